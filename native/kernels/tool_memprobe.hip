// gsx-memprobe: how much device memory does this process (pod) get?
//
//   gsx-memprobe [--device N] [--alloc BYTES[,BYTES...]] [--hold-ms MS] [--touch]
//                [--api malloc|async|finegrained|pitch|vmem|host] [--scratch KIB --blocks N]
//
// --api picks the allocation entry point (the isolation library must cap every one that takes HBM):
// hipMalloc, hipMallocAsync (stream-ordered pool), hipExtMallocWithFlags(fine-grained), hipMallocPitch,
// hipMemCreate (the virtual-memory API PyTorch's expandable segments use), or hipHostMalloc (host memory,
// which is not the device's and must not count).
//
// --streams N (with --scratch): the kernel runs on N streams at once (created before the code object loads), each
// over its own N blocks -- ROCr gives each hardware queue its own scratch, so they hold N times one dispatch's.
// The JSON then also carries the isolation library's per-queue scratch counters when it is loaded.
//
// --scratch loads gsx-scratch-KIB.hsaco (next to this executable) and launches, after the allocations, its kernel,
// whose every lane keeps a KIB-KiB private array (1, 4, 16 or 64) in scratch, over N 256-lane workgroups: the
// runtime sizes the queue's scratch for it behind any allocation API.  The JSON then carries the launch status and this process's VRAM as the kernel driver counts
// it (/sys/class/kfd/kfd/proc/<pid>/vram_*) before and after.
//
// Prints hipMemGetInfo before and after, then tries each allocation in turn (kept until exit) and prints one
// JSON line.  Operators run it inside a pod to see the HBM share the device plugin's isolation library enforces
// (native/isolate/gsx_isolate.cc); tests/test_gpu_isolate.py drives it against the share and past it.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <dirent.h>
#include <dlfcn.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

struct Held {
  void* p = nullptr;
  hipMemGenericAllocationHandle_t h{};
  bool vmem = false, host = false, async = false;
};

hipError_t alloc_one(const std::string& api, int dev, size_t bytes, bool touch, Held* out) {
  hipError_t r = hipErrorInvalidValue;
  if (api == "malloc") {
    r = hipMalloc(&out->p, bytes);
  } else if (api == "async") {
    out->async = true;
    r = hipMallocAsync(&out->p, bytes, nullptr);
    if (r == hipSuccess) r = hipStreamSynchronize(nullptr);
  } else if (api == "finegrained") {
    r = hipExtMallocWithFlags(&out->p, bytes, hipDeviceMallocFinegrained);
  } else if (api == "pitch") {
    size_t pitch = 0, width = 1 << 20;
    r = hipMallocPitch(&out->p, &pitch, width, (bytes + width - 1) / width);
  } else if (api == "host") {
    out->host = true;
    r = hipHostMalloc(&out->p, bytes, hipHostMallocDefault);
    return r;  // nothing to touch on the device
  } else if (api == "vmem") {
    out->vmem = true;
    hipMemAllocationProp prop{};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = dev;
    size_t gran = 0;
    r = hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum);
    if (r != hipSuccess) return r;
    size_t sz = (bytes + gran - 1) / gran * gran;
    r = hipMemCreate(&out->h, sz, &prop, 0);
    return r;  // created, not mapped: the cap is about the physical backing
  }
  if (r == hipSuccess && touch) r = hipMemset(out->p, 0x5a, bytes);
  if (r == hipSuccess) r = hipDeviceSynchronize();
  return r;
}

void free_one(const Held& h) {
  if (h.vmem) {
    (void)hipMemRelease(h.h);
  } else if (h.host) {
    (void)hipHostFree(h.p);
  } else if (h.async) {
    (void)hipFreeAsync(h.p, nullptr);
    (void)hipStreamSynchronize(nullptr);
  } else {
    (void)hipFree(h.p);
  }
}

// this process's VRAM as amdkfd accounts it (every GPU it has opened); -1 if the file is not there
long long kfd_vram() {
  char dir[128];
  std::snprintf(dir, sizeof dir, "/sys/class/kfd/kfd/proc/%d", static_cast<int>(getpid()));
  DIR* d = opendir(dir);
  if (!d) return -1;
  long long sum = -1;
  while (dirent* e = readdir(d)) {
    if (std::strncmp(e->d_name, "vram_", 5) != 0) continue;
    char path[512];
    std::snprintf(path, sizeof path, "%s/%s", dir, e->d_name);
    FILE* f = std::fopen(path, "r");
    if (!f) continue;
    long long v = 0;
    if (std::fscanf(f, "%lld", &v) == 1) sum = (sum < 0 ? 0 : sum) + v;
    std::fclose(f);
  }
  closedir(d);
  return sum;
}

// the HSA runtime's scratch thresholds for the first GPU agent (HIP has initialised the runtime already)
struct ScratchLimits {
  uint64_t max = 0, current = 0;
  hsa_agent_t agent{};
  bool found = false;
};

hsa_status_t find_gpu(hsa_agent_t a, void* data) {
  auto* sl = static_cast<ScratchLimits*>(data);
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS || t != HSA_DEVICE_TYPE_GPU) {
    return HSA_STATUS_SUCCESS;
  }
  sl->agent = a;
  sl->found = true;
  (void)hsa_agent_get_info(a, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_SCRATCH_LIMIT_MAX), &sl->max);
  (void)hsa_agent_get_info(a, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_SCRATCH_LIMIT_CURRENT), &sl->current);
  return HSA_STATUS_INFO_BREAK;
}

ScratchLimits scratch_limits() {
  ScratchLimits sl;
  (void)hsa_iterate_agents(find_gpu, &sl);
  return sl;
}

// the directory of this executable (the scratch probe's code objects sit next to it)
std::string exe_dir() {
  char buf[4096];
  ssize_t n = readlink("/proc/self/exe", buf, sizeof buf - 1);
  if (n <= 0) return ".";
  buf[n] = 0;
  std::string p(buf);
  size_t cut = p.rfind('/');
  return cut == std::string::npos ? "." : p.substr(0, cut);
}

// load gsx-scratch-<kib>.hsaco and run its kernel over `blocks` 256-lane workgroups; *stage names the step that
// failed ("load": the code object was refused, e.g. by the isolation library's scratch check)
hipError_t run_scratch(int kib, int blocks, int nstreams, const char** stage) {
  // the streams first: their hardware queues exist when the code object loads (the isolation library charges the
  // worst kernel's scratch on every queue then)
  *stage = "stream";
  std::vector<hipStream_t> streams;
  hipError_t r = hipSuccess;
  for (int i = 0; i < nstreams && nstreams > 1; ++i) {
    hipStream_t st = nullptr;
    r = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    if (r != hipSuccess) break;
    streams.push_back(st);
  }
  auto cleanup = [&] {
    for (hipStream_t st : streams) (void)hipStreamDestroy(st);
  };
  if (r != hipSuccess) {
    cleanup();
    return r;
  }
  if (streams.empty()) streams.push_back(nullptr);
  *stage = "load";
  hipModule_t mod = nullptr;
  const std::string path = exe_dir() + "/gsx-scratch-" + std::to_string(kib) + ".hsaco";
  r = hipModuleLoad(&mod, path.c_str());
  if (r != hipSuccess) {
    cleanup();
    return r;
  }
  hipFunction_t fn = nullptr;
  r = hipModuleGetFunction(&fn, mod, "gsx_scratch_kernel");
  if (r != hipSuccess) {
    cleanup();
    return r;
  }
  *stage = "launch";
  int* out = nullptr;
  r = hipMalloc(&out, static_cast<size_t>(blocks) * 256 * sizeof(int) * streams.size());
  if (r != hipSuccess) {
    cleanup();
    return r;
  }
  int seed = 3;
  for (size_t i = 0; i < streams.size() && r == hipSuccess; ++i) {
    int* o = out + i * static_cast<size_t>(blocks) * 256;
    void* args[] = {&o, &seed};
    r = hipModuleLaunchKernel(fn, static_cast<unsigned>(blocks), 1, 1, 256, 1, 1, 0, streams[i], args, nullptr);
  }
  hipError_t s = hipDeviceSynchronize();
  if (r == hipSuccess) r = s;
  (void)hipFree(out);
  if (streams[0] != nullptr) cleanup();
  *stage = r == hipSuccess ? "" : "launch";
  return r;
}

// the isolation library's per-queue scratch counters, when it is loaded in this process: {worst, queues, refused}
bool iso_scratch_queues(unsigned long long out[3]) {
  const char* tl = std::getenv("HSA_TOOLS_LIB");
  if (!tl) return false;
  std::string libs(tl);
  size_t p = 0;
  while (p <= libs.size()) {
    size_t q = libs.find_first_of(" :", p);
    if (q == std::string::npos) q = libs.size();
    std::string one = libs.substr(p, q - p);
    if (one.find("gsx_isolate") != std::string::npos) {
      void* h = dlopen(one.c_str(), RTLD_NOW | RTLD_NOLOAD);
      if (!h) return false;
      auto fn = reinterpret_cast<void (*)(uint64_t*)>(dlsym(h, "gsx_isolate_scratch_queues"));
      if (!fn) return false;
      uint64_t v[3];
      fn(v);
      for (int i = 0; i < 3; ++i) out[i] = v[i];
      return true;
    }
    p = q + 1;
  }
  return false;
}

}  // namespace

int main(int argc, char** argv) {
  int dev = 0, hold_ms = 0, scratch_kib = 0, blocks = 8192, nstreams = 1;
  long long set_limit = -1;
  bool touch = false;
  std::string api = "malloc";
  std::vector<size_t> sizes;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--device") && i + 1 < argc) {
      dev = std::atoi(argv[++i]);
    } else if (!std::strcmp(argv[i], "--alloc") && i + 1 < argc) {
      std::string s(argv[++i]);
      size_t p = 0;
      while (p < s.size()) {
        size_t q = s.find(',', p);
        if (q == std::string::npos) q = s.size();
        sizes.push_back(std::strtoull(s.substr(p, q - p).c_str(), nullptr, 10));
        p = q + 1;
      }
    } else if (!std::strcmp(argv[i], "--hold-ms") && i + 1 < argc) {
      hold_ms = std::atoi(argv[++i]);
    } else if (!std::strcmp(argv[i], "--touch")) {
      touch = true;
    } else if (!std::strcmp(argv[i], "--scratch") && i + 1 < argc) {
      scratch_kib = std::atoi(argv[++i]);
    } else if (!std::strcmp(argv[i], "--scratch-limit") && i + 1 < argc) {
      set_limit = std::atoll(argv[++i]);
    } else if (!std::strcmp(argv[i], "--blocks") && i + 1 < argc) {
      blocks = std::atoi(argv[++i]);
    } else if (!std::strcmp(argv[i], "--streams") && i + 1 < argc) {
      nstreams = std::atoi(argv[++i]);
    } else if (!std::strcmp(argv[i], "--api") && i + 1 < argc) {
      api = argv[++i];
    } else {
      std::fprintf(stderr, "usage: %s [--device N] [--alloc B,...] [--hold-ms MS] [--touch] [--api A] [--scratch KIB --blocks N --streams N --scratch-limit B]\n", argv[0]);
      return 2;
    }
  }
  if (hipSetDevice(dev) != hipSuccess) {
    std::fprintf(stderr, "hipSetDevice(%d) failed\n", dev);
    return 1;
  }
  size_t free0 = 0, total0 = 0;
  hipError_t e = hipMemGetInfo(&free0, &total0);
  if (e != hipSuccess) {
    std::fprintf(stderr, "hipMemGetInfo: %s\n", hipGetErrorString(e));
    return 1;
  }
  std::vector<Held> held;
  std::string rows;
  for (size_t b : sizes) {
    Held h;
    hipError_t r = alloc_one(api, dev, b, touch, &h);
    bool ok = r == hipSuccess && (h.p != nullptr || h.vmem);
    if (ok) held.push_back(h);
    (void)hipGetLastError();  // an OOM is sticky in some HIP versions' last-error slot
    char buf[256];
    std::snprintf(buf, sizeof buf, "%s{\"bytes\":%zu,\"ok\":%s,\"err\":\"%s\"}", rows.empty() ? "" : ",", b,
                  ok ? "true" : "false", ok ? "" : hipGetErrorName(r));
    rows += buf;
  }
  std::string scratch = "null";
  if (scratch_kib > 0) {
    if (set_limit >= 0) {
      ScratchLimits sl = scratch_limits();
      if (sl.found) (void)hsa_amd_agent_set_async_scratch_limit(sl.agent, static_cast<size_t>(set_limit));
    }
    long long v0 = kfd_vram();
    const char* stage = "";
    hipError_t r = run_scratch(scratch_kib, blocks, nstreams, &stage);
    (void)hipGetLastError();
    long long v1 = kfd_vram();
    size_t f = 0, t = 0;
    (void)hipMemGetInfo(&f, &t);
    unsigned long long sq[3] = {0, 0, 0};
    const bool have_iso = iso_scratch_queues(sq);
    char buf[768];
    std::snprintf(buf, sizeof buf,
                  "{\"kib_per_lane\":%d,\"blocks\":%d,\"streams\":%d,\"ok\":%s,\"err\":\"%s\",\"stage\":\"%s\","
                  "\"kfd_vram_before\":%lld,\"kfd_vram_after\":%lld,\"free_after\":%zu,\"iso\":%s,"
                  "\"iso_worst\":%llu,\"iso_queues\":%llu,\"iso_queues_refused\":%llu}",
                  scratch_kib, blocks, nstreams, r == hipSuccess ? "true" : "false",
                  r == hipSuccess ? "" : hipGetErrorName(r), stage, v0, v1, f, have_iso ? "true" : "false", sq[0],
                  sq[1], sq[2]);
    scratch = buf;
  }
  size_t free1 = 0, total1 = 0;
  (void)hipMemGetInfo(&free1, &total1);
  ScratchLimits sl = scratch_limits();
  std::printf("{\"device\":%d,\"api\":\"%s\",\"total\":%zu,\"free\":%zu,\"allocs\":[%s],\"free_after\":%zu,"
              "\"total_after\":%zu,\"scratch\":%s,\"kfd_vram\":%lld,\"scratch_limit_max\":%llu,"
              "\"scratch_limit_current\":%llu}\n", dev, api.c_str(), total0, free0, rows.c_str(), free1, total1,
              scratch.c_str(), kfd_vram(), static_cast<unsigned long long>(sl.max),
              static_cast<unsigned long long>(sl.current));
  std::fflush(stdout);
  if (hold_ms > 0) usleep(static_cast<useconds_t>(hold_ms) * 1000u);
  for (const Held& h : held) free_one(h);
  return 0;
}
