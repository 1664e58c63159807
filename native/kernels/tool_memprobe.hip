// gsx-memprobe: how much device memory does this process (pod) get?
//
//   gsx-memprobe [--device N] [--alloc BYTES[,BYTES...]] [--hold-ms MS] [--touch]
//                [--api malloc|async|finegrained|pitch|vmem|host]
//
// --api picks the allocation entry point (the isolation library must cap every one that takes HBM):
// hipMalloc, hipMallocAsync (stream-ordered pool), hipExtMallocWithFlags(fine-grained), hipMallocPitch,
// hipMemCreate (the virtual-memory API PyTorch's expandable segments use), or hipHostMalloc (host memory,
// which is not the device's and must not count).
//
// Prints hipMemGetInfo before and after, then tries each allocation in turn (kept until exit) and prints one
// JSON line.  Operators run it inside a pod to see the HBM share the device plugin's isolation library enforces
// (native/isolate/gsx_isolate.cc); tests/test_gpu_isolate.py drives it against the share and past it.
#include <hip/hip_runtime.h>
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

}  // namespace

int main(int argc, char** argv) {
  int dev = 0, hold_ms = 0;
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
    } else if (!std::strcmp(argv[i], "--api") && i + 1 < argc) {
      api = argv[++i];
    } else {
      std::fprintf(stderr, "usage: %s [--device N] [--alloc B,...] [--hold-ms MS] [--touch] [--api A]\n", argv[0]);
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
  size_t free1 = 0, total1 = 0;
  (void)hipMemGetInfo(&free1, &total1);
  std::printf("{\"device\":%d,\"api\":\"%s\",\"total\":%zu,\"free\":%zu,\"allocs\":[%s],\"free_after\":%zu,"
              "\"total_after\":%zu}\n", dev, api.c_str(), total0, free0, rows.c_str(), free1, total1);
  std::fflush(stdout);
  if (hold_ms > 0) usleep(static_cast<useconds_t>(hold_ms) * 1000u);
  for (const Held& h : held) free_one(h);
  return 0;
}
