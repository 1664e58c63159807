// Host-only test of libgsx_isolate.so against a fake HSA runtime (no GPU, no ROCr).
//
// The test plays ROCr: it builds a CoreApiTable / AmdExtTable whose entries are fakes below, calls the
// library's OnLoad exactly as ROCr's tools loader does, and then calls through the (now hooked) tables.
// Checked: queues get the pod's CU mask, later set_mask calls are intersected with it, GPU-pool allocations
// are capped at the share (CPU pools are not), pool size / available memory report the share, frees give
// bytes back, and the ledger is shared by processes: a forked child sees the parent's bytes, and a dead
// process's bytes stop counting.
//
//   isolate_test <path to libgsx_isolate.so> <scratch dir>
#include <dlfcn.h>
#include <hsa/hsa.h>
#include <hsa/hsa_api_trace.h>
#include <hsa/hsa_ext_amd.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

static int g_fail = 0;
#define CHECK(c)                                                     \
  do {                                                               \
    if (!(c)) {                                                      \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                      \
    }                                                                \
  } while (0)

constexpr uint64_t GPU_POOL = 1, CPU_POOL = 2, GPU_AGENT = 10, CPU_AGENT = 11;
constexpr size_t POOL_SIZE = size_t{288} << 30;
static std::vector<uint32_t> g_last_mask;
static hsa_queue_t g_queue;

static hsa_queue_t g_more[16];
static int g_nmore = 0;
static bool g_fail_create = false;  // the runtime refuses the next queue creations
static hsa_status_t fake_queue_create(hsa_agent_t, uint32_t, hsa_queue_type32_t, void (*)(hsa_status_t, hsa_queue_t*, void*),
                                      void*, uint32_t, uint32_t, hsa_queue_t** q) {
  if (g_fail_create) return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  *q = g_nmore == 0 ? &g_queue : &g_more[g_nmore - 1];
  if (g_nmore < 16) g_nmore++;
  g_last_mask.clear();
  return HSA_STATUS_SUCCESS;
}
static hsa_status_t fake_queue_destroy(hsa_queue_t*) { return HSA_STATUS_SUCCESS; }
static hsa_status_t fake_set_mask(const hsa_queue_t*, uint32_t nbits, const uint32_t* m) {
  g_last_mask.assign(m, m + (nbits + 31) / 32);
  return HSA_STATUS_SUCCESS;
}
static hsa_status_t fake_pool_get_info(hsa_amd_memory_pool_t p, hsa_amd_memory_pool_info_t a, void* v) {
  switch (a) {
    case HSA_AMD_MEMORY_POOL_INFO_SEGMENT: *static_cast<hsa_amd_segment_t*>(v) = HSA_AMD_SEGMENT_GLOBAL; break;
    case HSA_AMD_MEMORY_POOL_INFO_LOCATION:
      *static_cast<hsa_amd_memory_pool_location_t*>(v) =
          p.handle == GPU_POOL ? HSA_AMD_MEMORY_POOL_LOCATION_GPU : HSA_AMD_MEMORY_POOL_LOCATION_CPU;
      break;
    case HSA_AMD_MEMORY_POOL_INFO_SIZE: *static_cast<size_t*>(v) = POOL_SIZE; break;
    default: return HSA_STATUS_ERROR_INVALID_ARGUMENT;
  }
  return HSA_STATUS_SUCCESS;
}
static bool g_slow_alloc = false;  // widen the window between the share check and the allocation's record
static hsa_status_t fake_pool_allocate(hsa_amd_memory_pool_t, size_t size, uint32_t, void** ptr) {
  if (g_slow_alloc) usleep(100000);
  *ptr = std::malloc(16);  // a unique address stands in for the device allocation
  return *ptr ? HSA_STATUS_SUCCESS : HSA_STATUS_ERROR_OUT_OF_RESOURCES;
}
static hsa_status_t fake_pool_free(void* p) {
  std::free(p);
  return HSA_STATUS_SUCCESS;
}
static hsa_status_t fake_agent_get_info(hsa_agent_t a, hsa_agent_info_t attr, void* v) {
  if (attr == HSA_AGENT_INFO_DEVICE) {
    *static_cast<hsa_device_type_t*>(v) = a.handle == GPU_AGENT ? HSA_DEVICE_TYPE_GPU : HSA_DEVICE_TYPE_CPU;
    return HSA_STATUS_SUCCESS;
  }
  if (static_cast<int>(attr) == static_cast<int>(HSA_AMD_AGENT_INFO_MEMORY_AVAIL)) {
    *static_cast<uint64_t*>(v) = POOL_SIZE;
    return HSA_STATUS_SUCCESS;
  }
  switch (static_cast<int>(attr)) {  // an MI355X: 256 CUs x 32 wave slots of 64 lanes, 32 GiB scratch at most
    case HSA_AMD_AGENT_INFO_COMPUTE_UNIT_COUNT: *static_cast<uint32_t*>(v) = 256; return HSA_STATUS_SUCCESS;
    case HSA_AMD_AGENT_INFO_MAX_WAVES_PER_CU: *static_cast<uint32_t*>(v) = 32; return HSA_STATUS_SUCCESS;
    case HSA_AGENT_INFO_WAVEFRONT_SIZE: *static_cast<uint32_t*>(v) = 64; return HSA_STATUS_SUCCESS;
    case HSA_AMD_AGENT_INFO_SCRATCH_LIMIT_MAX: *static_cast<uint64_t*>(v) = uint64_t{32} << 30; return HSA_STATUS_SUCCESS;
    default: break;
  }
  return HSA_STATUS_ERROR_INVALID_ARGUMENT;
}

// ---- a fake loader: executable handle -> the private bytes per lane of its kernels
static std::vector<std::vector<uint32_t>> g_exes;
static uint64_t g_scratch_limit_set = 0;
static hsa_status_t fake_freeze(hsa_executable_t, const char*) { return HSA_STATUS_SUCCESS; }
static hsa_status_t fake_iterate_symbols(hsa_executable_t e,
                                         hsa_status_t (*cb)(hsa_executable_t, hsa_executable_symbol_t, void*),
                                         void* data) {
  for (size_t k = 0; k < g_exes[e.handle].size(); ++k) {
    hsa_status_t s = cb(e, hsa_executable_symbol_t{(e.handle << 16) | k}, data);
    if (s != HSA_STATUS_SUCCESS) return s;
  }
  return HSA_STATUS_SUCCESS;
}
static hsa_status_t fake_symbol_get_info(hsa_executable_symbol_t sym, hsa_executable_symbol_info_t attr, void* v) {
  switch (attr) {
    case HSA_EXECUTABLE_SYMBOL_INFO_TYPE: *static_cast<hsa_symbol_kind_t*>(v) = HSA_SYMBOL_KIND_KERNEL; break;
    case HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE:
      *static_cast<uint32_t*>(v) = g_exes[sym.handle >> 16][sym.handle & 0xffff];
      break;
    case HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_DYNAMIC_CALLSTACK: *static_cast<bool*>(v) = false; break;
    case HSA_EXECUTABLE_SYMBOL_INFO_AGENT: *static_cast<hsa_agent_t*>(v) = hsa_agent_t{GPU_AGENT}; break;
    default: return HSA_STATUS_ERROR_INVALID_ARGUMENT;
  }
  return HSA_STATUS_SUCCESS;
}
static hsa_status_t fake_set_scratch_limit(hsa_agent_t, size_t threshold) {
  g_scratch_limit_set = threshold;
  return HSA_STATUS_SUCCESS;
}

static CoreApiTable core;
static AmdExtTable amd;

static hsa_status_t alloc(uint64_t pool, size_t gib, void** p) {
  return amd.hsa_amd_memory_pool_allocate_fn(hsa_amd_memory_pool_t{pool}, gib << 30, 0, p);
}

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  std::string dir = argv[2];
  std::string conf = dir + "/isolation.conf", ledger = dir + "/hbm.ledger";
  FILE* f = std::fopen(conf.c_str(), "w");
  // 32 CUs: CUs 0-7 of every other 32-CU block
  std::fprintf(f, "# written by the device plugin\ncu_mask=0x000000ff,0x00000000,0x000000ff,0x00000000,"
                  "0x000000ff,0x00000000,0x000000ff,0x00000000\nhbm_limit_bytes=%llu\nledger=%s\n",
               static_cast<unsigned long long>(size_t{100} << 30), ledger.c_str());
  std::fclose(f);
  setenv("GSX_ISOLATION_CONFIG", conf.c_str(), 1);
  unsetenv("HSA_TOOLS_LIB");

  void* h = dlopen(argv[1], RTLD_NOW);
  if (!h) {
    std::fprintf(stderr, "dlopen: %s\n", dlerror());
    return 1;
  }
  // the preload constructor put the library into HSA_TOOLS_LIB
  const char* tl = std::getenv("HSA_TOOLS_LIB");
  CHECK(tl != nullptr && std::strstr(tl, "gsx_isolate") != nullptr);

  std::memset(&core, 0, sizeof core);
  std::memset(&amd, 0, sizeof amd);
  core.version.minor_id = sizeof(CoreApiTable);
  amd.version.minor_id = sizeof(AmdExtTable);
  core.hsa_queue_create_fn = fake_queue_create;
  core.hsa_queue_destroy_fn = fake_queue_destroy;
  core.hsa_agent_get_info_fn = fake_agent_get_info;
  amd.hsa_amd_queue_cu_set_mask_fn = fake_set_mask;
  amd.hsa_amd_memory_pool_get_info_fn = fake_pool_get_info;
  amd.hsa_amd_memory_pool_allocate_fn = fake_pool_allocate;
  amd.hsa_amd_memory_pool_free_fn = fake_pool_free;
  core.hsa_executable_freeze_fn = fake_freeze;
  core.hsa_executable_iterate_symbols_fn = fake_iterate_symbols;
  core.hsa_executable_symbol_get_info_fn = fake_symbol_get_info;
  amd.hsa_amd_agent_set_async_scratch_limit_fn = fake_set_scratch_limit;
  HsaApiTable table;
  std::memset(&table, 0, sizeof table);
  table.core_ = &core;
  table.amd_ext_ = &amd;
  auto onload = reinterpret_cast<bool (*)(HsaApiTable*, uint64_t, uint64_t, const char* const*)>(dlsym(h, "OnLoad"));
  auto stats = reinterpret_cast<void (*)(uint64_t*)>(dlsym(h, "gsx_isolate_stats"));
  CHECK(onload && stats);
  CHECK(onload(&table, 3, 0, nullptr));
  CHECK(core.hsa_queue_create_fn != fake_queue_create);

  // ---- CU partition
  hsa_queue_t* q = nullptr;
  CHECK(core.hsa_queue_create_fn(hsa_agent_t{GPU_AGENT}, 1024, HSA_QUEUE_TYPE_MULTI, nullptr, nullptr, 0, 0, &q) ==
        HSA_STATUS_SUCCESS);
  CHECK(g_last_mask.size() == 8 && g_last_mask[0] == 0xff && g_last_mask[1] == 0 && g_last_mask[6] == 0xff);
  std::vector<uint32_t> all(8, 0xffffffffu);
  // "all CUs": stays inside the partition, and succeeds (HIP fails a stream on any other status)
  CHECK(amd.hsa_amd_queue_cu_set_mask_fn(q, 256, all.data()) == HSA_STATUS_SUCCESS);
  CHECK(g_last_mask.size() == 8 && g_last_mask[0] == 0xff && g_last_mask[1] == 0);
  CHECK(amd.hsa_amd_queue_cu_set_mask_fn(q, 0, nullptr) == HSA_STATUS_SUCCESS);  // reset: the partition again
  CHECK(g_last_mask[0] == 0xff && g_last_mask[2] == 0xff);
  std::vector<uint32_t> narrow(8, 0);
  narrow[0] = 0x0f;  // a narrower request inside the partition is honoured as is
  CHECK(amd.hsa_amd_queue_cu_set_mask_fn(q, 256, narrow.data()) == HSA_STATUS_SUCCESS);
  CHECK(g_last_mask[0] == 0x0f && g_last_mask[2] == 0);
  std::vector<uint32_t> outside(8, 0);
  outside[1] = 0xff;  // entirely outside: keeps the partition
  amd.hsa_amd_queue_cu_set_mask_fn(q, 256, outside.data());
  CHECK(g_last_mask[0] == 0xff && g_last_mask[1] == 0);

  // ---- HBM share
  size_t sz = 0;
  CHECK(amd.hsa_amd_memory_pool_get_info_fn(hsa_amd_memory_pool_t{GPU_POOL}, HSA_AMD_MEMORY_POOL_INFO_SIZE, &sz) ==
        HSA_STATUS_SUCCESS);
  CHECK(sz == size_t{100} << 30);
  CHECK(amd.hsa_amd_memory_pool_get_info_fn(hsa_amd_memory_pool_t{CPU_POOL}, HSA_AMD_MEMORY_POOL_INFO_SIZE, &sz) ==
        HSA_STATUS_SUCCESS);
  CHECK(sz == POOL_SIZE);
  void *a = nullptr, *b = nullptr, *c = nullptr, *big = nullptr;
  CHECK(alloc(GPU_POOL, 60, &a) == HSA_STATUS_SUCCESS);
  CHECK(alloc(GPU_POOL, 50, &b) == HSA_STATUS_ERROR_OUT_OF_RESOURCES);  // 110 > 100
  CHECK(alloc(CPU_POOL, 500, &big) == HSA_STATUS_SUCCESS);             // host memory is not the share
  uint64_t avail = 0;
  CHECK(core.hsa_agent_get_info_fn(hsa_agent_t{GPU_AGENT}, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_MEMORY_AVAIL),
                                   &avail) == HSA_STATUS_SUCCESS);
  CHECK(avail == uint64_t{40} << 30);
  CHECK(alloc(GPU_POOL, 40, &c) == HSA_STATUS_SUCCESS);  // exactly the share
  CHECK(amd.hsa_amd_memory_pool_free_fn(c) == HSA_STATUS_SUCCESS);

  // ---- the ledger is per pod: a forked child sees the parent's 60 GiB
  pid_t pid = fork();
  if (pid == 0) {
    void *x = nullptr, *y = nullptr;
    int bad = 0;
    if (alloc(GPU_POOL, 50, &x) != HSA_STATUS_ERROR_OUT_OF_RESOURCES) bad |= 1;  // 60 + 50 > 100
    if (alloc(GPU_POOL, 30, &y) != HSA_STATUS_SUCCESS) bad |= 2;                 // 60 + 30 fits
    _exit(bad);  // dies holding 30 GiB: its slot stops counting with it
  }
  int st = 0;
  waitpid(pid, &st, 0);
  CHECK(WIFEXITED(st) && WEXITSTATUS(st) == 0);
  void* d = nullptr;
  CHECK(alloc(GPU_POOL, 40, &d) == HSA_STATUS_SUCCESS);  // the dead child's 30 GiB are not held against us

  // a second, independent process of the same pod (another container: same ledger file, new process)
  int up[2], down[2];  // child -> parent, parent -> child
  CHECK(pipe(up) == 0 && pipe(down) == 0);
  pid = fork();
  if (pid == 0) {
    // parent holds 100 of 100 now: nothing fits until it frees
    void* x = nullptr;
    int bad = alloc(GPU_POOL, 1, &x) == HSA_STATUS_ERROR_OUT_OF_RESOURCES ? 0 : 1;
    char ch;
    if (write(up[1], "r", 1) != 1) bad |= 4;
    if (read(down[0], &ch, 1) != 1) bad |= 8;  // parent freed 40
    if (alloc(GPU_POOL, 40, &x) != HSA_STATUS_SUCCESS) bad |= 2;
    _exit(bad);
  }
  char ch;
  CHECK(read(up[0], &ch, 1) == 1);
  CHECK(amd.hsa_amd_memory_pool_free_fn(d) == HSA_STATUS_SUCCESS);
  CHECK(write(down[1], "g", 1) == 1);
  waitpid(pid, &st, 0);
  CHECK(WIFEXITED(st) && WEXITSTATUS(st) == 0);

  uint64_t sv[5];
  stats(sv);
  CHECK(sv[0] == 1 && sv[2] >= 1 && sv[3] == uint64_t{60} << 30 && sv[4] == 2);
  CHECK(amd.hsa_amd_memory_pool_free_fn(a) == HSA_STATUS_SUCCESS);
  stats(sv);
  CHECK(sv[3] == 0);
  amd.hsa_amd_memory_pool_free_fn(big);

  // ---- two processes of the pod allocate at once: the check and the reservation are one step under
  // the ledger lock, so of two 60 GiB allocations against the 100 GiB share exactly one succeeds, however slow
  // the runtime's allocation between the check and its record
  g_slow_alloc = true;
  int go[2], res[2];
  CHECK(pipe(go) == 0 && pipe(res) == 0);
  pid_t kids[2];
  for (int k = 0; k < 2; ++k) {
    kids[k] = fork();
    if (kids[k] == 0) {
      char c;
      if (read(go[0], &c, 1) != 1) _exit(9);
      void* x = nullptr;
      char ok = alloc(GPU_POOL, 60, &x) == HSA_STATUS_SUCCESS ? '1' : '0';
      if (write(res[1], &ok, 1) != 1) _exit(9);
      if (read(go[0], &c, 1) != 1) _exit(9);  // hold the allocation until both answered
      _exit(0);
    }
  }
  CHECK(write(go[1], "gg", 2) == 2);
  int granted = 0;
  for (int k = 0; k < 2; ++k) {
    char c = 0;
    CHECK(read(res[0], &c, 1) == 1);
    granted += c == '1';
  }
  CHECK(write(go[1], "gg", 2) == 2);
  for (int k = 0; k < 2; ++k) waitpid(kids[k], &st, 0);
  CHECK(granted == 1);
  g_slow_alloc = false;

  // ---- scratch: a loaded code object charges its worst kernel (lane bytes in 256-byte granules x 64 lanes x 32
  // waves x 256 CUs) against the share, sets the agent's async scratch limit to it, and is refused if it cannot fit
  auto scratch = reinterpret_cast<void (*)(uint64_t*)>(dlsym(h, "gsx_isolate_scratch"));
  CHECK(scratch != nullptr);
  g_exes = {{0, 1040, 200}, {4112}, {16400}, {0}};
  const uint64_t slots = uint64_t{64} * 32 * 256;
  uint64_t sc[3];
  CHECK(core.hsa_executable_freeze_fn(hsa_executable_t{0}, nullptr) == HSA_STATUS_SUCCESS);
  scratch(sc);
  CHECK(sc[0] == 1280 * slots && sc[1] == 0 && sc[2] == 1280 * slots && g_scratch_limit_set == 1280 * slots);
  stats(sv);
  CHECK(sv[3] == 1280 * slots);  // part of this process's share
  CHECK(core.hsa_executable_freeze_fn(hsa_executable_t{3}, nullptr) == HSA_STATUS_SUCCESS);  // no scratch: no change
  CHECK(core.hsa_executable_freeze_fn(hsa_executable_t{1}, nullptr) == HSA_STATUS_SUCCESS);  // raised, not added
  scratch(sc);
  CHECK(sc[0] == 4352 * slots && g_scratch_limit_set == 4352 * slots);
  void* e = nullptr;
  CHECK(alloc(GPU_POOL, 95, &e) == HSA_STATUS_SUCCESS);  // 95 GiB + 2.3 GB of scratch: fits the 100 GiB share
  // 16400 bytes a lane: 8.7 GB at full occupancy, more than the share has left
  CHECK(core.hsa_executable_freeze_fn(hsa_executable_t{2}, nullptr) == HSA_STATUS_ERROR_OUT_OF_RESOURCES);
  scratch(sc);
  CHECK(sc[0] == 4352 * slots && sc[1] == 1);
  CHECK(amd.hsa_amd_memory_pool_free_fn(e) == HSA_STATUS_SUCCESS);
  CHECK(core.hsa_executable_freeze_fn(hsa_executable_t{2}, nullptr) == HSA_STATUS_SUCCESS);  // room again
  scratch(sc);
  CHECK(sc[0] == 16640 * slots);

  // ---- scratch is per queue (ROCr gives each hardware queue its own): every queue past the first adds the worst
  // kernel's scratch to the charge; a queue that no longer fits is refused, a destroyed one gives its share back
  auto squeues = reinterpret_cast<void (*)(uint64_t*)>(dlsym(h, "gsx_isolate_scratch_queues"));
  CHECK(squeues != nullptr);
  uint64_t sq[3];
  squeues(sq);
  CHECK(sq[0] == 16640 * slots && sq[1] == 1 && sq[2] == 0);  // the CU-partition test's queue
  const uint64_t per = 16640 * slots;                          // ~8.7 GB a queue
  std::vector<hsa_queue_t*> extra;
  for (;;) {
    hsa_queue_t* x = nullptr;
    hsa_status_t qs = core.hsa_queue_create_fn(hsa_agent_t{GPU_AGENT}, 1024, HSA_QUEUE_TYPE_MULTI, nullptr, nullptr,
                                               0, 0, &x);
    if (qs != HSA_STATUS_SUCCESS) {
      CHECK(qs == HSA_STATUS_ERROR_OUT_OF_RESOURCES);
      break;
    }
    extra.push_back(x);
    CHECK(extra.size() < 16);
  }
  scratch(sc);
  squeues(sq);
  const uint64_t fit = (uint64_t{100} << 30) / per;  // queues whose scratch the 100 GiB share holds
  CHECK(sq[1] == fit && sq[2] == 1 && sc[0] == per * fit && extra.size() + 1 == fit);
  stats(sv);
  CHECK(sv[3] == per * fit);  // charged against the share like an allocation
  CHECK(core.hsa_queue_destroy_fn(extra.back()) == HSA_STATUS_SUCCESS);
  scratch(sc);
  squeues(sq);
  CHECK(sq[1] == fit - 1 && sc[0] == per * (fit - 1));
  // with every queue able to run it at once, a code object raising the worst kernel is charged on each
  g_exes.push_back({20496});  // 20496 bytes a lane (20736 in granules)
  CHECK(core.hsa_executable_freeze_fn(hsa_executable_t{4}, nullptr) == HSA_STATUS_ERROR_OUT_OF_RESOURCES);
  for (size_t k = 0; k + 1 < extra.size(); ++k) CHECK(core.hsa_queue_destroy_fn(extra[k]) == HSA_STATUS_SUCCESS);
  squeues(sq);
  CHECK(sq[1] == 1);
  CHECK(core.hsa_executable_freeze_fn(hsa_executable_t{4}, nullptr) == HSA_STATUS_SUCCESS);  // one queue: fits
  scratch(sc);
  CHECK(sc[0] == 20736 * slots);
  // a queue is counted and its share charged in one step before the runtime creates it; one the runtime
  // fails gives both back (the count and the charge of a second queue that was never made)
  g_fail_create = true;
  hsa_queue_t* nq = nullptr;
  CHECK(core.hsa_queue_create_fn(hsa_agent_t{GPU_AGENT}, 1024, HSA_QUEUE_TYPE_MULTI, nullptr, nullptr, 0, 0, &nq) ==
        HSA_STATUS_ERROR_OUT_OF_RESOURCES);
  g_fail_create = false;
  squeues(sq);
  scratch(sc);
  CHECK(sq[1] == 1 && sc[0] == 20736 * slots);
  stats(sv);
  CHECK(sv[3] == 20736 * slots);
  CHECK(core.hsa_queue_create_fn(hsa_agent_t{GPU_AGENT}, 1024, HSA_QUEUE_TYPE_MULTI, nullptr, nullptr, 0, 0, &nq) ==
        HSA_STATUS_SUCCESS);
  squeues(sq);
  scratch(sc);
  CHECK(sq[1] == 2 && sc[0] == 2 * 20736 * slots);
  CHECK(core.hsa_queue_destroy_fn(nq) == HSA_STATUS_SUCCESS);
  squeues(sq);
  scratch(sc);
  CHECK(sq[1] == 1 && sc[0] == 20736 * slots);
  if (g_fail == 0) std::printf("isolate_test: OK\n");
  return g_fail ? 1 : 0;
}
