// libgsx_isolate.so — enforced per-pod GPU isolation for MI355X (the "integrate Nvidia MPS" roadmap item of the
// reference, /root/reference/README.md:77, which docs/designs/designs.md:25-28 leaves to the application).
//
// The device plugin used to hand a pod its share only as advice: HSA_CU_MASK in the container env (a process
// that drops it gets all 256 CUs) and GSX_GPU_MEM_FRACTION (honoured only by cooperating PyTorch code).  This
// library moves both into the HSA runtime, underneath HIP, so that an arbitrary HIP/HSA program is confined:
//
//  * it is an HSA tools library: ROCr dlopen()s every library named in HSA_TOOLS_LIB during hsa_init() and
//    calls its OnLoad() with the live API dispatch table; OnLoad swaps in the hooks below;
//  * CU partition: every queue the process creates (hsa_queue_create, hsa_amd_queue_intercept_create) gets the
//    pod's CU mask before it is returned, and every later hsa_amd_queue_cu_set_mask (hipExtStreamCreateWithCUMask,
//    a "reset to all CUs" with count 0, ...) is intersected with it — a queue can narrow its partition, never
//    leave it;
//  * HBM share: device-memory allocations (hsa_amd_memory_pool_allocate on a GPU pool, hsa_amd_vmem_handle_create)
//    are accounted against the pod's gpu-mem share and fail with HSA_STATUS_ERROR_OUT_OF_RESOURCES (hipMalloc:
//    hipErrorOutOfMemory) beyond it.  The account is per pod, not per process: every process of the pod (every
//    container, every fork) holds a slot in one shared ledger file; a slot counts while its owner lives (an OFD
//    byte-range lock the kernel drops when the process dies, so a crashed process never leaks its share);
//  * the GPU pools report the share as their size and the agent reports (share - used) as available memory, so
//    hipMemGetInfo / torch.cuda.mem_get_info / the PyTorch caching allocator see a device of the pod's size.
//
// Configuration is a root-written file the plugin mounts read-only: /run/gsx/isolation.conf (a container cannot
// edit or hide it).  Only when that path does not exist is $GSX_ISOLATION_CONFIG consulted (tests, host runs).
//     cu_mask=0x000000ff,0x00000000,...   (32-bit words, CU c = bit c%32 of word c/32; GSX_CU_MASK format)
//     hbm_limit_bytes=68719476736
//     ledger=/run/gsx/hbm.ledger
// Loaded through /etc/ld.so.preload (mounted by the plugin), the constructor below adds the library to
// HSA_TOOLS_LIB before the program's first HIP call, so unsetting environment variables does not escape it.
// Not covered: statically linked programs, and processes that drive /dev/kfd ioctls directly.
#include <dlfcn.h>
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <hsa/hsa.h>
#include <hsa/hsa_api_trace.h>
#include <hsa/hsa_ext_amd.h>
#include <pthread.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <unordered_map>
#include <vector>

#define GSX_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

constexpr const char* kFixedConfig = "/run/gsx/isolation.conf";
constexpr uint64_t kMagic = 0x31304d4248585347ull;  // "GSXHBM01"
constexpr int kSlots = 256;

struct LedgerFile {
  uint64_t magic;
  uint64_t reserved[7];          // 64-byte header; byte 0 is the ledger's mutex (an OFD write lock)
  uint64_t bytes[kSlots];        // slot i = device bytes held by the process that holds the lock on byte 64+i
};

struct Config {
  std::vector<uint32_t> cu_mask;  // empty: no CU partition
  uint64_t hbm_limit = 0;         // 0: no cap
  std::string ledger;             // empty: per-process account
  std::string source;
  bool verbose = false;
};

// Process state is never destroyed: HIP's own static destructors (which run after ours, the library having
// been loaded after libamdhip64) still free device memory through the hooks at exit.
Config& g_cfg = *new Config;
std::mutex& g_mu = *new std::mutex;  // the process-local half of the ledger lock (OFD locks do not exclude threads)
std::unordered_map<uintptr_t, uint64_t>& g_allocs = *new std::unordered_map<uintptr_t, uint64_t>;  // ptr -> bytes
uint64_t g_local_used = 0;        // this process's device bytes (the ledger slot mirrors it)
int g_fd = -1;
LedgerFile* g_map = nullptr;
int g_slot = -1;
std::atomic<uint64_t> g_stats_queues{0}, g_stats_masked{0}, g_stats_denied{0}, g_stats_reduced{0};

// the runtime's own entry points, saved by OnLoad
decltype(hsa_queue_create)* real_queue_create = nullptr;
decltype(hsa_agent_get_info)* real_agent_get_info = nullptr;
decltype(hsa_amd_queue_cu_set_mask)* real_cu_set_mask = nullptr;
decltype(hsa_amd_queue_intercept_create)* real_intercept_create = nullptr;
decltype(hsa_amd_memory_pool_get_info)* real_pool_get_info = nullptr;
decltype(hsa_amd_memory_pool_allocate)* real_pool_allocate = nullptr;
decltype(hsa_amd_memory_pool_free)* real_pool_free = nullptr;
decltype(hsa_amd_vmem_handle_create)* real_vmem_create = nullptr;
decltype(hsa_amd_vmem_handle_release)* real_vmem_release = nullptr;

#define GSX_LOG(...)                                                        \
  do {                                                                      \
    if (g_cfg.verbose) {                                                    \
      std::fprintf(stderr, "gsx-isolate[%d]: ", static_cast<int>(getpid())); \
      std::fprintf(stderr, __VA_ARGS__);                                    \
      std::fputc('\n', stderr);                                             \
    }                                                                       \
  } while (0)

std::string trim(const std::string& s) {
  size_t a = s.find_first_not_of(" \t\r\n"), b = s.find_last_not_of(" \t\r\n");
  return a == std::string::npos ? std::string() : s.substr(a, b - a + 1);
}

bool parse_config(const char* path, Config* out) {
  FILE* f = std::fopen(path, "r");
  if (!f) return false;
  char line[4096];
  while (std::fgets(line, sizeof line, f)) {
    std::string l = trim(line);
    if (l.empty() || l[0] == '#') continue;
    size_t eq = l.find('=');
    if (eq == std::string::npos) continue;
    std::string k = trim(l.substr(0, eq)), v = trim(l.substr(eq + 1));
    if (k == "cu_mask") {
      size_t i = 0;
      while (i < v.size()) {
        size_t j = v.find(',', i);
        if (j == std::string::npos) j = v.size();
        std::string w = trim(v.substr(i, j - i));
        if (!w.empty()) out->cu_mask.push_back(static_cast<uint32_t>(std::strtoul(w.c_str(), nullptr, 16)));
        i = j + 1;
      }
    } else if (k == "hbm_limit_bytes") {
      out->hbm_limit = std::strtoull(v.c_str(), nullptr, 10);
    } else if (k == "ledger") {
      out->ledger = v;
    } else if (k == "verbose") {
      out->verbose = v == "1" || v == "true";
    }
  }
  std::fclose(f);
  bool any = false;
  for (uint32_t w : out->cu_mask) any = any || w != 0;
  if (!any) out->cu_mask.clear();  // an all-zero mask would stop every queue: treat it as "no partition"
  out->source = path;
  return true;
}

const char* config_path() {
  struct stat st;
  if (::stat(kFixedConfig, &st) == 0) return kFixedConfig;
  const char* e = std::getenv("GSX_ISOLATION_CONFIG");
  return e && *e ? e : nullptr;
}

// ------------------------------------------------------------------ shared per-pod HBM ledger
int ofd_lock(int fd, short type, off_t off, bool wait) {
  struct flock fl;
  std::memset(&fl, 0, sizeof fl);
  fl.l_type = type;
  fl.l_whence = SEEK_SET;
  fl.l_start = off;
  fl.l_len = 1;
  int r;
  do {
    r = ::fcntl(fd, wait ? F_OFD_SETLKW : F_OFD_SETLK, &fl);
  } while (r != 0 && errno == EINTR);
  return r;
}

bool slot_alive(int fd, int i) {
  struct flock fl;
  std::memset(&fl, 0, sizeof fl);
  fl.l_type = F_WRLCK;
  fl.l_whence = SEEK_SET;
  fl.l_start = static_cast<off_t>(offsetof(LedgerFile, bytes) + i);
  fl.l_len = 1;
  if (::fcntl(fd, F_OFD_GETLK, &fl) != 0) return false;
  return fl.l_type != F_UNLCK;  // another open file description holds the slot: its process is alive
}

// open + map the ledger and claim a free slot (caller holds g_mu); false: fall back to a per-process account
bool ledger_open() {
  if (g_map) return true;
  if (g_cfg.ledger.empty()) return false;
  int fd = ::open(g_cfg.ledger.c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0666);
  if (fd < 0) return false;
  if (ofd_lock(fd, F_WRLCK, 0, true) != 0) {
    ::close(fd);
    return false;
  }
  struct stat st;
  if (::fstat(fd, &st) != 0 || (st.st_size < static_cast<off_t>(sizeof(LedgerFile)) &&
                                ::ftruncate(fd, sizeof(LedgerFile)) != 0)) {
    ofd_lock(fd, F_UNLCK, 0, false);
    ::close(fd);
    return false;
  }
  void* p = ::mmap(nullptr, sizeof(LedgerFile), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (p == MAP_FAILED) {
    ofd_lock(fd, F_UNLCK, 0, false);
    ::close(fd);
    return false;
  }
  auto* m = static_cast<LedgerFile*>(p);
  if (m->magic != kMagic) {
    std::memset(m, 0, sizeof(LedgerFile));
    m->magic = kMagic;
  }
  int slot = -1;
  for (int i = 0; i < kSlots && slot < 0; ++i) {
    if (slot_alive(fd, i)) continue;
    if (ofd_lock(fd, F_WRLCK, static_cast<off_t>(offsetof(LedgerFile, bytes) + i), false) == 0) slot = i;
  }
  if (slot < 0) {
    ofd_lock(fd, F_UNLCK, 0, false);
    ::munmap(p, sizeof(LedgerFile));
    ::close(fd);
    return false;
  }
  m->bytes[slot] = g_local_used;  // a dead owner's count is dropped with its slot
  ofd_lock(fd, F_UNLCK, 0, false);
  g_fd = fd;
  g_map = m;
  g_slot = slot;
  GSX_LOG("ledger %s slot %d", g_cfg.ledger.c_str(), slot);
  return true;
}

// bytes the whole pod holds on the device, this process included (caller holds g_mu and the ledger lock)
uint64_t pod_used_locked() {
  if (!g_map) return g_local_used;
  uint64_t sum = g_local_used;
  for (int i = 0; i < kSlots; ++i) {
    if (i == g_slot || g_map->bytes[i] == 0) continue;
    if (slot_alive(g_fd, i)) sum += g_map->bytes[i];
  }
  return sum;
}

struct LedgerGuard {
  bool held = false;
  LedgerGuard() {
    if (g_map) held = ofd_lock(g_fd, F_WRLCK, 0, true) == 0;
  }
  ~LedgerGuard() {
    if (held) ofd_lock(g_fd, F_UNLCK, 0, false);
  }
};

void after_fork_child() {
  // the child shares the parent's open file description (and so its slot lock): give it its own slot
  if (g_map) ::munmap(g_map, sizeof(LedgerFile));
  if (g_fd >= 0) ::close(g_fd);
  g_map = nullptr;
  g_fd = -1;
  g_slot = -1;
  g_allocs.clear();
  g_local_used = 0;
  new (&g_mu) std::mutex();
}

// ------------------------------------------------------------------ pool / agent classification
bool is_gpu_pool(hsa_amd_memory_pool_t pool) {
  static std::mutex& mu = *new std::mutex;
  static std::unordered_map<uint64_t, bool>& cache = *new std::unordered_map<uint64_t, bool>;
  {
    std::lock_guard<std::mutex> l(mu);
    auto it = cache.find(pool.handle);
    if (it != cache.end()) return it->second;
  }
  hsa_amd_segment_t seg = HSA_AMD_SEGMENT_GLOBAL;
  hsa_amd_memory_pool_location_t loc = HSA_AMD_MEMORY_POOL_LOCATION_CPU;
  bool gpu = real_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) == HSA_STATUS_SUCCESS &&
             seg == HSA_AMD_SEGMENT_GLOBAL &&
             real_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_LOCATION, &loc) == HSA_STATUS_SUCCESS &&
             loc == HSA_AMD_MEMORY_POOL_LOCATION_GPU;
  std::lock_guard<std::mutex> l(mu);
  cache[pool.handle] = gpu;
  return gpu;
}

bool is_gpu_agent(hsa_agent_t agent) {
  hsa_device_type_t t = HSA_DEVICE_TYPE_CPU;
  return real_agent_get_info(agent, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_GPU;
}

// ------------------------------------------------------------------ CU partition hooks
void apply_mask(hsa_queue_t* q) {
  if (g_cfg.cu_mask.empty() || q == nullptr) return;
  hsa_status_t s = real_cu_set_mask(q, static_cast<uint32_t>(32 * g_cfg.cu_mask.size()), g_cfg.cu_mask.data());
  if (s == HSA_STATUS_SUCCESS || static_cast<int>(s) == static_cast<int>(HSA_STATUS_CU_MASK_REDUCED)) g_stats_masked++;
}

hsa_status_t hook_queue_create(hsa_agent_t agent, uint32_t size, hsa_queue_type32_t type,
                               void (*cb)(hsa_status_t, hsa_queue_t*, void*), void* data, uint32_t priv,
                               uint32_t group, hsa_queue_t** queue) {
  hsa_status_t s = real_queue_create(agent, size, type, cb, data, priv, group, queue);
  if (s == HSA_STATUS_SUCCESS && queue) {
    g_stats_queues++;
    apply_mask(*queue);
  }
  return s;
}

hsa_status_t hook_intercept_create(hsa_agent_t agent, uint32_t size, hsa_queue_type32_t type,
                                   void (*cb)(hsa_status_t, hsa_queue_t*, void*), void* data, uint32_t priv,
                                   uint32_t group, hsa_queue_t** queue) {
  hsa_status_t s = real_intercept_create(agent, size, type, cb, data, priv, group, queue);
  if (s == HSA_STATUS_SUCCESS && queue) {
    g_stats_queues++;
    apply_mask(*queue);
  }
  return s;
}

hsa_status_t hook_cu_set_mask(const hsa_queue_t* q, uint32_t nbits, const uint32_t* mask) {
  if (g_cfg.cu_mask.empty()) return real_cu_set_mask(q, nbits, mask);
  // the queue may narrow its partition, never leave it: AND with the pod's mask ("0 bits" = all CUs = the pod's)
  std::vector<uint32_t> m(g_cfg.cu_mask);
  bool reduced = false;
  if (nbits != 0 && mask != nullptr) {
    size_t words = (nbits + 31) / 32;
    bool any = false;
    for (size_t i = 0; i < m.size(); ++i) {
      uint32_t w = i < words ? mask[i] : 0u;
      if (i + 1 == words && nbits % 32) w &= (1u << (nbits % 32)) - 1u;
      reduced = reduced || (w & ~m[i]) != 0;
      m[i] &= w;
      any = any || m[i] != 0;
    }
    if (!any) m = g_cfg.cu_mask;  // nothing of the request lies in the partition: keep the partition
  }
  hsa_status_t s = real_cu_set_mask(q, static_cast<uint32_t>(32 * m.size()), m.data());
  g_stats_masked++;
  if (reduced) g_stats_reduced++;
  // a request that reached outside the partition is honoured only inside it, silently (as under MPS): HIP
  // treats any status but SUCCESS from this call as a failed stream creation
  return static_cast<int>(s) == static_cast<int>(HSA_STATUS_CU_MASK_REDUCED) ? HSA_STATUS_SUCCESS : s;
}

// ------------------------------------------------------------------ HBM share hooks
hsa_status_t hook_pool_allocate(hsa_amd_memory_pool_t pool, size_t size, uint32_t flags, void** ptr) {
  if (g_cfg.hbm_limit == 0 || !is_gpu_pool(pool)) return real_pool_allocate(pool, size, flags, ptr);
  std::lock_guard<std::mutex> l(g_mu);
  ledger_open();
  LedgerGuard lg;
  uint64_t used = pod_used_locked();
  if (used + size > g_cfg.hbm_limit) {
    g_stats_denied++;
    GSX_LOG("denied %zu bytes (pod holds %llu of %llu)", size, static_cast<unsigned long long>(used),
            static_cast<unsigned long long>(g_cfg.hbm_limit));
    return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  }
  hsa_status_t s = real_pool_allocate(pool, size, flags, ptr);
  if (s == HSA_STATUS_SUCCESS && ptr && *ptr) {
    g_allocs[reinterpret_cast<uintptr_t>(*ptr)] = size;
    g_local_used += size;
    if (g_map) g_map->bytes[g_slot] = g_local_used;
  }
  return s;
}

hsa_status_t hook_pool_free(void* ptr) {
  if (g_cfg.hbm_limit != 0 && ptr) {
    std::lock_guard<std::mutex> l(g_mu);
    auto it = g_allocs.find(reinterpret_cast<uintptr_t>(ptr));
    if (it != g_allocs.end()) {
      LedgerGuard lg;
      g_local_used -= it->second;
      if (g_map) g_map->bytes[g_slot] = g_local_used;
      g_allocs.erase(it);
    }
  }
  return real_pool_free(ptr);
}

hsa_status_t hook_vmem_create(hsa_amd_memory_pool_t pool, size_t size, hsa_amd_memory_type_t type, uint64_t flags,
                              hsa_amd_vmem_alloc_handle_t* handle) {
  if (g_cfg.hbm_limit == 0 || !is_gpu_pool(pool)) return real_vmem_create(pool, size, type, flags, handle);
  std::lock_guard<std::mutex> l(g_mu);
  ledger_open();
  LedgerGuard lg;
  if (pod_used_locked() + size > g_cfg.hbm_limit) {
    g_stats_denied++;
    return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  }
  hsa_status_t s = real_vmem_create(pool, size, type, flags, handle);
  if (s == HSA_STATUS_SUCCESS && handle) {
    g_allocs[static_cast<uintptr_t>(handle->handle) | (uintptr_t{1} << 63)] = size;
    g_local_used += size;
    if (g_map) g_map->bytes[g_slot] = g_local_used;
  }
  return s;
}

hsa_status_t hook_vmem_release(hsa_amd_vmem_alloc_handle_t handle) {
  hsa_status_t s = real_vmem_release(handle);
  if (g_cfg.hbm_limit != 0 && s == HSA_STATUS_SUCCESS) {
    std::lock_guard<std::mutex> l(g_mu);
    auto it = g_allocs.find(static_cast<uintptr_t>(handle.handle) | (uintptr_t{1} << 63));
    if (it != g_allocs.end()) {
      LedgerGuard lg;
      g_local_used -= it->second;
      if (g_map) g_map->bytes[g_slot] = g_local_used;
      g_allocs.erase(it);
    }
  }
  return s;
}

// the device looks the size of the share: pool size / max allocation clamp to it, available = share - pod's use
hsa_status_t hook_pool_get_info(hsa_amd_memory_pool_t pool, hsa_amd_memory_pool_info_t attr, void* value) {
  hsa_status_t s = real_pool_get_info(pool, attr, value);
  if (s != HSA_STATUS_SUCCESS || g_cfg.hbm_limit == 0 || value == nullptr) return s;
  if ((attr == HSA_AMD_MEMORY_POOL_INFO_SIZE || attr == HSA_AMD_MEMORY_POOL_INFO_ALLOC_MAX_SIZE) && is_gpu_pool(pool)) {
    size_t* v = static_cast<size_t*>(value);
    if (*v > g_cfg.hbm_limit) *v = static_cast<size_t>(g_cfg.hbm_limit);
  }
  return s;
}

hsa_status_t hook_agent_get_info(hsa_agent_t agent, hsa_agent_info_t attr, void* value) {
  hsa_status_t s = real_agent_get_info(agent, attr, value);
  if (s != HSA_STATUS_SUCCESS || g_cfg.hbm_limit == 0 || value == nullptr) return s;
  if (static_cast<int>(attr) == static_cast<int>(HSA_AMD_AGENT_INFO_MEMORY_AVAIL) && is_gpu_agent(agent)) {
    uint64_t used;
    {
      std::lock_guard<std::mutex> l(g_mu);
      ledger_open();
      LedgerGuard lg;
      used = pod_used_locked();
    }
    uint64_t room = used >= g_cfg.hbm_limit ? 0 : g_cfg.hbm_limit - used;
    uint64_t* v = static_cast<uint64_t*>(value);
    if (*v > room) *v = room;
  }
  return s;
}

template <typename Table, typename Fn>
bool has_field(const Table* t, Fn Table::*field) {
  // ApiTableVersion.minor_id is the table's size as the runtime built it: an older runtime's table may end
  // before a field this library was compiled against
  return t != nullptr && reinterpret_cast<const char*>(&(t->*field)) + sizeof(Fn) <=
                             reinterpret_cast<const char*>(t) + t->version.minor_id;
}

void crash_report(int sig) {
  // debugging aid (GSX_ISOLATION_VERBOSE): where did a process under this library fault?
  void* frames[64];
  int n = backtrace(frames, 64);
  char msg[64];
  int m = std::snprintf(msg, sizeof msg, "gsx-isolate[%d]: signal %d\n", static_cast<int>(getpid()), sig);
  if (m > 0) (void)!::write(2, msg, static_cast<size_t>(m));
  backtrace_symbols_fd(frames, n, 2);
  ::signal(sig, SIG_DFL);
  ::raise(sig);
}

std::string self_path() {
  Dl_info info;
  if (dladdr(reinterpret_cast<void*>(&self_path), &info) && info.dli_fname) return info.dli_fname;
  return "";
}

}  // namespace

// ------------------------------------------------------------------ HSA tools-library entry points
GSX_EXPORT bool OnLoad(HsaApiTable* table, uint64_t runtime_version, uint64_t failed_tool_count,
                       const char* const* failed_tool_names) {
  if (std::getenv("GSX_ISOLATION_VERBOSE")) {
    g_cfg.verbose = true;
    ::signal(SIGSEGV, crash_report);
    ::signal(SIGBUS, crash_report);
    GSX_LOG("OnLoad(runtime %llu, failed tools %llu): core table %u bytes, amd_ext %u bytes (ours %zu / %zu)",
            static_cast<unsigned long long>(runtime_version), static_cast<unsigned long long>(failed_tool_count),
            table && table->core_ ? table->core_->version.minor_id : 0u,
            table && table->amd_ext_ ? table->amd_ext_->version.minor_id : 0u, sizeof(CoreApiTable),
            sizeof(AmdExtTable));
  }
  const char* path = config_path();
  if (!path || !parse_config(path, &g_cfg)) {
    if (path) std::fprintf(stderr, "gsx-isolate: cannot read %s; not isolating\n", path);
    return true;  // nothing to enforce: stay loaded and inert
  }
  if (std::getenv("GSX_ISOLATION_VERBOSE")) g_cfg.verbose = true;
  if (table == nullptr || table->core_ == nullptr || table->amd_ext_ == nullptr) return false;
  CoreApiTable* core = table->core_;
  AmdExtTable* amd = table->amd_ext_;
  if (!has_field(core, &CoreApiTable::hsa_queue_create_fn) || !has_field(core, &CoreApiTable::hsa_agent_get_info_fn) ||
      !has_field(amd, &AmdExtTable::hsa_amd_queue_cu_set_mask_fn) ||
      !has_field(amd, &AmdExtTable::hsa_amd_memory_pool_free_fn)) {
    std::fprintf(stderr, "gsx-isolate: HSA API table too old; refusing to run unconfined\n");
    return false;
  }
  real_queue_create = core->hsa_queue_create_fn;
  real_agent_get_info = core->hsa_agent_get_info_fn;
  real_cu_set_mask = amd->hsa_amd_queue_cu_set_mask_fn;
  real_pool_get_info = amd->hsa_amd_memory_pool_get_info_fn;
  real_pool_allocate = amd->hsa_amd_memory_pool_allocate_fn;
  real_pool_free = amd->hsa_amd_memory_pool_free_fn;
  core->hsa_queue_create_fn = hook_queue_create;
  core->hsa_agent_get_info_fn = hook_agent_get_info;
  amd->hsa_amd_queue_cu_set_mask_fn = hook_cu_set_mask;
  amd->hsa_amd_memory_pool_get_info_fn = hook_pool_get_info;
  amd->hsa_amd_memory_pool_allocate_fn = hook_pool_allocate;
  amd->hsa_amd_memory_pool_free_fn = hook_pool_free;
  if (has_field(amd, &AmdExtTable::hsa_amd_queue_intercept_create_fn)) {
    real_intercept_create = amd->hsa_amd_queue_intercept_create_fn;
    amd->hsa_amd_queue_intercept_create_fn = hook_intercept_create;
  }
  if (has_field(amd, &AmdExtTable::hsa_amd_vmem_handle_release_fn)) {
    real_vmem_create = amd->hsa_amd_vmem_handle_create_fn;
    real_vmem_release = amd->hsa_amd_vmem_handle_release_fn;
    amd->hsa_amd_vmem_handle_create_fn = hook_vmem_create;
    amd->hsa_amd_vmem_handle_release_fn = hook_vmem_release;
  }
  pthread_atfork(nullptr, nullptr, after_fork_child);
  int cus = 0;
  for (uint32_t w : g_cfg.cu_mask) cus += __builtin_popcount(w);
  GSX_LOG("%s: %d CUs, hbm_limit %llu bytes", g_cfg.source.c_str(), cus,
          static_cast<unsigned long long>(g_cfg.hbm_limit));
  return true;
}

GSX_EXPORT void OnUnload() {}

// counters for tests and for the workload's self-report: queues created, mask applications, allocations
// denied, this process's device bytes, mask requests narrowed to the partition
GSX_EXPORT void gsx_isolate_stats(uint64_t out[5]) {
  out[0] = g_stats_queues.load();
  out[1] = g_stats_masked.load();
  out[2] = g_stats_denied.load();
  out[4] = g_stats_reduced.load();
  std::lock_guard<std::mutex> l(g_mu);
  out[3] = g_local_used;
}

// loaded by /etc/ld.so.preload or LD_PRELOAD: make sure ROCr loads us as a tools library (before any hsa_init)
__attribute__((constructor)) static void gsx_isolate_preload() {
  if (!config_path()) return;
  std::string me = self_path();
  if (me.empty()) return;
  const char* cur = std::getenv("HSA_TOOLS_LIB");
  std::string v = cur ? cur : "";
  if (v.find(me) != std::string::npos) return;
  v = v.empty() ? me : me + " " + v;
  ::setenv("HSA_TOOLS_LIB", v.c_str(), 1);
}
