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
//    hipMemGetInfo / torch.cuda.mem_get_info / the PyTorch caching allocator see a device of the pod's size;
//  * scratch (private memory), which ROCr allocates behind every allocation API: when a code object is loaded
//    (hsa_executable_freeze) each kernel's worst case is computed (private bytes per lane, 256-byte granules, x
//    wavefront size x waves per CU x CUs, at most the agent's SCRATCH_LIMIT_MAX) and the process's charge is
//    raised to the largest one, reserved against the share like an allocation; the agent's async scratch limit
//    (the scratch ROCr keeps assigned to queues) is set to that charge.  A code object whose kernel cannot fit is
//    refused (HSA_STATUS_ERROR_OUT_OF_RESOURCES: hipModuleLoad / the launch fails) instead of running over the
//    share.  Scratch is per queue (ROCr gives each hardware queue its own), so the charge is the worst kernel's
//    scratch times the live queues the process created: a queue whose share no longer fits is refused at creation
//    (hipStreamCreate fails cleanly), a code object that would overflow it on every queue at load.
//
// Configuration is a root-written file the plugin mounts read-only: /run/gsx/isolation.conf (a container cannot
// edit or hide it).  Only when that path does not exist is $GSX_ISOLATION_CONFIG consulted (tests, host runs).
//     cu_mask=0x000000ff,0x00000000,...   (32-bit words, CU c = bit c%32 of word c/32; GSX_CU_MASK format)
//     hbm_limit_bytes=68719476736
//     ledger=/run/gsx/hbm.ledger
// Loaded through /etc/ld.so.preload (mounted by the plugin), the constructor below adds the library to
// HSA_TOOLS_LIB before the program's first HIP call, and the library's own hsa_init (which precedes the runtime's
// in the global symbol scope) puts it back right before the runtime reads it: a process that unsets or rewrites
// HSA_TOOLS_LIB itself before its first HIP call is still confined.
// Copies: device->device copies are HIP's blit kernels on the stream's (masked) queue, host<->device copies run on
// the SDMA engines (profiles/r04_blit/); a process asking for HSA_ENABLE_SDMA=0 (ROCr's own blit queues, unhooked)
// gets it turned back on when the library is preloaded.
// Not covered: statically linked programs, and processes that drive /dev/kfd ioctls directly.  It confines
// programs, not adversaries (like MPS): a process can rewrite its own pod's ledger file.
//
// Portability: the library is loaded into whatever userland the container image has, and a preload that fails to
// load is skipped by ld.so with only a warning.  So it needs nothing but libc: no C++ runtime (plain data, pthread
// mutexes, its own hash table; built with -fno-exceptions -fno-rtti and linked without libstdc++) and no glibc
// symbol newer than 2.14 (stat/fstat@2.33 and dladdr@2.34 are avoided).  tests/test_isolation.py checks both.
#include <elf.h>
#include <errno.h>
#include <link.h>
#include <execinfo.h>
#include <fcntl.h>
#include <hsa/hsa.h>
#include <hsa/hsa_api_trace.h>
#include <hsa/hsa_ext_amd.h>
#include <pthread.h>
#include <signal.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>

#define GSX_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

const char kFixedConfig[] = "/run/gsx/isolation.conf";
constexpr uint64_t kMagic = 0x31304d4248585347ull;  // "GSXHBM01"
constexpr int kSlots = 256;
constexpr int kMaxMaskWords = 64;  // 2048 CUs

struct LedgerFile {
  uint64_t magic;
  uint64_t reserved[7];          // 64-byte header; byte 0 is the ledger's mutex (an OFD write lock)
  uint64_t bytes[kSlots];        // slot i = device bytes held by the process that holds the lock on byte 64+i
};

// Plain data only: no constructors or destructors run for process state (HIP's own static destructors, which
// run after ours, still free device memory through the hooks at exit), and no C++ runtime library is needed.
struct Config {
  uint32_t cu_mask[kMaxMaskWords];
  int cu_words;                   // 0: no CU partition
  uint64_t hbm_limit;             // 0: no cap
  char ledger[1024];              // "": per-process account
  char source[1024];
  bool verbose;
};

Config g_cfg;
pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;  // process-local half of the ledger lock (OFD locks do not
                                                    // exclude threads of one process)
uint64_t g_local_used = 0;        // this process's device bytes (the ledger slot mirrors it)
int g_fd = -1;
LedgerFile* g_map = nullptr;
int g_slot = -1;
uint64_t g_stats_queues = 0, g_stats_masked = 0, g_stats_denied = 0, g_stats_reduced = 0;  // __atomic ops
uint64_t g_scratch_charged = 0;   // this process's scratch reservation, part of g_local_used (g_mu)
uint64_t g_scratch_refused = 0;   // code objects refused for their scratch (__atomic)
uint64_t g_scratch_limit = 0;     // the async scratch limit last set on the agent (0: never)
// Scratch is per queue: ROCr gives each hardware queue its own scratch, so N queues running the worst loaded kernel
// at the same instant hold N times its scratch.  The charge is the worst kernel's scratch times the live queues this
// process created (at least one): a queue whose share of it no longer fits is refused, as is a code object that
// raises the worst past what the share has left for every queue (g_mu)
uint64_t g_scratch_worst = 0;     // the worst loaded kernel's scratch for one queue
// live queues created through the hooks, counted from the moment their creation is charged (charge_queue) so that
// two creations at once each see the other; at most kMaxTracked, each one then tracked in g_queues
uint64_t g_scratch_queues = 0;
uint64_t g_scratch_queue_refused = 0;  // queues refused for their scratch
constexpr int kMaxTracked = 1024;
hsa_queue_t* g_queues[kMaxTracked];  // the live queues counted in g_scratch_queues
int g_nqueues_tracked = 0;

// the runtime's own entry points, saved by OnLoad
decltype(hsa_queue_create)* real_queue_create = nullptr;
decltype(hsa_queue_destroy)* real_queue_destroy = nullptr;
decltype(hsa_agent_get_info)* real_agent_get_info = nullptr;
decltype(hsa_amd_queue_cu_set_mask)* real_cu_set_mask = nullptr;
decltype(hsa_amd_queue_intercept_create)* real_intercept_create = nullptr;
decltype(hsa_amd_memory_pool_get_info)* real_pool_get_info = nullptr;
decltype(hsa_amd_memory_pool_allocate)* real_pool_allocate = nullptr;
decltype(hsa_amd_memory_pool_free)* real_pool_free = nullptr;
decltype(hsa_amd_vmem_handle_create)* real_vmem_create = nullptr;
decltype(hsa_amd_vmem_handle_release)* real_vmem_release = nullptr;
decltype(hsa_executable_freeze)* real_freeze = nullptr;
decltype(hsa_executable_iterate_symbols)* real_iterate_symbols = nullptr;
decltype(hsa_executable_symbol_get_info)* real_symbol_get_info = nullptr;
decltype(hsa_amd_agent_set_async_scratch_limit)* real_set_scratch_limit = nullptr;

#define GSX_LOG(...)                                                   \
  do {                                                                 \
    if (g_cfg.verbose) {                                               \
      fprintf(stderr, "gsx-isolate[%d]: ", static_cast<int>(getpid())); \
      fprintf(stderr, __VA_ARGS__);                                    \
      fputc('\n', stderr);                                             \
    }                                                                  \
  } while (0)

void bump(uint64_t* c) { __atomic_fetch_add(c, 1, __ATOMIC_RELAXED); }

struct Lock {  // scoped pthread mutex
  pthread_mutex_t* m;
  explicit Lock(pthread_mutex_t* mu) : m(mu) { pthread_mutex_lock(m); }
  ~Lock() { pthread_mutex_unlock(m); }
};

// ------------------------------------------------------------------ live allocations (ptr / handle -> bytes)
// open addressing, linear probing; key 0 = empty, 1 = tombstone (pointers and tagged handles are neither)
struct Entry {
  uintptr_t key;
  uint64_t bytes;
};
Entry* g_tab = nullptr;
size_t g_cap = 0, g_fill = 0;  // g_fill: live entries + tombstones

size_t hash_key(uintptr_t k) {
  uint64_t x = k;
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  return static_cast<size_t>(x);
}

void tab_insert_raw(Entry* tab, size_t cap, uintptr_t k, uint64_t v) {
  for (size_t i = hash_key(k) & (cap - 1);; i = (i + 1) & (cap - 1)) {
    if (tab[i].key == 0) {
      tab[i].key = k;
      tab[i].bytes = v;
      return;
    }
  }
}

bool tab_put(uintptr_t k, uint64_t v) {  // g_mu held
  if ((g_fill + 1) * 4 >= g_cap * 3) {
    size_t live = 0;
    for (size_t i = 0; i < g_cap; ++i) live += g_tab[i].key > 1;
    size_t cap = 1024;
    while ((live + 1) * 2 >= cap) cap *= 2;
    Entry* t = static_cast<Entry*>(calloc(cap, sizeof(Entry)));
    if (!t) return false;
    for (size_t i = 0; i < g_cap; ++i) {
      if (g_tab[i].key > 1) tab_insert_raw(t, cap, g_tab[i].key, g_tab[i].bytes);
    }
    free(g_tab);
    g_tab = t;
    g_cap = cap;
    g_fill = live;
  }
  tab_insert_raw(g_tab, g_cap, k, v);
  g_fill++;
  return true;
}

bool tab_take(uintptr_t k, uint64_t* v) {  // g_mu held
  if (g_cap == 0) return false;
  for (size_t i = hash_key(k) & (g_cap - 1);; i = (i + 1) & (g_cap - 1)) {
    if (g_tab[i].key == 0) return false;
    if (g_tab[i].key == k) {
      *v = g_tab[i].bytes;
      g_tab[i].key = 1;
      return true;
    }
  }
}

// ------------------------------------------------------------------ configuration
char* trim(char* s) {
  while (*s == ' ' || *s == '\t') ++s;
  char* e = s + strlen(s);
  while (e > s && (e[-1] == ' ' || e[-1] == '\t' || e[-1] == '\r' || e[-1] == '\n')) *--e = 0;
  return s;
}

bool parse_config(const char* path, Config* out) {
  FILE* f = fopen(path, "r");
  if (!f) return false;
  char line[4096];
  while (fgets(line, sizeof line, f)) {
    char* l = trim(line);
    if (!*l || *l == '#') continue;
    char* eq = strchr(l, '=');
    if (!eq) continue;
    *eq = 0;
    char* k = trim(l);
    char* v = trim(eq + 1);
    if (!strcmp(k, "cu_mask")) {
      out->cu_words = 0;
      for (char* p = v; *p && out->cu_words < kMaxMaskWords;) {
        char* end = nullptr;
        unsigned long w = strtoul(p, &end, 16);
        if (end == p) break;
        out->cu_mask[out->cu_words++] = static_cast<uint32_t>(w);
        p = end;
        while (*p == ',' || *p == ' ') ++p;
      }
    } else if (!strcmp(k, "hbm_limit_bytes")) {
      out->hbm_limit = strtoull(v, nullptr, 10);
    } else if (!strcmp(k, "ledger")) {
      snprintf(out->ledger, sizeof out->ledger, "%s", v);
    } else if (!strcmp(k, "verbose")) {
      out->verbose = !strcmp(v, "1") || !strcmp(v, "true");
    }
  }
  fclose(f);
  bool any = false;
  for (int i = 0; i < out->cu_words; ++i) any = any || out->cu_mask[i] != 0;
  if (!any) out->cu_words = 0;  // an all-zero mask would stop every queue: treat it as "no partition"
  snprintf(out->source, sizeof out->source, "%s", path);
  return true;
}

const char* config_path() {
  if (access(kFixedConfig, F_OK) == 0) return kFixedConfig;
  const char* e = getenv("GSX_ISOLATION_CONFIG");
  return e && *e ? e : nullptr;
}

// ------------------------------------------------------------------ shared per-pod HBM ledger
int ofd_lock(int fd, short type, off_t off, bool wait) {
  struct flock fl;
  memset(&fl, 0, sizeof fl);
  fl.l_type = type;
  fl.l_whence = SEEK_SET;
  fl.l_start = off;
  fl.l_len = 1;
  int r;
  do {
    r = fcntl(fd, wait ? F_OFD_SETLKW : F_OFD_SETLK, &fl);
  } while (r != 0 && errno == EINTR);
  return r;
}

bool slot_alive(int fd, int i) {
  struct flock fl;
  memset(&fl, 0, sizeof fl);
  fl.l_type = F_WRLCK;
  fl.l_whence = SEEK_SET;
  fl.l_start = static_cast<off_t>(offsetof(LedgerFile, bytes) + i);
  fl.l_len = 1;
  if (fcntl(fd, F_OFD_GETLK, &fl) != 0) return false;
  return fl.l_type != F_UNLCK;  // another open file description holds the slot: its process is alive
}

// open + map the ledger and claim a free slot (caller holds g_mu); false: fall back to a per-process account
bool ledger_open() {
  if (g_map) return true;
  if (!g_cfg.ledger[0]) return false;
  int fd = open(g_cfg.ledger, O_RDWR | O_CREAT | O_CLOEXEC, 0666);
  if (fd < 0) return false;
  if (ofd_lock(fd, F_WRLCK, 0, true) != 0) {
    close(fd);
    return false;
  }
  off_t size = lseek(fd, 0, SEEK_END);
  if (size < 0 || (size < static_cast<off_t>(sizeof(LedgerFile)) && ftruncate(fd, sizeof(LedgerFile)) != 0)) {
    ofd_lock(fd, F_UNLCK, 0, false);
    close(fd);
    return false;
  }
  void* p = mmap(nullptr, sizeof(LedgerFile), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (p == MAP_FAILED) {
    ofd_lock(fd, F_UNLCK, 0, false);
    close(fd);
    return false;
  }
  auto* m = static_cast<LedgerFile*>(p);
  if (m->magic != kMagic) {
    memset(m, 0, sizeof(LedgerFile));
    m->magic = kMagic;
  }
  int slot = -1;
  for (int i = 0; i < kSlots && slot < 0; ++i) {
    if (slot_alive(fd, i)) continue;
    if (ofd_lock(fd, F_WRLCK, static_cast<off_t>(offsetof(LedgerFile, bytes) + i), false) == 0) slot = i;
  }
  if (slot < 0) {
    ofd_lock(fd, F_UNLCK, 0, false);
    munmap(p, sizeof(LedgerFile));
    close(fd);
    return false;
  }
  m->bytes[slot] = g_local_used;  // a dead owner's count is dropped with its slot
  ofd_lock(fd, F_UNLCK, 0, false);
  g_fd = fd;
  g_map = m;
  g_slot = slot;
  GSX_LOG("ledger %s slot %d", g_cfg.ledger, slot);
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

void publish_locked() {
  if (g_map) g_map->bytes[g_slot] = g_local_used;
}

void after_fork_child() {
  // the child shares the parent's open file description (and so its slot lock): give it its own slot; the
  // parent's device allocations are not the child's
  if (g_map) munmap(g_map, sizeof(LedgerFile));
  if (g_fd >= 0) close(g_fd);
  g_map = nullptr;
  g_fd = -1;
  g_slot = -1;
  if (g_tab) memset(g_tab, 0, g_cap * sizeof(Entry));
  g_fill = 0;
  g_local_used = 0;
  g_scratch_charged = 0;  // the parent's loaded code objects are not the child's charge
  g_scratch_worst = 0;
  g_scratch_queues = 0;
  g_nqueues_tracked = 0;
  pthread_mutex_t fresh = PTHREAD_MUTEX_INITIALIZER;
  g_mu = fresh;
}

// ------------------------------------------------------------------ pool / agent classification
struct PoolKind {
  uint64_t handle;
  bool gpu;
};
PoolKind g_pools[256];
int g_npools = 0;
pthread_mutex_t g_pool_mu = PTHREAD_MUTEX_INITIALIZER;

bool is_gpu_pool(hsa_amd_memory_pool_t pool) {
  {
    Lock l(&g_pool_mu);
    for (int i = 0; i < g_npools; ++i) {
      if (g_pools[i].handle == pool.handle) return g_pools[i].gpu;
    }
  }
  hsa_amd_segment_t seg = HSA_AMD_SEGMENT_GLOBAL;
  hsa_amd_memory_pool_location_t loc = HSA_AMD_MEMORY_POOL_LOCATION_CPU;
  bool gpu = real_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) == HSA_STATUS_SUCCESS &&
             seg == HSA_AMD_SEGMENT_GLOBAL &&
             real_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_LOCATION, &loc) == HSA_STATUS_SUCCESS &&
             loc == HSA_AMD_MEMORY_POOL_LOCATION_GPU;
  Lock l(&g_pool_mu);
  if (g_npools < static_cast<int>(sizeof g_pools / sizeof g_pools[0])) g_pools[g_npools++] = PoolKind{pool.handle, gpu};
  return gpu;
}

bool is_gpu_agent(hsa_agent_t agent) {
  hsa_device_type_t t = HSA_DEVICE_TYPE_CPU;
  return real_agent_get_info(agent, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_GPU;
}

// ------------------------------------------------------------------ CU partition hooks
void apply_mask(hsa_queue_t* q) {
  if (g_cfg.cu_words == 0 || q == nullptr) return;
  hsa_status_t s = real_cu_set_mask(q, static_cast<uint32_t>(32 * g_cfg.cu_words), g_cfg.cu_mask);
  if (s == HSA_STATUS_SUCCESS || static_cast<int>(s) == static_cast<int>(HSA_STATUS_CU_MASK_REDUCED)) {
    bump(&g_stats_masked);
  }
}

bool reserve_locked(uint64_t size);
void unreserve_locked(uint64_t size);

// A new queue's share of the scratch charge (the worst loaded kernel's scratch, for every queue past the first):
// reserved before the queue exists, and the queue counted in the same step (a second creation racing this one sees
// it and pays its own share); false = refused (the share has no room for another queue's scratch, or the process
// already has kMaxTracked live queues -- one this library could not track would never give its charge back).
// *counted: queue_created() must settle the count (keep it, or roll it back if the runtime fails the creation)
bool charge_queue(uint64_t* extra, bool* counted) {
  *extra = 0;
  *counted = false;
  if (g_cfg.hbm_limit == 0) return true;
  Lock l(&g_mu);
  if (g_scratch_queues >= static_cast<uint64_t>(kMaxTracked)) {
    g_scratch_queue_refused++;
    fprintf(stderr, "gsx-isolate: %d live queues, the most this library tracks; refusing to create another\n",
            kMaxTracked);
    return false;
  }
  if (g_scratch_worst != 0 && g_scratch_queues != 0) {  // the first queue's scratch is already charged
    if (!reserve_locked(g_scratch_worst)) {
      g_scratch_queue_refused++;
      fprintf(stderr,
              "gsx-isolate: another queue can need %llu bytes of scratch for the kernels loaded, more than the pod's "
              "share has left; refusing to create it\n",
              static_cast<unsigned long long>(g_scratch_worst));
      return false;
    }
    g_scratch_charged += g_scratch_worst;
    *extra = g_scratch_worst;
  }
  g_scratch_queues++;
  *counted = true;
  return true;
}

void queue_created(hsa_queue_t* q, uint64_t extra, bool counted, bool ok) {
  if (!counted) return;
  Lock l(&g_mu);
  if (!ok) {  // the runtime did not create it: the count and the share charged for it go back
    g_scratch_queues--;
    if (extra) {
      unreserve_locked(extra);
      g_scratch_charged -= extra;
    }
    return;
  }
  g_queues[g_nqueues_tracked++] = q;  // room: g_nqueues_tracked <= g_scratch_queues <= kMaxTracked
}

hsa_status_t hook_queue_create(hsa_agent_t agent, uint32_t size, hsa_queue_type32_t type,
                               void (*cb)(hsa_status_t, hsa_queue_t*, void*), void* data, uint32_t priv,
                               uint32_t group, hsa_queue_t** queue) {
  uint64_t extra;
  bool counted;
  if (!charge_queue(&extra, &counted)) return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  hsa_status_t s = real_queue_create(agent, size, type, cb, data, priv, group, queue);
  const bool ok = s == HSA_STATUS_SUCCESS && queue;
  queue_created(ok ? *queue : nullptr, extra, counted, ok);
  if (ok) {
    bump(&g_stats_queues);
    apply_mask(*queue);
  }
  return s;
}

hsa_status_t hook_intercept_create(hsa_agent_t agent, uint32_t size, hsa_queue_type32_t type,
                                   void (*cb)(hsa_status_t, hsa_queue_t*, void*), void* data, uint32_t priv,
                                   uint32_t group, hsa_queue_t** queue) {
  uint64_t extra;
  bool counted;
  if (!charge_queue(&extra, &counted)) return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  hsa_status_t s = real_intercept_create(agent, size, type, cb, data, priv, group, queue);
  const bool ok = s == HSA_STATUS_SUCCESS && queue;
  queue_created(ok ? *queue : nullptr, extra, counted, ok);
  if (ok) {
    bump(&g_stats_queues);
    apply_mask(*queue);
  }
  return s;
}

// a queue this library counted goes: its share of the scratch charge is released
hsa_status_t hook_queue_destroy(hsa_queue_t* q) {
  hsa_status_t s = real_queue_destroy(q);
  if (s != HSA_STATUS_SUCCESS || g_cfg.hbm_limit == 0) return s;
  Lock l(&g_mu);
  for (int i = 0; i < g_nqueues_tracked; ++i) {
    if (g_queues[i] != q) continue;
    g_queues[i] = g_queues[--g_nqueues_tracked];
    const uint64_t before = g_scratch_worst * (g_scratch_queues > 1 ? g_scratch_queues : 1);
    g_scratch_queues--;
    const uint64_t after = g_scratch_worst * (g_scratch_queues > 1 ? g_scratch_queues : 1);
    if (before > after) {
      unreserve_locked(before - after);
      g_scratch_charged -= before - after;
    }
    break;
  }
  return s;
}

hsa_status_t hook_cu_set_mask(const hsa_queue_t* q, uint32_t nbits, const uint32_t* mask) {
  if (g_cfg.cu_words == 0) return real_cu_set_mask(q, nbits, mask);
  // the queue may narrow its partition, never leave it: AND with the pod's mask ("0 bits" = all CUs = the pod's)
  uint32_t m[kMaxMaskWords];
  const int n = g_cfg.cu_words;
  memcpy(m, g_cfg.cu_mask, sizeof(uint32_t) * static_cast<size_t>(n));
  bool reduced = false;
  if (nbits != 0 && mask != nullptr) {
    size_t words = (nbits + 31) / 32;
    bool any = false;
    for (int i = 0; i < n; ++i) {
      uint32_t w = static_cast<size_t>(i) < words ? mask[i] : 0u;
      if (static_cast<size_t>(i) + 1 == words && nbits % 32) w &= (1u << (nbits % 32)) - 1u;
      reduced = reduced || (w & ~m[i]) != 0;
      m[i] &= w;
      any = any || m[i] != 0;
    }
    if (!any) memcpy(m, g_cfg.cu_mask, sizeof(uint32_t) * static_cast<size_t>(n));  // nothing of it lies inside
  }
  hsa_status_t s = real_cu_set_mask(q, static_cast<uint32_t>(32 * n), m);
  bump(&g_stats_masked);
  if (reduced) bump(&g_stats_reduced);
  // a request that reached outside the partition is honoured only inside it, silently (as under MPS): HIP
  // treats any status but SUCCESS from this call as a failed stream creation
  return static_cast<int>(s) == static_cast<int>(HSA_STATUS_CU_MASK_REDUCED) ? HSA_STATUS_SUCCESS : s;
}

// ------------------------------------------------------------------ HBM share hooks
constexpr uintptr_t kHandleTag = uintptr_t{1} << 63;  // vmem handles and pointers share the table

// Reserve `size` bytes of the pod's share if they fit (g_mu held): the check and the reservation happen under
// the cross-process ledger lock in one step, so two processes of one pod can never both pass the check for the
// last bytes of the share and then both allocate.  false = over the share (nothing reserved).
bool reserve_locked(uint64_t size) {
  ledger_open();
  LedgerGuard lg;
  uint64_t used = pod_used_locked();
  if (used + size > g_cfg.hbm_limit) {
    bump(&g_stats_denied);
    GSX_LOG("denied %llu bytes (pod holds %llu of %llu)", static_cast<unsigned long long>(size),
            static_cast<unsigned long long>(used), static_cast<unsigned long long>(g_cfg.hbm_limit));
    return false;
  }
  g_local_used += size;
  publish_locked();
  return true;
}

// the reserved bytes were not allocated after all (g_mu held)
void unreserve_locked(uint64_t size) {
  LedgerGuard lg;
  g_local_used -= size;
  publish_locked();
}

// the reserved bytes are now the allocation `key` (g_mu held)
void record_locked(uintptr_t key, uint64_t size) {
  if (!tab_put(key, size)) {
    // out of host memory for the table: the bytes cannot be matched to their free; keep them charged
    // (never under-count the share)
    return;
  }
}

void forget_locked(uintptr_t key) {
  uint64_t bytes = 0;
  if (!tab_take(key, &bytes)) return;
  LedgerGuard lg;
  g_local_used -= bytes;
  publish_locked();
}

hsa_status_t hook_pool_allocate(hsa_amd_memory_pool_t pool, size_t size, uint32_t flags, void** ptr) {
  if (g_cfg.hbm_limit == 0 || !is_gpu_pool(pool)) return real_pool_allocate(pool, size, flags, ptr);
  Lock l(&g_mu);
  if (!reserve_locked(size)) return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  hsa_status_t s = real_pool_allocate(pool, size, flags, ptr);
  if (s == HSA_STATUS_SUCCESS && ptr && *ptr) {
    record_locked(reinterpret_cast<uintptr_t>(*ptr), size);
  } else {
    unreserve_locked(size);
  }
  return s;
}

hsa_status_t hook_pool_free(void* ptr) {
  if (g_cfg.hbm_limit != 0 && ptr) {
    Lock l(&g_mu);
    forget_locked(reinterpret_cast<uintptr_t>(ptr));
  }
  return real_pool_free(ptr);
}

hsa_status_t hook_vmem_create(hsa_amd_memory_pool_t pool, size_t size, hsa_amd_memory_type_t type, uint64_t flags,
                              hsa_amd_vmem_alloc_handle_t* handle) {
  if (g_cfg.hbm_limit == 0 || !is_gpu_pool(pool)) return real_vmem_create(pool, size, type, flags, handle);
  Lock l(&g_mu);
  if (!reserve_locked(size)) return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  hsa_status_t s = real_vmem_create(pool, size, type, flags, handle);
  if (s == HSA_STATUS_SUCCESS && handle) {
    record_locked(static_cast<uintptr_t>(handle->handle) | kHandleTag, size);
  } else {
    unreserve_locked(size);
  }
  return s;
}

hsa_status_t hook_vmem_release(hsa_amd_vmem_alloc_handle_t handle) {
  hsa_status_t s = real_vmem_release(handle);
  if (g_cfg.hbm_limit != 0 && s == HSA_STATUS_SUCCESS) {
    Lock l(&g_mu);
    forget_locked(static_cast<uintptr_t>(handle.handle) | kHandleTag);
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
      Lock l(&g_mu);
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

// ------------------------------------------------------------------ scratch (private memory)
constexpr uint64_t kDynamicStackBytes = 1024;  // HIP's default per-lane stack for kernels with a dynamic call stack
constexpr uint64_t kScratchGranule = 256;      // per-lane scratch is allocated in 256-byte granules

// The most scratch one dispatch of a kernel can make ROCr allocate on `agent`: every wave slot of every CU busy.
uint64_t kernel_scratch_worst(hsa_agent_t agent, uint32_t private_bytes, bool dynamic_stack) {
  uint64_t lane = private_bytes + (dynamic_stack ? kDynamicStackBytes : 0);
  if (lane == 0) return 0;
  lane = (lane + kScratchGranule - 1) / kScratchGranule * kScratchGranule;
  uint32_t cus = 0, waves = 0, wave = 64;
  real_agent_get_info(agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_COMPUTE_UNIT_COUNT), &cus);
  real_agent_get_info(agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_MAX_WAVES_PER_CU), &waves);
  real_agent_get_info(agent, HSA_AGENT_INFO_WAVEFRONT_SIZE, &wave);
  uint64_t worst = lane * wave * (waves ? waves : 32) * (cus ? cus : 1);
  uint64_t cap = 0;
  if (real_agent_get_info(agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_SCRATCH_LIMIT_MAX), &cap) ==
          HSA_STATUS_SUCCESS &&
      cap != 0 && worst > cap) {
    worst = cap;  // ROCr runs such a dispatch on fewer waves
  }
  return worst;
}

struct ScratchScan {
  uint64_t worst;
  hsa_agent_t agent;
  bool have_agent;
};

hsa_status_t scan_symbol(hsa_executable_t, hsa_executable_symbol_t sym, void* data) {
  auto* scan = static_cast<ScratchScan*>(data);
  hsa_symbol_kind_t kind = HSA_SYMBOL_KIND_VARIABLE;
  if (real_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_TYPE, &kind) != HSA_STATUS_SUCCESS ||
      kind != HSA_SYMBOL_KIND_KERNEL) {
    return HSA_STATUS_SUCCESS;
  }
  uint32_t priv = 0;
  bool dynamic_stack = false;
  hsa_agent_t agent{};
  real_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &priv);
  real_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_DYNAMIC_CALLSTACK, &dynamic_stack);
  if (real_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_AGENT, &agent) != HSA_STATUS_SUCCESS ||
      !is_gpu_agent(agent)) {
    return HSA_STATUS_SUCCESS;
  }
  uint64_t w = kernel_scratch_worst(agent, priv, dynamic_stack);
  if (w > scan->worst) {
    scan->worst = w;
    scan->agent = agent;
    scan->have_agent = true;
  }
  return HSA_STATUS_SUCCESS;
}

// A loaded code object may raise the process's scratch charge to its worst kernel; one that cannot fit in the
// share is refused (the runtime would otherwise allocate its scratch behind the share's back).
hsa_status_t hook_freeze(hsa_executable_t exe, const char* options) {
  hsa_status_t st = real_freeze(exe, options);
  if (st != HSA_STATUS_SUCCESS || g_cfg.hbm_limit == 0 || !real_iterate_symbols || !real_symbol_get_info) return st;
  ScratchScan scan{0, {}, false};
  real_iterate_symbols(exe, scan_symbol, &scan);
  uint64_t limit = 0;
  {
    Lock l(&g_mu);
    if (scan.worst <= g_scratch_worst) return st;
    // every live queue (at least one) may run the new worst kernel at the same instant
    const uint64_t queues = g_scratch_queues > 1 ? g_scratch_queues : 1;
    const uint64_t extra = (scan.worst - g_scratch_worst) * queues;
    if (!reserve_locked(extra)) {
      __atomic_fetch_add(&g_scratch_refused, 1, __ATOMIC_RELAXED);
      fprintf(stderr,
              "gsx-isolate: a kernel of this code object can need %llu bytes of scratch on each of %llu queue(s), "
              "more than the pod's share has left; refusing to load it\n",
              static_cast<unsigned long long>(scan.worst), static_cast<unsigned long long>(queues));
      return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
    }
    g_scratch_charged += extra;
    g_scratch_worst = scan.worst;
    limit = scan.worst;
  }
  // the scratch ROCr keeps assigned to this agent's queues stays within what is charged; bigger dispatches get
  // use-once scratch (also within the charge: no loaded kernel needs more)
  if (real_set_scratch_limit && scan.have_agent &&
      real_set_scratch_limit(scan.agent, static_cast<size_t>(limit)) == HSA_STATUS_SUCCESS) {
    __atomic_store_n(&g_scratch_limit, limit, __ATOMIC_RELAXED);
  }
  GSX_LOG("scratch charge raised to %llu bytes", static_cast<unsigned long long>(limit));
  return st;
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
  int m = snprintf(msg, sizeof msg, "gsx-isolate[%d]: signal %d\n", static_cast<int>(getpid()), sig);
  if (m > 0) (void)!write(2, msg, static_cast<size_t>(m));
  backtrace_symbols_fd(frames, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

// the mapped file that contains this function (/proc/self/maps: no dladdr, whose symbol version would tie the
// library to the build host's glibc); "" if not found
void self_path(char* out, size_t cap) {
  out[0] = 0;
  uintptr_t me = reinterpret_cast<uintptr_t>(&self_path);
  FILE* f = fopen("/proc/self/maps", "r");
  if (!f) return;
  char line[4096];
  while (fgets(line, sizeof line, f)) {
    unsigned long lo = 0, hi = 0;
    if (sscanf(line, "%lx-%lx", &lo, &hi) != 2 || me < lo || me >= hi) continue;
    const char* path = strchr(line, '/');
    if (path) snprintf(out, cap, "%s", path);
    break;
  }
  fclose(f);
  trim(out);
}

}  // namespace

// ------------------------------------------------------------------ HSA tools-library entry points
GSX_EXPORT bool OnLoad(HsaApiTable* table, uint64_t runtime_version, uint64_t failed_tool_count,
                       const char* const* failed_tool_names) {
  (void)failed_tool_names;
  if (getenv("GSX_ISOLATION_VERBOSE")) {
    g_cfg.verbose = true;
    signal(SIGSEGV, crash_report);
    signal(SIGBUS, crash_report);
    GSX_LOG("OnLoad(runtime %llu, failed tools %llu): core table %u bytes, amd_ext %u bytes (ours %zu / %zu)",
            static_cast<unsigned long long>(runtime_version), static_cast<unsigned long long>(failed_tool_count),
            table && table->core_ ? table->core_->version.minor_id : 0u,
            table && table->amd_ext_ ? table->amd_ext_->version.minor_id : 0u, sizeof(CoreApiTable),
            sizeof(AmdExtTable));
  }
  const char* path = config_path();
  if (!path || !parse_config(path, &g_cfg)) {
    if (path) fprintf(stderr, "gsx-isolate: cannot read %s; not isolating\n", path);
    return true;  // nothing to enforce: stay loaded and inert
  }
  if (getenv("GSX_ISOLATION_VERBOSE")) g_cfg.verbose = true;
  if (table == nullptr || table->core_ == nullptr || table->amd_ext_ == nullptr) return false;
  CoreApiTable* core = table->core_;
  AmdExtTable* amd = table->amd_ext_;
  if (!has_field(core, &CoreApiTable::hsa_queue_create_fn) || !has_field(core, &CoreApiTable::hsa_agent_get_info_fn) ||
      !has_field(amd, &AmdExtTable::hsa_amd_queue_cu_set_mask_fn) ||
      !has_field(amd, &AmdExtTable::hsa_amd_memory_pool_free_fn)) {
    fprintf(stderr, "gsx-isolate: HSA API table too old; refusing to run unconfined\n");
    return false;
  }
  real_queue_create = core->hsa_queue_create_fn;
  real_agent_get_info = core->hsa_agent_get_info_fn;
  if (has_field(core, &CoreApiTable::hsa_queue_destroy_fn)) {
    real_queue_destroy = core->hsa_queue_destroy_fn;
    core->hsa_queue_destroy_fn = hook_queue_destroy;
  }
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
  if (g_cfg.hbm_limit != 0 && has_field(core, &CoreApiTable::hsa_executable_iterate_symbols_fn)) {
    real_freeze = core->hsa_executable_freeze_fn;
    real_iterate_symbols = core->hsa_executable_iterate_symbols_fn;
    real_symbol_get_info = core->hsa_executable_symbol_get_info_fn;
    core->hsa_executable_freeze_fn = hook_freeze;
    if (has_field(amd, &AmdExtTable::hsa_amd_agent_set_async_scratch_limit_fn)) {
      real_set_scratch_limit = amd->hsa_amd_agent_set_async_scratch_limit_fn;
    }
  }
  if (has_field(amd, &AmdExtTable::hsa_amd_vmem_handle_release_fn)) {
    real_vmem_create = amd->hsa_amd_vmem_handle_create_fn;
    real_vmem_release = amd->hsa_amd_vmem_handle_release_fn;
    amd->hsa_amd_vmem_handle_create_fn = hook_vmem_create;
    amd->hsa_amd_vmem_handle_release_fn = hook_vmem_release;
  }
  pthread_atfork(nullptr, nullptr, after_fork_child);
  int cus = 0;
  for (int i = 0; i < g_cfg.cu_words; ++i) cus += __builtin_popcount(g_cfg.cu_mask[i]);
  GSX_LOG("%s: %d CUs, hbm_limit %llu bytes", g_cfg.source, cus, static_cast<unsigned long long>(g_cfg.hbm_limit));
  return true;
}

GSX_EXPORT void OnUnload() {}

// counters for tests and for the workload's self-report: queues created, mask applications, allocations
// denied, this process's device bytes, mask requests narrowed to the partition
// scratch: this process's charge, code objects refused for their scratch, the async scratch limit last set
GSX_EXPORT void gsx_isolate_scratch(uint64_t out[3]) {
  out[1] = __atomic_load_n(&g_scratch_refused, __ATOMIC_RELAXED);
  out[2] = __atomic_load_n(&g_scratch_limit, __ATOMIC_RELAXED);
  Lock l(&g_mu);
  out[0] = g_scratch_charged;
}

// per-queue scratch: the worst loaded kernel's scratch for one queue, live queues counted, queues refused
GSX_EXPORT void gsx_isolate_scratch_queues(uint64_t out[3]) {
  Lock l(&g_mu);
  out[0] = g_scratch_worst;
  out[1] = g_scratch_queues;
  out[2] = g_scratch_queue_refused;
}

GSX_EXPORT void gsx_isolate_stats(uint64_t out[5]) {
  out[0] = __atomic_load_n(&g_stats_queues, __ATOMIC_RELAXED);
  out[1] = __atomic_load_n(&g_stats_masked, __ATOMIC_RELAXED);
  out[2] = __atomic_load_n(&g_stats_denied, __ATOMIC_RELAXED);
  out[4] = __atomic_load_n(&g_stats_reduced, __ATOMIC_RELAXED);
  Lock l(&g_mu);
  out[3] = g_local_used;
}

namespace {

// make sure ROCr loads this library as a tools library: HSA_TOOLS_LIB names it (prepended to whatever else)
void ensure_tools_lib() {
  if (!config_path()) return;
  // with SDMA off ROCr copies host<->device with blit kernels on queues of its own, which no hook sees (so they
  // would run on every CU): keep the copy engines on (only when the runtime has not read its flags yet)
  const char* sdma = getenv("HSA_ENABLE_SDMA");
  if (sdma && !strcmp(sdma, "0")) setenv("HSA_ENABLE_SDMA", "1", 1);
  char me[4096];
  self_path(me, sizeof me);
  if (!me[0]) return;
  const char* cur = getenv("HSA_TOOLS_LIB");
  if (cur && strstr(cur, me)) return;
  size_t n = strlen(me) + (cur ? strlen(cur) + 1 : 0) + 1;
  char* v = static_cast<char*>(malloc(n));
  if (!v) return;
  if (cur && *cur) {
    snprintf(v, n, "%s %s", me, cur);
  } else {
    snprintf(v, n, "%s", me);
  }
  setenv("HSA_TOOLS_LIB", v, 1);
  free(v);
}

// The runtime's own hsa_init, found without libdl (which would tie the library to a newer glibc or add a
// dependency): walk the loaded objects (dl_iterate_phdr, libc) to libhsa-runtime64 and look the symbol up in its
// GNU hash table.
uint32_t gnu_hash(const char* s) {
  uint32_t h = 5381;
  for (; *s; ++s) h = (h << 5) + h + static_cast<uint8_t>(*s);
  return h;
}

struct SymQuery {
  const char* name;
  void* addr;
};

int find_in_hsa_runtime(struct dl_phdr_info* info, size_t, void* data) {
  auto* q = static_cast<SymQuery*>(data);
  if (!info->dlpi_name || !strstr(info->dlpi_name, "libhsa-runtime64")) return 0;
  const ElfW(Addr) base = info->dlpi_addr;
  const ElfW(Dyn)* dyn = nullptr;
  for (int i = 0; i < info->dlpi_phnum; ++i) {
    if (info->dlpi_phdr[i].p_type == PT_DYNAMIC) dyn = reinterpret_cast<const ElfW(Dyn)*>(base + info->dlpi_phdr[i].p_vaddr);
  }
  if (!dyn) return 0;
  const ElfW(Sym)* symtab = nullptr;
  const char* strtab = nullptr;
  const uint32_t* gh = nullptr;
  auto addr = [base](ElfW(Addr) p) { return p < base ? p + base : p; };  // relocated in place by ld.so, or not
  for (; dyn->d_tag != DT_NULL; ++dyn) {
    if (dyn->d_tag == DT_SYMTAB) symtab = reinterpret_cast<const ElfW(Sym)*>(addr(dyn->d_un.d_ptr));
    if (dyn->d_tag == DT_STRTAB) strtab = reinterpret_cast<const char*>(addr(dyn->d_un.d_ptr));
    if (dyn->d_tag == DT_GNU_HASH) gh = reinterpret_cast<const uint32_t*>(addr(dyn->d_un.d_ptr));
  }
  if (!symtab || !strtab || !gh) return 0;
  const uint32_t nbuckets = gh[0], symoffset = gh[1], bloom_size = gh[2];
  if (nbuckets == 0) return 0;
  const uint32_t* buckets = gh + 4 + bloom_size * (sizeof(ElfW(Addr)) / 4);
  const uint32_t* chain = buckets + nbuckets;
  const uint32_t h = gnu_hash(q->name);
  for (uint32_t i = buckets[h % nbuckets]; i >= symoffset && i != 0; ++i) {
    const uint32_t ch = chain[i - symoffset];
    const ElfW(Sym)& sym = symtab[i];
    if ((h | 1) == (ch | 1) && sym.st_shndx != SHN_UNDEF && strcmp(q->name, strtab + sym.st_name) == 0) {
      q->addr = reinterpret_cast<void*>(base + sym.st_value);
      return 1;
    }
    if (ch & 1) break;
  }
  return 0;
}

}  // namespace

// loaded by /etc/ld.so.preload or LD_PRELOAD: make sure ROCr loads us as a tools library (before any hsa_init)
__attribute__((constructor)) static void gsx_isolate_preload() { ensure_tools_lib(); }

// Preloaded, this definition precedes libhsa-runtime64's in the global scope, so HIP's (and any program's) call
// reaches it first: HSA_TOOLS_LIB is put back right before the runtime reads it, whatever the process did to its
// environment since it started (os.environ.pop("HSA_TOOLS_LIB") before import torch, setenv, clearenv).
GSX_EXPORT hsa_status_t hsa_init() {
  ensure_tools_lib();
  static hsa_status_t (*real)() = nullptr;
  if (!real) {
    SymQuery q{"hsa_init", nullptr};
    dl_iterate_phdr(find_in_hsa_runtime, &q);
    real = reinterpret_cast<hsa_status_t (*)()>(q.addr);
  }
  if (!real || reinterpret_cast<void*>(real) == reinterpret_cast<void*>(&hsa_init)) {
    fprintf(stderr, "gsx-isolate: the HSA runtime's hsa_init not found; refusing to run unconfined\n");
    return HSA_STATUS_ERROR;
  }
  return real();
}
