#include "introspect.h"

#include <cxxabi.h>
#include <dirent.h>
#include <dlfcn.h>
#include <elf.h>
#include <execinfo.h>
#include <link.h>
#include <pthread.h>
#include <signal.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <fstream>
#include <iterator>
#include <thread>
#include <unordered_map>

namespace gsx {
namespace introspect {

namespace {

uint64_t mono_ns() {
  return static_cast<uint64_t>(
      std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
          .count());
}

void atomic_max(std::atomic<uint64_t>* a, uint64_t v) {
  uint64_t cur = a->load(std::memory_order_relaxed);
  while (v > cur && !a->compare_exchange_weak(cur, v, std::memory_order_relaxed)) {
  }
}

constexpr int kMaxFrames = 48;

// One capture slot: the requester arms it for a tid, that thread's handler fills it.
struct Slot {
  std::atomic<int> state{0};  // 0 idle, 1 armed, 2 filled
  std::atomic<int> tid{0};
  void* pcs[kMaxFrames];
  int n = 0;
};

Slot g_slot;
std::mutex g_capture_mu;
std::atomic<bool> g_installed{false};
int g_sig = 0;

int gettid_() { return static_cast<int>(::syscall(SYS_gettid)); }

void on_sample(int, siginfo_t*, void*) {
  int saved = errno;
  if (g_slot.state.load(std::memory_order_acquire) == 1 && g_slot.tid.load(std::memory_order_relaxed) == gettid_()) {
    g_slot.n = ::backtrace(g_slot.pcs, kMaxFrames);
    g_slot.state.store(2, std::memory_order_release);
  }
  errno = saved;
}

std::string comm_of(int tid) {
  std::ifstream f("/proc/self/task/" + std::to_string(tid) + "/comm");
  std::string s;
  std::getline(f, s);
  return s;
}

// Function symbols of every loaded object from its ELF .symtab (static symbols included: the engine is
// built with -fvisibility=hidden, so dladdr alone would only ever name PyInit__engine).
struct Sym {
  uintptr_t addr, size;
  std::string name;
};

void load_symtab(const std::string& path, uintptr_t base, std::vector<Sym>* out) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return;
  std::string img((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  if (img.size() < sizeof(Elf64_Ehdr) || std::memcmp(img.data(), ELFMAG, SELFMAG) != 0) return;
  const auto* eh = reinterpret_cast<const Elf64_Ehdr*>(img.data());
  if (eh->e_ident[EI_CLASS] != ELFCLASS64 || eh->e_shoff == 0 ||
      eh->e_shoff + uint64_t(eh->e_shnum) * sizeof(Elf64_Shdr) > img.size()) {
    return;
  }
  const auto* sh = reinterpret_cast<const Elf64_Shdr*>(img.data() + eh->e_shoff);
  for (int i = 0; i < eh->e_shnum; ++i) {
    if (sh[i].sh_type != SHT_SYMTAB || sh[i].sh_link >= eh->e_shnum) continue;
    const Elf64_Shdr& str = sh[sh[i].sh_link];
    if (sh[i].sh_offset + sh[i].sh_size > img.size() || str.sh_offset + str.sh_size > img.size()) continue;
    const auto* syms = reinterpret_cast<const Elf64_Sym*>(img.data() + sh[i].sh_offset);
    size_t n = sh[i].sh_size / sizeof(Elf64_Sym);
    for (size_t k = 0; k < n; ++k) {
      if (ELF64_ST_TYPE(syms[k].st_info) != STT_FUNC || syms[k].st_value == 0 || syms[k].st_name >= str.sh_size) {
        continue;
      }
      out->push_back({base + syms[k].st_value, syms[k].st_size, std::string(img.data() + str.sh_offset + syms[k].st_name)});
    }
  }
}

const std::vector<Sym>& symbols() {
  static std::vector<Sym> syms = [] {
    std::vector<Sym> v;
    struct Obj {
      std::string path;
      uintptr_t base;
    };
    std::vector<Obj> objs;
    ::dl_iterate_phdr(
        [](dl_phdr_info* info, size_t, void* data) {
          auto* o = static_cast<std::vector<Obj>*>(data);
          std::string path = info->dlpi_name && *info->dlpi_name ? info->dlpi_name : "/proc/self/exe";
          o->push_back({path, static_cast<uintptr_t>(info->dlpi_addr)});
          return 0;
        },
        &objs);
    for (auto& o : objs) load_symtab(o.path, o.base, &v);
    std::sort(v.begin(), v.end(), [](const Sym& a, const Sym& b) { return a.addr < b.addr; });
    return v;
  }();
  return syms;
}

std::string demangle(const char* name) {
  int st = 0;
  char* dm = abi::__cxa_demangle(name, nullptr, nullptr, &st);
  std::string out = st == 0 && dm ? dm : name;
  std::free(dm);
  // keep collapsed-stack lines readable: drop argument lists of demangled C++ names
  size_t paren = out.find('(');
  if (paren != std::string::npos && paren > 0) out.resize(paren);
  return out;
}

std::string symbolize(void* pc) {
  static std::mutex mu;
  static std::unordered_map<void*, std::string> cache;
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(pc);
  if (it != cache.end()) return it->second;
  std::string out;
  const auto& syms = symbols();
  uintptr_t a = reinterpret_cast<uintptr_t>(pc) - 1;  // return addresses point past the call
  auto ub = std::upper_bound(syms.begin(), syms.end(), a, [](uintptr_t x, const Sym& s) { return x < s.addr; });
  if (ub != syms.begin()) {
    const Sym& s = *std::prev(ub);
    if (a < s.addr + std::max<uintptr_t>(s.size, 1)) out = demangle(s.name.c_str());
  }
  Dl_info info;
  if (out.empty() && ::dladdr(pc, &info) && info.dli_sname) out = demangle(info.dli_sname);
  if (out.empty()) {
    const char* obj = (::dladdr(pc, &info) && info.dli_fname) ? std::strrchr(info.dli_fname, '/') : nullptr;
    char b[96];
    std::snprintf(b, sizeof(b), "%s+%p", obj ? obj + 1 : "?", pc);
    out = b;
  }
  cache.emplace(pc, out);
  return out;
}

}  // namespace

void name_thread(const std::string& name) {
  std::string n = "gsx-" + name;
  if (n.size() > 15) n.resize(15);
  ::pthread_setname_np(::pthread_self(), n.c_str());
}

bool install() {
  if (g_installed.load()) return true;
  std::lock_guard<std::mutex> g(g_capture_mu);
  if (g_installed.load()) return true;
  void* warm[4];
  ::backtrace(warm, 4);  // loads the unwinder now, not inside a signal handler
  g_sig = SIGRTMIN + 5;
  struct sigaction sa;
  std::memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = on_sample;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigemptyset(&sa.sa_mask);
  if (::sigaction(g_sig, &sa, nullptr) != 0) return false;
  g_installed.store(true);
  return true;
}

std::string symbol_at(uintptr_t pc) {
  std::string s = symbolize(reinterpret_cast<void*>(pc + 1));  // symbolize() looks up pc - 1
  return s.find("+0x") != std::string::npos && s.find('?') == 0 ? std::string() : s;
}

std::vector<int> thread_ids() {
  std::vector<int> out;
  DIR* d = ::opendir("/proc/self/task");
  if (!d) return out;
  while (dirent* e = ::readdir(d)) {
    if (e->d_name[0] < '0' || e->d_name[0] > '9') continue;
    out.push_back(std::atoi(e->d_name));
  }
  ::closedir(d);
  return out;
}

std::vector<Sample> capture(const std::vector<int>& tids_in, double timeout_s) {
  std::vector<Sample> out;
  if (!install()) return out;
  std::vector<int> tids = tids_in.empty() ? thread_ids() : tids_in;
  const int self = gettid_();
  std::lock_guard<std::mutex> g(g_capture_mu);
  for (int tid : tids) {
    Sample s;
    s.tid = tid;
    s.comm = comm_of(tid);
    if (tid == self) {  // our own stack: no signal needed
      void* pcs[kMaxFrames];
      int n = ::backtrace(pcs, kMaxFrames);
      for (int i = 1; i < n; ++i) s.frames.push_back(symbolize(pcs[i]));
      s.ok = true;
      out.push_back(std::move(s));
      continue;
    }
    g_slot.tid.store(tid, std::memory_order_relaxed);
    g_slot.state.store(1, std::memory_order_release);
    if (::syscall(SYS_tgkill, ::getpid(), tid, g_sig) != 0) {
      g_slot.state.store(0);
      continue;  // exited meanwhile
    }
    uint64_t deadline = mono_ns() + static_cast<uint64_t>(timeout_s * 1e9);
    while (g_slot.state.load(std::memory_order_acquire) != 2 && mono_ns() < deadline) {
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    int expected = 2;
    if (g_slot.state.compare_exchange_strong(expected, 0)) {
      // frame 0 is the handler, frame 1 the kernel's signal trampoline
      for (int i = 2; i < g_slot.n; ++i) s.frames.push_back(symbolize(g_slot.pcs[i]));
      s.ok = true;
    } else {
      // disarm; a handler that runs late sees state != 1 and does nothing
      g_slot.state.store(0, std::memory_order_release);
    }
    out.push_back(std::move(s));
  }
  return out;
}

void ProfiledMutex::lock() {
  if (!m_.try_lock()) {
    uint64_t t0 = mono_ns();
    m_.lock();
    uint64_t w = mono_ns() - t0;
    contended_.fetch_add(1, std::memory_order_relaxed);
    wait_ns_.fetch_add(w, std::memory_order_relaxed);
    atomic_max(&max_wait_ns_, w);
  }
  n_.fetch_add(1, std::memory_order_relaxed);
  acquired_ns_ = mono_ns();
}

bool ProfiledMutex::try_lock() {
  if (!m_.try_lock()) return false;
  n_.fetch_add(1, std::memory_order_relaxed);
  acquired_ns_ = mono_ns();
  return true;
}

void ProfiledMutex::unlock() {
  uint64_t h = mono_ns() - acquired_ns_;
  hold_ns_.fetch_add(h, std::memory_order_relaxed);
  atomic_max(&max_hold_ns_, h);
  m_.unlock();
}

MutexStats ProfiledMutex::stats() const {
  MutexStats s;
  s.acquisitions = n_.load();
  s.contended = contended_.load();
  s.wait_s = static_cast<double>(wait_ns_.load()) * 1e-9;
  s.max_wait_s = static_cast<double>(max_wait_ns_.load()) * 1e-9;
  s.hold_s = static_cast<double>(hold_ns_.load()) * 1e-9;
  s.max_hold_s = static_cast<double>(max_hold_ns_.load()) * 1e-9;
  return s;
}

}  // namespace introspect
}  // namespace gsx
