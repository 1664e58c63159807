// Native-thread introspection for the extender's /debug/pprof/* (the reference serves Go's net/http/pprof,
// pkg/routes/pprof.go:10-64, which sees every goroutine of the process that serves filter / bind).
//
// Here filter / bind run on C++ epoll loops and a bind pool, the informers on reflector threads: a
// Python-only profiler sees none of them.  This module gives /debug/pprof the native view:
//
//   * every native thread names itself (pthread_setname_np, visible in /proc/self/task/<tid>/comm, top -H,
//     gdb) so per-thread CPU time can be attributed;
//   * capture(): a stack sample of any thread of the process.  The requester sends a real-time signal to
//     the thread (tgkill); its handler records backtrace() into a slot; the requester symbolises outside the
//     handler (dladdr + demangling).  Handlers are installed with SA_RESTART, but that does NOT restart
//     recv / send on sockets with SO_RCVTIMEO / SO_SNDTIMEO (signal(7)): those return EINTR, and every
//     caller retries them (plain sockets and SSL_read / SSL_write alike, apiclient.cc); epoll_wait returns
//     EINTR, which every loop already tolerates;
//   * ProfiledMutex: the ledger's mutex, counting acquisitions, contended acquisitions, wait and hold time
//     (the /debug/pprof/mutex and block profiles).
#pragma once

#include <atomic>
#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

namespace gsx {
namespace introspect {

// Name the calling thread ("gsx-" prefix added; truncated to the kernel's 15 characters).
void name_thread(const std::string& name);

// Install the sampling signal handler (idempotent).  False if the signal could not be installed.
bool install();

struct Sample {
  int tid = 0;
  std::string comm;              // /proc/self/task/<tid>/comm
  std::vector<std::string> frames;  // innermost first, symbolised
  bool ok = false;                // false: the thread did not answer in time (blocked signal, exited)
};

// Stack samples of the given threads of this process (all threads when empty).  One capture at a time.
std::vector<Sample> capture(const std::vector<int>& tids, double timeout_s = 0.05);

// Thread ids of this process (/proc/self/task).
std::vector<int> thread_ids();

// Function name covering `pc` (ELF .symtab of the loaded objects, then dladdr); "" when unknown.
std::string symbol_at(uintptr_t pc);

struct MutexStats {
  uint64_t acquisitions = 0, contended = 0;
  double wait_s = 0, max_wait_s = 0, hold_s = 0, max_hold_s = 0;
};

// std::mutex with contention accounting; BasicLockable (std::lock_guard / std::unique_lock).
class ProfiledMutex {
 public:
  void lock();
  bool try_lock();
  void unlock();
  MutexStats stats() const;

 private:
  std::mutex m_;
  uint64_t acquired_ns_ = 0;  // written under m_
  std::atomic<uint64_t> n_{0}, contended_{0}, wait_ns_{0}, max_wait_ns_{0}, hold_ns_{0}, max_hold_ns_{0};
};

}  // namespace introspect
}  // namespace gsx
