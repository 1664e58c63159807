// Per-GPU pod runtime endpoint in C++ (the CRI-runtime role of the node):
// the node agent starts / stops pods on a GPU through it.  Counterpart of
// deviceplugin/runtime.py (HbmArenaRuntime + RuntimeShim) without Python on
// the admission path: the request thread carves the pod's 2 MiB-aligned slice
// out of the GPU's HBM arena, stamps it and verifies every resident slice with
// ONE call into libgsx_kernels.so (gsx_hbm_admit_n: two kernel launches, one
// stream sync), and answers.  A slice is a list of extents taken first-fit
// from the arena's holes: the extender accounts a device's memory as one
// number (like HBM behind the GPU's page tables), so a pod that fits the
// device's free bytes must be admitted even when no single hole is big enough.
//
//   POST   /v1/pods/<uid>  {"dev","bytes","cus","verify"} -> {"bad": n} | 409 {"error"}
//   DELETE /v1/pods/<uid>
//   GET    /v1/stats
//
// With arena_addr == 0 (no GPU) only the slice accounting runs.
#pragma once

#include <cstdint>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "ctlserver.h"

namespace gsx {

struct PodRuntimeConfig {
  int dev = 0;
  uint64_t arena_bytes = 0;
  uint64_t arena_addr = 0;  // device pointer of the arena (0: accounting only)
  void* stream = nullptr;   // hipStream_t for the admission kernels
  uint64_t stride = 1 << 20;
  std::string kernels_lib;  // path of libgsx_kernels.so (already loaded by the process)
};

class PodRuntime {
 public:
  explicit PodRuntime(PodRuntimeConfig cfg);
  ~PodRuntime();
  bool init(std::string* err);  // resolves the kernel entry points
  // `cpus`: where the endpoint's threads run (the CRI-runtime role gets a CPU of its own; empty: inherit)
  int serve(const std::string& host, int port, std::string* err, std::vector<int> cpus = {});
  void stop();
  // Admission without HTTP (tests): returns bad stamps, -1 with *err on failure.
  int64_t admit(const std::string& uid, uint64_t bytes, bool verify, std::string* err);
  bool release(const std::string& uid);
  int64_t verify_all(std::string* err);
  uint64_t admitted() const { return admitted_; }
  uint64_t failed() const { return failed_; }
  uint64_t bad() const { return bad_; }
  uint64_t batches() const { return batches_; }  // GPU admission calls (one per group of concurrent admissions)
  uint64_t resident_bytes() const;
  size_t resident() const;

 private:
  struct Slice {
    std::vector<std::pair<uint64_t, uint64_t>> ext;  // (offset, bytes), offset-ordered
    uint64_t size, tag;
  };
  CtlServer::Reply handle(const http::Message& m);
  // Stamp `uid`'s extents (if `stamp`) and verify the resident slices (all of them, or only `uid`'s when
  // !verify); mu_ held.  Returns bad stamps, -1 with *err.
  int64_t run_admit(bool stamp, const std::string& uid, bool verify, std::string* err);
  // Group commit: admissions that arrive while one is on the GPU are carved and admitted together, one
  // stamp launch + one verify launch + one sync for the group.
  struct Pending {
    std::string uid;
    uint64_t bytes;
    bool verify;
    bool done = false;
    int64_t result = 0;
    std::string err;
  };
  bool carve_locked(const std::string& uid, uint64_t bytes, std::string* err);  // mu_ held
  void admit_group_locked(const std::vector<Pending*>& group);                   // mu_ held

  PodRuntimeConfig cfg_;
  mutable std::mutex mu_;
  std::map<std::string, Slice> slices_;  // uid -> slice
  uint64_t admitted_ = 0, failed_ = 0, bad_ = 0, batches_ = 0;
  std::mutex qmu_;  // the admission queue; never held with mu_ across a GPU call
  std::condition_variable qcv_;
  std::vector<Pending*> queue_;
  bool leading_ = false;  // a thread is admitting a group
  std::unique_ptr<CtlServer> srv_;
  void* lib_ = nullptr;
  int (*set_device_)(int) = nullptr;
  int (*admit_n_)(void*, const void*, int, int, int, uint64_t, uint64_t*) = nullptr;
  const char* (*last_error_)() = nullptr;
};

}  // namespace gsx
