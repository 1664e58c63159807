// The device plugin's Allocate path in native code, on the one matcher (allocstate.h) — used by the shipped
// plugin's native gRPC server (bindings: _engine.DpServer) for the common case, with the Python plugin
// (deviceplugin/plugin.py allocate_container) answering everything else, and by the Python code itself for the
// pieces that must have one implementation: the container response (build_response, the reference's env
// contract plus /dev nodes and the CU partition) and the enforced-isolation files (isolation_prepare).
//
// Fast path of one Allocate (one container request, as kubelet sends them): match the earliest-ASSUME_TIME
// pending pod of that size; a later container of a committed pod is answered from the pod's state; a first
// container commits ASSIGNED=true with a resourceVersion-guarded PATCH.  Anything unusual -- no candidate, an
// unknown or physically full GPU (by the Allocate records), a pod in a reconciliation exchange, a failed PATCH --
// returns false and the Python slow path (refresh, wait for annotations, reconcile, guard, retries) decides.
#pragma once

#include <cstdint>
#include <map>
#include <unordered_map>
#include <memory>
#include <string>
#include <string_view>
#include <vector>

#include "allocstate.h"
#include "apiclient.h"
#include "dpproto.h"
#include "model.h"

namespace gsx {

struct DpDevice {
  int index = 0;
  std::string bdf;
  int cu_count = 256;
  int64_t total_bytes = 0, share_bytes = 0;
  int64_t units = 0;                // capacity in the advertised unit
  std::vector<std::string> nodes;   // /dev/kfd, /dev/dri/renderD*, ... (mount mode "isolated")
  bool healthy = true;
};

struct DpConfig {
  std::string node;
  Profile profile;
  std::string mount_mode = "isolated";
  int64_t unit_bytes = int64_t{1} << 30;
  std::string iso_dir;  // enforced isolation host directory ("" = advisory)
  bool guard = false;   // reconciliation on: refuse a first container on a GPU its records say is full
  ApiConfig api;
  // early answer: a first container's Allocate is answered once its record is in `journal` (appended, one JSON
  // line per Allocate), and the ASSIGNED patch follows; the pod stays claimed (in flight) until the patch lands.
  // kubelet admits a node's pods one at a time, so the apiserver round trip leaves its admission path.
  bool early_answer = false;
  std::string journal;
};

// ---- the single implementations the Python plugin calls too
dp::ContainerResponse build_response(const AllocPod& pod, const DpDevice& d, int64_t container_units,
                                     const std::vector<int>& cus, const std::string& mount_mode, const Profile& p);
std::string isolation_config_text(const std::vector<int>& cus, int cu_count, int64_t limit_bytes);
// Writes <host_dir>/pods/<uid>/{isolation.conf,hbm.ledger}; fills the Allocate mounts / envs.
bool isolation_prepare(const std::string& host_dir, const std::string& uid, const std::vector<int>& cus, int cu_count,
                       int64_t limit_bytes, bool host_process, std::vector<dp::MountMsg>* mounts,
                       std::map<std::string, std::string>* envs, std::string* err);

struct DpEvent {  // what the Python side learns after a fast-path Allocate
  std::string uid, key, aid, iso, pod_json;
  bool committed = false;  // a first container (ASSIGNED patch) rather than a later one
  // another pending pod of the same size waits for another GPU: a kubelet admission batch may have served this
  // allocation to that pod (the reconciliation looks at once)
  bool ambiguous = false;
  bool patch_only = false;  // early answer: the ASSIGNED patch of an Allocate answered before landed (pod_json)
  double t_handler = 0, t_match = 0, t_patch = 0, t_isolate = 0;
};

// A first container waiting for its ASSIGNED patch.  The PATCH runs off the owner's thread (the plugin's event
// loop must never block on the apiserver -- in tests the apiserver is served by that very loop); begin / finish
// and every AllocState access stay on the owner's thread.
struct DpPending {
  uint64_t call = 0;
  std::string request;  // the Allocate request, for the slow path if the PATCH fails
  AllocPod pod;
  bool whole = false, had_cus = false;
  int64_t units = 0;
  std::vector<std::string> ids;
  bool on_gpu = false;  // every ID lies on the pod's GPU
  bool ambiguous = false;  // DpEvent::ambiguous
  dp::ContainerResponse cr;
  std::string iso, path, body;
  double t0 = 0, tm = 0, ti0 = 0, ti1 = 0, tp0 = 0, tp1 = 0;
  bool answered = false;  // early answer: kubelet has its response; only the patch remains
  bool retry = false;     // finish() asks for the patch to be run again
  int attempts = 0;
  double not_before = 0;  // early-answer retry: not before this CLOCK_MONOTONIC time (backoff)
  // filled by the worker
  bool ok = false;
  int status = 0;
  std::string resp, err;
};

enum class DpStep { Answered, AnsweredPending, Pending, Slow };

class DpCore {
 public:
  DpCore(DpConfig cfg, AllocState* state);
  ~DpCore();
  DpCore(const DpCore&) = delete;
  DpCore& operator=(const DpCore&) = delete;
  void set_devices(std::vector<DpDevice> devs, std::map<std::string, int> id_owner);
  void set_state(AllocState* state) { state_ = state; }  // the device layout changed: a rebuilt state
  const std::map<int, DpDevice>& devices() const { return devs_; }

  // true: answered (*resp = the response message); false: the slow path answers (*why says why)
  bool preferred(const std::string& req, std::string* resp, std::string* why);
  // Answered: *resp / *ev set.  Pending: *pend holds the PATCH to run (then finish()).  AnsweredPending (early
  // answer): *resp / *ev set and *pend holds the PATCH still to run.  Slow: Python answers.
  DpStep allocate(const std::string& req, std::string* resp, DpEvent* ev, std::unique_ptr<DpPending>* pend,
                  std::string* why);
  // after the PATCH: true = answered (*resp / *ev); false = undone, the slow path answers.  For an early-answered
  // Allocate nothing is answered: *ev->patch_only carries the committed pod, or p.retry asks for another run at
  // p.not_before (transport / 5xx / transient 409: capped exponential backoff, for as long as the pod exists);
  // 404, a UID-precondition 409 (re-created) or a pod the state no longer has: nothing left to commit.
  bool finish(DpPending& p, std::string* resp, DpEvent* ev, std::string* why);
  // the worker's half: the blocking apiserver call
  void run_patch(DpPending& p);

  struct Stats {
    uint64_t fast_allocate = 0, fast_preferred = 0, slow_allocate = 0, slow_preferred = 0, patch_failures = 0;
    uint64_t journal_failures = 0;  // early-answer journal lines that did not reach the file (then early answer off)
    uint64_t commits_gone = 0;  // early-answer commits whose pod was gone (404 / re-created): released at once
    uint64_t guard_by_ids = 0;  // the records said full, kubelet's IDs said there is room
    // fast-path Allocate phases, summed seconds over `phased` answers: decode, match, guard + CU claim, response
    // build, commit body, record (incl. the physical account), journal line, response encode
    double ph_decode = 0, ph_match = 0, ph_claim = 0, ph_build = 0, ph_body = 0, ph_record = 0, ph_journal = 0,
           ph_encode = 0;
    uint64_t phased = 0;
  };
  const Stats& stats() const { return stats_; }
  // early answer: the journal's lines move to <journal>.old (appended if a previous checkpoint left one) and the
  // journal starts empty; the caller deletes .old once the checkpoint holding those records is in place.  Called
  // under the state lock, so no Allocate falls between the records snapshot and the rotation.
  bool journal_rotate(std::string* err);
  bool journaling() const { return jfd_ >= 0; }
  // the mapping trimmed to its lines and closed (the endpoint is closing: no Allocate is answered after this)
  void journal_close() { journal_unmap(true); }
  // closing: an ASSIGNED commit in flight fails at once instead of waiting out the apiserver (an early-answered one
  // is in the journal, and the restarted plugin lands it)
  void abort_requests() {
    if (api_) api_->abort();
  }
  const std::string& journal_path() const { return cfg_.journal; }
  int64_t physical_used(int dev) const;
  bool ids_on(const std::vector<std::string>& ids, int dev) const;

 private:
  DpConfig cfg_;
  AllocState* state_;
  std::unique_ptr<ApiClient> api_;
  std::map<int, DpDevice> devs_;
  std::unordered_map<std::string, int> id_owner_;
  std::unordered_map<std::string_view, int> id_owner_view_;  // keys view id_owner_'s strings
  std::unordered_map<int, std::string> id_prefix_;  // dev -> its IDs' common prefix (empty map: use the lookups)
  static constexpr std::string_view kIdSep = "-_-";  // deviceplugin/plugin.py: ID_SEP
  bool id_on(std::string_view id, int dev) const;
  uint64_t aid_ = 0;
  // The early-answer journal: a MAP_SHARED mapping of the file (a line is durable against a crash of this process
  // once copied in, as a write(2) to the page cache is, without a syscall per Allocate).  The file is sized ahead in
  // kJournalChunk steps; bytes past jlen_ are zeros until it is trimmed (close, rotation).
  int jfd_ = -1;
  char* jmap_ = nullptr;
  size_t jcap_ = 0, jlen_ = 0;
  static constexpr size_t kJournalChunk = size_t(1) << 20;
  bool journal_map(int fd, std::string* err);  // maps fd, jlen_ = its whole lines
  void journal_unmap(bool trim);
  Stats stats_;
  void record_and_answer(DpPending& p, std::string* resp, DpEvent* ev);
  bool journal_append(const AllocRecord& r);  // false: the line did not reach the file
};

}  // namespace gsx
