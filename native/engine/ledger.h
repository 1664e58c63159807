// GPU-share ledger: node -> device -> pod accounting and the binpack policy.
//
// Reference: pkg/cache/{cache,nodeinfo,deviceinfo}.go.  Same observable
// policy (single-device fit in filter, best-fit with lowest-index ties in
// bind, used memory = sum of the pods' SHARED_GPU_MEM_POD annotations,
// Succeeded/Failed pods not counted), re-designed for throughput:
//   * per-device used counters are maintained incrementally (the reference
//     re-parses every pod annotation on every query, deviceinfo.go:41-54);
//   * signed arithmetic, no uint underflow on over-commit (nodeinfo.go:260);
//   * bind reserves memory up front ("assume"), so concurrent binds on one
//     node need no lock held across apiserver round-trips (nodeinfo.go:141);
//   * capacity / device-count changes rebuild the node (cache.go:144-157
//     only rebuilt on the non-gpushare -> gpushare transition);
//   * heterogeneous per-device totals via a node annotation.
#pragma once

#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <list>
#include <map>
#include <mutex>
#include <string>
#include <atomic>
#include <unordered_map>
#include <unordered_set>
#include <deque>
#include <vector>

#include <string_view>

#include "introspect.h"
#include "model.h"

namespace gsx {

// A pod's CU-partition request (deviceplugin/allocator.py CU_COUNT_ANNOTATION).
constexpr std::string_view kCuCountAnnotation = "gpushare.amd.com/cu-count";

enum class Check : int { Ok = 0, NodeNotFound = 1, NotGPUShare = 2, Insufficient = 3 };

struct PodRec {
  std::string uid, ns, name, node;
  int64_t dev = -1;      // device index on node (-1: not placed)
  int64_t hold = -1;     // second device charged while a reconciliation moves the pod (-1: none)
  int64_t mem = 0;       // accounted memory (annotation POD / assumed request)
  int64_t request = 0;   // container-limit sum (inspect "usedGPU" per pod)
  bool terminal = false; // Succeeded/Failed -> not counted
  bool deleting = false;
  bool assumed = false;  // reserved by bind, not yet observed with annotations
  bool bound = false;    // bind round-trips finished successfully
  double assumed_at = 0;
  double bound_at = 0;   // when the bind's apiserver write succeeded
  double deadline = 0;   // expiry of an assumed+bound reservation
  bool accounted = false;
  int64_t held_on = -1;  // the hold device actually charged by account() (node may have changed since)
  int64_t assume_ns = 0;      // ASSUME_TIME written by our bind
  bool unannotated = false;   // observed bound to its node WITHOUT the allocation annotations we sent
  bool repair_queued = false;
  // a device-plugin move in flight (begin_move): the target device is charged too until the informer shows the
  // pod there (or the move fails), so nothing else is placed into the room it takes
  int64_t move_to = -1;
  int64_t moved_on = -1;  // the move target actually charged by account()
  double move_at = 0;
};

// POST /gpushare-scheduler/move: the device plugin asks the extender -- the one writer of *_IDX -- to rewrite a
// bound pod's allocation record (a reconciliation exchange step, a hold release, a move off a physically full GPU).
struct MoveRequest {
  std::string uid, node;
  int64_t from = -1;       // the device the caller's view has the pod on (the ledger must agree)
  int64_t to = -1;         // the new *_IDX (-1: best fit with room, other than `from`)
  // the exchange partner: the pod on `to` that this move's hold swaps with (step 1: the request carries
  // hold-idx = `from` and a hold-partner naming it), or the pod holding `to` that took this pod's GPU (step 2).  A
  // verified partner's share is credited on `to` (it leaves `to`), so an exchange of two sizes is checked on the
  // final state of both GPUs, not refused for the room the partner still occupies
  std::string partner;
  // the pod's container already runs on `to` (a drift repair, or taking over the allocation it holds there): the
  // device plugin's published unaccounted use on `to` includes it, and moves into the annotations
  bool physical_on_to = false;
  int64_t req_hold = -1;        // hold-idx the move request writes (-1: none)
  std::string req_hold_partner; // uid named by the hold-partner the move request writes
};

// A pod this extender bound whose allocation annotations the apiserver did not keep (an apiserver or
// admission webhook that drops Binding.metadata.annotations): what to write back onto it.
struct AnnotationRepair {
  std::string uid, ns, name, node;
  int64_t dev = -1, dev_total = -1, mem = 0, assume_ns = 0;
};

struct DevState {
  int64_t total = 0;
  int64_t used = 0;
  int64_t npods = 0;
  int64_t held = 0;  // the part of `used` charged by exchange holds (pods leaving this device once the hold clears)
};

struct NodeState {
  std::string name;
  std::string address;
  int64_t total = 0;  // node capacity
  int64_t count = 0;
  std::vector<int64_t> dev_totals_override;
  std::vector<DevState> devs;
  std::unordered_set<std::string> pods;  // uids whose rec.node == name
  bool landing_order = false;            // NodeView::landing_order
  // the device plugin's unaccounted use (POST /gpushare-scheduler/physical): units kubelet's containers hold on a
  // device whose pods the annotations put elsewhere, or that are gone -- a kubelet admission batch served two pods
  // each other's allocations and the exchange of their records has not landed, or the pod an allocation was built
  // for was deleted while another pod's container holds it.  Charged on top of the annotations, so such a device
  // takes no bind into room its containers already fill.  Empty: none published (or expired, extra_until)
  std::vector<int64_t> extra;
  double extra_until = 0;
  bool publishes = false;      // NodeView::publishes
  bool published = false;      // a publication of the node's plugin arrived in this epoch
  double pub_wait_until = 0;   // binds to the node wait for that publication until then (0: no wait)
  bool gpushare() const { return total > 0 && count > 0; }
  int64_t used_eff(size_t i) const { return devs[i].used + (i < extra.size() ? extra[i] : 0); }
  int64_t free_of(size_t i) const { return devs[i].total - used_eff(i); }
};

struct Stats {
  uint64_t filter_calls = 0, filter_nodes_ok = 0, filter_nodes_failed = 0;
  uint64_t assume_ok = 0, assume_fail = 0, bind_ok = 0, bind_fail = 0;
  uint64_t expired = 0, overcommit_events = 0, pod_upserts = 0, pod_removes = 0;
  uint64_t expiry_deferred = 0;  // GC passes that kept an overdue reservation until a LIST could confirm it
  uint64_t annotations_missing = 0;  // binds observed bound without the annotations they carried
  uint64_t moves_ok = 0, moves_refused = 0, moves_failed = 0;  // device-plugin allocation-record writes
  uint64_t partner_claims_refused = 0;
  uint64_t unaccounted_updates = 0, unaccounted_expired = 0;  // the device plugin's unaccounted-use publications  // a move naming a partner the ledger does not show in an exchange with it
};

class Ledger {
 public:
  explicit Ledger(Profile p) : profile_(std::move(p)) {}
  const Profile& profile() const { return profile_; }

  // ---- nodes (informer-driven) ----
  // Returns true when the device layout was (re)built.
  bool upsert_node(const NodeView& nv);
  bool remove_node(const std::string& name);
  bool has_node(const std::string& name) const;

  // ---- pods (informer-driven; cache.go:89-127) ----
  // Returns 1 if the pod is (now) accounted to a device, 0 if skipped
  // (no nodeName / no valid device index).
  int upsert_pod(const PodView& v);
  bool remove_pod(const std::string& uid);
  bool known(const std::string& uid) const;
  // 0 unknown, 1 accounted from annotations, 2 assumed (bind reservation not
  // yet confirmed by the informer).  The controller uses it to decide whether
  // an update event must be synced (pkg/gpushare/controller.go:257-305).
  int pod_state(const std::string& uid, int64_t* dev) const;
  // Binds observed without their annotations since the last call (see AnnotationRepair)
  std::vector<AnnotationRepair> drain_repairs();
  // Bind order (see bind ordering below):
  //   kOrderAuto (default): ASSUME_TIME order on nodes whose device plugin matches by ASSUME_TIME (the
  //     reference's contract), none on nodes that advertise landing-order matching (allocstate.h);
  //   kOrderStrict: ASSUME_TIME order everywhere;
  //   kOrderRelaxed: no bind waits for another anywhere.  Safe only where the device plugin reconciles its
  //     Allocates with kubelet's PodResources record (deviceplugin/reconcile.py).
  enum OrderMode : int { kOrderAuto = 0, kOrderStrict = 1, kOrderRelaxed = 2 };
  void set_order_mode(OrderMode m) { order_mode_.store(m); }
  OrderMode order_mode() const { return static_cast<OrderMode>(order_mode_.load()); }
  static const char* order_mode_name(OrderMode m) {
    return m == kOrderStrict ? "strict" : m == kOrderRelaxed ? "relaxed" : "auto";
  }
  // true: binds to this node wait for earlier equal-size binds headed for another GPU
  bool node_ordered_locked(const std::string& node) const;

  // ---- scheduling verbs ----
  Check check(const std::string& node, int64_t req) const;  // nodeinfo.go:113-137
  // Reserve a device for a pod being bound (best fit, nodeinfo.go:209-252).
  // Returns device index >= 0, or -1 insufficient, -2 node not found,
  // -3 node not gpushare, -4 bind already in flight for this uid.
  int64_t assume(const std::string& uid, const std::string& ns, const std::string& name,
                 const std::string& node, int64_t req, int64_t* dev_total);
  void finish_bind(const std::string& uid, bool ok, double ttl_s);
  // Validate a move and reserve its target: 0 ok (*to resolved; the pod is charged on both devices until the
  // informer confirms it on the target, or end_move(false)); 1 the pod is not bound to that node here; 2 stale (the
  // ledger has it on another device); 3 no room on the target (and no equal-size partner makes the move
  // sum-neutral); 4 a bind or another move of the pod is in flight.
  int begin_move(MoveRequest* m, std::string* why);
  void end_move(const std::string& uid, bool ok);

  // ---- bind ordering, shared by the native front end and the Python slow path ----
  // kubelet admits a node's pods in the order their bindings land, and the device plugin gives a request
  // of N units to the earliest-ASSUME_TIME unassigned pod of that size (docs/designs/designs.md:93-103):
  // two equal-size pods headed for different GPUs of one node must reach the apiserver in ASSUME_TIME
  // order.  assume_ordered() (ledger mutex held) reserves the device, stamps ASSUME_TIME and enters the
  // in-flight set in one step; bind_wait() (ledger mutex NOT held) blocks only while an earlier
  // equal-size bind of that node is in flight whose pod is not interchangeable with this one: another GPU,
  // or a different CU-partition request (`cu_count`, the gpushare.amd.com/cu-count annotation; the plugin
  // would hand one pod's partition size to the other's container); bind_leave() ends the entry.
  int64_t assume_ordered(const std::string& uid, const std::string& ns, const std::string& name,
                         const std::string& node, int64_t req, int64_t* dev_total, uint64_t* seq, int64_t* assume_ns,
                         const std::string& cu_count = std::string());
  bool bind_blocked(uint64_t seq);
  void bind_wait(uint64_t seq, const std::atomic<bool>* stop);
  void bind_leave(uint64_t seq);
  uint64_t bind_order_waits() const { return order_waits_.load(); }
  // total / longest time binds spent held back by bind_wait (seconds)
  double bind_order_wait_s() const { return static_cast<double>(order_wait_ns_.load()) * 1e-9; }
  double bind_order_wait_max_s() const { return static_cast<double>(order_wait_max_ns_.load()) * 1e-9; }
  // Expire stale reservations.  A bound reservation the pod informer has not confirmed within its TTL is
  // dropped only if a pod LIST that *started after the bind succeeded* (`confirmed_list_start`, steady-clock
  // seconds; 0 = none) was applied without confirming it: then the apiserver really has no such binding.
  // Otherwise -- watch stalled, apiserver unreachable -- the device stays reserved (never over-committed)
  // and `*need_relist` is set so the caller forces a LIST.  Binds that never finished expire after 600 s.
  int gc(double confirmed_list_start, bool* need_relist);

  // ---- observation ----
  std::string inspect_json(const std::string& node, bool* found) const;
  std::vector<std::pair<int64_t, int64_t>> node_devices(const std::string& node) const;
  // the device plugin's unaccounted use per device of `node` (empty: withdraw), valid for ttl_s; false: unknown node
  bool set_unaccounted(const std::string& node, const std::vector<int64_t>& extra, double ttl_s);
  // A new extender epoch (process start, or this replica became the leader): the unaccounted use its predecessor
  // was told is unknown here, so binds to every node whose plugin publishes wait (at most hold_s) for that plugin's
  // first publication of the epoch -- the plugin republishes as soon as it sees the epoch change.  hold_s 0: off.
  void begin_epoch(double hold_s);
  // seconds a bind to `node` still waits for its plugin's publication (0: none)
  double publication_wait(const std::string& node) const;
  std::vector<int64_t> node_unaccounted(const std::string& node) const;
  std::vector<std::string> node_names() const;
  Stats stats() const { return stats_; }
  Stats& mutable_stats() { return stats_; }
  size_t pod_count() const { return pods_.size(); }
  const NodeState* node(const std::string& name) const {
    auto it = nodes_.find(name);
    return it == nodes_.end() ? nullptr : &it->second;
  }

  static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  }

  introspect::ProfiledMutex& mu() { return mu_; }

  // ---- pods seen by the filter verb (native bind fast path) ----
  // The filter request carries the whole v1.Pod; remembering (uid -> ns,
  // name, request) lets the native bind skip the lister lookup.  Bounded FIFO.
  struct PendingPod {
    std::string ns, name;
    int64_t req = 0;
    std::string cu_count;  // gpushare.amd.com/cu-count annotation ("" none): part of the bind-order class
    std::string rv;        // metadata.resourceVersion the scheduler saw (update-mode precondition)
  };
  void remember_pending(const std::string& uid, PendingPod p);
  bool pending(const std::string& uid, PendingPod* out) const;
  void forget_pending(const std::string& uid);
  // live filter-time records and the length of their eviction-order queue (bounded by 2x live + 1024)
  size_t pending_count() const { return pending_.size(); }
  size_t pending_queue_len() const { return pending_order_.size(); }

 private:
  void account(PodRec& r);
  void unaccount(PodRec& r);
  void rebuild(NodeState& n);
  void erase_pod(std::unordered_map<std::string, PodRec>::iterator it);

  Profile profile_;
  std::map<std::string, NodeState> nodes_;  // ordered: deterministic inspect
  std::unordered_map<std::string, PodRec> pods_;
  std::vector<AnnotationRepair> repairs_;
  double pub_hold_s_ = 0;  // begin_epoch(): nodes first seen later in the epoch wait that long too
  void arm_publication_wait(NodeState& n);
  void queue_repair(PodRec& r);
  Stats stats_;
  mutable introspect::ProfiledMutex mu_;  // every caller locks it; contention is exported to /debug/pprof/mutex
  std::unordered_map<std::string, PendingPod> pending_;
  std::deque<std::string> pending_order_;
  // in-flight binds (order_mu_ nests inside the ledger mutex, never around it)
  struct InflightBind {
    std::string node;
    int64_t size, dev;
    uint64_t seq;
    std::string cu_count;
    bool ordered = true;                        // node_ordered_locked() when the bind was assumed
    std::condition_variable* waiter = nullptr;  // set while its bind sits in bind_wait()
  };
  bool blocked_locked(const InflightBind& me) const;
  std::mutex order_mu_;
  std::atomic<int> order_mode_{kOrderAuto};
  std::list<InflightBind> inflight_;
  uint64_t order_seq_ = 0;
  int64_t last_assume_ns_ = 0;
  std::atomic<uint64_t> order_waits_{0}, order_wait_ns_{0}, order_wait_max_ns_{0};
};

// Full filter verb on a raw ExtenderArgs body; returns the
// ExtenderFilterResult JSON with the reference's Go field names
// (vendor/k8s.io/kubernetes/pkg/scheduler/api/types.go:273-284).
std::string filter_body(Ledger& l, std::string_view body);

// Prioritize verb: HostPriorityList scoring nodes by best-fit tightness (0..10).
std::string prioritize_body(Ledger& l, std::string_view body);

}  // namespace gsx
