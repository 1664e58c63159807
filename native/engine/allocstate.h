// The device plugin's allocation state: ONE implementation of the Allocate matching contract, used by the
// shipped gRPC device plugin (Python, through the _engine binding: deviceplugin/state.py) and by the compiled
// kubelet stand-in (native/nodeagent).
//
// The contract (reconstructed from docs/designs/designs.md:93-103 and docs/designs/sequence.jpg; the plugin
// itself is not in the reference tree): kubelet asks for N fake device IDs and never says for
// which pod; the plugin serves the earliest-ASSUME_TIME pending pod bound to its node whose request is N and
// whose ASSIGNED annotation is "false", and flips ASSIGNED to "true" (the commit point).  On top of that:
//
//  * candidates: Pending pods of this node, ASSIGNED=false, *_IDX naming one of our GPUs, not claimed by an
//    Allocate whose ASSIGNED patch is in flight; ordered by (landing, ASSUME_TIME, creationTimestamp, ns/name).
//    `landing` is the resourceVersion at which the pod was first seen bound to this node: kubelet admits
//    the pods of its node one at a time in the order its watch delivers them (one admission batch per watch
//    event: the apiserver config source pushes every event, kubelet's pod config merges it into an ADD of
//    the pods it had not seen), and that order is resourceVersion order for every watcher.  So the earliest
//    landed candidate is the pod kubelet is admitting, whatever order the extender's binds reached the
//    apiserver in; with binds landing in ASSUME_TIME order (the reference's only guarantee) the two keys
//    agree.  The plugin advertises this on its node (gpushare.amd.com/allocate-order=landing) and the
//    extender then binds equal-size pods for different GPUs concurrently (ledger.h, bind ordering).  Only a
//    multi-pod admission batch (kubelet's initial LIST after a restart, sorted by creationTimestamp) can
//    still disagree; deviceplugin/reconcile.py repairs those from kubelet's PodResources record;
//  * multi-container pods: kubelet calls Allocate once per container.  The first container commits the pod;
//    the remaining container sizes are kept until allocated ("partial").  After a restart the progress of an
//    ASSIGNED=true Pending pod is unknown, so any of its sizes is accepted again;
//  * CU partitions (the MPS stand-in, README.md:77): per GPU, owned per pod UID, spread round-robin over the
//    XCDs; rebuilt from the gpushare.amd.com/cu-mask annotation of assigned pods, released when a pod
//    completes or disappears;
//  * allocation records: every Allocate with kubelet's device IDs, the pod it was matched to and what it
//    handed out; deviceplugin/reconcile.py compares them with kubelet's PodResources record.
//
// Not thread-safe: callers serialise (the Python plugin runs on one event loop; the node agent holds its mutex).
#pragma once

#include <cstdint>
#include <deque>
#include <map>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "json.h"
#include "model.h"

namespace gsx {

// Per-device CU ledger.  A partition of n CUs takes the free CUs in round-robin XCD order (xcc0 cu0,
// xcc1 cu0, ..., logical CU ids are xcc-major blocks of cu/xcc), so every pod keeps a share of every L2 slice.
class CuPartitioner {
 public:
  explicit CuPartitioner(int cu = 256, int xcc = 8);
  // the pod's partition (the same one again if it already holds one); false + *err when it does not fit
  bool allocate(const std::string& uid, int n, std::vector<int>* out, std::string* err);
  int release(const std::string& uid);  // CUs freed
  // an existing partition (from a pod's cu-mask annotation); CUs another pod owns stay with it: returns them
  std::vector<int> adopt(const std::string& uid, const std::vector<int>& cus);
  void swap_owners(const std::string& a, const std::string& b);
  bool holds(const std::string& uid) const { return held_.count(uid) != 0; }
  std::vector<int> held_by(const std::string& uid) const;
  const std::unordered_map<std::string, std::vector<int>>& held() const { return held_; }
  int free_count() const;
  int cu_count() const { return cu_; }
  int xcc_count() const { return xcc_; }

 private:
  int cu_, xcc_;
  std::vector<std::string> owner_;
  std::unordered_map<std::string, std::vector<int>> held_;
};

std::string cu_words(const std::vector<int>& cus, int cu_count);  // "0x000000ff,0x00000000,..."
std::vector<int> parse_cu_words(const std::string& words);
std::string cu_ranges(const std::vector<int>& cus);  // "0-7,32-39" (HSA_CU_MASK list syntax)

struct AllocPod {
  std::string uid, key, ns, name, rv, phase, creation, node;
  int64_t dev = -1;           // *_IDX annotation
  int64_t request = 0;        // sum of container limits
  std::vector<int64_t> containers;  // container limits > 0, in spec order
  int64_t assume_time = -1;
  int64_t landed = -1;        // set by AllocState::observe: resourceVersion first seen bound to the node
  int64_t dev_total = -1;     // *_DEV annotation
  std::string assigned;       // ASSIGNED annotation value ("" absent)
  bool complete = false;
  // deletionTimestamp set, phase not terminal: kubelet is stopping its containers.  Complete for matching (no
  // Allocate serves it), but the scheduler extender keeps its share charged until the object is gone
  // (controller.cc sync), so the annotated account below keeps it too
  bool terminating = false;
  double grace_s = -1;        // metadata.deletionGracePeriodSeconds (-1 absent)
  // spec.terminationGracePeriodSeconds: the apiserver's defaulting writes 30 into every pod it stores; absent only
  // from the fakes' pods, which they delete at once (tests/fixtures/fakeapi.py delete) -- 0
  double term_grace_s = 0;
  int cu_count = 0;           // gpushare.amd.com/cu-count
  std::string cu_mask;        // gpushare.amd.com/cu-mask
  int64_t hold_idx = -1;      // gpushare.amd.com/hold-idx
  std::string hold_partner;   // gpushare.amd.com/hold-partner
  // the pod object as the apiserver sent it, when a feed kept it (the shipped plugin's pod feed and its own PATCH
  // responses: the Python side reads pod objects from here instead of running a second watch); "" otherwise
  std::string raw;
  bool pending() const { return phase == "Pending" || phase.empty(); }
};

// Build an AllocPod from a pod object on a JSON tape (the node agent's informer).
bool parse_alloc_pod(const json::Doc& d, uint32_t pod, const Profile& p, AllocPod* out);

struct AllocRecord {
  std::string aid;
  std::vector<std::string> ids;  // kubelet's device IDs, sorted
  std::string uid;               // the pod whose annotations describe this allocation
  int64_t dev = -1, units = 0;
  std::string cu_mask;
  std::string owner;             // the pod kubelet gave the IDs to ("" until PodResources said so)
  double t = 0;
  std::string iso;               // isolation directory key the container's mounts point at
  // every ID lies on `dev` (by the plugin's fake-ID layout): kubelet's own per-ID accounting then bounds what
  // physically runs on that GPU (false: unknown or mixed -- only the records can tell)
  bool on_gpu = false;
  const std::string& holder() const { return owner.empty() ? uid : owner; }
};

struct AllocStats {
  uint64_t cu_released = 0, cu_adopted = 0, cu_conflicts = 0, partial_released = 0, pods_released = 0,
           records_dropped = 0, matches = 0, match_misses = 0;
};

class AllocState {
 public:
  AllocState(std::string node, const std::vector<std::pair<int, std::pair<int, int>>>& devices);  // idx -> (cu, xcc)

  // ---- informer feed
  // An added / updated pod.  Returns false if ignored as a stale copy (older resourceVersion).
  bool observe(const AllocPod& p);
  void release(const std::string& uid);  // completed / deleted
  // A pod the apiserver deleted (a watch DELETE): released, and its UID remembered, so that a copy of it still in
  // flight (a second feed that lags, a PATCH response read after the delete) cannot bring it back with its CU
  // partition.  UIDs are never reused; a complete pod is remembered the same way (terminal phases and deletion
  // timestamps are never undone).  Kept for kTombstoneS seconds.
  //
  // A pod deleted while live here (never seen terminating, not terminal: a force delete) with kubelet reporting
  // owners: kubelet drops it from PodResources and frees its device IDs at once, but its containers get their
  // termination grace to exit.  What they hold lingers on its GPUs (physical_used, and no per-ID bound there) until
  // `now` (wall seconds; <0: the clock) + spec.terminationGracePeriodSeconds + kLingerSlackS.
  void deleted(const std::string& uid, double now = -1.0);
  static constexpr double kLingerSlackS = 2.0;
  // off: kubelet's PodResources report is taken as the truth about a force-deleted pod's containers (a kubelet that
  // lists them until they have stopped, like the node agent stand-in): what they hold stays held until kubelet no
  // longer lists it (prune_held), and is published as unaccounted use meanwhile (gone_held)
  void set_linger(bool on) { linger_on_ = on; }
  // the matcher skips the partner of an unfinished exchange (candidates); off only to show what that prevents
  void set_skip_partners(bool on) { skip_partners_ = on; }
  bool linger_enabled() const { return linger_on_; }
  int64_t lingering(int64_t dev) const;  // units of force-deleted pods' containers still counted on `dev`
  // units kubelet still lists on `dev` for pods this view no longer has -- deleted pods' containers that have not
  // stopped yet, the extender freed their share with the objects -- once two reports in a row, kGoneHeldMinS apart
  // at least, have listed them after the pod went (a container that stops within that is never published: the
  // physical guard still counts it.  Published and withdrawn a pass later, a fast stop held the extender's room for
  // a poll interval -- a 10 ms wave in the headline bench on MI355X)
  int64_t gone_held(int64_t dev) const;
  static constexpr double kGoneHeldMinS = 0.05;
  size_t linger_count() const { return linger_.size(); }
  void tombstone(const std::string& uid);
  bool is_tombstoned(const std::string& uid) const { return gone_.count(uid) != 0; }
  static constexpr double kTombstoneS = 600.0;
  // A complete LIST of this node's pods (already observed): anything held that is not in `live` is gone.
  void resync(const std::unordered_set<std::string>& live, double now = -1.0);
  std::vector<std::string> holders() const;
  // ---- terminating pods (AllocPod::terminating): what the extender still charges for them, per GPU
  int64_t terminating_used(int64_t dev) const;
  // the GPU a terminating pod's annotation names (-1: not terminating here)
  int64_t terminating_dev(const std::string& uid) const;
  size_t terminating_count() const { return terminating_.size(); }

  // ---- Allocate
  std::vector<const AllocPod*> candidates() const;
  // (pod, whole_pod) for an Allocate of `units`: a whole pod of that size (earliest ASSUME_TIME), else a later
  // container of a pod whose first container was allocated, else the first container of a multi-container
  // pod that has a container of that size.
  std::pair<const AllocPod*, bool> match(int64_t units);
  int64_t preferred_device(int64_t units);
  bool unannotated(int64_t units) const;
  bool claim_cus(const std::string& uid, std::vector<int>* out, std::string* err);
  void set_inflight(const std::string& uid, bool on);
  bool inflight(const std::string& uid) const { return inflight_.count(uid) != 0; }
  void first_container_committed(const std::string& uid, int64_t units, bool whole);
  void later_container_allocated(const std::string& uid, int64_t units);

  // ---- allocation records
  // `on_gpu`: every ID lies on the pod's GPU (set here, not by a later mark_on_gpu: one key and hash fewer)
  AllocRecord& record(const std::string& uid, const std::vector<std::string>& ids, int64_t units,
                      const std::string& cu_mask, const std::string& aid, double t, bool on_gpu = false);
  void add_record(AllocRecord r);  // restored from a checkpoint
  bool drop_record(const std::string& aid);
  const AllocRecord* record_for_ids(std::vector<std::string> ids) const;
  AllocRecord* record_by_aid(const std::string& aid);
  void set_owner(const std::string& aid, const std::string& owner);
  // With kubelet's PodResources reconciled (`on`), a record whose holder kubelet has not reported yet is not
  // dropped with the pod it was built for: after a swap another pod's container may be running with it.  The
  // reconciler drops it once kubelet no longer lists its IDs.
  void set_owners_reported(bool on) {
    owners_reported_ = on;
    if (!on) owners_expected_ = false;  // nobody will report: records and holds end with their pods again
  }
  bool owners_reported() const { return owners_reported_; }
  // A PodResources reconciler runs but has not reported yet: a pod's going does not end the allocations built
  // for it (another container may hold one: a swap), until kubelet's first report says who holds what.
  void expect_owner_reports(bool on) { owners_expected_ = on; }
  bool owners_known() const { return owners_reported_ || owners_expected_; }
  // After the annotations of P and Q were exchanged because P holds `aid` (built for Q): that record now
  // describes P, whatever described P describes Q, and the CU partitions follow.
  void move_records(const std::string& p_uid, const std::string& q_uid, const std::string& aid);
  const std::map<std::string, AllocRecord>& records() const { return records_; }
  // ---- what kubelet has handed out (the physical account)
  // One entry per Allocate answered, keyed by kubelet's device IDs: the GPU the container was given and its units.
  // Kept apart from the records' reconciliation bookkeeping (exchanges re-label records; pods come and go): an
  // entry leaves only when kubelet no longer reports its IDs (prune_held), or -- with nobody reporting -- with the
  // pod it was built for.  physical_used() is what really runs on a GPU, whatever the annotations say.
  int64_t physical_used(int64_t dev) const;
  void mark_on_gpu(const std::string& aid, bool on);
  size_t off_gpu_records() const { return off_gpu_; }  // entries whose IDs do not all lie on their GPU
  // those of them whose container runs on GPU `dev`: while there are none, kubelet's per-ID accounting bounds what
  // runs on `dev` (every unit there holds one of its IDs)
  size_t off_gpu_records_on(int64_t dev) const;
  // kubelet's PodResources answer, requested at `asked` (wall seconds): entries made more than `grace` before it whose
  // IDs it does not list are gone (their containers stopped) -- unless the pod kubelet last reported holding them is
  // live here (kubelet stops listing a force-deleted pod at once; the delete reaches this view a moment later and
  // makes the entry linger).  An entry held by a force-deleted pod -- or never reported while a force-deleted pod's
  // containers may still run (kubelet gave the IDs to a pod deleted before its admission) -- lingers until that pod's
  // kill deadline.  Lingering entries past their time go.  Returns how many left.
  size_t prune_held(const std::vector<std::vector<std::string>>& listed, double asked, double grace);
  size_t held_count() const { return held_.size(); }
  // what was handed out with these IDs: false if nothing this plugin knows of
  bool held_for(std::vector<std::string> ids, int64_t* dev, int64_t* units, double* t, std::string* cu_mask) const;
  std::vector<AllocRecord> take_dropped();  // records dropped since the last call (isolation cleanup)
  bool dropped_pending() const { return !dropped_.empty(); }

  const AllocPod* pod(const std::string& uid) const;
  const AllocPod* pod_by_key(const std::string& key) const;
  const std::unordered_map<std::string, AllocPod>& pods() const { return pods_; }
  const std::unordered_map<std::string, std::vector<int64_t>>& partial() const { return partial_; }
  CuPartitioner* cus(int dev);
  const std::map<int, CuPartitioner>& all_cus() const { return cus_; }
  bool has_device(int64_t dev) const { return cus_.count(static_cast<int>(dev)) != 0; }
  const AllocStats& stats() const { return stats_; }
  const std::string& node() const { return node_; }

 private:
  std::string node_;
  std::map<int, CuPartitioner> cus_;
  std::unordered_map<std::string, AllocPod> pods_;        // uid -> non-complete pods on this node
  struct Terminating {
    int64_t dev = -1, request = 0, hold = -1;
  };
  std::unordered_map<std::string, Terminating> terminating_;  // uid -> terminating pods on this node
  std::unordered_map<std::string, double> gone_;          // deleted / complete UIDs -> when (see deleted())
  std::deque<std::pair<double, std::string>> gone_order_;
  std::unordered_map<std::string, std::string> keys_;     // ns/name -> uid
  std::unordered_map<std::string, std::vector<int64_t>> partial_;  // uid -> container sizes not yet allocated
  std::unordered_set<std::string> local_commits_, inflight_;
  std::map<std::string, AllocRecord> records_;            // aid -> record
  // an ID set as one string: the sorted IDs joined by '\n' (one allocation and one hash per lookup, where a
  // vector key cost a copy of every ID string and element-wise compares on the Allocate path)
  static std::string id_key(const std::vector<std::string>& sorted_ids);
  std::unordered_map<std::string, std::string> by_ids_;  // id_key -> aid
  std::vector<AllocRecord> dropped_;
  struct Held {
    int64_t dev = -1, units = 0;
    double t = 0;
    std::string uid;  // the pod the allocation was built for (pruned with it when nobody reports owners)
    bool on_gpu = false;
    std::string cu_mask;  // the CU partition handed out with it
    std::string owner;    // the pod kubelet last reported holding the IDs (set_owner)
    bool listed = false;  // kubelet's last report listed the IDs (prune_held)
    int gone_reports = 0; // reports in a row that listed them after their holder had gone (holder_gone)
    double gone_since = 0;  // when the first of those reports was asked for
  };
  double last_prune_ = 0;  // when the last report prune_held saw was asked for
  bool holder_gone(const Held& h) const;
  struct Linger {
    int64_t dev = -1, units = 0;
    double until = 0;
  };
  std::vector<Linger> linger_;                     // held entries of force-deleted pods' containers
  std::unordered_map<int64_t, int64_t> linger_units_;  // dev -> their units
  std::unordered_map<int64_t, size_t> linger_n_;       // dev -> their count
  // force-deleted pods, by UID and by "~ns/name" -> when kubelet has killed their containers (wall seconds)
  std::unordered_map<std::string, double> forced_;
  std::unordered_map<std::string, double> deleted_;  // uid -> when deleted() saw it go (gone_held; kept kTombstoneS)
  bool linger_on_ = true;
  bool skip_partners_ = true;
  void linger(const Held& h, double until);
  void unlinger(const Linger& l);
  void force_gone(const std::string& uid, double now);  // deleted() / resync(): a live pod gone outright
  // a held entry kubelet stopped listing: when the force-deleted pod that may still run it is dead by (0: none)
  double ghost_until(const Held& h) const;

  std::unordered_map<std::string, Held> held_;  // id_key(sorted kubelet IDs) -> what was handed out with them
  std::unordered_map<int64_t, int64_t> phys_;     // dev -> sum of held_ units (kept in step)
  size_t off_gpu_ = 0;                             // held_ entries with on_gpu == false
  std::unordered_map<int64_t, size_t> off_gpu_dev_;  // ... per GPU their container runs on
  void off_gpu_count(int64_t dev, int d);
  void hold(const std::string& ids_key, Held h);
  void unhold(std::unordered_map<std::string, Held>::iterator it);
  bool owners_reported_ = false;
  bool owners_expected_ = false;
  AllocStats stats_;
};

}  // namespace gsx
