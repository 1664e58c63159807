// Native cluster-state sync controller: pod / node reflectors -> ledger.
//
// Counterpart of pkg/gpushare/controller.go + pkg/cache/cache.go:49-127 (and
// of the asyncio controller in core/controller.py, which it replaces on the
// default extender path).  Same observable rules:
//
//   * only pods requesting gpu-mem pass the event filter, with
//     FilteringResourceEventHandler transitions (controller.go:77-100);
//   * add -> sync; update -> sync iff (known and now complete) or (unknown /
//     bind-assumed and annotated with a device index) or (device index
//     rewritten) (controller.go:257-305); delete -> sync with the remembered
//     object (controller.go:307-332, removePodCache);
//   * syncPod (controller.go:174-205): gone -> remove; complete -> remove;
//     otherwise add-or-update from annotations;
//   * BuildCache (cache.go:49-74) on the first pod LIST, plus a consistency
//     check that reports over-committed devices instead of wrapping uints;
//   * nodes go straight into the ledger; capacity changes rebuild the node.
//
// Differences by design: events are applied on the reflector thread the
// moment they are decoded (ledger operations cannot fail, so the reference's
// rate-limited retry queue has nothing to retry), there is no 1 s sleep per
// synced item (controller.go:218-223), and all state is guarded by mutexes
// (the reference raced on removePodCache and the node map).
#pragma once

#include <atomic>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "informer.h"
#include "ledger.h"

namespace gsx {

struct ControllerConfig {
  ApiConfig api;
  double resync_s = 30.0;  // informer resync (cmd/main.go:28); 0 disables
  int watch_timeout_s = 300;
};

struct ControllerStats {
  uint64_t pod_events = 0, node_events = 0, syncs = 0, removes = 0, upserts = 0, resyncs = 0;
  uint64_t pod_lists = 0, node_lists = 0, pod_watches = 0, node_watches = 0, watch_errors = 0;
  uint64_t pod_list_pages = 0, node_list_pages = 0;
  uint64_t recovered = 0;  // pods replayed by BuildCache
};

class Controller {
 public:
  Controller(Ledger* l, ControllerConfig cfg);
  ~Controller();
  // Starts the node reflector, waits for it, then the pod reflector
  // (controller.go:118-128 waits for nodes, then pods); false on timeout.
  bool start(double sync_timeout_s, std::string* err);
  void stop();
  bool synced() const;
  // Lister: raw JSON of the last observed gpu-share pod `ns/name`.
  bool get_pod(const std::string& key, std::string* raw) const;
  bool has_pod(const std::string& key) const;
  std::vector<std::tuple<std::string, int, int64_t, int64_t>> overcommitted() const;
  ControllerStats stats() const;
  std::string last_error() const;
  // Reservation GC gated on the pod reflector (Ledger::gc): an overdue bind reservation is dropped only
  // once a LIST begun after its binding has been applied without confirming it; until then a re-list is
  // forced (a stalled or unanswered watch never makes a held device look free).
  int gc_reservations(bool* relist_requested);
  double pod_list_start() const;
  void request_pod_relist();

 private:
  struct Entry {
    PodView v;
    bool share = false;  // passes the gpu-mem filter
    std::string raw;     // object JSON (gpu-share pods only; lister)
  };

  void on_pod_list(const ListView& lv);
  void on_pod_event(Ev ev, const json::Doc& d, uint32_t obj);
  void on_node_list(const ListView& lv);
  void on_node_event(Ev ev, const json::Doc& d, uint32_t obj);
  bool decode(const json::Doc& d, uint32_t obj, Entry* e) const;
  // handler semantics (called with smu_ held)
  void h_add(const std::string& key);
  void h_update(const Entry& old, const std::string& key);
  void h_delete(const std::string& key, const Entry& gone);
  void sync(const std::string& key);
  void build_cache();
  void resync_loop();

  Ledger* l_;
  ControllerConfig cfg_;
  std::unique_ptr<Reflector> pods_, nodes_;
  mutable std::mutex smu_;  // store_, removed_, stats_, overcommitted_
  std::unordered_map<std::string, Entry> store_;    // ns/name -> last state
  std::unordered_map<std::string, Entry> removed_;  // removePodCache
  bool built_ = false;
  ControllerStats stats_;
  std::vector<std::tuple<std::string, int, int64_t, int64_t>> overcommitted_;
  std::unordered_set<std::string> listed_nodes_;  // guarded by the ledger mutex
  std::thread resync_th_;
  std::atomic<bool> stop_{false};
  std::mutex rmu_;
  std::condition_variable rcv_;
};

}  // namespace gsx
