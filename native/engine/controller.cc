#include "controller.h"
#include "introspect.h"

#include <chrono>
#include <unordered_set>

namespace gsx {

namespace {

std::string key_of(const PodView& v) { return v.ns.empty() ? v.name : v.ns + "/" + v.name; }

}  // namespace

Controller::Controller(Ledger* l, ControllerConfig cfg) : l_(l), cfg_(std::move(cfg)) {
  ReflectorConfig pr;
  pr.path = "/api/v1/pods";
  pr.watch_timeout_s = cfg_.watch_timeout_s;
  ReflectorHandler ph;
  ph.on_list = [this](const ListView& lv) { on_pod_list(lv); };
  ph.on_event = [this](Ev ev, const json::Doc& d, uint32_t obj) { on_pod_event(ev, d, obj); };
  pods_ = std::make_unique<Reflector>(cfg_.api, pr, ph);
  ReflectorConfig nr;
  nr.path = "/api/v1/nodes";
  nr.watch_timeout_s = cfg_.watch_timeout_s;
  ReflectorHandler nh;
  nh.on_list = [this](const ListView& lv) { on_node_list(lv); };
  nh.on_event = [this](Ev ev, const json::Doc& d, uint32_t obj) { on_node_event(ev, d, obj); };
  nodes_ = std::make_unique<Reflector>(cfg_.api, nr, nh);
}

Controller::~Controller() { stop(); }

bool Controller::start(double sync_timeout_s, std::string* err) {
  stop_.store(false);
  nodes_->start();
  if (!nodes_->wait_synced(sync_timeout_s)) {
    *err = "node informer did not sync: " + nodes_->last_error();
    return false;
  }
  pods_->start();
  if (!pods_->wait_synced(sync_timeout_s)) {
    *err = "pod informer did not sync: " + pods_->last_error();
    return false;
  }
  if (cfg_.resync_s > 0 && !resync_th_.joinable()) resync_th_ = std::thread([this] {
    introspect::name_thread("resync");
    resync_loop();
  });
  return true;
}

void Controller::stop() {
  stop_.store(true);
  rcv_.notify_all();
  if (pods_) pods_->stop();
  if (nodes_) nodes_->stop();
  if (resync_th_.joinable()) resync_th_.join();
}

bool Controller::synced() const { return pods_->synced() && nodes_->synced(); }

double Controller::pod_list_start() const { return pods_->last_list_start(); }

void Controller::request_pod_relist() { pods_->request_relist(); }

int Controller::gc_reservations(bool* relist_requested) {
  bool need = false;
  int n;
  {
    std::lock_guard<introspect::ProfiledMutex> g(l_->mu());
    n = l_->gc(pods_->last_list_start(), &need);
  }
  if (need) pods_->request_relist();
  if (relist_requested) *relist_requested = need;
  return n;
}

std::string Controller::last_error() const {
  std::string e = pods_->last_error();
  return e.empty() ? nodes_->last_error() : e;
}

bool Controller::get_pod(const std::string& key, std::string* raw) const {
  std::lock_guard<std::mutex> g(smu_);
  auto it = store_.find(key);
  if (it == store_.end() || !it->second.share) return false;
  *raw = it->second.raw;
  return true;
}

bool Controller::has_pod(const std::string& key) const {
  std::lock_guard<std::mutex> g(smu_);
  auto it = store_.find(key);
  return it != store_.end() && it->second.share;
}

std::vector<std::tuple<std::string, int, int64_t, int64_t>> Controller::overcommitted() const {
  std::lock_guard<std::mutex> g(smu_);
  return overcommitted_;
}

ControllerStats Controller::stats() const {
  std::lock_guard<std::mutex> g(smu_);
  ControllerStats s = stats_;
  s.pod_lists = pods_->relists();
  s.node_lists = nodes_->relists();
  s.pod_watches = pods_->rewatches();
  s.node_watches = nodes_->rewatches();
  s.watch_errors = pods_->errors() + nodes_->errors();
  s.pod_list_pages = pods_->list_pages();
  s.node_list_pages = nodes_->list_pages();
  return s;
}

bool Controller::decode(const json::Doc& d, uint32_t obj, Entry* e) const {
  if (!parse_pod(d, obj, l_->profile(), &e->v)) return false;
  e->share = e->v.request > 0;  // IsGPUsharingPod (pod.go:40-42)
  if (e->share) e->raw.assign(d.raw(obj));
  return true;
}

// ---------------------------------------------------------------- sync

void Controller::sync(const std::string& key) {
  // controller.go:174-205
  stats_.syncs++;
  auto it = store_.find(key);
  if (it == store_.end() || !it->second.share) {
    auto gone = removed_.find(key);
    if (gone != removed_.end()) {
      {
        std::lock_guard<introspect::ProfiledMutex> g(l_->mu());
        l_->remove_pod(gone->second.v.uid);
      }
      stats_.removes++;
      removed_.erase(gone);
    }
    return;
  }
  removed_.erase(key);
  const PodView& v = it->second.v;
  std::lock_guard<introspect::ProfiledMutex> g(l_->mu());
  // controller.go:193-195 frees a pod at IsCompletePod, i.e. already at its deletionTimestamp.  Here a terminating
  // pod stays charged until its object is gone (the DELETED event, above) or its phase turns terminal: kubelet
  // stops its containers during the grace period, and kube-scheduler's own NodeInfo counts it until then too
  // ("deleting pods still count -- keep (conservative)")
  if (v.terminal()) {
    l_->remove_pod(v.uid);
    stats_.removes++;
    return;
  }
  l_->upsert_pod(v);
  stats_.upserts++;
}

void Controller::h_add(const std::string& key) { sync(key); }

void Controller::h_update(const Entry& old, const std::string& key) {
  // controller.go:257-305 enqueue rules (+ "assumed by our bind, now observed",
  // "device index rewritten" and "reconciliation hold set or cleared")
  const Entry& cur = store_[key];
  int64_t dev = -1;
  int state;
  {
    std::lock_guard<introspect::ProfiledMutex> g(l_->mu());
    state = l_->pod_state(cur.v.uid, &dev);
  }
  bool enqueue = false;
  if (state != 0 && (cur.v.terminal() || cur.v.deleting != old.v.deleting)) {
    enqueue = true;  // now terminal (freed), or terminating (still charged; inspect lists it no more)
  } else if (cur.v.dev_idx >= 0 && (state == 0 || state == 2)) {
    enqueue = true;
  } else if (state == 1 && cur.v.dev_idx != dev) {
    enqueue = true;
  } else if (state != 0 && cur.v.hold_idx != old.v.hold_idx) {
    enqueue = true;
  } else if (state == 2 && cur.v.dev_idx < 0 && !cur.v.node.empty()) {
    enqueue = true;  // our reservation, bound, but without its annotations: the ledger queues a repair
  }
  if (enqueue) sync(key);
}

void Controller::h_delete(const std::string& key, const Entry& gone) {
  removed_[key] = gone;
  sync(key);
}

// ---------------------------------------------------------------- pods

void Controller::on_pod_event(Ev ev, const json::Doc& d, uint32_t obj) {
  Entry e;
  if (!decode(d, obj, &e)) return;
  std::string key = key_of(e.v);
  std::lock_guard<std::mutex> g(smu_);
  stats_.pod_events++;
  if (ev == Ev::Deleted) {
    auto it = store_.find(key);
    Entry old;
    bool had = it != store_.end();
    if (had) {
      old = std::move(it->second);
      store_.erase(it);
    }
    const Entry& gone = had ? old : e;
    if (gone.share) h_delete(key, gone);
    return;
  }
  auto it = store_.find(key);
  if (it == store_.end()) {
    bool share = e.share;
    store_.emplace(key, std::move(e));
    if (share) h_add(key);
    return;
  }
  Entry old = std::move(it->second);
  it->second = std::move(e);
  bool was = old.share, now = it->second.share;
  if (was && now) {
    h_update(old, key);
  } else if (now) {
    h_add(key);
  } else if (was) {
    h_delete(key, old);
  }
}

void Controller::on_pod_list(const ListView& lv) {
  std::unordered_map<std::string, Entry> fresh;
  fresh.reserve(lv.size());
  for (size_t k = 0; k < lv.size(); ++k) {
    Entry e;
    if (!decode(lv.doc(k), lv.obj(k), &e)) continue;
    std::string key = key_of(e.v);
    fresh[key] = std::move(e);
  }
  std::lock_guard<std::mutex> g(smu_);
  std::unordered_map<std::string, Entry> old;
  old.swap(store_);
  // client-go Replace(): deletes for objects that vanished while not watching
  for (auto& kv : old) {
    if (fresh.count(kv.first) == 0 && kv.second.share) h_delete(kv.first, kv.second);
  }
  store_ = std::move(fresh);
  if (!built_) {
    build_cache();
    built_ = true;
    return;
  }
  for (auto& kv : store_) {
    auto o = old.find(kv.first);
    if (o == old.end()) {
      if (kv.second.share) h_add(kv.first);
      continue;
    }
    if (o->second.v.rv == kv.second.v.rv) continue;
    bool was = o->second.share, now = kv.second.share;
    if (was && now) {
      h_update(o->second, kv.first);
    } else if (now) {
      h_add(kv.first);
    } else if (was) {
      h_delete(kv.first, o->second);
    }
  }
}

void Controller::build_cache() {
  // cache.go:49-74: replay annotated, scheduled pods (annotations are the
  // durable allocation record), then the informer's initial adds.
  uint64_t n = 0;
  {
    std::lock_guard<introspect::ProfiledMutex> g(l_->mu());
    for (auto& kv : store_) {
      const PodView& v = kv.second.v;
      if (!kv.second.share || v.terminal()) continue;  // a terminating pod still holds its share (sync)
      if (v.annot_mem > 0 && !v.node.empty()) {
        if (l_->upsert_pod(v) > 0) ++n;
      }
    }
  }
  for (auto& kv : store_) {
    if (kv.second.share) sync(kv.first);
  }
  stats_.recovered += n;
  // consistency check: report devices whose annotations add
  // up to more than capacity instead of wrapping (nodeinfo.go:260)
  overcommitted_.clear();
  std::lock_guard<introspect::ProfiledMutex> g(l_->mu());
  for (const std::string& node : l_->node_names()) {
    auto devs = l_->node_devices(node);
    for (size_t i = 0; i < devs.size(); ++i) {
      if (devs[i].second > devs[i].first) {
        overcommitted_.emplace_back(node, static_cast<int>(i), devs[i].second, devs[i].first);
      }
    }
  }
}

void Controller::resync_loop() {
  // Informer resync (cmd/main.go:28): every stored pod is re-delivered as an
  // update, so a missed transition is eventually applied.
  while (!stop_.load()) {
    {
      std::unique_lock<std::mutex> lk(rmu_);
      rcv_.wait_for(lk, std::chrono::duration<double>(cfg_.resync_s), [this] { return stop_.load(); });
    }
    if (stop_.load()) return;
    std::lock_guard<std::mutex> g(smu_);
    stats_.resyncs++;
    std::vector<std::string> keys;
    keys.reserve(store_.size());
    for (auto& kv : store_) {
      if (kv.second.share) keys.push_back(kv.first);
    }
    for (const auto& k : keys) {
      auto it = store_.find(k);
      if (it != store_.end()) h_update(it->second, k);
    }
  }
}

// ---------------------------------------------------------------- nodes

void Controller::on_node_event(Ev ev, const json::Doc& d, uint32_t obj) {
  NodeView nv;
  if (!parse_node(d, obj, l_->profile(), &nv)) return;
  {
    std::lock_guard<std::mutex> g(smu_);
    stats_.node_events++;
  }
  std::lock_guard<introspect::ProfiledMutex> g(l_->mu());
  if (ev == Ev::Deleted) {
    l_->remove_node(nv.name);
    listed_nodes_.erase(nv.name);
  } else {
    l_->upsert_node(nv);
    listed_nodes_.insert(nv.name);
  }
}

void Controller::on_node_list(const ListView& lv) {
  std::unordered_set<std::string> seen;
  std::lock_guard<introspect::ProfiledMutex> g(l_->mu());
  for (size_t k = 0; k < lv.size(); ++k) {
    NodeView nv;
    if (!parse_node(lv.doc(k), lv.obj(k), l_->profile(), &nv)) continue;
    seen.insert(nv.name);
    l_->upsert_node(nv);
  }
  // Replace(): nodes this informer delivered before that are gone now
  for (const std::string& n : listed_nodes_) {
    if (seen.count(n) == 0) l_->remove_node(n);
  }
  listed_nodes_ = std::move(seen);
}

}  // namespace gsx
