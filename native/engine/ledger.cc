#include "ledger.h"

#include <algorithm>
#include <cstdio>

namespace gsx {

// ---------------------------------------------------------------- accounting

void Ledger::account(PodRec& r) {
  if (r.accounted) return;
  if (r.dev < 0 || r.terminal) return;
  auto it = nodes_.find(r.node);
  if (it == nodes_.end()) return;
  NodeState& n = it->second;
  if (r.dev >= static_cast<int64_t>(n.devs.size())) return;
  DevState& d = n.devs[static_cast<size_t>(r.dev)];
  d.used += r.mem;
  d.npods += 1;
  if (d.used > d.total) stats_.overcommit_events++;
  // a pod being moved between devices is charged on both until the move completes: never under-counted
  r.held_on = (r.hold >= 0 && r.hold != r.dev && r.hold < static_cast<int64_t>(n.devs.size())) ? r.hold : -1;
  if (r.held_on >= 0) {
    n.devs[static_cast<size_t>(r.held_on)].used += r.mem;
    n.devs[static_cast<size_t>(r.held_on)].held += r.mem;
  }
  r.moved_on = (r.move_to >= 0 && r.move_to != r.dev && r.move_to != r.held_on &&
                r.move_to < static_cast<int64_t>(n.devs.size()))
                   ? r.move_to
                   : -1;
  if (r.moved_on >= 0) n.devs[static_cast<size_t>(r.moved_on)].used += r.mem;
  r.accounted = true;
}

void Ledger::unaccount(PodRec& r) {
  if (!r.accounted) return;
  auto it = nodes_.find(r.node);
  r.accounted = false;
  if (it == nodes_.end()) return;
  NodeState& n = it->second;
  if (r.dev < 0 || r.dev >= static_cast<int64_t>(n.devs.size())) return;
  DevState& d = n.devs[static_cast<size_t>(r.dev)];
  d.used -= r.mem;
  d.npods -= 1;
  if (r.held_on >= 0 && r.held_on < static_cast<int64_t>(n.devs.size())) {
    n.devs[static_cast<size_t>(r.held_on)].used -= r.mem;
    n.devs[static_cast<size_t>(r.held_on)].held -= r.mem;
  }
  r.held_on = -1;
  if (r.moved_on >= 0 && r.moved_on < static_cast<int64_t>(n.devs.size())) {
    n.devs[static_cast<size_t>(r.moved_on)].used -= r.mem;
  }
  r.moved_on = -1;
}

void Ledger::rebuild(NodeState& n) {
  // nodeinfo.go:29-45: count devices, total/count each (homogeneous); the
  // per-device annotation, when it matches the count, is exact.
  n.devs.assign(static_cast<size_t>(n.count > 0 ? n.count : 0), DevState{});
  bool use_override = static_cast<int64_t>(n.dev_totals_override.size()) == n.count && n.count > 0;
  for (int64_t i = 0; i < n.count; ++i) {
    n.devs[static_cast<size_t>(i)].total =
        use_override ? n.dev_totals_override[static_cast<size_t>(i)] : (n.total / n.count);
  }
  for (const auto& uid : n.pods) {
    auto pit = pods_.find(uid);
    if (pit == pods_.end()) continue;
    pit->second.accounted = false;
    account(pit->second);
  }
}

bool Ledger::upsert_node(const NodeView& nv) {
  auto it = nodes_.find(nv.name);
  if (it == nodes_.end()) {
    NodeState n;
    n.name = nv.name;
    n.address = nv.address;
    n.total = nv.total;
    n.count = nv.count;
    n.dev_totals_override = nv.dev_totals;
    n.landing_order = nv.landing_order;
    n.publishes = nv.publishes;
    arm_publication_wait(n);
    // adopt pods that arrived before their node
    for (auto& kv : pods_) {
      if (kv.second.node == nv.name) n.pods.insert(kv.first);
    }
    auto res = nodes_.emplace(nv.name, std::move(n));
    rebuild(res.first->second);
    return true;
  }
  NodeState& n = it->second;
  n.address = nv.address;
  n.landing_order = nv.landing_order;
  if (nv.publishes != n.publishes) {
    n.publishes = nv.publishes;
    arm_publication_wait(n);
  }
  if (n.total == nv.total && n.count == nv.count && n.dev_totals_override == nv.dev_totals) return false;
  n.total = nv.total;
  n.count = nv.count;
  n.dev_totals_override = nv.dev_totals;
  rebuild(n);
  return true;
}

bool Ledger::remove_node(const std::string& name) {
  auto it = nodes_.find(name);
  if (it == nodes_.end()) return false;
  for (const auto& uid : it->second.pods) {
    auto pit = pods_.find(uid);
    if (pit != pods_.end()) pit->second.accounted = false;
  }
  nodes_.erase(it);
  return true;
}

bool Ledger::has_node(const std::string& name) const { return nodes_.count(name) != 0; }

// ---------------------------------------------------------------- pods

void Ledger::erase_pod(std::unordered_map<std::string, PodRec>::iterator it) {
  unaccount(it->second);
  auto nit = nodes_.find(it->second.node);
  if (nit != nodes_.end()) nit->second.pods.erase(it->first);
  pods_.erase(it);
}

int Ledger::upsert_pod(const PodView& v) {
  stats_.pod_upserts++;
  auto it = pods_.find(v.uid);
  if (v.node.empty()) {
    // cache.go:91-95 skips unscheduled pods.  An assumed reservation stays:
    // this is the annotation write racing ahead of the Binding.
    if (it != pods_.end() && it->second.assumed) return it->second.dev >= 0 ? 1 : 0;
    return 0;
  }
  if (it != pods_.end()) {
    PodRec& r = it->second;
    unaccount(r);
    if (r.node != v.node) {
      auto oit = nodes_.find(r.node);
      if (oit != nodes_.end()) oit->second.pods.erase(r.uid);
      r.node = v.node;
      auto nit = nodes_.find(r.node);
      if (nit != nodes_.end()) nit->second.pods.insert(r.uid);
    }
    r.ns = v.ns;
    r.name = v.name;
    r.request = v.request;
    r.terminal = v.terminal();
    r.deleting = v.deleting;
    if (v.dev_idx >= 0) {
      r.dev = v.dev_idx;
      r.mem = v.annot_mem;
      r.hold = v.hold_idx;
      if (r.move_to >= 0 && r.dev == r.move_to) r.move_to = -1;  // the move is confirmed
      r.assumed = false;  // observed with annotations: reservation confirmed
      r.unannotated = false;
    } else if (!r.assumed) {
      r.dev = -1;
    } else if (r.dev >= 0) {
      // our reservation, bound to its node, but the allocation annotations the Binding carried are missing:
      // the apiserver did not copy them (the reservation stays; the server writes them back)
      r.unannotated = true;
      queue_repair(r);
    }
    account(r);
    return r.dev >= 0 ? 1 : 0;
  }
  if (v.dev_idx < 0) return 0;  // nodeinfo.go:89-110 only adds pods with an idx
  PodRec r;
  r.uid = v.uid;
  r.ns = v.ns;
  r.name = v.name;
  r.node = v.node;
  r.dev = v.dev_idx;
  r.hold = v.hold_idx;
  r.mem = v.annot_mem;
  r.request = v.request;
  r.terminal = v.terminal();
  r.deleting = v.deleting;
  auto res = pods_.emplace(v.uid, std::move(r));
  auto nit = nodes_.find(v.node);
  if (nit != nodes_.end()) nit->second.pods.insert(v.uid);
  account(res.first->second);
  return 1;
}

bool Ledger::remove_pod(const std::string& uid) {
  auto it = pods_.find(uid);
  if (it == pods_.end()) return false;
  stats_.pod_removes++;
  erase_pod(it);
  return true;
}

bool Ledger::known(const std::string& uid) const { return pods_.count(uid) != 0; }

int Ledger::pod_state(const std::string& uid, int64_t* dev) const {
  auto it = pods_.find(uid);
  if (it == pods_.end()) {
    *dev = -1;
    return 0;
  }
  *dev = it->second.dev;
  return it->second.assumed ? 2 : 1;
}

// ---------------------------------------------------------------- verbs

Check Ledger::check(const std::string& node, int64_t req) const {
  auto it = nodes_.find(node);
  if (it == nodes_.end()) return Check::NodeNotFound;
  const NodeState& n = it->second;
  if (!n.gpushare()) return Check::NotGPUShare;
  for (size_t i = 0; i < n.devs.size(); ++i) {
    if (n.free_of(i) >= req) return Check::Ok;
  }
  return Check::Insufficient;
}

int64_t Ledger::assume(const std::string& uid, const std::string& ns, const std::string& name,
                       const std::string& node, int64_t req, int64_t* dev_total) {
  auto nit = nodes_.find(node);
  if (nit == nodes_.end()) {
    stats_.assume_fail++;
    return -2;
  }
  NodeState& n = nit->second;
  if (!n.gpushare()) {
    stats_.assume_fail++;
    return -3;
  }
  auto pit = pods_.find(uid);
  if (pit != pods_.end()) {
    PodRec& r = pit->second;
    if (r.assumed && !r.bound) {
      stats_.assume_fail++;
      return -4;
    }
    if (r.node == node && r.dev >= 0 && r.dev < static_cast<int64_t>(n.devs.size()) && !r.terminal) {
      // idempotent re-bind of an already placed pod: keep its record as is
      if (dev_total) *dev_total = n.devs[static_cast<size_t>(r.dev)].total;
      stats_.assume_ok++;
      return r.dev;
    }
    erase_pod(pit);
  }
  // best fit: smallest free >= req, lowest index on ties (nodeinfo.go:219-232)
  int64_t cand = -1;
  int64_t cand_free = 0;
  for (size_t i = 0; i < n.devs.size(); ++i) {
    int64_t free = n.free_of(i);
    if (free >= req && (cand < 0 || free < cand_free)) {
      cand = static_cast<int64_t>(i);
      cand_free = free;
    }
  }
  if (cand < 0 || req <= 0) {
    // nodeinfo.go:218: a pod with no gpu-mem request is never placed
    stats_.assume_fail++;
    return -1;
  }
  PodRec r;
  r.uid = uid;
  r.ns = ns;
  r.name = name;
  r.node = node;
  r.dev = cand;
  r.mem = req;
  r.request = req;
  r.assumed = true;
  r.assumed_at = now_s();
  auto res = pods_.emplace(uid, std::move(r));
  n.pods.insert(uid);
  account(res.first->second);
  if (dev_total) *dev_total = n.devs[static_cast<size_t>(cand)].total;
  stats_.assume_ok++;
  return cand;
}

int64_t Ledger::assume_ordered(const std::string& uid, const std::string& ns, const std::string& name,
                               const std::string& node, int64_t req, int64_t* dev_total, uint64_t* seq,
                               int64_t* assume_ns, const std::string& cu_count) {
  int64_t dev = assume(uid, ns, name, node, req, dev_total);
  if (dev < 0) return dev;
  int64_t now = std::chrono::duration_cast<std::chrono::nanoseconds>(
                    std::chrono::system_clock::now().time_since_epoch()).count();
  std::lock_guard<std::mutex> o(order_mu_);
  last_assume_ns_ = std::max(now, last_assume_ns_ + 1);  // strictly increasing in assume order
  *assume_ns = last_assume_ns_;
  auto pit = pods_.find(uid);
  if (pit != pods_.end()) pit->second.assume_ns = last_assume_ns_;
  *seq = ++order_seq_;
  inflight_.push_back(InflightBind{node, req, dev, *seq, cu_count, node_ordered_locked(node)});
  return dev;
}

bool Ledger::node_ordered_locked(const std::string& node) const {
  switch (order_mode()) {
    case kOrderStrict:
      return true;
    case kOrderRelaxed:
      return false;
    default: {
      auto it = nodes_.find(node);
      return it == nodes_.end() || !it->second.landing_order;
    }
  }
}

bool Ledger::blocked_locked(const InflightBind& me) const {
  if (!me.ordered) return false;
  for (const auto& f : inflight_) {
    if (f.seq < me.seq && f.node == me.node && f.size == me.size && (f.dev != me.dev || f.cu_count != me.cu_count)) {
      return true;
    }
  }
  return false;
}

bool Ledger::bind_blocked(uint64_t seq) {
  std::lock_guard<std::mutex> o(order_mu_);
  for (const auto& f : inflight_) {
    if (f.seq == seq) return blocked_locked(f);
  }
  return false;
}

void Ledger::bind_wait(uint64_t seq, const std::atomic<bool>* stop) {
  std::unique_lock<std::mutex> o(order_mu_);
  // the entry is looked up by seq after every wake, never kept across one: bind_leave(seq) may run while we
  // sleep (a cancelled Python caller's cleanup) and free it; then nobody references our cv any more
  auto find = [this, seq]() -> InflightBind* {
    for (auto& f : inflight_) {
      if (f.seq == seq) return &f;
    }
    return nullptr;
  };
  InflightBind* me = find();
  if (!me || !blocked_locked(*me)) return;
  order_waits_.fetch_add(1, std::memory_order_relaxed);
  auto t0 = std::chrono::steady_clock::now();
  // a condition variable of our own: bind_leave() wakes exactly the binds it unblocks (a shared one woke
  // every waiter of the node on every completed bind, and they queued for the extender's CPUs to re-check)
  std::condition_variable cv;
  me->waiter = &cv;
  while (true) {
    me = find();
    if (me == nullptr) break;  // left while we waited: the entry (and its pointer to cv) is gone
    if (!blocked_locked(*me) || (stop && stop->load())) {
      me->waiter = nullptr;
      break;
    }
    cv.wait_for(o, std::chrono::milliseconds(100));  // timeout: notice `stop`
  }
  uint64_t ns = static_cast<uint64_t>(
      std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count());
  order_wait_ns_.fetch_add(ns, std::memory_order_relaxed);
  uint64_t cur = order_wait_max_ns_.load(std::memory_order_relaxed);
  while (ns > cur && !order_wait_max_ns_.compare_exchange_weak(cur, ns, std::memory_order_relaxed)) {
  }
}

void Ledger::bind_leave(uint64_t seq) {
  std::lock_guard<std::mutex> o(order_mu_);
  for (const auto& f : inflight_) {
    // a waiter still blocked on the entry being removed (its caller gave up): wake it so it sees it is gone
    if (f.seq == seq && f.waiter) f.waiter->notify_one();
  }
  inflight_.remove_if([seq](const InflightBind& f) { return f.seq == seq; });
  // notify under order_mu_: a waiter's cv lives on its stack until it has re-taken the mutex
  for (const auto& f : inflight_) {
    if (f.waiter && !blocked_locked(f)) f.waiter->notify_one();
  }
}

void Ledger::finish_bind(const std::string& uid, bool ok, double ttl_s) {
  auto it = pods_.find(uid);
  if (it == pods_.end()) return;
  if (!ok) {
    stats_.bind_fail++;
    if (it->second.assumed) erase_pod(it);
    return;
  }
  stats_.bind_ok++;
  it->second.bound = true;
  it->second.bound_at = now_s();
  it->second.deadline = it->second.bound_at + ttl_s;
  if (it->second.unannotated) queue_repair(it->second);  // the watch event raced the binding's response
}

int Ledger::begin_move(MoveRequest* m, std::string* why) {
  auto pit = pods_.find(m->uid);
  if (pit == pods_.end() || pit->second.node != m->node || pit->second.terminal || pit->second.dev < 0) {
    *why = "pod " + m->uid + " is not bound to node " + m->node + " in the extender's ledger";
    stats_.moves_refused++;
    return 1;
  }
  PodRec& r = pit->second;
  if ((r.assumed && !r.bound) || r.move_to >= 0) {
    *why = "a bind or another move of the pod is in flight";
    stats_.moves_refused++;
    return 4;
  }
  if (r.dev != m->from) {
    *why = "stale: the ledger has the pod on GPU " + std::to_string(r.dev) + ", not " + std::to_string(m->from);
    stats_.moves_refused++;
    return 2;
  }
  NodeState& n = nodes_.at(r.node);
  const int64_t ndev = static_cast<int64_t>(n.devs.size());
  if (m->to < 0) {  // best fit among the other devices (nodeinfo.go:209-252)
    int64_t best = -1, best_free = 0;
    for (int64_t i = 0; i < ndev; ++i) {
      const int64_t free = n.free_of(static_cast<size_t>(i));
      if (i != m->from && free >= r.mem && (best < 0 || free < best_free)) {
        best = i;
        best_free = free;
      }
    }
    m->to = best;
  }
  if (m->to < 0 || m->to >= ndev) {
    *why = "no GPU of node " + m->node + " has room for " + std::to_string(r.mem);
    stats_.moves_refused++;
    return 3;
  }
  if (m->to != r.dev) {
    // An exchange with a partner the ledger can verify:
    //  step 1 -- Q is on `to`, and this write charges the pod on `from` too (hold-idx = from) and names Q as
    //            the hold's partner: Q will take `from` in step 2;
    //  step 2 -- Q (the partner named here) already took this pod's GPU and holds `to` until this lands (or, before
    //            the informer has seen step 1 land, Q is still on `to` with its move to this pod's GPU charged).
    // An exchange only relabels who runs where, so it is checked on `to`'s final annotation sum (the holds on
    // `to` go, a partner still on `to` leaves) and never refused when it adds no load there (the reference's
    // equal-size exchange).  Any other move also counts the device plugin's unaccounted use.
    const DevState& d = n.devs[static_cast<size_t>(m->to)];
    const size_t ti = static_cast<size_t>(m->to);
    bool exchange = false;
    int64_t partner_mem = 0, leaving = 0;
    if (!m->partner.empty() && m->partner != m->uid) {
      auto q = pods_.find(m->partner);
      if (q != pods_.end() && q->second.node == r.node && !q->second.terminal) {
        const PodRec& Q = q->second;
        const bool step1 = Q.dev == m->to && m->req_hold == r.dev && m->req_hold_partner == m->partner;
        const bool step2_seen = Q.hold == m->to && Q.dev == r.dev;
        const bool step2_early = Q.dev == m->to && Q.move_to == r.dev;
        exchange = step1 || step2_seen || step2_early;
        partner_mem = Q.mem;
        leaving = (step1 || step2_early) ? Q.mem : 0;  // step 2 seen: Q's charge on `to` is its hold (in `held`)
      }
      if (!exchange) stats_.partner_claims_refused++;
    }
    bool fits;
    if (exchange) {
      fits = r.mem <= partner_mem || d.used - d.held - leaving + r.mem <= d.total;
    } else {
      // after the move: the annotations gain the pod; if its container already runs there, its share leaves the
      // unaccounted use it was part of
      const int64_t ex = ti < n.extra.size() ? n.extra[ti] : 0;
      fits = d.used + r.mem + (m->physical_on_to ? std::max<int64_t>(0, ex - r.mem) : ex) <= d.total;
    }
    if (!fits) {
      *why = "GPU " + std::to_string(m->to) + " of node " + m->node + " has " + std::to_string(n.free_of(ti)) +
             " free" + (exchange ? " (" + std::to_string(leaving) + " leaving)" : std::string()) +
             ", the pod needs " + std::to_string(r.mem);
      stats_.moves_refused++;
      return 3;
    }
    unaccount(r);
    r.move_to = m->to;
    r.move_at = now_s();
    account(r);
  }
  return 0;
}

void Ledger::end_move(const std::string& uid, bool ok) {
  auto pit = pods_.find(uid);
  if (pit == pods_.end()) return;
  PodRec& r = pit->second;
  if (ok) {
    stats_.moves_ok++;
    return;  // the target stays charged until the informer shows the pod there
  }
  stats_.moves_failed++;
  if (r.move_to < 0) return;
  unaccount(r);
  r.move_to = -1;
  account(r);
}

void Ledger::queue_repair(PodRec& r) {
  if (!r.bound || r.repair_queued || r.dev < 0) return;
  r.repair_queued = true;
  stats_.annotations_missing++;
  AnnotationRepair a;
  a.uid = r.uid;
  a.ns = r.ns;
  a.name = r.name;
  a.node = r.node;
  a.dev = r.dev;
  a.mem = r.mem;
  a.assume_ns = r.assume_ns;
  auto nit = nodes_.find(r.node);
  if (nit != nodes_.end() && r.dev < static_cast<int64_t>(nit->second.devs.size())) {
    a.dev_total = nit->second.devs[static_cast<size_t>(r.dev)].total;
  }
  repairs_.push_back(std::move(a));
}

std::vector<AnnotationRepair> Ledger::drain_repairs() {
  std::vector<AnnotationRepair> out;
  out.swap(repairs_);
  return out;
}

int Ledger::gc(double confirmed_list_start, bool* need_relist) {
  double now = now_s();
  int n = 0;
  bool relist = false;
  for (auto& kv : nodes_) {
    // an unaccounted-use publication its device plugin stopped refreshing (the plugin is gone): annotations only
    if (!kv.second.extra.empty() && kv.second.extra_until < now) {
      kv.second.extra.clear();
      stats_.unaccounted_expired++;
    }
  }
  for (auto& kv : pods_) {
    // a move the informer never confirmed (the pod's record was rewritten again since): its target charge goes
    PodRec& r = kv.second;
    if (r.move_to >= 0 && now - r.move_at > 30.0) {
      unaccount(r);
      r.move_to = -1;
      account(r);
    }
  }
  for (auto it = pods_.begin(); it != pods_.end();) {
    const PodRec& r = it->second;
    bool expire = false;
    if (r.assumed && r.bound && r.unannotated) {
      // seen bound on its node (only the annotations are missing): never expired, the repair confirms it
    } else if (r.assumed && r.bound && r.deadline < now) {
      // overdue: only a LIST begun after the binding was written can prove the binding absent
      if (confirmed_list_start > r.bound_at) {
        expire = true;
      } else {
        relist = true;
        stats_.expiry_deferred++;
      }
    } else if (r.assumed && !r.bound && now - r.assumed_at > 600.0) {
      expire = true;  // a bind that never finished (crashed worker)
    }
    if (expire) {
      auto cur = it++;
      erase_pod(cur);
      ++n;
    } else {
      ++it;
    }
  }
  stats_.expired += static_cast<uint64_t>(n);
  if (need_relist) *need_relist = relist;
  return n;
}

// ---------------------------------------------------------------- inspect

bool Ledger::set_unaccounted(const std::string& node, const std::vector<int64_t>& extra, double ttl_s) {
  auto it = nodes_.find(node);
  if (it == nodes_.end()) return false;
  it->second.extra = extra;
  it->second.extra_until = extra.empty() ? 0 : now_s() + ttl_s;
  it->second.published = true;
  it->second.pub_wait_until = 0;
  stats_.unaccounted_updates++;
  return true;
}

void Ledger::arm_publication_wait(NodeState& n) {
  n.pub_wait_until = (n.publishes && !n.published && pub_hold_s_ > 0) ? now_s() + pub_hold_s_ : 0;
}

void Ledger::begin_epoch(double hold_s) {
  pub_hold_s_ = hold_s > 0 ? hold_s : 0;
  for (auto& kv : nodes_) {
    kv.second.published = false;
    arm_publication_wait(kv.second);
  }
}

double Ledger::publication_wait(const std::string& node) const {
  auto it = nodes_.find(node);
  if (it == nodes_.end() || it->second.pub_wait_until <= 0) return 0;
  const double left = it->second.pub_wait_until - now_s();
  return left > 0 ? left : 0;
}

std::vector<int64_t> Ledger::node_unaccounted(const std::string& node) const {
  auto it = nodes_.find(node);
  return it == nodes_.end() ? std::vector<int64_t>() : it->second.extra;
}

std::vector<std::pair<int64_t, int64_t>> Ledger::node_devices(const std::string& node) const {
  std::vector<std::pair<int64_t, int64_t>> out;
  auto it = nodes_.find(node);
  if (it == nodes_.end()) return out;
  for (const DevState& d : it->second.devs) out.emplace_back(d.total, d.used);
  return out;
}

std::vector<std::string> Ledger::node_names() const {
  std::vector<std::string> out;
  out.reserve(nodes_.size());
  for (const auto& kv : nodes_) out.push_back(kv.first);
  return out;
}

namespace {
void append_int(std::string* o, int64_t v) {
  char buf[32];
  int n = std::snprintf(buf, sizeof(buf), "%lld", static_cast<long long>(v));
  o->append(buf, static_cast<size_t>(n));
}
}  // namespace

std::string Ledger::inspect_json(const std::string& node, bool* found) const {
  // Schema of pkg/scheduler/gpushare-inspect.go:14-38 (lowercase tags).
  std::string o;
  o.reserve(256);
  o.append("{\"nodes\":[");
  bool first_node = true;
  *found = true;
  auto emit = [&](const NodeState& n) {
    if (!first_node) o.push_back(',');
    first_node = false;
    // per-device pod lists, sorted for determinism
    std::vector<std::vector<const PodRec*>> per(n.devs.size());
    for (const auto& uid : n.pods) {
      auto pit = pods_.find(uid);
      if (pit == pods_.end()) continue;
      const PodRec& r = pit->second;
      if (r.dev < 0 || r.dev >= static_cast<int64_t>(n.devs.size())) continue;
      if (r.deleting || r.terminal) continue;  // AssignedNonTerminatedPod
      per[static_cast<size_t>(r.dev)].push_back(&r);
    }
    int64_t used_total = 0;
    for (const DevState& d : n.devs) used_total += d.used;
    o.append("{\"name\":");
    json::append_quoted(&o, n.name);
    o.append(",\"totalGPU\":");
    append_int(&o, n.total);
    o.append(",\"usedGPU\":");
    append_int(&o, used_total);
    o.append(",\"devs\":[");
    for (size_t i = 0; i < n.devs.size(); ++i) {
      if (i) o.push_back(',');
      o.append("{\"id\":");
      append_int(&o, static_cast<int64_t>(i));
      o.append(",\"totalGPU\":");
      append_int(&o, n.devs[i].total);
      o.append(",\"usedGPU\":");
      append_int(&o, n.devs[i].used);
      o.append(",\"pods\":[");
      auto& lst = per[i];
      std::sort(lst.begin(), lst.end(), [](const PodRec* a, const PodRec* b) {
        return a->ns != b->ns ? a->ns < b->ns : a->name < b->name;
      });
      for (size_t k = 0; k < lst.size(); ++k) {
        if (k) o.push_back(',');
        o.append("{\"name\":");
        json::append_quoted(&o, lst[k]->name);
        o.append(",\"namespace\":");
        json::append_quoted(&o, lst[k]->ns);
        o.append(",\"usedGPU\":");
        append_int(&o, lst[k]->request);
        o.push_back('}');
      }
      o.append("]}");
    }
    o.append("]}");
  };
  std::string err;
  if (node.empty()) {
    for (const auto& kv : nodes_) emit(kv.second);
  } else {
    auto it = nodes_.find(node);
    if (it == nodes_.end()) {
      *found = false;
      err = "node \"" + node + "\" not found";
    } else {
      emit(it->second);
    }
  }
  o.push_back(']');
  if (!err.empty()) {
    o.append(",\"error\":");
    json::append_quoted(&o, err);
  }
  o.push_back('}');
  return o;
}

// ---------------------------------------------------------------- pending pods

void Ledger::remember_pending(const std::string& uid, PendingPod p) {
  auto it = pending_.find(uid);
  if (it != pending_.end()) {
    it->second = std::move(p);
    return;
  }
  constexpr size_t kMax = 65536;
  while (pending_.size() >= kMax && !pending_order_.empty()) {
    pending_.erase(pending_order_.front());
    pending_order_.pop_front();
  }
  pending_.emplace(uid, std::move(p));
  pending_order_.push_back(uid);
  if (pending_order_.size() > 2 * pending_.size() + 1024) {
    // drop ids already forgotten (bound pods) so the order queue stays proportional to the live set; each pass
    // removes at least half the queue, so the cost is amortised O(1) per pod
    std::deque<std::string> keep;
    for (auto& u : pending_order_) {
      if (pending_.count(u)) keep.push_back(u);
    }
    pending_order_.swap(keep);
  }
}

bool Ledger::pending(const std::string& uid, PendingPod* out) const {
  auto it = pending_.find(uid);
  if (it == pending_.end()) return false;
  *out = it->second;
  return true;
}

void Ledger::forget_pending(const std::string& uid) { pending_.erase(uid); }

// ---------------------------------------------------------------- filter verb

std::string filter_body(Ledger& l, std::string_view body) {
  l.mutable_stats().filter_calls++;
  json::Doc d;
  std::string err;
  auto error_result = [](const std::string& e) {
    std::string o("{\"Nodes\":null,\"NodeNames\":null,\"FailedNodes\":null,\"Error\":");
    json::append_quoted(&o, e);
    o.push_back('}');
    return o;
  };
  if (!d.parse(body, &err)) return error_result(err);
  if (d.at(0).type != json::T::Object) {
    return error_result("json: cannot unmarshal value into Go value of type api.ExtenderArgs");
  }
  int64_t pod = d.find(0, "Pod", true);
  if (pod < 0 || d.at(static_cast<uint32_t>(pod)).type != json::T::Object) {
    return error_result("ExtenderArgs.Pod is required");
  }
  const Profile& p = l.profile();
  int64_t req = pod_limits_sum(d, static_cast<uint32_t>(pod), p.resource);
  {
    int64_t u = d.path(static_cast<uint32_t>(pod), {"metadata", "uid"});
    if (u >= 0 && d.at(static_cast<uint32_t>(u)).type == json::T::String) {
      Ledger::PendingPod pp;
      int64_t nm = d.path(static_cast<uint32_t>(pod), {"metadata", "name"});
      int64_t ns = d.path(static_cast<uint32_t>(pod), {"metadata", "namespace"});
      if (nm >= 0) pp.name = d.str(static_cast<uint32_t>(nm));
      pp.ns = ns >= 0 ? d.str(static_cast<uint32_t>(ns)) : std::string("default");
      pp.req = req;
      int64_t cu = d.path(static_cast<uint32_t>(pod), {"metadata", "annotations", kCuCountAnnotation});
      if (cu >= 0 && d.at(static_cast<uint32_t>(cu)).type == json::T::String) pp.cu_count = d.str(static_cast<uint32_t>(cu));
      int64_t rv = d.path(static_cast<uint32_t>(pod), {"metadata", "resourceVersion"});
      if (rv >= 0 && d.at(static_cast<uint32_t>(rv)).type == json::T::String) pp.rv = d.str(static_cast<uint32_t>(rv));
      l.remember_pending(d.str(static_cast<uint32_t>(u)), std::move(pp));
    }
  }

  // Candidate nodes: NodeNames (nodeCacheCapable) or Nodes.items.
  struct Cand {
    std::string name;
    int64_t item = -1;  // tape index of the v1.Node when given as NodeList
  };
  std::vector<Cand> cands;
  bool by_names = false, by_nodes = false;
  int64_t names = d.find(0, "NodeNames", true);
  if (names >= 0 && d.at(static_cast<uint32_t>(names)).type == json::T::Array) {
    by_names = true;
    uint32_t end = d.at(static_cast<uint32_t>(names)).skip;
    for (uint32_t i = static_cast<uint32_t>(names) + 1; i < end; i = d.next(i)) {
      cands.push_back(Cand{d.str(i), -1});
    }
  }
  int64_t nodes = d.find(0, "Nodes", true);
  if (!by_names && nodes >= 0 && d.at(static_cast<uint32_t>(nodes)).type == json::T::Object) {
    int64_t items = d.find(static_cast<uint32_t>(nodes), "items");
    if (items >= 0 && d.at(static_cast<uint32_t>(items)).type == json::T::Array) {
      by_nodes = true;
      uint32_t end = d.at(static_cast<uint32_t>(items)).skip;
      for (uint32_t i = static_cast<uint32_t>(items) + 1; i < end; i = d.next(i)) {
        std::string nm;
        int64_t m = d.path(i, {"metadata", "name"});
        if (m >= 0) nm = d.str(static_cast<uint32_t>(m));
        cands.push_back(Cand{nm, static_cast<int64_t>(i)});
      }
    }
  }

  std::vector<const Cand*> ok;
  std::vector<std::pair<std::string, std::string>> failed;
  ok.reserve(cands.size());
  for (const Cand& c : cands) {
    Check r = l.check(c.name, req);
    switch (r) {
      case Check::Ok:
        ok.push_back(&c);
        break;
      case Check::NodeNotFound:
        failed.emplace_back(c.name, "node \"" + c.name + "\" not found");
        break;
      case Check::NotGPUShare:
        failed.emplace_back(c.name, "The node " + c.name + " is not for GPU share, need skip");
        break;
      case Check::Insufficient:
        failed.emplace_back(c.name, "Insufficient GPU Memory in one device");
        break;
    }
  }
  l.mutable_stats().filter_nodes_ok += ok.size();
  l.mutable_stats().filter_nodes_failed += failed.size();
  // Go marshals map keys sorted; duplicates collapse (last wins).
  std::stable_sort(failed.begin(), failed.end(),
                   [](const auto& a, const auto& b) { return a.first < b.first; });

  std::string o;
  o.reserve(64 + 24 * cands.size());
  o.append("{\"Nodes\":");
  if (by_nodes) {
    o.append("{\"metadata\":{},\"items\":[");
    for (size_t i = 0; i < ok.size(); ++i) {
      if (i) o.push_back(',');
      o.append(d.raw(static_cast<uint32_t>(ok[i]->item)));
    }
    o.append("]}");
  } else {
    o.append("null");
  }
  o.append(",\"NodeNames\":");
  if (by_names || by_nodes) {
    o.push_back('[');
    for (size_t i = 0; i < ok.size(); ++i) {
      if (i) o.push_back(',');
      json::append_quoted(&o, ok[i]->name);
    }
    o.push_back(']');
  } else {
    o.append("[]");
  }
  o.append(",\"FailedNodes\":{");
  bool first = true;
  for (size_t i = 0; i < failed.size(); ++i) {
    if (i + 1 < failed.size() && failed[i + 1].first == failed[i].first) continue;
    if (!first) o.push_back(',');
    first = false;
    json::append_quoted(&o, failed[i].first);
    o.push_back(':');
    json::append_quoted(&o, failed[i].second);
  }
  o.append("},\"Error\":\"\"}");
  return o;
}

}  // namespace gsx

namespace gsx {

// ---------------------------------------------------------------- prioritize verb (ours)
//
// The reference registers only filter + bind (config/scheduler-policy-config.json:7-8),
// so kube-scheduler spreads gpushare pods across nodes by its default scores
// and binpacking happens only inside a node.  This verb scores every node by
// how tightly the pod would fit its best-fit device: 10 = exact fit, 0 = does
// not fit / empty device of a node that has a partly used one elsewhere, so
// "binpack-first" also holds across nodes.  Wire format: HostPriorityList
// [{"Host": name, "Score": 0..10}] (kube-scheduler extender API).
std::string prioritize_body(Ledger& l, std::string_view body) {
  json::Doc d;
  std::string err;
  if (!d.parse(body, &err) || d.at(0).type != json::T::Object) return "[]";
  int64_t pod = d.find(0, "Pod", true);
  if (pod < 0 || d.at(static_cast<uint32_t>(pod)).type != json::T::Object) return "[]";
  int64_t req = pod_limits_sum(d, static_cast<uint32_t>(pod), l.profile().resource);
  std::vector<std::string> names;
  int64_t nn = d.find(0, "NodeNames", true);
  if (nn >= 0 && d.at(static_cast<uint32_t>(nn)).type == json::T::Array) {
    uint32_t end = d.at(static_cast<uint32_t>(nn)).skip;
    for (uint32_t i = static_cast<uint32_t>(nn) + 1; i < end; i = d.next(i)) names.push_back(d.str(i));
  } else {
    int64_t nodes = d.find(0, "Nodes", true);
    if (nodes >= 0 && d.at(static_cast<uint32_t>(nodes)).type == json::T::Object) {
      int64_t items = d.find(static_cast<uint32_t>(nodes), "items");
      if (items >= 0 && d.at(static_cast<uint32_t>(items)).type == json::T::Array) {
        uint32_t end = d.at(static_cast<uint32_t>(items)).skip;
        for (uint32_t i = static_cast<uint32_t>(items) + 1; i < end; i = d.next(i)) {
          int64_t m = d.path(i, {"metadata", "name"});
          names.push_back(m >= 0 ? d.str(static_cast<uint32_t>(m)) : std::string());
        }
      }
    }
  }
  std::string o("[");
  for (size_t k = 0; k < names.size(); ++k) {
    int64_t score = 0;
    const NodeState* n = l.node(names[k]);
    if (n && n->gpushare() && req > 0) {
      int64_t best = -1, best_total = 1;
      for (size_t di = 0; di < n->devs.size(); ++di) {
        const DevState& dv = n->devs[di];
        int64_t left = n->free_of(di) - req;
        if (left >= 0 && (best < 0 || left < best)) {
          best = left;
          best_total = dv.total > 0 ? dv.total : 1;
        }
      }
      if (best >= 0) score = 10 - (10 * best + best_total - 1) / best_total;  // ceil: only an exact fit scores 10
      if (score < 0) score = 0;
    }
    if (k) o.push_back(',');
    o.append("{\"Host\":");
    json::append_quoted(&o, names[k]);
    o.append(",\"Score\":");
    o.append(std::to_string(score));
    o.push_back('}');
  }
  o.push_back(']');
  return o;
}

}  // namespace gsx
