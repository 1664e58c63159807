#include "allocstate.h"

#include <chrono>
#include <unordered_set>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <stdexcept>
#include <tuple>

#include "quantity.h"

namespace gsx {

// ---------------------------------------------------------------- CU partitions

CuPartitioner::CuPartitioner(int cu, int xcc) : cu_(cu), xcc_(std::max(1, xcc)), owner_(static_cast<size_t>(cu)) {}

bool CuPartitioner::allocate(const std::string& uid, int n, std::vector<int>* out, std::string* err) {
  auto h = held_.find(uid);
  if (h != held_.end() && !h->second.empty()) {
    *out = h->second;
    return true;
  }
  if (n <= 0 || n > cu_) {
    *err = "invalid CU partition size " + std::to_string(n);
    return false;
  }
  const int per = cu_ / xcc_;
  std::vector<int> got;
  for (int i = 0; i < per && static_cast<int>(got.size()) < n; ++i) {
    for (int x = 0; x < xcc_ && static_cast<int>(got.size()) < n; ++x) {
      int c = x * per + i;
      if (owner_[static_cast<size_t>(c)].empty()) got.push_back(c);
    }
  }
  if (static_cast<int>(got.size()) < n) {
    int free = free_count();
    *err = "only " + std::to_string(free) + " CUs free, " + std::to_string(n) + " requested";
    return false;
  }
  std::sort(got.begin(), got.end());
  for (int c : got) owner_[static_cast<size_t>(c)] = uid;
  held_[uid] = got;
  *out = got;
  return true;
}

int CuPartitioner::release(const std::string& uid) {
  auto h = held_.find(uid);
  if (h == held_.end()) return 0;
  int n = static_cast<int>(h->second.size());
  for (int c : h->second) owner_[static_cast<size_t>(c)].clear();
  held_.erase(h);
  return n;
}

std::vector<int> CuPartitioner::adopt(const std::string& uid, const std::vector<int>& cus) {
  std::vector<int> clash, got;
  std::vector<int> sorted(cus);
  std::sort(sorted.begin(), sorted.end());
  sorted.erase(std::unique(sorted.begin(), sorted.end()), sorted.end());
  for (int c : sorted) {
    if (c < 0 || c >= cu_) continue;
    std::string& o = owner_[static_cast<size_t>(c)];
    if (!o.empty() && o != uid) {
      clash.push_back(c);
      continue;
    }
    o = uid;
    got.push_back(c);
  }
  if (!got.empty()) {
    std::vector<int>& mine = held_[uid];
    mine.insert(mine.end(), got.begin(), got.end());
    std::sort(mine.begin(), mine.end());
    mine.erase(std::unique(mine.begin(), mine.end()), mine.end());
  }
  return clash;
}

void CuPartitioner::swap_owners(const std::string& a, const std::string& b) {
  if (a == b) return;
  std::vector<int> pa, pb;
  auto ia = held_.find(a);
  if (ia != held_.end()) {
    pa = std::move(ia->second);
    held_.erase(ia);
  }
  auto ib = held_.find(b);
  if (ib != held_.end()) {
    pb = std::move(ib->second);
    held_.erase(ib);
  }
  for (int c : pa) owner_[static_cast<size_t>(c)] = b;
  for (int c : pb) owner_[static_cast<size_t>(c)] = a;
  if (!pa.empty()) held_[b] = std::move(pa);
  if (!pb.empty()) held_[a] = std::move(pb);
}

std::vector<int> CuPartitioner::held_by(const std::string& uid) const {
  auto h = held_.find(uid);
  return h == held_.end() ? std::vector<int>() : h->second;
}

int CuPartitioner::free_count() const {
  int n = 0;
  for (const auto& o : owner_) n += o.empty() ? 1 : 0;
  return n;
}

std::string cu_words(const std::vector<int>& cus, int cu_count) {
  std::vector<uint32_t> w(static_cast<size_t>((cu_count + 31) / 32), 0);
  for (int c : cus) {
    if (c >= 0 && c < cu_count) w[static_cast<size_t>(c / 32)] |= 1u << (c % 32);
  }
  std::string o;
  char b[16];
  for (size_t i = 0; i < w.size(); ++i) {
    std::snprintf(b, sizeof(b), "%s0x%08x", i ? "," : "", w[i]);
    o.append(b);
  }
  return o;
}

std::vector<int> parse_cu_words(const std::string& words) {
  std::vector<int> out;
  size_t i = 0;
  int wi = 0;
  while (i < words.size()) {
    size_t j = words.find(',', i);
    if (j == std::string::npos) j = words.size();
    std::string tok = words.substr(i, j - i);
    size_t a = tok.find_first_not_of(" \t"), b = tok.find_last_not_of(" \t");
    if (a != std::string::npos) {
      tok = tok.substr(a, b - a + 1);
      char* end = nullptr;
      unsigned long v = std::strtoul(tok.c_str(), &end, 16);
      if (end == tok.c_str() || *end != '\0') throw std::invalid_argument("bad CU mask word: " + tok);
      for (int bit = 0; bit < 32; ++bit) {
        if (v >> bit & 1ul) out.push_back(32 * wi + bit);
      }
      ++wi;
    }
    i = j + 1;
  }
  return out;
}

std::string cu_ranges(const std::vector<int>& in) {
  std::vector<int> cus(in);
  std::sort(cus.begin(), cus.end());
  std::string o;
  size_t i = 0;
  while (i < cus.size()) {
    size_t j = i;
    while (j + 1 < cus.size() && cus[j + 1] == cus[j] + 1) ++j;
    if (!o.empty()) o.push_back(',');
    o.append(std::to_string(cus[i]));
    if (j > i) o.append("-").append(std::to_string(cus[j]));
    i = j + 1;
  }
  return o;
}

// ---------------------------------------------------------------- pods from the informer

bool parse_alloc_pod(const json::Doc& d, uint32_t pod, const Profile& p, AllocPod* out) {
  PodView v;
  if (!parse_pod(d, pod, p, &v)) return false;
  out->uid = v.uid;
  out->ns = v.ns;
  out->name = v.name;
  out->key = v.ns.empty() ? v.name : v.ns + "/" + v.name;
  out->rv = v.rv;
  out->phase = v.phase;
  out->node = v.node;
  out->dev = v.dev_idx;
  out->request = v.request;
  out->assume_time = v.assume_time;
  out->dev_total = v.annot_dev_total;
  out->complete = v.complete();
  out->terminating = v.deleting && !v.terminal();
  int64_t gp = d.path(pod, {"metadata", "deletionGracePeriodSeconds"});
  int64_t gv = -1;
  out->grace_s = (gp >= 0 && d.as_int(static_cast<uint32_t>(gp), &gv)) ? static_cast<double>(gv) : -1.0;
  int64_t tg = d.path(pod, {"spec", "terminationGracePeriodSeconds"});
  int64_t tv = 0;
  out->term_grace_s = (tg >= 0 && d.as_int(static_cast<uint32_t>(tg), &tv) && tv >= 0) ? static_cast<double>(tv) : 0.0;
  out->cu_mask = v.cu_mask;
  out->hold_idx = v.hold_idx;
  out->assigned.clear();
  out->cu_count = 0;
  out->hold_partner.clear();
  int64_t an = d.path(pod, {"metadata", "annotations"});
  if (an >= 0 && d.at(static_cast<uint32_t>(an)).type == json::T::Object) {
    uint32_t a = static_cast<uint32_t>(an);
    int64_t i = d.find(a, p.a_assigned);
    if (i >= 0) out->assigned = d.str(static_cast<uint32_t>(i));
    i = d.find(a, "gpushare.amd.com/cu-count");
    if (i >= 0) out->cu_count = std::atoi(d.str(static_cast<uint32_t>(i)).c_str());
    i = d.find(a, "gpushare.amd.com/hold-partner");
    if (i >= 0) out->hold_partner = d.str(static_cast<uint32_t>(i));
  }
  int64_t ct = d.path(pod, {"metadata", "creationTimestamp"});
  out->creation = ct >= 0 ? d.str(static_cast<uint32_t>(ct)) : std::string();
  out->containers.clear();
  int64_t cs = d.path(pod, {"spec", "containers"});
  if (cs >= 0 && d.at(static_cast<uint32_t>(cs)).type == json::T::Array) {
    uint32_t end = d.at(static_cast<uint32_t>(cs)).skip;
    for (uint32_t c = static_cast<uint32_t>(cs) + 1; c < end; c = d.next(c)) {
      if (d.at(c).type != json::T::Object) continue;
      int64_t lim = d.path(c, {"resources", "limits"});
      int64_t v2 = 0;
      if (lim >= 0 && quantity_of(d, d.find(static_cast<uint32_t>(lim), p.resource), &v2) && v2 > 0) {
        out->containers.push_back(v2);
      }
    }
  }
  return true;
}

// ---------------------------------------------------------------- state

namespace {
bool older_rv(const std::string& a, const std::string& b) {
  // resourceVersion a < b, when both are integers (the apiserver's are; compare nothing otherwise)
  char* ea = nullptr;
  char* eb = nullptr;
  long long x = std::strtoll(a.c_str(), &ea, 10), y = std::strtoll(b.c_str(), &eb, 10);
  if (a.empty() || b.empty() || *ea != '\0' || *eb != '\0') return false;
  return x < y;
}

auto order_key(const AllocPod& p) { return std::tie(p.landed, p.assume_time, p.creation, p.key); }

int64_t rv_int(const std::string& rv) {
  char* e = nullptr;
  long long x = std::strtoll(rv.c_str(), &e, 10);
  return rv.empty() || *e != '\0' ? -1 : static_cast<int64_t>(x);
}
}  // namespace

AllocState::AllocState(std::string node, const std::vector<std::pair<int, std::pair<int, int>>>& devices)
    : node_(std::move(node)) {
  for (const auto& d : devices) cus_.emplace(d.first, CuPartitioner(d.second.first, d.second.second));
}

bool AllocState::observe(const AllocPod& p) {
  if (p.uid.empty()) return false;
  if (gone_.count(p.uid)) {  // deleted or complete: a late copy never brings it back
    auto t = terminating_.find(p.uid);
    if (t != terminating_.end() && p.complete && !p.terminating) terminating_.erase(t);  // now terminal
    return false;
  }
  auto prev = pods_.find(p.uid);
  if (prev != pods_.end() && older_rv(p.rv, prev->second.rv)) return false;  // a slow LIST racing the watch
  if (p.complete) {
    tombstone(p.uid);
    release(p.uid);
    if (p.terminating && p.node == node_ && p.request > 0 && p.dev >= 0) {
      terminating_[p.uid] = Terminating{p.dev, p.request, p.hold_idx};
    } else {
      terminating_.erase(p.uid);  // terminal now: the extender freed it
    }
    return true;
  }
  if (p.node != node_ || p.request <= 0) {
    release(p.uid);
    return true;
  }
  // the landing key survives every later copy of the pod (annotation patches, status, our own PATCH response)
  const int64_t landed = prev != pods_.end() && prev->second.landed != INT64_MAX ? prev->second.landed : -1;
  AllocPod& cur = pods_[p.uid];
  cur = p;
  // no integer resourceVersion (never from an apiserver, whose are etcd revisions): landing unknown, the
  // order falls back to ASSUME_TIME
  cur.landed = landed >= 0 ? landed : (rv_int(p.rv) >= 0 ? rv_int(p.rv) : INT64_MAX);
  keys_[p.key] = p.uid;
  if (p.assigned != "true") return true;
  // an assigned pod owns its CU partition (rebuilt after a restart, or another agent's record)
  auto cp = cus_.find(static_cast<int>(p.dev));
  if (!p.cu_mask.empty() && cp != cus_.end() && !cp->second.holds(p.uid)) {
    std::vector<int> cus;
    try {
      cus = parse_cu_words(p.cu_mask);
    } catch (const std::exception&) {
      cus.clear();
    }
    auto clash = cp->second.adopt(p.uid, cus);
    stats_.cu_adopted++;
    if (!clash.empty()) {
      stats_.cu_conflicts++;
      std::fprintf(stderr, "[gsx-allocstate] pod %s: %zu CU(s) of GPU %lld already owned by another pod\n",
                   p.key.c_str(), clash.size(), static_cast<long long>(p.dev));
    }
  }
  if (!p.pending()) {
    if (partial_.erase(p.uid)) stats_.partial_released++;
  } else if (p.containers.size() > 1 && !local_commits_.count(p.uid) && !partial_.count(p.uid)) {
    partial_[p.uid] = p.containers;  // restarted between containers: accept any of its sizes
  }
  return true;
}

void AllocState::release(const std::string& uid) {
  if (uid.empty()) return;
  int n = 0;
  for (auto& kv : cus_) n += kv.second.release(uid);
  stats_.cu_released += static_cast<uint64_t>(n);
  if (partial_.erase(uid)) stats_.partial_released++;
  auto it = pods_.find(uid);
  if (it != pods_.end()) {
    stats_.pods_released++;
    auto k = keys_.find(it->second.key);
    if (k != keys_.end() && k->second == uid) keys_.erase(k);
    pods_.erase(it);
  }
  local_commits_.erase(uid);
  inflight_.erase(uid);
  std::vector<std::string> gone;
  for (const auto& kv : records_) {
    const AllocRecord& r = kv.second;
    if (r.owner == uid || (r.owner.empty() && r.uid == uid && !owners_known())) gone.push_back(kv.first);
  }
  for (const auto& aid : gone) drop_record(aid);
  if (!owners_known()) {
    // nobody reports what kubelet holds: an allocation is taken to end with the pod it was built for
    for (auto h = held_.begin(); h != held_.end();) {
      auto cur = h++;
      if (cur->second.uid == uid) unhold(cur);
    }
  }
}

void AllocState::tombstone(const std::string& uid) {
  if (uid.empty()) return;
  const double now = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  while (!gone_order_.empty() && (gone_order_.front().first < now - kTombstoneS || gone_order_.size() > 200000)) {
    auto it = gone_.find(gone_order_.front().second);
    if (it != gone_.end() && it->second == gone_order_.front().first) gone_.erase(it);
    gone_order_.pop_front();
  }
  gone_[uid] = now;
  gone_order_.emplace_back(now, uid);
}

void AllocState::deleted(const std::string& uid, double now) {
  if (now < 0) now = std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
  deleted_[uid] = now;
  force_gone(uid, now);
  tombstone(uid);
  release(uid);
  terminating_.erase(uid);
}

void AllocState::force_gone(const std::string& uid, double now) {
  auto p = pods_.find(uid);
  // (with kubelet's report as the truth -- set_linger(false) -- the entries simply stay held until kubelet stops
  // listing them: prune_held, gone_held)
  if (linger_on_ && p != pods_.end() && owners_known()) {
    // live until now: a force delete.  Its containers (the entries it holds, or was built for and nobody else was
    // reported holding) keep their GPU share until kubelet has killed them: their termination grace from now
    if (now < 0) now = std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
    const double until = now + std::min(std::max(p->second.term_grace_s, 0.0), 600.0) + kLingerSlackS;
    forced_[uid] = until;
    forced_["~" + p->second.key] = until;  // the reconciler's name for a holder it no longer knows (GONE)
    std::vector<std::string> keys;
    for (const auto& kv : records_) {
      const AllocRecord& r = kv.second;
      if (!r.ids.empty() && (r.owner == uid || (r.owner.empty() && r.uid == uid))) keys.push_back(id_key(r.ids));
    }
    for (auto h = held_.begin(); h != held_.end(); ++h) {
      if (h->second.owner == uid) keys.push_back(h->first);
    }
    for (const auto& k : keys) {
      auto h = held_.find(k);
      if (h == held_.end()) continue;
      linger(h->second, until);
      unhold(h);
    }
  }
}

double AllocState::ghost_until(const Held& h) const {
  if (!h.owner.empty()) {
    auto f = forced_.find(h.owner);
    return f == forced_.end() ? 0.0 : f->second;
  }
  // never reported: kubelet may have given the IDs to any pod force-deleted before its admission
  double until = 0;
  for (const auto& kv : forced_) until = std::max(until, kv.second);
  return until;
}

int64_t AllocState::terminating_used(int64_t dev) const {
  int64_t n = 0;
  for (const auto& kv : terminating_) {
    // a hold charges the hold device too (the extender's ledger.cc account())
    if (kv.second.dev == dev || (kv.second.hold >= 0 && kv.second.hold == dev)) n += kv.second.request;
  }
  return n;
}

int64_t AllocState::terminating_dev(const std::string& uid) const {
  auto it = terminating_.find(uid);
  return it == terminating_.end() ? -1 : it->second.dev;
}

std::vector<std::string> AllocState::holders() const {
  std::unordered_set<std::string> out;
  for (const auto& kv : pods_) out.insert(kv.first);
  for (const auto& kv : partial_) out.insert(kv.first);
  out.insert(local_commits_.begin(), local_commits_.end());
  for (const auto& c : cus_) {
    for (const auto& h : c.second.held()) out.insert(h.first);
  }
  return std::vector<std::string>(out.begin(), out.end());
}

void AllocState::resync(const std::unordered_set<std::string>& live, double now) {
  for (const auto& uid : holders()) {
    if (live.count(uid)) continue;
    force_gone(uid, now);  // gone while live here: deleted outright (not tombstoned: a LIST may lag a watch)
    release(uid);
  }
  for (auto it = terminating_.begin(); it != terminating_.end();) {
    if (!live.count(it->first)) {
      it = terminating_.erase(it);
    } else {
      ++it;
    }
  }
}

std::vector<const AllocPod*> AllocState::candidates() const {
  // the partner Q an unfinished reconciliation exchange names (P's hold-partner): its fields are about to be
  // rewritten (step 2), so no Allocate may be served to it with the old ones meanwhile -- served on the GPU it is
  // leaving, it would stay there while the extender has already credited that room to P (tests/interleave.py,
  // reconcile.py _finish_holds).  Holds are rare and short: a scan, no index
  std::unordered_set<std::string> partners;
  for (const auto& kv : pods_) {
    if (!skip_partners_) break;
    const std::string& hp = kv.second.hold_partner;
    if (hp.empty()) continue;
    const size_t k = hp.find("\"uid\"");
    const size_t q1 = k == std::string::npos ? k : hp.find('"', hp.find(':', k) + 1);
    const size_t q2 = q1 == std::string::npos ? q1 : hp.find('"', q1 + 1);
    if (q2 != std::string::npos) partners.insert(hp.substr(q1 + 1, q2 - q1 - 1));
  }
  std::vector<const AllocPod*> out;
  for (const auto& kv : pods_) {
    const AllocPod& r = kv.second;
    if (r.pending() && r.assigned == "false" && has_device(r.dev) && !inflight_.count(r.uid) &&
        (partners.empty() || !partners.count(r.uid))) {
      out.push_back(&r);
    }
  }
  std::sort(out.begin(), out.end(), [](const AllocPod* a, const AllocPod* b) { return order_key(*a) < order_key(*b); });
  return out;
}

std::pair<const AllocPod*, bool> AllocState::match(int64_t units) {
  auto cands = candidates();
  for (const AllocPod* r : cands) {
    if (r->request == units) {
      stats_.matches++;
      return {r, true};
    }
  }
  const AllocPod* best = nullptr;
  for (const auto& kv : partial_) {
    auto it = pods_.find(kv.first);
    if (it == pods_.end() || inflight_.count(kv.first)) continue;
    if (std::find(kv.second.begin(), kv.second.end(), units) == kv.second.end()) continue;
    if (!best || order_key(it->second) < order_key(*best)) best = &it->second;
  }
  if (best) {
    stats_.matches++;
    return {best, false};
  }
  for (const AllocPod* r : cands) {
    if (std::find(r->containers.begin(), r->containers.end(), units) != r->containers.end()) {
      stats_.matches++;
      return {r, false};
    }
  }
  stats_.match_misses++;
  return {nullptr, false};
}

int64_t AllocState::preferred_device(int64_t units) {
  auto m = match(units);
  return m.first ? m.first->dev : -1;
}

bool AllocState::unannotated(int64_t units) const {
  for (const auto& kv : pods_) {
    const AllocPod& r = kv.second;
    if (r.pending() && r.dev < 0 && r.assigned != "true" && r.request == units && !inflight_.count(r.uid)) return true;
  }
  return false;
}

bool AllocState::claim_cus(const std::string& uid, std::vector<int>* out, std::string* err) {
  out->clear();
  auto it = pods_.find(uid);
  if (it == pods_.end()) {
    *err = "pod " + uid + " is not on this node";
    return false;
  }
  const AllocPod& p = it->second;
  if (p.cu_count <= 0) return true;
  auto cp = cus_.find(static_cast<int>(p.dev));
  if (cp == cus_.end()) {
    *err = "pod " + p.key + " annotated with GPU " + std::to_string(p.dev) + ", not on this node";
    return false;
  }
  return cp->second.allocate(uid, p.cu_count, out, err);
}

void AllocState::set_inflight(const std::string& uid, bool on) {
  if (on) {
    inflight_.insert(uid);
  } else {
    inflight_.erase(uid);
  }
}

void AllocState::first_container_committed(const std::string& uid, int64_t units, bool whole) {
  local_commits_.insert(uid);
  if (whole) return;
  auto it = pods_.find(uid);
  if (it == pods_.end()) return;
  std::vector<int64_t> left = it->second.containers;
  auto f = std::find(left.begin(), left.end(), units);
  if (f != left.end()) left.erase(f);
  if (!left.empty()) partial_[uid] = std::move(left);
}

void AllocState::later_container_allocated(const std::string& uid, int64_t units) {
  auto it = partial_.find(uid);
  if (it == partial_.end()) return;
  auto f = std::find(it->second.begin(), it->second.end(), units);
  if (f != it->second.end()) it->second.erase(f);
  if (it->second.empty()) partial_.erase(it);
}

// ---------------------------------------------------------------- records

AllocRecord& AllocState::record(const std::string& uid, const std::vector<std::string>& ids_in, int64_t units,
                                const std::string& cu_mask, const std::string& aid, double t, bool on_gpu) {
  std::vector<std::string> ids(ids_in);
  // kubelet passes GetPreferredAllocation's pick back in the plugin's own (sorted) order: usually nothing to sort
  if (!std::is_sorted(ids.begin(), ids.end())) std::sort(ids.begin(), ids.end());
  const std::string key = ids.empty() ? std::string() : id_key(ids);
  if (!ids.empty()) {
    auto old = by_ids_.find(key);
    if (old != by_ids_.end()) drop_record(old->second);  // kubelet re-used the IDs of a finished pod
  }
  AllocRecord r;
  r.aid = aid;
  r.uid = uid;
  auto p = pods_.find(uid);
  r.dev = p != pods_.end() ? p->second.dev : -1;
  r.units = units;
  r.cu_mask = cu_mask;
  r.t = t;
  r.on_gpu = on_gpu;
  if (!ids.empty()) by_ids_[key] = aid;
  if (!ids.empty()) hold(key, Held{r.dev, units, t, uid, on_gpu, cu_mask});
  r.ids = std::move(ids);
  auto res = records_.insert_or_assign(aid, std::move(r));
  return res.first->second;
}

void AllocState::add_record(AllocRecord r) {
  std::sort(r.ids.begin(), r.ids.end());
  const std::string key = r.ids.empty() ? std::string() : id_key(r.ids);
  if (!r.ids.empty()) by_ids_[key] = r.aid;
  std::string aid = r.aid;
  // a restored record: its allocation is held until kubelet's report says otherwise
  if (!r.ids.empty() && !held_.count(key)) hold(key, Held{r.dev, r.units, r.t, r.uid, r.on_gpu, r.cu_mask, r.owner});
  records_.insert_or_assign(aid, std::move(r));
}

std::string AllocState::id_key(const std::vector<std::string>& sorted_ids) {
  size_t n = 0;
  for (const auto& id : sorted_ids) n += id.size() + 1;
  std::string k;
  k.reserve(n);
  for (const auto& id : sorted_ids) {
    k.append(id);
    k.push_back('\n');
  }
  return k;
}

void AllocState::linger(const Held& h, double until) {
  if (h.dev < 0 || h.units <= 0) return;
  linger_.push_back(Linger{h.dev, h.units, until});
  linger_units_[h.dev] += h.units;
  linger_n_[h.dev]++;
}

bool AllocState::holder_gone(const Held& h) const {
  const std::string& who = h.owner.empty() ? h.uid : h.owner;
  // a holder kubelet lists but this view does not know ("~ns/name"), one deleted, or one never seen (a restart);
  // not a complete pod (a finished Job's object stays, and some kubelets keep listing it)
  if (!who.empty() && who[0] == '~') return true;
  return !pods_.count(who) && !terminating_.count(who) && (deleted_.count(who) || !gone_.count(who));
}

int64_t AllocState::gone_held(int64_t dev) const {
  int64_t n = 0;
  for (const auto& kv : held_) {
    const Held& h = kv.second;
    if (h.dev == dev && h.listed && h.gone_reports >= 2 && last_prune_ - h.gone_since >= kGoneHeldMinS) n += h.units;
  }
  return n;
}

int64_t AllocState::lingering(int64_t dev) const {
  auto it = linger_units_.find(dev);
  return it == linger_units_.end() ? 0 : it->second;
}

void AllocState::hold(const std::string& ids, Held h) {
  auto prev = held_.find(ids);
  if (prev != held_.end()) {
    // kubelet re-used the IDs: their container finished -- or its pod was force-deleted (kubelet frees the IDs at
    // once) and this view has not seen the delete yet: its container may still be stopping
    const Held& ph = prev->second;
    auto o = ph.owner.empty() || !linger_on_ ? pods_.end() : pods_.find(ph.owner);
    if (o != pods_.end() && o->first != h.uid) {
      linger(ph, h.t + std::min(std::max(o->second.term_grace_s, 0.0), 600.0) + kLingerSlackS);
    } else if (linger_on_) {
      const double until = ghost_until(ph);
      if (until > h.t) linger(ph, until);
    }
    unhold(prev);
  }
  if (h.dev >= 0) phys_[h.dev] += h.units;
  if (!h.on_gpu) off_gpu_count(h.dev, +1);
  held_.emplace(ids, std::move(h));
}

void AllocState::unhold(std::unordered_map<std::string, Held>::iterator it) {
  const Held& h = it->second;
  if (h.dev >= 0) {
    int64_t& u = phys_[h.dev];
    u -= h.units;
    if (u == 0) phys_.erase(h.dev);
  }
  if (!h.on_gpu) off_gpu_count(h.dev, -1);
  held_.erase(it);
}

int64_t AllocState::physical_used(int64_t dev) const {
  auto it = phys_.find(dev);
  return (it == phys_.end() ? 0 : it->second) + lingering(dev);
}

void AllocState::mark_on_gpu(const std::string& aid, bool on) {
  auto it = records_.find(aid);
  if (it == records_.end()) return;
  it->second.on_gpu = on;
  auto h = held_.find(id_key(it->second.ids));
  if (h == held_.end() || h->second.on_gpu == on) return;
  h->second.on_gpu = on;
  off_gpu_count(h->second.dev, on ? -1 : +1);
}

void AllocState::off_gpu_count(int64_t dev, int d) {
  off_gpu_ = static_cast<size_t>(static_cast<int64_t>(off_gpu_) + d);
  size_t& n = off_gpu_dev_[dev];
  n = static_cast<size_t>(static_cast<int64_t>(n) + d);
  if (n == 0) off_gpu_dev_.erase(dev);
}

size_t AllocState::off_gpu_records_on(int64_t dev) const {
  // a lingering container holds no ID kubelet still counts: kubelet's per-ID accounting no longer bounds `dev`
  auto it = off_gpu_dev_.find(dev);
  auto ln = linger_n_.find(dev);
  return (it == off_gpu_dev_.end() ? 0 : it->second) + (ln == linger_n_.end() ? 0 : ln->second);
}

bool AllocState::held_for(std::vector<std::string> ids, int64_t* dev, int64_t* units, double* t,
                          std::string* cu_mask) const {
  std::sort(ids.begin(), ids.end());
  auto it = held_.find(id_key(ids));
  if (it == held_.end()) return false;
  *dev = it->second.dev;
  *units = it->second.units;
  *t = it->second.t;
  *cu_mask = it->second.cu_mask;
  return true;
}

size_t AllocState::prune_held(const std::vector<std::vector<std::string>>& listed_in, double asked, double grace) {
  std::unordered_set<std::string> listed;
  for (auto ids : listed_in) {
    std::sort(ids.begin(), ids.end());
    listed.insert(id_key(ids));
  }
  size_t n = 0;
  last_prune_ = asked;
  for (auto it = held_.begin(); it != held_.end();) {
    auto cur = it++;
    cur->second.listed = listed.count(cur->first) != 0;
    cur->second.gone_reports = cur->second.listed && holder_gone(cur->second) ? cur->second.gone_reports + 1 : 0;
    if (cur->second.gone_reports == 1) cur->second.gone_since = asked;
    if (!cur->second.listed && asked - cur->second.t > grace) {
      const Held& h = cur->second;
      if (!h.owner.empty() && pods_.count(h.owner)) continue;  // live here: see the header
      // held by a force-deleted pod (kubelet stopped listing it at the delete, perhaps before this view knew the
      // pod was gone -- one deleted between its binding and its admission): counted until its kill deadline
      const double until = linger_on_ ? ghost_until(h) : 0.0;
      if (until > asked) linger(h, until);
      unhold(cur);
      n++;
    }
  }
  for (auto it = deleted_.begin(); it != deleted_.end();) {
    if (it->second < asked - kTombstoneS) {
      it = deleted_.erase(it);
    } else {
      ++it;
    }
  }
  for (auto it = forced_.begin(); it != forced_.end();) {
    if (it->second <= asked) {
      it = forced_.erase(it);
    } else {
      ++it;
    }
  }
  for (auto it = linger_.begin(); it != linger_.end();) {
    if (it->until > asked) {
      ++it;
      continue;
    }
    unlinger(*it);
    it = linger_.erase(it);
    n++;
  }
  return n;
}

void AllocState::unlinger(const Linger& l) {
  if ((linger_units_[l.dev] -= l.units) <= 0) linger_units_.erase(l.dev);
  if (--linger_n_[l.dev] == 0) linger_n_.erase(l.dev);
}

bool AllocState::drop_record(const std::string& aid) {
  auto it = records_.find(aid);
  if (it == records_.end()) return false;
  auto b = by_ids_.find(id_key(it->second.ids));
  if (b != by_ids_.end() && b->second == aid) by_ids_.erase(b);
  stats_.records_dropped++;
  dropped_.push_back(std::move(it->second));
  records_.erase(it);
  return true;
}

const AllocRecord* AllocState::record_for_ids(std::vector<std::string> ids) const {
  std::sort(ids.begin(), ids.end());
  auto b = by_ids_.find(id_key(ids));
  if (b == by_ids_.end()) return nullptr;
  auto it = records_.find(b->second);
  return it == records_.end() ? nullptr : &it->second;
}

AllocRecord* AllocState::record_by_aid(const std::string& aid) {
  auto it = records_.find(aid);
  return it == records_.end() ? nullptr : &it->second;
}

void AllocState::set_owner(const std::string& aid, const std::string& owner) {
  auto it = records_.find(aid);
  if (it == records_.end()) return;
  it->second.owner = owner;
  if (it->second.ids.empty()) return;
  auto h = held_.find(id_key(it->second.ids));
  if (h != held_.end()) h->second.owner = owner;
}

void AllocState::move_records(const std::string& p_uid, const std::string& q_uid, const std::string& aid) {
  for (auto& kv : records_) {
    if (kv.first != aid && kv.second.uid == p_uid) kv.second.uid = q_uid;
  }
  auto it = records_.find(aid);
  if (it != records_.end()) it->second.uid = p_uid;
  for (auto& kv : cus_) kv.second.swap_owners(p_uid, q_uid);
}

std::vector<AllocRecord> AllocState::take_dropped() {
  std::vector<AllocRecord> out;
  out.swap(dropped_);
  return out;
}

const AllocPod* AllocState::pod(const std::string& uid) const {
  auto it = pods_.find(uid);
  return it == pods_.end() ? nullptr : &it->second;
}

const AllocPod* AllocState::pod_by_key(const std::string& key) const {
  auto k = keys_.find(key);
  return k == keys_.end() ? nullptr : pod(k->second);
}

CuPartitioner* AllocState::cus(int dev) {
  auto it = cus_.find(dev);
  return it == cus_.end() ? nullptr : &it->second;
}

}  // namespace gsx
