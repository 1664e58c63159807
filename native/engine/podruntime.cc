#include "podruntime.h"

#include <dlfcn.h>

#include <algorithm>
#include <cstdio>
#include <set>
#include <vector>

#include "json.h"

namespace gsx {

namespace {

constexpr uint64_t kAlign = 2ull << 20;

// Per-pod stamp tag: FNV-1a of the uid, odd (never 0 = "unstamped").
uint64_t tag_of(const std::string& uid) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : uid) {
    h ^= c;
    h *= 1099511628211ull;
  }
  return h | 1;
}

// layout of gsx_slice in gsx_kernels.h
struct GsxSlice {
  uint64_t addr, bytes, tag;
};

}  // namespace

PodRuntime::PodRuntime(PodRuntimeConfig cfg) : cfg_(std::move(cfg)) {}

PodRuntime::~PodRuntime() {
  stop();
  if (lib_) dlclose(lib_);
}

bool PodRuntime::init(std::string* err) {
  if (!cfg_.arena_addr) return true;  // accounting only
  lib_ = dlopen(cfg_.kernels_lib.c_str(), RTLD_NOW | RTLD_LOCAL);
  if (!lib_) {
    *err = std::string("dlopen ") + cfg_.kernels_lib + ": " + dlerror();
    return false;
  }
  set_device_ = reinterpret_cast<int (*)(int)>(dlsym(lib_, "gsx_set_device"));
  admit_n_ = reinterpret_cast<int (*)(void*, const void*, int, int, int, uint64_t, uint64_t*)>(
      dlsym(lib_, "gsx_hbm_admit_n"));
  last_error_ = reinterpret_cast<const char* (*)()>(dlsym(lib_, "gsx_last_error"));
  if (!set_device_ || !admit_n_ || !last_error_) {
    *err = "libgsx_kernels.so lacks gsx_set_device / gsx_hbm_admit_n";
    return false;
  }
  if (!cfg_.stream || cfg_.stride < 16 || cfg_.stride % 16) {
    *err = "pod runtime needs a stream and a 16-B multiple stamp stride";
    return false;
  }
  return true;
}

int PodRuntime::serve(const std::string& host, int port, std::string* err, std::vector<int> cpus) {
  srv_ = std::make_unique<CtlServer>([this](const http::Message& m) { return handle(m); });
  srv_->set_cpus(std::move(cpus));
  return srv_->start(host, port, err);
}

void PodRuntime::stop() {
  if (srv_) srv_->stop();
}

uint64_t PodRuntime::resident_bytes() const {
  std::lock_guard<std::mutex> g(mu_);
  uint64_t b = 0;
  for (auto& kv : slices_) b += kv.second.size;
  return b;
}

size_t PodRuntime::resident() const {
  std::lock_guard<std::mutex> g(mu_);
  return slices_.size();
}

int64_t PodRuntime::run_admit(bool stamp, const std::string& uid, bool verify, std::string* err) {
  if (!cfg_.arena_addr) return 0;
  std::vector<GsxSlice> sl;
  auto add = [&](const Slice& s) {
    for (auto& e : s.ext) sl.push_back(GsxSlice{cfg_.arena_addr + e.first, e.second, s.tag});
  };
  auto mine = slices_.find(uid);
  if (mine != slices_.end()) add(mine->second);  // the new pod's extents first: they are the ones stamped
  const int n_stamp = stamp ? static_cast<int>(sl.size()) : 0;
  if (verify) {
    for (auto& kv : slices_) {
      if (kv.first != uid) add(kv.second);
    }
  }
  if (sl.empty()) return 0;
  uint64_t bad = 0;
  int rc = set_device_(cfg_.dev);
  if (rc == 0) rc = admit_n_(cfg_.stream, sl.data(), static_cast<int>(sl.size()), n_stamp, 1, cfg_.stride, &bad);
  if (rc != 0) {
    *err = std::string("gsx_hbm_admit_n: ") + last_error_();
    return -1;
  }
  return static_cast<int64_t>(bad);
}

bool PodRuntime::carve_locked(const std::string& uid, uint64_t bytes, std::string* err) {
  uint64_t size = (bytes + kAlign - 1) / kAlign * kAlign;
  // extents from the arena's holes in offset order (first fit; one extent unless fragmented)
  std::vector<std::pair<uint64_t, uint64_t>> used;
  for (auto& kv : slices_) used.insert(used.end(), kv.second.ext.begin(), kv.second.ext.end());
  std::sort(used.begin(), used.end());
  Slice s{{}, size, tag_of(uid)};
  uint64_t pos = 0, need = size;
  auto take = [&](uint64_t end) {
    if (need && end > pos) {
      uint64_t n = std::min(need, end - pos);
      s.ext.emplace_back(pos, n);
      need -= n;
    }
  };
  for (auto& u : used) {
    take(u.first);
    pos = std::max(pos, u.first + u.second);
  }
  take(cfg_.arena_bytes);
  if (need) {
    *err = "arena exhausted: need " + std::to_string(size) + " B, " + std::to_string(size - need) + " free of " +
           std::to_string(cfg_.arena_bytes);
    return false;
  }
  slices_[uid] = std::move(s);
  return true;
}

void PodRuntime::admit_group_locked(const std::vector<Pending*>& group) {
  std::vector<Pending*> fresh, again;
  bool verify_all = false;
  for (Pending* p : group) {
    if (slices_.count(p->uid)) {
      again.push_back(p);  // idempotent re-admission (or the same uid twice in one group)
    } else if (!carve_locked(p->uid, p->bytes, &p->err)) {
      failed_++;
      p->result = -1;
      continue;
    } else {
      fresh.push_back(p);
    }
    verify_all = verify_all || p->verify;
  }
  if (fresh.empty() && again.empty()) return;
  // the group's new extents first (stamped), then -- if any admission asked for it -- every other resident
  // slice, so one launch pair checks that no new stamp landed in another pod's slice
  std::vector<GsxSlice> sl;
  std::set<std::string> listed;
  for (Pending* p : fresh) {
    for (auto& e : slices_[p->uid].ext) sl.push_back(GsxSlice{cfg_.arena_addr + e.first, e.second, slices_[p->uid].tag});
    listed.insert(p->uid);
  }
  const int n_stamp = static_cast<int>(sl.size());
  for (auto& kv : slices_) {
    if (listed.count(kv.first)) continue;
    bool own = false;
    for (Pending* p : again) own = own || p->uid == kv.first;
    if (!verify_all && !own) continue;
    for (auto& e : kv.second.ext) sl.push_back(GsxSlice{cfg_.arena_addr + e.first, e.second, kv.second.tag});
  }
  uint64_t bad = 0;
  int rc = 0;
  if (cfg_.arena_addr && !sl.empty()) {
    rc = set_device_(cfg_.dev);
    if (rc == 0) rc = admit_n_(cfg_.stream, sl.data(), static_cast<int>(sl.size()), n_stamp, 1, cfg_.stride, &bad);
    batches_++;
  }
  if (rc != 0) {
    std::string e = std::string("gsx_hbm_admit_n: ") + last_error_();
    for (Pending* p : fresh) {
      slices_.erase(p->uid);
      failed_++;
      p->result = -1;
      p->err = e;
    }
    for (Pending* p : again) {
      p->result = -1;
      p->err = e;
    }
    return;
  }
  bad_ += bad;
  // An admission that asked for verification answers for every resident slice (the group's total).  One that
  // did not is charged only with its own slice (another pod's corrupted slice must not fail it): on
  // the rare bad group its extents are verified once more on their own.
  auto own_bad = [&](Pending* p) -> int64_t {
    if (p->verify || bad == 0) return static_cast<int64_t>(bad);
    std::vector<GsxSlice> mine;
    auto it = slices_.find(p->uid);
    if (it == slices_.end()) return 0;
    for (auto& e : it->second.ext) mine.push_back(GsxSlice{cfg_.arena_addr + e.first, e.second, it->second.tag});
    uint64_t b = 0;
    if (!mine.empty() && admit_n_(cfg_.stream, mine.data(), static_cast<int>(mine.size()), 0, 1, cfg_.stride, &b) != 0) {
      return static_cast<int64_t>(bad);  // cannot tell: keep the conservative answer
    }
    return static_cast<int64_t>(b);
  };
  for (Pending* p : fresh) {
    admitted_++;
    p->result = own_bad(p);
  }
  for (Pending* p : again) p->result = own_bad(p);  // its slice was re-verified in the launch
}

int64_t PodRuntime::admit(const std::string& uid, uint64_t bytes, bool verify, std::string* err) {
  Pending me{uid, bytes, verify};
  std::unique_lock<std::mutex> q(qmu_);
  queue_.push_back(&me);
  while (!me.done) {
    if (leading_) {
      qcv_.wait(q);
      continue;
    }
    // lead: admit everything queued so far as one group; admissions arriving meanwhile form the next one
    leading_ = true;
    std::vector<Pending*> group;
    group.swap(queue_);
    q.unlock();
    try {
      std::lock_guard<std::mutex> g(mu_);
      admit_group_locked(group);
    } catch (const std::exception& e) {
      // the group fails, but leadership is handed back below: a throw here must not park every later admission
      for (Pending* p : group) {
        if (p->result >= 0 && p->err.empty()) {
          p->result = -1;
          p->err = std::string("admission: ") + e.what();
        }
      }
    }
    q.lock();
    for (Pending* p : group) p->done = true;
    leading_ = false;
    qcv_.notify_all();
  }
  if (me.result < 0) *err = me.err;
  return me.result;
}

bool PodRuntime::release(const std::string& uid) {
  std::lock_guard<std::mutex> g(mu_);
  return slices_.erase(uid) > 0;
}

int64_t PodRuntime::verify_all(std::string* err) {
  std::lock_guard<std::mutex> g(mu_);
  return run_admit(false, std::string(), true, err);
}

CtlServer::Reply PodRuntime::handle(const http::Message& m) {
  CtlServer::Reply rep;
  std::string_view path = m.path();
  const std::string_view pre = "/v1/pods/";
  if (path.substr(0, pre.size()) == pre && path.size() > pre.size()) {
    std::string uid(path.substr(pre.size()));
    if (m.method == "POST") {
      json::Doc d;
      std::string err;
      int64_t bytes = 0;
      bool verify = true;
      if (d.parse(m.body, &err)) {
        int64_t b = d.find(0, "bytes");
        if (b >= 0) d.as_int(static_cast<uint32_t>(b), &bytes);
        int64_t v = d.find(0, "verify");
        if (v >= 0) verify = d.at(static_cast<uint32_t>(v)).type != json::T::False;
      }
      if (bytes <= 0) {
        rep.status = 400;
        rep.body = "{\"error\":\"bytes must be > 0\"}";
        return rep;
      }
      int64_t bad = admit(uid, static_cast<uint64_t>(bytes), verify, &err);
      if (bad < 0) {
        rep.status = 409;
        rep.body = "{\"error\":";
        json::append_quoted(&rep.body, err);
        rep.body.push_back('}');
        return rep;
      }
      rep.body = "{\"bad\":" + std::to_string(bad) + "}";
      return rep;
    }
    if (m.method == "DELETE") {
      rep.status = release(uid) ? 200 : 404;
      return rep;
    }
  }
  if (m.method == "GET" && path == "/v1/stats") {
    std::lock_guard<std::mutex> g(mu_);
    char b[256];
    std::snprintf(b, sizeof(b),
                  "{\"admitted\":%llu,\"failed\":%llu,\"bad\":%llu,\"resident\":%zu,\"batches\":%llu,\"native\":true}",
                  (unsigned long long)admitted_, (unsigned long long)failed_, (unsigned long long)bad_,
                  slices_.size(), (unsigned long long)batches_);
    rep.body = b;
    return rep;
  }
  rep.status = 404;
  rep.body = "{\"error\":\"not found\"}";
  return rep;
}

}  // namespace gsx
