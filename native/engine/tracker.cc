#include "tracker.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <deque>
#include <thread>
#include <unordered_set>

namespace gsx {

namespace {

std::string str_at(const json::Doc& d, int64_t i) { return i >= 0 ? d.str(static_cast<uint32_t>(i)) : std::string(); }

}  // namespace

PodTracker::PodTracker(const ApiConfig& cfg, const std::string& ns, const std::string& label_selector) {
  ReflectorConfig rc;
  rc.path = ns.empty() ? "/api/v1/pods" : "/api/v1/namespaces/" + ns + "/pods";
  rc.label_selector = label_selector;
  ReflectorHandler h;
  auto key_of = [](const json::Doc& d, uint32_t obj) {
    std::string ns_ = str_at(d, d.path(obj, {"metadata", "namespace"}));
    std::string name = str_at(d, d.path(obj, {"metadata", "name"}));
    return ns_.empty() ? name : ns_ + "/" + name;
  };
  h.on_list = [this, key_of](const ListView& lv) {
    std::lock_guard<std::mutex> g(mu_);
    pods_.clear();
    for (size_t k = 0; k < lv.size(); ++k) {
      const json::Doc& d = lv.doc(k);
      uint32_t i = lv.obj(k);
      St& s = pods_[key_of(d, i)];
      s.node = str_at(d, d.path(i, {"spec", "nodeName"}));
      s.phase = str_at(d, d.path(i, {"status", "phase"}));
    }
    cv_.notify_all();
  };
  h.on_event = [this, key_of](Ev ev, const json::Doc& d, uint32_t obj) {
    std::string key = key_of(d, obj);
    std::lock_guard<std::mutex> g(mu_);
    if (ev == Ev::Deleted) {
      pods_.erase(key);
    } else {
      St& s = pods_[key];
      s.node = str_at(d, d.path(obj, {"spec", "nodeName"}));
      s.phase = str_at(d, d.path(obj, {"status", "phase"}));
    }
    cv_.notify_all();
  };
  r_ = std::make_unique<Reflector>(cfg, rc, h);
}

PodTracker::~PodTracker() { stop(); }

bool PodTracker::start(double timeout_s, std::string* err) {
  r_->start();
  if (!r_->wait_synced(timeout_s)) {
    *err = "tracker did not sync: " + r_->last_error();
    return false;
  }
  return true;
}

void PodTracker::stop() {
  if (r_) r_->stop();
  cv_.notify_all();
}

size_t PodTracker::size() const {
  std::lock_guard<std::mutex> g(mu_);
  return pods_.size();
}

bool PodTracker::ok_locked(const std::string& key, int cond, std::string* err) const {
  auto it = pods_.find(key);
  switch (cond) {
    case Bound:
      return it != pods_.end() && !it->second.node.empty();
    case Running:
      if (it != pods_.end() && it->second.phase == "Failed") *err = "pod " + key + " Failed";
      return it != pods_.end() && it->second.phase == "Running";
    case Stopped:
      return it == pods_.end() || it->second.phase == "Succeeded" || it->second.phase == "Failed";
    default:
      return it == pods_.end();
  }
}

std::string PodTracker::wait(const std::vector<std::string>& keys, int cond, double timeout_s) {
  auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  std::unique_lock<std::mutex> lk(mu_);
  size_t i = 0;  // keys before i already satisfied the condition (monotone within one wave)
  while (true) {
    std::string err;
    while (i < keys.size() && ok_locked(keys[i], cond, &err)) ++i;
    if (!err.empty()) return err;
    if (i == keys.size()) return std::string();
    if (cv_.wait_until(lk, deadline) == std::cv_status::timeout) {
      while (i < keys.size() && ok_locked(keys[i], cond, &err)) ++i;
      if (i == keys.size()) return std::string();
      return "timeout: " + std::to_string(keys.size() - i) + " pods not " +
             (cond == Bound ? "bound" : cond == Running ? "Running" : cond == Stopped ? "stopped" : "gone") + ", e.g. " + keys[i];
    }
  }
}

BatchClient::~BatchClient() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : helpers_) t.join();
}

void BatchClient::work_on(const std::vector<Req>& reqs, std::vector<std::pair<int, std::string>>* out) {
  while (true) {
    size_t i = next_.fetch_add(1);
    if (i >= reqs.size()) return;
    int status = 0;
    std::string body, err;
    const auto& r = reqs[i];
    if (api_.request(std::get<0>(r), std::get<1>(r), std::get<2>(r), "application/json", &status, &body, &err)) {
      (*out)[i] = {status, std::move(body)};
    } else {
      (*out)[i] = {-1, err};
    }
  }
}

void BatchClient::helper(int me) {
  uint64_t seen = 0;
  std::unique_lock<std::mutex> lk(mu_);
  while (true) {
    cv_.wait(lk, [&] { return stop_ || (gen_ != seen && me < want_); });
    if (stop_) return;
    seen = gen_;
    const std::vector<Req>* reqs = reqs_;
    auto* out = out_;
    ++busy_;
    lk.unlock();
    work_on(*reqs, out);
    lk.lock();
    if (--busy_ == 0) done_cv_.notify_all();
  }
}

std::vector<std::pair<int, std::string>> BatchClient::run(const std::vector<Req>& reqs, int concurrency) {
  std::lock_guard<std::mutex> one(run_mu_);  // one batch at a time
  std::vector<std::pair<int, std::string>> out(reqs.size());
  const int n = std::max(1, std::min<int>(concurrency, static_cast<int>(reqs.size())));
  {
    std::lock_guard<std::mutex> g(mu_);
    while (static_cast<int>(helpers_.size()) < n - 1) {
      const int k = static_cast<int>(helpers_.size());
      helpers_.emplace_back([this, k] { helper(k); });
    }
    reqs_ = &reqs;
    out_ = &out;
    next_.store(0);
    want_ = n - 1;
    ++gen_;
  }
  if (n > 1) cv_.notify_all();
  work_on(reqs, &out);
  std::unique_lock<std::mutex> lk(mu_);
  // every helper that joined this batch has finished its request before `out` goes out of scope; one that wakes
  // late finds the batch taken (next_ past the end) and leaves at once
  done_cv_.wait(lk, [&] { return busy_ == 0; });
  want_ = 0;
  reqs_ = nullptr;
  out_ = nullptr;
  return out;
}

}  // namespace gsx

namespace gsx {

namespace {
double mono() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
}  // namespace

// Constant-rate arrivals (an open loop: a slow stack does not slow the arrivals down, so queueing shows as latency
// instead of a lower offered rate -- no coordinated omission).  Pod i arrives at t0 + i / rate; creators send it
// then (or as soon as one is free), and every stage time counts from that arrival.  A pod seen Running is deleted
// (after hold_s) by the deleters, so the node's room turns over and the run measures the stack's sustained
// throughput with many pods in flight, not its capacity.
bool OpenLoop::run(const OpenLoopConfig& c, std::vector<OpenLoopPod>* pods, std::string* err, int* create_errors,
                   int* delete_errors) {
  const size_t n = static_cast<size_t>(std::max(1.0, c.rate * c.duration_s));
  pods->assign(n, OpenLoopPod{});
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::pair<double, size_t>> dq;  // (not before, pod) to delete
  std::atomic<int> cerr{0}, derr{0};
  std::atomic<size_t> next{0}, gone{0};
  std::atomic<bool> stop{false};
  const std::string prefix = "ol-" + c.run + "-";
  auto index_of = [&](const json::Doc& d, uint32_t obj) -> int64_t {
    std::string name = str_at(d, d.path(obj, {"metadata", "name"}));
    if (name.compare(0, prefix.size(), prefix) != 0) return -1;
    char* e = nullptr;
    long long i = std::strtoll(name.c_str() + prefix.size(), &e, 10);
    return (e && *e == '\0' && i >= 0 && static_cast<size_t>(i) < n) ? i : -1;
  };
  auto observe = [&](Ev ev, const json::Doc& d, uint32_t obj) {
    int64_t i = index_of(d, obj);
    if (i < 0) return;
    const double now = mono();
    std::lock_guard<std::mutex> g(mu);
    OpenLoopPod& p = (*pods)[static_cast<size_t>(i)];
    if (ev == Ev::Deleted) {
      if (p.gone == 0) {
        p.gone = now;
        gone.fetch_add(1);
        cv.notify_all();
      }
      return;
    }
    if (p.bound == 0 && !str_at(d, d.path(obj, {"spec", "nodeName"})).empty()) p.bound = now;
    std::string phase = str_at(d, d.path(obj, {"status", "phase"}));
    if (p.running == 0 && (phase == "Running" || phase == "Failed")) {
      p.running = now;
      p.failed = phase == "Failed";
      dq.emplace_back(now + c.hold_s, static_cast<size_t>(i));
      cv.notify_all();
    }
  };
  ReflectorConfig rc;
  rc.path = "/api/v1/namespaces/" + c.ns + "/pods";
  rc.label_selector = c.label_key + "=" + c.run;
  ReflectorHandler h;
  h.on_list = [&](const ListView& lv) {
    for (size_t k = 0; k < lv.size(); ++k) observe(Ev::Modified, lv.doc(k), lv.obj(k));
  };
  h.on_event = [&](Ev ev, const json::Doc& d, uint32_t obj) { observe(ev, d, obj); };
  Reflector r(cfg_, rc, h);
  r.start();
  if (!r.wait_synced(30)) {
    *err = "open-loop watch did not sync: " + r.last_error();
    r.stop();
    return false;
  }
  const std::string coll = "/api/v1/namespaces/" + c.ns + "/pods";
  const double t0 = mono() + 0.01;
  std::vector<std::thread> th;
  for (int k = 0; k < std::max(1, c.creators); ++k) {
    th.emplace_back([&] {
      ApiClient api(cfg_);
      std::string body, resp, e;
      while (!stop.load()) {
        size_t i = next.fetch_add(1);
        if (i >= n) return;
        const double at = t0 + static_cast<double>(i) / c.rate;
        const double wait = at - mono();
        if (wait > 0) std::this_thread::sleep_for(std::chrono::duration<double>(wait));
        body = c.pod_tmpl;
        const std::string name = prefix + std::to_string(i);
        for (size_t pos = body.find("__NAME__"); pos != std::string::npos; pos = body.find("__NAME__", pos))
          body.replace(pos, 8, name);
        int status = 0;
        bool ok = api.request("POST", coll, body, "application/json", &status, &resp, &e) && status == 201;
        std::lock_guard<std::mutex> g(mu);
        (*pods)[i].arrival = at;
        (*pods)[i].created = mono();
        if (!ok) {
          cerr.fetch_add(1);
          (*pods)[i].gone = (*pods)[i].created;  // never existed: nothing to wait for
          gone.fetch_add(1);
          cv.notify_all();
        }
      }
    });
  }
  for (int k = 0; k < std::max(1, c.deleters); ++k) {
    th.emplace_back([&] {
      ApiClient api(cfg_);
      std::string resp, e;
      const std::string opts = c.grace < 0 ? std::string("{\"kind\":\"DeleteOptions\",\"apiVersion\":\"v1\"}")
                                           : "{\"kind\":\"DeleteOptions\",\"apiVersion\":\"v1\",\"gracePeriodSeconds\":" +
                                                 std::to_string(c.grace) + "}";
      while (true) {
        size_t i;
        {
          std::unique_lock<std::mutex> lk(mu);
          while (true) {
            if (stop.load()) return;
            if (!dq.empty() && dq.front().first <= mono()) break;
            double w = dq.empty() ? 0.05 : std::max(0.0, dq.front().first - mono());
            cv.wait_for(lk, std::chrono::duration<double>(std::min(w, 0.05)));
          }
          i = dq.front().second;
          dq.pop_front();
        }
        int status = 0;
        bool ok = api.request("DELETE", coll + "/" + prefix + std::to_string(i), opts, "application/json", &status,
                              &resp, &e) && (status == 200 || status == 404);
        std::lock_guard<std::mutex> g(mu);
        (*pods)[i].deleted = mono();
        if (!ok) derr.fetch_add(1);
      }
    });
  }
  {
    const double end = t0 + c.duration_s + c.drain_s;
    std::unique_lock<std::mutex> lk(mu);
    while (gone.load() < n && mono() < end) cv.wait_for(lk, std::chrono::milliseconds(20));
  }
  stop.store(true);
  cv.notify_all();
  for (auto& t : th) t.join();
  r.stop();
  *create_errors = cerr.load();
  *delete_errors = derr.load();
  return true;
}

}  // namespace gsx
