#include "tracker.h"

#include <atomic>
#include <chrono>
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
             (cond == Bound ? "bound" : cond == Running ? "Running" : "gone") + ", e.g. " + keys[i];
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
