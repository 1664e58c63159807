// gsx-schedsim: kube-scheduler stand-in speaking the extender protocol, in C++.
//
// There is no kube-scheduler in this environment.  This
// replays what it does for a pod requesting a managed extended resource
// (config/scheduler-policy-config.json:4-19), like sim/scheduler.py but
// compiled, so the benchmark measures the extender rather than a Python
// load generator (kube-scheduler itself is compiled Go):
//
//   scheduling cycle (one thread, serial, one pod at a time):
//     NodeResourcesFit on the node aggregate of gpu-mem (ignoredByScheduler:
//     false) -> POST <prefix>/filter {Pod, NodeNames} (nodeCacheCapable) ->
//     pick a node (binpack | spread | first) -> assume the pod on it;
//   binding cycle (a pool of threads, many in flight):
//     POST <prefix>/bind; any error drops the assumption and the pod is
//     retried after a backoff (routes.go:139-143 answers 500).
//
// Pods and nodes come from native reflectors (informer.cc).  Per-pod timings
// are served for the benchmark:
//   POST /v1/timings ["ns/name",...] -> {"ns/name": {seen, filtered, bound,
//        filter_rtt, bind_rtt, attempts, node, error}}  (steady clock seconds)
//   POST /v1/forget  ["ns/name",...]
//   GET  /v1/stats
//
//   gsx-schedsim --apiserver URL --extender URL [--profile shared-gpu|aliyun]
//                [--node-policy binpack|spread|first] [--bind-threads N]
//                [--port P] [--port-file F] [--scheduler-name S]
//                [--nodes-to-score adaptive|all|<percent>]
//
// Node sampling follows kube-scheduler's numFeasibleNodesToFind: below 100
// nodes every feasible node goes to the extender; above, the search stops once
// max(100, N * p / 100) feasible nodes were found, with the adaptive
// p = max(5, 50 - N / 125) percent (percentageOfNodesToScore unset), starting
// where the previous cycle stopped (nextStartNodeIndex).
#include <signal.h>
#include <unistd.h>

#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <fstream>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "apiclient.h"
#include "ctlserver.h"
#include "informer.h"
#include "json.h"
#include "model.h"
#include "quantity.h"

using namespace gsx;

namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Timing {
  double seen = 0, filtered = 0, bound = 0, filter_rtt = 0, bind_rtt = 0;
  int attempts = 0;
  std::string node, error;
};

struct PodInfo {
  std::string uid, ns, name, rv, node, sched;
  bool complete = false, terminal = false;
  int64_t request = 0;
  std::string raw;  // object JSON while pending (the filter request carries it)
};

struct BindJob {
  std::string key, ns, name, uid, node;
};

int64_t quantity_at(const json::Doc& d, int64_t idx) {
  if (idx < 0) return -1;
  int64_t v = 0;
  const json::Val& x = d.at(static_cast<uint32_t>(idx));
  std::string s = x.type == json::T::String ? d.str(static_cast<uint32_t>(idx)) : std::string(d.raw(static_cast<uint32_t>(idx)));
  return parse_quantity(s, &v) ? v : -1;
}

class Sim {
 public:
  Sim(ApiConfig api, ApiConfig ext, Profile p, std::string policy, std::string sched_name, int bind_threads,
      double backoff, double score_pct = 0)
      : p_(std::move(p)), policy_(std::move(policy)), sched_(std::move(sched_name)), ext_(ext), backoff_(backoff),
        score_pct_(score_pct) {
    ReflectorConfig pr;
    pr.path = "/api/v1/pods";
    ReflectorHandler ph;
    ph.on_list = [this](const ListView& lv) {
      std::lock_guard<std::mutex> g(mu_);
      std::unordered_set<std::string> seen;
      for (size_t k = 0; k < lv.size(); ++k) seen.insert(on_pod_locked(lv.doc(k), lv.obj(k)));
      std::vector<std::string> gone;
      for (auto& kv : pods_) {
        if (!seen.count(kv.first)) gone.push_back(kv.first);
      }
      for (auto& k : gone) on_pod_delete_locked(k);
      cv_.notify_all();
    };
    ph.on_event = [this](Ev ev, const json::Doc& d, uint32_t obj) {
      std::lock_guard<std::mutex> g(mu_);
      if (ev == Ev::Deleted) {
        PodView v;
        parse_pod(d, obj, p_, &v);
        on_pod_delete_locked(v.ns + "/" + v.name);
      } else {
        on_pod_locked(d, obj);
      }
      cv_.notify_all();
    };
    pods_r_ = std::make_unique<Reflector>(api, pr, ph);
    ReflectorConfig nr;
    nr.path = "/api/v1/nodes";
    ReflectorHandler nh;
    nh.on_list = [this](const ListView& lv) {
      std::lock_guard<std::mutex> g(mu_);
      nodes_.clear();
      for (size_t k = 0; k < lv.size(); ++k) on_node_locked(lv.doc(k), lv.obj(k));
      cv_.notify_all();
    };
    nh.on_event = [this](Ev ev, const json::Doc& d, uint32_t obj) {
      std::lock_guard<std::mutex> g(mu_);
      if (ev == Ev::Deleted) {
        int64_t n = d.path(obj, {"metadata", "name"});
        if (n >= 0) nodes_.erase(d.str(static_cast<uint32_t>(n)));
      } else {
        on_node_locked(d, obj);
      }
      cv_.notify_all();
    };
    nodes_r_ = std::make_unique<Reflector>(api, nr, nh);
    filter_api_ = std::make_unique<ApiClient>(ext_);
    bind_api_ = std::make_unique<ApiClient>(ext_);
    nbind_ = bind_threads;
  }

  bool start(std::string* err) {
    nodes_r_->start();
    pods_r_->start();
    if (!nodes_r_->wait_synced(60) || !pods_r_->wait_synced(60)) {
      *err = "informers did not sync: " + pods_r_->last_error() + " " + nodes_r_->last_error();
      return false;
    }
    sched_th_ = std::thread([this] { schedule_loop(); });
    for (int i = 0; i < nbind_; ++i) bind_th_.emplace_back([this] { bind_loop(); });
    return true;
  }

  void stop() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    bcv_.notify_all();
    if (sched_th_.joinable()) sched_th_.join();
    for (auto& t : bind_th_) t.join();
    pods_r_->stop();
    nodes_r_->stop();
  }

  CtlServer::Reply handle(const http::Message& req) {
    CtlServer::Reply rep;
    std::string_view path = req.path();
    if (req.method == "POST" && (path == "/v1/timings" || path == "/v1/forget")) {
      json::Doc d;
      std::string err;
      if (!d.parse(req.body, &err) || d.at(0).type != json::T::Array) {
        rep.status = 400;
        rep.body = "{\"error\":\"expected a JSON array of keys\"}";
        return rep;
      }
      std::lock_guard<std::mutex> g(mu_);
      if (path == "/v1/forget") {
        uint32_t end = d.at(0).skip;
        for (uint32_t i = 1; i < end; i = d.next(i)) timings_.erase(d.str(i));
        rep.body = "{\"ok\":true}";
        return rep;
      }
      std::string& o = rep.body;
      o.push_back('{');
      bool first = true;
      uint32_t end = d.at(0).skip;
      char num[512];
      for (uint32_t i = 1; i < end; i = d.next(i)) {
        std::string k = d.str(i);
        auto it = timings_.find(k);
        if (it == timings_.end()) continue;
        const Timing& t = it->second;
        if (!first) o.push_back(',');
        first = false;
        json::append_quoted(&o, k);
        std::snprintf(num, sizeof(num),
                      ":{\"seen\":%.9f,\"filtered\":%.9f,\"bound\":%.9f,\"filter_rtt\":%.9f,\"bind_rtt\":%.9f,"
                      "\"attempts\":%d,\"node\":",
                      t.seen, t.filtered, t.bound, t.filter_rtt, t.bind_rtt, t.attempts);
        o.append(num);
        json::append_quoted(&o, t.node);
        o.append(",\"error\":");
        json::append_quoted(&o, t.error);
        o.push_back('}');
      }
      o.push_back('}');
      return rep;
    }
    if (req.method == "GET" && path == "/v1/stats") {
      std::lock_guard<std::mutex> g(mu_);
      char buf[512];
      std::snprintf(buf, sizeof(buf),
                    "{\"scheduled\":%llu,\"bound\":%llu,\"bind_errors\":%llu,\"unschedulable\":%llu,"
                    "\"filter_calls\":%llu,\"pending\":%zu,\"native\":true}",
                    (unsigned long long)scheduled_, (unsigned long long)bound_, (unsigned long long)bind_errors_,
                    (unsigned long long)unschedulable_, (unsigned long long)filter_calls_, queue_.size());
      rep.body = buf;
      return rep;
    }
    rep.status = 404;
    rep.body = "{\"error\":\"not found\"}";
    return rep;
  }

 private:
  // ---------------------------------------------------------------- intake
  bool pending(const PodInfo& pi) const { return pi.node.empty() && pi.sched == sched_ && !pi.complete; }

  std::string on_pod_locked(const json::Doc& d, uint32_t obj) {
    PodView v;
    parse_pod(d, obj, p_, &v);
    std::string key = v.ns + "/" + v.name;
    PodInfo& pi = pods_[key];
    pi.uid = v.uid;
    pi.ns = v.ns;
    pi.name = v.name;
    pi.rv = v.rv;
    pi.node = v.node;
    pi.complete = v.complete();
    pi.terminal = v.terminal();
    pi.request = v.request;
    int64_t sn = d.path(obj, {"spec", "schedulerName"});
    pi.sched = sn >= 0 ? d.str(static_cast<uint32_t>(sn)) : std::string("default-scheduler");
    account_locked(key, &pi);
    if (pending(pi)) {
      pi.raw.assign(d.raw(obj));
      if (!queued_.count(key) && !assumed_.count(key)) {
        queued_.insert(key);
        Timing& t = timings_[key];
        if (t.seen == 0) t.seen = now_s();
        queue_.push_back(key);
      }
    } else {
      pi.raw.clear();
    }
    return key;
  }

  void on_pod_delete_locked(const std::string& key) {
    account_locked(key, nullptr);
    unassume_locked(key);
    pods_.erase(key);
  }

  // NodeResourcesFit bookkeeping: placed (observed bound, not terminal) + assumed.
  void account_locked(const std::string& key, const PodInfo* pi) {
    auto old = placed_.find(key);
    if (old != placed_.end()) {
      used_[old->second.first] -= old->second.second;
      placed_.erase(old);
    }
    if (!pi) return;
    if (!pi->node.empty() && !pi->terminal) {
      placed_[key] = {pi->node, pi->request};
      used_[pi->node] += pi->request;
      unassume_locked(key);
    }
  }

  void unassume_locked(const std::string& key) {
    auto a = assumed_.find(key);
    if (a != assumed_.end()) {
      used_[a->second.first] -= a->second.second;
      assumed_.erase(a);
    }
  }

  void on_node_locked(const json::Doc& d, uint32_t obj) {
    int64_t n = d.path(obj, {"metadata", "name"});
    if (n < 0) return;
    std::string name = d.str(static_cast<uint32_t>(n));
    int64_t alloc = -1;
    int64_t a = d.path(obj, {"status", "allocatable"});
    if (a >= 0) alloc = quantity_at(d, d.find(static_cast<uint32_t>(a), p_.resource));
    if (alloc < 0) {
      int64_t c = d.path(obj, {"status", "capacity"});
      if (c >= 0) alloc = quantity_at(d, d.find(static_cast<uint32_t>(c), p_.resource));
    }
    nodes_[name] = alloc < 0 ? 0 : alloc;
  }

  // ---------------------------------------------------------------- scheduling cycle
  void retry_later_locked(const std::string& key) { delayed_.push_back({now_s() + backoff_, key}); }

  void schedule_loop() {
    std::unique_lock<std::mutex> lk(mu_);
    while (!stop_) {
      double now = now_s();
      // due retries go back to the queue
      for (auto it = delayed_.begin(); it != delayed_.end();) {
        if (it->first <= now) {
          auto pit = pods_.find(it->second);
          if (pit != pods_.end() && pending(pit->second) && !queued_.count(it->second) &&
              !assumed_.count(it->second)) {
            queued_.insert(it->second);
            queue_.push_back(it->second);
          }
          it = delayed_.erase(it);
        } else {
          ++it;
        }
      }
      if (queue_.empty()) {
        double wait = 0.05;
        for (auto& dl : delayed_) wait = std::min(wait, std::max(0.0, dl.first - now));
        cv_.wait_for(lk, std::chrono::duration<double>(wait));
        continue;
      }
      std::string key = std::move(queue_.front());
      queue_.pop_front();
      queued_.erase(key);
      schedule_one_locked(key, lk);
    }
  }

  void schedule_one_locked(const std::string& key, std::unique_lock<std::mutex>& lk) {
    auto pit = pods_.find(key);
    if (pit == pods_.end() || !pending(pit->second)) return;
    PodInfo pi = pit->second;  // copy: the lock is dropped around the filter call
    Timing& tm = timings_[key];
    if (tm.seen == 0) tm.seen = now_s();
    tm.attempts++;
    // NodeResourcesFit on the aggregate (name order, like the Python simulator's list order), stopping at
    // kube-scheduler's numFeasibleNodesToFind from a rotating start index
    std::vector<std::string> cands;
    const size_t n_all = nodes_.size();
    const size_t want = feasible_to_find(n_all);
    if (node_order_.size() != n_all) {
      node_order_.clear();
      for (auto& kv : nodes_) node_order_.push_back(kv.first);
    }
    size_t processed = 0;
    for (size_t k = 0; k < n_all && cands.size() < want; ++k) {
      const std::string& name = node_order_[(next_start_ + k) % n_all];
      ++processed;
      auto nit = nodes_.find(name);
      if (nit == nodes_.end()) continue;
      int64_t used = used_.count(name) ? used_[name] : 0;
      if (pi.request == 0 || nit->second - used >= pi.request) cands.push_back(name);
    }
    if (n_all) next_start_ = (next_start_ + processed) % n_all;
    if (cands.empty()) {
      unschedulable_++;
      tm.error = "0 nodes available: Insufficient " + p_.resource;
      retry_later_locked(key);
      return;
    }
    std::vector<std::string> names;
    if (pi.request > 0) {
      std::string body;
      body.reserve(pi.raw.size() + 64 + 32 * cands.size());
      body.append("{\"Pod\":").append(pi.raw).append(",\"Nodes\":null,\"NodeNames\":[");
      for (size_t i = 0; i < cands.size(); ++i) {
        if (i) body.push_back(',');
        json::append_quoted(&body, cands[i]);
      }
      body.append("]}");
      lk.unlock();
      double t0 = now_s();
      int status = 0;
      std::string resp, err;
      bool ok = filter_api_->request("POST", "/gpushare-scheduler/filter", body, "application/json", &status, &resp,
                                     &err);
      double rtt = now_s() - t0;
      std::string ferr;
      if (ok) {
        json::Doc d;
        std::string perr;
        if (!d.parse(resp, &perr)) {
          ferr = "bad filter response: " + perr;
        } else {
          int64_t e = d.find(0, "Error", true);
          if (e >= 0 && d.at(static_cast<uint32_t>(e)).type == json::T::String) ferr = d.str(static_cast<uint32_t>(e));
          int64_t nn = d.find(0, "NodeNames", true);
          if (nn >= 0 && d.at(static_cast<uint32_t>(nn)).type == json::T::Array) {
            uint32_t end = d.at(static_cast<uint32_t>(nn)).skip;
            for (uint32_t i = static_cast<uint32_t>(nn) + 1; i < end; i = d.next(i)) names.push_back(d.str(i));
          }
        }
      } else {
        ferr = err;
      }
      lk.lock();
      Timing& t2 = timings_[key];
      t2.filter_rtt = rtt;
      filter_calls_++;
      if (!ferr.empty()) {
        t2.error = ferr;
        retry_later_locked(key);
        return;
      }
      // the pod may have changed while the lock was dropped
      auto again = pods_.find(key);
      if (again == pods_.end() || !pending(again->second)) return;
    } else {
      names = cands;
    }
    Timing& t3 = timings_[key];
    if (names.empty()) {
      unschedulable_++;
      t3.error = "extender filtered all nodes";
      retry_later_locked(key);
      return;
    }
    std::string node = pick_locked(names);
    t3.filtered = now_s();
    assumed_[key] = {node, pi.request};
    used_[node] += pi.request;
    scheduled_++;
    jobs_.push_back(BindJob{key, pi.ns, pi.name, pi.uid, node});
    bcv_.notify_one();
  }

  size_t feasible_to_find(size_t n) const {
    if (score_pct_ == 100 || n < 100) return n;  // all nodes (minFeasibleNodesToFind = 100)
    double pct = score_pct_;
    if (pct <= 0) pct = std::max(5.0, 50.0 - static_cast<double>(n) / 125.0);  // adaptive
    size_t k = static_cast<size_t>(static_cast<double>(n) * pct / 100.0);
    return std::max<size_t>(100, k);
  }

  std::string pick_locked(const std::vector<std::string>& names) {
    if (policy_ == "first" || names.size() == 1) return names[0];
    auto free_of = [&](const std::string& n) {
      auto it = nodes_.find(n);
      int64_t used = used_.count(n) ? used_[n] : 0;
      return it == nodes_.end() ? 0 : it->second - used;
    };
    std::string best = names[0];
    int64_t bf = free_of(best);
    for (size_t i = 1; i < names.size(); ++i) {
      int64_t f = free_of(names[i]);
      bool better = policy_ == "spread" ? (f > bf || (f == bf && names[i] > best))
                                        : (f < bf || (f == bf && names[i] < best));
      if (better) {
        best = names[i];
        bf = f;
      }
    }
    return best;
  }

  // ---------------------------------------------------------------- binding cycle
  void bind_loop() {
    std::unique_lock<std::mutex> lk(mu_);
    while (true) {
      bcv_.wait(lk, [this] { return stop_ || !jobs_.empty(); });
      if (stop_) return;
      BindJob j = std::move(jobs_.front());
      jobs_.pop_front();
      lk.unlock();
      std::string body = "{\"PodName\":";
      json::append_quoted(&body, j.name);
      body.append(",\"PodNamespace\":");
      json::append_quoted(&body, j.ns);
      body.append(",\"PodUID\":");
      json::append_quoted(&body, j.uid);
      body.append(",\"Node\":");
      json::append_quoted(&body, j.node);
      body.push_back('}');
      double t0 = now_s();
      int status = 0;
      std::string resp, err;
      bool ok = bind_api_->request("POST", "/gpushare-scheduler/bind", body, "application/json", &status, &resp, &err);
      double t1 = now_s();
      std::string berr;
      if (!ok) {
        berr = err;
      } else {
        json::Doc d;
        std::string perr;
        if (d.parse(resp, &perr)) {
          int64_t e = d.find(0, "Error", true);
          if (e >= 0 && d.at(static_cast<uint32_t>(e)).type == json::T::String) berr = d.str(static_cast<uint32_t>(e));
        }
        if (berr.empty() && status != 200) berr = "HTTP " + std::to_string(status);
      }
      lk.lock();
      Timing& t = timings_[j.key];
      t.bind_rtt = t1 - t0;
      if (!berr.empty()) {
        bind_errors_++;
        t.error = berr;
        unassume_locked(j.key);
        retry_later_locked(j.key);
        cv_.notify_all();
        continue;
      }
      t.bound = t1;
      t.node = j.node;
      t.error.clear();
      bound_++;
    }
  }

  Profile p_;
  std::string policy_, sched_;
  ApiConfig ext_;
  double backoff_;
  double score_pct_ = 0;  // percentageOfNodesToScore: 0 adaptive, 100 all
  std::vector<std::string> node_order_;  // node names in order (rebuilt when the set changes size)
  size_t next_start_ = 0;
  int nbind_ = 16;
  std::unique_ptr<Reflector> pods_r_, nodes_r_;
  std::unique_ptr<ApiClient> filter_api_, bind_api_;
  std::mutex mu_;
  std::condition_variable cv_, bcv_;
  bool stop_ = false;
  std::unordered_map<std::string, PodInfo> pods_;
  std::map<std::string, int64_t> nodes_;  // name -> allocatable gpu-mem (ordered)
  std::unordered_map<std::string, int64_t> used_;
  std::unordered_map<std::string, std::pair<std::string, int64_t>> placed_, assumed_;
  std::unordered_set<std::string> queued_;
  std::deque<std::string> queue_;
  std::vector<std::pair<double, std::string>> delayed_;
  std::deque<BindJob> jobs_;
  std::unordered_map<std::string, Timing> timings_;
  uint64_t scheduled_ = 0, bound_ = 0, bind_errors_ = 0, unschedulable_ = 0, filter_calls_ = 0;
  std::thread sched_th_;
  std::vector<std::thread> bind_th_;
};

volatile sig_atomic_t g_stop = 0;
void on_sig(int) { g_stop = 1; }

}  // namespace

int main(int argc, char** argv) {
  std::string apiserver, extender, profile = "shared-gpu", policy = "binpack", host = "127.0.0.1", port_file;
  std::string sched = "default-scheduler";
  int port = 0, bind_threads = 16;
  double backoff = 0.05, score_pct = 0;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto val = [&](const char* name) -> std::string {
      if (i + 1 >= argc) {
        std::fprintf(stderr, "missing value for %s\n", name);
        std::exit(2);
      }
      return argv[++i];
    };
    if (a == "--apiserver") apiserver = val("--apiserver");
    else if (a == "--extender") extender = val("--extender");
    else if (a == "--profile") profile = val("--profile");
    else if (a == "--node-policy") policy = val("--node-policy");
    else if (a == "--host") host = val("--host");
    else if (a == "--port") port = std::atoi(val("--port").c_str());
    else if (a == "--port-file") port_file = val("--port-file");
    else if (a == "--bind-threads" || a == "--max-inflight-binds") bind_threads = std::max(1, std::min(256, std::atoi(val("--bind-threads").c_str())));
    else if (a == "--scheduler-name") sched = val("--scheduler-name");
    else if (a == "--retry-backoff") backoff = std::atof(val("--retry-backoff").c_str());
    else if (a == "--nodes-to-score") {
      std::string v = val("--nodes-to-score");
      score_pct = v == "adaptive" ? 0 : v == "all" ? 100 : std::atof(v.c_str());
    }
    else if (a == "-h" || a == "--help") {
      std::printf("usage: gsx-schedsim --apiserver URL --extender URL [--profile P] [--node-policy binpack|spread|first]\n"
                  "                    [--bind-threads N] [--port P] [--port-file F] [--scheduler-name S]\n");
      return 0;
    } else {
      std::fprintf(stderr, "unknown argument %s\n", a.c_str());
      return 2;
    }
  }
  if (apiserver.empty() || extender.empty()) {
    std::fprintf(stderr, "--apiserver and --extender are required\n");
    return 2;
  }
  signal(SIGPIPE, SIG_IGN);
  struct sigaction sa;
  std::memset(&sa, 0, sizeof(sa));
  sa.sa_handler = on_sig;
  sigaction(SIGTERM, &sa, nullptr);
  sigaction(SIGINT, &sa, nullptr);
  ApiConfig api;
  api.server = apiserver;
  ApiConfig ext;
  ext.server = extender;
  ext.timeout_s = 60;
  // bind threads beyond 64 cannot keep their own idle connection in the pool
  Sim sim(api, ext, profile_by_name(profile), policy, sched, std::min(bind_threads, 64), backoff, score_pct);
  std::string err;
  if (!sim.start(&err)) {
    std::fprintf(stderr, "gsx-schedsim: %s\n", err.c_str());
    return 1;
  }
  CtlServer srv([&](const http::Message& m) { return sim.handle(m); });
  int bound = srv.start(host, port, &err);
  if (bound < 0) {
    std::fprintf(stderr, "gsx-schedsim: %s\n", err.c_str());
    return 1;
  }
  if (!port_file.empty()) {
    std::string tmp = port_file + ".tmp";
    {
      std::ofstream f(tmp);
      f << bound;
    }
    std::rename(tmp.c_str(), port_file.c_str());
  }
  while (!g_stop) ::usleep(20000);
  srv.stop();
  sim.stop();
  return 0;
}
