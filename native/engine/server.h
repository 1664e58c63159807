// Native HTTP front end of the scheduler extender.
//
// The reference extender is a Go net/http server (cmd/main.go:119-128,
// pkg/routes/routes.go).  Here the hot verbs are served entirely in C++:
//
//   POST /gpushare-scheduler/filter   native ledger check (no GIL)
//   POST /gpushare-scheduler/bind     native reserve + one apiserver
//                                     POST pods/{name}/binding carrying the
//                                     allocation annotations (bind pool)
//   GET  /gpushare-scheduler/inspect  native
//   GET  /version                     native
//
// Every bind is decided here, including the ones the filter never saw (the pod
// then comes from the controller's lister or one live GET, gpushare-bind.go:
// 44-65) and both bind modes; a client-side QPS limit (--kube-qps) is a token
// bucket in front of every apiserver call this server makes.  Anything else
// (/metrics, /debug/pprof/*, /healthz) is proxied to the Python aiohttp app on
// a loopback port, so the observable API is one server.
//
// Design: N event-loop threads, each with its own SO_REUSEPORT listening
// socket and epoll set (the kernel spreads connections); blocking work (the
// apiserver round trip, proxying) runs on a small thread pool and completes
// back to the owning loop through an eventfd.  One request per connection is
// in flight at a time, so responses stay ordered.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <list>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "apiclient.h"
#include "http.h"
#include "ledger.h"

namespace gsx {

struct ServerConfig {
  std::string host = "0.0.0.0";
  int port = 0;
  int threads = 2;
  int pool_threads = 16;
  int fallback_port = 0;      // Python app on 127.0.0.1 (0: none)
  // bind_mode "update": the reference's two calls, annotate the pod (merge patch, resourceVersion precondition,
  // one retry on the optimistic-lock conflict) then POST a plain Binding (pkg/cache/nodeinfo.go:145-189)
  bool update_mode = false;
  double reservation_ttl = 60.0;
  // client-side apiserver rate limit of the bind / move calls (client-go's QPS / Burst); qps <= 0: unlimited
  double qps = 0.0;
  int burst = 10;
  ApiConfig api;
  size_t max_body = 64u << 20;
  // who may call the device plugin's endpoints (/move, /physical): "none" (anyone who reaches the port: tests, a
  // loopback-only deployment) or "tokenreview" (a bearer token the apiserver's TokenReview authenticates as one of
  // plugin_users, e.g. system:serviceaccount:kube-system:gpushare-device-plugin; cached plugin_auth_ttl seconds)
  std::string plugin_auth = "none";
  std::vector<std::string> plugin_users;
  double plugin_auth_ttl = 60.0;
  // after a (re)start or a leader change, binds to a node whose device plugin publishes its unaccounted GPU use wait
  // at most this long for the plugin's first publication of the new epoch (Ledger::begin_epoch); 0: no wait
  double publication_hold_s = 5.0;
};

struct BindFailure {
  std::string ns, name, uid, node, message;
};

struct LatencyHist {
  static constexpr int kBuckets = 15;
  static const double kBounds[kBuckets];
  std::atomic<uint64_t> counts[kBuckets + 1];
  std::atomic<uint64_t> n{0};
  std::atomic<uint64_t> sum_ns{0};
  LatencyHist() {
    for (auto& c : counts) c.store(0);
  }
  void observe(double seconds);
};

struct ServerStats {
  std::atomic<uint64_t> requests{0}, filters{0}, binds{0}, bind_ok{0}, bind_fail{0}, proxied{0}, bad_requests{0},
      inspects{0}, connections{0}, api_calls{0}, conflicts_retried{0}, bind_order_waits{0}, moves{0}, moves_failed{0},
      unfiltered_binds{0}, live_gets{0}, qps_waits{0}, physical_posts{0}, plugin_auth_denied{0},
      token_reviews{0}, backoffs{0}, publication_waits{0}, physical_refused{0};
  LatencyHist filter_lat, bind_lat, api_lat;
};

class NativeServer {
 public:
  NativeServer(Ledger* ledger, ServerConfig cfg);
  ~NativeServer();
  // Binds and starts the loops; returns the bound port (> 0) or -1 with *err.
  int start(std::string* err);
  void stop();
  int port() const { return port_; }
  const ServerStats& stats() const { return stats_; }
  // apiserver responses sent again after a 429 / Retry-After (ApiClient), and the seconds waited for them
  uint64_t api_throttled() const { return api_ ? api_->throttled() : 0; }
  double api_throttle_wait_s() const { return api_ ? api_->throttle_wait_s() : 0.0; }
  std::vector<BindFailure> drain_failures();
  // HA standby: a replica that does not hold the leader Lease refuses binds (and the device plugin's /move and
  // /physical).  Becoming the leader starts a new epoch (new_epoch).
  void set_binds_enabled(bool on);
  // this extender's epoch: a boot id and the number of times it became the leader ("<boot>.<n>").  Answered on
  // GET .../epoch and with every /physical and /move; a device plugin that sees it change republishes at once
  std::string epoch() const;
  // switch to the reference's annotate-then-bind calls at run time (the apiserver dropped Binding annotations)
  void set_update_mode(bool on) { update_mode_.store(on); }
  bool update_mode() const { return update_mode_.load(); }
  bool binds_enabled() const { return binds_enabled_.load(); }
  // the controller's lister: raw JSON of the pod "ns/name" (false: not held).  Set before start().
  using Lister = std::function<bool(const std::string& key, std::string* raw)>;
  void set_lister(Lister f) { lister_ = std::move(f); }

 private:
  struct Loop;
  struct Conn;
  struct Job {
    Loop* loop;
    uint64_t conn_id;
    int kind;  // 0 bind, 1 proxy, 2 move, 3 physical
    http::Message req;
    double t0;
  };

  void run_loop(Loop* lp);
  void on_readable(Loop* lp, Conn* c);
  void process(Loop* lp, Conn* c);
  void safe_process(Loop* lp, Conn* c);  // process() that closes only this connection on an exception
  void dispatch(Loop* lp, Conn* c, http::Message& req);
  void respond(Loop* lp, Conn* c, std::string resp, bool keep_alive);
  void flush(Loop* lp, Conn* c);
  void close_conn(Loop* lp, Conn* c);
  void complete(Loop* lp, uint64_t conn_id, std::string resp, bool keep_alive);
  void drain_completions(Loop* lp);
  void pool_main();
  void submit(Job j);
  std::string do_bind(const http::Message& req);
  // the pod of a bind the filter did not see here: lister first, one live GET when the lister does not hold
  // it under that UID; false with the reference's error string (gpushare-bind.go:44-65)
  bool lookup_pod(const std::string& ns, const std::string& name, const std::string& uid, bool live,
                  Ledger::PendingPod* out, std::string* err);
  // one apiserver call behind the QPS limit
  bool api_call(const char* method, const std::string& target, const std::string& body, const char* ct, int* status,
                std::string* resp, std::string* err);
  void throttle();
  std::string do_proxy(const http::Message& req);
  // token_node: the node the caller's token is bound to (its TokenReview's node-name claim), "" when it has none
  std::string do_move(const http::Message& req, const std::string& token_node = std::string());
  std::string do_physical(const http::Message& req, const std::string& token_node = std::string());
  // the caller of a device-plugin endpoint is the plugin (ServerConfig::plugin_auth); false with the 401/403 answer
  bool plugin_authorized(const http::Message& req, std::string* resp, std::string* token_node);
  std::string bind_error_response(const std::string& msg) const;
  void record_failure(BindFailure f);
  void new_epoch();
  // wait (bounded) until `node`'s device plugin has published in this epoch; false: stopping
  void wait_publication(const std::string& node);
  std::string boot_id_;
  std::atomic<uint64_t> epoch_gen_{0};
  std::mutex pub_mu_;
  std::condition_variable pub_cv_;
  std::atomic<uint64_t> publication_wait_ns_{0};

  Ledger* l_;
  ServerConfig cfg_;
  int port_ = -1;
  std::atomic<bool> stop_{false};
  std::atomic<bool> binds_enabled_{true};
  std::atomic<bool> update_mode_{false};
  std::vector<std::unique_ptr<Loop>> loops_;
  std::vector<std::thread> loop_threads_;
  std::vector<std::thread> pool_threads_;
  std::mutex jmu_;
  std::condition_variable jcv_;
  std::deque<Job> jobs_;
  std::unique_ptr<ApiClient> api_;
  std::unique_ptr<ApiClient> fallback_;
  Lister lister_;
  std::mutex qmu_;  // token bucket
  double q_tokens_ = 0.0, q_last_ = 0.0;
  std::mutex fmu_;
  std::vector<BindFailure> failures_;
  // TokenReview cache: token -> verdict until `until` (allowed, or denied: a denial is cached briefly too, so a
  // caller repeating a bad token does not cost the apiserver a review per request), and the node its pod is on
  struct Authz {
    double until = 0;
    bool allowed = false;
    int status = 0;
    std::string msg, node;
  };
  std::mutex amu_;
  std::unordered_map<std::string, Authz> authz_cache_;
  double review_tokens_ = 0, review_last_ = 0;  // token bucket for reviews not answered from the cache
  ServerStats stats_;
  // bind ordering lives in the ledger (Ledger::assume_ordered / bind_wait / bind_leave): one in-flight
  // set for the native binds and the Python slow path alike
};

}  // namespace gsx
