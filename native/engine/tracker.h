// Load-generator helpers for the benchmark's wave driver, in C++ so the
// driver process measures the cluster rather than its own JSON decoding:
//
//   PodTracker   a reflector over the wave's pods (namespace + label selector)
//                that answers "are all these pods bound / Running / gone?"
//                with a blocking wait woken by watch events;
//   BatchClient  issues a list of apiserver requests concurrently over a
//                keep-alive connection pool (the wave's pod creates);
//   OpenLoop     constant-rate pod arrivals with every pod's stages timed
//                (arrival -> bound -> Running -> deleted -> gone), each pod
//                deleted once it runs: the sustained throughput of the whole
//                stack with many pods in flight (bench.py --open-loop).
#pragma once

#include <atomic>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "apiclient.h"
#include "informer.h"

namespace gsx {

class PodTracker {
 public:
  // Stopped: gone, or in a terminal phase (its kubelet stopped the containers of a gracefully deleted pod and
  // reported it; the object goes a moment later)
  enum Cond : int { Bound = 0, Running = 1, Gone = 2, Stopped = 3 };
  PodTracker(const ApiConfig& cfg, const std::string& ns, const std::string& label_selector);
  ~PodTracker();
  bool start(double timeout_s, std::string* err);
  void stop();
  // "" once every key satisfies `cond`; "timeout ..." or "pod <key> Failed" otherwise.
  std::string wait(const std::vector<std::string>& keys, int cond, double timeout_s);
  size_t size() const;

 private:
  struct St {
    std::string node, phase;
  };
  bool ok_locked(const std::string& key, int cond, std::string* err) const;

  std::unique_ptr<Reflector> r_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::unordered_map<std::string, St> pods_;
};

struct OpenLoopConfig {
  std::string ns = "default";
  std::string label_key = "gsx-ol";  // the run's pods carry label_key=<run> (the watch selects them)
  std::string run;
  // the pod object with __NAME__ where its name goes (its labels must include label_key: run)
  std::string pod_tmpl;
  double rate = 1000;        // arrivals per second
  double duration_s = 2.0;   // arrivals for this long
  double warm_s = 0.5;       // the first warm_s of arrivals are not counted
  double hold_s = 0.0;       // a pod runs this long before it is deleted
  double drain_s = 20.0;     // after the last arrival: wait this long for the pods to run and go
  int creators = 16, deleters = 16;
  // DELETE's gracePeriodSeconds: < 0 sends none (the pod's spec.terminationGracePeriodSeconds: a graceful deletion
  // its kubelet ends once the containers stopped), 0 deletes outright (a force delete)
  int grace = -1;
};

struct OpenLoopPod {
  double arrival = 0, created = 0, bound = 0, running = 0, deleted = 0, gone = 0;
  bool failed = false;
};

class OpenLoop {
 public:
  explicit OpenLoop(const ApiConfig& cfg) : cfg_(cfg) {}
  // runs to the end (all pods gone, or drain_s passed); false + *err only when the watch never synced
  bool run(const OpenLoopConfig& c, std::vector<OpenLoopPod>* pods, std::string* err, int* create_errors,
           int* delete_errors);

 private:
  ApiConfig cfg_;
};

class BatchClient {
 public:
  using Req = std::tuple<std::string, std::string, std::string>;
  explicit BatchClient(const ApiConfig& cfg) : api_(cfg) {}
  ~BatchClient();
  // (method, path, body) -> (status or -1, response body / transport error).  The helper threads are kept between
  // calls (a wave's creates used to start and join up to 15 threads inside the timed wave)
  std::vector<std::pair<int, std::string>> run(const std::vector<Req>& reqs, int concurrency);

 private:
  void work_on(const std::vector<Req>& reqs, std::vector<std::pair<int, std::string>>* out);
  void helper(int me);

  ApiClient api_;
  std::mutex run_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<std::thread> helpers_;
  // the batch in progress: helpers with index < want_ join it
  const std::vector<Req>* reqs_ = nullptr;
  std::vector<std::pair<int, std::string>>* out_ = nullptr;
  std::atomic<size_t> next_{0};
  uint64_t gen_ = 0;
  int want_ = 0, busy_ = 0;
  bool stop_ = false;
};

}  // namespace gsx
