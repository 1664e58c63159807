// Load-generator helpers for the benchmark's wave driver, in C++ so the
// driver process measures the cluster rather than its own JSON decoding:
//
//   PodTracker   a reflector over the wave's pods (namespace + label selector)
//                that answers "are all these pods bound / Running / gone?"
//                with a blocking wait woken by watch events;
//   BatchClient  issues a list of apiserver requests concurrently over a
//                keep-alive connection pool (the wave's pod creates).
#pragma once

#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "apiclient.h"
#include "informer.h"

namespace gsx {

class PodTracker {
 public:
  enum Cond : int { Bound = 0, Running = 1, Gone = 2 };
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

class BatchClient {
 public:
  explicit BatchClient(const ApiConfig& cfg) : api_(cfg) {}
  // (method, path, body) -> (status or -1, response body / transport error)
  std::vector<std::pair<int, std::string>> run(
      const std::vector<std::tuple<std::string, std::string, std::string>>& reqs, int concurrency);

 private:
  ApiClient api_;
};

}  // namespace gsx
