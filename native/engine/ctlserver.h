// Small blocking HTTP/1.1 server for low-rate control endpoints of the native
// tools (scheduler simulator timings / stats).  One thread per connection,
// keep-alive, request handler called serially per connection.  The extender's
// own hot verbs are served by NativeServer (server.h), not by this.
#pragma once

#include <atomic>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "http.h"

namespace gsx {

class CtlServer {
 public:
  // Handler: request -> (status, content type, body).
  struct Reply {
    int status = 200;
    std::string content_type = "application/json";
    std::string body;
  };
  using Handler = std::function<Reply(const http::Message&)>;

  explicit CtlServer(Handler h) : h_(std::move(h)) {}
  ~CtlServer() { stop(); }
  // Returns the bound port or -1 (*err).
  int start(const std::string& host, int port, std::string* err);
  // CPUs the server's threads (acceptor, connections) run on; empty: inherit the creator's.  Before start().
  void set_cpus(std::vector<int> cpus) { cpus_ = std::move(cpus); }
  void stop();

 private:
  void accept_loop();
  void serve_conn(int fd);

  void pin_thread() const;

  Handler h_;
  std::vector<int> cpus_;
  int lfd_ = -1;
  std::atomic<bool> stop_{false};
  std::thread acc_;
  std::mutex mu_;
  std::vector<int> conns_;
  std::map<uint64_t, std::thread> threads_;  // per connection; joined once finished (see accept_loop)
  std::vector<uint64_t> finished_;            // connections whose thread has returned
  uint64_t next_conn_ = 0;
};

}  // namespace gsx
