// Blocking HTTP/1.1 client with a keep-alive connection pool (plain TCP or
// TLS via OpenSSL) for the native bind path: one POST pods/{name}/binding per
// bind.  Replaces client-go's REST client on the hot path
// (pkg/cache/nodeinfo.go:150-189); no client-side QPS throttle by default
// (client-go's 5 QPS / burst 10 is what caps the reference at ~2.5 binds/s).
#pragma once

#include <atomic>
#include <condition_variable>
#include <functional>
#include <string_view>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "http.h"

typedef struct ssl_ctx_st SSL_CTX;
typedef struct ssl_st SSL;

namespace gsx {

struct ApiConfig {
  std::string server;  // http(s)://host:port
  std::string token;   // bearer token
  std::string token_file;      // re-read every token_reload_s (kubelet rotates projected SA tokens)
  double token_reload_s = 60.0;
  std::string ca_file, cert_file, key_file;
  bool insecure = false;
  double timeout_s = 30.0;
  std::string user_agent = "gpushare-schd-extender-amd/0.1.0 (native)";
  // client-go's contract (vendor/k8s.io/client-go/rest/request.go:658-734,973-995): a 429 Too Many Requests (API
  // Priority and Fairness rejected the request before it ran, so any method is safe to repeat), or a 5xx that
  // carries Retry-After, is sent again after the server's Retry-After -- at most max_attempts sends in all.  A 429
  // without Retry-After waits a capped exponential backoff with jitter instead (backoff_base_s doubling up to
  // backoff_max_s).  A 5xx without Retry-After is returned to the caller: a write may have been applied, and the
  // caller knows whether repeating it is safe (the bind path does, with its own backoff).  max_attempts 1: off.
  int max_attempts = 10;
  double backoff_base_s = 0.005, backoff_max_s = 1.0;
  double retry_after_max_s = 30.0;  // a longer Retry-After is clamped (kube-apiserver's APF sends 1-8 s)
};

// Lets another thread end a running ApiClient::stream() (shuts the socket).
struct StreamHandle {
  std::atomic<int> fd{-1};
  std::atomic<bool> aborted{false};
  void abort();
};

class ApiClient {
 public:
  explicit ApiClient(ApiConfig cfg);
  ~ApiClient();
  bool ok() const { return ok_; }
  const std::string& init_error() const { return init_err_; }

  // Performs one request; returns false only on transport errors (then *err
  // is set).  HTTP error statuses are returned in *status.
  bool request(const std::string& method, const std::string& path, const std::string& body,
               const char* content_type, int* status, std::string* resp, std::string* err,
               std::string* resp_content_type = nullptr);

  // Streams one GET on a dedicated connection (watch).  Decoded body bytes
  // (chunked or length / close delimited) go to on_data; returning false
  // from it ends the stream.  For HTTP status >= 400 the body is collected
  // into *error_body instead.  Returns false on transport errors (*err set);
  // a stream that ends cleanly (server timeout, abort) returns true.
  // idle_timeout_s bounds a silent connection.
  bool stream(const std::string& path, int* status, std::string* error_body,
              const std::function<bool(std::string_view)>& on_data, std::string* err, StreamHandle* h,
              double idle_timeout_s);

  // The owner is closing: the sockets of requests in flight are shut (they fail with a transport error at once
  // instead of waiting out a slow apiserver) and later requests fail without connecting.
  void abort();

  uint64_t requests() const { return requests_; }
  uint64_t reconnects() const { return reconnects_; }
  // responses answered 429 / 5xx-with-Retry-After that were sent again, and the time spent waiting for that
  uint64_t throttled() const { return throttled_; }
  double throttle_wait_s() const { return static_cast<double>(throttle_wait_ns_.load()) * 1e-9; }
  // the wait before resending a request answered `status` with Retry-After `retry_after` ("" absent) on send
  // `attempt` (0-based); < 0: not retried (see ApiConfig::max_attempts)
  static double retry_wait(const ApiConfig& cfg, const std::string& method, int status, const std::string& retry_after,
                           int attempt, double jitter01);

 private:
  struct Conn {
    int fd = -1;
    SSL* ssl = nullptr;
    std::string rbuf;
  };
  bool request_once(const std::string& req, int* status, std::string* resp, std::string* err,
                    std::string* resp_content_type, std::string* retry_after);
  bool wait_or_abort(double seconds);  // false: abort() was called
  std::mutex wait_mu_;
  std::condition_variable wait_cv_;
  std::atomic<uint64_t> throttled_{0}, throttle_wait_ns_{0};
  Conn* acquire(std::string* err);
  Conn* connect_new(std::string* err);
  std::string request_head(const std::string& method, const std::string& path, size_t body_len,
                           const char* content_type, bool has_body) const;
  void release(Conn* c, bool reuse);
  void close_conn(Conn* c);
  bool send_all(Conn* c, const std::string& data);
  long recv_some(Conn* c, char* buf, size_t n);

  ApiConfig cfg_;
  std::string bearer() const;  // cfg_.token, refreshed from cfg_.token_file when it is due
  mutable std::mutex tok_mu_;
  mutable std::string tok_;
  mutable double tok_at_ = 0.0;
  http::Url url_;
  SSL_CTX* ctx_ = nullptr;
  bool ok_ = false;
  std::string init_err_;
  std::mutex mu_;
  std::vector<Conn*> idle_;
  std::vector<int> busy_;  // fds of requests in flight (guarded by mu_), for abort()
  bool aborted_ = false;   // guarded by mu_
  std::atomic<uint64_t> requests_{0}, reconnects_{0};
};

}  // namespace gsx
