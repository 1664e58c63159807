// Blocking HTTP/1.1 client with a keep-alive connection pool (plain TCP or
// TLS via OpenSSL) for the native bind path: one POST pods/{name}/binding per
// bind.  Replaces client-go's REST client on the hot path
// (pkg/cache/nodeinfo.go:150-189); no client-side QPS throttle by default
// (client-go's 5 QPS / burst 10 is what caps the reference at ~2.5 binds/s).
#pragma once

#include <atomic>
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
  std::string ca_file, cert_file, key_file;
  bool insecure = false;
  double timeout_s = 30.0;
  std::string user_agent = "gpushare-schd-extender-amd/0.1.0 (native)";
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

  uint64_t requests() const { return requests_; }
  uint64_t reconnects() const { return reconnects_; }

 private:
  struct Conn {
    int fd = -1;
    SSL* ssl = nullptr;
    std::string rbuf;
  };
  Conn* acquire(std::string* err);
  void release(Conn* c, bool reuse);
  void close_conn(Conn* c);
  bool send_all(Conn* c, const std::string& data);
  long recv_some(Conn* c, char* buf, size_t n);

  ApiConfig cfg_;
  http::Url url_;
  SSL_CTX* ctx_ = nullptr;
  bool ok_ = false;
  std::string init_err_;
  std::mutex mu_;
  std::vector<Conn*> idle_;
  std::atomic<uint64_t> requests_{0}, reconnects_{0};
};

}  // namespace gsx
