#include "apiclient.h"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <openssl/err.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <fstream>
#include <sstream>
#include <cstdio>
#include <cstring>
#include <algorithm>

namespace gsx {

namespace {

std::string ssl_err() {
  unsigned long e = ERR_get_error();
  char buf[256];
  ERR_error_string_n(e, buf, sizeof(buf));
  return buf;
}

bool is_ip(const std::string& h) {
  unsigned char b[16];
  return inet_pton(AF_INET, h.c_str(), b) == 1 || inet_pton(AF_INET6, h.c_str(), b) == 1;
}

}  // namespace

ApiClient::ApiClient(ApiConfig cfg) : cfg_(std::move(cfg)) {
  if (!http::parse_url(cfg_.server, &url_)) {
    init_err_ = "bad apiserver url: " + cfg_.server;
    return;
  }
  if (url_.tls) {
    ctx_ = SSL_CTX_new(TLS_client_method());
    if (!ctx_) {
      init_err_ = "SSL_CTX_new: " + ssl_err();
      return;
    }
    SSL_CTX_set_min_proto_version(ctx_, TLS1_2_VERSION);
    if (cfg_.insecure) {
      SSL_CTX_set_verify(ctx_, SSL_VERIFY_NONE, nullptr);
    } else {
      SSL_CTX_set_verify(ctx_, SSL_VERIFY_PEER, nullptr);
      int r = cfg_.ca_file.empty() ? SSL_CTX_set_default_verify_paths(ctx_)
                                   : SSL_CTX_load_verify_locations(ctx_, cfg_.ca_file.c_str(), nullptr);
      if (r != 1) {
        init_err_ = "loading CA: " + ssl_err();
        return;
      }
    }
    if (!cfg_.cert_file.empty() && !cfg_.key_file.empty()) {
      if (SSL_CTX_use_certificate_chain_file(ctx_, cfg_.cert_file.c_str()) != 1 ||
          SSL_CTX_use_PrivateKey_file(ctx_, cfg_.key_file.c_str(), SSL_FILETYPE_PEM) != 1) {
        init_err_ = "loading client cert: " + ssl_err();
        return;
      }
    }
  }
  ok_ = true;
}

ApiClient::~ApiClient() {
  std::lock_guard<std::mutex> g(mu_);
  for (Conn* c : idle_) {
    close_conn(c);
    delete c;
  }
  idle_.clear();
  if (ctx_) SSL_CTX_free(ctx_);
}

void ApiClient::abort() {
  {
    std::lock_guard<std::mutex> g(mu_);
    aborted_ = true;
    for (int fd : busy_) ::shutdown(fd, SHUT_RDWR);
  }
  std::lock_guard<std::mutex> w(wait_mu_);
  wait_cv_.notify_all();
}

bool ApiClient::wait_or_abort(double seconds) {
  std::unique_lock<std::mutex> w(wait_mu_);
  return !wait_cv_.wait_for(w, std::chrono::duration<double>(seconds), [this] {
    std::lock_guard<std::mutex> g(mu_);
    return aborted_;
  });
}

double ApiClient::retry_wait(const ApiConfig& cfg, const std::string& method, int status,
                             const std::string& retry_after, int attempt, double jitter01) {
  (void)method;  // 429s are rejected before any handler ran: every verb is safe to repeat
  if (attempt + 1 >= cfg.max_attempts) return -1;
  const bool throttled = status == 429;
  if (!throttled && status < 500) return -1;
  if (!retry_after.empty()) {
    char* end = nullptr;
    double s = std::strtod(retry_after.c_str(), &end);
    // seconds (client-go reads an integer; a fraction is honoured too); an HTTP-date is treated as absent
    if (end != retry_after.c_str() && *end == '\0' && s >= 0) return std::min(s, cfg.retry_after_max_s);
  }
  if (!throttled) return -1;  // 5xx without Retry-After: the caller decides
  double b = cfg.backoff_base_s * static_cast<double>(1ull << std::min(attempt, 20));
  b = std::min(b, cfg.backoff_max_s);
  return b * (0.5 + 0.5 * jitter01);  // jitter: [b/2, b)
}

void ApiClient::close_conn(Conn* c) {
  if (c->ssl) {
    SSL_shutdown(c->ssl);
    SSL_free(c->ssl);
    c->ssl = nullptr;
  }
  if (c->fd >= 0) ::close(c->fd);
  c->fd = -1;
}

ApiClient::Conn* ApiClient::acquire(std::string* err) {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (!idle_.empty()) {
      Conn* c = idle_.back();
      idle_.pop_back();
      return c;
    }
  }
  return connect_new(err);
}

ApiClient::Conn* ApiClient::connect_new(std::string* err) {
  addrinfo hints;
  std::memset(&hints, 0, sizeof(hints));
  hints.ai_socktype = SOCK_STREAM;
  hints.ai_family = AF_UNSPEC;
  addrinfo* res = nullptr;
  std::string port = std::to_string(url_.port);
  int gr = getaddrinfo(url_.host.c_str(), port.c_str(), &hints, &res);
  if (gr != 0) {
    *err = std::string("resolve ") + url_.host + ": " + gai_strerror(gr);
    return nullptr;
  }
  int fd = -1;
  for (addrinfo* a = res; a; a = a->ai_next) {
    fd = ::socket(a->ai_family, a->ai_socktype | SOCK_CLOEXEC, a->ai_protocol);
    if (fd < 0) continue;
    timeval tv;
    tv.tv_sec = static_cast<long>(cfg_.timeout_s);
    tv.tv_usec = static_cast<long>((cfg_.timeout_s - static_cast<double>(tv.tv_sec)) * 1e6);
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
    setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    if (::connect(fd, a->ai_addr, a->ai_addrlen) == 0) break;
    ::close(fd);
    fd = -1;
  }
  freeaddrinfo(res);
  if (fd < 0) {
    *err = "connect " + cfg_.server + ": " + std::strerror(errno);
    return nullptr;
  }
  Conn* c = new Conn();
  c->fd = fd;
  if (url_.tls) {
    c->ssl = SSL_new(ctx_);
    SSL_set_fd(c->ssl, fd);
    if (!is_ip(url_.host)) SSL_set_tlsext_host_name(c->ssl, url_.host.c_str());  // no IP literals in SNI (RFC 6066)
    if (!cfg_.insecure) {
      X509_VERIFY_PARAM* p = SSL_get0_param(c->ssl);
      if (is_ip(url_.host)) {
        X509_VERIFY_PARAM_set1_ip_asc(p, url_.host.c_str());
      } else {
        X509_VERIFY_PARAM_set1_host(p, url_.host.c_str(), 0);
      }
    }
    if (SSL_connect(c->ssl) != 1) {
      *err = "TLS handshake with " + cfg_.server + ": " + ssl_err();
      close_conn(c);
      delete c;
      return nullptr;
    }
  }
  ++reconnects_;
  return c;
}

void ApiClient::release(Conn* c, bool reuse) {
  if (!reuse) {
    close_conn(c);
    delete c;
    return;
  }
  std::lock_guard<std::mutex> g(mu_);
  if (idle_.size() >= 64) {
    close_conn(c);
    delete c;
    return;
  }
  idle_.push_back(c);
}

namespace {
// An SSL call that failed only because a signal interrupted the underlying recv/send: the /debug/pprof stack
// sampler signals every native thread, and on sockets with SO_RCVTIMEO/SO_SNDTIMEO the kernel never restarts
// those calls (signal(7)), SA_RESTART or not.  A timeout (EAGAIN) is not retried.
bool ssl_interrupted(SSL* ssl, int r, int saved_errno) {
  int e = SSL_get_error(ssl, r);
  return (e == SSL_ERROR_SYSCALL || e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE) && saved_errno == EINTR;
}
}  // namespace

bool ApiClient::send_all(Conn* c, const std::string& data) {
  size_t off = 0;
  while (off < data.size()) {
    long w;
    if (c->ssl) {
      errno = 0;
      int r = SSL_write(c->ssl, data.data() + off, static_cast<int>(data.size() - off));
      int err = errno;
      if (r <= 0) {
        if (ssl_interrupted(c->ssl, r, err)) continue;  // SSL_write must be repeated with the same arguments
        return false;
      }
      w = r;
    } else {
      w = ::send(c->fd, data.data() + off, data.size() - off, MSG_NOSIGNAL);
      if (w < 0) {
        if (errno == EINTR) continue;
        return false;
      }
    }
    off += static_cast<size_t>(w);
  }
  return true;
}

long ApiClient::recv_some(Conn* c, char* buf, size_t n) {
  if (c->ssl) {
    while (true) {
      errno = 0;
      int r = SSL_read(c->ssl, buf, static_cast<int>(n));
      int err = errno;
      if (r > 0) return r;
      if (ssl_interrupted(c->ssl, r, err)) continue;
      return SSL_get_error(c->ssl, r) == SSL_ERROR_ZERO_RETURN ? 0 : -1;
    }
  }
  while (true) {
    long r = ::recv(c->fd, buf, n, 0);
    if (r < 0 && errno == EINTR) continue;
    return r;
  }
}

std::string ApiClient::bearer() const {
  if (cfg_.token_file.empty()) return cfg_.token;
  const double now = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  std::lock_guard<std::mutex> g(tok_mu_);
  if (tok_at_ == 0.0 || now - tok_at_ >= cfg_.token_reload_s) {
    tok_at_ = now;
    std::ifstream f(cfg_.token_file);
    std::stringstream ss;
    if (f) ss << f.rdbuf();
    std::string t = ss.str();
    while (!t.empty() && (t.back() == '\n' || t.back() == '\r' || t.back() == ' ')) t.pop_back();
    if (!t.empty()) {
      tok_ = t;
    } else if (tok_.empty()) {
      tok_ = cfg_.token;  // unreadable file: keep what we were given
    }
  }
  return tok_;
}

std::string ApiClient::request_head(const std::string& method, const std::string& path, size_t body_len,
                                    const char* content_type, bool has_body) const {
  std::string req;
  req.reserve(256 + body_len);
  req.append(method).append(" ").append(url_.prefix).append(path).append(" HTTP/1.1\r\nHost: ");
  req.append(url_.host);
  if ((url_.tls && url_.port != 443) || (!url_.tls && url_.port != 80)) req.append(":").append(std::to_string(url_.port));
  req.append("\r\nUser-Agent: ").append(cfg_.user_agent);
  req.append("\r\nAccept: application/json\r\n");
  const std::string tok = bearer();
  if (!tok.empty()) req.append("Authorization: Bearer ").append(tok).append("\r\n");
  if (has_body) {
    req.append("Content-Type: ").append(content_type ? content_type : "application/json").append("\r\n");
    req.append("Content-Length: ").append(std::to_string(body_len)).append("\r\n");
  }
  req.append("\r\n");
  return req;
}

void StreamHandle::abort() {
  aborted.store(true);
  int fd_ = fd.load();
  if (fd_ >= 0) ::shutdown(fd_, SHUT_RDWR);
}

bool ApiClient::stream(const std::string& path, int* status, std::string* error_body,
                       const std::function<bool(std::string_view)>& on_data, std::string* err, StreamHandle* h,
                       double idle_timeout_s) {
  if (!ok_) {
    *err = init_err_;
    return false;
  }
  if (h->aborted.load()) return true;
  Conn* c = connect_new(err);
  if (!c) return false;
  struct Closer {
    ApiClient* self;
    Conn* c;
    StreamHandle* h;
    ~Closer() {
      h->fd.store(-1);
      self->close_conn(c);
      delete c;
    }
  } closer{this, c, h};
  h->fd.store(c->fd);
  if (h->aborted.load()) return true;  // abort raced with the connect
  timeval tv;
  tv.tv_sec = static_cast<long>(idle_timeout_s);
  tv.tv_usec = 0;
  setsockopt(c->fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  if (!send_all(c, request_head("GET", path, 0, nullptr, false))) {
    if (h->aborted.load()) return true;
    *err = "send to apiserver failed";
    return false;
  }
  ++requests_;
  char buf[65536];
  std::string head;
  http::Message m;
  long content_length = -1;
  bool chunked = false;
  long hl = 0;
  while (true) {
    long r = recv_some(c, buf, sizeof(buf));
    if (r <= 0) {
      if (h->aborted.load()) return true;
      *err = r == 0 ? "apiserver closed the watch before responding" : "watch read failed";
      return false;
    }
    head.append(buf, static_cast<size_t>(r));
    std::string perr;
    hl = http::parse_head(head.data(), head.size(), false, &m, &perr, &content_length, &chunked);
    if (hl < 0) {
      *err = "bad watch response: " + perr;
      return false;
    }
    if (hl > 0) break;
  }
  *status = m.status;
  const bool is_err = m.status >= 400;
  http::Dechunker dech;
  bool stop = false;
  long long left = content_length;  // -1: until close (when not chunked)
  auto emit = [&](std::string_view piece) {
    if (stop || piece.empty()) return;
    if (is_err) {
      error_body->append(piece);
    } else if (!on_data(piece)) {
      stop = true;
    }
  };
  auto consume = [&](const char* p, size_t n) -> int {
    if (chunked) return dech.feed(p, n, emit);
    if (left >= 0) {
      size_t take = static_cast<size_t>(std::min<long long>(left, static_cast<long long>(n)));
      emit(std::string_view(p, take));
      left -= static_cast<long long>(take);
      return left == 0 ? 1 : 0;
    }
    emit(std::string_view(p, n));
    return 0;
  };
  int st = consume(head.data() + hl, head.size() - static_cast<size_t>(hl));
  while (st == 0 && !stop) {
    long r = recv_some(c, buf, sizeof(buf));
    if (r == 0) break;  // server closed: end of stream
    if (r < 0) {
      if (h->aborted.load()) return true;
      *err = "watch read failed";
      return false;
    }
    st = consume(buf, static_cast<size_t>(r));
  }
  if (st < 0) {
    *err = "bad chunked framing in watch stream";
    return false;
  }
  return true;
}

bool ApiClient::request(const std::string& method, const std::string& path, const std::string& body,
                        const char* content_type, int* status, std::string* resp, std::string* err,
                        std::string* resp_content_type) {
  if (!ok_) {
    *err = init_err_;
    return false;
  }
  const bool has_body = !body.empty() || method == "POST" || method == "PUT" || method == "PATCH";
  thread_local uint64_t rng = 0x9e3779b97f4a7c15ull ^ reinterpret_cast<uintptr_t>(&rng);
  for (int attempt = 0;; ++attempt) {
    // the head is rebuilt per send: a rotated service-account token is picked up between attempts
    std::string req = request_head(method, path, body.size(), content_type, has_body);
    req.append(body);
    std::string retry_after;
    if (!request_once(req, status, resp, err, resp_content_type, &retry_after)) return false;
    if (*status != 429 && (*status < 500 || retry_after.empty())) return true;
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    const double wait = retry_wait(cfg_, method, *status, retry_after, attempt,
                                   static_cast<double>(rng >> 11) * (1.0 / 9007199254740992.0));
    if (wait < 0) return true;  // out of attempts (or not retried): the caller sees the status
    throttled_.fetch_add(1, std::memory_order_relaxed);
    throttle_wait_ns_.fetch_add(static_cast<uint64_t>(wait * 1e9), std::memory_order_relaxed);
    if (!wait_or_abort(wait)) {
      *err = "apiserver client closed";
      return false;
    }
  }
}

bool ApiClient::request_once(const std::string& req, int* status, std::string* resp, std::string* err,
                             std::string* resp_content_type, std::string* retry_after) {

  // a request in flight is listed (abort() shuts its socket) until its connection is released
  auto done = [this](Conn* c, bool reuse) {
    {
      std::lock_guard<std::mutex> g(mu_);
      busy_.erase(std::remove(busy_.begin(), busy_.end(), c->fd), busy_.end());
      reuse = reuse && !aborted_;
    }
    release(c, reuse);
  };
  for (int attempt = 0; attempt < 2; ++attempt) {
    Conn* c = acquire(err);
    if (!c) return false;
    bool aborted;
    {
      std::lock_guard<std::mutex> g(mu_);
      aborted = aborted_;
      if (!aborted) busy_.push_back(c->fd);
    }
    if (aborted) {
      release(c, false);
      *err = "apiserver client closed";
      return false;
    }
    bool fresh_fail = false;
    if (!send_all(c, req)) {
      done(c, false);
      if (attempt == 0) continue;  // stale keep-alive connection: retry once on a new one
      *err = "send to apiserver failed";
      return false;
    }
    http::Message m;
    std::string perr;
    char buf[65536];
    c->rbuf.clear();
    http::MessageParser parser(false);  // a large chunked LIST page is decoded once, not re-parsed per read
    while (true) {
      long got = parser.parse(c->rbuf.data(), c->rbuf.size(), &m, &perr);
      if (got > 0) break;
      if (got < 0) {
        done(c, false);
        *err = "bad response from apiserver: " + perr;
        return false;
      }
      long r = recv_some(c, buf, sizeof(buf));
      if (r == 0) {
        long got2 = parser.parse(c->rbuf.data(), c->rbuf.size(), &m, &perr, 64u << 20, true);
        if (got2 > 0) break;
        fresh_fail = c->rbuf.empty();
        break;
      }
      if (r < 0) {
        fresh_fail = c->rbuf.empty();
        break;
      }
      c->rbuf.append(buf, static_cast<size_t>(r));
    }
    if (m.status == 0) {
      done(c, false);
      if (fresh_fail && attempt == 0) continue;
      *err = "apiserver closed the connection";
      return false;
    }
    ++requests_;
    *status = m.status;
    if (resp_content_type) {
      const std::string* ct = m.header("content-type");
      *resp_content_type = ct ? *ct : std::string();
    }
    if (m.status == 429 || m.status >= 500) {
      const std::string* ra = m.header("retry-after");
      *retry_after = ra ? *ra : std::string();
    }
    *resp = std::move(m.body);
    done(c, m.keep_alive && !m.body_until_close);
    return true;
  }
  *err = "apiserver request failed";
  return false;
}

}  // namespace gsx
