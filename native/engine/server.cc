#include "server.h"
#include "quantity.h"
#include "introspect.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <random>

#include "json.h"

namespace gsx {

const double LatencyHist::kBounds[LatencyHist::kBuckets] = {0.0001, 0.00025, 0.0005, 0.001, 0.0025,
                                                             0.005,  0.01,    0.025,  0.05,  0.1,
                                                             0.25,   0.5,     1.0,    2.5,   5.0};

void LatencyHist::observe(double s) {
  int i = 0;
  while (i < kBuckets && s > kBounds[i]) ++i;
  counts[i].fetch_add(1, std::memory_order_relaxed);
  n.fetch_add(1, std::memory_order_relaxed);
  sum_ns.fetch_add(static_cast<uint64_t>(s * 1e9), std::memory_order_relaxed);
}

namespace {

constexpr uint64_t kListenId = 1;
constexpr uint64_t kEventId = 2;
constexpr const char* kPrefix = "/gpushare-scheduler";
constexpr const char* kVersion = "0.1.0";
// the device plugin's allocation annotations a move may write besides *_IDX and ASSIGNED (models/profile.py)
constexpr std::string_view kAnnCuMask = "gpushare.amd.com/cu-mask";
constexpr std::string_view kAnnHoldIdx = "gpushare.amd.com/hold-idx";
constexpr std::string_view kAnnHoldPartner = "gpushare.amd.com/hold-partner";
constexpr std::string_view kAnnReconciled = "gpushare.amd.com/reconciled";

double mono() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void set_nonblock(int fd) { fcntl(fd, F_SETFL, fcntl(fd, F_GETFL, 0) | O_NONBLOCK); }

std::string error_body(const std::string& msg) {
  std::string o("{\"Error\":");
  json::append_quoted(&o, msg);
  o.push_back('}');
  return o;
}

// Go-style lookup of a string member of the ExtenderBindingArgs object.
bool arg_str(const json::Doc& d, const char* key, std::string* out) {
  int64_t i = d.find(0, key, true);
  if (i < 0) {
    out->clear();
    return true;
  }
  const json::Val& v = d.at(static_cast<uint32_t>(i));
  if (v.type == json::T::Null) {
    out->clear();
    return true;
  }
  if (v.type != json::T::String) return false;
  *out = d.str(static_cast<uint32_t>(i));
  return true;
}

// encoding/json's name for a JSON value that cannot fill a Go string field
const char* go_json_type(json::T t) {
  switch (t) {
    case json::T::Object: return "object";
    case json::T::Array: return "array";
    case json::T::True:
    case json::T::False: return "bool";
    default: return "number";
  }
}

// ExtenderBindingArgs (types.go:287-296) as encoding/json decodes it: keys match case-insensitively, null leaves
// a field empty, any other non-string is the decoder's type error
bool binding_args(const json::Doc& d, std::string* name, std::string* ns, std::string* uid, std::string* node,
                  std::string* err) {
  const char* keys[4] = {"PodName", "PodNamespace", "PodUID", "Node"};
  std::string* outs[4] = {name, ns, uid, node};
  for (int k = 0; k < 4; ++k) {
    if (arg_str(d, keys[k], outs[k])) continue;
    int64_t i = d.find(0, keys[k], true);
    *err = std::string("json: cannot unmarshal ") + go_json_type(d.at(static_cast<uint32_t>(i)).type) +
           " into Go struct field ExtenderBindingArgs." + keys[k] + " of type string";
    return false;
  }
  return true;
}

std::string status_message(const std::string& body, int status) {
  json::Doc d;
  std::string e;
  if (!body.empty() && d.parse(body, &e) && d.at(0).type == json::T::Object) {
    int64_t m = d.find(0, "message");
    if (m >= 0 && d.at(static_cast<uint32_t>(m)).type == json::T::String) return d.str(static_cast<uint32_t>(m));
  }
  return "apiserver returned HTTP " + std::to_string(status);
}

std::string url_escape_path(const std::string& s) {
  static const char* hex = "0123456789ABCDEF";
  std::string o;
  for (unsigned char c : s) {
    if (std::isalnum(c) || c == '-' || c == '.' || c == '_' || c == '~') {
      o.push_back(static_cast<char>(c));
    } else {
      o.push_back('%');
      o.push_back(hex[c >> 4]);
      o.push_back(hex[c & 15]);
    }
  }
  return o;
}

}  // namespace

struct NativeServer::Conn {
  int fd = -1;
  uint64_t id = 0;
  std::string in;
  http::MessageParser parser;  // resumes across reads: a trickled request is parsed once, not once per read
  std::string out;
  size_t out_off = 0;
  bool busy = false;
  bool close_after = false;
  bool want_write = false;
};

struct NativeServer::Loop {
  int ep = -1;
  int lfd = -1;
  int efd = -1;
  uint64_t next_id = 16;
  std::unordered_map<uint64_t, Conn*> conns;
  std::mutex cmu;
  std::deque<std::tuple<uint64_t, std::string, bool>> done;
};

NativeServer::NativeServer(Ledger* ledger, ServerConfig cfg) : l_(ledger), cfg_(std::move(cfg)) {
  update_mode_.store(cfg_.update_mode);
  std::random_device rd;
  char b[24];
  std::snprintf(b, sizeof(b), "%08x%08x", rd(), rd());
  boot_id_ = b;
}

void NativeServer::set_binds_enabled(bool on) {
  const bool was = binds_enabled_.exchange(on);
  if (on && !was && port_ > 0) new_epoch();  // became the leader (before start(): start() begins the first epoch)
}

std::string NativeServer::epoch() const { return boot_id_ + "." + std::to_string(epoch_gen_.load()); }

void NativeServer::new_epoch() {
  epoch_gen_.fetch_add(1);
  {
    std::lock_guard<introspect::ProfiledMutex> g(l_->mu());
    l_->begin_epoch(cfg_.publication_hold_s);
  }
  std::lock_guard<std::mutex> p(pub_mu_);
  pub_cv_.notify_all();
}

void NativeServer::wait_publication(const std::string& node) {
  double t0 = 0;
  while (!stop_.load()) {
    double left;
    {
      std::lock_guard<introspect::ProfiledMutex> g(l_->mu());
      left = l_->publication_wait(node);
    }
    if (left <= 0) break;
    if (t0 == 0) {
      t0 = mono();
      stats_.publication_waits.fetch_add(1, std::memory_order_relaxed);
    }
    std::unique_lock<std::mutex> p(pub_mu_);
    pub_cv_.wait_for(p, std::chrono::duration<double>(std::min(left, 0.05)));
  }
  if (t0 > 0) publication_wait_ns_.fetch_add(static_cast<uint64_t>((mono() - t0) * 1e9), std::memory_order_relaxed);
}

NativeServer::~NativeServer() { stop(); }

int NativeServer::start(std::string* err) {
  if (cfg_.threads < 1) cfg_.threads = 1;
  if (cfg_.pool_threads < 1) cfg_.pool_threads = 1;
  if (!cfg_.api.server.empty()) {
    api_.reset(new ApiClient(cfg_.api));
    if (!api_->ok()) {
      *err = "apiserver client: " + api_->init_error();
      return -1;
    }
  }
  if (cfg_.fallback_port > 0) {
    ApiConfig fc;
    fc.server = "http://127.0.0.1:" + std::to_string(cfg_.fallback_port);
    fc.timeout_s = 120.0;
    fallback_.reset(new ApiClient(fc));
  }
  int port = cfg_.port;
  for (int i = 0; i < cfg_.threads; ++i) {
    std::unique_ptr<Loop> lp(new Loop());
    addrinfo hints;
    std::memset(&hints, 0, sizeof(hints));
    hints.ai_family = AF_UNSPEC;
    hints.ai_socktype = SOCK_STREAM;
    hints.ai_flags = AI_PASSIVE | AI_NUMERICHOST;
    addrinfo* res = nullptr;
    std::string ps = std::to_string(port);
    int gr = getaddrinfo(cfg_.host.empty() ? nullptr : cfg_.host.c_str(), ps.c_str(), &hints, &res);
    if (gr != 0) {
      *err = std::string("listen address ") + cfg_.host + ": " + gai_strerror(gr);
      return -1;
    }
    int fd = ::socket(res->ai_family, SOCK_STREAM | SOCK_CLOEXEC, 0);
    int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    setsockopt(fd, SOL_SOCKET, SO_REUSEPORT, &one, sizeof(one));
    if (::bind(fd, res->ai_addr, res->ai_addrlen) != 0 || ::listen(fd, 1024) != 0) {
      *err = std::string("bind/listen on port ") + ps + ": " + std::strerror(errno);
      freeaddrinfo(res);
      ::close(fd);
      return -1;
    }
    freeaddrinfo(res);
    if (port == 0) {
      sockaddr_storage ss;
      socklen_t sl = sizeof(ss);
      getsockname(fd, reinterpret_cast<sockaddr*>(&ss), &sl);
      port = ss.ss_family == AF_INET6 ? ntohs(reinterpret_cast<sockaddr_in6*>(&ss)->sin6_port)
                                      : ntohs(reinterpret_cast<sockaddr_in*>(&ss)->sin_port);
    }
    set_nonblock(fd);
    lp->lfd = fd;
    lp->ep = epoll_create1(EPOLL_CLOEXEC);
    lp->efd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    epoll_event ev;
    ev.events = EPOLLIN;
    ev.data.u64 = kListenId;
    epoll_ctl(lp->ep, EPOLL_CTL_ADD, lp->lfd, &ev);
    ev.data.u64 = kEventId;
    epoll_ctl(lp->ep, EPOLL_CTL_ADD, lp->efd, &ev);
    loops_.push_back(std::move(lp));
  }
  if (binds_enabled_.load()) new_epoch();  // the first epoch: what a predecessor was told is unknown here
  port_ = port;
  int li = 0;
  for (auto& lp : loops_) {
    loop_threads_.emplace_back([this, p = lp.get(), li] {
      introspect::name_thread("http-" + std::to_string(li));
      run_loop(p);
    });
    ++li;
  }
  for (int i = 0; i < cfg_.pool_threads; ++i) {
    pool_threads_.emplace_back([this, i] {
      introspect::name_thread("bind-" + std::to_string(i));
      pool_main();
    });
  }
  return port_;
}

void NativeServer::stop() {
  if (stop_.exchange(true)) return;
  for (auto& lp : loops_) {
    uint64_t one = 1;
    if (write(lp->efd, &one, sizeof(one)) < 0) {
    }
  }
  jcv_.notify_all();
  for (auto& t : loop_threads_) t.join();
  for (auto& t : pool_threads_) t.join();
  loop_threads_.clear();
  pool_threads_.clear();
  for (auto& lp : loops_) {
    for (auto& kv : lp->conns) {
      ::close(kv.second->fd);
      delete kv.second;
    }
    lp->conns.clear();
    ::close(lp->lfd);
    ::close(lp->efd);
    ::close(lp->ep);
  }
  loops_.clear();
}

std::vector<BindFailure> NativeServer::drain_failures() {
  std::lock_guard<std::mutex> g(fmu_);
  std::vector<BindFailure> out;
  out.swap(failures_);
  return out;
}

void NativeServer::record_failure(BindFailure f) {
  std::lock_guard<std::mutex> g(fmu_);
  if (failures_.size() < 4096) failures_.push_back(std::move(f));
}

// ------------------------------------------------------------------ event loop

void NativeServer::run_loop(Loop* lp) {
  epoll_event evs[128];
  while (!stop_.load()) {
    int n = epoll_wait(lp->ep, evs, 128, 500);
    for (int i = 0; i < n; ++i) {
      uint64_t id = evs[i].data.u64;
      if (id == kListenId) {
        while (true) {
          int cfd = accept4(lp->lfd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
          if (cfd < 0) break;
          int one = 1;
          setsockopt(cfd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
          Conn* c = new Conn();
          c->fd = cfd;
          c->id = lp->next_id++;
          lp->conns[c->id] = c;
          epoll_event ev;
          ev.events = EPOLLIN | EPOLLRDHUP;
          ev.data.u64 = c->id;
          epoll_ctl(lp->ep, EPOLL_CTL_ADD, cfd, &ev);
          stats_.connections.fetch_add(1, std::memory_order_relaxed);
        }
      } else if (id == kEventId) {
        uint64_t v;
        while (read(lp->efd, &v, sizeof(v)) > 0) {
        }
        drain_completions(lp);
      } else {
        auto it = lp->conns.find(id);
        if (it == lp->conns.end()) continue;
        Conn* c = it->second;
        if (evs[i].events & (EPOLLERR | EPOLLHUP)) {
          close_conn(lp, c);
          continue;
        }
        if (evs[i].events & EPOLLOUT) {
          flush(lp, c);
          if (lp->conns.find(id) == lp->conns.end()) continue;
        }
        if (evs[i].events & (EPOLLIN | EPOLLRDHUP)) on_readable(lp, c);
      }
    }
  }
}

void NativeServer::on_readable(Loop* lp, Conn* c) {
  char buf[65536];
  bool eof = false;
  while (true) {
    ssize_t r = ::recv(c->fd, buf, sizeof(buf), 0);
    if (r > 0) {
      c->in.append(buf, static_cast<size_t>(r));
      if (c->in.size() > cfg_.max_body + (64u << 10)) {
        close_conn(lp, c);
        return;
      }
      if (static_cast<size_t>(r) < sizeof(buf)) break;  // drained; level-triggered epoll reports more input
      continue;
    }
    if (r == 0) eof = true;
    break;  // EAGAIN or error
  }
  uint64_t id = c->id;
  safe_process(lp, c);
  if (eof && lp->conns.count(id)) {
    Conn* cc = lp->conns[id];
    if (!cc->busy && cc->out_off >= cc->out.size()) {
      close_conn(lp, cc);
    } else {
      cc->close_after = true;
    }
  }
}

void NativeServer::safe_process(Loop* lp, Conn* c) {
  uint64_t id = c->id;
  try {
    process(lp, c);
  } catch (const std::exception& e) {
    // one malformed or hostile request must never take the loop thread (and the extender) down
    stats_.bad_requests.fetch_add(1, std::memory_order_relaxed);
    std::fprintf(stderr, "[gsx-engine] request dropped: %s\n", e.what());
    auto it = lp->conns.find(id);
    if (it != lp->conns.end()) close_conn(lp, it->second);
  }
}

void NativeServer::process(Loop* lp, Conn* c) {
  uint64_t id = c->id;
  while (!c->busy && !c->in.empty()) {
    http::Message req;
    std::string perr;
    long used = c->parser.parse(c->in.data(), c->in.size(), &req, &perr, cfg_.max_body);
    if (used == 0) return;
    if (used < 0) {
      stats_.bad_requests.fetch_add(1, std::memory_order_relaxed);
      respond(lp, c, http::response(400, "text/plain", perr, false), false);
      return;
    }
    c->in.erase(0, static_cast<size_t>(used));
    stats_.requests.fetch_add(1, std::memory_order_relaxed);
    dispatch(lp, c, req);
    if (!lp->conns.count(id)) return;
  }
}

void NativeServer::respond(Loop* lp, Conn* c, std::string resp, bool keep_alive) {
  c->out.append(resp);
  if (!keep_alive) c->close_after = true;
  flush(lp, c);
}

void NativeServer::flush(Loop* lp, Conn* c) {
  while (c->out_off < c->out.size()) {
    ssize_t w = ::send(c->fd, c->out.data() + c->out_off, c->out.size() - c->out_off, MSG_NOSIGNAL);
    if (w > 0) {
      c->out_off += static_cast<size_t>(w);
      continue;
    }
    if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
      if (!c->want_write) {
        epoll_event ev;
        ev.events = EPOLLIN | EPOLLRDHUP | EPOLLOUT;
        ev.data.u64 = c->id;
        epoll_ctl(lp->ep, EPOLL_CTL_MOD, c->fd, &ev);
        c->want_write = true;
      }
      return;
    }
    close_conn(lp, c);
    return;
  }
  c->out.clear();
  c->out_off = 0;
  if (c->want_write) {
    epoll_event ev;
    ev.events = EPOLLIN | EPOLLRDHUP;
    ev.data.u64 = c->id;
    epoll_ctl(lp->ep, EPOLL_CTL_MOD, c->fd, &ev);
    c->want_write = false;
  }
  if (c->close_after && !c->busy) close_conn(lp, c);
}

void NativeServer::close_conn(Loop* lp, Conn* c) {
  epoll_ctl(lp->ep, EPOLL_CTL_DEL, c->fd, nullptr);
  ::close(c->fd);
  lp->conns.erase(c->id);
  delete c;
}

void NativeServer::complete(Loop* lp, uint64_t conn_id, std::string resp, bool keep_alive) {
  {
    std::lock_guard<std::mutex> g(lp->cmu);
    lp->done.emplace_back(conn_id, std::move(resp), keep_alive);
  }
  uint64_t one = 1;
  if (write(lp->efd, &one, sizeof(one)) < 0) {
  }
}

void NativeServer::drain_completions(Loop* lp) {
  std::deque<std::tuple<uint64_t, std::string, bool>> done;
  {
    std::lock_guard<std::mutex> g(lp->cmu);
    done.swap(lp->done);
  }
  for (auto& t : done) {
    auto it = lp->conns.find(std::get<0>(t));
    if (it == lp->conns.end()) continue;  // client went away meanwhile
    Conn* c = it->second;
    c->busy = false;
    uint64_t id = c->id;
    respond(lp, c, std::move(std::get<1>(t)), std::get<2>(t));
    if (lp->conns.count(id)) safe_process(lp, c);
  }
}

// ------------------------------------------------------------------ routing

void NativeServer::dispatch(Loop* lp, Conn* c, http::Message& req) {
  double t0 = mono();
  std::string_view path = req.path();
  const bool ka = req.keep_alive;
  const std::string pre(kPrefix);
  if (req.method == "POST" && path == pre + "/filter") {
    stats_.filters.fetch_add(1, std::memory_order_relaxed);
    std::string out;
    {
      std::lock_guard<introspect::ProfiledMutex> g(l_->mu());
      out = filter_body(*l_, req.body);
    }
    stats_.filter_lat.observe(mono() - t0);
    respond(lp, c, http::response(200, "application/json", out, ka), ka);
    return;
  }
  if (req.method == "POST" && path == pre + "/prioritize") {
    std::string out;
    {
      std::lock_guard<introspect::ProfiledMutex> g(l_->mu());
      out = prioritize_body(*l_, req.body);
    }
    respond(lp, c, http::response(200, "application/json", out, ka), ka);
    return;
  }
  if (req.method == "POST" && path == pre + "/bind") {
    stats_.binds.fetch_add(1, std::memory_order_relaxed);
    c->busy = true;
    submit(Job{lp, c->id, 0, std::move(req), t0});
    return;
  }
  if (req.method == "POST" && path == pre + "/physical") {
    stats_.physical_posts.fetch_add(1, std::memory_order_relaxed);
    c->busy = true;
    submit(Job{lp, c->id, 3, std::move(req), t0});
    return;
  }
  if (req.method == "POST" && path == pre + "/move") {
    stats_.moves.fetch_add(1, std::memory_order_relaxed);
    c->busy = true;
    submit(Job{lp, c->id, 2, std::move(req), t0});
    return;
  }
  if (req.method == "GET" && (path == pre + "/inspect" || path == pre + "/inspect/" ||
                              path.substr(0, pre.size() + 9) == pre + "/inspect/")) {
    std::string node;
    if (path.size() > pre.size() + 9) node = std::string(path.substr(pre.size() + 9));
    stats_.inspects.fetch_add(1, std::memory_order_relaxed);
    std::string out;
    bool found;
    {
      std::lock_guard<introspect::ProfiledMutex> g(l_->mu());
      out = l_->inspect_json(node, &found);
    }
    respond(lp, c, http::response(200, "application/json", out, ka), ka);
    return;
  }
  if (req.method == "GET" && path == pre + "/epoch") {
    std::string out = "{\"epoch\":\"" + epoch() + "\",\"leader\":" + (binds_enabled_.load() ? "true" : "false") + "}";
    respond(lp, c, http::response(200, "application/json", out, ka), ka);
    return;
  }
  if (req.method == "GET" && path == "/version") {
    respond(lp, c, http::response(200, "text/plain; charset=utf-8", kVersion, ka), ka);
    return;
  }
  if (fallback_) {
    c->busy = true;
    submit(Job{lp, c->id, 1, std::move(req), t0});
    return;
  }
  respond(lp, c, http::response(404, "text/plain", "404 page not found\n", ka), ka);
}

void NativeServer::submit(Job j) {
  {
    std::lock_guard<std::mutex> g(jmu_);
    jobs_.push_back(std::move(j));
  }
  jcv_.notify_one();
}

void NativeServer::pool_main() {
  while (true) {
    Job j;
    {
      std::unique_lock<std::mutex> g(jmu_);
      jcv_.wait(g, [this] { return stop_.load() || !jobs_.empty(); });
      if (stop_.load() && jobs_.empty()) return;
      j = std::move(jobs_.front());
      jobs_.pop_front();
    }
    std::string resp;
    const bool ka = j.req.keep_alive;
    try {
      if (j.kind == 0) {
        resp = do_bind(j.req);
        stats_.bind_lat.observe(mono() - j.t0);
      } else if (j.kind == 2 || j.kind == 3) {
        std::string token_node;
        if (plugin_authorized(j.req, &resp, &token_node)) {
          resp = j.kind == 2 ? do_move(j.req, token_node) : do_physical(j.req, token_node);
        }
      } else {
        resp = do_proxy(j.req);
      }
    } catch (const std::exception& e) {
      // as in the loop threads: one request that throws must not terminate the extender (a pool thread has no
      // handler above it); kube-scheduler retries a bind that answers 500
      stats_.bad_requests.fetch_add(1, std::memory_order_relaxed);
      std::fprintf(stderr, "[gsx-engine] %s failed: %s\n", j.kind == 0 ? "bind" : "proxied request", e.what());
      resp = http::response(500, "application/json", error_body(std::string("internal error: ") + e.what()), true);
    }
    complete(j.loop, j.conn_id, std::move(resp), ka);
  }
}

std::string NativeServer::bind_error_response(const std::string& msg) const {
  return http::response(500, "application/json", error_body(msg), true);
}

std::string NativeServer::do_proxy(const http::Message& req) {
  stats_.proxied.fetch_add(1, std::memory_order_relaxed);
  if (!fallback_) return http::response(404, "text/plain", "404 page not found\n", true);
  const std::string* ct = req.header("content-type");
  int status = 0;
  std::string body, err, rct;
  if (!fallback_->request(req.method, req.target, req.body, ct ? ct->c_str() : "application/json", &status, &body,
                          &err, &rct)) {
    return http::response(502, "text/plain", "fallback: " + err, true);
  }
  return http::response(status, rct, body, true);
}

// Native bind: reserve on the ledger, then one POST pods/{name}/binding whose
// metadata.annotations carry the allocation record (pkg/utils/pod.go:192-206).
std::string NativeServer::do_bind(const http::Message& req) {
  if (!binds_enabled_.load()) {
    return bind_error_response("this extender replica is not the leader");
  }
  if (!api_) return bind_error_response("the extender has no apiserver client");
  json::Doc d;
  std::string perr;
  if (!d.parse(req.body, &perr)) return bind_error_response(perr);
  if (d.at(0).type != json::T::Object) {
    return bind_error_response("json: cannot unmarshal value into Go value of type api.ExtenderBindingArgs");
  }
  std::string name, ns, uid, node;
  if (!binding_args(d, &name, &ns, &uid, &node, &perr)) return bind_error_response(perr);
  // a new epoch does not know what the node's containers hold beyond the annotations: its plugin republishes
  // as soon as it sees the epoch change, and the placement below must count that
  wait_publication(node);
  Ledger::PendingPod pp;
  int64_t dev = -1, dev_total = -1, assume_ns = 0;
  uint64_t seq = 0;
  const Profile& prof = l_->profile();
  bool filtered;
  {
    std::lock_guard<introspect::ProfiledMutex> g(l_->mu());
    filtered = l_->pending(uid, &pp) && pp.name == name && pp.ns == ns;
    // reservation, ASSUME_TIME and the ordering sequence in one step
    if (filtered) dev = l_->assume_ordered(uid, ns, name, node, pp.req, &dev_total, &seq, &assume_ns, pp.cu_count);
  }
  if (!filtered) {
    // never filtered here (a restart between filter and bind, another replica's filter): the pod's request
    // comes from the lister or the apiserver
    stats_.unfiltered_binds.fetch_add(1, std::memory_order_relaxed);
    std::string err;
    if (!lookup_pod(ns, name, uid, false, &pp, &err)) {
      stats_.bind_fail.fetch_add(1, std::memory_order_relaxed);
      record_failure(BindFailure{ns, name, uid, node, err});
      return bind_error_response(err);
    }
    std::lock_guard<introspect::ProfiledMutex> g(l_->mu());
    dev = l_->assume_ordered(uid, ns, name, node, pp.req, &dev_total, &seq, &assume_ns, pp.cu_count);
  }
  if (dev < 0) {
    std::string msg;
    if (dev == -2) {
      msg = "node \"" + node + "\" not found";
    } else if (dev == -3) {
      msg = "The node " + node + " is not for GPU share, need skip";
    } else if (dev == -4) {
      msg = "bind of pod " + name + " in ns " + ns + " is already in progress";
    } else {
      msg = "The node " + node + " can't place the pod " + name + " in ns " + ns;  // nodeinfo.go:170
    }
    stats_.bind_fail.fetch_add(1, std::memory_order_relaxed);
    record_failure(BindFailure{ns, name, uid, node, msg});
    return bind_error_response(msg);
  }
  struct Done {  // leave the in-flight set however the bind ends
    Ledger* l;
    uint64_t seq;
    ~Done() { l->bind_leave(seq); }
  } done{l_, seq};
  // the allocation record (pkg/utils/pod.go:192-206)
  std::string ann;
  ann.reserve(256);
  auto kv = [&](const std::string& k, const std::string& v, bool last) {
    json::append_quoted(&ann, k);
    ann.push_back(':');
    json::append_quoted(&ann, v);
    if (!last) ann.push_back(',');
  };
  kv(prof.a_idx, std::to_string(dev), false);
  kv(prof.a_dev, std::to_string(dev_total), false);
  kv(prof.a_pod, std::to_string(pp.req), false);
  kv(prof.a_assigned, "false", false);
  kv(prof.a_assume, std::to_string(assume_ns), true);
  const std::string pod_path = "/api/v1/namespaces/" + url_escape_path(ns) + "/pods/" + url_escape_path(name);
  const std::string path = pod_path + "/binding";
  std::string msg;
  bool ok = false;
  auto call = [&](const char* method, const std::string& target, const std::string& body, const char* ct,
                  int* status, std::string* resp) {
    std::string err;
    bool sent = api_call(method, target, body, ct, status, resp, &err);
    if (!sent) msg = err;
    return sent;
  };
  auto fail = [&](const std::string& m) {
    {
      std::lock_guard<introspect::ProfiledMutex> g(l_->mu());
      l_->finish_bind(uid, false, cfg_.reservation_ttl);
    }
    stats_.bind_fail.fetch_add(1, std::memory_order_relaxed);
    record_failure(BindFailure{ns, name, uid, node, m});
    return bind_error_response(m);
  };
  // a 5xx the apiserver sent without Retry-After (ApiClient already waited out 429s and Retry-After 5xx): sent
  // again after a capped exponential backoff with jitter, the reservation kept meanwhile
  auto backoff = [this](int attempt) {
    thread_local uint64_t r = 0x2545f4914f6cdd1dull ^ reinterpret_cast<uintptr_t>(&r);
    r ^= r << 13;
    r ^= r >> 7;
    r ^= r << 17;
    const double b = std::min(0.2, 0.005 * static_cast<double>(1 << std::min(attempt, 6)));
    stats_.backoffs.fetch_add(1, std::memory_order_relaxed);
    std::this_thread::sleep_for(std::chrono::duration<double>(b * (0.5 + 0.5 * static_cast<double>(r >> 11) *
                                                                            (1.0 / 9007199254740992.0))));
  };
  constexpr int kServerErrorAttempts = 5;
  const bool update_mode = update_mode_.load();
  if (update_mode) {
    // the reference's first call: write the annotations, guarded by the resourceVersion the scheduler saw;
    // on the optimistic-lock conflict retry once on the latest version (nodeinfo.go:150-168).  Not ordered:
    // a pod without spec.nodeName is no device-plugin candidate yet
    int conflicts = 0;
    for (int attempt = 0; attempt < kServerErrorAttempts; ++attempt) {
      std::string patch = "{\"metadata\":{";
      if (attempt == 0 && conflicts == 0 && !pp.rv.empty()) {
        patch.append("\"resourceVersion\":");
        json::append_quoted(&patch, pp.rv);
        patch.push_back(',');
      }
      patch.append("\"annotations\":{").append(ann).append("}}}");
      int status = 0;
      std::string body;
      if (!call("PATCH", pod_path, patch, "application/merge-patch+json", &status, &body)) return fail(msg);
      if (status == 200 || status == 201) break;
      msg = status_message(body, status);
      if (conflicts == 0 && status == 409) {  // a conflict is detected by status, not by message
        ++conflicts;
        stats_.conflicts_retried.fetch_add(1, std::memory_order_relaxed);
        continue;
      }
      if (status >= 500 && attempt + 1 < kServerErrorAttempts) {  // the same annotations again: idempotent
        backoff(attempt);
        continue;
      }
      return fail(msg);
    }
  }
  // Binding object; in "binding" mode it carries the annotations, which kube-apiserver copies onto the pod
  std::string b;
  b.reserve(512);
  b.append("{\"apiVersion\":\"v1\",\"kind\":\"Binding\",\"metadata\":{\"name\":");
  json::append_quoted(&b, name);
  b.append(",\"namespace\":");
  json::append_quoted(&b, ns);
  b.append(",\"uid\":");
  json::append_quoted(&b, uid);
  if (!update_mode) b.append(",\"annotations\":{").append(ann).push_back('}');
  b.append("},\"target\":{\"apiVersion\":\"v1\",\"kind\":\"Node\",\"name\":");
  json::append_quoted(&b, node);
  b.append("}}");
  // kubelet admits a node's pods in the order their bindings land, and the device plugin gives a request
  // of N units to the earliest-ASSUME_TIME unassigned pod of that size (docs/designs/designs.md:93-103).
  // Two equal-size pods headed for different GPUs of one node must therefore land in ASSUME_TIME order,
  // or each container is started with the other's GPU.  The reference got this from its node lock held
  // across the API calls (pkg/cache/nodeinfo.go:141-189); here only such a pair waits, everything else
  // (other nodes, other sizes, the same GPU) binds concurrently.
  if (l_->bind_blocked(seq)) {
    stats_.bind_order_waits.fetch_add(1, std::memory_order_relaxed);
    l_->bind_wait(seq, &stop_);
  }
  for (int attempt = 0, conflicts = 0; attempt < kServerErrorAttempts; ++attempt) {
    int status = 0;
    std::string body;
    if (!call("POST", path, b, "application/json", &status, &body)) break;
    if (status == 200 || status == 201) {
      ok = true;
      break;
    }
    msg = status_message(body, status);
    if (status == 409 && msg.find("Precondition failed") != std::string::npos) {
      // UID mismatch (the pod was re-created under its name): the reference's exact error comes from a live
      // GET (gpushare-bind.go:44-65)
      Ledger::PendingPod live;
      std::string err;
      if (!lookup_pod(ns, name, uid, true, &live, &err)) msg = err;
      break;
    }
    if (status == 409 && msg.find("already assigned") == std::string::npos && conflicts < 2) {
      ++conflicts;
      stats_.conflicts_retried.fetch_add(1, std::memory_order_relaxed);
      continue;
    }
    if (status >= 500 && attempt + 1 < kServerErrorAttempts) {
      backoff(attempt);
      continue;
    }
    break;
  }
  {
    std::lock_guard<introspect::ProfiledMutex> g(l_->mu());
    l_->finish_bind(uid, ok, cfg_.reservation_ttl);
    if (ok) l_->forget_pending(uid);
  }
  if (!ok) {
    stats_.bind_fail.fetch_add(1, std::memory_order_relaxed);
    record_failure(BindFailure{ns, name, uid, node, msg});
    return bind_error_response(msg);
  }
  stats_.bind_ok.fetch_add(1, std::memory_order_relaxed);
  return http::response(200, "application/json", "{\"Error\":\"\"}", true);
}

void NativeServer::throttle() {
  if (cfg_.qps <= 0) return;
  double wait;
  {
    std::lock_guard<std::mutex> g(qmu_);
    const double now = mono();
    const double burst = std::max(1, cfg_.burst);
    if (q_last_ == 0.0) q_tokens_ = burst;
    q_tokens_ = std::min(burst, q_tokens_ + (now - q_last_) * cfg_.qps);
    q_last_ = now;
    q_tokens_ -= 1.0;  // reserved now, so waiters queue in arrival order
    wait = q_tokens_ < 0 ? -q_tokens_ / cfg_.qps : 0.0;
  }
  if (wait > 0) {
    stats_.qps_waits.fetch_add(1, std::memory_order_relaxed);
    std::this_thread::sleep_for(std::chrono::duration<double>(wait));
  }
}

bool NativeServer::api_call(const char* method, const std::string& target, const std::string& body, const char* ct,
                            int* status, std::string* resp, std::string* err) {
  throttle();
  double t0 = mono();
  stats_.api_calls.fetch_add(1, std::memory_order_relaxed);
  bool sent = api_->request(method, target, body, ct, status, resp, err);
  stats_.api_lat.observe(mono() - t0);
  return sent;
}

bool NativeServer::lookup_pod(const std::string& ns, const std::string& name, const std::string& uid, bool live,
                              Ledger::PendingPod* out, std::string* err) {
  std::string raw;
  json::Doc d;
  std::string perr;
  auto uid_of = [&d]() {
    int64_t u = d.path(0, {"metadata", "uid"});
    return u >= 0 && d.at(static_cast<uint32_t>(u)).type == json::T::String ? d.str(static_cast<uint32_t>(u))
                                                                             : std::string();
  };
  bool have = !live && lister_ && lister_(ns + "/" + name, &raw) && d.parse(raw, &perr) &&
              d.at(0).type == json::T::Object && uid_of() == uid;
  if (!have) {
    stats_.live_gets.fetch_add(1, std::memory_order_relaxed);
    int status = 0;
    raw.clear();
    if (!api_call("GET", "/api/v1/namespaces/" + url_escape_path(ns) + "/pods/" + url_escape_path(name), "",
                  "application/json", &status, &raw, err)) {
      return false;
    }
    if (status != 200) {
      *err = status_message(raw, status);
      return false;
    }
    if (!d.parse(raw, &perr) || d.at(0).type != json::T::Object) {
      *err = "apiserver returned an unreadable pod: " + perr;
      return false;
    }
    const std::string puid = uid_of();
    if (puid != uid) {
      *err = "The pod " + name + " in ns " + ns + "'s uid is " + puid + ", and it's not equal with expected " + uid;
      return false;
    }
  }
  out->ns = ns;
  out->name = name;
  out->req = pod_limits_sum(d, 0, l_->profile().resource);
  out->cu_count.clear();
  out->rv.clear();
  int64_t cu = d.path(0, {"metadata", "annotations", kCuCountAnnotation});
  if (cu >= 0 && d.at(static_cast<uint32_t>(cu)).type == json::T::String) out->cu_count = d.str(static_cast<uint32_t>(cu));
  int64_t rv = d.path(0, {"metadata", "resourceVersion"});
  if (rv >= 0 && d.at(static_cast<uint32_t>(rv)).type == json::T::String) out->rv = d.str(static_cast<uint32_t>(rv));
  return true;
}

// The device plugin's allocation-record writes (deviceplugin/reconcile.py, plugin.py move_unstarted): the extender
// is the one writer of *_IDX, as the reference's node lock made it (pkg/cache/nodeinfo.go:139-168).  Under the
// ledger mutex the move is checked against the ledger (the pod is where the caller thinks; the target has room,
// counting in-flight binds and other moves, unless an equal-size partner makes it an exchange) and the target is
// reserved; then one merge patch, guarded by the caller's resourceVersion, writes *_IDX with the other allocation
// fields the caller sends (ASSIGNED, cu-mask, hold-idx / hold-partner, reconciled).  409 on any refusal or
// conflict: the caller re-plans from fresh state.
//
//   {"namespace","name","uid","node","resourceVersion","from","to","partner","annotations":{k: "v" | null}}
//   -> 200 {"Error":"","to":N,"pod":{...}} | 409 {"Error":"..."} | 4xx/5xx {"Error":"..."}
std::string NativeServer::do_move(const http::Message& req, const std::string& token_node) {
  auto answer = [](int status, const std::string& body) { return http::response(status, "application/json", body, true); };
  if (!binds_enabled_.load()) return answer(503, error_body("this extender replica is not the leader"));
  if (!api_) return answer(501, error_body("no apiserver client"));
  json::Doc d;
  std::string perr;
  if (!d.parse(req.body, &perr) || d.at(0).type != json::T::Object) return answer(400, error_body("bad move request: " + perr));
  std::string ns, name, uid, node, rv, partner;
  if (!arg_str(d, "namespace", &ns) || !arg_str(d, "name", &name) || !arg_str(d, "uid", &uid) ||
      !arg_str(d, "node", &node) || !arg_str(d, "resourceVersion", &rv) || !arg_str(d, "partner", &partner) ||
      ns.empty() || name.empty() || uid.empty() || node.empty() || rv.empty()) {
    return answer(400, error_body("move needs namespace, name, uid, node and resourceVersion"));
  }
  if (!token_node.empty() && token_node != node) {  // the ledger checks the pod is on `node`
    stats_.plugin_auth_denied.fetch_add(1, std::memory_order_relaxed);
    return answer(403, error_body("the caller's token is bound to node " + token_node + ", not " + node));
  }
  MoveRequest m;
  m.uid = uid;
  m.node = node;
  m.partner = partner;
  int64_t pi = d.find(0, "physical_on_to");
  m.physical_on_to = pi >= 0 && d.at(static_cast<uint32_t>(pi)).type == json::T::True;
  int64_t v;
  int64_t fi = d.find(0, "from");
  int64_t ti = d.find(0, "to");
  if (fi < 0 || !d.as_int(static_cast<uint32_t>(fi), &m.from)) return answer(400, error_body("move needs from"));
  if (ti >= 0 && d.as_int(static_cast<uint32_t>(ti), &v)) m.to = v;
  // the other allocation fields (string values, or null to remove an annotation): only the ones a move rewrites --
  // ASSIGNED, the CU partition, the exchange hold and its partner, the reconciliation count.  The pod's share
  // (POD / DEV) is fixed and its GPU is `to`; nothing else of the pod is the device plugin's to write.
  const Profile& prof = l_->profile();
  std::string extra;
  int64_t ai = d.find(0, "annotations");
  if (ai >= 0 && d.at(static_cast<uint32_t>(ai)).type == json::T::Object) {
    const uint32_t obj = static_cast<uint32_t>(ai);
    for (uint32_t k = obj + 1; k < d.at(obj).skip;) {
      const uint32_t val = k + 1;
      const json::T t = d.at(val).type;
      const std::string key = d.str(k);
      if (key == prof.a_idx || key == prof.a_pod || key == prof.a_dev) {
        return answer(400, error_body("the move request names the pod's GPU in from / to, and its share is fixed"));
      }
      if (key != prof.a_assigned && key != kAnnCuMask && key != kAnnHoldIdx && key != kAnnHoldPartner &&
          key != kAnnReconciled) {
        return answer(400, error_body("a move writes only " + prof.a_assigned + ", " + std::string(kAnnCuMask) + ", " +
                                      std::string(kAnnHoldIdx) + ", " + std::string(kAnnHoldPartner) + " and " +
                                      std::string(kAnnReconciled) + "; not " + key));
      }
      if (t != json::T::String && t != json::T::Null) return answer(400, error_body("annotation values are strings or null"));
      if (t == json::T::String && key == kAnnHoldIdx) {
        int64_t hv;
        if (parse_atoi(d.str(val), &hv) && hv >= 0) m.req_hold = hv;
      }
      if (t == json::T::String && key == kAnnHoldPartner) {
        json::Doc hp;
        std::string herr;
        const std::string hsrc = d.str(val);  // the tape points into its source: keep it alive
        if (hp.parse(hsrc, &herr) && hp.at(0).type == json::T::Object) {
          int64_t ui = hp.find(0, "uid");
          if (ui >= 0 && hp.at(static_cast<uint32_t>(ui)).type == json::T::String) {
            m.req_hold_partner = hp.str(static_cast<uint32_t>(ui));
          }
        }
      }
      extra.push_back(',');
      json::append_quoted(&extra, key);
      extra.push_back(':');
      extra.append(d.raw(val));
      k = d.next(val);
    }
  }
  std::string why;
  int rc;
  {
    std::lock_guard<introspect::ProfiledMutex> g(l_->mu());
    rc = l_->begin_move(&m, &why);
  }
  if (rc != 0) return answer(rc == 1 ? 404 : 409, error_body(why));
  std::string patch = "{\"metadata\":{\"resourceVersion\":";
  json::append_quoted(&patch, rv);
  patch.append(",\"annotations\":{");
  json::append_quoted(&patch, prof.a_idx);
  patch.append(":\"").append(std::to_string(m.to)).append("\"").append(extra).append("}}}");
  const std::string target = "/api/v1/namespaces/" + url_escape_path(ns) + "/pods/" + url_escape_path(name);
  int status = 0;
  std::string body, err;
  const bool sent = api_call("PATCH", target, patch, "application/merge-patch+json", &status, &body, &err);
  const bool ok = sent && status >= 200 && status < 300;
  {
    std::lock_guard<introspect::ProfiledMutex> g(l_->mu());
    l_->end_move(uid, ok);
  }
  if (!ok) {
    stats_.moves_failed.fetch_add(1, std::memory_order_relaxed);
    if (!sent) return answer(502, error_body("apiserver: " + err));
    return answer(status == 409 ? 409 : (status >= 500 ? 502 : status), error_body(status_message(body, status)));
  }
  std::string out = "{\"Error\":\"\",\"epoch\":\"" + epoch() + "\",\"to\":" + std::to_string(m.to) + ",\"pod\":";
  out.append(body).push_back('}');
  return answer(200, out);
}

bool NativeServer::plugin_authorized(const http::Message& req, std::string* resp, std::string* token_node) {
  if (cfg_.plugin_auth != "tokenreview") return true;
  auto deny = [&](int status, const std::string& msg) {
    stats_.plugin_auth_denied.fetch_add(1, std::memory_order_relaxed);
    *resp = http::response(status, "application/json", error_body(msg), true);
    return false;
  };
  const std::string* h = req.header("authorization");
  if (!h || h->size() <= 7 || h->compare(0, 7, "Bearer ") != 0) {
    return deny(401, "the device plugin's endpoints need its service-account token (Authorization: Bearer)");
  }
  const std::string token = h->substr(7);
  const double now = mono();
  {
    std::lock_guard<std::mutex> g(amu_);
    auto it = authz_cache_.find(token);
    if (it != authz_cache_.end() && it->second.until > now) {
      if (!it->second.allowed) return deny(it->second.status, it->second.msg);
      *token_node = it->second.node;
      return true;
    }
    // reviews the cache cannot answer are rate limited (20 a second, bursts of 40): a stream of made-up tokens
    // must not turn into a stream of TokenReviews against the apiserver
    review_tokens_ = std::min(40.0, review_tokens_ + (now - review_last_) * 20.0);
    review_last_ = now;
    if (review_tokens_ < 1.0) return deny(429, "too many token reviews; retry shortly");
    review_tokens_ -= 1.0;
  }
  if (!api_) return deny(503, "no apiserver client to review the token");
  auto remember = [&](Authz a) {
    std::lock_guard<std::mutex> g(amu_);
    if (authz_cache_.size() > 1024) authz_cache_.clear();
    authz_cache_[token] = std::move(a);
  };
  auto refuse = [&](int status, const std::string& msg) {
    remember(Authz{now + 10.0, false, status, msg, std::string()});
    return deny(status, msg);
  };
  // TokenReview (authentication.k8s.io/v1): the apiserver says whose token it is
  std::string body = "{\"apiVersion\":\"authentication.k8s.io/v1\",\"kind\":\"TokenReview\",\"spec\":{\"token\":";
  json::append_quoted(&body, token);
  body.append("}}");
  stats_.token_reviews.fetch_add(1, std::memory_order_relaxed);
  int status = 0;
  std::string out, err;
  if (!api_call("POST", "/apis/authentication.k8s.io/v1/tokenreviews", body, "application/json", &status, &out, &err) ||
      status < 200 || status >= 300) {
    return deny(503, "token review failed: " + (err.empty() ? std::to_string(status) : err));  // not cached
  }
  json::Doc d;
  std::string perr;
  if (!d.parse(out, &perr) || d.at(0).type != json::T::Object) return deny(503, "token review: bad answer");
  const int64_t au = d.path(0, {"status", "authenticated"});
  const int64_t un = d.path(0, {"status", "user", "username"});
  if (au < 0 || d.at(static_cast<uint32_t>(au)).type != json::T::True || un < 0) {
    return refuse(401, "the token is not authenticated");
  }
  const std::string user = d.str(static_cast<uint32_t>(un));
  bool allowed = false;
  for (const auto& u : cfg_.plugin_users) allowed = allowed || u == user;
  if (!allowed) return refuse(403, "user " + user + " may not write allocation records");
  // a bound service-account token names the node its pod runs on (status.user.extra, Kubernetes >= 1.30): the
  // plugin of one node may then write only that node's records
  std::string node;
  const int64_t ex = d.path(0, {"status", "user", "extra", "authentication.kubernetes.io/node-name"});
  if (ex >= 0 && d.at(static_cast<uint32_t>(ex)).type == json::T::Array) {
    const uint32_t arr = static_cast<uint32_t>(ex), first = d.first_child(arr);
    if (first < d.next(arr) && d.at(first).type == json::T::String) node = d.str(first);
  }
  remember(Authz{now + cfg_.plugin_auth_ttl, true, 200, std::string(), node});
  *token_node = node;
  return true;
}

// The device plugin's unaccounted use (deviceplugin/plugin.py publish_physical): units kubelet's containers hold on
// each device of its node whose pods the annotations put on another device, or that are gone (a kubelet admission
// batch served two equal-size pods each other's allocations and the exchange of their records has not landed, or
// the pod an allocation was built for was deleted while another pod's container holds it).  The ledger charges it
// on top of the annotations, so the deletion of a pod whose allocation another pod's container holds never frees
// that device for the next bind.  Withdrawn (unaccounted: null) once the records agree; it expires on its own after
// `ttl` seconds unless refreshed (a plugin that died).
//
//   {"node": "n", "unaccounted": [u0, u1, ...] | null, "ttl": s}  ->  200 {"Error":""} | 400 | 404
std::string NativeServer::do_physical(const http::Message& req, const std::string& token_node) {
  auto answer = [](int status, const std::string& body) { return http::response(status, "application/json", body, true); };
  if (!binds_enabled_.load()) {
    // a standby keeps no publication the leader would need: the plugin must not count this one as delivered
    stats_.physical_refused.fetch_add(1, std::memory_order_relaxed);
    return answer(503, error_body("this extender replica is not the leader"));
  }
  json::Doc d;
  std::string perr;
  if (!d.parse(req.body, &perr) || d.at(0).type != json::T::Object) return answer(400, error_body("bad request: " + perr));
  std::string node;
  if (!arg_str(d, "node", &node) || node.empty()) return answer(400, error_body("physical needs node"));
  if (!token_node.empty() && token_node != node) {
    stats_.plugin_auth_denied.fetch_add(1, std::memory_order_relaxed);
    return answer(403, error_body("the caller's token is bound to node " + token_node + ", not " + node));
  }
  std::vector<int64_t> used;
  int64_t ui = d.find(0, "unaccounted");
  if (ui >= 0 && d.at(static_cast<uint32_t>(ui)).type == json::T::Array) {
    const uint32_t arr = static_cast<uint32_t>(ui);
    for (uint32_t k = arr + 1; k < d.at(arr).skip; k = d.next(k)) {
      int64_t v;
      if (!d.as_int(k, &v) || v < 0) return answer(400, error_body("unaccounted: non-negative integers"));
      used.push_back(v);
    }
  } else if (ui >= 0 && d.at(static_cast<uint32_t>(ui)).type != json::T::Null) {
    return answer(400, error_body("unaccounted: an array or null"));
  }
  double ttl = 60.0;  // seconds, fractions allowed (the plugin sends 60.0), at most 600
  int64_t ti = d.find(0, "ttl");
  if (ti >= 0 && d.at(static_cast<uint32_t>(ti)).type == json::T::Number) {
    const std::string txt(d.raw(static_cast<uint32_t>(ti)));
    const double tv = std::strtod(txt.c_str(), nullptr);
    if (tv > 0) ttl = std::min(tv, 600.0);
  }
  bool ok;
  {
    std::lock_guard<introspect::ProfiledMutex> g(l_->mu());
    ok = l_->set_unaccounted(node, used, ttl);
  }
  if (!ok) return answer(404, error_body("node " + node + " is not in the extender's ledger"));
  {
    std::lock_guard<std::mutex> p(pub_mu_);
    pub_cv_.notify_all();  // binds waiting for this node's first publication of the epoch
  }
  return answer(200, "{\"Error\":\"\",\"epoch\":\"" + epoch() + "\"}");
}

}  // namespace gsx
