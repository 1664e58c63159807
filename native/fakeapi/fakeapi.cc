// gsx-fakeapi: fake kube-apiserver in C++ (pods, nodes, events, leases,
// bindings) -- the compiled counterpart of k8s/fakeapi.py with the same REST
// subset and semantics, for benchmarks where the asyncio one would be the
// bottleneck (a real kube-apiserver is compiled Go in front of etcd):
//
//   * LIST + chunked WATCH with resourceVersion (one global counter, as etcd
//     gives kube-apiserver), 410 Gone for compacted history, field selectors
//     (dotted paths, = / !=) and label selectors (=, !=, exists, !exists);
//   * optimistic concurrency on PUT / PATCH (409 with client-go's exact
//     message, pkg/cache/nodeinfo.go:14-16), server-owned metadata;
//   * POST pods/<name>/binding sets spec.nodeName once and merges the
//     Binding's annotations into the pod (kube-apiserver's
//     setPodHostAndAnnotations), plus a PodScheduled condition;
//   * JSON merge patch (strategic merge patch treated as merge patch),
//     DeleteCollection with selectors, DELETE preconditions.uid;
//   * graceful pod deletion as kube-apiserver does it: a bound, non-terminal
//     pod only gets deletionTimestamp; its kubelet removes the object with a
//     grace-0 delete once the containers stopped (no timer here);
//   * fault injection (POST /fake/faults): conflict_rate, error_rate,
//     throttle_rate + retry_after (429 Too Many Requests), latency_ms,
//     drop_watch_after, expire_watches, hold_watches, drop_watches_now;
//     GET /fake/stats.
//
// Concurrency (a real kube-apiserver serves requests on many cores in front of
// one etcd revision counter): N epoll loops, each with its own SO_REUSEPORT
// listener and the connections it accepted.  A loop parses requests and JSON
// bodies and sends responses and watch chunks without any lock; the object
// store, the revision counter, the watch history and the watcher registry sit
// behind one state mutex, held only while a request mutates or reads them.
// Watch events are appended under that mutex to the watcher's buffer in
// revision order and sent by the loop that owns the watch connection (woken
// through its eventfd), one chunk per watcher per loop iteration.
//
// --watch-loop (with --threads N >= 2): loop 0 serves only watch streams and has no listener; loops 1..N-1
// accept and serve requests.  A request that becomes a watch is handed over with its connection, so a write
// emits its events to watcher buffers (state mutex) and at most one eventfd wakes the watch loop per batch;
// the request loops never send watch chunks and never wake each other.  At N = 8 on the MI355X box it does not
// move the wave either (per-wave p50 17.3-18.8k pods/s in every layout, profiles/r03e/watchloop_ab.md).
//
// Default 1 loop.  Measured on the MI355X box (bench.py, fake devices, N=8:
// 32 pods per wave, ~5 writes per pod): 4 loops were slower (10.7k vs 13.6k
// pods/s) -- each write is still serialised under the mutex, its hold time
// doubled once objects bounce between cores, and an event produced on one loop
// for a watch owned by another costs a wakeup hop on the wave's critical path.
// More loops pay off for many independent clients, not for one latency-bound
// chain of dependent writes.  GET /fake/stats reports lock wait / hold times.
//
//   gsx-fakeapi [--host 127.0.0.1] [--port 0] [--port-file F] [--history N] [--threads N]
//               [--watch-flush request|iteration] [--watch-loop]
#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <signal.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <deque>
#include <fstream>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "http.h"
#include "jdom.h"
#include "json.h"

using namespace gsx;

namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

std::string now_iso() {
  time_t t = time(nullptr);
  struct tm tmv;
  gmtime_r(&t, &tmv);
  char b[32];
  strftime(b, sizeof(b), "%Y-%m-%dT%H:%M:%SZ", &tmv);
  return b;
}

std::mt19937_64& rng() {
  static std::mt19937_64 r(std::random_device{}());
  return r;
}

std::string uuid4() {
  uint64_t a = rng()(), b = rng()();
  a = (a & 0xffffffffffff0fffull) | 0x0000000000004000ull;
  b = (b & 0x3fffffffffffffffull) | 0x8000000000000000ull;
  char s[40];
  std::snprintf(s, sizeof(s), "%08x-%04x-%04x-%04x-%012llx", static_cast<unsigned>(a >> 32),
                static_cast<unsigned>((a >> 16) & 0xffff), static_cast<unsigned>(a & 0xffff),
                static_cast<unsigned>(b >> 48), static_cast<unsigned long long>(b & 0xffffffffffffull));
  return s;
}

std::string url_unescape(std::string_view s) {
  std::string o;
  o.reserve(s.size());
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '%' && i + 2 < s.size()) {
      o.push_back(static_cast<char>(std::strtol(std::string(s.substr(i + 1, 2)).c_str(), nullptr, 16)));
      i += 2;
    } else if (s[i] == '+') {
      o.push_back(' ');
    } else {
      o.push_back(s[i]);
    }
  }
  return o;
}

std::map<std::string, std::string> parse_query(std::string_view target) {
  std::map<std::string, std::string> q;
  size_t qm = target.find('?');
  if (qm == std::string_view::npos) return q;
  std::string_view s = target.substr(qm + 1);
  size_t i = 0;
  while (i <= s.size()) {
    size_t j = s.find('&', i);
    if (j == std::string_view::npos) j = s.size();
    std::string_view kv = s.substr(i, j - i);
    size_t eq = kv.find('=');
    if (!kv.empty()) {
      q[url_unescape(kv.substr(0, eq))] = eq == std::string_view::npos ? "" : url_unescape(kv.substr(eq + 1));
    }
    i = j + 1;
  }
  return q;
}

std::vector<std::string> split(std::string_view s, char c) {
  std::vector<std::string> out;
  size_t i = 0;
  while (i <= s.size()) {
    size_t j = s.find(c, i);
    if (j == std::string_view::npos) j = s.size();
    out.emplace_back(s.substr(i, j - i));
    i = j + 1;
  }
  return out;
}

std::string trim(std::string s) {
  while (!s.empty() && s.back() == ' ') s.pop_back();
  size_t i = 0;
  while (i < s.size() && s[i] == ' ') ++i;
  return s.substr(i);
}

// A parsed label / field selector ("a=b,c!=d,e,!f"), matched many times per
// watch stream without re-splitting the string.
struct Selector {
  enum Op { Eq, Ne, Exists, NotExists };
  struct Term {
    std::string key, val;
    Op op;
  };
  std::vector<Term> terms;
  bool field = false;  // field selector: dotted paths, no existence terms

  static Selector parse(const std::string& sel, bool field) {
    Selector out;
    out.field = field;
    for (std::string term : split(sel, ',')) {
      term = trim(term);
      if (term.empty()) continue;
      Term t;
      size_t ne = term.find("!=");
      size_t eq = term.find('=');
      if (ne != std::string::npos) {
        t = {trim(term.substr(0, ne)), trim(term.substr(ne + 2)), Ne};
      } else if (eq != std::string::npos) {
        std::string val = term.substr(eq + 1);
        if (!val.empty() && val[0] == '=') val.erase(0, 1);  // "=="
        t = {trim(term.substr(0, eq)), trim(val), Eq};
      } else if (field) {
        t = {term, std::string(), Eq};  // malformed field term: never matches a non-empty value
      } else if (term[0] == '!') {
        t = {term.substr(1), std::string(), NotExists};
      } else {
        t = {term, std::string(), Exists};
      }
      out.terms.push_back(std::move(t));
    }
    return out;
  }

  bool matches(const jd::Value& obj) const {
    if (terms.empty()) return true;
    const jd::Value* labels = nullptr;
    if (!field) {
      const jd::Value* md = obj.get("metadata");
      labels = md ? md->get("labels") : nullptr;
    }
    for (const Term& t : terms) {
      if (field) {
        const jd::Value* v = obj.at_path(t.key);
        bool same = (v ? v->scalar_text() : std::string()) == t.val;
        if ((t.op == Eq) != same) return false;
        continue;
      }
      const jd::Value* v = labels ? labels->get(t.key) : nullptr;
      switch (t.op) {
        case Eq:
          if (!v || !v->is_str() || v->s != t.val) return false;
          break;
        case Ne:
          if (v && v->is_str() && v->s == t.val) return false;
          break;
        case Exists:
          if (!v) return false;
          break;
        case NotExists:
          if (v) return false;
          break;
      }
    }
    return true;
  }
};

std::string status_body(int code, const std::string& reason, const std::string& message, const std::string& name = "",
                        const std::string& kind = "") {
  std::string o = "{\"kind\":\"Status\",\"apiVersion\":\"v1\",\"metadata\":{},\"status\":\"Failure\",\"message\":";
  json::append_quoted(&o, message);
  o.append(",\"reason\":");
  json::append_quoted(&o, reason);
  o.append(",\"code\":").append(std::to_string(code));
  if (!name.empty()) {
    o.append(",\"details\":{\"name\":");
    json::append_quoted(&o, name);
    o.append(",\"kind\":");
    json::append_quoted(&o, kind);
    o.push_back('}');
  }
  o.push_back('}');
  return o;
}

struct HttpError {
  int code;
  std::string body;
};

HttpError conflict(const std::string& kind, const std::string& name) {
  return {409, status_body(409, "Conflict",
                           "Operation cannot be fulfilled on " + kind + " \"" + name +
                               "\": the object has been modified; please apply your changes to the latest version and "
                               "try again",
                           name, kind)};
}

HttpError not_found(const std::string& kind, const std::string& name) {
  return {404, status_body(404, "NotFound", kind + " \"" + name + "\" not found", name, kind)};
}

// A stored object: immutable once stored (writes replace the pointer), with
// its serialisation cached for GET / LIST / watch / write responses.
struct Obj {
  std::shared_ptr<const jd::Value> vp;  // shared with the DELETED copy of the object (make_deleted)
  int64_t rv = 0;                       // metadata.resourceVersion
  std::string json;
  std::string ns, name;
  const jd::Value& v() const { return *vp; }
};
using ObjP = std::shared_ptr<const Obj>;

ObjP make_obj(jd::Value v) {
  auto o = std::make_shared<Obj>();
  const jd::Value* md = v.get("metadata");
  if (md) {
    o->ns = md->str_or("namespace");
    o->name = md->str_or("name");
    o->rv = std::atoll(md->str_or("resourceVersion").c_str());
  }
  o->vp = std::make_shared<const jd::Value>(std::move(v));
  o->json = jd::dump(*o->vp);
  return o;
}

// The object as its DELETED event carries it: the last stored state under a new resourceVersion.  Its JSON is the
// stored JSON with that one value replaced, and it shares the stored object's tree (the watchers' selectors read
// labels and fields, which the deletion does not change): no deep copy and re-serialisation per deleted pod, a
// DeleteCollection of a wave's pods being a loop of them.  Falls back to a copy when the value is not unique.
ObjP make_deleted(const ObjP& cur, const std::string& rv) {
  const jd::Value* md = cur->v().get("metadata");
  const std::string old = "\"resourceVersion\":\"" + (md ? md->str_or("resourceVersion") : std::string()) + "\"";
  const size_t at = cur->json.find(old);
  if (at == std::string::npos || cur->json.find(old, at + 1) != std::string::npos) {
    jd::Value gone = cur->v();
    gone.member("metadata").set("resourceVersion", jd::Value::string(rv));
    return make_obj(std::move(gone));
  }
  auto o = std::make_shared<Obj>();
  o->vp = cur->vp;
  o->ns = cur->ns;
  o->name = cur->name;
  o->rv = std::atoll(rv.c_str());
  o->json.reserve(cur->json.size() + 8);
  o->json.append(cur->json, 0, at).append("\"resourceVersion\":\"").append(rv).append("\"");
  o->json.append(cur->json, at + old.size(), std::string::npos);
  return o;
}

struct Event {
  int64_t rv;
  std::string kind;
  std::shared_ptr<const std::string> line;
  ObjP obj;
};

struct Watcher;
struct Loop;

// A client connection; touched only by the loop that accepted it.
struct Conn {
  int fd = -1;
  uint64_t id = 0;
  std::string rbuf, wbuf;
  bool want_close = false;
  bool busy = false;                // a delayed response is pending
  bool handoff = false;             // became a watch owned by the watch loop: moves there after this request
  std::shared_ptr<Watcher> watch;   // streaming
  bool epollout = false;
};

// A watch stream.  `pending`, `dirty`, `closed` and `end_requested` are guarded
// by the state mutex; the rest is fixed at creation or owned by `owner`.
using Lines = std::vector<std::shared_ptr<const std::string>>;
struct Watcher {
  uint64_t conn_id;
  Loop* owner = nullptr;
  std::string kind, ns;
  Selector fsel, lsel;
  // the event lines queued for the next chunk: shared with the history and with every other watcher of the event
  // (a DeleteCollection of a wave's pods fans each line out to every pod watcher; it is copied once, into the
  // connection's buffer)
  Lines pending;
  uint64_t sent = 0, drop_after = 0;
  double deadline = 0;  // 0: none
  std::atomic<bool> closed{false};  // written under the state mutex, read anywhere
  bool dirty = false;          // queued on owner->dirty
  bool end_requested = false;  // another loop asked the owner to end it
  bool adopted = true;         // its connection is in owner->conns (false while handed over to the watch loop)
};

struct Delayed {
  double due;
  uint64_t conn;
  http::Message req;
};

struct Held {
  uint64_t conn;
  http::Message req;
};

// One event loop: its listener, eventfd and connections (owner-only), plus
// the watchers with events to send (`dirty`, `signaled`: state mutex).
struct Loop {
  int idx = 0;
  int ep = -1, lfd = -1, efd = -1;
  std::unordered_map<uint64_t, std::unique_ptr<Conn>> conns;
  std::vector<std::shared_ptr<Watcher>> mine;  // watches on this loop's connections
  std::vector<Delayed> delayed;
  std::vector<Held> held;
  std::vector<std::shared_ptr<Watcher>> dirty;
  std::vector<std::unique_ptr<Conn>> inbox;  // watch connections handed over by request loops (state mutex)
  bool signaled = false;
  std::atomic<bool> has_dirty{false};  // `dirty` is non-empty (checked before taking the mutex)
  // owner-written, read by /fake/stats
  std::atomic<uint64_t> busy_ns{0}, max_iter_ns{0}, flush_ns{0}, flushes{0};
  std::thread th;
};

thread_local Loop* tl_loop = nullptr;
// --watch-loop: a request loop wakes the watch loop once, at the end of its iteration, for all the events its
// requests of that iteration produced (as the single loop sends them in one chunk per watcher per iteration)
thread_local Loop* tl_deferred_wake = nullptr;

struct Faults {
  double conflict_rate = 0, error_rate = 0, latency_ms = 0;
  // API Priority and Fairness: this share of non-watch /api/v1 requests answers 429 with Retry-After: retry_after
  // seconds (fractional in tests; kube-apiserver sends whole seconds)
  double throttle_rate = 0, retry_after = 1;
  int64_t drop_watch_after = 0, expire_watches = 0;
  bool hold_watches = false;
  // an apiserver (or admission webhook) that does not copy Binding.metadata.annotations onto the pod
  bool drop_binding_annotations = false;
  std::string json() const {
    char b[448];
    std::snprintf(b, sizeof(b),
                  "{\"conflict_rate\":%g,\"error_rate\":%g,\"latency_ms\":%g,\"drop_watch_after\":%lld,"
                  "\"expire_watches\":%lld,\"hold_watches\":%s,\"drop_binding_annotations\":%s,"
                  "\"throttle_rate\":%g,\"retry_after\":%g}",
                  conflict_rate, error_rate, latency_ms, (long long)drop_watch_after, (long long)expire_watches,
                  hold_watches ? "true" : "false", drop_binding_annotations ? "true" : "false", throttle_rate,
                  retry_after);
    return b;
  }
};

struct Reply {
  int status = 200;
  std::string body;
  const char* ct = "application/json";
  std::string headers;  // extra header lines ("Name: value\r\n")
};

class Server;

// The state mutex with wait / hold accounting for /fake/stats.
struct LockStats {
  std::atomic<uint64_t> n{0}, wait_ns{0}, max_wait_ns{0}, hold_ns{0}, max_hold_ns{0};
};

inline uint64_t mono_ns() {
  return static_cast<uint64_t>(
      std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count());
}

inline void atomic_max(std::atomic<uint64_t>& a, uint64_t v) {
  uint64_t cur = a.load(std::memory_order_relaxed);
  while (v > cur && !a.compare_exchange_weak(cur, v, std::memory_order_relaxed)) {
  }
}

class StateLock {
 public:
  StateLock(std::mutex& m, LockStats& st) : m_(m), st_(st) {
    uint64_t t0 = mono_ns();
    m_.lock();
    t1_ = mono_ns();
    st_.n.fetch_add(1, std::memory_order_relaxed);
    st_.wait_ns.fetch_add(t1_ - t0, std::memory_order_relaxed);
    atomic_max(st_.max_wait_ns, t1_ - t0);
  }
  ~StateLock() {
    uint64_t h = mono_ns() - t1_;
    m_.unlock();
    st_.hold_ns.fetch_add(h, std::memory_order_relaxed);
    atomic_max(st_.max_hold_ns, h);
  }
  StateLock(const StateLock&) = delete;
  StateLock& operator=(const StateLock&) = delete;

 private:
  std::mutex& m_;
  LockStats& st_;
  uint64_t t1_ = 0;
};

class Server {
 public:
  Server(size_t history, int threads, bool flush_per_request, bool watch_loop)
      : history_max_(history), nloops_(std::max(1, std::min(64, threads))), flush_per_request_(flush_per_request),
        watch_loop_(watch_loop && nloops_ >= 2) {
    for (const char* k : {"pods", "nodes", "events", "leases"}) store_[k];
  }

  // One SO_REUSEPORT listener per loop on the same port (the first picks it when `port` is 0).
  int listen_on(const std::string& host, int port, std::string* err) {
    for (int i = 0; i < nloops_; ++i) {
      auto L = std::make_unique<Loop>();
      L->idx = i;
      if (watch_loop_ && i == 0) {  // the watch loop: no listener, only its eventfd and adopted connections
        L->ep = epoll_create1(EPOLL_CLOEXEC);
        L->efd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
        epoll_event ev;
        ev.events = EPOLLIN;
        ev.data.u64 = kWakeId;
        epoll_ctl(L->ep, EPOLL_CTL_ADD, L->efd, &ev);
        loops_.push_back(std::move(L));
        continue;
      }
      L->lfd = ::socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
      int one = 1;
      setsockopt(L->lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
      setsockopt(L->lfd, SOL_SOCKET, SO_REUSEPORT, &one, sizeof(one));
      sockaddr_in a;
      std::memset(&a, 0, sizeof(a));
      a.sin_family = AF_INET;
      a.sin_port = htons(static_cast<uint16_t>(port));
      inet_pton(AF_INET, host.c_str(), &a.sin_addr);
      if (::bind(L->lfd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || ::listen(L->lfd, 1024) != 0) {
        *err = std::string("bind/listen: ") + std::strerror(errno);
        return -1;
      }
      socklen_t len = sizeof(a);
      getsockname(L->lfd, reinterpret_cast<sockaddr*>(&a), &len);
      port = ntohs(a.sin_port);
      L->ep = epoll_create1(EPOLL_CLOEXEC);
      L->efd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
      epoll_event ev;
      ev.events = EPOLLIN;
      ev.data.u64 = kListenId;
      epoll_ctl(L->ep, EPOLL_CTL_ADD, L->lfd, &ev);
      ev.data.u64 = kWakeId;
      epoll_ctl(L->ep, EPOLL_CTL_ADD, L->efd, &ev);
      loops_.push_back(std::move(L));
    }
    return port;
  }

  void run(volatile sig_atomic_t* stop) {
    for (size_t i = 1; i < loops_.size(); ++i) {
      Loop* L = loops_[i].get();
      L->th = std::thread([this, L, stop] { loop_main(L, stop); });
    }
    loop_main(loops_[0].get(), stop);
    for (size_t i = 1; i < loops_.size(); ++i) loops_[i]->th.join();
  }

 private:
  static constexpr uint64_t kListenId = 0, kWakeId = 1;

  void loop_main(Loop* L, volatile sig_atomic_t* stop) {
    tl_loop = L;
    std::vector<epoll_event> evs(256);
    while (!*stop) {
      int timeout = next_timeout_ms(L);
      int n = epoll_wait(L->ep, evs.data(), static_cast<int>(evs.size()), timeout);
      double t_iter = now_s();
      if (watch_loop_ && L->idx == 0) adopt_watches(L);
      for (int i = 0; i < n; ++i) {
        uint64_t id = evs[i].data.u64;
        if (id == kListenId) {
          accept_all(L);
          continue;
        }
        if (id == kWakeId) {
          uint64_t v;
          while (::read(L->efd, &v, sizeof(v)) > 0) {
          }
          continue;
        }
        auto it = L->conns.find(id);
        if (it == L->conns.end()) continue;
        Conn* c = it->second.get();
        if (evs[i].events & (EPOLLERR | EPOLLHUP)) {
          close_conn(L, c);
          continue;
        }
        if (evs[i].events & EPOLLIN) on_readable(L, c);
        if (L->conns.count(id) && (evs[i].events & EPOLLOUT)) flush_conn(L, c);
      }
      run_timers(L);
      if (tl_deferred_wake != nullptr) {
        wake(tl_deferred_wake);
        tl_deferred_wake = nullptr;
      }
      double t_flush = now_s();
      if (flush_watchers(L)) {
        L->flushes.fetch_add(1, std::memory_order_relaxed);
        L->flush_ns.fetch_add(static_cast<uint64_t>((now_s() - t_flush) * 1e9), std::memory_order_relaxed);
      }
      uint64_t iter_ns = static_cast<uint64_t>((now_s() - t_iter) * 1e9);
      L->busy_ns.fetch_add(iter_ns, std::memory_order_relaxed);  // loop time outside epoll_wait
      atomic_max(L->max_iter_ns, iter_ns);
    }
    // leave every connection of this loop closed
    std::vector<Conn*> all;
    for (auto& kv : L->conns) all.push_back(kv.second.get());
    for (Conn* c : all) close_conn(L, c);
  }

  // ---------------------------------------------------------------- connections
  void accept_all(Loop* L) {
    while (true) {
      int fd = ::accept4(L->lfd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (fd < 0) return;
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      auto c = std::make_unique<Conn>();
      c->fd = fd;
      c->id = next_id_.fetch_add(1) + 2;  // 0 / 1: listener / eventfd
      epoll_event ev;
      ev.events = EPOLLIN | EPOLLRDHUP;
      ev.data.u64 = c->id;
      epoll_ctl(L->ep, EPOLL_CTL_ADD, fd, &ev);
      L->conns[c->id] = std::move(c);
    }
  }

  void close_conn(Loop* L, Conn* c) {
    if (c->watch) {
      StateLock g(smu_, lstats_);
      c->watch->closed = true;
    }
    epoll_ctl(L->ep, EPOLL_CTL_DEL, c->fd, nullptr);
    ::close(c->fd);
    L->conns.erase(c->id);
  }

  void on_readable(Loop* L, Conn* c) {
    char buf[65536];
    while (true) {
      long r = ::recv(c->fd, buf, sizeof(buf), 0);
      if (r > 0) {
        c->rbuf.append(buf, static_cast<size_t>(r));
        if (static_cast<size_t>(r) < sizeof(buf)) break;  // drained (level-triggered epoll wakes us for more)
        continue;
      }
      if (r == 0) {
        close_conn(L, c);
        return;
      }
      if (errno == EINTR) continue;
      break;  // EAGAIN
    }
    process(L, c);
  }

  void process(Loop* L, Conn* c) {
    uint64_t id = c->id;
    while (!c->busy && !c->watch && !c->rbuf.empty()) {
      http::Message req;
      std::string perr;
      long got = http::parse(c->rbuf.data(), c->rbuf.size(), true, &req, &perr);
      if (got == 0) return;
      if (got < 0) {
        respond(L, c, Reply{400, status_body(400, "BadRequest", perr)}, false);
        return;
      }
      c->rbuf.erase(0, static_cast<size_t>(got));
      handle(L, c, req, true);
      if (!L->conns.count(id)) return;
      if (flush_per_request_) {
        // push this write's watch events now, as kube-apiserver's per-watcher goroutines do, instead of at
        // the end of the loop iteration (a burst of creates then reaches the watchers one by one)
        flush_watchers(L);
        if (!L->conns.count(id)) return;
      }
    }
  }

  // A request body parsed outside the state mutex (JSON decoding is the costly part of a write).
  struct Body {
    bool ok = true;
    jd::Value v;
    std::string err;
  };

  static jd::Value take_body(Body& b) {
    if (!b.ok) throw HttpError{400, status_body(400, "BadRequest", "invalid JSON: " + b.err)};
    return std::move(b.v);
  }

  // `fresh`: the request has not been through the injected-latency queue yet.
  void handle(Loop* L, Conn* c, http::Message& req, bool fresh) {
    bool is_watch = false;
    {
      auto q = parse_query(req.target);
      auto w = q.find("watch");
      is_watch = w != q.end() && (w->second == "1" || w->second == "true");
    }
    Body body;
    if (!req.body.empty() && (req.method == "POST" || req.method == "PUT" || req.method == "PATCH")) {
      body.ok = jd::parse(req.body, &body.v, &body.err);
    } else {
      body.v = jd::Value::object();
    }
    std::string cls = route_class(req);
    Reply rep;
    bool reply = true;
    {
      StateLock g(smu_, lstats_);
      if (fresh) counts_[req.method]++;
      if (fresh && faults_.latency_ms > 0 && !is_watch) {
        c->busy = true;
        L->delayed.push_back({now_s() + faults_.latency_ms / 1000.0, c->id, std::move(req)});
        return;
      }
      double t0 = now_s();
      RouteTime& rt = route_time_[cls];
      rt.n++;
      if (!is_watch && faults_.throttle_rate > 0 && req.path().substr(0, 8) == "/api/v1/" &&
          std::uniform_real_distribution<double>(0, 1)(rng()) < faults_.throttle_rate) {
        counts_["injected_throttle"]++;
        char ra[64];
        std::snprintf(ra, sizeof(ra), "Retry-After: %g\r\n", faults_.retry_after);
        rep.status = 429;
        rep.headers = ra;
        rep.body = status_body(429, "TooManyRequests", "Too many requests, please try again later.");
      } else {
        try {
          reply = route(L, c, req, body, &rep);  // false: became a watch stream (or is held)
        } catch (const HttpError& e) {
          rep.status = e.code;
          rep.body = e.body;
        }
      }
      rt.s += now_s() - t0;
    }
    if (reply) {
      respond(L, c, rep, req.keep_alive);
    } else if (c->handoff) {
      hand_over(L, c);
    } else if (!c->wbuf.empty() || c->want_close) {
      flush_conn(L, c);
    }
  }

  // A request loop's connection that became a watch: off this loop's epoll, into the watch loop's inbox.
  void hand_over(Loop* L, Conn* c) {
    c->handoff = false;
    epoll_ctl(L->ep, EPOLL_CTL_DEL, c->fd, nullptr);
    auto it = L->conns.find(c->id);
    std::unique_ptr<Conn> up = std::move(it->second);
    L->conns.erase(it);
    Loop* W = loops_[0].get();
    StateLock g(smu_, lstats_);
    W->inbox.push_back(std::move(up));
    W->signaled = true;
    wake(W);
  }

  // The watch loop: take over the handed-over connections, then send what their watchers hold.
  void adopt_watches(Loop* L) {
    std::vector<std::unique_ptr<Conn>> in;
    {
      StateLock g(smu_, lstats_);
      if (L->inbox.empty()) return;
      in.swap(L->inbox);
      for (auto& c : in) {
        c->watch->adopted = true;
        if (c->watch->closed) continue;
        L->mine.push_back(c->watch);
        mark_dirty_locked(c->watch);  // no-op if an event already queued it here (flushed once adopted)
      }
    }
    for (auto& c : in) {
      Conn* raw = c.get();
      if (raw->watch->closed) {
        ::close(raw->fd);
        continue;
      }
      epoll_event ev;
      ev.events = EPOLLIN | EPOLLRDHUP;
      ev.data.u64 = raw->id;
      epoll_ctl(L->ep, EPOLL_CTL_ADD, raw->fd, &ev);
      raw->epollout = false;
      L->conns[raw->id] = std::move(c);
      flush_conn(L, raw);  // the response head (and anything the request loop had queued)
    }
  }

  // "METHOD kind[/sub]" (names and namespaces dropped) for the per-route time table of /fake/stats.
  static std::string route_class(const http::Message& req) {
    std::vector<std::string> seg = split(std::string(req.path()), '/');
    std::string k;
    if (seg.size() >= 4 && seg[1] == "api" && seg[2] == "v1") {
      size_t at = seg[3] == "namespaces" && seg.size() >= 6 ? 5 : 3;
      k = seg[at];
      if (seg.size() == at + 3) k += "/" + seg[at + 2];
      if (seg.size() == at + 1 && req.target.find("watch=") != std::string::npos) k += "?watch";
    } else {
      k = std::string(req.path());
    }
    return req.method + " " + k;
  }

  void respond(Loop* L, Conn* c, const Reply& r, bool keep_alive) {
    c->wbuf.append(http::response(r.status, r.ct, r.body, keep_alive, r.headers));
    if (!keep_alive) c->want_close = true;
    flush_conn(L, c);
  }

  void flush_conn(Loop* L, Conn* c) {
    while (!c->wbuf.empty()) {
      long w = ::send(c->fd, c->wbuf.data(), c->wbuf.size(), MSG_NOSIGNAL);
      if (w > 0) {
        c->wbuf.erase(0, static_cast<size_t>(w));
        continue;
      }
      if (w < 0 && errno == EINTR) continue;
      if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
        if (!c->epollout) {
          epoll_event ev;
          ev.events = EPOLLIN | EPOLLOUT | EPOLLRDHUP;
          ev.data.u64 = c->id;
          epoll_ctl(L->ep, EPOLL_CTL_MOD, c->fd, &ev);
          c->epollout = true;
        }
        return;
      }
      close_conn(L, c);
      return;
    }
    if (c->epollout) {
      epoll_event ev;
      ev.events = EPOLLIN | EPOLLRDHUP;
      ev.data.u64 = c->id;
      epoll_ctl(L->ep, EPOLL_CTL_MOD, c->fd, &ev);
      c->epollout = false;
    }
    if (c->want_close) close_conn(L, c);
  }

  void wake(Loop* L) {
    uint64_t one = 1;
    ssize_t r = ::write(L->efd, &one, sizeof(one));
    (void)r;
  }

  // ---------------------------------------------------------------- timers
  int next_timeout_ms(Loop* L) {
    double now = now_s();
    double next = now + 1.0;
    for (auto& d : L->delayed) next = std::min(next, d.due);
    for (auto& w : L->mine) {
      if (w->deadline > 0) next = std::min(next, w->deadline);
    }
    if (!L->held.empty()) next = std::min(next, now + 0.005);
    double ms = (next - now) * 1000.0;
    return ms <= 0 ? 0 : static_cast<int>(ms) + 1;
  }

  void run_timers(Loop* L) {
    double now = now_s();
    if (!L->delayed.empty()) {
      std::vector<Delayed> due;
      for (auto it = L->delayed.begin(); it != L->delayed.end();) {
        if (it->due <= now) {
          due.push_back(std::move(*it));
          it = L->delayed.erase(it);
        } else {
          ++it;
        }
      }
      for (auto& d : due) {
        auto it = L->conns.find(d.conn);
        if (it == L->conns.end()) continue;
        Conn* c = it->second.get();
        c->busy = false;
        handle(L, c, d.req, false);
        if (L->conns.count(d.conn)) process(L, c);
      }
    }
    if (!L->mine.empty()) {
      // prune closed watches and end the expired ones (timeoutSeconds)
      std::vector<std::shared_ptr<Watcher>> expired, keep;
      for (auto& w : L->mine) {
        if (w->closed) continue;
        if (w->deadline > 0 && w->deadline <= now) {
          expired.push_back(w);
        } else {
          keep.push_back(w);
        }
      }
      L->mine.swap(keep);
      for (auto& w : expired) end_watch(L, w);
    }
    if (!L->held.empty()) {
      bool hold;
      {
        StateLock g(smu_, lstats_);
        hold = faults_.hold_watches;
      }
      if (!hold) {
        auto held = std::move(L->held);
        L->held.clear();
        for (auto& h : held) {
          auto it = L->conns.find(h.conn);
          if (it == L->conns.end()) continue;
          Conn* c = it->second.get();
          c->busy = false;
          handle(L, c, h.req, false);
          if (L->conns.count(h.conn)) process(L, c);
        }
      }
    }
  }

  // ---------------------------------------------------------------- watch
  // State mutex held: append the event to every matching watcher and queue the
  // watcher on its owner loop (woken unless it is the calling loop, which
  // flushes at the end of its iteration).
  void emit(const std::string& kind, const char* etype, const ObjP& o) {
    const int64_t rv = o->rv;
    auto line = std::make_shared<std::string>();
    line->reserve(o->json.size() + 32);
    line->append("{\"type\":\"").append(etype).append("\",\"object\":").append(o->json).append("}\n");
    if (history_.size() >= history_max_) {
      oldest_rv_ = history_.front().rv;  // watches from before this are told 410 Gone
      history_.pop_front();
    }
    history_.push_back(Event{rv, kind, line, o});
    for (auto& w : watchers_) {
      if (!w->closed && w->kind == kind && wants(*w, *o)) {
        w->pending.push_back(line);
        mark_dirty_locked(w);
      }
    }
  }

  void mark_dirty_locked(const std::shared_ptr<Watcher>& w) {
    if (w->dirty) return;
    w->dirty = true;
    Loop* L = w->owner;
    L->dirty.push_back(w);
    L->has_dirty.store(true);
    if (L != tl_loop && !L->signaled) {
      L->signaled = true;
      if (watch_loop_ && tl_loop != nullptr && tl_loop->idx != 0) {
        tl_deferred_wake = L;
      } else {
        wake(L);
      }
    }
  }

  bool wants(const Watcher& w, const Obj& o) const {
    if (!w.ns.empty() && o.ns != w.ns) return false;
    return w.fsel.matches(o.v()) && w.lsel.matches(o.v());
  }

  // Send what this loop's dirty watchers accumulated: buffers are taken under the
  // state mutex, the socket writes happen outside it.
  // Returns whether there was anything to send.
  bool flush_watchers(Loop* L) {
    struct Out {
      std::shared_ptr<Watcher> w;
      Lines data;
      bool end;
    };
    std::vector<Out> outs;
    if (!L->has_dirty.exchange(false)) return false;
    {
      StateLock g(smu_, lstats_);
      L->signaled = false;
      if (L->dirty.empty()) return false;
      for (auto& w : L->dirty) {
        w->dirty = false;
        if (w->closed || !w->adopted) continue;  // not adopted yet: adopt_watches re-queues it
        Out o{w, std::move(w->pending), w->end_requested};
        w->pending.clear();
        // one chunk per loop iteration; count events for drop_watch_after
        w->sent += static_cast<uint64_t>(o.data.size());
        if (w->drop_after && w->sent >= w->drop_after) {
          counts_["watch_dropped"]++;
          o.end = true;
        }
        outs.push_back(std::move(o));
      }
      L->dirty.clear();
      watchers_.erase(std::remove_if(watchers_.begin(), watchers_.end(),
                                     [](const std::shared_ptr<Watcher>& w) { return w->closed.load(); }),
                      watchers_.end());
    }
    for (auto& o : outs) {
      auto it = L->conns.find(o.w->conn_id);
      if (it == L->conns.end()) {
        StateLock g(smu_, lstats_);
        o.w->closed = true;
        continue;
      }
      Conn* c = it->second.get();
      append_chunk(c, o.data);
      if (o.end) {
        end_watch(L, o.w);
        continue;
      }
      flush_conn(L, c);
    }
    return true;
  }

  // One HTTP chunk of event lines onto the connection's buffer.
  static void append_chunk(Conn* c, const Lines& lines) {
    size_t n = 0;
    for (const auto& l : lines) n += l->size();
    if (!n) return;
    char hdr[32];
    std::snprintf(hdr, sizeof(hdr), "%zx\r\n", n);
    c->wbuf.reserve(c->wbuf.size() + n + 40);
    c->wbuf.append(hdr);
    for (const auto& l : lines) c->wbuf.append(*l);
    c->wbuf.append("\r\n");
  }

  // Owner loop only: send what is pending, the terminating chunk, and close.
  void end_watch(Loop* L, const std::shared_ptr<Watcher>& w) {
    Lines rest;
    {
      StateLock g(smu_, lstats_);
      if (w->closed) return;
      w->closed = true;
      rest = std::move(w->pending);
      w->pending.clear();
    }
    auto it = L->conns.find(w->conn_id);
    if (it == L->conns.end()) return;
    Conn* c = it->second.get();
    c->watch = nullptr;
    append_chunk(c, rest);
    c->wbuf.append("0\r\n\r\n");
    c->want_close = true;
    flush_conn(L, c);
  }

  // State mutex held (called from route).  Returns false: the request became a
  // (held) watch stream; the caller flushes what was queued on the connection.
  bool start_watch(Loop* L, Conn* c, const http::Message& req, const std::string& kind, const std::string& ns,
                   const std::map<std::string, std::string>& q) {
    if (faults_.hold_watches) {
      c->busy = true;
      L->held.push_back({c->id, req});
      return false;
    }
    std::string head = "HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nTransfer-Encoding: chunked\r\n\r\n";
    auto get = [&](const char* k) {
      auto it = q.find(k);
      return it == q.end() ? std::string() : it->second;
    };
    if (faults_.expire_watches > 0) {
      faults_.expire_watches--;
      counts_["watch_expired"]++;
      std::string line = "{\"type\":\"ERROR\",\"object\":" +
                         status_body(410, "Expired", "too old resource version (injected)") + "}\n";
      char hdr[32];
      std::snprintf(hdr, sizeof(hdr), "%zx\r\n", line.size());
      c->wbuf.append(head).append(hdr).append(line).append("\r\n0\r\n\r\n");
      c->want_close = true;
      return false;
    }
    auto w = std::make_shared<Watcher>();
    w->conn_id = c->id;
    w->owner = L;
    w->kind = kind;
    w->ns = ns;
    w->fsel = Selector::parse(get("fieldSelector"), true);
    w->lsel = Selector::parse(get("labelSelector"), false);
    w->drop_after = static_cast<uint64_t>(std::max<int64_t>(0, faults_.drop_watch_after));
    std::string to = get("timeoutSeconds");
    if (!to.empty() && std::atof(to.c_str()) > 0) w->deadline = now_s() + std::atof(to.c_str());
    std::string rvs = get("resourceVersion");
    if (!rvs.empty() && rvs != "0") {
      int64_t rv = std::atoll(rvs.c_str());
      if (oldest_rv_ && rv < oldest_rv_) {
        std::string line = "{\"type\":\"ERROR\",\"object\":" +
                           status_body(410, "Expired", "too old resource version: " + std::to_string(rv) + " (" +
                                                           std::to_string(oldest_rv_) + ")") +
                           "}\n";
        char hdr[32];
        std::snprintf(hdr, sizeof(hdr), "%zx\r\n", line.size());
        c->wbuf.append(head).append(hdr).append(line).append("\r\n0\r\n\r\n");
        c->want_close = true;
        return false;
      }
      // backlog: history after rv (binary search: history is rv-ordered)
      auto it = std::upper_bound(history_.begin(), history_.end(), rv,
                                 [](int64_t v, const Event& e) { return v < e.rv; });
      for (; it != history_.end(); ++it) {
        if (it->kind == kind && wants(*w, *it->obj)) w->pending.push_back(it->line);
      }
    } else {
      for (auto& kv : store_[kind]) {
        if (wants(*w, *kv.second)) {
          auto line = std::make_shared<std::string>();
          line->reserve(kv.second->json.size() + 32);
          line->append("{\"type\":\"ADDED\",\"object\":").append(kv.second->json).append("}\n");
          w->pending.push_back(std::move(line));
        }
      }
    }
    c->wbuf.append(head);
    c->watch = w;
    watchers_.push_back(w);
    if (watch_loop_ && L->idx != 0) {
      w->owner = loops_[0].get();
      w->adopted = false;
      c->handoff = true;  // handle() moves the connection after this request
      return false;
    }
    L->mine.push_back(w);
    if (!w->pending.empty()) mark_dirty_locked(w);
    return false;
  }

  // ---------------------------------------------------------------- store
  using Key = std::pair<std::string, std::string>;
  std::string bump() { return std::to_string(++rv_); }

  ObjP get_obj(const std::string& kind, const std::string& ns, const std::string& name) {
    auto& m = store_[kind];
    auto it = m.find({kind == "nodes" ? std::string() : ns, name});
    if (it == m.end()) throw not_found(kind, name);
    return it->second;
  }

  void maybe_error() {
    if (faults_.error_rate > 0 && std::uniform_real_distribution<double>(0, 1)(rng()) < faults_.error_rate) {
      counts_["injected_error"]++;
      throw HttpError{500, status_body(500, "InternalError", "injected fault")};
    }
  }

  bool injected_conflict() {
    if (faults_.conflict_rate > 0 && std::uniform_real_distribution<double>(0, 1)(rng()) < faults_.conflict_rate) {
      counts_["injected_conflict"]++;
      return true;
    }
    return false;
  }

  ObjP do_create(const std::string& kind, jd::Value obj, const std::string& ns) {
    jd::Value& md = obj.member("metadata");
    if (kind != "nodes") {
      if (!ns.empty()) md.set("namespace", jd::Value::string(ns));
      if (!md.get("namespace")) md.set("namespace", jd::Value::string("default"));
    }
    std::string name = md.str_or("name");
    if (name.empty()) {
      std::string gen = md.str_or("generateName");
      if (gen.empty()) throw HttpError{422, status_body(422, "Invalid", "metadata.name: Required value")};
      name = gen + uuid4().substr(0, 5);
      md.set("name", jd::Value::string(name));
    }
    Key key{kind == "nodes" ? std::string() : md.str_or("namespace"), name};
    auto& m = store_[kind];
    if (m.count(key)) throw HttpError{409, status_body(409, "AlreadyExists", kind + " \"" + name + "\" already exists")};
    if (md.str_or("uid").empty()) md.set("uid", jd::Value::string(uuid4()));
    if (!md.get("creationTimestamp")) md.set("creationTimestamp", jd::Value::string(now_iso()));
    if (kind == "pods") {
      jd::Value& st = obj.member("status");
      if (!st.get("phase")) st.set("phase", jd::Value::string("Pending"));
      obj.member("spec");
    }
    md.set("resourceVersion", jd::Value::string(bump()));
    ObjP o = make_obj(std::move(obj));
    m[key] = o;
    emit(kind, "ADDED", o);
    return o;
  }

  static void keep_server_fields(const jd::Value& cur_md, jd::Value* md) {
    for (const char* f : {"uid", "creationTimestamp", "namespace", "name", "deletionTimestamp"}) {
      const jd::Value* v = cur_md.get(f);
      if (v) md->set(f, *v);
    }
  }

  ObjP do_replace(const std::string& kind, const std::string& ns, const std::string& name, jd::Value obj,
                  const std::string& sub) {
    ObjP cur = get_obj(kind, ns, name);
    const jd::Value& cmd = *cur->v().get("metadata");
    const jd::Value* omd = obj.get("metadata");
    std::string want = omd ? omd->str_or("resourceVersion") : std::string();
    if (!want.empty() && want != cmd.str_or("resourceVersion")) throw conflict(kind, name);
    if (kind == "pods" && injected_conflict()) throw conflict(kind, name);
    jd::Value nv;
    if (sub == "status") {
      nv = cur->v();
      const jd::Value* st = obj.get("status");
      nv.set("status", st ? *st : jd::Value::object());
    } else {
      nv = std::move(obj);
      jd::Value& md = nv.member("metadata");
      keep_server_fields(cmd, &md);
      if (kind == "pods") {
        const jd::Value* cs = cur->v().get("spec");
        const jd::Value* on = cs ? cs->get("nodeName") : nullptr;
        jd::Value& spec = nv.member("spec");
        if (on && on->is_str() && !on->s.empty()) {
          spec.set("nodeName", *on);
        } else {
          spec.erase("nodeName");
        }
        const jd::Value* cst = cur->v().get("status");
        nv.set("status", cst ? *cst : jd::Value::object());
      }
    }
    nv.member("metadata").set("resourceVersion", jd::Value::string(bump()));
    ObjP o = make_obj(std::move(nv));
    store_[kind][{kind == "nodes" ? std::string() : ns, name}] = o;
    emit(kind, "MODIFIED", o);
    return o;
  }

  ObjP do_patch(const std::string& kind, const std::string& ns, const std::string& name, jd::Value patch,
                const std::string& sub) {
    ObjP cur = get_obj(kind, ns, name);
    const jd::Value& cmd = *cur->v().get("metadata");
    const jd::Value* pmd = patch.get("metadata");
    std::string want = pmd ? pmd->str_or("resourceVersion") : std::string();
    if (!want.empty() && want != cmd.str_or("resourceVersion")) throw conflict(kind, name);
    // a merge patch that names another metadata.uid than the stored object's: kube-apiserver applies the patch and
    // its update validation refuses the changed immutable field (422 Invalid) -- a PATCH carries no UID
    // precondition (only a PUT's object or a Binding does: 409 below)
    std::string want_uid = pmd ? pmd->str_or("uid") : std::string();
    if (!want_uid.empty() && want_uid != cmd.str_or("uid")) {
      throw HttpError{422, status_body(422, "Invalid", kind == "pods" ? "Pod \"" + name + "\" is invalid: metadata.uid: "
                                                                          "Invalid value: \"" + want_uid +
                                                                          "\": field is immutable"
                                                                    : "metadata.uid: Invalid value: \"" + want_uid +
                                                                          "\": field is immutable")};
    }
    if (kind == "pods" && injected_conflict()) throw conflict(kind, name);
    if (sub == "status") {
      jd::Value p = jd::Value::object();
      const jd::Value* st = patch.get("status");
      p.set("status", st ? *st : jd::Value::object());
      patch = std::move(p);
    } else if (kind == "pods") {
      jd::Value* spec = patch.get("spec");
      if (spec && spec->is_obj()) spec->erase("nodeName");
      if (sub.empty()) patch.erase("status");
    }
    jd::Value nv = cur->v();
    jd::merge_patch(&nv, patch);
    jd::Value& md = nv.member("metadata");
    keep_server_fields(cmd, &md);
    md.set("resourceVersion", jd::Value::string(bump()));
    ObjP o = make_obj(std::move(nv));
    store_[kind][{kind == "nodes" ? std::string() : ns, name}] = o;
    emit(kind, "MODIFIED", o);
    return o;
  }

  void do_bind(const std::string& ns, const std::string& name, const jd::Value& binding) {
    ObjP cur = get_obj("pods", ns, name);
    const jd::Value& cmd = *cur->v().get("metadata");
    const jd::Value* bmd = binding.get("metadata");
    std::string buid = bmd ? bmd->str_or("uid") : std::string();
    if (!buid.empty() && buid != cmd.str_or("uid")) {
      throw HttpError{409, status_body(409, "Conflict", "Precondition failed: UID in precondition: " + buid +
                                                            ", UID in object meta: " + cmd.str_or("uid"))};
    }
    if (injected_conflict()) throw conflict("pods", name);
    const jd::Value* cs = cur->v().get("spec");
    std::string cur_node = cs ? cs->str_or("nodeName") : std::string();
    if (!cur_node.empty()) {
      throw HttpError{409, status_body(409, "Conflict", "pod " + name + " is already assigned to node \"" + cur_node + "\"")};
    }
    if (cmd.get("deletionTimestamp") && !cmd.get("deletionTimestamp")->is_null()) {
      throw HttpError{409, status_body(409, "Conflict", "pod " + name + " is being deleted")};
    }
    const jd::Value* tgt = binding.get("target");
    std::string target = tgt ? tgt->str_or("name") : std::string();
    if (target.empty()) throw HttpError{422, status_body(422, "Invalid", "target.name: Required value")};
    jd::Value nv = cur->v();
    nv.member("spec").set("nodeName", jd::Value::string(target));
    const jd::Value* ann = bmd ? bmd->get("annotations") : nullptr;
    if (faults_.drop_binding_annotations) ann = nullptr;
    if (ann && ann->is_obj() && !ann->o.empty()) {
      jd::Value& a = nv.member("metadata").member("annotations");
      for (const auto& m : ann->o) a.set(m.first, m.second);
    }
    jd::Value& st = nv.member("status");
    jd::Value* conds = st.get("conditions");
    if (!conds || conds->k != jd::Value::Arr) {
      st.set("conditions", jd::Value::array());
      conds = st.get("conditions");
    }
    jd::Value c = jd::Value::object();
    c.set("type", jd::Value::string("PodScheduled"));
    c.set("status", jd::Value::string("True"));
    c.set("lastTransitionTime", jd::Value::string(now_iso()));
    conds->a.push_back(std::move(c));
    nv.member("metadata").set("resourceVersion", jd::Value::string(bump()));
    ObjP o = make_obj(std::move(nv));
    store_["pods"][{ns, name}] = o;
    emit("pods", "MODIFIED", o);
  }

  // DELETE as kube-apiserver answers it.  A bound pod that is not terminal is deleted gracefully: it gets
  // deletionTimestamp and stays until a delete with grace 0 -- its kubelet's, once the containers stopped (the
  // kubelet stand-ins, gsxtools/agent.py and native/nodeagent, do that).  grace < 0 (none given) takes the pod's
  // spec.terminationGracePeriodSeconds, absent: 0 (the pods the harness builds carry none).  `uid`: the
  // DeleteOptions' preconditions.uid (409 on mismatch).
  ObjP do_delete(const std::string& kind, const std::string& ns, const std::string& name, double grace,
                 const std::string& uid = std::string()) {
    ObjP cur = get_obj(kind, ns, name);
    Key key{kind == "nodes" ? std::string() : ns, name};
    const jd::Value& cmd0 = *cur->v().get("metadata");
    if (!uid.empty() && uid != cmd0.str_or("uid")) {
      throw HttpError{409, status_body(409, "Conflict", "Precondition failed: UID in precondition: " + uid +
                                                            ", UID in object meta: " + cmd0.str_or("uid"))};
    }
    const jd::Value* cs = cur->v().get("spec");
    if (kind == "pods" && grace < 0 && cs) {
      const jd::Value* tg = cs->get("terminationGracePeriodSeconds");
      grace = (tg && tg->k == jd::Value::Num) ? std::atof(tg->s.c_str()) : 0;
    }
    const jd::Value* st = cur->v().get("status");
    std::string phase = st ? st->str_or("phase") : std::string();
    if (kind == "pods" && grace > 0 && cs && !cs->str_or("nodeName").empty() && phase != "Succeeded" &&
        phase != "Failed") {
      const jd::Value& cmd = *cur->v().get("metadata");
      const jd::Value* dt = cmd.get("deletionTimestamp");
      if (dt && !dt->is_null()) return cur;
      jd::Value nv = cur->v();
      jd::Value& md = nv.member("metadata");
      md.set("deletionTimestamp", jd::Value::string(now_iso()));
      md.set("deletionGracePeriodSeconds", jd::Value::number(static_cast<int64_t>(grace)));
      md.set("resourceVersion", jd::Value::string(bump()));
      ObjP o = make_obj(std::move(nv));
      store_[kind][key] = o;
      emit(kind, "MODIFIED", o);
      return o;
    }
    store_[kind].erase(key);
    ObjP o = make_deleted(cur, bump());
    emit(kind, "DELETED", o);
    return o;
  }

  // ---------------------------------------------------------------- routing
  // DeleteOptions: gracePeriodSeconds (query or body; -1 none given) and preconditions.uid (body)
  static double grace_of(const http::Message& req, const std::map<std::string, std::string>& q,
                         std::string* uid = nullptr) {
    double grace = -1;
    if (!req.body.empty()) {
      jd::Value v;
      std::string err;
      if (jd::parse(req.body, &v, &err)) {
        const jd::Value* g = v.get("gracePeriodSeconds");
        if (g && g->k == jd::Value::Num) grace = std::atof(g->s.c_str());
        const jd::Value* pc = v.get("preconditions");
        if (uid && pc && pc->is_obj()) *uid = pc->str_or("uid");
      }
    }
    auto it = q.find("gracePeriodSeconds");
    if (it != q.end()) grace = std::atof(it->second.c_str());
    return grace;
  }

  // LIST, optionally paginated like kube-apiserver: `limit` caps the items of one response and
  // metadata.continue ("<rv>:<ns>/<name>" of the last item sent) resumes after it, in key order; every
  // page reports the first page's resourceVersion.
  std::string list_json(const std::string& kind, const std::string& ns, const std::string& fsel,
                        const std::string& lsel, int64_t limit = 0, const std::string& cont = std::string()) {
    static const std::map<std::string, std::string> lists = {
        {"pods", "PodList"}, {"nodes", "NodeList"}, {"events", "EventList"}, {"leases", "LeaseList"}};
    auto& m = store_[kind];
    auto it = m.begin();
    std::string list_rv = std::to_string(rv_);
    if (!cont.empty()) {
      size_t colon = cont.find(':'), slash = cont.find('/', colon == std::string::npos ? 0 : colon);
      if (colon == std::string::npos || slash == std::string::npos) {
        throw HttpError{400, status_body(400, "BadRequest", "invalid continue token")};
      }
      list_rv = cont.substr(0, colon);
      it = m.upper_bound(Key{cont.substr(colon + 1, slash - colon - 1), cont.substr(slash + 1)});
    }
    std::string items;
    bool first = true;
    int64_t n = 0;
    std::string next;
    const Key* last_sent = nullptr;
    Selector fs = Selector::parse(fsel, true), ls = Selector::parse(lsel, false);
    for (; it != m.end(); ++it) {
      if (!ns.empty() && it->second->ns != ns) continue;
      if (!fs.matches(it->second->v()) || !ls.matches(it->second->v())) continue;
      if (limit > 0 && n == limit) {  // more matching items remain: continue after the last one sent
        next = list_rv + ":" + last_sent->first + "/" + last_sent->second;
        break;
      }
      if (!first) items.push_back(',');
      first = false;
      items.append(it->second->json);
      last_sent = &it->first;
      ++n;
    }
    std::string o = "{\"kind\":\"" + lists.at(kind) + "\",\"apiVersion\":\"v1\",\"metadata\":{\"resourceVersion\":\"" +
                    list_rv + "\"";
    if (!next.empty()) {
      o.append(",\"continue\":");
      json::append_quoted(&o, next);
    }
    o.append("},\"items\":[");
    o.append(items);
    o.append("]}");
    return o;
  }

  // Collection routes: (kind, ns) for "/api/v1/<kind>", "/api/v1/namespaces/<ns>/<kind>",
  // "/apis/coordination.k8s.io/v1/namespaces/<ns>/leases"; item routes add name and subresource.
  bool route(Loop* L, Conn* c, http::Message& req, Body& body, Reply* rep) {
    std::string path(req.path());
    auto q = parse_query(req.target);
    const std::string& m = req.method;
    if (path == "/version") {
      rep->body = "{\"major\":\"1\",\"minor\":\"30\",\"gitVersion\":\"v1.30.0-gsx-fake-native\",\"platform\":\"linux/amd64\"}";
      return true;
    }
    if (path == "/healthz") {
      rep->body = "ok";
      rep->ct = "text/plain";
      return true;
    }
    if (path == "/api") {
      rep->body = "{\"kind\":\"APIVersions\",\"versions\":[\"v1\"]}";
      return true;
    }
    if (path == "/fake/faults") {
      if (m == "POST") {
        jd::Value b = take_body(body);
        auto num = [&](const char* k, double* dst) {
          const jd::Value* v = b.get(k);
          if (v && v->k == jd::Value::Num) *dst = std::atof(v->s.c_str());
        };
        auto inum = [&](const char* k, int64_t* dst) {
          const jd::Value* v = b.get(k);
          if (v && v->k == jd::Value::Num) *dst = std::atoll(v->s.c_str());
        };
        num("conflict_rate", &faults_.conflict_rate);
        num("error_rate", &faults_.error_rate);
        num("latency_ms", &faults_.latency_ms);
        num("throttle_rate", &faults_.throttle_rate);
        num("retry_after", &faults_.retry_after);
        inum("drop_watch_after", &faults_.drop_watch_after);
        inum("expire_watches", &faults_.expire_watches);
        const jd::Value* h = b.get("hold_watches");
        if (h && h->k == jd::Value::Bool) faults_.hold_watches = h->b;
        const jd::Value* dba = b.get("drop_binding_annotations");
        if (dba && dba->k == jd::Value::Bool) faults_.drop_binding_annotations = dba->b;
        const jd::Value* seed = b.get("seed");
        if (seed && seed->k == jd::Value::Num) rng().seed(static_cast<uint64_t>(std::atoll(seed->s.c_str())));
        const jd::Value* drop = b.get("drop_watches_now");
        if (drop && drop->k == jd::Value::Bool && drop->b) {
          for (auto& w : watchers_) {  // each owner loop ends its own watches
            if (w->closed) continue;
            w->end_requested = true;
            mark_dirty_locked(w);
          }
        }
      }
      rep->body = faults_.json();
      return true;
    }
    // {"token": "...", "user": "...", "node": "..."}: what a TokenReview answers (node: the bound token's
    // authentication.kubernetes.io/node-name claim, optional)
    if (path == "/fake/tokens" && m == "POST") {
      jd::Value b = take_body(body);
      const jd::Value* t = b.get("token");
      const jd::Value* u = b.get("user");
      const jd::Value* nd = b.get("node");
      if (t && t->k == jd::Value::Str && u && u->k == jd::Value::Str) {
        tokens_[t->s] = {u->s, nd && nd->k == jd::Value::Str ? nd->s : std::string()};
      }
      rep->body = "{}";
      return true;
    }
    if (path == "/apis/authentication.k8s.io/v1/tokenreviews" && m == "POST") {
      jd::Value b = take_body(body);
      const jd::Value* spec = b.get("spec");
      const jd::Value* t = spec ? spec->get("token") : nullptr;
      auto it = (t && t->k == jd::Value::Str) ? tokens_.find(t->s) : tokens_.end();
      counts_["tokenreviews"]++;
      std::string o = "{\"kind\":\"TokenReview\",\"apiVersion\":\"authentication.k8s.io/v1\",\"status\":{";
      if (it != tokens_.end()) {
        o.append("\"authenticated\":true,\"user\":{\"username\":");
        json::append_quoted(&o, it->second.first);
        if (!it->second.second.empty()) {
          o.append(",\"extra\":{\"authentication.kubernetes.io/node-name\":[");
          json::append_quoted(&o, it->second.second);
          o.append("]}");
        }
        o.append("}}}");
      } else {
        o.append("\"authenticated\":false}}");
      }
      rep->status = 201;
      rep->body = o;
      return true;
    }
    if (path == "/fake/stats") {
      std::string o = "{\"rv\":" + std::to_string(rv_) + ",\"native\":true,\"counts\":{";
      bool first = true;
      for (auto& kv : counts_) {
        if (!first) o.push_back(',');
        first = false;
        json::append_quoted(&o, kv.first);
        o.append(":").append(std::to_string(kv.second));
      }
      size_t live = 0;
      for (auto& w : watchers_) live += w->closed ? 0 : 1;
      char mx[96];
      uint64_t busy = 0, mxi = 0, fl = 0, fln = 0;
      for (auto& lp : loops_) {
        busy += lp->busy_ns.load();
        mxi = std::max<uint64_t>(mxi, lp->max_iter_ns.load());
        fl += lp->flush_ns.load();
        fln += lp->flushes.load();
      }
      char lk[256];
      std::snprintf(lk, sizeof(lk),
                    "},\"lock\":{\"n\":%llu,\"wait_ms\":%.3f,\"max_wait_ms\":%.3f,\"hold_ms\":%.3f,\"max_hold_ms\":%.3f}",
                    (unsigned long long)lstats_.n.load(), lstats_.wait_ns.load() / 1e6, lstats_.max_wait_ns.load() / 1e6,
                    lstats_.hold_ns.load() / 1e6, lstats_.max_hold_ns.load() / 1e6);
      o.append(lk);
      std::snprintf(mx, sizeof(mx), ",\"max_iter_ms\":%.3f,\"busy_ms\":%.3f,\"loops\":%zu,\"route_ms\":{", mxi / 1e6,
                    busy / 1e6, loops_.size());
      o.append(mx);
      first = true;
      std::snprintf(mx, sizeof(mx), "\"watch-flush\":[%llu,%.3f]", (unsigned long long)fln, fl / 1e6);
      o.append(mx);
      first = false;
      for (auto& kv : route_time_) {
        if (!first) o.push_back(',');
        first = false;
        json::append_quoted(&o, kv.first);
        std::snprintf(mx, sizeof(mx), ":[%llu,%.3f]", (unsigned long long)kv.second.n, kv.second.s * 1e3);
        o.append(mx);
      }
      o.push_back('}');
      o.append(",\"watchers\":").append(std::to_string(live));
      for (auto& kv : store_) o.append(",\"" + kv.first + "\":" + std::to_string(kv.second.size()));
      o.push_back('}');
      rep->body = o;
      return true;
    }
    std::vector<std::string> seg = split(path, '/');  // "", "api", "v1", ...
    std::string kind, ns, name, sub;
    bool coll = false;
    if (seg.size() >= 4 && seg[1] == "api" && seg[2] == "v1") {
      if (seg[3] == "namespaces" && seg.size() >= 6) {
        ns = seg[4];
        kind = seg[5];
        if (seg.size() == 6) {
          coll = true;
        } else {
          name = seg[6];
          if (seg.size() == 8) sub = seg[7];
          if (seg.size() > 8) throw HttpError{404, status_body(404, "NotFound", "the server could not find the requested resource")};
        }
        if (kind == "bindings" && coll && m == "POST") {
          jd::Value b = take_body(body);
          maybe_error();
          const jd::Value* bmd = b.get("metadata");
          do_bind(ns, bmd ? bmd->str_or("name") : std::string(), b);
          rep->status = 201;
          rep->body = "{\"kind\":\"Status\",\"apiVersion\":\"v1\",\"metadata\":{},\"status\":\"Success\",\"code\":201}";
          return true;
        }
      } else if (seg.size() == 4) {
        kind = seg[3];
        coll = true;
      } else if (seg[3] == "nodes") {
        kind = "nodes";
        name = seg[4];
        if (seg.size() == 6) sub = seg[5];
      }
    } else if (seg.size() >= 7 && seg[1] == "apis" && seg[2] == "coordination.k8s.io" && seg[3] == "v1" &&
               seg[4] == "namespaces" && seg[6] == "leases") {
      ns = seg[5];
      kind = "leases";
      if (seg.size() == 7) {
        coll = true;
      } else {
        name = seg[7];
      }
    }
    if (!store_.count(kind) || (kind == "nodes" && !ns.empty())) {
      throw HttpError{404, status_body(404, "NotFound", "the server could not find the requested resource")};
    }
    if (coll) {
      if (m == "GET") {
        auto w = q.find("watch");
        if (w != q.end() && (w->second == "1" || w->second == "true")) return start_watch(L, c, req, kind, ns, q);
        int64_t limit = q.count("limit") ? std::atoll(q["limit"].c_str()) : 0;
        rep->body = list_json(kind, ns, q.count("fieldSelector") ? q["fieldSelector"] : "",
                              q.count("labelSelector") ? q["labelSelector"] : "", limit,
                              q.count("continue") ? q["continue"] : "");
        return true;
      }
      if (m == "POST") {
        jd::Value b = take_body(body);
        if (kind == "pods") maybe_error();
        rep->status = 201;
        rep->body = do_create(kind, std::move(b), ns)->json;
        return true;
      }
      if (m == "DELETE" && kind != "nodes") {
        double grace = grace_of(req, q);
        std::string fsel = q.count("fieldSelector") ? q["fieldSelector"] : "";
        std::string lsel = q.count("labelSelector") ? q["labelSelector"] : "";
        std::vector<std::string> names;
        Selector fs = Selector::parse(fsel, true), ls = Selector::parse(lsel, false);
        for (auto& kv : store_[kind]) {
          if (!ns.empty() && kv.second->ns != ns) continue;
          if (fs.matches(kv.second->v()) && ls.matches(kv.second->v())) names.push_back(kv.second->name);
        }
        std::string o = "{\"kind\":\"PodList\",\"apiVersion\":\"v1\",\"metadata\":{},\"items\":[";
        for (size_t i = 0; i < names.size(); ++i) {
          if (i) o.push_back(',');
          o.append(do_delete(kind, ns, names[i], grace)->json);
        }
        o.append("]}");
        rep->body = o;
        return true;
      }
      throw HttpError{405, status_body(405, "MethodNotAllowed", "method not allowed")};
    }
    if (sub == "binding" && kind == "pods" && m == "POST") {
      jd::Value b = take_body(body);
      maybe_error();
      do_bind(ns, name, b);
      rep->status = 201;
      rep->body = "{\"kind\":\"Status\",\"apiVersion\":\"v1\",\"metadata\":{},\"status\":\"Success\",\"code\":201}";
      return true;
    }
    if (!sub.empty() && sub != "status") {
      throw HttpError{404, status_body(404, "NotFound", "the server could not find the requested resource")};
    }
    if (m == "GET" && sub.empty()) {
      rep->body = get_obj(kind, ns, name)->json;
      return true;
    }
    if (m == "PUT") {
      jd::Value b = take_body(body);
      if (kind == "pods") maybe_error();
      rep->body = do_replace(kind, ns, name, std::move(b), sub)->json;
      return true;
    }
    if (m == "PATCH") {
      const std::string* ct = req.header("content-type");
      if (ct && ct->find("json-patch+json") != std::string::npos) {
        rep->status = 415;
        rep->body = status_body(415, "UnsupportedMediaType", "json-patch not supported");
        return true;
      }
      jd::Value b = take_body(body);
      if (kind == "pods") maybe_error();
      rep->body = do_patch(kind, ns, name, std::move(b), sub)->json;
      return true;
    }
    if (m == "DELETE" && sub.empty()) {
      std::string uid;
      double grace = grace_of(req, q, &uid);
      rep->body = do_delete(kind, ns, name, grace, uid)->json;
      return true;
    }
    throw HttpError{405, status_body(405, "MethodNotAllowed", "method not allowed")};
  }

  struct RouteTime {
    uint64_t n = 0;
    double s = 0;
  };

  size_t history_max_;
  std::map<std::string, RouteTime> route_time_;
  int nloops_;
  std::vector<std::unique_ptr<Loop>> loops_;
  LockStats lstats_;
  const bool flush_per_request_;  // --watch-flush request
  const bool watch_loop_;         // --watch-loop: loop 0 owns every watch stream
  std::mutex smu_;  // the state below: store, revision, history, watchers, faults, counters
  std::atomic<uint64_t> next_id_{0};
  std::vector<std::shared_ptr<Watcher>> watchers_;
  std::map<std::string, std::map<Key, ObjP>> store_;
  std::deque<Event> history_;
  int64_t rv_ = 0, oldest_rv_ = 0;
  Faults faults_;
  std::map<std::string, std::pair<std::string, std::string>> tokens_;  // TokenReview: token -> (user, node)
  std::map<std::string, uint64_t> counts_;
};

volatile sig_atomic_t g_stop = 0;
void on_sig(int) { g_stop = 1; }

}  // namespace

int main(int argc, char** argv) {
  std::string host = "127.0.0.1", port_file;
  int port = 0;
  size_t history = 200000;
  int threads = 1;
  bool flush_per_request = false, watch_loop = false;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto val = [&]() -> std::string {
      if (i + 1 >= argc) {
        std::fprintf(stderr, "missing value for %s\n", a.c_str());
        std::exit(2);
      }
      return argv[++i];
    };
    if (a == "--host") host = val();
    else if (a == "--port") port = std::atoi(val().c_str());
    else if (a == "--port-file") port_file = val();
    else if (a == "--history") history = static_cast<size_t>(std::max(1, std::atoi(val().c_str())));
    else if (a == "--threads") threads = std::atoi(val().c_str());
    else if (a == "--watch-loop") watch_loop = true;
    else if (a == "--watch-flush") {
      std::string m = val();
      if (m != "request" && m != "iteration") {
        std::fprintf(stderr, "--watch-flush: request | iteration\n");
        return 2;
      }
      flush_per_request = m == "request";
    } else if (a == "-h" || a == "--help") {
      std::printf("usage: gsx-fakeapi [--host H] [--port P] [--port-file F] [--history N] [--threads N]\n"
                  "                   [--watch-flush request|iteration] [--watch-loop]\n");
      return 0;
    } else {
      std::fprintf(stderr, "unknown argument %s\n", a.c_str());
      return 2;
    }
  }
  signal(SIGPIPE, SIG_IGN);
  struct sigaction sa;
  std::memset(&sa, 0, sizeof(sa));
  sa.sa_handler = on_sig;
  sigaction(SIGTERM, &sa, nullptr);
  sigaction(SIGINT, &sa, nullptr);
  Server srv(history, threads, flush_per_request, watch_loop);
  std::string err;
  int bound = srv.listen_on(host, port, &err);
  if (bound < 0) {
    std::fprintf(stderr, "gsx-fakeapi: %s\n", err.c_str());
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
  std::printf("fake-apiserver (native) listening on http://%s:%d\n", host.c_str(), bound);
  std::fflush(stdout);
  srv.run(&g_stop);
  return 0;
}
