// gRPC over HTTP/2 on libnghttp2 (see h2.h).  The library is dlopen'ed and its C ABI declared here (the
// image ships libnghttp2.so.14 but not its headers); only the frame header of nghttp2_frame is read.
#include "h2.h"

#include <dlfcn.h>
#include <fcntl.h>
#include <poll.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/un.h>
#include <time.h>
#include <unistd.h>

#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <mutex>

extern "C" {
typedef struct nghttp2_session nghttp2_session;
typedef struct nghttp2_session_callbacks nghttp2_session_callbacks;
typedef struct {
  uint8_t* name;
  uint8_t* value;
  size_t namelen;
  size_t valuelen;
  uint8_t flags;
} nghttp2_nv;
typedef struct {
  size_t length;
  int32_t stream_id;
  uint8_t type;
  uint8_t flags;
  uint8_t reserved;
} nghttp2_frame_hd;
typedef union {
  nghttp2_frame_hd hd;  // every frame type starts with it; nothing else is read here
} nghttp2_frame;
typedef union {
  int fd;
  void* ptr;
} nghttp2_data_source;
typedef ssize_t (*nghttp2_data_source_read_callback)(nghttp2_session*, int32_t, uint8_t*, size_t, uint32_t*,
                                                      nghttp2_data_source*, void*);
typedef struct {
  nghttp2_data_source source;
  nghttp2_data_source_read_callback read_callback;
} nghttp2_data_provider;
typedef struct {
  int32_t settings_id;
  uint32_t value;
} nghttp2_settings_entry;
typedef int (*nghttp2_on_begin_headers_callback)(nghttp2_session*, const nghttp2_frame*, void*);
typedef int (*nghttp2_on_header_callback)(nghttp2_session*, const nghttp2_frame*, const uint8_t*, size_t,
                                          const uint8_t*, size_t, uint8_t, void*);
typedef int (*nghttp2_on_data_chunk_recv_callback)(nghttp2_session*, uint8_t, int32_t, const uint8_t*, size_t,
                                                   void*);
typedef int (*nghttp2_on_frame_recv_callback)(nghttp2_session*, const nghttp2_frame*, void*);
typedef int (*nghttp2_on_stream_close_callback)(nghttp2_session*, int32_t, uint32_t, void*);
}

namespace gsx::h2 {
namespace {

constexpr uint8_t kData = 0x0, kHeaders = 0x1;
constexpr uint8_t kFlagEndStream = 0x01;
constexpr uint32_t kDataEof = 0x01, kDataNoEndStream = 0x02;
constexpr int kErrDeferred = -508;
constexpr int32_t kMaxConcurrentStreams = 0x3;
constexpr int32_t kInitialWindowSize = 0x4;
constexpr int32_t kMaxFrameSize = 0x5;
// Flow-control windows and frame size both ends announce: a GetPreferredAllocation of an 8-GPU node lists every
// free unit ID (~2,300 IDs, ~70 KB), past HTTP/2's default 64 KiB window -- the sender would stall for a
// WINDOW_UPDATE round trip on kubelet's serial admission path, and send five 16 KiB DATA frames
constexpr int32_t kWindow = 16 << 20;
constexpr int32_t kFrame = 1 << 20;
constexpr uint32_t kCancel = 0x8;

struct Lib {
  int (*callbacks_new)(nghttp2_session_callbacks**);
  void (*callbacks_del)(nghttp2_session_callbacks*);
  void (*set_on_begin_headers)(nghttp2_session_callbacks*, nghttp2_on_begin_headers_callback);
  void (*set_on_header)(nghttp2_session_callbacks*, nghttp2_on_header_callback);
  void (*set_on_data_chunk_recv)(nghttp2_session_callbacks*, nghttp2_on_data_chunk_recv_callback);
  void (*set_on_frame_recv)(nghttp2_session_callbacks*, nghttp2_on_frame_recv_callback);
  void (*set_on_stream_close)(nghttp2_session_callbacks*, nghttp2_on_stream_close_callback);
  int (*server_new)(nghttp2_session**, const nghttp2_session_callbacks*, void*);
  int (*client_new)(nghttp2_session**, const nghttp2_session_callbacks*, void*);
  void (*session_del)(nghttp2_session*);
  int (*submit_settings)(nghttp2_session*, uint8_t, const nghttp2_settings_entry*, size_t);
  int (*set_local_window_size)(nghttp2_session*, uint8_t, int32_t, int32_t) = nullptr;
  int (*submit_response)(nghttp2_session*, int32_t, const nghttp2_nv*, size_t, const nghttp2_data_provider*);
  int (*submit_trailer)(nghttp2_session*, int32_t, const nghttp2_nv*, size_t);
  int32_t (*submit_request)(nghttp2_session*, const void*, const nghttp2_nv*, size_t, const nghttp2_data_provider*,
                            void*);
  int (*submit_rst_stream)(nghttp2_session*, uint8_t, int32_t, uint32_t);
  int (*resume_data)(nghttp2_session*, int32_t);
  ssize_t (*mem_recv)(nghttp2_session*, const uint8_t*, size_t);
  ssize_t (*mem_send)(nghttp2_session*, const uint8_t**);
  int (*want_read)(nghttp2_session*);
  int (*want_write)(nghttp2_session*);
  const char* (*strerror)(int);
};

Lib g_lib;
bool g_loaded = false;
std::string g_load_err;
std::once_flag g_once;

template <typename F>
bool sym(void* h, const char* name, F* out) {
  *out = reinterpret_cast<F>(dlsym(h, name));
  if (!*out) g_load_err = std::string("libnghttp2 lacks ") + name;
  return *out != nullptr;
}

void load() {
  // GSX_NGHTTP2_LIB: the library to load instead (an image with another soname, or a test hiding it)
  const char* want = std::getenv("GSX_NGHTTP2_LIB");
  void* h = dlopen(want && *want ? want : "libnghttp2.so.14", RTLD_NOW | RTLD_LOCAL);
  if (!h && !(want && *want)) h = dlopen("libnghttp2.so", RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    g_load_err = std::string("dlopen libnghttp2: ") + dlerror();
    return;
  }
  Lib& l = g_lib;
  g_loaded = sym(h, "nghttp2_session_callbacks_new", &l.callbacks_new) &&
             sym(h, "nghttp2_session_callbacks_del", &l.callbacks_del) &&
             sym(h, "nghttp2_session_callbacks_set_on_begin_headers_callback", &l.set_on_begin_headers) &&
             sym(h, "nghttp2_session_callbacks_set_on_header_callback", &l.set_on_header) &&
             sym(h, "nghttp2_session_callbacks_set_on_data_chunk_recv_callback", &l.set_on_data_chunk_recv) &&
             sym(h, "nghttp2_session_callbacks_set_on_frame_recv_callback", &l.set_on_frame_recv) &&
             sym(h, "nghttp2_session_callbacks_set_on_stream_close_callback", &l.set_on_stream_close) &&
             sym(h, "nghttp2_session_server_new", &l.server_new) && sym(h, "nghttp2_session_client_new", &l.client_new) &&
             sym(h, "nghttp2_session_del", &l.session_del) && sym(h, "nghttp2_submit_settings", &l.submit_settings) &&
             sym(h, "nghttp2_submit_response", &l.submit_response) && sym(h, "nghttp2_submit_trailer", &l.submit_trailer) &&
             sym(h, "nghttp2_submit_request", &l.submit_request) &&
             sym(h, "nghttp2_submit_rst_stream", &l.submit_rst_stream) &&
             sym(h, "nghttp2_session_resume_data", &l.resume_data) && sym(h, "nghttp2_session_mem_recv", &l.mem_recv) &&
             sym(h, "nghttp2_session_mem_send", &l.mem_send) && sym(h, "nghttp2_session_want_read", &l.want_read) &&
             sym(h, "nghttp2_session_want_write", &l.want_write) && sym(h, "nghttp2_strerror", &l.strerror);
  if (g_loaded) sym(h, "nghttp2_session_set_local_window_size", &l.set_local_window_size);  // optional (1.7+)
}

// the settings above, on a new session (either end)
void big_windows(nghttp2_session* s, bool server) {
  nghttp2_settings_entry iv[3] = {{kInitialWindowSize, kWindow}, {kMaxFrameSize, kFrame}, {kMaxConcurrentStreams, 256}};
  g_lib.submit_settings(s, 0, iv, server ? 3 : 2);
  if (g_lib.set_local_window_size) g_lib.set_local_window_size(s, 0, 0, kWindow);  // the connection's window
}

nghttp2_nv nv(const std::string& n, const std::string& v) {
  return nghttp2_nv{reinterpret_cast<uint8_t*>(const_cast<char*>(n.data())),
                    reinterpret_cast<uint8_t*>(const_cast<char*>(v.data())), n.size(), v.size(), 0};
}

double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

bool set_nonblock(int fd) {
  int fl = fcntl(fd, F_GETFL, 0);
  return fl >= 0 && fcntl(fd, F_SETFL, fl | O_NONBLOCK) == 0;
}

sockaddr_un unix_addr(const std::string& path, bool* ok) {
  sockaddr_un a{};
  a.sun_family = AF_UNIX;
  *ok = path.size() < sizeof(a.sun_path);
  if (*ok) std::memcpy(a.sun_path, path.c_str(), path.size() + 1);
  return a;
}

}  // namespace

bool available(std::string* err) {
  std::call_once(g_once, load);
  if (!g_loaded && err) *err = g_load_err;
  return g_loaded;
}

std::string grpc_frame(const std::string& payload) {
  std::string out(5, '\0');
  uint32_t n = static_cast<uint32_t>(payload.size());
  out[1] = static_cast<char>(n >> 24);
  out[2] = static_cast<char>(n >> 16);
  out[3] = static_cast<char>(n >> 8);
  out[4] = static_cast<char>(n);
  out += payload;
  return out;
}

bool grpc_unframe(std::string* buf, std::vector<std::string>* out) {
  size_t off = 0;
  while (buf->size() - off >= 5) {
    const auto* p = reinterpret_cast<const uint8_t*>(buf->data() + off);
    if (p[0] != 0) return false;  // compressed: never negotiated here
    uint32_t n = (uint32_t(p[1]) << 24) | (uint32_t(p[2]) << 16) | (uint32_t(p[3]) << 8) | uint32_t(p[4]);
    if (buf->size() - off - 5 < n) break;
    out->emplace_back(buf->data() + off + 5, n);
    off += 5 + n;
  }
  buf->erase(0, off);
  return true;
}

// ====================================================================== server
struct Server::Stream {
  int32_t id = 0;
  uint64_t call = 0;
  std::string path, in;
  bool dispatched = false;
  bool headers_sent = false;  // response HEADERS submitted (with a data provider)
  std::string out;
  size_t out_off = 0;
  bool eof = false, trailers = false, deferred = false;
  int status = 0;
  std::string message;
};

struct Server::Conn {
  int fd = -1;
  nghttp2_session* s = nullptr;
  Server* srv = nullptr;
  std::map<int32_t, std::unique_ptr<Stream>> streams;
  std::string wbuf;
  bool want_out = false;
  bool dead = false;
};

struct Callbacks {
  static Server::Stream* stream(Server::Conn* c, int32_t id) {
    auto it = c->streams.find(id);
    return it == c->streams.end() ? nullptr : it->second.get();
  }
  static int begin_headers(nghttp2_session*, const nghttp2_frame* f, void* ud) {
    auto* c = static_cast<Server::Conn*>(ud);
    if (f->hd.type != kHeaders || stream(c, f->hd.stream_id)) return 0;  // trailers of a request: ignore
    auto s = std::make_unique<Server::Stream>();
    s->id = f->hd.stream_id;
    c->streams[s->id] = std::move(s);
    return 0;
  }
  static int header(nghttp2_session*, const nghttp2_frame* f, const uint8_t* n, size_t nl, const uint8_t* v, size_t vl,
                    uint8_t, void* ud) {
    auto* c = static_cast<Server::Conn*>(ud);
    Server::Stream* s = stream(c, f->hd.stream_id);
    if (s && nl == 5 && std::memcmp(n, ":path", 5) == 0) s->path.assign(reinterpret_cast<const char*>(v), vl);
    return 0;
  }
  static int data(nghttp2_session*, uint8_t, int32_t id, const uint8_t* d, size_t n, void* ud) {
    auto* c = static_cast<Server::Conn*>(ud);
    Server::Stream* s = stream(c, id);
    if (!s) return 0;
    if (s->in.empty() && n >= 5) {
      // the gRPC length prefix sizes the message: one allocation, not a doubling per chunk (kubelet's
      // GetPreferredAllocation lists every free ID of the node, ~60 KB on 8 GPUs)
      const uint32_t len = (static_cast<uint32_t>(d[1]) << 24) | (static_cast<uint32_t>(d[2]) << 16) |
                           (static_cast<uint32_t>(d[3]) << 8) | static_cast<uint32_t>(d[4]);
      if (len > n - 5 && len <= (64u << 20)) s->in.reserve(5 + static_cast<size_t>(len));
    }
    s->in.append(reinterpret_cast<const char*>(d), n);
    return 0;
  }
  static int frame(nghttp2_session*, const nghttp2_frame* f, void* ud) {
    auto* c = static_cast<Server::Conn*>(ud);
    if ((f->hd.type == kHeaders || f->hd.type == kData) && (f->hd.flags & kFlagEndStream)) {
      Server::Stream* s = stream(c, f->hd.stream_id);
      if (s && !s->dispatched) {
        s->dispatched = true;
        c->srv->ready_.push_back({c, s});
      }
    }
    return 0;
  }
  static int closed(nghttp2_session*, int32_t id, uint32_t, void* ud) {
    auto* c = static_cast<Server::Conn*>(ud);
    auto it = c->streams.find(id);
    if (it != c->streams.end()) {
      c->srv->calls_by_id_.erase(it->second->call);
      // a request still waiting in ready_ must not be dispatched after this
      for (auto& r : c->srv->ready_) {
        if (r.second == it->second.get()) r.second = nullptr;
      }
      c->streams.erase(it);
    }
    return 0;
  }
  static ssize_t read(nghttp2_session* sess, int32_t id, uint8_t* buf, size_t len, uint32_t* flags,
                      nghttp2_data_source* src, void* ud) {
    auto* c = static_cast<Server::Conn*>(ud);
    Server::Stream* s = stream(c, id);
    if (!s) {
      *flags |= kDataEof;
      return 0;
    }
    size_t left = s->out.size() - s->out_off;
    if (left > 0) {
      size_t n = left < len ? left : len;
      std::memcpy(buf, s->out.data() + s->out_off, n);
      s->out_off += n;
      if (s->out_off == s->out.size()) {
        s->out.clear();
        s->out_off = 0;
      }
      return static_cast<ssize_t>(n);
    }
    if (!s->eof) {
      s->deferred = true;
      return kErrDeferred;
    }
    *flags |= kDataEof;
    if (s->trailers) {
      *flags |= kDataNoEndStream;
      std::string st = std::to_string(s->status);
      std::vector<nghttp2_nv> tr;
      std::string k1 = "grpc-status", k2 = "grpc-message";
      tr.push_back(nv(k1, st));
      if (!s->message.empty()) tr.push_back(nv(k2, s->message));
      g_lib.submit_trailer(sess, id, tr.data(), tr.size());
    }
    return 0;
  }
};

Server::Server(const std::string& unix_path, Handler handler) : path_(unix_path), handler_(std::move(handler)) {
  if (!available(&err_)) return;
  bool fits;
  sockaddr_un a = unix_addr(path_, &fits);
  if (!fits) {
    err_ = "socket path too long";
    return;
  }
  ::unlink(path_.c_str());
  lfd_ = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC | SOCK_NONBLOCK, 0);
  if (lfd_ < 0 || ::bind(lfd_, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0 || ::listen(lfd_, 64) != 0) {
    err_ = std::string("listen ") + path_ + ": " + std::strerror(errno);
    return;
  }
  ep_ = ::epoll_create1(EPOLL_CLOEXEC);
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.fd = lfd_;
  if (ep_ < 0 || ::epoll_ctl(ep_, EPOLL_CTL_ADD, lfd_, &ev) != 0) {
    err_ = std::string("epoll: ") + std::strerror(errno);
    return;
  }
  ok_ = true;
}

Server::~Server() {
  while (!conns_.empty()) close_conn(conns_.begin()->first);
  if (ep_ >= 0) ::close(ep_);
  if (lfd_ >= 0) {
    ::close(lfd_);
    ::unlink(path_.c_str());
  }
}

void Server::accept_all() {
  for (;;) {
    int fd = ::accept4(lfd_, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
    if (fd < 0) return;
    auto c = std::make_unique<Conn>();
    c->fd = fd;
    c->srv = this;
    nghttp2_session_callbacks* cbs = nullptr;
    g_lib.callbacks_new(&cbs);
    g_lib.set_on_begin_headers(cbs, &Callbacks::begin_headers);
    g_lib.set_on_header(cbs, &Callbacks::header);
    g_lib.set_on_data_chunk_recv(cbs, &Callbacks::data);
    g_lib.set_on_frame_recv(cbs, &Callbacks::frame);
    g_lib.set_on_stream_close(cbs, &Callbacks::closed);
    int rv = g_lib.server_new(&c->s, cbs, c.get());
    g_lib.callbacks_del(cbs);
    if (rv != 0) {
      ::close(fd);
      continue;
    }
    big_windows(c->s, true);
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.fd = fd;
    ::epoll_ctl(ep_, EPOLL_CTL_ADD, fd, &ev);
    Conn* raw = c.get();
    conns_[fd] = std::move(c);
    conns_total_++;
    flush_conn(raw);
  }
}

bool Server::read_conn(Conn* c) {
  char buf[65536];
  for (;;) {
    ssize_t n = ::recv(c->fd, buf, sizeof buf, 0);
    if (n > 0) {
      ssize_t r = g_lib.mem_recv(c->s, reinterpret_cast<const uint8_t*>(buf), static_cast<size_t>(n));
      if (r < 0) return false;
      // a short read that completed a request drained the socket: no second recv just to meet EAGAIN (a syscall
      // per kubelet call; the epoll registration is level-triggered, so bytes that land meanwhile wake the owner
      // again).  A short read inside a request (a 25 KB GetPreferredAllocation arrives in several pieces while
      // the sender still copies it in) reads on.
      if (static_cast<size_t>(n) < sizeof buf && !ready_.empty()) return true;
      continue;
    }
    if (n == 0) return false;
    if (errno == EINTR) continue;
    return errno == EAGAIN || errno == EWOULDBLOCK;
  }
}

bool Server::flush_conn(Conn* c) {
  for (;;) {
    const uint8_t* data = nullptr;
    ssize_t n = g_lib.mem_send(c->s, &data);
    if (n < 0) return false;
    if (n == 0) break;
    c->wbuf.append(reinterpret_cast<const char*>(data), static_cast<size_t>(n));
  }
  while (!c->wbuf.empty()) {
    ssize_t n = ::send(c->fd, c->wbuf.data(), c->wbuf.size(), MSG_NOSIGNAL);
    if (n > 0) {
      c->wbuf.erase(0, static_cast<size_t>(n));
      continue;
    }
    if (n < 0 && errno == EINTR) continue;
    if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
    return false;
  }
  bool want = !c->wbuf.empty();
  if (want != c->want_out) {
    epoll_event ev{};
    ev.events = EPOLLIN | (want ? EPOLLOUT : 0);
    ev.data.fd = c->fd;
    ::epoll_ctl(ep_, EPOLL_CTL_MOD, c->fd, &ev);
    c->want_out = want;
  }
  return g_lib.want_read(c->s) || g_lib.want_write(c->s) || !c->wbuf.empty();
}

void Server::close_conn(int fd) {
  auto it = conns_.find(fd);
  if (it == conns_.end()) return;
  Conn* c = it->second.get();
  for (auto& kv : c->streams) calls_by_id_.erase(kv.second->call);
  for (auto& r : ready_) {
    if (r.first == c) r.second = nullptr;
  }
  ::epoll_ctl(ep_, EPOLL_CTL_DEL, fd, nullptr);
  g_lib.session_del(c->s);
  ::close(fd);
  conns_.erase(it);
}

void Server::dispatch(Conn* c, Stream* s) {
  s->call = next_call_++;
  calls_by_id_[s->call] = {c->fd, s->id};
  calls_++;
  std::vector<std::string> msgs;
  Call call;
  call.id = s->call;
  call.path = s->path;
  if (!grpc_unframe(&s->in, &msgs) || msgs.size() != 1) {
    respond(s->call, 13, "gsx: expected exactly one uncompressed request message");
    return;
  }
  call.message = std::move(msgs[0]);
  handler_(*this, call);
}

int Server::poll() {
  if (!ok_) return 0;
  epoll_event evs[64];
  int dispatched = 0;
  for (;;) {
    int n = ::epoll_wait(ep_, evs, 64, 0);
    if (n <= 0) break;
    std::vector<int> dead;
    for (int i = 0; i < n; ++i) {
      int fd = evs[i].data.fd;
      if (fd == lfd_) {
        accept_all();
        continue;
      }
      auto it = conns_.find(fd);
      if (it == conns_.end()) continue;
      Conn* c = it->second.get();
      bool alive = true;
      if (evs[i].events & (EPOLLIN | EPOLLHUP | EPOLLERR)) alive = read_conn(c);
      if (alive) {
        std::vector<std::pair<Conn*, Stream*>> ready;
        ready.swap(ready_);
        for (auto& r : ready) {
          if (r.second) {
            dispatch(r.first, r.second);
            dispatched++;
          }
        }
        auto still = conns_.find(fd);
        if (still == conns_.end()) continue;
        alive = flush_conn(c);
      }
      if (!alive) dead.push_back(fd);
    }
    for (int fd : dead) close_conn(fd);
    if (n < 64) break;
  }
  return dispatched;
}

void Server::watch_fd(int fd) {
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.fd = fd;
  ::epoll_ctl(ep_, EPOLL_CTL_ADD, fd, &ev);
}

Server::Stream* Server::find(uint64_t call, Conn** conn) {
  auto it = calls_by_id_.find(call);
  if (it == calls_by_id_.end()) return nullptr;
  auto c = conns_.find(it->second.first);
  if (c == conns_.end()) return nullptr;
  auto s = c->second->streams.find(it->second.second);
  if (s == c->second->streams.end()) return nullptr;
  *conn = c->second.get();
  return s->second.get();
}

void Server::submit(Conn* c, Stream* s) {
  if (!s->headers_sent) {
    s->headers_sent = true;
    std::string k1 = ":status", v1 = "200", k2 = "content-type", v2 = "application/grpc";
    nghttp2_nv hdr[2] = {nv(k1, v1), nv(k2, v2)};
    nghttp2_data_provider dp;
    dp.source.ptr = s;
    dp.read_callback = &Callbacks::read;
    g_lib.submit_response(c->s, s->id, hdr, 2, &dp);
  } else if (s->deferred) {
    s->deferred = false;
    g_lib.resume_data(c->s, s->id);
  }
  if (!flush_conn(c)) close_conn(c->fd);
}

bool Server::respond(uint64_t call, int status, const std::string& payload_or_message) {
  Conn* c = nullptr;
  Stream* s = find(call, &c);
  if (!s) return false;
  if (status != 0 && !s->headers_sent) {
    // trailers-only response
    s->headers_sent = true;
    std::string k1 = ":status", v1 = "200", k2 = "content-type", v2 = "application/grpc", k3 = "grpc-status",
                v3 = std::to_string(status), k4 = "grpc-message";
    std::string msg = payload_or_message;
    for (char& ch : msg) {
      if (ch == '\r' || ch == '\n') ch = ' ';
    }
    nghttp2_nv hdr[4] = {nv(k1, v1), nv(k2, v2), nv(k3, v3), nv(k4, msg)};
    g_lib.submit_response(c->s, s->id, hdr, msg.empty() ? 3 : 4, nullptr);
    if (!flush_conn(c)) close_conn(c->fd);
    return true;
  }
  if (status == 0) s->out += grpc_frame(payload_or_message);
  s->eof = true;
  s->trailers = true;
  s->status = status;
  if (status != 0) s->message = payload_or_message;
  submit(c, s);
  return true;
}

bool Server::stream_send(uint64_t call, const std::string& payload) {
  Conn* c = nullptr;
  Stream* s = find(call, &c);
  if (!s || s->eof) return false;
  s->out += grpc_frame(payload);
  submit(c, s);
  return true;
}

bool Server::stream_end(uint64_t call, int status, const std::string& message) {
  Conn* c = nullptr;
  Stream* s = find(call, &c);
  if (!s) return false;
  s->eof = true;
  s->trailers = true;
  s->status = status;
  s->message = message;
  submit(c, s);
  return true;
}

std::vector<uint64_t> Server::open_streams(const std::string& path) const {
  std::vector<uint64_t> out;
  for (const auto& kv : calls_by_id_) {
    auto c = conns_.find(kv.second.first);
    if (c == conns_.end()) continue;
    auto s = c->second->streams.find(kv.second.second);
    if (s != c->second->streams.end() && s->second->path == path && !s->second->eof) out.push_back(kv.first);
  }
  return out;
}

// ====================================================================== client
struct Client::Impl {
  std::string path;
  int fd = -1;
  nghttp2_session* s = nullptr;
  std::string wbuf;
  // the one call in flight
  int32_t sid = -1;
  std::string req_frame;
  size_t req_off = 0;
  std::string body;
  std::string grpc_status, grpc_message, http_status;
  bool closed = false;
  size_t want_msgs = 0;
  std::vector<std::string>* sink = nullptr;
  // GSX_H2_CLIENT_SPIN_US: poll without sleeping this long into a call before blocking for its answer (a caller
  // making serial calls, like kubelet's admission, then does not pay a sleep / wake-up per answer)
  double spin_s = [] {
    const char* v = std::getenv("GSX_H2_CLIENT_SPIN_US");
    return v ? std::atof(v) * 1e-6 : 0.0;
  }();

  ~Impl() { drop(); }
  void drop() {
    if (s) g_lib.session_del(s);
    s = nullptr;
    if (fd >= 0) ::close(fd);
    fd = -1;
  }

  static int on_header(nghttp2_session*, const nghttp2_frame* f, const uint8_t* n, size_t nl, const uint8_t* v,
                       size_t vl, uint8_t, void* ud) {
    auto* c = static_cast<Impl*>(ud);
    if (f->hd.stream_id != c->sid) return 0;
    std::string name(reinterpret_cast<const char*>(n), nl), val(reinterpret_cast<const char*>(v), vl);
    if (name == "grpc-status") c->grpc_status = val;
    else if (name == "grpc-message") c->grpc_message = val;
    else if (name == ":status") c->http_status = val;
    return 0;
  }
  static int on_data(nghttp2_session*, uint8_t, int32_t id, const uint8_t* d, size_t n, void* ud) {
    auto* c = static_cast<Impl*>(ud);
    if (id == c->sid) c->body.append(reinterpret_cast<const char*>(d), n);
    return 0;
  }
  static int on_close(nghttp2_session*, int32_t id, uint32_t, void* ud) {
    auto* c = static_cast<Impl*>(ud);
    if (id == c->sid) c->closed = true;
    return 0;
  }
  static ssize_t read_req(nghttp2_session*, int32_t, uint8_t* buf, size_t len, uint32_t* flags, nghttp2_data_source*,
                          void* ud) {
    auto* c = static_cast<Impl*>(ud);
    size_t left = c->req_frame.size() - c->req_off;
    size_t n = left < len ? left : len;
    std::memcpy(buf, c->req_frame.data() + c->req_off, n);
    c->req_off += n;
    if (c->req_off == c->req_frame.size()) *flags |= kDataEof;
    return static_cast<ssize_t>(n);
  }

  bool connect(std::string* err) {
    if (s) return true;
    bool fits;
    sockaddr_un a = unix_addr(path, &fits);
    if (!fits) {
      *err = "socket path too long";
      return false;
    }
    fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (fd < 0 || ::connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0) {
      *err = std::string("connect ") + path + ": " + std::strerror(errno);
      drop();
      return false;
    }
    set_nonblock(fd);
    nghttp2_session_callbacks* cbs = nullptr;
    g_lib.callbacks_new(&cbs);
    g_lib.set_on_header(cbs, &Impl::on_header);
    g_lib.set_on_data_chunk_recv(cbs, &Impl::on_data);
    g_lib.set_on_stream_close(cbs, &Impl::on_close);
    int rv = g_lib.client_new(&s, cbs, this);
    g_lib.callbacks_del(cbs);
    if (rv != 0) {
      *err = "nghttp2_session_client_new failed";
      drop();
      return false;
    }
    big_windows(s, false);
    return true;
  }

  // drive the session until pred() or the deadline; false on transport failure / timeout (*err)
  template <typename Pred>
  bool run(Pred pred, double deadline, std::string* err) {
    char buf[65536];
    const double spin_until = spin_s > 0 ? now_s() + spin_s : 0;
    for (;;) {
      for (;;) {
        const uint8_t* data = nullptr;
        ssize_t n = g_lib.mem_send(s, &data);
        if (n < 0) {
          *err = g_lib.strerror(static_cast<int>(n));
          return false;
        }
        if (n == 0) break;
        wbuf.append(reinterpret_cast<const char*>(data), static_cast<size_t>(n));
      }
      while (!wbuf.empty()) {
        ssize_t n = ::send(fd, wbuf.data(), wbuf.size(), MSG_NOSIGNAL);
        if (n > 0) {
          wbuf.erase(0, static_cast<size_t>(n));
        } else if (n < 0 && errno == EINTR) {
          continue;
        } else if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
          break;
        } else {
          *err = std::string("send: ") + std::strerror(errno);
          return false;
        }
      }
      if (pred()) return true;
      double left = deadline - now_s();
      if (left <= 0) {
        *err = "deadline exceeded";
        return false;
      }
      pollfd p{fd, static_cast<short>(POLLIN | (wbuf.empty() ? 0 : POLLOUT)), 0};
      const bool spinning = spin_until > 0 && now_s() < spin_until;
      int r = ::poll(&p, 1, spinning ? 0 : static_cast<int>(left * 1000) + 1);
      if (r == 0 && spinning) continue;
      if (r < 0 && errno != EINTR) {
        *err = std::string("poll: ") + std::strerror(errno);
        return false;
      }
      if (r > 0 && (p.revents & (POLLIN | POLLHUP | POLLERR))) {
        ssize_t n = ::recv(fd, buf, sizeof buf, 0);
        if (n == 0) {
          *err = "connection closed";
          return false;
        }
        if (n < 0 && errno != EAGAIN && errno != EINTR) {
          *err = std::string("recv: ") + std::strerror(errno);
          return false;
        }
        if (n > 0 && g_lib.mem_recv(s, reinterpret_cast<const uint8_t*>(buf), static_cast<size_t>(n)) < 0) {
          *err = "malformed HTTP/2 from the server";
          return false;
        }
      }
    }
  }

  bool start(const std::string& rpc, const std::string& req, std::string* err) {
    if (!connect(err)) return false;
    body.clear();
    grpc_status.clear();
    grpc_message.clear();
    http_status.clear();
    closed = false;
    req_frame = grpc_frame(req);
    req_off = 0;
    std::string k[6] = {":method", ":scheme", ":path", ":authority", "content-type", "te"};
    std::string v[6] = {"POST", "http", rpc, "localhost", "application/grpc", "trailers"};
    nghttp2_nv hdr[6];
    for (int i = 0; i < 6; ++i) hdr[i] = nv(k[i], v[i]);
    nghttp2_data_provider dp;
    dp.source.ptr = nullptr;
    dp.read_callback = &Impl::read_req;
    sid = g_lib.submit_request(s, nullptr, hdr, 6, &dp, nullptr);
    if (sid < 0) {
      *err = g_lib.strerror(sid);
      drop();
      return false;
    }
    return true;
  }
};

Client::Client(const std::string& unix_path) : impl_(std::make_unique<Impl>()) { impl_->path = unix_path; }
Client::~Client() = default;

bool Client::call(const std::string& path, const std::string& req, std::string* resp, int* status, std::string* err,
                  double timeout_s) {
  *status = -1;
  if (!available(err)) return false;
  Impl& c = *impl_;
  if (!c.start(path, req, err)) return false;
  if (!c.run([&] { return c.closed; }, now_s() + timeout_s, err)) {
    c.drop();
    return false;
  }
  *status = c.grpc_status.empty() ? 2 : std::atoi(c.grpc_status.c_str());
  if (*status != 0) {
    *err = c.grpc_message.empty() ? "grpc-status " + c.grpc_status : c.grpc_message;
    return false;
  }
  std::vector<std::string> msgs;
  if (!grpc_unframe(&c.body, &msgs) || msgs.size() != 1) {
    *err = "expected one response message";
    *status = 13;
    return false;
  }
  *resp = std::move(msgs[0]);
  return true;
}

bool Client::stream(const std::string& path, const std::string& req, size_t max_messages,
                    std::vector<std::string>* out, int* status, std::string* err, double timeout_s) {
  *status = -1;
  if (!available(err)) return false;
  Impl& c = *impl_;
  if (!c.start(path, req, err)) return false;
  std::vector<std::string> msgs;
  bool ok = c.run(
      [&] {
        grpc_unframe(&c.body, &msgs);
        return c.closed || msgs.size() >= max_messages;
      },
      now_s() + timeout_s, err);
  if (!ok) {
    c.drop();
    return false;
  }
  for (auto& m : msgs) out->push_back(std::move(m));
  if (!c.closed) {
    g_lib.submit_rst_stream(c.s, 0, c.sid, kCancel);
    std::string e2;
    c.run([] { return true; }, now_s() + 1.0, &e2);
    *status = 0;
    return true;
  }
  *status = c.grpc_status.empty() ? 0 : std::atoi(c.grpc_status.c_str());
  if (*status != 0) *err = c.grpc_message;
  return *status == 0;
}

}  // namespace gsx::h2
