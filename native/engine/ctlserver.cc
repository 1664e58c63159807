#include "ctlserver.h"
#include "introspect.h"

#include <arpa/inet.h>
#include <pthread.h>
#include <sched.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstring>

namespace gsx {

void CtlServer::pin_thread() const {
  if (cpus_.empty()) return;
  cpu_set_t set;
  CPU_ZERO(&set);
  for (int c : cpus_) {
    if (c >= 0 && c < CPU_SETSIZE) CPU_SET(c, &set);
  }
  pthread_setaffinity_np(pthread_self(), sizeof(set), &set);  // best effort: a CPU outside the cgroup is ignored
}

int CtlServer::start(const std::string& host, int port, std::string* err) {
  lfd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (lfd_ < 0) {
    *err = std::string("socket: ") + std::strerror(errno);
    return -1;
  }
  int one = 1;
  setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a;
  std::memset(&a, 0, sizeof(a));
  a.sin_family = AF_INET;
  a.sin_port = htons(static_cast<uint16_t>(port));
  if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1) {
    *err = "bad listen address " + host;
    return -1;
  }
  if (::bind(lfd_, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || ::listen(lfd_, 64) != 0) {
    *err = std::string("bind/listen: ") + std::strerror(errno);
    ::close(lfd_);
    lfd_ = -1;
    return -1;
  }
  socklen_t len = sizeof(a);
  getsockname(lfd_, reinterpret_cast<sockaddr*>(&a), &len);
  acc_ = std::thread([this] {
    introspect::name_thread("ctl-accept");
    pin_thread();
    accept_loop();
  });
  return ntohs(a.sin_port);
}

void CtlServer::stop() {
  if (stop_.exchange(true)) return;
  if (lfd_ >= 0) ::shutdown(lfd_, SHUT_RDWR);
  if (acc_.joinable()) acc_.join();
  if (lfd_ >= 0) ::close(lfd_);
  lfd_ = -1;
  std::map<uint64_t, std::thread> ts;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (int fd : conns_) ::shutdown(fd, SHUT_RDWR);
    ts.swap(threads_);
    finished_.clear();
  }
  for (auto& kv : ts) kv.second.join();
}

void CtlServer::accept_loop() {
  while (!stop_.load()) {
    int fd = ::accept4(lfd_, nullptr, nullptr, SOCK_CLOEXEC);
    if (fd < 0) {
      if (errno == EINTR) continue;
      return;
    }
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    std::vector<std::thread> done;
    {
      std::lock_guard<std::mutex> g(mu_);
      if (stop_.load()) {
        ::close(fd);
        return;
      }
      // reap the threads of closed connections (a joinable thread keeps its stack until it is joined)
      for (uint64_t id : finished_) {
        auto it = threads_.find(id);
        if (it == threads_.end()) continue;
        done.push_back(std::move(it->second));
        threads_.erase(it);
      }
      finished_.clear();
      conns_.push_back(fd);
      const uint64_t id = next_conn_++;
      threads_.emplace(id, std::thread([this, fd, id] {
        introspect::name_thread("ctl-conn");
        pin_thread();
        serve_conn(fd);
        std::lock_guard<std::mutex> g2(mu_);
        finished_.push_back(id);
      }));
    }
    for (auto& t : done) t.join();  // returned or about to: outside the lock their epilogue needs
  }
}

void CtlServer::serve_conn(int fd) {
  std::string buf;
  char tmp[16384];
  bool open = true;
  http::MessageParser parser;
  while (open && !stop_.load()) {
    http::Message req;
    std::string perr;
    long got = parser.parse(buf.data(), buf.size(), &req, &perr, 64u << 20);
    if (got < 0) break;
    if (got == 0) {
      long r = ::recv(fd, tmp, sizeof(tmp), 0);
      if (r <= 0) {
        if (r < 0 && errno == EINTR) continue;
        break;
      }
      buf.append(tmp, static_cast<size_t>(r));
      continue;
    }
    buf.erase(0, static_cast<size_t>(got));
    Reply rep;
    try {
      rep = h_(req);
    } catch (const std::exception& e) {  // a connection thread has no handler above it: answer, do not terminate
      std::fprintf(stderr, "[gsx-ctl] request failed: %s\n", e.what());
      rep.status = 500;
      rep.body = "{\"error\":\"internal error\"}";
    }
    std::string out = http::response(rep.status, rep.content_type, rep.body, req.keep_alive);
    size_t off = 0;
    while (off < out.size()) {
      long w = ::send(fd, out.data() + off, out.size() - off, MSG_NOSIGNAL);
      if (w < 0) {
        if (errno == EINTR) continue;
        open = false;
        break;
      }
      off += static_cast<size_t>(w);
    }
    if (!req.keep_alive) break;
  }
  std::lock_guard<std::mutex> g(mu_);
  conns_.erase(std::remove(conns_.begin(), conns_.end(), fd), conns_.end());
  ::close(fd);
}

}  // namespace gsx
