// Local microbenchmark of the h2 transport (native/engine/h2.cc): a polling server thread answering 300 B, one client
// making serial unary calls, against a raw unix-socket ping-pong.  Build after `python native/build.py nodeagent`:
//   g++ -O3 -std=c++17 -Inative/engine scripts/experiments/h2bench.cc build/obj/tool_h2.o -o /tmp/h2bench -lpthread -ldl
//   GSX_H2_CLIENT_SPIN_US=1000 /tmp/h2bench 40 30000   (request bytes, calls)
#include "h2.h"
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <sched.h>
#include <unistd.h>
#include <sys/socket.h>
#include <sys/un.h>
using namespace gsx;
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
static void pin(int c) { cpu_set_t s; CPU_ZERO(&s); CPU_SET(c, &s); sched_setaffinity(0, sizeof s, &s); }
int main(int argc, char** argv) {
  int reqsz = argc > 1 ? atoi(argv[1]) : 40;
  int n = argc > 2 ? atoi(argv[2]) : 20000;
  std::string path = "/tmp/h2bench.sock";
  std::string resp(300, 'r');
  std::atomic<bool> stop{false};
  h2::Server srv(path, [&](h2::Server& s, const h2::Call& c) { s.respond(c.id, 0, resp); });
  if (!srv.ok()) { printf("srv: %s\n", srv.init_error().c_str()); return 1; }
  std::thread t([&] { pin(2); while (!stop.load(std::memory_order_relaxed)) srv.poll(); });
  pin(4);
  h2::Client cl(path);
  std::string req(reqsz, 'q'), out, err; int st;
  for (int i = 0; i < 1000; ++i) cl.call("/v1beta1.DevicePlugin/Allocate", req, &out, &st, &err);
  double t0 = now();
  for (int i = 0; i < n; ++i) if (!cl.call("/v1beta1.DevicePlugin/Allocate", req, &out, &st, &err)) { printf("err %s\n", err.c_str()); break; }
  double dt = now() - t0;
  printf("h2 req=%d rtt_us=%.2f\n", reqsz, dt / n * 1e6);
  stop = true; t.join();
  // raw ping-pong over a socketpair with the server spinning on nonblocking recv
  int sv[2]; socketpair(AF_UNIX, SOCK_STREAM, 0, sv);
  std::thread e([&] { pin(2); char b[65536]; for (int i = 0; i < n + 1000; ++i) { size_t got = 0; while (got < (size_t)reqsz) { ssize_t k = recv(sv[1], b, sizeof b, MSG_DONTWAIT); if (k > 0) got += k; } send(sv[1], resp.data(), resp.size(), 0); } });
  char b[65536];
  auto pp = [&] { send(sv[0], req.data(), req.size(), 0); size_t got = 0; while (got < resp.size()) { ssize_t k = recv(sv[0], b, sizeof b, MSG_DONTWAIT); if (k > 0) got += k; } };
  for (int i = 0; i < 1000; ++i) pp();
  t0 = now();
  for (int i = 0; i < n; ++i) pp();
  printf("raw req=%d rtt_us=%.2f\n", reqsz, (now() - t0) / n * 1e6);
  e.join();
}
