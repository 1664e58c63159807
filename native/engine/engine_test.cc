// Host-side unit + stress test of the native engine, built with sanitizers:
//   ASan+UBSan: python native/build.py asan   -> build/engine_test_asan
//   TSan:       python native/build.py tsan   -> build/engine_test_tsan
// (the reference had no race detection at all; its cache had
// two data races.)  The stress part runs the epoll front end with 8 client
// threads doing filter + bind against a tiny in-process "apiserver".
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cassert>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <memory>
#include <vector>

#include "allocstate.h"
#include "dpproto.h"
#include "http.h"
#include "json.h"
#include "ledger.h"
#include "model.h"
#include "quantity.h"
#include "server.h"
#include "tracker.h"

using namespace gsx;

static int g_fail = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                    \
    }                                                              \
  } while (0)

static void test_json() {
  json::Doc d;
  std::string err;
  CHECK(d.parse(R"({"Pod":{"metadata":{"name":"a\u00e9","uid":"u1"}},"nodenames":["n1","n2"]})", &err));
  CHECK(d.find(0, "pod", true) >= 0);
  CHECK(d.find(0, "pod", false) < 0);
  int64_t nn = d.find(0, "NodeNames", true);
  CHECK(nn >= 0 && d.at(static_cast<uint32_t>(nn)).count == 2);
  int64_t nm = d.path(static_cast<uint32_t>(d.find(0, "Pod")), {"metadata", "name"});
  CHECK(nm >= 0 && d.str(static_cast<uint32_t>(nm)) == "a\xc3\xa9");
  json::Doc bad;
  CHECK(!bad.parse("{\"a\":", &err) && err == "unexpected end of JSON input");
  CHECK(!bad.parse("[1,]", &err));
  std::string q;
  json::append_quoted(&q, "<&>\"\n");
  CHECK(q == "\"\\u003c\\u0026\\u003e\\\"\\n\"");
}

static void test_quantity() {
  int64_t v;
  CHECK(parse_quantity("64Gi", &v) && v == (int64_t(64) << 30));
  CHECK(parse_quantity("1.5", &v) && v == 2);
  CHECK(parse_quantity("500m", &v) && v == 1);
  CHECK(parse_quantity("1e3", &v) && v == 1000);
  CHECK(!parse_quantity("1Kib", &v));
  CHECK(parse_atoi("-12", &v) && v == -12);
  CHECK(!parse_atoi(" 1", &v));
}

static std::string pod_json(const std::string& name, const std::string& uid, int mem) {
  return "{\"metadata\":{\"name\":\"" + name + "\",\"namespace\":\"default\",\"uid\":\"" + uid +
         "\"},\"spec\":{\"containers\":[{\"name\":\"c\",\"resources\":{\"limits\":{\"shared-gpu/gpu-mem\":\"" +
         std::to_string(mem) + "\"}}}]},\"status\":{\"phase\":\"Pending\"}}";
}

static void test_ledger() {
  Ledger l{Profile()};
  NodeView nv;
  nv.name = "n";
  nv.total = 4 * 16276;
  nv.count = 4;
  l.upsert_node(nv);
  // design doc bind example: free {12207, 8138, 4069, 16276}, request 8138 -> GPU1
  const int64_t used[3] = {16276 - 12207, 16276 - 8138, 16276 - 4069};
  for (int i = 0; i < 3; ++i) {
    PodView v;
    v.uid = "x" + std::to_string(i);
    v.name = v.uid;
    v.ns = "default";
    v.node = "n";
    v.dev_idx = i;
    v.annot_mem = used[i];
    v.phase = "Running";
    CHECK(l.upsert_pod(v) == 1);
  }
  int64_t total = 0;
  CHECK(l.assume("u", "default", "p", "n", 8138, &total) == 1 && total == 16276);
  CHECK(l.assume("u", "default", "p", "n", 8138, &total) == -4);  // in flight
  l.finish_bind("u", false, 0);
  CHECK(l.node_devices("n")[1].second == 8138);
  CHECK(l.check("n", 16276) == Check::Ok);
  CHECK(l.check("n", 16277) == Check::Insufficient);
  CHECK(l.check("zz", 1) == Check::NodeNotFound);
  std::string body = "{\"Pod\":" + pod_json("q", "uq", 16276) + ",\"NodeNames\":[\"n\",\"zz\"]}";
  std::string out = filter_body(l, body);
  CHECK(out.find("\"NodeNames\":[\"n\"]") != std::string::npos);
  CHECK(out.find("\"zz\":\"node \\\"zz\\\" not found\"") != std::string::npos);
  Ledger::PendingPod pp;
  CHECK(l.pending("uq", &pp) && pp.req == 16276 && pp.name == "q");
  // 200k pods filtered then bound: the eviction-order queue stays proportional to the live records
  for (int i = 0; i < 200000; ++i) {
    std::string u = "soak-" + std::to_string(i);
    l.remember_pending(u, pp);
    l.forget_pending(u);
  }
  CHECK(l.pending_count() == 1 && l.pending_queue_len() <= 2 * l.pending_count() + 1024 + 1);
  CHECK(l.pending("uq", &pp));
}

static void test_http() {
  http::Message m;
  std::string err;
  std::string two = "POST /a?x=1 HTTP/1.1\r\nHost: h\r\nContent-Length: 3\r\n\r\nabcGET /b HTTP/1.1\r\n\r\n";
  long n = http::parse(two.data(), two.size(), true, &m, &err);
  CHECK(n > 0 && m.method == "POST" && m.path() == "/a" && m.body == "abc" && m.keep_alive);
  long n2 = http::parse(two.data() + n, two.size() - static_cast<size_t>(n), true, &m, &err);
  CHECK(n2 > 0 && m.method == "GET" && m.body.empty());
  std::string ch = "HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n3\r\nabc\r\n2\r\nde\r\n0\r\n\r\n";
  CHECK(http::parse(ch.data(), ch.size() - 3, false, &m, &err) == 0);  // incomplete
  CHECK(http::parse(ch.data(), ch.size(), false, &m, &err) == static_cast<long>(ch.size()) && m.body == "abcde");
  std::string close = "HTTP/1.0 200 OK\r\n\r\nxyz";
  CHECK(http::parse(close.data(), close.size(), false, &m, &err) == 0);
  CHECK(http::parse(close.data(), close.size(), false, &m, &err, true) > 0 && m.body == "xyz" && !m.keep_alive);
  // hostile chunk sizes: a size that would wrap body.size() + sz, a signed size, garbage
  const char* hostile[] = {"5\r\nhello\r\nfffffffffffffffb\r\n", "5\r\nhello\r\n-1\r\n", "0x5\r\nhello\r\n0\r\n\r\n",
                           "ffffffffffffffffff\r\n", "\r\n", "4 4\r\nabcd\r\n0\r\n\r\n"};
  for (const char* b : hostile) {
    std::string req = std::string("POST /f HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n") + b;
    CHECK(http::parse(req.data(), req.size(), true, &m, &err, false, 1 << 20) == -1);
  }
  std::string big = "POST /f HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n5\r\nhello\r\n100000\r\n";
  CHECK(http::parse(big.data(), big.size(), true, &m, &err, false, 1 << 20) == -1 && err == "body too large");
  std::string okc = "POST /f HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n5;ext=1\r\nhello\r\nA\r\n0123456789\r\n0\r\n\r\n";
  CHECK(http::parse(okc.data(), okc.size(), true, &m, &err, false, 1 << 20) == static_cast<long>(okc.size()) &&
        m.body == "hello0123456789");
  size_t sz = 0;
  CHECK(!http::parse_chunk_size("fffffffffffffffb", size_t(-1) / 2, &sz));
  CHECK(http::parse_chunk_size("7fffffffffffffff", size_t(-1) / 2, &sz) && sz == size_t(-1) / 2);
  CHECK(!http::parse_chunk_size("+5", 100, &sz) && !http::parse_chunk_size("", 100, &sz));
  http::Dechunker dc;
  CHECK(dc.feed("-1\r\n", 4, [](std::string_view) {}) == -1);
  http::Url u;
  CHECK(http::parse_url("https://[::1]:6443/pre/", &u) && u.tls && u.host == "::1" && u.port == 6443 &&
        u.prefix == "/pre");
}

// The connection parser must agree with the one-shot parser however the bytes are split across reads.
static void test_request_parser() {
  const std::string reqs[] = {
      "POST /a?x=1 HTTP/1.1\r\nHost: h\r\nContent-Length: 3\r\n\r\nabc",
      "GET /b HTTP/1.1\r\nConnection: close\r\n\r\n",
      "POST /f HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n5;ext=1\r\nhello\r\nA\r\n0123456789\r\n0\r\nX-T: 1\r\n\r\n",
      "POST /g HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n1\r\na\r\n1\r\nb\r\n1\r\nc\r\n0\r\n\r\n",
  };
  std::string stream;
  for (const auto& r : reqs) stream += r;
  for (size_t step : {size_t(1), size_t(2), size_t(3), size_t(7), size_t(64), stream.size()}) {
    http::MessageParser rp;
    std::string in;
    std::vector<http::Message> got;
    for (size_t off = 0; off < stream.size(); off += step) {
      in.append(stream, off, step);
      while (!in.empty()) {
        http::Message m;
        std::string err;
        long used = rp.parse(in.data(), in.size(), &m, &err, 1 << 20);
        CHECK(used >= 0);
        if (used <= 0) break;
        in.erase(0, static_cast<size_t>(used));
        got.push_back(std::move(m));
      }
    }
    CHECK(in.empty() && got.size() == 4);
    if (got.size() != 4) continue;
    for (size_t i = 0; i < 4; ++i) {
      http::Message ref;
      std::string err;
      CHECK(http::parse(reqs[i].data(), reqs[i].size(), true, &ref, &err, false, 1 << 20) ==
            static_cast<long>(reqs[i].size()));
      CHECK(got[i].method == ref.method && got[i].target == ref.target && got[i].body == ref.body &&
            got[i].keep_alive == ref.keep_alive && got[i].headers == ref.headers);
    }
  }
  // responses (the apiserver client): chunked, 204 without a body, and a body delimited by the close
  {
    const std::string ch = "HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n3\r\nabc\r\n2\r\nde\r\n0\r\n\r\n";
    const std::string nc = "HTTP/1.1 204 No Content\r\n\r\n";
    for (size_t k = 1; k <= ch.size(); ++k) {
      http::MessageParser rp(false);
      http::Message m;
      std::string err;
      long r = rp.parse(ch.data(), k, &m, &err);
      if (k < ch.size()) CHECK(r == 0);
      if (k == ch.size()) CHECK(r == static_cast<long>(k) && m.status == 200 && m.body == "abcde");
      if (k < ch.size()) {  // the rest arrives: the parser resumes from its state
        r = rp.parse(ch.data(), ch.size(), &m, &err);
        CHECK(r == static_cast<long>(ch.size()) && m.body == "abcde");
      }
    }
    http::MessageParser rp(false);
    http::Message m;
    std::string err;
    CHECK(rp.parse(nc.data(), nc.size(), &m, &err) == static_cast<long>(nc.size()) && m.status == 204);
    const std::string cl = "HTTP/1.0 200 OK\r\n\r\nxyz";
    CHECK(rp.parse(cl.data(), cl.size(), &m, &err) == 0);
    CHECK(rp.parse(cl.data(), cl.size(), &m, &err, 64u << 20, true) == static_cast<long>(cl.size()) &&
          m.body == "xyz" && m.body_until_close && !m.keep_alive);
  }
  // the same hostile framing is refused, also when it arrives one byte at a time
  const char* hostile[] = {"5\r\nhello\r\nfffffffffffffffb\r\n", "5\r\nhello\r\n-1\r\n", "0x5\r\nhello\r\n0\r\n\r\n",
                           "5\r\nhello\r\n100000\r\n"};
  for (const char* b : hostile) {
    std::string req = std::string("POST /f HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n") + b;
    http::MessageParser rp;
    long r = 0;
    http::Message m;
    std::string err;
    for (size_t k = 1; k <= req.size() && r == 0; ++k) r = rp.parse(req.data(), k, &m, &err, 1 << 20);
    CHECK(r == -1);
  }
  // a head or a chunk-size line that never ends is cut off at 64 KiB instead of being re-scanned forever
  {
    http::MessageParser rp;
    http::Message m;
    std::string err;
    std::string head = "GET / HTTP/1.1\r\nX: " + std::string(70000, 'a');
    CHECK(rp.parse(head.data(), 1000, &m, &err, 1 << 20) == 0);
    CHECK(rp.parse(head.data(), head.size(), &m, &err, 1 << 20) == -1 && err == "header too large");
    std::string sl = "POST /f HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n" + std::string(70000, '0');
    http::MessageParser rp2;
    CHECK(rp2.parse(sl.data(), sl.size(), &m, &err, 1 << 20) == -1);
  }
  // 100k one-byte chunks trickled in 16-byte reads: linear work (this loop would be ~10^10 byte scans if every
  // read re-parsed the buffer from the start)
  {
    std::string big = "POST /t HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n";
    for (int i = 0; i < 100000; ++i) big += "1\r\nz\r\n";
    big += "0\r\n\r\n";
    http::MessageParser rp;
    http::Message m;
    std::string err;
    long r = 0;
    for (size_t k = 16;; k += 16) {
      k = std::min(k, big.size());
      r = rp.parse(big.data(), k, &m, &err, 1 << 20);
      if (r != 0 || k == big.size()) break;
    }
    CHECK(r == static_cast<long>(big.size()) && m.body == std::string(100000, 'z'));
  }
}

// ---------------------------------------------------------------- stress

static int listen_any(int* port) {
  int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a;
  std::memset(&a, 0, sizeof(a));
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  ::bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a));
  ::listen(fd, 128);
  socklen_t sl = sizeof(a);
  getsockname(fd, reinterpret_cast<sockaddr*>(&a), &sl);
  *port = ntohs(a.sin_port);
  return fd;
}

// minimal "kube-apiserver": answers every request with 201 Created, keep-alive
static void fake_apiserver(int lfd, std::atomic<bool>* stop, std::atomic<int>* bindings) {
  std::vector<std::thread> conns;
  while (!stop->load()) {
    int c = ::accept(lfd, nullptr, nullptr);
    if (c < 0) break;
    conns.emplace_back([c, bindings] {
      std::string buf;
      char tmp[8192];
      while (true) {
        http::Message m;
        std::string err;
        long n = http::parse(buf.data(), buf.size(), true, &m, &err);
        if (n > 0) {
          buf.erase(0, static_cast<size_t>(n));
          if (m.path().find("/binding") != std::string_view::npos) bindings->fetch_add(1);
          std::string r = http::response(201, "application/json", "{\"kind\":\"Status\",\"code\":201}", true);
          if (::send(c, r.data(), r.size(), MSG_NOSIGNAL) < 0) break;
          continue;
        }
        if (n < 0) break;
        ssize_t got = ::recv(c, tmp, sizeof(tmp), 0);
        if (got <= 0) break;
        buf.append(tmp, static_cast<size_t>(got));
      }
      ::close(c);
    });
  }
  for (auto& t : conns) t.join();
}

static std::string roundtrip(int fd, const std::string& req) {
  if (::send(fd, req.data(), req.size(), MSG_NOSIGNAL) < 0) return {};
  std::string buf;
  char tmp[8192];
  while (true) {
    http::Message m;
    std::string err;
    if (http::parse(buf.data(), buf.size(), false, &m, &err) > 0) return std::to_string(m.status) + " " + m.body;
    ssize_t got = ::recv(fd, tmp, sizeof(tmp), 0);
    if (got <= 0) return {};
    buf.append(tmp, static_cast<size_t>(got));
  }
}

static void test_server_stress() {
  int aport = 0;
  int alfd = listen_any(&aport);
  std::atomic<bool> stop{false};
  std::atomic<int> bindings{0};
  std::thread api(fake_apiserver, alfd, &stop, &bindings);

  Ledger l{Profile()};
  NodeView nv;
  nv.name = "n";
  nv.total = 8 * 1000;
  nv.count = 8;
  l.upsert_node(nv);
  ServerConfig cfg;
  cfg.host = "127.0.0.1";
  cfg.threads = 3;
  cfg.pool_threads = 6;
  cfg.api.server = "http://127.0.0.1:" + std::to_string(aport);
  std::unique_ptr<NativeServer> srv(new NativeServer(&l, cfg));
  std::string err;
  int port = srv->start(&err);
  CHECK(port > 0);
  const int kThreads = 8, kPods = 40;
  std::atomic<int> ok{0}, failed{0};
  std::vector<std::thread> cs;
  for (int t = 0; t < kThreads; ++t) {
    cs.emplace_back([&, t] {
      int fd = ::socket(AF_INET, SOCK_STREAM, 0);
      sockaddr_in a;
      std::memset(&a, 0, sizeof(a));
      a.sin_family = AF_INET;
      a.sin_port = htons(static_cast<uint16_t>(port));
      a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
      if (::connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0) {
        failed.fetch_add(kPods);
        return;
      }
      for (int i = 0; i < kPods; ++i) {
        std::string uid = "u" + std::to_string(t) + "-" + std::to_string(i);
        std::string name = "p" + std::to_string(t) + "-" + std::to_string(i);
        std::string fb = "{\"Pod\":" + pod_json(name, uid, 25) + ",\"NodeNames\":[\"n\"]}";
        std::string r1 = roundtrip(fd, "POST /gpushare-scheduler/filter HTTP/1.1\r\nContent-Length: " +
                                           std::to_string(fb.size()) + "\r\n\r\n" + fb);
        std::string bb = "{\"PodName\":\"" + name + "\",\"PodNamespace\":\"default\",\"PodUID\":\"" + uid +
                         "\",\"Node\":\"n\"}";
        std::string r2 = roundtrip(fd, "POST /gpushare-scheduler/bind HTTP/1.1\r\nContent-Length: " +
                                           std::to_string(bb.size()) + "\r\n\r\n" + bb);
        if (r2.rfind("200 ", 0) == 0) {
          ok.fetch_add(1);
        } else {
          failed.fetch_add(1);
        }
        (void)r1;
      }
      ::close(fd);
    });
  }
  for (auto& t : cs) t.join();
  // 8 devices x 1000 / 25 = 320 slots for 320 pods: every bind fits exactly once
  CHECK(ok.load() == kThreads * kPods);
  CHECK(failed.load() == 0);
  CHECK(bindings.load() == kThreads * kPods);
  {
    std::lock_guard<introspect::ProfiledMutex> g(l.mu());
    for (auto& d : l.node_devices("n")) CHECK(d.second == 1000);
  }
  srv.reset();  // stops the loops and closes the keep-alive apiserver connections
  stop.store(true);
  ::shutdown(alfd, SHUT_RDWR);
  ::close(alfd);
  api.join();
}

// Landing-order Allocate matching (allocstate.h) and the per-node bind order it lets the ledger drop (ledger.h).
static void test_landing_order() {
  AllocState st("n", {{0, {256, 8}}, {1, {256, 8}}});
  auto pod = [](const char* uid, const char* rv, int64_t dev, int64_t assume) {
    AllocPod p;
    p.uid = uid;
    p.key = std::string("default/") + uid;
    p.ns = "default";
    p.name = uid;
    p.rv = rv;
    p.phase = "Pending";
    p.node = "n";
    p.dev = dev;
    p.request = 8;
    p.containers = {8};
    p.assume_time = assume;
    p.assigned = "false";
    return p;
  };
  CHECK(st.observe(pod("late", "5", 0, 30)));    // assumed last, landed first
  CHECK(st.observe(pod("early", "9", 1, 10)));
  auto c = st.candidates();
  CHECK(c.size() == 2 && c[0]->uid == "late" && c[1]->uid == "early");
  CHECK(st.observe(pod("late", "12", 0, 30)));   // a later copy keeps its landing
  CHECK(st.match(8).first && st.match(8).first->uid == "late");
  CHECK(!st.observe(pod("early", "3", 1, 10)));  // an older copy is ignored
  AllocPod norv = pod("norv", "", 0, 1);         // no integer resourceVersion: ASSUME_TIME decides, after both
  CHECK(st.observe(norv));
  c = st.candidates();
  CHECK(c.size() == 3 && c[2]->uid == "norv");

  for (int mode = 0; mode < 3; ++mode) {  // auto / strict / relaxed on a landing-order node and a plain one
    for (int landing = 0; landing < 2; ++landing) {
      Ledger l{Profile()};
      l.set_order_mode(static_cast<Ledger::OrderMode>(mode));
      NodeView nv;
      nv.name = "n";
      nv.total = 2 * 16;
      nv.count = 2;
      nv.landing_order = landing == 1;
      l.upsert_node(nv);
      int64_t total = 0, ns = 0;
      uint64_t sa = 0, sb = 0;
      CHECK(l.assume_ordered("ua", "default", "a", "n", 10, &total, &sa, &ns) == 0);
      CHECK(l.assume_ordered("ub", "default", "b", "n", 10, &total, &sb, &ns) == 1);
      const bool want_blocked = mode == Ledger::kOrderStrict || (mode == Ledger::kOrderAuto && !landing);
      CHECK(l.bind_blocked(sb) == want_blocked);
      CHECK(!l.bind_blocked(sa));
      l.bind_leave(sa);
      CHECK(!l.bind_blocked(sb));
      l.bind_leave(sb);
    }
  }
}

// The wave driver's BatchClient (persistent helper threads, tracker.cc) over many batches of mixed concurrency, and
// ApiClient::abort shutting requests in flight against an apiserver that never answers.
static void silent_apiserver(int lfd, std::atomic<bool>* stop) {
  std::vector<int> held;
  while (!stop->load()) {
    int c = ::accept(lfd, nullptr, nullptr);
    if (c < 0) break;
    held.push_back(c);  // read nothing, answer nothing
  }
  for (int c : held) ::close(c);
}

static void test_batch_client_and_abort() {
  int aport = 0;
  int alfd = listen_any(&aport);
  std::atomic<bool> stop{false};
  std::atomic<int> bindings{0};
  std::thread api(fake_apiserver, alfd, &stop, &bindings);
  ApiConfig cfg;
  cfg.server = "http://127.0.0.1:" + std::to_string(aport);
  {
    BatchClient bc(cfg);
    for (int k = 0; k < 60; ++k) {
      std::vector<BatchClient::Req> reqs;
      for (int i = 0; i < 3 + k % 20; ++i) reqs.emplace_back("POST", "/api/v1/namespaces/d/pods/p" + std::to_string(i) + "/binding", "{}");
      auto out = bc.run(reqs, (k % 3 == 0) ? 1 : (k % 3 == 1 ? 4 : 16));
      CHECK(out.size() == reqs.size());
      for (auto& o : out) CHECK(o.first == 201);
    }
  }
  CHECK(bindings.load() > 0);
  // abort: two requests stuck on an apiserver that never answers fail at once, and later ones fail without waiting
  int sport = 0;
  int slfd = listen_any(&sport);
  std::atomic<bool> sstop{false};
  std::thread silent(silent_apiserver, slfd, &sstop);
  ApiConfig scfg;
  scfg.server = "http://127.0.0.1:" + std::to_string(sport);
  ApiClient c(scfg);
  std::atomic<int> failed{0};
  std::vector<std::thread> ts;
  for (int i = 0; i < 2; ++i) {
    ts.emplace_back([&] {
      int st = 0;
      std::string resp, err;
      if (!c.request("PATCH", "/api/v1/namespaces/d/pods/x", "{}", "application/merge-patch+json", &st, &resp, &err)) {
        failed.fetch_add(1);
      }
    });
  }
  ::usleep(200000);  // both are waiting for an answer
  const auto t0 = std::chrono::steady_clock::now();
  c.abort();
  for (auto& t : ts) t.join();
  CHECK(failed.load() == 2);
  CHECK(std::chrono::steady_clock::now() - t0 < std::chrono::seconds(5));
  int st = 0;
  std::string resp, err;
  CHECK(!c.request("GET", "/api/v1/pods", "", "application/json", &st, &resp, &err));
  stop.store(true);
  sstop.store(true);
  ::shutdown(alfd, SHUT_RDWR);
  ::shutdown(slfd, SHUT_RDWR);
  ::close(alfd);
  ::close(slfd);
  api.join();
  silent.join();
}

// The one-pass Allocate response encoder against the straightforward one: byte-identical output for empty and
// multi-container responses, empty strings (absent fields), read-only mounts and values over 127 bytes.
static void test_allocate_response_encoding() {
  std::vector<dp::ContainerResponse> none;
  CHECK(dp::encode_allocate_response_selfcheck(none));
  dp::ContainerResponse a;
  a.envs["HIP_VISIBLE_DEVICES"] = "0";
  a.envs["EMPTY"] = "";
  a.envs[std::string(200, 'k')] = std::string(300, 'v');
  a.annotations["gpushare.amd.com/pod"] = "default/p/uid";
  a.mounts.push_back(dp::MountMsg{"/run/gsx/isolation.conf", "/var/lib/gsx/x/isolation.conf", true});
  a.mounts.push_back(dp::MountMsg{"/c", "", false});
  a.devices.push_back(dp::DeviceSpecMsg{"/dev/kfd", "/dev/kfd", "rw"});
  a.devices.push_back(dp::DeviceSpecMsg{"", "", ""});
  dp::ContainerResponse b;  // an empty container
  std::vector<dp::ContainerResponse> two{a, b};
  CHECK(dp::encode_allocate_response_selfcheck({a}));
  CHECK(dp::encode_allocate_response_selfcheck(two));
  std::vector<dp::ContainerResponse> back;
  CHECK(dp::decode_allocate_response(dp::encode_allocate_response(two), &back) && back.size() == 2 &&
        back[0].envs.size() == 3 && back[0].mounts.size() == 2 && back[0].devices.size() == 2);
}

int main() {
  test_json();
  test_quantity();
  test_ledger();
  test_landing_order();
  test_http();
  test_request_parser();
  test_server_stress();
  test_batch_client_and_abort();
  test_allocate_response_encoding();
  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("engine_test: all checks passed\n");
  return 0;
}
