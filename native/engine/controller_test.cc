// Concurrency stress of the extender's native stack, built under sanitizers:
//   ThreadSanitizer:   python native/build.py tsan   -> build/controller_test_tsan
//   ASan + UBSan:      python native/build.py asan   -> build/controller_test_asan
// (engine_test.cc never constructed Controller / Reflector, which run two reflector
// threads and a resync thread whose locks nest with the server pool's.)
//
// Against a real gsx-fakeapi (started by tests/test_sanitizers.py; `--apiserver URL`), for a few seconds:
//   * Controller: pod + node reflectors (paginated LISTs, watches, forced re-lists), resync thread;
//   * NativeServer: 2 epoll loops + 8 pool threads serving filter / bind storms from 6 client threads,
//     native binds POSTing pods/binding to the apiserver;
//   * churn: a creator and a deleter thread, watch drops injected through /fake/faults;
//   * reservation GC + forced re-lists, inspect / stats readers;
//   * PodTracker (tracker.cc) watching the churn label, PodRuntime (podruntime.cc, accounting only)
//     admitting and releasing slices from two threads.
// Invariants checked at the end: no device over-committed, every thread made progress, clean stops.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <deque>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "apiclient.h"
#include "controller.h"
#include "json.h"
#include "ledger.h"
#include "podruntime.h"
#include "server.h"
#include "tracker.h"

using namespace gsx;

static int g_fail = 0;
#define CHECK(c)                                                                     \
  do {                                                                               \
    if (!(c)) {                                                                      \
      std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c);     \
      ++g_fail;                                                                      \
    }                                                                                \
  } while (0)

namespace {

constexpr int kNodes = 6, kDevs = 4, kDevUnits = 100, kPodUnits = 10;

std::string node_json(int i) {
  char b[512];
  std::snprintf(b, sizeof(b),
                "{\"apiVersion\":\"v1\",\"kind\":\"Node\",\"metadata\":{\"name\":\"n%d\",\"labels\":{\"gpushare\":"
                "\"true\"}},\"status\":{\"capacity\":{\"shared-gpu/gpu-mem\":\"%d\",\"shared-gpu/gpu-count\":\"%d\"},"
                "\"addresses\":[{\"type\":\"InternalIP\",\"address\":\"10.0.0.%d\"}]}}",
                i, kDevs * kDevUnits, kDevs, i + 1);
  return b;
}

std::string pod_json(const std::string& name) {
  return "{\"apiVersion\":\"v1\",\"kind\":\"Pod\",\"metadata\":{\"name\":\"" + name +
         "\",\"namespace\":\"default\",\"labels\":{\"gsx-stress\":\"1\"}},\"spec\":{\"schedulerName\":\"default-"
         "scheduler\",\"containers\":[{\"name\":\"c\",\"resources\":{\"limits\":{\"shared-gpu/gpu-mem\":\"" +
         std::to_string(kPodUnits) + "\"}}}]},\"status\":{\"phase\":\"Pending\"}}";
}

struct Created {
  std::string name, uid, raw;
};

class Queue {
 public:
  void push(Created c) {
    std::lock_guard<std::mutex> g(mu_);
    q_.push_back(std::move(c));
  }
  bool pop(Created* out) {
    std::lock_guard<std::mutex> g(mu_);
    if (q_.empty()) return false;
    *out = std::move(q_.front());
    q_.pop_front();
    return true;
  }

 private:
  std::mutex mu_;
  std::deque<Created> q_;
};

double now_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

}  // namespace

int main(int argc, char** argv) {
  std::string apiserver;
  double seconds = 3.0;
  for (int i = 1; i + 1 < argc; ++i) {
    if (std::strcmp(argv[i], "--apiserver") == 0) apiserver = argv[++i];
    else if (std::strcmp(argv[i], "--seconds") == 0) seconds = std::atof(argv[++i]);
  }
  if (apiserver.empty()) {
    std::fprintf(stderr, "usage: controller_test --apiserver URL [--seconds S]\n");
    return 2;
  }
  ApiConfig api;
  api.server = apiserver;
  ApiClient admin(api);
  int st = 0;
  std::string resp, err;
  for (int i = 0; i < kNodes; ++i) {
    CHECK(admin.request("POST", "/api/v1/nodes", node_json(i), "application/json", &st, &resp, &err) && st == 201);
  }

  Ledger ledger{Profile()};
  ControllerConfig cc;
  cc.api = api;
  cc.resync_s = 0.2;  // exercise the resync thread against the reflectors
  Controller ctl(&ledger, cc);
  CHECK(ctl.start(30, &err));
  ServerConfig sc;
  sc.host = "127.0.0.1";
  sc.threads = 2;
  sc.pool_threads = 8;
  sc.api = api;
  sc.reservation_ttl = 0.3;
  NativeServer srv(&ledger, sc);
  int port = srv.start(&err);
  CHECK(port > 0);
  ApiConfig ext;
  ext.server = "http://127.0.0.1:" + std::to_string(port);
  PodTracker tracker(api, "default", "gsx-stress=1");
  CHECK(tracker.start(30, &err));
  PodRuntimeConfig rc;
  rc.arena_bytes = uint64_t(1) << 34;
  PodRuntime runtime(rc);
  CHECK(runtime.init(&err));

  std::atomic<bool> stop{false};
  std::atomic<uint64_t> created{0}, filtered{0}, bound{0}, bind_errors{0}, deleted{0}, gcs{0}, reads{0},
      admits{0};
  Queue to_bind, to_delete;
  std::vector<std::thread> th;

  th.emplace_back([&] {  // creator
    ApiClient c(api);
    uint64_t i = 0;
    while (!stop.load()) {
      std::string name = "s" + std::to_string(i++), body = pod_json(name), r, e;
      int s = 0;
      if (!c.request("POST", "/api/v1/namespaces/default/pods", body, "application/json", &s, &r, &e) || s != 201) {
        continue;
      }
      json::Doc d;
      std::string pe;
      if (!d.parse(r, &pe)) continue;
      int64_t u = d.path(0, {"metadata", "uid"});
      to_bind.push({name, u >= 0 ? d.str(static_cast<uint32_t>(u)) : std::string(), r});
      created++;
      if (created.load() % 50 == 0) std::this_thread::sleep_for(std::chrono::milliseconds(2));
    }
  });
  for (int t = 0; t < 6; ++t) {  // scheduler stand-ins: filter, then bind to the first feasible node
    th.emplace_back([&] {
      ApiClient c(ext);
      std::string names = "[";
      for (int i = 0; i < kNodes; ++i) names += std::string(i ? "," : "") + "\"n" + std::to_string(i) + "\"";
      names += "]";
      Created p;
      while (!stop.load()) {
        if (!to_bind.pop(&p)) {
          std::this_thread::sleep_for(std::chrono::microseconds(200));
          continue;
        }
        std::string fb = "{\"Pod\":" + p.raw + ",\"NodeNames\":" + names + "}", r, e;
        int s = 0;
        if (!c.request("POST", "/gpushare-scheduler/filter", fb, "application/json", &s, &r, &e) || s != 200) continue;
        filtered++;
        json::Doc d;
        std::string pe;
        if (!d.parse(r, &pe)) continue;
        int64_t nn = d.find(0, "NodeNames");
        if (nn < 0 || d.at(static_cast<uint32_t>(nn)).type != json::T::Array || d.at(static_cast<uint32_t>(nn)).count == 0) {
          to_delete.push(p);  // full cluster: let the deleter free room
          continue;
        }
        std::string node = d.str(static_cast<uint32_t>(nn) + 1);
        std::string bb = "{\"PodName\":\"" + p.name + "\",\"PodNamespace\":\"default\",\"PodUID\":\"" + p.uid +
                         "\",\"Node\":\"" + node + "\"}";
        if (c.request("POST", "/gpushare-scheduler/bind", bb, "application/json", &s, &r, &e) && s == 200) {
          bound++;
        } else {
          bind_errors++;
        }
        to_delete.push(p);
      }
    });
  }
  th.emplace_back([&] {  // deleter: churn lags the binds a little
    ApiClient c(api);
    Created p;
    while (!stop.load()) {
      if (!to_delete.pop(&p)) {
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
        continue;
      }
      std::string r, e;
      int s = 0;
      if (c.request("DELETE", "/api/v1/namespaces/default/pods/" + p.name, "", nullptr, &s, &r, &e)) deleted++;
    }
  });
  th.emplace_back([&] {  // reservation GC, forced re-lists, injected watch drops
    ApiClient c(api);
    int k = 0;
    while (!stop.load()) {
      bool relist = false;
      ctl.gc_reservations(&relist);
      gcs++;
      if (++k % 15 == 0) ctl.request_pod_relist();
      if (k % 40 == 0) {
        std::string r, e;
        int s = 0;
        c.request("POST", "/fake/faults", "{\"drop_watches_now\":true}", "application/json", &s, &r, &e);
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
  });
  th.emplace_back([&] {  // observers: inspect, stats, lister
    while (!stop.load()) {
      {
        std::lock_guard<introspect::ProfiledMutex> g(ledger.mu());
        bool found = false;
        std::string js = ledger.inspect_json("", &found);
        CHECK(!js.empty());
      }
      ControllerStats cs = ctl.stats();
      (void)cs;
      std::string raw;
      ctl.get_pod("default/s1", &raw);
      (void)srv.stats();
      (void)tracker.size();
      reads++;
      std::this_thread::sleep_for(std::chrono::microseconds(500));
    }
  });
  for (int t = 0; t < 2; ++t) {  // the per-GPU runtime endpoint's admissions and releases
    th.emplace_back([&, t] {
      std::mt19937 rng(static_cast<unsigned>(t + 1));
      int i = 0;
      while (!stop.load()) {
        std::string uid = "rt" + std::to_string(t) + "-" + std::to_string(i++ % 64), e;
        if (rng() % 2) {
          if (runtime.admit(uid, uint64_t(1) << 28, true, &e) >= 0) admits++;
        } else {
          runtime.release(uid);
        }
      }
    });
  }

  double t0 = now_s();
  while (now_s() - t0 < seconds) std::this_thread::sleep_for(std::chrono::milliseconds(20));
  stop.store(true);
  for (auto& t : th) t.join();

  // settle: the informer catches up with the deletes, GC drops what no LIST confirms
  for (int i = 0; i < 100; ++i) {
    bool relist = false;
    ctl.gc_reservations(&relist);
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
  {
    std::lock_guard<introspect::ProfiledMutex> g(ledger.mu());
    for (int i = 0; i < kNodes; ++i) {
      for (auto& d : ledger.node_devices("n" + std::to_string(i))) CHECK(d.second <= d.first);
    }
  }
  std::printf("created=%llu filtered=%llu bound=%llu bind_errors=%llu deleted=%llu gc=%llu reads=%llu admits=%llu "
              "pod_lists=%llu\n",
              (unsigned long long)created.load(), (unsigned long long)filtered.load(),
              (unsigned long long)bound.load(), (unsigned long long)bind_errors.load(),
              (unsigned long long)deleted.load(), (unsigned long long)gcs.load(), (unsigned long long)reads.load(),
              (unsigned long long)admits.load(), (unsigned long long)ctl.stats().pod_lists);
  CHECK(created.load() > 50 && bound.load() > 20 && deleted.load() > 20 && gcs.load() > 10 && admits.load() > 10);
  CHECK(ctl.stats().pod_lists >= 2);  // forced re-lists happened
  tracker.stop();
  runtime.stop();
  srv.stop();
  ctl.stop();
  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("controller_test: all checks passed\n");
  return 0;
}
