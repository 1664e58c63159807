// gsx-nodeagent: kubelet + device-plugin + container-runtime stand-in for one
// node, in C++ (the compiled counterpart of gsxtools/agent.py).
//
// Where there is no kubelet (bench.py on the GPU box, simulators), this drives
// the device plugin's Allocate logic for every pod bound to the node and
// starts the pod on its GPU's runtime endpoint -- the tail of the reference's
// sequence diagram (docs/designs/sequence.jpg, docs/designs/designs.md:93-103):
//
//   bound pod, ASSIGNED=false ──► Allocate(N ids): the earliest-ASSUME_TIME
//   unassigned pod of that size on this node ──► PATCH ASSIGNED=true with a
//   resourceVersion precondition (the commit point; 409 -> retry) ──► container
//   env (HIP_VISIBLE_DEVICES, *_IDX/_DEV/_POD/_CONTAINER, memory fraction,
//   optional CU partition) ──► POST <runtime>/v1/pods/<uid>: the pod's slice of
//   the GPU's HBM arena is stamped by a HIP kernel and every resident slice is
//   verified ──► PATCH status Running.
//   completed / deleted pod ──► DELETE <runtime>/v1/pods/<uid>, CUs released.
//   terminating pod (deletionTimestamp, graceful delete) ──► its containers stop (--stop-delay seconds, at most
//   its grace period) ──► DELETE <runtime>/v1/pods/<uid> ──► PATCH status Succeeded ──► DELETE the pod with
//   gracePeriodSeconds 0 and a UID precondition: kubelet, not the apiserver, ends a graceful deletion.
//
// Devices and runtime endpoints come from the node's annotations
// (gpushare.amd.com/devices, gpushare.amd.com/runtime-endpoints), written by
// the device plugin / the benchmark.  Control endpoints:
//   GET /v1/stats, GET /v1/allocations/<uid> (container env of the Allocate).
//
// The matching decision is AllocState (native/engine/allocstate.h), shared with the shipped gRPC device plugin.
//
//   gsx-nodeagent --apiserver URL --node NAME [--profile P] [--unit GiB]
//                 [--workers N] [--no-verify] [--serial-admission] [--port-file F]
//                 [--plugin-socket S | --plugin-spawn PYTHON] [--batch-window SECONDS]
//
// Admission: with the shipped plugin (--plugin-socket / --plugin-spawn), or with --serial-admission for the
// in-process matcher, pods are admitted one at a time in the order the informer met them, as kubelet does (the
// Allocate, and the plugin's ASSIGNED commit inside it, are serial); starting the container (runtime + Running
// patch) runs on the workers in parallel, as kubelet's pod workers do.  Without it the in-process matcher admits
// on all workers at once.
#include <poll.h>
#include <signal.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <fstream>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "allocstate.h"
#include "apiclient.h"
#include "ctlserver.h"
#include "dpcore.h"
#include "dpproto.h"
#include "h2.h"
#include "informer.h"
#include "introspect.h"
#include "json.h"
#include "model.h"
#include "quantity.h"

using namespace gsx;

namespace {

void put_varint(std::string* o, uint64_t v) {  // protobuf base-128 varint
  while (v >= 0x80) {
    o->push_back(static_cast<char>((v & 0x7f) | 0x80));
    v >>= 7;
  }
  o->push_back(static_cast<char>(v));
}

const char* kDevInfoAnn = "gpushare.amd.com/devices";
const char* kEndpointsAnn = "gpushare.amd.com/runtime-endpoints";
const char* kCuMaskAnn = "gpushare.amd.com/cu-mask";
const char* kAssignTimeAnn = "gpushare.amd.com/assign-time";

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int64_t unix_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::system_clock::now().time_since_epoch())
      .count();
}

struct Device {
  int index = 0;
  std::string bdf;
  int cu = 256, xcc = 8;
  int render = -1, card = -1;
  // a partition sharing one HBM pool (CPX/NPS1): its process sees the whole pool, so the memory
  // fraction is scaled by share/total (deviceplugin/allocator.py build_response)
  int64_t total_bytes = 0, share_bytes = 0;
  std::string endpoint;
};

// The Allocate matching, CU partitions and multi-container progress are the device plugin's own
// (native/engine/allocstate.h, the same code deviceplugin/state.py runs): this agent only plays kubelet
// and the container runtime around it.

class Agent {
 public:
  Agent(ApiConfig api, std::string node, Profile p, int64_t unit_bytes, int workers, bool verify)
      : api_cfg_(api), node_(std::move(node)), p_(std::move(p)), unit_(unit_bytes), nworkers_(workers),
        verify_(verify), api_(api) {}

  bool load_devices(double timeout_s, std::string* err) {
    double deadline = now_s() + timeout_s;
    while (true) {
      int status = 0;
      std::string body, e;
      if (api_.request("GET", "/api/v1/nodes/" + node_, std::string(), nullptr, &status, &body, &e) && status == 200) {
        json::Doc d;
        std::string perr;
        if (d.parse(body, &perr)) {
          int64_t an = d.path(0, {"metadata", "annotations"});
          int64_t inv = an >= 0 ? d.find(static_cast<uint32_t>(an), kDevInfoAnn) : -1;
          int64_t eps = an >= 0 ? d.find(static_cast<uint32_t>(an), kEndpointsAnn) : -1;
          if (inv >= 0 && eps >= 0 && parse_devices(d.str(static_cast<uint32_t>(inv)), d.str(static_cast<uint32_t>(eps))))
            return true;
        }
      }
      if (now_s() > deadline) {
        *err = "node " + node_ + " never published devices + runtime endpoints";
        return false;
      }
      ::usleep(50000);
    }
  }

  // kubelet admits a node's pods one at a time (Allocate included): with this set the in-process matcher does too
  void set_serial_admission(bool on) { serial_admission_ = on; }

  void set_plugin_socket(const std::string& s) { plugin_sock_ = s; }
  // how long a container takes to stop after SIGTERM (graceful deletion), capped by the pod's grace period
  void set_stop_delay(double s) { stop_delay_ = std::max(0.0, s); }
  void set_batch_window(double s) { batch_window_ = s; }
  void set_plugin_spawn(const std::string& python, const std::string& apiserver, const std::string& profile,
                        const std::string& unit) {
    spawn_python_ = python;
    spawn_api_ = apiserver;
    spawn_profile_ = profile;
    spawn_unit_ = unit;
  }

  // Run the shipped device plugin as a child process on this node's inventory (the fake device backend fed the
  // node's published devices; no kubelet registration, no PodResources: this stand-in serves neither).
  bool spawn_plugin(std::string* err) {
    char tmpl[] = "/tmp/gsx-na-XXXXXX";
    if (!::mkdtemp(tmpl)) {
      *err = std::string("mkdtemp: ") + std::strerror(errno);
      return false;
    }
    std::string dir = tmpl;
    std::string spec = dir + "/devices.json";
    {
      std::ofstream f(spec);
      f << "[";
      bool first = true;
      for (const auto& kv : devices_) {
        const Device& d = kv.second;
        if (!first) f << ",";
        first = false;
        std::string bdf;
        json::append_quoted(&bdf, d.bdf);
        f << "{\"index\":" << d.index << ",\"bdf\":" << bdf << ",\"total_bytes\":" << d.total_bytes
          << ",\"share_bytes\":" << d.share_bytes << ",\"cu_count\":" << d.cu << ",\"xcc_count\":" << d.xcc
          << ",\"render_minor\":" << d.render << ",\"card_minor\":" << d.card << "}";
      }
      f << "]";
    }
    // kubelet's PodResources API, served by this agent (pr_serve): the plugin reconciles its Allocate records
    // against it, as under a real kubelet
    pr_sock_ = dir + "/pod-resources.sock";
    if (!pr_start(err)) return false;
    std::vector<std::string> args = {spawn_python_, "-m", "gpushare_scheduler_extender_amd.deviceplugin", "--node", node_,
                                     "--apiserver", spawn_api_, "--profile", spawn_profile_, "--unit", spawn_unit_,
                                     "--backend", "fake", "--socket-dir", dir, "--no-publish", "--no-register",
                                     "--podresources-socket", pr_sock_, "--isolation", "advisory", "--health-interval",
                                     "3600", "--log-level", "warning", "--debug-port", "0", "--debug-port-file",
                                     dir + "/debug.port"};
    const char* ext_url = std::getenv("GSX_EXTENDER_URL");
    if (!ext_url || !*ext_url) args.push_back("--no-extender");  // a harness run without an extender
    plugin_debug_file_ = dir + "/debug.port";
    pid_t pid = ::fork();
    if (pid < 0) {
      *err = std::string("fork: ") + std::strerror(errno);
      return false;
    }
    if (pid == 0) {
      ::setenv("GSX_FAKE_DEVICES", spec.c_str(), 1);
      std::vector<char*> argv;
      for (auto& a : args) argv.push_back(const_cast<char*>(a.c_str()));
      argv.push_back(nullptr);
      ::execv(spawn_python_.c_str(), argv.data());
      ::_exit(127);
    }
    plugin_pid_ = pid;
    plugin_sock_ = dir + "/gpushare-amd.sock";
    return true;
  }
  bool start(std::string* err) {
    if (!spawn_python_.empty() && !spawn_plugin(err)) return false;
    if (!plugin_sock_.empty() && !plugin_connect(120, err)) return false;
    ReflectorConfig rc;
    rc.path = "/api/v1/pods";
    rc.field_selector = "spec.nodeName=" + node_;
    ReflectorHandler h;
    h.on_list = [this](const ListView& lv) {
      std::lock_guard<std::mutex> g(mu_);
      std::unordered_set<std::string> seen, live;
      for (size_t k = 0; k < lv.size(); ++k) seen.insert(on_pod_locked(lv.doc(k), lv.obj(k), &live));
      std::vector<std::string> gone;
      for (auto& kv : keys_) {
        if (!seen.count(kv.first)) gone.push_back(kv.first);
      }
      for (auto& k : gone) on_delete_locked(k);
      state_->resync(live);
      wake_locked();
    };
    h.on_event = [this](Ev ev, const json::Doc& d, uint32_t obj) {
      // the event is read before the agent's lock is taken: the admitting worker needs that lock between its
      // two calls to the plugin, and a wave of N x 4 pods brings ~5 events per pod
      if (ev == Ev::Deleted) {
        PodView v;
        parse_pod(d, obj, p_, &v);
        std::lock_guard<std::mutex> g(mu_);
        on_delete_locked(v.ns + "/" + v.name);
        wake_locked();
      } else {
        AllocPod ap;
        parse_alloc_pod(d, obj, p_, &ap);
        std::lock_guard<std::mutex> g(mu_);
        on_pod_parsed_locked(ap, nullptr);
        wake_locked();
      }
    };
    pods_r_ = std::make_unique<Reflector>(api_cfg_, rc, h);
    pods_r_->start();
    if (!pods_r_->wait_synced(60)) {
      *err = "pod informer did not sync: " + pods_r_->last_error();
      return false;
    }
    target_workers_ = static_cast<size_t>(std::max(nworkers_, 1));
    for (int i = 0; i < nworkers_; ++i) {
      workers_.emplace_back([this, i] {
        introspect::name_thread("na-worker");
        worker(static_cast<size_t>(i));
      });
    }
    ready_.store(true);
    return true;
  }

  void stop() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    stop_flag_.store(true);
    cv_.notify_all();
    park_cv_.notify_all();
    for (auto& t : workers_) t.join();
    if (pods_r_) pods_r_->stop();
    pr_stop();
    if (plugin_pid_ > 0) {
      ::kill(plugin_pid_, SIGTERM);
      for (int i = 0; i < 100 && ::waitpid(plugin_pid_, nullptr, WNOHANG) == 0; ++i) ::usleep(50000);
      ::kill(plugin_pid_, SIGKILL);
      ::waitpid(plugin_pid_, nullptr, WNOHANG);
      plugin_pid_ = -1;
    }
  }

  CtlServer::Reply handle(const http::Message& req) {
    CtlServer::Reply rep;
    std::string_view path = req.path();
    std::lock_guard<std::mutex> g(mu_);
    if (req.method == "GET" && path == "/v1/stats") {
      if (!ready_.load()) {  // as the Python agent: 503 until the pod informer has synced and workers run
        rep.status = 503;
        rep.body = "{}";
        return rep;
      }
      std::vector<double> lat = latency_;
      std::sort(lat.begin(), lat.end());
      double p50 = lat.empty() ? 0 : lat[lat.size() / 2];
      const double n = admitted_ ? static_cast<double>(admitted_) : 1.0;
      const double fn = finals_done_ ? static_cast<double>(finals_done_) : 1.0;
      char b[2560];
      std::snprintf(b, sizeof(b),
                    "{\"admitted\":%llu,\"failed\":%llu,\"bad_stamps\":%llu,\"conflicts\":%llu,\"running\":%zu,"
                    "\"stopping\":%zu,\"releases_queued\":%zu,"
                    "\"admit_p50_ms\":%.3f,\"admit_max_ms\":%.3f,\"max_ms\":{\"queue\":%.3f,\"assign_patch\":%.3f,"
                    "\"runtime\":%.3f,\"running_patch\":%.3f},\"mean_ms\":{\"queue\":%.4f,\"assign_patch\":%.4f,"
                    "\"runtime\":%.4f,\"running_patch\":%.4f},\"status_retries\":%llu,\"api_connects\":%llu,"
                    "\"plugin_calls_mean_ms\":{\"n\":%llu,\"slot_wait\":%.4f,\"get_preferred\":%.4f,\"allocate\":%.4f,"
                    "\"encode_preferred\":%.4f,\"gap\":%.4f,\"n_gap\":%llu,\"gap_loop\":%.4f,\"gap_list\":%.4f,"
                    "\"gap_handoff\":%.4f,\"relock\":%.4f,\"gap_kept\":%.4f,\"n_gap_kept\":%llu},"
                    "\"mismatch\":%llu,\"podresources_calls\":%llu,\"plugin_debug\":\"%s\",\"finalized\":%llu,"
                    "\"finalize_mean_ms\":{\"wake\":%.4f,\"stop\":%.4f,\"status\":%.4f,\"delete\":%.4f},"
                    "\"native\":true}",
                    (unsigned long long)admitted_, (unsigned long long)failed_, (unsigned long long)bad_,
                    (unsigned long long)conflicts_, running_.size(), stopping_.size(), releases_.size(), p50 * 1e3, lat.empty() ? 0.0 : lat.back() * 1e3,
                    max_queue_ * 1e3, max_patch_ * 1e3, max_runtime_ * 1e3, max_status_ * 1e3, sum_queue_ / n * 1e3,
                    sum_patch_ / n * 1e3, sum_runtime_ / n * 1e3, sum_status_ / n * 1e3,
                    (unsigned long long)status_retries_.load(), (unsigned long long)api_.reconnects(),
                    (unsigned long long)dp_calls_, sum_dp_slot_ / std::max<double>(1.0, dp_calls_) * 1e3,
                    sum_dp_pref_ / std::max<double>(1.0, dp_calls_) * 1e3,
                    sum_dp_alloc_ / std::max<double>(1.0, dp_calls_) * 1e3,
                    sum_dp_enc_ / std::max<double>(1.0, dp_calls_) * 1e3,
                    sum_dp_gap_ / std::max<double>(1.0, n_dp_gap_) * 1e3, (unsigned long long)n_dp_gap_,
                    sum_gap_loop_ / std::max<double>(1.0, n_dp_gap_) * 1e3,
                    sum_gap_list_ / std::max<double>(1.0, n_dp_gap_) * 1e3,
                    sum_gap_handoff_ / std::max<double>(1.0, n_dp_gap_) * 1e3,
                    sum_dp_relock_ / std::max<double>(1.0, dp_calls_) * 1e3,
                    sum_gap_kept_ / std::max<double>(1.0, n_gap_kept_) * 1e3, (unsigned long long)n_gap_kept_,
                    (unsigned long long)mismatch_,
                    (unsigned long long)pr_calls_.load(), plugin_debug_url().c_str(),
                    (unsigned long long)finals_done_, sum_fin_wake_ / fn * 1e3, sum_fin_release_ / fn * 1e3,
                    sum_fin_status_ / fn * 1e3, sum_fin_delete_ / fn * 1e3);
      rep.body = b;
      return rep;
    }
    if (req.method == "POST" && path == "/v1/config") {
      // {"verify": bool}: whether an admission verifies every resident slice of its GPU (default) or only its own
      // (bench.py's open-loop rows: hundreds of resident pods, the stand-in runtime's check is not the stack under test)
      // {"workers": n}: at least n pod workers (kubelet's pod workers are one goroutine per pod; these block on the
      // runtime call and the Running patch, so at 5 ms per apiserver call 16 of them start ~3k pods/s at most)
      json::Doc d;
      std::string e;
      if (d.parse(req.body, &e)) {
        int64_t v = d.find(0, "verify");
        if (v >= 0) verify_ = d.at(static_cast<uint32_t>(v)).type == json::T::True;
        int64_t w = d.find(0, "workers");
        int64_t nw = 0;
        if (w >= 0 && d.as_int(static_cast<uint32_t>(w), &nw)) {
          nw = std::max<int64_t>(1, std::min<int64_t>(nw, 256));
          target_workers_ = static_cast<size_t>(nw);
          while (workers_.size() < target_workers_ && !stop_) {
            const size_t me = workers_.size();
            workers_.emplace_back([this, me] {
              introspect::name_thread("na-worker");
              worker(me);
            });
          }
          park_cv_.notify_all();
        }
      }
      rep.body = std::string("{\"verify\":") + (verify_ ? "true" : "false") + ",\"workers\":" +
                 std::to_string(target_workers_) + "}";
      return rep;
    }
    const std::string_view pre = "/v1/allocations/";
    if (req.method == "GET" && path.substr(0, pre.size()) == pre) {
      auto it = allocations_.find(std::string(path.substr(pre.size())));
      if (it == allocations_.end()) {
        rep.status = 404;
        rep.body = "{}";
      } else {
        rep.body = it->second;
      }
      return rep;
    }
    rep.status = 404;
    rep.body = "{\"error\":\"not found\"}";
    return rep;
  }

 private:
  struct Final {
    double due;
    std::string uid, ns, name;
    bool ran;  // a container of it was running (or starting) when the deletion was seen
  };

  bool parse_devices(const std::string& inv, const std::string& eps) {
    json::Doc di, de;
    std::string e;
    if (!di.parse(inv, &e) || !de.parse(eps, &e)) return false;
    if (di.at(0).type != json::T::Array || de.at(0).type != json::T::Object) return false;
    std::map<int, Device> devs;
    uint32_t end = di.at(0).skip;
    for (uint32_t i = 1; i < end; i = di.next(i)) {
      if (di.at(i).type != json::T::Object) continue;
      Device d;
      int64_t v;
      auto geti = [&](const char* k, int* dst) {
        int64_t x = di.find(i, k);
        if (x >= 0 && di.as_int(static_cast<uint32_t>(x), &v)) *dst = static_cast<int>(v);
      };
      geti("index", &d.index);
      geti("cu", &d.cu);
      geti("xcc", &d.xcc);
      geti("render", &d.render);
      geti("card", &d.card);
      int64_t tb = di.find(i, "total_bytes");
      if (tb >= 0) di.as_int(static_cast<uint32_t>(tb), &d.total_bytes);
      int64_t sb = di.find(i, "share_bytes");
      if (sb >= 0) di.as_int(static_cast<uint32_t>(sb), &d.share_bytes);
      int64_t b = di.find(i, "bdf");
      if (b >= 0) d.bdf = di.str(static_cast<uint32_t>(b));
      int64_t ep = de.find(0, std::to_string(d.index));
      if (ep < 0) return false;  // every GPU needs its runtime endpoint
      d.endpoint = de.str(static_cast<uint32_t>(ep));
      devs[d.index] = d;
    }
    if (devs.empty()) return false;
    std::vector<std::pair<int, std::pair<int, int>>> cu_layout;
    for (auto& kv : devs) cu_layout.push_back({kv.first, {kv.second.cu, kv.second.xcc}});
    state_ = std::make_unique<AllocState>(node_, cu_layout);
    for (auto& kv : devs) {
      ApiConfig rc;
      rc.server = kv.second.endpoint;
      rc.timeout_s = 60;
      runtimes_.emplace(kv.first, std::make_unique<ApiClient>(rc));
    }
    devices_ = std::move(devs);
    return true;
  }

  // ---------------------------------------------------------------- informer handlers (agent.py _on_pod)
  std::string on_pod_locked(const json::Doc& d, uint32_t obj, std::unordered_set<std::string>* live) {
    AllocPod ap;
    parse_alloc_pod(d, obj, p_, &ap);
    return on_pod_parsed_locked(ap, live);
  }

  std::string on_pod_parsed_locked(const AllocPod& ap, std::unordered_set<std::string>* live) {
    const std::string key = ap.key;
    const std::string uid = ap.uid;
    if (live) live->insert(uid);
    keys_[key] = uid;
    if (ap.terminating && (ap.dev < 0 || state_->has_device(ap.dev))) {
      // graceful deletion: kubelet stops the containers, then removes the object itself (finalize_locked)
      if (finals_set_.insert(uid).second) {
        const bool runs = running_.count(uid) != 0 || state_->inflight(uid);
        double delay = runs ? std::min(stop_delay_, ap.grace_s >= 0 ? ap.grace_s : stop_delay_) : 0.0;
        finals_.push_back(Final{now_s() + delay, uid, ap.ns, ap.name, runs});
        ++added_;
      }
      state_->release(uid);  // CUs: no new container of it starts
      return key;
    }
    if (ap.complete) {
      stop_pod_locked(uid);
      state_->release(uid);  // CUs too, also for pods this agent did not start (e.g. before a restart)
      return key;
    }
    state_->observe(ap);  // candidates, CU partitions of assigned pods, multi-container progress
    if (ap.request <= 0 || !state_->has_device(ap.dev)) return key;
    if (ap.assigned == "false" && !state_->inflight(uid) && !running_.count(uid) && !queued_.count(uid)) {
      queued_.insert(uid);
      seen_.emplace(uid, now_s());
      if (batch_window_ > 0) {
        // kubelet's restart case: the pods met within the window are admitted as one batch, sorted by
        // creationTimestamp (as kubelet sorts the pods of its initial LIST), not in the order they landed
        if (batch_.empty()) batch_deadline_ = now_s() + batch_window_;
        batch_.push_back({ap.creation, key});
      } else {
        queue_.push_back(key);
      }
      ++added_;
    }
    return key;
  }

  void on_delete_locked(const std::string& key) {
    auto it = keys_.find(key);
    if (it == keys_.end()) return;
    std::string uid = it->second;
    keys_.erase(it);
    finals_set_.erase(uid);
    stop_pod_locked(uid);
    state_->tombstone(uid);  // a late copy of it (a PATCH response) never re-queues it
    if (!state_->inflight(uid)) state_->release(uid);  // the admitting worker owns it until its patch resolves
  }

  void release_cus_locked(const std::string& uid) {
    if (state_->inflight(uid)) return;
    for (auto& kv : devices_) {
      if (CuPartitioner* cp = state_->cus(kv.first)) cp->release(uid);
    }
  }

  void stop_pod_locked(const std::string& uid) {
    auto r = running_.find(uid);
    if (r == running_.end()) return;
    int dev = r->second;
    running_.erase(r);
    running_bytes_.erase(uid);
    // the container's device IDs stay taken, and PodResources keeps listing it, until the runtime has stopped it
    // (release_one): this kubelet's report is the truth about what still runs (the plugin's
    // GSX_PLUGIN_FORCE_DELETE=report).  (kubelet frees a force-deleted pod's devices, and stops listing it, at once)
    auto ui = used_ids_.find(uid);
    auto uk = uid_key_.find(uid);
    if (ui != used_ids_.end() && uk != uid_key_.end()) {
      stopping_[uid] = {uk->second, ui->second};
      used_ids_.erase(ui);
      uid_key_.erase(uk);
    } else {
      forget_ids_locked(uid);
    }
    for (auto& kv : devices_) {
      if (CuPartitioner* cp = state_->cus(kv.first)) cp->release(uid);
    }
    allocations_.erase(uid);
    releases_.push_back({uid, dev});
    ++added_;
  }

  // One worker per new work item (an event that queued nothing wakes nobody).
  void wake_locked() {
    for (; added_ > 0; --added_) cv_.notify_one();
  }

  // ---------------------------------------------------------------- admission (agent.py _admit)
  void worker(size_t me) {
    std::unique_lock<std::mutex> lk(mu_);
    std::unique_lock<std::mutex> slot(dp_mu_, std::defer_lock);  // the admission slot, when this worker holds it
    while (true) {
      // past the configured number of workers (POST /v1/config lowered it): parked apart, so that a wake-up meant
      // for a working one never lands here
      while (me >= target_workers_ && !stop_) park_cv_.wait(lk);
      double now = now_s();
      if (!batch_.empty() && now >= batch_deadline_) {
        std::stable_sort(batch_.begin(), batch_.end());
        for (auto& b : batch_) queue_.push_back(std::move(b.second));
        batch_.clear();
        cv_.notify_all();
      }
      for (auto it = delayed_.begin(); it != delayed_.end();) {
        if (it->first <= now) {
          queue_.push_back(it->second);
          it = delayed_.erase(it);
        } else {
          ++it;
        }
      }
      if (stop_) return;
      const bool serial = dp_ || serial_admission_;
      // kubelet admits one pod at a time, in the order it met them (its sync loop), and its pod workers start the
      // admitted containers in parallel.  The worker holding the admission slot pops the queue's front only while
      // it holds the slot (taken under mu_, never waited for: a worker that popped first but reached the slot later
      // would reorder the Allocates), and with the plugin it keeps the slot for the next pod, leaving the start of
      // the one it admitted to another worker (starts_): admissions follow each other with no thread hand-off
      const bool kept = slot.owns_lock();  // still holding the slot from this worker's previous admission
      if (!queue_.empty() && (!serial || slot.owns_lock() || slot.try_lock())) {
        admit_kept_ = kept;
        std::string key = std::move(queue_.front());
        queue_.pop_front();
        auto kit = keys_.find(key);
        if (kit == keys_.end()) continue;
        queued_.erase(kit->second);
        admit_locked(key, lk, serial ? &slot : nullptr);
        continue;
      }
      if (slot.owns_lock()) {  // nothing left to admit: another worker may take the slot
        slot.unlock();
        cv_.notify_all();
      }
      if (!releases_.empty()) {
        auto rel = releases_.front();
        releases_.pop_front();
        release_one(rel, lk);
        continue;
      }
      if (!starts_.empty()) {
        auto start = std::move(starts_.front());
        starts_.pop_front();
        start(lk);
        continue;
      }
      auto fin = std::find_if(finals_.begin(), finals_.end(), [now](const Final& f) { return f.due <= now; });
      if (fin != finals_.end()) {
        Final f = *fin;
        finals_.erase(fin);
        finalize_locked(f, lk);
        continue;
      }
      double wait = 0.05;
      for (auto& f : finals_) wait = std::min(wait, std::max(0.0, f.due - now));
      for (auto& dl : delayed_) wait = std::min(wait, std::max(0.0, dl.first - now));
      if (!batch_.empty()) wait = std::min(wait, std::max(0.0, batch_deadline_ - now));
      cv_.wait_for(lk, std::chrono::duration<double>(wait));
    }
  }

  // The container response is the plugin's own (native/engine/dpcore.cc build_response, mount mode "isolated":
  // only this GPU's nodes), kept as JSON for GET /v1/allocations/<uid>.
  static std::string allocation_json(const dp::ContainerResponse& r) {
    std::string o = "{\"envs\":{";
    bool first = true;
    for (const auto& kv : r.envs) {
      if (!first) o.push_back(',');
      first = false;
      json::append_quoted(&o, kv.first);
      o.push_back(':');
      json::append_quoted(&o, kv.second);
    }
    o.append("},\"devices\":[");
    for (size_t i = 0; i < r.devices.size(); ++i) {
      if (i) o.push_back(',');
      o.append("{\"container_path\":");
      json::append_quoted(&o, r.devices[i].container_path);
      o.append(",\"host_path\":");
      json::append_quoted(&o, r.devices[i].host_path);
      o.append(",\"permissions\":");
      json::append_quoted(&o, r.devices[i].permissions);
      o.push_back('}');
    }
    o.append("]}");
    return o;
  }

  std::string build_envs_locked(const AllocPod& pod, const Device& dev, const std::vector<int>& cus) {
    DpDevice d;
    d.index = dev.index;
    d.bdf = dev.bdf;
    d.cu_count = dev.cu;
    d.total_bytes = dev.total_bytes;
    d.share_bytes = dev.share_bytes;
    d.nodes = {"/dev/kfd"};
    if (dev.render >= 0) d.nodes.push_back("/dev/dri/renderD" + std::to_string(dev.render));
    if (dev.card >= 0) d.nodes.push_back("/dev/dri/card" + std::to_string(dev.card));
    return allocation_json(build_response(pod, d, pod.request, cus, "isolated", p_));
  }

  // ---------------------------------------------------------------- kubelet + the shipped device plugin
  // With --plugin-socket / --plugin-spawn the Allocate is not decided here: like kubelet, this agent asks the
  // plugin (GetPreferredAllocation, then Allocate with those IDs) over the device-plugin gRPC API and starts the
  // pod it admitted with whatever came back (never re-routed: a swap is the plugin's to repair, from this agent's
  // PodResources record), as kubelet does.
  bool plugin_connect(double timeout_s, std::string* err) {
    dp_ = std::make_unique<h2::Client>(plugin_sock_);
    double deadline = now_s() + timeout_s;
    while (true) {
      std::vector<std::string> msgs;
      int st = 0;
      std::string e;
      if (dp_->stream("/v1beta1.DevicePlugin/ListAndWatch", std::string(), 1, &msgs, &st, &e, 5.0) && !msgs.empty()) {
        std::vector<dp::DeviceMsg> devs;
        if (dp::decode_list_and_watch(msgs[0], &devs)) {
          all_ids_.clear();
          for (const auto& d : devs) {
            if (d.health == "Healthy") all_ids_.push_back(d.id);
          }
          id_index_.clear();
          id_field_.clear();
          for (size_t i = 0; i < all_ids_.size(); ++i) {
            id_index_.emplace(all_ids_[i], i);
            // the ID as GetPreferredAllocation's field 1 (available_deviceIDs), encoded once
            std::string f(1, '\x0a');
            put_varint(&f, all_ids_[i].size());
            f.append(all_ids_[i]);
            id_field_.push_back(std::move(f));
          }
          id_used_.assign(all_ids_.size(), 0);
          id_fields_.clear();
          id_field_off_.assign(1, 0);
          for (const auto& f : id_field_) {
            id_fields_.append(f);
            id_field_off_.push_back(id_fields_.size());
          }
          // as kubelet: GetPreferredAllocation only if the plugin's options advertise it
          std::string opts;
          bool pre = false;
          if (dp_->call("/v1beta1.DevicePlugin/GetDevicePluginOptions", std::string(), &opts, &st, &e) &&
              dp::decode_options(opts, &pre, &preferred_)) {
            return true;
          }
        }
      }
      if (now_s() > deadline) {
        *err = "device plugin at " + plugin_sock_ + " never answered ListAndWatch: " + e;
        return false;
      }
      dp_ = std::make_unique<h2::Client>(plugin_sock_);
      ::usleep(50000);
    }
  }

  // `slot`: the admission slot (held when admissions are serial); given up once the Allocate is answered, as
  // kubelet's pod workers start containers after admission, in parallel
  void admit_via_plugin_locked(std::string key, std::unique_lock<std::mutex>& lk, std::unique_lock<std::mutex>* slot) {
    const double te = now_s();  // gap split: loop + pop before this, the free-ID list after it
    const AllocPod* mine = state_->pod_by_key(key);
    if (!mine) return;
    const std::string my_uid = mine->uid, my_key = key;
    if (running_.count(my_uid) || state_->inflight(my_uid)) return;
    const int64_t units = mine->request;
    // kubelet's free IDs: every healthy ID no running container holds, as indices into all_ids_ (fixed once the
    // plugin is connected); without GetPreferredAllocation only the first `units` are needed, kubelet's own pick
    std::vector<uint32_t> free_idx;
    // with GetPreferredAllocation: the free IDs as runs of all_ids_ (a pod's IDs are consecutive, so a node holds a
    // few dozen runs), each copied from the pre-encoded field image in one piece
    std::vector<std::pair<size_t, size_t>> runs;
    size_t n_free = 0, field_bytes = 0;
    if (preferred_) {
      const size_t n = all_ids_.size();
      const char* used = id_used_.data();
      size_t i = 0;
      while (i < n) {
        const void* f = std::memchr(used + i, 0, n - i);  // the next free ID
        if (!f) break;
        i = static_cast<size_t>(static_cast<const char*>(f) - used);
        const void* u = std::memchr(used + i, 1, n - i);  // the next used one ends the run
        const size_t j = u ? static_cast<size_t>(static_cast<const char*>(u) - used) : n;
        runs.emplace_back(i, j);
        n_free += j - i;
        field_bytes += id_field_off_[j] - id_field_off_[i];
        i = j;
      }
    } else {
      free_idx.reserve(static_cast<size_t>(std::max<int64_t>(units, 0)));
      for (size_t i = 0; i < all_ids_.size(); ++i) {
        if (id_used_[i]) continue;
        ++n_free;
        if (static_cast<int64_t>(free_idx.size()) < units) {
          free_idx.push_back(static_cast<uint32_t>(i));
        } else {
          break;
        }
      }
    }
    if (static_cast<int64_t>(n_free) < units && !stopping_.empty()) {
      // IDs of containers still stopping: finish those releases here, then look again
      std::vector<int> devs;
      for (const auto& kv : devices_) devs.push_back(kv.first);
      for (int d : devs) drain_releases_locked(d, lk);
      queued_.insert(my_uid);
      queue_.push_front(key);
      return;
    }
    if (static_cast<int64_t>(n_free) < units) {
      std::fprintf(stderr, "[gsx-nodeagent] %s: %lld units requested, %zu IDs free\n", key.c_str(),
                   static_cast<long long>(units), n_free);
      queued_.insert(my_uid);
      delayed_.push_back({now_s() + 0.01, key});
      return;
    }
    const double tl = now_s();
    state_->set_inflight(my_uid, true);
    const double t0 = seen_.count(my_uid) ? seen_[my_uid] : now_s();
    const double prev_done = last_admitted_;
    const bool wake_starter = start_queued_;  // the previous admission's start, signalled outside the lock
    start_queued_ = false;
    lk.unlock();
    if (wake_starter) cv_.notify_one();
    std::string resp, err;
    int st = 0;
    std::vector<std::vector<std::string>> chosen;
    std::vector<dp::ContainerResponse> crs;
    const double tp0 = now_s();
    bool ok;
    double ts = 0, tpref = 0, tenc = 0;
    {
      // the worker holds the admission slot (dp_mu_) from the queue pop on: kubelet admits one pod at a time
      ts = now_s();
      if (preferred_) {
        // kubelet's request: one container, every free ID (the fields encoded at connect), then the size
        std::string size_field(1, '\x18');
        put_varint(&size_field, static_cast<uint64_t>(units));
        std::string req(1, '\x0a');
        put_varint(&req, field_bytes + size_field.size());
        req.reserve(req.size() + field_bytes + size_field.size());
        for (const auto& r : runs) req.append(id_fields_, id_field_off_[r.first], id_field_off_[r.second] - id_field_off_[r.first]);
        req.append(size_field);
        tenc = now_s() - ts;
        ok = dp_->call("/v1beta1.DevicePlugin/GetPreferredAllocation", req, &resp, &st, &err) &&
             dp::decode_preferred_response(resp, &chosen) && chosen.size() == 1;
      } else {
        // kubelet's own pick (devicesToAllocate without a preference): the first free IDs
        chosen.assign(1, {});
        for (uint32_t i : free_idx) chosen[0].push_back(all_ids_[i]);
        ok = true;
      }
      tpref = now_s();
      ok = ok && dp_->call("/v1beta1.DevicePlugin/Allocate", dp::encode_allocate_request(chosen), &resp, &st, &err) &&
           dp::decode_allocate_response(resp, &crs) && crs.size() == 1;
    }
    const double tp1 = now_s();
    // the admission slot is given up only once the IDs are recorded as used (below): kubelet's device manager
    // records an allocation before its next admission, which must never be offered the same IDs
    auto release_slot = [slot] {
      if (slot && slot->owns_lock()) slot->unlock();
    };
    lk.lock();
    sum_dp_relock_ += now_s() - tp1;  // taking the agent's lock back after the Allocate (pod watch, pod workers)
    dp_calls_++;
    sum_dp_slot_ += ts - tp0;  // waiting for the admission slot (another pod's calls)
    sum_dp_pref_ += tpref - ts;
    sum_dp_alloc_ += tp1 - tpref;
    sum_dp_enc_ += tenc;
    if (prev_done > 0 && ts - prev_done < 0.002) {  // back to back: from the last admission's end to this one's calls
      sum_dp_gap_ += ts - prev_done;
      sum_gap_loop_ += te - prev_done;
      sum_gap_list_ += tl - te;
      sum_gap_handoff_ += ts - tl;
      n_dp_gap_++;
      if (admit_kept_) {
        sum_gap_kept_ += ts - prev_done;
        n_gap_kept_++;
      }
    }
    state_->set_inflight(my_uid, false);
    if (!ok) {
      failed_++;
      release_slot();
      std::fprintf(stderr, "[gsx-nodeagent] Allocate for %s failed: %d %s\n", key.c_str(), st, err.c_str());
      lk.unlock();
      std::string stj = "{\"status\":{\"phase\":\"Failed\",\"reason\":\"UnexpectedAdmissionError\",\"message\":";
      json::append_quoted(&stj, "Allocate failed: " + err);
      stj.append("}}");
      patch_status("/api/v1/namespaces/" + mine_ns(my_key) + "/pods/" + mine_name(my_key), stj);
      lk.lock();
      return;
    }
    const dp::ContainerResponse& cr = crs[0];
    // kubelet never re-routes an allocation: the container of the pod it admitted starts with whatever the plugin
    // answered.  An answer built for another pod (the plugin names it in the gpushare.amd.com/pod container
    // annotation) is a swap the plugin repairs from this agent's PodResources record, as under a real kubelet
    std::string who = cr.annotations.count("gpushare.amd.com/pod") ? cr.annotations.at("gpushare.amd.com/pod") : "";
    size_t cut = who.rfind('/');
    if (cut != std::string::npos && who.substr(cut + 1) != my_uid) {
      mismatch_++;
      std::fprintf(stderr, "[gsx-nodeagent] %s admitted with the allocation built for %s\n", my_key.c_str(),
                   who.c_str());
    }
    auto kit = keys_.find(my_key);
    if (running_.count(my_uid) || kit == keys_.end() || kit->second != my_uid) {  // gone meanwhile
      release_slot();
      return;
    }
    used_ids_[my_uid] = chosen[0];
    uid_key_[my_uid] = my_key;
    mark_used_locked(chosen[0], 1);  // recorded before the next admission: it is never offered these IDs
    last_admitted_ = now_s();
    auto idx = cr.envs.find(p_.a_idx);
    const int dev_idx = idx == cr.envs.end() ? -1 : std::atoi(idx->second.c_str());
    if (!devices_.count(dev_idx)) {
      forget_ids_locked(my_uid);
      return;
    }
    state_->set_inflight(my_uid, true);
    // a pod worker starts the container (reading the plugin's answer there, off the admission path); this worker
    // goes on with the next admission (it keeps the slot) and wakes a pod worker once it has let go of the lock
    starts_.push_back([this, my_key, my_uid, units, dev_idx, cr = std::move(crs[0]), t0, tp0,
                       tp1](std::unique_lock<std::mutex>& l) {
      std::vector<int> cus;
      auto cm = cr.envs.find("GSX_CU_MASK");
      if (cm != cr.envs.end()) {
        try {
          cus = parse_cu_words(cm->second);
        } catch (const std::exception&) {
          cus.clear();
        }
      }
      // the container's share is what the plugin's env says it got (SHARED_GPU_MEM_CONTAINER)
      auto ce = cr.envs.find(p_.env_container);
      const int64_t request = ce == cr.envs.end() ? units : std::max<int64_t>(1, std::atoll(ce->second.c_str()));
      start_pod_locked(my_key, my_uid, request, dev_idx, cus, allocation_json(cr),
                       "/api/v1/namespaces/" + mine_ns(my_key) + "/pods/" + mine_name(my_key), t0, tp0, tp1, l);
    });
    start_queued_ = true;
  }

  // the spawned plugin's /healthz, /metrics and /debug/state (its reconciliation and endpoint counters)
  std::string plugin_debug_url() {
    if (plugin_debug_url_.empty() && !plugin_debug_file_.empty()) {
      std::ifstream f(plugin_debug_file_);
      int port = 0;
      if (f >> port && port > 0) plugin_debug_url_ = "http://127.0.0.1:" + std::to_string(port);
    }
    return plugin_debug_url_;
  }

  void mark_used_locked(const std::vector<std::string>& ids, char used) {
    for (const auto& id : ids) {
      auto it = id_index_.find(id);
      if (it != id_index_.end()) id_used_[it->second] = used;
    }
  }

  void forget_ids_locked(const std::string& uid) {
    auto ui = used_ids_.find(uid);
    if (ui != used_ids_.end()) {
      mark_used_locked(ui->second, 0);
      used_ids_.erase(ui);
    }
    uid_key_.erase(uid);
  }

  // ---------------------------------------------------------------- kubelet's PodResources API (v1 List / Get)
  // What kubelet's device manager recorded: the device IDs each admitted container holds, until the pod goes.
  bool pr_start(std::string* err) {
    pr_srv_ = std::make_unique<h2::Server>(pr_sock_, [this](h2::Server& s, const h2::Call& c) { pr_call(s, c); });
    if (!pr_srv_->ok()) {
      *err = "PodResources endpoint: " + pr_srv_->init_error();
      return false;
    }
    pr_thread_ = std::thread([this] {
      introspect::name_thread("na-podres");
      const int ep = pr_srv_->fd();
      while (!pr_stop_.load()) {
        pollfd pf{ep, POLLIN, 0};
        ::poll(&pf, 1, 100);
        pr_srv_->poll();
      }
    });
    return true;
  }

  void pr_stop() {
    if (!pr_thread_.joinable()) return;
    pr_stop_.store(true);
    pr_thread_.join();
    pr_srv_.reset();
  }

  void pr_call(h2::Server& s, const h2::Call& call) {
    pr_calls_.fetch_add(1);
    const std::string svc = "/v1.PodResourcesLister/";
    if (call.path.compare(0, svc.size(), svc) != 0) {
      s.respond(call.id, 12, "unknown service " + call.path);
      return;
    }
    const std::string m = call.path.substr(svc.size());
    if (m == "GetAllocatableResources") {
      s.respond(call.id, 0, std::string());
      return;
    }
    if (m != "List") {
      s.respond(call.id, 12, "unknown method " + m);
      return;
    }
    std::vector<dp::PodDevicesMsg> out;
    {
      std::lock_guard<std::mutex> g(mu_);
      out.reserve(used_ids_.size());
      for (const auto& kv : used_ids_) {
        auto k = uid_key_.find(kv.first);
        if (k == uid_key_.end()) continue;
        dp::PodDevicesMsg e;
        e.ns = mine_ns(k->second);
        e.name = mine_name(k->second);
        e.container = "main";
        e.resource = p_.resource;
        e.ids = kv.second;
        out.push_back(std::move(e));
      }
      for (const auto& kv : stopping_) {  // containers of deleted pods the runtime has not stopped yet
        dp::PodDevicesMsg e;
        e.ns = mine_ns(kv.second.first);
        e.name = mine_name(kv.second.first);
        e.container = "main";
        e.resource = p_.resource;
        e.ids = kv.second.second;
        out.push_back(std::move(e));
      }
    }
    s.respond(call.id, 0, dp::encode_pod_resources_list(out));
  }

  static std::string mine_ns(const std::string& key) { return key.substr(0, key.find('/')); }
  static std::string mine_name(const std::string& key) { return key.substr(key.find('/') + 1); }

  void admit_locked(std::string key, std::unique_lock<std::mutex>& lk, std::unique_lock<std::mutex>* slot) {
    if (dp_) {
      admit_via_plugin_locked(std::move(key), lk, slot);
      return;
    }
    const AllocPod* mine = state_->pod_by_key(key);
    if (!mine) return;
    std::string uid = mine->uid;
    if (running_.count(uid) || state_->inflight(uid)) return;
    const int64_t units = mine->request;
    // kubelet's Allocate(N ids), answered by the device plugin's matcher: the earliest-ASSUME_TIME unassigned
    // pod of that size
    auto m = state_->match(units);
    if (!m.first) return;
    const AllocPod pod = *m.first;
    if (pod.uid != uid) {
      // an earlier same-size pod wins this Allocate; ours is served by the next one
      queued_.insert(uid);
      queue_.push_back(key);
      ++added_;
      wake_locked();
      key = pod.key;
      uid = pod.uid;
    }
    state_->set_inflight(uid, true);
    double t0 = seen_.count(uid) ? seen_[uid] : now_s();
    int dev_idx = static_cast<int>(pod.dev);
    const Device dev = devices_.at(dev_idx);
    std::vector<int> cus;
    CuPartitioner* cp = state_->cus(dev_idx);
    const bool had_cus = cp && cp->holds(uid);
    {
      std::string e;
      if (!state_->claim_cus(uid, &cus, &e)) {
        std::fprintf(stderr, "[gsx-nodeagent] %s: %s\n", key.c_str(), e.c_str());
        state_->set_inflight(uid, false);
        return;
      }
    }
    std::string envs = build_envs_locked(pod, dev, cus);
    lk.unlock();

    // commit point: ASSIGNED=true guarded by the resourceVersion we decided on
    std::string patch = "{\"metadata\":{\"resourceVersion\":";
    json::append_quoted(&patch, pod.rv);
    patch.append(",\"annotations\":{");
    json::append_quoted(&patch, p_.a_assigned);
    patch.append(":\"true\",");
    json::append_quoted(&patch, kAssignTimeAnn);
    patch.append(":\"").append(std::to_string(unix_ns())).append("\"");
    if (!cus.empty()) {
      patch.push_back(',');
      json::append_quoted(&patch, kCuMaskAnn);
      patch.push_back(':');
      json::append_quoted(&patch, cu_words(cus, dev.cu));
    }
    patch.append("}}}");
    std::string path = "/api/v1/namespaces/" + pod.ns + "/pods/" + pod.name;
    int status = 0;
    std::string resp, err;
    double tp0 = now_s();
    bool ok = api_.request("PATCH", path, patch, "application/merge-patch+json", &status, &resp, &err);
    double tp1 = now_s();
    if (slot && slot->owns_lock()) {  // the Allocate (its commit) is done: the next admission may go
      slot->unlock();
      cv_.notify_one();
    }
    if (!ok || status >= 300) {
      lk.lock();
      if (!cus.empty() && !had_cus && cp) cp->release(uid);
      state_->set_inflight(uid, false);
      // 409: stale copy, retry from the informer's latest version; 5xx / transport: the apiserver is
      // unhealthy, retry with backoff (kubelet retries Allocate-time failures the same way); 4xx: give up
      const bool retry = !ok || status == 409 || status >= 500;
      if (ok && status == 409) conflicts_++;
      if (retry && !queued_.count(uid)) {
        int& n = assign_retries_[uid];
        n++;
        queued_.insert(uid);
        delayed_.push_back({now_s() + std::min(0.2, 0.001 * (1 << std::min(n, 8))), key});
      }
      if (!retry || (ok && status >= 500)) {
        std::fprintf(stderr, "[gsx-nodeagent] ASSIGNED patch of %s failed: %s %d %s\n", key.c_str(), err.c_str(),
                     status, resp.substr(0, 200).c_str());
      }
      return;
    }
    // a container runtime tears down before it starts: every release already decided for this GPU
    // reaches the runtime before this pod's slice is carved (the next wave's pods may be bound the
    // moment the extender's ledger frees the device, while another worker is still releasing)
    // the PATCH answered the committed pod: the matcher sees ASSIGNED=true now, not when the watch event comes
    // (until then it would still offer this pod to the next Allocate, whose commit would fail on the stale rv)
    AllocPod committed;
    json::Doc cd;
    std::string cerr;
    bool have = cd.parse(resp, &cerr) && parse_alloc_pod(cd, 0, p_, &committed);
    lk.lock();
    if (have) state_->observe(committed);
    state_->first_container_committed(uid, units, true);
    start_pod_locked(key, uid, pod.request, dev_idx, cus, envs, path, t0, tp0, tp1, lk);
  }

  // Start a pod whose Allocate is done on its GPU's runtime (slice stamped + every resident slice verified), then
  // report it Running.  mu_ held on entry and exit.
  void start_pod_locked(const std::string& key, const std::string& uid, int64_t request, int dev_idx,
                        const std::vector<int>& cus, const std::string& envs, const std::string& path, double t0,
                        double tp0, double tp1, std::unique_lock<std::mutex>& lk) {
    CuPartitioner* cp = state_->cus(dev_idx);
    drain_releases_locked(dev_idx, lk);
    lk.unlock();
    // start the pod on its GPU's runtime: slice stamped + every resident slice verified
    std::string body ="{\"dev\":" + std::to_string(dev_idx) + ",\"bytes\":" + std::to_string(request * unit_) +
                       ",\"cus\":";
    if (cus.empty()) {
      body.append("null");
    } else {
      body.push_back('[');
      for (size_t i = 0; i < cus.size(); ++i) {
        if (i) body.push_back(',');
        body.append(std::to_string(cus[i]));
      }
      body.push_back(']');
    }
    body.append(",\"verify\":").append(verify_ ? "true" : "false").append("}");
    std::string rresp;
    int rst = runtime_call(dev_idx, "POST", "/v1/pods/" + uid, body, &rresp);
    double tp2 = now_s();
    int64_t bad = 0;
    std::string why;
    if (rst != 200) {
      why = "runtime HTTP " + std::to_string(rst) + ": " + rresp.substr(0, 200);
    } else {
      json::Doc d;
      std::string perr;
      if (d.parse(rresp, &perr)) {
        int64_t b = d.find(0, "bad");
        if (b >= 0) d.as_int(static_cast<uint32_t>(b), &bad);
      }
      if (bad) why = std::to_string(bad) + " bad HBM stamps after admitting " + key;
    }
    if (!why.empty()) {
      lk.lock();
      if (rst == 409) {  // what this agent believes the GPU holds, next to the runtime's refusal
        int64_t sum = 0;
        std::string who;
        for (const auto& kv : running_) {
          if (kv.second != dev_idx) continue;
          auto b = running_bytes_.find(kv.first);
          const int64_t n = b == running_bytes_.end() ? -1 : b->second / unit_;
          sum += n;
          who += " " + kv.first.substr(0, 8) + ":" + std::to_string(n);
        }
        size_t rel = 0;
        for (const auto& r : releases_) rel += r.second == dev_idx;
        why += " (agent: " + std::to_string(sum) + " units running on GPU " + std::to_string(dev_idx) + ":" + who +
               "; " + std::to_string(rel) + " releases queued, " + std::to_string(releasing_[dev_idx]) + " in flight)";
      }
      failed_++;
      bad_ += static_cast<uint64_t>(bad);
      if (!cus.empty() && cp) cp->release(uid);
      state_->set_inflight(uid, false);
      forget_ids_locked(uid);
      lk.unlock();
      if (rst == 200) runtime_call(dev_idx, "DELETE", "/v1/pods/" + uid, std::string(), nullptr);
      std::fprintf(stderr, "[gsx-nodeagent] admission of %s on GPU %d failed: %s\n", key.c_str(), dev_idx, why.c_str());
      std::string st = "{\"status\":{\"phase\":\"Failed\",\"reason\":\"UnexpectedAdmissionError\",\"message\":";
      json::append_quoted(&st, why);
      st.append("}}");
      patch_status(path, st);
      lk.lock();
      return;
    }
    lk.lock();
    running_[uid] = dev_idx;
    running_bytes_[uid] = request * unit_;
    allocations_[uid] = envs;
    admitted_++;
    lk.unlock();
    patch_status(path, "{\"status\":{\"phase\":\"Running\"}}");
    double tp3 = now_s();
    lk.lock();
    max_patch_ = std::max(max_patch_, tp1 - tp0);
    max_runtime_ = std::max(max_runtime_, tp2 - tp1);
    max_status_ = std::max(max_status_, tp3 - tp2);
    max_queue_ = std::max(max_queue_, tp0 - t0);
    sum_queue_ += tp0 - t0;
    sum_patch_ += tp1 - tp0;
    sum_runtime_ += tp2 - tp1;
    sum_status_ += tp3 - tp2;
    latency_.push_back(now_s() - t0);
    if (latency_.size() > 100000) latency_.erase(latency_.begin(), latency_.begin() + 50000);
    seen_.erase(uid);
    state_->set_inflight(uid, false);
    assign_retries_.erase(uid);
    // deleted while we were admitting: release now
    auto pk = keys_.find(key);
    if (pk == keys_.end() || pk->second != uid) {
      stop_pod_locked(uid);
      state_->release(uid);
    }
    wake_locked();
  }

  // kubelet's status manager: a pod status update is retried until the apiserver takes it (409 / 5xx /
  // transport errors), with capped backoff; 404 (pod gone) ends it.  mu_ not held.
  void patch_status(const std::string& path, const std::string& body) {
    for (int attempt = 0; attempt < 50 && !stop_flag_.load(); ++attempt) {
      int status = 0;
      std::string resp, err;
      bool ok = api_.request("PATCH", path + "/status", body, "application/merge-patch+json", &status, &resp, &err);
      if (ok && (status < 300 || status == 404 || (status >= 400 && status < 500 && status != 409 && status != 429)))
        return;
      status_retries_.fetch_add(1);
      std::this_thread::sleep_for(std::chrono::microseconds(std::min(100000, 500 << std::min(attempt, 8))));
    }
  }

  // The end of a graceful deletion, as kubelet does it: the containers have stopped (runtime slice released), the
  // terminal phase is reported, and the object is deleted with grace 0 under a UID precondition (a pod re-created
  // under the same name is not touched).  mu_ held on entry and exit, dropped around the API calls.
  void finalize_locked(const Final& f, std::unique_lock<std::mutex>& lk) {
    const double t0 = now_s();
    sum_fin_wake_ += std::max(0.0, t0 - f.due);
    stop_pod_locked(f.uid);
    for (auto it = releases_.begin(); it != releases_.end(); ++it) {
      if (it->first != f.uid) continue;
      auto rel = *it;
      releases_.erase(it);
      release_one(rel, lk);
      break;
    }
    finals_done_++;
    const double t1 = now_s();
    sum_fin_release_ += t1 - t0;
    lk.unlock();
    const std::string path = "/api/v1/namespaces/" + f.ns + "/pods/" + f.name;
    if (f.ran) patch_status(path, "{\"status\":{\"phase\":\"Succeeded\"}}");
    const double t2 = now_s();
    std::string body = "{\"kind\":\"DeleteOptions\",\"apiVersion\":\"v1\",\"gracePeriodSeconds\":0,"
                       "\"preconditions\":{\"uid\":";
    json::append_quoted(&body, f.uid);
    body.append("}}");
    for (int attempt = 0; attempt < 50 && !stop_flag_.load(); ++attempt) {
      int status = 0;
      std::string resp, err;
      bool ok = api_.request("DELETE", path, body, "application/json", &status, &resp, &err);
      // 409: the UID precondition failed (another pod has the name now); 404: already gone
      if (ok && (status < 300 || status == 404 || status == 409 || (status >= 400 && status < 500 && status != 429)))
        break;
      status_retries_.fetch_add(1);
      std::this_thread::sleep_for(std::chrono::microseconds(std::min(100000, 500 << std::min(attempt, 8))));
    }
    lk.lock();
    sum_fin_status_ += t2 - t1;
    sum_fin_delete_ += now_s() - t2;
  }

  // DELETE a pod's slice on its runtime; mu_ held on entry and exit, dropped around the call.
  void release_one(const std::pair<std::string, int>& rel, std::unique_lock<std::mutex>& lk) {
    releasing_[rel.second]++;
    lk.unlock();
    runtime_call(rel.second, "DELETE", "/v1/pods/" + rel.first, std::string(), nullptr);
    lk.lock();
    auto st = stopping_.find(rel.first);
    if (st != stopping_.end()) {
      mark_used_locked(st->second.second, 0);
      stopping_.erase(st);
    }
    if (--releasing_[rel.second] == 0) cv_.notify_all();
  }

  // Run this GPU's queued releases on the calling worker and wait for the ones other workers have in
  // flight (they never wait on anything, so this cannot deadlock); mu_ held.
  void drain_releases_locked(int dev, std::unique_lock<std::mutex>& lk) {
    while (true) {
      auto it = std::find_if(releases_.begin(), releases_.end(), [dev](const auto& r) { return r.second == dev; });
      if (it != releases_.end()) {
        auto rel = *it;
        releases_.erase(it);
        release_one(rel, lk);
        continue;
      }
      if (releasing_[dev] == 0 || stop_) return;
      cv_.wait(lk);
    }
  }

  int runtime_call(int dev, const char* method, const std::string& path, const std::string& body, std::string* out) {
    auto it = runtimes_.find(dev);
    if (it == runtimes_.end()) return -1;
    int status = 0;
    std::string resp, err;
    if (!it->second->request(method, path, body, "application/json", &status, &resp, &err)) return -1;
    if (out) *out = std::move(resp);
    return status;
  }

  ApiConfig api_cfg_;
  std::string node_;
  Profile p_;
  int64_t unit_;
  int nworkers_;
  bool verify_;  // (mu_) POST /v1/config
  bool serial_admission_ = false;  // set_serial_admission
  ApiClient api_;
  std::map<int, Device> devices_;
  std::unique_ptr<AllocState> state_;  // the device plugin's matcher (allocstate.h)
  std::string plugin_sock_;             // --plugin-socket: Allocate through the shipped plugin (gRPC)
  std::string spawn_python_, spawn_api_, spawn_profile_, spawn_unit_;  // --plugin-spawn: run that plugin ourselves
  pid_t plugin_pid_ = -1;
  std::unique_ptr<h2::Client> dp_;
  std::mutex dp_mu_;
  std::vector<std::string> all_ids_;
  std::unordered_map<std::string, std::vector<std::string>> used_ids_;  // uid -> the IDs its Allocate took
  std::unordered_map<std::string, size_t> id_index_;                     // ID -> its place in all_ids_
  std::vector<std::string> id_field_;  // per all_ids_ entry: the ID encoded as GetPreferredAllocation's field 1
  std::string id_fields_;                // the same fields back to back, in all_ids_ order
  std::vector<size_t> id_field_off_;     // entry i's field starts at id_field_off_[i] (size all_ids_ + 1)
  bool start_queued_ = false;          // starts_ got a pod no pod worker was woken for yet
  std::vector<char> id_used_;  // per all_ids_ entry: held by a running container (the union of used_ids_)
  std::unordered_map<std::string, std::string> uid_key_;                 // uid -> ns/name of every used_ids_ pod
  std::string pr_sock_;                    // kubelet's PodResources API socket (with --plugin-spawn)
  std::string plugin_debug_file_, plugin_debug_url_;
  std::unordered_map<std::string, int64_t> running_bytes_;  // uid -> bytes its slice was carved with
  bool preferred_ = false;  // the plugin advertises GetPreferredAllocation
  std::unique_ptr<h2::Server> pr_srv_;
  std::thread pr_thread_;
  std::atomic<bool> pr_stop_{false};
  std::atomic<uint64_t> pr_calls_{0};
  uint64_t mismatch_ = 0;  // admissions answered with an allocation built for another pod (swaps)
  double batch_window_ = 0;  // --batch-window: > 0 admits the pods met within it as one creationTimestamp batch
  double batch_deadline_ = 0;
  std::vector<std::pair<std::string, std::string>> batch_;  // (creationTimestamp, ns/name) of the open batch
  std::unordered_map<std::string, std::string> keys_;  // ns/name -> uid of every pod the informer delivered
  std::map<int, std::unique_ptr<ApiClient>> runtimes_;
  std::unique_ptr<Reflector> pods_r_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::condition_variable park_cv_;  // workers past target_workers_ wait here
  size_t target_workers_ = 1;
  bool stop_ = false;
  std::unordered_map<std::string, int> running_;
  std::unordered_set<std::string> queued_;
  std::unordered_map<std::string, double> seen_;
  std::unordered_map<std::string, std::string> allocations_;
  std::deque<std::string> queue_;
  std::deque<std::function<void(std::unique_lock<std::mutex>&)>> starts_;  // admitted pods to start (pod workers)
  std::vector<std::pair<double, std::string>> delayed_;
  std::deque<std::pair<std::string, int>> releases_;
  std::vector<Final> finals_;                 // graceful deletions to end (finalize_locked)
  // uid -> (ns/name, device IDs) of stopped pods whose runtime slice is still being released
  std::unordered_map<std::string, std::pair<std::string, std::vector<std::string>>> stopping_;
  std::unordered_set<std::string> finals_set_;
  uint64_t finals_done_ = 0;
  // where a graceful deletion's end goes (seconds summed over finals_done_): the event to a worker, the container
  // stop (runtime release), the terminal-phase report, the grace-0 delete
  double sum_fin_wake_ = 0, sum_fin_release_ = 0, sum_fin_status_ = 0, sum_fin_delete_ = 0;
  double stop_delay_ = 0;
  std::map<int, int> releasing_;  // per GPU: DELETEs in flight on some worker
  std::unordered_map<std::string, int> assign_retries_;  // per pod: ASSIGNED patch attempts (backoff)
  std::atomic<uint64_t> status_retries_{0};
  std::atomic<bool> stop_flag_{false};
  std::atomic<bool> ready_{false};
  std::vector<double> latency_;
  uint64_t admitted_ = 0, failed_ = 0, bad_ = 0, conflicts_ = 0;
  int added_ = 0;  // work items queued since the last wake_locked()
  // worst case per admission step (seconds): queue wait, ASSIGNED patch, runtime admit, Running patch
  double max_queue_ = 0, max_patch_ = 0, max_runtime_ = 0, max_status_ = 0;
  double sum_queue_ = 0, sum_patch_ = 0, sum_runtime_ = 0, sum_status_ = 0;  // over admitted_ pods
  uint64_t dp_calls_ = 0;  // GetPreferredAllocation + Allocate pairs to the plugin (--plugin-socket / --plugin-spawn)
  double sum_dp_slot_ = 0, sum_dp_pref_ = 0, sum_dp_alloc_ = 0, sum_dp_enc_ = 0, sum_dp_gap_ = 0;
  // the gap split: record + start queued + worker loop + pop (loop), free-ID list (list), unlock + wake (handoff)
  double sum_gap_loop_ = 0, sum_gap_list_ = 0, sum_gap_handoff_ = 0, sum_dp_relock_ = 0;
  // back-to-back admissions by the worker that kept the slot (no queue-empty release in between)
  double sum_gap_kept_ = 0;
  uint64_t n_gap_kept_ = 0;
  bool admit_kept_ = false;
  uint64_t n_dp_gap_ = 0;
  double last_admitted_ = 0;  // when the last admission's IDs were recorded
  std::vector<std::thread> workers_;
};

volatile sig_atomic_t g_stop = 0;
void on_sig(int) { g_stop = 1; }

}  // namespace

int main(int argc, char** argv) {
  std::string apiserver, node, profile = "shared-gpu", unit = "GiB", port_file, host = "127.0.0.1", plugin_socket, plugin_python;
  int workers = 16, port = 0;
  double batch_window = 0, stop_delay = 0;
  bool verify = true, serial = false;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto val = [&](const char* name) -> std::string {
      if (i + 1 >= argc) {
        std::fprintf(stderr, "missing value for %s\n", name);
        std::exit(2);
      }
      return argv[++i];
    };
    if (a == "--apiserver") apiserver = val("--apiserver");
    else if (a == "--node") node = val("--node");
    else if (a == "--profile") profile = val("--profile");
    else if (a == "--unit") unit = val("--unit");
    else if (a == "--workers") workers = std::max(1, std::min(128, std::atoi(val("--workers").c_str())));
    else if (a == "--no-verify") verify = false;
    else if (a == "--serial-admission") serial = true;
    else if (a == "--port") port = std::atoi(val("--port").c_str());
    else if (a == "--port-file") port_file = val("--port-file");
    else if (a == "--plugin-socket") plugin_socket = val("--plugin-socket");
    else if (a == "--plugin-spawn") plugin_python = val("--plugin-spawn");
    else if (a == "--batch-window") batch_window = std::atof(val("--batch-window").c_str());
    else if (a == "--stop-delay") stop_delay = std::atof(val("--stop-delay").c_str());
    else if (a == "-h" || a == "--help") {
      std::printf("usage: gsx-nodeagent --apiserver URL --node NAME [--profile P] [--unit GiB|MiB] [--workers N]\n"
                  "                     [--no-verify] [--serial-admission] [--port P] [--port-file F]\n"
                  "                     [--plugin-socket S | --plugin-spawn PYTHON] [--batch-window SECONDS]\n"
                  "                     [--stop-delay SECONDS]\n");
      return 0;
    } else {
      std::fprintf(stderr, "unknown argument %s\n", a.c_str());
      return 2;
    }
  }
  if (apiserver.empty() || node.empty()) {
    std::fprintf(stderr, "--apiserver and --node are required\n");
    return 2;
  }
  int64_t unit_bytes = unit == "MiB" ? (1ll << 20) : unit == "GB" ? 1000000000ll : unit == "MB" ? 1000000ll : (1ll << 30);
  signal(SIGPIPE, SIG_IGN);
  struct sigaction sa;
  std::memset(&sa, 0, sizeof(sa));
  sa.sa_handler = on_sig;
  sigaction(SIGTERM, &sa, nullptr);
  sigaction(SIGINT, &sa, nullptr);
  ApiConfig api;
  api.server = apiserver;
  Agent agent(api, node, profile_by_name(profile), unit_bytes, workers, verify);
  agent.set_plugin_socket(plugin_socket);
  agent.set_serial_admission(serial);
  agent.set_batch_window(batch_window);
  agent.set_stop_delay(stop_delay);
  if (!plugin_python.empty()) agent.set_plugin_spawn(plugin_python, apiserver, profile, unit);
  std::string err;
  CtlServer srv([&](const http::Message& m) { return agent.handle(m); });
  int bound = srv.start(host, port, &err);
  if (bound < 0) {
    std::fprintf(stderr, "gsx-nodeagent: %s\n", err.c_str());
    return 1;
  }
  // readiness for the process harness: published before waiting for the node's inventory
  if (!port_file.empty()) {
    std::string tmp = port_file + ".tmp";
    {
      std::ofstream f(tmp);
      f << bound;
    }
    std::rename(tmp.c_str(), port_file.c_str());
  }
  if (!agent.load_devices(600, &err) || !agent.start(&err)) {
    std::fprintf(stderr, "gsx-nodeagent: %s\n", err.c_str());
    srv.stop();
    return 1;
  }
  while (!g_stop) ::usleep(20000);
  srv.stop();
  agent.stop();
  return 0;
}
