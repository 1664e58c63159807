// pybind11 bindings for the native ledger engine (module `_engine`).
//
// The Python control plane (asyncio I/O) owns no scheduling state: every
// filter/bind decision and all accounting happen here, behind one mutex.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <poll.h>
#include <pthread.h>
#include <sched.h>
#include <sys/eventfd.h>
#include <sys/timerfd.h>
#include <time.h>
#include <unistd.h>

#include <condition_variable>
#include <deque>
#include <memory>
#include <map>
#include <mutex>
#include <thread>

#include "allocstate.h"
#include "dpcore.h"
#include "h2.h"
#include "introspect.h"
#include "ledger.h"
#include "quantity.h"
#include "controller.h"
#include "server.h"
#include "tracker.h"
#include "podruntime.h"

namespace py = pybind11;
using namespace gsx;

namespace {

Profile profile_from(const py::dict& d) {
  Profile p;
  auto get = [&](const char* k, std::string* dst) {
    if (d.contains(k)) *dst = d[k].cast<std::string>();
  };
  get("resource", &p.resource);
  get("count", &p.count);
  get("annotation_idx", &p.a_idx);
  get("annotation_pod", &p.a_pod);
  get("annotation_dev", &p.a_dev);
  get("annotation_assigned", &p.a_assigned);
  get("annotation_assume_time", &p.a_assume);
  get("annotation_node_devices", &p.a_node_devs);
  get("env_container", &p.env_container);
  return p;
}

std::string_view view_of(const py::bytes& b) {
  char* buf;
  Py_ssize_t len;
  if (PyBytes_AsStringAndSize(b.ptr(), &buf, &len) != 0) throw py::error_already_set();
  return std::string_view(buf, static_cast<size_t>(len));
}

bool parse_pod_bytes(const py::bytes& b, const Profile& p, PodView* out, std::string* err) {
  json::Doc d;
  if (!d.parse(view_of(b), err)) return false;
  // accept either a bare pod or a watch event {"type":..,"object":pod}
  uint32_t root = 0;
  int64_t obj = d.find(0, "object");
  if (obj >= 0 && d.find(0, "type") >= 0) root = static_cast<uint32_t>(obj);
  if (!parse_pod(d, root, p, out)) {
    *err = "not a pod object";
    return false;
  }
  return true;
}

bool parse_node_bytes(const py::bytes& b, const Profile& p, NodeView* out, std::string* err) {
  json::Doc d;
  if (!d.parse(view_of(b), err)) return false;
  uint32_t root = 0;
  int64_t obj = d.find(0, "object");
  if (obj >= 0 && d.find(0, "type") >= 0) root = static_cast<uint32_t>(obj);
  if (!parse_node(d, root, p, out)) {
    *err = "not a node object";
    return false;
  }
  return true;
}

ApiConfig api_from(const py::dict& api) {
  ApiConfig c;
  auto get = [&](const char* k, std::string* dst) {
    if (api.contains(k) && !api[k].is_none()) *dst = api[k].cast<std::string>();
  };
  get("server", &c.server);
  get("token", &c.token);
  get("token_file", &c.token_file);
  if (api.contains("token_reload_s")) c.token_reload_s = api["token_reload_s"].cast<double>();
  get("ca_file", &c.ca_file);
  get("cert_file", &c.cert_file);
  get("key_file", &c.key_file);
  if (api.contains("insecure")) c.insecure = api["insecure"].cast<bool>();
  return c;
}

class Engine {
 public:
  explicit Engine(const py::dict& profile) : l_(profile_from(profile)) {}

  py::dict profile() const {
    const Profile& p = l_.profile();
    py::dict d;
    d["resource"] = p.resource;
    d["count"] = p.count;
    d["annotation_idx"] = p.a_idx;
    d["annotation_pod"] = p.a_pod;
    d["annotation_dev"] = p.a_dev;
    d["annotation_assigned"] = p.a_assigned;
    d["annotation_assume_time"] = p.a_assume;
    d["annotation_node_devices"] = p.a_node_devs;
    return d;
  }

  bool upsert_node(const std::string& name, int64_t total, int64_t count, std::vector<int64_t> devs,
                   const std::string& address) {
    NodeView nv;
    nv.name = name;
    nv.total = total;
    nv.count = count;
    nv.dev_totals = std::move(devs);
    nv.address = address;
    std::lock_guard<introspect::ProfiledMutex> g(l_.mu());
    return l_.upsert_node(nv);
  }

  py::tuple upsert_node_json(const py::bytes& b) {
    NodeView nv;
    std::string err;
    if (!parse_node_bytes(b, l_.profile(), &nv, &err)) throw py::value_error(err);
    bool rebuilt;
    {
      std::lock_guard<introspect::ProfiledMutex> g(l_.mu());
      rebuilt = l_.upsert_node(nv);
    }
    return py::make_tuple(nv.name, rebuilt);
  }

  bool remove_node(const std::string& name) {
    std::lock_guard<introspect::ProfiledMutex> g(l_.mu());
    return l_.remove_node(name);
  }

  bool has_node(const std::string& name) {
    std::lock_guard<introspect::ProfiledMutex> g(l_.mu());
    return l_.has_node(name);
  }

  py::tuple node_info(const std::string& name) {
    std::lock_guard<introspect::ProfiledMutex> g(l_.mu());
    const NodeState* n = l_.node(name);
    if (!n) return py::make_tuple();
    return py::make_tuple(n->total, n->count, n->address);
  }

  int upsert_pod(const PodView& v) {
    std::lock_guard<introspect::ProfiledMutex> g(l_.mu());
    return l_.upsert_pod(v);
  }

  bool remove_pod(const std::string& uid) {
    std::lock_guard<introspect::ProfiledMutex> g(l_.mu());
    return l_.remove_pod(uid);
  }

  bool known(const std::string& uid) {
    std::lock_guard<introspect::ProfiledMutex> g(l_.mu());
    return l_.known(uid);
  }

  py::tuple pod_state(const std::string& uid) {
    int64_t dev;
    int st;
    {
      std::lock_guard<introspect::ProfiledMutex> g(l_.mu());
      st = l_.pod_state(uid, &dev);
    }
    return py::make_tuple(st, dev);
  }

  // Upsert straight from a raw pod / watch-event JSON (informer fast path).
  int upsert_pod_json(const py::bytes& b) {
    PodView v;
    std::string err;
    if (!parse_pod_bytes(b, l_.profile(), &v, &err)) throw py::value_error(err);
    std::lock_guard<introspect::ProfiledMutex> g(l_.mu());
    return l_.upsert_pod(v);
  }

  int check(const std::string& node, int64_t req) {
    std::lock_guard<introspect::ProfiledMutex> g(l_.mu());
    return static_cast<int>(l_.check(node, req));
  }

  py::bytes filter(const py::bytes& body) {
    std::string_view v = view_of(body);
    std::string out;
    {
      py::gil_scoped_release rel;
      std::lock_guard<introspect::ProfiledMutex> g(l_.mu());
      out = filter_body(l_, v);
    }
    return py::bytes(out);
  }

  py::bytes prioritize(const py::bytes& body) {
    std::string_view v = view_of(body);
    std::string out;
    {
      py::gil_scoped_release rel;
      std::lock_guard<introspect::ProfiledMutex> g(l_.mu());
      out = prioritize_body(l_, v);
    }
    return py::bytes(out);
  }

  py::tuple assume(const std::string& uid, const std::string& ns, const std::string& name,
                   const std::string& node, int64_t req) {
    int64_t dev_total = -1;
    std::lock_guard<introspect::ProfiledMutex> g(l_.mu());
    int64_t dev = l_.assume(uid, ns, name, node, req, &dev_total);
    return py::make_tuple(dev, dev_total);
  }

  // (dev, dev_total, seq, assume_ns): reservation + ASSUME_TIME + entry in the shared bind-order set
  py::tuple assume_ordered(const std::string& uid, const std::string& ns, const std::string& name,
                           const std::string& node, int64_t req, const std::string& cu_count) {
    int64_t dev_total = -1, assume_ns = 0;
    uint64_t seq = 0;
    std::lock_guard<introspect::ProfiledMutex> g(l_.mu());
    int64_t dev = l_.assume_ordered(uid, ns, name, node, req, &dev_total, &seq, &assume_ns, cu_count);
    return py::make_tuple(dev, dev_total, seq, assume_ns);
  }

  bool bind_blocked(uint64_t seq) { return l_.bind_blocked(seq); }

  void bind_wait(uint64_t seq) {
    py::gil_scoped_release rel;
    l_.bind_wait(seq, nullptr);
  }

  void bind_leave(uint64_t seq) { l_.bind_leave(seq); }

  void finish_bind(const std::string& uid, bool ok, double ttl) {
    std::lock_guard<introspect::ProfiledMutex> g(l_.mu());
    l_.finish_bind(uid, ok, ttl);
  }

  // (expired, need_relist): see Ledger::gc; list_start is the start time of the last applied pod LIST
  py::tuple gc(double list_start) {
    bool need = false;
    int n;
    {
      std::lock_guard<introspect::ProfiledMutex> g(l_.mu());
      n = l_.gc(list_start, &need);
    }
    return py::make_tuple(n, need);
  }

  // (expired, relist_requested) with the native controller's pod reflector as the confirming LIST source
  py::tuple controller_gc() {
    if (!ctl_) return gc(0.0);
    bool need = false;
    int n;
    {
      py::gil_scoped_release rel;
      n = ctl_->gc_reservations(&need);
    }
    return py::make_tuple(n, need);
  }

  py::tuple inspect(const std::string& node) {
    bool found;
    std::string s;
    {
      std::lock_guard<introspect::ProfiledMutex> g(l_.mu());
      s = l_.inspect_json(node, &found);
    }
    return py::make_tuple(py::bytes(s), found);
  }

  std::vector<std::pair<int64_t, int64_t>> node_devices(const std::string& node) {
    std::lock_guard<introspect::ProfiledMutex> g(l_.mu());
    return l_.node_devices(node);
  }

  std::vector<int64_t> node_unaccounted(const std::string& node) {
    std::lock_guard<introspect::ProfiledMutex> g(l_.mu());
    return l_.node_unaccounted(node);
  }

  // The ledger halves of the device plugin's endpoints (server.cc do_move / do_physical run the same calls around
  // their apiserver write), for in-process protocol harnesses (tests/test_interleavings.py): (rc, to, why) -- rc as
  // Ledger::begin_move.
  py::tuple begin_move(const std::string& uid, const std::string& node, int64_t from, int64_t to,
                       const std::string& partner, bool physical_on_to, int64_t req_hold,
                       const std::string& req_hold_partner) {
    MoveRequest m;
    m.uid = uid;
    m.node = node;
    m.from = from;
    m.to = to;
    m.partner = partner;
    m.physical_on_to = physical_on_to;
    m.req_hold = req_hold;
    m.req_hold_partner = req_hold_partner;
    std::string why;
    int rc;
    {
      std::lock_guard<introspect::ProfiledMutex> g(l_.mu());
      rc = l_.begin_move(&m, &why);
    }
    return py::make_tuple(rc, m.to, why);
  }

  void end_move(const std::string& uid, bool ok) {
    std::lock_guard<introspect::ProfiledMutex> g(l_.mu());
    l_.end_move(uid, ok);
  }

  bool set_unaccounted(const std::string& node, const std::vector<int64_t>& extra, double ttl_s) {
    std::lock_guard<introspect::ProfiledMutex> g(l_.mu());
    return l_.set_unaccounted(node, extra, ttl_s);
  }

  void begin_epoch(double hold_s) {
    std::lock_guard<introspect::ProfiledMutex> g(l_.mu());
    l_.begin_epoch(hold_s);
  }

  double publication_wait(const std::string& node) {
    std::lock_guard<introspect::ProfiledMutex> g(l_.mu());
    return l_.publication_wait(node);
  }

  std::vector<std::string> node_names() {
    std::lock_guard<introspect::ProfiledMutex> g(l_.mu());
    return l_.node_names();
  }

  py::dict stats() {
    Stats s;
    size_t pods;
    {
      std::lock_guard<introspect::ProfiledMutex> g(l_.mu());
      s = l_.stats();
      pods = l_.pod_count();
    }
    py::dict d;
    d["filter_calls"] = s.filter_calls;
    d["filter_nodes_ok"] = s.filter_nodes_ok;
    d["filter_nodes_failed"] = s.filter_nodes_failed;
    d["assume_ok"] = s.assume_ok;
    d["assume_fail"] = s.assume_fail;
    d["bind_ok"] = s.bind_ok;
    d["bind_fail"] = s.bind_fail;
    d["expired"] = s.expired;
    d["expiry_deferred"] = s.expiry_deferred;
    d["annotations_missing"] = s.annotations_missing;
    d["moves_ok"] = s.moves_ok;
    d["moves_refused"] = s.moves_refused;
    d["partner_claims_refused"] = s.partner_claims_refused;
    d["unaccounted_updates"] = s.unaccounted_updates;
    d["unaccounted_expired"] = s.unaccounted_expired;
    d["moves_failed"] = s.moves_failed;
    d["overcommit_events"] = s.overcommit_events;
    d["pod_upserts"] = s.pod_upserts;
    d["pod_removes"] = s.pod_removes;
    d["pods"] = pods;
    // binds held back for ASSUME_TIME order, native and Python paths together
    d["bind_order_waits"] = l_.bind_order_waits();
    d["bind_order_wait_s"] = l_.bind_order_wait_s();
    return d;
  }

  // ---- native HTTP front end (server.h) ----
  int serve(const std::string& host, int port, int threads, int pool_threads, int fallback_port, double ttl,
            const py::dict& api, bool update_mode, double qps, int burst, const std::string& plugin_auth,
            const std::vector<std::string>& plugin_users) {
    if (srv_) throw std::runtime_error("native server already running");
    ServerConfig cfg;
    cfg.host = host;
    cfg.port = port;
    cfg.threads = threads;
    cfg.pool_threads = pool_threads;
    cfg.fallback_port = fallback_port;
    cfg.update_mode = update_mode;
    cfg.reservation_ttl = ttl;
    cfg.qps = qps;
    cfg.burst = burst;
    cfg.api = api_from(api);
    if (plugin_auth != "none" && plugin_auth != "tokenreview") throw std::invalid_argument("plugin_auth: none|tokenreview");
    cfg.plugin_auth = plugin_auth;
    cfg.plugin_users = plugin_users;
    if (const char* h = std::getenv("GSX_PUBLICATION_HOLD_S")) cfg.publication_hold_s = std::atof(h);
    srv_.reset(new NativeServer(&l_, cfg));
    // the controller outlives the server (stop_server runs before stop_controller)
    srv_->set_lister([this](const std::string& key, std::string* raw) { return ctl_ && ctl_->get_pod(key, raw); });
    srv_->set_binds_enabled(binds_enabled_);
    if (update_mode_) srv_->set_update_mode(true);
    std::string err;
    int p = srv_->start(&err);
    if (p < 0) {
      srv_.reset();
      throw std::runtime_error(err);
    }
    return p;
  }

  // ---- native controller (controller.h): reflectors -> ledger ----
  void start_controller(const py::dict& api, double resync_s, double sync_timeout_s, int watch_timeout_s) {
    if (ctl_) throw std::runtime_error("native controller already running");
    ControllerConfig cfg;
    cfg.api = api_from(api);
    cfg.resync_s = resync_s;
    cfg.watch_timeout_s = watch_timeout_s;
    ctl_.reset(new Controller(&l_, cfg));
    std::string err;
    bool ok;
    {
      py::gil_scoped_release rel;
      ok = ctl_->start(sync_timeout_s, &err);
    }
    if (!ok) {
      {
        py::gil_scoped_release rel;
        ctl_->stop();
      }
      ctl_.reset();
      throw std::runtime_error(err);
    }
  }

  void stop_controller() {
    if (ctl_) {
      py::gil_scoped_release rel;
      ctl_->stop();
    }
    ctl_.reset();
  }

  bool controller_synced() const { return ctl_ && ctl_->synced(); }

  py::object controller_get_pod(const std::string& key) {
    std::string raw;
    if (!ctl_ || !ctl_->get_pod(key, &raw)) return py::none();
    return py::bytes(raw);
  }

  py::list controller_overcommitted() {
    py::list out;
    if (!ctl_) return out;
    for (auto& t : ctl_->overcommitted()) {
      out.append(py::make_tuple(std::get<0>(t), std::get<1>(t), std::get<2>(t), std::get<3>(t)));
    }
    return out;
  }

  py::dict controller_stats() {
    py::dict d;
    if (!ctl_) return d;
    ControllerStats s = ctl_->stats();
    d["pod_events"] = s.pod_events;
    d["node_events"] = s.node_events;
    d["syncs"] = s.syncs;
    d["removes"] = s.removes;
    d["upserts"] = s.upserts;
    d["pod_lists"] = s.pod_lists;
    d["node_lists"] = s.node_lists;
    d["pod_rewatches"] = s.pod_watches;
    d["node_rewatches"] = s.node_watches;
    d["watch_errors"] = s.watch_errors;
    d["pod_list_pages"] = s.pod_list_pages;
    d["node_list_pages"] = s.node_list_pages;
    d["resyncs"] = s.resyncs;
    d["recovered"] = s.recovered;
    d["last_error"] = ctl_->last_error();
    return d;
  }

  void stop_server() {
    if (srv_) {
      py::gil_scoped_release rel;
      srv_->stop();
    }
    srv_.reset();
  }

  py::dict server_stats() {
    py::dict d;
    if (!srv_) return d;
    const ServerStats& s = srv_->stats();
    d["requests"] = s.requests.load();
    d["filters"] = s.filters.load();
    d["binds"] = s.binds.load();
    d["bind_order_waits"] = s.bind_order_waits.load();
    d["bind_order_wait_s"] = l_.bind_order_wait_s();
    d["bind_order_wait_max_s"] = l_.bind_order_wait_max_s();
    d["bind_ok"] = s.bind_ok.load();
    d["bind_fail"] = s.bind_fail.load();
    d["proxied"] = s.proxied.load();
    d["bad_requests"] = s.bad_requests.load();
    d["inspects"] = s.inspects.load();
    d["connections"] = s.connections.load();
    d["api_calls"] = s.api_calls.load();
    d["conflicts_retried"] = s.conflicts_retried.load();
    d["moves"] = s.moves.load();
    d["unfiltered_binds"] = s.unfiltered_binds.load();
    d["live_gets"] = s.live_gets.load();
    d["qps_waits"] = s.qps_waits.load();
    d["moves_failed"] = s.moves_failed.load();
    d["physical_posts"] = s.physical_posts.load();
    d["plugin_auth_denied"] = s.plugin_auth_denied.load();
    d["token_reviews"] = s.token_reviews.load();
    d["backoffs"] = s.backoffs.load();
    d["publication_waits"] = s.publication_waits.load();
    d["physical_refused"] = s.physical_refused.load();
    d["epoch"] = srv_->epoch();
    d["api_throttled"] = srv_->api_throttled();
    d["api_throttle_wait_s"] = srv_->api_throttle_wait_s();
    auto hist = [](const LatencyHist& h) {
      py::dict o;
      py::list bounds, counts;
      for (int i = 0; i < LatencyHist::kBuckets; ++i) bounds.append(LatencyHist::kBounds[i]);
      for (int i = 0; i <= LatencyHist::kBuckets; ++i) counts.append(h.counts[i].load());
      o["bounds"] = bounds;
      o["counts"] = counts;
      o["n"] = h.n.load();
      o["sum"] = static_cast<double>(h.sum_ns.load()) / 1e9;
      return o;
    };
    d["filter_latency"] = hist(s.filter_lat);
    d["bind_latency"] = hist(s.bind_lat);
    d["api_latency"] = hist(s.api_lat);
    return d;
  }

  // ---- introspection for /debug/pprof (introspect.h) ----
  py::dict ledger_mutex() {
    introspect::MutexStats m = l_.mu().stats();
    py::dict d;
    d["acquisitions"] = m.acquisitions;
    d["contended"] = m.contended;
    d["wait_s"] = m.wait_s;
    d["max_wait_s"] = m.max_wait_s;
    d["hold_s"] = m.hold_s;
    d["max_hold_s"] = m.max_hold_s;
    return d;
  }

  void set_binds_enabled(bool on) {
    binds_enabled_ = on;
    if (srv_) srv_->set_binds_enabled(on);
  }

  py::list drain_annotation_repairs() {
    std::vector<AnnotationRepair> rs;
    {
      std::lock_guard<introspect::ProfiledMutex> g(l_.mu());
      rs = l_.drain_repairs();
    }
    py::list out;
    for (auto& a : rs) {
      py::dict d;
      d["uid"] = a.uid;
      d["namespace"] = a.ns;
      d["name"] = a.name;
      d["node"] = a.node;
      d["dev"] = a.dev;
      d["dev_total"] = a.dev_total;
      d["mem"] = a.mem;
      d["assume_ns"] = a.assume_ns;
      out.append(d);
    }
    return out;
  }

  void set_bind_order(const std::string& m) {
    if (m == "auto") {
      l_.set_order_mode(Ledger::kOrderAuto);
    } else if (m == "strict") {
      l_.set_order_mode(Ledger::kOrderStrict);
    } else if (m == "relaxed") {
      l_.set_order_mode(Ledger::kOrderRelaxed);
    } else {
      throw py::value_error("bind order must be auto, strict or relaxed");
    }
  }
  std::string bind_order() const { return Ledger::order_mode_name(l_.order_mode()); }

  void set_update_mode(bool on) {
    update_mode_ = on;
    if (srv_) srv_->set_update_mode(on);
  }

  py::list drain_bind_failures() {
    py::list out;
    if (!srv_) return out;
    for (auto& f : srv_->drain_failures()) {
      py::dict d;
      d["namespace"] = f.ns;
      d["name"] = f.name;
      d["uid"] = f.uid;
      d["node"] = f.node;
      d["message"] = f.message;
      out.append(d);
    }
    return out;
  }

  size_t pending_count() {
    std::lock_guard<introspect::ProfiledMutex> g(l_.mu());
    return l_.pending_count();
  }

  ~Engine() {
    stop_server();
    stop_controller();
  }

  PodView parse_pod(const py::bytes& b) {
    PodView v;
    std::string err;
    if (!parse_pod_bytes(b, l_.profile(), &v, &err)) throw py::value_error(err);
    return v;
  }

 private:
  Ledger l_;
  bool update_mode_ = false;
  std::unique_ptr<NativeServer> srv_;  // declared after l_: destroyed (stopped) first
  std::unique_ptr<Controller> ctl_;
  bool binds_enabled_ = true;
};

}  // namespace

namespace {

// Benchmark wave-driver helpers (tracker.h); blocking calls drop the GIL.
class PyPodTracker {
 public:
  PyPodTracker(const py::dict& api, const std::string& ns, const std::string& label_selector)
      : t_(api_from(api), ns, label_selector) {}
  void start(double timeout) {
    std::string err;
    bool ok;
    {
      py::gil_scoped_release rel;
      ok = t_.start(timeout, &err);
    }
    if (!ok) throw std::runtime_error(err);
  }
  void stop() {
    py::gil_scoped_release rel;
    t_.stop();
  }
  std::string wait(const std::vector<std::string>& keys, int cond, double timeout) {
    py::gil_scoped_release rel;
    return t_.wait(keys, cond, timeout);
  }
  size_t size() const { return t_.size(); }

 private:
  PodTracker t_;
};

// The reflector the extender's controller and the plugin's pod feed run, with a plain key -> resourceVersion
// view: tests/test_k8s.py holds it against the Python informer the device plugin still runs (the one Python
// twin left, fenced by that cross-check).
class PyReflectorProbe {
 public:
  PyReflectorProbe(const py::dict& api, const std::string& path, const std::string& field_selector, int page) {
    ReflectorConfig rc;
    rc.path = path;
    rc.field_selector = field_selector;
    rc.list_page_size = page;
    ReflectorHandler h;
    h.on_list = [this](const ListView& lv) {
      std::map<std::string, std::string> fresh;
      for (size_t k = 0; k < lv.size(); ++k) {
        std::string key, rv;
        if (key_rv(lv.doc(k), lv.obj(k), &key, &rv)) fresh[key] = rv;
      }
      std::lock_guard<std::mutex> g(mu_);
      view_.swap(fresh);
      lists_++;
    };
    h.on_event = [this](Ev ev, const json::Doc& d, uint32_t obj) {
      std::string key, rv;
      if (!key_rv(d, obj, &key, &rv)) return;
      std::lock_guard<std::mutex> g(mu_);
      if (ev == Ev::Deleted) {
        view_.erase(key);
      } else {
        view_[key] = rv;
      }
      events_++;
    };
    r_ = std::make_unique<Reflector>(api_from(api), rc, h);
  }
  ~PyReflectorProbe() { stop(); }
  void start() { r_->start(); }
  void stop() {
    if (r_) {
      py::gil_scoped_release rel;
      r_->stop();
    }
  }
  bool wait_synced(double t) {
    py::gil_scoped_release rel;
    return r_->wait_synced(t);
  }
  void request_relist() { r_->request_relist(); }
  py::dict view() {
    py::dict d;
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : view_) d[py::str(kv.first)] = kv.second;
    return d;
  }
  py::dict stats() {
    py::dict d;
    d["relists"] = r_->relists();
    d["rewatches"] = r_->rewatches();
    d["errors"] = r_->errors();
    d["resource_version"] = r_->resource_version();
    std::lock_guard<std::mutex> g(mu_);
    d["lists"] = lists_;
    d["events"] = events_;
    return d;
  }

 private:
  static bool key_rv(const json::Doc& d, uint32_t obj, std::string* key, std::string* rv) {
    int64_t n = d.path(obj, {"metadata", "name"});
    if (n < 0) return false;
    int64_t ns = d.path(obj, {"metadata", "namespace"});
    int64_t r = d.path(obj, {"metadata", "resourceVersion"});
    *key = (ns >= 0 ? d.str(static_cast<uint32_t>(ns)) + "/" : std::string()) + d.str(static_cast<uint32_t>(n));
    *rv = r >= 0 ? d.str(static_cast<uint32_t>(r)) : std::string();
    return true;
  }
  std::unique_ptr<Reflector> r_;
  std::mutex mu_;
  std::map<std::string, std::string> view_;
  uint64_t lists_ = 0, events_ = 0;
};

class PyBatchClient {
 public:
  explicit PyBatchClient(const py::dict& api) : c_(api_from(api)) {}
  py::list run(const std::vector<std::tuple<std::string, std::string, py::bytes>>& reqs, int concurrency) {
    std::vector<std::tuple<std::string, std::string, std::string>> rq;
    rq.reserve(reqs.size());
    for (const auto& r : reqs) rq.emplace_back(std::get<0>(r), std::get<1>(r), std::string(std::get<2>(r)));
    std::vector<std::pair<int, std::string>> out;
    {
      py::gil_scoped_release rel;
      out = c_.run(rq, concurrency);
    }
    py::list l;
    for (auto& o : out) l.append(py::make_tuple(o.first, py::bytes(o.second)));
    return l;
  }

 private:
  BatchClient c_;
};

// bench.py --open-loop: constant-rate arrivals, every pod's stage times (tracker.h OpenLoop)
py::dict open_loop_run(const py::dict& api, const std::string& run, const std::string& pod_tmpl, double rate,
                       double duration_s, double warm_s, double hold_s, double drain_s, int creators, int deleters,
                       const std::string& ns, int grace) {
  OpenLoopConfig c;
  c.grace = grace;
  c.run = run;
  c.pod_tmpl = pod_tmpl;
  c.rate = rate;
  c.duration_s = duration_s;
  c.warm_s = warm_s;
  c.hold_s = hold_s;
  c.drain_s = drain_s;
  c.creators = creators;
  c.deleters = deleters;
  c.ns = ns;
  OpenLoop ol(api_from(api));
  std::vector<OpenLoopPod> pods;
  std::string err;
  int ce = 0, de = 0;
  bool ok;
  {
    py::gil_scoped_release rel;
    ok = ol.run(c, &pods, &err, &ce, &de);
  }
  if (!ok) throw std::runtime_error(err);
  py::list l;
  for (const auto& p : pods) l.append(py::make_tuple(p.arrival, p.created, p.bound, p.running, p.deleted, p.gone, p.failed));
  py::dict d;
  d["pods"] = l;
  d["create_errors"] = ce;
  d["delete_errors"] = de;
  return d;
}

class PyPodRuntime {
 public:
  PyPodRuntime(int dev, uint64_t arena_bytes, uint64_t arena_addr, uint64_t stream, uint64_t stride,
               const std::string& kernels_lib) {
    PodRuntimeConfig c;
    c.dev = dev;
    c.arena_bytes = arena_bytes;
    c.arena_addr = arena_addr;
    c.stream = reinterpret_cast<void*>(stream);
    c.stride = stride;
    c.kernels_lib = kernels_lib;
    r_ = std::make_unique<PodRuntime>(c);
    std::string err;
    if (!r_->init(&err)) throw std::runtime_error(err);
  }
  int serve(const std::string& host, int port, std::vector<int> cpus) {
    std::string err;
    int p = r_->serve(host, port, &err, std::move(cpus));
    if (p < 0) throw std::runtime_error(err);
    return p;
  }
  void stop() {
    py::gil_scoped_release rel;
    r_->stop();
  }
  int64_t admit(const std::string& uid, uint64_t bytes, bool verify) {
    std::string err;
    int64_t bad;
    {
      py::gil_scoped_release rel;
      bad = r_->admit(uid, bytes, verify, &err);
    }
    if (bad < 0) throw std::runtime_error(err);
    return bad;
  }
  bool release(const std::string& uid) { return r_->release(uid); }
  int64_t verify() {
    std::string err;
    int64_t bad;
    {
      py::gil_scoped_release rel;
      bad = r_->verify_all(&err);
    }
    if (bad < 0) throw std::runtime_error(err);
    return bad;
  }
  py::dict stats() const {
    py::dict d;
    d["admitted"] = r_->admitted();
    d["batches"] = r_->batches();
    d["failed"] = r_->failed();
    d["bad"] = r_->bad();
    d["resident"] = r_->resident();
    d["resident_bytes"] = r_->resident_bytes();
    return d;
  }

 private:
  std::unique_ptr<PodRuntime> r_;
};

}  // namespace

// ---------------------------------------------------------------- device plugin: native gRPC server
py::dict container_response_dict(const dp::ContainerResponse& r) {
  py::dict d;
  d["envs"] = r.envs;
  d["annotations"] = r.annotations;
  py::list mounts, devices;
  for (const auto& m : r.mounts) {
    py::dict e;
    e["container_path"] = m.container_path;
    e["host_path"] = m.host_path;
    e["read_only"] = m.read_only;
    mounts.append(e);
  }
  for (const auto& x : r.devices) {
    py::dict e;
    e["container_path"] = x.container_path;
    e["host_path"] = x.host_path;
    e["permissions"] = x.permissions;
    devices.append(e);
  }
  d["mounts"] = mounts;
  d["devices"] = devices;
  return d;
}

DpDevice dp_device_from(const py::dict& d) {
  DpDevice x;
  x.index = d["index"].cast<int>();
  if (d.contains("bdf")) x.bdf = d["bdf"].cast<std::string>();
  if (d.contains("cu_count")) x.cu_count = d["cu_count"].cast<int>();
  if (d.contains("total_bytes")) x.total_bytes = d["total_bytes"].cast<int64_t>();
  if (d.contains("share_bytes")) x.share_bytes = d["share_bytes"].cast<int64_t>();
  if (d.contains("units")) x.units = d["units"].cast<int64_t>();
  if (d.contains("nodes")) x.nodes = d["nodes"].cast<std::vector<std::string>>();
  if (d.contains("healthy")) x.healthy = d["healthy"].cast<bool>();
  return x;
}

// The device plugin's allocation state is shared by the plugin's Python code (state.py, through the AllocState /
// CuPartitioner bindings) and the native endpoint's serving thread.  One process-wide lock guards it: every binding
// of those classes takes it (py::call_guard), and so does the serving thread for each pass.  The serving thread
// never takes the GIL, so a Python caller holding the GIL while it waits for this lock cannot deadlock with it.
std::recursive_mutex& alloc_mu() {
  static std::recursive_mutex m;
  return m;
}
struct AllocLock {
  AllocLock() { alloc_mu().lock(); }
  ~AllocLock() { alloc_mu().unlock(); }
  AllocLock(const AllocLock&) = delete;
  AllocLock& operator=(const AllocLock&) = delete;
};

// The plugin's gRPC endpoint in native code, driven by the plugin's asyncio loop (add_reader(fd, poll)).
// GetDevicePluginOptions / ListAndWatch / PreStartContainer are answered here; GetPreferredAllocation and
// Allocate take DpCore's fast path and otherwise come back from poll() as pending calls for the Python handlers,
// answered with respond().
class PyDpServer {
 public:
  static constexpr const char* kSvc = "/v1beta1.DevicePlugin/";
  PyDpServer(const std::string& socket, AllocState& state, const py::dict& cfg) {
    DpConfig c;
    c.node = cfg["node"].cast<std::string>();
    c.profile = profile_from(cfg["profile"].cast<py::dict>());
    if (cfg.contains("mount_mode")) c.mount_mode = cfg["mount_mode"].cast<std::string>();
    if (cfg.contains("unit_bytes")) c.unit_bytes = cfg["unit_bytes"].cast<int64_t>();
    if (cfg.contains("iso_dir") && !cfg["iso_dir"].is_none()) c.iso_dir = cfg["iso_dir"].cast<std::string>();
    if (cfg.contains("guard")) c.guard = cfg["guard"].cast<bool>();
    if (cfg.contains("api") && !cfg["api"].is_none()) c.api = api_from(cfg["api"].cast<py::dict>());
    if (cfg.contains("early_answer")) c.early_answer = cfg["early_answer"].cast<bool>();
    if (cfg.contains("journal") && !cfg["journal"].is_none()) c.journal = cfg["journal"].cast<std::string>();
    if (cfg.contains("fast")) fast_ = cfg["fast"].cast<bool>();
    if (cfg.contains("spin_us")) spin_us_ = cfg["spin_us"].cast<double>();
    if (cfg.contains("py_event_ms")) py_event_s_ = cfg["py_event_ms"].cast<double>() * 1e-3;
    if (cfg.contains("preferred")) preferred_ = cfg["preferred"].cast<bool>();
    node_ = c.node;
    profile_ = c.profile;
    state_ = &state;
    core_ = std::make_unique<DpCore>(std::move(c), &state);
    srv_ = std::make_unique<h2::Server>(socket, [this](h2::Server& s, const h2::Call& call) { on_call(s, call); });
    if (!srv_->ok()) throw std::runtime_error(srv_->init_error());
    efd_ = ::eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    srv_->watch_fd(efd_);
    tfd_ = ::timerfd_create(CLOCK_MONOTONIC, TFD_NONBLOCK | TFD_CLOEXEC);
    srv_->watch_fd(tfd_);
    // the ASSIGNED commits of early-answered Allocates are independent (one pod each): several in flight, so the
    // node's admission rate is not capped at one commit per apiserver round trip (1 ms: 1,000 pods/s; the open-loop
    // rows of bench.py found that bound).  Worker 0 also runs the synchronous patches, in order
    int nw = 8;
    if (const char* e = std::getenv("GSX_PLUGIN_COMMIT_THREADS")) nw = std::max(1, std::min(64, std::atoi(e)));
    for (int i = 0; i < nw; ++i) {
      workers_.emplace_back([this, i] {
        introspect::name_thread("dp-worker");
        work(i);
      });
    }
  }
  ~PyDpServer() {
    stop_serving();
    if (feed_r_) feed_r_->stop();
    stop_worker();
    if (efd_ >= 0) ::close(efd_);
    if (tfd_ >= 0) ::close(tfd_);
    if (pyfd_ >= 0) ::close(pyfd_);
  }

  // Serve from a native thread instead of the owner's event loop: accept, read, the fast paths, the pod feed
  // and the patch completions run as soon as their fd is ready, however busy the Python loop is (its own pod
  // informer decodes every event of the node).  The state lock (alloc_mu) guards the shared state: every Python
  // call into it takes the lock, and so does the thread for each pass (microseconds of C++).  Returns an eventfd that
  // turns readable when calls for the Python slow path or fast-path events wait for poll().
  int start_serving() {
    if (serving_.joinable()) return pyfd_;
    pyfd_ = ::eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    stop_serving_ = false;
    {
      std::lock_guard<std::mutex> l(wmu_);
      serving_on_ = true;  // from now on the serving thread runs the synchronous patches (todo_) itself
    }
    serving_ = std::thread([this] { serve(); });
    return pyfd_;
  }

  // This node's pods straight into the allocation state from a native reflector (the plugin's Python informer,
  // slower to decode a burst of events, keeps its own views): an Allocate that kubelet sends right after the
  // binding finds its pod without waiting for Python.  Events are applied on the owner's thread, in poll().
  void start_feed(const py::dict& api) {
    if (feed_r_) return;
    ReflectorConfig rc;
    rc.path = "/api/v1/pods";
    rc.field_selector = "spec.nodeName=" + node_;
    ReflectorHandler h;
    h.on_list = [this](const ListView& lv) {
      Feed f;
      f.resync = true;
      for (size_t k = 0; k < lv.size(); ++k) {
        AllocPod ap;
        if (parse_alloc_pod(lv.doc(k), lv.obj(k), profile_, &ap)) {
          ap.raw = std::string(lv.doc(k).raw(lv.obj(k)));
          f.pods.push_back(std::move(ap));
        }
      }
      push_feed(std::move(f));
    };
    h.on_event = [this](Ev ev, const json::Doc& d, uint32_t obj) {
      Feed f;
      AllocPod ap;
      if (!parse_alloc_pod(d, obj, profile_, &ap)) return;
      if (ev != Ev::Deleted) ap.raw = std::string(d.raw(obj));
      f.deleted = ev == Ev::Deleted;
      f.pods.push_back(std::move(ap));
      push_feed(std::move(f));
    };
    feed_r_ = std::make_unique<Reflector>(api_from(api), rc, h);
    feed_r_->start();
  }

  // the feed's first LIST has arrived (false: timeout or no feed); poll() then applies it
  bool feed_synced(double timeout_s) {
    if (!feed_r_) return false;
    py::gil_scoped_release nogil;
    return feed_r_->wait_synced(timeout_s);
  }

  int fd() const { return srv_ ? srv_->fd() : -1; }

  py::tuple poll() {
    if (serving_.joinable()) {
      uint64_t n;
      (void)!::read(pyfd_, &n, sizeof n);  // the serving thread did the pass; collect what it left for Python
    } else {
      one_pass();
    }
    py::list pending, events;
    for (auto& p : pending_) pending.append(py::make_tuple(std::get<0>(p), std::get<1>(p), py::bytes(std::get<2>(p))));
    pending_.clear();
    for (auto& e : events_) {
      py::dict d;
      d["uid"] = e.uid;
      d["key"] = e.key;
      d["aid"] = e.aid;
      d["iso"] = e.iso;
      d["committed"] = e.committed;
      d["ambiguous"] = e.ambiguous;
      d["patch_only"] = e.patch_only;
      d["pod_json"] = py::bytes(e.pod_json);
      d["t_handler"] = e.t_handler;
      d["t_match"] = e.t_match;
      d["t_patch"] = e.t_patch;
      d["t_isolate"] = e.t_isolate;
      events.append(d);
    }
    events_.clear();
    return py::make_tuple(pending, events);
  }

  void one_pass() {
    // clear the wake-up first, then drain: a feed event or patch completion after this read signals again
    uint64_t n;
    if (efd_ >= 0) (void)!::read(efd_, &n, sizeof n);
    drain_feed();
    if (srv_) srv_->poll();
    drain_feed();
    retry_waiting(false);
    finish_patches();
    retry_waiting(true);
    passes_++;
  }

  // Early answer: the records to checkpoint, and the journal rotated to <journal>.old in the same step (under the
  // state lock, so no Allocate falls between the two).  The caller writes the checkpoint and deletes .old only once
  // it is in place: a failed or interrupted checkpoint loses no journaled record.  Returns (records, rotated, err).
  py::tuple journal_checkpoint() {
    py::list out;
    if (state_) {
      for (const auto& kv : state_->records()) {
        const AllocRecord& r = kv.second;
        py::dict d;
        d["aid"] = r.aid;
        d["ids"] = r.ids;
        d["uid"] = r.uid;
        d["dev"] = r.dev;
        d["units"] = r.units;
        d["cu_mask"] = r.cu_mask;
        d["owner"] = r.owner;
        d["t"] = r.t;
        d["iso"] = r.iso;
        d["on_gpu"] = r.on_gpu;
        out.append(d);
      }
    }
    std::string err;
    const bool rotated = core_->journal_rotate(&err);
    return py::make_tuple(out, rotated, err);
  }

  bool respond(uint64_t call, int status, const py::bytes& payload) {
    return srv_ && srv_->respond(call, status, std::string(view_of(payload)));
  }

  void set_devices(const py::list& devs, const std::map<std::string, int>& id_owner) {
    std::vector<DpDevice> v;
    for (const auto& d : devs) v.push_back(dp_device_from(d.cast<py::dict>()));
    core_->set_devices(std::move(v), id_owner);
  }

  // the encoded ListAndWatchResponse; every open ListAndWatch stream gets it
  void set_device_list(const py::bytes& msg) {
    device_list_ = std::string(view_of(msg));
    have_list_ = true;
    if (!srv_) return;
    for (uint64_t id : srv_->open_streams(std::string(kSvc) + "ListAndWatch")) srv_->stream_send(id, device_list_);
  }

  void set_fast(bool on) { fast_ = on; }
  void set_ready(bool on) { ready_ = on; }
  void set_state(AllocState& state) {
    core_->set_state(&state);
    state_ = &state;
  }

  size_t bg_backlog() {
    std::lock_guard<std::mutex> l(wmu_);
    return todo_bg_.size();
  }

  py::dict stats() {
    py::dict d;
    const auto& s = core_->stats();
    d["fast_allocate"] = s.fast_allocate;
    d["fast_preferred"] = s.fast_preferred;
    d["slow_allocate"] = s.slow_allocate;
    d["slow_preferred"] = s.slow_preferred;
    d["patch_failures"] = s.patch_failures;
    d["journal_failures"] = s.journal_failures;
    d["commits_gone"] = s.commits_gone;
    d["guard_by_ids"] = s.guard_by_ids;
    if (s.phased) {
      const double k = 1e6 / static_cast<double>(s.phased);
      d["allocate_phases_us"] = py::dict(py::arg("decode") = s.ph_decode * k, py::arg("match") = s.ph_match * k,
                                         py::arg("claim") = s.ph_claim * k, py::arg("build") = s.ph_build * k,
                                         py::arg("body") = s.ph_body * k, py::arg("record") = s.ph_record * k,
                                         py::arg("journal") = s.ph_journal * k, py::arg("encode") = s.ph_encode * k);
    }
    d["calls"] = srv_ ? srv_->calls() : 0;
    d["spins"] = spins_;
    d["loop_iters"] = loop_iters_;
    d["spin_iters"] = spin_iters_;
    d["connections"] = srv_ ? srv_->connections() : 0;
    d["fast"] = fast_;
    d["last_slow_reason"] = last_why_;
    d["waited"] = waited_;
    d["wait_ms"] = py::dict(py::arg("total") = wait_s_ * 1e3, py::arg("max") = wait_max_s_ * 1e3);
    d["feed_events"] = feed_events_;
    if (feed_r_) {
      d["feed_relists"] = feed_r_->relists();
      d["feed_rewatches"] = feed_r_->rewatches();
      d["feed_errors"] = feed_r_->errors();
    }
    d["feed"] = static_cast<bool>(feed_r_);
    d["serving_thread"] = serving_.joinable();
    d["journaling"] = core_->journaling();
    d["early_answer_backlog"] = static_cast<uint64_t>(bg_backlog());
    d["passes"] = passes_;
    // time inside the handlers (decode, match, respond), per call: what the plugin adds to kubelet's round trip
    d["lock_wait"] = py::dict(py::arg("total_ms") = 1e3 * lock_wait_s_, py::arg("max_us") = 1e6 * lock_wait_max_s_,
                              py::arg("over_5us") = lock_waits_);
    d["handler_us"] = py::dict(py::arg("get_preferred") = h_pref_n_ ? 1e6 * h_pref_s_ / h_pref_n_ : 0.0,
                               py::arg("allocate") = h_alloc_n_ ? 1e6 * h_alloc_s_ / h_alloc_n_ : 0.0,
                               py::arg("n_preferred") = h_pref_n_, py::arg("n_allocate") = h_alloc_n_,
                               py::arg("max_preferred") = 1e6 * h_pref_max_, py::arg("max_allocate") = 1e6 * h_alloc_max_);
    return d;
  }

  void close() {
    if (core_) core_->abort_requests();
    stop_serving();
    if (feed_r_) feed_r_->stop();
    stop_worker();
    AllocLock lock;
    finish_patches();
    if (srv_) {
      for (uint64_t id : srv_->open_streams(std::string(kSvc) + "ListAndWatch")) srv_->stream_end(id, 0, "");
      srv_->poll();
    }
    srv_.reset();
    if (core_) core_->journal_close();
  }

 private:
  void on_call(h2::Server& s, const h2::Call& call) {
    const double t0 = mono();
    handle_call(s, call);
    const double dt = mono() - t0;
    const std::string_view m(call.path);
    auto ends = [&m](std::string_view suf) { return m.size() >= suf.size() && m.substr(m.size() - suf.size()) == suf; };
    if (ends("/GetPreferredAllocation")) {
      h_pref_s_ += dt;
      h_pref_n_++;
      h_pref_max_ = std::max(h_pref_max_, dt);
    } else if (ends("/Allocate")) {
      h_alloc_s_ += dt;
      h_alloc_n_++;
      h_alloc_max_ = std::max(h_alloc_max_, dt);
    }
  }

  void handle_call(h2::Server& s, const h2::Call& call) {
    if (!ready_) {  // opened early for its pod feed, not serving yet (records and unlanded commits come first)
      s.respond(call.id, 14, "device plugin starting");
      return;
    }
    const std::string svc = kSvc;
    if (call.path.compare(0, svc.size(), svc) != 0) {
      s.respond(call.id, 12, "unknown service " + call.path);
      return;
    }
    std::string m = call.path.substr(svc.size());
    std::string resp, why;
    if (m == "GetDevicePluginOptions") {
      s.respond(call.id, 0, dp::encode_options(false, preferred_));
    } else if (m == "PreStartContainer") {
      s.respond(call.id, 0, std::string());
    } else if (m == "ListAndWatch") {
      if (have_list_) s.stream_send(call.id, device_list_);
    } else if (m == "GetPreferredAllocation" && fast_ && core_->preferred(call.message, &resp, &why)) {
      s.respond(call.id, 0, resp);
    } else if (m == "GetPreferredAllocation" && fast_ && feed_r_ && why == kNoPodYet) {
      wait_for_pod(call.id, m, call.message);
    } else if (m == "Allocate" && fast_) {
      DpEvent ev;
      std::unique_ptr<DpPending> pend;
      DpStep step = core_->allocate(call.message, &resp, &ev, &pend, &why);
      if (step == DpStep::Answered || step == DpStep::AnsweredPending) {
        s.respond(call.id, 0, resp);
        events_.push_back(std::move(ev));
        if (step == DpStep::AnsweredPending) queue_patch(std::move(pend), call.id, call.message);
      } else if (step == DpStep::Pending) {
        pend->call = call.id;
        pend->request = call.message;
        std::lock_guard<std::mutex> l(wmu_);
        todo_.push_back(std::move(pend));
        if (!serving_.joinable()) wcv_.notify_all();  // the serving thread runs its patches itself
      } else if (feed_r_ && why == kNoCandidate) {
        wait_for_pod(call.id, m, call.message);
      } else {
        last_why_ = why;
        pending_.emplace_back(call.id, m, call.message);
      }
    } else if (m == "GetPreferredAllocation" || m == "Allocate") {
      if (!why.empty()) last_why_ = why;
      pending_.emplace_back(call.id, m, call.message);
    } else {
      s.respond(call.id, 12, "unknown method " + m);
    }
  }

  void serve() {
    pthread_setname_np(pthread_self(), "gsx-dp-serve");
    const int ep = srv_ ? srv_->fd() : -1;
    // kubelet's calls come in bursts (GetPreferredAllocation, then Allocate, then the next pod's): after a pass
    // the thread polls without sleeping for spin_us_ before it blocks, so the next call of the burst does not pay
    // a sleep / wake-up of this thread (and of its idle core) on kubelet's serial admission path
    double spin_until = 0;
    for (;;) {
      pollfd pf{ep, POLLIN, 0};
      loop_iters_++;
      if (mono() < spin_until) {
        if (::poll(&pf, 1, 0) == 0 && !(py_deferred_ && mono() >= py_due_)) {
          spin_iters_++;
          if (stop_serving_) return;  // read without the lock: only a faster exit; checked again below
          // give the CPU to another runnable thread of this process (the pod feed, the commit worker): on the one
          // core a DaemonSet pod gets they would otherwise wait out the spin (run-delay 216 % of the timed region,
          // profiles/r05_session7/)
          sched_yield();
          continue;
        }
      } else {
        int ms = 100;
        if (py_deferred_) ms = std::max(0, std::min(ms, static_cast<int>((py_due_ - mono()) * 1e3) + 1));
        ::poll(&pf, 1, ms);
      }
      const double tl0 = mono();
      std::unique_lock<std::recursive_mutex> lock(alloc_mu());  // the state lock, not the GIL
      const double tl = mono() - tl0;
      lock_wait_s_ += tl;
      lock_wait_max_s_ = std::max(lock_wait_max_s_, tl);
      lock_waits_ += tl > 5e-6;
      if (stop_serving_ || !srv_) return;
      one_pass();
      // the ASSIGNED patches of this pass's Allocates, here rather than on the worker (two thread hops fewer on
      // kubelet's serial admission); the state lock is released around each apiserver call
      for (;;) {
        std::unique_ptr<DpPending> p;
        {
          std::lock_guard<std::mutex> l(wmu_);
          if (todo_.empty()) break;
          p = std::move(todo_.front());
          todo_.pop_front();
        }
        lock.unlock();
        core_->run_patch(*p);
        lock.lock();
        {
          std::lock_guard<std::mutex> l(wmu_);
          done_.push_back(std::move(p));
        }
        finish_patches();
        if (stop_serving_ || !srv_) return;
      }
      // spin only after a pass that served kubelet (its calls come in bursts: GetPreferredAllocation, Allocate, the
      // next pod's); a pass woken by the pod feed, a patch completion or the idle timeout blocks again at once, so an
      // idle or trickling node costs no polling core
      const uint64_t calls = srv_ ? srv_->calls() : 0;
      spin_until = (spin_us_ > 0 && calls != calls_seen_) ? mono() + spin_us_ * 1e-6 : 0;
      if (spin_until > 0) spins_++;
      calls_seen_ = calls;
      // also when the feed released a pod whose records went: Python cleans up their isolation files.  Calls for
      // the Python slow path wake it at once; bookkeeping events (answered Allocates, landed commits) at most every
      // py_event_s_: a Python pass takes the state lock, and one per Allocate would sit in the next admission's way
      const bool urgent = !pending_.empty();
      if (urgent || !events_.empty() || (state_ && state_->dropped_pending())) {
        const double now = mono();
        if (urgent || now - py_signal_at_ >= py_event_s_) {
          uint64_t one = 1;
          (void)!::write(pyfd_, &one, sizeof one);
          py_signal_at_ = now;
          py_deferred_ = false;
        } else if (!py_deferred_) {
          py_deferred_ = true;
          py_due_ = py_signal_at_ + py_event_s_;
        }
      } else {
        // nothing left for Python (it drained the events on a wake-up of its own): no deferred signal is due.  A
        // deferral left standing made every later poll time out at once -- the thread took the state lock for an
        // empty pass hundreds of thousands of times a second until the next event (round 4's busy plugin core)
        py_deferred_ = false;
      }
    }
  }

  // Not under the state lock (the thread needs it to finish its pass); the GIL is released while joining.
  void stop_serving() {
    if (!serving_.joinable()) return;
    {
      AllocLock lock;
      stop_serving_ = true;
    }
    uint64_t one = 1;
    (void)!::write(efd_, &one, sizeof one);
    py::gil_scoped_release nogil;
    serving_.join();
    {
      std::lock_guard<std::mutex> l(wmu_);
      serving_on_ = false;  // synchronous patches left in todo_ go to the worker again
    }
    wcv_.notify_all();
  }

  static constexpr const char* kNoCandidate = "no candidate";
  static constexpr const char* kNoPodYet = "no pending pod of that size known yet";
  static constexpr double kWaitS = 0.02;  // how long a call waits for its pod's event before Python takes it

  struct Feed {
    bool resync = false, deleted = false;
    std::vector<AllocPod> pods;
  };
  struct Waiting {
    uint64_t call;
    std::string method, message;
    double deadline;
    double t0 = 0;  // when it started waiting
  };

  static double mono() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
  }

  void push_feed(Feed f) {
    {
      std::lock_guard<std::mutex> l(fmu_);
      feed_.push_back(std::move(f));
    }
    uint64_t one = 1;
    (void)!::write(efd_, &one, sizeof one);
  }

  void drain_feed() {
    std::vector<Feed> fs;
    {
      std::lock_guard<std::mutex> l(fmu_);
      fs.swap(feed_);
    }
    for (auto& f : fs) {
      feed_events_ += f.pods.size();
      if (f.resync) {
        std::unordered_set<std::string> live;
        for (const auto& ap : f.pods) {
          live.insert(ap.uid);
          state_->observe(ap);
        }
        state_->resync(live);
      } else if (f.deleted) {
        for (const auto& ap : f.pods) state_->deleted(ap.uid);
      } else {
        for (const auto& ap : f.pods) state_->observe(ap);
      }
    }
  }

  void arm_timer() {
    if (waiting_.empty()) return;
    double first = waiting_.front().deadline;
    for (const auto& w : waiting_) first = std::min(first, w.deadline);
    double dt = std::max(0.0005, first - mono());
    itimerspec its{};
    its.it_value.tv_sec = static_cast<time_t>(dt);
    its.it_value.tv_nsec = static_cast<long>((dt - static_cast<double>(its.it_value.tv_sec)) * 1e9);
    ::timerfd_settime(tfd_, 0, &its, nullptr);
  }

  void wait_for_pod(uint64_t call, const std::string& method, const std::string& message) {
    const double now = mono();
    waiting_.push_back({call, method, message, now + kWaitS, now});
    waited_++;
    arm_timer();
  }

  // calls that found no pod yet: again through the fast path; past their deadline, to Python
  void retry_waiting(bool expire) {
    uint64_t n;
    if (tfd_ >= 0) (void)!::read(tfd_, &n, sizeof n);
    if (waiting_.empty() || !srv_) return;
    std::vector<Waiting> still;
    const double now = mono();
    auto waited = [&](const Waiting& w) {  // how long a call waited for its pod's event (the feed's lag)
      const double dt = now - w.t0;
      wait_s_ += dt;
      wait_max_s_ = std::max(wait_max_s_, dt);
    };
    for (auto& w : waiting_) {
      std::string resp, why;
      if (w.method == "GetPreferredAllocation") {
        if (core_->preferred(w.message, &resp, &why)) {
          srv_->respond(w.call, 0, resp);
          waited(w);
          continue;
        }
      } else {
        DpEvent ev;
        std::unique_ptr<DpPending> pend;
        DpStep step = core_->allocate(w.message, &resp, &ev, &pend, &why);
        if (step == DpStep::Answered || step == DpStep::AnsweredPending) {
          srv_->respond(w.call, 0, resp);
          waited(w);
          events_.push_back(std::move(ev));
          if (step == DpStep::AnsweredPending) queue_patch(std::move(pend), w.call, w.message);
          continue;
        }
        if (step == DpStep::Pending) {
          waited(w);
          pend->call = w.call;
          pend->request = w.message;
          std::lock_guard<std::mutex> l(wmu_);
          todo_.push_back(std::move(pend));
          if (!serving_.joinable()) wcv_.notify_all();
          continue;
        }
        if (why != kNoCandidate) {
          last_why_ = why;
          pending_.emplace_back(w.call, w.method, w.message);
          continue;
        }
      }
      if (expire && now >= w.deadline) {
        waited(w);
        last_why_ = why;
        pending_.emplace_back(w.call, w.method, w.message);
      } else {
        still.push_back(std::move(w));
      }
    }
    waiting_.swap(still);
    arm_timer();
  }

  // the ASSIGNED patches run here, never on the owner's event loop
  // Takes the synchronous patches (todo_) only while no serving thread runs them itself, and the early-answered
  // commits (todo_bg_) once their backoff (not_before) has passed.
  void work(int me) {
    for (;;) {
      std::unique_ptr<DpPending> p;
      {
        std::unique_lock<std::mutex> l(wmu_);
        for (;;) {
          if (me == 0 && (!serving_on_ || stopping_) && !todo_.empty()) {
            p = std::move(todo_.front());
            todo_.pop_front();
            break;
          }
          // stopping: early-answered commits still queued are left to the journal (a restarted plugin lands them)
          if (stopping_) return;
          if (todo_bg_.empty()) {
            wcv_.wait(l);
            continue;
          }
          const double now = mono();
          auto it = std::find_if(todo_bg_.begin(), todo_bg_.end(),
                                 [now](const std::unique_ptr<DpPending>& q) { return q->not_before <= now; });
          if (it != todo_bg_.end()) {
            p = std::move(*it);
            todo_bg_.erase(it);
            break;
          }
          double first = todo_bg_.front()->not_before;
          for (const auto& q : todo_bg_) first = std::min(first, q->not_before);
          wcv_.wait_for(l, std::chrono::duration<double>(first - now));
        }
      }
      core_->run_patch(*p);
      {
        std::lock_guard<std::mutex> l(wmu_);
        done_.push_back(std::move(p));
      }
      uint64_t one = 1;
      (void)!::write(efd_, &one, sizeof one);
    }
  }

  void stop_worker() {
    if (workers_.empty()) return;
    {
      std::lock_guard<std::mutex> l(wmu_);
      stopping_ = true;
    }
    wcv_.notify_all();
    for (auto& w : workers_) w.join();
    workers_.clear();
  }

  void queue_patch(std::unique_ptr<DpPending> pend, uint64_t call, const std::string& message) {
    if (call) {
      pend->call = call;
      pend->request = message;
    }
    std::lock_guard<std::mutex> l(wmu_);
    if (pend->answered) {
      todo_bg_.push_back(std::move(pend));
      wcv_.notify_all();  // any worker (worker 0 may be the one a synchronous patch needs)
      return;
    }
    todo_.push_back(std::move(pend));
    if (!serving_.joinable()) wcv_.notify_all();  // worker 0 takes it (the serving thread runs its patches itself)
  }

  void finish_patches() {
    std::deque<std::unique_ptr<DpPending>> done;
    {
      std::lock_guard<std::mutex> l(wmu_);
      done.swap(done_);
    }
    for (auto& p : done) {
      std::string resp, why;
      DpEvent ev;
      if (p->answered) {  // early answer: kubelet has its response; only the commit's outcome remains
        core_->finish(*p, &resp, &ev, &why);
        if (p->retry) {
          queue_patch(std::move(p), 0, std::string());
        } else if (ev.patch_only) {
          events_.push_back(std::move(ev));
        }
        continue;
      }
      if (core_->finish(*p, &resp, &ev, &why)) {
        if (srv_) srv_->respond(p->call, 0, resp);
        events_.push_back(std::move(ev));
      } else {
        last_why_ = why;
        pending_.emplace_back(p->call, std::string("Allocate"), p->request);
      }
    }
  }

  std::string node_;
  Profile profile_;
  AllocState* state_ = nullptr;
  std::unique_ptr<Reflector> feed_r_;
  std::mutex fmu_;
  std::vector<Feed> feed_;
  std::vector<Waiting> waiting_;
  uint64_t waited_ = 0, feed_events_ = 0;
  double wait_s_ = 0, wait_max_s_ = 0;  // calls that waited for their pod's event: total / longest wait
  int tfd_ = -1;
  std::vector<std::thread> workers_;
  std::mutex wmu_;
  std::condition_variable wcv_;
  std::deque<std::unique_ptr<DpPending>> todo_, done_;
  // early-answered commits: always on the worker, so a slow apiserver never holds up the serving thread
  std::deque<std::unique_ptr<DpPending>> todo_bg_;
  bool stopping_ = false;
  bool serving_on_ = false;  // (wmu_) a serving thread runs todo_ itself
  int efd_ = -1;
  std::unique_ptr<DpCore> core_;
  std::unique_ptr<h2::Server> srv_;
  std::vector<std::tuple<uint64_t, std::string, std::string>> pending_;
  std::vector<DpEvent> events_;
  std::string device_list_, last_why_;
  bool have_list_ = false, fast_ = true;
  // start_serving(): the pass runs on this thread, the GIL as the state mutex
  std::thread serving_;
  std::atomic<bool> stop_serving_{false};  // written under the state lock
  int pyfd_ = -1;              // readable: pending_ / events_ waiting for poll()
  double h_pref_s_ = 0, h_alloc_s_ = 0, h_pref_max_ = 0, h_alloc_max_ = 0;
  bool ready_ = true;       // false: every call is answered UNAVAILABLE (set_ready)
  bool preferred_ = false;  // cfg "preferred": advertise GetPreferredAllocation (kubelet then calls it per admission)
  double py_event_s_ = 0.002;  // cfg "py_event_ms": how often answered Allocates are handed to Python at most
  double py_signal_at_ = 0, py_due_ = 0;
  bool py_deferred_ = false;
  double lock_wait_s_ = 0, lock_wait_max_s_ = 0;  // the serving thread waiting for the state lock (Python holds it)
  uint64_t lock_waits_ = 0;                        // waits over 5 us
  uint64_t h_pref_n_ = 0, h_alloc_n_ = 0;
  double spin_us_ = 1000;      // poll without sleeping this long after a pass (cfg "spin_us"; 0: always block)
  uint64_t calls_seen_ = 0;    // kubelet calls served as of the last pass (a pass that served none does not spin)
  uint64_t spins_ = 0;
  uint64_t loop_iters_ = 0, spin_iters_ = 0;
  uint64_t passes_ = 0;
};

PYBIND11_MODULE(_engine, m) {
  m.def(
      "native_symbol", [](uint64_t pc) { return introspect::symbol_at(static_cast<uintptr_t>(pc)); },
      "Function name at a program counter of this process ('' when unknown).");
  m.def(
      "native_stacks",
      [](std::vector<int> tids, double timeout) {
        std::vector<introspect::Sample> got;
        {
          py::gil_scoped_release rel;  // Python threads must be able to run their handlers too
          got = introspect::capture(tids, timeout);
        }
        py::list out;
        for (auto& smp : got) out.append(py::make_tuple(smp.tid, smp.comm, smp.ok, smp.frames));
        return out;
      },
      py::arg("tids") = std::vector<int>(), py::arg("timeout") = 0.05,
      "Stack samples (tid, comm, ok, frames innermost-first) of this process's threads (all when tids is empty).");

  m.doc() = "gpushare MI355X native ledger engine";

  py::class_<PodView>(m, "PodView")
      .def(py::init<>())
      .def_readwrite("uid", &PodView::uid)
      .def_readwrite("name", &PodView::name)
      .def_readwrite("namespace", &PodView::ns)
      .def_readwrite("node", &PodView::node)
      .def_readwrite("phase", &PodView::phase)
      .def_readwrite("resource_version", &PodView::rv)
      .def_readwrite("deleting", &PodView::deleting)
      .def_readwrite("request", &PodView::request)
      .def_readwrite("dev_idx", &PodView::dev_idx)
      .def_readwrite("annot_mem", &PodView::annot_mem)
      .def_readwrite("has_annot_mem", &PodView::has_annot_mem)
      .def_readwrite("annot_dev_total", &PodView::annot_dev_total)
      .def_readwrite("assigned", &PodView::assigned)
      .def_readwrite("assume_time", &PodView::assume_time)
      .def_readwrite("cu_mask", &PodView::cu_mask)
      .def_readwrite("hold_idx", &PodView::hold_idx)
      .def_property_readonly("terminal", &PodView::terminal)
      .def_property_readonly("complete", &PodView::complete)
      .def_property_readonly("assigned_non_terminated", &PodView::assigned_non_terminated)
      .def("__repr__", [](const PodView& v) {
        return "<PodView " + v.ns + "/" + v.name + " uid=" + v.uid + " node=" + v.node +
               " req=" + std::to_string(v.request) + " idx=" + std::to_string(v.dev_idx) + ">";
      });

  py::class_<Engine>(m, "Engine")
      .def(py::init<const py::dict&>(), py::arg("profile") = py::dict())
      .def("profile", &Engine::profile)
      .def("upsert_node", &Engine::upsert_node, py::arg("name"), py::arg("total"), py::arg("count"),
           py::arg("dev_totals") = std::vector<int64_t>(), py::arg("address") = std::string())
      .def("upsert_node_json", &Engine::upsert_node_json)
      .def("remove_node", &Engine::remove_node)
      .def("has_node", &Engine::has_node)
      .def("node_info", &Engine::node_info)
      .def("upsert_pod", &Engine::upsert_pod)
      .def("remove_pod", &Engine::remove_pod)
      .def("known", &Engine::known)
      .def("pod_state", &Engine::pod_state)
      .def("upsert_pod_json", &Engine::upsert_pod_json)
      .def("check", &Engine::check)
      .def("filter", &Engine::filter)
      .def("prioritize", &Engine::prioritize)
      .def("assume", &Engine::assume)
      .def("finish_bind", &Engine::finish_bind, py::arg("uid"), py::arg("ok"), py::arg("ttl") = 30.0)
      .def("gc", &Engine::gc, py::arg("list_start") = 0.0)
      .def("assume_ordered", &Engine::assume_ordered, py::arg("uid"), py::arg("ns"), py::arg("name"),
           py::arg("node"), py::arg("req"), py::arg("cu_count") = std::string())
      .def("bind_blocked", &Engine::bind_blocked)
      .def("bind_wait", &Engine::bind_wait)
      .def("bind_leave", &Engine::bind_leave)
      .def("controller_gc", &Engine::controller_gc)
      .def("inspect", &Engine::inspect, py::arg("node") = std::string())
      .def("node_devices", &Engine::node_devices)
      .def("node_names", &Engine::node_names)
      .def("stats", &Engine::stats)
      .def("parse_pod", &Engine::parse_pod)
      .def("serve", &Engine::serve, py::arg("host"), py::arg("port"), py::arg("threads") = 2,
           py::arg("pool_threads") = 16, py::arg("fallback_port") = 0, py::arg("ttl") = 60.0,
           py::arg("api") = py::dict(), py::arg("update_mode") = false, py::arg("qps") = 0.0, py::arg("burst") = 10,
           py::arg("plugin_auth") = "none", py::arg("plugin_users") = std::vector<std::string>())
      .def("node_unaccounted", [](Engine& e, const std::string& node) { return e.node_unaccounted(node); })
      .def("begin_move", &Engine::begin_move, py::arg("uid"), py::arg("node"), py::arg("from_dev"), py::arg("to") = -1,
           py::arg("partner") = std::string(), py::arg("physical_on_to") = false, py::arg("req_hold") = -1,
           py::arg("req_hold_partner") = std::string())
      .def("end_move", &Engine::end_move)
      .def("set_unaccounted", &Engine::set_unaccounted, py::arg("node"), py::arg("extra"), py::arg("ttl") = 60.0)
      .def("begin_epoch", &Engine::begin_epoch)
      .def("publication_wait", &Engine::publication_wait)
      .def("stop_server", &Engine::stop_server)
      .def("start_controller", &Engine::start_controller, py::arg("api"), py::arg("resync") = 30.0,
           py::arg("sync_timeout") = 60.0, py::arg("watch_timeout") = 300)
      .def("stop_controller", &Engine::stop_controller)
      .def("controller_synced", &Engine::controller_synced)
      .def("controller_get_pod", &Engine::controller_get_pod)
      .def("controller_overcommitted", &Engine::controller_overcommitted)
      .def("controller_stats", &Engine::controller_stats)
      .def("server_stats", &Engine::server_stats)
      .def("ledger_mutex", &Engine::ledger_mutex)
      .def("drain_bind_failures", &Engine::drain_bind_failures)
      .def("set_binds_enabled", &Engine::set_binds_enabled)
      .def("set_update_mode", &Engine::set_update_mode)
      .def("set_bind_order", &Engine::set_bind_order)
      .def_property_readonly("bind_order", &Engine::bind_order)
      .def("drain_annotation_repairs", &Engine::drain_annotation_repairs)
      .def("pending_count", &Engine::pending_count);

  py::class_<PyPodTracker>(m, "PodTracker")
      .def(py::init<const py::dict&, const std::string&, const std::string&>(), py::arg("api"),
           py::arg("namespace") = std::string(), py::arg("label_selector") = std::string())
      .def("start", &PyPodTracker::start, py::arg("timeout") = 30.0)
      .def("stop", &PyPodTracker::stop)
      .def("wait", &PyPodTracker::wait, py::arg("keys"), py::arg("cond"), py::arg("timeout") = 120.0)
      .def("size", &PyPodTracker::size);
  m.attr("TRACK_BOUND") = static_cast<int>(PodTracker::Bound);
  m.attr("TRACK_RUNNING") = static_cast<int>(PodTracker::Running);
  m.attr("TRACK_GONE") = static_cast<int>(PodTracker::Gone);
  m.attr("TRACK_STOPPED") = static_cast<int>(PodTracker::Stopped);
  py::class_<PyReflectorProbe>(m, "ReflectorProbe")
      .def(py::init<const py::dict&, const std::string&, const std::string&, int>(), py::arg("api"),
           py::arg("path") = "/api/v1/pods", py::arg("field_selector") = "", py::arg("page") = 500)
      .def("start", &PyReflectorProbe::start)
      .def("stop", &PyReflectorProbe::stop)
      .def("wait_synced", &PyReflectorProbe::wait_synced, py::arg("timeout") = 10.0)
      .def("request_relist", &PyReflectorProbe::request_relist)
      .def("view", &PyReflectorProbe::view)
      .def("stats", &PyReflectorProbe::stats);

  m.def("open_loop_run", &open_loop_run, py::arg("api"), py::arg("run"), py::arg("pod_tmpl"), py::arg("rate"),
        py::arg("duration_s") = 2.0, py::arg("warm_s") = 0.5, py::arg("hold_s") = 0.0, py::arg("drain_s") = 20.0,
        py::arg("creators") = 16, py::arg("deleters") = 16, py::arg("ns") = "default", py::arg("grace") = -1);
  py::class_<PyBatchClient>(m, "BatchClient")
      .def(py::init<const py::dict&>())
      .def("run", &PyBatchClient::run, py::arg("requests"), py::arg("concurrency") = 8);

  py::class_<PyPodRuntime>(m, "PodRuntime")
      .def(py::init<int, uint64_t, uint64_t, uint64_t, uint64_t, const std::string&>(), py::arg("dev"),
           py::arg("arena_bytes"), py::arg("arena_addr") = 0, py::arg("stream") = 0, py::arg("stride") = 1 << 20,
           py::arg("kernels_lib") = std::string())
      .def("serve", &PyPodRuntime::serve, py::arg("host") = "127.0.0.1", py::arg("port") = 0,
           py::arg("cpus") = std::vector<int>())
      .def("stop", &PyPodRuntime::stop)
      .def("admit", &PyPodRuntime::admit, py::arg("uid"), py::arg("bytes"), py::arg("verify") = true)
      .def("release", &PyPodRuntime::release)
      .def("verify", &PyPodRuntime::verify)
      .def("stats", &PyPodRuntime::stats);


  // ---- the device plugin's allocation state (allocstate.h): one implementation for the gRPC plugin and the
  // compiled node agent
  py::class_<CuPartitioner>(m, "CuPartitioner")
      .def(py::init<int, int>(), py::arg("cu_count") = 256, py::arg("xcc_count") = 8)
      .def("allocate", [](CuPartitioner& c, const std::string& uid, int n) {
             std::vector<int> out;
             std::string err;
             if (!c.allocate(uid, n, &out, &err)) throw py::value_error(err);
             return out;
           }, py::call_guard<AllocLock>())
      .def("release", &CuPartitioner::release, py::call_guard<AllocLock>())
      .def("adopt", &CuPartitioner::adopt, py::call_guard<AllocLock>())
      .def("swap_owners", &CuPartitioner::swap_owners, py::call_guard<AllocLock>())
      .def("holds", &CuPartitioner::holds, py::call_guard<AllocLock>())
      .def("held_by", &CuPartitioner::held_by, py::call_guard<AllocLock>())
      .def("held", [](const CuPartitioner& c) {
        py::dict d;
        for (const auto& kv : c.held()) d[py::str(kv.first)] = kv.second;
        return d;
      }, py::call_guard<AllocLock>())
      .def("free_count", &CuPartitioner::free_count, py::call_guard<AllocLock>())
      .def_property_readonly("cu_count", &CuPartitioner::cu_count)
      .def_property_readonly("xcc_count", &CuPartitioner::xcc_count);
  m.def("cu_words", &cu_words, py::call_guard<AllocLock>());
  m.def("parse_cu_words", [](const std::string& w) {
    try {
      return parse_cu_words(w);
    } catch (const std::invalid_argument& e) {
      throw py::value_error(e.what());
    }
  }, py::call_guard<AllocLock>());
  m.def("cu_ranges", &cu_ranges, py::call_guard<AllocLock>());

  py::class_<AllocPod>(m, "AllocPod")
      .def(py::init<>())
      .def_readwrite("uid", &AllocPod::uid)
      .def_readwrite("key", &AllocPod::key)
      .def_readwrite("namespace", &AllocPod::ns)
      .def_readwrite("name", &AllocPod::name)
      .def_readwrite("rv", &AllocPod::rv)
      .def_readwrite("phase", &AllocPod::phase)
      .def_readwrite("creation", &AllocPod::creation)
      .def_readwrite("node", &AllocPod::node)
      .def_readwrite("dev", &AllocPod::dev)
      .def_readwrite("request", &AllocPod::request)
      .def_readwrite("containers", &AllocPod::containers)
      .def_readwrite("assume_time", &AllocPod::assume_time)
      .def_readwrite("dev_total", &AllocPod::dev_total)
      .def_readwrite("assigned", &AllocPod::assigned)
      .def_readwrite("complete", &AllocPod::complete)
      .def_readwrite("terminating", &AllocPod::terminating)
      .def_readwrite("term_grace_s", &AllocPod::term_grace_s)
      .def_readwrite("cu_count", &AllocPod::cu_count)
      .def_readwrite("cu_mask", &AllocPod::cu_mask)
      .def_readwrite("hold_idx", &AllocPod::hold_idx)
      .def_readwrite("hold_partner", &AllocPod::hold_partner)
      .def_readwrite("raw", &AllocPod::raw)
      .def_property_readonly("pending", &AllocPod::pending);

  auto rec_dict = [](const AllocRecord& r) {
    py::dict d;
    d["aid"] = r.aid;
    d["ids"] = r.ids;
    d["uid"] = r.uid;
    d["dev"] = r.dev;
    d["units"] = r.units;
    d["cu_mask"] = r.cu_mask;
    d["owner"] = r.owner;
    d["t"] = r.t;
    d["iso"] = r.iso;
    d["on_gpu"] = r.on_gpu;
    return d;
  };
  py::class_<AllocState>(m, "AllocState")
      .def(py::init([](const std::string& node, const std::vector<std::tuple<int, int, int>>& devs) {
             std::vector<std::pair<int, std::pair<int, int>>> d;
             for (const auto& t : devs) d.push_back({std::get<0>(t), {std::get<1>(t), std::get<2>(t)}});
             return new AllocState(node, d);
           }),
           py::arg("node"), py::arg("devices"))
      .def("observe", &AllocState::observe, py::call_guard<AllocLock>())
      .def("release", &AllocState::release, py::call_guard<AllocLock>())
      .def("deleted", &AllocState::deleted, py::arg("uid"), py::arg("now") = -1.0, py::call_guard<AllocLock>())
      .def("lingering", &AllocState::lingering, py::call_guard<AllocLock>())
      .def("gone_held", &AllocState::gone_held, py::call_guard<AllocLock>())
      .def("set_linger", &AllocState::set_linger, py::call_guard<AllocLock>())
      .def("set_skip_partners", &AllocState::set_skip_partners, py::call_guard<AllocLock>())
      .def("linger_enabled", &AllocState::linger_enabled, py::call_guard<AllocLock>())
      .def("linger_count", &AllocState::linger_count, py::call_guard<AllocLock>())
      .def("is_tombstoned", &AllocState::is_tombstoned, py::call_guard<AllocLock>())
      .def("resync", [](AllocState& s, const std::vector<std::string>& live, double now) {
        s.resync(std::unordered_set<std::string>(live.begin(), live.end()), now);
      }, py::arg("live"), py::arg("now") = -1.0, py::call_guard<AllocLock>())
      .def("holders", &AllocState::holders, py::call_guard<AllocLock>())
      .def("has_pod", [](const AllocState& s, const std::string& uid) { return s.pod(uid) != nullptr; }, py::call_guard<AllocLock>())
      // ns/name -> uid through the state's key index (the reconciliation looks up every pod kubelet reports)
      .def("uid_for_key", [](const AllocState& s, const std::string& key) -> std::string {
        const AllocPod* p = s.pod_by_key(key);
        return p ? p->uid : std::string();
      }, py::call_guard<AllocLock>())
      // the native state's view of a pod (the one the matcher decided on): the fields an Allocate acts on
      .def("pod_view", [](const AllocState& s, const std::string& uid) -> py::object {
             const AllocPod* p = s.pod(uid);
             if (!p) return py::none();
             py::dict d;
             d["rv"] = p->rv;
             d["phase"] = p->phase;
             d["dev"] = p->dev;
             d["assigned"] = p->assigned;
             d["cu_mask"] = p->cu_mask;
             d["hold_idx"] = p->hold_idx;
             d["hold_partner"] = p->hold_partner;
             return d;
           }, py::call_guard<AllocLock>())
      // every pod the state holds, for the Python views: (uid, key, ns, name, rv, phase, dev, request, containers,
      // assume_time, creation, assigned, complete, cu_count, cu_mask, hold_idx, hold_partner)
      .def("pod_views", [](const AllocState& s) {
        std::vector<AllocPod> copy;
        {
          AllocLock lock;
          copy.resize(s.pods().size());
          size_t i = 0;
          for (const auto& kv : s.pods()) {  // every field but the raw JSON
            const AllocPod& p = kv.second;
            AllocPod& c = copy[i++];
            c.uid = p.uid, c.key = p.key, c.ns = p.ns, c.name = p.name, c.rv = p.rv, c.phase = p.phase;
            c.creation = p.creation, c.dev = p.dev, c.request = p.request, c.containers = p.containers;
            c.assume_time = p.assume_time, c.assigned = p.assigned, c.complete = p.complete;
            c.cu_count = p.cu_count, c.cu_mask = p.cu_mask, c.hold_idx = p.hold_idx, c.hold_partner = p.hold_partner;
          }
        }
        py::list out;
        for (const AllocPod& p : copy) {
          out.append(py::make_tuple(p.uid, p.key, p.ns, p.name, p.rv, p.phase, p.dev, p.request, p.containers,
                                    p.assume_time, p.creation, p.assigned, p.complete, p.cu_count, p.cu_mask,
                                    p.hold_idx, p.hold_partner));
        }
        return out;
      })
      .def("pod_full", [](const AllocState& s, const std::string& uid) -> py::object {
        const AllocPod* pp = s.pod(uid);
        if (!pp) return py::none();
        const AllocPod& p = *pp;
        return py::make_tuple(p.uid, p.key, p.ns, p.name, p.rv, p.phase, p.dev, p.request, p.containers,
                              p.assume_time, p.creation, p.assigned, p.complete, p.cu_count, p.cu_mask, p.hold_idx,
                              p.hold_partner);
      }, py::call_guard<AllocLock>())
      .def("pod_json", [](const AllocState& s, const std::string& uid) -> py::object {
        const AllocPod* p = s.pod(uid);
        if (!p || p->raw.empty()) return py::none();
        return py::bytes(p->raw);
      }, py::call_guard<AllocLock>())
      .def("pod_uids", [](const AllocState& s) {
        std::vector<std::string> out;
        for (const auto& kv : s.pods()) out.push_back(kv.first);
        return out;
      }, py::call_guard<AllocLock>())
      .def("candidates", [](const AllocState& s) {
        std::vector<std::string> out;
        for (const AllocPod* p : s.candidates()) out.push_back(p->uid);
        return out;
      }, py::call_guard<AllocLock>())
      .def("match", [](AllocState& s, int64_t units) {
        auto m = s.match(units);
        return py::make_tuple(m.first ? py::object(py::str(m.first->uid)) : py::object(py::none()), m.second);
      }, py::call_guard<AllocLock>())
      .def("preferred_device", &AllocState::preferred_device, py::call_guard<AllocLock>())
      .def("unannotated", &AllocState::unannotated, py::call_guard<AllocLock>())
      .def("claim_cus", [](AllocState& s, const std::string& uid) {
             std::vector<int> out;
             std::string err;
             if (!s.claim_cus(uid, &out, &err)) throw py::value_error(err);
             return out;
           }, py::call_guard<AllocLock>())
      .def("set_inflight", &AllocState::set_inflight, py::call_guard<AllocLock>())
      .def("set_owners_reported", &AllocState::set_owners_reported, py::call_guard<AllocLock>())
      .def("owners_reported", &AllocState::owners_reported, py::call_guard<AllocLock>())
      .def("expect_owner_reports", &AllocState::expect_owner_reports, py::call_guard<AllocLock>())
      .def("inflight", &AllocState::inflight, py::call_guard<AllocLock>())
      .def("first_container_committed", &AllocState::first_container_committed, py::call_guard<AllocLock>())
      .def("later_container_allocated", &AllocState::later_container_allocated, py::call_guard<AllocLock>())
      .def("partial", [](const AllocState& s) {
        py::dict d;
        for (const auto& kv : s.partial()) d[py::str(kv.first)] = kv.second;
        return d;
      }, py::call_guard<AllocLock>())
      .def("record", [rec_dict](AllocState& s, const std::string& uid, const std::vector<std::string>& ids, int64_t units,
                      const std::string& cu_mask, const std::string& aid, double t, const std::string& iso) {
             AllocRecord& r = s.record(uid, ids, units, cu_mask, aid, t);
             r.iso = iso;
             return rec_dict(r);
           },
           py::arg("uid"), py::arg("ids"), py::arg("units"), py::arg("cu_mask"), py::arg("aid"), py::arg("t") = 0.0,
           py::arg("iso") = std::string(), py::call_guard<AllocLock>())
      .def("add_record", [](AllocState& s, const py::dict& d) {
             AllocRecord r;
             r.aid = d["aid"].cast<std::string>();
             r.ids = d.contains("ids") ? d["ids"].cast<std::vector<std::string>>() : std::vector<std::string>();
             r.uid = d.contains("uid") ? d["uid"].cast<std::string>() : std::string();
             r.dev = d.contains("dev") ? d["dev"].cast<int64_t>() : -1;
             r.units = d.contains("units") ? d["units"].cast<int64_t>() : 0;
             r.cu_mask = d.contains("cu_mask") ? d["cu_mask"].cast<std::string>() : std::string();
             r.owner = d.contains("owner") ? d["owner"].cast<std::string>() : std::string();
             r.t = d.contains("t") ? d["t"].cast<double>() : 0.0;
             r.iso = d.contains("iso") ? d["iso"].cast<std::string>() : std::string();
             r.on_gpu = d.contains("on_gpu") && d["on_gpu"].cast<bool>();
             s.add_record(std::move(r));
           }, py::call_guard<AllocLock>())
      .def("drop_record", &AllocState::drop_record, py::call_guard<AllocLock>())
      .def("mark_on_gpu", &AllocState::mark_on_gpu, py::call_guard<AllocLock>())
      .def("physical_used", &AllocState::physical_used, py::call_guard<AllocLock>())
      .def("terminating_used", &AllocState::terminating_used, py::call_guard<AllocLock>())
      .def("terminating_dev", &AllocState::terminating_dev, py::call_guard<AllocLock>())
      .def("terminating_count", &AllocState::terminating_count, py::call_guard<AllocLock>())
      .def("off_gpu_records", &AllocState::off_gpu_records, py::call_guard<AllocLock>())
      .def("off_gpu_records_on", &AllocState::off_gpu_records_on, py::call_guard<AllocLock>())
      .def("prune_held", &AllocState::prune_held, py::arg("listed"), py::arg("asked"), py::arg("grace"),
           py::call_guard<AllocLock>())
      .def("held_count", &AllocState::held_count, py::call_guard<AllocLock>())
      .def("held_for", [](const AllocState& s, const std::vector<std::string>& ids) -> py::object {
             int64_t dev = -1, units = 0;
             double t = 0;
             std::string cu;
             if (!s.held_for(ids, &dev, &units, &t, &cu)) return py::none();
             py::dict d;
             d["dev"] = dev;
             d["units"] = units;
             d["t"] = t;
             d["cu_mask"] = cu;
             return d;
           }, py::call_guard<AllocLock>())
      .def("record_for_ids", [rec_dict](const AllocState& s, const std::vector<std::string>& ids) -> py::object {
             const AllocRecord* r = s.record_for_ids(ids);
             return r ? py::object(rec_dict(*r)) : py::object(py::none());
           }, py::call_guard<AllocLock>())
      .def("get_record", [rec_dict](AllocState& s, const std::string& aid) -> py::object {
             AllocRecord* r = s.record_by_aid(aid);
             return r ? py::object(rec_dict(*r)) : py::object(py::none());
           }, py::call_guard<AllocLock>())
      .def("set_owner", &AllocState::set_owner, py::call_guard<AllocLock>())
      .def("move_records", &AllocState::move_records, py::call_guard<AllocLock>())
      // copied under the state lock, converted to Python objects after it (the serving thread may be waiting)
      .def("records", [rec_dict](const AllocState& s) {
             std::vector<AllocRecord> copy;
             {
               AllocLock lock;
               copy.reserve(s.records().size());
               for (const auto& kv : s.records()) copy.push_back(kv.second);
             }
             py::list out;
             for (const auto& r : copy) out.append(rec_dict(r));
             return out;
           })
      .def("record_count", [](const AllocState& s) { return s.records().size(); }, py::call_guard<AllocLock>())
      .def("take_dropped", [rec_dict](AllocState& s) {
             py::list out;
             for (const auto& r : s.take_dropped()) out.append(rec_dict(r));
             return out;
           }, py::call_guard<AllocLock>())
      .def("cus", [](AllocState& s, int dev) { return s.cus(dev); }, py::return_value_policy::reference_internal, py::call_guard<AllocLock>())
      .def("devices", [](const AllocState& s) {
        std::vector<int> out;
        for (const auto& kv : s.all_cus()) out.push_back(kv.first);
        return out;
      }, py::call_guard<AllocLock>())
      .def("stats", [](const AllocState& s) {
        const AllocStats& st = s.stats();
        py::dict d;
        d["cu_released"] = st.cu_released;
        d["cu_adopted"] = st.cu_adopted;
        d["cu_conflicts"] = st.cu_conflicts;
        d["partial_released"] = st.partial_released;
        d["pods_released"] = st.pods_released;
        d["records_dropped"] = st.records_dropped;
        d["matches"] = st.matches;
        d["match_misses"] = st.match_misses;
        return d;
      }, py::call_guard<AllocLock>());

  // ApiClient's wait before resending a request answered `status` (Retry-After `retry_after`); < 0: not resent
  m.def("api_retry_wait", [](int status, const std::string& retry_after, int attempt, double jitter01) {
    return ApiClient::retry_wait(ApiConfig{}, "GET", status, retry_after, attempt, jitter01);
  });
  m.def("parse_quantity", [](const std::string& s) {
    int64_t v;
    if (!parse_quantity(s, &v)) throw py::value_error("quantities must match the regular expression");
    return v;
  });
  m.def("json_quote", [](const std::string& s) {
    std::string o;
    json::append_quoted(&o, s);
    return o;
  });
  m.def("json_validate", [](const py::bytes& b) {
    json::Doc d;
    std::string err;
    bool ok = d.parse(view_of(b), &err);
    return py::make_tuple(ok, err, static_cast<int64_t>(d.size()));
  });

  // ---- device plugin: native gRPC endpoint + the response / isolation code the Python plugin shares
  m.def("h2_available", []() {
    std::string err;
    bool ok = h2::available(&err);
    return py::make_tuple(ok, err);
  });
  m.def("build_response",
        [](const AllocPod& pod, const py::dict& dev, int64_t units, const std::vector<int>& cus,
           const std::string& mount_mode, const py::dict& profile) {
          return container_response_dict(
              build_response(pod, dp_device_from(dev), units, cus, mount_mode, profile_from(profile)));
        });
  m.def("isolation_config_text", &isolation_config_text);
  m.def("isolation_prepare", [](const std::string& host_dir, const std::string& uid, const std::vector<int>& cus,
                                int cu_count, int64_t limit, bool host_process) {
    std::vector<dp::MountMsg> mounts;
    std::map<std::string, std::string> envs;
    std::string err;
    if (!isolation_prepare(host_dir, uid, cus, cu_count, limit, host_process, &mounts, &envs, &err))
      throw std::runtime_error(err);
    py::list ml;
    for (const auto& x : mounts) {
      py::dict e;
      e["container_path"] = x.container_path;
      e["host_path"] = x.host_path;
      e["read_only"] = x.read_only;
      ml.append(e);
    }
    return py::make_tuple(ml, envs);
  });
  py::class_<PyDpServer>(m, "DpServer")
      .def(py::init<const std::string&, AllocState&, const py::dict&>(), py::keep_alive<1, 3>())
      .def("fd", &PyDpServer::fd)
      .def("poll", &PyDpServer::poll, py::call_guard<AllocLock>())
      .def("start_serving", &PyDpServer::start_serving, py::call_guard<AllocLock>())
      .def("journal_checkpoint", &PyDpServer::journal_checkpoint, py::call_guard<AllocLock>())
      .def("respond", &PyDpServer::respond, py::call_guard<AllocLock>())
      .def("set_devices", &PyDpServer::set_devices, py::call_guard<AllocLock>())
      .def("set_device_list", &PyDpServer::set_device_list, py::call_guard<AllocLock>())
      .def("set_fast", &PyDpServer::set_fast, py::call_guard<AllocLock>())
      .def("set_ready", &PyDpServer::set_ready, py::call_guard<AllocLock>())
      .def("set_state", &PyDpServer::set_state, py::keep_alive<1, 2>(), py::call_guard<AllocLock>())
      .def("start_feed", &PyDpServer::start_feed, py::call_guard<AllocLock>())
      .def("feed_synced", &PyDpServer::feed_synced, py::arg("timeout") = 30.0)
      .def("stats", &PyDpServer::stats, py::call_guard<AllocLock>())
      .def("close", &PyDpServer::close);
  py::class_<h2::Client>(m, "H2Client")
      .def(py::init<const std::string&>())
      .def("call", [](h2::Client& c, const std::string& path, const py::bytes& req, double timeout) {
        std::string resp, err;
        int status = 0;
        bool ok;
        std::string r(view_of(req));
        {
          py::gil_scoped_release nogil;
          ok = c.call(path, r, &resp, &status, &err, timeout);
        }
        return py::make_tuple(ok ? 0 : status, py::bytes(ok ? resp : err));
      }, py::arg("path"), py::arg("req"), py::arg("timeout") = 10.0);
  // test client (the compiled kubelet stand-in uses h2::Client directly)
  m.def("h2_call", [](const std::string& sock, const std::string& path, const py::bytes& req, double timeout) {
    h2::Client c(sock);
    std::string resp, err;
    int status = 0;
    bool ok;
    {
      py::gil_scoped_release nogil;
      ok = c.call(path, std::string(view_of(req)), &resp, &status, &err, timeout);
    }
    return py::make_tuple(ok ? 0 : status, py::bytes(ok ? resp : err));
  });
}
