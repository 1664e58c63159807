// pybind11 module `_mxdev`: amdsmi-backed device inventory for the device plugin.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <memory>
#include <mutex>

#include "mxdev.h"

namespace py = pybind11;

namespace {

py::dict to_dict(const mxdev::DeviceRec& r) {
  py::dict d;
  d["index"] = r.index;
  d["name"] = r.name.empty() ? std::string("AMD Instinct MI355X") : r.name;
  d["arch"] = r.arch;
  d["bdf"] = r.bdf;
  d["uuid"] = r.uuid;
  d["total_bytes"] = r.total_bytes;
  d["cu_count"] = r.cu_count > 0 ? r.cu_count : 256;
  d["xcc_count"] = r.xcc_count;
  d["render_minor"] = r.render_minor;
  d["card_minor"] = r.card_minor;
  d["kfd_id"] = r.kfd_id;
  d["partition"] = r.partition;
  d["memory_partition"] = r.memory_partition;
  d["partition_id"] = r.partition_id;
  d["pool"] = r.pool;
  d["healthy"] = r.healthy;
  d["numa_node"] = r.numa_node;
  py::dict links;
  for (size_t j = 0; j < r.link_types.size(); ++j) links[py::int_(j)] = r.link_types[j];
  d["links"] = links;
  return d;
}

class Session {
 public:
  explicit Session(const std::string& backend) {
    std::string err;
    b_.reset(mxdev::make_backend(backend, &err));
    if (!b_) throw std::runtime_error(err);
  }
  std::string name() const { return b_->name(); }
  py::list devices() {
    std::vector<mxdev::DeviceRec> v;
    std::string err;
    {
      py::gil_scoped_release rel;
      std::lock_guard<std::mutex> g(mu_);
      if (!b_->enumerate(&v, &err)) throw std::runtime_error(err);
    }
    py::list out;
    for (auto& r : v) out.append(to_dict(r));
    return out;
  }
  py::dict health(int index) {
    mxdev::DeviceRec r;
    std::string err;
    bool ok;
    {
      py::gil_scoped_release rel;
      std::lock_guard<std::mutex> g(mu_);
      ok = b_->health(index, &r, &err);
    }
    if (!ok) throw std::runtime_error(err);
    py::dict d;
    d["healthy"] = r.healthy;
    d["reason"] = r.reason;
    d["ecc_uncorrectable"] = r.ecc_uncorrectable;
    d["ecc_correctable"] = r.ecc_correctable;
    d["ras_umc_uncorrectable"] = r.ras_umc_uncorrectable;
    d["ras_gfx_uncorrectable"] = r.ras_gfx_uncorrectable;
    d["ras_sdma_uncorrectable"] = r.ras_sdma_uncorrectable;
    d["ras_xgmi_uncorrectable"] = r.ras_xgmi_uncorrectable;
    d["ras_xgmi_correctable"] = r.ras_xgmi_correctable;
    d["xgmi_error"] = r.xgmi_error;
    d["thermal_throttle"] = r.thermal_throttle;
    d["power_throttle"] = r.power_throttle;
    d["partition"] = r.partition;
    d["memory_partition"] = r.memory_partition;
    return d;
  }
  void inject(int index, const std::string& what) {
    std::string err;
    std::lock_guard<std::mutex> g(mu_);
    if (!b_->inject(index, what, &err)) throw std::runtime_error(err);
  }
  void watch_events() {
    std::string err;
    std::lock_guard<std::mutex> g(mu_);
    if (!b_->watch_events(&err)) throw std::runtime_error(err);
  }
  py::list poll_events(int timeout_ms) {
    std::vector<mxdev::Event> ev;
    {
      py::gil_scoped_release rel;  // may block up to timeout_ms
      ev = b_->poll_events(timeout_ms);
    }
    py::list out;
    for (auto& e : ev) {
      py::dict d;
      d["index"] = e.index;
      d["type"] = e.type;
      d["name"] = e.name;
      d["message"] = e.message;
      out.append(d);
    }
    return out;
  }

 private:
  std::unique_ptr<mxdev::Backend> b_;
  std::mutex mu_;
};

}  // namespace

PYBIND11_MODULE(_mxdev, m) {
  m.doc() = "MI355X device inventory / health / topology over amdsmi (dlopen'ed)";
  py::class_<Session>(m, "Session")
      .def(py::init<const std::string&>(), py::arg("backend") = "auto")
      .def_property_readonly("backend", &Session::name)
      .def("devices", &Session::devices)
      .def("health", &Session::health)
      .def("watch_events", &Session::watch_events)
      .def("poll_events", &Session::poll_events, py::arg("timeout_ms") = 1000)
      .def("inject", &Session::inject, py::arg("index"), py::arg("what"));
  m.def("fake_spec_ok", [](const std::string& s) {
    std::vector<mxdev::DeviceRec> v;
    std::string err;
    return mxdev::fake_spec(s, &v, &err);
  });
}
