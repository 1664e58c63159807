#include "mxdev.h"

#include <dlfcn.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <regex>

#include <amd_smi/amdsmi.h>

namespace mxdev {

namespace {

// ---------------------------------------------------------------- amdsmi via dlopen

struct Api {
  void* h = nullptr;
  decltype(&amdsmi_init) init = nullptr;
  decltype(&amdsmi_shut_down) shut_down = nullptr;
  decltype(&amdsmi_get_socket_handles) sockets = nullptr;
  decltype(&amdsmi_get_processor_handles) procs = nullptr;
  decltype(&amdsmi_get_processor_type) ptype = nullptr;
  decltype(&amdsmi_get_gpu_device_bdf) bdf = nullptr;
  decltype(&amdsmi_get_gpu_device_uuid) uuid = nullptr;
  decltype(&amdsmi_get_gpu_enumeration_info) enum_info = nullptr;
  decltype(&amdsmi_get_gpu_memory_total) mem_total = nullptr;
  decltype(&amdsmi_get_gpu_memory_usage) mem_usage = nullptr;
  decltype(&amdsmi_get_gpu_asic_info) asic = nullptr;
  decltype(&amdsmi_get_gpu_kfd_info) kfd = nullptr;
  decltype(&amdsmi_get_gpu_compute_partition) cpart = nullptr;
  decltype(&amdsmi_get_gpu_memory_partition) mpart = nullptr;
  decltype(&amdsmi_get_gpu_total_ecc_count) ecc = nullptr;
  decltype(&amdsmi_get_gpu_ecc_count) ecc_block = nullptr;
  decltype(&amdsmi_gpu_xgmi_error_status) xgmi_status = nullptr;
  decltype(&amdsmi_get_violation_status) violation = nullptr;
  decltype(&amdsmi_topo_get_link_type) link_type = nullptr;
  decltype(&amdsmi_topo_get_numa_node_number) numa = nullptr;
  decltype(&amdsmi_init_gpu_event_notification) evt_init = nullptr;
  decltype(&amdsmi_set_gpu_event_notification_mask) evt_mask = nullptr;
  decltype(&amdsmi_get_gpu_event_notification) evt_get = nullptr;
  decltype(&amdsmi_status_code_to_string) status_str = nullptr;

  template <typename F>
  bool sym(F* f, const char* name, bool required, std::string* err) {
    *f = reinterpret_cast<F>(dlsym(h, name));
    if (!*f && required) {
      *err = std::string("amdsmi symbol missing: ") + name;
      return false;
    }
    return true;
  }

  bool load(std::string* err) {
    // GSX_AMDSMI_LIB: another amdsmi library first (tests load native/mxdev/fake_amdsmi.cc, a shuffled topology)
    const char* over = std::getenv("GSX_AMDSMI_LIB");
    if (over && *over) h = dlopen(over, RTLD_NOW | RTLD_LOCAL | RTLD_DEEPBIND);
    const char* cands[] = {"/opt/rocm/lib/libamd_smi.so", "libamd_smi.so.26", "libamd_smi.so"};
    for (const char* c : cands) {
      if (h) break;
      h = dlopen(c, RTLD_NOW | RTLD_LOCAL | RTLD_DEEPBIND);
    }
    if (!h) {
      *err = std::string("dlopen libamd_smi failed: ") + dlerror();
      return false;
    }
    return sym(&init, "amdsmi_init", true, err) && sym(&shut_down, "amdsmi_shut_down", true, err) &&
           sym(&sockets, "amdsmi_get_socket_handles", true, err) &&
           sym(&procs, "amdsmi_get_processor_handles", true, err) &&
           sym(&ptype, "amdsmi_get_processor_type", false, err) &&
           sym(&bdf, "amdsmi_get_gpu_device_bdf", true, err) && sym(&uuid, "amdsmi_get_gpu_device_uuid", false, err) &&
           sym(&enum_info, "amdsmi_get_gpu_enumeration_info", false, err) &&
           sym(&mem_total, "amdsmi_get_gpu_memory_total", true, err) &&
           sym(&mem_usage, "amdsmi_get_gpu_memory_usage", false, err) &&
           sym(&asic, "amdsmi_get_gpu_asic_info", false, err) && sym(&kfd, "amdsmi_get_gpu_kfd_info", false, err) &&
           sym(&cpart, "amdsmi_get_gpu_compute_partition", false, err) &&
           sym(&mpart, "amdsmi_get_gpu_memory_partition", false, err) &&
           sym(&ecc, "amdsmi_get_gpu_total_ecc_count", false, err) &&
           sym(&ecc_block, "amdsmi_get_gpu_ecc_count", false, err) &&
           sym(&xgmi_status, "amdsmi_gpu_xgmi_error_status", false, err) &&
           sym(&violation, "amdsmi_get_violation_status", false, err) &&
           sym(&link_type, "amdsmi_topo_get_link_type", false, err) &&
           sym(&numa, "amdsmi_topo_get_numa_node_number", false, err) &&
           sym(&evt_init, "amdsmi_init_gpu_event_notification", false, err) &&
           sym(&evt_mask, "amdsmi_set_gpu_event_notification_mask", false, err) &&
           sym(&evt_get, "amdsmi_get_gpu_event_notification", false, err) &&
           sym(&status_str, "amdsmi_status_code_to_string", false, err);
  }

  std::string why(amdsmi_status_t st) const {
    const char* s = nullptr;
    if (status_str && status_str(st, &s) == AMDSMI_STATUS_SUCCESS && s) return s;
    return "amdsmi status " + std::to_string(static_cast<int>(st));
  }
};

const char* event_name(int t) {
  switch (t) {
    case AMDSMI_EVT_NOTIF_VMFAULT: return "VMFAULT";
    case AMDSMI_EVT_NOTIF_THERMAL_THROTTLE: return "THERMAL_THROTTLE";
    case AMDSMI_EVT_NOTIF_GPU_PRE_RESET: return "GPU_PRE_RESET";
    case AMDSMI_EVT_NOTIF_GPU_POST_RESET: return "GPU_POST_RESET";
    case AMDSMI_EVT_NOTIF_QUEUE_EVICTION: return "QUEUE_EVICTION";
    case AMDSMI_EVT_NOTIF_QUEUE_RESTORE: return "QUEUE_RESTORE";
    default: return "OTHER";
  }
}

std::string bdf_str(amdsmi_bdf_t b) {
  char buf[32];
  std::snprintf(buf, sizeof(buf), "%04llx:%02llx:%02llx.%llx", static_cast<unsigned long long>(b.bdf.domain_number),
                static_cast<unsigned long long>(b.bdf.bus_number), static_cast<unsigned long long>(b.bdf.device_number),
                static_cast<unsigned long long>(b.bdf.function_number));
  return buf;
}

class AmdSmi : public Backend {
 public:
  ~AmdSmi() override {
    if (inited_ && api_.shut_down) api_.shut_down();
  }

  bool open(std::string* err) {
    if (!api_.load(err)) return false;
    amdsmi_status_t st = api_.init(AMDSMI_INIT_AMD_GPUS);
    if (st != AMDSMI_STATUS_SUCCESS) {
      *err = "amdsmi_init: " + api_.why(st);
      return false;
    }
    inited_ = true;
    return true;
  }

  std::string name() const override { return "amdsmi"; }

  bool handles(std::vector<amdsmi_processor_handle>* out, std::string* err) {
    uint32_t ns = 0;
    amdsmi_status_t st = api_.sockets(&ns, nullptr);
    if (st != AMDSMI_STATUS_SUCCESS) {
      *err = "amdsmi_get_socket_handles: " + api_.why(st);
      return false;
    }
    std::vector<amdsmi_socket_handle> socks(ns);
    if (ns) api_.sockets(&ns, socks.data());
    for (uint32_t s = 0; s < ns; ++s) {
      uint32_t np = 0;
      if (api_.procs(socks[s], &np, nullptr) != AMDSMI_STATUS_SUCCESS) continue;
      std::vector<amdsmi_processor_handle> ps(np);
      if (np) api_.procs(socks[s], &np, ps.data());
      for (auto p : ps) {
        if (api_.ptype) {
          processor_type_t t;
          if (api_.ptype(p, &t) == AMDSMI_STATUS_SUCCESS && t != AMDSMI_PROCESSOR_TYPE_AMD_GPU) continue;
        }
        out->push_back(p);
      }
    }
    return true;
  }

  bool enumerate(std::vector<DeviceRec>* out, std::string* err) override {
    handles_.clear();
    if (!handles(&handles_, err)) return false;
    std::vector<std::pair<int, DeviceRec>> recs;
    int ordinal = 0;
    for (auto p : handles_) {
      DeviceRec r;
      r.index = ordinal;
      amdsmi_bdf_t b;
      if (api_.bdf(p, &b) == AMDSMI_STATUS_SUCCESS) r.bdf = bdf_str(b);
      if (api_.uuid) {
        char u[AMDSMI_MAX_STRING_LENGTH] = {0};
        unsigned int n = sizeof(u);
        if (api_.uuid(p, &n, u) == AMDSMI_STATUS_SUCCESS) r.uuid = u;
      }
      if (api_.enum_info) {
        amdsmi_enumeration_info_t e;
        std::memset(&e, 0, sizeof(e));
        if (api_.enum_info(p, &e) == AMDSMI_STATUS_SUCCESS) {
          r.render_minor = static_cast<int>(e.drm_render);
          r.card_minor = static_cast<int>(e.drm_card);
          r.hsa_id = static_cast<int>(e.hsa_id);
          r.index = static_cast<int>(e.hip_id);
        }
      }
      uint64_t tot = 0;
      if (api_.mem_total(p, AMDSMI_MEM_TYPE_VRAM, &tot) == AMDSMI_STATUS_SUCCESS) r.total_bytes = tot;
      if (api_.mem_usage) {
        uint64_t u = 0;
        if (api_.mem_usage(p, AMDSMI_MEM_TYPE_VRAM, &u) == AMDSMI_STATUS_SUCCESS) r.used_bytes = u;
      }
      if (api_.asic) {
        amdsmi_asic_info_t a;
        std::memset(&a, 0, sizeof(a));
        if (api_.asic(p, &a) == AMDSMI_STATUS_SUCCESS) {
          r.name = a.market_name;
          if (a.num_of_compute_units != 0xFFFFFFFFu) r.cu_count = static_cast<int>(a.num_of_compute_units);
        }
      }
      if (api_.kfd) {
        amdsmi_kfd_info_t k;
        std::memset(&k, 0, sizeof(k));
        if (api_.kfd(p, &k) == AMDSMI_STATUS_SUCCESS) {
          if (k.kfd_id != ~0ull) r.kfd_id = static_cast<int64_t>(k.kfd_id);
          if (k.current_partition_id != 0xFFFFFFFFu) r.partition_id = static_cast<int>(k.current_partition_id);
        }
      }
      if (api_.cpart) {
        char buf[64] = {0};
        if (api_.cpart(p, buf, sizeof(buf)) == AMDSMI_STATUS_SUCCESS && buf[0]) r.partition = buf;
      }
      if (api_.mpart) {
        char buf[64] = {0};
        if (api_.mpart(p, buf, sizeof(buf)) == AMDSMI_STATUS_SUCCESS) r.memory_partition = buf;
      }
      r.xcc_count = xcds_for_partition(r.partition);
      // partitions of one GPU differ only in the PCI function number
      r.pool = r.bdf.size() > 2 ? r.bdf.substr(0, r.bdf.size() - 2) : r.bdf;
      if (api_.numa) {
        uint32_t nn = 0;
        if (api_.numa(p, &nn) == AMDSMI_STATUS_SUCCESS) r.numa_node = static_cast<int>(nn);
      }
      std::string e2;
      health_of(p, &r, &e2);
      recs.emplace_back(ordinal, std::move(r));
      ++ordinal;
    }
    // link types between every pair (xGMI on MI355X OAM platforms)
    for (size_t i = 0; i < recs.size(); ++i) {
      auto& r = recs[i].second;
      r.link_types.assign(recs.size(), "UNKNOWN");
      for (size_t j = 0; j < recs.size(); ++j) {
        if (i == j) {
          r.link_types[j] = "SELF";
          continue;
        }
        if (!api_.link_type) continue;
        uint64_t hops = 0;
        amdsmi_link_type_t t;
        if (api_.link_type(handles_[i], handles_[j], &hops, &t) == AMDSMI_STATUS_SUCCESS) {
          r.link_types[j] = t == AMDSMI_LINK_TYPE_XGMI ? "XGMI" : t == AMDSMI_LINK_TYPE_PCIE ? "PCIE" : "OTHER";
        }
      }
    }
    std::sort(recs.begin(), recs.end(), [](const auto& a, const auto& b) { return a.second.index < b.second.index; });
    // link_types were built in amdsmi order; re-index them by HIP index
    std::vector<int> hip_of(recs.size());
    for (size_t k = 0; k < recs.size(); ++k) hip_of[static_cast<size_t>(recs[k].first)] = recs[k].second.index;
    order_ = hip_of;
    for (auto& pr : recs) {
      std::vector<std::string> lt(pr.second.link_types.size());
      for (size_t j = 0; j < lt.size(); ++j) {
        size_t dst = static_cast<size_t>(hip_of[j]);
        if (dst < lt.size()) lt[dst] = pr.second.link_types[j];
      }
      pr.second.link_types = lt;
      out->push_back(pr.second);
    }
    return true;
  }

  bool health_of(amdsmi_processor_handle p, DeviceRec* r, std::string* err) {
    // every counter is optional: unsupported (e.g. inside some VMs) is not unhealthy
    if (api_.ecc) {
      amdsmi_error_count_t ec;
      std::memset(&ec, 0, sizeof(ec));
      if (api_.ecc(p, &ec) == AMDSMI_STATUS_SUCCESS) {
        r->ecc_uncorrectable = ec.uncorrectable_count;
        r->ecc_correctable = ec.correctable_count;
      }
    }
    if (api_.ecc_block) {
      auto block = [&](amdsmi_gpu_block_t b, uint64_t* unc, uint64_t* cor) {
        amdsmi_error_count_t ec;
        std::memset(&ec, 0, sizeof(ec));
        if (api_.ecc_block(p, b, &ec) == AMDSMI_STATUS_SUCCESS) {
          *unc = ec.uncorrectable_count;
          if (cor) *cor = ec.correctable_count;
        }
      };
      block(AMDSMI_GPU_BLOCK_UMC, &r->ras_umc_uncorrectable, nullptr);
      block(AMDSMI_GPU_BLOCK_GFX, &r->ras_gfx_uncorrectable, nullptr);
      block(AMDSMI_GPU_BLOCK_SDMA, &r->ras_sdma_uncorrectable, nullptr);
      block(AMDSMI_GPU_BLOCK_XGMI_WAFL, &r->ras_xgmi_uncorrectable, &r->ras_xgmi_correctable);
    }
    if (api_.xgmi_status) {
      amdsmi_xgmi_status_t xs = AMDSMI_XGMI_STATUS_NO_ERRORS;
      if (api_.xgmi_status(p, &xs) == AMDSMI_STATUS_SUCCESS) r->xgmi_error = static_cast<int>(xs);
    }
    if (api_.violation) {
      amdsmi_violation_status_t v;
      std::memset(&v, 0, sizeof(v));
      if (api_.violation(p, &v) == AMDSMI_STATUS_SUCCESS) {
        auto on = [](uint8_t x) { return x == 1; };  // 0xFF = unsupported
        r->thermal_throttle = on(v.active_prochot_thrm) || on(v.active_socket_thrm) || on(v.active_hbm_thrm) ||
                              on(v.active_vr_thrm);
        r->power_throttle = on(v.active_ppt_pwr);
      }
    }
    // the partition modes are re-read every poll: a runtime change re-shapes the node's devices
    if (api_.cpart) {
      char buf[64] = {0};
      if (api_.cpart(p, buf, sizeof(buf)) == AMDSMI_STATUS_SUCCESS && buf[0]) r->partition = buf;
    }
    if (api_.mpart) {
      char buf[64] = {0};
      if (api_.mpart(p, buf, sizeof(buf)) == AMDSMI_STATUS_SUCCESS) r->memory_partition = buf;
    }
    classify(r);
    return true;
  }

  bool health(int index, DeviceRec* rec, std::string* err) override {
    if (handles_.empty()) {
      std::vector<DeviceRec> tmp;
      if (!enumerate(&tmp, err)) return false;
    }
    for (size_t k = 0; k < order_.size(); ++k) {
      if (order_[k] == index) return health_of(handles_[k], rec, err);
    }
    *err = "no device with index " + std::to_string(index);
    return false;
  }

  bool watch_events(std::string* err) override {
    if (!api_.evt_init || !api_.evt_mask || !api_.evt_get) {
      *err = "amdsmi event notification API not available";
      return false;
    }
    if (handles_.empty()) {
      std::vector<DeviceRec> tmp;
      if (!enumerate(&tmp, err)) return false;
    }
    uint64_t mask = AMDSMI_EVENT_MASK_FROM_INDEX(AMDSMI_EVT_NOTIF_VMFAULT) |
                    AMDSMI_EVENT_MASK_FROM_INDEX(AMDSMI_EVT_NOTIF_THERMAL_THROTTLE) |
                    AMDSMI_EVENT_MASK_FROM_INDEX(AMDSMI_EVT_NOTIF_GPU_PRE_RESET) |
                    AMDSMI_EVENT_MASK_FROM_INDEX(AMDSMI_EVT_NOTIF_GPU_POST_RESET);
    for (auto p : handles_) {
      amdsmi_status_t st = api_.evt_init(p);
      if (st != AMDSMI_STATUS_SUCCESS) {
        *err = "amdsmi_init_gpu_event_notification: " + api_.why(st);
        return false;
      }
      st = api_.evt_mask(p, mask);
      if (st != AMDSMI_STATUS_SUCCESS) {
        *err = "amdsmi_set_gpu_event_notification_mask: " + api_.why(st);
        return false;
      }
    }
    watching_ = true;
    return true;
  }

  std::vector<Event> poll_events(int timeout_ms) override {
    std::vector<Event> out;
    if (!watching_) return out;
    amdsmi_evt_notification_data_t data[16];
    uint32_t n = 16;
    if (api_.evt_get(timeout_ms, &n, data) != AMDSMI_STATUS_SUCCESS) return out;
    for (uint32_t i = 0; i < n; ++i) {
      int idx = -1;
      for (size_t k = 0; k < handles_.size(); ++k) {
        if (handles_[k] == data[i].processor_handle) idx = k < order_.size() ? order_[k] : static_cast<int>(k);
      }
      out.push_back(Event{idx, static_cast<int>(data[i].event), event_name(data[i].event), data[i].message});
    }
    return out;
  }

 private:
  Api api_;
  bool inited_ = false;
  bool watching_ = false;
  std::vector<amdsmi_processor_handle> handles_;
  std::vector<int> order_;  // amdsmi ordinal -> HIP index
};

// ---------------------------------------------------------------- fake backend

class Fake : public Backend {
 public:
  Fake(std::vector<DeviceRec> d, std::string spec) : devs_(std::move(d)), spec_(std::move(spec)) {}
  std::string name() const override { return "fake"; }
  bool enumerate(std::vector<DeviceRec>* out, std::string*) override {
    std::lock_guard<std::mutex> g(mu_);
    *out = devs_;
    return true;
  }
  bool health(int index, DeviceRec* rec, std::string* err) override {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& d : devs_) {
      if (d.index == index) {
        *rec = d;
        classify(rec);
        return true;
      }
    }
    *err = "no device with index " + std::to_string(index);
    return false;
  }
  bool watch_events(std::string*) override { return true; }
  std::vector<Event> poll_events(int timeout_ms) override {
    std::unique_lock<std::mutex> g(mu_);
    if (events_.empty()) cv_.wait_for(g, std::chrono::milliseconds(timeout_ms));
    std::vector<Event> out;
    out.swap(events_);
    return out;
  }
  bool inject(int index, const std::string& what, std::string* err) override {
    size_t eq = what.find('=');
    if (eq == std::string::npos) {
      *err = "inject wants key=value";
      return false;
    }
    std::string k = what.substr(0, eq), v = what.substr(eq + 1);
    std::lock_guard<std::mutex> g(mu_);
    if (k == "partition" || k == "memory_partition") {
      // the whole node re-partitions (amd-smi set on every GPU): the logical devices are generated again
      std::string mode = k == "partition" ? v : devs_.empty() ? "SPX" : devs_[0].partition;
      std::string nps = k == "memory_partition" ? v : devs_.empty() ? "NPS1" : devs_[0].memory_partition;
      size_t c1 = spec_.find(':');
      std::string base = c1 == std::string::npos ? spec_ : spec_.substr(0, c1);
      std::string spec = base + ":" + mode + (nps.empty() || nps == "NPS1" ? "" : ":" + nps);
      std::vector<DeviceRec> d;
      if (!fake_spec(spec, &d, err)) return false;
      devs_ = std::move(d);
      spec_ = spec;
      return true;
    }
    for (auto& d : devs_) {
      if (d.index != index) continue;
      uint64_t n = std::strtoull(v.c_str(), nullptr, 10);
      if (k == "ecc_uncorrectable") d.ecc_uncorrectable = n;
      else if (k == "ecc_correctable") d.ecc_correctable = n;
      else if (k == "ras_umc_uncorrectable") d.ras_umc_uncorrectable = n;
      else if (k == "ras_gfx_uncorrectable") d.ras_gfx_uncorrectable = n;
      else if (k == "ras_xgmi_uncorrectable") d.ras_xgmi_uncorrectable = n;
      else if (k == "xgmi_error") d.xgmi_error = static_cast<int>(n);
      else if (k == "thermal_throttle") d.thermal_throttle = n != 0;
      else if (k == "power_throttle") d.power_throttle = n != 0;
      else if (k == "event") {
        int t = v == "GPU_PRE_RESET" ? AMDSMI_EVT_NOTIF_GPU_PRE_RESET : v == "GPU_POST_RESET" ? AMDSMI_EVT_NOTIF_GPU_POST_RESET
                : v == "VMFAULT" ? AMDSMI_EVT_NOTIF_VMFAULT : AMDSMI_EVT_NOTIF_THERMAL_THROTTLE;
        events_.push_back(Event{index, t, event_name(t), "injected"});
        cv_.notify_all();
      } else {
        *err = "unknown fault " + k;
        return false;
      }
      return true;
    }
    *err = "no device with index " + std::to_string(index);
    return false;
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<DeviceRec> devs_;
  std::string spec_;
  std::vector<Event> events_;
};

}  // namespace

void classify(DeviceRec* r) {
  std::string why;
  auto add = [&](const std::string& s) { why += (why.empty() ? "" : ", ") + s; };
  if (r->ecc_uncorrectable) add("ecc uncorrectable=" + std::to_string(r->ecc_uncorrectable));
  if (r->ras_umc_uncorrectable) add("HBM (UMC) uncorrectable=" + std::to_string(r->ras_umc_uncorrectable));
  if (r->ras_gfx_uncorrectable) add("GFX uncorrectable=" + std::to_string(r->ras_gfx_uncorrectable));
  if (r->ras_sdma_uncorrectable) add("SDMA uncorrectable=" + std::to_string(r->ras_sdma_uncorrectable));
  if (r->ras_xgmi_uncorrectable) add("xGMI uncorrectable=" + std::to_string(r->ras_xgmi_uncorrectable));
  if (r->xgmi_error) add(r->xgmi_error == 2 ? "xGMI multiple errors" : "xGMI error");
  r->healthy = why.empty();
  r->reason = why;
}

int partitions_for_mode(const std::string& mode) {
  if (mode == "CPX") return 8;
  if (mode == "QPX") return 4;
  if (mode == "DPX") return 2;
  return 1;  // SPX / unknown
}

int xcds_for_partition(const std::string& mode) { return 8 / partitions_for_mode(mode); }

bool fake_spec(const std::string& spec, std::vector<DeviceRec>* out, std::string* err) {
  static const std::regex re(
      R"(^(\d+)x(\d+(?:\.\d+)?)(GB|GiB|MiB|MB)(?::(SPX|DPX|QPX|CPX))?(?::NPS(1|2|4|8))?$)");
  std::smatch m;
  if (!std::regex_match(spec, m, re)) {
    *err = "fake spec must look like 8x288GB, got '" + spec + "'";
    return false;
  }
  int n = std::stoi(m[1].str());
  double size = std::stod(m[2].str());
  std::string u = m[3].str();
  double mult = u == "GB" ? 1e9 : u == "GiB" ? 1073741824.0 : u == "MiB" ? 1048576.0 : 1e6;
  if (n <= 0 || n > 64) {
    *err = "fake device count out of range";
    return false;
  }
  const std::string mode = m[4].matched ? m[4].str() : "SPX";
  const int nps = m[5].matched ? std::stoi(m[5].str()) : 1;
  const int parts = partitions_for_mode(mode);
  if (nps > parts) {
    *err = "NPS" + std::to_string(nps) + " needs at least as many compute partitions (" + mode + ")";
    return false;
  }
  const int total = n * parts;
  if (total > 64) {
    *err = "fake logical device count out of range";
    return false;
  }
  out->clear();
  // each logical device reports the VRAM of its memory pool (the whole GPU in NPS1)
  const uint64_t pool_bytes = static_cast<uint64_t>(std::llround(size * mult)) / static_cast<uint64_t>(nps);
  for (int g = 0; g < n; ++g) {
    for (int p = 0; p < parts; ++p) {
      const int i = g * parts + p;
      DeviceRec r;
      r.index = i;
      r.name = "AMD Instinct MI355X";
      char bdf[32];
      std::snprintf(bdf, sizeof(bdf), "0000:%02x:00.%d", 0x05 + 0x10 * g, p);
      r.bdf = bdf;
      r.pool = r.bdf.substr(0, r.bdf.size() - 2);
      r.uuid = "fake-" + std::to_string(i);
      r.total_bytes = pool_bytes;
      r.cu_count = 256 / parts;
      r.xcc_count = 8 / parts;
      r.partition = mode;
      r.memory_partition = "NPS" + std::to_string(nps);
      r.partition_id = p;
      r.render_minor = parts == 1 ? 128 + 8 * i : 128 + i;
      r.card_minor = i + 1;
      r.kfd_id = i;
      r.hsa_id = i + 1;
      r.link_types.assign(static_cast<size_t>(total), "XGMI");
      r.link_types[static_cast<size_t>(i)] = "SELF";
      out->push_back(r);
    }
  }
  return true;
}

Backend* make_backend(const std::string& kind, std::string* err) {
  if (kind.rfind("fake:", 0) == 0) {
    std::vector<DeviceRec> d;
    if (!fake_spec(kind.substr(5), &d, err)) return nullptr;
    return new Fake(std::move(d), kind.substr(5));
  }
  if (kind == "amdsmi" || kind == "auto") {
    auto* b = new AmdSmi();
    if (!b->open(err)) {
      delete b;
      return nullptr;
    }
    return b;
  }
  *err = "unknown backend '" + kind + "'";
  return nullptr;
}

}  // namespace mxdev
