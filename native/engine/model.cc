#include "model.h"

#include "quantity.h"

namespace gsx {

bool quantity_of(const json::Doc& d, int64_t idx, int64_t* out) {
  if (idx < 0) return false;
  const json::Val& v = d.at(static_cast<uint32_t>(idx));
  if (v.type == json::T::String) {
    std::string s = d.str(static_cast<uint32_t>(idx));
    return parse_quantity(s, out);
  }
  if (v.type == json::T::Number) {
    return parse_quantity(d.raw(static_cast<uint32_t>(idx)), out);
  }
  return false;
}

namespace {

std::string str_at(const json::Doc& d, int64_t idx) {
  if (idx < 0) return std::string();
  return d.str(static_cast<uint32_t>(idx));
}

}  // namespace

int64_t pod_limits_sum(const json::Doc& d, uint32_t pod, const std::string& name) {
  int64_t total = 0;
  int64_t cs = d.path(pod, {"spec", "containers"});
  if (cs < 0 || d.at(static_cast<uint32_t>(cs)).type != json::T::Array) return 0;
  uint32_t end = d.at(static_cast<uint32_t>(cs)).skip;
  for (uint32_t c = static_cast<uint32_t>(cs) + 1; c < end; c = d.next(c)) {
    if (d.at(c).type != json::T::Object) continue;
    int64_t lim = d.path(c, {"resources", "limits"});
    if (lim < 0) continue;
    int64_t q = d.find(static_cast<uint32_t>(lim), name);
    int64_t v = 0;
    if (quantity_of(d, q, &v)) {
      if (v > 0 && total > INT64_MAX - v) {
        total = INT64_MAX;
      } else {
        total += v;
      }
    }
  }
  return total;
}

Profile profile_by_name(const std::string& name) {
  Profile p;
  if (name == "aliyun") {
    p.resource = "aliyun.com/gpu-mem";
    p.count = "aliyun.com/gpu-count";
    p.a_idx = "ALIYUN_COM_GPU_MEM_IDX";
    p.a_pod = "ALIYUN_COM_GPU_MEM_POD";
    p.a_dev = "ALIYUN_COM_GPU_MEM_DEV";
    p.a_assigned = "ALIYUN_COM_GPU_MEM_ASSIGNED";
    p.a_assume = "ALIYUN_COM_GPU_MEM_ASSUME_TIME";
    p.env_container = "ALIYUN_COM_GPU_MEM_CONTAINER";
  }
  return p;
}

bool parse_pod(const json::Doc& d, uint32_t pod, const Profile& p, PodView* out) {
  if (pod >= d.size() || d.at(pod).type != json::T::Object) return false;
  int64_t meta = d.find(pod, "metadata");
  if (meta >= 0 && d.at(static_cast<uint32_t>(meta)).type == json::T::Object) {
    uint32_t m = static_cast<uint32_t>(meta);
    out->uid = str_at(d, d.find(m, "uid"));
    out->name = str_at(d, d.find(m, "name"));
    out->ns = str_at(d, d.find(m, "namespace"));
    out->rv = str_at(d, d.find(m, "resourceVersion"));
    int64_t dt = d.find(m, "deletionTimestamp");
    out->deleting = dt >= 0 && d.at(static_cast<uint32_t>(dt)).type != json::T::Null;
    int64_t an = d.find(m, "annotations");
    if (an >= 0 && d.at(static_cast<uint32_t>(an)).type == json::T::Object) {
      uint32_t a = static_cast<uint32_t>(an);
      int64_t v;
      int64_t i = d.find(a, p.a_idx);
      if (i >= 0) {
        std::string s = str_at(d, i);
        out->dev_idx = parse_atoi(s, &v) ? v : -1;
        if (out->dev_idx < -1) out->dev_idx = -1;
      }
      i = d.find(a, p.a_pod);
      if (i >= 0) {
        std::string s = str_at(d, i);
        out->has_annot_mem = true;
        out->annot_mem = parse_atoi(s, &v) ? (v < 0 ? 0 : v) : 0;
      }
      i = d.find(a, p.a_dev);
      if (i >= 0) {
        std::string s = str_at(d, i);
        out->annot_dev_total = parse_atoi(s, &v) ? v : -1;
      }
      i = d.find(a, p.a_assigned);
      if (i >= 0) {
        std::string s = str_at(d, i);
        out->assigned = (s == "true") ? 1 : 0;
      }
      i = d.find(a, p.a_assume);
      if (i >= 0) {
        std::string s = str_at(d, i);
        out->assume_time = parse_atoi(s, &v) ? v : -1;
      }
      i = d.find(a, "gpushare.amd.com/cu-mask");
      if (i >= 0) out->cu_mask = str_at(d, i);
      i = d.find(a, "gpushare.amd.com/hold-idx");
      if (i >= 0) {
        std::string s = str_at(d, i);
        out->hold_idx = parse_atoi(s, &v) && v >= 0 ? v : -1;
      }
    }
  }
  out->node = str_at(d, d.path(pod, {"spec", "nodeName"}));
  out->phase = str_at(d, d.path(pod, {"status", "phase"}));
  out->request = pod_limits_sum(d, pod, p.resource);
  return true;
}

bool parse_node(const json::Doc& d, uint32_t node, const Profile& p, NodeView* out) {
  if (node >= d.size() || d.at(node).type != json::T::Object) return false;
  out->name = str_at(d, d.path(node, {"metadata", "name"}));
  int64_t cap = d.path(node, {"status", "capacity"});
  if (cap >= 0) {
    int64_t v = 0;
    if (quantity_of(d, d.find(static_cast<uint32_t>(cap), p.resource), &v)) out->total = v;
    v = 0;
    if (quantity_of(d, d.find(static_cast<uint32_t>(cap), p.count), &v)) out->count = v;
  }
  int64_t an = d.path(node, {"metadata", "annotations"});
  if (an >= 0) {
    int64_t i = d.find(static_cast<uint32_t>(an), p.a_node_devs);
    if (i >= 0) {
      std::string s = str_at(d, i);
      size_t start = 0;
      bool ok = true;
      std::vector<int64_t> vals;
      while (start <= s.size()) {
        size_t comma = s.find(',', start);
        std::string_view tok(s.data() + start, (comma == std::string::npos ? s.size() : comma) - start);
        int64_t v;
        if (!parse_atoi(tok, &v) || v < 0) {
          ok = false;
          break;
        }
        vals.push_back(v);
        if (comma == std::string::npos) break;
        start = comma + 1;
      }
      if (ok) out->dev_totals = std::move(vals);
    }
    out->landing_order = str_at(d, d.find(static_cast<uint32_t>(an), kAllocateOrderAnnotation)) == "landing";
    out->publishes = str_at(d, d.find(static_cast<uint32_t>(an), kPhysicalPublicationAnnotation)) == "true";
  }
  int64_t addrs = d.path(node, {"status", "addresses"});
  if (addrs >= 0 && d.at(static_cast<uint32_t>(addrs)).type == json::T::Array) {
    uint32_t end = d.at(static_cast<uint32_t>(addrs)).skip;
    for (uint32_t a = static_cast<uint32_t>(addrs) + 1; a < end; a = d.next(a)) {
      if (str_at(d, d.find(a, "type")) == "InternalIP") {
        out->address = str_at(d, d.find(a, "address"));
        break;
      }
    }
  }
  return true;
}

}  // namespace gsx
