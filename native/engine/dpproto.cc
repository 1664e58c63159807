#include "dpproto.h"

#include <cstring>

#include <algorithm>

#include <string_view>

namespace gsx::dp {
namespace {

// ------------------------------------------------------------------ writer
void varint(std::string* o, uint64_t v) {
  while (v >= 0x80) {
    o->push_back(static_cast<char>((v & 0x7f) | 0x80));
    v >>= 7;
  }
  o->push_back(static_cast<char>(v));
}
void tag(std::string* o, int field, int wire) { varint(o, (static_cast<uint64_t>(field) << 3) | wire); }
void bytes(std::string* o, int field, std::string_view s) {
  tag(o, field, 2);
  varint(o, s.size());
  o->append(s);
}
void str_if(std::string* o, int field, const std::string& s) {
  if (!s.empty()) bytes(o, field, s);
}
void boolean(std::string* o, int field, bool b) {
  if (!b) return;
  tag(o, field, 0);
  varint(o, 1);
}
void int_field(std::string* o, int field, int64_t v) {
  if (v == 0) return;
  tag(o, field, 0);
  varint(o, static_cast<uint64_t>(v));
}
std::string map_entry(const std::string& k, const std::string& v) {
  std::string e;
  str_if(&e, 1, k);
  str_if(&e, 2, v);
  return e;
}

// ------------------------------------------------------------------ reader
struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  explicit Reader(std::string_view s)
      : p(reinterpret_cast<const uint8_t*>(s.data())), end(reinterpret_cast<const uint8_t*>(s.data()) + s.size()) {}
  bool done() const { return p >= end; }
  bool varint(uint64_t* v) {
    *v = 0;
    for (int shift = 0; shift < 64 && p < end; shift += 7) {
      uint8_t b = *p++;
      *v |= static_cast<uint64_t>(b & 0x7f) << shift;
      if (!(b & 0x80)) return true;
    }
    return false;
  }
  // next field: number, wire type and (for wire 2) the payload; other wire types are skipped into *num only
  bool next(int* field, int* wire, std::string_view* payload, uint64_t* value) {
    uint64_t t;
    if (!varint(&t)) return false;
    *field = static_cast<int>(t >> 3);
    *wire = static_cast<int>(t & 7);
    switch (*wire) {
      case 0:
        return varint(value);
      case 1:
        if (end - p < 8) return false;
        p += 8;
        return true;
      case 2: {
        uint64_t n;
        if (!varint(&n) || static_cast<uint64_t>(end - p) < n) return false;
        *payload = std::string_view(reinterpret_cast<const char*>(p), n);  // a view into the message: no copy
        p += n;
        return true;
      }
      case 5:
        if (end - p < 4) return false;
        p += 4;
        return true;
      default:
        return false;
    }
  }
};

template <typename Fn>
bool each(std::string_view msg, Fn fn) {
  Reader r(msg);
  while (!r.done()) {
    int f, w;
    std::string_view pl;
    uint64_t v = 0;
    if (!r.next(&f, &w, &pl, &v)) return false;
    if (!fn(f, w, pl, v)) return false;
  }
  return true;
}

bool decode_map_entry(std::string_view e, std::string* k, std::string* v) {
  return each(e, [&](int f, int w, std::string_view pl, uint64_t) {
    if (w == 2 && f == 1) *k = pl;
    if (w == 2 && f == 2) *v = pl;
    return true;
  });
}

}  // namespace

std::string encode_options(bool pre_start_required, bool preferred_available) {
  std::string o;
  boolean(&o, 1, pre_start_required);
  boolean(&o, 2, preferred_available);
  return o;
}

std::string encode_list_and_watch(const std::vector<DeviceMsg>& devs) {
  std::string o;
  for (const auto& d : devs) {
    std::string m;
    str_if(&m, 1, d.id);
    str_if(&m, 2, d.health);
    if (!d.numa.empty()) {
      std::string topo;
      for (int64_t n : d.numa) {
        std::string node;
        int_field(&node, 1, n);
        bytes(&topo, 1, node);
      }
      bytes(&m, 3, topo);
    }
    bytes(&o, 1, m);
  }
  return o;
}

std::string encode_preferred_response(const std::vector<std::vector<std::string>>& per_container) {
  std::string o;
  for (const auto& ids : per_container) {
    std::string c;
    for (const auto& id : ids) bytes(&c, 1, id);
    bytes(&o, 1, c);
  }
  return o;
}

namespace {
// Sizes of the nested messages, so the response is written in one pass into one buffer (it answers every
// Allocate on kubelet's serial admission path): no temporary string per map entry, mount or device.
size_t varint_len(uint64_t v) {
  size_t n = 1;
  while (v >= 0x80) {
    v >>= 7;
    ++n;
  }
  return n;
}
size_t str_field_len(size_t n) { return n ? 1 + varint_len(n) + n : 0; }  // str_if: absent when empty
void str_field(std::string* o, int field, const std::string& s) {
  if (s.empty()) return;
  tag(o, field, 2);
  varint(o, s.size());
  o->append(s);
}
size_t entry_len(const std::string& k, const std::string& v) { return str_field_len(k.size()) + str_field_len(v.size()); }
void entry(std::string* o, int field, const std::string& k, const std::string& v) {
  tag(o, field, 2);
  varint(o, entry_len(k, v));
  str_field(o, 1, k);
  str_field(o, 2, v);
}
size_t mount_len(const MountMsg& m) {
  return str_field_len(m.container_path.size()) + str_field_len(m.host_path.size()) + (m.read_only ? 2 : 0);
}
size_t device_len(const DeviceSpecMsg& d) {
  return str_field_len(d.container_path.size()) + str_field_len(d.host_path.size()) +
         str_field_len(d.permissions.size());
}
size_t container_len(const ContainerResponse& r) {
  size_t n = 0;
  for (const auto& kv : r.envs) n += 1 + varint_len(entry_len(kv.first, kv.second)) + entry_len(kv.first, kv.second);
  for (const auto& m : r.mounts) n += 1 + varint_len(mount_len(m)) + mount_len(m);
  for (const auto& d : r.devices) n += 1 + varint_len(device_len(d)) + device_len(d);
  for (const auto& kv : r.annotations) n += 1 + varint_len(entry_len(kv.first, kv.second)) + entry_len(kv.first, kv.second);
  return n;
}

}  // namespace

std::string encode_allocate_response(const std::vector<ContainerResponse>& per_container) {
  size_t total = 0;
  std::vector<size_t> lens;
  lens.reserve(per_container.size());
  for (const auto& r : per_container) {
    lens.push_back(container_len(r));
    total += 1 + varint_len(lens.back()) + lens.back();
  }
  std::string o;
  o.reserve(total);
  for (size_t i = 0; i < per_container.size(); ++i) {
    const ContainerResponse& r = per_container[i];
    tag(&o, 1, 2);
    varint(&o, lens[i]);
    for (const auto& kv : r.envs) entry(&o, 1, kv.first, kv.second);
    for (const auto& m : r.mounts) {
      tag(&o, 2, 2);
      varint(&o, mount_len(m));
      str_field(&o, 1, m.container_path);
      str_field(&o, 2, m.host_path);
      if (m.read_only) {
        tag(&o, 3, 0);
        varint(&o, 1);
      }
    }
    for (const auto& d : r.devices) {
      tag(&o, 3, 2);
      varint(&o, device_len(d));
      str_field(&o, 1, d.container_path);
      str_field(&o, 2, d.host_path);
      str_field(&o, 3, d.permissions);
    }
    for (const auto& kv : r.annotations) entry(&o, 4, kv.first, kv.second);
  }
  return o;
}

namespace {
std::string encode_allocate_response_ref(const std::vector<ContainerResponse>& per_container) {
  std::string o;
  for (const auto& r : per_container) {
    std::string c;
    for (const auto& kv : r.envs) bytes(&c, 1, map_entry(kv.first, kv.second));
    for (const auto& m : r.mounts) {
      std::string e;
      str_if(&e, 1, m.container_path);
      str_if(&e, 2, m.host_path);
      boolean(&e, 3, m.read_only);
      bytes(&c, 2, e);
    }
    for (const auto& d : r.devices) {
      std::string e;
      str_if(&e, 1, d.container_path);
      str_if(&e, 2, d.host_path);
      str_if(&e, 3, d.permissions);
      bytes(&c, 3, e);
    }
    for (const auto& kv : r.annotations) bytes(&c, 4, map_entry(kv.first, kv.second));
    bytes(&o, 1, c);
  }
  return o;
}
}  // namespace

// The straightforward encoder the one-pass one must match byte for byte (tests: dp_selfcheck).
bool encode_allocate_response_selfcheck(const std::vector<ContainerResponse>& per_container) {
  return encode_allocate_response(per_container) == encode_allocate_response_ref(per_container);
}

std::string encode_allocate_request(const std::vector<std::vector<std::string>>& ids_per_container) {
  std::string o;
  for (const auto& ids : ids_per_container) {
    std::string c;
    for (const auto& id : ids) bytes(&c, 1, id);
    bytes(&o, 1, c);
  }
  return o;
}

std::string encode_preferred_request(const std::vector<PreferredRequest>& reqs) {
  std::string o;
  for (const auto& r : reqs) {
    std::string c;
    for (const auto& id : r.available) bytes(&c, 1, id);
    for (const auto& id : r.must_include) bytes(&c, 2, id);
    int_field(&c, 3, r.size);
    bytes(&o, 1, c);
  }
  return o;
}

bool decode_allocate_request(const std::string& msg, std::vector<std::vector<std::string>>* out) {
  return each(msg, [&](int f, int w, std::string_view pl, uint64_t) {
    if (f != 1 || w != 2) return true;
    std::vector<std::string> ids;
    bool ok = each(pl, [&](int f2, int w2, std::string_view pl2, uint64_t) {
      if (f2 == 1 && w2 == 2) ids.emplace_back(pl2);
      return true;
    });
    out->push_back(std::move(ids));
    return ok;
  });
}

bool decode_preferred_request(std::string_view msg, std::vector<PreferredRequestView>* out) {
  return each(msg, [&](int f, int w, std::string_view pl, uint64_t) {
    if (f != 1 || w != 2) return true;
    PreferredRequestView r;
    r.available.reserve(pl.size() / 16);  // kubelet lists every free ID of the node (~2,300 on 8 GPUs, ~24 B each)
    bool ok = each(pl, [&](int f2, int w2, std::string_view pl2, uint64_t v) {
      if (f2 == 1 && w2 == 2) r.available.push_back(pl2);
      if (f2 == 2 && w2 == 2) r.must_include.push_back(pl2);
      if (f2 == 3 && w2 == 0) r.size = static_cast<int32_t>(v);
      return true;
    });
    out->push_back(std::move(r));
    return ok;
  });
}

bool preferred_single(std::string_view msg, int32_t* size, std::string_view* container) {
  int n = 0;
  bool ok = each(msg, [&](int f, int w, std::string_view pl, uint64_t) {
    if (f == 1 && w == 2) {
      ++n;
      *container = pl;
    }
    return true;
  });
  if (!ok || n != 1) return false;
  bool must = false;
  *size = 0;
  ok = each(*container, [&](int f, int w, std::string_view, uint64_t v) {
    if (f == 2 && w == 2) must = true;
    if (f == 3 && w == 0) *size = static_cast<int32_t>(v);
    return true;
  });
  return ok && !must;
}

bool preferred_single_size(std::string_view msg, int32_t* size, std::string_view* container) {
  int n = 0;
  if (!each(msg, [&](int f, int w, std::string_view pl, uint64_t) {
        if (f == 1 && w == 2) {
          ++n;
          *container = pl;
        }
        return true;
      }) ||
      n != 1) {
    return false;
  }
  // the tail: tag 0x18 (field 3, varint), then the varint (continuation bytes >= 0x80, the last < 0x80).  An ID
  // byte is printable ASCII, so the tag byte cannot be part of one; the walk confirms it anyway
  const auto* b = reinterpret_cast<const uint8_t*>(container->data());
  size_t e = container->size();
  if (e < 2 || (b[e - 1] & 0x80)) return false;
  size_t i = e - 1;
  while (i > 0 && (b[i - 1] & 0x80) && e - i < 5) --i;
  if (i == 0 || b[i - 1] != 0x18) return false;
  uint64_t v = 0;
  for (size_t k = e; k-- > i;) v = (v << 7) | (b[k] & 0x7f);
  if (v == 0 || v > (1u << 30)) return false;
  *size = static_cast<int32_t>(v);
  return true;
}

bool pick_available(std::string_view container, int32_t size, std::string_view prefix,
                    std::vector<std::string_view>* mine, std::vector<std::string_view>* other) {
  const size_t cap = static_cast<size_t>(size), pn = prefix.size();
  const char* pre = prefix.data();
  Reader r(container);
  bool sized = false;
  while (!r.done()) {
    // the common entry, an available ID (tag 0x0a, a one-byte length), without the generic decoder
    if (*r.p == 0x0a && r.end - r.p >= 2 && r.p[1] < 0x80) {
      const size_t n = r.p[1];
      r.p += 2;
      if (static_cast<size_t>(r.end - r.p) < n) return false;
      const char* id = reinterpret_cast<const char*>(r.p);
      r.p += n;
      if (n > pn && pn && std::memcmp(id, pre, pn) == 0) {
        if (mine->size() < cap) mine->emplace_back(id, n);
      } else if (other->size() < cap) {
        other->emplace_back(id, n);
      }
      continue;
    }
    int f, w;
    std::string_view pl;
    uint64_t v = 0;
    if (!r.next(&f, &w, &pl, &v)) return false;
    if (f == 1 && w == 2) {  // a long ID (length >= 128)
      if (pl.size() > pn && pn && pl.compare(0, pn, prefix) == 0) {
        if (mine->size() < cap) mine->push_back(pl);
      } else if (other->size() < cap) {
        other->push_back(pl);
      }
    } else if (f == 2 && w == 2) {
      return false;  // must_include: the general path
    } else if (f == 3 && w == 0) {
      sized = static_cast<int64_t>(v) == size;
    }
  }
  return sized;
}

bool for_each_available(std::string_view container, const std::function<bool(std::string_view)>& fn) {
  bool stopped = false;
  const bool ok = each(container, [&](int f, int w, std::string_view pl, uint64_t) {
    if (f == 1 && w == 2 && !fn(pl)) {
      stopped = true;
      return false;  // the rest of the list is not read
    }
    return true;
  });
  return ok || stopped;
}

bool decode_list_and_watch(const std::string& msg, std::vector<DeviceMsg>* out) {
  return each(msg, [&](int f, int w, std::string_view pl, uint64_t) {
    if (f != 1 || w != 2) return true;
    DeviceMsg d;
    bool ok = each(pl, [&](int f2, int w2, std::string_view pl2, uint64_t) {
      if (f2 == 1 && w2 == 2) d.id = pl2;
      if (f2 == 2 && w2 == 2) d.health = pl2;
      return true;
    });
    out->push_back(std::move(d));
    return ok;
  });
}

bool decode_options(const std::string& msg, bool* pre_start_required, bool* preferred_available) {
  *pre_start_required = *preferred_available = false;
  return each(msg, [&](int f, int w, std::string_view, uint64_t v) {
    if (w == 0 && f == 1) *pre_start_required = v != 0;
    if (w == 0 && f == 2) *preferred_available = v != 0;
    return true;
  });
}

bool decode_preferred_response(const std::string& msg, std::vector<std::vector<std::string>>* out) {
  return decode_allocate_request(msg, out);  // same shape: repeated {1: repeated string}
}

bool decode_allocate_response(const std::string& msg, std::vector<ContainerResponse>* out) {
  return each(msg, [&](int f, int w, std::string_view pl, uint64_t) {
    if (f != 1 || w != 2) return true;
    ContainerResponse r;
    bool ok = each(pl, [&](int f2, int w2, std::string_view pl2, uint64_t) {
      if (w2 != 2) return true;
      std::string k, v;
      if (f2 == 1 && decode_map_entry(pl2, &k, &v)) r.envs[k] = v;
      if (f2 == 4 && decode_map_entry(pl2, &k, &v)) r.annotations[k] = v;
      if (f2 == 2) {
        MountMsg m;
        each(pl2, [&](int f3, int w3, std::string_view pl3, uint64_t v3) {
          if (f3 == 1 && w3 == 2) m.container_path = pl3;
          if (f3 == 2 && w3 == 2) m.host_path = pl3;
          if (f3 == 3 && w3 == 0) m.read_only = v3 != 0;
          return true;
        });
        r.mounts.push_back(std::move(m));
      }
      if (f2 == 3) {
        DeviceSpecMsg d;
        each(pl2, [&](int f3, int w3, std::string_view pl3, uint64_t) {
          if (f3 == 1 && w3 == 2) d.container_path = pl3;
          if (f3 == 2 && w3 == 2) d.host_path = pl3;
          if (f3 == 3 && w3 == 2) d.permissions = pl3;
          return true;
        });
        r.devices.push_back(std::move(d));
      }
      return true;
    });
    out->push_back(std::move(r));
    return ok;
  });
}

std::string encode_pod_resources_list(const std::vector<PodDevicesMsg>& entries) {
  // PodResources{1 name, 2 namespace, 3 repeated ContainerResources{1 name, 2 repeated ContainerDevices{
  // 1 resource_name, 2 repeated device_ids}}}; ListPodResourcesResponse{1 repeated PodResources}
  std::vector<std::pair<std::pair<std::string, std::string>, std::string>> pods;  // (ns, name) -> containers
  for (const auto& e : entries) {
    std::string dev;
    str_if(&dev, 1, e.resource);
    for (const auto& id : e.ids) bytes(&dev, 2, id);
    std::string c;
    str_if(&c, 1, e.container);
    bytes(&c, 2, dev);
    auto it = std::find_if(pods.begin(), pods.end(), [&](const auto& p) {
      return p.first.first == e.ns && p.first.second == e.name;
    });
    if (it == pods.end()) {
      pods.push_back({{e.ns, e.name}, std::string()});
      it = pods.end() - 1;
    }
    bytes(&it->second, 3, c);
  }
  std::string out;
  for (const auto& p : pods) {
    std::string pr;
    str_if(&pr, 1, p.first.second);
    str_if(&pr, 2, p.first.first);
    pr += p.second;
    bytes(&out, 1, pr);
  }
  return out;
}

bool decode_pod_resources_list(const std::string& msg, std::vector<PodDevicesMsg>* entries) {
  return each(msg, [&](int f, int w, std::string_view pr, uint64_t) {
    if (f != 1 || w != 2) return true;
    std::string ns, name;
    std::vector<std::string_view> containers;
    bool ok = each(pr, [&](int f2, int w2, std::string_view pl, uint64_t) {
      if (w2 != 2) return true;
      if (f2 == 1) name = pl;
      if (f2 == 2) ns = pl;
      if (f2 == 3) containers.push_back(pl);
      return true;
    });
    if (!ok) return false;
    for (auto c : containers) {
      std::string cname;
      std::vector<std::string_view> devs;
      if (!each(c, [&](int f3, int w3, std::string_view pl, uint64_t) {
            if (w3 == 2 && f3 == 1) cname = pl;
            if (w3 == 2 && f3 == 2) devs.push_back(pl);
            return true;
          })) {
        return false;
      }
      for (auto d : devs) {
        PodDevicesMsg m;
        m.ns = ns;
        m.name = name;
        m.container = cname;
        if (!each(d, [&](int f4, int w4, std::string_view pl, uint64_t) {
              if (w4 == 2 && f4 == 1) m.resource = pl;
              if (w4 == 2 && f4 == 2) m.ids.emplace_back(pl);
              return true;
            })) {
          return false;
        }
        entries->push_back(std::move(m));
      }
    }
    return true;
  });
}

}  // namespace gsx::dp
