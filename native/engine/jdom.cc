#include "jdom.h"

namespace gsx {
namespace jd {

const Value* Value::get(std::string_view key) const {
  if (k != Obj) return nullptr;
  for (const auto& m : o) {
    if (m.first == key) return &m.second;
  }
  return nullptr;
}

Value* Value::get(std::string_view key) {
  if (k != Obj) return nullptr;
  for (auto& m : o) {
    if (m.first == key) return &m.second;
  }
  return nullptr;
}

Value& Value::member(std::string_view key, bool force_obj) {
  if (k != Obj) {
    *this = object();
  }
  for (auto& m : o) {
    if (m.first == key) {
      if (force_obj && m.second.k != Obj) m.second = object();
      return m.second;
    }
  }
  o.emplace_back(std::string(key), force_obj ? object() : Value());
  return o.back().second;
}

void Value::set(std::string_view key, Value v) {
  if (k != Obj) *this = object();
  for (auto& m : o) {
    if (m.first == key) {
      m.second = std::move(v);
      return;
    }
  }
  o.emplace_back(std::string(key), std::move(v));
}

bool Value::erase(std::string_view key) {
  if (k != Obj) return false;
  for (auto it = o.begin(); it != o.end(); ++it) {
    if (it->first == key) {
      o.erase(it);
      return true;
    }
  }
  return false;
}

const Value* Value::at_path(std::string_view dotted) const {
  const Value* cur = this;
  size_t i = 0;
  while (cur && i <= dotted.size()) {
    size_t j = dotted.find('.', i);
    if (j == std::string_view::npos) j = dotted.size();
    cur = cur->get(dotted.substr(i, j - i));
    i = j + 1;
    if (j == dotted.size()) break;
  }
  return cur;
}

std::string Value::scalar_text() const {
  switch (k) {
    case Str:
    case Num:
      return s;
    case Bool:
      return b ? "True" : "False";  // Python str(bool), as the asyncio fake apiserver compares
    default:
      return std::string();
  }
}

std::string Value::str_or(std::string_view key, std::string dflt) const {
  const Value* v = get(key);
  return v && v->k == Str ? v->s : dflt;
}

bool from_doc(const json::Doc& d, uint32_t i, Value* out) {
  const json::Val& v = d.at(i);
  switch (v.type) {
    case json::T::Null:
      out->k = Value::Null;
      return true;
    case json::T::False:
    case json::T::True:
      out->k = Value::Bool;
      out->b = v.type == json::T::True;
      return true;
    case json::T::Number:
      out->k = Value::Num;
      out->s.assign(d.raw(i));
      return true;
    case json::T::String:
      out->k = Value::Str;
      out->s = d.str(i);
      return true;
    case json::T::Array: {
      out->k = Value::Arr;
      out->a.reserve(v.count);
      for (uint32_t c = i + 1; c < v.skip; c = d.next(c)) {
        out->a.emplace_back();
        if (!from_doc(d, c, &out->a.back())) return false;
      }
      return true;
    }
    case json::T::Object: {
      out->k = Value::Obj;
      out->o.reserve(v.count);
      for (uint32_t c = i + 1; c < v.skip;) {
        // member = key string record followed by the value subtree
        std::string key = d.str(c);
        uint32_t val = c + 1;
        Value x;
        if (!from_doc(d, val, &x)) return false;
        // duplicate keys: last one wins (Go encoding/json)
        bool dup = false;
        for (auto& m : out->o) {
          if (m.first == key) {
            m.second = std::move(x);
            dup = true;
            break;
          }
        }
        if (!dup) out->o.emplace_back(std::move(key), std::move(x));
        c = d.next(val);
      }
      return true;
    }
  }
  return false;
}

bool parse(std::string_view s, Value* out, std::string* err) {
  json::Doc d;
  if (!d.parse(s, err)) return false;
  *out = Value();
  return from_doc(d, 0, out);
}

void write(const Value& v, std::string* out) {
  switch (v.k) {
    case Value::Null:
      out->append("null");
      return;
    case Value::Bool:
      out->append(v.b ? "true" : "false");
      return;
    case Value::Num:
      out->append(v.s);
      return;
    case Value::Str:
      json::append_quoted(out, v.s);
      return;
    case Value::Arr:
      out->push_back('[');
      for (size_t i = 0; i < v.a.size(); ++i) {
        if (i) out->push_back(',');
        write(v.a[i], out);
      }
      out->push_back(']');
      return;
    case Value::Obj:
      out->push_back('{');
      for (size_t i = 0; i < v.o.size(); ++i) {
        if (i) out->push_back(',');
        json::append_quoted(out, v.o[i].first);
        out->push_back(':');
        write(v.o[i].second, out);
      }
      out->push_back('}');
      return;
  }
}

std::string dump(const Value& v) {
  std::string s;
  s.reserve(512);
  write(v, &s);
  return s;
}

void merge_patch(Value* target, const Value& patch) {
  if (patch.k != Value::Obj) {
    *target = patch;
    return;
  }
  if (target->k != Value::Obj) *target = Value::object();
  for (const auto& m : patch.o) {
    if (m.second.k == Value::Null) {
      target->erase(m.first);
    } else {
      Value* cur = target->get(m.first);
      if (cur) {
        merge_patch(cur, m.second);
      } else {
        Value nv;
        merge_patch(&nv, m.second);
        target->o.emplace_back(m.first, std::move(nv));
      }
    }
  }
}

}  // namespace jd
}  // namespace gsx
