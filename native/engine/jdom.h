// Mutable JSON values for the native fake kube-apiserver (object store,
// merge patches, server-owned metadata).  The extender's hot paths never
// build a DOM (they read the json.h tape); only the apiserver stand-in, which
// has to edit objects, uses this.  Objects keep member insertion order.
#pragma once

#include <cstdint>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

#include "json.h"

namespace gsx {
namespace jd {

struct Value {
  enum Kind : uint8_t { Null, Bool, Num, Str, Arr, Obj };
  Kind k = Null;
  bool b = false;
  std::string s;  // Num: literal text; Str: decoded value
  std::vector<Value> a;
  std::vector<std::pair<std::string, Value>> o;

  static Value string(std::string v) {
    Value x;
    x.k = Str;
    x.s = std::move(v);
    return x;
  }
  static Value number(int64_t v) {
    Value x;
    x.k = Num;
    x.s = std::to_string(v);
    return x;
  }
  static Value boolean(bool v) {
    Value x;
    x.k = Bool;
    x.b = v;
    return x;
  }
  static Value object() {
    Value x;
    x.k = Obj;
    return x;
  }
  static Value array() {
    Value x;
    x.k = Arr;
    return x;
  }

  bool is_obj() const { return k == Obj; }
  bool is_str() const { return k == Str; }
  bool is_null() const { return k == Null; }
  const Value* get(std::string_view key) const;
  Value* get(std::string_view key);
  // Member `key` (created as an empty object when missing or not an object
  // when `force_obj`).  Converts *this to an object if needed.
  Value& member(std::string_view key, bool force_obj = true);
  void set(std::string_view key, Value v);
  bool erase(std::string_view key);
  // Dotted path lookup ("spec.nodeName"); nullptr if absent.
  const Value* at_path(std::string_view dotted) const;
  // String form used by field selectors: strings as is, null/absent "",
  // numbers / bools as their literal.
  std::string scalar_text() const;
  std::string str_or(std::string_view key, std::string dflt = std::string()) const;
};

bool from_doc(const json::Doc& d, uint32_t i, Value* out);
bool parse(std::string_view s, Value* out, std::string* err);
void write(const Value& v, std::string* out);
std::string dump(const Value& v);
// RFC 7386 JSON merge patch.
void merge_patch(Value* target, const Value& patch);

}  // namespace jd
}  // namespace gsx
