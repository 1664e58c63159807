// Minimal tape JSON parser + Go-compatible writer helpers.
//
// The extender's hot paths (filter request bodies that carry a whole v1.Pod,
// informer watch events) are JSON.  The reference decodes them with Go's
// encoding/json into typed structs (pkg/routes/routes.go:72, :114).  Here a
// single pass builds a flat "tape" of value records (type + byte span +
// subtree skip index) so callers can look up the handful of fields they need
// without materialising a DOM of heap objects, and can slice raw sub-values
// (e.g. NodeList items) straight out of the request buffer.
#pragma once

#include <cstdint>
#include <cstring>
#include <string>
#include <string_view>
#include <vector>

namespace gsx {
namespace json {

enum class T : uint8_t { Null, False, True, Number, String, Array, Object };

struct Val {
  T type;
  bool escaped;    // string contains backslash escapes
  uint32_t begin;  // byte offset of value start (strings: first content byte)
  uint32_t end;    // byte offset one past value end (strings: closing quote)
  uint32_t skip;   // tape index of the first record after this subtree
  uint32_t count;  // arrays: elements; objects: members
};

class Doc {
 public:
  // Parses `src` (which must outlive the Doc).  Returns false and fills err
  // with a Go-style message on malformed input.
  bool parse(std::string_view src, std::string* err);

  std::string_view src() const { return src_; }
  const Val& at(uint32_t i) const { return tape_[i]; }
  size_t size() const { return tape_.size(); }
  bool empty() const { return tape_.empty(); }

  // Object member lookup.  Returns the tape index of the value or -1.
  // ci=true follows Go encoding/json: exact match wins, else ASCII
  // case-insensitive match (last one wins, as with duplicate keys).
  int64_t find(uint32_t obj, std::string_view key, bool ci = false) const;
  // Convenience path lookup through nested objects (exact keys).
  int64_t path(uint32_t obj, std::initializer_list<std::string_view> keys) const;

  // Raw text of the value (strings include their quotes).
  std::string_view raw(uint32_t i) const;
  // Decoded string value (unescaped); empty for non-strings.
  std::string str(uint32_t i) const;
  // String content view when no escapes are present (fast path).
  bool str_view(uint32_t i, std::string_view* out) const;
  // Integer value of a number record; false if not an integral number.
  bool as_int(uint32_t i, int64_t* out) const;

  // Iteration helpers: first child index and next sibling.
  uint32_t first_child(uint32_t i) const { return i + 1; }
  uint32_t next(uint32_t i) const { return tape_[i].skip; }

 private:
  bool parse_value(uint32_t depth);
  bool parse_string(uint32_t* idx);
  void fail(const char* what);
  void fail_char(const char* ctx);
  void skip_ws() {
    while (pos_ < n_) {
      char c = s_[pos_];
      if (c == ' ' || c == '\n' || c == '\t' || c == '\r') {
        ++pos_;
      } else {
        break;
      }
    }
  }

  std::string_view src_;
  const char* s_ = nullptr;
  uint32_t n_ = 0;
  uint32_t pos_ = 0;
  std::vector<Val> tape_;
  std::string* err_ = nullptr;
  bool failed_ = false;
};

// Decode JSON string escapes of s (content between quotes) into out.
bool unescape(std::string_view s, std::string* out);

// Append a JSON string literal using Go encoding/json's escaping rules
// (HTML-safe: <, >, & as < etc; U+2028/2029 escaped).
void append_quoted(std::string* out, std::string_view s);

}  // namespace json
}  // namespace gsx
