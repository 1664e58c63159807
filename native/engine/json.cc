#include "json.h"

#include <cstdio>
#include <cstdlib>

namespace gsx {
namespace json {

namespace {
constexpr uint32_t kMaxDepth = 512;

inline bool ieq(std::string_view a, std::string_view b) {
  if (a.size() != b.size()) return false;
  for (size_t i = 0; i < a.size(); ++i) {
    char x = a[i], y = b[i];
    if (x >= 'A' && x <= 'Z') x = char(x - 'A' + 'a');
    if (y >= 'A' && y <= 'Z') y = char(y - 'A' + 'a');
    if (x != y) return false;
  }
  return true;
}

inline int hexval(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

inline void put_utf8(std::string* out, uint32_t cp) {
  if (cp < 0x80) {
    out->push_back(char(cp));
  } else if (cp < 0x800) {
    out->push_back(char(0xC0 | (cp >> 6)));
    out->push_back(char(0x80 | (cp & 0x3F)));
  } else if (cp < 0x10000) {
    out->push_back(char(0xE0 | (cp >> 12)));
    out->push_back(char(0x80 | ((cp >> 6) & 0x3F)));
    out->push_back(char(0x80 | (cp & 0x3F)));
  } else {
    out->push_back(char(0xF0 | (cp >> 18)));
    out->push_back(char(0x80 | ((cp >> 12) & 0x3F)));
    out->push_back(char(0x80 | ((cp >> 6) & 0x3F)));
    out->push_back(char(0x80 | (cp & 0x3F)));
  }
}
}  // namespace

void Doc::fail(const char* what) {
  if (failed_) return;
  failed_ = true;
  if (err_) *err_ = what;
}

void Doc::fail_char(const char* ctx) {
  if (failed_) return;
  if (pos_ >= n_) {
    fail("unexpected end of JSON input");
    return;
  }
  char buf[160];
  unsigned char c = static_cast<unsigned char>(s_[pos_]);
  if (c >= 0x20 && c < 0x7f && c != '\'') {
    std::snprintf(buf, sizeof(buf), "invalid character '%c' %s", c, ctx);
  } else {
    std::snprintf(buf, sizeof(buf), "invalid character '\\x%02x' %s", c, ctx);
  }
  fail(buf);
}

bool Doc::parse(std::string_view src, std::string* err) {
  src_ = src;
  s_ = src.data();
  n_ = static_cast<uint32_t>(src.size());
  pos_ = 0;
  tape_.clear();
  tape_.reserve(64 + src.size() / 12);
  err_ = err;
  failed_ = false;
  skip_ws();
  if (pos_ >= n_) {
    fail("unexpected end of JSON input");
    return false;
  }
  if (!parse_value(0)) return false;
  skip_ws();
  if (pos_ != n_) {
    fail_char("after top-level value");
    return false;
  }
  return true;
}

bool Doc::parse_string(uint32_t* idx) {
  // s_[pos_] == '"'
  uint32_t start = ++pos_;
  bool esc = false;
  while (true) {
    // fast scan
    while (pos_ < n_) {
      unsigned char c = static_cast<unsigned char>(s_[pos_]);
      if (c == '"' || c == '\\' || c < 0x20) break;
      ++pos_;
    }
    if (pos_ >= n_) {
      fail("unexpected end of JSON input");
      return false;
    }
    char c = s_[pos_];
    if (c == '"') break;
    if (c == '\\') {
      esc = true;
      if (pos_ + 1 >= n_) {
        fail("unexpected end of JSON input");
        return false;
      }
      char e = s_[pos_ + 1];
      if (e == 'u') {
        if (pos_ + 6 > n_) {
          fail("unexpected end of JSON input");
          return false;
        }
        for (int k = 2; k < 6; ++k) {
          if (hexval(s_[pos_ + k]) < 0) {
            pos_ += k;
            fail_char("in \\u hexadecimal character escape");
            return false;
          }
        }
        pos_ += 6;
      } else if (e == '"' || e == '\\' || e == '/' || e == 'b' || e == 'f' || e == 'n' || e == 'r' ||
                 e == 't') {
        pos_ += 2;
      } else {
        ++pos_;
        fail_char("in string escape code");
        return false;
      }
      continue;
    }
    fail_char("in string literal");
    return false;
  }
  Val v{T::String, esc, start, pos_, 0, 0};
  *idx = static_cast<uint32_t>(tape_.size());
  tape_.push_back(v);
  tape_.back().skip = *idx + 1;
  ++pos_;  // closing quote
  return true;
}

bool Doc::parse_value(uint32_t depth) {
  if (depth > kMaxDepth) {
    fail("exceeded max depth");
    return false;
  }
  if (pos_ >= n_) {
    fail("unexpected end of JSON input");
    return false;
  }
  char c = s_[pos_];
  switch (c) {
    case '{': {
      uint32_t idx = static_cast<uint32_t>(tape_.size());
      tape_.push_back(Val{T::Object, false, pos_, 0, 0, 0});
      ++pos_;
      skip_ws();
      uint32_t count = 0;
      if (pos_ < n_ && s_[pos_] == '}') {
        ++pos_;
      } else {
        while (true) {
          skip_ws();
          if (pos_ >= n_) {
            fail("unexpected end of JSON input");
            return false;
          }
          if (s_[pos_] != '"') {
            fail_char("looking for beginning of object key string");
            return false;
          }
          uint32_t kidx;
          if (!parse_string(&kidx)) return false;
          skip_ws();
          if (pos_ >= n_) {
            fail("unexpected end of JSON input");
            return false;
          }
          if (s_[pos_] != ':') {
            fail_char("after object key");
            return false;
          }
          ++pos_;
          skip_ws();
          if (!parse_value(depth + 1)) return false;
          ++count;
          skip_ws();
          if (pos_ >= n_) {
            fail("unexpected end of JSON input");
            return false;
          }
          if (s_[pos_] == ',') {
            ++pos_;
            continue;
          }
          if (s_[pos_] == '}') {
            ++pos_;
            break;
          }
          fail_char("after object key:value pair");
          return false;
        }
      }
      tape_[idx].end = pos_;
      tape_[idx].count = count;
      tape_[idx].skip = static_cast<uint32_t>(tape_.size());
      return true;
    }
    case '[': {
      uint32_t idx = static_cast<uint32_t>(tape_.size());
      tape_.push_back(Val{T::Array, false, pos_, 0, 0, 0});
      ++pos_;
      skip_ws();
      uint32_t count = 0;
      if (pos_ < n_ && s_[pos_] == ']') {
        ++pos_;
      } else {
        while (true) {
          skip_ws();
          if (!parse_value(depth + 1)) return false;
          ++count;
          skip_ws();
          if (pos_ >= n_) {
            fail("unexpected end of JSON input");
            return false;
          }
          if (s_[pos_] == ',') {
            ++pos_;
            continue;
          }
          if (s_[pos_] == ']') {
            ++pos_;
            break;
          }
          fail_char("after array element");
          return false;
        }
      }
      tape_[idx].end = pos_;
      tape_[idx].count = count;
      tape_[idx].skip = static_cast<uint32_t>(tape_.size());
      return true;
    }
    case '"': {
      uint32_t idx;
      return parse_string(&idx);
    }
    case 't':
    case 'f':
    case 'n': {
      const char* lit = c == 't' ? "true" : (c == 'f' ? "false" : "null");
      size_t len = std::strlen(lit);
      for (size_t k = 0; k < len; ++k) {
        if (pos_ + k >= n_) {
          pos_ = n_;
          fail("unexpected end of JSON input");
          return false;
        }
        if (s_[pos_ + k] != lit[k]) {
          pos_ += static_cast<uint32_t>(k);
          fail_char(c == 't' ? "in literal true (expecting 'r')" : (c == 'f' ? "in literal false" : "in literal null"));
          return false;
        }
      }
      T t = c == 't' ? T::True : (c == 'f' ? T::False : T::Null);
      uint32_t idx = static_cast<uint32_t>(tape_.size());
      tape_.push_back(Val{t, false, pos_, pos_ + static_cast<uint32_t>(len), idx + 1, 0});
      pos_ += static_cast<uint32_t>(len);
      return true;
    }
    default: {
      if (c == '-' || (c >= '0' && c <= '9')) {
        uint32_t start = pos_;
        if (s_[pos_] == '-') ++pos_;
        if (pos_ >= n_) {
          fail("unexpected end of JSON input");
          return false;
        }
        if (s_[pos_] == '0') {
          ++pos_;
        } else if (s_[pos_] >= '1' && s_[pos_] <= '9') {
          while (pos_ < n_ && s_[pos_] >= '0' && s_[pos_] <= '9') ++pos_;
        } else {
          fail_char("in numeric literal");
          return false;
        }
        if (pos_ < n_ && s_[pos_] == '.') {
          ++pos_;
          if (pos_ >= n_ || !(s_[pos_] >= '0' && s_[pos_] <= '9')) {
            fail_char("after decimal point in numeric literal");
            return false;
          }
          while (pos_ < n_ && s_[pos_] >= '0' && s_[pos_] <= '9') ++pos_;
        }
        if (pos_ < n_ && (s_[pos_] == 'e' || s_[pos_] == 'E')) {
          ++pos_;
          if (pos_ < n_ && (s_[pos_] == '+' || s_[pos_] == '-')) ++pos_;
          if (pos_ >= n_ || !(s_[pos_] >= '0' && s_[pos_] <= '9')) {
            fail_char("in exponent of numeric literal");
            return false;
          }
          while (pos_ < n_ && s_[pos_] >= '0' && s_[pos_] <= '9') ++pos_;
        }
        uint32_t idx = static_cast<uint32_t>(tape_.size());
        tape_.push_back(Val{T::Number, false, start, pos_, idx + 1, 0});
        return true;
      }
      fail_char("looking for beginning of value");
      return false;
    }
  }
}

int64_t Doc::find(uint32_t obj, std::string_view key, bool ci) const {
  if (obj >= tape_.size() || tape_[obj].type != T::Object) return -1;
  int64_t ci_hit = -1;
  int64_t exact = -1;
  uint32_t i = obj + 1;
  const uint32_t stop = tape_[obj].skip;
  std::string tmp;
  while (i < stop) {
    const Val& k = tape_[i];
    uint32_t vi = i + 1;
    std::string_view kv(s_ + k.begin, k.end - k.begin);
    if (k.escaped) {
      tmp.clear();
      unescape(kv, &tmp);
      kv = tmp;
    }
    if (kv == key) {
      exact = vi;
    } else if (ci && ieq(kv, key)) {
      ci_hit = vi;
    }
    i = tape_[vi].skip;
  }
  return exact >= 0 ? exact : ci_hit;
}

int64_t Doc::path(uint32_t obj, std::initializer_list<std::string_view> keys) const {
  int64_t cur = obj;
  for (auto k : keys) {
    if (cur < 0) return -1;
    cur = find(static_cast<uint32_t>(cur), k, false);
  }
  return cur;
}

std::string_view Doc::raw(uint32_t i) const {
  const Val& v = tape_[i];
  if (v.type == T::String) return std::string_view(s_ + v.begin - 1, v.end - v.begin + 2);
  return std::string_view(s_ + v.begin, v.end - v.begin);
}

bool Doc::str_view(uint32_t i, std::string_view* out) const {
  const Val& v = tape_[i];
  if (v.type != T::String || v.escaped) return false;
  *out = std::string_view(s_ + v.begin, v.end - v.begin);
  return true;
}

std::string Doc::str(uint32_t i) const {
  const Val& v = tape_[i];
  if (v.type != T::String) return std::string();
  std::string_view sv(s_ + v.begin, v.end - v.begin);
  if (!v.escaped) return std::string(sv);
  std::string out;
  unescape(sv, &out);
  return out;
}

bool Doc::as_int(uint32_t i, int64_t* out) const {
  const Val& v = tape_[i];
  if (v.type != T::Number) return false;
  int64_t acc = 0;
  uint32_t p = v.begin;
  bool neg = false;
  if (s_[p] == '-') {
    neg = true;
    ++p;
  }
  for (; p < v.end; ++p) {
    char c = s_[p];
    if (c < '0' || c > '9') return false;
    if (acc > (INT64_MAX - (c - '0')) / 10) return false;
    acc = acc * 10 + (c - '0');
  }
  *out = neg ? -acc : acc;
  return true;
}

bool unescape(std::string_view s, std::string* out) {
  out->reserve(out->size() + s.size());
  for (size_t i = 0; i < s.size(); ++i) {
    char c = s[i];
    if (c != '\\') {
      out->push_back(c);
      continue;
    }
    if (i + 1 >= s.size()) return false;
    char e = s[++i];
    switch (e) {
      case '"': out->push_back('"'); break;
      case '\\': out->push_back('\\'); break;
      case '/': out->push_back('/'); break;
      case 'b': out->push_back('\b'); break;
      case 'f': out->push_back('\f'); break;
      case 'n': out->push_back('\n'); break;
      case 'r': out->push_back('\r'); break;
      case 't': out->push_back('\t'); break;
      case 'u': {
        // i points at 'u'; hex digits at i+1..i+4
        if (i + 4 >= s.size()) return false;
        uint32_t cp = 0;
        for (int k = 1; k <= 4; ++k) {
          int h = hexval(s[i + k]);
          if (h < 0) return false;
          cp = cp * 16 + static_cast<uint32_t>(h);
        }
        i += 4;  // i at last hex digit
        if (cp >= 0xD800 && cp < 0xDC00 && i + 6 < s.size() && s[i + 1] == '\\' && s[i + 2] == 'u') {
          uint32_t lo = 0;
          bool ok = true;
          for (int k = 3; ok && k <= 6; ++k) {
            int h = hexval(s[i + k]);
            if (h < 0) ok = false;
            lo = lo * 16 + static_cast<uint32_t>(h < 0 ? 0 : h);
          }
          if (ok && lo >= 0xDC00 && lo < 0xE000) {
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            i += 6;
          } else {
            cp = 0xFFFD;
          }
        } else if (cp >= 0xD800 && cp < 0xE000) {
          cp = 0xFFFD;
        }
        put_utf8(out, cp);
        break;
      }
      default:
        return false;
    }
  }
  return true;
}

namespace {
// 1 for bytes Go's encoding/json (HTML-safe) copies verbatim.
struct SafeTable {
  bool t[256];
  SafeTable() {
    for (int c = 0; c < 256; ++c) t[c] = c >= 0x20 && c < 0x80 && c != '"' && c != '\\' && c != '<' && c != '>' && c != '&';
  }
};
const SafeTable kSafe;
}  // namespace

void append_quoted(std::string* out, std::string_view s) {
  static const char* hex = "0123456789abcdef";
  out->push_back('"');
  size_t i = 0;
  const size_t n = s.size();
  while (i < n) {
    // bulk-copy the run of bytes that need no escaping
    size_t j = i;
    while (j < n && kSafe.t[static_cast<unsigned char>(s[j])]) ++j;
    if (j > i) {
      out->append(s.data() + i, j - i);
      i = j;
      if (i == n) break;
    }
    unsigned char c = static_cast<unsigned char>(s[i]);
    if (c < 0x80) {
      switch (c) {
        case '"': out->append("\\\""); break;
        case '\\': out->append("\\\\"); break;
        case '\n': out->append("\\n"); break;
        case '\r': out->append("\\r"); break;
        case '\t': out->append("\\t"); break;
        default:
          out->append("\\u00");
          out->push_back(hex[c >> 4]);
          out->push_back(hex[c & 0xF]);
      }
      ++i;
      continue;
    }
    // U+2028 / U+2029 are E2 80 A8 / E2 80 A9
    if (c == 0xE2 && i + 2 < n && static_cast<unsigned char>(s[i + 1]) == 0x80 &&
        (static_cast<unsigned char>(s[i + 2]) == 0xA8 || static_cast<unsigned char>(s[i + 2]) == 0xA9)) {
      out->append(static_cast<unsigned char>(s[i + 2]) == 0xA8 ? "\\u2028" : "\\u2029");
      i += 3;
      continue;
    }
    out->push_back(char(c));
    ++i;
  }
  out->push_back('"');
}

}  // namespace json
}  // namespace gsx
