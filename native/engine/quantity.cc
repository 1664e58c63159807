#include "quantity.h"

#include <climits>

namespace gsx {

namespace {
using i128 = __int128;
constexpr i128 kCap = (static_cast<i128>(1) << 100);  // saturation guard, far above INT64_MAX

inline i128 sat_mul(i128 a, i128 b) {
  if (a == 0 || b == 0) return 0;
  if (a > kCap / b) return kCap;
  i128 r = a * b;
  return r > kCap ? kCap : r;
}
}  // namespace

bool parse_quantity(std::string_view s, int64_t* out) {
  size_t i = 0, n = s.size();
  if (n == 0) return false;
  bool neg = false;
  if (s[i] == '+' || s[i] == '-') {
    neg = s[i] == '-';
    ++i;
  }
  i128 mant = 0;
  int exp10 = 0;
  int digits = 0;
  bool any = false;
  while (i < n && s[i] >= '0' && s[i] <= '9') {
    any = true;
    if (mant < kCap) {
      mant = mant * 10 + (s[i] - '0');
    } else {
      ++exp10;  // drop insignificant digits, keep magnitude
    }
    ++digits;
    ++i;
  }
  if (i < n && s[i] == '.') {
    ++i;
    while (i < n && s[i] >= '0' && s[i] <= '9') {
      any = true;
      if (mant < kCap / 10) {
        mant = mant * 10 + (s[i] - '0');
        --exp10;
      }
      ++i;
    }
  }
  if (!any) return false;
  (void)digits;
  int exp2 = 0;
  std::string_view suf = s.substr(i);
  if (suf.empty()) {
  } else if (suf == "Ki") {
    exp2 = 10;
  } else if (suf == "Mi") {
    exp2 = 20;
  } else if (suf == "Gi") {
    exp2 = 30;
  } else if (suf == "Ti") {
    exp2 = 40;
  } else if (suf == "Pi") {
    exp2 = 50;
  } else if (suf == "Ei") {
    exp2 = 60;
  } else if (suf == "n") {
    exp10 -= 9;
  } else if (suf == "u") {
    exp10 -= 6;
  } else if (suf == "m") {
    exp10 -= 3;
  } else if (suf == "k") {
    exp10 += 3;
  } else if (suf == "M") {
    exp10 += 6;
  } else if (suf == "G") {
    exp10 += 9;
  } else if (suf == "T") {
    exp10 += 12;
  } else if (suf == "P") {
    exp10 += 15;
  } else if (suf == "E") {
    exp10 += 18;
  } else if (suf[0] == 'e' || suf[0] == 'E') {
    size_t j = 1;
    bool eneg = false;
    if (j < suf.size() && (suf[j] == '+' || suf[j] == '-')) {
      eneg = suf[j] == '-';
      ++j;
    }
    if (j >= suf.size()) return false;
    int e = 0;
    for (; j < suf.size(); ++j) {
      if (suf[j] < '0' || suf[j] > '9') return false;
      if (e < 10000) e = e * 10 + (suf[j] - '0');
    }
    exp10 += eneg ? -e : e;
  } else {
    return false;
  }

  i128 v = mant;
  for (int k = 0; k < exp2; ++k) v = sat_mul(v, 2);
  if (exp10 >= 0) {
    for (int k = 0; k < exp10 && v < kCap; ++k) v = sat_mul(v, 10);
    if (neg) v = -v;
  } else {
    i128 div = 1;
    bool tiny = false;
    for (int k = 0; k < -exp10; ++k) {
      if (div > kCap / 10) {
        tiny = true;
        break;
      }
      div *= 10;
    }
    if (tiny) {
      // |value| < 1: ceil is 1 for positive non-zero, 0 for negative/zero
      v = (mant == 0) ? 0 : (neg ? 0 : 1);
    } else {
      i128 q = v / div, r = v % div;
      if (neg) {
        v = -q;  // ceil toward +inf for negatives truncates
      } else {
        v = q + (r != 0 ? 1 : 0);
      }
    }
  }
  if (v > static_cast<i128>(INT64_MAX)) v = INT64_MAX;
  if (v < static_cast<i128>(INT64_MIN)) v = INT64_MIN;
  *out = static_cast<int64_t>(v);
  return true;
}

bool parse_atoi(std::string_view s, int64_t* out) {
  if (s.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') {
    neg = s[0] == '-';
    i = 1;
    if (s.size() == 1) return false;
  }
  i128 acc = 0;
  for (; i < s.size(); ++i) {
    char c = s[i];
    if (c < '0' || c > '9') return false;
    acc = acc * 10 + (c - '0');
    if (acc > static_cast<i128>(INT64_MAX) + 1) return false;
  }
  if (neg) acc = -acc;
  if (acc > INT64_MAX || acc < INT64_MIN) return false;
  *out = static_cast<int64_t>(acc);
  return true;
}

}  // namespace gsx
