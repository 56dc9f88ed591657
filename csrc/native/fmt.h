// Number formatting that reproduces the text the reference pipeline emits.
//
//  * java_double: java.lang.Double.toString (Scala `x.toString`), used for flow
//    words ("80.0_3.0_5.0_2.0", flow_pre_lda.scala:349), the time column and
//    the scores of flow_results.csv / dns_results.csv (flow_post_lda.scala:238,
//    dns_post_lda.scala:320).  Digits are the shortest round-trip digits (the
//    JDK >= 19 algorithm; older JDKs occasionally printed one extra digit).
//  * py2_float: Python 2 str(float) / numpy<1.14 str(float64) = "%.12g" with
//    ".0" appended to integral results; doc_results.csv / word_results.csv
//    (lda_post.py:45,115-122).
//  * fixed10: C printf "%5.10f" (lda-c save_lda_model / save_gamma).
#pragma once
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>

namespace onin {

// Appends Java's Double.toString(d) to out.
inline void append_java_double(std::string& out, double d) {
  if (std::isnan(d)) { out += "NaN"; return; }
  if (std::isinf(d)) { out += d > 0 ? "Infinity" : "-Infinity"; return; }
  if (d == 0.0) { out += std::signbit(d) ? "-0.0" : "0.0"; return; }
  char buf[64];
  auto r = std::to_chars(buf, buf + sizeof(buf), d, std::chars_format::scientific);
  *r.ptr = 0;
  // buf = [-]D[.DDDD]e[+-]XX
  const char* p = buf;
  bool neg = false;
  if (*p == '-') { neg = true; ++p; }
  char digits[32];
  int nd = 0;
  while (*p && *p != 'e') {
    if (*p != '.') digits[nd++] = *p;
    ++p;
  }
  int e = std::atoi(p + 1);  // value = d1.d2d3.. * 10^e
  if (neg) out += '-';
  const double a = std::fabs(d);
  if (a >= 1e-3 && a < 1e7) {
    if (e >= 0) {
      for (int i = 0; i <= e; ++i) out += (i < nd ? digits[i] : '0');
      out += '.';
      if (nd > e + 1) out.append(digits + e + 1, nd - e - 1);
      else out += '0';
    } else {
      out += "0.";
      for (int i = 0; i < -e - 1; ++i) out += '0';
      out.append(digits, nd);
    }
  } else {
    out += digits[0];
    out += '.';
    if (nd > 1) out.append(digits + 1, nd - 1);
    else out += '0';
    out += 'E';
    char eb[8];
    int n = std::snprintf(eb, sizeof(eb), "%d", e);
    out.append(eb, n);
  }
}

inline std::string java_double(double d) {
  std::string s;
  append_java_double(s, d);
  return s;
}

// Python 2 str(float): repr-free "%.12g" plus ".0" on integral-looking output.
// std::to_chars(general, 12) is specified as printf("%.12g") in the C locale and
// is exact (Ryu-printf in libstdc++), ~4x faster than snprintf.
inline void append_py2_float(std::string& out, double d) {
  if (std::isnan(d)) { out += "nan"; return; }
  if (std::isinf(d)) { out += d > 0 ? "inf" : "-inf"; return; }
  char buf[40];
  auto r = std::to_chars(buf, buf + sizeof(buf), d, std::chars_format::general, 12);
  const int n = (int)(r.ptr - buf);
  out.append(buf, n);
  bool has = false;
  for (int i = 0; i < n; ++i)
    if (buf[i] == '.' || buf[i] == 'e') { has = true; break; }
  if (!has) out += ".0";
}

// printf("%5.10f"): finite values always exceed the 5-character field width, so
// to_chars(fixed, 10) (exact, same digits as glibc) is the whole conversion;
// nan / inf keep printf's padded spelling.
inline void append_fixed10(std::string& out, double d) {
  char buf[352];
  if (!std::isfinite(d)) {
    int n = std::snprintf(buf, sizeof(buf), "%5.10f", d);
    out.append(buf, n);
    return;
  }
  auto r = std::to_chars(buf, buf + sizeof(buf), d, std::chars_format::fixed, 10);
  out.append(buf, r.ptr - buf);
}

inline void append_int(std::string& out, long long v) {
  char buf[24];
  auto r = std::to_chars(buf, buf + sizeof(buf), v);
  out.append(buf, r.ptr - buf);
}

// java.lang.Double.parseDouble subset: trims ASCII whitespace/control chars
// (<= ' '), accepts an optional trailing d/D/f/F suffix, decimal and
// "NaN"/"Infinity" literals.  Returns false when the text is not a number
// (the reference would throw NumberFormatException).
inline bool java_parse_double(const char* b, const char* e, double* out) {
  while (b < e && (unsigned char)*b <= ' ') ++b;
  while (e > b && (unsigned char)e[-1] <= ' ') --e;
  if (b == e) return false;
  if (e - b > 1 && (e[-1] == 'd' || e[-1] == 'D' || e[-1] == 'f' || e[-1] == 'F')) {
    char c = e[-2];
    if ((c >= '0' && c <= '9') || c == '.') --e;
  }
  const char* s = b;
  bool neg = false;
  if (*s == '+' || *s == '-') { neg = *s == '-'; ++s; }
  const size_t n = e - s;
  if (n == 3 && std::memcmp(s, "NaN", 3) == 0) { *out = NAN; return true; }
  if (n == 8 && std::memcmp(s, "Infinity", 8) == 0) { *out = neg ? -INFINITY : INFINITY; return true; }
  // from_chars does not accept a leading '+'
  double v;
  auto r = std::from_chars(s, e, v, std::chars_format::general);
  if (r.ec != std::errc() || r.ptr != e) {
    // from_chars rejects "5." / ".5" forms?  It accepts ".5" and "5." per C strtod grammar;
    // anything else is not a Java double literal either.
    return false;
  }
  *out = neg ? -v : v;
  return true;
}

}  // namespace onin
