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
#include <cstdint>
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

// ---- fast paths from the shortest round-trip digits ---------------------------------------
//
// Let S be the shortest round-trip decimal of x (Ryu: fewest digits, then closest to x) and T a
// rounding midpoint of a P-digit grid.  T cannot lie strictly between x and S: T would then be in
// x's round-trip interval with fewer digits than S (or as many and closer to x), so Ryu would
// have picked it.  Hence rounding S to P digits gives the same result as rounding x, except when
// S itself IS a midpoint (its digit P is the last one and equals 5) -- those values take the
// exact (printf-equivalent) path.  ~4x faster than to_chars(general / fixed, precision).

// |a| finite, nonzero: dig[0..nd) with a = d0.d1d2... x 10^e; no trailing zeros.
inline int shortest_digits(double a, char* dig, int* e10) {
  char buf[40];
  auto r = std::to_chars(buf, buf + sizeof(buf), a, std::chars_format::scientific);
  int nd = 0;
  const char* p = buf;
  for (; p < r.ptr && *p != 'e'; ++p)
    if (*p != '.') dig[nd++] = *p;
  ++p;
  const bool neg = *p == '-';
  if (*p == '+' || *p == '-') ++p;
  int e = 0;
  for (; p < r.ptr; ++p) e = e * 10 + (*p - '0');
  *e10 = neg ? -e : e;
  while (nd > 1 && dig[nd - 1] == '0') --nd;
  return nd;
}

// Round dig to P significant digits (round half up is never needed: see above).  False on a
// midpoint (the caller takes the exact path).
inline bool round_digits(char* dig, int& nd, int& e, int P) {
  if (nd <= P) return true;
  if (P < 1) return false;
  const char c = dig[P];
  if (c == '5' && nd == P + 1) return false;
  nd = P;
  if (c >= '5') {
    int i = P - 1;
    while (i >= 0 && dig[i] == '9') dig[i--] = '0';
    if (i < 0) {
      dig[0] = '1';
      ++e;
    } else {
      ++dig[i];
    }
  }
  while (nd > 1 && dig[nd - 1] == '0') --nd;
  return true;
}

// digits -> double (Clinger's fast path: an integer mantissa < 2^53 times / over an exact power of
// ten is one correctly rounded operation); false outside it
inline bool digits_value(const char* dig, int nd, int e, bool neg, double* out) {
  static const double p10[] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                               1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
  if (nd > 15) return false;
  int64_t m = 0;
  for (int i = 0; i < nd; ++i) m = m * 10 + (dig[i] - '0');
  const int k = e - nd + 1;
  double v;
  if (k >= 0 && k <= 22) v = (double)m * p10[k];
  else if (k < 0 && k >= -22) v = (double)m / p10[-k];
  else return false;
  *out = neg ? -v : v;
  return true;
}

// Python 2 str(float): "%.12g" plus ".0" on integral-looking output.  `back` (optional) receives
// the value a reader parses from the text.
inline void append_py2_float(std::string& out, double d, double* back = nullptr) {
  if (std::isnan(d)) { out += "nan"; if (back) *back = d; return; }
  if (std::isinf(d)) { out += d > 0 ? "inf" : "-inf"; if (back) *back = d; return; }
  char dig[32];
  int e = 0, nd = 0;
  const size_t at = out.size();
  if (std::fabs(d) >= 2.2250738585072014e-308) {      // normal: 53 bits > 12 digits (see above)
    nd = shortest_digits(std::fabs(d), dig, &e);
    if (round_digits(dig, nd, e, 12)) {
      if (d < 0) out += '-';
      if (e < -4 || e >= 12) {
        out += dig[0];
        if (nd > 1) { out += '.'; out.append(dig + 1, nd - 1); }
        out += 'e';
        out += e < 0 ? '-' : '+';
        const int ae = e < 0 ? -e : e;
        if (ae < 10) out += '0';
        char eb[8];
        auto r = std::to_chars(eb, eb + sizeof(eb), ae);
        out.append(eb, r.ptr - eb);
      } else if (e >= 0) {
        for (int i = 0; i <= e; ++i) out += i < nd ? dig[i] : '0';
        if (nd > e + 1) { out += '.'; out.append(dig + e + 1, nd - e - 1); }
        else out += ".0";
      } else {
        out += "0.";
        out.append((size_t)(-e - 1), '0');
        out.append(dig, nd);
      }
      if (back && !digits_value(dig, nd, e, d < 0, back))
        std::from_chars(out.data() + at, out.data() + out.size(), *back);
      return;
    }
  }
  char buf[40];
  auto r = std::to_chars(buf, buf + sizeof(buf), d, std::chars_format::general, 12);
  const int n = (int)(r.ptr - buf);
  out.append(buf, n);
  bool has = false;
  for (int i = 0; i < n; ++i)
    if (buf[i] == '.' || buf[i] == 'e') { has = true; break; }
  if (!has) out += ".0";
  if (back) std::from_chars(out.data() + at, out.data() + out.size(), *back);
}

// printf("%5.10f"): finite values always exceed the 5-character field width, so the
// conversion is the exact 10-decimal rounding (fast path for 1e-9 <= |d| < 1e5, where half an
// ulp of d is far below the 1e-10 grid); nan / inf keep printf's padded spelling.
inline void append_fixed10(std::string& out, double d, double* back = nullptr) {
  const size_t at = out.size();
  const double a = std::fabs(d);
  if (a >= 1e-9 && a < 1e5) {
    char dig[32];
    int e = 0;
    int nd = shortest_digits(a, dig, &e);
    if (round_digits(dig, nd, e, e + 11)) {
      if (d < 0) out += '-';
      if (e >= 0) {
        for (int i = 0; i <= e; ++i) out += i < nd ? dig[i] : '0';
      } else {
        out += '0';
      }
      out += '.';
      for (int i = e + 1; i <= e + 10; ++i) out += (i >= 0 && i < nd) ? dig[i] : '0';
      if (back && !digits_value(dig, nd, e, d < 0, back))
        std::from_chars(out.data() + at, out.data() + out.size(), *back);
      return;
    }
  }
  char buf[352];
  if (!std::isfinite(d)) {
    int n = std::snprintf(buf, sizeof(buf), "%5.10f", d);
    out.append(buf, n);
  } else {
    auto r = std::to_chars(buf, buf + sizeof(buf), d, std::chars_format::fixed, 10);
    out.append(buf, r.ptr - buf);
  }
  if (back) std::from_chars(out.data() + at, out.data() + out.size(), *back);
}

// The exact (printf-equivalent) conversions, for tests of the fast paths above.
inline void append_py2_float_exact(std::string& out, double d) {
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

inline void append_fixed10_exact(std::string& out, double d) {
  char buf[352];
  int n = std::snprintf(buf, sizeof(buf), "%5.10f", d);
  out.append(buf, n);
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
