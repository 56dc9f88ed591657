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

// ---- exact fast paths without a decimal conversion library ---------------------------------
//
// "%.10f" and "%.12g" both print N = round-half-even(|x| * 10^k) for one k (10, or 11 - the
// decimal exponent).  With 10^k exact (0 <= k <= 22) that rounding is decided exactly from the
// error-free product x * 10^k = p + err.  No Ryu / printf on this path (2-5x cheaper); values
// outside it (|x| >= 1e11 for %.12g, >= 9e5 for %.10f, tiny or non-finite) take the exact
// library conversion.

inline const double* pow10_table() {
  static const double p10[] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                               1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
  return p10;
}

// 12 decimal digits of 0 <= n < 10^12, two at a time
inline void put_digits12(char* dig, int64_t n);

// the exact product a * b = p + e: one fused multiply-add (x86-64-v3 hosts), else Dekker's split
inline void two_prod(double a, double b, double* p, double* e) {
  *p = a * b;
#if defined(__FMA__)
  *e = __builtin_fma(a, b, -*p);
#else
  const double sp = 134217729.0;                // 2^27 + 1
  double t = sp * a, ah = t - (t - a), al = a - ah;
  t = sp * b;
  const double bh = t - (t - b), bl = b - bh;
  *e = ((ah * bh - *p) + ah * bl + al * bh) + al * bl;
#endif
}

// 10^i as the nearest double, i in [-12, 12] (decade of a value: a >= ten_pow(E + 1) -> E + 1)
inline double ten_pow(int i) {
  static const double t[25] = {1e-12, 1e-11, 1e-10, 1e-9, 1e-8, 1e-7, 1e-6, 1e-5, 1e-4, 1e-3, 1e-2, 1e-1, 1e0,
                               1e1,   1e2,   1e3,   1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11, 1e12};
  return t[i + 12];
}

inline const char* digit_pairs() {
  static const char pairs[] =
      "00010203040506070809101112131415161718192021222324252627282930313233343536373839"
      "40414243444546474849505152535455565758596061626364656667686970717273747576777879"
      "8081828384858687888990919293949596979899";
  return pairs;
}

inline void put_digits12(char* dig, int64_t n) {
  const char* pairs = digit_pairs();
  uint32_t hi = (uint32_t)(n / 1000000), lo = (uint32_t)(n % 1000000);
  for (int i = 4; i >= 0; i -= 2) {
    std::memcpy(dig + 6 + i, pairs + 2 * (lo % 100), 2);
    std::memcpy(dig + i, pairs + 2 * (hi % 100), 2);
    lo /= 100;
    hi /= 100;
  }
}

// round-half-even(a * 10^k) for a >= 0, 0 <= k <= 22, a * 10^k < 2^52
inline int64_t scaled_round(double a, int k) {
  double p, err;                                // a * 10^k = p + err exactly
  two_prod(a, pow10_table()[k], &p, &err);
  // floor(p) for 0 <= p < 2^53 (every caller): the truncating conversion, not a libm floor() call
  const double q = (double)(int64_t)p;
  const double f = p - q;                       // exact
  const int64_t n = (int64_t)q;
  // round up iff f + err > 1/2, ties to even; d = f - 1/2 is exact (Sterbenz for f in [1/4, 1], exact
  // below) and |err| <= half an ulp of p < 1/4, so one branch-free comparison decides every case (the
  // fraction is random in the formatted tables: a three-way branch mispredicted half the time)
  const double d = f - 0.5;
  return n + (int64_t)((d > -err) | ((d == -err) & (int)(n & 1)));
}

// digits -> double (Clinger's fast path: an integer mantissa < 2^53 times / over an exact power of
// ten is one correctly rounded operation, i.e. what strtod returns); false outside it
inline bool digits_value(const char* dig, int nd, int e, bool neg, double* out) {
  if (nd > 15) return false;
  int64_t m = 0;
  for (int i = 0; i < nd; ++i) m = m * 10 + (dig[i] - '0');
  const int k = e - nd + 1;
  double v;
  if (k >= 0 && k <= 22) v = (double)m * pow10_table()[k];
  else if (k < 0 && k >= -22) v = (double)m / pow10_table()[-k];
  else return false;
  *out = neg ? -v : v;
  return true;
}

// Python 2 str(float): "%.12g" plus ".0" on integral-looking output, written at w (at most 32 bytes);
// returns the end.  `back` (optional) receives the value a reader parses from the text.
inline char* put_py2_float(char* w, double d, double* back = nullptr) {
  char* const start = w;
  const double a = std::fabs(d);
  if (a >= 1e-11 && a < 1e11) {                 // 0 <= 11 - E <= 22: an exact power of ten
    uint64_t bits;
    std::memcpy(&bits, &a, 8);
    const int e2 = (int)((bits >> 52) & 0x7ff) - 1022;          // a in [2^(e2-1), 2^e2)
    int E = ((e2 - 1) * 78913) >> 18;          // floor((e2 - 1) log10 2) for |e2| < 1100: E or E - 1
    if (a >= ten_pow(E + 1)) ++E;               // almost always the decade now (the loop repairs the rest)
    int64_t N = 0;
    bool ok = false;
    for (int tries = 0; tries < 3; ++tries) {
      const int k = 11 - E;
      if (k < 0 || k > 22) break;
      N = scaled_round(a, k);
      if (N < 100000000000LL) { --E; continue; }
      if (N >= 1000000000000LL) {
        if (N == 1000000000000LL) { N = 100000000000LL; ++E; ok = true; break; }  // rounded up to 10^12
        ++E;
        continue;
      }
      ok = true;
      break;
    }
    if (ok) {
      char dig[12];
      put_digits12(dig, N);
      int nd = 12;
      while (nd > 1 && dig[nd - 1] == '0') --nd;
      if (d < 0) *w++ = '-';
      if (E < -4 || E >= 12) {
        *w++ = dig[0];
        if (nd > 1) { *w++ = '.'; std::memcpy(w, dig + 1, 11); w += nd - 1; }   // fixed-size copy
        *w++ = 'e';
        *w++ = E < 0 ? '-' : '+';
        const int ae = E < 0 ? -E : E;
        if (ae >= 100) *w++ = (char)('0' + ae / 100);
        *w++ = (char)('0' + ae / 10 % 10);
        *w++ = (char)('0' + ae % 10);
      } else if (E >= 0) {
        for (int i = 0; i <= E; ++i) *w++ = i < nd ? dig[i] : '0';
        *w++ = '.';
        if (nd > E + 1) { std::memcpy(w, dig + E + 1, nd - E - 1); w += nd - E - 1; }
        else *w++ = '0';
      } else {
        // -4 <= E <= -1: "0." and 0-3 zeros from one fixed copy, then the digits from another (both
        // fixed-size: the lengths vary value to value, and variable copies / loops mispredicted)
        std::memcpy(w, "0.000", 5);
        w += 1 - E;
        std::memcpy(w, dig, 12);
        w += nd;
      }
      if (back && !digits_value(dig, nd, E, d < 0, back)) std::from_chars(start, w, *back);
      return w;
    }
  }
  if (std::isnan(d)) { std::memcpy(w, "nan", 3); if (back) *back = d; return w + 3; }
  if (std::isinf(d)) {
    const char* t = d > 0 ? "inf" : "-inf";
    const size_t n = std::strlen(t);
    std::memcpy(w, t, n);
    if (back) *back = d;
    return w + n;
  }
  auto r = std::to_chars(w, w + 32, d, std::chars_format::general, 12);
  bool has = false;
  for (char* q = w; q < r.ptr; ++q)
    if (*q == '.' || *q == 'e') { has = true; break; }
  w = r.ptr;
  if (!has) { *w++ = '.'; *w++ = '0'; }
  if (back) std::from_chars(start, w, *back);
  return w;
}

// The value a reader parses from Python 2 str(d), without the text: the 12 significant digits N and
// decade E exactly as put_py2_float computes them, then N / 10^(11 - E) -- one correctly rounded
// division of exact operands, the same double strtod returns for the digits (Clinger; trailing zeros
// do not change the real number).  False outside 1e-11 <= |d| < 1e11 (the caller formats and parses).
inline bool py2_value(double d, double* out) {
  const double a = std::fabs(d);
  if (!(a >= 1e-11 && a < 1e11)) return false;
  uint64_t bits;
  std::memcpy(&bits, &a, 8);
  const int e2 = (int)((bits >> 52) & 0x7ff) - 1022;
  int E = ((e2 - 1) * 78913) >> 18;            // floor((e2 - 1) log10 2), as put_py2_float
  E += a >= ten_pow(E + 1) ? 1 : 0;             // (a select, not a data-dependent branch)
  {
    // the common case without branches on the data: E right, N in [10^11, 10^12], where N = 10^12 is
    // a round-up into the next decade (12 digits "100000000000" one decade up: the same value)
    int k = 11 - E;                             // 1 <= k <= 22 for 1e-11 <= a < 1e11
    int64_t N = scaled_round(a, k);
    if (__builtin_expect(N >= 100000000000LL && N <= 1000000000000LL, 1)) {
      const int up = N == 1000000000000LL ? 1 : 0;
      N = up ? 100000000000LL : N;
      k -= up;
      const double v = (double)N / pow10_table()[k];
      *out = std::copysign(v, d);
      return true;
    }
  }
  for (int tries = 0; tries < 3; ++tries) {
    const int k = 11 - E;
    if (k < 0 || k > 22) return false;
    int64_t N = scaled_round(a, k);
    if (N < 100000000000LL) { --E; continue; }
    if (N >= 1000000000000LL) {
      if (N == 1000000000000LL) { N = 100000000000LL; ++E; }
      else { ++E; continue; }
    }
    const int kk = 11 - E;
    if (kk < 0 || kk > 22) return false;
    const double v = (double)N / pow10_table()[kk];
    *out = d < 0 ? -v : v;
    return true;
  }
  return false;
}

inline void append_py2_float(std::string& out, double d, double* back = nullptr) {
  char buf[40];
  out.append(buf, put_py2_float(buf, d, back) - buf);
}

// printf("%5.10f"): finite values always exceed the 5-character field width, so the conversion
// is the exact 10-decimal rounding: N = round-half-even(|d| * 1e10) for |d| < 4.5e5 (N < 2^52),
// the exact printf-equivalent path beyond; nan / inf keep printf's padded spelling.
inline char* put_fixed10(char* w, double d, double* back = nullptr) {
  const double a = std::fabs(d);
  if (a < 4.5e5) {                              // |d| 1e10 < 2^52: the rounding error term is <= 1/4
    int64_t N = scaled_round(a, 10);
    const int64_t ip = N / 10000000000LL, fp = N % 10000000000LL;
    *w = '-';
    w += std::signbit(d) ? 1 : 0;               // branch-free sign (log beta: always '-'; gamma: never)
    const char* pr = digit_pairs();
    if (ip < 100) {                             // 1 or 2 integer digits without a data-dependent branch
      const int one = ip < 10;
      std::memcpy(w, pr + 2 * ip + one, 2);
      w += 2 - one;
    } else {
      w = std::to_chars(w, w + 24, ip).ptr;
    }
    *w++ = '.';
    // ten fraction digits as two independent five-digit halves (shorter dependency chains)
    const uint32_t hi = (uint32_t)(fp / 100000), lo = (uint32_t)(fp % 100000);
    w[0] = (char)('0' + hi / 10000);
    w[5] = (char)('0' + lo / 10000);
    const uint32_t h4 = hi % 10000, l4 = lo % 10000;
    std::memcpy(w + 1, pr + 2 * (h4 / 100), 2);
    std::memcpy(w + 3, pr + 2 * (h4 % 100), 2);
    std::memcpy(w + 6, pr + 2 * (l4 / 100), 2);
    std::memcpy(w + 8, pr + 2 * (l4 % 100), 2);
    w += 10;
    if (back) {
      const double x = (double)N / 1e10;
      *back = std::signbit(d) ? -x : x;
    }
    return w;
  }
  return nullptr;                               // caller takes the exact path (append_fixed10)
}

inline void append_fixed10(std::string& out, double d, double* back = nullptr) {
  char b[48];
  if (char* e = put_fixed10(b, d, back)) {
    out.append(b, e - b);
    return;
  }
  const size_t at = out.size();
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
  // fast path: at most 15 digits and at most one '.': N (the digits) is an exact integer and so is
  // 10^f (f fraction digits <= 15), so N / 10^f is the correctly rounded value Java returns
  if (n <= 16) {
    uint64_t N = 0;
    int nd = 0, f = -1;
    const char* q = s;
    for (; q < e; ++q) {
      const unsigned d = (unsigned)(unsigned char)*q - '0';
      if (d < 10) {
        N = N * 10 + d;
        ++nd;
        f += f >= 0;
      } else if (*q == '.' && f < 0) {
        f = 0;
      } else {
        break;
      }
    }
    if (q == e && nd > 0 && nd <= 15) {
      static constexpr double p10[16] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7,
                                         1e8, 1e9, 1e10, 1e11, 1e12, 1e13, 1e14, 1e15};
      double v = (double)N;
      if (f > 0) v /= p10[f];
      *out = neg ? -v : v;
      return true;
    }
  }
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
