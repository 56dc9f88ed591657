// fp64 math and wave-reduction helpers shared by the block Gauss-Seidel E-step kernels
// (lda_gs64.hip: the one-workgroup document kernels; experimental/lda_xsplit.hip: one document over the CUs of
// an XCD).  lda-c's arithmetic in short dependency chains for gfx950.
#pragma once
#include "common.h"
#include "kernels.h"
#include "log_table.h"

namespace oni {
namespace gs {

// c*phi rows are written once per E-step and read once by the suff-stats pass: nontemporal
// stores keep them from evicting the beta rows every document re-gathers each sweep
typedef double dvec2 __attribute__((ext_vector_type(2)));

constexpr int ilog2(int x) { return x <= 1 ? 0 : 1 + ilog2(x / 2); }
// 1/x for a positive normal double: v_rcp_f64 and two Newton steps (~1 ulp).
__device__ __forceinline__ double drcp(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = fma(-x, r, 1.0);
  r = fma(r, e, r);
  e = fma(-x, r, 1.0);
  return fma(r, e, r);
}

// fp64 VALU results have a ~30-cycle dependent latency on gfx950 (scripts/micro/fp64_latency.hip:
// a dependent v_fma_f64 chain runs at ~1/8 of the issue rate), so the transcendentals below are
// written for a short dependency chain: Estrin-scheme polynomials (depth log2(degree) + 1 instead
// of the degree) and one reciprocal where lda-c's digamma has seven.

// Natural log of a positive normal double: y = 2^e m, m in [sqrt(1/2), sqrt(2)),
// log m = 2 atanh(f) = 2f + f s P(s), f = (m - 1) / (m + 1), s = f^2 <= 0.0295, P through
// s^10 (truncation < 1e-17), ln 2 split hi / lo.  ~2 ulp; ~15 dependent steps (OCML's log: ~100
// instructions, ~490 cycles dependent).
__device__ __forceinline__ double flog(double y) {
  int e = __builtin_amdgcn_frexp_exp(y);
  double mt = __builtin_amdgcn_frexp_mant(y);            // [0.5, 1)
  const bool lo = mt < 0.70710678118654752;
  mt = lo ? mt + mt : mt;
  e = lo ? e - 1 : e;
  const double f = (mt - 1.0) * drcp(mt + 1.0);
  const double s = f * f, s2 = s * s, s4 = s2 * s2, s8 = s4 * s4;
  // c_i = 2 / (2 i + 3), i = 0..10
  const double a0 = fma(0.4, s, 0.66666666666666667), a1 = fma(0.22222222222222222, s, 0.28571428571428571);
  const double a2 = fma(0.15384615384615385, s, 0.18181818181818182);
  const double a3 = fma(0.11764705882352941, s, 0.13333333333333333);
  const double a4 = fma(0.095238095238095238, s, 0.10526315789473684);
  const double b0 = fma(a1, s2, a0), b1 = fma(a3, s2, a2), b2 = fma(0.086956521739130435, s2, a4);
  const double P = fma(b2, s8, fma(b1, s4, b0));
  const double de = (double)e;
  return fma(de, 6.93147180369123816490e-01, fma(de, 1.90821492927058770002e-10, fma(f * s, P, f + f)));
}

// exp(x) for |x| < 700: x = k ln 2 + r, |r| <= ln2 / 2, degree-12 Taylor polynomial in Estrin
// form (truncation < 2e-16 relative), 2^k by ldexp.
__device__ __forceinline__ double fexp(double x) {
  const double k = __builtin_rint(x * 1.44269504088896340736);
  const double r = fma(-k, 1.90821492927058770002e-10, fma(-k, 6.93147180369123816490e-01, x));
  const double r2 = r * r, r4 = r2 * r2, r8 = r4 * r4;
  const double a0 = 1.0 + r, a1 = fma(1.66666666666666667e-01, r, 0.5);
  const double a2 = fma(8.33333333333333333e-03, r, 4.16666666666666667e-02);
  const double a3 = fma(1.98412698412698413e-04, r, 1.38888888888888889e-03);
  const double a4 = fma(2.75573192239858907e-06, r, 2.48015873015873016e-05);
  const double a5 = fma(2.50521083854417188e-08, r, 2.75573192239858907e-07);
  const double b0 = fma(a1, r2, a0), b1 = fma(a3, r2, a2), b2 = fma(a5, r2, a4);
  const double c0 = fma(b1, r4, b0), c1 = fma(2.08767569878680990e-09, r4, b2);
  return __builtin_amdgcn_ldexp(fma(c1, r8, c0), (int)k);
}

// Natural log of a positive normal double by table: y = 2^e m, m in [1, 2), i = the top 7 bits of m's
// fraction, log y = e ln 2 + L_i + log1p(r), r = m inv_i - 1 (one fma, |r| <= 2^-8), log1p by a degree-6
// polynomial (truncation < 3e-18).  inv_i / L_i = -log(inv_i): log_table.h (scripts/gen_log_table.py),
// copied into the workgroup's LDS by log_table_fill.  <= 1 ulp for y >= 2 (host emulation with exact fma
// over 6 .. 1e4: 0.65 ulp); near y = 1 the e ln 2 + L cancellation leaves ~1e-16 absolute error (flog keeps
// the relative accuracy there).  17 VALU instructions and one ds_read_b128 against flog's ~36.
// LDS image: [0, 128) the log table {inv_i, L_i}, [128, 160) the exp table kExpTab as pairs
constexpr int kMathTabN = 160;
__device__ __forceinline__ void log_table_fill(dvec2* __restrict__ s) {
  for (int i = threadIdx.x; i < kMathTabN; i += blockDim.x)
    s[i] = i < 128 ? dvec2{kLogTab[i][0], kLogTab[i][1]} : dvec2{kExpTab[2 * (i - 128)], kExpTab[2 * (i - 128) + 1]};
}
__device__ __forceinline__ double flog_t(double y, const dvec2* __restrict__ tab) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(y);
  const unsigned hi = (unsigned)(b >> 32);
  const dvec2 c = tab[(hi >> 13) & 127u];
  const double mt = __longlong_as_double((long long)(((unsigned long long)((hi & 0x000FFFFFu) | 0x3FF00000u) << 32) |
                                                     (b & 0xFFFFFFFFull)));
  const double de = (double)((int)(hi >> 20) - 1023);
  const double r = fma(mt, c.x, -1.0);
  const double r2 = r * r;
  const double q1 = fma(r, 0.33333333333333333, -0.5);
  const double q3 = fma(r2, -0.16666666666666667, fma(r, 0.2, -0.25));
  const double p = fma(r2 * r2, q3, fma(r2, q1, r));
  return fma(de, 6.93147180369123816490e-01, fma(de, 1.90821492927058770002e-10, c.y + p));
}

// exp(x) for |x| < 700 by table: x = (64 e + j) ln 2 / 64 + r, |r| <= ln 2 / 128, exp x = 2^e T_j (1 + q(r)),
// q of degree 6 (truncation < 3e-20), T_j = RN(2^(j/64)) from the LDS image (log_table_fill).  <= 1 ulp
// (host emulation with exact fma over [-700, 10]); 17 VALU instructions against fexp's 21.
__device__ __forceinline__ double fexp_t(double x, const dvec2* __restrict__ tab) {
  const double kf = __builtin_rint(x * 92.332482616893657);
  const double r = fma(-kf, 0x1.a39ef35793c76p-39, fma(-kf, 0x1.62e42fee00000p-7, x));
  const int ki = (int)kf;
  const double T = reinterpret_cast<const double*>(tab + 128)[ki & 63];
  const double r2 = r * r;
  const double a = fma(r, 0.16666666666666667, 0.5);
  const double c = fma(r2, 0.0013888888888888889, fma(r, 0.0083333333333333333, 0.041666666666666667));
  const double q = fma(r2 * r2, c, fma(r2, a, r));
  return __builtin_amdgcn_ldexp(fma(T, q, T), ki >> 6);
}

// lda-c digamma (x + 6 shift, 4-term series, six recurrence terms) and
// E = exp(psi - m).  The six reciprocals 1/(x+i) are (dA B + dB A) / (A B) with
// A = x(x+1)(x+2), B = (x+3)(x+4)(x+5) (one reciprocal; A B < 1e54 for x < 1e9);
// E = (x+6) exp(rest - m) does not wait on the log.
// R1 (the throughput-bound kernels): one reciprocal R = 1 / (A B y) for both 1/y = A B R and the six terms
// (dA B + dB A) y R -- 3 instructions fewer, ~4 more dependent steps before the series (A B y < 1e63 for
// x < 1e9), a few ulp on terms that are not the log
// ET: exp by table too (off in the 16-lane kernel: 211 -> 243 VGPRs there and 2.5 % slower, r5ao)
template <bool TAB = false, bool R1 = false, bool ET = TAB>
__device__ __forceinline__ void psi_exp(double x, double m, double& psi, double& e, const dvec2* tab = nullptr) {
  const double y = x + 6.0;
  const double x1 = x + 1.0, x2 = x + 2.0, x3 = x + 3.0, x4 = x + 4.0, x5 = x + 5.0;
  const double A = x * x1 * x2, dA = fma(x, x1 + x2, x1 * x2);
  const double B = x3 * x4 * x5, dB = fma(x3, x4 + x5, x4 * x5);
  double iy, S;
  if constexpr (R1) {
    const double AB = A * B;
    const double R = drcp(AB * y);
    iy = AB * R;
    S = fma(dA, B, dB * A) * (y * R);
  } else {
    iy = drcp(y);
    S = fma(dA, B, dB * A) * drcp(A * B);
  }
  const double z = iy * iy;
  const double ser = fma(fma(0.004166666666667, z, -0.003968253986254), z * z,
                         fma(0.008333333333333, z, -0.083333333333333)) * z;
  const double rest = fma(-0.5, iy, ser) - S;
  psi = (TAB ? flog_t(y, tab) : flog(y)) + rest;
  e = y * (ET ? fexp_t(rest - m, tab) : fexp(rest - m));
}

// ln Gamma(x), x > 0: Stirling series at y = x + 6 (terms through 1/y^13, truncation
// < 1e-13 absolute) and the recurrence lnG(x) = lnG(x + 6) - ln(x (x+1) ... (x+5)).
// Same accuracy class as the libm lgamma lda-c calls, at a fraction of OCML's cost.
template <bool TAB = false>
__device__ __forceinline__ double lgamma_pos(double x, const dvec2* tab = nullptr) {
  const double y = x + 6.0;
  const double iy = drcp(y);
  const double z = iy * iy;
  const double ser = ((((((0.0064102564102564103 * z - 0.0019175269175269175) * z + 0.00084175084175084175) * z -
                         0.00059523809523809524) * z + 0.00079365079365079365) * z - 0.0027777777777777778) * z +
                      0.083333333333333333) * iy;
  const double p = x * (x + 1.0) * (x + 2.0) * ((x + 3.0) * (x + 4.0) * (x + 5.0));
  if constexpr (TAB)
    return (y - 0.5) * flog_t(y, tab) - y + 0.91893853320467274 + ser - flog_t(p, tab);
  else
    return (y - 0.5) * flog(y) - y + 0.91893853320467274 + ser - flog(p);
}

__device__ __forceinline__ double psi_only(double x) {
  double p, e;
  psi_exp(x, 0.0, p, e);
  return p;
}

// ---- symmetric lane reductions (every participating lane ends with the same bits) ----
// DIRECT: every exchange reads the partner lane itself (safe when only some lane groups are
// active); otherwise xor 4 may route through the lanes of a neighbouring group (two DPP moves,
// no LDS crossbar), which needs the whole 8-lane half-row active.
template <int MASK, bool DIRECT = true>
__device__ __forceinline__ double xsum(double x) {
  using namespace detail;
  if constexpr (MASK == 1) {
    return x + xchg<kQuadXor1>(x);
  } else if constexpr (MASK == 2) {
    return x + xchg<kQuadXor2>(x);
  } else if constexpr (MASK == 4 && !DIRECT) {
    // xor 4 = row_half_mirror (l -> 7 - l within 8) then quad_perm [3,2,1,0]
    return x + xchg<0x1B>(xchg<kRowHalfMirror>(x));
  } else if constexpr (MASK == 4) {
    const long long b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_ds_swizzle((int)(b & 0xffffffffLL), 0x101F);
    const int hi = __builtin_amdgcn_ds_swizzle((int)(b >> 32), 0x101F);
    return x + __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
  } else if constexpr (MASK == 8) {
    return x + xchg<0x128>(x);   // row_ror:8 == xor 8 inside a 16-lane row
  } else if constexpr (MASK == 16) {
    return swap_combine<false>(x, add<double>);
  } else {
    static_assert(MASK == 32, "lane mask");
    return swap_combine<true>(x, add<double>);
  }
}

// sum over lane bits [LO, HI)
template <int LO, int HI, bool DIRECT = true>
__device__ __forceinline__ double bits_sum(double x) {
  if constexpr (LO >= HI) {
    return x;
  } else {
    return bits_sum<LO + 1, HI, DIRECT>(xsum<(1 << LO), DIRECT>(x));
  }
}

__device__ __forceinline__ double params_vconv(const double* p) { return (double)(float)p[3]; }

// lda-c: converged = (L_old - L) / L_old; the loop runs while converged > VAR_CONVERGED
// and (var_iter < VAR_MAX_ITER or VAR_MAX_ITER == -1).
__device__ __forceinline__ bool var_continue(double conv, double vconv, int it, int vmi) {
  return conv > vconv && (it < vmi || vmi == -1);
}

// Sum KS per-lane values over the 64 lanes of a wave and store topic totals into out[k]:
// a reduce-scatter in registers, no LDS.  v_permlane32_swap (xor 32) and v_permlane16_swap
// (xor 16) each combine a PAIR of values with one swap per dword (lanes of one half keep the
// first value's sum, the other half the second's), leaving ceil(ceil(KS/2)/2) values per lane;
// these are summed over the 16 lanes of each row by DPP (quad xor 1 / 2, half-mirror + quad
// reverse = xor 4, row_ror 8 = xor 8).  Row rho = lane bits 5..4 then holds topics
// (bit5 ? H1 : 0) + (bit4 ? H2 : 0) + i, i < H2.  Needs all 64 lanes active.
__device__ __forceinline__ double swap_sum32(double first, double second) {
  // permlane32_swap(vdst = first, vsrc = second) exchanges vdst's upper half with vsrc's lower
  // half: vdst' = [first_lo, second_lo], vsrc' = [first_hi, second_hi], so the sum leaves lanes
  // 0-31 with first's total and lanes 32-63 with second's
  const unsigned long long f = (unsigned long long)__double_as_longlong(first);
  const unsigned long long g = (unsigned long long)__double_as_longlong(second);
  const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)f, (unsigned)g, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(f >> 32), (unsigned)(g >> 32), false, false);
  const double x = __longlong_as_double((long long)(((unsigned long long)hi[0] << 32) | lo[0]));
  const double y = __longlong_as_double((long long)(((unsigned long long)hi[1] << 32) | lo[1]));
  return x + y;
}
__device__ __forceinline__ double swap_sum16(double first, double second) {
  // permlane16_swap(vdst = first, vsrc = second) exchanges vdst's odd rows with vsrc's even rows:
  // the sum leaves rows 0 / 2 with first's total, rows 1 / 3 with second's
  const unsigned long long f = (unsigned long long)__double_as_longlong(first);
  const unsigned long long g = (unsigned long long)__double_as_longlong(second);
  const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)f, (unsigned)g, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(f >> 32), (unsigned)(g >> 32), false, false);
  const double x = __longlong_as_double((long long)(((unsigned long long)hi[0] << 32) | lo[0]));
  const double y = __longlong_as_double((long long)(((unsigned long long)hi[1] << 32) | lo[1]));
  return x + y;
}

// The same reduce-scatter with the totals left in registers: returns the topic whose total this lane
// holds (v), or -1 (at KS <= 32 only lanes with (lane & 15) < 8 hold one; lanes 8-15 of every row never)
template <int KS>
__device__ __forceinline__ int wave_topic_sums_reg(const double (&acc)[KS], int lane, double& v) {
  constexpr int H1 = (KS + 1) / 2, H2 = (H1 + 1) / 2;
  double a1[H1];
#pragma unroll
  for (int i = 0; i < H1; ++i) a1[i] = swap_sum32(acc[i], i + H1 < KS ? acc[i + H1] : 0.0);
  double a2[H2];
#pragma unroll
  for (int i = 0; i < H2; ++i) a2[i] = swap_sum16(a1[i], i + H2 < H1 ? a1[i + H2] : 0.0);
#pragma unroll
  for (int i = 0; i < H2; ++i) a2[i] = bits_sum<0, 4, false>(a2[i]);
  const int base = ((lane >> 5) & 1) * H1 + ((lane >> 4) & 1) * H2;
  const int i = lane & 15;
  v = 0.0;
#pragma unroll
  for (int ii = 0; ii < H2; ++ii) v = i == ii ? a2[ii] : v;
  const bool hi4 = (lane >> 4) & 1;
  return (i < H2 && (!hi4 || H2 + i < H1) && base + i < KS) ? base + i : -1;
}

template <int KS>
__device__ __forceinline__ void wave_topic_sums(const double (&acc)[KS], int lane, double* out) {
  double v;
  const int k = wave_topic_sums_reg<KS>(acc, lane, v);
  if (k >= 0) out[k] = v;
}

}  // namespace gs
}  // namespace oni
