// Shared device helpers for the oni_ml_amd CDNA4 (gfx950) kernels.
//
// * wave64 everywhere: group reductions are written for 64-lane wavefronts;
//   sub-wave groups (16/32 lanes) use shuffles bounded by their width so
//   several short documents can share one wavefront.
// * special functions follow the series used by lda-c's utils.c (digamma:
//   shift by 6 + asymptotic expansion), so the device E-step and the host
//   reference agree on the same approximation.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdexcept>
#include <string>

#define ONI_HIP_CHECK(expr)                                                        \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess) {                                                        \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(_e) + \
                               " at " + __FILE__ + ":" + std::to_string(__LINE__)); \
    }                                                                              \
  } while (0)

namespace oni {

// exp(-100): the value lda-c's M-step floor (log_prob_w = -100) contributes in
// the E-step.  It is an f32 subnormal; hipcc keeps f32 denormals by default.
constexpr float kExpMinus100 = 3.7200759760208e-44f;

// lda-c digamma (utils.c): x+6 shift, 4-term asymptotic series, then the six
// recurrence corrections.
// Reciprocals use v_rcp_f32 (1 ulp) instead of IEEE division (a 10-instruction
// div_scale/fmas/fixup sequence each): the E-step's per-topic phase is
// dominated by these.
__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }

__device__ __forceinline__ float digammaf_ldac(float x) {
  float p;
  x = x + 6.0f;
  const float ix = frcp(x);
  p = ix * ix;
  p = (((0.004166666666667f * p - 0.003968253986254f) * p + 0.008333333333333f) * p -
       0.083333333333333f) * p;
  p = p + __logf(x) - 0.5f * ix - frcp(x - 1.0f) - frcp(x - 2.0f) - frcp(x - 3.0f) - frcp(x - 4.0f) -
      frcp(x - 5.0f) - frcp(x - 6.0f);
  return p;
}

// log Gamma(x), x > 0: Stirling series at x + 6 and the recurrence (the form of
// lda-c's utils.c log_gamma), float with fast reciprocal / log.  About 1e-7
// relative, the precision of the float lgammaf it replaces, at a fraction of
// its cost.
__device__ __forceinline__ float lgammaf_fast(float x) {
  const float xs = x + 6.0f;
  const float ix = frcp(xs);
  const float z = ix * ix;
  const float ser = (((-0.000595238095238f * z + 0.000793650793651f) * z - 0.002777777777778f) * z +
                     0.083333333333333f) * ix;
  const float p = x * (x + 1.0f) * (x + 2.0f);
  const float q = (x + 3.0f) * (x + 4.0f) * (x + 5.0f);
  return (xs - 0.5f) * __logf(xs) - xs + 0.918938533204673f + ser - __logf(p) - __logf(q);
}

__device__ __forceinline__ double digamma_ldac(double x) {
  double p;
  x = x + 6.0;
  p = 1.0 / (x * x);
  p = (((0.004166666666667 * p - 0.003968253986254) * p + 0.008333333333333) * p -
       0.083333333333333) * p;
  p = p + log(x) - 0.5 / x - 1.0 / (x - 1.0) - 1.0 / (x - 2.0) - 1.0 / (x - 3.0) -
      1.0 / (x - 4.0) - 1.0 / (x - 5.0) - 1.0 / (x - 6.0);
  return p;
}

// ---------------------------------------------------------------------------
// Wavefront / group reductions.  G must be a power of two <= 64; all lanes of
// the group must be active (callers keep loop conditions group-uniform).
// ---------------------------------------------------------------------------
template <int G, typename T>
__device__ __forceinline__ T group_sum(T x) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) x += __shfl_xor(x, o, G);
  return x;
}

template <int G, typename T>
__device__ __forceinline__ T group_max(T x) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) {
    T y = __shfl_xor(x, o, G);
    x = x > y ? x : y;
  }
  return x;
}

// Wave-level LDS hand-off between lanes of ONE wavefront: orders the
// ds_writes before the ds_reads (same wave, so no s_barrier is needed and
// divergent groups never deadlock).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Multi-value butterfly: reduces v[0..N) over the G lanes of a group and
// leaves the total of value i in EVERY lane's v[i].  N*log2(G) shuffles.
template <int G, int N>
__device__ __forceinline__ void group_sum_vec(float (&v)[N]) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) {
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] += __shfl_xor(v[i], o, G);
  }
}

// Bijective XCD-aware remap of a 1-D grid (cdna_hip_programming.md §5 T1):
// consecutive logical blocks land on the same XCD (L2) for locality.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int nxcd = 8;
  if (nwg < nxcd) return bid;
  int q = nwg / nxcd, r = nwg % nxcd;
  int xcd = bid % nxcd, idx = bid / nxcd;
  int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + idx;
}

}  // namespace oni
