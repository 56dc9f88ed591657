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

// Device-side EM loop control (em_control.hip): once the convergence test has
// fired, every kernel of the iterations still queued behind it returns at once.
__device__ __forceinline__ bool gated(const double* gate) { return gate != nullptr && *gate != 0.0; }

// lda-c digamma (utils.c): x+6 shift, 4-term asymptotic series, then the six
// recurrence corrections.
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
//
// Within a 16-lane row the exchanges are DPP modifiers on the VALU op itself
// (quad_perm xor1 / xor2, row_half_mirror, row_mirror: no LDS crossbar), the
// 32-lane step a v_permlane16_swap, the 64-lane step a v_permlane32_swap (gfx950).
// Every step combines a lane with its partner commutatively, so all lanes of
// a group finish with bitwise the same total (the kernels rely on that:
// replicated topic state must not diverge between lanes).

namespace detail {
template <int CTRL>
__device__ __forceinline__ int dpp(int x) {
  return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xF, 0xF, true);
}
constexpr int kQuadXor1 = 0xB1;   // quad_perm [1,0,3,2]
constexpr int kQuadXor2 = 0x4E;   // quad_perm [2,3,0,1]
constexpr int kRowHalfMirror = 0x141;
constexpr int kRowMirror = 0x140;
constexpr int kSwzXor16 = 0x401F; // ds_swizzle bitmask mode: and 0x1f, or 0, xor 0x10

template <int CTRL>
__device__ __forceinline__ float xchg(float x) { return __int_as_float(dpp<CTRL>(__float_as_int(x))); }
template <int CTRL>
__device__ __forceinline__ double xchg(double x) {
  const long long b = __double_as_longlong(x);
  const int lo = dpp<CTRL>((int)(b & 0xffffffffLL)), hi = dpp<CTRL>((int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ float swz16(float x) {
  return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(x), kSwzXor16));
}
__device__ __forceinline__ double swz16(double x) {
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_ds_swizzle((int)(b & 0xffffffffLL), kSwzXor16);
  const int hi = __builtin_amdgcn_ds_swizzle((int)(b >> 32), kSwzXor16);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ float rdlane(float x, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), l)); }
__device__ __forceinline__ double rdlane(double x, int l) {
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// gfx950 v_permlane16_swap / v_permlane32_swap with both operands = x: returns
// (x of the even rows / lower half, x of the odd rows / upper half) in EVERY lane,
// so op(first, second) is the xor-16 / xor-32 combination with the same operand
// order in both partner lanes (bitwise identical) -- a VALU exchange, no LDS
// crossbar (ds_swizzle) and no v_readlane / SGPR round trip.
template <bool HALF>
__device__ __forceinline__ void swap_pair(unsigned x, unsigned& lo_part, unsigned& hi_part) {
  if constexpr (HALF) {
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    lo_part = r[0];
    hi_part = r[1];
  } else {
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    lo_part = r[0];
    hi_part = r[1];
  }
}
template <bool HALF, typename Op>
__device__ __forceinline__ float swap_combine(float x, Op op) {
  unsigned a, b;
  swap_pair<HALF>(__float_as_uint(x), a, b);
  return op(__uint_as_float(a), __uint_as_float(b));
}
template <bool HALF, typename Op>
__device__ __forceinline__ double swap_combine(double x, Op op) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(x);
  unsigned alo, blo, ahi, bhi;
  swap_pair<HALF>((unsigned)(u & 0xffffffffULL), alo, blo);
  swap_pair<HALF>((unsigned)(u >> 32), ahi, bhi);
  const double a = __longlong_as_double((long long)(((unsigned long long)ahi << 32) | alo));
  const double b = __longlong_as_double((long long)(((unsigned long long)bhi << 32) | blo));
  return op(a, b);
}
template <typename T>
__device__ __forceinline__ T add(T a, T b) { return a + b; }
template <typename T>
__device__ __forceinline__ T mx(T a, T b) { return a > b ? a : b; }
}  // namespace detail

template <int G, typename T, typename Op>
__device__ __forceinline__ T group_reduce(T x, Op op) {
  static_assert(G == 16 || G == 32 || G == 64, "group size must be 16, 32 or 64");
  using namespace detail;
  x = op(x, xchg<kQuadXor1>(x));
  x = op(x, xchg<kQuadXor2>(x));
  x = op(x, xchg<kRowHalfMirror>(x));
  x = op(x, xchg<kRowMirror>(x));
  if constexpr (G >= 32) x = swap_combine<false>(x, op);
  if constexpr (G == 64) x = swap_combine<true>(x, op);
  return x;
}

template <int G, typename T>
__device__ __forceinline__ T group_sum(T x) {
  return group_reduce<G>(x, [](T a, T b) { return a + b; });
}

template <int G, typename T>
__device__ __forceinline__ T group_max(T x) {
  return group_reduce<G>(x, [](T a, T b) { return a > b ? a : b; });
}

// Sum over the 64 lanes of a wave delivered to lane 63 only, all in DPP (no
// ds_swizzle, no v_readlane): the four row steps of group_reduce, then
// row_bcast:15 (rows 1, 3 add the last lane of rows 0, 2) and row_bcast:31
// (rows 2, 3 add lane 31).  For reductions whose result one lane stores: the
// ds_swizzle + readlane tail of group_reduce costs LDS-pipe round trips and
// readlane hazards per value (~2,000 cycles per variational iteration for the
// KS accumulators of the 4/8-wave document kernels, scripts/estep_phases.py).
namespace detail {
constexpr int kRowBcast15 = 0x142;
constexpr int kRowBcast31 = 0x143;
template <int CTRL, int ROWS>
__device__ __forceinline__ float bcast(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, ROWS, 0xF, false));
}
template <int CTRL, int ROWS>
__device__ __forceinline__ double bcast(double x) {
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffLL), CTRL, ROWS, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROWS, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
}  // namespace detail

template <typename T>
__device__ __forceinline__ T wave_sum_last(T x) {
  using namespace detail;
  x += xchg<kQuadXor1>(x);
  x += xchg<kQuadXor2>(x);
  x += xchg<kRowHalfMirror>(x);
  x += xchg<kRowMirror>(x);
  x += bcast<kRowBcast15, 0xA>(x);
  x += bcast<kRowBcast31, 0xC>(x);
  return x;   // lane 63: the total
}

// Wave-level LDS hand-off between lanes of ONE wavefront: orders the
// ds_writes before the ds_reads (same wave, so no s_barrier is needed and
// divergent groups never deadlock).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Workgroup barrier ordering LDS only: s_waitcnt lgkmcnt(0) + s_barrier, WITHOUT the
// vmcnt(0) wait of __syncthreads()' global release fence, so global loads issued before
// the barrier (prefetches of the next chunk's rows) stay in flight across it.  Only for
// kernels whose threads exchange data through LDS, never through global memory.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Multi-value all-reduce: the total of value i over the G lanes of a group in
// EVERY lane's v[i] (N independent DPP chains: good ILP, no LDS traffic).
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
