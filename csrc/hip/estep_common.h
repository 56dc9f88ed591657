// Device helpers shared by the E-step kernels (lda_estep.hip, lda_estep_split.hip).
#pragma once
#include "common.h"
#include "kernels.h"

namespace oni {

// One word-major beta row (KS topics, 16-byte aligned) into registers.
template <int KS>
__device__ __forceinline__ void load_row(const float* __restrict__ beta, int w, float (&row)[KS]) {
  const float4* p = reinterpret_cast<const float4*>(beta + (size_t)w * KS);
#pragma unroll
  for (int j = 0; j < KS / 4; ++j) {
    float4 v = p[j];
    row[4 * j + 0] = v.x;
    row[4 * j + 1] = v.y;
    row[4 * j + 2] = v.z;
    row[4 * j + 3] = v.w;
  }
}

// P = sum_k E_k * row_k with E read from LDS (broadcast: every lane of a group
// reads the same address).
template <int KS>
__device__ __forceinline__ float dot_lds(const float* sE, const float (&row)[KS]) {
  const float4* e4 = reinterpret_cast<const float4*>(sE);
  float p0 = 0.f, p1 = 0.f;
#pragma unroll
  for (int j = 0; j < KS / 4; ++j) {
    float4 e = e4[j];
    p0 = fmaf(e.x, row[4 * j + 0], p0);
    p1 = fmaf(e.y, row[4 * j + 1], p1);
    p0 = fmaf(e.z, row[4 * j + 2], p0);
    p1 = fmaf(e.w, row[4 * j + 3], p1);
  }
  return p0 + p1;
}

constexpr float kPMin = 1e-30f;

// lda-c's variational loop test  (L_old - L) / L_old > VAR_CONVERGED  with IEEE semantics
// (L_old == 0 on the first iteration: +-inf or NaN), evaluated without the f64 division:
// the sign of L_old decides the direction of the inequality.
__device__ __forceinline__ bool var_more(double lik_old, double L, double c) {
  // branch-free (selects, no exec-mask branches on the topic-phase chain):
  //   lik_old < 0: (lik_old - L) < c lik_old;  lik_old > 0: (lik_old - L) > c lik_old;
  //   lik_old == 0: (0 - L) / 0 = +inf (L < 0), -inf or NaN otherwise
  const double d = lik_old - L, t = c * lik_old;
  const bool neg = lik_old < 0.0, pos = lik_old > 0.0;
  const bool zero_case = !neg & !pos & (L < 0.0) & (c < INFINITY);
  return (neg & (d < t)) | (pos & (d > t)) | zero_case;
}

// r = c / P with v_rcp_f32 (1 ulp) instead of IEEE division: the correctly rounded
// f32 divide is a ~10-instruction div_scale / fmas / fixup sequence, a large share
// of the per-word work (P >= kPMin is a normal float, so rcp is exact to 1 ulp).
__device__ __forceinline__ float rdiv(float c, float P) { return c * __builtin_amdgcn_rcpf(P); }

// Beta rows each lane keeps in VGPRs across the variational iterations:
// 4-wave kernels (G64C, B4) and 8-wave kernels (B8, split segments; 2 waves per
// SIMD leave ~256 VGPRs per lane, so up to 8 rows of 20 topics fit).
constexpr int rows_per_lane_4w(int KS) { return KS <= 32 ? 4 : (KS <= 64 ? 2 : 1); }
constexpr int rows_per_lane_8w(int KS) { return KS <= 20 ? 6 : (KS <= 32 ? 3 : 1); }

// Per-launch scalars from device memory when the launch is graph-replayed:
// params = {alpha, lgamma(K alpha) - K lgamma(alpha), VAR_MAX_ITER, VAR_CONVERGED,
// done}.  Returns true when the EM loop has already converged (skip the launch).
template <typename Args>
__device__ __forceinline__ bool load_params(Args& a) {
  if (a.params) {
    if (a.params[kParamDone] != 0.0) return true;
    a.alpha = (float)a.params[0];
    a.lik_const = a.params[1];
    a.var_max_iter = (int)a.params[2];
    a.var_conv = (float)a.params[3];
  }
  return false;
}

// ---------------------------------------------------------------------------
// Split-document hand-off: iteration-tagged 8-byte granules {float, uint32 tag}.
// A 64-bit aligned relaxed atomic store / load is single-copy atomic, so a reader
// that sees the tag sees the value; agent scope makes the accesses coherent
// across XCDs (sc1, no stale L2 / L1 lines).  Tag = (launch epoch << 12) |
// (iteration & 0xfff): iteration bits separate it from it - 2 (the previous use
// of the parity buffer), the epoch separates launches.
// ---------------------------------------------------------------------------
constexpr long kSplitSpinLimit = 1L << 24;   // ~seconds of polling, then give up (error flag)

__device__ __forceinline__ unsigned split_tag(int epoch, int it) {
  return ((unsigned)(epoch & 0xfffff) << 12) | (unsigned)(it & 0xfff);
}

__device__ __forceinline__ void put_tagged(unsigned long long* p, float v, unsigned tag) {
  const unsigned long long g = ((unsigned long long)tag << 32) | (unsigned long long)__float_as_uint(v);
  __hip_atomic_store(p, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// sum_{q < n} value(x[q * stride]) in order q = 0, 1, ..., in double, each granule
// awaited until it carries `tag`; 8 loads in flight per round trip, and the granules still
// missing their tag are re-polled together (one round trip per poll, not one per stale
// granule).  Returns false on a timeout.
__device__ __forceinline__ bool tagged_sum(const unsigned long long* x, int n, int stride, unsigned tag, double& out) {
  double s = 0.0;
  long spins = 0;
  for (int q0 = 0; q0 < n; q0 += 8) {
    unsigned long long v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      v[u] = __hip_atomic_load(x + (size_t)min(q0 + u, n - 1) * stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (;;) {
      unsigned pending = 0;
#pragma unroll
      for (int u = 0; u < 8; ++u) pending |= (q0 + u < n && (unsigned)(v[u] >> 32) != tag) ? (1u << u) : 0u;
      if (pending == 0) break;
      if (++spins > kSplitSpinLimit) {
        out = __builtin_nan("");
        return false;
      }
      __builtin_amdgcn_s_sleep(1);
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if ((pending >> u) & 1u)
          v[u] = __hip_atomic_load(x + (size_t)(q0 + u) * stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (q0 + u < n) s += (double)__uint_as_float((unsigned)(v[u] & 0xffffffffu));
  }
  out = s;
  return true;
}

// Gather every segment's row (KS topic granules + the log-sum hi/lo pair) in segment
// order: lane-column k < KS + 2 of the calling wave sums its column over the n
// segments, all columns in flight together (one round-trip chain, not one per
// segment for the log-sum).  acc[j] = topic lane + 64 j (0 past KS), lsum = the
// document's log-sum; the same bits in every workgroup of the document.
template <int KS, int TJ>
__device__ __forceinline__ bool tagged_gather(const unsigned long long* x, int n, int stride, unsigned tag, int lane,
                                              float (&acc)[TJ], double& lsum) {
  constexpr int TX = (KS + 2 + 63) / 64;
  double v[TX];
  bool ok = true;
#pragma unroll
  for (int j = 0; j < TX; ++j) {
    const int k = lane + 64 * j;
    v[j] = 0.0;
    if (k < KS + 2) ok &= tagged_sum(x + k, n, stride, tag, v[j]);
  }
#pragma unroll
  for (int j = 0; j < TJ; ++j) acc[j] = (lane + 64 * j < KS) ? (float)v[j] : 0.f;
  lsum = __shfl(v[KS / 64], KS % 64) + __shfl(v[(KS + 1) / 64], (KS + 1) % 64);
  return ok;
}

// Publish one segment's iteration partials: lanes 0..63 of the calling wave write the
// KS topic granules (acc_of(k)), lane 0 also the log-sum pair.
template <int KS, typename AccOf>
__device__ __forceinline__ void publish_tagged(unsigned long long* row, AccOf acc_of, double lsum, int lane,
                                               unsigned tag) {
#pragma unroll
  for (int j = 0; j < (KS + 63) / 64; ++j) {
    const int k = lane + 64 * j;
    if (k < KS) put_tagged(row + k, acc_of(j), tag);
  }
  if (lane == 0) {
    const float hi = (float)lsum;
    const float lo = (float)(lsum - (double)hi);
    put_tagged(row + KS, hi, tag);
    put_tagged(row + KS + 1, lo, tag);
  }
}

// End of a split launch: the last segment of the document to get here bumps the
// document's epoch and resets the exit count (graph replays need no memset).
__device__ __forceinline__ void split_exit(int* counter, int n_docs, int nseg) {
  if (threadIdx.x == 0) {
    int* exits = counter + n_docs;
    if (__hip_atomic_fetch_add(exits, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nseg - 1) {
      __hip_atomic_store(exits, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace oni
