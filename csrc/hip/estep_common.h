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

}  // namespace oni
