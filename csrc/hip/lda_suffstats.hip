// Deterministic LDA sufficient statistics (lda-c doc_e_step):
//
//   class_word[w][k] = sum_{(d,n): w_n = w} c_n phi_nk
//                    = beta[w][k] * sum_{d in docs(w)} E[d][k] * r_{d,n}
//
// where E and r = c/P come from the fused E-step.  Instead of nnz*K float
// atomics (an order-dependent, atomic-rate-bound scatter), the corpus is also
// held in CSC (word-major) order and each word's topic vector is produced by
// exactly one group as a gather-reduce: bitwise reproducible run to run.
// Words are length-bucketed: light words share a wave (16 lanes each), heavy
// (Zipf-head) words get an 8-wave workgroup with a cross-wave LDS reduction.
#include <stdexcept>
#include <string>

#include "common.h"
#include "kernels.h"
#include "em_control.h"
#include "alpha_newton.h"

namespace oni {

template <int KS>
__device__ __forceinline__ void axpy_row(const float* __restrict__ e, int d, float r, float (&acc)[KS]) {
  const float4* p = reinterpret_cast<const float4*>(e + (size_t)d * KS);
#pragma unroll
  for (int j = 0; j < KS / 4; ++j) {
    float4 v = p[j];
    acc[4 * j + 0] = fmaf(r, v.x, acc[4 * j + 0]);
    acc[4 * j + 1] = fmaf(r, v.y, acc[4 * j + 1]);
    acc[4 * j + 2] = fmaf(r, v.z, acc[4 * j + 2]);
    acc[4 * j + 3] = fmaf(r, v.w, acc[4 * j + 3]);
  }
}

// acc += sum over this lane's CSC entries i = beg, beg + STRIDE, ... of r_i * E[doc_i].
// Four entries are in flight per lane (index loads, then the r / E-row gathers,
// then the FMAs): the gather chain is latency-bound, not bandwidth-bound.
template <int KS, int STRIDE>
__device__ __forceinline__ void gather_axpy(const SuffArgs& a, int i, int end, float (&acc)[KS]) {
  constexpr int U = KS <= 32 ? 4 : (KS <= 64 ? 2 : 1);   // registers: U rows of KS in flight
  for (; i + (U - 1) * STRIDE < end; i += U * STRIDE) {
    int d[U], ent[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      d[u] = a.csc_doc[i + u * STRIDE];
      ent[u] = a.csc_ent[i + u * STRIDE];
    }
    float r[U];
    float4 v[U][KS / 4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      r[u] = a.r[ent[u]];
      const float4* p = reinterpret_cast<const float4*>(a.e + (size_t)d[u] * KS);
#pragma unroll
      for (int j = 0; j < KS / 4; ++j) v[u][j] = p[j];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int j = 0; j < KS / 4; ++j) {
        acc[4 * j + 0] = fmaf(r[u], v[u][j].x, acc[4 * j + 0]);
        acc[4 * j + 1] = fmaf(r[u], v[u][j].y, acc[4 * j + 1]);
        acc[4 * j + 2] = fmaf(r[u], v[u][j].z, acc[4 * j + 2]);
        acc[4 * j + 3] = fmaf(r[u], v[u][j].w, acc[4 * j + 3]);
      }
    }
  }
  for (; i < end; i += STRIDE) axpy_row<KS>(a.e, a.csc_doc[i], a.r[a.csc_ent[i]], acc);
}

template <int KS>
__device__ __forceinline__ void store_cw(const SuffArgs& a, int w, const float (&acc)[KS]) {
  const float4* b = reinterpret_cast<const float4*>(a.beta + (size_t)w * KS);
  float4* o = reinterpret_cast<float4*>(a.cw + (size_t)w * KS);
#pragma unroll
  for (int j = 0; j < KS / 4; ++j) {
    float4 bv = b[j];
    o[j] = make_float4(bv.x * acc[4 * j + 0], bv.y * acc[4 * j + 1], bv.z * acc[4 * j + 2],
                       bv.w * acc[4 * j + 3]);
  }
}

template <int KS, int G>
__global__ __launch_bounds__(256) void lda_suff_group(SuffArgs a) {
  constexpr int GPB = 256 / G;
  const int t = threadIdx.x % G;
  const int item = blockIdx.x * GPB + threadIdx.x / G;
  if (item >= a.n_items || gated(a.gate)) return;
  const int w = a.order[item];
  const int beg = a.word_ptr[w], end = a.word_ptr[w + 1];
  float acc[KS];
#pragma unroll
  for (int k = 0; k < KS; ++k) acc[k] = 0.f;
  gather_axpy<KS, G>(a, beg + t, end, acc);
  group_sum_vec<G, KS>(acc);
  if (t == 0) store_cw<KS>(a, w, acc);
}

template <int KS, int NW>
__global__ __launch_bounds__(NW * 64) void lda_suff_block(SuffArgs a) {
  __shared__ float sRed[NW][KS];
  if (gated(a.gate)) return;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int w = a.order[blockIdx.x];
  const int beg = a.word_ptr[w], end = a.word_ptr[w + 1];
  float acc[KS];
#pragma unroll
  for (int k = 0; k < KS; ++k) acc[k] = 0.f;
  gather_axpy<KS, NW * 64>(a, beg + t, end, acc);
  group_sum_vec<64, KS>(acc);
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < KS; ++k) sRed[wv][k] = acc[k];
  }
  __syncthreads();
  if (t < KS) {
    float s = 0.f;
#pragma unroll
    for (int v = 0; v < NW; ++v) s += sRed[v][t];
    a.cw[(size_t)w * KS + t] = a.beta[(size_t)w * KS + t] * s;
  }
}

// One launch for all words (heavy words first), 256 threads per workgroup:
//   heavy  (> 1024 entries): one word per workgroup, 4 waves, cross-wave LDS sum
//   medium (65..1024):       one word per wave
//   light  (<= 64, empty):   one word per 16 lanes
// Each workgroup also writes the column sums of the class_word rows it produced
// (in double, fixed group order) to part[blockIdx.x][0..KS), so the per-topic
// totals need only a small second pass over the partials (colsum_partials)
// instead of a re-read of the whole [V][KS] matrix.
// Columns 0 / 1 of this workgroup's partial row (layout off == 2): its slice of the
// per-document likelihood and alpha_ss sums (wave 0; fixed order, so colsum_partials
// gives bitwise the same totals every run).  Called by every thread before any barrier.
__device__ __forceinline__ void scalar_slice(const SuffPartLayout& L, double* row) {
  if (L.off != 2 || threadIdx.x >= 64) return;
  const int t = threadIdx.x;
  double x = 0.0, y = 0.0;
  if (L.lik) {
    const int n = L.hi - L.lo, nb = (int)gridDim.x;
    const int per = (n + nb - 1) / nb;
    const int i0 = L.lo + (int)blockIdx.x * per, i1 = min(L.hi, i0 + per);
    for (int i = i0 + t; i < i1; i += 64) {
      x += L.lik[i];
      y += L.ass[i];
    }
  }
  x = group_sum<64>(x);
  y = group_sum<64>(y);
  if (t == 0) {
    row[0] = x;
    row[1] = y;
  }
}

template <int KS>
__global__ __launch_bounds__(256) void lda_suff_fused(SuffArgs a, int n_heavy, int n_medium, int n_light,
                                                      double* __restrict__ part, SuffPartLayout lay) {
  __shared__ float sRow[16][KS];
  if (gated(a.gate)) return;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  scalar_slice(lay, part + (size_t)blockIdx.x * lay.stride);
  part += lay.off;
  const int nbM = (n_medium + 3) / 4;
  const int b = blockIdx.x;
  float acc[KS];
#pragma unroll
  for (int k = 0; k < KS; ++k) acc[k] = 0.f;
  int ngroups;
  if (b < n_heavy) {
    const int w = a.order[b];
    gather_axpy<KS, 256>(a, a.word_ptr[w] + t, a.word_ptr[w + 1], acc);
    group_sum_vec<64, KS>(acc);
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < KS; ++k) sRow[wv][k] = acc[k];
    }
    __syncthreads();
    if (t < KS) {
      float s = 0.f;
#pragma unroll
      for (int v = 0; v < 4; ++v) s += sRow[v][t];
      const float c = a.beta[(size_t)w * KS + t] * s;
      a.cw[(size_t)w * KS + t] = c;
      part[(size_t)b * lay.stride + t] = (double)c;
    }
    return;
  } else if (b < n_heavy + nbM) {
    const int item = (b - n_heavy) * 4 + wv;
    const bool valid = item < n_medium;
    const int w = valid ? a.order[n_heavy + item] : 0;
    if (valid) gather_axpy<KS, 64>(a, a.word_ptr[w] + lane, a.word_ptr[w + 1], acc);
    group_sum_vec<64, KS>(acc);
    if (lane == 0) {
      if (valid) store_cw<KS>(a, w, acc);
      const float* bw = a.beta + (size_t)w * KS;
#pragma unroll
      for (int k = 0; k < KS; ++k) sRow[wv][k] = valid ? bw[k] * acc[k] : 0.f;
    }
    ngroups = 4;
  } else {
    const int g = t >> 4, q = t & 15;
    const int item = (b - n_heavy - nbM) * 16 + g;
    const bool valid = item < n_light;
    const int w = valid ? a.order[n_heavy + n_medium + item] : 0;
    if (valid) gather_axpy<KS, 16>(a, a.word_ptr[w] + q, a.word_ptr[w + 1], acc);
    group_sum_vec<16, KS>(acc);
    if (q == 0) {
      if (valid) store_cw<KS>(a, w, acc);
      const float* bw = a.beta + (size_t)w * KS;
#pragma unroll
      for (int k = 0; k < KS; ++k) sRow[g][k] = valid ? bw[k] * acc[k] : 0.f;
    }
    ngroups = 16;
  }
  __syncthreads();
  if (t < KS) {
    double s = 0.0;
    for (int g = 0; g < ngroups; ++g) s += (double)sRow[g][t];
    part[(size_t)b * lay.stride + t] = s;
  }
}

// Wide-topic variant (K > 32) of lda_suff_fused: a CSC entry's KS topics are split
// over TG lanes (E-row chunk c on lane c mod TG, as in lda_estep_wide.hip), so a
// lane holds ceil(KS/4/TG) float4 accumulators instead of KS floats and the
// kernel runs at 3-4 waves per SIMD instead of spilling at one.  Same group
// shapes as lda_suff_fused (heavy: one word per workgroup; medium: per wave;
// light: per 16 lanes), S = G/TG entry slots per word.  The slot partials meet in
// LDS and are added in slot order (bitwise reproducible); the word's row is then
// scaled by beta and written with the per-workgroup column sums.
template <int KS, int TG>
__global__ __launch_bounds__(256) void lda_suff_wide(SuffArgs a, int n_heavy, int n_medium, int n_light,
                                                     double* __restrict__ part, SuffPartLayout lay) {
  constexpr int C = KS / 4;
  constexpr int CPL = (C + TG - 1) / TG;
  constexpr int NSLOT = 256 / TG;
  constexpr int U = 4;   // entries in flight per lane
  __shared__ float4 sAcc4[NSLOT][C];
  __shared__ float sRow[16][KS];
  if (gated(a.gate)) return;
  scalar_slice(lay, part + (size_t)blockIdx.x * lay.stride);
  part += lay.off;
  const int t = threadIdx.x;
  const int b = blockIdx.x;
  const int nbM = (n_medium + 3) / 4;
  int G, item, nitems, base;
  if (b < n_heavy) {
    G = 256, item = b, nitems = n_heavy, base = 0;
  } else if (b < n_heavy + nbM) {
    G = 64, item = (b - n_heavy) * 4 + t / 64, nitems = n_medium, base = n_heavy;
  } else {
    G = 16, item = (b - n_heavy - nbM) * 16 + t / 16, nitems = n_light, base = n_heavy + n_medium;
  }
  const int S = G / TG;
  const int gi = t / G;                      // word group of this thread within the block
  const int s = (t % G) / TG, q = t % TG;
  const bool valid = item < nitems;
  const int w = valid ? a.order[base + item] : 0;
  float4 acc[CPL];
#pragma unroll
  for (int j = 0; j < CPL; ++j) acc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (valid) {
    int i = a.word_ptr[w] + s;
    const int end = a.word_ptr[w + 1];
    for (; i + (U - 1) * S < end; i += U * S) {
      int d[U];
      float r[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        d[u] = a.csc_doc[i + u * S];
        r[u] = a.r[a.csc_ent[i + u * S]];
      }
      float4 v[U][CPL];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float4* p = reinterpret_cast<const float4*>(a.e + (size_t)d[u] * KS);
#pragma unroll
        for (int j = 0; j < CPL; ++j) v[u][j] = (q + TG * j < C) ? p[q + TG * j] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int j = 0; j < CPL; ++j) {
          acc[j].x = fmaf(r[u], v[u][j].x, acc[j].x);
          acc[j].y = fmaf(r[u], v[u][j].y, acc[j].y);
          acc[j].z = fmaf(r[u], v[u][j].z, acc[j].z);
          acc[j].w = fmaf(r[u], v[u][j].w, acc[j].w);
        }
      }
    }
    for (; i < end; i += S) {
      const float r = a.r[a.csc_ent[i]];
      const float4* p = reinterpret_cast<const float4*>(a.e + (size_t)a.csc_doc[i] * KS);
#pragma unroll
      for (int j = 0; j < CPL; ++j) {
        if (q + TG * j < C) {
          const float4 v = p[q + TG * j];
          acc[j].x = fmaf(r, v.x, acc[j].x);
          acc[j].y = fmaf(r, v.y, acc[j].y);
          acc[j].z = fmaf(r, v.z, acc[j].z);
          acc[j].w = fmaf(r, v.w, acc[j].w);
        }
      }
    }
  }
  // slot partials -> LDS (global slot index t / TG)
#pragma unroll
  for (int j = 0; j < CPL; ++j)
    if (q + TG * j < C) sAcc4[t / TG][q + TG * j] = acc[j];
  __syncthreads();
  const float* sAcc = reinterpret_cast<const float*>(&sAcc4[0][0]);
  const int ngroups = 256 / G;
  for (int idx = t; idx < ngroups * KS; idx += 256) {
    const int g = idx / KS, k = idx % KS;
    const int it = (G == 256 ? item : item - gi + g);   // the item of word group g
    float v = 0.f;
    for (int u = 0; u < S; ++u) v += sAcc[(g * S + u) * KS + k];
    float c = 0.f;
    if (it < nitems) {
      const int wg = a.order[base + it];
      c = a.beta[(size_t)wg * KS + k] * v;
      a.cw[(size_t)wg * KS + k] = c;
    }
    sRow[g][k] = c;
  }
  __syncthreads();
  if (t < KS) {
    double sum = 0.0;
    for (int g = 0; g < ngroups; ++g) sum += (double)sRow[g][t];
    part[(size_t)b * lay.stride + t] = sum;
  }
}

int suff_fused_blocks(int n_heavy, int n_medium, int n_light) {
  return n_heavy + (n_medium + 3) / 4 + (n_light + 15) / 16;
}

template <int KS>
static void suff_fused_ks(const SuffArgs& a, int n_heavy, int n_medium, int n_light, double* part, bool wide,
                          const SuffPartLayout& lay, hipStream_t s) {
  const int nb = suff_fused_blocks(n_heavy, n_medium, n_light);
  if (nb <= 0) return;
  if (wide) {
    if constexpr (KS >= 32) {
      hipLaunchKernelGGL((lda_suff_wide<KS, (KS >= 100 ? 8 : 4)>), dim3(nb), dim3(256), 0, s, a, n_heavy, n_medium,
                         n_light, part, lay);
      ONI_HIP_CHECK(hipGetLastError());
      return;
    } else {
      throw std::runtime_error("lda_suffstats_fused: wide layout needs KS >= 32");
    }
  }
  hipLaunchKernelGGL((lda_suff_fused<KS>), dim3(nb), dim3(256), 0, s, a, n_heavy, n_medium, n_light, part, lay);
  ONI_HIP_CHECK(hipGetLastError());
}

void launch_lda_suffstats_fused(const SuffArgs& a, int n_heavy, int n_medium, int n_light, double* part, int KS,
                                bool wide, const SuffPartLayout& lay, hipStream_t s) {
  if (!((lay.off == 0 && lay.stride == KS) || (lay.off == 2 && lay.stride == KS + 2)))
    throw std::runtime_error("lda_suffstats_fused: partial layout must be [KS] or [2 + KS]");
  switch (KS) {
#define ONI_KS(X) \
  case X:         \
    suff_fused_ks<X>(a, n_heavy, n_medium, n_light, part, wide, lay, s); \
    break;
    ONI_FOR_EACH_KS(ONI_KS)
#undef ONI_KS
    default:
      throw std::runtime_error("lda_suffstats_fused: unsupported KS " + std::to_string(KS));
  }
}

template <int KS>
static void suff_ks(const SuffArgs& a, int variant, hipStream_t s) {
  if (a.n_items <= 0) return;
  switch (variant) {
    case kSuffG16:
      hipLaunchKernelGGL((lda_suff_group<KS, 16>), dim3((a.n_items + 15) / 16), dim3(256), 0, s, a);
      break;
    case kSuffG64:
      hipLaunchKernelGGL((lda_suff_group<KS, 64>), dim3((a.n_items + 3) / 4), dim3(256), 0, s, a);
      break;
    case kSuffB8:
      hipLaunchKernelGGL((lda_suff_block<KS, 8>), dim3(a.n_items), dim3(512), 0, s, a);
      break;
    default:
      throw std::runtime_error("lda_suffstats: unknown variant");
  }
  ONI_HIP_CHECK(hipGetLastError());
}

void launch_lda_suffstats(const SuffArgs& a, int variant, int KS, hipStream_t s) {
  switch (KS) {
#define ONI_KS(X) \
  case X:         \
    suff_ks<X>(a, variant, s); \
    break;
    ONI_FOR_EACH_KS(ONI_KS)
#undef ONI_KS
    default:
      throw std::runtime_error("lda_suffstats: unsupported KS " + std::to_string(KS));
  }
}

// ----------------------------------------------------------------- M-step ---
// lda-c lda_mle: log p(w|z) = log cw - log ct, floor -100 where
// cw == 0.  The E-step consumes exp(log p) directly, so this writes
// beta = cw / ct (exact division) or exp(-100).
__global__ __launch_bounds__(256) void lda_mstep_kernel(const float* __restrict__ cw,
                                                        const double* __restrict__ ct,
                                                        float* __restrict__ beta, int V, int K, int KS,
                                                        const double* gate) {
  if (gated(gate)) return;
  const int64_t total = (int64_t)V * KS;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(i % KS);
    float out = 0.f;
    if (k < K) {
      const float c = cw[i];
      out = c > 0.f ? (float)((double)c / ct[k]) : kExpMinus100;
    }
    beta[i] = out;
  }
}

// rows != nullptr: only those word rows (a rank's own words under the sparse class_word
// exchange -- the other rows of beta are never read on that rank).
__global__ __launch_bounds__(256) void lda_mstep_control_kernel(const float* __restrict__ cw,
                                                                const double* __restrict__ ct,
                                                                float* __restrict__ beta, int V, int K, int KS,
                                                                const int* __restrict__ rows, int n_rows,
                                                                EMControlArgs c, NewtonArgs nw) {
  if (c.params[kParamDone] != 0.0) return;
  // alpha Newton (lanes 0-1 of workgroup 0) beside the other workgroups' beta rows; its
  // agent-scope stores drain before this workgroup's completion count below
  if (nw.enabled && blockIdx.x == 0 && threadIdx.x < 64) {
    if (threadIdx.x < 2)
      alpha_newton_lanes(c.scalars, nw.num_docs, K, nw.estimate, c.params, nw.alpha_out, threadIdx.x);
    __builtin_amdgcn_s_waitcnt(0);
  }
  // float4 granules of the word-major [V][KS] matrices (KS % 4 == 0)
  const int q = KS / 4;
  const int total4 = (rows ? n_rows : V) * q;
  const float4* cw4 = reinterpret_cast<const float4*>(cw);
  float4* beta4 = reinterpret_cast<float4*>(beta);
  for (int g = blockIdx.x * blockDim.x + threadIdx.x; g < total4; g += gridDim.x * blockDim.x) {
    const int k0 = (g % q) * 4;
    const int i = rows ? rows[g / q] * q + g % q : g;
    const float4 v = cw4[i];
    float o[4];
    const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = k0 + j;
      o[j] = k < K ? (vv[j] > 0.f ? (float)((double)vv[j] / ct[k]) : kExpMinus100) : 0.f;
    }
    beta4[i] = make_float4(o[0], o[1], o[2], o[3]);
  }
  // Relaxed is enough: the control step reads what earlier kernels wrote (scalars, params,
  // ctl) plus this launch's alpha, which it loads at agent scope after the count has
  // seen workgroup 0 (whose write-through stores drained before its add).
  // (An acq_rel agent-scope RMW per workgroup costs an L2 writeback + invalidate each.)
  __syncthreads();
  if (threadIdx.x == 0) {
    if (__hip_atomic_fetch_add(c.done_count, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1) {
      __hip_atomic_store(c.done_count, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const double alpha_now = __hip_atomic_load(c.params, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      em_control_step(c.scalars, c.params, c.ctl, c.hist, c.hist_slots, alpha_now);
    }
  }
}

void launch_lda_mstep_control(const float* cw, const double* class_total, float* beta, int V, int K, int KS,
                              const int* rows, int n_rows, const EMControlArgs& c, const NewtonArgs& nw,
                              hipStream_t s) {
  const int64_t total = (int64_t)(rows ? n_rows : V) * KS;
  // 2 workgroups per CU: the completion count is a same-address atomic per workgroup
  int64_t blocks = (total / 4 + 255) / 256;
  if (blocks > 512) blocks = 512;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(lda_mstep_control_kernel, dim3((unsigned)blocks), dim3(256), 0, s, cw, class_total, beta, V,
                     K, KS, rows, n_rows, c, nw);
  ONI_HIP_CHECK(hipGetLastError());
}

__global__ void alpha_newton_kernel(const double* __restrict__ scalars, double num_docs, int K, int estimate,
                                    double* __restrict__ params, double* __restrict__ alpha_out) {
  const int lane = threadIdx.x;
  if (blockIdx.x != 0 || lane >= 2 || params[kParamDone] != 0.0) return;
  alpha_newton_lanes(scalars, num_docs, K, estimate, params, alpha_out, lane);
}

void launch_alpha_newton(const double* scalars, double num_docs, int K, bool estimate, double* params,
                         double* alpha_out, hipStream_t s) {
  hipLaunchKernelGGL(alpha_newton_kernel, dim3(1), dim3(64), 0, s, scalars, num_docs, K, estimate ? 1 : 0, params,
                     alpha_out);
  ONI_HIP_CHECK(hipGetLastError());
}

void launch_lda_mstep(const float* cw, const double* class_total, float* beta, int V, int K, int KS,
                      const double* gate, hipStream_t s) {
  const int64_t total = (int64_t)V * KS;
  if (total == 0) return;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(lda_mstep_kernel, dim3((unsigned)blocks), dim3(256), 0, s, cw, class_total, beta, V,
                     K, KS, gate);
  ONI_HIP_CHECK(hipGetLastError());
}

}  // namespace oni
