// Split-document E-step: one huge document over several workgroups
// (the sequence-/context-parallel analogue of SURVEY.md §5.7(a)).
//
// A document with N >> 1024 distinct words (NAT gateways, resolvers, busy
// servers: the heavy tail of IP "documents") would serialise its whole
// variational loop on one workgroup.  Here it is cut into `nseg` segments of
// `seg_words` words; workgroup s keeps its segment's beta rows in VGPRs for all
// variational iterations and every iteration
//
//   1. computes E from its (replicated) topic state,
//   2. reduces its segment's sum_n (c_n/P_n) beta_n  and  sum_n c_n log P_n
//      over its waves (LDS),
//   3. publishes them as iteration-tagged 8-byte granules {value, tag} to
//      xchg[it & 1][block] (relaxed agent-scope 64-bit stores: single-copy
//      atomic, so a reader that sees the tag sees the value),
//   4. polls the nseg segments' granules of this iteration directly (8 loads in
//      flight, s_sleep between rounds, bounded: a timeout sets `error`) and sums
//      them in segment order -- identical bits in every workgroup --
//   5. runs the same deterministic topic update, so all segments agree on gamma
//      and on the convergence decision without a second barrier.
// One write + the polling reads per iteration: no arrival counter and no wait for
// store completion (a counter-based barrier costs about two more fabric round
// trips per iteration -- the split chain is the E-step's critical path).
// Parity double-buffering makes one exchange per iteration sufficient: a
// workgroup can only overwrite buffer (it & 1) again at iteration it + 2, after
// every segment has read iteration it.  The tag holds the document's launch
// epoch, bumped by its last segment on exit, so granules of an earlier launch
// never match.  The launch is capped at kSplitMaxBlocks workgroups (one per CU),
// so all segments are co-resident and the exchange cannot deadlock.
#include <stdexcept>
#include <string>

#include "common.h"
#include "estep_common.h"
#include "kernels.h"

namespace oni {

namespace {

constexpr int kNW = 8;      // 8 waves x rows_per_lane_8w rows: 4096 words per segment at K <= 20
constexpr int kNT = kNW * 64;

}  // namespace

template <int KS, int CW>
__global__ __launch_bounds__(kNT) void lda_estep_split(EStepArgs a, SplitArgs s) {
  if (load_params(a)) return;
  __builtin_amdgcn_s_setprio(3);   // the longest serial chain of the EM step
  constexpr int TJ = (KS + 63) / 64;
  __shared__ float4 sE4[KS / 4];
  __shared__ float sRed[kNW][KS];
  __shared__ double sRedD[kNW];
  __shared__ int sFlag;

  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int b = blockIdx.x;
  const int d = s.seg_doc[b];
  const int seg = s.seg_index[b];
  const int nseg = s.seg_count[b];
  const int base = s.seg_base[b];
  int* counter = s.counter + s.doc_slot[b];
  const int epoch = __hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int dbeg = a.doc_ptr[d];
  const int Ndoc = a.doc_ptr[d + 1] - dbeg;
  const int beg = dbeg + seg * s.seg_words;
  const int N = min(s.seg_words, Ndoc - seg * s.seg_words);
  const int K = a.K;
  const float alpha = a.alpha;
  float* sE = reinterpret_cast<float*>(&sE4[0]);

  // ---- this workgroup's words in registers (seg_words <= kNT * CW) ----
  float bc[CW][KS];
  float cc[CW];
#pragma unroll
  for (int c = 0; c < CW; ++c) {
    const int n = t + kNT * c;
    if (n < N) {
      cc[c] = a.counts[beg + n];
      load_row<KS>(a.beta, a.word_idx[beg + n], bc[c]);
    } else {
      cc[c] = 0.f;
#pragma unroll
      for (int k = 0; k < KS; ++k) bc[c][k] = 0.f;
    }
  }
  // document total (every workgroup reads the whole doc's counts: O(N) once)
  double tot_l = 0.0;
  for (int n = t; n < Ndoc; n += kNT) tot_l += a.counts[dbeg + n];
  tot_l = group_sum<64>(tot_l);
  if (lane == 0) sRedD[wv] = tot_l;
  __syncthreads();
  double total = 0.0;
#pragma unroll
  for (int w = 0; w < kNW; ++w) total += sRedD[w];
  __syncthreads();

  float gam[TJ], psi[TJ], e[TJ];
  const float g0 = alpha + (float)(total / K);
  double lik_old = 0.0, L = 0.0, dsum_last = 0.0;
  float m = 0.f;
  int it = 0;
  const bool unbounded = a.var_max_iter < 0;
  if (wv == 0) {
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int k = lane + 64 * j;
      gam[j] = (k < K) ? g0 : 0.f;
      psi[j] = (k < K) ? digammaf_ldac(g0) : -INFINITY;
    }
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < TJ; ++j) mx = fmaxf(mx, psi[j]);
    m = group_max<64>(mx);
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int k = lane + 64 * j;
      e[j] = (k < K) ? __expf(psi[j] - m) : 0.f;
      if (k < KS) sE[k] = e[j];
    }
    float sg = 0.f;
#pragma unroll
    for (int j = 0; j < TJ; ++j) sg += gam[j];
    dsum_last = digammaf_ldac(group_sum<64>(sg));
    if (lane == 0) sFlag = (unbounded || a.var_max_iter > 0) ? 1 : 0;
  }
  __syncthreads();

  // optional phase timer (scripts/estep_phases.py): thread 0 of workgroup 0
  const bool timed = a.dbg != nullptr && b == 0 && t == 0;
  long long tm[6] = {0, 0, 0, 0, 0, 0}, t0 = 0;
  auto lap = [&](int i) {
    if (timed) {
      const long long t1 = clock64();
      tm[i] += t1 - t0;
      t0 = t1;
    }
  };
  if (timed) t0 = clock64();

  while (sFlag) {
    // ---- word pass over this segment ----
    float acc[KS];
#pragma unroll
    for (int k = 0; k < KS; ++k) acc[k] = 0.f;
    float lsum = 0.f;
#pragma unroll
    for (int c = 0; c < CW; ++c) {
      if (t + kNT * c < N) {
        const float P = fmaxf(dot_lds<KS>(sE, bc[c]), kPMin);
        const float r = rdiv(cc[c], P);
        lsum = fmaf(cc[c], log_normal(P), lsum);
#pragma unroll
        for (int k = 0; k < KS; ++k) acc[k] = fmaf(r, bc[c][k], acc[k]);
      }
    }
    lap(0);
    wave_sum_last_vec<KS>(acc);   // totals in lane 63
    const double lsum_w = wave_sum_last((double)lsum);
    if (lane == 63) {
#pragma unroll
      for (int k = 0; k < KS; ++k) sRed[wv][k] = acc[k];
      sRedD[wv] = lsum_w;
    }
    __syncthreads();
    lap(1);

    if (wv == 0) {
      ++it;
      const int par = it & 1;
      const unsigned tag = split_tag(epoch, it);
      constexpr int GR = KS + 2;
      // publish this segment's partials, then gather every segment's (in segment order)
      float part[TJ];
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int k = lane + 64 * j;
        float v = 0.f;
        if (k < KS) {
#pragma unroll
          for (int w = 0; w < kNW; ++w) v += sRed[w][k];
        }
        part[j] = v;
      }
      double lpart = 0.0;
#pragma unroll
      for (int w = 0; w < kNW; ++w) lpart += sRedD[w];
      unsigned long long* xb = s.xchg + (size_t)par * s.n_blocks * GR;
      publish_tagged<KS>(xb + (size_t)b * GR, [&](int j) { return part[j]; }, lpart, lane, tag);
      lap(2);
      float ak[TJ];
      double lsum_d;
      bool ok = tagged_gather<KS>(xb + (size_t)base * GR, nseg, GR, tag, lane, ak, lsum_d);
      lap(3);
      float gn[TJ];
      float sg = 0.f;
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        gn[j] = (lane + 64 * j < K) ? fmaf(e[j], ak[j], alpha) : 0.f;
        sg += gn[j];
      }
      ok = __all(ok);
      if (!ok && lane == 0) __hip_atomic_store(s.error, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // sum_k [lnG(g'_k) - (g'_k - a) psi(g_k)] + psi(S') (S' - K a): independent of psi(S');
      // KS <= 32: every topic in the low half-wave, 32-lane reductions
      constexpr int GL = KS <= 32 ? 32 : 64;
      double partl = 0.0;
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int k = lane + 64 * j;
        if (k < K) {
          float pn, lg;
          digamma_lgamma(gn[j], pn, lg);
          partl += (double)lg - (double)(gn[j] - alpha) * (double)psi[j];
          psi[j] = pn;
          gam[j] = gn[j];
        }
      }
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < TJ; ++j) mx = fmaxf(mx, psi[j]);
      const float S = group_sum<GL>(sg);
      const double termp = group_sum<GL>(partl);
      const float m_new = group_max<GL>(mx);   // next E beside the likelihood chain
      float e_new[TJ];
#pragma unroll
      for (int j = 0; j < TJ; ++j) e_new[j] = (lane + 64 * j < K) ? __expf(psi[j] - m_new) : 0.f;
      float dS, lgS;
      digamma_lgamma(S, dS, lgS);
      const double term = termp + (double)dS * ((double)S - (double)K * (double)alpha);
      L = a.lik_const - (double)lgS + term + (lsum_d + (double)m * total) - total * (double)dS;
      const bool more = var_more(lik_old, L, (double)a.var_conv);
      lik_old = L;
      dsum_last = dS;
      const bool cont = ok && more && (unbounded || it < a.var_max_iter);
      if (cont) {
        m = m_new;
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          const int k = lane + 64 * j;
          e[j] = e_new[j];
          if (k < KS) sE[k] = e[j];
        }
      }
      if (lane == 0) sFlag = cont ? 1 : 0;
      lap(4);
    }
    __syncthreads();
    lap(5);
  }
  if (timed) {
#pragma unroll
    for (int i = 0; i < 6; ++i) a.dbg[i] = tm[i];
    a.dbg[6] = it;
    a.dbg[7] = nseg;
  }

  // Every wave of this workgroup has passed its last exchange (the loop ends on a __syncthreads).
  split_exit(counter, s.n_docs, nseg);
  const bool failed = __hip_atomic_load(s.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;

  // ---- outputs: r for this segment; the document state from segment 0 ----
#pragma unroll
  for (int c = 0; c < CW; ++c) {
    const int n = t + kNT * c;
    if (n < N) a.r_out[beg + n] = rdiv(cc[c], fmaxf(dot_lds<KS>(sE, bc[c]), kPMin));
  }
  if (wv == 0 && seg == 0) {
    double ass = 0.0;
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int k = lane + 64 * j;
      if (k < KS) {
        a.gamma[(size_t)d * KS + k] = gam[j];
        a.e_out[(size_t)d * KS + k] = sE[k];
      }
      if (k < K) ass += (double)psi[j];
    }
    ass = group_sum<64>(ass);
    if (lane == 0) {
      a.lik[d] = failed ? __builtin_nan("") : L;   // a timed-out barrier surfaces as a NaN likelihood
      a.alpha_ss[d] = ass - (double)K * dsum_last;
      a.iters[d] = it;
    }
  }
}

template <int KS>
static void split_ks(const EStepArgs& a, const SplitArgs& s, hipStream_t st) {
  constexpr int CW = rows_per_lane_8w(KS);
  if (s.n_blocks <= 0) return;
  if (s.n_blocks > kSplitMaxBlocks) throw std::runtime_error("lda_estep_split: too many workgroups in one launch");
  if (s.seg_words > kNT * CW) throw std::runtime_error("lda_estep_split: segment larger than the register cache");
  hipLaunchKernelGGL((lda_estep_split<KS, CW>), dim3(s.n_blocks), dim3(kNT), 0, st, a, s);
  ONI_HIP_CHECK(hipGetLastError());
}

int split_segment_words(int KS) { return kNT * rows_per_lane_8w(KS); }

// Workgroups of the split kernel the device can hold at once (occupancy API x CU count).
template <int KS>
static int split_capacity_ks() {
  int dev = 0, per_cu = 0;
  hipDeviceProp_t p;
  ONI_HIP_CHECK(hipGetDevice(&dev));
  ONI_HIP_CHECK(hipGetDeviceProperties(&p, dev));
  ONI_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
      &per_cu, reinterpret_cast<const void*>(&lda_estep_split<KS, rows_per_lane_8w(KS)>), kNT, 0));
  return per_cu * p.multiProcessorCount;
}

int split_capacity(int KS) {
  switch (KS) {
#define ONI_KS(X) \
  case X:         \
    return split_capacity_ks<X>();
    ONI_FOR_EACH_KS(ONI_KS)
#undef ONI_KS
    default:
      throw std::runtime_error("split_capacity: unsupported KS " + std::to_string(KS));
  }
}
int block_words(int KS, int waves) { return waves * 64 * (waves == 8 ? rows_per_lane_8w(KS) : rows_per_lane_4w(KS)); }

void launch_lda_estep_split(const EStepArgs& a, const SplitArgs& s, int KS, hipStream_t st) {
  switch (KS) {
#define ONI_KS(X) \
  case X:         \
    split_ks<X>(a, s, st); \
    break;
    ONI_FOR_EACH_KS(ONI_KS)
#undef ONI_KS
    default:
      throw std::runtime_error("lda_estep_split: unsupported KS " + std::to_string(KS));
  }
}

}  // namespace oni
