// Fused variational E-step for LDA on CDNA4 (gfx950).
//
// Reference semantics: oni-lda-c `lda_inference` + `compute_likelihood`
// (call site /root/reference/ml_ops.sh:80).  lda-c updates
// gamma after every word (Gauss-Seidel, K digammas per word).  Here the doc is
// updated in Jacobi form, which has the same fixed point:
//
//   E_k      = exp(psi(gamma_k) - m)               (m = max_k psi, scale-free)
//   P_n      = sum_k E_k * beta[w_n][k]            (phinorm, scaled by e^-m)
//   gamma'_k = alpha + E_k * sum_n (c_n / P_n) beta[w_n][k]
//
// and the per-doc likelihood is evaluated in closed form (no per-(n,k) log):
//
//   L = lnG(K a) - K lnG(a) - lnG(S') + sum_k [(a-1)Y_k + lnG(g'_k) - (g'_k-1)Y_k
//       + (g'_k - a)(psi(g'_k) - psi(g_k))] + sum_n c_n (ln P_n + m) - T psi(S')
//   Y_k = psi(g'_k) - psi(S'),  S' = sum_k g'_k,  T = sum_n c_n
//
// which equals lda-c's compute_likelihood(phi(g), g') exactly in exact arithmetic.
// Convergence follows lda-c: iterate while (L_old - L)/L_old > var_conv and
// it < var_max_iter (-1 = unbounded), L_old starting at 0.
//
// Work decomposition (length-bucketed):
//   lda_estep_group<KS,G,CW>: G lanes (16/32/64) per document, 256/G docs per
//     block; lanes stride over words; the doc's first CW*G beta rows stay in
//     VGPRs across all variational iterations; per-topic transcendentals are
//     spread over lanes (topic k on lane k mod G); E is broadcast through LDS.
//   lda_estep_block<KS,NW,CW>: one long document per NW-wave workgroup (the
//     "long-context" analogue): words striped over NW*64 lanes, cross-wave
//     sums through LDS, wave 0 owns the per-topic state.
// Outputs per doc: gamma, the E vector of the final phi, r_n = c_n/P_n (so the
// sufficient statistics can be formed deterministically in lda_suffstats),
// likelihood, alpha sufficient statistic and the variational iteration count.
#include <stdexcept>
#include <string>

#include "common.h"
#include "estep_common.h"
#include "kernels.h"

namespace oni {


// ---------------------------------------------------------------------------
// Group kernel: G lanes per document.
// ---------------------------------------------------------------------------
template <int KS, int G, int CW>
__global__ __launch_bounds__(256) void lda_estep_group(EStepArgs a) {
  if (load_params(a)) return;
  constexpr int GPB = 256 / G;
  constexpr int TJ = (KS + G - 1) / G;
  __shared__ float4 sE4[GPB][KS / 4];
  __shared__ float sAcc[G == 64 ? GPB : 1][G == 64 ? KS : 1];   // one-wave documents: lane 63 -> topic lanes

  const int t = threadIdx.x % G;
  const int g = threadIdx.x / G;
  const int item = blockIdx.x * GPB + g;
  if (item >= a.n_items) return;  // group-uniform exit
  float* sE = reinterpret_cast<float*>(&sE4[g][0]);

  const int d = a.order[item];
  const int beg = a.doc_ptr[d];
  const int N = a.doc_ptr[d + 1] - beg;
  const int K = a.K;
  const float alpha = a.alpha;

  // ---- stage this lane's first CW words in registers ----
  float bc[CW][KS];
  float cc[CW];
  double tot_l = 0.0;
#pragma unroll
  for (int c = 0; c < CW; ++c) {
    const int n = t + G * c;
    if (n < N) {
      const int w = a.word_idx[beg + n];
      cc[c] = a.counts[beg + n];
      load_row<KS>(a.beta, w, bc[c]);
    } else {
      cc[c] = 0.f;
#pragma unroll
      for (int k = 0; k < KS; ++k) bc[c][k] = 0.f;
    }
    tot_l += cc[c];
  }
  for (int n = t + G * CW; n < N; n += G) tot_l += a.counts[beg + n];
  const double total = group_sum<G>(tot_l);
  const float totalf = (float)total;

  // ---- per-topic state (topic k = t + G*j) ----
  float gam[TJ], psi[TJ], e[TJ];
  const float g0 = alpha + (float)(total / K);
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int k = t + G * j;
    gam[j] = (k < K) ? g0 : 0.f;
    psi[j] = (k < K) ? digammaf_ldac(g0) : -INFINITY;
    e[j] = 0.f;
  }

  double lik_old = 0.0, L = 0.0, dsum_last = 0.0;
  bool more = 1.0 > (double)a.var_conv;   // lda-c starts with converged = 1
  int it = 0;
  float m = 0.f;
  const bool unbounded = a.var_max_iter < 0;

  {  // E_k = exp(psi_k - m) of the initial gamma; later E's come from the previous topic phase
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < TJ; ++j) mx = fmaxf(mx, psi[j]);
    m = group_max<G>(mx);
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int k = t + G * j;
      e[j] = (k < K) ? __expf(psi[j] - m) : 0.f;
      if (k < KS) sE[k] = e[j];
    }
  }
  while (more && (unbounded || it < a.var_max_iter)) {
    ++it;
    wave_lds_sync();   // sE of this iteration

    // ---- word pass ----
    float acc[KS];
#pragma unroll
    for (int k = 0; k < KS; ++k) acc[k] = 0.f;
    float lsum = 0.f;
#pragma unroll
    for (int c = 0; c < CW; ++c) {
      if (t + G * c < N) {
        const float P = fmaxf(dot_lds<KS>(sE, bc[c]), kPMin);
        const float r = rdiv(cc[c], P);
        lsum = fmaf(cc[c], log_normal(P), lsum);
#pragma unroll
        for (int k = 0; k < KS; ++k) acc[k] = fmaf(r, bc[c][k], acc[k]);
      }
    }
    for (int n = t + G * CW; n < N; n += G) {
      float row[KS];
      const int w = a.word_idx[beg + n];
      const float cnt = a.counts[beg + n];
      load_row<KS>(a.beta, w, row);
      const float P = fmaxf(dot_lds<KS>(sE, row), kPMin);
      const float r = rdiv(cnt, P);
      lsum = fmaf(cnt, log_normal(P), lsum);
#pragma unroll
      for (int k = 0; k < KS; ++k) acc[k] = fmaf(r, row[k], acc[k]);
    }
    double lsum_d;
    if constexpr (G == 64) {
      // one document per wave: DPP sums into lane 63 (no swizzle / readlane per value), handed to
      // the topic lanes through LDS
      wave_sum_last_vec<KS>(acc);
      lsum_d = __shfl(wave_sum_last((double)lsum), 63);
      if (t == 63) {
#pragma unroll
        for (int k = 0; k < KS; ++k) sAcc[g][k] = acc[k];
      }
      wave_lds_sync();
    } else {
      group_sum_vec<G, KS>(acc);
      lsum_d = group_sum<G>((double)lsum);
    }

    // ---- topic phase: gamma update + likelihood ----
    float gn[TJ];
    float sg = 0.f;
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int k = t + G * j;
      float ak = 0.f;
      if constexpr (G == 64) {
        if (k < KS) ak = sAcc[g][k];
      } else {
#pragma unroll
        for (int i = 0; i < KS; ++i) ak = (i == k) ? acc[i] : ak;
      }
      gn[j] = (k < K) ? fmaf(e[j], ak, alpha) : 0.f;
      sg += gn[j];
    }
    // sum_k [lnG(g'_k) + (g'_k - a)(psi(S') - psi(g_k))]
    //   = sum_k [lnG(g'_k) - (g'_k - a) psi(g_k)] + psi(S') (S' - K a): no wait for psi(S')
    double part = 0.0;
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int k = t + G * j;
      if (k < K) {
        float pn, lg;
        digamma_lgamma(gn[j], pn, lg);
        part += (double)lg - (double)(gn[j] - alpha) * (double)psi[j];
        psi[j] = pn;
        gam[j] = gn[j];
      }
    }
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < TJ; ++j) mx = fmaxf(mx, psi[j]);
    const float S = group_sum<G>(sg);
    const double termp = group_sum<G>(part);
    const float m_new = group_max<G>(mx);   // next E beside the likelihood chain
    float e_new[TJ];
#pragma unroll
    for (int j = 0; j < TJ; ++j) e_new[j] = (t + G * j < K) ? __expf(psi[j] - m_new) : 0.f;
    float dS, lgS;
    digamma_lgamma(S, dS, lgS);
    const double term = termp + (double)dS * ((double)S - (double)K * (double)alpha);
    L = a.lik_const - (double)lgS + term + (lsum_d + (double)m * total) - total * (double)dS;
    more = var_more(lik_old, L, (double)a.var_conv);
    lik_old = L;
    dsum_last = dS;
    if (more && (unbounded || it < a.var_max_iter)) {   // commit (E of the final phi stays otherwise)
      m = m_new;
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int k = t + G * j;
        e[j] = e_new[j];
        if (k < KS) sE[k] = e[j];
      }
    }
  }

  if (it == 0) {  // var_max_iter == 0: phi from the initial gamma
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < TJ; ++j) mx = fmaxf(mx, psi[j]);
    m = group_max<G>(mx);
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int k = t + G * j;
      e[j] = (k < K) ? __expf(psi[j] - m) : 0.f;
      if (k < KS) sE[k] = e[j];
    }
    float sg = 0.f;
#pragma unroll
    for (int j = 0; j < TJ; ++j) sg += gam[j];
    dsum_last = digammaf_ldac(group_sum<G>(sg));
    wave_lds_sync();
  }

  // ---- outputs ----
  double ass = 0.0;
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int k = t + G * j;
    if (k < KS) {
      a.gamma[(size_t)d * KS + k] = gam[j];
      a.e_out[(size_t)d * KS + k] = e[j];
    }
    if (k < K) ass += (double)psi[j];
  }
  ass = group_sum<G>(ass);
#pragma unroll
  for (int c = 0; c < CW; ++c) {
    const int n = t + G * c;
    if (n < N) a.r_out[beg + n] = rdiv(cc[c], fmaxf(dot_lds<KS>(sE, bc[c]), kPMin));
  }
  for (int n = t + G * CW; n < N; n += G) {
    float row[KS];
    load_row<KS>(a.beta, a.word_idx[beg + n], row);
    a.r_out[beg + n] = rdiv(a.counts[beg + n], fmaxf(dot_lds<KS>(sE, row), kPMin));
  }
  if (t == 0) {
    a.lik[d] = L;
    a.alpha_ss[d] = ass - (double)K * dsum_last;
    a.iters[d] = it;
  }
}

// ---------------------------------------------------------------------------
// Block kernel: one long document per workgroup of NW waves.
// ---------------------------------------------------------------------------
template <int KS, int NW, int CW>
__global__ __launch_bounds__(NW * 64) void lda_estep_block(EStepArgs a) {
  if (load_params(a)) return;
  // long documents are the EM step's critical path: win SIMD issue arbitration
  // against the short-document waves that share the CU (microarch guide, s_setprio)
  __builtin_amdgcn_s_setprio(2);
  constexpr int NT = NW * 64;
  constexpr int TJ = (KS + 63) / 64;  // topics per lane of wave 0
  __shared__ float4 sE4[KS / 4];
  __shared__ float sRed[NW][KS];
  __shared__ double sRedD[NW][2];
  __shared__ int sFlag;

  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wv = t >> 6;
  const int d = a.order[blockIdx.x];
  const int beg = a.doc_ptr[d];
  const int N = a.doc_ptr[d + 1] - beg;
  const int K = a.K;
  const float alpha = a.alpha;
  float* sE = reinterpret_cast<float*>(&sE4[0]);

  float bc[CW][KS];
  float cc[CW];
  double tot_l = 0.0;
#pragma unroll
  for (int c = 0; c < CW; ++c) {
    const int n = t + NT * c;
    if (n < N) {
      cc[c] = a.counts[beg + n];
      load_row<KS>(a.beta, a.word_idx[beg + n], bc[c]);
    } else {
      cc[c] = 0.f;
#pragma unroll
      for (int k = 0; k < KS; ++k) bc[c][k] = 0.f;
    }
    tot_l += cc[c];
  }
  for (int n = t + NT * CW; n < N; n += NT) tot_l += a.counts[beg + n];
  tot_l = group_sum<64>(tot_l);
  if (lane == 0) sRedD[wv][0] = tot_l;
  __syncthreads();
  double total = 0.0;
#pragma unroll
  for (int w = 0; w < NW; ++w) total += sRedD[w][0];
  __syncthreads();

  // wave 0 owns topic state
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
      e[j] = 0.f;
    }
    // first E
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

  const bool timed = a.dbg != nullptr && blockIdx.x == 0 && t == 0;
  long long tm[4] = {0, 0, 0, 0}, t0 = 0, t1 = 0;
  while (sFlag) {
    if (timed) t0 = clock64();
    // ---- word pass (all waves) ----
    float acc[KS];
#pragma unroll
    for (int k = 0; k < KS; ++k) acc[k] = 0.f;
    float lsum = 0.f;
#pragma unroll
    for (int c = 0; c < CW; ++c) {
      if (t + NT * c < N) {
        const float P = fmaxf(dot_lds<KS>(sE, bc[c]), kPMin);
        const float r = rdiv(cc[c], P);
        lsum = fmaf(cc[c], log_normal(P), lsum);
#pragma unroll
        for (int k = 0; k < KS; ++k) acc[k] = fmaf(r, bc[c][k], acc[k]);
      }
    }
    for (int n = t + NT * CW; n < N; n += NT) {
      float row[KS];
      const float cnt = a.counts[beg + n];
      load_row<KS>(a.beta, a.word_idx[beg + n], row);
      const float P = fmaxf(dot_lds<KS>(sE, row), kPMin);
      const float r = rdiv(cnt, P);
      lsum = fmaf(cnt, log_normal(P), lsum);
#pragma unroll
      for (int k = 0; k < KS; ++k) acc[k] = fmaf(r, row[k], acc[k]);
    }
    if (timed) { t1 = clock64(); tm[0] += t1 - t0; t0 = t1; }
    wave_sum_last_vec<KS>(acc);   // totals in lane 63
    const double lsum_w = wave_sum_last((double)lsum);
    if (lane == 63) {
#pragma unroll
      for (int k = 0; k < KS; ++k) sRed[wv][k] = acc[k];
      sRedD[wv][1] = lsum_w;
    }
    if (timed) { t1 = clock64(); tm[1] += t1 - t0; t0 = t1; }
    __syncthreads();
    if (timed) { t1 = clock64(); tm[2] += t1 - t0; t0 = t1; }

    // ---- topic phase (wave 0) ----
    if (wv == 0) {
      ++it;
      double lsum_d = 0.0;
#pragma unroll
      for (int w = 0; w < NW; ++w) lsum_d += sRedD[w][1];
      float gn[TJ];
      float sg = 0.f;
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int k = lane + 64 * j;
        float ak = 0.f;
        if (k < KS) {
#pragma unroll
          for (int w = 0; w < NW; ++w) ak += sRed[w][k];
        }
        gn[j] = (k < K) ? fmaf(e[j], ak, alpha) : 0.f;
        sg += gn[j];
      }
      // The topic-dependent part of the likelihood does not need psi(S'):
      //   sum_k [lnG(g'_k) + (g'_k - a)(psi(S') - psi(g_k))]
      //     = sum_k [lnG(g'_k) - (g'_k - a) psi(g_k)] + psi(S') (S' - K a)
      // so its reduction runs beside the S' reduction and psi(S') (shorter serial chain).  With
      // KS <= 32 every topic lives in the low half-wave: 32-lane reductions (no v_readlane step).
      constexpr int GR = KS <= 32 ? 32 : 64;
      double part = 0.0;
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int k = lane + 64 * j;
        if (k < K) {
          float pn, lg;
          digamma_lgamma(gn[j], pn, lg);
          part += (double)lg - (double)(gn[j] - alpha) * (double)psi[j];
          psi[j] = pn;
          gam[j] = gn[j];
        }
      }
      // the next E (max + exp of the new psi) is computed beside the likelihood chain and committed
      // only if the loop continues (E of the final phi stays otherwise)
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < TJ; ++j) mx = fmaxf(mx, psi[j]);
      const float S = group_sum<GR>(sg);
      const double termp = group_sum<GR>(part);
      const float m_new = group_max<GR>(mx);
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
      const bool cont = more && (unbounded || it < a.var_max_iter);
      if (cont) {  // next E (keeps sE = E of the final phi when stopping)
        m = m_new;
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          const int k = lane + 64 * j;
          e[j] = e_new[j];
          if (k < KS) sE[k] = e[j];
        }
      }
      if (lane == 0) sFlag = cont ? 1 : 0;
    }
    if (timed) { t1 = clock64(); tm[3] += t1 - t0; t0 = t1; }
    __syncthreads();
  }
  if (timed) {
    // [0] word pass  [1] cross-lane / LDS reductions  [2] barrier wait  [3] topic phase (wave 0)
    // [4] variational iterations  [5] words
    for (int i = 0; i < 4; ++i) a.dbg[i] = tm[i];
    a.dbg[4] = it;
    a.dbg[5] = N;
  }

  // ---- outputs ----
#pragma unroll
  for (int c = 0; c < CW; ++c) {
    const int n = t + NT * c;
    if (n < N) a.r_out[beg + n] = rdiv(cc[c], fmaxf(dot_lds<KS>(sE, bc[c]), kPMin));
  }
  for (int n = t + NT * CW; n < N; n += NT) {
    float row[KS];
    load_row<KS>(a.beta, a.word_idx[beg + n], row);
    a.r_out[beg + n] = rdiv(a.counts[beg + n], fmaxf(dot_lds<KS>(sE, row), kPMin));
  }
  if (wv == 0) {
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
      a.lik[d] = L;
      a.alpha_ss[d] = ass - (double)K * dsum_last;
      a.iters[d] = it;
    }
  }
}

// ---------------------------------------------------------------------------
// Thread kernel: one document per thread (tiny documents: half of all IP
// documents hold 1-2 distinct words).  No cross-lane traffic at all: the
// thread keeps gamma / psi / E / the accumulator in registers, streams its few
// beta rows from L2 and runs the whole variational loop serially.  64 documents
// share a wave; the plan sorts documents by length so a wave's documents have
// similar word counts.
// ---------------------------------------------------------------------------
template <int KS>
__global__ __launch_bounds__(256) void lda_estep_thread(EStepArgs a) {
  // The first TC beta rows stay in VGPRs across the variational iterations (the
  // median document has 2 words, so most threads never touch memory in the loop);
  // further words are fetched two rows at a time so their loads overlap.
  constexpr int TC = KS <= 12 ? 4 : (KS <= 20 ? 3 : 1);
  if (load_params(a)) return;
  const int item = blockIdx.x * 256 + threadIdx.x;
  if (item >= a.n_items) return;
  const int d = a.order[item];
  const int beg = a.doc_ptr[d];
  const int N = a.doc_ptr[d + 1] - beg;
  const int K = a.K;
  const float alpha = a.alpha;
  float bc[TC][KS], cc[TC];
  double total = 0.0;
#pragma unroll
  for (int c = 0; c < TC; ++c) {
    if (c < N) {
      cc[c] = a.counts[beg + c];
      load_row<KS>(a.beta, a.word_idx[beg + c], bc[c]);
    } else {
      cc[c] = 0.f;
#pragma unroll
      for (int k = 0; k < KS; ++k) bc[c][k] = 0.f;
    }
    total += cc[c];
  }
  for (int n = TC; n < N; ++n) total += a.counts[beg + n];
  float gam[KS], psi[KS], e[KS];
  const float g0 = alpha + (float)(total / K);
  const float p0 = digammaf_ldac(g0);
#pragma unroll
  for (int k = 0; k < KS; ++k) {
    gam[k] = k < K ? g0 : 0.f;
    psi[k] = k < K ? p0 : -INFINITY;
  }
  double lik_old = 0.0, L = 0.0, dsum_last = 0.0;
  bool more = 1.0 > (double)a.var_conv;   // lda-c starts with converged = 1
  float m = p0;
  int it = 0;
  const bool unbounded = a.var_max_iter < 0;
  auto compute_e = [&]() {
    float mx = -INFINITY;
#pragma unroll
    for (int k = 0; k < KS; ++k) mx = fmaxf(mx, psi[k]);
    m = mx;
#pragma unroll
    for (int k = 0; k < KS; ++k) e[k] = k < K ? __expf(psi[k] - m) : 0.f;
  };
  compute_e();
  {
    float sg = 0.f;
#pragma unroll
    for (int k = 0; k < KS; ++k) sg += gam[k];
    dsum_last = digammaf_ldac(sg);
  }
  while (more && (unbounded || it < a.var_max_iter)) {
    ++it;
    float acc[KS];
#pragma unroll
    for (int k = 0; k < KS; ++k) acc[k] = 0.f;
    float lsum = 0.f;
    // one word: P = E . beta_w, r = c / P, acc += r beta_w.  r_n is written every
    // iteration; the last write is r under the final E (no reload pass at the end).
    auto word = [&](const float (&row)[KS], float cnt, int n) {
      float p0_ = 0.f, p1_ = 0.f;
#pragma unroll
      for (int k = 0; k < KS; k += 2) {
        p0_ = fmaf(e[k], row[k], p0_);
        p1_ = fmaf(e[k + 1], row[k + 1], p1_);
      }
      const float P = fmaxf(p0_ + p1_, kPMin);
      const float r = rdiv(cnt, P);
      lsum = fmaf(cnt, log_normal(P), lsum);
#pragma unroll
      for (int k = 0; k < KS; ++k) acc[k] = fmaf(r, row[k], acc[k]);
      a.r_out[beg + n] = r;
    };
#pragma unroll
    for (int c = 0; c < TC; ++c)
      if (c < N) word(bc[c], cc[c], c);
    for (int n = TC; n < N; n += 2) {
      const bool two = n + 1 < N;
      float r0[KS], r1[KS];
      load_row<KS>(a.beta, a.word_idx[beg + n], r0);
      load_row<KS>(a.beta, a.word_idx[beg + (two ? n + 1 : n)], r1);
      const float c0 = a.counts[beg + n];
      const float c1 = two ? a.counts[beg + n + 1] : 0.f;
      word(r0, c0, n);
      if (two) word(r1, c1, n + 1);
    }
    float gn[KS];
    float S = 0.f;
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      gn[k] = k < K ? fmaf(e[k], acc[k], alpha) : 0.f;
      S += gn[k];
    }
    float dS, lgS;
    digamma_lgamma(S, dS, lgS);
    // sum_k [lnG(g'_k) - (g'_k - a) psi(g_k)] + psi(S') (S' - K a): independent of psi(S')
    double part = 0.0;
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      if (k < K) {
        float pn, lg;
        digamma_lgamma(gn[k], pn, lg);
        part += (double)lg - (double)(gn[k] - alpha) * (double)psi[k];
        psi[k] = pn;
        gam[k] = gn[k];
      }
    }
    const double term = part + (double)dS * ((double)S - (double)K * (double)alpha);
    L = a.lik_const - (double)lgS + term + ((double)lsum + (double)m * total) - total * (double)dS;
    more = var_more(lik_old, L, (double)a.var_conv);
    lik_old = L;
    dsum_last = dS;
    const bool cont = more && (unbounded || it < a.var_max_iter);
    if (cont) compute_e();
  }
  // outputs (E of the final phi; r_n was written by the last word pass)
  double ass = 0.0;
#pragma unroll
  for (int k = 0; k < KS; ++k) {
    a.gamma[(size_t)d * KS + k] = gam[k];
    a.e_out[(size_t)d * KS + k] = e[k];
    if (k < K) ass += (double)psi[k];
  }
  a.lik[d] = L;
  a.alpha_ss[d] = ass - (double)K * dsum_last;
  a.iters[d] = it;
}

// ---------------------------------------------------------------------------
// Host launcher
// ---------------------------------------------------------------------------
template <int KS>
static void launch_ks(const EStepArgs& a, int variant, hipStream_t s) {
  if (a.n_items <= 0) return;
  constexpr int CWS = rows_per_lane_4w(KS);
  constexpr int CW8 = rows_per_lane_8w(KS);
  switch (variant) {
    case kEStepG16:
      hipLaunchKernelGGL((lda_estep_group<KS, 16, 1>), dim3((a.n_items + 15) / 16), dim3(256), 0, s, a);
      break;
    case kEStepG32:
      hipLaunchKernelGGL((lda_estep_group<KS, 32, 1>), dim3((a.n_items + 7) / 8), dim3(256), 0, s, a);
      break;
    case kEStepG64:
      hipLaunchKernelGGL((lda_estep_group<KS, 64, 1>), dim3((a.n_items + 3) / 4), dim3(256), 0, s, a);
      break;
    case kEStepG64C:
      hipLaunchKernelGGL((lda_estep_group<KS, 64, CWS>), dim3((a.n_items + 3) / 4), dim3(256), 0, s, a);
      break;
    case kEStepB4:
      hipLaunchKernelGGL((lda_estep_block<KS, 4, CWS>), dim3(a.n_items), dim3(256), 0, s, a);
      break;
    case kEStepB8:
      hipLaunchKernelGGL((lda_estep_block<KS, 8, CW8>), dim3(a.n_items), dim3(512), 0, s, a);
      break;
    case kEStepT1:
      if constexpr (KS <= 32) {
        hipLaunchKernelGGL((lda_estep_thread<KS>), dim3((a.n_items + 255) / 256), dim3(256), 0, s, a);
      } else {
        throw std::runtime_error("lda_estep: thread-per-document variant needs KS <= 32");
      }
      break;
    default:
      throw std::runtime_error("lda_estep: unknown variant");
  }
  ONI_HIP_CHECK(hipGetLastError());
}

void launch_lda_estep(const EStepArgs& a, int variant, int KS, hipStream_t s) {
  if (variant >= kEStepW16) {
    launch_lda_estep_wide(a, variant, KS, s);
    return;
  }
  switch (KS) {
#define ONI_KS(X) \
  case X:         \
    launch_ks<X>(a, variant, s); \
    break;
    ONI_FOR_EACH_KS(ONI_KS)
#undef ONI_KS
    default:
      throw std::runtime_error("lda_estep: unsupported padded topic count " + std::to_string(KS));
  }
}

}  // namespace oni
