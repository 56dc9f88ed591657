// Wide-topic variational E-step (K >= 48) on CDNA4 (gfx950).
//
// Same Jacobi fixed point and closed-form likelihood as lda_estep.hip (oni-lda-c
// `lda_inference` + `compute_likelihood`, SURVEY.md C9c/C9d, call site
// /root/reference/ml_ops.sh:80), but a different lane layout.  The narrow
// kernels give every lane whole word rows (KS floats for the row, KS for the
// accumulator, KS per cached row): at K = 100 that is > 300 VGPRs, so they run
// at one wave per SIMD with scratch spills.  Here one word's KS topics are split
// over TG lanes ("topic groups"):
//
//   row chunk c (4 topics, 16 bytes), c < KS/4, lives on lane q = c mod TG of the
//   word's slot, at register index j = c / TG   -> CPL = ceil(KS/4/TG) float4s
//
// so a slot of TG lanes loads a 4*KS-byte row as TG-wide coalesced 64-byte
// pieces, each lane holds CPL float4 of row / accumulator / E, and the per-word
// normaliser P = sum_k E_k beta[w][k] is a partial dot per lane plus a TG-lane
// DPP reduction (quad_perm xor1/xor2, row_half_mirror: symmetric, so all TG lanes
// get bitwise the same P).  Per variational iteration:
//
//   word pass   lanes of slot s take words n = s, s + S, ... (S = slots per doc);
//               the first CW words of a lane stay in VGPRs across iterations,
//               further words stream from L2 / HBM (their r_n is written each pass)
//   slot sum    each lane stores its accumulator chunks to LDS [slot][KS]; topic
//               owners add the S slot rows in slot order (deterministic)
//   topic phase gamma' = alpha + E * acc, psi / lnGamma, likelihood terms, the
//               convergence test and the next E (LDS broadcast to the word layout)
//
// Kernels:
//   lda_estep_wgroup<KS,TG,G,CW>  G = 16/32/64 lanes per document, 256/G per block
//   lda_estep_wblock<KS,TG,NW,CW> one document per NW-wave workgroup (NW = 4, 8)
//   lda_estep_wsplit<KS,TG,CW>    one huge document over several 8-wave workgroups,
//                                 the cross-workgroup protocol of lda_estep_split.hip
#include <stdexcept>
#include <string>

#include "common.h"
#include "estep_common.h"
#include "kernels.h"

namespace oni {

namespace {

template <int KS, int TG>
struct Wide {
  static_assert(KS % 4 == 0, "KS must be a multiple of 4");
  static_assert(TG == 4 || TG == 8, "topic group of 4 or 8 lanes");
  static constexpr int C = KS / 4;                 // float4 chunks per row
  static constexpr int CPL = (C + TG - 1) / TG;    // chunks per lane (upper bound)
};

// Sum over the TG lanes of a topic group (aligned lanes, all active together).
template <int TG>
__device__ __forceinline__ float tg_sum(float x) {
  using namespace detail;
  x += xchg<kQuadXor1>(x);
  x += xchg<kQuadXor2>(x);
  if constexpr (TG == 8) x += xchg<kRowHalfMirror>(x);
  return x;
}

template <int KS, int TG>
__device__ __forceinline__ void load_chunks(const float* __restrict__ beta, int w, int q,
                                            float4 (&row)[Wide<KS, TG>::CPL]) {
  using W = Wide<KS, TG>;
  const float4* p = reinterpret_cast<const float4*>(beta + (size_t)w * KS);
#pragma unroll
  for (int j = 0; j < W::CPL; ++j) {
    const int c = q + TG * j;
    row[j] = (c < W::C) ? p[c] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

template <int CPL>
__device__ __forceinline__ float dot4(const float4 (&e)[CPL], const float4 (&row)[CPL]) {
  float p0 = 0.f, p1 = 0.f;
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    p0 = fmaf(e[j].x, row[j].x, p0);
    p1 = fmaf(e[j].y, row[j].y, p1);
    p0 = fmaf(e[j].z, row[j].z, p0);
    p1 = fmaf(e[j].w, row[j].w, p1);
  }
  return p0 + p1;
}

template <int CPL>
__device__ __forceinline__ void axpy4(float r, const float4 (&row)[CPL], float4 (&acc)[CPL]) {
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    acc[j].x = fmaf(r, row[j].x, acc[j].x);
    acc[j].y = fmaf(r, row[j].y, acc[j].y);
    acc[j].z = fmaf(r, row[j].z, acc[j].z);
    acc[j].w = fmaf(r, row[j].w, acc[j].w);
  }
}

// E chunks of this lane from the document's LDS E vector (KS floats).
template <int KS, int TG>
__device__ __forceinline__ void load_e(const float* sE, int q, float4 (&e)[Wide<KS, TG>::CPL]) {
  using W = Wide<KS, TG>;
  const float4* s4 = reinterpret_cast<const float4*>(sE);
#pragma unroll
  for (int j = 0; j < W::CPL; ++j) {
    const int c = q + TG * j;
    e[j] = (c < W::C) ? s4[c] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// This lane's accumulator chunks into its slot row of LDS ([slot][KS]).
template <int KS, int TG>
__device__ __forceinline__ void store_acc(float* sRow, int q, const float4 (&acc)[Wide<KS, TG>::CPL]) {
  using W = Wide<KS, TG>;
  float4* s4 = reinterpret_cast<float4*>(sRow);
#pragma unroll
  for (int j = 0; j < W::CPL; ++j) {
    const int c = q + TG * j;
    if (c < W::C) s4[c] = acc[j];
  }
}

// Register-cached words of one lane (the slot's first CW words).
template <int KS, int TG, int CW>
struct Cache {   // CW == 0: nothing cached (long documents stream every word)
  float4 bc[CW > 0 ? CW : 1][Wide<KS, TG>::CPL];
  float cc[CW > 0 ? CW : 1];
};

template <int KS, int TG, int CW>
__device__ __forceinline__ double load_cache(const EStepArgs& a, int beg, int N, int s, int S, int q,
                                             Cache<KS, TG, CW>& c) {
  double tot = 0.0;
#pragma unroll
  for (int i = 0; i < CW; ++i) {
    const int n = s + S * i;
    if (n < N) {
      c.cc[i] = a.counts[beg + n];
      load_chunks<KS, TG>(a.beta, a.word_idx[beg + n], q, c.bc[i]);
    } else {
      c.cc[i] = 0.f;
#pragma unroll
      for (int j = 0; j < Wide<KS, TG>::CPL; ++j) c.bc[i][j] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    tot += c.cc[i];
  }
  for (int n = s + S * CW; n < N; n += S) tot += a.counts[beg + n];
  return tot;   // counted once per slot lane q == 0 by the caller
}

// One pass over the lane's words under E (e): acc += r_n beta_n, lsum += c_n log P_n
// (lane q == 0 of each slot only).  Streamed words write r_n = c_n / P_n every pass,
// so the last pass leaves r under the final E.  UNR streamed words are in flight
// per lane (the long-document kernels are bound by bytes in flight per CU).
template <int KS, int TG, int CW, int UNR>
__device__ __forceinline__ void word_pass(const EStepArgs& a, int beg, int N, int s, int S, int q,
                                          const Cache<KS, TG, CW>& c, const float4 (&e)[Wide<KS, TG>::CPL],
                                          float4 (&acc)[Wide<KS, TG>::CPL], float& lsum) {
  constexpr int CPL = Wide<KS, TG>::CPL;
#pragma unroll
  for (int j = 0; j < CPL; ++j) acc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int i = 0; i < CW; ++i) {
    if (s + S * i < N) {   // slot-uniform
      const float P = fmaxf(tg_sum<TG>(dot4<CPL>(e, c.bc[i])), kPMin);
      const float r = rdiv(c.cc[i], P);
      if (q == 0) lsum = fmaf(c.cc[i], log_normal(P), lsum);
      axpy4<CPL>(r, c.bc[i], acc);
    }
  }
  int n = s + S * CW;
  for (; n + (UNR - 1) * S < N; n += UNR * S) {
    float4 rows[UNR][CPL];
    float cn[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      cn[u] = a.counts[beg + n + u * S];
      load_chunks<KS, TG>(a.beta, a.word_idx[beg + n + u * S], q, rows[u]);
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const float P = fmaxf(tg_sum<TG>(dot4<CPL>(e, rows[u])), kPMin);
      const float x = rdiv(cn[u], P);
      if (q == 0) {
        lsum = fmaf(cn[u], log_normal(P), lsum);
        a.r_out[beg + n + u * S] = x;
      }
      axpy4<CPL>(x, rows[u], acc);
    }
  }
  for (; n < N; n += S) {
    float4 r0[CPL];
    const float c0 = a.counts[beg + n];
    load_chunks<KS, TG>(a.beta, a.word_idx[beg + n], q, r0);
    const float P0 = fmaxf(tg_sum<TG>(dot4<CPL>(e, r0)), kPMin);
    const float x0 = rdiv(c0, P0);
    if (q == 0) {
      lsum = fmaf(c0, log_normal(P0), lsum);
      a.r_out[beg + n] = x0;
    }
    axpy4<CPL>(x0, r0, acc);
  }
}

// r_n of the cached words under the final E (and of streamed words when no
// variational iteration ran, var_max_iter == 0).
template <int KS, int TG, int CW>
__device__ __forceinline__ void write_r(const EStepArgs& a, int beg, int N, int s, int S, int q,
                                       const Cache<KS, TG, CW>& c, const float4 (&e)[Wide<KS, TG>::CPL],
                                       bool streamed) {
  constexpr int CPL = Wide<KS, TG>::CPL;
#pragma unroll
  for (int i = 0; i < CW; ++i) {
    const int n = s + S * i;
    if (n < N) {
      const float P = fmaxf(tg_sum<TG>(dot4<CPL>(e, c.bc[i])), kPMin);
      if (q == 0) a.r_out[beg + n] = rdiv(c.cc[i], P);
    }
  }
  if (streamed) {
    for (int n = s + S * CW; n < N; n += S) {
      float4 row[CPL];
      load_chunks<KS, TG>(a.beta, a.word_idx[beg + n], q, row);
      const float P = fmaxf(tg_sum<TG>(dot4<CPL>(e, row)), kPMin);
      if (q == 0) a.r_out[beg + n] = rdiv(a.counts[beg + n], P);
    }
  }
}

// Per-topic state of the topic phase: topic k = lane + GT * j (GT lanes, TJ topics each).
template <int KS, int GT>
struct Topics {
  static constexpr int TJ = (KS + GT - 1) / GT;
  float gam[TJ], psi[TJ], e[TJ];
};

template <int KS, int GT>
__device__ __forceinline__ void topics_init(Topics<KS, GT>& T, int lane, int K, float g0) {
  const float p0 = digammaf_ldac(g0);
#pragma unroll
  for (int j = 0; j < Topics<KS, GT>::TJ; ++j) {
    const int k = lane + GT * j;
    T.gam[j] = (k < K) ? g0 : 0.f;
    T.psi[j] = (k < K) ? p0 : -INFINITY;
    T.e[j] = 0.f;
  }
}

// E_k = exp(psi_k - m) into registers and the LDS E vector; returns m.
template <int KS, int GT>
__device__ __forceinline__ float topics_e(Topics<KS, GT>& T, int lane, int K, float* sE) {
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < Topics<KS, GT>::TJ; ++j) mx = fmaxf(mx, T.psi[j]);
  const float m = group_max<GT>(mx);
#pragma unroll
  for (int j = 0; j < Topics<KS, GT>::TJ; ++j) {
    const int k = lane + GT * j;
    T.e[j] = (k < K) ? __expf(T.psi[j] - m) : 0.f;
    if (k < KS) sE[k] = T.e[j];
  }
  return m;
}

template <int KS, int GT>
__device__ __forceinline__ float topics_gsum(const Topics<KS, GT>& T) {
  float sg = 0.f;
#pragma unroll
  for (int j = 0; j < Topics<KS, GT>::TJ; ++j) sg += T.gam[j];
  return group_sum<GT>(sg);
}

// gamma' = alpha + E * acc (acc[j] = summed accumulator of topic lane + GT*j),
// psi / lnGamma of gamma', the document likelihood.  Returns L; dS = psi(sum gamma').
template <int KS, int GT>
__device__ __forceinline__ double topics_update(Topics<KS, GT>& T, const float (&acc)[Topics<KS, GT>::TJ], int lane,
                                                int K, float alpha, double lik_const, double lsum, float m,
                                                double total, double& dsum) {
  constexpr int TJ = Topics<KS, GT>::TJ;
  float gn[TJ];
  float sg = 0.f;
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int k = lane + GT * j;
    gn[j] = (k < K) ? fmaf(T.e[j], acc[j], alpha) : 0.f;
    sg += gn[j];
  }
  // sum_k [lnG(g'_k) + (g'_k - a)(psi(S') - psi(g_k))]
  //   = sum_k [lnG(g'_k) - (g'_k - a) psi(g_k)] + psi(S') (S' - K a): no wait for psi(S')
  double part = 0.0;
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int k = lane + GT * j;
    if (k < K) {
      float pn, lg;
      digamma_lgamma(gn[j], pn, lg);
      part += (double)lg - (double)(gn[j] - alpha) * (double)T.psi[j];
      T.psi[j] = pn;
      T.gam[j] = gn[j];
    }
  }
  const float S = group_sum<GT>(sg);
  const double termp = group_sum<GT>(part);
  float dS, lgS;
  digamma_lgamma(S, dS, lgS);
  const double term = termp + (double)dS * ((double)S - (double)K * (double)alpha);
  dsum = dS;
  return lik_const - (double)lgS + term + (lsum + (double)m * total) - total * (double)dS;
}

template <int KS, int GT>
__device__ __forceinline__ void topics_out(const EStepArgs& a, const Topics<KS, GT>& T, int d, int lane, int K,
                                           double L, double dsum, int it) {
  double ass = 0.0;
#pragma unroll
  for (int j = 0; j < Topics<KS, GT>::TJ; ++j) {
    const int k = lane + GT * j;
    if (k < KS) {
      a.gamma[(size_t)d * KS + k] = T.gam[j];
      a.e_out[(size_t)d * KS + k] = T.e[j];
    }
    if (k < K) ass += (double)T.psi[j];
  }
  ass = group_sum<GT>(ass);
  if (lane == 0) {
    a.lik[d] = L;
    a.alpha_ss[d] = ass - (double)K * dsum;
    a.iters[d] = it;
  }
}

}  // namespace

// ---------------------------------------------------------------------------
// Group kernel: G lanes (S = G/TG slots) per document, 256/G documents per block.
// ---------------------------------------------------------------------------
template <int KS, int TG, int G, int CW, int UNR>
__global__ __launch_bounds__(256) void lda_estep_wgroup(EStepArgs a) {
  if (load_params(a)) return;
  using W = Wide<KS, TG>;
  using TP = Topics<KS, G>;
  constexpr int GPB = 256 / G;
  constexpr int S = G / TG;
  __shared__ float4 sE4[GPB][KS / 4];
  __shared__ float4 sAcc4[GPB][S][KS / 4];

  const int t = threadIdx.x % G;
  const int g = threadIdx.x / G;
  const int item = blockIdx.x * GPB + g;
  if (item >= a.n_items) return;   // group-uniform exit
  const int s = t / TG, q = t % TG;
  float* sE = reinterpret_cast<float*>(&sE4[g][0]);
  float* sAcc = reinterpret_cast<float*>(&sAcc4[g][0][0]);

  const int d = a.order[item];
  const int beg = a.doc_ptr[d];
  const int N = a.doc_ptr[d + 1] - beg;
  const int K = a.K;
  const float alpha = a.alpha;

  Cache<KS, TG, CW> cache;
  double tot_l = load_cache<KS, TG, CW>(a, beg, N, s, S, q, cache);
  const double total = group_sum<G>(q == 0 ? tot_l : 0.0);

  TP T;
  topics_init<KS, G>(T, t, K, alpha + (float)(total / K));
  float m = topics_e<KS, G>(T, t, K, sE);
  double dsum = digammaf_ldac(topics_gsum<KS, G>(T));
  wave_lds_sync();
  float4 e4[W::CPL];
  load_e<KS, TG>(sE, q, e4);

  double lik_old = 0.0, L = 0.0;
  bool more = 1.0 > (double)a.var_conv;   // lda-c starts with converged = 1
  int it = 0;
  const bool unbounded = a.var_max_iter < 0;
  while (more && (unbounded || it < a.var_max_iter)) {
    ++it;
    float4 acc4[W::CPL];
    float lsum = 0.f;
    word_pass<KS, TG, CW, UNR>(a, beg, N, s, S, q, cache, e4, acc4, lsum);
    store_acc<KS, TG>(sAcc + s * KS, q, acc4);
    const double lsum_d = group_sum<G>((double)lsum);
    wave_lds_sync();
    float acc[TP::TJ];
#pragma unroll
    for (int j = 0; j < TP::TJ; ++j) {
      const int k = t + G * j;
      float v = 0.f;
      if (k < KS) {
#pragma unroll
        for (int u = 0; u < S; ++u) v += sAcc[u * KS + k];
      }
      acc[j] = v;
    }
    L = topics_update<KS, G>(T, acc, t, K, alpha, a.lik_const, lsum_d, m, total, dsum);
    more = var_more(lik_old, L, (double)a.var_conv);
    lik_old = L;
    if (more && (unbounded || it < a.var_max_iter)) {
      m = topics_e<KS, G>(T, t, K, sE);
      wave_lds_sync();
      load_e<KS, TG>(sE, q, e4);
    }
  }
  write_r<KS, TG, CW>(a, beg, N, s, S, q, cache, e4, it == 0);
  topics_out<KS, G>(a, T, d, t, K, L, dsum, it);
}

// ---------------------------------------------------------------------------
// Block kernel: one document per NW-wave workgroup (S = 64*NW/TG slots).
// Slot sums: thread t adds slots [h*S/H, (h+1)*S/H) of topic t % 128 (H = NT/128
// partial rows), then wave 0 -- the owner of the topic state -- adds the H rows.
// ---------------------------------------------------------------------------
template <int KS, int TG, int NW, int CW, int UNR>
__global__ __launch_bounds__(NW * 64) void lda_estep_wblock(EStepArgs a) {
  if (load_params(a)) return;
  __builtin_amdgcn_s_setprio(2);   // long documents: the E-step's critical path
  static_assert(KS <= 128, "block slot reduction assumes KS <= 128");
  using W = Wide<KS, TG>;
  using TP = Topics<KS, 64>;
  constexpr int NT = NW * 64;
  constexpr int S = NT / TG;
  constexpr int H = NT / 128;
  constexpr int SH = S / H;
  __shared__ float4 sE4[KS / 4];
  __shared__ float4 sAcc4[S][KS / 4];
  __shared__ float sPart[H][128];
  __shared__ double sRedD[NW];
  __shared__ int sFlag;

  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int s = t / TG, q = t % TG;
  const int d = a.order[blockIdx.x];
  const int beg = a.doc_ptr[d];
  const int N = a.doc_ptr[d + 1] - beg;
  const int K = a.K;
  const float alpha = a.alpha;
  float* sE = reinterpret_cast<float*>(&sE4[0]);
  float* sAcc = reinterpret_cast<float*>(&sAcc4[0][0]);

  Cache<KS, TG, CW> cache;
  double tot_l = load_cache<KS, TG, CW>(a, beg, N, s, S, q, cache);
  tot_l = group_sum<64>(q == 0 ? tot_l : 0.0);
  if (lane == 0) sRedD[wv] = tot_l;
  __syncthreads();
  double total = 0.0;
#pragma unroll
  for (int w = 0; w < NW; ++w) total += sRedD[w];
  __syncthreads();

  TP T;
  double lik_old = 0.0, L = 0.0, dsum = 0.0;
  float m = 0.f;
  int it = 0;
  const bool unbounded = a.var_max_iter < 0;
  if (wv == 0) {
    topics_init<KS, 64>(T, lane, K, alpha + (float)(total / K));
    m = topics_e<KS, 64>(T, lane, K, sE);
    dsum = digammaf_ldac(topics_gsum<KS, 64>(T));
    if (lane == 0) sFlag = (unbounded || a.var_max_iter > 0) ? 1 : 0;
  }
  __syncthreads();
  const bool ran = sFlag != 0;   // false: var_max_iter == 0, no variational iteration
  float4 e4[W::CPL];
  load_e<KS, TG>(sE, q, e4);

  while (sFlag) {
    float4 acc4[W::CPL];
    float lsum = 0.f;
    word_pass<KS, TG, CW, UNR>(a, beg, N, s, S, q, cache, e4, acc4, lsum);
    store_acc<KS, TG>(sAcc + s * KS, q, acc4);
    const double lsum_w = group_sum<64>((double)lsum);
    if (lane == 0) sRedD[wv] = lsum_w;
    __syncthreads();
    {
      const int k = t & 127, h = t >> 7;
      if (k < KS) {
        float v = 0.f;
#pragma unroll 8
        for (int u = h * SH; u < (h + 1) * SH; ++u) v += sAcc[u * KS + k];
        sPart[h][k] = v;
      }
    }
    __syncthreads();
    if (wv == 0) {
      ++it;
      double lsum_d = 0.0;
#pragma unroll
      for (int w = 0; w < NW; ++w) lsum_d += sRedD[w];
      float acc[TP::TJ];
#pragma unroll
      for (int j = 0; j < TP::TJ; ++j) {
        const int k = lane + 64 * j;
        float v = 0.f;
        if (k < KS) {
#pragma unroll
          for (int h = 0; h < H; ++h) v += sPart[h][k];
        }
        acc[j] = v;
      }
      L = topics_update<KS, 64>(T, acc, lane, K, alpha, a.lik_const, lsum_d, m, total, dsum);
      const bool more = var_more(lik_old, L, (double)a.var_conv);
      lik_old = L;
      const bool cont = more && (unbounded || it < a.var_max_iter);
      if (cont) m = topics_e<KS, 64>(T, lane, K, sE);
      if (lane == 0) sFlag = cont ? 1 : 0;
    }
    __syncthreads();
    load_e<KS, TG>(sE, q, e4);
  }
  write_r<KS, TG, CW>(a, beg, N, s, S, q, cache, e4, !ran);
  if (wv == 0) topics_out<KS, 64>(a, T, d, lane, K, L, dsum, it);
}

// ---------------------------------------------------------------------------
// Split kernel: one huge document over nseg 8-wave workgroups; every variational
// iteration the segments exchange (acc[KS], lsum) through global memory behind a
// per-document arrival counter (protocol: lda_estep_split.hip).
// ---------------------------------------------------------------------------
namespace {
constexpr int kWNW = 8;
constexpr int kWNT = kWNW * 64;
}  // namespace

template <int KS, int TG, int CW, int UNR>
__global__ __launch_bounds__(kWNT) void lda_estep_wsplit(EStepArgs a, SplitArgs sp) {
  if (load_params(a)) return;
  __builtin_amdgcn_s_setprio(3);
  static_assert(KS <= 128, "block slot reduction assumes KS <= 128");
  using W = Wide<KS, TG>;
  using TP = Topics<KS, 64>;
  constexpr int S = kWNT / TG;
  constexpr int H = kWNT / 128;
  constexpr int SH = S / H;
  __shared__ float4 sE4[KS / 4];
  __shared__ float4 sAcc4[S][KS / 4];
  __shared__ float sPart[H][128];
  __shared__ double sRedD[kWNW];
  __shared__ int sFlag;

  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int s = t / TG, q = t % TG;
  const int b = blockIdx.x;
  const int d = sp.seg_doc[b];
  const int seg = sp.seg_index[b];
  const int nseg = sp.seg_count[b];
  const int base = sp.seg_base[b];
  int* counter = sp.counter + sp.doc_slot[b];
  const int epoch = __hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int dbeg = a.doc_ptr[d];
  const int Ndoc = a.doc_ptr[d + 1] - dbeg;
  const int beg = dbeg + seg * sp.seg_words;
  const int N = min(sp.seg_words, Ndoc - seg * sp.seg_words);
  const int K = a.K;
  const float alpha = a.alpha;
  float* sE = reinterpret_cast<float*>(&sE4[0]);
  float* sAcc = reinterpret_cast<float*>(&sAcc4[0][0]);

  Cache<KS, TG, CW> cache;
  load_cache<KS, TG, CW>(a, beg, N, s, S, q, cache);
  // document total: every workgroup reads the whole document's counts once
  double tot_l = 0.0;
  for (int n = t; n < Ndoc; n += kWNT) tot_l += a.counts[dbeg + n];
  tot_l = group_sum<64>(tot_l);
  if (lane == 0) sRedD[wv] = tot_l;
  __syncthreads();
  double total = 0.0;
#pragma unroll
  for (int w = 0; w < kWNW; ++w) total += sRedD[w];
  __syncthreads();

  TP T;
  double lik_old = 0.0, L = 0.0, dsum = 0.0;
  float m = 0.f;
  int it = 0;
  const bool unbounded = a.var_max_iter < 0;
  if (wv == 0) {
    topics_init<KS, 64>(T, lane, K, alpha + (float)(total / K));
    m = topics_e<KS, 64>(T, lane, K, sE);
    dsum = digammaf_ldac(topics_gsum<KS, 64>(T));
    if (lane == 0) sFlag = (unbounded || a.var_max_iter > 0) ? 1 : 0;
  }
  __syncthreads();
  const bool ran = sFlag != 0;
  float4 e4[W::CPL];
  load_e<KS, TG>(sE, q, e4);

  while (sFlag) {
    float4 acc4[W::CPL];
    float lsum = 0.f;
    word_pass<KS, TG, CW, UNR>(a, beg, N, s, S, q, cache, e4, acc4, lsum);
    store_acc<KS, TG>(sAcc + s * KS, q, acc4);
    const double lsum_w = group_sum<64>((double)lsum);
    if (lane == 0) sRedD[wv] = lsum_w;
    __syncthreads();
    {
      const int k = t & 127, h = t >> 7;
      if (k < KS) {
        float v = 0.f;
#pragma unroll 8
        for (int u = h * SH; u < (h + 1) * SH; ++u) v += sAcc[u * KS + k];
        sPart[h][k] = v;
      }
    }
    __syncthreads();
    if (wv == 0) {
      ++it;
      const int par = it & 1;
      const unsigned tag = split_tag(epoch, it);
      constexpr int GR = KS + 2;
      float part[TP::TJ];
#pragma unroll
      for (int j = 0; j < TP::TJ; ++j) {
        const int k = lane + 64 * j;
        float v = 0.f;
        if (k < KS) {
#pragma unroll
          for (int h = 0; h < H; ++h) v += sPart[h][k];
        }
        part[j] = v;
      }
      double lpart = 0.0;
#pragma unroll
      for (int w = 0; w < kWNW; ++w) lpart += sRedD[w];
      unsigned long long* xb = sp.xchg + (size_t)par * sp.n_blocks * GR;
      publish_tagged<KS>(xb + (size_t)b * GR, [&](int j) { return part[j]; }, lpart, lane, tag);
      // every segment's partials in segment order: identical bits in every workgroup
      float acc[TP::TJ];
      double lsum_d;
      bool ok = tagged_gather<KS>(xb + (size_t)base * GR, nseg, GR, tag, lane, acc, lsum_d);
      ok = __all(ok);
      if (!ok && lane == 0) __hip_atomic_store(sp.error, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      L = topics_update<KS, 64>(T, acc, lane, K, alpha, a.lik_const, lsum_d, m, total, dsum);
      const bool more = var_more(lik_old, L, (double)a.var_conv);
      lik_old = L;
      const bool cont = ok && more && (unbounded || it < a.var_max_iter);
      if (cont) m = topics_e<KS, 64>(T, lane, K, sE);
      if (lane == 0) sFlag = cont ? 1 : 0;
    }
    __syncthreads();
    load_e<KS, TG>(sE, q, e4);
  }

  split_exit(counter, sp.n_docs, nseg);
  const bool failed = __hip_atomic_load(sp.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  write_r<KS, TG, CW>(a, beg, N, s, S, q, cache, e4, !ran);
  if (wv == 0 && seg == 0) topics_out<KS, 64>(a, T, d, lane, K, failed ? __builtin_nan("") : L, dsum, it);
}

// ---------------------------------------------------------------------------
// Host launchers
// ---------------------------------------------------------------------------
namespace {
// topic-group width and register-cached words per lane: ~4 waves / SIMD (<= 128 VGPRs)
// for the group kernels -- 4 lanes per word up to KS = 64 (4 float4 per lane), 8 beyond
constexpr int wide_tg(int KS) { return KS >= 100 ? 8 : 4; }
constexpr int wide_cw(int KS) { return 2; }
// long documents (WB8, split): no register cache -- 20 variational iterations of a
// 4k..90k-word document re-stream it anyway -- and 4 words in flight per lane
constexpr int kLongCW = 0, kLongUNR = 4;

template <int KS>
void wide_ks(const EStepArgs& a, int variant, hipStream_t s) {
  constexpr int TG = wide_tg(KS), CW = wide_cw(KS);
  switch (variant) {
    case kEStepW16:
      hipLaunchKernelGGL((lda_estep_wgroup<KS, TG, 16, CW, 2>), dim3((a.n_items + 15) / 16), dim3(256), 0, s, a);
      break;
    case kEStepW32:
      hipLaunchKernelGGL((lda_estep_wgroup<KS, TG, 32, CW, 2>), dim3((a.n_items + 7) / 8), dim3(256), 0, s, a);
      break;
    case kEStepW64:
      hipLaunchKernelGGL((lda_estep_wgroup<KS, TG, 64, CW, 2>), dim3((a.n_items + 3) / 4), dim3(256), 0, s, a);
      break;
    case kEStepWB4:
      hipLaunchKernelGGL((lda_estep_wblock<KS, TG, 4, CW, 2>), dim3(a.n_items), dim3(256), 0, s, a);
      break;
    case kEStepWB8:
      hipLaunchKernelGGL((lda_estep_wblock<KS, TG, 8, kLongCW, kLongUNR>), dim3(a.n_items), dim3(512), 0, s, a);
      break;
    default:
      throw std::runtime_error("lda_estep_wide: unknown variant " + std::to_string(variant));
  }
  ONI_HIP_CHECK(hipGetLastError());
}

template <int KS>
void wsplit_ks(const EStepArgs& a, const SplitArgs& sp, hipStream_t st) {
  if (sp.n_blocks <= 0) return;
  if (sp.n_blocks > kSplitMaxBlocks) throw std::runtime_error("lda_estep_wsplit: too many workgroups in one launch");
  hipLaunchKernelGGL((lda_estep_wsplit<KS, wide_tg(KS), kLongCW, kLongUNR>), dim3(sp.n_blocks), dim3(kWNT), 0, st, a,
                     sp);
  ONI_HIP_CHECK(hipGetLastError());
}
}  // namespace

int wide_words(int KS, int lanes) { return (lanes / wide_tg(KS)) * wide_cw(KS); }

template <int KS>
static int wsplit_capacity_ks() {
  int dev = 0, per_cu = 0;
  hipDeviceProp_t p;
  ONI_HIP_CHECK(hipGetDevice(&dev));
  ONI_HIP_CHECK(hipGetDeviceProperties(&p, dev));
  ONI_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
      &per_cu, reinterpret_cast<const void*>(&lda_estep_wsplit<KS, wide_tg(KS), kLongCW, kLongUNR>), kWNT, 0));
  return per_cu * p.multiProcessorCount;
}

int wsplit_capacity(int KS) {
  switch (KS) {
#define ONI_KS(X) \
  case X:         \
    return wsplit_capacity_ks<X>();
    ONI_FOR_EACH_WIDE_KS(ONI_KS)
#undef ONI_KS
    default:
      throw std::runtime_error("wsplit_capacity: unsupported KS " + std::to_string(KS));
  }
}
int wide_slots(int KS, int lanes) { return lanes / wide_tg(KS); }

void launch_lda_estep_wide(const EStepArgs& a, int variant, int KS, hipStream_t s) {
  if (a.n_items <= 0) return;
  switch (KS) {
#define ONI_KS(X) \
  case X:         \
    wide_ks<X>(a, variant, s); \
    break;
    ONI_FOR_EACH_WIDE_KS(ONI_KS)
#undef ONI_KS
    default:
      throw std::runtime_error("lda_estep_wide: unsupported KS " + std::to_string(KS));
  }
}

void launch_lda_estep_wsplit(const EStepArgs& a, const SplitArgs& sp, int KS, hipStream_t st) {
  switch (KS) {
#define ONI_KS(X) \
  case X:         \
    wsplit_ks<X>(a, sp, st); \
    break;
    ONI_FOR_EACH_WIDE_KS(ONI_KS)
#undef ONI_KS
    default:
      throw std::runtime_error("lda_estep_wsplit: unsupported KS " + std::to_string(KS));
  }
}

}  // namespace oni
