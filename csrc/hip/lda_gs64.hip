// fp64 block Gauss-Seidel E-step, sufficient statistics and M-step (gfx950).
//
// Reference: oni-lda-c's lda_inference (call site /root/reference/ml_ops.sh:80;
// SURVEY.md C9c-C9h) computes in double and refreshes gamma and digamma(gamma)
// after EVERY word.  This engine keeps lda-c's arithmetic (double, lda-c's series
// digamma, lgamma, the -100 floor) and its schedule up to the block size: a
// document of n words is walked in chunks of W = ceil(n / U) words (U = gs_updates
// refreshes per sweep); a chunk's words take phi from one digamma vector, then
// gamma and digamma are refreshed.  n <= U is exactly lda-c's per-word schedule.
// The CPU oracle is csrc/native/lda_ref.cpp lda_inference(..., gs_updates).
//
// Chunk algebra (why no per-word phi state is needed): with E_k = exp(psi_k - m)
// (m = psi of the initial gamma, a per-document constant), P_n = sum_k E_k b_nk,
// r_n = c_n / P_n, the chunk's contribution to gamma is
//     new_jk = sum_{n in j} c_n phi_nk = E_k * S_k,   S_k = sum_{n in j} r_n b_nk,
// so a chunk update is gamma_k += new_jk - C_jk; C_jk = new_jk (C = the chunk's
// previous contribution, c_total/K before the first sweep), one table of U x KS
// doubles per document in LDS.  The per-sweep likelihood (lda-c compute_likelihood)
// collapses to
//     L = lgG(K a) - K lgG(a) - lgG(sum g) + sum_k lgG(g_k)
//         + sum_n c_n (m + log P_n) - sum_j sum_k psi_jk new_jk
// (the (a - 1), (g - 1) and (g - a) psi terms cancel exactly; psi_jk is the digamma
// the chunk's words saw).  The final sweep's c_n phi_nk = E_jk b_nk r_n rows are
// written per corpus entry; the suff-stats kernel gathers them in CSC order.
//
// Kernel shapes:
//   gs_tiny   TG lanes per document (KPL = KS / TG topics per lane), n <= NMAX words,
//             literal per-word schedule; the per-word contributions C[n][.] live in VGPRs.
//   gs_team   one wave / 4-wave / 8-wave workgroup per document.  Lanes are
//             (topic group q) x (word slot sl) with the slot in the low lane bits:
//             a word's P is an xor-16/32 (permlane swap) reduction over q, the slot
//             reduction of S is a row DPP reduction; cross-wave sums go through LDS in
//             wave order (bitwise reproducible).  Topic owners (one thread per topic)
//             run the refresh and broadcast E through LDS.
#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "alpha_newton.h"
#include "common.h"
#include "em_control.h"
#include "estep_common.h"
#include "gs_math.h"
#include "kernels.h"

namespace oni {
namespace gs {

constexpr double kExpM100 = 3.720075976020836e-44;   // exp(-100), lda-c's log-probability floor

constexpr int tg_of(int KS) { return KS <= 32 ? 4 : (KS <= 64 ? 8 : 16); }
constexpr int kpl_of(int KS) { return (KS + tg_of(KS) - 1) / tg_of(KS); }
// tiny kernel: wider topic groups than the team kernels (fewer topics, hence fewer
// digamma/exp chains and queue registers per lane)
constexpr int tiny_tg(int KS) { return KS <= 32 ? 8 : 16; }
constexpr int tiny_kpl(int KS) { return (KS + tiny_tg(KS) - 1) / tiny_tg(KS); }
constexpr int tiny_max(int KS) { return tiny_kpl(KS) <= 4 ? 8 : 4; }

// topic of a lane's i-th value in the team layouts (TeamShape::PAIR: consecutive pairs)
template <int TG, bool PAIR>
__device__ __forceinline__ int tk(int q, int i) { return PAIR ? 2 * q + (i & 1) + 2 * TG * (i >> 1) : q + TG * i; }

// a word's KPL values of this lane at constant offsets.  The row's last, partial topic group: lanes past KS
// re-read the group's last valid topic (the cache line a valid lane already fetches), so a row gather touches
// only the row's own lines -- reading on into the next row touched ~1.75 extra 128-B lines per 800-B row at
// KS = 100 (8.75 instead of 7).  Measured at 100 M events: team8 0.147 -> 0.141 ns per word-sweep (-4 %), team4
// -1 % (profiles/r6p_team4_rmax.md): these gathers are not bound by the lines they fetch.
// Those lanes' values only ever meet E = 0 or are never stored (every consumer guards tk < KS).
template <int KS, int KPL, int TG, bool PAIR>
__device__ __forceinline__ void load_row(const double* __restrict__ beta, int w, int q, double (&b)[KPL]) {
  const double* rb = beta + (size_t)w * KS;
  if constexpr (PAIR) {
    static_assert(KS % 2 == 0, "pair rows: even KS");
    const dvec2* r = reinterpret_cast<const dvec2*>(rb + 2 * q);
#pragma unroll
    for (int ii = 0; ii < KPL / 2; ++ii) {
      dvec2 v;
      if (2 * TG * (ii + 1) <= KS) {
        v = r[TG * ii];
      } else {
        const int last = (KS - 2 * TG * ii) / 2 - 1;     // the group's last valid pair (compile-time)
        v = *reinterpret_cast<const dvec2*>(rb + 2 * TG * ii + 2 * min(q, last));
      }
      b[2 * ii] = v.x;
      b[2 * ii + 1] = v.y;
    }
  } else {
    const double* brow = rb + q;
#pragma unroll
    for (int i = 0; i < KPL; ++i) {
      if (TG * (i + 1) <= KS)
        b[i] = brow[TG * i];
      else
        b[i] = rb[TG * i + min(q, KS - TG * i - 1)];
    }
  }
}

// ------------------------------------------------------------------ tiny ----
// C[j][.] (the current contribution of word j) is a register queue: word j always
// uses C[0], then the queue rotates left by one with the new value at the back, so
// the word loop is a runtime loop (one copy of the digamma/exp code, ~160 VGPRs)
// instead of an unrolled one (>256 VGPRs + scratch).  After a sweep of n words the
// queue is rotated back by (-n) mod NMAX in log2(NMAX) conditional stages.
template <int N, int KPL>
__device__ __forceinline__ void rotl1(double (&C)[N][KPL]) {
#pragma unroll
  for (int i = 0; i < KPL; ++i) {
    const double t0 = C[0][i];
#pragma unroll
    for (int j = 0; j < N - 1; ++j) C[j][i] = C[j + 1][i];
    C[N - 1][i] = t0;
  }
}

template <int N, int KPL, int B>
__device__ __forceinline__ void rotl_if(double (&C)[N][KPL], bool on) {
#pragma unroll
  for (int i = 0; i < KPL; ++i) {
    double T[N];
#pragma unroll
    for (int j = 0; j < N; ++j) T[j] = C[(j + B) % N][i];
#pragma unroll
    for (int j = 0; j < N; ++j) C[j][i] = on ? T[j] : C[j][i];
  }
}

template <int KS>
__global__ __launch_bounds__(256) void gs_tiny(GSArgs a) {
  constexpr int TG = tiny_tg(KS), KPL = tiny_kpl(KS), NMAX = tiny_max(KS);
  constexpr int LTG = ilog2(TG);
  static_assert(NMAX == 4 || NMAX == 8, "tiny queue length");
  constexpr int DPB = 256 / TG;
  // the document's beta rows and counts, staged once per E-step (every sweep reads them)
  constexpr int BST = NMAX * KS + 1;   // odd stride in doubles: groups of a wave hit different banks
  __shared__ double sB[DPB][BST];
  __shared__ double sN[DPB][NMAX];
  __shared__ dvec2 sLog[kMathTabN];          // flog_t's table
  if (a.params[kParamDone] != 0.0) return;
  log_table_fill(sLog);
  __syncthreads();
  const int t = threadIdx.x, q = t & (TG - 1), g = t / TG;
  const int item = blockIdx.x * DPB + g;
  if (item >= a.n_items) return;   // whole TG groups leave together
  const double alpha = a.params[0], lik_const = a.params[1];
  const int vmi = (int)a.params[2];
  const double vconv = params_vconv(a.params);
  const int K = a.K;
  const int d = a.order[item];
  if (d < 0) return;   // XCD placement gap (GSPlan.xcd_gaps): this document slot only
  const int s0 = a.doc_ptr[d];
  const int n = min(a.doc_ptr[d + 1] - s0, NMAX);
  const int* __restrict__ wrow = a.word_idx + s0;
  const float* __restrict__ crow = a.counts + s0;
  for (int x = q; x < n * KS; x += TG) {
    const int j = x / KS, k = x - j * KS;
    sB[g][j * KS + k] = a.beta[(size_t)wrow[j] * KS + k];
  }
  if (q < n) sN[g][q] = (double)crow[q];
  wave_lds_sync();
  double total = 0.0;
  for (int j = 0; j < n; ++j) total += sN[g][j];
  const double g0 = alpha + total / K;
  const double m = psi_only(g0);
  double gam[KPL], psi[KPL], E[KPL], C[NMAX][KPL];
#pragma unroll
  for (int i = 0; i < KPL; ++i) {
    const bool real = q + TG * i < K;
    gam[i] = real ? g0 : 1.0;   // padding topics hold gamma = 1 (finite refresh, never summed or stored)
    psi[i] = m;
    E[i] = real ? 1.0 : 0.0;
  }
#pragma unroll
  for (int j = 0; j < NMAX; ++j) {
    const double cj = j < n ? sN[g][j] : 0.0;
#pragma unroll
    for (int i = 0; i < KPL; ++i) C[j][i] = (q + TG * i < K) ? cj / K : 0.0;
  }
  double L = 0.0, L_old = 0.0, conv = 1.0, GS = 0.0;
  int it = 0;
  while (var_continue(conv, vconv, it, vmi)) {
    ++it;
    double lw = 0.0, lp = 0.0;
#pragma unroll 1
    for (int j = 0; j < n; ++j) {
      const double* brow = &sB[g][j * KS];
      const double c = sN[g][j];
      double b[KPL];
#pragma unroll
      for (int i = 0; i < KPL; ++i) b[i] = (q + TG * i < KS) ? brow[q + TG * i] : 0.0;
      double pp = 0.0;
#pragma unroll
      for (int i = 0; i < KPL; ++i) pp = fma(E[i], b[i], pp);
      const double P = bits_sum<0, LTG, false>(pp);
      const double r = c * drcp(P);
      lw = fma(c, flog_t(P, sLog), lw);
      // branch-free refresh: the KPL digamma/exp chains interleave (a topic-guarded psi_exp is a basic block
      // of its own and the chains ran one after another); padding topics have E = 0, so nw = 0, and keep
      // gamma = 1, E = 0
#pragma unroll
      for (int i = 0; i < KPL; ++i) {
        const bool real = q + TG * i < K;
        const double nw = E[i] * b[i] * r;
        lp = fma(psi[i], nw, lp);
        gam[i] += nw - C[0][i];
        C[0][i] = nw;
        double pn, en;
        // padding topics: gamma stays 1 (nw = 0, C = 0), psi finite and only ever multiplied by nw = 0
        psi_exp<true, true, (KS > 32)>(gam[i], m, pn, en, sLog);   // table exp: K > 32 only (r5aq)
        psi[i] = pn;
        E[i] = real ? en : 0.0;
      }
      rotl1(C);
    }
    // n rotations so far: rotate by (-n) mod NMAX back to word order
    const int rb = (NMAX - n) & (NMAX - 1);
    rotl_if<NMAX, KPL, 1>(C, rb & 1);
    rotl_if<NMAX, KPL, 2>(C, rb & 2);
    if constexpr (NMAX == 8) rotl_if<NMAX, KPL, 4>(C, rb & 4);
    double gs = 0.0, lg = 0.0;
#pragma unroll
    for (int i = 0; i < KPL; ++i) {
      if (q + TG * i < K) {
        gs += gam[i];
        lg += lgamma_pos<true>(gam[i], sLog);
      }
    }
    GS = bits_sum<0, LTG, false>(gs);
    lg = bits_sum<0, LTG, false>(lg);
    lp = bits_sum<0, LTG, false>(lp);
    L = lik_const - lgamma_pos(GS) + lg + fma(m, total, lw) - lp;
    conv = (L_old - L) / L_old;
    L_old = L;
  }
  double ps = 0.0;
#pragma unroll
  for (int i = 0; i < KPL; ++i) {
    const int k = q + TG * i;
    if (k < K) ps += psi[i];
    if (k < KS) a.gamma[(size_t)d * KS + k] = k < K ? gam[i] : 0.0;
  }
  ps = bits_sum<0, LTG, false>(ps);
#pragma unroll
  for (int j = 0; j < NMAX; ++j) {
    if (j < n) {
      double* row = a.cphi + (size_t)(s0 + j) * KS;
#pragma unroll
      for (int i = 0; i < KPL; ++i)
        if (q + TG * i < KS) __builtin_nontemporal_store(C[j][i], &row[q + TG * i]);
    }
  }
  if (q == 0) {
    a.lik[d] = L;
    a.alpha_ss[d] = ps - K * psi_only(GS);
    a.iters[d] = it;
  }
}

// ----------------------------------------------------------------- small ----
// Short documents (the tiny kernel's limit < n <= kGsSmallMax words): 16 lanes per document, four
// documents per wave, everything in registers except the per-chunk tables.  A word's P is a 16-lane
// DPP sum (every lane holds the bitwise same value), the refresh runs in the same lanes right after
// the chunk's last word -- no LDS, no barrier between the word and the refresh, which is what a
// per-word schedule (n <= U: every word is a chunk) pays for in the one-wave team kernel.  The chunk
// contributions C[j] and the E each chunk used (final pass) are per-lane private arrays (scratch).
constexpr int kGsSmallMax = 64;
constexpr int small_kpl(int KS) { return (KS + 15) / 16; }

template <int KS>
__global__ __launch_bounds__(256) void gs_small(GSArgs a) {
  static_assert(KS <= 32, "small kernel: KS <= 32");
  constexpr int TG = 16, KPL = small_kpl(KS);
  if (a.params[kParamDone] != 0.0) return;
  const int t = threadIdx.x, q = t & (TG - 1);
  const int item = blockIdx.x * (256 / TG) + t / TG;
  if (item >= a.n_items) return;   // whole 16-lane groups leave together
  const double alpha = a.params[0], lik_const = a.params[1];
  const int vmi = (int)a.params[2];
  const double vconv = params_vconv(a.params);
  const int K = a.K;
  const int d = a.order[item];
  if (d < 0) return;   // XCD placement gap (GSPlan.xcd_gaps): this document slot only
  const int s0 = a.doc_ptr[d], n = a.doc_ptr[d + 1] - s0;
  const int U = a.gs_updates;
  const int W = n > 0 ? (n + U - 1) / U : 1;
  const int nch = (n + W - 1) / W;
  const int* __restrict__ wrow = a.word_idx + s0;
  const float* __restrict__ crow = a.counts + s0;
  double C[kGsUMax][KPL], Et[kGsUMax][KPL];
  // counts: each lane sums a stride of the document, a 16-lane sum gives the total; chunk sums serially
  double total = 0.0;
  for (int p = q; p < n; p += TG) total += (double)crow[p];
  total = bits_sum<0, 4, false>(total);
  const double g0 = alpha + total / K;
  const double m = psi_only(g0);
  double gam[KPL], psi[KPL], E[KPL], lps[KPL];
  bool real[KPL];
#pragma unroll
  for (int i = 0; i < KPL; ++i) {
    real[i] = q + TG * i < K;
    gam[i] = real[i] ? g0 : 0.0;
    psi[i] = m;
    E[i] = real[i] ? 1.0 : 0.0;
  }
  for (int j = 0; j < nch; ++j) {
    const int n0 = j * W, n1 = min(n, n0 + W);
    double cs = 0.0;
    for (int p = n0; p < n1; ++p) cs += (double)crow[p];   // integer counts: exact in any order
#pragma unroll
    for (int i = 0; i < KPL; ++i) C[j][i] = real[i] ? cs / K : 0.0;
  }
  // one-word-ahead prefetch of (row, count); the word order wraps into the next sweep
  auto load_row = [&](int p, double (&b)[KPL]) {
    const double* brow = a.beta + (size_t)wrow[p] * KS;
#pragma unroll
    for (int i = 0; i < KPL; ++i) b[i] = (q + TG * i < KS) ? brow[q + TG * i] : 0.0;
  };
  double bn[KPL];
  double cn = 0.0;
  if (n > 0) {
    load_row(0, bn);
    cn = (double)crow[0];
  }
  double L = 0.0, L_old = 0.0, conv = 1.0, GS = 0.0;
  int it = 0;
  while (var_continue(conv, vconv, it, vmi)) {
    ++it;
    double lw = 0.0;
#pragma unroll
    for (int i = 0; i < KPL; ++i) lps[i] = 0.0;
    for (int j = 0; j < nch; ++j) {
      const int n0 = j * W, n1 = min(n, n0 + W);
      double acc[KPL];
#pragma unroll
      for (int i = 0; i < KPL; ++i) acc[i] = 0.0;
      for (int p = n0; p < n1; ++p) {
        double b[KPL];
#pragma unroll
        for (int i = 0; i < KPL; ++i) b[i] = bn[i];
        const double c = cn;
        const int pn = p + 1 < n ? p + 1 : 0;
        load_row(pn, bn);
        cn = (double)crow[pn];
        double pp = 0.0;
#pragma unroll
        for (int i = 0; i < KPL; ++i) pp = fma(E[i], b[i], pp);
        const double P = bits_sum<0, 4, false>(pp);
        const double r = c * drcp(P);
        lw = fma(c, flog(P), lw);
#pragma unroll
        for (int i = 0; i < KPL; ++i) acc[i] = fma(r, b[i], acc[i]);
      }
      // branch-free refresh (interleaved chains; padding topics: E = 0, nw = 0, psi stays m)
#pragma unroll
      for (int i = 0; i < KPL; ++i) {
        const double nw = E[i] * acc[i];
        Et[j][i] = E[i];
        lps[i] = fma(psi[i], nw, lps[i]);
        gam[i] += nw - C[j][i];
        double pn, en;
        psi_exp(real[i] ? gam[i] : 1.0, m, pn, en);
        psi[i] = real[i] ? pn : psi[i];
        E[i] = real[i] ? en : 0.0;
        C[j][i] = nw;
      }
    }
    double gs = 0.0, lg = 0.0, lp = 0.0;
#pragma unroll
    for (int i = 0; i < KPL; ++i) {
      if (real[i]) {
        gs += gam[i];
        lg += lgamma_pos(gam[i]);
        lp += lps[i];
      }
    }
    GS = bits_sum<0, 4, false>(gs);
    lg = bits_sum<0, 4, false>(lg);
    lp = bits_sum<0, 4, false>(lp);
    L = lik_const - lgamma_pos(GS) + lg + fma(m, total, lw) - lp;
    conv = (L_old - L) / L_old;
    L_old = L;
  }
  double ps = 0.0;
#pragma unroll
  for (int i = 0; i < KPL; ++i) {
    const int k = q + TG * i;
    if (real[i]) ps += psi[i];
    if (k < KS) a.gamma[(size_t)d * KS + k] = gam[i];
  }
  ps = bits_sum<0, 4, false>(ps);
  if (q == 0) {
    a.lik[d] = L;
    a.alpha_ss[d] = ps - K * psi_only(GS);
    a.iters[d] = it;
  }
  // final pass: c_n phi_nk = E_jk b_nk r_n with the final sweep's chunk E
  for (int j = 0; j < nch; ++j) {
    const int n0 = j * W, n1 = min(n, n0 + W);
    for (int p = n0; p < n1; ++p) {
      double b[KPL];
      load_row(p, b);
      double pp = 0.0;
#pragma unroll
      for (int i = 0; i < KPL; ++i) pp = fma(Et[j][i], b[i], pp);
      const double r = (double)crow[p] * drcp(bits_sum<0, 4, false>(pp));
      double* row = a.cphi + (size_t)(s0 + p) * KS;
#pragma unroll
      for (int i = 0; i < KPL; ++i)
        if (q + TG * i < KS) __builtin_nontemporal_store(Et[j][i] * b[i] * r, &row[q + TG * i]);
    }
  }
}

// ----------------------------------------------------------------- chain ----
// lda-c's per-word schedule and chunks of a few words at K > 32 (U > 32): one wave per document, lane l
// holding topics l and l + 64 (TC = ceil(KS / 64)).  A chunk's P is a full-wave sum, the refresh TC
// digamma/exp chains per lane with E, gamma, psi in registers: no LDS, no barrier.  At U = 1024 a document of
// 257-4,096 words is a chain of up to 1,024 refreshes per sweep; the one-wave team paid an LDS round trip
// each way per chunk and waited on the row of the next word, gathered one chunk (= one word) ahead (r5h:
// 3.9 k cycles per chunk).  Here the rows of the next D words are in flight in a register ring (their ids D
// words further ahead), so a chunk costs its arithmetic.  Chunk tables in the document's own c*phi rows:
// C_j in row j W, the E chunk j used in row j W + 1 (chunks of >= 2 words); every row access is by the lane
// owning the topic.  Words wrap into the next sweep (a stopped run discards D prefetched rows).
template <int KS, int D>
__global__ __launch_bounds__(256) void gs_chain(GSArgs a) {
  static_assert(KS <= 128, "gs_chain: KS <= 128");
  constexpr int TC = (KS + 63) / 64;
  // TC = 2: lane l holds the topic pair 2l, 2l + 1 and loads it with one 16-byte load (KS even)
  constexpr bool PAIR = TC == 2;
  __shared__ dvec2 sLog[kMathTabN];      // flog_t's table
  if (a.params[kParamDone] != 0.0) return;
  log_table_fill(sLog);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int item = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (item >= a.n_items) return;   // whole waves leave together
  const double alpha = a.params[0], lik_const = a.params[1];
  const int vmi = (int)a.params[2];
  const double vconv = params_vconv(a.params);
  const int K = a.K;
  const int d = a.order[item];
  if (d < 0) return;
  const int s0 = a.doc_ptr[d], n = a.doc_ptr[d + 1] - s0;
  if (n <= 0) return;              // (the planner never sends an empty document)
  const int U = a.gs_updates;
  const int W = (n + U - 1) / U;
  const int nch = (n + W - 1) / W;
  const int* __restrict__ wrow = a.word_idx + s0;
  const float* __restrict__ crow = a.counts + s0;
  double* __restrict__ rows = a.cphi + (size_t)s0 * KS;
  auto topic = [&](int o) -> int { return PAIR ? 2 * lane + o : lane + 64 * o; };
  auto owned = [&](int o) { return topic(o) < KS; };
  // a word's TC values of this lane (lanes past KS read into the next row: beta's pad row)
  auto row_of = [&](int w, double (&v)[TC]) {
    if constexpr (PAIR) {
      const dvec2 x = *reinterpret_cast<const dvec2*>(a.beta + (size_t)w * KS + 2 * lane);
      v[0] = x.x;
      v[1] = x.y;
    } else if constexpr (KS >= 64) {
      v[0] = a.beta[(size_t)w * KS + lane];
    } else {
      // KS <= 32 (lda-c's per-word schedule at K <= 32): lanes past KS hold no topic and read nothing
      // (64 - KS of them would run past beta's one pad row)
      v[0] = lane < KS ? a.beta[(size_t)w * KS + lane] : 0.0;
    }
  };
  double total = 0.0;
  for (int j = 0; j < nch; ++j) {
    const int n0 = j * W, n1 = min(n, n0 + W);
    double cs = 0.0;
    for (int p = n0; p < n1; ++p) cs += (double)crow[p];   // integer counts: exact
    total += cs;
#pragma unroll
    for (int o = 0; o < TC; ++o)
      if (owned(o)) rows[(size_t)n0 * KS + topic(o)] = topic(o) < K ? cs / K : 0.0;
  }
  const double g0 = alpha + total / K;
  const double m = psi_only(g0);
  double gam[TC], psi[TC], E[TC], Cn[TC], acc[TC];
#pragma unroll
  for (int o = 0; o < TC; ++o) {
    const int k = topic(o);
    gam[o] = k < K ? g0 : 0.0;
    psi[o] = m;
    E[o] = k < K ? 1.0 : 0.0;
    Cn[o] = owned(o) ? rows[k] : 0.0;   // C_0 (this lane's own store)
    acc[o] = 0.0;
  }
  // rings: rb / rc the rows and counts of words g .. g + D - 1, wi / wc the ids and counts of words
  // g + D .. g + 2D - 1 (word g in slot g mod D); beta's pad row covers the lanes past KS
  double rb[D][TC], rc[D];
  int wi[D];
  float wc[D];
#pragma unroll
  for (int t = 0; t < D; ++t) {
    const int p = t % n;
    row_of(wrow[p], rb[t]);
    rc[t] = (double)crow[p];
    const int p2 = (t + D) % n;
    wi[t] = wrow[p2];
    wc[t] = crow[p2];
  }
  double L = 0.0, L_old = 0.0, conv = 1.0, GS = 0.0;
  double lw = 0.0, lp = 0.0;
  int pw = 0, j = 0;               // word of the sweep, its chunk
  int cend = min(n, W);            // end of chunk j
  int g2 = 2 * D;                  // the word whose id the slot being consumed loads next (mod n)
  bool run = var_continue(conv, vconv, 0, vmi);
  int it = run ? 1 : 0;            // sweeps begun
  while (run) {
#pragma unroll
    for (int t = 0; t < D; ++t) {
      if (run) {
        // word pw: P over the whole wave, then its contribution to the chunk
        double pp = 0.0;
#pragma unroll
        for (int o = 0; o < TC; ++o) pp = fma(E[o], rb[t][o], pp);
        const double P = group_sum<64>(pp);
        const double c = rc[t];
        const double r = c * drcp(P);
        lw = fma(c, flog_t(P, sLog), lw);
#pragma unroll
        for (int o = 0; o < TC; ++o) acc[o] = fma(r, rb[t][o], acc[o]);
        // the slot's next row (word pw + D) and the id D words beyond it
        {
          row_of(wi[t], rb[t]);
          rc[t] = (double)wc[t];
          const int p2 = g2 % n;
          wi[t] = wrow[p2];
          wc[t] = crow[p2];
          ++g2;
        }
        if (++pw == cend) {
          // chunk j ends: its tables, then the refresh (branch-free: padding topics keep E = 0)
          const int n0 = j * W;
          const bool two = cend - n0 >= 2;
#pragma unroll
          for (int o = 0; o < TC; ++o) {
            if (owned(o)) {
              rows[(size_t)n0 * KS + topic(o)] = E[o] * acc[o];
              if (two) rows[(size_t)(n0 + 1) * KS + topic(o)] = E[o];
            }
          }
#pragma unroll
          for (int o = 0; o < TC; ++o) {
            const bool real = topic(o) < K;
            const double nw = E[o] * acc[o];
            lp = fma(psi[o], nw, lp);
            gam[o] = real ? gam[o] + (nw - Cn[o]) : gam[o];
            double pn, en;
            psi_exp<true>(real ? gam[o] : 1.0, m, pn, en, sLog);
            psi[o] = real ? pn : psi[o];
            E[o] = real ? en : 0.0;
            acc[o] = 0.0;
          }
          j = j + 1 < nch ? j + 1 : 0;
          cend = min(n, (j + 1) * W);
#pragma unroll
          for (int o = 0; o < TC; ++o) Cn[o] = owned(o) ? rows[(size_t)j * W * KS + topic(o)] : 0.0;
          if (pw == n) {
            // sweep end: lda-c's likelihood and convergence test
            double gs = 0.0, lg = 0.0;
#pragma unroll
            for (int o = 0; o < TC; ++o) {
              const bool real = topic(o) < K;
              const double l = lgamma_pos<true>(real ? gam[o] : 1.0, sLog);
              gs += real ? gam[o] : 0.0;
              lg += real ? l : 0.0;
            }
            GS = group_sum<64>(gs);
            const double LG = group_sum<64>(lg), LP = group_sum<64>(lp);
            L = lik_const - lgamma_pos(GS) + LG + fma(m, total, lw) - LP;
            conv = (L_old - L) / L_old;
            L_old = L;
            run = var_continue(conv, vconv, it, vmi);
            it += run ? 1 : 0;
            pw = 0;
            lw = 0.0;
            lp = 0.0;
          }
        }
      }
    }
  }
  double ps = 0.0;
#pragma unroll
  for (int o = 0; o < TC; ++o) {
    const int k = topic(o);
    if (k < K) ps += psi[o];
    if (owned(o)) a.gamma[(size_t)d * KS + k] = gam[o];
  }
  ps = group_sum<64>(ps);
  if (lane == 0) {
    a.lik[d] = L;
    a.alpha_ss[d] = ps - K * psi_only(GS);
    a.iters[d] = it;
  }
  // final pass over chunks of >= 2 words: c_n phi_nk = E_jk b_nk r_n with the final sweep's chunk E
  if (W < 2) return;
  for (int jj = 0; jj < nch; ++jj) {
    const int n0 = jj * W, n1 = min(n, n0 + W);
    if (n1 - n0 < 2) continue;
    double Ej[TC];
#pragma unroll
    for (int o = 0; o < TC; ++o) Ej[o] = owned(o) ? rows[(size_t)(n0 + 1) * KS + topic(o)] : 0.0;
    for (int p = n0; p < n1; ++p) {
      double b[TC], pp = 0.0;
      row_of(wrow[p], b);
#pragma unroll
      for (int o = 0; o < TC; ++o) pp = fma(Ej[o], b[o], pp);
      const double rr = (double)crow[p] * drcp(group_sum<64>(pp));
#pragma unroll
      for (int o = 0; o < TC; ++o)
        if (owned(o)) __builtin_nontemporal_store(Ej[o] * b[o] * rr, &rows[(size_t)p * KS + topic(o)]);
    }
  }
}

// ---------------------------------------------------------- small, K > 32 ----
// The one-wave range at K > 32 (short documents; at lda-c's per-word schedule every document whose chunks
// hold <= 2 words): 16 lanes per document, KPL = ceil(KS / 16) topics per lane, four documents per wave,
// no LDS and no barrier.  The one-wave team (gs_team<KS, 1>) spreads a chunk's words over 4 word slots, then
// pays a cross-slot reduction and an LDS round trip per chunk and refreshes 2 topics per lane with 28 of
// 128 lane slots idle at K = 100; here the word loop runs in the document's 16 lanes and the refresh is
// KPL independent digamma/exp chains per lane (100 of 112 lane slots busy at K = 100).  Chunk tables live in
// the document's own c*phi rows (gs_team's GM layout): C_j in row j W, the E chunk j used in row j W + 1
// (chunks of >= 2 words); a one-word chunk's C_j IS that word's c*phi, so documents of <= U words need no
// final pass.  Every access to a row is by the lane that owns the topic (same-lane program order).
// RQ: words of the NEXT chunk whose rows are gathered during this chunk (ids one chunk earlier still); the
// rest of a chunk streams in batches of RQ.  Row loads are brow[q + 16 i] at constant offsets: lanes whose
// topic is >= KS read into the next row (beta carries one zero pad row, LDAEngine), values that only ever
// meet E = 0 / are never stored -- the clamped index held two address VGPRs per load.
template <int N, int KPL>
__device__ __forceinline__ void quad_word_steps(const double (&E)[KPL], const double (*b)[KPL], const double* c,
                                                double (&acc)[KPL], double& lw, const dvec2* __restrict__ tab) {
  double P[N];
#pragma unroll
  for (int u = 0; u < N; ++u) {
    double p0 = 0.0, p1 = 0.0;
#pragma unroll
    for (int i = 0; i < KPL; i += 2) p0 = fma(E[i], b[u][i], p0);
#pragma unroll
    for (int i = 1; i < KPL; i += 2) p1 = fma(E[i], b[u][i], p1);
    P[u] = bits_sum<0, 4, false>(p0 + p1);
  }
#pragma unroll
  for (int u = 0; u < N; ++u) {
    const double Pu = c[u] > 0.0 ? P[u] : 1.0;
    const double r = c[u] * drcp(Pu);
    lw = fma(c[u], flog_t(Pu, tab), lw);
#pragma unroll
    for (int i = 0; i < KPL; ++i) acc[i] = fma(r, b[u][i], acc[i]);
  }
}

template <int KS, int RQ, int MINW = 1>
__global__ __launch_bounds__(256, MINW) void gs_smallw(GSArgs a) {
  static_assert(KS > 32, "gs_smallw: KS > 32 (gs_small covers KS <= 32)");
  // one topic per 8-byte lane: the pair layout (TeamShape::PAIR) measured slower here (K = 100 bucket 9.48 vs
  // 8.99 ms, r5s: 8 topics per lane instead of 7 and 235 vs 196 VGPRs), the 16-lane kernel being refresh-bound
  constexpr bool PAIR = false;
  constexpr int TG = 16, KPL = PAIR ? 2 * ((KS + 2 * TG - 1) / (2 * TG)) : (KS + TG - 1) / TG;
  __shared__ dvec2 sLog[kMathTabN];          // flog_t's table
  if (a.params[kParamDone] != 0.0) return;
  log_table_fill(sLog);
  __syncthreads();
  const int t = threadIdx.x, q = t & (TG - 1);
  const int item = blockIdx.x * (256 / TG) + t / TG;
  if (item >= a.n_items) return;   // whole 16-lane groups leave together
  const double alpha = a.params[0], lik_const = a.params[1];
  const int vmi = (int)a.params[2];
  const double vconv = params_vconv(a.params);
  const int K = a.K;
  const int d = a.order[item];
  if (d < 0) return;
  const int s0 = a.doc_ptr[d], n = a.doc_ptr[d + 1] - s0;
  if (n <= 0) return;              // (the planner never sends an empty document)
  const int U = a.gs_updates;
  const int W = (n + U - 1) / U;
  const int nch = (n + W - 1) / W;
  const int* __restrict__ wrow = a.word_idx + s0;
  const float* __restrict__ crow = a.counts + s0;
  double* __restrict__ rows = a.cphi + (size_t)s0 * KS;
  // chunk count sums: C_j = cs_j / K into row j W (integer counts: the sums are exact in any order)
  double total = 0.0;
  for (int j = 0; j < nch; ++j) {
    const int n0 = j * W, n1 = min(n, n0 + W);
    double cs;
    if (W == 1) {
      cs = (double)crow[n0];
    } else {
      cs = 0.0;
      for (int p = n0 + q; p < n1; p += TG) cs += (double)crow[p];
      cs = bits_sum<0, 4, false>(cs);
    }
    total += cs;
#pragma unroll
    for (int i = 0; i < KPL; ++i) {
      const int k = tk<TG, PAIR>(q, i);
      if (k < KS) rows[(size_t)n0 * KS + k] = k < K ? cs / K : 0.0;
    }
  }
  const double g0 = alpha + total / K;
  const double m = psi_only(g0);
  double gam[KPL], psi[KPL], E[KPL], Cn[KPL];
#pragma unroll
  for (int i = 0; i < KPL; ++i) {
    const int k = tk<TG, PAIR>(q, i);
    gam[i] = k < K ? g0 : 1.0;   // padding topics hold gamma = 1 (finite refresh, never summed or stored)
    psi[i] = m;
    E[i] = k < K ? 1.0 : 0.0;
    Cn[i] = k < KS ? rows[k] : 0.0;   // C_0 (this lane's own stores above)
  }
  // head of a chunk: its first RQ words (past the chunk's end: count 0, the chunk's last row again)
  int wn[RQ];
  float cn[RQ];
  double bq[RQ][KPL], cq[RQ];
  auto head_ids = [&](int j) {
    const int n0 = j * W, n1 = min(n, n0 + W);
#pragma unroll
    for (int r = 0; r < RQ; ++r) {
      const int pc = min(n0 + r, n1 - 1);
      wn[r] = wrow[pc];
      cn[r] = n0 + r < n1 ? crow[pc] : 0.0f;
    }
  };
  auto head_rows = [&]() {
#pragma unroll
    for (int r = 0; r < RQ; ++r) {
      cq[r] = (double)cn[r];
      load_row<KS, KPL, TG, PAIR>(a.beta, wn[r], q, bq[r]);
    }
  };
  head_ids(0);
  head_rows();
  head_ids(nch > 1 ? 1 : 0);
  double L = 0.0, L_old = 0.0, conv = 1.0, GS = 0.0;
  int it = 0;
  while (var_continue(conv, vconv, it, vmi)) {
    ++it;
    double lw = 0.0, lp = 0.0;   // lp: sum of psi_k nw_jk over this lane's topics and the chunks
    for (int j = 0; j < nch; ++j) {
      const int n0 = j * W, n1 = min(n, n0 + W);
      double acc[KPL];
#pragma unroll
      for (int i = 0; i < KPL; ++i) acc[i] = 0.0;
      quad_word_steps<RQ, KPL>(E, bq, cq, acc, lw, sLog);
      // the rest of the chunk: batches of RQ rows, a batch's loads in flight together
      for (int p0 = n0 + RQ; p0 < n1; p0 += RQ) {
        double c[RQ];
#pragma unroll
        for (int r = 0; r < RQ; ++r) {
          const int pc = min(p0 + r, n1 - 1);
          c[r] = p0 + r < n1 ? (double)crow[pc] : 0.0;
          load_row<KS, KPL, TG, PAIR>(a.beta, wrow[pc], q, bq[r]);
        }
        quad_word_steps<RQ, KPL>(E, bq, c, acc, lw, sLog);
      }
      // next chunk's head rows in flight during the refresh; ids of the one after
      const int j1 = j + 1 < nch ? j + 1 : 0;
      head_rows();
      head_ids(j1 + 1 < nch ? j1 + 1 : 0);
      const bool two = n1 - n0 >= 2;
      // this chunk's C_j (and E_j) rows; lanes past KS exist only in the last topic group (static test)
#pragma unroll
      for (int i = 0; i < KPL; ++i) {
        const int k = tk<TG, PAIR>(q, i);
        if (k < KS) {
          rows[(size_t)n0 * KS + k] = E[i] * acc[i];
          if (two) rows[(size_t)(n0 + 1) * KS + k] = E[i];
        }
      }
      // the refresh without branches: a topic-guarded psi_exp is a basic block of its own, so the KPL
      // chains would run one after another instead of interleaved (padding topics keep gamma = 1
      // and E = 0: nw = 0 there)
#pragma unroll
      for (int i = 0; i < KPL; ++i) {
        const bool real = tk<TG, PAIR>(q, i) < K;
        const double nw = E[i] * acc[i];
        lp = fma(psi[i], nw, lp);
        gam[i] += nw - Cn[i];
        double p, e;
        // padding topics: gamma stays 1 (nw = 0, C = 0), psi finite and only ever multiplied by nw = 0
        psi_exp<true, true, false>(gam[i], m, p, e, sLog);
        psi[i] = p;
        E[i] = real ? e : 0.0;
      }
      // C of the next chunk, after this chunk's row stores (nch == 1: the same row)
#pragma unroll
      for (int i = 0; i < KPL; ++i) {
        const int k = tk<TG, PAIR>(q, i);
        Cn[i] = (k < KS) ? rows[(size_t)j1 * W * KS + k] : 0.0;
      }
    }
    double gs = 0.0, lg = 0.0;
#pragma unroll
    for (int i = 0; i < KPL; ++i) {
      const bool real = tk<TG, PAIR>(q, i) < K;
      const double l = lgamma_pos<true>(real ? gam[i] : 1.0, sLog);
      gs += real ? gam[i] : 0.0;
      lg += real ? l : 0.0;
    }
    GS = bits_sum<0, 4, false>(gs);
    lg = bits_sum<0, 4, false>(lg);
    lp = bits_sum<0, 4, false>(lp);
    L = lik_const - lgamma_pos(GS) + lg + fma(m, total, lw) - lp;
    conv = (L_old - L) / L_old;
    L_old = L;
  }
  double ps = 0.0;
#pragma unroll
  for (int i = 0; i < KPL; ++i) {
    const int k = tk<TG, PAIR>(q, i);
    if (k < K) ps += psi[i];
    if (k < KS) a.gamma[(size_t)d * KS + k] = k < K ? gam[i] : 0.0;
  }
  ps = bits_sum<0, 4, false>(ps);
  if (q == 0) {
    a.lik[d] = L;
    a.alpha_ss[d] = ps - K * psi_only(GS);
    a.iters[d] = it;
  }
  // final pass over chunks of >= 2 words: c_n phi_nk = E_jk b_nk r_n with the final sweep's chunk E
  // (read from row j W + 1 before the chunk's rows are overwritten; the same lane's addresses only)
  if (W < 2) return;
  for (int j = 0; j < nch; ++j) {
    const int n0 = j * W, n1 = min(n, n0 + W);
    if (n1 - n0 < 2) continue;
    double Ej[KPL];
#pragma unroll
    for (int i = 0; i < KPL; ++i) {
      const int k = tk<TG, PAIR>(q, i);
      Ej[i] = k < KS ? rows[(size_t)(n0 + 1) * KS + k] : 0.0;
    }
    for (int p0 = n0; p0 < n1; p0 += RQ) {
      double b[RQ][KPL], c[RQ];
#pragma unroll
      for (int r = 0; r < RQ; ++r) {
        const int pc = min(p0 + r, n1 - 1);
        c[r] = (double)crow[pc];
        load_row<KS, KPL, TG, PAIR>(a.beta, wrow[pc], q, b[r]);
      }
#pragma unroll
      for (int r = 0; r < RQ; ++r) {
        if (p0 + r >= n1) break;
        double pp0 = 0.0, pp1 = 0.0;
#pragma unroll
        for (int i = 0; i < KPL; i += 2) pp0 = fma(Ej[i], b[r][i], pp0);
#pragma unroll
        for (int i = 1; i < KPL; i += 2) pp1 = fma(Ej[i], b[r][i], pp1);
        const double rr = c[r] * drcp(bits_sum<0, 4, false>(pp0 + pp1));
        double* row = rows + (size_t)(p0 + r) * KS;
#pragma unroll
        for (int i = 0; i < KPL; ++i) {
          const int k = tk<TG, PAIR>(q, i);
          if (k < KS) __builtin_nontemporal_store(Ej[i] * b[r][i] * rr, &row[k]);
        }
      }
    }
  }
}

// ------------------------------------------------------------------ team ----
// Threads of a document team exchange data through LDS only (lds_barrier keeps the
// next chunk's prefetched global loads in flight across the barrier).
template <int NW>
__device__ __forceinline__ void team_sync() {
  if constexpr (NW == 1)
    wave_lds_sync();
  else
    lds_barrier();
}

constexpr int team_threads(int KS, int NW) { return ((NW == 1 && KS <= 32) ? 4 : 1) * NW * 64; }

template <int KS, int NW>
struct TeamShape {
  static constexpr int DPB = (NW == 1 && KS <= 32) ? 4 : 1;   // documents per workgroup
  static constexpr int NTD = NW * 64;                          // threads per document
  static constexpr int TG = tg_of(KS);
  // PAIR (TG >= 8, KS > 32): a lane holds topic PAIRS 2q, 2q + 1 (+ 2 TG per pair) and loads each pair with one
  // 16-byte load -- half the load instructions of one topic per 8-byte lane; the row gathers of the K = 100
  // team kernels are issue-bound (a chunk's prefetch issue 2.5-4.5 k cycles, profiles/r5_k100.md)
  static constexpr bool PAIR = TG >= 8;
  static constexpr int KPL = PAIR ? 2 * ((KS + 2 * TG - 1) / (2 * TG)) : kpl_of(KS);
  static constexpr int NSW = 64 / TG;                          // word slots per wave
  static constexpr int LSW = ilog2(NSW);
  static constexpr int NS = NW * NSW;                          // word slots per document
  static constexpr int TO = (KS + NTD - 1) / NTD;              // topics owned per thread
  // prefetched words per slot per chunk (even).  The 4-wave team keeps one round at KS > 32 too, although it runs
  // 2 waves per SIMD at any VGPR count up to 256 (171 with one round): 2 or 3 rounds (205 / 230 VGPRs) measured
  // slower on the K = 100 shard (team4 bucket 5.89 ms at 1, 6.01 at 2, 6.28 at 3; profiles/r6p_team4_rmax.md)
  static constexpr int RMAX = NW >= 8 ? (KPL <= 5 ? 8 : 4) : 1;
};

// N words of the word phase, interleaved (independent dependency chains): P = sum_k E_k b_k over
// the TG lanes of each slot, r = c / P, acc += r b, lw += c log P.  A word with c == 0 (no word in
// that round) contributes nothing (its P is replaced by 1 before the reciprocal).
template <int N, int KPL, int LSW, bool TAB = false>
__device__ __forceinline__ void word_steps(const double (&E)[KPL], const double (*b)[KPL], const double* c,
                                           double (&acc)[KPL], double& lw, const dvec2* tab = nullptr) {
  double P[N];
#pragma unroll
  for (int u = 0; u < N; ++u) {
    double p0 = 0.0, p1 = 0.0;
#pragma unroll
    for (int i = 0; i < KPL; i += 2) p0 = fma(E[i], b[u][i], p0);
#pragma unroll
    for (int i = 1; i < KPL; i += 2) p1 = fma(E[i], b[u][i], p1);
    P[u] = bits_sum<LSW, 6>(p0 + p1);
  }
#pragma unroll
  for (int u = 0; u < N; ++u) {
    const double Pu = c[u] > 0.0 ? P[u] : 1.0;
    const double r = c[u] * drcp(Pu);
    lw = fma(c[u], TAB ? flog_t(Pu, tab) : flog(Pu), lw);
#pragma unroll
    for (int i = 0; i < KPL; ++i) acc[i] = fma(r, b[u][i], acc[i]);
  }
}

// RMAX streamed words of one slot (p0, p0 + NS, ...; past `end` counts 0 and re-reads a valid row):
// ids, then rows, then the word steps, so a batch costs about one gather latency
template <int RMAX, int KS, int KPL, int TG, int LSW, bool PAIR, bool TAB = false>
__device__ __forceinline__ void stream_batch(const double* __restrict__ beta, const int* __restrict__ wrow,
                                             const float* __restrict__ crow, int p0, int end, int NS, int q,
                                             const double (&E)[KPL], double (&b)[RMAX][KPL], double (&acc)[KPL],
                                             double& lw, const dvec2* tab = nullptr) {
  int w[RMAX];
  double c[RMAX];
#pragma unroll
  for (int r = 0; r < RMAX; ++r) {
    const int p = p0 + r * NS;
    const int pc = min(p, end - 1);
    w[r] = wrow[pc];
    c[r] = p < end ? (double)crow[pc] : 0.0;
  }
#pragma unroll
  for (int r = 0; r < RMAX; ++r) load_row<KS, KPL, TG, PAIR>(beta, w[r], q, b[r]);
  word_steps<RMAX, KPL, LSW, TAB>(E, b, c, acc, lw, tab);
}

// the streamed tail of one slot: full batches while >= 2 rounds remain, the last round alone (a
// lone word in a full batch paid RMAX rows and word steps; measured on the split kernel)
template <int RMAX, int KS, int KPL, int TG, int LSW, bool PAIR, bool TAB = false>
__device__ __forceinline__ void stream_tail(const double* __restrict__ beta, const int* __restrict__ wrow,
                                            const float* __restrict__ crow, int p0, int end, int NS, int q,
                                            const double (&E)[KPL], double (&b)[RMAX][KPL], double (&acc)[KPL],
                                            double& lw, const dvec2* tab = nullptr) {
  int p = p0;
  if (p + NS < end) {
    // the ids of batch i + 1 load while batch i's rows are in flight: a batch then waits one memory latency
    // (its rows), not two (ids, then rows)
    int w[RMAX];
    double c[RMAX];
#pragma unroll
    for (int r = 0; r < RMAX; ++r) {
      const int pr = p + r * NS;
      const int pc = min(pr, end - 1);
      w[r] = wrow[pc];
      c[r] = pr < end ? (double)crow[pc] : 0.0;
    }
    for (; p + NS < end; p += RMAX * NS) {
#pragma unroll
      for (int r = 0; r < RMAX; ++r) load_row<KS, KPL, TG, PAIR>(beta, w[r], q, b[r]);
      double cb[RMAX];
      const int pn = p + RMAX * NS;
#pragma unroll
      for (int r = 0; r < RMAX; ++r) {
        cb[r] = c[r];
        const int pr = pn + r * NS;
        const int pc = max(0, min(pr, end - 1));
        w[r] = wrow[pc];
        c[r] = pr < end ? (double)crow[pc] : 0.0;
      }
      word_steps<RMAX, KPL, LSW, TAB>(E, b, cb, acc, lw, tab);
    }
  }
  if (p < end) {
    double b1[1][KPL];
    stream_batch<1, KS, KPL, TG, LSW, PAIR, TAB>(beta, wrow, crow, p, end, NS, q, E, b1, acc, lw, tab);
  }
}

// MINW: minimum waves per SIMD requested from the register allocator (the LDS-free one-wave team
// at K > 32 is latency-bound on its per-word refresh chains: 3 waves per SIMD, 13.2 -> 11.7 ms on the
// K = 100 shard; 4 spilled, 19.5 ms -- profiles/r2_k100_split.md)
template <int KS, int NW, int MINW = 1, bool GMT = false>
__global__ __launch_bounds__(team_threads(KS, NW), MINW) void gs_team(GSArgs a) {
  using T = TeamShape<KS, NW>;
  // (KS <= 32 GMT, the parity mode: 4 / 2 prefetched rounds -- 8 spilled 284 bytes at KS = 20, 4 at KS 24-32)
  constexpr int DPB = T::DPB, NTD = T::NTD, TG = T::TG, KPL = T::KPL, NSW = T::NSW, LSW = T::LSW, NS = T::NS,
                TO = T::TO, RMAX = (GMT && KS <= 32) ? (T::RMAX < (KS <= 20 ? 4 : 2) ? T::RMAX : (KS <= 20 ? 4 : 2))
                                                         : T::RMAX;
  constexpr bool PAIR = T::PAIR;
  // GM (one-wave documents at KS > 32, and every team size when GMT: U > kGsUMax refreshes per
  // sweep): the chunk tables live in the document's own c*phi rows instead of LDS (2 x 32 x KS
  // doubles of LDS held one wave per CU to ~3 waves; U chunks of them do not fit at all): C_j in
  // row j W, the E chunk j used in row j W + 1 (chunks of >= 2 words).  A one-word chunk's C_j IS
  // that word's c*phi (E_j r b), so documents of <= U words need no final pass at all.
  constexpr bool GM = GMT || (NW == 1 && KS > 32);
  // KS <= 32 with U > kGsUMax (lda-c's per-word schedule at K <= 32): the 4- and 8-wave teams only (DPB == 1,
  // so the early returns stay workgroup-uniform); the one-wave range goes to gs_chain there
  static_assert(!GMT || KS > 32 || NW > 1, "U > kGsUMax at KS <= 32: 4- and 8-wave team kernels only");
  constexpr int UT = GM ? 1 : kGsUMax;
  __shared__ double sC[DPB][UT][KS];         // chunk contributions (previous sweep)
  __shared__ double sEt[DPB][UT][KS];        // E each chunk used (final pass)
  __shared__ double sE[DPB][KS];             // current E, broadcast
  __shared__ double sRed[DPB][NW][KS];       // per-wave slot sums
  __shared__ double sCs[DPB][UT];            // chunk count sums (GM: straight into the C_j rows)
  __shared__ double sScal[DPB][NW][4];       // per-wave sweep partials
  // KS > 32: flog_t's table for the per-word log and the refresh (DPB == 1 there: the workgroup is one
  // document, so every early return below is workgroup-uniform)
  constexpr bool TAB = KS > 32;
  __shared__ dvec2 sLog[TAB ? kMathTabN : 1];
  if (a.params[kParamDone] != 0.0) return;
  if constexpr (TAB) {
    log_table_fill(sLog);
    __syncthreads();
  }
  const int t = threadIdx.x % NTD, ds = threadIdx.x / NTD;
  const int item = blockIdx.x * DPB + ds;
  if (item >= a.n_items) return;             // NW == 1: one wave per document (no block barriers)
  const double alpha = a.params[0], lik_const = a.params[1];
  const int vmi = (int)a.params[2];
  const double vconv = params_vconv(a.params);
  const int K = a.K;
  const int lane = t & 63, wv = t >> 6;
  const int q = lane >> LSW, sl = lane & (NSW - 1);
  const int slot = wv * NSW + sl;
  const int d = a.order[item];
  if (d < 0) return;   // XCD placement gap (GSPlan.xcd_gaps): this document slot only
  const int s0 = a.doc_ptr[d], n = a.doc_ptr[d + 1] - s0;
  const int U = a.gs_updates;
  const int W = n > 0 ? (n + U - 1) / U : 1;
  const int nch = (n + W - 1) / W;           // <= U (host-checked: <= kGsUMax unless GM)
  const int nact = min(NW, (W + NSW - 1) / NSW);   // waves holding words of a chunk
  const bool active = wv < nact;
  const int* __restrict__ wrow = a.word_idx + s0;
  const float* __restrict__ crow = a.counts + s0;
  double(*C)[KS] = sC[ds];
  double(*Et)[KS] = sEt[ds];
  double* E_ = sE[ds];
  double total = 0.0;
  if constexpr (GM) {
    // a thread per chunk: its count sum Cs_j, and C_j = Cs_j / K straight into row j W (any number
    // of chunks); the document total from the per-thread sums (integer counts: exact in any order)
    double part = 0.0;
    for (int j = t; j < nch; j += NTD) {
      const int n0 = j * W, n1 = min(n, n0 + W);
      double cs = 0.0;
      for (int p = n0; p < n1; ++p) cs += (double)crow[p];
      part += cs;
      double* row = a.cphi + (size_t)(s0 + n0) * KS;
      for (int k = 0; k < KS; ++k) row[k] = k < K ? cs / K : 0.0;
    }
    part = group_sum<64>(part);
    if constexpr (NW == 1) {
      total = part;
    } else {
      if (lane == 0) sScal[ds][wv][0] = part;
      __syncthreads();   // also orders the C_j row stores before the topic owners read them
#pragma unroll
      for (int v = 0; v < NW; ++v) total += sScal[ds][v][0];
      __syncthreads();
    }
  } else {
    double* Cs = sCs[ds];
    for (int j = t; j < nch; j += NTD) Cs[j] = 0.0;
    team_sync<NW>();
    // integer counts: the LDS double atomics are exact in any order
    for (int p = t; p < n; p += NTD) atomicAdd(&Cs[p / W], (double)crow[p]);
    team_sync<NW>();
    for (int j = 0; j < nch; ++j) total += Cs[j];
  }
  const double g0 = alpha + total / K;
  const double m = psi_only(g0);
  double gam[TO], psi[TO], lps[TO];
#pragma unroll
  for (int o = 0; o < TO; ++o) {
    const int k = t + NTD * o;
    gam[o] = k < K ? g0 : 0.0;
    psi[o] = m;
    lps[o] = 0.0;
    if (k < KS) {
      E_[k] = k < K ? 1.0 : 0.0;
      if constexpr (!GM) {
        for (int j = 0; j < nch; ++j) C[j][k] = k < K ? sCs[ds][j] / K : 0.0;
      }
    }
  }
  // GM: C of the next chunk, loaded one chunk ahead (NW == 1: this wave wrote it, same-address
  // order; NW > 1: behind the __syncthreads above)
  double Cn[TO];
  if constexpr (GM) {
#pragma unroll
    for (int o = 0; o < TO; ++o) {
      const int k = t + NTD * o;
      Cn[o] = (k < KS && nch > 0) ? a.cphi[(size_t)s0 * KS + k] : 0.0;
    }
  }
  // chunk-ahead prefetch: the beta rows of chunk j + 1 are in flight while chunk j reduces and
  // refreshes (chunks wrap into the next sweep); chunk j + 1's word ids are loaded at the START of
  // chunk j (after its counts left the registers) and land during its word phase.  (Ids loaded two
  // chunks ahead just before the barrier had to be rotated into the loop-carried registers at the
  // loop latch, and that copy made the compiler wait for every outstanding load -- the row prefetch
  // included -- before barrier 1, putting the row latency in front of the refresh.)  Loads are
  // unconditional (clamped indices); a round without a word has count 0 (its row is real but unused).
  int wc[RMAX];
  float cc[RMAX];
  unsigned vc = 0;                            // valid-round mask
  double bc[RMAX][KPL];
  auto load_ids = [&](int j, int (&w)[RMAX], float (&c)[RMAX], unsigned& v) {
    const int n0 = j * W, n1 = min(n, n0 + W);
    v = 0;
#pragma unroll
    for (int r = 0; r < RMAX; ++r) {
      const int p = n0 + slot + r * NS;
      v |= (active && p < n1) ? (1u << r) : 0u;
      // rounds past the chunk end re-read the chunk's last word: the same address as a valid
      // lane, so no extra row is gathered (clamping to the document end fetched the next chunk's rows)
      const int pc = min(p, n1 - 1);
      w[r] = wrow[pc];
      c[r] = crow[pc];
    }
  };
  auto load_rows = [&](const int (&w)[RMAX]) {
    if (!active) return;   // wave-uniform: waves without words of a chunk gather no rows
#pragma unroll
    for (int r = 0; r < RMAX; ++r) {
      load_row<KS, KPL, TG, PAIR>(a.beta, w[r], q, bc[r]);   // constant offsets (beta's pad row: gs_smallw)
    }
  };
  if (nch > 0) {
    load_ids(0, wc, cc, vc);
    load_rows(wc);
  }
  team_sync<NW>();
  double L = 0.0, L_old = 0.0, conv = 1.0, GS = 0.0;
  int it = 0;
  const bool timer = a.dbg != nullptr && blockIdx.x == 0 && threadIdx.x == 0;
  long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  long long tc = timer ? clock64() : 0;
  auto tick = [&](int i) {
    if (timer) {
      const long long x = clock64();
      ph[i] += x - tc;
      tc = x;
    }
  };
  while (var_continue(conv, vconv, it, vmi)) {
    ++it;
    double lw = 0.0;
#pragma unroll
    for (int o = 0; o < TO; ++o) lps[o] = 0.0;
    for (int j = 0; j < nch; ++j) {
      ph[7] += timer ? 1 : 0;
      if (active) {
        const int n0 = j * W, n1 = min(n, n0 + W);
        // this chunk's counts out of the id registers, then the next chunk's ids into them
        double cr[RMAX];
#pragma unroll
        for (int r = 0; r < RMAX; ++r) cr[r] = ((vc >> r) & 1u) ? (double)cc[r] : 0.0;
        load_ids(j + 1 < nch ? j + 1 : 0, wc, cc, vc);
        double E[KPL], acc[KPL];
#pragma unroll
        for (int i = 0; i < KPL; ++i) {
          E[i] = (tk<TG, PAIR>(q, i) < KS) ? E_[tk<TG, PAIR>(q, i)] : 0.0;
          acc[i] = 0.0;
        }
        // rounds of this chunk (team-uniform): pairs of words in flight per slot
        const int R = (n1 - n0 + NS - 1) / NS;
        if constexpr (RMAX == 1) {
          word_steps<1, KPL, LSW, TAB>(E, bc, cr, acc, lw, sLog);
        } else if (R > 2) {
          word_steps<RMAX, KPL, LSW, TAB>(E, bc, cr, acc, lw, sLog);    // every round in flight at once
        } else {
          word_steps<2, KPL, LSW, TAB>(E, bc, cr, acc, lw, sLog);
        }
        // words beyond the prefetched rounds (documents longer than RMAX * NS * U): streamed in
        // batches of RMAX rows per slot with a batch's loads in flight together (bc is free until
        // the next chunk's prefetch below); one row at a time left the word phase latency-bound
        stream_tail<RMAX, KS, KPL, TG, LSW, PAIR, TAB>(a.beta, wrow, crow, n0 + slot + RMAX * NS, n1, NS, q, E, bc, acc,
                                                        lw, sLog);
        // next chunk's rows (its ids landed during the word phase)
        load_rows(wc);
        tick(0);
        // whole active waves; a one-word chunk (lda-c's per-word schedule: every chunk of a document of
        // <= U words) has its word in slot 0 and exact zeros in the other slots, so the sum is slot 0's
        if (n1 - n0 > 1) {
#pragma unroll
          for (int i = 0; i < KPL; ++i) acc[i] = bits_sum<0, LSW, false>(acc[i]);
        }
        if (sl == 0) {
#pragma unroll
          for (int i = 0; i < KPL; ++i)
            if (tk<TG, PAIR>(q, i) < KS) sRed[ds][wv][tk<TG, PAIR>(q, i)] = acc[i];
        }
        tick(1);
      }
      team_sync<NW>();
      tick(2);
      // gather, then a branch-free refresh (TO > 1: the chains of a thread interleave; a topic-guarded
      // psi_exp is a basic block of its own), then the table stores.  Padding topics: Eo = 0, nw = 0,
      // gamma = 0, psi = m, E = 0.
      double nwv[TO], Eov[TO], Env[TO];
#pragma unroll
      for (int o = 0; o < TO; ++o) {
        const int k = t + NTD * o;
        const int kc = k < KS ? k : KS - 1;
        // all NW loads issued together (a dynamic loop serialises LDS round trips)
        double S = 0.0;
#pragma unroll
        for (int v = 0; v < NW; ++v) S += v < nact ? sRed[ds][v][kc] : 0.0;
        Eov[o] = k < KS ? E_[kc] : 0.0;
        nwv[o] = Eov[o] * S;
        const double Cj = GM ? Cn[o] : C[j][kc];
        const bool real = k < K;
        lps[o] = fma(psi[o], nwv[o], lps[o]);
        gam[o] = real ? gam[o] + (nwv[o] - Cj) : gam[o];
        double pn, en;
        psi_exp<TAB>(real ? gam[o] : 1.0, m, pn, en, sLog);
        psi[o] = real ? pn : psi[o];
        Env[o] = real ? en : 0.0;
      }
#pragma unroll
      for (int o = 0; o < TO; ++o) {
        const int k = t + NTD * o;
        if (k < KS) {
          if constexpr (GM) {
            double* crw = a.cphi + (size_t)(s0 + j * W) * KS;
            crw[k] = nwv[o];
            if (min(n, (j + 1) * W) - j * W >= 2) crw[KS + k] = Eov[o];
            const int j1 = j + 1 < nch ? j + 1 : 0;
            Cn[o] = a.cphi[(size_t)(s0 + j1 * W) * KS + k];
          } else {
            C[j][k] = nwv[o];
            Et[j][k] = Eov[o];
          }
          E_[k] = Env[o];
        }
      }
      tick(3);
      team_sync<NW>();
      tick(4);
    }
    // sweep likelihood: wave partials -> LDS -> every thread sums in wave order
    double gs = 0.0, lg = 0.0, lp = 0.0;
#pragma unroll
    for (int o = 0; o < TO; ++o) {
      if (t + NTD * o < K) {
        gs += gam[o];
        lg += lgamma_pos<TAB>(gam[o], sLog);
        lp += lps[o];
      }
    }
    const double w0 = group_sum<64>(q == 0 ? lw : 0.0);
    const double w1 = group_sum<64>(gs), w2 = group_sum<64>(lg), w3 = group_sum<64>(lp);
    if (lane == 0) {
      sScal[ds][wv][0] = w0;
      sScal[ds][wv][1] = w1;
      sScal[ds][wv][2] = w2;
      sScal[ds][wv][3] = w3;
    }
    team_sync<NW>();
    double LW = 0.0, LG = 0.0, LP = 0.0;
    GS = 0.0;
#pragma unroll
    for (int v = 0; v < NW; ++v) {
      LW += sScal[ds][v][0];
      GS += sScal[ds][v][1];
      LG += sScal[ds][v][2];
      LP += sScal[ds][v][3];
    }
    L = lik_const - lgamma_pos(GS) + LG + fma(m, total, LW) - LP;
    conv = (L_old - L) / L_old;
    L_old = L;
    team_sync<NW>();
    tick(5);
  }
  if (timer)
    for (int i = 0; i < 8; ++i) a.dbg[i] = ph[i];
  // outputs
  double ps = 0.0;
#pragma unroll
  for (int o = 0; o < TO; ++o) {
    const int k = t + NTD * o;
    if (k < K) ps += psi[o];
    if (k < KS) a.gamma[(size_t)d * KS + k] = gam[o];
  }
  ps = group_sum<64>(ps);
  if (lane == 0) sScal[ds][wv][0] = ps;
  team_sync<NW>();
  if (t == 0) {
    double PS = 0.0;
    for (int v = 0; v < NW; ++v) PS += sScal[ds][v][0];
    a.lik[d] = L;
    a.alpha_ss[d] = PS - K * psi_only(GS);
    a.iters[d] = it;
  }
  // final pass: c_n phi_nk = E_jk b_nk r_n with the final sweep's chunk E (same P as the sweep)
  if constexpr (GM && NW > 1) {
    // every wave reads E_j from row n0 + 1 before any wave overwrites the chunk's rows: one
    // workgroup barrier per chunk, so the waves without words stay in the loop
    __syncthreads();   // the last sweep's C_j / E_j row stores (topic owners) before the reads
    for (int j = 0; j < nch; ++j) {
      const int n0 = j * W, n1 = min(n, n0 + W);
      if (n1 - n0 < 2) continue;           // team-uniform: a one-word chunk's row is its c*phi
      const double* er = a.cphi + (size_t)(s0 + n0 + 1) * KS;
      double E[KPL];
#pragma unroll
      for (int i = 0; i < KPL; ++i) E[i] = (tk<TG, PAIR>(q, i) < KS) ? er[tk<TG, PAIR>(q, i)] : 0.0;
      __syncthreads();
      if (active) {
        for (int p = n0 + slot; p < n1; p += NS) {
          const double* brow = a.beta + (size_t)wrow[p] * KS;
          const double c = (double)crow[p];
          double b[KPL];
#pragma unroll
          for (int i = 0; i < KPL; ++i) b[i] = (tk<TG, PAIR>(q, i) < KS) ? brow[tk<TG, PAIR>(q, i)] : 0.0;
          double pp = 0.0;
#pragma unroll
          for (int i = 0; i < KPL; ++i) pp = fma(E[i], b[i], pp);
          const double r = c * drcp(bits_sum<LSW, 6>(pp));
          double* row = a.cphi + (size_t)(s0 + p) * KS;
#pragma unroll
          for (int i = 0; i < KPL; ++i)
            if (tk<TG, PAIR>(q, i) < KS) __builtin_nontemporal_store(E[i] * b[i] * r, &row[tk<TG, PAIR>(q, i)]);
        }
      }
    }
    return;
  }
  if (!active) return;
  for (int j = 0; j < nch; ++j) {
    const int n0 = j * W, n1 = min(n, n0 + W);
    double E[KPL];
    if constexpr (GM) {
      // one-word chunk: its c*phi row already holds C_j; else E_j from row n0 + 1, read by the
      // whole wave before any lane overwrites the chunk's rows (the stores depend on the loads)
      if (n1 - n0 < 2) continue;
      const double* er = a.cphi + (size_t)(s0 + n0 + 1) * KS;
#pragma unroll
      for (int i = 0; i < KPL; ++i) E[i] = (tk<TG, PAIR>(q, i) < KS) ? er[tk<TG, PAIR>(q, i)] : 0.0;
    } else {
#pragma unroll
      for (int i = 0; i < KPL; ++i) E[i] = (tk<TG, PAIR>(q, i) < KS) ? Et[j][tk<TG, PAIR>(q, i)] : 0.0;
    }
    for (int p = n0 + slot; p < n1; p += NS) {
      const double* brow = a.beta + (size_t)wrow[p] * KS;
      const double c = (double)crow[p];
      double b[KPL];
#pragma unroll
      for (int i = 0; i < KPL; ++i) b[i] = (tk<TG, PAIR>(q, i) < KS) ? brow[tk<TG, PAIR>(q, i)] : 0.0;
      double pp = 0.0;
#pragma unroll
      for (int i = 0; i < KPL; ++i) pp = fma(E[i], b[i], pp);
      const double r = c * drcp(bits_sum<LSW, 6>(pp));
      double* row = a.cphi + (size_t)(s0 + p) * KS;
#pragma unroll
      for (int i = 0; i < KPL; ++i)
        if (tk<TG, PAIR>(q, i) < KS) __builtin_nontemporal_store(E[i] * b[i] * r, &row[tk<TG, PAIR>(q, i)]);
    }
  }
}

// ----------------------------------------------------------------- split ----
// One long document over G workgroups (K > 32).  Chunk j of a sweep
// (W = ceil(n / U) words) is cut into G contiguous ranges of ceil(W / G) words; workgroup g gathers
// and reduces its range's S_k = sum_n r_n b_nk and sum_n c_n log P_n, publishes them, and reads all
// G partials back in segment order (the same bits in every workgroup), so the G replicas of
// (gamma, psi, E, C) run the identical refresh and the identical lda-c convergence test: one
// exchange per chunk.  A double travels as two tagged 8-byte granules {uint32 half, uint32 tag}
// (relaxed agent-scope 64-bit stores / loads are single-copy atomic); tag = (launch epoch, chunk
// sequence number) (estep_common.h) and a parity double buffer: a workgroup reuses buffer (seq & 1)
// at seq + 2 only after every segment has published seq + 1, i.e. after every segment has finished
// reading seq.  The host caps a launch below the co-resident capacity (gs_split_capacity), so the
// exchange cannot deadlock; a bounded wait sets `error`.
__device__ __forceinline__ void put_tagged_bits(unsigned long long* p, unsigned v, unsigned tag) {
  __hip_atomic_store(p, ((unsigned long long)tag << 32) | (unsigned long long)v, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// Segment-order sums of the tagged doubles of TC columns (column c: granules x[u * stride + 2 c] and
// x[u * stride + 2 c + 1] = (lo, hi) bits of segment u's value, u < G <= GMX).  Every pass issues ALL
// TC x GMX x 2 loads back to back (unconditional, clamped indices) and then checks the tags; a pass that
// finds any stale granule is repeated whole.  Loads inside per-granule branches get a vmcnt(0) each -- one
// round trip per granule group; the round-3 form polled 4 segments per round trip, 2 x 4 serial round
// trips per chunk at G = 16, K = 100 (12.8 k cycles per chunk, profiles/r5f) -- and the microbenchmark
// (scripts/micro/xcd_exchange.hip) measured batched polls at half the per-granule form.  False on a timeout.
constexpr int kSplitMaxSeg = 16;   // GMX of the single-round gather (more: split_allreduce2)
template <int TC, int GMX, int NC>
__device__ __forceinline__ bool tagged_gather(const unsigned long long* x, int G, int stride, int lane, unsigned tag,
                                              double (&out)[TC]) {
  unsigned long long v[TC][GMX][2];
  long spins = 0;
  for (;;) {
#pragma unroll
    for (int o = 0; o < TC; ++o) {
      const int c = min(lane + 64 * o, NC - 1);
#pragma unroll
      for (int u = 0; u < GMX; ++u) {
        const unsigned long long* p = x + (size_t)min(u, G - 1) * stride + 2 * c;
        v[o][u][0] = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        v[o][u][1] = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    bool ok = true;
#pragma unroll
    for (int o = 0; o < TC; ++o)
#pragma unroll
      for (int u = 0; u < GMX; ++u)
        ok &= u >= G || ((unsigned)(v[o][u][0] >> 32) == tag && (unsigned)(v[o][u][1] >> 32) == tag);
    if (ok) break;
    if (++spins > kSplitSpinLimit) {
#pragma unroll
      for (int o = 0; o < TC; ++o) out[o] = __builtin_nan("");
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
#pragma unroll
  for (int o = 0; o < TC; ++o) {
    double s = 0.0;
#pragma unroll
    for (int u = 0; u < GMX; ++u)
      if (u < G)
        s += __longlong_as_double((long long)(((v[o][u][1] & 0xffffffffull) << 32) | (v[o][u][0] & 0xffffffffull)));
    out[o] = s;
  }
  return true;
}

// Two-phase exchange for G > kSplitMaxSeg segments (up to kSplitMaxSeg2): a single-round gather reads
// G x NC x 2 granules per segment -- linear in G, and past 16 segments more than the topic wave's registers
// can keep in flight -- so the columns are owned instead: segment g reduces columns c = g + G x (x < nown)
// over the G published partials (reduce-scatter: ~NC x 2 granules per segment, <= 4 per lane, all in one
// batched poll), publishes each owned total once with the chunk's tag into the document's totals row, and
// every segment then gathers the NC totals (all-gather: NC x 2 granules).  Two round trips whatever G is;
// each total is computed by exactly one segment, so every replica reads the same bits.  Buffer reuse: the
// totals row (seq & 1) is rewritten at seq + 2 only after its owner has read every segment's seq + 2
// partial, which a segment publishes only after it has gathered the seq + 1 totals, i.e. after it has
// finished reading seq's.  sPair: LDS scratch of >= NC + kSplitMaxSeg2 doubles (the topic wave only).
constexpr int kSplitMaxSeg2 = 128;   // two-phase exchange: two segments per topic-wave lane
template <int TC, int NC, int GR>
__device__ __forceinline__ bool split_allreduce2(const unsigned long long* __restrict__ xs, unsigned long long* xt,
                                                 int G, int g, int lane, unsigned tag, double* sPair,
                                                 double (&out)[TC]) {
  // pairs (column, segment) per lane: nown x G < NC + G when G < NC, = G <= kSplitMaxSeg2 otherwise, and
  // < 2 NC when NC / 2 < G < NC (nown = 2)
  constexpr int PMAX = ((2 * NC > kSplitMaxSeg2 ? 2 * NC : kSplitMaxSeg2) + 63) / 64;
  const int nown = g < NC ? (NC - 1 - g) / G + 1 : 0;        // uniform across the wave
  const int npair = nown * G;
  if (npair > 0) {
    int off[PMAX];
#pragma unroll
    for (int o = 0; o < PMAX; ++o) {
      const int i = min(lane + 64 * o, npair - 1);
      const int x = i / G, u = i - x * G;
      off[o] = u * GR + 2 * (g + G * x);
    }
    unsigned long long v[PMAX][2];
    long spins = 0;
    for (;;) {
#pragma unroll
      for (int o = 0; o < PMAX; ++o) {
        v[o][0] = __hip_atomic_load(xs + off[o], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        v[o][1] = __hip_atomic_load(xs + off[o] + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      bool ok = true;
#pragma unroll
      for (int o = 0; o < PMAX; ++o)
        ok &= lane + 64 * o >= npair || ((unsigned)(v[o][0] >> 32) == tag && (unsigned)(v[o][1] >> 32) == tag);
      if (ok) break;
      if (++spins > kSplitSpinLimit) {
#pragma unroll
        for (int o = 0; o < TC; ++o) out[o] = __builtin_nan("");
        return false;
      }
      __builtin_amdgcn_s_sleep(1);
    }
#pragma unroll
    for (int o = 0; o < PMAX; ++o)
      if (lane + 64 * o < npair)
        sPair[lane + 64 * o] =
            __longlong_as_double((long long)(((v[o][1] & 0xffffffffull) << 32) | (v[o][0] & 0xffffffffull)));
    wave_lds_sync();
    for (int x = 0; x < nown; ++x) {
      double s = (lane < G ? sPair[x * G + lane] : 0.0) + (lane + 64 < G ? sPair[x * G + lane + 64] : 0.0);
      s = group_sum<64>(s);   // fixed DPP tree: computed once, by this owner
      if (lane == 0) {
        const unsigned long long bits = (unsigned long long)__double_as_longlong(s);
        unsigned long long* row = xt + 2 * (g + G * x);
        put_tagged_bits(row, (unsigned)(bits & 0xffffffffull), tag);
        put_tagged_bits(row + 1, (unsigned)(bits >> 32), tag);
      }
    }
    wave_lds_sync();
  }
  return tagged_gather<TC, 1, NC>(xt, 1, GR, lane, tag, out);
}

// ------------------------------------------------------------ split kernel ----
// 7 word waves + 1 topic wave: the word waves leave their chunk partials in LDS, signal an LDS arrival
// counter and issue the NEXT chunk's row prefetch at once; the topic wave sums the waves, publishes the
// segment's tagged granules, sweeps the document's G segments and runs the refresh.  Its poll loads
// never queue behind row prefetches (vmcnt is in order per wave, and the hand-off price sits in the
// consumer's memory queue -- MI355X_MICROARCH handoff-1to1 / gather-pass), and a chunk costs one
// workgroup barrier.  (The round-2 form with all three roles in the same eight waves and three barriers
// per chunk was 3.82 vs 3.17 ms on the K = 50 split bucket and is gone; profiles/r3_tuning_log.md.)
// UM: chunk-table rows in LDS (U <= UM): 32, or 64 where 2 x 64 x KS doubles still fit the 64 KB of
// static LDS (KS <= 52: K = 50 at U = 64, the schedule that meets lda-c parity there,
// profiles/r3_precision_parity.md).  GM (U > UM at KS > 32, lda-c's per-word schedule): the chunk tables
// move to the launch's per-segment scratch sp.tab ([n_blocks][U][C_j | E_j][KS]; each replica reads only
// what it wrote itself) and C_j is loaded one chunk ahead, as gs_team's c*phi-row layout does.
template <int KS, int UM = kGsUMax, bool GM = false>
__global__ __launch_bounds__(512) void gs_splitw(GSArgs a, SplitArgs sp) {
  using T = TeamShape<KS, 8>;   // word-slot geometry and prefetch depth of the 8-wave team
  constexpr int NW = 7, NTD = (NW + 1) * 64, TG = T::TG, KPL = T::KPL, NSW = T::NSW, LSW = T::LSW, NS = NW * NSW,
                RMAX = T::RMAX;
  constexpr bool PAIR = T::PAIR;
  constexpr int NC = KS + 1;                 // exchanged columns: KS topic sums + the log-sum
  constexpr int GR = 2 * NC;                 // granules per segment row
  constexpr int TC = (NC + 63) / 64;         // columns per topic-wave lane
  constexpr int UT = GM ? 1 : UM;             // LDS chunk-table rows
  __shared__ double sC[UT][KS];
  __shared__ double sEt[UT][KS];
  __shared__ double sE[KS];
  __shared__ double sRed[NW][KS];
  __shared__ double sRedL[NW];
  __shared__ double sCs[GM ? kGsUMaxWide : UM];
  __shared__ double sScal[4];
  __shared__ int arrive[NW];   // per word wave: chunks whose partial sums it has left in sRed / sRedL
  __shared__ int sFail;
  __shared__ double sPair[KS > 32 ? 2 * NC + kSplitMaxSeg2 : 1];   // the two-phase exchange's values
  if (a.params[kParamDone] != 0.0) return;
  const int t = threadIdx.x, b = blockIdx.x;
  const int d = sp.seg_doc[b], g = sp.seg_index[b], G = sp.seg_count[b], base = sp.seg_base[b];
  const int dslot = sp.doc_slot[b];
  int* counter = sp.counter + dslot;
  const int epoch = __hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const double alpha = a.params[0], lik_const = a.params[1];
  const int vmi = (int)a.params[2];
  const double vconv = params_vconv(a.params);
  const int K = a.K;
  auto kc_ = [](int k) { return k < KS ? k : KS - 1; };   // an in-bounds LDS column for guarded reads
  const int lane = t & 63, wv = t >> 6;
  const bool topic_wave = wv == NW;
  const int q = lane >> LSW, sl = lane & (NSW - 1);
  const int slot = wv * NSW + sl;
  const int s0 = a.doc_ptr[d], n = a.doc_ptr[d + 1] - s0;   // n > 0 (host)
  const int U = a.gs_updates;
  const int W = (n + U - 1) / U;
  const int nch = (n + W - 1) / W;
  const int WG = (W + G - 1) / G;             // words of a chunk per segment
  const int nact = min(NW, (WG + NSW - 1) / NSW);
  const bool active = wv < nact;              // never the topic wave
  const int* __restrict__ wrow = a.word_idx + s0;
  const float* __restrict__ crow = a.counts + s0;
  // row j: C_j, then E_j; sp.tab_rows >= every batch document's nch (GSSplitPlan)
  double* __restrict__ tab = GM ? sp.tab + (size_t)b * sp.tab_rows * 2 * KS : nullptr;
  auto range = [&](int j, int& m0, int& m1) {
    const int n1 = min(n, (j + 1) * W);
    m0 = min(n1, j * W + g * WG);
    m1 = min(n1, m0 + WG);
  };
  if (GM && nch > sp.tab_rows) {   // a host plan error: every segment of d leaves (same nch), none waits
    if (t == 0) __hip_atomic_store(sp.error, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  if (sp.csum) {
    // the chunk count sums the plan computed once (GSSplitPlan.chunk_sums): no pass over the whole
    // document's counts in every segment (443 k words x 124 segments at config 5)
    const double* cs = sp.csum + (size_t)dslot * sp.csum_stride;
    for (int j = t; j < nch; j += NTD) sCs[j] = cs[j];
    if (t == 0) sFail = 0;
    if (t < NW) arrive[t] = 0;
  } else {
    for (int j = t; j < nch; j += NTD) sCs[j] = 0.0;
    if (t == 0) sFail = 0;
    if (t < NW) arrive[t] = 0;
    lds_barrier();
    for (int p = t; p < n; p += NTD) atomicAdd(&sCs[p / W], (double)crow[p]);   // integer counts: exact
  }
  lds_barrier();
  double total = 0.0;
  for (int j = 0; j < nch; ++j) total += sCs[j];
  const double g0 = alpha + total / K;
  const double m = psi_only(g0);
  const bool twt = a.dbg != nullptr && b == 0 && t == NW * 64;   // topic-wave timer lane
  const bool wwt = a.dbg != nullptr && b == 0 && t == 0;         // word-wave timer lane
  long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  long long tc = (twt || wwt) ? clock64() : 0;
  auto tick = [&](int i) {
    if (twt || wwt) {
      const long long x = clock64();
      ph[i] += x - tc;
      tc = x;
    }
  };
  double L = 0.0, L_old = 0.0, conv = 1.0, GS = 0.0;
  int it = 0;
  bool failed = false;
  auto sweep_end = [&]() {
    lds_barrier();
    GS = sScal[1];
    L = lik_const - lgamma_pos(GS) + sScal[2] + fma(m, total, sScal[0]) - sScal[3];
    conv = (L_old - L) / L_old;
    L_old = L;
    lds_barrier();
  };
  if (topic_wave) {
    // ------------------------------------------------------------ topic wave
    __builtin_amdgcn_s_setprio(3);   // its chain is the critical path; the word waves wait on it
    double gam[TC], psi[TC], lps[TC], Cn[TC];
#pragma unroll
    for (int o = 0; o < TC; ++o) {
      const int k = lane + 64 * o;
      gam[o] = k < K ? g0 : 0.0;
      psi[o] = m;
      lps[o] = 0.0;
      Cn[o] = 0.0;
      if (k < KS) {
        sE[k] = k < K ? 1.0 : 0.0;
        for (int j = 0; j < nch; ++j) {
          const double c0 = k < K ? sCs[j] / K : 0.0;
          if constexpr (GM)
            tab[(size_t)j * 2 * KS + k] = c0;
          else
            sC[j][k] = c0;
        }
        if constexpr (GM) Cn[o] = tab[k];   // C_0 (this lane's own store)
      }
    }
    double LWs = 0.0;
    int want = 0;
    lds_barrier();   // (1)
    while (!failed && var_continue(conv, vconv, it, vmi)) {
      ++it;
#pragma unroll
      for (int o = 0; o < TC; ++o) lps[o] = 0.0;
      for (int j = 0; j < nch; ++j) {
        ph[7] += twt ? 1 : 0;
        ++want;
        // this chunk's C_jk and E_k before the waits (the LDS reads are off the chain)
        double gC[TC], Eo[TC];
#pragma unroll
        for (int o = 0; o < TC; ++o) {
          const int k = lane + 64 * o;
          gC[o] = k < KS ? gam[o] - (GM ? Cn[o] : sC[j][kc_(k)]) : 0.0;
          Eo[o] = k < KS ? sE[k] : 0.0;
        }
        // the segment's column sums, in wave order as the waves arrive (one add after the last)
        double part[TC];
#pragma unroll
        for (int o = 0; o < TC; ++o) part[o] = 0.0;
#pragma unroll
        for (int v = 0; v < NW; ++v) {
          if (v < nact) {
            while (__hip_atomic_load(&arrive[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < want)
              __builtin_amdgcn_s_sleep(1);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
#pragma unroll
            for (int o = 0; o < TC; ++o) {
              const int c = lane + 64 * o;
              part[o] += c < KS ? sRed[v][c] : (c == KS ? sRedL[v] : 0.0);
            }
          }
        }
        tick(3);
        const int seq = (it - 1) * nch + j + 1;
        const unsigned tag = split_tag(epoch, seq);
        unsigned long long* xb = sp.xchg + (size_t)(seq & 1) * sp.n_blocks * GR;
        // publish this segment's column sums, then sweep the G segments
#pragma unroll
        for (int o = 0; o < TC; ++o) {
          const int c = lane + 64 * o;
          if (c < NC) {
            const unsigned long long bits = (unsigned long long)__double_as_longlong(part[o]);
            unsigned long long* row = xb + (size_t)b * GR + 2 * c;
            put_tagged_bits(row, (unsigned)(bits & 0xffffffffull), tag);
            put_tagged_bits(row + 1, (unsigned)(bits >> 32), tag);
          }
        }
        // one batched pass over every column and segment up to 8 segments; past that a pass per column
        // (TC x 16 x 2 granules in flight spilled at K = 100)
        double tot[TC];
        const unsigned long long* xs = xb + (size_t)base * GR;
        bool ok = true;
        if (G <= 4) {
          ok = tagged_gather<TC, 4, NC>(xs, G, GR, lane, tag, tot);
        } else if (G <= 8) {
          ok = tagged_gather<TC, 8, NC>(xs, G, GR, lane, tag, tot);
        } else if (G <= kSplitMaxSeg) {
#pragma unroll
          for (int o = 0; o < TC; ++o) {
            double t1[1];
            ok &= tagged_gather<1, kSplitMaxSeg, NC>(xs, G, GR, lane + 64 * o, tag, t1);
            tot[o] = t1[0];
          }
        } else if constexpr (KS > 32) {
          // the document's totals row, after the launch's 2 x n_blocks partial rows (KS <= 32 splits take at
          // most kSplitMaxSeg segments: GSSplitPlan; the narrow word layout has no registers to spare for it)
          unsigned long long* xt = sp.xchg + (size_t)2 * sp.n_blocks * GR +
                                   ((size_t)(seq & 1) * sp.n_docs + dslot) * GR;
          ok = split_allreduce2<TC, NC, GR>(xs, xt, G, g, lane, tag, sPair, tot);
        } else {
          ok = false;
        }
        tick(4);
        if (!ok) {
          sFail = 1;
          __hip_atomic_store(sp.error, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        // branch-free refresh: the TC chains of a lane interleave (padding / log-sum columns have
        // Eo = 0: nw = 0, and keep gamma = 0, psi = m, E = 0)
        double En[TC];
#pragma unroll
        for (int o = 0; o < TC; ++o) {
          const bool real = lane + 64 * o < K;
          const double nw = Eo[o] * tot[o];
          lps[o] = fma(psi[o], nw, lps[o]);
          gam[o] = real ? fma(Eo[o], tot[o], gC[o]) : gam[o];   // gamma_k + (new_jk - C_jk) in one rounding
          double pn, en;
          psi_exp(real ? gam[o] : 1.0, m, pn, en);
          psi[o] = real ? pn : psi[o];
          En[o] = real ? en : 0.0;
        }
#pragma unroll
        for (int o = 0; o < TC; ++o) {
          const int k = lane + 64 * o;
          if (k < KS) {
            if constexpr (GM) {
              tab[(size_t)j * 2 * KS + k] = Eo[o] * tot[o];
              tab[(size_t)j * 2 * KS + KS + k] = Eo[o];
              Cn[o] = tab[(size_t)(j + 1 < nch ? j + 1 : 0) * 2 * KS + k];   // after the store (nch == 1)
            } else {
              sC[j][k] = Eo[o] * tot[o];
              sEt[j][k] = Eo[o];
            }
            sE[k] = En[o];
          } else if (k == KS) {
            LWs += tot[o];
          }
        }
        tick(5);
        lds_barrier();   // (B) E of chunk j + 1 published
        if (sFail) {
          failed = true;
          break;
        }
      }
      if (failed) break;
      double gs = 0.0, lg = 0.0, lp = 0.0, lw = 0.0;
#pragma unroll
      for (int o = 0; o < TC; ++o) {
        const int k = lane + 64 * o;
        if (k < K) {
          gs += gam[o];
          lg += lgamma_pos(gam[o]);
          lp += lps[o];
        }
        if (k == KS) lw = LWs;
      }
      LWs = 0.0;
      const double w1 = group_sum<64>(gs), w2 = group_sum<64>(lg), w3 = group_sum<64>(lp), w0 = group_sum<64>(lw);
      if (lane == 0) {
        sScal[0] = w0;
        sScal[1] = w1;
        sScal[2] = w2;
        sScal[3] = w3;
      }
      sweep_end();
      tick(6);
    }
    if constexpr (GM) __syncthreads();   // pairs with the word waves': the E_j table stores before their final pass
    if (twt)
      for (int i = 3; i < 8; ++i) a.dbg[i] = ph[i];
    split_exit(counter, sp.n_docs, G);   // thread 0 only: a no-op here (kept beside the word waves' call)
    double ps = 0.0;
#pragma unroll
    for (int o = 0; o < TC; ++o) {
      const int k = lane + 64 * o;
      if (k < K) ps += psi[o];
      if (g == 0 && k < KS) a.gamma[(size_t)d * KS + k] = gam[o];
    }
    ps = group_sum<64>(ps);
    if (g == 0 && lane == 0) {
      a.lik[d] = failed ? __builtin_nan("") : L;   // a timed-out exchange surfaces as a NaN likelihood
      a.alpha_ss[d] = ps - K * psi_only(GS);
      a.iters[d] = it;
    }
    return;
  }
  // -------------------------------------------------------------- word waves
  int wc[RMAX], wn[RMAX];
  float cc[RMAX], cn[RMAX];
  unsigned vc = 0, vn = 0;
  double bc[RMAX][KPL];
  auto load_ids = [&](int j, int (&w)[RMAX], float (&c)[RMAX], unsigned& v) {
    int m0, m1;
    range(j, m0, m1);
    v = 0;
#pragma unroll
    for (int r = 0; r < RMAX; ++r) {
      const int p = m0 + slot + r * NS;
      v |= (active && p < m1) ? (1u << r) : 0u;
      const int pc = max(0, min(p, m1 - 1));
      w[r] = wrow[pc];
      c[r] = crow[pc];
    }
  };
  auto load_rows = [&](const int (&w)[RMAX], unsigned v) {
    if (!active) return;
#pragma unroll
    for (int r = 0; r < RMAX; ++r) {
      // unconditional, constant offsets: a round past the range re-reads a valid row of the document
      // and carries count 0 (beta's pad row covers topic lanes past KS: gs_smallw)
      load_row<KS, KPL, TG, PAIR>(a.beta, w[r], q, bc[r]);
    }
  };
  load_ids(0, wc, cc, vc);
  load_rows(wc, vc);
  load_ids(nch > 1 ? 1 : 0, wn, cn, vn);
  lds_barrier();   // (1)
  while (!failed && var_continue(conv, vconv, it, vmi)) {
    ++it;
    for (int j = 0; j < nch; ++j) {
      if (active) {
        int m0, m1;
        range(j, m0, m1);
        double E[KPL], acc[KPL], lw = 0.0;
#pragma unroll
        for (int i = 0; i < KPL; ++i) {
          E[i] = (tk<TG, PAIR>(q, i) < KS) ? sE[tk<TG, PAIR>(q, i)] : 0.0;
          acc[i] = 0.0;
        }
        double cr[RMAX];
#pragma unroll
        for (int r = 0; r < RMAX; ++r) cr[r] = ((vc >> r) & 1u) ? (double)cc[r] : 0.0;
        const int R = (m1 - m0 + NS - 1) / NS;
        if (R <= 1) {
          word_steps<1, KPL, LSW>(E, bc, cr, acc, lw);
        } else if (R <= 2 || RMAX <= 2) {
          word_steps<(RMAX < 2 ? RMAX : 2), KPL, LSW>(E, bc, cr, acc, lw);
        } else if (R <= 4 || RMAX <= 4) {
          word_steps<(RMAX < 4 ? RMAX : 4), KPL, LSW>(E, bc, cr, acc, lw);
        } else {
          word_steps<RMAX, KPL, LSW>(E, bc, cr, acc, lw);
        }
        stream_tail<RMAX, KS, KPL, TG, LSW, PAIR>(a.beta, wrow, crow, m0 + slot + RMAX * NS, m1, NS, q, E, bc, acc, lw);
#pragma unroll
        for (int i = 0; i < KPL; ++i) acc[i] = bits_sum<0, LSW, false>(acc[i]);
        lw = group_sum<64>(q == 0 ? lw : 0.0);
        if (sl == 0) {
#pragma unroll
          for (int i = 0; i < KPL; ++i)
            if (tk<TG, PAIR>(q, i) < KS) sRed[wv][tk<TG, PAIR>(q, i)] = acc[i];
        }
        if (lane == 0) sRedL[wv] = lw;
        // arrival (LDS only: no vmcnt wait), then the next chunk's rows -- beside the exchange
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        if (lane == 0) __hip_atomic_fetch_add(&arrive[wv], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        tick(0);
        const int j1 = j + 1 < nch ? j + 1 : 0;
        const int j2 = j1 + 1 < nch ? j1 + 1 : 0;
#pragma unroll
        for (int r = 0; r < RMAX; ++r) {
          wc[r] = wn[r];
          cc[r] = cn[r];
        }
        vc = vn;
        load_rows(wc, vc);
        load_ids(j2, wn, cn, vn);
        tick(1);
      }
      lds_barrier();   // (B)
      tick(2);
      if (sFail) {
        failed = true;
        break;
      }
    }
    if (failed) break;
    sweep_end();
  }
  if constexpr (GM) __syncthreads();     // the topic wave's E_j table stores are visible past this
  if (wwt)
    for (int i = 0; i < 3; ++i) a.dbg[i] = ph[i];
  // every thread of this workgroup is past its last exchange (the loops end on a barrier)
  split_exit(counter, sp.n_docs, G);
  // final pass over this segment's ranges: c_n phi_nk = E_jk b_nk r_n with the final sweep's chunk E
  if (!active) return;
  for (int j = 0; j < nch; ++j) {
    int m0, m1;
    range(j, m0, m1);
    double E[KPL];
#pragma unroll
    for (int i = 0; i < KPL; ++i) {
      const int k = tk<TG, PAIR>(q, i);
      E[i] = k < KS ? (GM ? tab[(size_t)j * 2 * KS + KS + k] : sEt[j][kc_(k)]) : 0.0;
    }
    for (int p = m0 + slot; p < m1; p += NS) {
      const double* brow = a.beta + (size_t)wrow[p] * KS;
      const double c = (double)crow[p];
      double bv[KPL];
#pragma unroll
      for (int i = 0; i < KPL; ++i) bv[i] = (tk<TG, PAIR>(q, i) < KS) ? brow[tk<TG, PAIR>(q, i)] : 0.0;
      double pp = 0.0;
#pragma unroll
      for (int i = 0; i < KPL; ++i) pp = fma(E[i], bv[i], pp);
      const double r = c * drcp(bits_sum<LSW, 6>(pp));
      double* row = a.cphi + (size_t)(s0 + p) * KS;
#pragma unroll
      for (int i = 0; i < KPL; ++i)
        if (tk<TG, PAIR>(q, i) < KS) __builtin_nontemporal_store(E[i] * bv[i] * r, &row[tk<TG, PAIR>(q, i)]);
    }
  }
}

// ------------------------------------------------------------- word team ----
// Word-per-lane team kernel for KS <= 32: every lane owns whole words (all KS topics in
// registers), so a word costs 2 KS FMAs, one reciprocal and one log per LANE instead of per
// topic group (the topic-group layout repeats the reciprocal, the log and the cross-lane P sum
// on TG lanes).  The per-chunk topic sums are a register reduce-scatter per wave
// (wave_topic_sums), then the topic owners add the waves in order.  Rows of the next chunk are
// prefetched as in gs_team.
constexpr int wteam_dpb(int NW) { return 1; }
constexpr int wteam_threads(int NW) { return wteam_dpb(NW) * NW * 64; }

template <int KS, int N>
__device__ __forceinline__ void wword_steps(const double (&E)[KS], const double (*b)[KS], const double* c,
                                            double (&acc)[KS], double& lw) {
  double P[N];
#pragma unroll
  for (int u = 0; u < N; ++u) {
    double p0 = 0.0, p1 = 0.0, p2 = 0.0, p3 = 0.0;
#pragma unroll
    for (int k = 0; k < KS; k += 4) {
      p0 = fma(E[k], b[u][k], p0);
      if (k + 1 < KS) p1 = fma(E[k + 1], b[u][k + 1], p1);
      if (k + 2 < KS) p2 = fma(E[k + 2], b[u][k + 2], p2);
      if (k + 3 < KS) p3 = fma(E[k + 3], b[u][k + 3], p3);
    }
    P[u] = (p0 + p1) + (p2 + p3);
  }
#pragma unroll
  for (int u = 0; u < N; ++u) {
    const double Pu = c[u] > 0.0 ? P[u] : 1.0;
    const double r = c[u] * drcp(Pu);
    lw = fma(c[u], flog(Pu), lw);
#pragma unroll
    for (int k = 0; k < KS; ++k) acc[k] = fma(r, b[u][k], acc[k]);
  }
}

// the row of word position p from a staged document copy ([n/64][KS/2][64] double2 tiles,
// launch_gs_stage): 64 consecutive positions are 16-byte-contiguous per topic pair, so a wave's
// gather of 64 words touches ~9 cache lines per instruction instead of 64 rows' worth
template <int KS>
__device__ __forceinline__ void load_row_staged(const dvec2* __restrict__ s, int p, double (&b)[KS]) {
  const dvec2* q = s + (size_t)(p >> 6) * (KS / 2) * 64 + (p & 63);
#pragma unroll
  for (int k = 0; k < KS / 2; ++k) {
    const dvec2 v = q[k * 64];
    b[2 * k] = v.x;
    b[2 * k + 1] = v.y;
  }
}

template <int KS>
__device__ __forceinline__ void load_row_full(const double* __restrict__ beta, int w, double (&b)[KS]) {
  const double2* p = reinterpret_cast<const double2*>(beta + (size_t)w * KS);
#pragma unroll
  for (int k = 0; k < KS / 2; ++k) {
    const double2 v = p[k];
    b[2 * k] = v.x;
    b[2 * k + 1] = v.y;
  }
}

template <int KS, int NW, int RMAX>
__global__ __launch_bounds__(wteam_threads(NW)) void gs_wteam(GSArgs a) {
  static_assert(KS <= 32 && KS % 2 == 0, "word team: KS <= 32");
  constexpr int DPB = wteam_dpb(NW), NTD = NW * 64, NS = NTD;
  __shared__ double sC[DPB][kGsUMax][KS];
  __shared__ double sEt[DPB][kGsUMax][KS];
  __shared__ double sE[DPB][KS];
  __shared__ double sRed[DPB][NW][KS];
  __shared__ double sCs[DPB][kGsUMax];
  __shared__ double sScal[DPB][NW][4];
  if (a.params[kParamDone] != 0.0) return;
  const int t = threadIdx.x % NTD, ds = threadIdx.x / NTD;
  const int item = blockIdx.x * DPB + ds;
  if (item >= a.n_items) return;
  const int d = a.order[item];
  if (d < 0) return;   // placement gap (GSPlan.isolate_longest)
  const double alpha = a.params[0], lik_const = a.params[1];
  const int vmi = (int)a.params[2];
  const double vconv = params_vconv(a.params);
  const int K = a.K;
  const int lane = t & 63, wv = t >> 6;
  const int s0 = a.doc_ptr[d], n = a.doc_ptr[d + 1] - s0;
  const int U = a.gs_updates;
  const int W = n > 0 ? (n + U - 1) / U : 1;
  const int nch = (n + W - 1) / W;
  const int nact = min(NW, (W + 63) / 64);
  const bool active = wv < nact;
  const int* __restrict__ wrow = a.word_idx + s0;
  const float* __restrict__ crow = a.counts + s0;
  double(*C)[KS] = sC[ds];
  double(*Et)[KS] = sEt[ds];
  double* E_ = sE[ds];
  double* Cs = sCs[ds];
  for (int j = t; j < nch; j += NTD) Cs[j] = 0.0;
  team_sync<NW>();
  for (int p = t; p < n; p += NTD) atomicAdd(&Cs[p / W], (double)crow[p]);
  team_sync<NW>();
  double total = 0.0;
  for (int j = 0; j < nch; ++j) total += Cs[j];
  const double g0 = alpha + total / K;
  const double m = psi_only(g0);
  // topic owner: thread t < KS (wave 0)
  const int k = t;
  double gam = k < K ? g0 : 0.0, psi = m, lps = 0.0;
  if (k < KS) {
    E_[k] = k < K ? 1.0 : 0.0;
    for (int j = 0; j < nch; ++j) C[j][k] = k < K ? Cs[j] / K : 0.0;
  }
  int wc[RMAX], wn[RMAX];
  float cc[RMAX], cn[RMAX];
  unsigned vc = 0, vn = 0;
  double bc[RMAX][KS];
  auto load_ids = [&](int j, int (&w)[RMAX], float (&c)[RMAX], unsigned& v) {
    const int n0 = j * W, n1 = min(n, n0 + W);
    v = 0;
#pragma unroll
    for (int r = 0; r < RMAX; ++r) {
      const int p = n0 + t + r * NS;
      v |= (active && p < n1) ? (1u << r) : 0u;
      // rounds past the chunk end re-read the chunk's last word: the same address as a valid
      // lane, so no extra row is gathered (clamping to the document end fetched the next chunk's rows)
      const int pc = min(p, n1 - 1);
      w[r] = wrow[pc];
      c[r] = crow[pc];
    }
  };
  // rounds without a word (past the chunk end) load nothing: exec-masked lanes return no data, and
  // the row return path (64 B/clk per CU) is what a chunk's word phase waits on
  auto load_rows = [&](const int (&w)[RMAX], unsigned v) {
    if (!active) return;   // wave-uniform
#pragma unroll
    for (int r = 0; r < RMAX; ++r) {
      if ((v >> r) & 1u) {
        load_row_full<KS>(a.beta, w[r], bc[r]);
      } else {
#pragma unroll
        for (int k = 0; k < KS; ++k) bc[r][k] = 0.0;
      }
    }
  };
  if (nch > 0) {
    load_ids(0, wc, cc, vc);
    load_rows(wc, vc);
    load_ids(nch > 1 ? 1 : 0, wn, cn, vn);
  }
  team_sync<NW>();
  double L = 0.0, L_old = 0.0, conv = 1.0, GS = 0.0;
  int it = 0;
  const bool timer = a.dbg != nullptr && blockIdx.x == 0 && threadIdx.x == 0;
  long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  long long tc = timer ? clock64() : 0;
  auto tick = [&](int i) {
    if (timer) {
      const long long x = clock64();
      ph[i] += x - tc;
      tc = x;
    }
  };
  while (var_continue(conv, vconv, it, vmi)) {
    ++it;
    double lw = 0.0;
    lps = 0.0;
    for (int j = 0; j < nch; ++j) {
      ph[7] += timer ? 1 : 0;
      if (active) {
        const int n0 = j * W, n1 = min(n, n0 + W);
        double E[KS], acc[KS];
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
          E[kk] = E_[kk];
          acc[kk] = 0.0;
        }
        double cr[RMAX];
#pragma unroll
        for (int r = 0; r < RMAX; ++r) cr[r] = ((vc >> r) & 1u) ? (double)cc[r] : 0.0;
        if (RMAX == 1 || n1 - n0 <= NS)
          wword_steps<KS, 1>(E, bc, cr, acc, lw);
        else
          wword_steps<KS, RMAX>(E, bc, cr, acc, lw);
        for (int p = n0 + t + RMAX * NS; p < n1; p += NS) {   // beyond the prefetched rounds
          double b[1][KS];
          load_row_full<KS>(a.beta, wrow[p], b[0]);
          const double cp = (double)crow[p];
          wword_steps<KS, 1>(E, b, &cp, acc, lw);
        }
        const int j1 = j + 1 < nch ? j + 1 : 0;
        const int j2 = j1 + 1 < nch ? j1 + 1 : 0;
#pragma unroll
        for (int r = 0; r < RMAX; ++r) {
          wc[r] = wn[r];
          cc[r] = cn[r];
        }
        vc = vn;
        load_rows(wc, vc);
        load_ids(j2, wn, cn, vn);
        tick(0);
        wave_topic_sums<KS>(acc, lane, sRed[ds][wv]);
        tick(1);
      }
      team_sync<NW>();
      tick(2);
      if (k < KS) {
        double S = 0.0;
#pragma unroll
        for (int v = 0; v < NW; ++v) S += v < nact ? sRed[ds][v][k] : 0.0;
        const double Eo = E_[k];
        const double nw = Eo * S;
        double En = 0.0;
        if (k < K) {
          lps = fma(psi, nw, lps);
          gam += nw - C[j][k];
          psi_exp(gam, m, psi, En);
        }
        C[j][k] = nw;
        Et[j][k] = Eo;
        E_[k] = En;
      }
      tick(3);
      team_sync<NW>();
      tick(4);
    }
    const bool own = k < K;
    const double w0 = group_sum<64>(lw);
    const double w1 = group_sum<64>(own ? gam : 0.0), w2 = group_sum<64>(own ? lgamma_pos(gam) : 0.0);
    const double w3 = group_sum<64>(own ? lps : 0.0);
    if (lane == 0) {
      sScal[ds][wv][0] = w0;
      sScal[ds][wv][1] = w1;
      sScal[ds][wv][2] = w2;
      sScal[ds][wv][3] = w3;
    }
    team_sync<NW>();
    double LW = 0.0, LG = 0.0, LP = 0.0;
    GS = 0.0;
#pragma unroll
    for (int v = 0; v < NW; ++v) {
      LW += sScal[ds][v][0];
      GS += sScal[ds][v][1];
      LG += sScal[ds][v][2];
      LP += sScal[ds][v][3];
    }
    L = lik_const - lgamma_pos(GS) + LG + fma(m, total, LW) - LP;
    conv = (L_old - L) / L_old;
    L_old = L;
    team_sync<NW>();
    tick(5);
  }
  if (timer)
    for (int i = 0; i < 8; ++i) a.dbg[i] = ph[i];
  const double ps = group_sum<64>(k < K ? psi : 0.0);
  if (k < KS) a.gamma[(size_t)d * KS + k] = gam;
  if (lane == 0) sScal[ds][wv][0] = ps;
  team_sync<NW>();
  if (t == 0) {
    double PS = 0.0;
    for (int v = 0; v < NW; ++v) PS += sScal[ds][v][0];
    a.lik[d] = L;
    a.alpha_ss[d] = PS - K * psi_only(GS);
    a.iters[d] = it;
  }
  if (!active) return;
  for (int j = 0; j < nch; ++j) {
    const int n0 = j * W, n1 = min(n, n0 + W);
    double E[KS];
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) E[kk] = Et[j][kk];
    for (int p = n0 + t; p < n1; p += NS) {
      double b[KS];
      load_row_full<KS>(a.beta, wrow[p], b);
      double p0 = 0.0, p1 = 0.0, p2 = 0.0, p3 = 0.0;
#pragma unroll
      for (int kk = 0; kk < KS; kk += 4) {
        p0 = fma(E[kk], b[kk], p0);
        if (kk + 1 < KS) p1 = fma(E[kk + 1], b[kk + 1], p1);
        if (kk + 2 < KS) p2 = fma(E[kk + 2], b[kk + 2], p2);
        if (kk + 3 < KS) p3 = fma(E[kk + 3], b[kk + 3], p3);
      }
      const double r = (double)crow[p] * drcp((p0 + p1) + (p2 + p3));
      dvec2* row = reinterpret_cast<dvec2*>(a.cphi + (size_t)(s0 + p) * KS);
#pragma unroll
      for (int kk = 0; kk < KS / 2; ++kk) {
        const dvec2 v = {E[2 * kk] * b[2 * kk] * r, E[2 * kk + 1] * b[2 * kk + 1] * r};
        __builtin_nontemporal_store(v, &row[kk]);
      }
    }
  }
}

// ------------------------------------------------- word team, topic wave ----
// The longest documents (gs_wteam measured: ~8.7k cycles per chunk, the critical path of the
// E-step).  NW word waves own the words; one extra TOPIC WAVE owns the K topics and runs the
// refresh.  The two roles run separate loops with the same barrier sequence, so:
//  - the word waves' registers (E, accumulators, the next chunk's prefetched rows) are not live
//    in the refresh code, which therefore needs no spills; in gs_wteam the refresh ran in wave 0
//    beside 256 live VGPRs and its spill reloads waited (vmcnt is in order) behind the next
//    chunk's row prefetch;
//  - the topic wave issues no global loads, so nothing queues in front of its LDS traffic;
//  - the word waves take log P of their words (only the sweep likelihood needs it) while the
//    topic wave refreshes, off the chunk's critical path.
// Arithmetic per word and per topic is that of gs_wteam (the likelihood's lw partial sums are
// grouped by wave, so the two kernels agree to rounding, not bitwise).
// EP (early prefetch): rounds u < EP of the next chunk's rows are gathered
// into bc[u] as soon as the axpy of round u has consumed them -- before the topic sums and the
// arrival -- so the address unit works beside the reduction; the other rounds after the arrival.
// (Measured slower and removed in round 5, records in profiles/r4_tuning_log.md: the topic wave summing
// the word waves' lane partials, 5 or 3 word waves, two early rounds, the LDS-ring loader variant.)
template <int KS, int NW, int RMAX, int EP = 0, bool STG = false>
__global__ __launch_bounds__((NW + 1) * 64) void gs_wsteam(GSArgs a) {
  static_assert(KS <= 32 && KS % 2 == 0, "word team: KS <= 32");
  constexpr int NTD = (NW + 1) * 64, NS = NW * 64;
  __shared__ double C[kGsUMax][KS];     // chunk contributions (previous sweep)
  __shared__ double Et[kGsUMax][KS];    // E each chunk used (final pass)
  __shared__ double E_[KS];             // current E, broadcast
  __shared__ double sRed[NW][KS];       // per-wave topic sums of a chunk
  __shared__ double Cs[kGsUMax];        // chunk count sums
  __shared__ double sScal[NW + 1][4];   // sweep partials: lw per word wave; gamma sums (topic wave)
  __shared__ int arrive[NW];            // per word wave: chunks whose topic sums it has left in sRed
  if (a.params[kParamDone] != 0.0) return;
  const int t = threadIdx.x;
  const int d = a.order[blockIdx.x];
  if (d < 0) return;                    // placement gap (GSPlan.isolate_longest): whole workgroup
  const double alpha = a.params[0], lik_const = a.params[1];
  const int vmi = (int)a.params[2];
  const double vconv = params_vconv(a.params);
  const int K = a.K;
  auto kc_ = [](int k) { return k < KS ? k : KS - 1; };   // an in-bounds LDS column for guarded reads
  const int lane = t & 63, wv = t >> 6;
  const bool topic_wave = wv == NW;
  const int s0 = a.doc_ptr[d], n = a.doc_ptr[d + 1] - s0;
  const int U = a.gs_updates;
  const int W = n > 0 ? (n + U - 1) / U : 1;
  const int nch = (n + W - 1) / W;
  const int nact = min(NW, (W + 63) / 64);
  const bool active = wv < nact;        // word waves holding words of a chunk (never the topic wave)
  const int* __restrict__ wrow = a.word_idx + s0;
  const float* __restrict__ crow = a.counts + s0;
  for (int j = t; j < nch; j += NTD) Cs[j] = 0.0;
  if (t < NW) arrive[t] = 0;
  lds_barrier();
  for (int p = t; p < n; p += NTD) atomicAdd(&Cs[p / W], (double)crow[p]);   // integer counts: exact
  lds_barrier();
  double total = 0.0;
  for (int j = 0; j < nch; ++j) total += Cs[j];
  const double g0 = alpha + total / K;
  const double m = psi_only(g0);
  const bool timer = a.dbg != nullptr && blockIdx.x == 0 && t == 0;
  long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  long long tc = timer ? clock64() : 0;
  auto tick = [&](int i) {
    if (timer) {
      const long long x = clock64();
      ph[i] += x - tc;
      tc = x;
    }
  };
  double L = 0.0, L_old = 0.0, conv = 1.0, GS = 0.0;
  int it = 0;
  // sweep likelihood from the partials every wave left in sScal (same order in every thread)
  auto sweep_end = [&]() {
    lds_barrier();
    double LW = 0.0;
#pragma unroll
    for (int v = 0; v < NW; ++v) LW += sScal[v][0];
    GS = sScal[NW][1];
    L = lik_const - lgamma_pos(GS) + sScal[NW][2] + fma(m, total, LW) - sScal[NW][3];
    conv = (L_old - L) / L_old;
    L_old = L;
    lds_barrier();
  };
  if (topic_wave) {
    // ------------------------------------------------------------ topic wave
    __builtin_amdgcn_s_setprio(3);   // its chain is the critical path; the word waves wait on it
    const int k = lane;
    int want = 0;
    // dbg[8..11] (the int64[16] timer of gs_estep): this wave's cycles waiting for the arrivals,
    // summing + refreshing, and at barrier B, summed over chunks
    const bool ttimer = a.dbg != nullptr && blockIdx.x == 0 && lane == 0;
    long long tph[8] = {0, 0, 0, 0, 0, 0, 0, 0};   // [4 + i]: chunk start -> wave v_i's arrival seen
    long long ttc = ttimer ? clock64() : 0;
    auto ttick = [&](int i) {
      if (ttimer) {
        const long long x = clock64();
        tph[i] += x - ttc;
        ttc = x;
      }
    };
    double gam = k < K ? g0 : 0.0, psi = m, lps = 0.0;
    // this lane's E_k stays in a register (the wave is E_'s only writer), and C_jk is read before
    // the arrival wait: after the last arrival only the sRed loads precede the refresh chain
    double Ecur = k < K ? 1.0 : 0.0;
    if (k < KS) {
      E_[k] = Ecur;
      for (int j = 0; j < nch; ++j) C[j][k] = k < K ? Cs[j] / K : 0.0;
    }
    lds_barrier();   // (1) E_ and C ready; word waves' first rows in flight
    while (var_continue(conv, vconv, it, vmi)) {
      ++it;
      lps = 0.0;
      for (int j = 0; j < nch; ++j) {
        // (A) the nact word waves' topic sums of chunk j are in sRed: summed in wave order as each
        // wave arrives, so after the last arrival one add remains (not nact dependent adds)
        ++want;
        ttick(3);
        const double gC = k < KS ? gam - C[j][k] : 0.0;
        double S = 0.0;
#pragma unroll
        for (int v = 0; v < NW; ++v) {
          if (v < nact) {
            while (__hip_atomic_load(&arrive[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < want)
              __builtin_amdgcn_s_sleep(1);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
            if (ttimer && (v == 0 || v == 3 || v == 4 || v == nact - 1))
              tph[v == 0 ? 4 : v == 3 ? 5 : v == 4 ? 6 : 7] += clock64() - ttc;
            S += k < KS ? sRed[v][k] : 0.0;
          }
        }
        ttick(0);
        if (k < KS) {
          const double Eo = Ecur;
          const double nw = Eo * S;
          double En = 0.0;
          if (k < K) {
            lps = fma(psi, nw, lps);
            gam = fma(Eo, S, gC);   // gamma_k + (new_jk - C_jk) in one rounding, off the nw product
            psi_exp(gam, m, psi, En);
          }
          E_[k] = En;
          C[j][k] = nw;
          Et[j][k] = Eo;
          Ecur = En;
        }
        ttick(1);
        lds_barrier();   // (B) E of chunk j + 1 published
        ttick(2);
      }
      const bool own = k < K;
      const double w1 = group_sum<64>(own ? gam : 0.0), w2 = group_sum<64>(own ? lgamma_pos(gam) : 0.0);
      const double w3 = group_sum<64>(own ? lps : 0.0);
      if (lane == 0) {
        sScal[NW][1] = w1;
        sScal[NW][2] = w2;
        sScal[NW][3] = w3;
      }
      sweep_end();
    }
    if (ttimer)
      for (int i = 0; i < 8; ++i) a.dbg[8 + i] = tph[i];
    const double ps = group_sum<64>(k < K ? psi : 0.0);
    if (k < KS) a.gamma[(size_t)d * KS + k] = gam;
    if (lane == 0) {
      a.lik[d] = L;
      a.alpha_ss[d] = ps - K * psi_only(GS);
      a.iters[d] = it;
    }
    return;
  }
  // -------------------------------------------------------------- word waves
  // STG: rows come from the document's staged copy (launch_gs_stage) indexed by word position, so
  // the ids below are positions; otherwise they are vocabulary ids into beta
  const dvec2* stg = nullptr;
  if constexpr (STG) stg = reinterpret_cast<const dvec2*>(a.stage) + a.stage_off[blockIdx.x];
  auto row_of = [&](int p) { return STG ? p : wrow[p]; };
  auto load_row = [&](int id, double(&b)[KS]) {
    if constexpr (STG)
      load_row_staged<KS>(stg, id, b);
    else
      load_row_full<KS>(a.beta, id, b);
  };
  int wc[RMAX], wn[RMAX];
  float cc[RMAX], cn[RMAX];
  unsigned vc = 0, vn = 0;
  double bc[RMAX][KS];
  auto load_ids = [&](int j, int (&w)[RMAX], float (&c)[RMAX], unsigned& v) {
    const int n0 = j * W, n1 = min(n, n0 + W);
    v = 0;
#pragma unroll
    for (int r = 0; r < RMAX; ++r) {
      const int p = n0 + t + r * NS;
      v |= (active && p < n1) ? (1u << r) : 0u;
      const int pc = min(p, n1 - 1);
      w[r] = row_of(pc);
      c[r] = crow[pc];
    }
  };
  auto load_rows = [&](const int (&w)[RMAX], unsigned v) {
    if (!active) return;   // wave-uniform
#pragma unroll
    for (int r = 0; r < RMAX; ++r) {
      if ((v >> r) & 1u) {   // rounds past the chunk end gather nothing
        load_row(w[r], bc[r]);
      } else {
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) bc[r][kk] = 0.0;
      }
    }
  };
  if (nch > 0) {
    load_ids(0, wc, cc, vc);
    load_rows(wc, vc);
    load_ids(nch > 1 ? 1 : 0, wn, cn, vn);
  }
  lds_barrier();   // (1)
  while (var_continue(conv, vconv, it, vmi)) {
    ++it;
    double lw = 0.0;
    for (int j = 0; j < nch; ++j) {
      ph[7] += timer ? 1 : 0;
      double P[RMAX], cr[RMAX];
      if (active) {
        const int n0 = j * W, n1 = min(n, n0 + W);
        double E[KS], acc[KS];
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
          E[kk] = E_[kk];
          acc[kk] = 0.0;
        }
#pragma unroll
        for (int r = 0; r < RMAX; ++r) cr[r] = ((vc >> r) & 1u) ? (double)cc[r] : 0.0;
        // dot, reciprocal and axpy now; log P after barrier A (beside the refresh)
#pragma unroll
        for (int u = 0; u < RMAX; ++u) {
          double p0 = 0.0, p1 = 0.0, p2 = 0.0, p3 = 0.0;
#pragma unroll
          for (int kk = 0; kk < KS; kk += 4) {
            p0 = fma(E[kk], bc[u][kk], p0);
            if (kk + 1 < KS) p1 = fma(E[kk + 1], bc[u][kk + 1], p1);
            if (kk + 2 < KS) p2 = fma(E[kk + 2], bc[u][kk + 2], p2);
            if (kk + 3 < KS) p3 = fma(E[kk + 3], bc[u][kk + 3], p3);
          }
          P[u] = cr[u] > 0.0 ? (p0 + p1) + (p2 + p3) : 1.0;
        }
        if (timer) {   // split of the word phase: E read + dot | reciprocal + axpy + prefetch issue
          __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0) only... values consumed below anyway
          const long long x = clock64();
          ph[6] += x - tc;
          tc = x;
        }
#pragma unroll
        for (int u = 0; u < RMAX; ++u) {
          const double r = cr[u] * drcp(P[u]);
#pragma unroll
          for (int kk = 0; kk < KS; ++kk) acc[kk] = fma(r, bc[u][kk], acc[kk]);
          if (u < EP) {   // bc[u] is free: the next chunk's round u (ids already here)
            __builtin_amdgcn_sched_barrier(0);   // keep the gather below the axpy (no second row set)
            if ((vn >> u) & 1u) {
              load_row(wn[u], bc[u]);
            } else {
#pragma unroll
              for (int kk = 0; kk < KS; ++kk) bc[u][kk] = 0.0;
            }
          }
        }
        for (int p = n0 + t + RMAX * NS; p < n1; p += NS) {   // beyond the prefetched rounds
          double b[1][KS];
          load_row(row_of(p), b[0]);
          const double cp = (double)crow[p];
          wword_steps<KS, 1>(E, b, &cp, acc, lw);
        }
        tick(0);
        wave_topic_sums<KS>(acc, lane, sRed[wv]);
        // (A) arrival: this wave's topic sums are in sRed.  A counter instead of a workgroup barrier,
        // so the refresh starts while the word waves are still issuing the next chunk's row loads
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");   // LDS only: no vmcnt wait
        if (lane == 0) __hip_atomic_fetch_add(&arrive[wv], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        tick(1);
        // prefetch of the next chunk's rows: a chunk's ~700 row gathers keep the CU's address unit busy
        // for ~2k cycles (64 B/clk) and the issuing wave blocks until they are queued -- now beside the
        // refresh instead of before it
        const int j1 = j + 1 < nch ? j + 1 : 0;
        const int j2 = j1 + 1 < nch ? j1 + 1 : 0;
#pragma unroll
        for (int r = 0; r < RMAX; ++r) {
          wc[r] = wn[r];
          cc[r] = cn[r];
        }
        vc = vn;
        if constexpr (EP == 0) {
          load_rows(wc, vc);
        } else if (active) {
#pragma unroll
          for (int r = EP; r < RMAX; ++r) {
            if ((vc >> r) & 1u) {
              load_row(wc[r], bc[r]);
            } else {
#pragma unroll
              for (int kk = 0; kk < KS; ++kk) bc[r][kk] = 0.0;
            }
          }
        }
        load_ids(j2, wn, cn, vn);
        tick(2);
#pragma unroll
        for (int u = 0; u < RMAX; ++u) lw = fma(cr[u], flog(P[u]), lw);
      }
      tick(3);
      lds_barrier();   // (B)
      tick(4);
    }
    const double w0 = group_sum<64>(lw);
    if (lane == 0) sScal[wv][0] = w0;
    sweep_end();
    tick(5);
  }
  if (timer)
    for (int i = 0; i < 8; ++i) a.dbg[i] = ph[i];
  // final pass: c_n phi_nk = E_jk b_nk r_n with the final sweep's chunk E (same P as the sweep)
  if (!active) return;
  for (int j = 0; j < nch; ++j) {
    const int n0 = j * W, n1 = min(n, n0 + W);
    double E[KS];
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) E[kk] = Et[j][kk];
    for (int p = n0 + t; p < n1; p += NS) {
      double b[KS];
      load_row(row_of(p), b);
      double p0 = 0.0, p1 = 0.0, p2 = 0.0, p3 = 0.0;
#pragma unroll
      for (int kk = 0; kk < KS; kk += 4) {
        p0 = fma(E[kk], b[kk], p0);
        if (kk + 1 < KS) p1 = fma(E[kk + 1], b[kk + 1], p1);
        if (kk + 2 < KS) p2 = fma(E[kk + 2], b[kk + 2], p2);
        if (kk + 3 < KS) p3 = fma(E[kk + 3], b[kk + 3], p3);
      }
      const double r = (double)crow[p] * drcp((p0 + p1) + (p2 + p3));
      dvec2* row = reinterpret_cast<dvec2*>(a.cphi + (size_t)(s0 + p) * KS);
#pragma unroll
      for (int kk = 0; kk < KS / 2; ++kk) {
        const dvec2 v = {E[2 * kk] * b[2 * kk] * r, E[2 * kk + 1] * b[2 * kk + 1] * r};
        __builtin_nontemporal_store(v, &row[kk]);
      }
    }
  }
}

// ------------------------------------------------------------ suff stats ----
// One word per workgroup (heavy) / wave (medium) / 16 lanes (light); a CSC entry's
// row is read by TG lanes (KPL topics each), S = G / TG entries in flight per group.
template <int KS>
__global__ __launch_bounds__(256) void gs_suff64(const int* __restrict__ word_ptr, const int* __restrict__ csc_ent,
                                                 const int* __restrict__ order, int n_heavy, int n_medium,
                                                 int n_light, const double* __restrict__ cphi,
                                                 double* cw, double* __restrict__ part,
                                                 const double* __restrict__ lik, const double* __restrict__ ass,
                                                 int lo, int hi, const double* gate,
                                                 const double* cw_base) {
  // one topic per lane: the paired 16-byte loads of the team kernels measured slower here (K = 100 early
  // pass 2.06 -> 2.62 ms, r5v); the c.phi pad row (em.py) is kept so PAIR stays a one-line switch
  constexpr int TG = tg_of(KS), NSLOT = 256 / TG;
  constexpr bool PAIR = false;
  constexpr int KPL = PAIR ? 2 * ((KS + 2 * TG - 1) / (2 * TG)) : kpl_of(KS);
  __shared__ double sAcc[NSLOT][KS];
  __shared__ double sRow[16][KS];
  if (gated(gate)) return;
  const int t = threadIdx.x, b = blockIdx.x;
  double* prow = part + (size_t)b * (KS + 2);
  // likelihood / alpha_ss slice of this workgroup (wave 0, fixed order)
  if (t < 64) {
    const int nd = hi - lo, nb = (int)gridDim.x;
    const int per = (nd + nb - 1) / nb;
    const int i0 = lo + b * per, i1 = min(hi, i0 + per);
    double x = 0.0, y = 0.0;
    if (lik)
      for (int i = i0 + t; i < i1; i += 64) {
        x += lik[i];
        y += ass[i];
      }
    x = group_sum<64>(x);
    y = group_sum<64>(y);
    if (t == 0) {
      prow[0] = x;
      prow[1] = y;
    }
  }
  const int nbM = (n_medium + 3) / 4;
  int G, item, nitems, base;
  if (b < n_heavy) {
    G = 256, item = b, nitems = n_heavy, base = 0;
  } else if (b < n_heavy + nbM) {
    G = 64, item = (b - n_heavy) * 4 + t / 64, nitems = n_medium, base = n_heavy;
  } else {
    G = 16, item = (b - n_heavy - nbM) * 16 + t / 16, nitems = n_light, base = n_heavy + n_medium;
  }
  const int S = G / TG, gi = t / G;
  const int sidx = (t % G) / TG, q = t % TG;
  const bool valid = item < nitems;
  double acc[KPL];
#pragma unroll
  for (int i = 0; i < KPL; ++i) acc[i] = 0.0;
  if (valid) {
    const int w = order[base + item];
    int e = word_ptr[w] + sidx;
    const int end = word_ptr[w + 1];
    for (; e + 3 * S < end; e += 4 * S) {
      double v[4][KPL];
#pragma unroll
      for (int u = 0; u < 4; ++u) load_row<KS, KPL, TG, PAIR>(cphi, csc_ent[e + u * S], q, v[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int i = 0; i < KPL; ++i) acc[i] += v[u][i];
    }
    for (; e < end; e += S) {
      double v[KPL];
      load_row<KS, KPL, TG, PAIR>(cphi, csc_ent[e], q, v);
#pragma unroll
      for (int i = 0; i < KPL; ++i) acc[i] += v[i];
    }
  }
#pragma unroll
  for (int i = 0; i < KPL; ++i)
    if (tk<TG, PAIR>(q, i) < KS) sAcc[t / TG][tk<TG, PAIR>(q, i)] = acc[i];
  __syncthreads();
  const int ngroups = 256 / G;
  for (int idx = t; idx < ngroups * KS; idx += 256) {
    const int g = idx / KS, k = idx % KS;
    const int it = (G == 256 ? item : item - gi + g);
    // cw_base (nullable): rows summed earlier from the other entries of each word (the early /
    // late split of the suff-stats and the c.phi windows, em.py), added first so the order is
    // fixed; cw_base == cw (in place) is allowed: each element is read, then written, by one thread
    const size_t row = it < nitems ? (size_t)order[base + it] * KS : 0;
    double v = (cw_base != nullptr && it < nitems) ? cw_base[row + k] : 0.0;
    for (int u = 0; u < S; ++u) v += sAcc[g * S + u][k];
    if (it < nitems) cw[row + k] = v;
    else v = 0.0;
    sRow[g][k] = v;
  }
  __syncthreads();
  if (t < KS) {
    double s = 0.0;
    for (int g = 0; g < ngroups; ++g) s += sRow[g][t];
    prow[2 + t] = s;
  }
}

// ------------------------------------------------------------ random init ---
// lda-c "random" start (random_initialize_ss): class_word[k][w] = 1/V + u, u ~ U[0, 1) from a
// counter-based generator, so the host (csrc/native, CPU backends) and the device produce the same
// bits without a host-side stream: u = splitmix64(splitmix64(seed) ^ (k V + w)) >> 11, x 2^-53.
__device__ __forceinline__ unsigned long long smix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__global__ __launch_bounds__(256) void init_random_ss_kernel(double* __restrict__ cw, int V, int K, int KS,
                                                             unsigned long long seed) {
  const unsigned long long s = smix64(seed);
  const double inv = 1.0 / (double)V;
  const long long total = (long long)V * KS;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int w = (int)(i / KS), k = (int)(i % KS);
    double v = 0.0;
    if (k < K) {
      const unsigned long long h = smix64(s ^ ((unsigned long long)k * (unsigned long long)V + (unsigned long long)w));
      v = inv + (double)(h >> 11) * 0x1.0p-53;
    }
    cw[i] = v;
  }
}

// ----------------------------------------------------------------- M-step ---
__device__ __forceinline__ double mle(double c, double ct) { return c > 0.0 ? c / ct : kExpM100; }

// SKS > 0: the trailing sf.blocks workgroups refill staged rows at KS = SKS (one thread per staged
// position: its word's row in SKS / 2 independent 16-byte loads, as gs_stage_kernel)
template <int SKS>
__global__ __launch_bounds__(256) void gs_mstep_control_kernel(const double* __restrict__ cw,
                                                               const double* __restrict__ ct,
                                                               double* __restrict__ beta, int V, int K, int KS,
                                                               const int* __restrict__ rows, int n_rows,
                                                               EMControlArgs c, NewtonArgs nw, StageFuseArgs sf) {
  if (c.params[kParamDone] != 0.0) return;
  // with the alpha Newton (a serial chain of ~10-20 digamma / trigamma / exp / log steps on two lanes),
  // block 0 runs only the Newton and the other blocks compute beta beside it
  const bool newton = nw.enabled && gridDim.x > 1;
  if (nw.enabled && blockIdx.x == 0 && threadIdx.x < 64) {
    if (threadIdx.x < 2)
      alpha_newton_lanes(c.scalars, nw.num_docs, K, nw.estimate, c.params, nw.alpha_out, threadIdx.x);
    __builtin_amdgcn_s_waitcnt(0);
  }
  const int hq = KS / 2;
  const int total2 = (rows ? n_rows : V) * hq;
  const double2* cw2 = reinterpret_cast<const double2*>(cw);
  double2* beta2 = reinterpret_cast<double2*>(beta);
  const int sb0 = (int)gridDim.x - sf.blocks;   // the trailing sf.blocks workgroups refill staged rows
  if constexpr (SKS > 0) {
    if ((int)blockIdx.x >= sb0) {
      // one thread per (tile, lane): the row's SKS / 2 pairs loaded together, mle(cw, ct) -- bit for bit
      // the beta entries -- stored one 16-byte element per pair in [tile][pair][64 lanes]
      constexpr int HQ = SKS / 2;
      const int n0 = sf.n_tiles[0] * 64, n1 = sf.n_sets > 1 ? sf.n_tiles[1] * 64 : 0;
      for (int e = ((int)blockIdx.x - sb0) * (int)blockDim.x + (int)threadIdx.x; e < n0 + n1;
           e += sf.blocks * (int)blockDim.x) {
        const int set = e < n0 ? 0 : 1;
        const int el = set ? e - n0 : e;
        const int t = el >> 6, l = el & 63;
        double2 v[HQ];
        if (l < sf.tile_cnt[set][t]) {
          const double2* row = cw2 + (size_t)sf.word_idx[sf.tile_ent[set][t] + l] * HQ;
#pragma unroll
          for (int k = 0; k < HQ; ++k) v[k] = row[k];
#pragma unroll
          for (int k = 0; k < HQ; ++k) {
            v[k].x = 2 * k < K ? mle(v[k].x, ct[2 * k]) : 0.0;
            v[k].y = 2 * k + 1 < K ? mle(v[k].y, ct[2 * k + 1]) : 0.0;
          }
        } else {
#pragma unroll
          for (int k = 0; k < HQ; ++k) v[k] = double2{0.0, 0.0};
        }
        double2* o = reinterpret_cast<double2*>(sf.out[set]) + (size_t)t * HQ * 64 + l;
#pragma unroll
        for (int k = 0; k < HQ; ++k) o[k * 64] = v[k];
      }
    }
  }
  if ((int)blockIdx.x < sb0) {
    const int bx = newton ? (int)blockIdx.x - 1 : (int)blockIdx.x, nbx = newton ? sb0 - 1 : sb0;
    for (int g = bx * blockDim.x + threadIdx.x; bx >= 0 && g < total2; g += nbx * blockDim.x) {
      const int k0 = (g % hq) * 2;
      const int i = rows ? rows[g / hq] * hq + g % hq : g;
      const double2 v = cw2[i];
      double2 o;
      o.x = k0 < K ? mle(v.x, ct[k0]) : 0.0;
      o.y = k0 + 1 < K ? mle(v.y, ct[k0 + 1]) : 0.0;
      beta2[i] = o;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (__hip_atomic_fetch_add(c.done_count, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1) {
      __hip_atomic_store(c.done_count, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const double alpha_now = __hip_atomic_load(c.params, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      em_control_step(c.scalars, c.params, c.ctl, c.hist, c.hist_slots, alpha_now);
    }
  }
}

__global__ __launch_bounds__(256) void gs_mstep_kernel(const double* __restrict__ cw, const double* __restrict__ ct,
                                                       double* __restrict__ beta, int V, int K, int KS,
                                                       const double* gate) {
  if (gated(gate)) return;
  const int64_t total = (int64_t)V * KS;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(i % KS);
    beta[i] = k < K ? mle(cw[i], ct[k]) : 0.0;
  }
}

// Staged rows of the longest documents (GSArgs::stage): one thread per double2 of the tiled copy,
// coalesced stores and 16-byte gathers from beta (the gathers are spread over the whole GPU here,
// instead of through the one CU that walks the document 20 times per E-step)
template <int KS>
__global__ __launch_bounds__(256) void gs_stage_kernel(const double* __restrict__ beta,
                                                       const int* __restrict__ word_idx,
                                                       const int* __restrict__ tile_ent,
                                                       const int* __restrict__ tile_cnt, int n_tiles,
                                                       dvec2* __restrict__ out, const double* gate) {
  if (gate != nullptr && *gate != 0.0) return;   // converged EM loop: the queued iterations are no-ops
  // one thread per (tile, lane): its word's whole row in KS / 2 independent 16-byte loads, stored
  // as one 16-byte element per topic pair (a wave's stores are 1 KB-contiguous per pair)
  const long long total = (long long)n_tiles * 64;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int t = (int)(i >> 6), l = (int)(i & 63);
    dvec2 v[KS / 2];
    if (l < tile_cnt[t]) {
      const dvec2* row = reinterpret_cast<const dvec2*>(beta + (size_t)word_idx[tile_ent[t] + l] * KS);
#pragma unroll
      for (int k = 0; k < KS / 2; ++k) v[k] = row[k];
    } else {
#pragma unroll
      for (int k = 0; k < KS / 2; ++k) v[k] = dvec2{0.0, 0.0};
    }
    dvec2* o = out + (size_t)t * (KS / 2) * 64 + l;
#pragma unroll
    for (int k = 0; k < KS / 2; ++k) o[k * 64] = v[k];
  }
}

}  // namespace gs

// ------------------------------------------------------------------ launch ---
template <int KS>
static void gs_estep_ks(const GSArgs& a, int variant, hipStream_t s) {
  if (a.n_items <= 0) return;
  switch (variant) {
    case kGsTiny: {
      constexpr int per = 256 / gs::tiny_tg(KS);
      hipLaunchKernelGGL((gs::gs_tiny<KS>), dim3((a.n_items + per - 1) / per), dim3(256), 0, s, a);
      break;
    }
    case kGsSmall: {
      if (KS <= 32 && a.gs_updates > kGsUMax)
        throw std::runtime_error("gs_estep: gs_small keeps its chunk tables in LDS (U <= 32 at KS <= 32)");
      if constexpr (KS <= 32)
        hipLaunchKernelGGL((gs::gs_small<KS>), dim3((a.n_items + 15) / 16), dim3(256), 0, s, a);
      else
        hipLaunchKernelGGL((gs::gs_smallw<KS, 2, (KS > 100 ? 1 : 2)>), dim3((a.n_items + 15) / 16), dim3(256), 0, s, a);
      break;
    }
    case kGsChain:
      hipLaunchKernelGGL((gs::gs_chain<KS, 8>), dim3((a.n_items + 3) / 4), dim3(256), 0, s, a);
      break;
    case kGsTeam1: {
      if (KS <= 32 && a.gs_updates > kGsUMax)
        throw std::runtime_error("gs_estep: the one-wave team keeps its chunk tables in LDS (U <= 32 at KS <= 32)");
      // one wave per document (<= 256 words, chunks of <= 8 words): the topic-group layout keeps
      // more lanes busy than one word per lane (measured 0.90 vs 1.13 ms on the headline corpus)
      constexpr int dpb = gs::TeamShape<KS, 1>::DPB;
      const dim3 grid((a.n_items + dpb - 1) / dpb), blk(dpb * 64);
      if constexpr (KS > 32) {
        // 3 waves per SIMD (168 VGPRs, 12 B spilled): K = 100 shard team1 13.2 -> 11.7 ms; 4 (128 VGPRs,
        // 100 B spilled) 19.5 ms (profiles/r2_k100_split.md)
        hipLaunchKernelGGL((gs::gs_team<KS, 1, 3>), grid, blk, 0, s, a);
      } else {
        hipLaunchKernelGGL((gs::gs_team<KS, 1>), grid, blk, 0, s, a);
      }
      break;
    }
    case kGsTeam4:
      if (KS <= 32 && a.gs_updates > kGsUMax) {
        // lda-c's per-word schedule at K <= 32: the topic-group team with its chunk tables in the c*phi rows
        hipLaunchKernelGGL((gs::gs_team<KS, 4, 1, true>), dim3(a.n_items), dim3(256), 0, s, a);
      } else if constexpr (KS <= 32) {
        // one wave per document, a word per lane, in-wave refresh: 2.128 / 2.129 / 2.143 vs 2.136 / 2.141 /
        // 2.144 ms per EM iteration for 3 word waves + a topic wave (3 A/B rounds, profiles/r3_tuning_log.md):
        // a quarter of the waves for the same chains leaves the CUs to the other buckets
        hipLaunchKernelGGL((gs::gs_wteam<KS, 1, 1>), dim3(a.n_items), dim3(64), 0, s, a);
      }
      else
        // KS > 32, any U: the chunk tables in the c*phi rows (GM) and 3 waves per SIMD.  The LDS-table form
        // (2 x 32 x KS doubles: 58 KB at K = 100) fits two workgroups per CU; this one (6.7 KB, 166 VGPRs, 12 B
        // spilled) three: team4 bucket 5.88 -> 4.78 ms on the 12.5 M-event shard, 38.1 -> 30.7 ms at 100 M
        // events (E-step graph 170.0 -> 167.1 ms); 4 waves per SIMD spill 160 B and gain less
        // (profiles/r6z_team4_gm.md)
        hipLaunchKernelGGL((gs::gs_team<KS, 4, 3, true>), dim3(a.n_items), dim3(256), 0, s, a);
      break;
    case kGsTeam8:
      if (KS <= 32 && a.gs_updates > kGsUMax) {
        if (a.stage != nullptr) throw std::runtime_error("gs_estep: no staged rows past U = 32 at KS <= 32");
        hipLaunchKernelGGL((gs::gs_team<KS, 8, 1, true>), dim3(a.n_items), dim3(512), 0, s, a);
      } else if constexpr (KS <= 32) {
        // longest documents: 7 word waves x 2 prefetched words per lane + a topic wave (5 x 3: 2.64 ms, 3 x 4:
        // 2.06 ms vs 1.74 per headline EM iteration; profiles/r4_tuning_log.md).  Staged rows (GSStage): every
        // next-chunk round gathered after the arrival (1.726-1.740 vs 1.824-1.833 ms for an early round-0
        // gather); rows gathered from beta (a plan past the staging budget): round 0 early (2.13-2.14 vs
        // 2.17-2.18 ms).  The LDS-ring and topic-wave-reduction variants were slower and are gone.
        if (a.stage != nullptr)
          hipLaunchKernelGGL((gs::gs_wsteam<KS, 7, 2, 0, true>), dim3(a.n_items), dim3(512), 0, s, a);
        else
          hipLaunchKernelGGL((gs::gs_wsteam<KS, 7, 2, 1>), dim3(a.n_items), dim3(512), 0, s, a);
      }
      else if (a.gs_updates > kGsUMax)
        hipLaunchKernelGGL((gs::gs_team<KS, 8, 1, true>), dim3(a.n_items), dim3(512), 0, s, a);
      else
        hipLaunchKernelGGL((gs::gs_team<KS, 8>), dim3(a.n_items), dim3(512), 0, s, a);
      break;
    default:
      throw std::runtime_error("gs_estep: unknown variant");
  }
  ONI_HIP_CHECK(hipGetLastError());
}

// every KS: U > kGsUMax keeps the chunk tables in the c*phi rows (gs_team GMT, gs_chain, gs_smallw at KS > 32)
int gs_umax(int KS) { (void)KS; return kGsUMaxWide; }

void launch_gs_stage(const double* beta, const int* word_idx, const int* tile_ent, const int* tile_cnt, int n_tiles,
                     double* stage, int KS, const double* gate, hipStream_t s) {
  if (n_tiles <= 0) return;
  if (KS > 32 || KS % 2) throw std::runtime_error("gs_stage: staged rows need an even KS <= 32");
  const long long total = (long long)n_tiles * 64;
  const unsigned blocks = (unsigned)std::min<long long>((total + 255) / 256, 16384);
  switch (KS) {
#define ONI_KS(X)                                                                                           \
  case X:                                                                                                   \
    if constexpr (X <= 32 && X % 2 == 0)                                                                    \
      hipLaunchKernelGGL((gs::gs_stage_kernel<X>), dim3(blocks), dim3(256), 0, s, beta, word_idx, tile_ent, \
                         tile_cnt, n_tiles, reinterpret_cast<gs::dvec2*>(stage), gate);                     \
    break;
    ONI_FOR_EACH_KS(ONI_KS)
#undef ONI_KS
    default:
      throw std::runtime_error("gs_stage: unsupported KS " + std::to_string(KS));
  }
  ONI_HIP_CHECK(hipGetLastError());
}

void launch_gs_estep(const GSArgs& a, int variant, int KS, hipStream_t s) {
  if (a.gs_updates < 1 || a.gs_updates > gs_umax(KS))
    throw std::runtime_error("gs_estep: gs_updates must be in [1, " + std::to_string(gs_umax(KS)) + "] at KS " +
                             std::to_string(KS));
  if (!a.params) throw std::runtime_error("gs_estep: params block required");
  switch (KS) {
#define ONI_KS(X)                       \
  case X:                               \
    gs_estep_ks<X>(a, variant, s);      \
    break;
    ONI_FOR_EACH_KS(ONI_KS)
#undef ONI_KS
    default:
      throw std::runtime_error("gs_estep: unsupported KS " + std::to_string(KS));
  }
}

int gs_tiny_max(int KS) {
  switch (KS) {
#define ONI_KS(X) \
  case X:         \
    return gs::tiny_max(X);
    ONI_FOR_EACH_KS(ONI_KS)
#undef ONI_KS
    default:
      throw std::runtime_error("gs_tiny_max: unsupported KS " + std::to_string(KS));
  }
}

template <int KS>
constexpr int split_umax_ks() { return KS <= 52 ? 64 : kGsUMax; }   // chunk tables in LDS

int gs_split_lds_umax(int KS) {
  switch (KS) {
#define ONI_KS(X) \
  case X:         \
    return split_umax_ks<X>();
    ONI_FOR_EACH_KS(ONI_KS)
#undef ONI_KS
    default:
      return kGsUMax;
  }
}

// past the LDS tables, KS > 32 keeps its chunk tables in the launch's scratch (gs_splitw GM)
int gs_split_umax(int KS) { return KS > 32 ? kGsUMaxWide : gs_split_lds_umax(KS); }

template <int KS>
static int gs_split_capacity_ks() {
  int dev = 0, per_cu = 0;
  hipDeviceProp_t p;
  ONI_HIP_CHECK(hipGetDevice(&dev));
  ONI_HIP_CHECK(hipGetDeviceProperties(&p, dev));
  // the U <= 64 instantiation holds the larger LDS tables: where it exists its residency bounds both
  if constexpr (split_umax_ks<KS>() > kGsUMax)
    ONI_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &per_cu, reinterpret_cast<const void*>(&gs::gs_splitw<KS, split_umax_ks<KS>()>), 512, 0));
  else
    ONI_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &per_cu, reinterpret_cast<const void*>(&gs::gs_splitw<KS>), 512, 0));
  return per_cu * p.multiProcessorCount;
}

int gs_split_capacity(int KS) {
  switch (KS) {
#define ONI_KS(X) \
  case X:         \
    return gs_split_capacity_ks<X>();
    ONI_FOR_EACH_KS(ONI_KS)
#undef ONI_KS
    default:
      throw std::runtime_error("gs_split_capacity: unsupported KS " + std::to_string(KS));
  }
}

void launch_gs_split(const GSArgs& a, const SplitArgs& s, int KS, hipStream_t st) {
  if (s.n_blocks <= 0) return;
  const int um = gs_split_umax(KS);
  if (a.gs_updates < 1 || a.gs_updates > um)
    throw std::runtime_error("gs_split: gs_updates must be in [1, " + std::to_string(um) + "] at KS " +
                             std::to_string(KS));
  if (!a.params) throw std::runtime_error("gs_split: params block required");
  switch (KS) {
#define ONI_KS(X)                                                                                          \
  case X:                                                                                                  \
    if (a.gs_updates > split_umax_ks<X>()) {                                                               \
      if constexpr (X > 32) {                                                                              \
        if (!s.tab) throw std::runtime_error("gs_split: U past the LDS chunk tables needs the tab scratch");   \
        hipLaunchKernelGGL((gs::gs_splitw<X, kGsUMax, true>), dim3(s.n_blocks), dim3(512), 0, st, a, s);   \
      }                                                                                                    \
    } else if (a.gs_updates > kGsUMax) {                                                                   \
      if constexpr (split_umax_ks<X>() > kGsUMax)                                                          \
        hipLaunchKernelGGL((gs::gs_splitw<X, split_umax_ks<X>()>), dim3(s.n_blocks), dim3(512), 0, st, a, s); \
    } else                                                                                                 \
      hipLaunchKernelGGL((gs::gs_splitw<X>), dim3(s.n_blocks), dim3(512), 0, st, a, s);                    \
    break;
    ONI_FOR_EACH_KS(ONI_KS)
#undef ONI_KS
    default:
      throw std::runtime_error("gs_split: unsupported KS " + std::to_string(KS));
  }
  ONI_HIP_CHECK(hipGetLastError());
}

int suff_fused_blocks(int n_heavy, int n_medium, int n_light) {
  return n_heavy + (n_medium + 3) / 4 + (n_light + 15) / 16;
}

void launch_gs_suff64(const int* word_ptr, const int* csc_ent, const int* order, int n_heavy, int n_medium,
                      int n_light, const double* cphi, double* cw, double* part, const double* lik,
                      const double* ass, int lo, int hi, int KS, const double* gate, hipStream_t s,
                      const double* cw_base) {
  const int nb = suff_fused_blocks(n_heavy, n_medium, n_light);
  if (nb <= 0) return;
  switch (KS) {
#define ONI_KS(X)                                                                                        \
  case X:                                                                                                \
    hipLaunchKernelGGL((gs::gs_suff64<X>), dim3(nb), dim3(256), 0, s, word_ptr, csc_ent, order, n_heavy, \
                       n_medium, n_light, cphi, cw, part, lik, ass, lo, hi, gate, cw_base);              \
    break;
    ONI_FOR_EACH_KS(ONI_KS)
#undef ONI_KS
    default:
      throw std::runtime_error("gs_suff64: unsupported KS " + std::to_string(KS));
  }
  ONI_HIP_CHECK(hipGetLastError());
}

void launch_gs_mstep_control(const double* cw, const double* class_total, double* beta, int V, int K, int KS,
                             const int* rows, int n_rows, const EMControlArgs& c, const NewtonArgs& nw,
                             hipStream_t s, StageFuseArgs sf) {
  const int64_t total = (int64_t)(rows ? n_rows : V) * KS;
  int64_t blocks = (total / 2 + 255) / 256;
  if (blocks > 512) blocks = 512;
  if (blocks < 1) blocks = 1;
  if (nw.enabled) blocks += 1;   // block 0: the alpha Newton alone
  sf.blocks = 0;
  if (sf.n_sets > 0) {
    if (sf.n_sets > 2 || KS > 32 || KS % 2 || !sf.word_idx)
      throw std::runtime_error("gs_mstep_control: staged rows need 1-2 sets, an even KS <= 32 and word_idx");
    long long pos = 0;
    for (int i = 0; i < sf.n_sets; ++i) {
      if (sf.n_tiles[i] > 0 && (!sf.tile_ent[i] || !sf.tile_cnt[i] || !sf.out[i]))
        throw std::runtime_error("gs_mstep_control: staged set without its tables");
      pos += (long long)std::max(sf.n_tiles[i], 0) * 64;
    }
    if (pos > INT32_MAX) throw std::runtime_error("gs_mstep_control: too many staged positions");
    sf.blocks = (int)std::min<long long>((pos + 255) / 256, 1024);   // one thread per staged position
    blocks += sf.blocks;
  }
  if (sf.blocks == 0) {
    hipLaunchKernelGGL(gs::gs_mstep_control_kernel<0>, dim3((unsigned)blocks), dim3(256), 0, s, cw, class_total,
                       beta, V, K, KS, rows, n_rows, c, nw, sf);
  } else {
    switch (KS) {
#define ONI_KS(X)                                                                                          \
  case X:                                                                                                  \
    if constexpr (X <= 32 && X % 2 == 0)                                                                   \
      hipLaunchKernelGGL((gs::gs_mstep_control_kernel<X>), dim3((unsigned)blocks), dim3(256), 0, s, cw,    \
                         class_total, beta, V, K, KS, rows, n_rows, c, nw, sf);                            \
    break;
      ONI_FOR_EACH_KS(ONI_KS)
#undef ONI_KS
      default:
        throw std::runtime_error("gs_mstep_control: staged rows at unsupported KS " + std::to_string(KS));
    }
  }
  ONI_HIP_CHECK(hipGetLastError());
}

void launch_init_random_ss(double* cw, int V, int K, int KS, unsigned long long seed, hipStream_t s) {
  const long long total = (long long)V * KS;
  if (total <= 0) return;
  long long blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(gs::init_random_ss_kernel, dim3((unsigned)blocks), dim3(256), 0, s, cw, V, K, KS, seed);
  ONI_HIP_CHECK(hipGetLastError());
}

void launch_gs_mstep(const double* cw, const double* class_total, double* beta, int V, int K, int KS,
                     const double* gate, hipStream_t s) {
  const int64_t total = (int64_t)V * KS;
  if (total == 0) return;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(gs::gs_mstep_kernel, dim3((unsigned)blocks), dim3(256), 0, s, cw, class_total, beta, V, K, KS,
                     gate);
  ONI_HIP_CHECK(hipGetLastError());
}

}  // namespace oni
