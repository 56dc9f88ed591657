// One long document over the CUs of one XCD, K <= 32 (the SP/CP analogue).
//
// Why: at K <= 32 the longest document of a day (22,721 words on the headline day) is a serial
// chain of 20 sweeps x U = 32 chunks.  On one workgroup (lda_gs64.hip gs_wsteam) a chunk costs
// ~2.7 us, most of it streaming the chunk's ~711 beta rows (114 KB) through ONE CU's memory pipe;
// the round-3 split kernel (gs_splitw) spread those rows over a few CUs but paid ~2 us per chunk
// for the exchange, whose polls queued behind the row prefetches in the same CU's memory queue.
//
// Here each of G one-wave workgroups (members) keeps ITS share of every chunk's rows resident in
// LDS for the whole E-step (G >= n x 8 KS / 150 KB: 27 members for the 22,721-word document), so
// after the start no member issues a global load except the exchange's own polls:
//   word phase   lane = word of the member's range of chunk j (rows from LDS, transposed [k][row]:
//                conflict-free), P = sum_k E_k b_k, r = c / P, acc_k = r b_k;
//   reduction    wave_topic_sums_reg (permlane swaps + DPP): topic totals left in registers;
//   publish      the lanes holding a topic total store it as ONE 16-byte granule {lo, tag, hi, tag}
//                (each 8-byte half self-tagged: a reader that sees both tags sees the value);
//   gather       lane (column c, part p) polls the granules of members [p G/NP, (p+1) G/NP) of
//                column c, sums them in member order (fixed tree), parts combined by a permlane32
//                swap: every member gets bitwise the same totals;
//   refresh      lane k < K: gamma_k += E_k S_k - C_jk, psi / E by psi_exp (gs_math.h), exactly the
//                arithmetic of the one-workgroup kernels, replicated in every member.
// The sweep's c log P sum (likelihood only) rides as column KS of the LAST chunk of each sweep;
// for the other chunks the logs are taken after the publish, beside the exchange latency.
//
// Placement: the host puts a document's members on blocks b = x + 8 m (one XCD under the observed
// round-robin dispatch; a speed matter only).  proto 0 stores write-through (sc1), valid for any
// placement.  proto 1 first runs one write-through round in which members exchange their
// HW_REG_XCC_ID; only if all share one XCD do they switch to L2-resident stores (the line stays in
// that XCD's L2, which every member's L1-bypassing sc1 load reads) -- otherwise they stay on sc1.
// Every wait is bounded (error flag, NaN likelihood -> RuntimeError on the host), never a hang.
// Tags: (launch epoch + 1, sequence number), parity double buffer as gs_split (lda_gs64.hip).
// Oracle: csrc/native/lda_ref.cpp lda_inference(..., gs_updates) (tests/test_gs64.py).
#include <stdexcept>
#include <string>

#include "common.h"
#include "estep_common.h"
#include "gs_math.h"
#include "kernels.h"

namespace oni {
namespace gs {

typedef unsigned xu4 __attribute__((ext_vector_type(4)));

template <int KS>
struct XGeom {
  // chunk tables C, Et (U <= 32 rows), E, chunk count sums, small scalars
  static constexpr int TAB = 2 * kGsUMax * KS * 8 + KS * 8 + kGsUMax * 8 + 512;
  // rows: KS doubles + one float count each; a multiple of 64 rows, within 160 KB of LDS
  static constexpr int ROWS = ((160 * 1024 - TAB - 1024) / (KS * 8 + 4)) / 64 * 64;
  static constexpr int NC = KS + 1;                // exchanged columns: KS topic sums + c log P
  static constexpr int CL = NC <= 32 ? 32 : 64;    // lanes per member part
  static constexpr int NP = 64 / CL;               // member parts per column
};

__device__ __forceinline__ unsigned xtag(int epoch, int seq) {
  return ((unsigned)((epoch + 1) & 0xfffff) << 12) | (unsigned)(seq & 0xfff);   // never 0 (zeroed buffers)
}

// one double as a 16-byte granule {lo, tag, hi, tag}: write-through (sc1) or L2-resident (default policy)
__device__ __forceinline__ void xput(__amdgpu_buffer_rsrc_t rs, int off, double v, unsigned tag, bool wt) {
  const unsigned long long bits = (unsigned long long)__double_as_longlong(v);
  const xu4 q = {(unsigned)bits, tag, (unsigned)(bits >> 32), tag};
  if (wt)
    __builtin_amdgcn_raw_buffer_store_b128(q, rs, off, 0, 16);
  else
    __builtin_amdgcn_raw_buffer_store_b128(q, rs, off, 0, 0);
}

// Sum of the granules (member u = 0..cnt-1 at off0 + u * stride bytes) carrying `tag`, in member order
// (fixed pairwise tree over MP slots, the absent ones 0.0: the same bits in every member).  Every pass
// issues all MP loads back to back -- a load inside a per-granule branch gets its own vmcnt(0) wait, one
// L2 round trip per granule (scripts/micro/xcd_exchange.hip: 2.3 -> 1.0 us per 32-member round) -- and
// a pass that finds any stale granule is repeated whole.  Loads bypass L1 (sc1): a line another CU
// rewrote is read from L2.
template <int MP>
__device__ __forceinline__ bool xsum(__amdgpu_buffer_rsrc_t rs, int off0, int stride, int cnt, unsigned tag,
                                     double& out) {
  double v[MP];
  long spins = 0;
  for (;;) {
    bool ok = true;
#pragma unroll
    for (int u = 0; u < MP; ++u) {
      const int uu = u < cnt ? u : 0;   // absent slots re-read member 0's granule (no extra line)
      const xu4 q = __builtin_amdgcn_raw_buffer_load_b128(rs, off0 + uu * stride, 0, 16);
      v[u] = u < cnt ? __longlong_as_double((long long)(((unsigned long long)q.z << 32) | q.x)) : 0.0;
      ok &= u >= cnt || (q.y == tag && q.w == tag);
    }
    asm volatile("" ::: "memory");   // the next pass re-issues the loads
    if (ok) break;
    if (++spins > kSplitSpinLimit) {
      out = __builtin_nan("");
      return false;
    }
  }
#pragma unroll
  for (int h = 1; h < MP; h *= 2)
#pragma unroll
    for (int u = 0; u + h < MP; u += 2 * h) v[u] += v[u + h];
  out = v[0];
  return true;
}

template <int KS>
__global__ __launch_bounds__(256) void gs_xsplit(GSArgs a, XSplitArgs sp) {
  static_assert(KS <= 32 && KS % 2 == 0, "xsplit: even KS <= 32");
  using X = XGeom<KS>;
  constexpr int ROWS = X::ROWS, NC = X::NC, CL = X::CL, NP = X::NP, MP = (32 + NP - 1) / NP;
  __shared__ double sB[KS * ROWS];          // this member's beta rows, [k][row], row = j WG + i
  __shared__ float sN[ROWS];                // their counts
  __shared__ double sC[kGsUMax][KS];        // chunk contributions (previous sweep)
  __shared__ double sEt[kGsUMax][KS];       // E each chunk used (final pass)
  __shared__ double sE[KS];                 // current E
  __shared__ double sCs[kGsUMax];           // chunk count sums (the whole chunk, every member's words)
  if (a.params[kParamDone] != 0.0) return;
  const int b = blockIdx.x, t = threadIdx.x;
  const int d = sp.seg_doc[b];
  if (d < 0) return;                        // a block of no document (the grid covers 8 XCD groups)
  const int g = sp.seg_index[b], G = sp.seg_count[b], base = sp.seg_base[b];
  int* counter = sp.counter + sp.doc_slot[b];
  const int epoch = __hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const double alpha = a.params[0], lik_const = a.params[1];
  const int vmi = (int)a.params[2];
  const double vconv = params_vconv(a.params);
  const int K = a.K;
  const int s0 = a.doc_ptr[d], n = a.doc_ptr[d + 1] - s0;   // n > 0 (host)
  const int U = a.gs_updates;                                // <= kGsUMax (host)
  const int W = (n + U - 1) / U;
  const int nch = (n + W - 1) / W;
  const int WG = (W + G - 1) / G;                            // nch x WG <= ROWS (host)
  const int* __restrict__ wrow = a.word_idx + s0;
  const float* __restrict__ crow = a.counts + s0;
  auto range = [&](int j, int& m0, int& m1) {
    const int n1 = min(n, (j + 1) * W);
    m0 = min(n1, j * W + g * WG);
    m1 = min(n1, m0 + WG);
  };
  // ---- load phase (4 waves): this member's rows into LDS, chunk count sums
  for (int j = t; j < kGsUMax; j += 256) sCs[j] = 0.0;
  __syncthreads();
  for (int p = t; p < n; p += 256) atomicAdd(&sCs[p / W], (double)crow[p]);   // integer counts: exact
  const int R = nch * WG;
  for (int r = t; r < R; r += 256) {
    const int j = r / WG, i = r - j * WG;
    int m0, m1;
    range(j, m0, m1);
    const bool ok = i < m1 - m0;
    const dvec2* brow = reinterpret_cast<const dvec2*>(a.beta + (size_t)(ok ? wrow[m0 + i] : 0) * KS);
#pragma unroll
    for (int k = 0; k < KS / 2; ++k) {
      const dvec2 v = ok ? brow[k] : dvec2{0.0, 0.0};
      sB[(2 * k) * ROWS + r] = v.x;
      sB[(2 * k + 1) * ROWS + r] = v.y;
    }
    sN[r] = ok ? crow[m0 + i] : 0.0f;
  }
  __syncthreads();
  if (t >= 64) return;                      // waves 1-3 only helped to load
  // ---- one wave from here on: no workgroup barrier, LDS ordered by wave_lds_sync
  const int lane = t;
  double total = 0.0;
  for (int j = 0; j < nch; ++j) total += sCs[j];
  const double g0 = alpha + total / K;
  const double m = psi_only(g0);
  const int bytes = 2 * sp.n_rows * NC * 16;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(sp.xchg, 0, bytes, 0x00020000);
  auto goff = [&](int seq, int row, int col) { return (((seq & 1) * sp.n_rows + row) * NC + col) * 16; };
  bool failed = false;
  // placement check (proto 1): one write-through round, seq 0, column 0 = this member's XCC id
  bool wt = true;
  if (sp.proto == 1) {
    const unsigned tag0 = xtag(epoch, 0);
    const unsigned xc = (unsigned)__builtin_amdgcn_s_getreg((3 << 11) | 20) & 0xfu;   // HW_REG_XCC_ID
    if (lane == 0) xput(rs, goff(0, base + g, 0), (double)xc, tag0, true);
    double other = (double)xc;
    if (lane < G) {
      double s;
      failed = !xsum<1>(rs, goff(0, base + lane, 0), 0, 1, tag0, s);
      other = s;
    }
    const bool same = __all(failed || other == (double)xc);
    failed = __any(failed);
    wt = !same;
    if (lane == 0 && g == 0) sp.placed[sp.doc_slot[b]] = same ? 1 : 0;
  }
  // topic state: lane k owns topic k (replicated in every member)
  const int k = lane;
  double gam = k < K ? g0 : 0.0, psi = m, lps = 0.0;
  double Ecur = k < K ? 1.0 : 0.0;
  if (k < KS) {
    sE[k] = Ecur;
    for (int j = 0; j < nch; ++j) sC[j][k] = k < K ? sCs[j] / K : 0.0;
  }
  wave_lds_sync();
  double L = 0.0, L_old = 0.0, conv = 1.0, GS = 0.0;
  int it = 0;
  // phase timer (scripts/bench_gs64.py --phases): member 0 of the launch's first document, cycles per
  // E-step of the word phase + reduction, publish -> gathered, refresh; chunks
  const bool timer = a.dbg != nullptr && base == 0 && g == 0;
  long long ph[4] = {0, 0, 0, 0};
  long long tc = timer ? clock64() : 0;
  auto tick = [&](int i) {
    if (timer) {
      const long long x = clock64();
      ph[i] += x - tc;
      tc = x;
    }
  };
  const int col = lane & (CL - 1), part = lane / CL;
  const int q0 = part * G / NP, q1 = (part + 1) * G / NP;
  while (!failed && var_continue(conv, vconv, it, vmi)) {
    ++it;
    lps = 0.0;
    double lw = 0.0, LWs = 0.0;
    for (int j = 0; j < nch; ++j) {
      const bool last = j == nch - 1;
      const int seq = (it - 1) * nch + j + 1;
      const unsigned tag = xtag(epoch, seq);
      int m0, m1;
      range(j, m0, m1);
      const int cnt = m1 - m0, row0 = j * WG;
      double E[KS], acc[KS];
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
        E[kk] = sE[kk];
        acc[kk] = 0.0;
      }
      const double gC = k < KS ? gam - sC[j][k] : 0.0;   // off the chain
      // word phase: round 0 keeps P and c for the deferred log, further rounds take it at once
      double P0 = 1.0, c0 = 0.0;
      for (int i0 = 0; i0 < cnt; i0 += 64) {
        const int i = i0 + lane;
        const int r = min(row0 + i, ROWS - 1);
        const double c = i < cnt ? (double)sN[r] : 0.0;
        double bv[KS];
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) bv[kk] = sB[kk * ROWS + r];
        double p0 = 0.0, p1 = 0.0, p2 = 0.0, p3 = 0.0;
#pragma unroll
        for (int kk = 0; kk < KS; kk += 4) {
          p0 = fma(E[kk], bv[kk], p0);
          if (kk + 1 < KS) p1 = fma(E[kk + 1], bv[kk + 1], p1);
          if (kk + 2 < KS) p2 = fma(E[kk + 2], bv[kk + 2], p2);
          if (kk + 3 < KS) p3 = fma(E[kk + 3], bv[kk + 3], p3);
        }
        const double P = c > 0.0 ? (p0 + p1) + (p2 + p3) : 1.0;
        const double rr = c * drcp(P);
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) acc[kk] = fma(rr, bv[kk], acc[kk]);
        if (i0 == 0) {
          P0 = P;
          c0 = c;
        } else {
          lw = fma(c, flog(P), lw);
        }
      }
      double v;
      const int tk = wave_topic_sums_reg<KS>(acc, lane, v);
      if (last) {   // the sweep's log sum rides on the last chunk: taken before the publish
        lw = fma(c0, flog(P0), lw);
        const double lws = group_sum<64>(lw);
        if (lane == 63) v = lws;
      }
      tick(0);
      if (tk >= 0) xput(rs, goff(seq, base + g, tk), v, tag, wt);
      if (lane == 63) xput(rs, goff(seq, base + g, KS), last ? v : 0.0, tag, wt);
      if (!last) lw = fma(c0, flog(P0), lw);   // beside the exchange latency
      // gather: column col over members [q0, q1), parts combined in order
      double S = 0.0;
      bool ok = true;
      if (col < NC) ok = xsum<MP>(rs, goff(seq, base + q0, col), NC * 16, q1 - q0, tag, S);
      if constexpr (NP == 2) S = detail::swap_combine<true>(S, detail::add<double>);
      tick(1);
      if (__any(!ok)) {
        failed = true;
        if (lane == 0) __hip_atomic_store(sp.error, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      // refresh (lane k < KS), the arithmetic of gs_wsteam's topic wave
      if (k < KS) {
        const double Eo = Ecur;
        const double nw = Eo * S;
        double En = 0.0;
        if (k < K) {
          lps = fma(psi, nw, lps);
          gam = fma(Eo, S, gC);
          psi_exp(gam, m, psi, En);
        }
        sE[k] = En;
        sC[j][k] = nw;
        sEt[j][k] = Eo;
        Ecur = En;
      } else if (k == KS) {
        LWs = S;   // meaningful on the last chunk only
      }
      wave_lds_sync();
      tick(2);
      ph[3] += timer ? 1 : 0;
    }
    if (failed) break;
    const bool own = k < K;
    GS = group_sum<64>(own ? gam : 0.0);
    const double LG = group_sum<64>(own ? lgamma_pos(gam) : 0.0);
    const double LP = group_sum<64>(own ? lps : 0.0);
    const double LW = detail::rdlane(LWs, KS);
    L = lik_const - lgamma_pos(GS) + LG + fma(m, total, LW) - LP;
    conv = (L_old - L) / L_old;
    L_old = L;
  }
  if (timer && lane == 0)
    for (int i = 0; i < 4; ++i) a.dbg[i] = ph[i];
  // every lane of this member is past its last exchange read
  split_exit(counter, sp.n_docs, G);
  const double ps = group_sum<64>(k < K ? psi : 0.0);
  if (g == 0) {
    if (k < KS) a.gamma[(size_t)d * KS + k] = gam;
    if (lane == 0) {
      a.lik[d] = failed ? __builtin_nan("") : L;   // a timed-out exchange surfaces as a NaN likelihood
      a.alpha_ss[d] = ps - K * psi_only(GS);
      a.iters[d] = it;
    }
  }
  if (failed) return;
  // final pass over this member's words: c_n phi_nk = E_jk b_nk r_n with the final sweep's chunk E
  for (int j = 0; j < nch; ++j) {
    int m0, m1;
    range(j, m0, m1);
    const int cnt = m1 - m0, row0 = j * WG;
    double E[KS];
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) E[kk] = sEt[j][kk];
    for (int i = lane; i < cnt; i += 64) {
      const int r = row0 + i;
      double bv[KS];
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) bv[kk] = sB[kk * ROWS + r];
      double p0 = 0.0, p1 = 0.0, p2 = 0.0, p3 = 0.0;
#pragma unroll
      for (int kk = 0; kk < KS; kk += 4) {
        p0 = fma(E[kk], bv[kk], p0);
        if (kk + 1 < KS) p1 = fma(E[kk + 1], bv[kk + 1], p1);
        if (kk + 2 < KS) p2 = fma(E[kk + 2], bv[kk + 2], p2);
        if (kk + 3 < KS) p3 = fma(E[kk + 3], bv[kk + 3], p3);
      }
      const double rr = (double)sN[r] * drcp((p0 + p1) + (p2 + p3));
      dvec2* out = reinterpret_cast<dvec2*>(a.cphi + (size_t)(s0 + m0 + i) * KS);
#pragma unroll
      for (int kk = 0; kk < KS / 2; ++kk) {
        const dvec2 w2 = {E[2 * kk] * bv[2 * kk] * rr, E[2 * kk + 1] * bv[2 * kk + 1] * rr};
        __builtin_nontemporal_store(w2, &out[kk]);
      }
    }
  }
}

}  // namespace gs

int gs_xsplit_rows(int KS) {
  switch (KS) {
#define ONI_KS(X) \
  case X:         \
    return (X <= 32 && X % 2 == 0) ? gs::XGeom<X>::ROWS : 0;
    ONI_FOR_EACH_KS(ONI_KS)
#undef ONI_KS
    default:
      return 0;
  }
}

void launch_gs_xsplit(const GSArgs& a, const XSplitArgs& s, int KS, hipStream_t st) {
  if (s.n_blocks <= 0) return;
  if (a.gs_updates < 1 || a.gs_updates > kGsUMax)
    throw std::runtime_error("gs_xsplit: gs_updates must be in [1, " + std::to_string(kGsUMax) + "]");
  if (!a.params) throw std::runtime_error("gs_xsplit: params block required");
  if (!s.xchg || !s.counter || !s.error || !s.placed || s.n_rows <= 0)
    throw std::runtime_error("gs_xsplit: exchange buffers required");
  switch (KS) {
#define ONI_KS(X)                                                                                  \
  case X:                                                                                          \
    if constexpr (X <= 32 && X % 2 == 0) {                                                         \
      hipLaunchKernelGGL((gs::gs_xsplit<X>), dim3(s.n_blocks), dim3(256), 0, st, a, s);            \
      break;                                                                                       \
    }                                                                                              \
    throw std::runtime_error("gs_xsplit: KS " + std::to_string(KS) + " (even KS <= 32 only)");
    ONI_FOR_EACH_KS(ONI_KS)
#undef ONI_KS
    default:
      throw std::runtime_error("gs_xsplit: unsupported KS " + std::to_string(KS));
  }
  ONI_HIP_CHECK(hipGetLastError());
}

}  // namespace oni
