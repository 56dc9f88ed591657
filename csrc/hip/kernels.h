// Host-visible launch interface of the oni_ml_amd HIP kernels (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace oni {

// Padded topic counts (row stride of word-major beta, multiple of 4) that have
// compiled kernel instantiations.  Any K is served by the next larger entry;
// padding topics carry beta = 0 and are masked in the per-topic phase.
// Device parameter block (double[kParamCount]) read by the E-step kernels and
// written by the alpha Newton / EM control kernels; kParamDone != 0 gates every
// kernel of the EM iteration (device-side convergence, em_control.hip).
constexpr int kParamDone = 4;
constexpr int kParamCount = 8;
constexpr int kHistCols = 6;

#define ONI_FOR_EACH_KS(X) X(8) X(12) X(16) X(20) X(24) X(32) X(52) X(64) X(100) X(128)

// Huge documents (the long-context analogue): one document over
// several workgroups that exchange their per-chunk partials through global memory
// as tagged granules (launch_gs_split).  All workgroups of one launch must be
// co-resident: the host caps a launch below gs_split_capacity(KS).
struct SplitArgs {
  const int* seg_doc;     // [n_blocks] document of each workgroup
  const int* seg_index;   // [n_blocks] segment number within its document
  const int* seg_count;   // [n_blocks] segments of that document
  const int* seg_base;    // [n_blocks] block id of the document's segment 0
  const int* doc_slot;    // [n_blocks] counter slot of the document
  int n_blocks;
  int tab_rows;           // rows per workgroup of `tab` (>= nch of every document of the launch)
  unsigned long long* xchg;  // tagged granules (parity double-buffer), layout per kernel; gs_splitw:
                             // [2][n_blocks][2 (KS + 1)] partials, then [2][n_docs][2 (KS + 1)] totals
  int* counter;           // [2][n_docs] per document: launch epoch (tags of different launches never
                          // match), exit count (the last segment out bumps the epoch, resets the count)
  int n_docs;             // documents in this launch
  int* error;             // set to 1 if a wait times out (never hangs the GPU)
  double* tab = nullptr;  // U > the LDS table rows (KS > 32): per-segment chunk tables [n_blocks][tab_rows][2][KS]
  const double* csum = nullptr;  // [n_docs][csum_stride] chunk count sums of each document (nullptr: the
  int csum_stride = 0;           // kernel sums the counts itself)
};

// Sufficient-statistic launches: workgroups for [heavy | medium | light] word lists
// (a heavy word per workgroup, 4 medium or 16 light words per workgroup).
int suff_fused_blocks(int n_heavy, int n_medium, int n_light);

// alpha Newton on the device: reads scalars[1] (alpha_ss), writes params[0..1]
// (alpha, lgamma(K alpha) - K lgamma(alpha)) and alpha_out[0].
// Skipped once params[kParamDone] is set.
void launch_alpha_newton(const double* scalars, double num_docs, int K, bool estimate, double* params,
                         double* alpha_out, hipStream_t s);

// Device-side EM convergence test (em_control.hip), the lda-c driver loop
//   while ((conv < 0 || conv > EM_CONVERGED || i <= 2) && i <= EM_MAX_ITER)
// evaluated after each iteration without a host round trip.  ctl (double[8]):
//   [0] previous likelihood  [1] EM_CONVERGED  [2] history slot  [3] iteration i
//   [4] EM_MAX_ITER  [5] stop allowed (0: never set done)
// scalars = {likelihood, alpha_ss}.  It appends {likelihood, conv, alpha (params[0]),
// VAR_MAX_ITER, alpha_ss, -} (kHistCols
// doubles) to hist[slot], doubles
// VAR_MAX_ITER in params when the likelihood decreased (lda-c), and sets
// params[kParamDone] when the loop ends.
void launch_em_control(const double* scalars, double* params, double* ctl, double* hist, int hist_slots,
                       hipStream_t s);

// M-step fused with the EM control step (launch_gs_mstep_control): the last workgroup to finish
// (every other one has read the gate) runs em_control_step.  done_count: one int, zero before the
// first launch, left zero by the kernel.
struct EMControlArgs {
  const double* scalars;
  double* params;
  double* ctl;
  double* hist;
  int hist_slots;
  int* done_count;
};
// alpha Newton fused into the M-step: workgroup 0 runs it (lanes 0-1) beside the beta
// rows of the other workgroups; the control step (last workgroup) reads its alpha.
struct NewtonArgs {
  int enabled;            // 0: params[0..1] are left as they are
  int estimate;           // lda-c "alpha estimate" (else only the lgamma constant is refreshed)
  double num_docs;
  double* alpha_out;      // [1]
};
// ------------------------------------------------- fp64 block Gauss-Seidel ---
// lda-c-faithful E-step (lda_gs64.hip): everything in double, gamma / digamma refreshed
// after every chunk of W = ceil(n / U) words (U = gs_updates refreshes per sweep; a
// document of n <= U words is lda-c's literal per-word schedule).  The CPU oracle is
// csrc/native/lda_ref.cpp lda_inference(..., gs_updates).
constexpr int kGsUMax = 32;          // largest U with the chunk tables in LDS
constexpr int kGsUMaxWide = 4096;    // largest U at KS > 32 (chunk tables in the c*phi rows, gs_team GM)
enum GsVariant : int {
  kGsTiny = 0,     // TG lanes per document, literal schedule, n <= gs_tiny_max(KS)
  kGsTeam1 = 1,    // one wave per document
  kGsTeam4 = 2,    // one 4-wave workgroup per document
  kGsTeam8 = 3,    // one 8-wave workgroup per document (8 prefetched words per slot and chunk)
  kGsSmall = 4,    // 16 lanes per document: KS <= 32 tiny < n <= 64 words (register state); KS > 32 the
                   // one-wave range (gs_smallw, chunk tables in the c*phi rows)
  kGsChain = 5,    // KS > 32, U > 32: one wave per document, a topic per lane, rows of the next 8 words in
                   // flight (the planner routes chunks of W <= GSPlan.CHAIN_MAX_W = 2 words here:
                   // lda-c's per-word schedule, ops/hip.py wide_u_edges)
};
struct GSArgs {
  const int* doc_ptr;     // [D+1]
  const int* word_idx;    // [nnz]
  const float* counts;    // [nnz] (integer valued)
  const int* order;       // [n_items] documents of this launch
  int n_items;
  const double* beta;     // [V][KS] p(w|z) = exp(log_prob_w), word-major; 0 for padding topics
  int K;
  int gs_updates;         // U, 1 <= U <= gs_umax(KS)
  const double* params;   // {alpha, lgamma(K a) - K lgamma(a), VAR_MAX_ITER, VAR_CONVERGED, done, ...}
  double* gamma;          // [D][KS]
  double* cphi;           // [nnz][KS] c_n * phi_nk of the final sweep (sufficient-statistic input)
  double* lik;            // [D]
  double* alpha_ss;       // [D]
  int* iters;             // [D]
  // optional phase timer (scripts/bench_gs64.py --phases): workgroup 0, thread 0 of the team kernels
  // accumulates clock64() cycles into dbg[0..7]: word phase, slot reduction, barrier 1, topic phase,
  // barrier 2, sweep likelihood, final pass, chunks
  long long* dbg = nullptr;
  // optional staged rows (kGsTeam8 at KS <= 32, launch_gs_stage): item i's document has its beta rows
  // copied in document order to stage + stage_off[i] (double2 units), tiled [n/64][KS/2][64] so that a
  // wave's 64 consecutive words are 16-byte-contiguous per topic pair; stage_off[i] < 0: not staged
  const double* stage = nullptr;
  const long long* stage_off = nullptr;
};
void launch_gs_estep(const GSArgs& a, int variant, int KS, hipStream_t s);
// stage[(t KS/2 + k) 64 + l] (double2) = beta row pair k of the word at corpus entry tile_ent[t] + l
// (l < tile_cnt[t], else 0): the staged rows of launch_gs_estep, filled after every M-step
void launch_gs_stage(const double* beta, const int* word_idx, const int* tile_ent, const int* tile_cnt, int n_tiles,
                     double* stage, int KS, const double* gate, hipStream_t s);   // gate: as gs_mstep
int gs_tiny_max(int KS);   // longest document of the kGsTiny kernel
int gs_umax(int KS);       // largest gs_updates the E-step accepts at row stride KS
int gs_split_umax(int KS); // largest gs_updates of the split kernel (KS > 32: kGsUMaxWide, else 32 / 64)
int gs_split_lds_umax(int KS);   // largest gs_updates with the chunk tables in LDS (64 at KS <= 52, else 32)
// One long document over s.seg_count[b] workgroups (8 waves each): every chunk is cut into
// that many word ranges whose partials are exchanged as tagged granules (2 per double,
// s.xchg = [2][n_blocks][2 (KS + 1)]); s.seg_words is unused.  Every segment of a launch
// must be co-resident: n_blocks <= gs_split_capacity(KS) (the host keeps a margin).
void launch_gs_split(const GSArgs& a, const SplitArgs& s, int KS, hipStream_t st);
int gs_split_capacity(int KS);

// One long document over the CUs of one XCD (K <= 32, experimental/lda_xsplit.hip): G one-wave workgroups
// (blocks b = x + 8 m of a launch of 8 x groups blocks share XCD x under the round-robin dispatch),
// each holding its share of every chunk's beta rows in LDS for the whole E-step, exchange their
// per-chunk partial topic sums as 16-byte self-tagged granules.  proto 1: L2-resident stores, used
// only after the members have checked (one write-through round per launch) that they share an XCD;
// otherwise (and proto 0) write-through stores.  All members of a launch must be co-resident.
struct XSplitArgs {
  const int* seg_doc;     // [n_blocks] document of each block, -1: none (the block leaves at once)
  const int* seg_index;   // [n_blocks] member number within its document
  const int* seg_count;   // [n_blocks] members of that document
  const int* seg_base;    // [n_blocks] exchange row of the document's member 0
  const int* doc_slot;    // [n_blocks] counter slot of the document
  int n_blocks;           // grid
  int n_rows;             // exchange rows (members over all documents of the launch)
  unsigned* xchg;         // [2][n_rows][KS + 1] granules {lo, tag, hi, tag}
  int* counter;           // [2][n_docs] launch epoch, exit count (as SplitArgs)
  int n_docs;
  int* error;             // set to 1 if a wait times out (never hangs the GPU)
  int proto;              // 0: write-through stores; 1: L2-resident stores after the placement check
  int* placed;            // [n_docs] written by member 0: 1 = members on one XCD (and proto 1 used)
};
void launch_gs_xsplit(const GSArgs& a, const XSplitArgs& s, int KS, hipStream_t st);
int gs_xsplit_rows(int KS);   // LDS row capacity of one member (its words over all chunks of a sweep)

// class_word[w] = sum over w's CSC entries of cphi rows (fixed order, no atomics); part
// [nb][2 + KS] per-workgroup {lik slice, alpha_ss slice, column sums} for colsum_partials.
void launch_gs_suff64(const int* word_ptr, const int* csc_ent, const int* order, int n_heavy, int n_medium,
                      int n_light, const double* cphi, double* cw, double* part, const double* lik,
                      const double* ass, int lo, int hi, int KS, const double* gate, hipStream_t s,
                      const double* cw_base = nullptr);   // cw[w] = cw_base[w] + sum (nullable)
// Staged rows refilled by the M-step launch itself (trailing workgroups): the next E-step's staged
// copies of the longest documents' beta rows (launch_gs_stage's layout) computed straight from cw and
// class_total, so no separate stage launch (and its inter-kernel gap) sits between the M-step and the
// longest-document kernel.  n_sets = 0: none.
struct StageFuseArgs {
  const int* word_idx = nullptr;
  const int* tile_ent[2] = {nullptr, nullptr};
  const int* tile_cnt[2] = {nullptr, nullptr};
  double* out[2] = {nullptr, nullptr};
  int n_tiles[2] = {0, 0};
  int n_sets = 0;
  int blocks = 0;     // set by the launcher
};
// fp64 M-step + alpha Newton (workgroup 0) + EM control (last workgroup) [+ staged rows]
void launch_gs_mstep_control(const double* cw, const double* class_total, double* beta, int V, int K, int KS,
                             const int* rows, int n_rows, const EMControlArgs& c, const NewtonArgs& nw,
                             hipStream_t s, StageFuseArgs sf = StageFuseArgs());
// lda-c random start on the device: cw[w][k] = 1/V + u(seed, k V + w) (k < K), 0 for padding;
// the same values as csrc/native random_ss (counter-based splitmix64).
void launch_init_random_ss(double* cw, int V, int K, int KS, unsigned long long seed, hipStream_t s);
void launch_gs_mstep(const double* cw, const double* class_total, double* beta, int V, int K, int KS,
                     const double* gate, hipStream_t s);

// ------------------------------------------------------------- reductions ---
// Deterministic reductions (reduce.hip).  gate (nullable): skip when *gate != 0.
// out[k] = sum_b part[b][k] (b in order), the second pass of the fused suff-stats.
void launch_colsum_partials(const double* part, int nb, int cols, double* out, const double* gate, hipStream_t s);
// out [K][V] = log(cw[v][k]) - log(ct[k]) (floor_v where cw == 0): the saved log beta in file order.
void launch_log_beta_t(const double* cw, int V, int K, int ld, const double* ct, double floor_v, double* out,
                       hipStream_t s);
// Sparse class_word exchange: out[rows[i]] = 0 + src_0 + src_1 + ... over row i's sources
// (CSR ptr/src; src >= 0: recv row, src < 0: the rank's own row own[rows[i]]), fp64, double2 granules.
void launch_rows_accumulate(const int* rows, const int* ptr, const int* src, const double* own, const double* recv,
                            double* out, int n_rows, int width, hipStream_t s);

// ---------------------------------------------------------------- scoring ---
struct ScoreArgs {
  const double* theta;    // [D][K] p(z|d)
  const double* phi;      // [V][K] p(w|z)
  int K;                  // topics summed (reference: 20)
  double dflt;            // value of the default vector used for misses
  const int* doc_a;       // [n] doc index or -1
  const int* word_a;      // [n] word index or -1
  const int* doc_b;       // [n] (flow: destination side) or nullptr
  const int* word_b;      // [n]
  int64_t n;
  double tol;
  double* score_a;        // [n]
  double* score_b;        // [n] or nullptr
  double* key;            // [n] min(score_a, score_b) (or score_a)
  uint8_t* flag;          // [n] key < tol
};
void launch_score_events(const ScoreArgs& a, hipStream_t s);

// ------------------------------------------------------------ flow words ---
struct FlowWordArgs {
  const double* hour;      // [n] col 4
  const double* minute;    // [n] col 5
  const double* second;    // [n] col 6
  const double* port_a;    // [n] col 10 (reference variable name: dport)
  const double* port_b;    // [n] col 11 (reference variable name: sport)
  const double* ipkt;      // [n] col 16
  const double* ibyt;      // [n] col 17
  const double* time_cuts; // [n_time_cuts]
  const double* ibyt_cuts;
  const double* ipkt_cuts;
  int n_time_cuts, n_ibyt_cuts, n_ipkt_cuts;
  int64_t n;
  double* time_out;        // [n] col 27
  int8_t* time_bin;        // [n]
  int8_t* ibyt_bin;        // [n]
  int8_t* ipkt_bin;        // [n]
  double* word_port;       // [n]
  int8_t* p_case;          // [n]
  int8_t* src_prefix;      // [n] 1 if src word carries "-1_"
  int8_t* dst_prefix;      // [n]
};
void launch_flow_words(const FlowWordArgs& a, hipStream_t s);

// bins[i*ncols + c] = #{cut in cuts_c : value_c[i] > cut}   (generic binning)
void launch_bin_columns(const double* const* values, const double* const* cuts, const int* ncuts,
                        int ncols, int64_t n, int8_t* bins, hipStream_t s);

}  // namespace oni
