// Deterministic reductions of the EM step (replacing generic torch reductions that
// cost 12-25 us each at these sizes):
//   * colsum_partials: {likelihood, alpha_ss, class_total} from the per-workgroup
//     partial rows of the suff-stats launch, added in workgroup order;
//   * rows_accumulate: the sparse class_word exchange's rank-order row sums (fp64).
// Every sum runs in a fixed order, so results are bitwise reproducible run to run
// and independent of stream scheduling.
#include <stdexcept>

#include "common.h"
#include "kernels.h"

namespace oni {

namespace {
constexpr int kRT = 256;   // threads per workgroup
}  // namespace

// out[k] = sum_b part[b][k] over the per-workgroup column sums of the fused
// suff-stats kernel: one workgroup per column, rows strided over 256 lanes with
// 8 loads in flight, fixed-order wave and cross-wave combination.
__global__ __launch_bounds__(kRT) void colsum_partials_kernel(const double* __restrict__ part, int nb, int cols,
                                                              double* __restrict__ out, const double* gate) {
  if (gated(gate)) return;
  __shared__ double sw[kRT / 64];
  const int k = blockIdx.x, t = threadIdx.x;
  double s = 0.0;
  for (int b0 = t; b0 < nb; b0 += 8 * kRT) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int b = b0 + u * kRT;
      v[u] = b < nb ? part[(size_t)b * cols + k] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  s = group_sum<64>(s);
  if ((t & 63) == 0) sw[t >> 6] = s;
  __syncthreads();
  if (t == 0) {
    double r = 0.0;
#pragma unroll
    for (int w = 0; w < kRT / 64; ++w) r += sw[w];
    out[k] = r;
  }
}

void launch_colsum_partials(const double* part, int nb, int cols, double* out, const double* gate, hipStream_t s) {
  if (cols <= 0) return;
  hipLaunchKernelGGL(colsum_partials_kernel, dim3(cols), dim3(kRT), 0, s, part, nb, cols, out, gate);
  ONI_HIP_CHECK(hipGetLastError());
}

// Sparse class_word exchange (parallel/dist.py VocabExchange.accumulate): one launch
// for the whole rank-order sum instead of a fill + one index_add per peer.  The fp64
// adds run in source order (own row at the rank's own position), starting from +0.0,
// so every rank holding a word computes bitwise the same row -- and the same bits as
// torch's index_fill_(0) + index_add_ per source in that order.  One thread per
// double2 granule of a row (KS is even for every compiled topic count).
__global__ __launch_bounds__(kRT) void rows_accumulate_kernel(const int* __restrict__ rows, const int* __restrict__ ptr,
                                                              const int* __restrict__ src,
                                                              const double2* __restrict__ own,
                                                              const double2* __restrict__ recv,
                                                              double2* __restrict__ out, int n_rows, int q) {
  const long g = (long)blockIdx.x * kRT + threadIdx.x;
  if (g >= (long)n_rows * q) return;
  const int i = (int)(g / q), c = (int)(g % q);
  const size_t dst = (size_t)rows[i] * q + c;
  double2 s = make_double2(0.0, 0.0);
  const int j1 = ptr[i + 1];
  for (int j = ptr[i]; j < j1; ++j) {
    const int from = src[j];
    const double2 v = from < 0 ? own[dst] : recv[(size_t)from * q + c];
    s.x += v.x;
    s.y += v.y;
  }
  out[dst] = s;
}

void launch_rows_accumulate(const int* rows, const int* ptr, const int* src, const double* own, const double* recv,
                            double* out, int n_rows, int width, hipStream_t s) {
  if (width % 2 != 0) throw std::runtime_error("rows_accumulate: width must be even");
  const long n = (long)n_rows * (width / 2);
  if (n <= 0) return;
  hipLaunchKernelGGL(rows_accumulate_kernel, dim3((unsigned)((n + kRT - 1) / kRT)), dim3(kRT), 0, s, rows, ptr, src,
                     reinterpret_cast<const double2*>(own), reinterpret_cast<const double2*>(recv),
                     reinterpret_cast<double2*>(out), n_rows, width / 2);
  ONI_HIP_CHECK(hipGetLastError());
}

}  // namespace oni

namespace oni {

// Model files (LAG saves, final.beta): out[k][v] = log(cw[v][k]) - log(ct[k]), or `floor` where cw[v][k] == 0 --
// lda-c's saved log beta, transposed to its [K][V] file order.  One thread per (k, v), v fastest: the [K][V]
// writes coalesce, the cw reads stride KS doubles (the whole matrix is read once).  Replaces torch's transpose /
// log / where chain on the save path: the same ocml log in the same order (bitwise the torch result), and no
// first use of torch's elementwise kernels inside the EM loop of a fresh process.
__global__ __launch_bounds__(kRT) void log_beta_t_kernel(const double* __restrict__ cw, int V, int K, int ld,
                                                         const double* __restrict__ ct, double floor_v,
                                                         double* __restrict__ out) {
  const long long i = (long long)blockIdx.x * kRT + threadIdx.x;
  if (i >= (long long)V * K) return;
  const int k = (int)(i / V), v = (int)(i - (long long)k * V);
  const double c = cw[(size_t)v * ld + k];
  out[i] = c > 0.0 ? log(c) - log(ct[k]) : floor_v;
}

void launch_log_beta_t(const double* cw, int V, int K, int ld, const double* ct, double floor_v, double* out,
                       hipStream_t s) {
  const long long n = (long long)V * K;
  if (n <= 0) return;
  hipLaunchKernelGGL(log_beta_t_kernel, dim3((unsigned)((n + kRT - 1) / kRT)), dim3(kRT), 0, s, cw, V, K, ld, ct,
                     floor_v, out);
  ONI_HIP_CHECK(hipGetLastError());
}

}  // namespace oni
