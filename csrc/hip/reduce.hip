// Deterministic two-pass reductions for the EM step (replacing generic torch
// reductions that cost 12-25 us each at these sizes):
//   * colsum: class_total[k] = sum_w class_word[w][k]  (f32 [V][KS] -> f64 [KS])
// Pass 1 writes one partial per workgroup, pass 2 (one workgroup) adds the
// partials in workgroup order, so results are bitwise reproducible run to run
// and independent of stream scheduling.
#include <stdexcept>

#include "common.h"
#include "kernels.h"

namespace oni {

namespace {
constexpr int kRB = 256;   // pass-1 workgroups
constexpr int kRT = 256;   // threads per workgroup
}  // namespace

__global__ __launch_bounds__(kRT) void colsum_pass1(const float* __restrict__ m, int rows, int cols,
                                                    double* __restrict__ part, const double* gate) {
  if (gated(gate)) return;
  __shared__ double sh[kRT];
  const int groups = kRT / cols;                   // row groups per workgroup
  const int t = threadIdx.x;
  const int g = t / cols, k = t % cols;
  const int per = (rows + gridDim.x - 1) / gridDim.x;
  const int r0 = blockIdx.x * per, r1 = min(rows, r0 + per);
  double s = 0.0;
  if (g < groups)
    for (int r = r0 + g; r < r1; r += groups) s += (double)m[(size_t)r * cols + k];
  sh[t] = s;
  __syncthreads();
  if (t < cols) {
    double v = 0.0;
    for (int q = 0; q < groups; ++q) v += sh[q * cols + t];
    part[(size_t)blockIdx.x * cols + t] = v;
  }
}

// One wave per column (columns round-robin over the 4 waves): lane l adds the
// partials l, l+64, l+128, l+192 (independent loads), then a fixed butterfly.
__global__ __launch_bounds__(kRT) void colsum_pass2(const double* __restrict__ part, int nb, int cols,
                                                    double* __restrict__ out, const double* gate) {
  if (gated(gate)) return;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int k = wv; k < cols; k += kRT / 64) {
    double v[kRB / 64];
#pragma unroll
    for (int j = 0; j < kRB / 64; ++j) {
      const int b = lane + 64 * j;
      v[j] = b < nb ? part[(size_t)b * cols + k] : 0.0;
    }
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < kRB / 64; ++j) s += v[j];
    s = group_sum<64>(s);
    if (lane == 0) out[k] = s;
  }
}

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
// for the whole rank-order sum instead of a fill + one index_add per peer.  The
// fp32 adds run in source order (own row at the rank's own position), so every
// rank holding a word computes bitwise the same row.
__global__ __launch_bounds__(kRT) void rows_accumulate_kernel(const int* __restrict__ rows, const int* __restrict__ ptr,
                                                              const int* __restrict__ src,
                                                              const float4* __restrict__ own,
                                                              const float4* __restrict__ recv,
                                                              float4* __restrict__ out, int n_rows, int q) {
  const long g = (long)blockIdx.x * kRT + threadIdx.x;
  if (g >= (long)n_rows * q) return;
  const int i = (int)(g / q), c = (int)(g % q);
  const size_t dst = (size_t)rows[i] * q + c;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int j = ptr[i]; j < ptr[i + 1]; ++j) {
    const int from = src[j];
    const float4 v = from < 0 ? own[dst] : recv[(size_t)from * q + c];
    s.x += v.x;
    s.y += v.y;
    s.z += v.z;
    s.w += v.w;
  }
  out[dst] = s;
}

void launch_rows_accumulate(const int* rows, const int* ptr, const int* src, const float* own, const float* recv,
                            float* out, int n_rows, int width, hipStream_t s) {
  if (width % 4 != 0) throw std::runtime_error("rows_accumulate: width must be a multiple of 4");
  const long n = (long)n_rows * (width / 4);
  if (n <= 0) return;
  hipLaunchKernelGGL(rows_accumulate_kernel, dim3((unsigned)((n + kRT - 1) / kRT)), dim3(kRT), 0, s, rows, ptr, src,
                     reinterpret_cast<const float4*>(own), reinterpret_cast<const float4*>(recv),
                     reinterpret_cast<float4*>(out), n_rows, width / 4);
  ONI_HIP_CHECK(hipGetLastError());
}

int reduce_scratch_doubles(int cols) { return kRB * (cols > 2 ? cols : 2); }

void launch_colsum(const float* m, int rows, int cols, double* out, double* scratch, const double* gate,
                   hipStream_t s) {
  if (cols <= 0 || cols > kRT) throw std::runtime_error("colsum: cols out of range");
  hipLaunchKernelGGL(colsum_pass1, dim3(kRB), dim3(kRT), 0, s, m, rows, cols, scratch, gate);
  hipLaunchKernelGGL(colsum_pass2, dim3(1), dim3(kRT), 0, s, scratch, kRB, cols, out, gate);
  ONI_HIP_CHECK(hipGetLastError());
}

}  // namespace oni
