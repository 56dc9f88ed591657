// Flow word-ification (reference: flow_pre_lda.scala:272-358 add_time,
// bin_ibyt_ipkt_time, adjust_port; SURVEY.md C4d/C4e, hot ops H10/H11).
//
// One thread per event computes, in strict IEEE double (no contraction):
//   time      = hour + minute/60 + second/3600            (col 27)
//   *_bin     = #{cut : value > cut}                      (cols 28-30)
//   word_port / p_case / "-1_" prefix side per adjust_port
// with the reference's column naming quirk preserved: a = col 10 is called
// `dport` and b = col 11 `sport` inside adjust_port.  Word strings are never
// built here; the host packs (port id, bins, prefix) into integer word keys.
#include <stdexcept>
#include <string>

#include "common.h"
#include "kernels.h"

namespace oni {

__device__ __forceinline__ int8_t count_gt(double v, const double* cuts, int n) {
  int b = 0;
  for (int i = 0; i < n; ++i) b += (v > cuts[i]) ? 1 : 0;
  return (int8_t)b;
}

__global__ __launch_bounds__(256) void flow_words_kernel(FlowWordArgs a) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const double t = __dadd_rn(__dadd_rn(a.hour[i], __ddiv_rn(a.minute[i], 60.0)), __ddiv_rn(a.second[i], 3600.0));
    a.time_out[i] = t;
    const int8_t tb = count_gt(t, a.time_cuts, a.n_time_cuts);
    const int8_t bb = count_gt(a.ibyt[i], a.ibyt_cuts, a.n_ibyt_cuts);
    const int8_t pb = count_gt(a.ipkt[i], a.ipkt_cuts, a.n_ipkt_cuts);
    a.time_bin[i] = tb;
    a.ibyt_bin[i] = bb;
    a.ipkt_bin[i] = pb;

    const double dp = a.port_a[i];  // reference "dport" = col 10
    const double sp = a.port_b[i];  // reference "sport" = col 11
    const double mn = dp < sp ? dp : sp;
    const double mx = dp > sp ? dp : sp;
    double wp;
    int8_t pc;
    if ((dp <= 1024.0 || sp <= 1024.0) && (dp > 1024.0 || sp > 1024.0) && mn != 0.0) {
      pc = 2;
      wp = mn;
    } else if (dp > 1024.0 && sp > 1024.0) {
      pc = 3;
      wp = 333333.0;
    } else if (dp == 0.0 && sp != 0.0) {
      pc = 4;
      wp = sp;
    } else if (sp == 0.0 && dp != 0.0) {
      pc = 4;
      wp = dp;
    } else {
      pc = 1;
      wp = (mn == 0.0) ? mx : 111111.0;
    }
    int8_t spre = 0, dpre = 0;
    if (pc == 2 && dp < sp) dpre = 1;
    else if (pc == 2 && sp < dp) spre = 1;
    else if (pc == 4 && dp == 0.0) spre = 1;
    else if (pc == 4 && sp == 0.0) dpre = 1;
    a.word_port[i] = wp;
    a.p_case[i] = pc;
    a.src_prefix[i] = spre;
    a.dst_prefix[i] = dpre;
  }
}

void launch_flow_words(const FlowWordArgs& a, hipStream_t s) {
  if (a.n <= 0) return;
  int64_t blocks = (a.n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(flow_words_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a);
  ONI_HIP_CHECK(hipGetLastError());
}

// Generic multi-column binning (DNS: frame_len, unix_tstamp, subdomain length,
// entropy, label count).  Column pointers live in a small device array.
struct BinCols {
  const double* v[8];
  const double* c[8];
  int nc[8];
};

__global__ __launch_bounds__(256) void bin_columns_kernel(BinCols bc, int ncols, int64_t n, int8_t* bins) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    for (int c = 0; c < ncols; ++c) bins[i * ncols + c] = count_gt(bc.v[c][i], bc.c[c], bc.nc[c]);
  }
}

void launch_bin_columns(const double* const* values, const double* const* cuts, const int* ncuts, int ncols,
                        int64_t n, int8_t* bins, hipStream_t s) {
  if (n <= 0) return;
  if (ncols > 8) throw std::runtime_error("bin_columns: at most 8 columns");
  BinCols bc{};
  for (int c = 0; c < ncols; ++c) {
    bc.v[c] = values[c];
    bc.c[c] = cuts[c];
    bc.nc[c] = ncuts[c];
  }
  int64_t blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(bin_columns_kernel, dim3((unsigned)blocks), dim3(256), 0, s, bc, ncols, n, bins);
  ONI_HIP_CHECK(hipGetLastError());
}

}  // namespace oni
