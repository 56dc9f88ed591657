// lda-c opt_alpha on the device, shared by the fused M-step launch
// (lda_gs64.hip) and the stand-alone kernel (em_control.hip).
#pragma once
#include "common.h"
#include "kernels.h"

namespace oni {

// ------------------------------------------------------- alpha on device ---
// lda-c opt_alpha (lda-alpha.c): Newton on log(alpha) for
//   alhood(a) = D (lnG(K a) - K lnG(a)) + (a - 1) ss
// started at 100, x10 restart on NaN, |df| <= 1e-5 or 1000 iterations, in
// double exactly as the host version (models/lda/special.py).  Two lanes;
// it reads alpha_ss from the E-step's reduction output and writes the next
// E-step's {alpha, lgamma(K a) - K lgamma(a)} into the device parameter block,
// so an EM iteration needs no host round trip besides the likelihood read-back.
__device__ inline double trigamma_ldac(double x) {
  x = x + 6.0;
  double p = 1.0 / (x * x);
  p = (((((0.075757575757576 * p - 0.033333333333333) * p + 0.0238095238095238) * p - 0.033333333333333) * p +
        0.166666666666667) * p + 1) / x + 0.5 * p;
  for (int i = 0; i < 6; ++i) {
    x = x - 1.0;
    p = 1.0 / (x * x) + p;
  }
  return p;
}

// Lanes 0 and 1 of the calling wave (both must call it): they evaluate each step's
// special functions at K a and a side by side (one digamma + one trigamma latency per
// Newton step instead of two of each) and carry the same scalar state.  Lane 0 writes
// params[0..1] and alpha_out with agent-scope (write-through) stores, so a workgroup of
// the same launch can read them after its own agent-scope loads (fused M-step).
__device__ __forceinline__ void alpha_newton_lanes(const double* __restrict__ scalars, double num_docs, int K,
                                                   int estimate, double* __restrict__ params,
                                                   double* __restrict__ alpha_out, int lane) {
  double a = params[0];
  if (estimate) {
    const double ss = scalars[1];
    const double D = num_docs;
    double init_a = 100.0, log_a = log(init_a), df;
    int iter = 0;
    do {
      ++iter;
      a = exp(log_a);
      if (isnan(a)) {
        init_a = init_a * 10.0;
        a = init_a;
        log_a = log(a);
      }
      const double x = lane == 0 ? K * a : a;
      const double dg = digamma_ldac(x), tg = trigamma_ldac(x);
      const double dg_ka = __shfl(dg, 0, 2), dg_a = __shfl(dg, 1, 2);
      const double tg_ka = __shfl(tg, 0, 2), tg_a = __shfl(tg, 1, 2);
      df = D * (K * dg_ka - K * dg_a) + ss;
      const double d2f = D * (K * K * tg_ka - K * tg_a);
      log_a = log_a - df / (d2f * a + df);
    } while (fabs(df) > 1e-5 && iter < 1000);
    a = exp(log_a);
  }
  const double lg = lgamma(lane == 0 ? a * K : a);
  const double lg_ka = __shfl(lg, 0, 2), lg_a = __shfl(lg, 1, 2);
  if (lane == 0) {
    __hip_atomic_store(params, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(params + 1, lg_ka - K * lg_a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(alpha_out, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace oni
