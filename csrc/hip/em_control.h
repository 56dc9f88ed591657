// lda-c EM loop step evaluated on the device (see em_control.hip); shared by the
// stand-alone control kernel and the fused M-step + control kernel.
#pragma once
#include "common.h"
#include "kernels.h"

namespace oni {

__device__ inline void em_control_step(const double* __restrict__ scalars, double* __restrict__ params,
                                double* __restrict__ ctl, double* __restrict__ hist, int hist_slots,
                                double alpha_now) {
  const double lik = scalars[0];
  const double L_old = ctl[0];
  // IEEE division reproduces the host's L_old == 0 conventions (+-inf / nan)
  const double conv = (L_old - lik) / L_old;
  if (conv < 0.0) params[2] = params[2] * 2.0;
  const double i = ctl[3] + 1.0;
  ctl[3] = i;
  ctl[0] = lik;
  const int slot = (int)ctl[2];
  if (slot < hist_slots) {
    double* h = hist + (size_t)kHistCols * slot;
    h[0] = lik;
    h[1] = conv;
    h[2] = alpha_now;   // alpha after this iteration's Newton
    h[3] = params[2];
    h[4] = scalars[1];
  }
  ctl[2] = (double)(slot + 1);
  const double em_conv = ctl[1], em_max = ctl[4];
  const bool cont = (conv < 0.0 || conv > em_conv || i <= 2.0) && i <= em_max;
  if (!cont && ctl[5] != 0.0) params[kParamDone] = 1.0;
}

}  // namespace oni
