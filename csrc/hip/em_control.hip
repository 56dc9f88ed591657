// Device-side EM driver step: the convergence test of lda-c's run_em loop
// (lda-estimate.c structure, call site ml_ops.sh:80)
//
//   converged = (likelihood_old - likelihood) / likelihood_old;
//   if (converged < 0) VAR_MAX_ITER = VAR_MAX_ITER * 2;
//   likelihood_old = likelihood;
//   while (((converged < 0) || (converged > EM_CONVERGED) || (i <= 2)) && (i <= EM_MAX_ITER))
//
// evaluated on the GPU after every EM iteration.  The host enqueues a batch of
// iterations (hipGraph replays) without waiting; once this kernel sets
// params[kParamDone], every kernel of the iterations still queued returns at
// once, so the device state is exactly that of the iteration that converged.
// The host reads the per-iteration history {likelihood, conv, alpha,
// VAR_MAX_ITER} once per batch instead of one blocking read-back per iteration.
#include "common.h"
#include "kernels.h"
#include "em_control.h"
#include "alpha_newton.h"

namespace oni {

__global__ void em_control_kernel(const double* __restrict__ scalars, double* __restrict__ params,
                                  double* __restrict__ ctl, double* __restrict__ hist, int hist_slots) {
  if (threadIdx.x != 0 || blockIdx.x != 0 || params[kParamDone] != 0.0) return;
  em_control_step(scalars, params, ctl, hist, hist_slots, params[0]);
}

void launch_em_control(const double* scalars, double* params, double* ctl, double* hist, int hist_slots,
                       hipStream_t s) {
  hipLaunchKernelGGL(em_control_kernel, dim3(1), dim3(64), 0, s, scalars, params, ctl, hist, hist_slots);
  ONI_HIP_CHECK(hipGetLastError());
}

__global__ void alpha_newton_kernel(const double* __restrict__ scalars, double num_docs, int K, int estimate,
                                    double* __restrict__ params, double* __restrict__ alpha_out) {
  const int lane = threadIdx.x;
  if (blockIdx.x != 0 || lane >= 2 || params[kParamDone] != 0.0) return;
  alpha_newton_lanes(scalars, num_docs, K, estimate, params, alpha_out, lane);
}

void launch_alpha_newton(const double* scalars, double num_docs, int K, bool estimate, double* params,
                         double* alpha_out, hipStream_t s) {
  hipLaunchKernelGGL(alpha_newton_kernel, dim3(1), dim3(64), 0, s, scalars, num_docs, K, estimate ? 1 : 0, params,
                     alpha_out);
  ONI_HIP_CHECK(hipGetLastError());
}

}  // namespace oni
