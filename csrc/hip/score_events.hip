// Fused event scoring (reference: flow_post_lda.scala:227-248, dns_post_lda.scala:312-331;
// SURVEY.md C5c/C7c, hot op H12).
//
//   score = sum_{k<K} theta[doc][k] * phi[word][k]     (sequential, no FMA, f64)
//
// The reference evaluates this on the JVM in strict IEEE double: one rounded
// multiply and one rounded add per topic, in topic order.  __dmul_rn/__dadd_rn
// keep hipcc from contracting into FMAs so the printed scores (Java
// Double.toString) match bit for bit.  A miss (unknown doc or word) uses the
// constant default vector (flow 0.05, dns 0.1 in the reference).
// The kernel also writes key = min(src, dst) (flow) and the `key < TOL`
// predicate consumed by the compaction that follows.
#include <stdexcept>
#include <string>

#include "common.h"
#include "kernels.h"

namespace oni {

__device__ __forceinline__ double score_one(const double* __restrict__ theta, const double* __restrict__ phi,
                                            int K, double dflt, int d, int w) {
  // HIP compiles with -ffp-contract=fast; the JVM rounds the product and the sum separately.
#pragma clang fp contract(off)
  const double* tr = d >= 0 ? theta + (size_t)d * K : nullptr;
  const double* pr = w >= 0 ? phi + (size_t)w * K : nullptr;
  double s = 0.0;
  for (int k = 0; k < K; ++k) {
    const double tk = tr ? tr[k] : dflt;
    const double pk = pr ? pr[k] : dflt;
    const double prod = tk * pk;  // contract(off): rounded product, then rounded sum
    s = s + prod;
  }
  return s;
}

__global__ __launch_bounds__(256) void score_events_kernel(ScoreArgs a) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const double sa = score_one(a.theta, a.phi, a.K, a.dflt, a.doc_a[i], a.word_a[i]);
    double key = sa;
    a.score_a[i] = sa;
    if (a.doc_b) {
      const double sb = score_one(a.theta, a.phi, a.K, a.dflt, a.doc_b[i], a.word_b[i]);
      a.score_b[i] = sb;
      key = sa < sb ? sa : sb;  // breeze/scala min on two doubles
    }
    a.key[i] = key;
    a.flag[i] = key < a.tol ? 1 : 0;
  }
}

void launch_score_events(const ScoreArgs& a, hipStream_t s) {
  if (a.n <= 0) return;
  int64_t blocks = (a.n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(score_events_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a);
  ONI_HIP_CHECK(hipGetLastError());
}

}  // namespace oni
