// fp64 VALU latency / throughput probe on gfx950: cycles per dependent op (one chain) and per
// independent op (8 chains), for v_fma_f64, v_rcp_f64 and the engine's flog / fexp helpers.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ __forceinline__ double drcp(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = fma(-x, r, 1.0); r = fma(r, e, r); e = fma(-x, r, 1.0); return fma(r, e, r);
}

template <int MODE, int CH>
__global__ void probe(double* out, long long* cyc, int iters, double seed) {
  double v[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) v[c] = seed + threadIdx.x * 1e-3 + c;
  long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      if constexpr (MODE == 0) v[c] = fma(v[c], 0.999999, 1e-7);
      else if constexpr (MODE == 1) v[c] = __builtin_amdgcn_rcp(v[c]) + 1.0;
      else if constexpr (MODE == 2) v[c] = drcp(v[c]) + 1.0;
      else if constexpr (MODE == 3) v[c] = log(v[c]) + 3.0;
      else if constexpr (MODE == 4) v[c] = exp(v[c] * 0.01) + 0.5;
      else if constexpr (MODE == 5) v[c] = fmaf((float)v[c], 0.999999f, 1e-7f);
    }
  }
  long long t1 = clock64();
  double s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += v[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE, int CH>
void run(const char* name, int waves_per_simd) {
  double* out; long long* cyc;
  const int blocks = 256 * 4 * waves_per_simd;   // waves of 64 threads
  hipMalloc(&out, sizeof(double) * blocks * 64);
  hipMalloc(&cyc, sizeof(long long) * blocks);
  const int iters = 2000;
  hipLaunchKernelGGL((probe<MODE, CH>), dim3(blocks), dim3(64), 0, 0, out, cyc, iters, 1.5);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a);
  hipLaunchKernelGGL((probe<MODE, CH>), dim3(blocks), dim3(64), 0, 0, out, cyc, iters, 1.5);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  std::vector<long long> c(blocks);
  hipMemcpy(c.data(), cyc, sizeof(long long) * blocks, hipMemcpyDeviceToHost);
  double avg = 0; for (auto x : c) avg += x; avg /= blocks;
  // clock64 = s_memtime (100 MHz? no: shader clock) -> report per op in clock64 units and ns from events
  const double ops = (double)iters * CH;
  printf("%-10s chains=%d waves/SIMD=%d : %.2f clk64/op per wave, wall %.3f ms, %.3f ns/op/wave-chain-step\n", name, CH,
         waves_per_simd, avg / ops, ms, ms * 1e6 / (iters * (double)CH));
  hipFree(out); hipFree(cyc);
}

int main() {
  for (int w : {1, 4}) {
    run<0, 1>("fma64", w); run<0, 8>("fma64", w);
    run<5, 1>("fma32", w); run<5, 8>("fma32", w);
    run<1, 1>("rcp64", w); run<1, 8>("rcp64", w);
    run<2, 1>("drcp", w); run<2, 8>("drcp", w);
    run<3, 1>("log64", w); run<3, 8>("log64", w);
    run<4, 1>("exp64", w); run<4, 8>("exp64", w);
  }
  return 0;
}
