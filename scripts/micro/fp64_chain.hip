// Dependent-latency probe (gfx950): 16 dependent ops per loop trip, one wave per SIMD, cycles from
// s_memtime; fp64 FMA, fp32 FMA, fp64 add after a DPP move, permlane32 swap, LDS round trip.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ void chain(double* out, long long* cyc, int iters) {
  __shared__ double lds[64];
  double v = 1.0 + threadIdx.x * 1e-9;
  float f = 1.0f + threadIdx.x * 1e-6f;
  lds[threadIdx.x] = v;
  __syncthreads();
  long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if constexpr (MODE == 0) v = fma(v, 0.999999, 1e-7);
      if constexpr (MODE == 1) f = fmaf(f, 0.999999f, 1e-7f);
      if constexpr (MODE == 2) {
        const long long b = __double_as_longlong(v);
        const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0xB1, 0xF, 0xF, true);
        const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0xB1, 0xF, 0xF, true);
        v = 0.5 * (v + __longlong_as_double(((long long)hi << 32) | (unsigned)lo));
      }
      if constexpr (MODE == 3) {
        const auto r = __builtin_amdgcn_permlane32_swap((unsigned)__double_as_longlong(v), (unsigned)__double_as_longlong(v), false, false);
        v = v + (double)r[0] * 1e-30;
      }
      if constexpr (MODE == 4) {
        lds[threadIdx.x] = v;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        v = lds[(threadIdx.x + 1) & 63] * 0.999999;
      }
      if constexpr (MODE == 5) v = __builtin_amdgcn_rcp(v) + 0.5;
    }
  }
  long long t1 = clock64();
  out[blockIdx.x * 64 + threadIdx.x] = v + f;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE>
void run(const char* name) {
  double* out; long long* cyc;
  (void)hipMalloc(&out, sizeof(double) * 1024 * 64);
  (void)hipMalloc(&cyc, sizeof(long long) * 1024);
  const int iters = 4000;
  hipLaunchKernelGGL((chain<MODE>), dim3(1024), dim3(64), 0, 0, out, cyc, iters);
  (void)hipDeviceSynchronize();
  hipLaunchKernelGGL((chain<MODE>), dim3(1024), dim3(64), 0, 0, out, cyc, iters);
  (void)hipDeviceSynchronize();
  long long c[1024];
  (void)hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < 1024; ++i) avg += c[i];
  avg /= 1024;
  printf("%-22s %.2f clk per dependent step\n", name, avg / (iters * 16.0));
  (void)hipFree(out); (void)hipFree(cyc);
}

int main() {
  run<0>("fma_f64");
  run<1>("fma_f32");
  run<2>("dpp(2x32)+add+mul f64");
  run<3>("permlane32_swap+fma");
  run<4>("lds write+read (wave)");
  run<5>("rcp_f64+add");
  return 0;
}
