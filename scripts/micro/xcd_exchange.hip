// Per-chunk all-gather of a split document (verdict r4, "Next round" item 1: the go / no-go probe).
//
// G workgroups (one wave each) share a document chunk; every chunk each publishes NC = KS + 1 doubles
// (K = 20: 20 topic sums + the log-sum) and reads back all G rows, summing them in member order, so
// every replica runs the same refresh.  This program times that exchange alone, R rounds back to back
// (round r publishes with tag r into parity buffer r & 1), under:
//   placement  same   = group g = blocks b = g mod 8 (one XCD under round-robin dispatch; checked
//                        with HW_REG_XCC_ID per block and reported)
//              spread = group g = blocks [g G, (g + 1) G) (dealt over the 8 XCDs)
//   granule    8      = a double as two 8-byte {u32 half, u32 tag} (the round-3 split kernel's form)
//              16     = a double as one 16-byte {lo, tag, hi, tag} (each 8-byte half self-tagged)
//   store      sc1    = write-through stores (the valid cross-XCD form)
//              plain  = default-policy stores: the line stays in the XCD's L2, which a same-XCD
//                        reader's sc1 load (L1 bypass) reads; only meaningful with placement same
//   groups     1 (alone) or 8 (every XCD running its own group: the loaded chip)
// Every value read is checked against the value its producer wrote for that round (torn or stale
// granules count as errors; a poll that exceeds the spin limit counts as a timeout and the kernel
// moves on, so no configuration can hang the GPU).
//
// Build: hipcc --offload-arch=gfx950 -O3 scripts/micro/xcd_exchange.hip -o build/xcd_exchange
// Run:   build/xcd_exchange [rounds]          (prints one line per configuration)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned u2 __attribute__((ext_vector_type(2)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));

constexpr int NC = 21;                 // exchanged columns per member (K = 20)
constexpr int MAXG = 32;               // members per group
constexpr int PER = (MAXG + 2) / 3;    // members per lane part (3 parts of 21 lanes)
constexpr long kSpin = 1L << 16;       // polls per granule set before giving up (then the block stops)

struct Args {
  unsigned* buf;          // granules: [2][8][MAXG][NC] x 16 B (either format fits)
  int G, rounds, spread, groups;
  unsigned* xcc;          // [blocks] XCC id | (HW_ID << 8)
  long long* cyc;         // [blocks] clock64 cycles of the round loop
  int* err;               // [blocks] value mismatches
  int* tmo;               // [blocks] timed-out polls
  double* out;            // [blocks] checksum (keeps the sums alive)
};

__device__ __forceinline__ double expect(int m, int c, int r) { return (double)(m * 64 + c) + 0.25 * r; }

template <int FMT, int ST, int SENT = 0>
__global__ __launch_bounds__(64) void xchg(Args a) {
  const int b = blockIdx.x, l = threadIdx.x;
  const int G = a.G;
  const int grp = a.spread ? b / G : b % 8;
  const int mem = a.spread ? b % G : b / 8;
  if (l == 0) a.xcc[b] = (__builtin_amdgcn_s_getreg((3 << 11) | 20) & 0xf) | ((unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4) << 8);
  if (grp >= a.groups) return;
  const int bytes = 2 * 8 * MAXG * NC * 16;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(a.buf, 0, bytes, 0x00020000);
  const int c = l % NC, p = l / NC;                  // lane = (column, part); lane 63 idle
  const int m0 = p * G / 3, m1 = (p + 1) * G / 3;
  constexpr int AUX = ST ? 16 : 0;
  auto slot_off = [&](int par, int m, int col) { return (((par * 8 + grp) * MAXG + m) * NC + col) * 16; };
  double chk = 0.0;
  int errc = 0, tmoc = 0;
  const long long t0 = clock64();
  for (int r = 1; r <= a.rounds; ++r) {
    const unsigned tag = (unsigned)r;
    const int par = r & 1;
    if (l < NC) {
      const unsigned long long bits = (unsigned long long)__double_as_longlong(expect(mem, l, r));
      const unsigned lo = (unsigned)bits, hi = (unsigned)(bits >> 32);
      const int o = slot_off(par, mem, l);
      if constexpr (FMT == 16) {
        const u4 v = {lo, tag, hi, tag};
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, o, 0, AUX);
      } else {
        const u2 v0 = {lo, tag}, v1 = {hi, tag};
        __builtin_amdgcn_raw_buffer_store_b64(v0, rs, o, 0, AUX);
        __builtin_amdgcn_raw_buffer_store_b64(v1, rs, o + 8, 0, AUX);
      }
    }
    double s = 0.0;
    if constexpr (SENT) {
      // sentinel poll: lane m < G polls member m's column-0 granule (one 16-B load per lane per pass);
      // the bulk sweep below then mostly finds every granule in place on its first pass
      long spins = 0;
      bool rdy = l >= G;
      while (!__all(rdy)) {
        if (!rdy) {
          const int o = slot_off(par, l, 0);
          if constexpr (FMT == 16) {
            const u4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 16);
            rdy = v.y == tag && v.w == tag;
          } else {
            const u2 v0 = __builtin_amdgcn_raw_buffer_load_b64(rs, o, 0, 16);
            rdy = v0.y == tag;
          }
        }
        asm volatile("" ::: "memory");
        if (++spins > kSpin) {
          ++tmoc;
          break;
        }
      }
    }
    if (p < 3 && tmoc == 0) {
      // every pass issues ALL of this lane's granule loads back to back (no branch between them: a load
      // inside a per-granule branch gets its own vmcnt(0) wait, i.e. one L2 round trip per granule), then
      // checks the tags; a pass with any stale granule is repeated whole
      unsigned lo[PER], hi[PER];
      long spins = 0;
      for (;;) {
        bool ok = true;
#pragma unroll
        for (int u = 0; u < PER; ++u) {
          const int m = min(m0 + u, m1 - 1 < m0 ? m0 : m1 - 1);
          const int o = slot_off(par, m, c);
          if constexpr (FMT == 16) {
            const u4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 16);
            lo[u] = v.x;
            hi[u] = v.z;
            ok &= (m0 + u >= m1) || (v.y == tag && v.w == tag);
          } else {
            const u2 v0 = __builtin_amdgcn_raw_buffer_load_b64(rs, o, 0, 16);
            const u2 v1 = __builtin_amdgcn_raw_buffer_load_b64(rs, o + 8, 0, 16);
            lo[u] = v0.x;
            hi[u] = v1.x;
            ok &= (m0 + u >= m1) || (v0.y == tag && v1.y == tag);
          }
        }
        asm volatile("" ::: "memory");
        if (ok) break;
        if (++spins > kSpin) {
          ++tmoc;
          break;
        }
      }
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        if (m0 + u < m1) {
          const double v = __longlong_as_double((long long)(((unsigned long long)hi[u] << 32) | lo[u]));
          errc += (v != expect(m0 + u, c, r)) ? 1 : 0;
          s += v;
        }
      }
    }
    // parts combined in order: every group member gets the same bits
    const double s1 = __shfl(s, min(c + NC, 63), 64), s2 = __shfl(s, min(c + 2 * NC, 63), 64);
    chk += (p == 0) ? (s + s1) + s2 : 0.0;
    // a timed-out member stops (its peers then time out too): a broken form ends in ~0.1 s, not hours
    if (__any(tmoc != 0)) break;
  }
  const long long t1 = clock64();
  for (int o = 32; o > 0; o >>= 1) {
    errc += __shfl_xor(errc, o, 64);
    tmoc += __shfl_xor(tmoc, o, 64);
  }
  if (l == 0) {
    a.cyc[b] = t1 - t0;
    a.err[b] = errc;
    a.tmo[b] = tmoc;
  }
  a.out[b * 64 + l] = chk;
}

template <int FMT, int ST, int SENT = 0>
static void run(int G, int spread, int groups, int rounds, unsigned* buf) {
  const int nb = 8 * G;
  Args a{};
  a.buf = buf;
  a.G = G;
  a.rounds = rounds;
  a.spread = spread;
  a.groups = groups;
  (void)hipMalloc(&a.xcc, nb * sizeof(unsigned));
  (void)hipMalloc(&a.cyc, nb * sizeof(long long));
  (void)hipMalloc(&a.err, nb * sizeof(int));
  (void)hipMalloc(&a.tmo, nb * sizeof(int));
  (void)hipMalloc(&a.out, nb * 64 * sizeof(double));
  (void)hipMemset(a.cyc, 0, nb * sizeof(long long));
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float ms = 0.f;
  for (int rep = 0; rep < 2; ++rep) {   // the first launch warms the code object and the buffers
    (void)hipMemset(buf, 0, 2 * 8 * MAXG * NC * 16);
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL((xchg<FMT, ST, SENT>), dim3(nb), dim3(64), 0, 0, a);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
  }
  std::vector<unsigned> x(nb);
  std::vector<long long> cy(nb);
  std::vector<int> er(nb), tm(nb);
  (void)hipMemcpy(x.data(), a.xcc, nb * sizeof(unsigned), hipMemcpyDeviceToHost);
  (void)hipMemcpy(cy.data(), a.cyc, nb * sizeof(long long), hipMemcpyDeviceToHost);
  (void)hipMemcpy(er.data(), a.err, nb * sizeof(int), hipMemcpyDeviceToHost);
  (void)hipMemcpy(tm.data(), a.tmo, nb * sizeof(int), hipMemcpyDeviceToHost);
  long long errs = 0, tmos = 0, cmax = 0;
  int mixed = 0;
  for (int g = 0; g < groups; ++g) {
    int first = -1;
    for (int m = 0; m < G; ++m) {
      const int b = spread ? g * G + m : g + 8 * m;
      errs += er[b];
      tmos += tm[b];
      cmax = cy[b] > cmax ? cy[b] : cmax;
      const int xc = (int)(x[b] & 0xf);
      if (first < 0) first = xc;
      else if (xc != first) mixed = 1;
    }
  }
  // dispatch check over the whole grid: does block b sit on the XCD of block b mod 8?
  int rr_ok = 1;
  for (int b = 8; b < nb; ++b) rr_ok &= (x[b] & 0xf) == (x[b % 8] & 0xf);
  printf("granule=%2d store=%-5s poll=%-4s G=%2d place=%-6s groups=%d  us/round=%.3f  clk/round=%.0f  "
         "one_xcd_per_group=%s rr_placement=%s errors=%lld timeouts=%lld  xcc(b0..7)=",
         FMT, ST ? "sc1" : "plain", SENT ? "sent" : "all", G, spread ? "spread" : "same", groups, 1000.0 * ms / rounds,
         (double)cmax / rounds, mixed ? "no" : "yes", rr_ok ? "yes" : "no", errs, tmos);
  for (int b = 0; b < 8 && b < nb; ++b) printf("%u", x[b] & 0xf);
  printf("\n");
  fflush(stdout);
  (void)hipFree(a.xcc);
  (void)hipFree(a.cyc);
  (void)hipFree(a.err);
  (void)hipFree(a.tmo);
  (void)hipFree(a.out);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 2000;
  unsigned* buf;
  (void)hipMalloc(&buf, 2 * 8 * MAXG * NC * 16);
  // v3: r5a / r5b issued each granule load inside a per-granule branch, so the compiler waited for every
  // load before the next (one L2 round trip per granule); every pass now issues all loads back to back
  const int Gs[] = {2, 8, 16, 24, 32};
  for (int groups : {1, 8}) {
    for (int G : Gs) {
      run<16, 0, 0>(G, 0, groups, rounds, buf);
      run<16, 0, 1>(G, 0, groups, rounds, buf);
      run<16, 1, 1>(G, 0, groups, rounds, buf);
      if (groups == 1) run<16, 1, 1>(G, 1, groups, rounds, buf);
    }
  }
  (void)hipFree(buf);
  return 0;
}
