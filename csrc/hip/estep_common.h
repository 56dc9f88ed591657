// Device helpers of the split-document E-step kernels (lda_gs64.hip gs_splitw).
#pragma once
#include "common.h"
#include "kernels.h"

namespace oni {

// ---------------------------------------------------------------------------
// Split-document hand-off: tagged 8-byte granules {uint32 half of a double, uint32 tag}.
// A 64-bit aligned relaxed atomic store / load is single-copy atomic, so a reader
// that sees the tag sees the value; agent scope makes the accesses coherent
// across XCDs (sc1, no stale L2 / L1 lines).  Tag = (launch epoch << 12) |
// (iteration & 0xfff): iteration bits separate it from it - 2 (the previous use
// of the parity buffer), the epoch separates launches.
// ---------------------------------------------------------------------------
constexpr long kSplitSpinLimit = 1L << 24;   // ~seconds of polling, then give up (error flag)

__device__ __forceinline__ unsigned split_tag(int epoch, int it) {
  return ((unsigned)(epoch & 0xfffff) << 12) | (unsigned)(it & 0xfff);
}

// End of a split launch: the last segment of the document to get here bumps the
// document's epoch and resets the exit count (graph replays need no memset).
__device__ __forceinline__ void split_exit(int* counter, int n_docs, int nseg) {
  if (threadIdx.x == 0) {
    int* exits = counter + n_docs;
    if (__hip_atomic_fetch_add(exits, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nseg - 1) {
      __hip_atomic_store(exits, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace oni
