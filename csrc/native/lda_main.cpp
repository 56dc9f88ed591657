// `lda` executable with oni-lda-c's command line (reference call site
// /root/reference/ml_ops.sh:80):
//
//   lda est <alpha> <k> <settings> <nproc> <corpus> <random|seeded|model-prefix> <dir> [--gs-updates U]
//   lda inf <settings> <model-prefix> <corpus> <save-prefix> [--gs-updates U]
//
// --gs-updates U (an addition; default 0 = lda-c's literal per-word schedule): gamma / digamma refreshed
// after every chunk of ceil(n / U) words -- the block Gauss-Seidel schedule of the MI355X engine
// (csrc/hip/lda_gs64.hip), so a CPU baseline can be measured on the GPU's own schedule.
//
// <nproc> is the number of document shards (oni-lda-c's MPI ranks); shards run
// on threads of this process (ONI_THREADS, default: hardware threads) instead
// of MPI processes.  This is the CPU reference / baseline engine; the MI355X
// engine is `python -m oni_ml_amd.lda` with the same arguments.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>

#include "lda_ref.h"

static void usage() {
  std::fprintf(stderr,
               "usage: lda est [initial alpha] [k] [settings] [nproc] [data] [random/seeded/*] [directory]"
               " [--gs-updates U]\n"
               "       lda inf [settings] [model] [data] [name] [--gs-updates U]\n");
}

// trailing "--gs-updates U" after the positional arguments; -1: malformed
static int gs_updates_flag(int argc, char** argv, int first) {
  int u = 0;
  for (int i = first; i < argc; ++i) {
    if (std::strcmp(argv[i], "--gs-updates") == 0 && i + 1 < argc) {
      char* end = nullptr;
      const long v = std::strtol(argv[++i], &end, 10);
      if (!end || *end || v < 0 || v > (1 << 20)) return -1;
      u = (int)v;
    } else {
      return -1;
    }
  }
  return u;
}

int main(int argc, char** argv) {
  try {
    int threads = (int)std::thread::hardware_concurrency();
    if (const char* t = std::getenv("ONI_THREADS")) threads = std::atoi(t);
    uint64_t seed = 4357;
    if (const char* s = std::getenv("ONI_SEED")) seed = std::strtoull(s, nullptr, 10);
    if (argc >= 9 && std::strcmp(argv[1], "est") == 0) {
      double alpha = std::atof(argv[2]);
      int K = std::atoi(argv[3]);
      onin::LdacSettings st = onin::read_ldac_settings(argv[4]);
      st.gs_updates = gs_updates_flag(argc, argv, 9);
      if (st.gs_updates < 0) {
        usage();
        return 1;
      }
      int nproc = std::atoi(argv[5]);
      onin::LdacCorpus c = onin::read_ldac_corpus(argv[6]);
      std::printf("number of docs    : %d\nnumber of terms   : %d\n", c.num_docs(), c.num_terms);
      if (st.gs_updates > 0) std::printf("schedule          : block Gauss-Seidel, %d refreshes per sweep\n", st.gs_updates);
      int it = onin::ldac_estimate(c, K, alpha, st, argv[7], argv[8], nproc, threads, seed, true);
      std::printf("em iterations: %d\n", it);
      return 0;
    }
    if (argc >= 6 && std::strcmp(argv[1], "inf") == 0) {
      onin::LdacSettings st = onin::read_ldac_settings(argv[2]);
      st.gs_updates = gs_updates_flag(argc, argv, 6);
      if (st.gs_updates < 0) {
        usage();
        return 1;
      }
      onin::LdacCorpus c = onin::read_ldac_corpus(argv[4]);
      onin::ldac_infer(c, argv[3], st, argv[5], 1, threads);
      return 0;
    }
    usage();
    return 1;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "lda: %s\n", e.what());
    return 2;
  }
}
