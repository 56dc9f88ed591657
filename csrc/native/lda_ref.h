// CPU reference of oni-lda-c (upstream lda-c variational EM with document
// sharding), used as (a) the exact-semantics oracle for the HIP engine and (b)
// the measured CPU baseline.  Float64 throughout, Gauss-Seidel
// per-word gamma updates exactly as lda-c's lda_inference.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace onin {

struct LdacCorpus {
  std::vector<int64_t> doc_ptr;   // [D+1]
  std::vector<int32_t> words;     // [nnz]
  std::vector<int32_t> counts;    // [nnz]
  int num_terms = 0;
  int max_length = 0;
  int num_docs() const { return (int)doc_ptr.size() - 1; }
};

struct LdacSettings {
  int var_max_iter = 20;
  float var_converged = 1e-6f;
  int em_max_iter = 100;
  float em_converged = 1e-4f;
  bool estimate_alpha = true;
  int gs_updates = 0;   // 0: lda-c's per-word schedule; U > 0: block Gauss-Seidel (lda_ref.cpp)
};

// Result of one E-step over a document range.
struct EStepOut {
  double likelihood = 0.0;
  double alpha_ss = 0.0;
  std::vector<double> class_word;   // [K][V]
  std::vector<double> class_total;  // [K]
  std::vector<double> gamma;        // [D][K]
  std::vector<int32_t> iters;       // [D]
  std::vector<double> doc_lik;      // [D]
};

double ldac_digamma(double x);
double ldac_trigamma(double x);
double ldac_log_sum(double a, double b);
double ldac_opt_alpha(double ss, int D, int K);

// E-step over all docs of the corpus with `log_beta` [K][V].  Work is split into
// `nshards` contiguous nnz-balanced document shards (the MPI ranks of
// oni-lda-c) run on `threads` threads; shard statistics are reduced in shard
// order, so the result depends on nshards but never on threads.
EStepOut ldac_estep(const int64_t* doc_ptr, const int32_t* words, const double* counts, int D, int V, int K,
                    const double* log_beta, double alpha, int var_max_iter, float var_converged, int nshards,
                    int threads, int gs_updates = 0);

// run_em's final pass: a fresh lda_inference of every document under the final model, and for every
// corpus entry the topic of its largest phi (the first maximum; write_word_assignment).
std::vector<int32_t> ldac_word_assignments(const int64_t* doc_ptr, const int32_t* words, const double* counts, int D,
                                           int V, int K, const double* log_beta, double alpha, int var_max_iter,
                                           float var_converged, int gs_updates, int threads);

LdacCorpus read_ldac_corpus(const std::string& path);
LdacSettings read_ldac_settings(const std::string& path);

// Full `lda est` (random | seeded | <model prefix>) with lda-c outputs in dir.
int ldac_estimate(const LdacCorpus& c, int K, double alpha_init, const LdacSettings& st, const std::string& start,
                  const std::string& dir, int nshards, int threads, uint64_t seed, bool verbose);
// `lda inf`: gamma + likelihoods for a corpus under a saved model.
int ldac_infer(const LdacCorpus& c, const std::string& model_prefix, const LdacSettings& st,
               const std::string& save_prefix, int nshards, int threads);

}  // namespace onin
