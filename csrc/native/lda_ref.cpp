// oni-lda-c semantics on the CPU (see lda_ref.h).  The algorithm is upstream
// lda-c's variational EM (Blei): per-document coordinate ascent with the
// gamma vector updated after every word, lda-c's series digamma/trigamma,
// the -100 log-probability floor, Newton on log(alpha), EM loop with
// VAR_MAX_ITER doubling, LAG=5 snapshots and lda-c's text formats.
// Document sharding follows oni-lda-c's MPI layout (call site
// /root/reference/ml_ops.sh:80; outputs README.md:116-121).
#include "lda_ref.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <random>
#include <sstream>
#include <stdexcept>
#include <sys/stat.h>
#include <atomic>
#include <thread>

namespace onin {

static constexpr int kLag = 5;
static constexpr double kNewtonThresh = 1e-5;
static constexpr int kMaxAlphaIter = 1000;
static constexpr int kNumInit = 1;

double ldac_digamma(double x) {
  x = x + 6;
  double p = 1 / (x * x);
  p = (((0.004166666666667 * p - 0.003968253986254) * p + 0.008333333333333) * p - 0.083333333333333) * p;
  p = p + std::log(x) - 0.5 / x - 1 / (x - 1) - 1 / (x - 2) - 1 / (x - 3) - 1 / (x - 4) - 1 / (x - 5) -
      1 / (x - 6);
  return p;
}

double ldac_trigamma(double x) {
  x = x + 6;
  double p = 1 / (x * x);
  p = (((((0.075757575757576 * p - 0.033333333333333) * p + 0.0238095238095238) * p - 0.033333333333333) * p +
        0.166666666666667) * p + 1) / x + 0.5 * p;
  for (int i = 0; i < 6; i++) {
    x = x - 1;
    p = 1 / (x * x) + p;
  }
  return p;
}

double ldac_log_sum(double a, double b) {
  if (a < b) return b + std::log(1 + std::exp(a - b));
  return a + std::log(1 + std::exp(b - a));
}

static double d_alhood(double a, double ss, int D, int K) {
  return D * (K * ldac_digamma(K * a) - K * ldac_digamma(a)) + ss;
}
static double d2_alhood(double a, int D, int K) {
  return D * (K * K * ldac_trigamma(K * a) - K * ldac_trigamma(a));
}

double ldac_opt_alpha(double ss, int D, int K) {
  double init_a = 100;
  double log_a = std::log(init_a);
  int iter = 0;
  double df;
  do {
    iter++;
    double a = std::exp(log_a);
    if (std::isnan(a)) {
      init_a = init_a * 10;
      a = init_a;
      log_a = std::log(a);
    }
    df = d_alhood(a, ss, D, K);
    double d2f = d2_alhood(a, D, K);
    log_a = log_a - df / (d2f * a + df);
  } while ((std::fabs(df) > kNewtonThresh) && (iter < kMaxAlphaIter));
  return std::exp(log_a);
}

namespace {

struct DocView {
  const int32_t* w;
  const double* c;
  int n;
  double total;
};

struct Workspace {
  std::vector<double> phi, oldphi, dig;
  void ensure(int n, int K) {
    if ((int)phi.size() < n * K) phi.resize((size_t)n * K);
    if ((int)oldphi.size() < K) oldphi.resize(K);
    dig.resize(K);
  }
};

// lgamma without the global `signgam` write of std::lgamma (a data race between
// inference threads, found by the ThreadSanitizer self-test).
inline double lgam(double x) {
  int sign;
  return lgamma_r(x, &sign);
}

double compute_likelihood(const DocView& d, const double* lb, int V, int K, double alpha, const double* phi,
                          const double* gam, double* dig) {
  double gsum = 0;
  for (int k = 0; k < K; k++) {
    dig[k] = ldac_digamma(gam[k]);
    gsum += gam[k];
  }
  const double digsum = ldac_digamma(gsum);
  double L = lgam(alpha * K) - K * lgam(alpha) - lgam(gsum);
  for (int k = 0; k < K; k++) {
    L += (alpha - 1) * (dig[k] - digsum) + lgam(gam[k]) - (gam[k] - 1) * (dig[k] - digsum);
    for (int n = 0; n < d.n; n++) {
      const double p = phi[(size_t)n * K + k];
      if (p > 0) L += d.c[n] * (p * ((dig[k] - digsum) - std::log(p) + lb[(size_t)k * V + d.w[n]]));
    }
  }
  return L;
}

// lda_inference: returns the document likelihood; gam/phi hold the final state.
// gs_updates = 0: lda-c's literal schedule (gamma and digamma refreshed after every
// word).  gs_updates = U > 0: block Gauss-Seidel, the schedule of the fp64 HIP
// engine -- a document of n words is walked in chunks of W = ceil(n / U) words;
// the words of a chunk take their phi from the same digamma vector, then gamma and
// digamma are refreshed (at most U refreshes per sweep; n <= U is the literal
// schedule).  Everything else (init, likelihood, convergence test) is lda-c's.
double lda_inference(const DocView& d, const double* lb, int V, int K, double alpha, int var_max_iter,
                     float var_converged, double* gam, Workspace& ws, int* iters, int gs_updates) {
  ws.ensure(d.n, K);
  const int W = gs_updates > 0 ? std::max(1, (d.n + gs_updates - 1) / gs_updates) : 1;
  if ((int)ws.oldphi.size() < W * K) ws.oldphi.resize((size_t)W * K);
  double* phi = ws.phi.data();
  double* dig = ws.dig.data();
  double* old = ws.oldphi.data();
  for (int k = 0; k < K; k++) {
    gam[k] = alpha + d.total / K;
    dig[k] = ldac_digamma(gam[k]);
    for (int n = 0; n < d.n; n++) phi[(size_t)n * K + k] = 1.0 / K;
  }
  double converged = 1, L = 0, L_old = 0;
  int it = 0;
  while (converged > var_converged && (it < var_max_iter || var_max_iter == -1)) {
    it++;
    for (int n0 = 0; n0 < d.n; n0 += W) {
      const int n1 = std::min(d.n, n0 + W);
      for (int n = n0; n < n1; n++) {
        double* ph = phi + (size_t)n * K;
        double* o = old + (size_t)(n - n0) * K;
        double phisum = 0;
        for (int k = 0; k < K; k++) {
          o[k] = ph[k];
          ph[k] = dig[k] + lb[(size_t)k * V + d.w[n]];
          phisum = k > 0 ? ldac_log_sum(phisum, ph[k]) : ph[k];
        }
        for (int k = 0; k < K; k++) ph[k] = std::exp(ph[k] - phisum);
      }
      for (int n = n0; n < n1; n++) {
        const double* ph = phi + (size_t)n * K;
        const double* o = old + (size_t)(n - n0) * K;
        for (int k = 0; k < K; k++) gam[k] = gam[k] + d.c[n] * (ph[k] - o[k]);
      }
      for (int k = 0; k < K; k++) dig[k] = ldac_digamma(gam[k]);
    }
    L = compute_likelihood(d, lb, V, K, alpha, phi, gam, dig);
    converged = (L_old - L) / L_old;
    L_old = L;
  }
  if (iters) *iters = it;
  return L;
}

std::vector<std::pair<int, int>> shard_ranges(const int64_t* doc_ptr, int D, int nshards) {
  std::vector<std::pair<int, int>> r;
  if (nshards < 1) nshards = 1;
  const double nnz = (double)doc_ptr[D];
  int prev = 0;
  for (int s = 1; s <= nshards; ++s) {
    int b = D;
    if (s < nshards) {
      const double target = nnz * s / nshards;
      b = (int)(std::lower_bound(doc_ptr, doc_ptr + D + 1, (int64_t)std::ceil(target)) - doc_ptr);
      b = std::max(prev, std::min(b, D));
    }
    r.emplace_back(prev, b);
    prev = b;
  }
  return r;
}

}  // namespace

EStepOut ldac_estep(const int64_t* doc_ptr, const int32_t* words, const double* counts, int D, int V, int K,
                    const double* log_beta, double alpha, int var_max_iter, float var_converged, int nshards,
                    int threads, int gs_updates) {
  // Shards (emulated MPI ranks) are processed one after another; inside a shard
  // documents are inferred in parallel chunks that keep their final phi, and
  // the statistics are then accumulated in document order (words partitioned
  // over threads), so every sum runs in lda-c's sequential order and the
  // result is independent of `threads`.
  auto shards = shard_ranges(doc_ptr, D, nshards);
  if (threads < 1) threads = 1;
  EStepOut out;
  out.gamma.assign((size_t)D * K, 0.0);
  out.iters.assign(D, 0);
  out.class_word.assign((size_t)K * V, 0.0);
  out.class_total.assign(K, 0.0);
  std::vector<double> cw((size_t)K * V), ct(K), ass(D);
  out.doc_lik.assign(D, 0.0);
  std::vector<double>& lik = out.doc_lik;
  const int64_t kChunkNnz = 1 << 22;
  std::vector<double> phi;
  std::vector<Workspace> ws(threads);
  for (auto [s0, s1] : shards) {
    std::fill(cw.begin(), cw.end(), 0.0);
    std::fill(ct.begin(), ct.end(), 0.0);
    double sl = 0.0, sa = 0.0;
    int d0 = s0;
    while (d0 < s1) {
      int d1 = d0 + 1;
      while (d1 < s1 && doc_ptr[d1 + 1] - doc_ptr[d0] <= kChunkNnz) ++d1;
      const int64_t e0 = doc_ptr[d0], e1 = doc_ptr[d1];
      phi.resize((size_t)(e1 - e0) * K);
      std::atomic<int> next{d0};
      auto infer = [&](int t) {
        for (int di = next.fetch_add(1); di < d1; di = next.fetch_add(1)) {
          DocView d{words + doc_ptr[di], counts + doc_ptr[di], (int)(doc_ptr[di + 1] - doc_ptr[di]), 0.0};
          for (int n = 0; n < d.n; n++) d.total += d.c[n];
          double* gam = out.gamma.data() + (size_t)di * K;
          lik[di] = lda_inference(d, log_beta, V, K, alpha, var_max_iter, var_converged, gam, ws[t], &out.iters[di],
                                  gs_updates);
          std::memcpy(phi.data() + (size_t)(doc_ptr[di] - e0) * K, ws[t].phi.data(), sizeof(double) * d.n * K);
          double gsum = 0, dsum = 0;
          for (int k = 0; k < K; k++) {
            gsum += gam[k];
            dsum += ldac_digamma(gam[k]);
          }
          ass[di] = dsum - K * ldac_digamma(gsum);
        }
      };
      auto accumulate = [&](int t) {
        const int w0 = (int)((int64_t)V * t / threads), w1 = (int)((int64_t)V * (t + 1) / threads);
        for (int64_t j = e0; j < e1; ++j) {
          const int w = words[j];
          if (w < w0 || w >= w1) continue;
          const double c = counts[j];
          const double* ph = phi.data() + (size_t)(j - e0) * K;
          for (int k = 0; k < K; k++) cw[(size_t)k * V + w] += c * ph[k];
        }
      };
      std::vector<std::thread> th;
      for (int t = 1; t < threads; ++t) th.emplace_back(infer, t);
      infer(0);
      for (auto& x : th) x.join();
      th.clear();
      for (int t = 1; t < threads; ++t) th.emplace_back(accumulate, t);
      accumulate(0);
      for (int64_t j = e0; j < e1; ++j) {
        const double c = counts[j];
        const double* ph = phi.data() + (size_t)(j - e0) * K;
        for (int k = 0; k < K; k++) ct[k] += c * ph[k];
      }
      for (int di = d0; di < d1; ++di) {
        sl += lik[di];
        // lda-c accumulates alpha_ss term by term: += psi(g_k) ... -= K psi(sum)
        sa += ass[di];
      }
      for (auto& x : th) x.join();
      d0 = d1;
    }
    // rank-ordered reduction (MPI_Reduce equivalent, deterministic)
    out.likelihood += sl;
    out.alpha_ss += sa;
    for (size_t i = 0; i < cw.size(); ++i) out.class_word[i] += cw[i];
    for (int k = 0; k < K; ++k) out.class_total[k] += ct[k];
  }
  return out;
}

// ------------------------------------------------------------------ I/O ----

LdacCorpus read_ldac_corpus(const std::string& path) {
  std::ifstream f(path);
  if (!f) throw std::runtime_error("cannot open corpus " + path);
  LdacCorpus c;
  c.doc_ptr.push_back(0);
  std::string line;
  int maxw = -1;
  while (std::getline(f, line)) {
    if (line.empty() || line == "\r") continue;
    const char* p = line.c_str();
    char* e;
    long n = std::strtol(p, &e, 10);
    if (e == p) throw std::runtime_error("bad corpus line: " + line);
    p = e;
    for (long i = 0; i < n; ++i) {
      long w = std::strtol(p, &e, 10);
      if (e == p || *e != ':') throw std::runtime_error("bad corpus entry in line: " + line);
      p = e + 1;
      long cnt = std::strtol(p, &e, 10);
      if (e == p) throw std::runtime_error("bad corpus count in line: " + line);
      p = e;
      c.words.push_back((int32_t)w);
      c.counts.push_back((int32_t)cnt);
      maxw = std::max(maxw, (int)w);
    }
    c.max_length = std::max(c.max_length, (int)n);
    c.doc_ptr.push_back((int64_t)c.words.size());
  }
  c.num_terms = maxw + 1;
  return c;
}

LdacSettings read_ldac_settings(const std::string& path) {
  std::ifstream f(path);
  if (!f) throw std::runtime_error("cannot open settings " + path);
  LdacSettings s;
  std::string all((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  char alpha_action[100] = {0};
  if (std::sscanf(all.c_str(), "var max iter %d\nvar convergence %f\nem max iter %d\nem convergence %f\nalpha %99s",
                  &s.var_max_iter, &s.var_converged, &s.em_max_iter, &s.em_converged, alpha_action) != 5)
    throw std::runtime_error("malformed settings file " + path);
  s.estimate_alpha = std::strcmp(alpha_action, "fixed") != 0;
  return s;
}

namespace {

void save_model(const std::string& prefix, const std::vector<double>& lb, int K, int V, double alpha) {
  std::string s;
  s.reserve((size_t)K * V * 15);
  char buf[64];
  for (int k = 0; k < K; k++) {
    for (int w = 0; w < V; w++) {
      int n = std::snprintf(buf, sizeof(buf), " %5.10f", lb[(size_t)k * V + w]);
      s.append(buf, n);
    }
    s += '\n';
  }
  FILE* f = std::fopen((prefix + ".beta").c_str(), "w");
  if (!f) throw std::runtime_error("cannot write " + prefix + ".beta");
  std::fwrite(s.data(), 1, s.size(), f);
  std::fclose(f);
  f = std::fopen((prefix + ".other").c_str(), "w");
  if (!f) throw std::runtime_error("cannot write " + prefix + ".other");
  std::fprintf(f, "num_topics %d \n", K);
  std::fprintf(f, "num_terms %d \n", V);
  std::fprintf(f, "alpha %5.10f \n", alpha);
  std::fclose(f);
}

void save_gamma(const std::string& path, const std::vector<double>& g, int D, int K) {
  std::string s;
  char buf[64];
  for (int d = 0; d < D; d++) {
    for (int k = 0; k < K; k++) {
      int n = std::snprintf(buf, sizeof(buf), k ? " %5.10f" : "%5.10f", g[(size_t)d * K + k]);
      s.append(buf, n);
    }
    s += '\n';
  }
  FILE* f = std::fopen(path.c_str(), "w");
  if (!f) throw std::runtime_error("cannot write " + path);
  std::fwrite(s.data(), 1, s.size(), f);
  std::fclose(f);
}

void mle(const std::vector<double>& cw, const std::vector<double>& ct, int K, int V, std::vector<double>& lb) {
  lb.resize((size_t)K * V);
  for (int k = 0; k < K; k++)
    for (int w = 0; w < V; w++) {
      const double c = cw[(size_t)k * V + w];
      lb[(size_t)k * V + w] = c > 0 ? std::log(c) - std::log(ct[k]) : -100;
    }
}

bool load_model(const std::string& prefix, int& K, int& V, double& alpha, std::vector<double>& lb) {
  FILE* f = std::fopen((prefix + ".other").c_str(), "r");
  if (!f) return false;
  float a = 0;
  if (std::fscanf(f, "num_topics %d ", &K) != 1 || std::fscanf(f, "num_terms %d ", &V) != 1 ||
      std::fscanf(f, "alpha %f", &a) != 1) {
    std::fclose(f);
    throw std::runtime_error("malformed " + prefix + ".other");
  }
  std::fclose(f);
  alpha = a;
  f = std::fopen((prefix + ".beta").c_str(), "r");
  if (!f) throw std::runtime_error("missing " + prefix + ".beta");
  lb.resize((size_t)K * V);
  for (size_t i = 0; i < lb.size(); ++i) {
    float x;
    if (std::fscanf(f, "%f", &x) != 1) {
      std::fclose(f);
      throw std::runtime_error("short " + prefix + ".beta");
    }
    lb[i] = x;
  }
  std::fclose(f);
  return true;
}

std::vector<double> to_double(const std::vector<int32_t>& v) { return std::vector<double>(v.begin(), v.end()); }

}  // namespace

int ldac_estimate(const LdacCorpus& c, int K, double alpha_init, const LdacSettings& st0, const std::string& start,
                  const std::string& dir, int nshards, int threads, uint64_t seed, bool verbose) {
  LdacSettings st = st0;
  const int D = c.num_docs(), V = c.num_terms;
  ::mkdir(dir.c_str(), 0755);
  std::vector<double> cnt = to_double(c.counts);
  std::vector<double> lb;
  double alpha = alpha_init;
  std::mt19937_64 rng(seed);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  if (start == "random" || start == "seeded") {
    std::vector<double> cw((size_t)K * V, 0.0), ct(K, 0.0);
    for (int k = 0; k < K; k++) {
      if (start == "seeded") {
        for (int i = 0; i < kNumInit; i++) {
          int d = (int)std::floor(U(rng) * D);
          for (int64_t j = c.doc_ptr[d]; j < c.doc_ptr[d + 1]; ++j) cw[(size_t)k * V + c.words[j]] += c.counts[j];
        }
        for (int w = 0; w < V; w++) {
          cw[(size_t)k * V + w] += 1.0;
          ct[k] += cw[(size_t)k * V + w];
        }
      } else {
        for (int w = 0; w < V; w++) {
          cw[(size_t)k * V + w] += 1.0 / V + U(rng);
          ct[k] += cw[(size_t)k * V + w];
        }
      }
    }
    mle(cw, ct, K, V, lb);
  } else {
    int K2 = 0, V2 = 0;
    if (!load_model(start, K2, V2, alpha, lb)) throw std::runtime_error("cannot load model " + start);
    if (K2 != K || V2 != V) throw std::runtime_error("model shape does not match corpus/topics");
  }
  save_model(dir + "/000", lb, K, V, alpha);
  FILE* lf = std::fopen((dir + "/likelihood.dat").c_str(), "w");
  int i = 0;
  double L_old = 0, conv = 1;
  EStepOut r;
  while (((conv < 0) || (conv > st.em_converged) || (i <= 2)) && (i <= st.em_max_iter)) {
    i++;
    auto t0 = std::chrono::steady_clock::now();
    r = ldac_estep(c.doc_ptr.data(), c.words.data(), cnt.data(), D, V, K, lb.data(), alpha, st.var_max_iter,
                   st.var_converged, nshards, threads, st.gs_updates);
    mle(r.class_word, r.class_total, K, V, lb);
    if (st.estimate_alpha) alpha = ldac_opt_alpha(r.alpha_ss, D, K);
    conv = (L_old - r.likelihood) / L_old;
    if (conv < 0) st.var_max_iter = st.var_max_iter * 2;
    L_old = r.likelihood;
    std::fprintf(lf, "%10.10f\t%5.5e\n", r.likelihood, conv);
    std::fflush(lf);
    if (verbose) {
      double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      std::printf("**** em iteration %d **** L=%.6f conv=%.5e alpha=%.6f %.3fs\n", i, r.likelihood, conv, alpha, s);
      std::fflush(stdout);
    }
    if ((i % kLag) == 0) {
      char tag[16];
      std::snprintf(tag, sizeof(tag), "%03d", i);
      save_model(dir + "/" + tag, lb, K, V, alpha);
      save_gamma(dir + "/" + tag + ".gamma", r.gamma, D, K);
    }
  }
  std::fclose(lf);
  save_model(dir + "/final", lb, K, V, alpha);
  save_gamma(dir + "/final.gamma", r.gamma, D, K);
  // word assignments under the final model (a fresh lda_inference per document, run_em's final pass)
  const std::vector<int32_t> z = ldac_word_assignments(c.doc_ptr.data(), c.words.data(), cnt.data(), D, V, K, lb.data(),
                                                       alpha, st.var_max_iter, st.var_converged, st.gs_updates, threads);
  FILE* wf = std::fopen((dir + "/word-assignments.dat").c_str(), "w");
  for (int d = 0; d < D; d++) {
    std::fprintf(wf, "%03d", (int)(c.doc_ptr[d + 1] - c.doc_ptr[d]));
    for (int64_t e = c.doc_ptr[d]; e < c.doc_ptr[d + 1]; e++) std::fprintf(wf, " %04d:%02d", c.words[e], z[e]);
    std::fprintf(wf, "\n");
  }
  std::fclose(wf);
  return i;
}

std::vector<int32_t> ldac_word_assignments(const int64_t* doc_ptr, const int32_t* words, const double* counts, int D,
                                           int V, int K, const double* log_beta, double alpha, int var_max_iter,
                                           float var_converged, int gs_updates, int threads) {
  std::vector<int32_t> z(doc_ptr[D], 0);
  threads = std::max(1, threads);
  std::atomic<int> next{0};
  auto work = [&]() {
    Workspace ws;
    std::vector<double> gam(K);
    for (int d; (d = next.fetch_add(1)) < D;) {
      DocView dv{words + doc_ptr[d], counts + doc_ptr[d], (int)(doc_ptr[d + 1] - doc_ptr[d]), 0};
      for (int n = 0; n < dv.n; n++) dv.total += dv.c[n];
      lda_inference(dv, log_beta, V, K, alpha, var_max_iter, var_converged, gam.data(), ws, nullptr, gs_updates);
      for (int n = 0; n < dv.n; n++) {
        int best = 0;   // write_word_assignment: the first maximum
        for (int k = 1; k < K; k++)
          if (ws.phi[(size_t)n * K + k] > ws.phi[(size_t)n * K + best]) best = k;
        z[doc_ptr[d] + n] = best;
      }
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < threads; ++t) th.emplace_back(work);
  work();
  for (auto& x : th) x.join();
  return z;
}

int ldac_infer(const LdacCorpus& c, const std::string& model_prefix, const LdacSettings& st,
               const std::string& save_prefix, int nshards, int threads) {
  int K = 0, V = 0;
  double alpha = 0;
  std::vector<double> lb;
  if (!load_model(model_prefix, K, V, alpha, lb)) throw std::runtime_error("cannot load model " + model_prefix);
  const int D = c.num_docs();
  std::vector<double> cnt = to_double(c.counts);
  for (int32_t w : c.words)
    if (w >= V) throw std::runtime_error("corpus word id beyond model vocabulary");
  // per-document likelihoods need per-doc values: run docs individually in shards
  std::vector<double> gamma((size_t)D * K), lik(D);
  auto shards = shard_ranges(c.doc_ptr.data(), D, std::max(1, threads));
  std::vector<std::thread> th;
  for (auto [lo, hi] : shards) {
    th.emplace_back([&, lo = lo, hi = hi]() {
      Workspace ws;
      for (int d = lo; d < hi; d++) {
        DocView dv{c.words.data() + c.doc_ptr[d], cnt.data() + c.doc_ptr[d], (int)(c.doc_ptr[d + 1] - c.doc_ptr[d]), 0};
        for (int n = 0; n < dv.n; n++) dv.total += dv.c[n];
        lik[d] = lda_inference(dv, lb.data(), V, K, alpha, st.var_max_iter, st.var_converged,
                               gamma.data() + (size_t)d * K, ws, nullptr, st.gs_updates);
      }
    });
  }
  for (auto& x : th) x.join();
  (void)nshards;
  save_gamma(save_prefix + "-gamma.dat", gamma, D, K);
  FILE* f = std::fopen((save_prefix + "-lda-lhood.dat").c_str(), "w");
  for (int d = 0; d < D; d++) std::fprintf(f, "%5.5f\n", lik[d]);
  std::fclose(f);
  return D;
}

}  // namespace onin
