// Native runtime self-test, built by oni_ml_amd/_build.py `sanitize` under
// ThreadSanitizer / AddressSanitizer+UBSan (SURVEY.md §5.2 race detection).
// Exercises every multithreaded path of the host runtime with several thread
// counts and checks the results do not depend on them:
//   * TextTable ingest (per-thread parse + ordered dictionary merge)
//   * write_rows (per-thread formatting into ordered buffers)
//   * dns_features (per-thread parse + dictionary merge)
//   * ldac_estep (parallel inference + word-partitioned accumulation)
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "dns.h"
#include "lda_ref.h"
#include "table.h"

using namespace onin;

static int failures = 0;
#define CHECK(c)                                                     \
  do {                                                               \
    if (!(c)) {                                                      \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                    \
    }                                                                \
  } while (0)

static std::string slurp(const std::string& p) {
  std::ifstream f(p);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  std::mt19937 rng(7);
  // ---- CSV ingest ---------------------------------------------------------
  const std::string csv = dir + "/selftest_in.csv";
  {
    std::ofstream f(csv);
    f << "h0,h1,h2,h3\n";
    for (int i = 0; i < 200000; ++i) {
      f << (rng() % 1000) << ",10.0." << (rng() % 50) << "." << (rng() % 200) << ",10.1." << (rng() % 30) << ".1,"
        << (rng() % 7) << (i % 9973 == 0 ? ",\n" : "\n");
      if (i % 50021 == 0) f << "h0,h1,h2,h3\n";
    }
  }
  std::vector<ColVec<double>> nums;
  std::vector<ColVec<int32_t>> ids;
  std::vector<std::vector<std::string>> names;
  for (int th : {1, 3, 8}) {
    TextTable t(4, {0, 3}, {{1, 2}});
    t.load_files({csv}, true, th);
    t.append_text("5,10.9.9.9,10.0.0.1,3\n6,10.9.9.8,10.0.0.2,4", 1000, th);
    nums.push_back(t.num[0]);
    ids.push_back(t.ids[1]);
    names.push_back(t.dicts[0].names);
    CHECK(t.rows.size() == 200002);
    CHECK(t.n_header == 5);
    // formatted writer with all column kinds
    std::vector<int64_t> order;
    for (int64_t i = (int64_t)t.rows.size() - 1; i >= 0; i -= 3) order.push_back(i);
    std::vector<double> f64(t.rows.size());
    std::vector<int64_t> i64(t.rows.size());
    for (size_t i = 0; i < f64.size(); ++i) {
      f64[i] = t.num[0][i] / 7.0;
      i64[i] = (int64_t)i;
    }
    std::vector<OutCol> cols(4);
    cols[0].kind = OutCol::kTable;
    cols[0].table = &t;
    cols[1].kind = OutCol::kJava;
    cols[1].f64 = f64.data();
    cols[2].kind = OutCol::kInt;
    cols[2].i64 = i64.data();
    cols[3].kind = OutCol::kPair;
    cols[3].names = &t.dicts[0].names;
    cols[3].idx = t.ids[0].data();
    cols[3].idx2 = t.ids[1].data();
    const std::string out = dir + "/selftest_out_" + std::to_string(th) + ".csv";
    write_rows(out, order.data(), (int64_t)order.size(), cols, ",", false, th);
  }
  CHECK(nums[0] == nums[1] && nums[1] == nums[2]);
  CHECK(ids[0] == ids[1] && ids[1] == ids[2]);
  CHECK(names[0] == names[1] && names[1] == names[2]);
  CHECK(slurp(dir + "/selftest_out_1.csv") == slurp(dir + "/selftest_out_8.csv"));
  CHECK(slurp(dir + "/selftest_out_3.csv") == slurp(dir + "/selftest_out_8.csv"));

  // ---- DNS features --------------------------------------------------------
  std::string data;
  std::vector<int64_t> off{0};
  const char* parts[] = {"www", "mail", "a1b2c3", "x", "cdn", "co", "uk", "com", "in-addr", "arpa", "intel"};
  for (int i = 0; i < 100000; ++i) {
    int n = 1 + rng() % 5;
    std::string s;
    for (int j = 0; j < n; ++j) {
      if (j) s += '.';
      s += parts[rng() % 11];
    }
    data += s;
    off.push_back((int64_t)data.size());
  }
  std::vector<std::string> cc{"uk", "de", "jp", ""}, top{"mail", "cdn"};
  DnsFeatures a = dns_features(data.data(), off.data(), (int64_t)off.size() - 1, cc, top, "intel", 1);
  DnsFeatures b = dns_features(data.data(), off.data(), (int64_t)off.size() - 1, cc, top, "intel", 8);
  CHECK(a.domain_id == b.domain_id && a.sub_id == b.sub_id && a.entropy == b.entropy && a.domains == b.domains);

  // ---- lda-c E-step --------------------------------------------------------
  const int D = 3000, V = 500, K = 8;
  std::vector<int64_t> ptr{0};
  std::vector<int32_t> w;
  std::vector<double> c;
  for (int d = 0; d < D; ++d) {
    int n = 1 + rng() % (d % 50 == 0 ? 300 : 12);
    for (int j = 0; j < n; ++j) {
      w.push_back((int32_t)(rng() % V));
      c.push_back(1 + rng() % 4);
    }
    ptr.push_back((int64_t)w.size());
  }
  std::vector<double> lb((size_t)K * V);
  std::uniform_real_distribution<double> U(0.1, 1.0);
  for (int k = 0; k < K; ++k) {
    double s = 0;
    for (int v = 0; v < V; ++v) s += (lb[(size_t)k * V + v] = U(rng));
    for (int v = 0; v < V; ++v) lb[(size_t)k * V + v] = std::log(lb[(size_t)k * V + v] / s);
  }
  EStepOut e1 = ldac_estep(ptr.data(), w.data(), c.data(), D, V, K, lb.data(), 0.5, 20, 1e-6f, 4, 1);
  EStepOut e8 = ldac_estep(ptr.data(), w.data(), c.data(), D, V, K, lb.data(), 0.5, 20, 1e-6f, 4, 8);
  CHECK(e1.likelihood == e8.likelihood && e1.class_word == e8.class_word && e1.gamma == e8.gamma);
  CHECK(std::isfinite(e1.likelihood));

  std::printf("native selftest: %s\n", failures ? "FAILED" : "ok");
  return failures ? 1 : 0;
}
