// pybind11 module `_oninative`: the C++ host runtime of oni_ml_amd.
//   * TextTable     - multithreaded CSV ingest with the reference's semantics
//   * write_rows    - multithreaded formatted writer (Java / Python-2 / lda-c formats)
//   * dns_features  - DNS query-name parsing + Scala-order entropy
//   * lda_estep_ldac / opt_alpha / digamma - lda-c reference numerics
//   * java_double / py2_float - formatting helpers (tests, small outputs)
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <atomic>
#include <charconv>
#include <cstring>
#include <limits>
#include <thread>

#include "corpus_io.h"
#include "dns.h"
#include "fmt.h"
#include "lda_ref.h"
#include "table.h"

namespace py = pybind11;
using namespace onin;

static int default_threads();

// dst <- src in 32 MB pieces over up to default_threads() threads (a config-5 table column is 0.8 GB;
// the pieces also first-touch the new numpy buffer in parallel)
static void par_copy(void* dst, const void* src, size_t bytes) {
  constexpr size_t piece = size_t(32) << 20;
  const size_t np = (bytes + piece - 1) / piece;
  if (np <= 1) {
    if (bytes) std::memcpy(dst, src, bytes);
    return;
  }
  const int T = (int)std::min<size_t>(np, (size_t)default_threads());
  std::atomic<size_t> next{0};
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([&] {
      for (size_t i; (i = next.fetch_add(1)) < np;) {
        const size_t a = i * piece;
        std::memcpy((char*)dst + a, (const char*)src + a, std::min(piece, bytes - a));
      }
    });
  for (auto& x : th) x.join();
}

template <typename T, typename A>
static py::array_t<T> to_np(const std::vector<T, A>& v) {
  py::array_t<T> a(v.size());
  if (!v.empty()) {
    T* dst = a.mutable_data();
    py::gil_scoped_release rel;
    par_copy(dst, v.data(), v.size() * sizeof(T));
  }
  return a;
}

// Consecutive text chunks -> one numpy uint8 array (the row-sharded writers hand it to os.pwrite or
// to a byte all-to-all).
static py::array_t<uint8_t> join_chunks(const std::vector<std::string>& chunks) {
  int64_t total = 0;
  for (const auto& c : chunks) total += (int64_t)c.size();
  py::array_t<uint8_t> out(total);
  uint8_t* dst = out.mutable_data();
  {
    py::gil_scoped_release rel;
    for (const auto& c : chunks) {
      std::memcpy(dst, c.data(), c.size());
      dst += c.size();
    }
  }
  return out;
}

// Host threads a native call takes when the caller passes none (threads <= 0), resolved at CALL time:
// the calling thread's own setting (set_default_threads(n, this_thread=True): a background writer leaves
// the rank's GPU-driving thread some CPUs), else the process setting (the rank's budget, oni_ml_amd/
// ops/native.py from knobs.threads / utils/hostres.py), else min(hardware threads, 16).
static std::atomic<int> g_default_threads{0};
static thread_local int t_default_threads = 0;
static int default_threads() {
  if (t_default_threads > 0) return t_default_threads;
  const int g = g_default_threads.load(std::memory_order_relaxed);
  if (g > 0) return g;
  unsigned n = std::thread::hardware_concurrency();
  return n ? (int)std::min(n, 16u) : 4;
}
static int resolve_threads(int threads) { return threads > 0 ? threads : default_threads(); }

// Background writers (threads marked by set_default_threads(n, this_thread=True)) draw their worker
// threads from ONE process-wide pool (set_background_pool): the lda_pre writer and the model writers
// running side by side share the rank's budget instead of each taking it whole -- more runnable threads
// than the cgroup's CPU quota throttle the whole process, the thread driving the GPU with it.
static std::atomic<int> g_bg_free{-1};   // free tokens; -1: no pool configured (no limit)
struct BgThreads {
  int n = 0, taken = 0;
  explicit BgThreads(int want) {
    n = want;
    if (t_default_threads <= 0 || g_bg_free.load() < 0) return;   // not a background writer / no pool
    int cur = g_bg_free.load();
    while (taken < want && cur > 0) {
      if (g_bg_free.compare_exchange_weak(cur, cur - 1)) {
        ++taken;
        cur = g_bg_free.load();
      }
    }
    n = std::max(1, taken);   // an exhausted pool still makes progress on one thread
  }
  ~BgThreads() {
    if (taken) g_bg_free.fetch_add(taken);
  }
};

// Keeps numpy arrays / name lists alive while the writer runs.
struct ColHolder {
  std::vector<py::object> keep;
  std::vector<std::vector<std::string>> names;
};

static std::vector<OutCol> build_cols(const py::list& spec, ColHolder& h, int64_t n_rows_needed) {
  std::vector<OutCol> cols;
  h.names.reserve(spec.size());
  for (auto item : spec) {
    py::tuple t = item.cast<py::tuple>();
    std::string kind = t[0].cast<std::string>();
    OutCol c{};
    if (kind == "table") {
      c.kind = OutCol::kTable;
      c.table = t[1].cast<TextTable*>();
      h.keep.push_back(t[1]);
      if (t.size() > 2) {
        auto m = py::array_t<int64_t, py::array::c_style | py::array::forcecast>::ensure(t[2]);
        if (!m || m.size() < n_rows_needed) throw std::invalid_argument("table row map too short");
        const int64_t nr = (int64_t)c.table->rows.size();
        for (py::ssize_t i = 0; i < m.size(); ++i)
          if (m.data()[i] < 0 || m.data()[i] >= nr) throw std::invalid_argument("table row map out of range");
        h.keep.push_back(m);
        c.rowmap = m.data();
      }
    } else if (kind == "java" || kind == "py2row" || kind == "fixedrow") {
      auto a = py::array_t<double, py::array::c_style | py::array::forcecast>::ensure(t[1]);
      if (!a) throw std::invalid_argument("float64 array expected");
      h.keep.push_back(a);
      c.f64 = a.data();
      if (kind == "java") {
        c.kind = OutCol::kJava;
        if (a.size() < n_rows_needed) throw std::invalid_argument("java column too short");
      } else {
        c.kind = kind == "py2row" ? OutCol::kPy2Row : OutCol::kFixedRow;
        if (a.ndim() != 2) throw std::invalid_argument("row column needs a 2-D array");
        c.width = (int)a.shape(1);
        if (a.shape(0) < n_rows_needed) throw std::invalid_argument("row column too short");
        c.text = t.size() > 2 ? t[2].cast<std::string>() : std::string(" ");
        if (t.size() > 3 && !t[3].is_none()) {
          // optional read-back target: a writable float64 array of the same shape
          auto o = t[3].cast<py::array_t<double, py::array::c_style>>();
          if (o.ndim() != 2 || o.shape(0) != a.shape(0) || o.shape(1) != a.shape(1))
            throw std::invalid_argument("read-back array shape differs from the row column");
          h.keep.push_back(o);
          c.parsed = o.mutable_data();
        }
      }
    } else if (kind == "int") {
      auto a = py::array_t<int64_t, py::array::c_style | py::array::forcecast>::ensure(t[1]);
      if (!a) throw std::invalid_argument("int64 array expected");
      if (a.size() < n_rows_needed) throw std::invalid_argument("int column too short");
      h.keep.push_back(a);
      c.kind = OutCol::kInt;
      c.i64 = a.data();
    } else if (kind == "dict" || kind == "pair") {
      h.names.push_back(t[1].cast<std::vector<std::string>>());
      c.names = &h.names.back();
      auto a = py::array_t<int32_t, py::array::c_style | py::array::forcecast>::ensure(t[2]);
      if (!a || a.size() < n_rows_needed) throw std::invalid_argument("index column too short");
      h.keep.push_back(a);
      c.idx = a.data();
      const int64_t nn = (int64_t)c.names->size();
      for (py::ssize_t i = 0; i < a.size(); ++i)
        if (c.idx[i] >= nn || (kind == "pair" && c.idx[i] < 0)) throw std::invalid_argument("index out of range");
      c.kind = kind == "dict" ? OutCol::kDict : OutCol::kPair;
      if (kind == "pair") {
        auto b = py::array_t<int32_t, py::array::c_style | py::array::forcecast>::ensure(t[3]);
        if (!b || b.size() < n_rows_needed) throw std::invalid_argument("pair column too short");
        for (py::ssize_t i = 0; i < b.size(); ++i)
          if (b.data()[i] >= nn || b.data()[i] < 0) throw std::invalid_argument("index out of range");
        h.keep.push_back(b);
        c.idx2 = b.data();
      }
    } else if (kind == "const") {
      c.kind = OutCol::kConst;
      c.text = t[1].cast<std::string>();
    } else {
      throw std::invalid_argument("unknown column kind " + kind);
    }
    cols.push_back(std::move(c));
  }
  return cols;
}

// The module is built for x86-64-v3 (table.cpp scans lines with AVX2 compares): on a host without
// AVX2 / FMA refuse to import with a clear message instead of dying on SIGILL in the first ingest.
__attribute__((target("arch=x86-64"))) static bool host_has_avx2_fma() {
  __builtin_cpu_init();
  return __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma");
}

PYBIND11_MODULE(_oninative, m) {
  if (!host_has_avx2_fma())
    throw py::import_error("_oninative needs an x86-64-v3 CPU (AVX2 + FMA); this host lacks them");
  m.doc() = "oni_ml_amd C++ host runtime";

  py::class_<TextTable>(m, "TextTable")
      .def(py::init<int, std::vector<int>, std::vector<std::vector<int>>>(), py::arg("ncols"),
           py::arg("numeric_cols"), py::arg("dict_groups"))
      .def("load_files",
           [](TextTable& t, const std::vector<std::string>& paths, bool drop_header, int threads) {
             return t.load_files(paths, drop_header, resolve_threads(threads));
           },
           py::arg("paths"), py::arg("drop_header") = true, py::arg("threads") = 0,
           py::call_guard<py::gil_scoped_release>())
      .def("load_range",
           [](TextTable& t, const std::string& path, int64_t begin, int64_t end, const std::string& header,
              bool drop_header, int threads) {
             return t.load_range(path, begin, end, header, drop_header, resolve_threads(threads));
           },
           py::arg("path"), py::arg("begin"), py::arg("end"), py::arg("header"), py::arg("drop_header") = true,
           py::arg("threads") = 0, py::call_guard<py::gil_scoped_release>())
      .def("append_text",
           [](TextTable& t, const std::string& text, int64_t weight, int threads) {
             return t.append_text(text, weight, resolve_threads(threads));
           },
           py::arg("text"), py::arg("weight") = 1, py::arg("threads") = 0, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("num_rows", [](const TextTable& t) { return (int64_t)t.rows.size(); })
      .def_readonly("header", &TextTable::header)
      .def_readonly("n_bad_fields", &TextTable::n_bad_fields)
      .def_readonly("n_bad_numeric", &TextTable::n_bad_numeric)
      .def_readonly("n_header", &TextTable::n_header)
      .def("numeric", [](const TextTable& t, int col) {
        int s = t.numeric_slot(col);
        if (s < 0) throw std::invalid_argument("column not parsed as numeric");
        return to_np(t.num[s]);
      })
      .def("dict_ids", [](const TextTable& t, int col) {
        int s = t.dict_slot(col);
        if (s < 0) throw std::invalid_argument("column not dictionary-encoded");
        return to_np(t.ids[s]);
      })
      .def("dict_names", [](const TextTable& t, int group) {
        if (group < 0 || group >= (int)t.dicts.size()) throw std::invalid_argument("bad group");
        return t.dicts[group].names;
      })
      .def("dict_bytes", [](const TextTable& t, int group) {
        // the group's names as (concatenated UTF-8 bytes, int64 offsets [n + 1]): the row-sharded
        // dictionary merge packs them into fixed-width integer rows without a Python loop
        if (group < 0 || group >= (int)t.dicts.size()) throw std::invalid_argument("bad group");
        const auto& names = t.dicts[group].names;
        py::array_t<int64_t> off(names.size() + 1);
        int64_t* o = off.mutable_data();
        o[0] = 0;
        for (size_t i = 0; i < names.size(); ++i) o[i + 1] = o[i] + (int64_t)names[i].size();
        py::array_t<uint8_t> data(o[names.size()]);
        uint8_t* d = data.mutable_data();
        for (size_t i = 0; i < names.size(); ++i) std::memcpy(d + o[i], names[i].data(), names[i].size());
        return py::make_tuple(data, off);
      })
      .def("weights", [](const TextTable& t) { return to_np(t.weight); })
      .def("row_text", [](const TextTable& t, int64_t i) {
        if (i < 0 || i >= (int64_t)t.rows.size()) throw std::out_of_range("row");
        return std::string(t.row_text((size_t)i));
      });

  m.def(
      "write_rows",
      [](const std::string& path, py::object order, py::list spec, const std::string& sep, bool append,
         int threads, int64_t n) {
        ColHolder h;
        const int64_t* ord = nullptr;
        py::array_t<int64_t, py::array::c_style | py::array::forcecast> oa;
        int64_t max_row = n - 1;
        if (!order.is_none()) {
          oa = py::array_t<int64_t, py::array::c_style | py::array::forcecast>::ensure(order);
          ord = oa.data();
          n = oa.size();
          max_row = -1;
          for (int64_t i = 0; i < n; ++i) max_row = std::max(max_row, ord[i]);
          for (int64_t i = 0; i < n; ++i)
            if (ord[i] < 0) throw std::invalid_argument("negative row index");
        }
        auto cols = build_cols(spec, h, max_row + 1);
        for (auto& c : cols)
          if (c.kind == OutCol::kTable && !c.rowmap && max_row >= (int64_t)c.table->rows.size())
            throw std::invalid_argument("row index beyond table");
        threads = resolve_threads(threads);
        BgThreads bg(threads);
        py::gil_scoped_release rel;
        return write_rows(path, ord, n, cols, sep, append, bg.n);
      },
      py::arg("path"), py::arg("order"), py::arg("cols"), py::arg("sep") = ",", py::arg("append") = false,
      py::arg("threads") = 0, py::arg("n") = -1);
  m.def("set_default_threads", [](int n, bool this_thread) {
    if (this_thread)
      t_default_threads = n;
    else
      g_default_threads.store(n, std::memory_order_relaxed);
  }, py::arg("n"), py::arg("this_thread") = false);
  m.def("get_default_threads", []() { return default_threads(); });
  m.def("set_background_pool", [](int n) { g_bg_free.store(n); }, py::arg("n"));
  m.def("background_pool_free", []() { return g_bg_free.load(); });

  m.def(
      "format_rows",
      [](py::object order, py::list spec, const std::string& sep, int threads, int64_t n, bool row_ends) {
        ColHolder h;
        const int64_t* ord = nullptr;
        py::array_t<int64_t, py::array::c_style | py::array::forcecast> oa;
        int64_t max_row = n - 1;
        if (!order.is_none()) {
          oa = py::array_t<int64_t, py::array::c_style | py::array::forcecast>::ensure(order);
          ord = oa.data();
          n = oa.size();
          max_row = -1;
          for (int64_t i = 0; i < n; ++i) {
            if (ord[i] < 0) throw std::invalid_argument("negative row index");
            max_row = std::max(max_row, ord[i]);
          }
        }
        if (n < 0) throw std::invalid_argument("format_rows needs n or order");
        auto cols = build_cols(spec, h, max_row + 1);
        for (auto& c : cols)
          if (c.kind == OutCol::kTable && !c.rowmap && max_row >= (int64_t)c.table->rows.size())
            throw std::invalid_argument("row index beyond table");
        std::vector<int64_t> ends;
        std::vector<std::string> chunks;
        {
          py::gil_scoped_release rel;
          chunks = format_rows(ord, n, cols, sep, threads <= 0 ? default_threads() : threads, row_ends ? &ends : nullptr);
        }
        py::array_t<uint8_t> text = join_chunks(chunks);
        if (!row_ends) return py::object(text);
        return py::object(py::make_tuple(text, to_np(ends)));
      },
      py::arg("order"), py::arg("cols"), py::arg("sep") = ",", py::arg("threads") = 0, py::arg("n") = -1,
      py::arg("row_ends") = false);

  m.def(
      "dns_features",
      [](py::buffer data, py::array_t<int64_t, py::array::c_style | py::array::forcecast> offsets,
         std::vector<std::string> cc, std::vector<std::string> top, std::string special, int threads) {
        py::buffer_info bi = data.request();
        const int64_t n = offsets.size() - 1;
        if (n < 0) throw std::invalid_argument("offsets must have n+1 entries");
        const int64_t* off = offsets.data();
        for (int64_t i = 0; i < n; ++i)
          if (off[i] > off[i + 1] || off[i] < 0) throw std::invalid_argument("non-monotone offsets");
        if (n >= 0 && off[n] > (int64_t)(bi.size * bi.itemsize)) throw std::invalid_argument("offsets beyond data");
        DnsFeatures F;
        {
          py::gil_scoped_release rel;
          F = dns_features((const char*)bi.ptr, off, n, cc, top, special, resolve_threads(threads));
        }
        py::dict d;
        d["domain_id"] = to_np(F.domain_id);
        d["subdomain_id"] = to_np(F.sub_id);
        d["subdomain_length"] = to_np(F.sub_len);
        d["num_periods"] = to_np(F.num_parts);
        d["entropy"] = to_np(F.entropy);
        d["top_domain"] = to_np(F.top);
        d["domains"] = F.domains;
        d["subdomains"] = F.subs;
        return d;
      },
      py::arg("data"), py::arg("offsets"), py::arg("country_codes"), py::arg("top_domains"),
      py::arg("special") = "intel", py::arg("threads") = 0);

  // Concatenate byte spans of one buffer in the given order (the result-file merge: rows received
  // from every rank, put in global sort order).
  m.def(
      "concat_spans",
      [](py::array_t<uint8_t, py::array::c_style> src, py::array_t<int64_t, py::array::c_style | py::array::forcecast> starts,
         py::array_t<int64_t, py::array::c_style | py::array::forcecast> lens) {
        const int64_t n = starts.size();
        if (lens.size() != n) throw std::invalid_argument("starts / lens differ in length");
        const int64_t* s = starts.data();
        const int64_t* l = lens.data();
        const int64_t cap = src.size();
        int64_t total = 0;
        for (int64_t i = 0; i < n; ++i) {
          if (s[i] < 0 || l[i] < 0 || s[i] + l[i] > cap) throw std::invalid_argument("span out of range");
          total += l[i];
        }
        py::array_t<uint8_t> out(total);
        uint8_t* d = out.mutable_data();
        const uint8_t* b = src.data();
        {
          py::gil_scoped_release rel;
          for (int64_t i = 0; i < n; ++i) {
            std::memcpy(d, b + s[i], l[i]);
            d += l[i];
          }
        }
        return out;
      },
      py::arg("src"), py::arg("starts"), py::arg("lens"));

  m.def("scala_entropy", [](const std::string& s) { return scala_entropy(s); });
  m.def("java_double", [](double d) { return java_double(d); });
  m.def("py2_float", [](double d) {
    std::string s;
    append_py2_float(s, d);
    return s;
  });
  m.def("java_parse_double", [](const std::string& s) -> py::object {
    double v;
    if (!java_parse_double(s.data(), s.data() + s.size(), &v)) return py::none();
    return py::float_(v);
  });
  m.def("java_double_array", [](py::array_t<double, py::array::c_style | py::array::forcecast> a) {
    std::vector<std::string> out;
    out.reserve(a.size());
    for (py::ssize_t i = 0; i < a.size(); ++i) out.push_back(java_double(a.data()[i]));
    return out;
  });

  // Flow word strings of integer word keys (features/flow.py FlowWordSpace.decode):
  // key = (((port * NT + tb) * NB + bb) * NP + pb) * 2 + prefix -> "[-1_]<port>_<tb>_<bb>_<pb>", every
  // number in Java Double.toString form (flow_pre_lda.scala:349).  Heads (one per port and side) and
  // tails (one per bin triple) are formatted once; the words are concatenated without the GIL into
  // one buffer, then turned into str objects.
  m.def("flow_word_names", [](py::array_t<double, py::array::c_style | py::array::forcecast> ports, int NT, int NB,
                              int NP, py::array_t<int64_t, py::array::c_style | py::array::forcecast> keys) {
    const int64_t np_ = ports.size(), nk = keys.size();
    const int64_t nt = (int64_t)NT * NB * NP;
    if (NT <= 0 || NB <= 0 || NP <= 0) throw std::invalid_argument("flow_word_names: empty bin range");
    std::vector<std::string> heads(2 * np_), tails(nt);
    const int nb = std::max(NT, std::max(NB, NP));
    std::vector<std::string> bstr(nb);
    for (int i = 0; i < nb; ++i) bstr[i] = java_double((double)i);
    for (int64_t p = 0; p < np_; ++p) {
      const std::string ps = java_double(ports.data()[p]);
      heads[2 * p] = ps + "_";
      heads[2 * p + 1] = "-1_" + ps + "_";
    }
    for (int t = 0; t < NT; ++t)
      for (int b = 0; b < NB; ++b)
        for (int q = 0; q < NP; ++q) tails[((int64_t)t * NB + b) * NP + q] = bstr[t] + "_" + bstr[b] + "_" + bstr[q];
    std::string buf;
    std::vector<int64_t> ends(nk);
    const int64_t* k = keys.data();
    {
      py::gil_scoped_release rel;
      buf.reserve((size_t)nk * 24);
      for (int64_t i = 0; i < nk; ++i) {
        const int64_t key = k[i];
        const int64_t rest = key >> 1, tail = rest % nt, port = rest / nt;
        if (key < 0 || port >= np_) throw std::out_of_range("flow_word_names: key outside the word space");
        buf += heads[2 * port + (key & 1)];
        buf += tails[tail];
        ends[i] = (int64_t)buf.size();
      }
    }
    py::list out(nk);
    int64_t s = 0;
    for (int64_t i = 0; i < nk; ++i) {
      PyObject* o = PyUnicode_FromStringAndSize(buf.data() + s, (Py_ssize_t)(ends[i] - s));
      if (!o) throw py::error_already_set();
      PyList_SET_ITEM(out.ptr(), (Py_ssize_t)i, o);
      s = ends[i];
    }
    return out;
  });

  // ECDF cuts of float64 columns on the host, without the GIL (the flow input prefetch runs them while the
  // main thread imports torch; numpy's unique held the GIL long enough to slow the import, r6ak):
  // the rule and bits of features/quantiles.py ecdf_cuts -- values ordered by their int64 radix keys
  // (-0.0 below +0.0, every NaN canonical and last, ties in row order), runs of equal values under
  // `!=` (NaN never equal), exact int64 weight sums, F = cum / total in double, cut_q = the last run
  // value with F < q, max(cut, 0) taken as a select.  One thread per column.
  m.def("ecdf_cuts_cols", [](std::vector<py::array_t<double, py::array::c_style | py::array::forcecast>> cols,
                             py::object weights, std::vector<std::vector<double>> levels) {
    if (cols.size() != levels.size()) throw std::invalid_argument("ecdf_cuts_cols: one level list per column");
    const size_t nc = cols.size();
    std::vector<const double*> vp(nc);
    std::vector<int64_t> n(nc);
    for (size_t c = 0; c < nc; ++c) vp[c] = cols[c].data(), n[c] = cols[c].size();
    const int64_t* w = nullptr;
    py::array_t<int64_t, py::array::c_style | py::array::forcecast> wa;
    if (!weights.is_none()) {
      wa = py::array_t<int64_t, py::array::c_style | py::array::forcecast>::ensure(weights);
      if (!wa) throw std::invalid_argument("ecdf_cuts_cols: int64 weights expected");
      w = wa.data();
      for (size_t c = 0; c < nc; ++c)
        if (wa.size() < n[c]) throw std::invalid_argument("ecdf_cuts_cols: weights shorter than a column");
    }
    std::vector<std::vector<double>> out(nc);
    {
      py::gil_scoped_release rel;
      auto one = [&](size_t c) {
        const double* v = vp[c];
        const int64_t N = n[c];
        const std::vector<double>& q = levels[c];
        std::vector<double>& res = out[c];
        res.assign(q.size(), 0.0);
        if (N == 0) return;
        // the runs of the device's sorted order without a sort of the rows: distinct values by hashing their
        // int64 order keys (+0.0 and -0.0 one run under `!=`; the cut of either is +0.0), the distinct keys
        // sorted, then every NaN row a run of its own, last, in row order (NaN != NaN)
        // (open addressing, grown at half load: the table follows the distinct count, not the rows)
        size_t cap = 1 << 12, used = 0;
        int sh = 64 - __builtin_ctzll(cap);
        std::vector<int64_t> hk(cap, INT64_MIN), hw(cap, 0);
        auto slot = [&](int64_t k) {
          size_t h = (size_t)(((uint64_t)k * 0x9E3779B97F4A7C15ull) >> sh);
          while (hk[h] != INT64_MIN && hk[h] != k) h = (h + 1) & (cap - 1);
          return h;
        };
        std::vector<int64_t> nan_w;
        for (int64_t i = 0; i < N; ++i) {
          double x = v[i];
          const int64_t wi = w ? w[i] : 1;
          if (x != x) {
            nan_w.push_back(wi);
            continue;
          }
          if (x == 0.0) x = 0.0;
          int64_t k;
          std::memcpy(&k, &x, 8);
          k = k < 0 ? (k ^ INT64_MAX) : k;
          size_t h = slot(k);
          if (hk[h] == INT64_MIN) {
            if (2 * (used + 1) > cap) {   // grow, re-insert, and find k's slot again
              std::vector<int64_t> ok(std::move(hk)), ow(std::move(hw));
              cap <<= 1;
              sh = 64 - __builtin_ctzll(cap);
              hk.assign(cap, INT64_MIN);
              hw.assign(cap, 0);
              for (size_t j = 0; j < ok.size(); ++j)
                if (ok[j] != INT64_MIN) {
                  const size_t g = slot(ok[j]);
                  hk[g] = ok[j];
                  hw[g] = ow[j];
                }
              h = slot(k);
            }
            hk[h] = k;
            ++used;
          }
          hw[h] += wi;
        }
        std::vector<std::pair<int64_t, int64_t>> kw;
        for (size_t h = 0; h < cap; ++h)
          if (hk[h] != INT64_MIN) kw.emplace_back(hk[h], hw[h]);
        std::sort(kw.begin(), kw.end());
        std::vector<double> uv;
        std::vector<int64_t> cum;
        uv.reserve(kw.size() + nan_w.size());
        cum.reserve(kw.size() + nan_w.size());
        int64_t acc = 0;
        for (const auto& e : kw) {
          int64_t k = e.first < 0 ? (e.first ^ INT64_MAX) : e.first;
          double x;
          std::memcpy(&x, &k, 8);
          uv.push_back(x);
          cum.push_back(acc += e.second);
        }
        for (int64_t wi : nan_w) {
          uv.push_back(std::numeric_limits<double>::quiet_NaN());
          cum.push_back(acc += wi);
        }
        const double tot = (double)acc;
        for (size_t j = 0; j < q.size(); ++j) {
          // searchsorted(F, q, left) - 1: the last run with F < q
          int64_t lo = 0, hi = (int64_t)cum.size();
          while (lo < hi) {
            const int64_t mid = (lo + hi) / 2;
            if ((double)cum[(size_t)mid] / tot < q[j]) lo = mid + 1;
            else hi = mid;
          }
          const double cand = lo - 1 >= 0 ? uv[(size_t)(lo - 1)] : 0.0;
          res[j] = cand > 0 ? cand : 0.0;
        }
      };
      std::vector<std::thread> th;
      for (size_t c = 1; c < nc; ++c) th.emplace_back(one, c);
      if (nc) one(0);
      for (auto& t : th) t.join();
    }
    return out;
  });

  // DNS word strings of mixed-radix word keys (features/dns.py DnsWordSpace.decode):
  // key = ((top * r0 + d0) * r1 + d1 ...) * len(tail) + q -> "<top>_<d0>_<d1>..._<tail[q]>" (dns_pre_lda.scala's
  // word: the top-domain flag, the five bins, the query-type / response-code pair).
  m.def("radix_word_names", [](py::array_t<int64_t, py::array::c_style | py::array::forcecast> keys,
                               std::vector<int64_t> radix, std::vector<std::string> tail) {
    const int64_t nk = keys.size(), nq = std::max<int64_t>(1, (int64_t)tail.size());
    for (int64_t r : radix)
      if (r <= 0) throw std::invalid_argument("radix_word_names: radix must be positive");
    const int64_t* k = keys.data();
    std::string buf;
    std::vector<int64_t> ends(nk);
    {
      py::gil_scoped_release rel;
      buf.reserve((size_t)nk * 24);
      std::vector<int64_t> d(radix.size());
      char tmp[24];
      for (int64_t i = 0; i < nk; ++i) {
        int64_t x = k[i];
        if (x < 0) throw std::out_of_range("radix_word_names: negative key");
        const int64_t q = x % nq;
        x /= nq;
        for (size_t j = radix.size(); j-- > 0;) {
          d[j] = x % radix[j];
          x /= radix[j];
        }
        auto put = [&](int64_t v) {
          auto r = std::to_chars(tmp, tmp + sizeof(tmp), v);
          buf.append(tmp, r.ptr);
        };
        put(x);
        for (int64_t v : d) {
          buf += '_';
          put(v);
        }
        buf += '_';
        buf += tail.at((size_t)q);   // (no tail: out_of_range, as the Python form's IndexError)
        ends[i] = (int64_t)buf.size();
      }
    }
    py::list out(nk);
    int64_t s = 0;
    for (int64_t i = 0; i < nk; ++i) {
      PyObject* o = PyUnicode_FromStringAndSize(buf.data() + s, (Py_ssize_t)(ends[i] - s));
      if (!o) throw py::error_already_set();
      PyList_SET_ITEM(out.ptr(), (Py_ssize_t)i, o);
      s = ends[i];
    }
    return out;
  });

  // Value round trips through the reference's text hand-offs: "%5.10f"
  // (final.gamma / final.beta read back by lda_post.py) and Python-2 str
  // (doc_results.csv / word_results.csv read back by the Scala scorers).
  auto roundtrip = [](py::array_t<double, py::array::c_style | py::array::forcecast> a, int mode, int threads) {
    py::array_t<double> out(a.request().shape);
    const double* src = a.data();
    double* dst = out.mutable_data();
    const int64_t n = a.size();
    if (threads <= 0) threads = default_threads();
    if (n < 65536) threads = 1;
    {
      py::gil_scoped_release rel;
      auto work = [&](int t) {
        std::string s;
        for (int64_t i = n * t / threads; i < n * (t + 1) / threads; ++i) {
          if (mode == 1 && py2_value(src[i], dst + i)) continue;     // no text needed
          s.clear();
          if (mode == 0) append_fixed10(s, src[i], dst + i);
          else append_py2_float(s, src[i], dst + i);
        }
      };
      std::vector<std::thread> th;
      for (int t = 1; t < threads; ++t) th.emplace_back(work, t);
      work(0);
      for (auto& x : th) x.join();
    }
    return out;
  };
  // Fast shortest-digit formatting (fmt.h) against the exact printf-equivalent conversions:
  // (text mismatches, read-back mismatches, first bad index or -1).
  m.def("fmt_selfcheck", [](py::array_t<double, py::array::c_style | py::array::forcecast> a, int mode) {
    const double* src = a.data();
    int64_t bad_text = 0, bad_value = 0, first = -1;
    {
      py::gil_scoped_release rel;
      std::string f, x;
      for (py::ssize_t i = 0; i < a.size(); ++i) {
        f.clear();
        x.clear();
        double back = 0, ref = 0;
        if (mode == 0) { append_fixed10(f, src[i], &back); append_fixed10_exact(x, src[i]); }
        else { append_py2_float(f, src[i], &back); append_py2_float_exact(x, src[i]); }
        std::from_chars(x.data() + (x[0] == ' ' ? x.find_first_not_of(' ') : 0), x.data() + x.size(), ref);
        const bool tb = f != x, vb = !(back == ref || (back != back && ref != ref));
        bad_text += tb;
        bad_value += vb;
        if ((tb || vb) && first < 0) first = i;
      }
    }
    return py::make_tuple(bad_text, bad_value, first);
  });
  m.def("roundtrip_fixed10", [roundtrip](py::array_t<double, py::array::c_style | py::array::forcecast> a, int threads) {
    return roundtrip(a, 0, threads);
  }, py::arg("a"), py::arg("threads") = 0);
  m.def("roundtrip_py2", [roundtrip](py::array_t<double, py::array::c_style | py::array::forcecast> a, int threads) {
    return roundtrip(a, 1, threads);
  }, py::arg("a"), py::arg("threads") = 0);

  // lda_post.py's normalisations with numpy's arithmetic, row-parallel: each sum runs left to right in
  // double like np.cumsum(..., axis=1)[:, -1] (and Python's builtin sum), each quotient is one IEEE
  // division -- bitwise numpy's results, without its [rows, K] cumsum temporary (config 5: 5.7 M x 100)
  m.def("doc_topics", [](py::array_t<double, py::array::c_style | py::array::forcecast> g, int threads) {
    if (g.ndim() != 2) throw std::invalid_argument("gamma must be [D, K]");
    const int64_t D = g.shape(0), K = g.shape(1);
    py::array_t<double> out({D, K});
    const double* src = g.data();
    double* dst = out.mutable_data();
    if (threads <= 0) threads = default_threads();
    if (D * K < (1 << 16)) threads = 1;
    {
      py::gil_scoped_release rel;
      auto work = [&](int t) {
        for (int64_t d = D * t / threads; d < D * (t + 1) / threads; ++d) {
          const double* r = src + d * K;
          double* o = dst + d * K;
          double s = 0.0;
          for (int64_t k = 0; k < K; ++k) s += r[k];
          if (s > 0) {
            for (int64_t k = 0; k < K; ++k) o[k] = r[k] / s;
          } else {
            for (int64_t k = 0; k < K; ++k) o[k] = 0.0;
          }
        }
      };
      std::vector<std::thread> th;
      for (int t = 1; t < threads; ++t) th.emplace_back(work, t);
      work(0);
      for (auto& x : th) x.join();
    }
    return out;
  }, py::arg("gamma"), py::arg("threads") = 0);
  // p(w|z): raw [K, V] (exp log beta, numpy's exp) -> [V, K] with each topic over its sequential sum
  m.def("topic_normalize_t", [](py::array_t<double, py::array::c_style | py::array::forcecast> raw, int threads) {
    if (raw.ndim() != 2) throw std::invalid_argument("raw must be [K, V]");
    const int64_t K = raw.shape(0), V = raw.shape(1);
    py::array_t<double> out({V, K});
    const double* src = raw.data();
    double* dst = out.mutable_data();
    if (threads <= 0) threads = default_threads();
    if (K * V < (1 << 16)) threads = 1;
    std::vector<double> total((size_t)K, 0.0);
    {
      py::gil_scoped_release rel;
      const int ts = (int)std::min<int64_t>(threads, std::max<int64_t>(K, 1));
      auto sums = [&](int t) {                    // one thread per block of topics
        for (int64_t k = K * t / ts; k < K * (t + 1) / ts; ++k) {
          const double* r = src + k * V;
          double s = 0.0;
          for (int64_t v = 0; v < V; ++v) s += r[v];
          total[(size_t)k] = s;
        }
      };
      auto tr = [&](int t) {
        constexpr int64_t B = 64;                 // words per block: K x B reads, B x K writes
        const int64_t a = V * t / threads, b = V * (t + 1) / threads;
        for (int64_t lo = a; lo < b; lo += B) {
          const int64_t hi = std::min(lo + B, b);
          for (int64_t k = 0; k < K; ++k) {
            const double* r = src + k * V;
            const double tk = total[(size_t)k];
            for (int64_t v = lo; v < hi; ++v) dst[v * K + k] = r[v] / tk;
          }
        }
      };
      {
        std::vector<std::thread> th;
        for (int t = 1; t < ts; ++t) th.emplace_back(sums, t);
        sums(0);
        for (auto& x : th) x.join();
      }
      std::vector<std::thread> th;
      for (int t = 1; t < threads; ++t) th.emplace_back(tr, t);
      tr(0);
      for (auto& x : th) x.join();
    }
    return out;
  }, py::arg("raw"), py::arg("threads") = 0);

  // lda-c corpus text (model.dat)
  m.def(
      "write_ldac_corpus",
      [](const std::string& path, py::array_t<int64_t, py::array::c_style | py::array::forcecast> ptr,
         py::array_t<int32_t, py::array::c_style | py::array::forcecast> words,
         py::array_t<int64_t, py::array::c_style | py::array::forcecast> counts, int threads, bool assignments) {
        const int64_t D = (int64_t)ptr.size() - 1;
        if (D < 0) throw std::invalid_argument("doc_ptr must have D+1 entries");
        const int64_t* p = ptr.data();
        if (p[0] != 0 || p[D] != (int64_t)words.size() || words.size() != counts.size())
          throw std::invalid_argument("inconsistent corpus arrays");
        for (int64_t d = 0; d < D; ++d)
          if (p[d] > p[d + 1]) throw std::invalid_argument("non-monotone doc_ptr");
        if (threads <= 0) threads = default_threads();
        BgThreads bg(threads);
        py::gil_scoped_release rel;
        if (assignments)
          for (int64_t i = 0; i < (int64_t)counts.size(); ++i)
            if (counts.data()[i] < 0 || words.data()[i] < 0) throw std::invalid_argument("negative word or topic");
        return write_corpus_text(path, p, D, words.data(), counts.data(), bg.n, assignments);
      },
      py::arg("path"), py::arg("doc_ptr"), py::arg("words"), py::arg("counts"), py::arg("threads") = 0,
      py::arg("assignments") = false);
  m.def(
      "format_ldac_corpus",
      [](py::array_t<int64_t, py::array::c_style | py::array::forcecast> ptr,
         py::array_t<int32_t, py::array::c_style | py::array::forcecast> words,
         py::array_t<int64_t, py::array::c_style | py::array::forcecast> counts, int threads, bool assignments) {
        const int64_t D = (int64_t)ptr.size() - 1;
        if (D < 0) throw std::invalid_argument("doc_ptr must have D+1 entries");
        const int64_t* p = ptr.data();
        if (p[0] != 0 || p[D] != (int64_t)words.size() || words.size() != counts.size())
          throw std::invalid_argument("inconsistent corpus arrays");
        for (int64_t d = 0; d < D; ++d)
          if (p[d] > p[d + 1]) throw std::invalid_argument("non-monotone doc_ptr");
        if (threads <= 0) threads = default_threads();
        std::vector<std::string> chunks;
        {
          py::gil_scoped_release rel;
          chunks = format_corpus_text(p, D, words.data(), counts.data(), threads, assignments);
        }
        return join_chunks(chunks);
      },
      py::arg("doc_ptr"), py::arg("words"), py::arg("counts"), py::arg("threads") = 0,
      py::arg("assignments") = false);
  m.def(
      "read_ldac_corpus",
      [](const std::string& path, int threads) {
        if (threads <= 0) threads = default_threads();
        TextCorpus c;
        {
          py::gil_scoped_release rel;
          c = read_corpus_text(path, threads);
        }
        return py::make_tuple(to_np(c.doc_ptr), to_np(c.words), to_np(c.counts));
      },
      py::arg("path"), py::arg("threads") = 0);

  // lda-c "random" start: [K, V] class_word = 1/V + u, the counter-based generator of the HIP
  // init_random_ss kernel (csrc/hip/lda_gs64.hip), so every backend starts from the same bits
  m.def(
      "random_ss",
      [](int K, int V, unsigned long long seed, int threads) {
        if (K < 0 || V < 0) throw std::invalid_argument("K, V must be >= 0");
        py::array_t<double> out({(py::ssize_t)K, (py::ssize_t)V});
        double* o = out.mutable_data();
        if (threads <= 0) threads = default_threads();
        {
          py::gil_scoped_release rel;
          auto mix = [](unsigned long long x) {
            x += 0x9E3779B97F4A7C15ull;
            x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
            x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
            return x ^ (x >> 31);
          };
          const unsigned long long s = mix(seed);
          const double inv = 1.0 / (double)V;
          const long long total = (long long)K * V;
          auto work = [&](int t) {
            for (long long i = total * t / threads; i < total * (t + 1) / threads; ++i)
              o[i] = inv + (double)(mix(s ^ (unsigned long long)i) >> 11) * 0x1.0p-53;
          };
          std::vector<std::thread> th;
          for (int t = 1; t < threads; ++t) th.emplace_back(work, t);
          work(0);
          for (auto& x : th) x.join();
        }
        return out;
      },
      py::arg("K"), py::arg("V"), py::arg("seed"), py::arg("threads") = 0);

  // ---------------------------------------------------------------- lda-c --
  m.def("digamma", &ldac_digamma);
  m.def("trigamma", &ldac_trigamma);
  m.def("log_sum", &ldac_log_sum);
  m.def("opt_alpha", &ldac_opt_alpha, py::arg("ss"), py::arg("D"), py::arg("K"));
  m.def(
      "lda_assign_ldac",
      [](py::array_t<int64_t, py::array::c_style | py::array::forcecast> doc_ptr,
         py::array_t<int32_t, py::array::c_style | py::array::forcecast> words,
         py::array_t<double, py::array::c_style | py::array::forcecast> counts,
         py::array_t<double, py::array::c_style | py::array::forcecast> log_beta, double alpha, int var_max_iter,
         double var_conv, int threads, int gs_updates) {
        const int D = (int)doc_ptr.size() - 1;
        if (log_beta.ndim() != 2) throw std::invalid_argument("log_beta must be [K, V]");
        const int K = (int)log_beta.shape(0), V = (int)log_beta.shape(1);
        if (words.size() != counts.size() || doc_ptr.data()[D] != words.size())
          throw std::invalid_argument("inconsistent corpus arrays");
        for (py::ssize_t i = 0; i < words.size(); ++i)
          if (words.data()[i] < 0 || words.data()[i] >= V) throw std::invalid_argument("word id out of range");
        if (threads <= 0) threads = default_threads();
        std::vector<int32_t> z;
        {
          py::gil_scoped_release rel;
          z = ldac_word_assignments(doc_ptr.data(), words.data(), counts.data(), D, V, K, log_beta.data(), alpha,
                                    var_max_iter, (float)var_conv, gs_updates, threads);
        }
        return to_np(z);
      },
      py::arg("doc_ptr"), py::arg("words"), py::arg("counts"), py::arg("log_beta"), py::arg("alpha"),
      py::arg("var_max_iter"), py::arg("var_conv"), py::arg("threads") = 0, py::arg("gs_updates") = 0);
  m.def(
      "lda_estep_ldac",
      [](py::array_t<int64_t, py::array::c_style | py::array::forcecast> doc_ptr,
         py::array_t<int32_t, py::array::c_style | py::array::forcecast> words,
         py::array_t<double, py::array::c_style | py::array::forcecast> counts,
         py::array_t<double, py::array::c_style | py::array::forcecast> log_beta, double alpha, int var_max_iter,
         double var_conv, int nshards, int threads, int gs_updates) {
        const int D = (int)doc_ptr.size() - 1;
        if (log_beta.ndim() != 2) throw std::invalid_argument("log_beta must be [K, V]");
        const int K = (int)log_beta.shape(0), V = (int)log_beta.shape(1);
        if (words.size() != counts.size() || doc_ptr.data()[D] != words.size())
          throw std::invalid_argument("inconsistent corpus arrays");
        for (py::ssize_t i = 0; i < words.size(); ++i)
          if (words.data()[i] < 0 || words.data()[i] >= V) throw std::invalid_argument("word id out of range");
        if (threads <= 0) threads = default_threads();
        EStepOut r;
        {
          py::gil_scoped_release rel;
          r = ldac_estep(doc_ptr.data(), words.data(), counts.data(), D, V, K, log_beta.data(), alpha,
                         var_max_iter, (float)var_conv, nshards, threads, gs_updates);
        }
        py::dict d;
        d["likelihood"] = r.likelihood;
        d["alpha_ss"] = r.alpha_ss;
        py::array_t<double> cw({K, V});
        std::memcpy(cw.mutable_data(), r.class_word.data(), r.class_word.size() * sizeof(double));
        d["class_word"] = cw;
        d["class_total"] = to_np(r.class_total);
        py::array_t<double> g({D, K});
        if (!r.gamma.empty()) std::memcpy(g.mutable_data(), r.gamma.data(), r.gamma.size() * sizeof(double));
        d["gamma"] = g;
        d["iters"] = to_np(r.iters);
        d["doc_likelihood"] = to_np(r.doc_lik);
        return d;
      },
      py::arg("doc_ptr"), py::arg("words"), py::arg("counts"), py::arg("log_beta"), py::arg("alpha"),
      py::arg("var_max_iter"), py::arg("var_conv"), py::arg("nshards") = 1, py::arg("threads") = 0,
      py::arg("gs_updates") = 0);
}
