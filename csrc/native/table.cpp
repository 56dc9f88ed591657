#include "table.h"

#include <algorithm>
#include <charconv>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <stdexcept>
#include <thread>

#include "fmt.h"

namespace onin {

namespace {

struct LocalDict {
  std::vector<std::string_view> names;
  std::unordered_map<std::string_view, int32_t> index;
  int32_t get_or_add(std::string_view s) {
    auto it = index.find(s);
    if (it != index.end()) return it->second;
    int32_t id = (int32_t)names.size();
    names.push_back(s);
    index.emplace(s, id);
    return id;
  }
};

struct LocalOut {
  std::vector<uint64_t> off;
  std::vector<uint32_t> len;
  std::vector<std::vector<double>> num;
  std::vector<std::vector<int32_t>> ids;
  std::vector<LocalDict> dicts;
  int64_t bad_fields = 0, bad_numeric = 0, header = 0;
};

inline bool is_ws(char c) { return (unsigned char)c <= ' '; }

// Number of fields String.split(",") returns for [b, e).
inline int java_split_count(const char* b, const char* e) {
  if (b == e) return 1;
  const char* t = e;
  while (t > b && t[-1] == ',') --t;
  if (t == b) return 0;  // only separators: every field empty and trailing
  int n = 1;
  for (const char* p = b; p < t; ++p) n += (*p == ',');
  return n;
}

std::vector<size_t> split_points(const std::string& s, int parts) {
  std::vector<size_t> pts{0};
  const size_t n = s.size();
  for (int i = 1; i < parts; ++i) {
    size_t p = n * i / parts;
    if (p < pts.back()) p = pts.back();
    while (p < n && s[p - 1] != '\n') ++p;
    pts.push_back(p);
  }
  pts.push_back(n);
  return pts;
}

}  // namespace

TextTable::TextTable(int ncols_, std::vector<int> numeric_cols_, std::vector<std::vector<int>> dict_groups_)
    : ncols(ncols_), numeric_cols(std::move(numeric_cols_)), dict_groups(std::move(dict_groups_)) {
  for (int c : numeric_cols)
    if (c < 0 || c >= ncols) throw std::invalid_argument("numeric column out of range");
  num.resize(numeric_cols.size());
  for (size_t g = 0; g < dict_groups.size(); ++g)
    for (int c : dict_groups[g]) {
      if (c < 0 || c >= ncols) throw std::invalid_argument("dictionary column out of range");
      dict_col_group.push_back((int)g);
      dict_col_index.push_back(c);
    }
  ids.resize(dict_col_index.size());
  dicts.resize(dict_groups.size());
}

int TextTable::numeric_slot(int col) const {
  for (size_t i = 0; i < numeric_cols.size(); ++i)
    if (numeric_cols[i] == col) return (int)i;
  return -1;
}

int TextTable::dict_slot(int col) const {
  for (size_t i = 0; i < dict_col_index.size(); ++i)
    if (dict_col_index[i] == col) return (int)i;
  return -1;
}

void TextTable::load_files(const std::vector<std::string>& paths, bool drop_hdr, int threads) {
  drop_header = drop_hdr;
  bool first = true;
  for (const auto& p : paths) {
    std::ifstream f(p, std::ios::binary);
    if (!f) throw std::runtime_error("cannot open " + p);
    f.seekg(0, std::ios::end);
    std::string s((size_t)f.tellg(), '\0');
    f.seekg(0);
    f.read(s.data(), (std::streamsize)s.size());
    if (first && drop_header) {
      size_t e = s.find('\n');
      header = s.substr(0, e == std::string::npos ? s.size() : e);
      if (!header.empty() && header.back() == '\r') header.pop_back();
    }
    first = false;
    if (!s.empty() && s.back() != '\n') s.push_back('\n');
    chunks.push_back(std::move(s));
    ingest_chunk((uint32_t)(chunks.size() - 1), 1, threads);
  }
}

void TextTable::load_range(const std::string& path, int64_t begin, int64_t end, const std::string& hdr,
                           bool drop_hdr, int threads) {
  drop_header = drop_hdr;
  header = hdr;
  if (!header.empty() && header.back() == '\r') header.pop_back();
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  f.seekg(0, std::ios::end);
  const int64_t size = (int64_t)f.tellg();
  begin = std::max<int64_t>(0, std::min(begin, size));
  end = std::max(begin, std::min(end, size));
  // first line starting at or after `begin`
  int64_t b = begin;
  if (b > 0) {
    f.seekg(b - 1);
    char c = 0;
    f.get(c);
    if (c != '\n') {
      std::string rest;
      std::getline(f, rest);                 // the line begun before `begin` belongs to the previous range
      b = (int64_t)f.tellg();
      if (b < 0) b = size;                   // no newline after it: nothing of ours in the file
    }
  }
  // first line starting at or after `end` (our last line runs up to it)
  int64_t e = end;
  if (e < size && e > 0) {
    f.clear();
    f.seekg(e - 1);
    char c = 0;
    f.get(c);
    if (c != '\n') {
      std::string rest;
      std::getline(f, rest);
      e = (int64_t)f.tellg();
      if (e < 0) e = size;
    }
  }
  if (b >= e) return;
  f.clear();
  f.seekg(b);
  std::string s((size_t)(e - b), '\0');
  f.read(s.data(), (std::streamsize)s.size());
  if (!s.empty() && s.back() != '\n') s.push_back('\n');
  chunks.push_back(std::move(s));
  ingest_chunk((uint32_t)(chunks.size() - 1), 1, threads);
}

void TextTable::append_text(std::string text, int32_t w, int threads) {
  if (!text.empty() && text.back() != '\n') text.push_back('\n');
  chunks.push_back(std::move(text));
  ingest_chunk((uint32_t)(chunks.size() - 1), w, threads);
}

void TextTable::ingest_chunk(uint32_t cid, int32_t w, int threads) {
  const std::string& s = chunks[cid];
  if (threads < 1) threads = 1;
  if (s.size() < (1u << 20)) threads = 1;
  auto pts = split_points(s, threads);
  const int T = (int)pts.size() - 1;
  std::vector<LocalOut> outs(T);
  const int NN = (int)numeric_cols.size(), ND = (int)dict_col_index.size();
  // column -> (numeric slot, dict slot)
  std::vector<int> nslot(ncols, -1), dslot(ncols, -1);
  for (int i = 0; i < NN; ++i) nslot[numeric_cols[i]] = i;
  for (int i = 0; i < ND; ++i) dslot[dict_col_index[i]] = i;

  auto work = [&](int t) {
    LocalOut& o = outs[t];
    o.num.resize(NN);
    o.ids.resize(ND);
    o.dicts.resize(dicts.size());
    std::vector<const char*> fb(ncols), fe(ncols);
    std::vector<double> vals(NN);
    std::vector<std::string_view> svals(ND);
    const char* base = s.data();
    size_t p = pts[t];
    const size_t end = pts[t + 1];
    while (p < end) {
      const char* lb = base + p;
      const char* nl = (const char*)std::memchr(lb, '\n', end - p);
      const char* le = nl ? nl : base + end;
      p = (le - base) + 1;
      if (le > lb && le[-1] == '\r') --le;
      if (drop_header && (size_t)(le - lb) == header.size() && std::memcmp(lb, header.data(), header.size()) == 0) {
        ++o.header;
        continue;
      }
      if (java_split_count(lb, le) != ncols) { ++o.bad_fields; continue; }
      const char* tb = lb;
      const char* te = le;
      while (tb < te && is_ws(*tb)) ++tb;
      while (te > tb && is_ws(te[-1])) --te;
      while (te > tb && te[-1] == ',') --te;  // trailing empty fields vanish in split + mkString
      if (java_split_count(tb, te) != ncols) { ++o.bad_fields; continue; }
      // field boundaries
      int f = 0;
      const char* q = tb;
      fb[0] = tb;
      for (; q < te; ++q) {
        if (*q == ',') {
          fe[f] = q;
          fb[++f] = q + 1;
        }
      }
      fe[f] = te;
      bool ok = true;
      for (int i = 0; i < NN && ok; ++i) {
        const int c = numeric_cols[i];
        ok = java_parse_double(fb[c], fe[c], &vals[i]);
      }
      if (!ok) { ++o.bad_numeric; continue; }
      o.off.push_back((uint64_t)(tb - base));
      o.len.push_back((uint32_t)(te - tb));
      for (int i = 0; i < NN; ++i) o.num[i].push_back(vals[i]);
      for (int i = 0; i < ND; ++i) {
        const int c = dict_col_index[i];
        o.ids[i].push_back(o.dicts[dict_col_group[i]].get_or_add(std::string_view(fb[c], fe[c] - fb[c])));
      }
    }
  };
  if (T == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back(work, t);
    for (auto& x : th) x.join();
  }
  // ordered merge
  for (int t = 0; t < T; ++t) {
    LocalOut& o = outs[t];
    n_bad_fields += o.bad_fields;
    n_bad_numeric += o.bad_numeric;
    n_header += o.header;
    std::vector<std::vector<int32_t>> remap(dicts.size());
    for (size_t g = 0; g < dicts.size(); ++g) {
      remap[g].resize(o.dicts[g].names.size());
      for (size_t j = 0; j < o.dicts[g].names.size(); ++j) remap[g][j] = dicts[g].get_or_add(o.dicts[g].names[j]);
    }
    const size_t n = o.off.size();
    for (size_t r = 0; r < n; ++r) rows.push_back(RowSpan{cid, o.len[r], o.off[r]});
    weight.insert(weight.end(), n, w);
    for (int i = 0; i < NN; ++i) num[i].insert(num[i].end(), o.num[i].begin(), o.num[i].end());
    for (int i = 0; i < ND; ++i) {
      auto& rm = remap[dict_col_group[i]];
      for (int32_t v : o.ids[i]) ids[i].push_back(rm[v]);
    }
  }
}

// ------------------------------------------------------------------ writer --

static void format_row(std::string& out, int64_t r, const std::vector<OutCol>& cols, const std::string& sep) {
  for (size_t c = 0; c < cols.size(); ++c) {
    if (c) out += sep;
    const OutCol& k = cols[c];
    switch (k.kind) {
      case OutCol::kTable: {
        auto v = k.table->row_text((size_t)(k.rowmap ? k.rowmap[r] : r));
        out.append(v.data(), v.size());
        break;
      }
      case OutCol::kJava:
        append_java_double(out, k.f64[r]);
        break;
      case OutCol::kInt:
        append_int(out, k.i64[r]);
        break;
      case OutCol::kDict: {
        int32_t i = k.idx[r];
        if (i >= 0) out += (*k.names)[i];
        break;
      }
      case OutCol::kPair: {
        // flow ip_pair (flow_pre_lda.scala:328-329): "sip dip" if sip < dip (String order) else "dip sip"
        const std::string& a = (*k.names)[k.idx[r]];
        const std::string& b = (*k.names)[k.idx2[r]];
        if (a < b) { out += a; out += ' '; out += b; }
        else { out += b; out += ' '; out += a; }
        break;
      }
      case OutCol::kConst:
        out += k.text;
        break;
      case OutCol::kPy2Row:
      case OutCol::kFixedRow: {
        const double* row = k.f64 + (size_t)r * k.width;
        double* back = k.parsed ? k.parsed + (size_t)r * k.width : nullptr;
        for (int j = 0; j < k.width; ++j) {
          if (j) out += k.text;
          const size_t at = out.size();
          if (k.kind == OutCol::kPy2Row) append_py2_float(out, row[j]);
          else append_fixed10(out, row[j]);
          if (back) std::from_chars(out.data() + at, out.data() + out.size(), back[j]);
        }
        break;
      }
    }
  }
  out += '\n';
}

int64_t write_rows(const std::string& path, const int64_t* order, int64_t n, const std::vector<OutCol>& cols,
                   const std::string& sep, bool append, int threads) {
  FILE* f = std::fopen(path.c_str(), append ? "ab" : "wb");
  if (!f) throw std::runtime_error("cannot open for writing: " + path);
  if (threads < 1) threads = 1;
  // Rows per thread block: ~2^16 cells of work per block, so wide rows (a K x V
  // .beta file has K rows of V values) still spread over every thread.
  int64_t cells = 0;
  for (const OutCol& c : cols) cells += (c.kind == OutCol::kPy2Row || c.kind == OutCol::kFixedRow) ? c.width : 1;
  const int64_t block = std::max<int64_t>(1, (int64_t(1) << 16) / std::max<int64_t>(1, cells));
  int64_t written = 0;
  std::vector<std::string> bufs(threads);
  for (int64_t b0 = 0; b0 < n; b0 += block * threads) {
    auto work = [&](int t) {
      std::string& s = bufs[t];
      s.clear();
      const int64_t lo = b0 + t * block, hi = std::min(n, lo + block);
      for (int64_t i = lo; i < hi; ++i) format_row(s, order ? order[i] : i, cols, sep);
    };
    if (threads == 1 || n - b0 <= block) {
      work(0);
      for (int t = 1; t < threads; ++t) bufs[t].clear();
    } else {
      std::vector<std::thread> th;
      for (int t = 0; t < threads; ++t) th.emplace_back(work, t);
      for (auto& x : th) x.join();
    }
    for (auto& s : bufs) {
      if (!s.empty() && std::fwrite(s.data(), 1, s.size(), f) != s.size()) {
        std::fclose(f);
        throw std::runtime_error("short write: " + path);
      }
      written += (int64_t)s.size();
    }
  }
  if (std::fclose(f) != 0) throw std::runtime_error("close failed: " + path);
  return written;
}

}  // namespace onin
