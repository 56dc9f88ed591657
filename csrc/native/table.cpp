#include "table.h"

#include <future>

#include <immintrin.h>

#include <algorithm>
#include <charconv>
#include <cstdio>
#include <atomic>
#include <chrono>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <fcntl.h>
#include <fstream>
#include <unistd.h>
#include <stdexcept>
#include <thread>

#include "fmt.h"

namespace onin {

namespace {

// ONI_PROFILE contains "table": ingest and writer timings on stderr
bool table_profile() {
  static const bool on = [] {
    const char* e = std::getenv("ONI_PROFILE");
    return e && std::strstr(e, "table") != nullptr;
  }();
  return on;
}

struct alignas(64) LocalOut {
  std::vector<uint64_t> off;
  std::vector<uint32_t> len;
  std::vector<std::vector<double>> num;
  std::vector<std::vector<int32_t>> ids;
  std::vector<LocalNames> dicts;
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

template <class Text>
std::vector<size_t> split_points(const Text& s, int parts) {
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

template <class F>
void run_parallel(int n, int threads, F&& f) {
  threads = std::max(1, std::min(threads, n));
  if (threads == 1) {
    for (int i = 0; i < n; ++i) f(i);
    return;
  }
  std::atomic<int> next{0};
  std::vector<std::thread> th;
  for (int t = 0; t < threads; ++t)
    th.emplace_back([&] {
      for (int i; (i = next.fetch_add(1)) < n;) f(i);
    });
  for (auto& x : th) x.join();
}

// [off, off + n) of `path` into out, `threads` preads in parallel
void read_bytes(const std::string& path, int64_t off, int64_t n, char* out, int threads) {
  const int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) throw std::runtime_error("cannot open " + path);
  const int64_t piece = std::max<int64_t>(int64_t(8) << 20, (n + threads - 1) / std::max(1, threads));
  const int np = (int)((n + piece - 1) / piece);
  std::atomic<bool> bad{false};
  run_parallel(np, threads, [&](int i) {
    int64_t at = i * piece, left = std::min(piece, n - at);
    while (left > 0) {
      const ssize_t r = ::pread(fd, out + at, (size_t)left, off + at);
      if (r <= 0) { bad = true; return; }
      at += r;
      left -= r;
    }
  });
  ::close(fd);
  if (bad) throw std::runtime_error("read failed: " + path);
}

}  // namespace

// ------------------------------------------------------------------ dictionary --

uint64_t hash_bytes(const char* p, size_t n) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ (n * 0xff51afd7ed558ccdull);
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    h = (h ^ v) * 0xbf58476d1ce4e5b9ull;
    h ^= h >> 31;
    p += 8;
    n -= 8;
  }
  if (n) {
    uint64_t v = 0;
    std::memcpy(&v, p, n);
    h = (h ^ v) * 0x94d049bb133111ebull;
    h ^= h >> 29;
  }
  h *= 0xbf58476d1ce4e5b9ull;
  return h ^ (h >> 32);
}

StringDict::StringDict() : shards_(kShards) {}

std::string_view StringDict::Shard::store(std::string_view s) {
  if (s.size() > arena_left) {
    const size_t cap = std::max<size_t>(size_t(1) << 20, s.size());
    arena.emplace_back(new char[cap]);
    arena_at = arena.back().get();
    arena_left = cap;
  }
  std::memcpy(arena_at, s.data(), s.size());
  std::string_view v(arena_at, s.size());
  arena_at += s.size();
  arena_left -= s.size();
  return v;
}

int32_t StringDict::find(std::string_view s) const {
  const uint64_t h = hash_bytes(s.data(), s.size());
  const Shard& sh = shards_[shard_of(h)];
  const int64_t k = sh.index.find(h, s, [&](size_t i) { return sh.keys[i]; });
  return k < 0 ? -1 : (int32_t)sh.val[k];
}

int32_t StringDict::get_or_add(std::string_view s) {
  const uint64_t h = hash_bytes(s.data(), s.size());
  Shard& sh = shards_[shard_of(h)];
  const int64_t k = sh.index.find(h, s, [&](size_t i) { return sh.keys[i]; });
  if (k >= 0) return (int32_t)sh.val[k];
  const int32_t id = (int32_t)names.size();
  names.emplace_back(s);
  sh.keys.push_back(sh.store(s));
  sh.val.push_back(id);
  sh.index.insert(h);
  return id;
}

void StringDict::merge(const std::vector<const LocalNames*>& parts, std::vector<std::vector<int32_t>>& remap,
                       int threads) {
  const int T = (int)parts.size();
  remap.assign(T, {});
  // shard buckets of each part, in local (first-appearance) order
  std::vector<std::vector<std::vector<int32_t>>> bkt(T, std::vector<std::vector<int32_t>>(kShards));
  std::vector<std::vector<int64_t>> res(T);
  std::vector<std::vector<uint8_t>> first(T);
  run_parallel(T, threads, [&](int t) {
    const auto& L = *parts[t];
    res[t].resize(L.names.size());
    first[t].assign(L.names.size(), 0);
    remap[t].resize(L.names.size());
    for (size_t j = 0; j < L.names.size(); ++j) bkt[t][shard_of(L.hash[j])].push_back((int32_t)j);
  });
  // shard-parallel lookup / insert: parts visited in order, so the first part (and first local
  // index) that sees a new name owns it
  std::vector<std::vector<int64_t>> pending(kShards);
  run_parallel(kShards, threads, [&](int s) {
    Shard& sh = shards_[s];
    for (int t = 0; t < T; ++t) {
      const auto& L = *parts[t];
      for (int32_t j : bkt[t][s]) {
        const std::string_view name = L.names[j];
        const uint64_t h = L.hash[j];
        int64_t k = sh.index.find(h, name, [&](size_t i) { return sh.keys[i]; });
        if (k < 0) {
          k = (int64_t)sh.keys.size();
          sh.keys.push_back(sh.store(name));
          sh.val.push_back(~((int64_t)t << 32 | j));
          sh.index.insert(h);
          pending[s].push_back(k);
          first[t][j] = 1;
        }
        res[t][j] = sh.val[k];
      }
    }
  });
  // new ids in (part, local index) order
  std::vector<int64_t> base(T + 1, (int64_t)names.size());
  for (int t = 0; t < T; ++t) {
    int64_t c = 0;
    for (uint8_t f : first[t]) c += f;
    base[t + 1] = base[t] + c;
  }
  if (base[T] > INT32_MAX) throw std::runtime_error("dictionary exceeds 2^31 entries");
  names.resize((size_t)base[T]);
  run_parallel(T, threads, [&](int t) {
    int64_t id = base[t];
    for (size_t j = 0; j < first[t].size(); ++j)
      if (first[t][j]) {
        remap[t][j] = (int32_t)id;
        names[(size_t)id++] = std::string(parts[t]->names[j]);
      }
  });
  auto decode = [&](int64_t v) {
    const int64_t c = ~v;
    return remap[(int)(c >> 32)][(size_t)(c & 0xffffffff)];
  };
  run_parallel(T, threads, [&](int t) {
    for (size_t j = 0; j < res[t].size(); ++j)
      if (!first[t][j]) remap[t][j] = res[t][j] >= 0 ? (int32_t)res[t][j] : decode(res[t][j]);
  });
  run_parallel(kShards, threads, [&](int s) {
    for (int64_t k : pending[s]) shards_[s].val[k] = decode(shards_[s].val[k]);
  });
}

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
  std::vector<int64_t> sizes;
  int64_t total = 0;
  for (const auto& p : paths) {
    std::ifstream f(p, std::ios::binary | std::ios::ate);
    if (!f) throw std::runtime_error("cannot open " + p);
    sizes.push_back((int64_t)f.tellg());
    total += sizes.back();
  }
  int64_t left = total;
  // file i + 1 is read on a thread (a quarter of the threads) while file i is parsed
  auto read_file = [&](size_t i, int th) {
    TextChunk s((size_t)sizes[i]);
    read_bytes(paths[i], 0, sizes[i], s.data(), th);
    return s;
  };
  std::future<TextChunk> next;
  for (size_t i = 0; i < paths.size(); ++i) {
    TextChunk s = next.valid() ? next.get() : read_file(i, threads);
    if (i + 1 < paths.size())
      next = std::async(std::launch::async, read_file, i + 1, std::max(1, threads / 4));
    if (i == 0 && drop_header) {
      const char* e = (const char*)std::memchr(s.data(), '\n', s.size());
      header.assign(s.data(), e ? (size_t)(e - s.data()) : s.size());
      if (!header.empty() && header.back() == '\r') header.pop_back();
    }
    s.ensure_newline();
    chunks.push_back(std::move(s));
    ingest_chunk((uint32_t)(chunks.size() - 1), 1, threads);
    left -= sizes[i];
    // after the first file: room for the remaining files' rows at the observed bytes per row
    if (i == 0 && left > 0 && !rows.empty()) reserve_rows(rows.size() + (size_t)((double)left / bytes_in * rows.size() * 1.02));
  }
}

void TextTable::reserve_rows(size_t n) {
  rows.reserve(n);
  weight.reserve(n);
  for (auto& v : num) v.reserve(n);
  for (auto& v : ids) v.reserve(n);
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
  f.close();
  TextChunk s((size_t)(e - b));
  read_bytes(path, b, e - b, s.data(), threads);
  s.ensure_newline();
  chunks.push_back(std::move(s));
  ingest_chunk((uint32_t)(chunks.size() - 1), 1, threads);
}

void TextTable::append_text(std::string text, int32_t w, int threads) {
  TextChunk s(text.size());
  std::memcpy(s.data(), text.data(), text.size());
  s.ensure_newline();
  chunks.push_back(std::move(s));
  ingest_chunk((uint32_t)(chunks.size() - 1), w, threads);
}

void TextTable::ingest_chunk(uint32_t cid, int32_t w, int threads) {
  const TextChunk& s = chunks[cid];
  if (threads < 1) threads = 1;
  if (s.size() < (1u << 20)) threads = 1;
  auto pts = split_points(s, threads);
  const int T = (int)pts.size() - 1;
  const double bytes_per_row = rows.empty() ? 64.0 : (double)bytes_in / rows.size();
  bytes_in += (int64_t)s.size();
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
    const size_t guess = (size_t)((pts[t + 1] - pts[t]) / bytes_per_row * 1.05) + 16;
    o.off.reserve(guess);
    o.len.reserve(guess);
    for (auto& v : o.num) v.reserve(guess);
    for (auto& v : o.ids) v.reserve(guess);
    std::vector<const char*> fb(ncols), fe(ncols);
    std::vector<double> vals(NN);
    std::vector<uint64_t> dh(ND);
    const char* base = s.data();
    size_t p = pts[t];
    const size_t end = pts[t + 1];
    const char* const lim = base + end;
    const __m256i vcomma = _mm256_set1_epi8(','), vnl = _mm256_set1_epi8('\n');
    while (p < end) {
      const char* lb = base + p;
      // one pass over the line, 32 bytes at a time: its end and its first ncols - 1 commas
      int f = 0;
      auto commas = [&](uint32_t m, const char* at) {
        for (; m; m &= m - 1) {
          const char* c = at + __builtin_ctz(m);
          if (f + 1 < ncols) {
            fe[f] = c;
            fb[f + 1] = c + 1;
          }
          ++f;
        }
      };
      fb[0] = lb;
      const char* q = lb;
      for (;;) {
        if (q + 32 <= lim) {
          const __m256i v = _mm256_loadu_si256((const __m256i*)q);
          const uint32_t mc = (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, vcomma));
          const uint32_t mn = (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, vnl));
          if (mn) {
            const int stop = __builtin_ctz(mn);
            commas(mc & ((1u << stop) - 1u), q);
            q += stop;
            break;
          }
          commas(mc, q);
          q += 32;
        } else {
          for (; q < lim && *q != '\n'; ++q)
            if (*q == ',') commas(1u, q);
          break;
        }
      }
      const char* le = q;
      p = (le - base) + 1;
      if (le > lb && le[-1] == '\r') --le;
      if (drop_header && (size_t)(le - lb) == header.size() && std::memcmp(lb, header.data(), header.size()) == 0) {
        ++o.header;
        continue;
      }
      const char* tb = lb;
      const char* te = le;
      if (!(f == ncols - 1 && le > lb && !is_ws(*lb) && !is_ws(le[-1]) && le[-1] != ',')) {
        // not the plain form (ncols fields, nothing to trim, no trailing empty field): the reference's
        // split / trim / split rules in full
        if (java_split_count(lb, le) != ncols) { ++o.bad_fields; continue; }
        while (tb < te && is_ws(*tb)) ++tb;
        while (te > tb && is_ws(te[-1])) --te;
        while (te > tb && te[-1] == ',') --te;  // trailing empty fields vanish in split + mkString
        if (java_split_count(tb, te) != ncols) { ++o.bad_fields; continue; }
        f = 0;
        fb[0] = tb;
        for (const char* r = tb; r < te; ++r) {
          if (*r == ',') {
            fe[f] = r;
            fb[++f] = r + 1;
          }
        }
      }
      fe[f] = te;
      for (int i = 0; i < ND; ++i) {
        const int c = dict_col_index[i];
        dh[i] = hash_bytes(fb[c], fe[c] - fb[c]);
        o.dicts[dict_col_group[i]].prefetch(dh[i]);
      }
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
        o.ids[i].push_back(o.dicts[dict_col_group[i]].get_or_add(std::string_view(fb[c], fe[c] - fb[c]), dh[i]));
      }
    }
  };
  const auto tp0 = std::chrono::steady_clock::now();
  run_parallel(T, T, work);
  const auto tp1 = std::chrono::steady_clock::now();
  // ordered merge: dictionaries (shard-parallel), then every thread's rows copied to its offset
  std::vector<std::vector<std::vector<int32_t>>> remap(dicts.size());
  for (size_t g = 0; g < dicts.size(); ++g) {
    std::vector<const LocalNames*> parts(T);
    for (int t = 0; t < T; ++t) parts[t] = &outs[t].dicts[g];
    dicts[g].merge(parts, remap[g], threads);
  }
  const auto tp2 = std::chrono::steady_clock::now();
  std::vector<size_t> at(T + 1, rows.size());
  for (int t = 0; t < T; ++t) {
    n_bad_fields += outs[t].bad_fields;
    n_bad_numeric += outs[t].bad_numeric;
    n_header += outs[t].header;
    at[t + 1] = at[t] + outs[t].off.size();
  }
  rows.resize(at[T]);      // ColVec: no fill here; every element is written below, thread-parallel
  weight.resize(at[T]);
  for (int i = 0; i < NN; ++i) num[i].resize(at[T]);
  for (int i = 0; i < ND; ++i) ids[i].resize(at[T]);
  run_parallel(T, threads, [&](int t) {
    LocalOut& o = outs[t];
    const size_t n = o.off.size(), a = at[t];
    for (size_t r = 0; r < n; ++r) rows[a + r] = RowSpan{cid, o.len[r], o.off[r]};
    std::fill(weight.begin() + a, weight.begin() + a + n, w);
    for (int i = 0; i < NN; ++i) std::copy(o.num[i].begin(), o.num[i].end(), num[i].begin() + a);
    for (int i = 0; i < ND; ++i) {
      const auto& rm = remap[dict_col_group[i]][t];
      int32_t* dst = ids[i].data() + a;
      for (size_t r = 0; r < n; ++r) dst[r] = rm[o.ids[i][r]];
    }
    std::vector<std::vector<double>>().swap(o.num);
  });
  if (table_profile()) {
    const auto tp3 = std::chrono::steady_clock::now();
    auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    std::fprintf(stderr, "ingest chunk %u: %zu bytes parse %.1f ms dict %.1f ms rows %.1f ms\n", cid, s.size(),
                 ms(tp0, tp1), ms(tp1, tp2), ms(tp2, tp3));
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
        // the row's values formatted into a per-thread scratch row (room for the widest fast-path text
        // per value), appended once; the rare exact-path value goes through a std::string
        const double* row = k.f64 + (size_t)r * k.width;
        double* back = k.parsed ? k.parsed + (size_t)r * k.width : nullptr;
        const size_t ts = k.text.size();
        thread_local std::vector<char> scratch;
        const size_t need = (size_t)k.width * (40 + ts);
        if (scratch.size() < need) scratch.resize(need);
        char* const s0 = scratch.data();
        char* w = s0;
        for (int j = 0; j < k.width; ++j) {
          if (j) { std::memcpy(w, k.text.data(), ts); w += ts; }
          double* bj = back ? back + j : nullptr;
          if (k.kind == OutCol::kPy2Row) {
            w = put_py2_float(w, row[j], bj);
          } else if (char* e = put_fixed10(w, row[j], bj)) {
            w = e;
          } else {
            out.append(s0, w - s0);
            append_fixed10(out, row[j], bj);
            w = s0;
          }
        }
        out.append(s0, w - s0);
        break;
      }
    }
  }
  out += '\n';
}

// values [j0, j1) of row r of a row column (kPy2Row / kFixedRow), each after its in-row separator
// (none before value 0) -- format_row's text for that range
static void format_row_values(std::string& out, const OutCol& k, int64_t r, int64_t j0, int64_t j1) {
  const double* row = k.f64 + (size_t)r * k.width;
  double* back = k.parsed ? k.parsed + (size_t)r * k.width : nullptr;
  char b[64];
  for (int64_t j = j0; j < j1; ++j) {
    if (j) out += k.text;
    double* bj = back ? back + j : nullptr;
    if (k.kind == OutCol::kPy2Row) {
      out.append(b, put_py2_float(b, row[j], bj) - b);
    } else if (char* e = put_fixed10(b, row[j], bj)) {
      out.append(b, e - b);
    } else {
      append_fixed10(out, row[j], bj);
    }
  }
}

// Few very wide rows (a K x V .beta file: 100 rows of 4.5 M values at config 5): one row per thread
// left most threads idle in the last batches; here each row's values are cut into one segment per
// thread, and the row is written as its scalar columns, then the segments in order.
// A formatting exception (e.g. bad_alloc on a multi-GB row) must not leave a writer thread joinable:
// the std::thread destructor would call std::terminate instead of letting the caller report the error.
struct JoinGuard {
  std::thread& t;
  ~JoinGuard() {
    if (t.joinable()) t.join();
  }
};

static int64_t write_wide_rows(FILE* f, const int64_t* order, int64_t n, const std::vector<OutCol>& cols,
                               const std::string& sep, int threads, int& werr) {
  const OutCol& k = cols.back();
  std::vector<OutCol> head(cols.begin(), cols.end() - 1);
  // two buffer sets: a writer thread writes row i while the threads format row i + 1
  std::vector<std::string> seg[2] = {std::vector<std::string>((size_t)threads),
                                     std::vector<std::string>((size_t)threads)};
  std::string pre[2];
  int64_t written = 0;
  std::thread writer;
  auto flush = [&](int set) {
    if (!pre[set].empty() && std::fwrite(pre[set].data(), 1, pre[set].size(), f) != pre[set].size())
      werr = errno ? errno : EIO;
    written += (int64_t)pre[set].size();
    for (auto& x : seg[set]) {
      if (werr) return;
      if (!x.empty() && std::fwrite(x.data(), 1, x.size(), f) != x.size()) werr = errno ? errno : EIO;
      written += (int64_t)x.size();
    }
  };
  JoinGuard guard{writer};
  int set = 0;
  for (int64_t i = 0; i < n; ++i, set ^= 1) {
    const int64_t r = order ? order[i] : i;
    pre[set].clear();
    if (!head.empty()) {
      format_row(pre[set], r, head, sep);
      pre[set].pop_back();                     // format_row's newline
      pre[set] += sep;
    }
    const int64_t W = k.width;
    std::vector<std::string>& cur = seg[set];
    run_parallel(threads, threads, [&](int t) {
      std::string s;
      s.swap(cur[(size_t)t]);
      s.clear();
      const int64_t j0 = W * t / threads, j1 = W * (t + 1) / threads;
      s.reserve((size_t)(j1 - j0) * 18);
      format_row_values(s, k, r, j0, j1);
      s.swap(cur[(size_t)t]);
    });
    cur.back() += '\n';
    if (writer.joinable()) writer.join();
    if (werr) break;
    writer = std::thread(flush, set);
  }
  if (writer.joinable()) writer.join();
  return written;
}

int64_t write_rows(const std::string& path, const int64_t* order, int64_t n, const std::vector<OutCol>& cols,
                   const std::string& sep, bool append, int threads) {
  FILE* f = std::fopen(path.c_str(), append ? "ab" : "wb");
  if (!f) throw std::runtime_error("cannot open for writing: " + path + ": " + std::strerror(errno));
  if (threads < 1) threads = 1;
  if (!cols.empty() && (cols.back().kind == OutCol::kPy2Row || cols.back().kind == OutCol::kFixedRow) &&
      cols.back().width >= (1 << 16) && n < 2 * (int64_t)threads && threads > 1) {
    bool scalar_head = true;
    for (size_t c = 0; c + 1 < cols.size(); ++c)
      scalar_head = scalar_head && cols[c].kind != OutCol::kPy2Row && cols[c].kind != OutCol::kFixedRow;
    if (scalar_head) {
      int werr = 0;
      int64_t written = 0;
      try {
        written = write_wide_rows(f, order, n, cols, sep, threads, werr);
      } catch (...) {
        std::fclose(f);
        throw;
      }
      if (werr) {
        std::fclose(f);
        throw std::runtime_error("short write: " + path + ": " + std::strerror(werr));
      }
      if (std::fclose(f) != 0) throw std::runtime_error("close failed: " + path);
      return written;
    }
  }
  // Rows per thread block: ~2^18 cells of work per block, so wide rows (a K x V
  // .beta file has K rows of V values) still spread over every thread.
  int64_t cells = 0;
  for (const OutCol& c : cols) cells += (c.kind == OutCol::kPy2Row || c.kind == OutCol::kFixedRow) ? c.width : 1;
  const int64_t block = std::max<int64_t>(1, (int64_t(1) << 18) / std::max<int64_t>(1, cells));
  // Two buffer sets: one writer thread writes batch b while the others format batch b + 1 (writes
  // to one file serialise in the kernel anyway -- parallel pwrite measured slower).
  int64_t written = 0;
  std::vector<std::string> bufs[2] = {std::vector<std::string>(threads), std::vector<std::string>(threads)};
  std::thread writer;
  int werr = 0;
  auto flush = [&](int set) {
    for (auto& s : bufs[set]) {
      if (werr) return;
      if (!s.empty() && std::fwrite(s.data(), 1, s.size(), f) != s.size()) werr = errno ? errno : EIO;
      written += (int64_t)s.size();
    }
  };
  struct CloseOnThrow {   // declared before the join guard: the writer is joined first, then f closed
    FILE* f;
    bool armed = true;
    ~CloseOnThrow() {
      if (armed) std::fclose(f);
    }
  } closer{f};
  JoinGuard guard{writer};
  int set = 0;
  double t_fmt = 0, t_wait = 0;
  const auto t_all = std::chrono::steady_clock::now();
  auto since = [](std::chrono::steady_clock::time_point a) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
  };
  for (int64_t b0 = 0; b0 < n; b0 += block * threads, set ^= 1) {
    const auto tb = std::chrono::steady_clock::now();
    std::vector<std::string>& cur = bufs[set];
    const int nt = (int)std::min<int64_t>(threads, (n - b0 + block - 1) / block);
    run_parallel(threads, nt, [&](int t) {
      std::string s;                    // a local, not cur[t]: adjacent string headers would share
      s.swap(cur[t]);                   // cache lines and every append would bounce them
      s.clear();
      const int64_t lo = b0 + t * block, hi = std::min(n, lo + block);
      if (hi > lo) s.reserve((size_t)(hi - lo) * (size_t)cells * 18);   // no regrowth copies (30 ns per cell)
      for (int64_t i = lo; i < hi; ++i) format_row(s, order ? order[i] : i, cols, sep);
      s.swap(cur[t]);
    });
    t_fmt += since(tb);
    const auto tw = std::chrono::steady_clock::now();
    if (writer.joinable()) writer.join();
    t_wait += since(tw);
    if (werr) break;
    writer = std::thread(flush, set);
  }
  if (writer.joinable()) writer.join();
  closer.armed = false;
  if (table_profile())
    std::fprintf(stderr, "write_rows %s: %lld rows, %d threads, format %.1f ms, writer wait %.1f ms, total %.1f ms\n",
                 path.c_str(), (long long)n, threads, t_fmt, t_wait, since(t_all));
  if (werr) {
    std::fclose(f);
    throw std::runtime_error("short write: " + path + ": " + std::strerror(werr));
  }
  if (std::fclose(f) != 0) throw std::runtime_error("close failed: " + path);
  return written;
}

std::vector<std::string> format_rows(const int64_t* order, int64_t n, const std::vector<OutCol>& cols,
                                     const std::string& sep, int threads, std::vector<int64_t>* row_ends) {
  if (threads < 1) threads = 1;
  int64_t cells = 0;
  for (const OutCol& c : cols) cells += (c.kind == OutCol::kPy2Row || c.kind == OutCol::kFixedRow) ? c.width : 1;
  const int64_t block = std::max<int64_t>(1, (int64_t(1) << 16) / std::max<int64_t>(1, cells));
  const int64_t nb = (n + block - 1) / block;
  std::vector<std::string> out(nb);
  if (row_ends) row_ends->assign(n, 0);
  if (nb > INT32_MAX) throw std::invalid_argument("format_rows: too many rows");
  run_parallel((int)nb, threads, [&](int b) {
    std::string s;
    const int64_t lo = b * block, hi = std::min(n, lo + block);
    if (hi > lo) s.reserve((size_t)(hi - lo) * (size_t)cells * 18);   // no regrowth copies (30 ns per cell)
    for (int64_t i = lo; i < hi; ++i) {
      format_row(s, order ? order[i] : i, cols, sep);
      if (row_ends) (*row_ends)[i] = (int64_t)s.size();        // block-local for now
    }
    out[b].swap(s);
  });
  if (row_ends) {
    int64_t base = 0;
    for (int64_t b = 0; b < nb; ++b) {
      const int64_t lo = b * block, hi = std::min(n, lo + block);
      for (int64_t i = lo; i < hi; ++i) (*row_ends)[i] += base;
      base += (int64_t)out[b].size();
    }
  }
  return out;
}

}  // namespace onin
