#include "corpus_io.h"

#include <algorithm>
#include <charconv>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace onin {

namespace {

inline void put_int(std::string& s, int64_t v) {
  char b[24];
  auto r = std::to_chars(b, b + sizeof(b), v);
  s.append(b, r.ptr - b);
}

// printf "%0<W>d" for v >= 0
inline void put_int_pad(std::string& s, int64_t v, int width) {
  char b[24];
  auto r = std::to_chars(b, b + sizeof(b), v);
  for (int64_t k = r.ptr - b; k < width; ++k) s += '0';
  s.append(b, r.ptr - b);
}

template <typename F>
void parallel_for(int threads, F&& f) {
  if (threads <= 1) { f(0); return; }
  std::vector<std::thread> th;
  for (int t = 1; t < threads; ++t) th.emplace_back(f, t);
  f(0);
  for (auto& x : th) x.join();
}

}  // namespace

namespace {

// blocks of ~2^18 entries so heavy-tailed document lengths still balance
std::vector<int64_t> corpus_blocks(const int64_t* ptr, int64_t D) {
  const int64_t nnz = ptr[D];
  const int64_t per = std::max<int64_t>(1, nnz / std::max<int64_t>(1, (nnz >> 18)));
  std::vector<int64_t> cuts{0};
  for (int64_t d = 0; d < D;) {
    const int64_t target = ptr[d] + per;
    int64_t e = std::upper_bound(ptr + d, ptr + D + 1, target) - ptr;
    e = std::min<int64_t>(std::max<int64_t>(e - 1, d + 1), D);
    cuts.push_back(e);
    d = e;
  }
  return cuts;
}

void format_docs(std::string& s, const int64_t* ptr, int64_t d0, int64_t d1, const int32_t* w, const int64_t* c,
                 bool assignments) {
  for (int64_t d = d0; d < d1; ++d) {
    if (assignments) {
      put_int_pad(s, ptr[d + 1] - ptr[d], 3);
      for (int64_t i = ptr[d]; i < ptr[d + 1]; ++i) {
        s += ' ';
        put_int_pad(s, w[i], 4);
        s += ':';
        put_int_pad(s, c[i], 2);
      }
    } else {
      put_int(s, ptr[d + 1] - ptr[d]);
      for (int64_t i = ptr[d]; i < ptr[d + 1]; ++i) {
        s += ' ';
        put_int(s, w[i]);
        s += ':';
        put_int(s, c[i]);
      }
    }
    s += '\n';
  }
}

}  // namespace

int64_t write_corpus_text(const std::string& path, const int64_t* ptr, int64_t D, const int32_t* w,
                          const int64_t* c, int threads, bool assignments) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) throw std::runtime_error("cannot open for writing: " + path);
  threads = std::max(1, threads);
  const std::vector<int64_t> cuts = corpus_blocks(ptr, D);
  const int64_t nb = (int64_t)cuts.size() - 1;
  int64_t written = 0;
  std::vector<std::string> bufs(threads);
  for (int64_t b0 = 0; b0 < nb; b0 += threads) {
    parallel_for(std::min<int64_t>(threads, nb - b0), [&](int t) {
      std::string& s = bufs[t];
      s.clear();
      format_docs(s, ptr, cuts[b0 + t], cuts[b0 + t + 1], w, c, assignments);
    });
    for (int64_t t = 0; t < std::min<int64_t>(threads, nb - b0); ++t) {
      const std::string& s = bufs[t];
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

std::vector<std::string> format_corpus_text(const int64_t* ptr, int64_t D, const int32_t* w, const int64_t* c,
                                            int threads, bool assignments) {
  threads = std::max(1, threads);
  const std::vector<int64_t> cuts = corpus_blocks(ptr, D);
  const int64_t nb = (int64_t)cuts.size() - 1;
  std::vector<std::string> out(std::max<int64_t>(nb, 0));
  for (int64_t b0 = 0; b0 < nb; b0 += threads)
    parallel_for(std::min<int64_t>(threads, nb - b0),
                 [&](int t) { format_docs(out[b0 + t], ptr, cuts[b0 + t], cuts[b0 + t + 1], w, c, assignments); });
  return out;
}

TextCorpus read_corpus_text(const std::string& path, int threads) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("cannot open: " + path);
  std::fseek(f, 0, SEEK_END);
  const long sz = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  std::string buf((size_t)std::max(0L, sz), '\0');
  if (sz > 0 && std::fread(&buf[0], 1, (size_t)sz, f) != (size_t)sz) {
    std::fclose(f);
    throw std::runtime_error("short read: " + path);
  }
  std::fclose(f);
  threads = std::max(1, std::min<int>(threads, (int)(buf.size() >> 16) + 1));
  // chunk boundaries at line starts
  std::vector<size_t> start(threads + 1, buf.size());
  start[0] = 0;
  for (int t = 1; t < threads; ++t) {
    size_t p = buf.size() * t / threads;
    while (p < buf.size() && buf[p - 1] != '\n') ++p;
    start[t] = std::max(p, start[t - 1]);
  }
  struct Part {
    std::vector<int64_t> len;
    std::vector<int32_t> w;
    std::vector<int64_t> c;
    std::string err;
  };
  std::vector<Part> parts(threads);
  parallel_for(threads, [&](int t) {
    Part& P = parts[t];
    const char* p = buf.data() + start[t];
    const char* end = buf.data() + start[t + 1];
    auto skip_ws = [&](const char*& q, const char* e) {
      while (q < e && (*q == ' ' || *q == '\t' || *q == '\r')) ++q;
    };
    while (p < end) {
      const char* eol = static_cast<const char*>(std::memchr(p, '\n', end - p));
      if (!eol) eol = end;
      const char* q = p;
      skip_ws(q, eol);
      if (q < eol) {
        int64_t n = 0;
        auto r = std::from_chars(q, eol, n);
        if (r.ec != std::errc() || n < 0) { P.err = "bad entry count"; return; }
        q = r.ptr;
        int64_t got = 0;
        for (;;) {
          skip_ws(q, eol);
          if (q >= eol) break;
          int32_t wi = 0;
          int64_t ci = 0;
          r = std::from_chars(q, eol, wi);
          if (r.ec != std::errc() || r.ptr >= eol || *r.ptr != ':') { P.err = "bad w:c pair"; return; }
          r = std::from_chars(r.ptr + 1, eol, ci);
          if (r.ec != std::errc()) { P.err = "bad w:c pair"; return; }
          q = r.ptr;
          P.w.push_back(wi);
          P.c.push_back(ci);
          ++got;
        }
        if (got != n) {
          P.err = "model.dat line declares " + std::to_string(n) + " entries, has " + std::to_string(got);
          return;
        }
        P.len.push_back(n);
      }
      p = eol + 1;
    }
  });
  TextCorpus out;
  size_t D = 0, nnz = 0;
  for (auto& P : parts) {
    if (!P.err.empty()) throw std::runtime_error(P.err);
    D += P.len.size();
    nnz += P.w.size();
  }
  out.doc_ptr.reserve(D + 1);
  out.doc_ptr.push_back(0);
  out.words.reserve(nnz);
  out.counts.reserve(nnz);
  for (auto& P : parts) {
    for (int64_t n : P.len) out.doc_ptr.push_back(out.doc_ptr.back() + n);
    out.words.insert(out.words.end(), P.w.begin(), P.w.end());
    out.counts.insert(out.counts.end(), P.c.begin(), P.c.end());
  }
  return out;
}

}  // namespace onin
