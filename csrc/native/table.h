// Columnar text table: multithreaded CSV ingest with the reference's
// line/field semantics, plus the multithreaded formatted writer.
//
// Reference semantics reproduced (flow_pre_lda.scala:22-26,249-250,268-270;
// flow_post_lda.scala:128-137):
//  * sc.textFile line splitting (\n, optional \r stripped);
//  * removeHeader drops EVERY line equal to the first line of the input;
//  * Java String.split(","): trailing empty fields are dropped, a row is kept
//    only if it then has exactly `ncols` fields (checked on the raw line and on
//    the trimmed line that is actually split);
//  * numeric fields parse with java.lang.Double.parseDouble rules; a field that
//    would throw NumberFormatException drops the row (counted) instead of
//    failing the whole job;
//  * the row text kept for output is the trimmed line without its trailing
//    empty fields, i.e. exactly `row.mkString(",")` of the split row.
// String columns are dictionary-encoded at ingest: ids are assigned in
// first-appearance order (row-major, columns of one dictionary group in column
// order), computed per thread and merged in input order, so the result does
// not depend on the thread count.
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <string_view>
#include <type_traits>
#include <unordered_map>
#include <utility>
#include <vector>

namespace onin {

// std::allocator whose value-initialising construct() default-initialises instead: resize() of a
// column leaves the new elements untouched, so the rows of an ingested chunk are first written (and
// their pages first touched) by the threads that copy them in, not by a serial zero fill
template <class T>
struct DefaultInit : std::allocator<T> {
  template <class U>
  struct rebind { using other = DefaultInit<U>; };
  DefaultInit() = default;
  template <class U>
  DefaultInit(const DefaultInit<U>&) noexcept {}
  template <class U>
  void construct(U* p) noexcept(std::is_nothrow_default_constructible<U>::value) { ::new ((void*)p) U; }
  template <class U, class... A>
  void construct(U* p, A&&... a) { ::new ((void*)p) U(std::forward<A>(a)...); }
};
template <class T>
using ColVec = std::vector<T, DefaultInit<T>>;

struct RowSpan {
  uint32_t chunk;
  uint32_t len;
  uint64_t off;
};

// 64-bit hash of a byte string (8-byte multiply-xorshift rounds).
uint64_t hash_bytes(const char* p, size_t n);

// Open-addressing index over an external key list: slot -> key id + 1, linear probing on the
// precomputed hash, grown at half load.  Keys are compared through `key(id)`.
struct FlatIndex {
  std::vector<uint32_t> slot;
  std::vector<uint64_t> hash;   // per key id
  size_t mask = 0;
  template <class Key>
  int64_t find(uint64_t h, std::string_view s, const Key& key) const {
    if (slot.empty()) return -1;
    for (size_t i = h & mask;; i = (i + 1) & mask) {
      const uint32_t v = slot[i];
      if (v == 0) return -1;
      if (hash[v - 1] == h && key(v - 1) == s) return v - 1;
    }
  }
  void insert(uint64_t h) {      // the next key id (= hash.size()) with hash h
    hash.push_back(h);
    if (2 * hash.size() > slot.size()) rehash(std::max<size_t>(64, 4 * hash.size()));
    else place(h, (uint32_t)hash.size());
  }

 private:
  void place(uint64_t h, uint32_t v) {
    size_t i = h & mask;
    while (slot[i] != 0) i = (i + 1) & mask;
    slot[i] = v;
  }
  void rehash(size_t n) {
    size_t cap = 64;
    while (cap < n) cap <<= 1;
    slot.assign(cap, 0);
    mask = cap - 1;
    for (size_t k = 0; k < hash.size(); ++k) place(hash[k], (uint32_t)(k + 1));
  }
};

// One thread's first-appearance name list (string_views into the text being ingested).  The index
// holds keys of up to 16 bytes (every IPv4 address) inline in its slots, so a lookup touches one slot
// line instead of slot -> hash -> name -> text (the ingest's hottest path: two lookups per flow row);
// a longer key's slot holds its hash and is compared through `names`.
struct LocalNames {
  std::vector<std::string_view> names;
  std::vector<uint64_t> hash;    // per id (the merge's shard key)
  struct Slot {
    uint64_t k0, k1;             // key bytes (<= 16) zero-padded, or (hash, 0) for a longer key
    uint32_t id1;                // id + 1; 0 = empty
    uint32_t len;
  };
  std::vector<Slot> slot;
  size_t mask = 0;

  int32_t get_or_add(std::string_view s) { return get_or_add(s, hash_bytes(s.data(), s.size())); }
  // the slot line of hash h into cache ahead of get_or_add(s, h) (the ingest issues it before parsing
  // the row's numbers)
  void prefetch(uint64_t h) const {
    if (!slot.empty()) __builtin_prefetch(&slot[h & mask]);
  }
  int32_t get_or_add(std::string_view s, uint64_t h) {
    const size_t n = s.size();
    uint64_t k0 = 0, k1 = 0;
    if (n <= 16) {
      std::memcpy(&k0, s.data(), n < 8 ? n : 8);
      if (n > 8) std::memcpy(&k1, s.data() + 8, n - 8);
    } else {
      k0 = h;
    }
    if (2 * (names.size() + 1) > slot.size()) grow();
    for (size_t i = h & mask;; i = (i + 1) & mask) {
      Slot& x = slot[i];
      if (x.id1 == 0) {
        x = Slot{k0, k1, (uint32_t)names.size() + 1, (uint32_t)n};
        names.push_back(s);
        hash.push_back(h);
        return (int32_t)(names.size() - 1);
      }
      if (x.len == n && x.k0 == k0 && x.k1 == k1 && (n <= 16 || names[x.id1 - 1] == s)) return (int32_t)(x.id1 - 1);
    }
  }

 private:
  void grow() {
    std::vector<Slot> old;
    old.swap(slot);
    slot.assign(std::max<size_t>(64, 2 * old.size()), Slot{0, 0, 0, 0});
    mask = slot.size() - 1;
    for (const Slot& x : old)
      if (x.id1) {
        size_t i = hash[x.id1 - 1] & mask;
        while (slot[i].id1) i = (i + 1) & mask;
        slot[i] = x;
      }
  }
};

// Global dictionary: ids in first-appearance order.  The index is split into hash shards so
// merging T threads' first-appearance lists runs in parallel (merge(): shard-parallel lookup /
// insert, then a prefix over threads assigns the new ids in (thread, local index) order -- the
// order a serial pass over the rows would have produced).
class StringDict {
 public:
  std::vector<std::string> names;
  static constexpr int kShards = 64;
  StringDict();
  int32_t get_or_add(std::string_view s);
  int32_t find(std::string_view s) const;
  // remap[t][j] = global id of parts[t]->names[j]
  void merge(const std::vector<const LocalNames*>& parts, std::vector<std::vector<int32_t>>& remap, int threads);

 private:
  struct Shard {
    FlatIndex index;
    std::vector<std::string_view> keys;       // into arena
    std::vector<int64_t> val;                 // global id, or ~(t << 32 | j) while a merge is pending
    std::vector<std::unique_ptr<char[]>> arena;
    size_t arena_left = 0;
    char* arena_at = nullptr;
    std::string_view store(std::string_view s);
  };
  std::vector<Shard> shards_;
  static int shard_of(uint64_t h) { return (int)((h >> 40) % kShards); }
};

// Owned input text (not zero-filled: read straight into the buffer).
struct TextChunk {
  std::unique_ptr<char[]> buf;
  size_t n = 0;
  explicit TextChunk(size_t size) : buf(new char[size + 1]), n(size) {}
  const char* data() const { return buf.get(); }
  char* data() { return buf.get(); }
  size_t size() const { return n; }
  char operator[](size_t i) const { return buf[i]; }
  void ensure_newline() { if (n == 0 || buf[n - 1] != '\n') buf[n++] = '\n'; }   // capacity is size + 1
};

class TextTable {
 public:
  int ncols = 0;
  std::vector<int> numeric_cols;                 // columns parsed as double
  std::vector<std::vector<int>> dict_groups;     // columns sharing one dictionary
  std::vector<TextChunk> chunks;                 // owned text
  int64_t bytes_in = 0;                          // text ingested so far (row-count estimates)
  ColVec<RowSpan> rows;
  ColVec<int32_t> weight;                        // per-row multiplicity (feedback rows: DUPFACTOR)
  std::vector<ColVec<double>> num;               // [numeric_cols.size()][rows]
  std::vector<ColVec<int32_t>> ids;              // per dict column (flattened over groups) [rows]
  std::vector<int> dict_col_group;               // dict column slot -> group
  std::vector<int> dict_col_index;               // dict column slot -> column index
  std::vector<StringDict> dicts;                 // one per group
  std::string header;
  bool drop_header = false;
  int64_t n_bad_fields = 0, n_bad_numeric = 0, n_header = 0;

  TextTable(int ncols, std::vector<int> numeric_cols, std::vector<std::vector<int>> dict_groups);
  void load_files(const std::vector<std::string>& paths, bool drop_header, int threads);
  // Row-sharded ingest: the lines of `path` whose first byte lies in [begin, end) (a line belongs to the
  // range holding its first byte, so N ranges of one file partition its lines exactly).  `hdr` is the
  // header line of the job's first file (the reference's filter(_ != header) rule, applied to every line).
  void load_range(const std::string& path, int64_t begin, int64_t end, const std::string& hdr, bool drop_header,
                  int threads);
  void append_text(std::string text, int32_t w, int threads);  // newline-separated lines
  void reserve_rows(size_t n);
  std::string_view row_text(size_t i) const {
    const RowSpan& r = rows[i];
    return std::string_view(chunks[r.chunk].data() + r.off, r.len);
  }
  int numeric_slot(int col) const;
  int dict_slot(int col) const;

 private:
  void ingest_chunk(uint32_t chunk_id, int32_t w, int threads);
};

// One output column of a formatted writer.
struct OutCol {
  enum Kind { kTable, kJava, kInt, kDict, kPair, kConst, kPy2Row, kFixedRow } kind;
  const TextTable* table = nullptr;
  const int64_t* rowmap = nullptr;      // kTable: output row r prints table row rowmap[r] (or r)
  const double* f64 = nullptr;          // kJava / kPy2Row / kFixedRow (row-major [n][width])
  const int64_t* i64 = nullptr;         // kInt
  const int32_t* idx = nullptr;         // kDict / kPair (a)
  const int32_t* idx2 = nullptr;        // kPair (b)
  const std::vector<std::string>* names = nullptr;
  std::string text;                     // kConst, or the separator inside a row for kPy2Row/kFixedRow
  int width = 0;                        // kPy2Row / kFixedRow
  double* parsed = nullptr;             // kPy2Row / kFixedRow, optional [n][width]: each printed value read
                                        // back (strtod of its own text), so a reader's view of the file
                                        // comes with the write instead of a second format pass
};

// Writes one line per entry of `order` (row indices), columns joined by sep.
// Returns bytes written.  Formatting runs on `threads` threads; output order is
// exactly `order`.
int64_t write_rows(const std::string& path, const int64_t* order, int64_t n, const std::vector<OutCol>& cols,
                   const std::string& sep, bool append, int threads);

// In-memory variant (the row-sharded writers: every rank formats its own rows, then writes them at
// its byte offset of the shared file): the text of the rows in `order` as consecutive chunks, and
// optionally the end offset (over the concatenated chunks) of every row.
std::vector<std::string> format_rows(const int64_t* order, int64_t n, const std::vector<OutCol>& cols,
                                     const std::string& sep, int threads, std::vector<int64_t>* row_ends);

}  // namespace onin
