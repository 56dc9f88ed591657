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
#include <cstdint>
#include <memory>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

namespace onin {

struct RowSpan {
  uint32_t chunk;
  uint32_t len;
  uint64_t off;
};

class StringDict {
 public:
  std::vector<std::string> names;
  std::unordered_map<std::string, int32_t> index;
  int32_t get_or_add(std::string_view s) {
    auto it = index.find(std::string(s));
    if (it != index.end()) return it->second;
    int32_t id = (int32_t)names.size();
    names.emplace_back(s);
    index.emplace(names.back(), id);
    return id;
  }
  int32_t find(std::string_view s) const {
    auto it = index.find(std::string(s));
    return it == index.end() ? -1 : it->second;
  }
};

class TextTable {
 public:
  int ncols = 0;
  std::vector<int> numeric_cols;                 // columns parsed as double
  std::vector<std::vector<int>> dict_groups;     // columns sharing one dictionary
  std::vector<std::string> chunks;               // owned text
  std::vector<RowSpan> rows;
  std::vector<int32_t> weight;                   // per-row multiplicity (feedback rows: DUPFACTOR)
  std::vector<std::vector<double>> num;          // [numeric_cols.size()][rows]
  std::vector<std::vector<int32_t>> ids;         // per dict column (flattened over groups) [rows]
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

}  // namespace onin
