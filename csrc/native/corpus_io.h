// lda-c corpus text format ("N w:c w:c ...", one document per line; lda_pre.py:89-94,
// read by oni-lda-c's read_data) — multithreaded writer and reader.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace onin {

struct TextCorpus {
  std::vector<int64_t> doc_ptr;  // D + 1
  std::vector<int32_t> words;
  std::vector<int64_t> counts;
};

// Writes D lines; returns the number of bytes written.  assignments = false: model.dat
// ("%d" length, " %d:%d" word:count); true: lda-c's word-assignments.dat ("%03d" length,
// " %04d:%02d" word:topic, write_word_assignment).
int64_t write_corpus_text(const std::string& path, const int64_t* doc_ptr, int64_t D, const int32_t* words,
                          const int64_t* counts, int threads, bool assignments = false);

// The same text in memory (the row-sharded writers), as consecutive chunks.
std::vector<std::string> format_corpus_text(const int64_t* doc_ptr, int64_t D, const int32_t* words,
                                            const int64_t* counts, int threads, bool assignments = false);

// Parses a model.dat file.  Blank lines are skipped; a line whose declared
// entry count differs from its w:c pairs throws std::runtime_error.
TextCorpus read_corpus_text(const std::string& path, int threads);

}  // namespace onin
