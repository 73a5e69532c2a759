// Input parser and result writer (root rank only — PDF p.5: one process reads and writes).
//
// Reference: fscanf-based reading (main.c:76-108) with an OpenMP loop that calls fscanf on the
// shared stdin from many threads (bug B2: nondeterministic record order) and unbounded %s reads
// (bug B12). Output: printf per row (main.c:199-211).
//
// Here: the whole stream is read in bulk, the header is tokenised sequentially, and the record area
// is tokenised + upper-cased + encoded by a two-pass OpenMP scan (count, prefix-sum, fill), so the
// order is always input order and the thread count only changes speed.
#pragma once

#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "moc/common.hpp"
#include "moc/problem.hpp"

namespace moc {

struct ParseOptions {
  bool strict_limits = false;  // enforce PDF limits: |Seq1| <= 3000, |Seq2| <= 2000
  int64_t max_l1 = 0;          // 0 = unlimited
  int64_t max_l2 = 0;          // 0 = unlimited
};

// Reads the whole stream into memory (bulk fread; no per-token stdio).
uvector<char> read_stream(FILE* f);

// Two-phase parser of an in-memory input: the constructor reads the header and counts the records and
// letters (parallel pass 1); fill() encodes them into caller-provided buffers (parallel pass 2) — e.g.
// straight into a node-shared window, with no intermediate copy. `data` must outlive fill().
class BulkParser {
 public:
  BulkParser(const char* data, size_t len, const ParseOptions& opt = {});
  const Weights& weights() const { return weights_; }
  const std::vector<uint8_t>& seq1() const { return seq1_; }
  int64_t count() const { return n_; }
  int64_t total_chars() const { return total_chars_; }
  // codes[0..total_chars()), offsets[0..count()] (offsets[0] = 0); throws on non-letters / limits.
  void fill(uint8_t* codes, int64_t* offsets) const;
  // n * (L1 - avg + 1) * avg from the mean record length (before fill; for engine selection).
  int64_t cells_estimate() const;

 private:
  Weights weights_{};
  std::vector<uint8_t> seq1_;
  int64_t n_ = 0, total_chars_ = 0, l2_cap_ = 0;
  const char* area_ = nullptr;
  size_t area_len_ = 0;
  int nthreads_ = 1;
  std::vector<size_t> start_;
  std::vector<int64_t> tok_count_, char_count_;
};

// Parses "W1 W2 W3 W4 / Seq1 / N / Seq2 x N" (PDF p.5-6). Whitespace of any kind (incl. CRLF)
// separates tokens, exactly like fscanf %d/%s. Throws moc::Error with a precise message.
Problem parse_problem(const char* data, size_t len, const ParseOptions& opt = {});

// Incremental reader for the streaming mode (`final --batch-records=B`): parses the
// header up front, then hands out the records in bounded batches, so host memory is O(batch) instead of
// O(input). Same token rules and error messages as parse_problem. skip() consumes records without
// encoding them (`--skip-records`, resuming a partially printed run).
class StreamReader {
 public:
  explicit StreamReader(FILE* f, const ParseOptions& opt = {}, size_t block_bytes = size_t{32} << 20);
  const Weights& weights() const { return weights_; }
  const std::vector<uint8_t>& seq1() const { return seq1_; }
  int64_t count() const { return count_; }         // number_of_sequences from the header
  int64_t next_index() const { return next_; }     // index of the next record to be read
  int64_t skip(int64_t records);                   // returns the number actually skipped
  // Parses up to max_records (and, after the first record, at most max_chars letters) of the following
  // records into `out` (offsets rebased to 0). Returns the number of records (0 once all are read).
  int64_t next_batch(int64_t max_records, RecordBatch& out, int64_t max_chars = INT64_MAX);

 private:
  bool token(const char*& b, const char*& e);  // next token, refilling the buffer as needed
  FILE* f_;
  ParseOptions opt_;
  std::vector<char> buf_;
  size_t pos_ = 0, len_ = 0;
  bool eof_ = false;
  Weights weights_{};
  std::vector<uint8_t> seq1_;
  int64_t count_ = 0, next_ = 0, l2_cap_ = 0;
};

// Formats "#i: score: S, n: N, k: K\n" rows (main.c:204) for results[0..n), numbering from
// first_index, in parallel, then writes them with one fwrite.
void write_results(FILE* f, const Result* results, int64_t n, int64_t first_index = 0);
std::string format_results(const Result* results, int64_t n, int64_t first_index = 0);

}  // namespace moc
