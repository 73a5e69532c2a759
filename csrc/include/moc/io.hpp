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

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "moc/common.hpp"
#include "moc/partition.hpp"
#include "moc/problem.hpp"
#include "moc/wire.hpp"

namespace moc {

struct ParseOptions {
  bool strict_limits = false;  // enforce PDF limits: |Seq1| <= 3000, |Seq2| <= 2000
  int64_t max_l1 = 0;          // 0 = unlimited
  int64_t max_l2 = 0;          // 0 = unlimited
};

// Reads the whole stream into memory (bulk fread; no per-token stdio).
uvector<char> read_stream(FILE* f);
// Bytes left in a regular-file stream (from its position), or -1 for pipes / terminals / empty files.
int64_t regular_input_bytes(FILE* f);
// Reads up to `want` bytes of a regular file into dst (large reads: parallel preads); returns the count.
size_t read_regular_into(FILE* f, char* dst, size_t want);

// Pieces of the record area that hold a contiguous run of records (a rank's slice): piece q covers
// bytes [byte_begin, byte_end) of the area; its first token is record `tok` and its first letter is letter
// `chr` of the slice (both relative to the slice's first record / letter).
struct AreaPiece {
  int64_t byte_begin = 0, byte_end = 0, tok = 0, chr = 0;
};
struct AreaSlice {
  int64_t first_record = 0, records = 0, letters = 0;
  std::vector<AreaPiece> pieces;
};
// What pass 2 saw in a slice: the length range, and the first offending records (global indices, -1: none).
struct FillReport {
  int64_t min_len = INT64_MAX, max_len = 0;
  int64_t bad_record = -1;                 // first record holding a non-letter
  int64_t long_record = -1, long_len = 0;  // first record over the Seq2 length limit
  int64_t cells = 0;                       // search cells of the slice (record_cells over its records)
};

// Two-phase parser of an in-memory input. The constructor reads the header; pass 1 counts the tokens and
// letters of the record area in chunks (cut at whitespace); pass 2 encodes any contiguous slice of the
// records into caller-provided buffers — as byte codes or straight into the 5-bit packed wire format.
// Pass 1 can run on one process (count = true) or cooperatively: every rank of a node counts a share of
// the chunks of the node-shared text, the counts are exchanged, and each rank then encodes its own slice
// into its own (NUMA-local, page-locked) buffers. `data` must outlive the parser.
class BulkParser {
 public:
  BulkParser(const char* data, size_t len, const ParseOptions& opt = {}, bool count = true);
  // A parser over a bare record area without a header — one batch of a streaming job: its first `n`
  // tokens are the records, the problem (weights, Seq1, Seq2 length cap) comes from the job's header, and
  // pass 1 is the caller's chunk table (set_chunks).
  BulkParser(const char* area, size_t len, const Weights& w, const std::vector<uint8_t>& seq1, int64_t l2_cap,
             int64_t n);
  const Weights& weights() const { return weights_; }
  const std::vector<uint8_t>& seq1() const { return seq1_; }
  int64_t count() const { return n_; }
  int64_t total_chars() const { return total_chars_; }  // after pass 1
  int64_t area_bytes() const { return static_cast<int64_t>(area_len_); }
  int64_t l2_cap() const { return l2_cap_; }

  // ---- pass 1
  // nchunks+1 chunk boundaries (byte offsets in the area), each moved forward past the token it cuts.
  std::vector<int64_t> chunk_starts(int nchunks) const;
  // Tokens / letters of chunks [c0, c1) -> toks[c - c0], chars[c - c0] (OpenMP over the chunks).
  void count_chunks(const std::vector<int64_t>& starts, int c0, int c1, int64_t* toks, int64_t* chars) const;
  // Installs the chunk table (per-chunk counts of ALL chunks); throws when the area holds fewer than
  // count() records. Only the first count() tokens are records (trailing tokens are ignored).
  void set_chunks(std::vector<int64_t> starts, const int64_t* toks, const int64_t* chars);
  int nchunks() const { return static_cast<int>(start_.size()) - 1; }
  // Records / letters before chunk c (prefix arrays of the table, clipped to count() records).
  int64_t chunk_first_record(int c) const { return std::min(tok_pre_[c], n_); }
  int64_t chunk_first_letter(int c) const;

  // ---- pass 2
  AreaSlice slice(int64_t rec_begin, int64_t rec_end) const;
  // Encodes slice s: letters as bytes into codes[0..s.letters) and/or packed into `packed` (either may be
  // null): `pack` 5 = 5-bit packed, packed[0..packed5_bytes(s.letters)); 33 = P33 fields (moc::pack33),
  // packed[0..packed33_bytes(s.letters)).
  // Record boundaries (each output optional): dense
  // offsets[0..s.records] rebased to 0; sparse offsets (moc/wire.hpp, stride 2^kSparseShift)
  // sparse[0..sparse_count(s.records, kSparseShift)); lengths len16[0..s.records), saturated at 65535
  // (the report's max_len tells whether they are exact).
  FillReport fill_slice(const AreaSlice& s, uint8_t* codes, uint8_t* packed, int64_t* offsets,
                        int64_t* sparse = nullptr, uint16_t* len16 = nullptr, int pack = 5) const;
  // Throws the error a sequential reader would report first for this report (`first` = the report's
  // slice start; validates the score range for its longest record).
  void check(const FillReport& r) const;
  // All records: codes[0..total_chars()), offsets[0..count()] (offsets[0] = 0); throws on errors.
  void fill(uint8_t* codes, int64_t* offsets) const;
  // n * (L1 - avg + 1) * avg from the mean record length (pass 1's letters, or the area size before it).
  int64_t cells_estimate() const;
  // Mean record length: exact after pass 1, else the area's bytes less one separator per record.
  int64_t mean_length_estimate() const;
  // Exact cost (moc/partition.hpp) of all tokens of chunks [c0, c1) -> costs[c - c0] (OpenMP over chunks).
  void chunk_costs(const std::vector<int64_t>& starts, int c0, int c1, const CostModel& m, double* costs) const;
  // Installs exact chunk costs for cost_split (all chunks, same model); without them it estimates.
  void set_chunk_costs(std::vector<double> costs);
  // Rank bounds without a lengths array (after pass 1): the record index where the cost of records
  // [first, count()) reaches part/parts of their total. Chunk costs are exact when installed (else the
  // records at the chunk's mean length), walks are exact inside the chunk that holds the split. Monotone
  // in part, and the same on every rank holding the same chunk table, so each rank computes its own
  // [split(r), split(r + 1)) without a collective.
  int64_t cost_split(int64_t first, int part, int parts, const CostModel& m) const;

 private:
  struct Located {
    int64_t byte = 0, chr = 0;  // area byte just after token t-1 (or the chunk start) and letters before t
  };
  Located locate(int64_t t) const;  // position of the boundary before record t (t <= tokens in the area)
  Weights weights_{};
  std::vector<uint8_t> seq1_;
  int64_t n_ = 0, total_chars_ = 0, l2_cap_ = 0;
  const char* area_ = nullptr;
  size_t area_len_ = 0;
  std::vector<int64_t> start_, tok_pre_, chr_pre_;  // chunk table: nchunks+1 entries each
  std::vector<double> cost_;                        // optional exact chunk costs (nchunks entries)
};

// fscanf's separators: ' ' and \t \n \v \f \r (0x09..0x0d)
inline bool is_input_space(unsigned char c) { return c == ' ' || static_cast<unsigned char>(c - 9) <= 4; }
// Tokens and letters (non-space bytes) of text [p, p + len) that starts at a token start or at whitespace
// (pass 1; vectorised, no branches per byte).
void count_tokens(const char* p, size_t len, int64_t* tokens, int64_t* letters);

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
  // Hands the bytes read past the last consumed token to the caller (appended to `out`), which reads the
  // rest of the stream itself; true when the stream is already at its end.
  bool take_rest(uvector<char>& out);

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
// The same for consecutive runs of results in any wire format (e.g. every rank's slice in its own format),
// decoded row by row while formatting.
void write_results(FILE* f, const std::vector<ResultRun>& runs, int64_t first_index = 0);
std::string format_results(const Result* results, int64_t n, int64_t first_index = 0);
// Exact bytes of the rows write_results produces for these runs (a sizing pass, no formatting).
int64_t formatted_bytes(const std::vector<ResultRun>& runs, int64_t first_index = 0);
// Formats the rows and writes them into the regular file `fd` at byte offset `at` (parallel pwrite), so
// several processes can each write their own rows of one output file; returns the bytes written.
int64_t write_results_at(int fd, int64_t at, const std::vector<ResultRun>& runs, int64_t first_index = 0);

}  // namespace moc
