// The root's view of a streamed input's record area and its batch cutter (pass 1 ahead of the batches),
// shared by the node's streaming flow (flow_stream.cpp) and the device transports' (flow_device_stream.cpp).
#pragma once

#include <cstdio>
#include <deque>
#include <vector>

#include "moc/io.hpp"
#include "moc/problem.hpp"

namespace moc {

constexpr int64_t kMiB = int64_t{1} << 20;

// The text of the record area. Absolute offsets count from the first byte after the header ("area
// offsets"): a mapped --input file, or a stream read on demand into a buffer that drops consumed text.
class AreaText {
 public:
  AreaText(const char* mapped, int64_t bytes) : map_(mapped), hi_(bytes), eof_(true) {}
  AreaText(uvector<char> head, bool eof, FILE* f) : buf_(std::move(head)), len_(static_cast<int64_t>(buf_.size())),
                                                      hi_(len_), eof_(eof), f_(f) {}
  bool mapped() const { return map_ != nullptr; }
  const char* at(int64_t abs) const { return map_ ? map_ + abs : buf_.data() + (abs - base_); }
  int64_t hi() const { return hi_; }  // end of the loaded text
  bool eof() const { return eof_; }   // hi() is the end of the input
  // stream input: text before `abs` is no longer needed (dropped lazily, when the buffer needs room)
  void drop_before(int64_t abs) { drop_ = std::max(drop_, abs); }
  // stream input: loads at least `want` more bytes unless the input ends first; false if nothing new
  bool load_more(int64_t want);

 private:
  const char* map_ = nullptr;
  uvector<char> buf_;
  int64_t base_ = 0, len_ = 0, drop_ = 0;
  int64_t hi_ = 0;
  bool eof_ = true;
  FILE* f_ = nullptr;
};

struct Chunk {
  int64_t begin = 0, end = 0, toks = 0, chars = 0;  // area offsets; begin at a token start or whitespace
};

// One batch as the root cut it: area [begin, end) (whole counted chunks; the records are its first n
// tokens), its chunk table, and where the next batch starts.
struct BatchCut {
  int64_t n = 0, letters = 0, begin = 0, end = 0, next = 0;
  std::vector<Chunk> chunks;
};

// Root: pass 1 ahead of the batches, and the cuts.
class Cutter {
 public:
  explicit Cutter(AreaText& t) : t_(t) {}
  // Cuts the next batch: records are taken while fewer than max_rec are taken and (none is taken yet or
  // fewer than max_chr letters are) — StreamReader::next_batch's rule.
  BatchCut take(int64_t max_rec, int64_t max_chr);
  // Counts one more batch's worth of text ahead of the batches taken so far (at most `batches` ahead); false
  // when that much is counted already or the text is done. Work for the wait on the GPU's start-up.
  bool count_ahead(int64_t max_rec, int64_t max_chr, int64_t batches);

 private:
  // Counts the next region of the text (parallel chunks cut at whitespace), sized from the density seen.
  void extend(int64_t max_rec, int64_t max_chr);

  AreaText& t_;
  std::deque<Chunk> chunks_;  // counted, not yet taken
  int64_t counted_ = 0;       // area offset where counting continues
  int64_t tok_ahead_ = 0, chr_ahead_ = 0;
  int64_t seen_bytes_ = 0, seen_toks_ = 0, seen_chars_ = 0;
};

}  // namespace moc
