// AreaText / Cutter (text_cut.hpp): the root's pass 1 ahead of a streamed job's batches.
#include "text_cut.hpp"

#include <omp.h>
#include <sys/mman.h>

#include <algorithm>
#include <cstring>

namespace moc {

namespace {
constexpr int kMadvPopulateRead = 22;  // MADV_POPULATE_READ (Linux 5.14); older headers lack the name
}

bool AreaText::load_more(int64_t want) {
  if (map_ || eof_) return false;
  want = std::max<int64_t>(want, 4 * kMiB);
  if (len_ + want > static_cast<int64_t>(buf_.size()) && drop_ > base_) {  // room: drop the consumed prefix
    const int64_t keep = hi_ - drop_;
    std::memmove(buf_.data(), buf_.data() + (drop_ - base_), static_cast<size_t>(keep));
    base_ = drop_;
    len_ = keep;
  }
  if (len_ + want > static_cast<int64_t>(buf_.size()))
    buf_.resize(static_cast<size_t>(std::max<int64_t>(len_ + want, 2 * static_cast<int64_t>(buf_.size()))));
  const size_t room = buf_.size() - static_cast<size_t>(len_);
  const size_t got = read_regular_into(f_, buf_.data() + len_, room);
  if (got < room) {
    if (std::ferror(f_)) throw Error("error while reading input stream");
    eof_ = true;
  }
  len_ += static_cast<int64_t>(got);
  hi_ = base_ + len_;
  return got > 0;
}

BatchCut Cutter::take(int64_t max_rec, int64_t max_chr) {
  while (!(tok_ahead_ >= max_rec || chr_ahead_ >= max_chr) && !(t_.eof() && counted_ >= t_.hi())) extend(max_rec, max_chr);
  BatchCut cut;
  cut.begin = cut.next = chunks_.empty() ? counted_ : chunks_.front().begin;
  int64_t taken = 0, letters = 0;
  size_t used = 0;
  bool split = false;
  Chunk rest;
  for (; used < chunks_.size(); ++used) {
    if (taken >= max_rec || (taken > 0 && letters >= max_chr)) break;
    const Chunk& c = chunks_[used];
    cut.chunks.push_back(c);
    if (c.toks == 0 || (taken + c.toks <= max_rec && letters + c.chars - 1 < max_chr)) {  // whole chunk
      taken += c.toks;
      letters += c.chars;
      cut.next = c.end;
      continue;
    }
    // the batch ends inside this chunk (or its last token is the first over a limit): token walk
    const unsigned char* ua = reinterpret_cast<const unsigned char*>(t_.at(c.begin));
    int64_t i = 0, tk = 0, ch = 0;
    const int64_t e = c.end - c.begin;
    bool stop = false;
    while (i < e) {
      while (i < e && is_input_space(ua[i])) ++i;
      if (i >= e) break;
      if (taken + tk >= max_rec || (taken + tk > 0 && letters + ch >= max_chr)) {
        stop = true;
        break;
      }
      int64_t j = i;
      while (j < e && !is_input_space(ua[j])) ++j;
      ++tk;
      ch += j - i;
      i = j;
    }
    taken += tk;
    letters += ch;
    if (stop) {
      cut.next = c.begin + i;
      rest = Chunk{c.begin + i, c.end, c.toks - tk, c.chars - ch};
      split = true;
      ++used;
      break;
    }
    cut.next = c.end;
  }
  chunks_.erase(chunks_.begin(), chunks_.begin() + static_cast<std::ptrdiff_t>(used));
  if (split) chunks_.push_front(rest);
  tok_ahead_ = chr_ahead_ = 0;
  for (const Chunk& c : chunks_) {
    tok_ahead_ += c.toks;
    chr_ahead_ += c.chars;
  }
  cut.n = taken;
  cut.letters = letters;
  cut.end = cut.chunks.empty() ? cut.begin : cut.chunks.back().end;
  return cut;
}
bool Cutter::count_ahead(int64_t max_rec, int64_t max_chr, int64_t batches) {
  if (t_.eof() && counted_ >= t_.hi()) return false;
  const bool by_rec = max_rec < INT64_MAX, by_chr = max_chr < INT64_MAX;
  if ((by_rec && tok_ahead_ >= batches * max_rec) || (!by_rec && by_chr && chr_ahead_ >= batches * max_chr) ||
      (!by_rec && !by_chr))
    return false;
  const int64_t before = counted_;
  extend(by_rec ? tok_ahead_ + max_rec : INT64_MAX, by_chr ? chr_ahead_ + max_chr : INT64_MAX);
  return counted_ > before;
}

// ~1 MiB chunks: the walk to a batch's cut scans at most one, and the ranks' encode of a batch gets pieces
// small enough to balance over their threads
void Cutter::extend(int64_t max_rec, int64_t max_chr) {
  const double bpt = seen_toks_ > 0 ? static_cast<double>(seen_bytes_) / seen_toks_ : 16.0;
  const double bpl = seen_chars_ > 0 ? static_cast<double>(seen_bytes_) / seen_chars_ : 2.0;
  double want = std::min(max_rec < INT64_MAX ? (max_rec - tok_ahead_) * bpt : 1e18,
                         max_chr < INT64_MAX ? (max_chr - chr_ahead_) * bpl : 1e18);
  if (seen_toks_ == 0) want = std::min(want, 8.0 * kMiB);  // a first probe of the density
  const int64_t region = std::clamp<int64_t>(static_cast<int64_t>(want * 1.02) + kMiB, kMiB, int64_t{1} << 30);
  int64_t end = counted_ + region;
  while (end > t_.hi() && t_.load_more(end - t_.hi())) {
  }
  if (end >= t_.hi()) {
    end = t_.hi();
    if (!t_.eof()) {  // the loaded text ends inside a token: the region ends before it
      const unsigned char* ua = reinterpret_cast<const unsigned char*>(t_.at(counted_));
      int64_t e = end - counted_;
      while (e > 0 && !is_input_space(ua[e - 1])) --e;
      if (e == 0) {  // one token longer than everything loaded: load until it ends
        t_.load_more(end - counted_);
        return;
      }
      end = counted_ + e;
    }
  } else {  // move forward past the token the region end cuts
    while (true) {
      const unsigned char* ua = reinterpret_cast<const unsigned char*>(t_.at(counted_));
      int64_t e = end - counted_;
      const int64_t lim = t_.hi() - counted_;
      while (e < lim && e > 0 && !is_input_space(ua[e - 1])) ++e;
      end = counted_ + e;
      if (e < lim || t_.eof() || is_input_space(ua[e - 1])) break;
      if (!t_.load_more(kMiB)) break;
    }
  }
  const int64_t len = end - counted_;
  if (len <= 0) return;
  // ~1 MiB chunks: the walk to a batch's cut scans at most one, and the ranks' encode of a batch gets
  // pieces small enough to balance over their threads
  const int nt = static_cast<int>(std::clamp<int64_t>(len / kMiB, 1, 1 << 14));
  const unsigned char* ua = reinterpret_cast<const unsigned char*>(t_.at(counted_));
  std::vector<Chunk> parts(static_cast<size_t>(nt));
  std::vector<int64_t> b(static_cast<size_t>(nt) + 1);
  b[0] = 0;
  for (int q = 1; q < nt; ++q) {  // chunk starts move forward past the token they cut
    int64_t x = std::max(len * q / nt, b[q - 1]);
    while (x < len && x > 0 && !is_input_space(ua[x - 1])) ++x;
    b[q] = x;
  }
  b[nt] = len;
  const bool mapped = t_.mapped();
#pragma omp parallel for schedule(dynamic, 4) if (nt > 2)
  for (int q = 0; q < nt; ++q) {
    Chunk& c = parts[q];
    c.begin = counted_ + b[q];
    c.end = counted_ + b[q + 1];
    const char* at = reinterpret_cast<const char*>(ua) + b[q];
    if (mapped) {  // the chunk's page tables in one call rather than a fault per 64 KiB (28 % faster reads of a
                   // mapped file on the box, profiles/populate_probe_box.log; ignored before Linux 5.14)
      const uintptr_t a0 = reinterpret_cast<uintptr_t>(at) & ~uintptr_t{4095};
      (void)madvise(reinterpret_cast<void*>(a0), static_cast<size_t>(reinterpret_cast<uintptr_t>(at) + (b[q + 1] - b[q]) - a0),
                    kMadvPopulateRead);
    }
    count_tokens(at, static_cast<size_t>(b[q + 1] - b[q]), &c.toks, &c.chars);
  }
  for (const Chunk& c : parts) {
    if (c.end <= c.begin) continue;
    chunks_.push_back(c);
    tok_ahead_ += c.toks;
    chr_ahead_ += c.chars;
    seen_toks_ += c.toks;
    seen_chars_ += c.chars;
  }
  seen_bytes_ += len;
  counted_ = end;
}
}  // namespace moc
