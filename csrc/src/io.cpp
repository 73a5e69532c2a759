#include "moc/io.hpp"

#include <fcntl.h>
#include <omp.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <memory>

#include "moc/runtime/releaser.hpp"
#include "moc/simd.hpp"

namespace moc {

namespace {

inline bool is_space(unsigned char c) { return is_input_space(c); }

// letter -> code (1..26, either case), 0 for anything else
struct CodeTable {
  uint8_t v[256];
  CodeTable() {
    for (int c = 0; c < 256; ++c) v[c] = static_cast<uint8_t>(letter_code(static_cast<unsigned char>(c)));
  }
  uint8_t operator[](unsigned char c) const { return v[c]; }
};
const CodeTable kCodeOf;

struct Cursor {
  const char* p;
  const char* end;
  // Returns the next whitespace-delimited token [b, e) or false at end of input.
  bool next(const char*& b, const char*& e) {
    while (p < end && is_space(static_cast<unsigned char>(*p))) ++p;
    if (p >= end) return false;
    b = p;
    while (p < end && !is_space(static_cast<unsigned char>(*p))) ++p;
    e = p;
    return true;
  }
};

int64_t parse_int(const char* b, const char* e, const char* what) {
  std::string tok(b, e);
  char* stop = nullptr;
  errno = 0;
  long long v = std::strtoll(tok.c_str(), &stop, 10);
  if (errno != 0 || stop != tok.c_str() + tok.size())
    throw Error(std::string("expected an integer for ") + what + ", got '" + tok + "'");
  return v;
}

}  // namespace

size_t read_regular_into(FILE* f, char* dst, size_t want) {
  const long pos = std::ftell(f);
  if (pos < 0 || want <= (size_t{8} << 20)) {
    const size_t got = std::fread(dst, 1, want, f);
    if (got < want && std::ferror(f)) throw Error("error while reading input stream");
    return got;
  }
  // large file: the copy out of the page cache split over the OpenMP threads (one fread is a
  // single-threaded, page-faulting memcpy of the whole file)
  const int fd = fileno(f);
  // chunks of 1..16 MiB, at least two per thread
  const size_t kChunk = std::clamp(want / (2 * static_cast<size_t>(std::max(1, omp_get_max_threads()))), size_t{1} << 20,
                                   size_t{16} << 20);
  const int64_t nchunks = static_cast<int64_t>((want + kChunk - 1) / kChunk);
  std::vector<size_t> got(static_cast<size_t>(nchunks), 0);
  int failed = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(| : failed)
  for (int64_t c = 0; c < nchunks; ++c) {
    const size_t b = static_cast<size_t>(c) * kChunk, e = std::min(want, b + kChunk);
    size_t at = b;
    while (at < e) {
      const ssize_t r = pread(fd, dst + at, e - at, static_cast<off_t>(pos) + static_cast<off_t>(at));
      if (r < 0 && errno == EINTR) continue;
      if (r < 0) {
        failed = 1;
        break;
      }
      if (r == 0) break;
      at += static_cast<size_t>(r);
    }
    got[static_cast<size_t>(c)] = at - b;
  }
  if (failed) throw Error("error while reading input stream");
  // the file as it was at fstat time; a short chunk means it shrank: keep the contiguous prefix
  size_t len = 0;
  for (int64_t c = 0; c < nchunks; ++c) {
    len += got[static_cast<size_t>(c)];
    if (got[static_cast<size_t>(c)] < std::min(want, static_cast<size_t>(c + 1) * kChunk) - static_cast<size_t>(c) * kChunk)
      break;
  }
  (void)std::fseek(f, static_cast<long>(pos) + static_cast<long>(len), SEEK_SET);
  return len;
}

int64_t regular_input_bytes(FILE* f) {
  struct stat st;
  if (fstat(fileno(f), &st) != 0 || !S_ISREG(st.st_mode) || st.st_size <= 0) return -1;
  const long pos = std::ftell(f);
  return pos < 0 ? -1 : std::max<int64_t>(0, static_cast<int64_t>(st.st_size) - pos);
}

uvector<char> read_stream(FILE* f) {
  uvector<char> buf;
  size_t len = 0;
  const int64_t size = regular_input_bytes(f);
  if (size > 0) {
    // regular file: one allocation of the remaining size (+1 to detect growth), one read
    const size_t want = static_cast<size_t>(size) + 1;
    buf.resize(want);  // not touched yet (default-init): the advice below applies to every page
    if (want > (size_t{64} << 20)) {
      constexpr uintptr_t kHuge = uintptr_t{2} << 20;  // 2 MiB pages for the buffer
      const uintptr_t lo = (reinterpret_cast<uintptr_t>(buf.data()) + kHuge - 1) & ~(kHuge - 1);
      const uintptr_t hi = (reinterpret_cast<uintptr_t>(buf.data()) + want) & ~(kHuge - 1);
      if (hi > lo) (void)madvise(reinterpret_cast<void*>(lo), hi - lo, MADV_HUGEPAGE);
    }
    len = read_regular_into(f, buf.data(), want - 1);
    if (len < want - 1) {  // it shrank
      buf.resize(len);
      return buf;
    }
    // a file that grew after fstat continues through the stream loop below
    const size_t more = std::fread(buf.data() + len, 1, 1, f);
    len += more;
    if (!more) {
      if (std::ferror(f)) throw Error("error while reading input stream");
      buf.resize(len);
      return buf;
    }
  }
  // pipe / terminal (or a file that grew): read in growing blocks; new memory is not zero-filled
  size_t cap = std::max<size_t>(buf.size(), size_t{1} << 20);
  buf.resize(cap);
  while (true) {
    const size_t got = std::fread(buf.data() + len, 1, cap - len, f);
    len += got;
    if (len < cap) {
      if (std::ferror(f)) throw Error("error while reading input stream");
      break;
    }
    cap *= 2;
    buf.resize(cap);
  }
  buf.resize(len);
  return buf;
}

BulkParser::BulkParser(const char* data, size_t len, const ParseOptions& opt, bool count) {
  Cursor cur{data, data + len};
  const char *b, *e;
  static const char* wname[4] = {"W1", "W2", "W3", "W4"};
  for (int i = 0; i < 4; ++i) {
    if (!cur.next(b, e)) throw Error(std::string("unexpected end of input while reading ") + wname[i]);
    int64_t v = parse_int(b, e, wname[i]);
    if (v < 0 || v > INT32_MAX) throw Error(std::string(wname[i]) + " out of range");
    weights_.w[i] = static_cast<int32_t>(v);
  }
  if (!cur.next(b, e)) throw Error("unexpected end of input while reading Seq1");
  seq1_ = encode_sequence(b, e - b);
  if (!cur.next(b, e)) throw Error("unexpected end of input while reading the number of sequences");
  n_ = parse_int(b, e, "number_of_sequences");
  if (n_ < 0) throw Error("number_of_sequences must be >= 0");

  const int64_t l1_cap = opt.strict_limits ? kSpecMaxSeq1 : opt.max_l1;
  l2_cap_ = opt.strict_limits ? kSpecMaxSeq2 : opt.max_l2;
  if (l1_cap > 0 && static_cast<int64_t>(seq1_.size()) > l1_cap)
    throw Error("Seq1 has " + std::to_string(seq1_.size()) + " letters, limit is " + std::to_string(l1_cap));
  area_ = cur.p;
  area_len_ = static_cast<size_t>(cur.end - cur.p);
  total_chars_ = -1;
  if (count) {  // pass 1 on this process: one chunk per OpenMP thread
    const int nt = area_len_ < (size_t{1} << 16) ? 1 : std::max(1, omp_get_max_threads());
    std::vector<int64_t> st = chunk_starts(nt), tk(static_cast<size_t>(nt)), ch(static_cast<size_t>(nt));
    count_chunks(st, 0, nt, tk.data(), ch.data());
    set_chunks(std::move(st), tk.data(), ch.data());
  }
}

BulkParser::BulkParser(const char* area, size_t len, const Weights& w, const std::vector<uint8_t>& seq1,
                       int64_t l2_cap, int64_t n)
    : weights_(w), seq1_(seq1), n_(n), total_chars_(-1), l2_cap_(l2_cap), area_(area), area_len_(len) {}

std::vector<int64_t> BulkParser::chunk_starts(int nchunks) const {
  nchunks = std::max(1, nchunks);
  const int64_t len = static_cast<int64_t>(area_len_);
  const unsigned char* ua = reinterpret_cast<const unsigned char*>(area_);
  std::vector<int64_t> s(static_cast<size_t>(nchunks) + 1, 0);
  for (int t = 1; t < nchunks; ++t) {
    // from the previous boundary when that already lies past this one: every byte is scanned at most
    // once, even inside a token longer than many chunks
    int64_t x = std::max(len * t / nchunks, s[t - 1]);
    while (x < len && x > 0 && !is_space(ua[x - 1])) ++x;
    s[t] = x;
  }
  s[nchunks] = len;
  return s;
}

namespace {
bool count_simd_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("MOC_FILL_SIMD");
    if (e && std::strcmp(e, "0") == 0) return false;
    __builtin_cpu_init();
    return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw");
  }();
  return on;
}

// count_tokens, 64 bytes per step: whitespace mask by byte compares; tokens = non-space bytes after
// whitespace, letters = non-space bytes (two popcounts per 64 bytes).
__attribute__((target("avx512f,avx512bw,popcnt"))) void count_tokens_avx512(const unsigned char* ua, size_t len,
                                                                              int64_t* tokens, int64_t* letters) {
  const __m512i k9 = _mm512_set1_epi8(9), k4 = _mm512_set1_epi8(4), kSp = _mm512_set1_epi8(' ');
  uint64_t prev_ws = 1, nt = 0, nc = 0;
  for (size_t i = 0; i < len; i += 64) {
    const size_t nb = std::min<size_t>(64, len - i);
    const __mmask64 in = nb == 64 ? ~__mmask64{0} : (__mmask64{1} << nb) - 1;
    const __m512i v = _mm512_maskz_loadu_epi8(in, ua + i);
    const __mmask64 ws = _mm512_cmpeq_epi8_mask(v, kSp) | _mm512_cmple_epu8_mask(_mm512_sub_epi8(v, k9), k4) | ~in;
    nt += _mm_popcnt_u64(~ws & ((ws << 1) | prev_ws));
    nc += _mm_popcnt_u64(~ws);
    prev_ws = ws >> 63;
  }
  *tokens = static_cast<int64_t>(nt);
  *letters = static_cast<int64_t>(nc);
}
}  // namespace

void count_tokens(const char* p, size_t len, int64_t* tokens, int64_t* letters) {
  const unsigned char* ua = reinterpret_cast<const unsigned char*>(p);
  if (count_simd_enabled()) {
    count_tokens_avx512(ua, len, tokens, letters);
    return;
  }
  int64_t nt = 0, nc = 0;
  if (len > 0) {  // the text starts at a token start or at whitespace
    const int64_t first = is_space(ua[0]) ? 0 : 1;
    nt = first;
    nc = first;
    // pass 1 (branch-free): tokens = space->letter transitions, letters = non-space bytes. Independent
    // iterations (the previous byte is re-read, not carried) vectorise; 8-bit lanes summed per 255-byte
    // block so the counters cannot overflow
    for (size_t blk = 1; blk < len; blk += 255) {
      const size_t be = std::min(len, blk + 255);
      unsigned t_cnt = 0, c_cnt = 0;
      for (size_t i = blk; i < be; ++i) {
        const unsigned char ch = ua[i], q = ua[i - 1];
        const unsigned lt = (ch != ' ') & (static_cast<unsigned char>(ch - 9) > 4);  // ch is a token byte
        const unsigned ps = (q == ' ') | (static_cast<unsigned char>(q - 9) <= 4);   // q is whitespace
        t_cnt += lt & ps;
        c_cnt += lt;
      }
      nt += t_cnt;
      nc += c_cnt;
    }
  }
  *tokens = nt;
  *letters = nc;
}

void BulkParser::count_chunks(const std::vector<int64_t>& starts, int c0, int c1, int64_t* toks,
                              int64_t* chars) const {
  // Iterations are chunks, not thread ids: correct whatever number of threads OpenMP delivers.
#pragma omp parallel for schedule(dynamic, 1) if (c1 - c0 > 1 && starts[c1] - starts[c0] > (int64_t{1} << 16))
  for (int c = c0; c < c1; ++c)
    count_tokens(area_ + starts[c], static_cast<size_t>(starts[c + 1] - starts[c]), toks + (c - c0), chars + (c - c0));
}

void BulkParser::set_chunks(std::vector<int64_t> starts, const int64_t* toks, const int64_t* chars) {
  start_ = std::move(starts);
  const int nch = static_cast<int>(start_.size()) - 1;
  tok_pre_.assign(static_cast<size_t>(nch) + 1, 0);
  chr_pre_.assign(static_cast<size_t>(nch) + 1, 0);
  for (int c = 0; c < nch; ++c) {
    tok_pre_[c + 1] = tok_pre_[c] + toks[c];
    chr_pre_[c + 1] = chr_pre_[c] + chars[c];
  }
  const int64_t total_tokens = tok_pre_[nch];
  if (total_tokens < n_)
    throw Error("expected " + std::to_string(n_) + " Seq2 records, found only " + std::to_string(total_tokens));
  // only the first n tokens are records (extra trailing tokens are ignored, like the reference)
  total_chars_ = total_tokens == n_ ? chr_pre_[nch] : locate(n_).chr;
}

int64_t BulkParser::chunk_first_letter(int c) const { return tok_pre_[c] <= n_ ? chr_pre_[c] : total_chars_; }

BulkParser::Located BulkParser::locate(int64_t t) const {
  Located l;
  if (t <= 0) return l;
  // chunk c holds token t-1: tok_pre_[c] <= t-1 < tok_pre_[c+1]
  const int c = static_cast<int>(std::upper_bound(tok_pre_.begin(), tok_pre_.end(), t - 1) - tok_pre_.begin()) - 1;
  const unsigned char* ua = reinterpret_cast<const unsigned char*>(area_);
  int64_t i = start_[c];
  const int64_t e = start_[c + 1];
  int64_t k = tok_pre_[c], chr = chr_pre_[c];
  while (k < t && i < e) {
    while (i < e && is_space(ua[i])) ++i;
    const int64_t b = i;
    while (i < e && !is_space(ua[i])) ++i;
    chr += i - b;
    ++k;
  }
  l.byte = i;
  l.chr = chr;
  return l;
}

AreaSlice BulkParser::slice(int64_t rec_begin, int64_t rec_end) const {
  if (start_.empty()) throw Error("BulkParser::slice before pass 1");
  rec_begin = std::clamp<int64_t>(rec_begin, 0, n_);
  rec_end = std::clamp<int64_t>(rec_end, rec_begin, n_);
  AreaSlice s;
  s.first_record = rec_begin;
  s.records = rec_end - rec_begin;
  if (s.records == 0) return s;
  const Located lo = locate(rec_begin), hi = locate(rec_end);
  s.letters = hi.chr - lo.chr;
  const int nch = nchunks();
  for (int c = 0; c < nch; ++c) {
    const int64_t b = std::max(start_[c], lo.byte), e = std::min(start_[c + 1], hi.byte);
    if (b >= e) continue;
    AreaPiece p;
    p.byte_begin = b;
    p.byte_end = e;
    p.tok = b == lo.byte ? 0 : tok_pre_[c] - rec_begin;
    p.chr = b == lo.byte ? 0 : chr_pre_[c] - lo.chr;
    s.pieces.push_back(p);
  }
  return s;
}

namespace {
// Letter codes of 16 input bytes ((c & 0x1F): 'A'/'a' -> 1 ... 'Z'/'z' -> 26), with bit masks of the
// whitespace bytes (as is_space) and of the bytes that are letters.
inline __m128i encode16(const unsigned char* src, unsigned& space_mask, unsigned& letter_mask) {
  const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src));
  const __m128i t = _mm_sub_epi8(v, _mm_set1_epi8(9));  // \t \n \v \f \r -> 0..4
  const __m128i ws = _mm_or_si128(_mm_cmpeq_epi8(v, _mm_set1_epi8(' ')),
                                  _mm_cmpeq_epi8(_mm_min_epu8(t, _mm_set1_epi8(4)), t));
  const __m128i u = _mm_sub_epi8(_mm_and_si128(v, _mm_set1_epi8(static_cast<char>(0xDF))), _mm_set1_epi8('A'));
  const __m128i letter = _mm_cmpeq_epi8(_mm_min_epu8(u, _mm_set1_epi8(25)), u);
  space_mask = static_cast<unsigned>(_mm_movemask_epi8(ws));
  letter_mask = static_cast<unsigned>(_mm_movemask_epi8(letter));
  return _mm_and_si128(v, _mm_set1_epi8(0x1F));
}
}  // namespace

namespace {
// 8 letter codes (one per byte, < 32) -> their 40-bit 5-bit packed form (char j at bits [5j, 5j+5)).
inline uint64_t compress8(uint64_t x) {
  x &= 0x1F1F1F1F1F1F1F1Full;
  x = (x & 0x001F001F001F001Full) | ((x >> 3) & 0x03E003E003E003E0ull);
  x = (x & 0x000003FF000003FFull) | ((x >> 6) & 0x000FFC00000FFC00ull);
  x = (x & 0x00000000000FFFFFull) | ((x >> 12) & 0x000000FFFFF00000ull);
  return x;
}
constexpr int64_t kStage = int64_t{1} << 16;  // letters staged per thread before packing

struct PieceOut {
  FillReport rep;
  int64_t rec_base = 0;                       // global index of the piece's first record
  std::vector<std::pair<int64_t, uint8_t>> stragglers;  // packed mode: letters of partial groups
};

// One piece of a slice for the vector encoder: text bytes [bb, be) (starting at a token start or at
// whitespace, ending after its last token), its letters [a, b) and first token (slice-relative), and the
// outputs of fill_slice.
struct PieceJob {
  const unsigned char* ua;
  size_t bb, be;
  int64_t a, b, tok0;
  uint8_t* codes;
  uint8_t* packed;
  int64_t* offs;
  int64_t* sparse;
  uint16_t* len16;
  int64_t G, GB;
  bool p33;
  int64_t l2_cap, L1;
};

// MOC_FILL_SIMD=0 selects the portable SSE2 encoder (A/B, and hosts without AVX-512 VBMI2 use it anyway).
bool fill_simd_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("MOC_FILL_SIMD");
    if (e && std::strcmp(e, "0") == 0) return false;
    __builtin_cpu_init();
    return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
           __builtin_cpu_supports("avx512vbmi") && __builtin_cpu_supports("avx512vbmi2");
  }();
  return on;
}

#define MOC_AVX512 __attribute__((target("avx512f,avx512bw,avx512vbmi,avx512vbmi2,bmi,bmi2,popcnt,lzcnt")))
using simd::p33_block_avx512;

// Pass 2 of one piece, 64 text bytes per step: whitespace / letter masks by byte compares, the letter codes
// compacted with vpcompressb (register form) and stored under a mask, token starts as mask bits (a
// non-space byte after whitespace); each token's start letter is a popcount of the compacted bytes before
// it, so a record costs a few scalar operations and a byte costs none. Returns false — the caller then
// runs the scalar encoder for the piece, which names the offending record — on a non-letter byte or a
// record over the length limit.
// Packs the staged letters [st.base, hi) of a piece (and copies them to codes when both are wanted): whole
// groups straight into the packed stream; letters of the piece's first partial group and, at the end, of
// its last one go to the stragglers (fixed up once the whole slice is encoded).
struct Stager {
  uint8_t* stage;
  int64_t base;
  bool head_done;
};
MOC_AVX512 void stage_flush(const PieceJob& j, PieceOut& po, Stager& st, int64_t hi, bool final) {
  const int64_t G = j.G, GB = j.GB;
  if (j.codes) std::memcpy(j.codes + st.base, st.stage, static_cast<size_t>(hi - st.base));
  int64_t cur = st.base;
  if (!st.head_done) {
    const int64_t g0 = (j.a + G - 1) / G * G, hend = std::min(g0, hi);
    if (hend < g0 && !final) return;
    for (int64_t c = cur; c < hend; ++c) po.stragglers.emplace_back(c, st.stage[c - st.base]);
    cur = hend;
    st.head_done = true;
  }
  const int64_t ng = (hi - cur) / G;
  const uint8_t* src = st.stage + (cur - st.base);
  uint8_t* dst = j.packed + GB * (cur / G);
  if (j.p33) {
    for (int64_t g = 0; g < ng; ++g) p33_block_avx512(src + kP33Letters * g, dst + kP33Bytes * g);
  } else {
    for (int64_t g = 0; g < ng; ++g) {
      uint64_t x;
      std::memcpy(&x, src + 8 * g, 8);
      x = compress8(x);
      std::memcpy(dst + 5 * g, &x, g + 1 < ng ? 8 : 5);
    }
  }
  cur += G * ng;
  if (final) {
    for (int64_t c = cur; c < hi; ++c) po.stragglers.emplace_back(c, st.stage[c - st.base]);
  } else {
    std::memmove(st.stage, st.stage + (cur - st.base), static_cast<size_t>(hi - cur));
    st.base = cur;
  }
}

// Record bookkeeping of the per-block path: lengths (and the sparse offsets' record starts) of a piece.
struct Book {
  int64_t tok, mn, mx, cells;
};
// One record closed by scalar code (a token that crossed a block boundary): letters [start, start + L).
MOC_AVX512 inline void close_record(Book& bk, const PieceJob& j, int64_t start, int64_t L) {
  constexpr int64_t kMask = (int64_t{1} << kSparseShift) - 1;
  bk.mn = std::min(bk.mn, L);
  bk.mx = std::max(bk.mx, L);
  bk.cells += L <= j.L1 ? (j.L1 - L + 1) * L : 0;
  if (j.sparse && (bk.tok & kMask) == 0) j.sparse[bk.tok >> kSparseShift] = start;
  if (j.len16) j.len16[bk.tok] = static_cast<uint16_t>(L < 65535 ? L : 65535);
  ++bk.tok;
}

MOC_AVX512 bool fill_piece_avx512(const PieceJob& j, PieceOut& po) {
  thread_local std::vector<uint8_t> stage_tl;
  if (j.packed && stage_tl.size() < static_cast<size_t>(kStage + 128)) stage_tl.resize(static_cast<size_t>(kStage + 128));
  Stager st{j.packed ? stage_tl.data() : nullptr, j.packed ? j.a : 0, false};  // sink[x - base] = letter x
  uint8_t* const sink_base = j.packed ? st.stage : j.codes;
  const __m512i k1F = _mm512_set1_epi8(0x1F), kDF = _mm512_set1_epi8(static_cast<char>(0xDF));
  const __m512i kA = _mm512_set1_epi8('A'), k25 = _mm512_set1_epi8(25), k9 = _mm512_set1_epi8(9);
  const __m512i k4 = _mm512_set1_epi8(4), kSp = _mm512_set1_epi8(' ');
  const int64_t L1 = j.L1, cap = j.l2_cap > 0 ? j.l2_cap : INT64_MAX;
  constexpr int64_t kMask = (int64_t{1} << kSparseShift) - 1;
  int64_t* const offs = j.offs;
  int64_t* const sparse = j.sparse;
  uint16_t* const len16 = j.len16;
  int64_t pos = j.a, tok = j.tok0, cur = -1;
  int64_t mn = INT64_MAX, mx = 0, cells = 0;
  uint64_t prev_ws = 1;
  // Without dense offsets (the narrow wire form: lengths + sparse offsets) records are booked per block:
  // the tokens that start and end inside a block get their lengths as (end byte - start byte + 1) from two
  // vpcompressb of the byte positions, stored as uint16 in one masked store, with min / max / search cells
  // accumulated in vector registers; only a token crossing a block boundary is closed by scalar code.
  const bool per_block = offs == nullptr;
  alignas(64) static constexpr uint8_t kIota[64] = {
      0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21,
      22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 36, 37, 38, 39, 40, 41, 42, 43,
      44, 45, 46, 47, 48, 49, 50, 51, 52, 53, 54, 55, 56, 57, 58, 59, 60, 61, 62, 63};
  const __m512i iota = _mm512_load_si512(reinterpret_cast<const void*>(kIota)), one8 = _mm512_set1_epi8(1);
  const __m512i vL1 = _mm512_set1_epi64(L1), vL1p1 = _mm512_set1_epi64(L1 + 1);
  __m512i vmin = _mm512_set1_epi8(static_cast<char>(0xFF)), vmax = _mm512_setzero_si512(), vcells = _mm512_setzero_si512();
  Book bk{tok, INT64_MAX, 0, 0};
  int64_t open_len = -1, open_start = 0;  // the token running past the previous block: letters so far, start
  for (size_t i = j.bb; i < j.be; i += 64) {
    const size_t nb = std::min<size_t>(64, j.be - i);
    const __mmask64 in = nb == 64 ? ~__mmask64{0} : (__mmask64{1} << nb) - 1;
    const __m512i v = _mm512_maskz_loadu_epi8(in, j.ua + i);
    const __mmask64 ws = _mm512_cmpeq_epi8_mask(v, kSp) | _mm512_cmple_epu8_mask(_mm512_sub_epi8(v, k9), k4) | ~in;
    const __mmask64 nonws = ~ws;
    const __mmask64 letter = _mm512_cmple_epu8_mask(_mm512_sub_epi8(_mm512_and_si512(v, kDF), kA), k25);
    if (nonws & ~letter) return false;  // a non-letter: the scalar encoder reports it
    const __mmask64 starts = nonws & ((ws << 1) | prev_ws);
    prev_ws = ws >> 63;
    const int cnt = static_cast<int>(_mm_popcnt_u64(nonws));
    if (j.packed && pos - st.base > kStage) stage_flush(j, po, st, pos, false);
    _mm512_mask_storeu_epi8(sink_base + (pos - st.base), cnt == 64 ? ~__mmask64{0} : (__mmask64{1} << cnt) - 1,
                            _mm512_maskz_compress_epi8(nonws, _mm512_and_si512(v, k1F)));
    if (per_block) {
      const uint64_t nw = nonws;
      uint64_t E = nw & ~(nw >> 1) & 0x7FFFFFFFFFFFFFFFull;  // last letter of a token ending in this block
      if (open_len >= 0) {
        if (!(nw & 1)) {
          close_record(bk, j, open_start, open_len);
          open_len = -1;
        } else if (E) {
          close_record(bk, j, open_start, open_len + static_cast<int64_t>(_tzcnt_u64(E)) + 1);
          E &= E - 1;
          open_len = -1;
        } else {
          open_len += 64;  // no whitespace in the block
        }
      }
      if (starts) {
        const int ns = static_cast<int>(_mm_popcnt_u64(starts)), ne = static_cast<int>(_mm_popcnt_u64(E));
        const __m512i sp = _mm512_maskz_compress_epi8(starts, iota);
        if (ne > 0) {  // ne <= 32: a token and its separator take two bytes at least
          const __m512i L8 = _mm512_add_epi8(_mm512_sub_epi8(_mm512_maskz_compress_epi8(E, iota), sp), one8);
          const __mmask64 cm = (__mmask64{1} << ne) - 1;
          vmin = _mm512_mask_min_epu8(vmin, cm, vmin, L8);
          vmax = _mm512_mask_max_epu8(vmax, cm, vmax, L8);
          if (len16)
            _mm512_mask_storeu_epi16(len16 + bk.tok, static_cast<__mmask32>(cm),
                                     _mm512_cvtepu8_epi16(_mm512_castsi512_si256(L8)));
          alignas(64) uint8_t lb[64];
          _mm512_store_si512(reinterpret_cast<void*>(lb), L8);
          for (int k = 0; k < ne; k += 8) {  // search cells (L1 + 1 - L) * L of the lengths <= L1
            const __m512i L = _mm512_cvtepu8_epi64(_mm_loadl_epi64(reinterpret_cast<const __m128i*>(lb + k)));
            const __mmask8 lm = static_cast<__mmask8>((ne - k >= 8 ? 0xFFu : (1u << (ne - k)) - 1u) &
                                                      _mm512_cmple_epu64_mask(L, vL1));
            vcells = _mm512_mask_add_epi64(vcells, lm, vcells, _mm512_mul_epu32(_mm512_sub_epi64(vL1p1, L), L));
          }
          const int64_t k0 = (-bk.tok) & kMask;  // the record of this block that opens a sparse entry (if any)
          if (sparse && k0 < ne) {
            alignas(64) uint8_t sb[64];
            _mm512_store_si512(reinterpret_cast<void*>(sb), sp);
            sparse[(bk.tok + k0) >> kSparseShift] = pos + static_cast<int64_t>(_mm_popcnt_u64(nw & ((uint64_t{1} << sb[k0]) - 1)));
          }
          bk.tok += ne;
        }
        if (ns > ne) {  // the last token runs to the block end (and possibly past it)
          open_len = 64 - (63 - static_cast<int64_t>(_lzcnt_u64(starts)));
          open_start = pos + cnt - open_len;
        }
      }
      pos += cnt;
      continue;
    }
    for (uint64_t m = starts; m; m &= m - 1) {
      const int64_t S = pos + static_cast<int64_t>(_mm_popcnt_u64(nonws & (_blsi_u64(m) - 1)));
      if (cur >= 0) {  // the previous token, letters [cur, S), is record `tok`
        const int64_t L = S - cur;
        mn = std::min(mn, L);
        mx = std::max(mx, L);
        cells += L <= L1 ? (L1 - L + 1) * L : 0;
        if (sparse && (tok & kMask) == 0) sparse[tok >> kSparseShift] = cur;
        if (len16) len16[tok] = static_cast<uint16_t>(L < 65535 ? L : 65535);
        if (offs) offs[tok + 1] = S;
        ++tok;
      }
      cur = S;
    }
    pos += cnt;
  }
  if (per_block) {
    if (open_len >= 0) close_record(bk, j, open_start, open_len);
    alignas(64) uint8_t lb[64];
    _mm512_store_si512(reinterpret_cast<void*>(lb), vmin);
    uint8_t vmn = 255, vmx = 0;
    for (int k = 0; k < 64; ++k) vmn = std::min(vmn, lb[k]);
    _mm512_store_si512(reinterpret_cast<void*>(lb), vmax);
    for (int k = 0; k < 64; ++k) vmx = std::max(vmx, lb[k]);
    mn = vmn != 255 ? std::min<int64_t>(bk.mn, vmn) : bk.mn;  // in-block lengths are <= 64: 255 = none
    mx = std::max<int64_t>(bk.mx, vmx);
    cells = bk.cells + _mm512_reduce_add_epi64(vcells);
    tok = bk.tok;
  } else if (cur >= 0) {
    const int64_t L = pos - cur;
    mn = std::min(mn, L);
    mx = std::max(mx, L);
    cells += L <= L1 ? (L1 - L + 1) * L : 0;
    if (sparse && (tok & kMask) == 0) sparse[tok >> kSparseShift] = cur;
    if (len16) len16[tok] = static_cast<uint16_t>(L < 65535 ? L : 65535);
    if (offs) offs[tok + 1] = pos;
    ++tok;
  }
  if (mx > cap) return false;  // a record over the limit: the scalar encoder reports the first one
  if (j.packed) stage_flush(j, po, st, pos, true);
  po.rep.min_len = mn;
  po.rep.max_len = mx;
  po.rep.cells = cells;
  return true;
}
}  // namespace

FillReport BulkParser::fill_slice(const AreaSlice& s, uint8_t* codes, uint8_t* packed5, int64_t* offs, int64_t* sparse,
                                  uint16_t* len16, int pack) const {
  if (pack != 5 && pack != 33) throw Error("fill_slice: pack must be 5 or 33");
  // letters per group and bytes per group of the packed stream: 8 -> 5 (5-bit), 56 -> 33 (P33: a block of
  // eight 33-bit fields)
  const bool p33 = pack == 33;
  const int64_t G = p33 ? kP33Letters : 8, GB = p33 ? kP33Bytes : 5;
  if (offs) offs[0] = 0;
  constexpr int64_t kSparseMask = (int64_t{1} << kSparseShift) - 1;
  const int np = static_cast<int>(s.pieces.size());
  const unsigned char* ua = reinterpret_cast<const unsigned char*>(area_);
  const int64_t l2_cap = l2_cap_;
  const int64_t L1 = static_cast<int64_t>(seq1_.size());
  const size_t vec_in_end = area_len_ >= 16 ? area_len_ - 16 : 0;  // 16-byte loads stay in the area
  std::vector<PieceOut> out(static_cast<size_t>(np));
  const bool simd = fill_simd_enabled();
  // one piece per iteration (dynamic): correct for any number of delivered threads; a small slice is
  // encoded on the calling thread (no team start-up for a reference-sized input)
#pragma omp parallel for schedule(dynamic, 1) if (np > 1 && s.letters > (int64_t{1} << 16))
  for (int q = 0; q < np; ++q) {
    const AreaPiece& pc = s.pieces[q];
    PieceOut& po = out[q];
    const int64_t a = pc.chr, b = q + 1 < np ? s.pieces[q + 1].chr : s.letters;  // this piece's letters [a, b)
    po.rec_base = s.first_record + pc.tok;
    if (simd) {
      const PieceJob pj{ua,    static_cast<size_t>(pc.byte_begin), static_cast<size_t>(pc.byte_end), a, b, pc.tok,
                        codes, packed5, offs, sparse, len16, G, GB, p33, l2_cap, L1};
      if (fill_piece_avx512(pj, po)) continue;
      po = PieceOut{};  // an input error in this piece: the scalar pass below finds and reports it
      po.rec_base = s.first_record + pc.tok;
    }
    std::vector<uint8_t> stage(packed5 ? static_cast<size_t>(kStage + 64) : 0);
    // sink of the encoded letters: `codes` at the slice position, else the staging buffer
    int64_t base = packed5 ? a : 0;  // slice letter index of stage[0]
    bool head_done = false;
    auto flush = [&](int64_t hi, bool final) {  // packs staged letters [base, hi) (and copies them to codes)
      if (codes) std::memcpy(codes + base, stage.data(), static_cast<size_t>(hi - base));
      int64_t cur = base;
      if (!head_done) {  // letters before the piece's first whole group: fixed up after the loop
        const int64_t g0 = (a + G - 1) / G * G, hend = std::min(g0, hi);
        if (hend < g0 && !final) return;
        for (int64_t c = cur; c < hend; ++c) po.stragglers.emplace_back(c, stage[static_cast<size_t>(c - base)]);
        cur = hend;
        head_done = true;
      }
      const int64_t ng = (hi - cur) / G;
      const uint8_t* src = stage.data() + (cur - base);
      uint8_t* dst = packed5 + GB * (cur / G);
      if (p33) {
        for (int64_t g = 0; g < ng; ++g) p33_block_full(src + kP33Letters * g, dst + kP33Bytes * g);
      } else {
        for (int64_t g = 0; g < ng; ++g) {
          uint64_t x;
          std::memcpy(&x, src + 8 * g, 8);
          x = compress8(x);
          // 8-byte stores run 3 zero bytes into the next group, which the next store rewrites; the last
          // group of the run writes its 5 bytes only (the next group may belong to another piece)
          std::memcpy(dst + 5 * g, &x, g + 1 < ng ? 8 : 5);
        }
      }
      cur += G * ng;
      if (final) {
        for (int64_t c = cur; c < hi; ++c) po.stragglers.emplace_back(c, stage[static_cast<size_t>(c - base)]);
      } else {
        std::memmove(stage.data(), stage.data() + (cur - base), static_cast<size_t>(hi - cur));
        base = cur;
      }
    };
    uint8_t* sink = packed5 ? stage.data() : codes;
    int64_t tok = pc.tok, pos = a;
    int64_t first_bad = -1, lt = -1, ll = 0, mn = INT64_MAX, mx = 0, cells = 0;
    size_t i = static_cast<size_t>(pc.byte_begin);
    const size_t e = static_cast<size_t>(pc.byte_end);
    while (i < e) {
      while (i < e && is_space(ua[i])) ++i;
      if (i >= e) break;
      const int64_t p0 = pos;
      unsigned bad = 0;
      while (true) {
        if (packed5 && pos - base > kStage) flush(pos, false);  // mid-token is fine: groups are by position
        // 16-byte SSE2 blocks wherever a full block can be read from the area and stored into the sink
        // (byte mode: within this piece's letters only — a store past them would race with the next piece)
        const int64_t lim = packed5 ? base + kStage + 48 : b;
        if (i <= vec_in_end && pos + 16 <= lim) {
          unsigned sp, ok;
          const __m128i codes16 = encode16(ua + i, sp, ok);
          _mm_storeu_si128(reinterpret_cast<__m128i*>(sink + (pos - base)), codes16);
          // letters up to the first space (or the piece end); a token of >= 16 letters takes another block
          const size_t take = std::min<size_t>(sp ? static_cast<size_t>(__builtin_ctz(sp)) : 16, e - i);
          bad |= ~ok & ((1u << take) - 1u);
          i += take;
          pos += static_cast<int64_t>(take);
          if (take < 16) break;
          continue;
        }
        // tail: near the end of the area or of the piece (or of the staging buffer)
        int64_t room = lim - pos;
        while (i < e && !is_space(ua[i]) && room-- > 0) {
          const uint8_t code = kCodeOf[ua[i++]];
          bad |= (code == 0);
          sink[pos++ - base] = code;
        }
        if (i >= e || is_space(ua[i])) break;
      }
      const int64_t L = pos - p0;
      if (bad && first_bad < 0) first_bad = tok;
      if (l2_cap > 0 && L > l2_cap && lt < 0) {
        lt = tok;
        ll = L;
      }
      mn = std::min(mn, L);
      mx = std::max(mx, L);
      cells += record_cells(L1, L);
      if (sparse && (tok & kSparseMask) == 0) sparse[tok >> kSparseShift] = p0;
      if (len16) len16[tok] = static_cast<uint16_t>(std::min<int64_t>(L, 65535));
      if (offs) offs[tok + 1] = pos;
      ++tok;
    }
    if (packed5) flush(pos, true);
    po.rep.min_len = mn;
    po.rep.max_len = mx;
    po.rep.bad_record = first_bad < 0 ? -1 : s.first_record + first_bad;
    po.rep.long_record = lt < 0 ? -1 : s.first_record + lt;
    po.rep.long_len = ll;
    po.rep.cells = cells;
  }
  FillReport r;
  for (const PieceOut& po : out) {
    r.min_len = std::min(r.min_len, po.rep.min_len);
    r.max_len = std::max(r.max_len, po.rep.max_len);
    r.cells += po.rep.cells;
    if (po.rep.bad_record >= 0 && (r.bad_record < 0 || po.rep.bad_record < r.bad_record)) r.bad_record = po.rep.bad_record;
    if (po.rep.long_record >= 0 && (r.long_record < 0 || po.rep.long_record < r.long_record)) {
      r.long_record = po.rep.long_record;
      r.long_len = po.rep.long_len;
    }
  }
  if (packed5 && p33) {
    // blocks holding letters of two pieces (or the slice's last, partial block) hold stragglers only (a piece
    // packs whole blocks): each one's letters gathered in order and encoded once (letters past the slice = 1)
    uint8_t tmp[kP33Letters];
    int64_t blk = -1;
    for (const PieceOut& po : out)
      for (const auto& sc : po.stragglers) {
        if (sc.first / kP33Letters != blk) {
          if (blk >= 0) p33_block_full(tmp, packed5 + kP33Bytes * blk);
          blk = sc.first / kP33Letters;
          std::memset(tmp, 1, sizeof tmp);
        }
        tmp[sc.first % kP33Letters] = sc.second;
      }
    if (blk >= 0) p33_block_full(tmp, packed5 + kP33Bytes * blk);
  } else if (packed5) {
    // groups holding letters of two pieces (or the slice's last, partial group): zeroed, then assembled
    for (const PieceOut& po : out)
      for (const auto& sc : po.stragglers) std::memset(packed5 + GB * (sc.first / G), 0, static_cast<size_t>(GB));
    for (const PieceOut& po : out)
      for (const auto& sc : po.stragglers) {
        const int64_t bit = 5 * sc.first;
        const uint32_t v = static_cast<uint32_t>(sc.second & 31u) << (bit & 7);
        packed5[bit >> 3] |= static_cast<uint8_t>(v);
        packed5[(bit >> 3) + 1] |= static_cast<uint8_t>(v >> 8);
      }
  }
  if (packed5) {  // read slack past the last group
    const int64_t used = GB * ((s.letters + G - 1) / G);
    const int64_t total = p33 ? packed33_bytes(s.letters) : packed5_bytes(s.letters);
    std::memset(packed5 + used, 0, static_cast<size_t>(total - used));
  }
  if (sparse) sparse[sparse_count(s.records, kSparseShift) - 1] = s.letters;
  return r;
}

void BulkParser::check(const FillReport& r) const {
  // the record a sequential reader meets first; on that record the length limit is reported first
  if (r.long_record >= 0 && (r.bad_record < 0 || r.long_record <= r.bad_record))
    throw Error("Seq2 record #" + std::to_string(r.long_record) + " has " + std::to_string(r.long_len) +
                " letters, limit is " + std::to_string(l2_cap_));
  if (r.bad_record >= 0)
    throw Error("Seq2 record #" + std::to_string(r.bad_record) + " contains a non-letter character");
  validate_score_range(weights_, std::max<int64_t>(r.max_len, 1));
}

void BulkParser::fill(uint8_t* codes, int64_t* offs) const {
  const AreaSlice s = slice(0, n_);
  if (s.records == 0) {
    offs[0] = 0;
    validate_score_range(weights_, 1);
    return;
  }
  check(fill_slice(s, codes, nullptr, offs));
}

int64_t BulkParser::mean_length_estimate() const {
  if (n_ <= 0) return 0;
  const int64_t letters = total_chars_ >= 0 ? total_chars_ : std::max<int64_t>(0, static_cast<int64_t>(area_len_) - n_);
  return letters / n_;
}

int64_t BulkParser::cells_estimate() const {
  const int64_t L1 = static_cast<int64_t>(seq1_.size());
  if (n_ <= 0) return 0;
  // before pass 1: the area's bytes less one separator per record
  const int64_t letters = total_chars_ >= 0 ? total_chars_ : std::max<int64_t>(0, static_cast<int64_t>(area_len_) - n_);
  const int64_t avg = std::max<int64_t>(1, letters / n_);
  return avg <= L1 ? n_ * (L1 - avg + 1) * avg : 0;
}

void BulkParser::chunk_costs(const std::vector<int64_t>& starts, int c0, int c1, const CostModel& m,
                             double* costs) const {
  const unsigned char* ua = reinterpret_cast<const unsigned char*>(area_);
  const int64_t L1 = static_cast<int64_t>(seq1_.size());
#pragma omp parallel for schedule(dynamic, 1) if (c1 - c0 > 1 && starts[c1] - starts[c0] > (int64_t{1} << 16))
  for (int c = c0; c < c1; ++c) {
    int64_t i = starts[c];
    const int64_t e = starts[c + 1];
    double acc = 0.0;
    while (i < e) {
      while (i < e && is_space(ua[i])) ++i;
      if (i >= e) break;
      const int64_t b = i;
      while (i < e && !is_space(ua[i])) ++i;
      acc += record_cost(L1, i - b, m);
    }
    costs[c - c0] = acc;
  }
}

void BulkParser::set_chunk_costs(std::vector<double> costs) { cost_ = std::move(costs); }

int64_t BulkParser::cost_split(int64_t first, int part, int parts, const CostModel& m) const {
  if (start_.empty()) throw Error("BulkParser::cost_split before pass 1");
  first = std::clamp<int64_t>(first, 0, n_);
  if (part <= 0 || first >= n_) return first;
  if (part >= parts) return n_;
  const int64_t L1 = static_cast<int64_t>(seq1_.size());
  const int nch = nchunks();
  const unsigned char* ua = reinterpret_cast<const unsigned char*>(area_);
  // exact cost of the records of chunk c inside [first, n) (walks the chunk's tokens); stops once the
  // running total (from `acc`) reaches `target` and returns the split record there, else -1
  auto walk = [&](int c, double& acc, double target) -> int64_t {
    const int64_t t_end = std::min(tok_pre_[c + 1], n_);
    int64_t i = start_[c], t = tok_pre_[c];
    const int64_t e = start_[c + 1];
    while (t < t_end && i < e) {
      while (i < e && is_space(ua[i])) ++i;
      const int64_t b = i;
      while (i < e && !is_space(ua[i])) ++i;
      if (t >= first) {
        const double next = acc + record_cost(L1, i - b, m);
        if (next >= target) return (target - acc) < (next - target) ? t : t + 1;
        acc = next;
      }
      ++t;
    }
    return -1;
  };
  // chunk costs: exact ones from pass 1 (chunk_costs) for chunks wholly inside [first, n), a walk for the
  // two boundary chunks, else the records at the chunk's mean length
  std::vector<double> pre(static_cast<size_t>(nch) + 1, 0.0);
  for (int c = 0; c < nch; ++c) {
    const int64_t t0 = std::max(tok_pre_[c], first), t1 = std::min(tok_pre_[c + 1], n_);
    const int64_t toks = tok_pre_[c + 1] - tok_pre_[c];
    double est = 0.0;
    if (t1 > t0) {
      if (t1 - t0 < toks) {
        walk(c, est, std::numeric_limits<double>::infinity());
      } else if (!cost_.empty()) {
        est = cost_[static_cast<size_t>(c)];
      } else {
        const int64_t avg = (chr_pre_[c + 1] - chr_pre_[c] + toks / 2) / toks;
        est = static_cast<double>(toks) * record_cost(L1, avg, m);
      }
    }
    pre[c + 1] = pre[c] + est;
  }
  const double target = pre[nch] * part / parts;
  if (target <= 0.0) return first;
  const int c = static_cast<int>(std::lower_bound(pre.begin() + 1, pre.end(), target) - pre.begin()) - 1;
  if (c >= nch) return n_;
  double acc = pre[c];  // exact inside the chunk holding the target
  const int64_t t = walk(c, acc, target);
  return t >= 0 ? t : std::max(first, std::min(tok_pre_[c + 1], n_));
}

Problem parse_problem(const char* data, size_t len, const ParseOptions& opt) {
  BulkParser p(data, len, opt);
  Problem prob;
  prob.weights = p.weights();
  prob.seq1 = p.seq1();
  prob.seq2.codes.resize(static_cast<size_t>(p.total_chars()));  // uninitialised: fill writes every byte
  prob.seq2.offsets.resize(static_cast<size_t>(p.count()) + 1);
  p.fill(prob.seq2.codes.data(), prob.seq2.offsets.data());
  return prob;
}

// ---- streaming reader ---------------------------------------------------------------------------

StreamReader::StreamReader(FILE* f, const ParseOptions& opt, size_t block_bytes) : f_(f), opt_(opt) {
  buf_.resize(std::max<size_t>(block_bytes, 4096));
  const char *b, *e;
  static const char* wname[4] = {"W1", "W2", "W3", "W4"};
  for (int i = 0; i < 4; ++i) {
    if (!token(b, e)) throw Error(std::string("unexpected end of input while reading ") + wname[i]);
    int64_t v = parse_int(b, e, wname[i]);
    if (v < 0 || v > INT32_MAX) throw Error(std::string(wname[i]) + " out of range");
    weights_.w[i] = static_cast<int32_t>(v);
  }
  if (!token(b, e)) throw Error("unexpected end of input while reading Seq1");
  seq1_ = encode_sequence(b, e - b);
  if (!token(b, e)) throw Error("unexpected end of input while reading the number of sequences");
  count_ = parse_int(b, e, "number_of_sequences");
  if (count_ < 0) throw Error("number_of_sequences must be >= 0");
  const int64_t l1_cap = opt_.strict_limits ? kSpecMaxSeq1 : opt_.max_l1;
  l2_cap_ = opt_.strict_limits ? kSpecMaxSeq2 : opt_.max_l2;
  if (l1_cap > 0 && static_cast<int64_t>(seq1_.size()) > l1_cap)
    throw Error("Seq1 has " + std::to_string(seq1_.size()) + " letters, limit is " + std::to_string(l1_cap));
}

bool StreamReader::token(const char*& b, const char*& e) {
  // skip whitespace
  while (true) {
    while (pos_ < len_ && is_space(static_cast<unsigned char>(buf_[pos_]))) ++pos_;
    if (pos_ < len_) break;
    if (eof_) return false;
    pos_ = len_ = 0;
    len_ = std::fread(buf_.data(), 1, buf_.size(), f_);
    if (len_ < buf_.size()) {
      if (std::ferror(f_)) throw Error("error while reading input stream");
      eof_ = true;
    }
  }
  // token [pos_, q); extend the buffer while it runs into the end of the loaded data
  size_t q = pos_;
  while (true) {
    while (q < len_ && !is_space(static_cast<unsigned char>(buf_[q]))) ++q;
    if (q < len_ || eof_) break;
    // move the partial token to the front (grow if it fills the buffer) and read more
    const size_t keep = len_ - pos_;
    if (pos_ > 0) std::memmove(buf_.data(), buf_.data() + pos_, keep);
    if (keep == buf_.size()) buf_.resize(buf_.size() * 2);
    q = keep;
    pos_ = 0;
    const size_t got = std::fread(buf_.data() + keep, 1, buf_.size() - keep, f_);
    len_ = keep + got;
    if (len_ < buf_.size()) {
      if (std::ferror(f_)) throw Error("error while reading input stream");
      eof_ = true;
    }
  }
  b = buf_.data() + pos_;
  e = buf_.data() + q;
  pos_ = q;
  return true;
}

bool StreamReader::take_rest(uvector<char>& out) {
  const size_t at = out.size();
  out.resize(at + (len_ - pos_));
  if (len_ > pos_) std::memcpy(out.data() + at, buf_.data() + pos_, len_ - pos_);
  pos_ = len_;
  return eof_;
}

int64_t StreamReader::skip(int64_t records) {
  const char *b, *e;
  int64_t done = 0;
  while (done < records && next_ < count_) {
    if (!token(b, e))
      throw Error("expected " + std::to_string(count_) + " Seq2 records, found only " + std::to_string(next_));
    ++next_;
    ++done;
  }
  return done;
}

int64_t StreamReader::next_batch(int64_t max_records, RecordBatch& out, int64_t max_chars) {
  // Region by region: the loaded buffer's complete tokens are split into per-thread chunks at
  // whitespace, counted (tokens, letters) in parallel, cut where the batch ends (max_records, or the first
  // record that starts with >= max_chars letters already in the batch), then encoded in parallel. Errors
  // name the smallest offending record, the length check first, as a record-by-record scan would.
  out.codes.clear();
  out.offsets.assign(1, 0);
  const int64_t want = std::min(max_records, count_ - next_);
  int64_t got = 0, max_len = 0;
  auto missing = [&] {
    return Error("expected " + std::to_string(count_) + " Seq2 records, found only " + std::to_string(next_));
  };
  while (got < want) {
    if (got > 0 && static_cast<int64_t>(out.codes.size()) >= max_chars) break;
    // ---- the region [pos_, cut) of complete tokens (refill / grow until there is one, or EOF)
    while (pos_ < len_ && is_space(static_cast<unsigned char>(buf_[pos_]))) ++pos_;
    size_t cut = 0;
    while (true) {
      if (pos_ < len_) {
        if (eof_) {
          cut = len_;
        } else {
          cut = len_;
          while (cut > pos_ && !is_space(static_cast<unsigned char>(buf_[cut - 1]))) --cut;
        }
        if (cut > pos_) break;
      } else if (eof_) {
        throw missing();
      }
      const size_t keep = len_ - pos_;  // a partial token (or nothing) moves to the front
      if (pos_ > 0 && keep) std::memmove(buf_.data(), buf_.data() + pos_, keep);
      if (keep == buf_.size()) buf_.resize(buf_.size() * 2);
      pos_ = 0;
      // a regular file refills with parallel preads (one fread is a single-threaded copy out of the page
      // cache: it was the streaming mode's critical path at 1.1 G letters)
      const size_t rd = read_regular_into(f_, buf_.data() + keep, buf_.size() - keep);
      len_ = keep + rd;
      if (len_ < buf_.size()) {
        if (std::ferror(f_)) throw Error("error while reading input stream");
        eof_ = true;
      }
      while (pos_ < len_ && is_space(static_cast<unsigned char>(buf_[pos_]))) ++pos_;
    }
    const unsigned char* ua = reinterpret_cast<const unsigned char*>(buf_.data());
    const size_t rlen = cut - pos_;
    const int nt = rlen > (size_t{1} << 20) ? std::max(1, omp_get_max_threads()) : 1;
    std::vector<size_t> cb(static_cast<size_t>(nt) + 1);
    for (int t = 0; t <= nt; ++t) cb[t] = pos_ + rlen * static_cast<size_t>(t) / nt;
    for (int t = 1; t < nt; ++t) {  // chunk starts move forward past the token they cut
      size_t x = cb[t];
      while (x < cut && !is_space(ua[x - 1])) ++x;
      cb[t] = std::max(x, cb[t - 1]);
    }
    cb[nt] = cut;
    std::vector<int64_t> ctok(static_cast<size_t>(nt) + 1, 0), cchr(static_cast<size_t>(nt) + 1, 0);
#pragma omp parallel for num_threads(nt) schedule(static, 1)
    for (int t = 0; t < nt; ++t) {
      int64_t k = 0, c = 0;
      if (cb[t] < cb[t + 1]) {
        k = c = is_space(ua[cb[t]]) ? 0 : 1;
        for (size_t i = cb[t] + 1; i < cb[t + 1]; ++i) {
          const unsigned lt = !is_space(ua[i]);
          k += lt & is_space(ua[i - 1]);
          c += lt;
        }
      }
      ctok[t + 1] = k;
      cchr[t + 1] = c;
    }
    // ---- where this batch ends inside the region: whole chunks, then a token scan of the last one
    const int64_t base_chars = static_cast<int64_t>(out.codes.size());
    int64_t tk = 0, ch = 0;  // tokens / letters taken from the region so far
    int last = nt;           // chunks [0, last) are taken whole
    size_t end_pos = cut;
    for (int t = 0; t < nt; ++t) {
      // whole chunk: it stays within the record limit, and even its last token (which starts at most
      // one letter before the chunk's end) starts below max_chars
      const bool whole = ctok[t + 1] == 0 ||
                         (got + tk + ctok[t + 1] <= want && base_chars + ch + cchr[t + 1] - 1 < max_chars);
      if (whole) {
        tk += ctok[t + 1];
        ch += cchr[t + 1];
        continue;
      }
      // token scan of chunk t
      size_t i = cb[t];
      const size_t e = cb[t + 1];
      while (got + tk < want) {
        while (i < e && is_space(ua[i])) ++i;
        if (i >= e) break;
        if (got + tk > 0 && base_chars + ch >= max_chars) break;
        size_t j = i;
        while (j < e && !is_space(ua[j])) ++j;
        ++tk;
        ch += static_cast<int64_t>(j - i);
        i = j;
      }
      end_pos = i;
      last = t;
      break;
    }
    if (last < nt) cb[last + 1] = end_pos;  // chunk `last` is encoded up to the cut; later ones not at all
    const int nenc = last < nt ? last + 1 : nt;
    // per-chunk prefix of the (possibly truncated) counts
    if (last < nt) {
      int64_t k0 = 0, c0 = 0;
      for (int t = 0; t < last; ++t) {
        k0 += ctok[t + 1];
        c0 += cchr[t + 1];
      }
      ctok[last + 1] = tk - k0;
      cchr[last + 1] = ch - c0;
    }
    for (int t = 0; t < nenc; ++t) {
      ctok[t + 1] += ctok[t];
      cchr[t + 1] += cchr[t];
    }
    // ---- encode (parallel), checking lengths and letters
    const size_t at_tok = out.offsets.size() - 1;
    out.codes.resize(static_cast<size_t>(base_chars + ch));
    out.offsets.resize(at_tok + 1 + static_cast<size_t>(tk));
    uint8_t* codes = out.codes.data() + base_chars;
    int64_t* offs = out.offsets.data() + at_tok;
    std::vector<int64_t> err_tok(static_cast<size_t>(nenc), -1), err_len(static_cast<size_t>(nenc), 0),
        mx(static_cast<size_t>(nenc), 0);
    std::vector<int> err_kind(static_cast<size_t>(nenc), 0);
#pragma omp parallel for num_threads(nt) schedule(static, 1)
    for (int t = 0; t < nenc; ++t) {
      int64_t k = ctok[t], pos = cchr[t], m = 0;
      size_t i = cb[t];
      const size_t e = cb[t + 1];
      while (i < e) {
        while (i < e && is_space(ua[i])) ++i;
        if (i >= e) break;
        const int64_t p0 = pos;
        unsigned bad = 0;
        while (i < e && !is_space(ua[i])) {
          const uint8_t code = kCodeOf[ua[i++]];
          bad |= (code == 0);
          codes[pos++] = code;
        }
        const int64_t L = pos - p0;
        if (err_tok[t] < 0 && ((l2_cap_ > 0 && L > l2_cap_) || bad)) {
          err_tok[t] = k;
          err_kind[t] = (l2_cap_ > 0 && L > l2_cap_) ? 1 : 2;
          err_len[t] = L;
        }
        m = std::max(m, L);
        offs[++k] = base_chars + pos;
      }
      mx[t] = m;
    }
    for (int t = 0; t < nenc; ++t) {
      if (err_tok[t] >= 0) {
        const int64_t rec = next_ + err_tok[t];
        if (err_kind[t] == 1)
          throw Error("Seq2 record #" + std::to_string(rec) + " has " + std::to_string(err_len[t]) +
                      " letters, limit is " + std::to_string(l2_cap_));
        throw Error("Seq2 record #" + std::to_string(rec) + " contains a non-letter character");
      }
      max_len = std::max(max_len, mx[t]);
    }
    pos_ = end_pos;
    next_ += tk;
    got += tk;
  }
  if (got) validate_score_range(weights_, std::max<int64_t>(max_len, 1));
  return got;
}

// ---- writer -------------------------------------------------------------------------------------

namespace {
// ---- result rows: "#<idx>: score: <s>, n: <n>, k: <k>\n" (main.c:204), formatted without printf:
// two-digit table for the numbers, and a running decimal counter for the row index (consecutive rows
// differ in the last digit(s) only, so no division per row for the longest number).
constexpr char kDigitPairs[201] =
    "00010203040506070809101112131415161718192021222324252627282930313233343536373839"
    "40414243444546474849505152535455565758596061626364656667686970717273747576777879"
    "8081828384858687888990919293949596979899";

// Every writer below may store up to kSlack bytes past the text it emits (fixed-size copies instead of
// variable-length memcpy calls); each row's next piece overwrites them, and buffers carry kSlack spare.
constexpr int kSlack = 64;

inline char* put_uint(char* p, uint64_t u) {
  if (u < 10) {
    *p = static_cast<char>('0' + u);
    return p + 1;
  }
  if (u < 100) {
    std::memcpy(p, kDigitPairs + 2 * u, 2);
    return p + 2;
  }
  char tmp[48];
  char* e = tmp + 24;
  char* q = e;
  while (u >= 100) {
    const unsigned d = static_cast<unsigned>(u % 100);
    u /= 100;
    q -= 2;
    q[0] = kDigitPairs[2 * d];
    q[1] = kDigitPairs[2 * d + 1];
  }
  if (u >= 10) {
    q -= 2;
    q[0] = kDigitPairs[2 * u];
    q[1] = kDigitPairs[2 * u + 1];
  } else {
    *--q = static_cast<char>('0' + u);
  }
  std::memcpy(p, q, 24);  // fixed size: at most 20 digits, the rest is slack
  return p + (e - q);
}
inline char* put_int(char* p, int64_t v) {
  if (v < 0) {
    *p++ = '-';
    return put_uint(p, static_cast<uint64_t>(-(v + 1)) + 1);
  }
  return put_uint(p, static_cast<uint64_t>(v));
}
template <size_t N>
inline char* put_lit(char* p, const char (&s)[N]) {
  std::memcpy(p, s, N - 1);
  return p + N - 1;
}

// Decimal counter for the row index: digits live right-aligned in buf[0, 20).
struct RowCounter {
  char buf[48];  // [20, 48): padding read by the fixed-size copy in put()
  int first;     // index of the most significant digit
  explicit RowCounter(int64_t v) {
    char tmp[48];
    char* e = put_uint(tmp, static_cast<uint64_t>(v));
    const int n = static_cast<int>(e - tmp);
    first = 20 - n;
    std::memset(buf, 0, sizeof buf);
    std::memcpy(buf + first, tmp, static_cast<size_t>(n));
  }
  char* put(char* p) const {
    std::memcpy(p, buf + first, 24);
    return p + (20 - first);
  }
  void next() {
    int i = 19;
    while (i >= first && buf[i] == '9') buf[i--] = '0';
    if (i >= first) {
      ++buf[i];
    } else {
      buf[--first] = '1';
    }
  }
};

inline char* format_row(char* p, RowCounter& idx, const Result& r) {
  *p++ = '#';
  p = idx.put(p);
  idx.next();
  p = put_lit(p, ": score: ");
  p = put_int(p, r.score);
  p = put_lit(p, ", n: ");
  p = put_int(p, r.n);
  p = put_lit(p, ", k: ");
  p = put_int(p, r.k);
  *p++ = '\n';
  return p;
}
// '#' + 19 index digits + ": score: " + 11 + ", n: " + 11 + ", k: " + 11 + '\n'
constexpr int kMaxRow = 1 + 19 + 9 + 11 + 5 + 11 + 5 + 11 + 1;

// R2 results take at most 65 536 distinct values, so a large R2 run prints from a table of every code's
// row tail ": score: S, n: N, k: K\n" (one 48-byte slot each, built in parallel once per parameter set):
// a row is then '#', the index counter and one fixed-size copy (no decode divisions, no digit loops).
struct R2Tails {
  static constexpr int kSlot = 48;  // longest tail: 9 + 6 + 5 + 6 + 5 + 6 + 1 = 38 bytes
  R2Params r2;
  uvector<char> text;        // 65536 * kSlot
  std::vector<uint8_t> len;  // tail length per code
  explicit R2Tails(const R2Params& p) : r2(p), text(size_t{65536} * kSlot), len(65536) {
#pragma omp parallel for schedule(static)
    for (int c = 0; c < 65536; ++c) {
      const uint16_t code = static_cast<uint16_t>(c);
      const Result x = decode_result(&code, ResultFormat::R2, r2, 0);
      char tmp[kSlot + kSlack + 64];
      char* q = put_lit(tmp, ": score: ");
      q = put_int(q, x.score);
      q = put_lit(q, ", n: ");
      q = put_int(q, x.n);
      q = put_lit(q, ", k: ");
      q = put_int(q, x.k);
      *q++ = '\n';
      std::memcpy(text.data() + size_t{kSlot} * c, tmp, kSlot);
      len[c] = static_cast<uint8_t>(q - tmp);
    }
  }
};

// Rows of a sequence of result runs (one per rank slice, each in its own wire format), by global row.
struct RowSource {
  const std::vector<ResultRun>& runs;
  std::vector<int64_t> pre;  // pre[r] = rows before run r
  std::vector<std::shared_ptr<const R2Tails>> tails;  // per run: table path for large R2 runs
  explicit RowSource(const std::vector<ResultRun>& r) : runs(r), pre(r.size() + 1, 0), tails(r.size()) {
    for (size_t i = 0; i < r.size(); ++i) {
      pre[i + 1] = pre[i] + r[i].n;
      if (r[i].fmt != ResultFormat::R2 || r[i].n < (int64_t{1} << 18) || r[i].r2.j <= 0 || r[i].r2.kw <= 0) continue;
      for (size_t q = 0; q < i && !tails[i]; ++q)  // ranks of one job usually share the parameters
        if (tails[q] && tails[q]->r2.smin == r[i].r2.smin && tails[q]->r2.kw == r[i].r2.kw && tails[q]->r2.j == r[i].r2.j)
          tails[i] = tails[q];
      if (!tails[i]) tails[i] = std::make_shared<const R2Tails>(r[i].r2);
    }
  }
  int64_t total() const { return pre.back(); }
  // formats rows [rb, re) at p (writes up to kSlack bytes past the returned end)
  char* format(char* p, int64_t rb, int64_t re, int64_t first_index) const {
    RowCounter idx(first_index + rb);
    size_t r = static_cast<size_t>(std::upper_bound(pre.begin(), pre.end(), rb) - pre.begin()) - 1;
    for (int64_t i = rb; i < re;) {
      while (r + 1 < pre.size() && pre[r + 1] <= i) ++r;
      const ResultRun& run = runs[r];
      const int64_t e = std::min(re, pre[r + 1]);
      int64_t j = i - pre[r];
      if (tails[r]) {
        const uint16_t* codes = static_cast<const uint16_t*>(run.data);
        const char* text = tails[r]->text.data();
        const uint8_t* len = tails[r]->len.data();
        for (; i < e; ++i, ++j) {
          const unsigned c = codes[j];
          *p = '#';
          p = idx.put(p + 1);
          idx.next();
          std::memcpy(p, text + size_t{R2Tails::kSlot} * c, R2Tails::kSlot);
          p += len[c];
        }
      } else {
        for (; i < e; ++i, ++j) p = format_row(p, idx, decode_result(run.data, run.fmt, run.r2, j));
      }
    }
    return p;
  }
};
}  // namespace

std::string format_results(const Result* results, int64_t n, int64_t first_index) {
  const std::vector<ResultRun> runs = {ResultRun{results, ResultFormat::R12, R2Params{}, n}};
  const RowSource src(runs);
  const int parts_n = n > 65536 ? std::max(1, omp_get_max_threads()) : 1;
  std::vector<std::string> parts(static_cast<size_t>(parts_n));
  // iterations are parts, not thread ids: every part is formatted whatever number of threads runs
#pragma omp parallel for schedule(static, 1) num_threads(parts_n)
  for (int t = 0; t < parts_n; ++t) {
    const int64_t b = n * t / parts_n, e = n * (t + 1) / parts_n;
    std::string& s = parts[t];
    s.resize(static_cast<size_t>(e - b) * kMaxRow + kSlack);
    char* p = src.format(s.data(), b, e, first_index);
    s.resize(static_cast<size_t>(p - s.data()));
  }
  size_t total = 0;
  for (auto& s : parts) total += s.size();
  std::string out;
  out.reserve(total);
  for (auto& s : parts) out += s;
  return out;
}

void write_results(FILE* f, const Result* results, int64_t n, int64_t first_index) {
  write_results(f, std::vector<ResultRun>{ResultRun{results, ResultFormat::R12, R2Params{}, n}}, first_index);
}

void write_results(FILE* f, const std::vector<ResultRun>& runs, int64_t first_index) {
  // Rows are formatted in parallel into per-part buffers (never zero-filled, never concatenated), decoding
  // each run's wire format on the fly (R2 through a table of row tails, R4/R8 straight from the ranks'
  // result slices, no expansion). Blocks of 64 K rows per part keep the buffers small (~2 MB per part,
  // reused): page-faulting fresh multi-100 MB buffers cost more than the formatting (1.2 s of 1.6 s for
  // 33 M rows here). A regular file gets each part written at its own offset (pwrite, in parallel; a
  // shared file mapping with parallel page faults was 4.6x slower on the MI355X box's /tmp,
  // tools/write_probe.cpp). Anything else (under mpiexec stdout is a pipe to the MPICH proxy) is written
  // by one background thread in order, double-buffered: block k goes out while block k+1 is formatted.
  // Parallel loops iterate over parts, not thread ids (OMP_DYNAMIC / thread limits deliver fewer threads).
  const RowSource src(runs);
  const int64_t n = src.total();
  const int nparts = n > 65536 ? std::max(1, omp_get_max_threads()) : 1;
  const int64_t kBlock = int64_t{65536} * nparts;
  std::fflush(f);
  const int fd = fileno(f);
  struct stat st;
  off_t file_pos = -1;
  // (not with O_APPEND: Linux pwrite then ignores the offset)
  const int fl = fcntl(fd, F_GETFL);
  if (fl >= 0 && !(fl & O_APPEND) && fstat(fd, &st) == 0 && S_ISREG(st.st_mode)) file_pos = lseek(fd, 0, SEEK_CUR);
  // regular files: every part is written at its own offset by the thread that formatted it (parallel
  // pwrite measured faster than one ordered writer on tmpfs: 0.32 vs 0.40 s for 20 M rows here);
  // MOC_WRITER=ordered selects the ordered background writer for them too (A/B)
  const char* wenv = std::getenv("MOC_WRITER");
  const bool parallel_file = file_pos >= 0 && nparts > 1 && !(wenv && std::strcmp(wenv, "ordered") == 0);
  const bool async = !parallel_file && n > kBlock;
  std::vector<uvector<char>> part_sets[2];
  std::vector<size_t> used_sets[2];
  for (int s2 = 0; s2 < (async ? 2 : 1); ++s2) {
    part_sets[s2].resize(static_cast<size_t>(nparts));
    used_sets[s2].assign(static_cast<size_t>(nparts) + 1, 0);
  }
  std::atomic<bool> write_error{false};
  // writes one formatted block in order (the writer thread, or inline for small outputs)
  auto write_block = [f, fd, nparts, &file_pos, &write_error](const std::vector<uvector<char>>& parts,
                                                               const std::vector<size_t>& used) {
    for (int t = 0; t < nparts && !write_error; ++t) {
      const size_t len = used[t + 1];
      if (file_pos < 0) {
        if (std::fwrite(parts[t].data(), 1, len, f) != len) write_error = true;
        continue;
      }
      for (size_t done = 0; done < len;) {
        const ssize_t w = pwrite(fd, parts[t].data() + done, len - done, file_pos);
        if (w <= 0) {
          write_error = true;
          break;
        }
        done += static_cast<size_t>(w);
        file_pos += static_cast<off_t>(w);
      }
    }
  };
  BackgroundReleaser writer;  // FIFO worker: the ordered writes
  int set = 0;
  for (int64_t b = 0; b < n && !write_error; b += kBlock) {
    const int64_t e = std::min(n, b + kBlock), m = e - b;
    std::vector<uvector<char>>& parts = part_sets[set];
    std::vector<size_t>& used = used_sets[set];
#pragma omp parallel for schedule(static, 1) num_threads(nparts)
    for (int t = 0; t < nparts; ++t) {
      const int64_t rb = b + m * t / nparts, re = b + m * (t + 1) / nparts;
      uvector<char>& buf = parts[t];
      buf.resize(static_cast<size_t>(re - rb) * kMaxRow + kSlack);
      char* p = src.format(buf.data(), rb, re, first_index);
      used[t + 1] = static_cast<size_t>(p - buf.data());
    }
    if (parallel_file) {
      used[0] = 0;
      for (int q = 0; q < nparts; ++q) used[q + 1] += used[q];  // used[t] = byte offset of part t
#pragma omp parallel for schedule(static, 1) num_threads(nparts)
      for (int t = 0; t < nparts; ++t) {
        const size_t len = used[t + 1] - used[t];
        for (size_t done = 0; done < len;) {
          const ssize_t w =
              pwrite(fd, parts[t].data() + done, len - done, file_pos + static_cast<off_t>(used[t] + done));
          if (w <= 0) {
            write_error = true;
            break;
          }
          done += static_cast<size_t>(w);
        }
      }
      file_pos += static_cast<off_t>(used[nparts]);
    } else if (async) {
      writer.drain();  // the previous block (the other buffer set) is out: that set is free again
      writer.defer([&write_block, &parts, &used] { write_block(parts, used); });
      set ^= 1;
    } else {
      write_block(parts, used);
    }
  }
  writer.stop();
  if (file_pos >= 0 && lseek(fd, file_pos, SEEK_SET) < 0) write_error = true;
  if (write_error) throw Error("error while writing the results");
  std::fflush(f);
}

namespace {
inline int64_t dec_digits(uint64_t u) {
  int64_t d = 1;
  while (u >= 10) {
    u /= 10;
    ++d;
  }
  return d;
}
inline int64_t int_chars(int64_t v) { return v < 0 ? 1 + dec_digits(static_cast<uint64_t>(-(v + 1)) + 1) : dec_digits(static_cast<uint64_t>(v)); }
// total decimal digits of the integers [a, b)
int64_t digits_of_range(int64_t a, int64_t b) {
  int64_t total = 0;
  for (int64_t lo = 1, d = 1; lo <= b && d <= 19; lo *= 10, ++d) {
    const int64_t hi = d == 19 ? INT64_MAX : lo * 10;  // numbers with d digits: [lo, hi) (0 counts as 1 digit)
    const int64_t s = std::max(a, d == 1 ? int64_t{0} : lo), e = std::min(b, hi);
    if (e > s) total += d * (e - s);
  }
  return total;
}
}  // namespace

int64_t formatted_bytes(const std::vector<ResultRun>& runs, int64_t first_index) {
  const RowSource src(runs);
  const int64_t n = src.total();
  int64_t tails = 0;
  for (size_t r = 0; r < runs.size(); ++r) {
    const ResultRun& run = runs[r];
    int64_t t = 0;
    if (src.tails[r]) {
      const uint16_t* codes = static_cast<const uint16_t*>(run.data);
      const uint8_t* len = src.tails[r]->len.data();
#pragma omp parallel for reduction(+ : t) schedule(static) if (run.n > 65536)
      for (int64_t i = 0; i < run.n; ++i) t += len[codes[i]];
    } else {
#pragma omp parallel for reduction(+ : t) schedule(static) if (run.n > 65536)
      for (int64_t i = 0; i < run.n; ++i) {
        const Result x = decode_result(run.data, run.fmt, run.r2, i);
        t += 9 + int_chars(x.score) + 5 + int_chars(x.n) + 5 + int_chars(x.k) + 1;
      }
    }
    tails += t;
  }
  return n + digits_of_range(first_index, first_index + n) + tails;  // '#' + index + tail per row
}

int64_t write_results_at(int fd, int64_t at, const std::vector<ResultRun>& runs, int64_t first_index) {
  // write_results' parallel-file path at a given offset: several processes fill one file, each its rows
  const RowSource src(runs);
  const int64_t n = src.total();
  const int nparts = n > 65536 ? std::max(1, omp_get_max_threads()) : 1;
  const int64_t kBlock = int64_t{65536} * nparts;
  std::vector<uvector<char>> parts(static_cast<size_t>(nparts));
  std::vector<size_t> used(static_cast<size_t>(nparts) + 1, 0);
  std::atomic<bool> write_error{false};
  int64_t pos = at;
  for (int64_t b = 0; b < n && !write_error; b += kBlock) {
    const int64_t e = std::min(n, b + kBlock), m = e - b;
#pragma omp parallel for schedule(static, 1) num_threads(nparts)
    for (int t = 0; t < nparts; ++t) {
      const int64_t rb = b + m * t / nparts, re = b + m * (t + 1) / nparts;
      uvector<char>& buf = parts[t];
      buf.resize(static_cast<size_t>(re - rb) * kMaxRow + kSlack);
      char* p = src.format(buf.data(), rb, re, first_index);
      used[t + 1] = static_cast<size_t>(p - buf.data());
    }
    used[0] = 0;
    for (int q = 0; q < nparts; ++q) used[q + 1] += used[q];
#pragma omp parallel for schedule(static, 1) num_threads(nparts)
    for (int t = 0; t < nparts; ++t) {
      const size_t len = used[t + 1] - used[t];
      for (size_t done = 0; done < len;) {
        const ssize_t w = pwrite(fd, parts[t].data() + done, len - done, pos + static_cast<off_t>(used[t] + done));
        if (w <= 0) {
          write_error = true;
          break;
        }
        done += static_cast<size_t>(w);
      }
    }
    pos += static_cast<int64_t>(used[nparts]);
  }
  if (write_error) throw Error("error while writing the results");
  return pos - at;
}

}  // namespace moc
