// Wire formats of the search: how letters, record lengths and results travel between host memory, the
// GPU and the ranks. Host-only and ROCm-free, so the `final` binary (which links no ROCm library) can
// write the narrow input formats in its parser and print straight from the narrow result formats.
//
// Reference: one byte per letter in a fixed 2000-byte stride per record (main.c:93, scattered whole at
// main.c:174) and three separate int arrays of results (main.c:123-125, gathered at main.c:195-197).
//
//   letters  33-bit fields of 7 letters (moc::pack33, 4.714 bits per letter), the 5-bit packed stream
//            (char j at bits [5j, 5j+5), little endian: moc::pack5), or bytes (problem.hpp)
//   lengths  8-, 4- (two per byte, low nibble first) or 3-bit (bits [3i, 3i+3), LSB first) above a base
//   results  R12 (moc::Result) / R8 / R4 / R2 (one uint16 mixed-radix code per record)
#pragma once

#include <cstdint>
#include <vector>

#include "moc/common.hpp"
#include "moc/problem.hpp"

namespace moc {

// Result wire formats (device -> host). R12 is moc::Result; R8/R4/R2 are chosen automatically when the
// problem's bounds fit, to cut the D2H bytes per record by 1.5x / 3x / 6x.
enum class ResultFormat : int32_t { R12 = 0, R8 = 1, R4 = 2, R2 = 3 };
struct R8 {
  int32_t score;
  uint16_t n, k;
};
struct R4 {
  int16_t score;  // INT16_MIN encodes "no candidate" (INT_MIN)
  uint8_t n, k;
};
static_assert(sizeof(R8) == 8 && sizeof(R4) == 4, "packed result formats");
// R2: one uint16 per record, code = (score - smin) * j + n * kw + k (mixed radix), 0xFFFF = no
// candidate. Valid for a batch whose lengths lie in the [min_l2, max_l2] the parameters were made for.
struct R2Params {
  int32_t smin = 0;  // lowest possible score
  int32_t kw = 0;    // radix of k (>= max_l2)
  int32_t j = 0;     // radix of the score code (> every n * kw + k)
};
constexpr uint16_t kR2None = 0xFFFF;
inline int result_bytes(ResultFormat f) {
  return f == ResultFormat::R12 ? 12 : f == ResultFormat::R8 ? 8 : f == ResultFormat::R4 ? 4 : 2;
}
// R2 parameters for a problem (L1, pair-score range [min_t, max_t]) and a record-length range; false
// when the codes would not fit 16 bits.
bool r2_params(int64_t L1, int64_t min_l2, int64_t max_l2, int32_t min_t, int32_t max_t, R2Params& p);
// Smallest of R12/R8/R4 able to hold every result of a problem with these bounds.
ResultFormat pick_result_format(int64_t L1, int64_t max_l2, int32_t max_abs_weight);
// Expands packed results to moc::Result (host side); `r2` is required for R2.
void expand_results(const void* in, ResultFormat f, int64_t n, Result* out, const R2Params* r2 = nullptr);

// Row i of a result array in format f.
inline Result decode_result(const void* in, ResultFormat f, const R2Params& r2, int64_t i) {
  switch (f) {
    case ResultFormat::R2: {
      const uint16_t c = static_cast<const uint16_t*>(in)[i];
      if (c == kR2None) return no_candidate();
      const int32_t idx = c % r2.j;
      return Result{c / r2.j + r2.smin, idx / r2.kw, idx % r2.kw};
    }
    case ResultFormat::R4: {
      const R4 x = static_cast<const R4*>(in)[i];
      return Result{x.score == INT16_MIN ? kNoCandidateScore : x.score, x.n, x.k};
    }
    case ResultFormat::R8: {
      const R8 x = static_cast<const R8*>(in)[i];
      return Result{x.score, x.n, x.k};
    }
    default:
      return static_cast<const Result*>(in)[i];
  }
}

// A run of consecutive results in one wire format (e.g. one rank's slice of a job, printed in order).
struct ResultRun {
  const void* data = nullptr;
  ResultFormat fmt = ResultFormat::R12;
  R2Params r2{};
  int64_t n = 0;
};

// ---- narrow record lengths -------------------------------------------------------------------------
// `bits` 6 is not a bit width but the base-6 form: lengths of at most 6 values above the base, 8 records'
// lengths as one 21-bit base-6 number (6^8 = 1 679 616 < 2^21, record 8o+j as digit j of octet o), three
// octets per aligned little-endian 64-bit word (bits [21f, 21f+21)): 2.667 bits per length (log2 6 = 2.585)
// against 3 for the 3-bit fields; the kernels load a tile's words with aligned 8-byte loads.
constexpr int kLenBase6 = 6;
// Bytes of n lengths at `bits` (3: + one readable slack byte, the kernels load two bytes per length).
inline int64_t narrow_lengths_bytes(int64_t n, int bits) {
  return bits == kLenBase6 ? 8 * ((n + 23) / 24) : bits == 3 ? (3 * n + 7) / 8 + 1 : bits == 4 ? (n + 1) / 2 : n;
}
// Narrowest of base-6 / 3 / 4 / 8 bits able to hold lengths in [min_l2, max_l2] above base min_l2; 0 when none does.
inline int narrow_length_bits(int64_t min_l2, int64_t max_l2) {
  const int64_t span = max_l2 - min_l2;
  return span <= 5 ? kLenBase6 : span <= 7 ? 3 : span <= 15 ? 4 : max_l2 <= 255 ? 8 : 0;
}
// lengths from CSR offsets (offsets[i+1] - offsets[i] - base) -> out[0..narrow_lengths_bytes(n, bits)),
// OpenMP over groups of 8 records (no two threads share an output byte). bits 8 stores the raw length.
void pack_lengths(const int64_t* offsets, int64_t n, int bits, int64_t base, uint8_t* out);
// Length of record i of a narrow lengths array (test helper / host decode).
int64_t narrow_length(const uint8_t* lengths, int bits, int64_t base, int64_t i);
// The same packing from plain uint16 lengths (the parser's per-slice scratch).
void pack_lengths16(const uint16_t* lengths, int64_t n, int bits, int64_t base, uint8_t* out);

// ---- sparse offsets ---------------------------------------------------------------------------------
// The streaming kernels read a record's letter offset only at tile boundaries (multiples of 64 records)
// and at the batch end, and take every length from the narrow lengths. So the parser's narrow wire
// format keeps one int64 offset per 2^shift records: entry j = offset of record min(j << shift, n),
// j = 0 .. ceil(n / 2^shift) — 1/64 of the bytes of CSR offsets (which cost 8 B per record against the
// 5.3 B of packed letters of an input6-shaped record).
constexpr int kSparseShift = 6;
inline int64_t sparse_count(int64_t n, int shift) { return ((n + (int64_t{1} << shift) - 1) >> shift) + 1; }
// Entry of record r (a multiple of 2^shift, or r == n).
inline int64_t sparse_index(int64_t r, int shift) { return (r + (int64_t{1} << shift) - 1) >> shift; }
// Dense CSR offsets out[0..n] (absolute, out[0] = sparse[0]) from sparse offsets + narrow lengths.
void expand_offsets(const int64_t* sparse, int shift, const uint8_t* lengths, int bits, int64_t base, int64_t n,
                    int64_t* out);

// One host batch in the wire formats above: what `final`'s parser writes for a rank's slice and what the
// engines take. `offsets` is dense (off_shift 0, n+1 entries) or sparse (off_shift > 0, lengths required).
struct WireBatch {
  const uint8_t* letters = nullptr;  // P33 fields, 5-bit packed (packed5) or one byte per letter;
  bool packed5 = false;              // record i at letter offsets[i]
  bool packed33 = false;             // P33 fields (moc::pack33)
  const int64_t* offsets = nullptr;
  int off_shift = 0;
  const uint8_t* lengths = nullptr;  // narrow lengths (optional with dense offsets)
  int len_bits = 8;
  int64_t len_base = 0;
  int64_t n = 0;
  int64_t min_l2 = -1, max_l2 = -1;  // length range (-1: unknown; required with sparse offsets)
  bool device = false;               // every pointer is device memory of the engine's GPU
  int64_t first_letter() const { return offsets[0]; }
  int64_t end_letter() const { return offsets[off_shift ? sparse_count(n, off_shift) - 1 : n]; }
  int64_t letter_bytes() const {
    const int64_t L = end_letter() - first_letter();
    if (packed33) return p33_end_byte(end_letter()) - p33_first_byte(first_letter());
    return packed5 ? (5 * L + 7) / 8 : L;
  }
  int64_t offset_entries() const { return off_shift ? sparse_count(n, off_shift) : n + 1; }
  int64_t length_bytes() const { return lengths ? narrow_lengths_bytes(n, len_bits) : 0; }
};

}  // namespace moc
