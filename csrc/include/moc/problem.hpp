// Problem model: weights + Seq1 + a CSR batch of Seq2 records, all letters already encoded 1..26.
//
// Reference equivalent: weights int[4] (main.c:55), seq1 = malloc(3000) (main.c:66) and the
// fixed-stride seq2_all[N*2000] buffer (main.c:93). A fixed 2000-byte stride wastes >99% of the
// scatter bytes on input6 and overflows on a 2000-letter record (bug B12), so records are packed
// CSR here: codes[] concatenated, offsets[N+1].
#pragma once

#include <cstdint>
#include <cstring>
#include <memory>
#include <vector>

#include <sys/mman.h>

#include "moc/common.hpp"

namespace moc {

// Allocator whose resize() leaves new elements default-initialised (not zeroed): batch buffers are
// written in full right after they are sized, so zero-filling hundreds of MB first is pure waste.
template <typename T>
struct DefaultInitAllocator : std::allocator<T> {
  template <typename U>
  struct rebind {
    using other = DefaultInitAllocator<U>;
  };
  DefaultInitAllocator() = default;
  template <typename U>
  DefaultInitAllocator(const DefaultInitAllocator<U>&) noexcept {}
  template <typename U>
  void construct(U* p) noexcept {
    ::new (static_cast<void*>(p)) U;
  }
  template <typename U, typename... Args>
  void construct(U* p, Args&&... args) {
    ::new (static_cast<void*>(p)) U(std::forward<Args>(args)...);
  }
  // Large arrays (>= 32 MiB: a parsed batch's letters and offsets, input text) are their own mappings,
  // advised for 2 MiB pages: 512x fewer first-touch faults than malloc's 4 KiB ones (a 2.2 GB parse of
  // 1.14 G letters spent most of its time faulting pages in).
  static constexpr size_t kMapBytes = size_t{32} << 20;
  T* allocate(size_t n) {
    const size_t bytes = n * sizeof(T);
    if (bytes < kMapBytes) return std::allocator<T>::allocate(n);
    void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) throw std::bad_alloc();
    const uintptr_t huge = uintptr_t{2} << 20;
    const uintptr_t lo = (reinterpret_cast<uintptr_t>(p) + huge - 1) & ~(huge - 1);
    const uintptr_t hi = (reinterpret_cast<uintptr_t>(p) + bytes) & ~(huge - 1);
    if (hi > lo) (void)madvise(reinterpret_cast<void*>(lo), hi - lo, MADV_HUGEPAGE);
    return static_cast<T*>(p);
  }
  void deallocate(T* p, size_t n) {
    const size_t bytes = n * sizeof(T);
    if (bytes < kMapBytes) {
      std::allocator<T>::deallocate(p, n);
      return;
    }
    munmap(p, bytes);
  }
};
template <typename T>
using uvector = std::vector<T, DefaultInitAllocator<T>>;

struct RecordBatch {
  uvector<uint8_t> codes;    // concatenated letter codes (1..26)
  uvector<int64_t> offsets;  // size N+1, offsets[0] == 0

  RecordBatch() : offsets(1, 0) {}
  int64_t size() const { return static_cast<int64_t>(offsets.size()) - 1; }
  int64_t length(int64_t i) const { return offsets[i + 1] - offsets[i]; }
  const uint8_t* record(int64_t i) const { return codes.data() + offsets[i]; }
  int64_t total_chars() const { return offsets.back(); }
  int64_t max_length() const;
  void push_back(const uint8_t* c, int64_t n);
  // Contiguous slice [b, e) re-based to offset 0.
  RecordBatch slice(int64_t b, int64_t e) const;
};

struct Problem {
  Weights weights;
  std::vector<uint8_t> seq1;  // letter codes
  RecordBatch seq2;

  int64_t L1() const { return static_cast<int64_t>(seq1.size()); }
};

// Number of candidate cells the O(L1*L2) search touches for one record: (L1-L2+1)*L2, 0 if L2 > L1.
inline int64_t record_cells(int64_t L1, int64_t L2) { return L2 <= L1 ? (L1 - L2 + 1) * L2 : 0; }

// Throws moc::Error when the int32 score arithmetic (shared by the CPU and device engines, as in the
// reference's int counters, cudaFunctions.cu:103,161) could overflow for this problem.
void validate_score_range(const Weights& w, int64_t max_len2);

// ---- 5-bit packed letter codes ("packed CSR") ----------------------------------------------------------
// Letter j of the concatenated stream occupies bits [5j, 5j+5) of a little-endian byte stream, so a
// record keeps its char offsets (bit offset = 5 * char offset). 26 letters need 5 bits: the stream is
// 5/8 of the byte codes, i.e. 37.5% fewer bytes over PCIe / xGMI for every transfer of the batch.
inline int64_t packed5_bytes(int64_t n_chars) { return (5 * n_chars + 7) / 8 + 16; }  // + read slack
// codes[0..n) (values < 32) -> out[0..packed5_bytes(n)) (OpenMP; slack bytes zeroed).
void pack5(const uint8_t* codes, int64_t n, uint8_t* out);
// Inverse for chars [begin, begin + n) of a packed stream.
void unpack5(const uint8_t* packed, int64_t begin, int64_t n, uint8_t* out);

// ---- 33-bit letter fields ("P33": 4.714 bits per letter) -------------------------------------------------
// Letters 7f .. 7f+6 form field f, the value sum_i (code - 1) * 26^i (26^7 = 8 031 810 176 < 2^33) stored
// at bits [33f, 33f+33) of a little-endian bit stream. Eight fields (56 letters) fill exactly 33 bytes, so
// blocks of 56 letters are byte-aligned: the unit of parallel encoding and of a reader's byte ranges.
// 5.7% fewer bytes than 5-bit packing (log2 26 = 4.700 is the floor; round 3's 5-letters-in-3-bytes groups,
// retired in round 4, took 4.8); a field decodes with 32-bit arithmetic only
// (the first division as (v >> 1) / 13, the other six on a value < 2^29).
constexpr int kP33Field = 7, kP33Letters = 56, kP33Bytes = 33;
inline int64_t packed33_bytes(int64_t n_chars) { return kP33Bytes * ((n_chars + kP33Letters - 1) / kP33Letters) + 16; }
// Field value of up to 7 codes (codes 0 count as 1).
inline uint64_t p33_field(const uint8_t* c, int m = kP33Field) {
  uint64_t v = 0;
  for (int j = m - 1; j >= 0; --j) v = v * 26u + (c[j] > 1 ? c[j] - 1u : 0u);
  return v;
}
// One whole 33-byte block from 56 codes: the field as two 32-bit Horner chains (letters 0..3 < 26^4,
// 4..6 < 26^3) joined once, eight fields at bits 33k assembled into 4 words + 1 byte. Inline: the parser
// calls it per 56 letters.
inline uint32_t p33_digit(uint8_t c) { return c > 1 ? c - 1u : 0u; }
inline void p33_block_full(const uint8_t* c, uint8_t* out) {
  uint64_t f[8];
  for (int k = 0; k < 8; ++k) {
    const uint8_t* p = c + 7 * k;
    const uint32_t lo = ((p33_digit(p[3]) * 26u + p33_digit(p[2])) * 26u + p33_digit(p[1])) * 26u + p33_digit(p[0]);
    const uint32_t hi = (p33_digit(p[6]) * 26u + p33_digit(p[5])) * 26u + p33_digit(p[4]);
    f[k] = lo + static_cast<uint64_t>(hi) * 456976u;
  }
  const uint64_t w[4] = {f[0] | f[1] << 33, f[1] >> 31 | f[2] << 2 | f[3] << 35, f[3] >> 29 | f[4] << 4 | f[5] << 37,
                         f[5] >> 27 | f[6] << 6 | f[7] << 39};
  std::memcpy(out, w, 32);
  out[32] = static_cast<uint8_t>(f[7] >> 25);
}
// One 33-byte block from 56 codes (m < 56: the codes past m count as 1).
void p33_block(const uint8_t* c, uint8_t* out, int m = kP33Letters);
// codes[0..n) -> out[0..packed33_bytes(n)) (OpenMP; slack bytes zeroed).
void pack33(const uint8_t* codes, int64_t n, uint8_t* out);
// Letters [begin, begin + n) back as codes 1..26.
void unpack33(const uint8_t* packed, int64_t begin, int64_t n, uint8_t* out);
// Byte range of a P33 stream holding letters [c0, c1): [first, end).
inline int64_t p33_first_byte(int64_t c0) { return (33 * (c0 / kP33Field)) >> 3; }
inline int64_t p33_end_byte(int64_t c1) { return (33 * ((c1 + kP33Field - 1) / kP33Field) + 7) >> 3; }

// Encodes an ASCII string (letters only, any case) into codes; throws on a non-letter.
std::vector<uint8_t> encode_sequence(const char* s, int64_t n);
std::string decode_sequence(const uint8_t* codes, int64_t n);

}  // namespace moc
