#include "moc/problem.hpp"

#include "moc/simd.hpp"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>

namespace moc {

int64_t RecordBatch::max_length() const {
  int64_t m = 0;
  for (int64_t i = 0; i < size(); ++i) m = std::max(m, length(i));
  return m;
}

void RecordBatch::push_back(const uint8_t* c, int64_t n) {
  codes.insert(codes.end(), c, c + n);
  offsets.push_back(offsets.back() + n);
}

RecordBatch RecordBatch::slice(int64_t b, int64_t e) const {
  RecordBatch out;
  if (e <= b) return out;
  const int64_t base = offsets[b];
  out.codes.assign(codes.begin() + base, codes.begin() + offsets[e]);
  out.offsets.resize(e - b + 1);
  for (int64_t i = b; i <= e; ++i) out.offsets[i - b] = offsets[i] - base;
  return out;
}

void validate_score_range(const Weights& w, int64_t max_len2) {
  int64_t m = 0;
  for (int i = 0; i < 4; ++i) {
    if (w.w[i] < 0) throw Error("weights must be non-negative (PDF p.2), got " + std::to_string(w.w[i]));
    m = std::max<int64_t>(m, w.w[i]);
  }
  // Device keys hold 2*max|T|*L2 in int32 with headroom; the CPU engine matches bit-for-bit.
  if (m * std::max<int64_t>(max_len2, 1) >= (int64_t{1} << 29))
    throw Error("max weight * max Seq2 length = " + std::to_string(m * max_len2) +
                " exceeds the int32 score range supported (< 2^29)");
}

void pack5(const uint8_t* codes, int64_t n, uint8_t* out) {
  const int64_t groups = (n + 7) / 8;  // 8 chars -> 5 bytes, independent per group
#pragma omp parallel for schedule(static) if (groups > 65536)
  for (int64_t g = 0; g < groups; ++g) {
    uint64_t v = 0;
    const int64_t b = g * 8;
    const int m = static_cast<int>(std::min<int64_t>(8, n - b));
    for (int j = 0; j < m; ++j) v |= static_cast<uint64_t>(codes[b + j] & 31u) << (5 * j);
    uint8_t* o = out + g * 5;
    for (int j = 0; j < 5; ++j) o[j] = static_cast<uint8_t>(v >> (8 * j));
  }
  const int64_t used = groups * 5, total = packed5_bytes(n);
  for (int64_t i = used; i < total; ++i) out[i] = 0;
}

void unpack5(const uint8_t* packed, int64_t begin, int64_t n, uint8_t* out) {
#pragma omp parallel for schedule(static) if (n > (1 << 20))
  for (int64_t i = 0; i < n; ++i) {
    const int64_t bit = 5 * (begin + i);
    const uint32_t lo = packed[bit >> 3], hi = packed[(bit >> 3) + 1];
    out[i] = static_cast<uint8_t>(((lo | (hi << 8)) >> (bit & 7)) & 31u);
  }
}

void p33_block(const uint8_t* c, uint8_t* out, int m) {
  if (m >= kP33Letters) {
    p33_block_full(c, out);
    return;
  }
  uint64_t w[5] = {0, 0, 0, 0, 0};  // 264 bits + room for the last field's spill
  for (int f = 0; f < kP33Letters / kP33Field; ++f) {
    const int have = std::max(0, std::min(kP33Field, m - kP33Field * f));
    const uint64_t v = p33_field(c + kP33Field * f, have);
    const int bit = 33 * f;
    w[bit >> 6] |= v << (bit & 63);
    if ((bit & 63) + 33 > 64) w[(bit >> 6) + 1] |= v >> (64 - (bit & 63));
  }
  std::memcpy(out, w, kP33Bytes);
}

namespace simd {
bool p33_available() {
  static const bool on = [] {
    const char* e = std::getenv("MOC_FILL_SIMD");
    if (e && std::strcmp(e, "0") == 0) return false;
    __builtin_cpu_init();
    return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") && __builtin_cpu_supports("avx512vbmi");
  }();
  return on;
}
}  // namespace simd

namespace {
// whole 56-letter blocks [g0, g1) of pack33 with the vector field arithmetic
MOC_SIMD_P33 void pack33_blocks_simd(const uint8_t* codes, int64_t g0, int64_t g1, uint8_t* out) {
  for (int64_t g = g0; g < g1; ++g) simd::p33_block_avx512(codes + g * kP33Letters, out + g * kP33Bytes);
}
}  // namespace

void pack33(const uint8_t* codes, int64_t n, uint8_t* out) {
  const int64_t blocks = (n + kP33Letters - 1) / kP33Letters;
  const int64_t full = n / kP33Letters;
  if (simd::p33_available()) {  // whole blocks in parallel runs of 4096, the last partial one below
    const int64_t runs = (full + 4095) / 4096;
#pragma omp parallel for schedule(static) if (runs > 4)
    for (int64_t r = 0; r < runs; ++r) pack33_blocks_simd(codes, 4096 * r, std::min(full, 4096 * (r + 1)), out);
    if (full < blocks) p33_block(codes + full * kP33Letters, out + full * kP33Bytes, static_cast<int>(n - full * kP33Letters));
  } else {
#pragma omp parallel for schedule(static) if (blocks > 16384)
    for (int64_t g = 0; g < blocks; ++g) {
      const int64_t b = g * kP33Letters;
      p33_block(codes + b, out + g * kP33Bytes, static_cast<int>(std::min<int64_t>(kP33Letters, n - b)));
    }
  }
  const int64_t used = blocks * kP33Bytes, total = packed33_bytes(n);
  for (int64_t i = used; i < total; ++i) out[i] = 0;
}

void unpack33(const uint8_t* packed, int64_t begin, int64_t n, uint8_t* out) {
#pragma omp parallel for schedule(static) if (n > (1 << 20))
  for (int64_t i = 0; i < n; ++i) {
    const int64_t x = begin + i, f = x / kP33Field, bit = 33 * f;
    uint64_t w = 0;
    std::memcpy(&w, packed + (bit >> 3), 5);  // 33 bits from a 0..7 bit offset fit 5 bytes
    uint64_t v = (w >> (bit & 7)) & ((uint64_t{1} << 33) - 1);
    for (int64_t j = x - f * kP33Field; j > 0; --j) v /= 26u;
    out[i] = static_cast<uint8_t>(v % 26u + 1u);
  }
}

std::vector<uint8_t> encode_sequence(const char* s, int64_t n) {
  std::vector<uint8_t> out(n);
  for (int64_t i = 0; i < n; ++i) {
    int c = letter_code(static_cast<unsigned char>(s[i]));
    if (c == 0) throw Error(std::string("non-letter character '") + s[i] + "' in sequence");
    out[i] = static_cast<uint8_t>(c);
  }
  return out;
}

std::string decode_sequence(const uint8_t* codes, int64_t n) {
  std::string s(n, '?');
  for (int64_t i = 0; i < n; ++i) s[i] = code_letter(codes[i]);
  return s;
}

}  // namespace moc
