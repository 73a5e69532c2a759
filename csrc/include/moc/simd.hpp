// AVX-512 (VBMI) forms of the letter encoders (moc/problem.hpp), for host code that dispatches on the CPU
// at run time: header-only and `static inline` with a target attribute, so they inline into callers built
// for the same target (the parser's vector encoder, pack33) while the rest of the binary stays generic.
#pragma once

#include <immintrin.h>

#include <cstdint>
#include <cstring>

namespace moc {
namespace simd {

#define MOC_SIMD_P33 __attribute__((target("avx512f,avx512bw,avx512vbmi")))

// AVX-512 F + BW + VBMI present (and MOC_FILL_SIMD is not "0"): p33_block_avx512 may run.
bool p33_available();

// One P33 block (moc::p33_block_full) with the digit arithmetic on 64-bit lanes: the 56 codes are permuted
// into 8 lanes of 7 digits, vpmaddubsw / vpmaddwd form each lane's base-26 halves (digits 0..3 and 4..6)
// and one 32x32 multiply joins them; the eight 33-bit fields are then laid out as p33_block_full does.
MOC_SIMD_P33 static inline void p33_block_avx512(const uint8_t* c, uint8_t* out) {
  // lane k, byte j <- code 7k + j (byte 7 of every lane is zeroed by the mask below)
  alignas(64) static constexpr uint8_t kIdxBytes[64] = {
      0,  1,  2,  3,  4,  5,  6,  0, 7,  8,  9,  10, 11, 12, 13, 0, 14, 15, 16, 17, 18, 19, 20, 0,
      21, 22, 23, 24, 25, 26, 27, 0, 28, 29, 30, 31, 32, 33, 34, 0, 35, 36, 37, 38, 39, 40, 41, 0,
      42, 43, 44, 45, 46, 47, 48, 0, 49, 50, 51, 52, 53, 54, 55, 0};
  const __m512i kIdx = _mm512_load_si512(reinterpret_cast<const void*>(kIdxBytes));
  const __m512i x = _mm512_subs_epu8(_mm512_maskz_loadu_epi8((__mmask64{1} << 56) - 1, c), _mm512_set1_epi8(1));
  const __m512i y = _mm512_maskz_permutexvar_epi8(0x7F7F7F7F7F7F7F7Full, kIdx, x);
  const __m512i w = _mm512_maddubs_epi16(y, _mm512_set1_epi16(static_cast<short>(1 | (26 << 8))));
  const __m512i d = _mm512_madd_epi16(w, _mm512_set1_epi32(1 | (676 << 16)));
  const __m512i f = _mm512_add_epi64(_mm512_and_si512(d, _mm512_set1_epi64(0xFFFFFFFFll)),
                                     _mm512_mul_epu32(_mm512_srli_epi64(d, 32), _mm512_set1_epi64(456976)));
  alignas(64) uint64_t fv[8];
  _mm512_store_si512(reinterpret_cast<void*>(fv), f);
  const uint64_t wv[4] = {fv[0] | fv[1] << 33, fv[1] >> 31 | fv[2] << 2 | fv[3] << 35,
                          fv[3] >> 29 | fv[4] << 4 | fv[5] << 37, fv[5] >> 27 | fv[6] << 6 | fv[7] << 39};
  std::memcpy(out, wv, 32);
  out[32] = static_cast<uint8_t>(fv[7] >> 25);
}

}  // namespace simd
}  // namespace moc
