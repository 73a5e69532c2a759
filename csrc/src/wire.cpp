// Wire formats (moc/wire.hpp): result-format selection / decoding and narrow record lengths.
#include "moc/wire.hpp"

#include <omp.h>

#include <algorithm>
#include <climits>
#include <cstring>

namespace moc {

ResultFormat pick_result_format(int64_t L1, int64_t max_l2, int32_t max_abs_weight) {
  const int64_t smax = static_cast<int64_t>(std::max(max_abs_weight, 1)) * std::max<int64_t>(max_l2, 1);
  if (L1 <= 255 && max_l2 <= 255 && smax < 32767) return ResultFormat::R4;
  if (L1 <= 65535 && max_l2 <= 65535) return ResultFormat::R8;
  return ResultFormat::R12;
}

bool r2_params(int64_t L1, int64_t min_l2, int64_t max_l2, int32_t min_t, int32_t max_t, R2Params& p) {
  min_l2 = std::max<int64_t>(min_l2, 1);
  max_l2 = std::max(max_l2, min_l2);
  const int64_t smin = std::min(static_cast<int64_t>(min_t) * min_l2, static_cast<int64_t>(min_t) * max_l2);
  const int64_t smax = std::max(static_cast<int64_t>(max_t) * min_l2, static_cast<int64_t>(max_t) * max_l2);
  const int64_t kw = max_l2;
  const int64_t j = std::max<int64_t>(L1 - min_l2 + 1, 1) * kw;  // > (L1 - min_l2) * kw + (kw - 1) >= n*kw + k
  if ((smax - smin + 1) * j > kR2None) return false;            // 0xFFFF stays free for "no candidate"
  p.smin = static_cast<int32_t>(smin);
  p.kw = static_cast<int32_t>(kw);
  p.j = static_cast<int32_t>(j);
  return true;
}

void expand_results(const void* in, ResultFormat f, int64_t n, Result* out, const R2Params* r2) {
  if (f == ResultFormat::R12) {
    if (in != out) std::memmove(out, in, sizeof(Result) * static_cast<size_t>(n));
    return;
  }
  if (f == ResultFormat::R2 && (!r2 || r2->j <= 0 || r2->kw <= 0)) throw Error("expand_results: R2 needs its parameters");
#pragma omp parallel for schedule(static) if (n > 65536)
  for (int64_t i = 0; i < n; ++i) {
    if (f == ResultFormat::R2) {
      const uint16_t c = static_cast<const uint16_t*>(in)[i];
      if (c == kR2None) {
        out[i] = Result{INT32_MIN, 0, 0};
      } else {
        const int32_t idx = c % r2->j;
        out[i] = Result{c / r2->j + r2->smin, idx / r2->kw, idx % r2->kw};
      }
    } else if (f == ResultFormat::R8) {
      const R8 x = static_cast<const R8*>(in)[i];
      out[i] = Result{x.score, x.n, x.k};
    } else {
      const R4 x = static_cast<const R4*>(in)[i];
      out[i] = Result{x.score == INT16_MIN ? INT32_MIN : x.score, x.n, x.k};
    }
  }
}

namespace {
// Base-6 words: word w holds records [24w, 24w+24) (digits past n are 0). len(i) - base, i in [0, n).
// Each field is a sum of independent digit * 6^j terms (no serial Horner chain), and only the last word
// checks for records past n.
template <typename LenOf>
void pack_base6(int64_t n, uint8_t* out, LenOf len_of) {
  static constexpr uint32_t kPow6[8] = {1u, 6u, 36u, 216u, 1296u, 7776u, 46656u, 279936u};
  const int64_t words = (n + 23) / 24, full = n / 24;
#pragma omp parallel for schedule(static) if (words > 65536)
  for (int64_t w = 0; w < full; ++w) {
    uint64_t word = 0;
    for (int f = 0; f < 3; ++f) {
      uint32_t v = 0;
      for (int j = 0; j < 8; ++j) v += static_cast<uint32_t>(len_of(24 * w + 8 * f + j)) * kPow6[j];
      word |= static_cast<uint64_t>(v) << (21 * f);
    }
    std::memcpy(out + 8 * w, &word, 8);
  }
  for (int64_t w = full; w < words; ++w) {
    uint64_t word = 0;
    for (int f = 0; f < 3; ++f) {
      uint32_t v = 0;
      for (int j = 0; j < 8; ++j) {
        const int64_t i = 24 * w + 8 * f + j;
        if (i < n) v += static_cast<uint32_t>(len_of(i)) * kPow6[j];
      }
      word |= static_cast<uint64_t>(v) << (21 * f);
    }
    std::memcpy(out + 8 * w, &word, 8);
  }
}
}  // namespace

void pack_lengths(const int64_t* offsets, int64_t n, int bits, int64_t base, uint8_t* out) {
  if (bits == kLenBase6) {
    pack_base6(n, out, [&](int64_t i) { return offsets[i + 1] - offsets[i] - base; });
    return;
  }
  if (bits != 3 && bits != 4 && bits != 8) throw Error("pack_lengths: bits must be 3, 4, 6 (base 6) or 8");
  const int64_t groups = (n + 7) / 8;  // 8 records -> 3 / 4 / 8 bytes, independent per group
#pragma omp parallel for schedule(static) if (groups > 65536)
  for (int64_t g = 0; g < groups; ++g) {
    const int64_t b = g * 8;
    const int m = static_cast<int>(std::min<int64_t>(8, n - b));
    uint64_t v = 0;
    for (int j = 0; j < m; ++j) {
      const uint64_t L = static_cast<uint64_t>(offsets[b + j + 1] - offsets[b + j] - (bits == 8 ? 0 : base));
      v |= L << (bits * j);
    }
    const int nb = bits == 3 ? (3 * m + 7) / 8 : bits == 4 ? (m + 1) / 2 : m;
    for (int j = 0; j < nb; ++j) out[g * bits + j] = static_cast<uint8_t>(v >> (8 * j));
  }
  if (bits == 3 && n >= 0) out[narrow_lengths_bytes(n, 3) - 1] = 0;  // slack byte
}

void pack_lengths16(const uint16_t* lengths, int64_t n, int bits, int64_t base, uint8_t* out) {
  if (bits == kLenBase6) {
    pack_base6(n, out, [&](int64_t i) { return static_cast<int64_t>(lengths[i]) - base; });
    return;
  }
  if (bits != 3 && bits != 4 && bits != 8) throw Error("pack_lengths16: bits must be 3, 4, 6 (base 6) or 8");
  const int64_t groups = (n + 7) / 8;
#pragma omp parallel for schedule(static) if (groups > 65536)
  for (int64_t g = 0; g < groups; ++g) {
    const int64_t b = g * 8;
    const int m = static_cast<int>(std::min<int64_t>(8, n - b));
    uint64_t v = 0;
    for (int j = 0; j < m; ++j) v |= static_cast<uint64_t>(lengths[b + j] - (bits == 8 ? 0 : base)) << (bits * j);
    const int nb = bits == 3 ? (3 * m + 7) / 8 : bits == 4 ? (m + 1) / 2 : m;
    for (int j = 0; j < nb; ++j) out[g * bits + j] = static_cast<uint8_t>(v >> (8 * j));
  }
  if (bits == 3 && n >= 0) out[narrow_lengths_bytes(n, 3) - 1] = 0;  // slack byte
}

void expand_offsets(const int64_t* sparse, int shift, const uint8_t* lengths, int bits, int64_t base, int64_t n,
                    int64_t* out) {
  const int64_t S = int64_t{1} << shift, blocks = (n + S - 1) / S;
  // every block of 2^shift records starts at its sparse entry: independent prefix sums
#pragma omp parallel for schedule(static) if (blocks > 4096)
  for (int64_t j = 0; j < blocks; ++j) {
    int64_t o = sparse[j];
    const int64_t e = std::min(n, (j + 1) * S);
    for (int64_t i = j * S; i < e; ++i) {
      out[i] = o;
      o += narrow_length(lengths, bits, base, i);
    }
  }
  out[n] = sparse[sparse_count(n, shift) - 1];
}

int64_t narrow_length(const uint8_t* lengths, int bits, int64_t base, int64_t i) {
  if (bits == 8) return lengths[i];
  if (bits == kLenBase6) {
    uint64_t word;
    std::memcpy(&word, lengths + 8 * (i / 24), 8);
    uint32_t v = static_cast<uint32_t>(word >> (21 * ((i / 8) % 3))) & 0x1FFFFFu;
    for (int64_t j = i % 8; j > 0; --j) v /= 6u;
    return base + v % 6u;
  }
  if (bits == 4) return base + ((lengths[i / 2] >> (4 * (i & 1))) & 15);
  const int64_t bit = 3 * i;
  const uint32_t w = lengths[bit >> 3] | (static_cast<uint32_t>(lengths[(bit >> 3) + 1]) << 8);
  return base + ((w >> (bit & 7)) & 7);
}

}  // namespace moc
