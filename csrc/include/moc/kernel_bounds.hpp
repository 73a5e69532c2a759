// Exactness rules of the narrow-integer fast paths, in one place.
//
// The reference scores in plain int (cudaFunctions.cu:103,161). The gfx950 kernels run most batches in
// narrower arithmetic: packed int16 running sums, int8 difference profiles, int32 keys with k packed
// into the low bits. Each form is exact only while no intermediate can wrap. The host picks a form per
// batch with the functions below, and nothing else decides:
//   * the launchers (swipe_kernels.hip, short_kernels.hip, align_kernels.hip, build_profile16) call them;
//   * HipEngine records the form each solve ran (EngineStats::forms);
//   * moc_kernel_forms (capi.h) predicts the forms without a GPU;
//   * csrc/tests/test_core.cpp replays each form's arithmetic on the host, with the same wrap-around, at
//     the bound (exact) and one step past it (the replay wraps, and the rule refuses the form).
//
// Notation: W = max |T| over the pair-score table (max of |W1..W4|), L2 = the batch's longest record
// that is searched (records longer than Seq1 are never scored). Along a diagonal o the kernels sum
// Dt[c][j] = T[c][Seq1[j]] - T[c][Seq1[j+1]], so |Dt| <= 2W and |D_o(k)| <= 2 W L2 = dmax. The bound is
// reached: Seq1 = "AZAZ...", Seq2 = a piece of Seq1 at an even offset, W1 = W4 = W gives Dt = 2W at
// every step (tests/test_extremes.py builds exactly that input).
#pragma once

#include <algorithm>
#include <cstdint>

namespace moc {
namespace bounds {

// |D_o(k)| <= 2 W L2 for every diagonal and prefix length.
inline int64_t diff_bound(int32_t max_abs_weight, int64_t max_l2) {
  return 2 * static_cast<int64_t>(std::max(max_abs_weight, 1)) * std::max<int64_t>(max_l2, 1);
}

// ---- swipe kernel (swipe_impl.hpp): one lane per record, int16 running sums per offset pair.
// Record words per lane (4 letters each): 4 for records <= 16 letters, 8 for <= 32, 12 for <= 48, 16 for
// <= 64, 24 for <= 96, 32 for <= 128 (the longest records the kernel takes). The words size the LDS tables
// (and P33's decode slices), so input1's records of 32..41 letters take 12, not 16.
constexpr int64_t kSwipeMaxL2 = 128;
inline int swipe_record_words(int64_t max_l2) {
  return max_l2 <= 16 ? 4 : max_l2 <= 32 ? 8 : max_l2 <= 48 ? 12 : max_l2 <= 64 ? 16 : max_l2 <= 96 ? 24 : 32;
}
// Bits for k in the int16 keys: k <= 4 * l2w < 2^kb.
constexpr int swipe_kbits(int l2w) {
  int b = 1;
  while ((1 << b) <= 4 * l2w) ++b;
  return b;
}
enum class SwipeKeys { None, KBits, RK };
// Key form of the swipe kernel for a batch:
//   KBits: E = D * 2^kb + (2^kb - 1 - k) in int16. Its largest value is dmax * 2^kb + 2^kb - 2, so
//          dmax * 2^kb + 2^kb < 32767 keeps every key (and B2 = max E) exact.
//   RK:    E = D in int16 (|D| <= dmax < 32767); k is re-found on the winning diagonal afterwards.
//          Records of more than 32 letters (l2w >= 12) always take it: no room for 6 k bits.
//   None:  dmax >= 32767.
// The selection keys carry score + 2^15 in 16 bits: |score| <= W L2 = dmax / 2 < 2^14 under either form; the
// anchor diagonal is summed in int32 from an int32 table (swipe_build_tables), so W itself is not bounded.
inline SwipeKeys swipe_keys(int32_t max_abs_weight, int64_t max_l2) {
  const int64_t dmax = diff_bound(max_abs_weight, max_l2);
  if (dmax >= 32767) return SwipeKeys::None;
  const int l2w = swipe_record_words(max_l2);
  const int kb = swipe_kbits(l2w);
  return (l2w >= 12 || (dmax << kb) + (int64_t{1} << kb) >= 32767) ? SwipeKeys::RK : SwipeKeys::KBits;
}

// ---- short kernel (short_kernels.hip): one lane per offset.
// Pk form: the profile holds (Dt << 16 | S) and one packed int16 add advances D_o (high half, |D| <= dmax)
// and Tot_o (low half, |Tot| <= W L2 < dmax). Exact when dmax < 32767.
inline bool short_pk_exact(int32_t max_abs_weight, int64_t max_l2) {
  return diff_bound(max_abs_weight, max_l2) < 32767;
}

// ---- int32 hot keys of the short (non-Pk) and tile kernels: key = D << shift | (2^shift - 1 - k), with
// 2^shift > L2 >= k. Exact when dmax << shift < 2^31; 0 means 64-bit keys. `max_l2` is capped at L1 + 1 by
// the caller (longer records are not searched).
inline int32_t key_shift(int32_t max_abs_weight, int64_t max_l2) {
  int shift = 1;
  while ((int64_t{1} << shift) < max_l2 + 1) ++shift;  // mask = 2^shift - 1 >= every k used (<= L2)
  if (shift > 24 || (diff_bound(max_abs_weight, max_l2) << shift) >= (int64_t{1} << 31)) return 0;
  return shift;
}

// ---- tile16 / MFMA sweeps (tile16_kernels.hip, tile_mfma_kernels.hip): Dt as int8 bytes of a profile,
// summed in int16 halves for at most kProf16Fold steps before being folded into int32, so the int16
// partial sums stay within kProf16Fold * 128 = 8192. T itself is read as int8 (anchor diagonals).
constexpr int kProf16Fold = 64;
// dmin/dmax: the extreme Dt over letter pairs (including the zero pad past Seq1); tabs: max |T|.
inline bool profile16_exact(int32_t dmin, int32_t dmax, int32_t tabs) {
  return dmin >= -128 && dmax <= 127 && tabs <= 127;
}
static_assert(kProf16Fold * 128 < 32768, "tile16 int16 partial sums");
// The int16 profile (one Dt per entry, staged into widened images only): |Dt| <= 511 keeps a 64-step partial
// sum within int16 (64 * 511 = 32704); T is read from the int32 LUT.
inline bool profile16_i16_exact(int32_t dmin, int32_t dmax) { return dmin >= -511 && dmax <= 511; }
static_assert(kProf16Fold * 511 < 32768, "tile16 int16 partial sums, int16 profile");

// tile16's per-lane selection in 32-bit keys: ((score + 2^(31 - IB)) << IB) | (2^IB - 1 - idx), idx = 2o +
// mutated <= 2 L1 + 1 < 2^IB. Exact when every score fits the 32 - IB score bits: |score| <= max|T| * L2
// < 2^(31 - IB). Returns IB, or 0 when the 64-bit keys are needed.
inline int tile16_key32_bits(int64_t L1, int32_t max_abs_t, int64_t max_l2) {
  int ib = 1;
  while ((int64_t{1} << ib) <= 2 * L1 + 1) ++ib;
  if (ib > 24) return 0;
  return static_cast<int64_t>(max_abs_t) * max_l2 < (int64_t{1} << (31 - ib)) ? ib : 0;
}

// Form bits reported per solve (EngineStats::forms; Python: stats()["forms"]).
enum FormBits : int32_t {
  kFormSwipeKBits = 1,    // swipe, int16 keys with k bits
  kFormSwipeRK = 2,       // swipe, int16 sums, k re-walked
  kFormShortPk = 4,       // short, packed (D, Tot) int16 pairs
  kFormShortKey32 = 8,    // short, int32 keys
  kFormShortKey64 = 16,   // short, int64 keys
  kFormTile16 = 32,       // tile16, int8 profile + int16 partial sums
  kFormTilesKey32 = 64,   // LUT tile kernel, int32 keys
  kFormTilesKey64 = 128,  // LUT tile kernel, int64 keys
  kFormMfma = 256,        // matrix-core sweep over the tile16 profile
  kFormTile16Key32 = 512, // tile16's per-lane selection in 32-bit keys (tile16_key32_bits)
  kFormTile16I16 = 1024,  // tile16 over the int16 profile (profile16_i16_exact)
  kFormTile16Slide = 2048,  // tile16 in sliding widened windows (long records, widened image past the LDS)
};

}  // namespace bounds
}  // namespace moc
