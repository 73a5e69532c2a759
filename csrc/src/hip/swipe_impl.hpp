// Inter-record SIMD kernel for short records (input6-shaped: |Seq1| <= 200, |Seq2| <= 64, <= 64 offsets).
//
// One LANE = one whole record (vs. one lane per offset in short_kernels.hip): every lane keeps all its
// offsets' running diagonal sums in registers as packed int16 pairs, so
//   * no cross-lane traffic at all in the hot loop (no DPP, no segmented reductions per record),
//   * two cells per VALU op (v_pk_add_u16 / v_pk_max_i16),
//   * the profile row segment a lane needs at step i is read with NOFF/4 aligned ds_read_b64: the block
//     keeps kCopies = 4 copies of the int16 profile, copy s shifted left by s columns, so step i reads copy
//     (i mod 4) at column i - (i mod 4) (a multiple of 4 -> 8-byte aligned).
// The profile holds the diagonal DIFFERENCES Dt[c][j] = S[c][j] - S[c][j+1] (S = T[c][Seq1[j]], 0 past
// Seq1 and in the padding row 0), pre-scaled and pre-biased: Pf[c][j] = Dt[c][j] * 2^KB - 1. A lane's
// running sum for offset o after step i is then already the selection key of the mutant k = i + 1,
//     E_o(i) = D_o(i+1) * 2^KB + (KMASK - (i+1)),    D_o(k) = sum_{i<k} Dt[c_i][o+i],
// (larger D first, then smaller k), so per step and per pair of offsets (2m, 2m+1):
//     E2[m] += (Pf[c][i+2m], Pf[c][i+2m+1])            v_pk_add_u16
//     B2[m]  = max(B2[m], E2[m])                       v_pk_max_i16
// i.e. 1 VALU op per cell. Tot_o is not summed per cell: each lane sums the anchor diagonal
// Tot_NOFF = sum_i T[c_i][Seq1[NOFF + i]] from an int32 table at[i][c] in LDS (0 past Seq1, consistent with
// the profile) and recovers Tot_o = Tot_{o+1} + D_o(L2) by a suffix pass over its offsets in the epilogue,
// with D_o(L2) = (E_o(steps-1) - (KMASK - steps)) >> KB (steps past a record's end add the padding row, Dt 0).
// A wave runs steps = its longest record's length.
// Exactness: int16 arithmetic is exact because the host only selects this kernel when
// 2*max|W|*max|Seq2|*2^KB + 2^KB < 32767 (no key can wrap) — moc/kernel_bounds.hpp swipe_keys, replayed at
// and past the bound by csrc/tests/test_core.cpp test_swipe_replay_bounds. When the weights leave
// no room for k in the keys but the sums still fit int16 (input1: W1 = 100, |Seq2| <= 41), the RK form
// runs: Pf = Dt, the running sums are D_o(k) themselves, B2 keeps max_k D_o(k), and after the selection
// each lane whose winner is a mutant re-walks that one diagonal for the first k reaching the best D.
// Two kernels share the lane search (swipe_lane): swipe_search_kernel streams block tiles through LDS
// (zero-copy from pinned host memory: the host streams), swipe_direct_kernel lets each wave take 64 records
// straight from HBM (device-resident batches).
//
// This header holds the kernel templates; swipe_group.inc instantiates them, one code object per letter
// form (bytes, P33) and offsets per lane, and swipe_kernels.hip holds the host-side configuration,
// dispatch and launch.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "kernel_common.hpp"

namespace moc {
namespace dev {

using namespace kc;

namespace swipe {
constexpr int kBlock = 256;
constexpr int kMaxTile = 2048;  // records per tile: up to 8 per thread in the tile's length scan
// length fields per thread in a tile's scan: 8 for P33 letters (host streams take 2048-record tiles), 4
// for byte letters (device-resident batches: 512-record tiles, fewer registers)
constexpr int rpt_of(int lf) { return lf == 0 ? 4 : 8; }
constexpr int kLdsBudget = 80 * 1024;
constexpr int kMaxV = 4;  // 16-byte letter vectors per thread per tile (register prefetch)
// Shifted copies of the profile in LDS: a step's row segment is read in 8-byte ds_read_b64 chunks at a column
// multiple of 4, so copy s = i mod 4 serves step i (see swipe_build_tables for the bank mapping).
constexpr int kChunk = 8;               // bytes per LDS read (4 int16 entries)
constexpr int kCopies = kChunk / 2;     // shifted copies

typedef short s16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ s16x2 as_s16x2(uint32_t v) { return __builtin_bit_cast(s16x2, v); }
__device__ __forceinline__ uint32_t as_u32(s16x2 v) { return __builtin_bit_cast(uint32_t, v); }

// The profile's geometry is a compile-time function of the instance (NOFF, L2W), so every LDS address in the
// hot loop is the lane's letter times a constant plus an immediate offset. A step i < 4 L2W reads columns
// [8 (i >> 3), 8 (i >> 3) + NOFF) of a row (the RK re-walk: < NOFF + steps); rows are a multiple of 16
// entries, which keeps the rows' bank offsets a bijection of the letter (swipe_build_tables).
constexpr int swipe_row(int noff, int l2w) { return (4 * l2w + noff + 8 + 7) & ~7; }  // int16 entries
constexpr int swipe_stride(int noff, int l2w) { return 2 * swipe_row(noff, l2w) + 8; }  // bytes between rows
constexpr int swipe_copy_bytes(int noff, int l2w) { return kAlphabet * swipe_stride(noff, l2w); }
constexpr int swipe_prof_bytes(int noff, int l2w) { return kCopies * swipe_copy_bytes(noff, l2w); }
// anchor table: int32 [4 * l2w steps][32 letters]
constexpr int swipe_anchor_bytes(int l2w) { return 4 * l2w * 32 * 4; }

struct SwipeLayout {
  int prof_bytes = 0;   // 8 shifted copies of the Dt profile (swipe_prof_bytes)
  int s_off = 0;        // anchor table: at[i][c] = T[c][Seq1[NOFF + i]] (0 past Seq1), int32, swipe_anchor_bytes
  int loff_off = 0, codes_off = 0, res_off = 0, raw_off = 0, total = 0;  // raw: P33 bytes as loaded
  int wave_bytes = 0;  // lane-direct P33: one wave's slice of decoded field slots (direct_layout)
  int pairs_off = 0;   // lane-direct P33: the digit-pair table (build_p33_pair_table)
};

inline int al16(int x) { return (x + 15) & ~15; }

// P33 tiles: the loaded field bytes (33 bits per 7 letters, + alignment) of at most codes_cap letters
inline int p33_raw_cap(int codes_cap) { return (33 * (codes_cap / 7 + 2) + 7) / 8 + 32; }
// LDS bytes of a tile's raw (still encoded) letters by letter form
inline int raw_cap(int lf, int codes_cap) { return lf == 2 ? p33_raw_cap(codes_cap) : 0; }
inline int letter_form(const ShortArgs& a) { return a.packed33 ? 2 : 0; }

inline SwipeLayout swipe_layout(int L1, int noff, int l2w, int tile_records, int codes_cap, int fb, int lf) {
  SwipeLayout l;
  l.prof_bytes = swipe_prof_bytes(noff, l2w);
  l.s_off = l.prof_bytes;
  l.loff_off = l.s_off + swipe_anchor_bytes(l2w);
  l.codes_off = l.loff_off + al16((tile_records + 1) * 4 + 64);  // + misc: 16 ints
  l.res_off = l.codes_off + al16(codes_cap);
  l.raw_off = l.res_off + al16(tile_records * fb);
  l.total = l.raw_off + al16(raw_cap(lf, codes_cap));
  return l;
}

}  // namespace swipe

using namespace swipe;

// The block's LDS tables, built once per block (before a barrier):
//  * kCopies shifted int16 difference-profile copies: copy s, row c, entry j' holds Pf[c][j' + s], at byte
//    s * copy_bytes + c * stride + 2 j'. A step's read is 8-byte chunks of one row (the lane's letter), so the
//    32 lanes of a ds_read_b64 group (2 banks each, 64 banks) read 32 rows at the same column; the row stride
//    of 2 row + 8 bytes (row a multiple of 8 entries) puts row c's chunk on bank pair
//    (c (row / 4 + 1) + chunk) mod 32, a bijection of c mod 32 — all 27 letters on distinct bank pairs, and
//    lanes with the same letter read the same address (a broadcast): conflict-free. (16-byte chunks give a
//    16-lane group only 16 bank quads for 26 letters: 39 % of the LDS cycles were conflicts, PMC round 5.)
//    The address is one multiply-add of the letter plus immediate offsets.
//  * the anchor table at[i][c] = T[c][Seq1[NOFF + i]] (int32: letter c of step i on bank (32 i + c) mod 64,
//    conflict-free; 0 past Seq1 and for the padding letter 0), read at the lane's letter plus an immediate
//    offset: the anchor diagonal Tot_NOFF costs one LDS read per step.
template <bool RK, int KB, int NOFF, int L2W>
__device__ __forceinline__ void swipe_build_tables(unsigned char* smem, const ProblemView& pv, int tid, int nthreads) {
  constexpr int row = swipe_row(NOFF, L2W), stride = swipe_stride(NOFF, L2W), cb = swipe_copy_bytes(NOFF, L2W);
  const int L1 = pv.L1;
  constexpr int n = kCopies * kAlphabet * row;
  for (int e = tid; e < n; e += nthreads) {
    const int s = e / (kAlphabet * row), rem = e - s * (kAlphabet * row), c = rem / row, jj = rem - c * row;
    const int j = jj + s;  // the column entry jj of copy s holds
    const int sj = (c >= 1 && j < L1) ? pv.lut[c * kLutStride + pv.seq1[j]] : 0;
    const int sn = (c >= 1 && j + 1 < L1) ? pv.lut[c * kLutStride + pv.seq1[j + 1]] : 0;
    *reinterpret_cast<short*>(smem + s * cb + c * stride + 2 * jj) =
        static_cast<short>(RK ? sj - sn : (sj - sn) * (1 << KB) - 1);  // Pf = Dt * 2^KB - 1 (header)
  }
  int* at = reinterpret_cast<int*>(smem + swipe_prof_bytes(NOFF, L2W));
  for (int e = tid; e < swipe_anchor_bytes(L2W) / 4; e += nthreads) {
    const int i = e >> 5, c = e & 31, j = NOFF + i;
    at[e] = c >= 1 && c < kAlphabet && j < L1 ? pv.lut[c * kLutStride + pv.seq1[j]] : 0;
  }
}

// A record's letters (rs = byte position of its first letter in `l32`) -> NW aligned words, bits past the
// record end zeroed (they add row 0 = 0). Lanes that are not `on` get zeros and read nothing.
template <int NW>
__device__ __forceinline__ void record_words(const uint32_t* l32, int rs, int L2, bool on, uint32_t (&wd)[NW]) {
  const int wb = rs >> 2;
  const int sh = (rs & 3) * 8;
  const int rbits = 8 * L2;
  uint32_t prev = on ? l32[wb] : 0u;
#pragma unroll
  for (int k = 0; k < NW; ++k) {
    const uint32_t nxt = on ? l32[wb + k + 1] : 0u;
    uint32_t w = sh ? ((prev >> sh) | (nxt << (32 - sh))) : prev;
    const int left = rbits - 32 * k;  // record bits in this word
    w = left >= 32 ? w : (left <= 0 ? 0u : (w & ((1u << left) - 1u)));
    wd[k] = on ? w : 0u;
    prev = nxt;
  }
}

// One lane's search of its record (L2W words of letters, `on`: the lane searches; every lane of the wave
// must call it — the step count is the wave's longest record). max_l2: the batch's longest record.
template <int NOFF, int L2W, bool RK>
__device__ __forceinline__ Result swipe_lane(const unsigned char* smem, const uint32_t (&wd)[L2W], int L2, bool on,
                                             int L1, int max_l2, int sem) {
  constexpr int KB = RK ? 1 : bounds::swipe_kbits(L2W);
  constexpr int KMASK = (1 << KB) - 1;
  constexpr int NP = NOFF / 2;  // packed accumulators
  constexpr int stride = swipe_stride(NOFF, L2W), cb = swipe_copy_bytes(NOFF, L2W);
  const int steps = wave_max_small(on ? L2 : 0);  // L2 <= 4 * L2W <= 128 here (wave_max_small: < 256)
  const int* at = reinterpret_cast<const int*>(smem + swipe_prof_bytes(NOFF, L2W));

  uint32_t E2[NP], B2[NP];
  int anchor = 0;  // Tot_NOFF: the diagonal just past this lane's offsets
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    E2[q] = RK ? 0u : (static_cast<uint32_t>(KMASK) << 16) | KMASK;  // E_o(-1) = KMASK: D 0, k 0
    B2[q] = 0x80008000u;  // (INT16_MIN, INT16_MIN)
  }
#pragma unroll
  for (int i0 = 0; i0 < 4 * L2W; i0 += kCopies) {
    if (i0 >= steps) break;  // wave-uniform
#pragma unroll
    for (int s = 0; s < kCopies; ++s) {
      const int i = i0 + s;
      // wave-uniform (scalar branch): a wave stops at its longest record, not at the next multiple of
      // kCopies steps; the copy index s stays a compile-time constant
      if (i >= steps) break;
      const int c = (wd[i >> 2] >> (8 * (i & 3))) & 0xff;
      // copy s holds column j' + s at j': columns i .. i + NOFF - 1 are the 8-byte chunks from column i0
      const unsigned char* rowp = smem + (s * cb + 2 * i0) + __umul24(c, stride);
      uint32_t v[NP];
#pragma unroll
      for (int q = 0; q < NOFF / 4; ++q) {
        // a relaxed atomic load: one ds_read_b64 per chunk (plain loads get paired into ds_read2_b64, which
        // reads at half the rate over 32 banks — conflicts again — and needs an address add per pair)
        const uint64_t x = __atomic_load_n(reinterpret_cast<const uint64_t*>(rowp + 8 * q), __ATOMIC_RELAXED);
        v[2 * q + 0] = static_cast<uint32_t>(x);
        v[2 * q + 1] = static_cast<uint32_t>(x >> 32);
      }
      anchor += at[32 * i + c];
#pragma unroll
      for (int q = 0; q < NP; ++q) E2[q] = as_u32(as_s16x2(E2[q]) + as_s16x2(v[q]));
#pragma unroll
      for (int q = 0; q < NP; ++q) B2[q] = as_u32(__builtin_elementwise_max(as_s16x2(B2[q]), as_s16x2(E2[q])));
    }
  }

  // ---- per-lane selection over the record's offsets: 32-bit keys (score + 2^15) << 16 | ~(o << KB | k),
  //      0 = none (RK: the low bits are ~(o << 1 | mutated)). The offsets run from the top down through one
  //      chain value C_o = (Tot_o + 2^15) << 16 + ~(o << KB | 0): the un-mutated candidate's key IS C_o, and
  //      the best mutant's key is C_{o+1} + ((d << 16) | (KMASK - k)) + 1 (d = its D_o(k)); so per offset one
  //      op takes D_o(L2) << 16 (plus the step of the index field) out of the packed sums, one add moves the
  //      chain, one byte permute builds the mutant's (d, k) word, one add3 its key and one max3 selects —
  //      five full-rate ops, half the former epilogue (round-5 roofline: a third of the kernel's issue).
  //      Mod-2^32 arithmetic is exact: every Tot_o + 2^15 and score + 2^15 fits 16 bits (the swipe_keys
  //      bound), and the index field never carries into the score.
  //      The valid offsets are prefixes: the un-mutated candidate at o < lim0 (o <= last = L1-L2 under the
  //      spec semantics or when L2 == L1, else o < last), the mutants at o < lim1 = last (L2 >= 2). Below
  //      wlo every searching lane's candidates are valid (no limit tests), from whi up none is (the chain
  //      only): both wave-uniform, applied per group of 4 offsets.
  const int last = L1 - L2;
  const bool spec = sem == static_cast<int>(Semantics::Spec);
  const int lim0 = on ? last + ((spec || L2 == L1) ? 1 : 0) : 0;
  const int lim1 = on && L2 >= 2 ? last : 0;
  const int wlo = __builtin_amdgcn_ballot_w64(on && L2 < 2) != 0 ? 0 : L1 - steps;
  const int wmin = 255 - wave_max_small(on ? 255 - L2 : 0);  // the wave's shortest searching record
  const int whi = max(L1 - wmin + (spec ? 1 : 0), 1);
  (void)max_l2;
  // packed per offset pair (one op per two offsets): D_o(L2) (E >> KB: E = D * 2^KB + KMASK - steps and
  // steps <= KMASK), the best mutant's D_o(k) and its KMASK - k
  uint32_t dq2[NP], bd2[NP], bl2[NP];
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    dq2[q] = RK ? E2[q] : as_u32(as_s16x2(E2[q]) >> static_cast<short>(KB));
    bd2[q] = RK ? B2[q] : as_u32(as_s16x2(B2[q]) >> static_cast<short>(KB));
    bl2[q] = RK ? 0u : B2[q] & (static_cast<uint32_t>(KMASK) * 0x10001u);
  }
  constexpr uint32_t kStep = 1u << KB;  // ~(o << KB) - ~((o + 1) << KB)
  uint32_t best = 0;
  // C_NOFF from the anchor diagonal Tot_NOFF (the index field may borrow: only C_o for o < NOFF is a key)
  uint32_t C = (static_cast<uint32_t>(anchor + 32768) << 16) + (0xffffu - (static_cast<uint32_t>(NOFF) << KB));
  auto offset = [&](const int o, const int mode) {  // mode 0: valid everywhere, 1: limit tests, 2: chain only
    const int q = o >> 1;
    const bool hi = o & 1;
    const uint32_t ds = hi ? (dq2[q] & 0xffff0000u) | kStep : (dq2[q] << 16) | kStep;
    if (mode == 2) {
      C += ds;
      return;
    }
    // (d << 16) | (KMASK - k): the halves of the pair's packed D and k words (RK: d << 16)
    const uint32_t m = RK ? (hi ? bd2[q] & 0xffff0000u : bd2[q] << 16)
                          : __builtin_amdgcn_perm(bd2[q], bl2[q], hi ? 0x07060302u : 0x05040100u);
    uint32_t k1 = C + m + 1u;  // the best mutant of offset o, from C_{o+1}
    C += ds;                   // C_o
    uint32_t k0 = C;           // the un-mutated candidate of offset o
    if (mode == 1) {
      k0 = o < lim0 ? k0 : 0u;
      k1 = o < lim1 ? k1 : 0u;
    }
    best = max(best, max(k0, k1));
  };
  // groups of 4 offsets, from the top (one wave-uniform branch per group, not per offset)
#pragma unroll
  for (int g = NOFF / 4 - 1; g >= 0; --g) {
    if (4 * g >= whi) {
#pragma unroll
      for (int o = 4 * g + 3; o >= 4 * g; --o) offset(o, 2);
    } else if (4 * g + 3 >= wlo) {
#pragma unroll
      for (int o = 4 * g + 3; o >= 4 * g; --o) offset(o, 1);
    } else {
#pragma unroll
      for (int o = 4 * g + 3; o >= 4 * g; --o) offset(o, 0);
    }
  }
  if (!on) best = 0u;
  int kw = 0;  // RK: the winning mutant's k
  if (RK) {
    // the first k of the winning offset's diagonal with the largest D_o(k): a mutant wins only with a D
    // above D_o(L2) (at k >= L2 the sums stay D_o(L2), and the un-mutated candidate wins that tie), so
    // that k is below L2
    const bool walk = best != 0u && ((0xffffu - (best & 0xffffu)) & 1u);
    if (__builtin_amdgcn_ballot_w64(walk) != 0) {  // wave-uniform
      const int ow = static_cast<int>((0xffffu - (best & 0xffffu)) >> 1);
      int run = 0, top = INT32_MIN;
#pragma unroll
      for (int i = 0; i < 4 * L2W; ++i) {
        if (i >= steps) break;  // wave-uniform
        const int c = (wd[i >> 2] >> (8 * (i & 3))) & 0xff;
        run += *reinterpret_cast<const short*>(smem + __umul24(c, stride) + 2 * (ow + i));  // copy 0: column ow + i
        kw = run > top ? i + 1 : kw;
        top = max(top, run);
      }
    }
  }
  if (best == 0u) return Result{INT32_MIN, 0, 0};
  const uint32_t idx = 0xffffu - (best & 0xffffu);
  return RK ? Result{static_cast<int>(best >> 16) - 32768, static_cast<int>(idx >> 1), (idx & 1u) ? kw : 0}
            : Result{static_cast<int>(best >> 16) - 32768, static_cast<int>(idx >> KB), static_cast<int>(idx & KMASK)};
}

// LF: letter format of `a.codes` — 0 bytes, 2 P33 fields (decoded to bytes in LDS per tile).
// RK: keys without k bits (the weights leave no room for them in int16): the running sums are plain
// D_o(k), B2 keeps max_k D_o(k), and the winner's k is re-found afterwards on its diagonal.
template <int NOFF, int L2W, int LF, bool RK>
__global__ __launch_bounds__(kBlock) void swipe_search_kernel(ProblemView pv, ShortArgs a, SwipeLayout lay) {
  constexpr bool P33 = LF == 2;
  constexpr int kRpt = rpt_of(LF);
  constexpr int NW = L2W;  // record words (4 letters each) held per lane
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int* loff = reinterpret_cast<int*>(smem + lay.loff_off);
  int* misc = loff + a.tile_records + 1;
  uint8_t* codes_l = smem + lay.codes_off;
  uint8_t* res_l = smem + lay.res_off;
  uint8_t* raw_l = smem + lay.raw_off;  // P33: the tile's encoded bytes as loaded
  const int L1 = pv.L1;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int KB = RK ? 1 : bounds::swipe_kbits(L2W);  // k bits of the int16 keys (moc/kernel_bounds.hpp)

  const int fb = fmt_bytes(a.fmt);
  // tiles [0, tail_from) hold tile_records records, the rest tail_records (the batch's last work, cut finer
  // so the blocks finish together)
  const int64_t big_end = a.tail_records ? min(a.n, a.tail_from * a.tile_records) : a.n;
  const int64_t n_tiles = a.tail_records ? a.tail_from + (a.n - big_end + a.tail_records - 1) / a.tail_records
                                         : (a.n + a.tile_records - 1) / a.tile_records;
  auto tile_first = [&](int64_t t) -> int64_t {
    return t < a.tail_from ? t * a.tile_records : big_end + (t - a.tail_from) * a.tail_records;
  };
  auto tile_size = [&](int64_t t) -> int64_t { return t < a.tail_from ? a.tile_records : a.tail_records; };
  const int sem = pv.semantics;
  const bool spec = sem == static_cast<int>(Semantics::Spec);

  // ---- tile fetch: the next tile's lengths and letters are loaded into registers while the current
  //      tile is being scored, so the PCIe / HBM read latency hides behind the compute (the streaming
  //      path is bound by host-link bytes: keep the link busy all the time).
  // Byte-letter batches without narrow lengths (device-resident: records by dense offsets) load their
  // tile's offsets in fetch() and take the lengths from them when the tile is staged: subtracting at the load
  // would make every thread wait there for the loads' return, so the next tile's loads would not stay in
  // flight behind the current tile's scoring (device-resident input6 0.573 -> 0.547 ms,
  // profiles/swipe_lds_ab_r4/). Narrow length forms (the host streams') decode at the load: deferring the
  // base-6 words measured 0.2 % slower on the headline.
  constexpr bool kDeferLens = LF == 0 && kRpt == 4;
  struct Fetch {
    int64_t t, rb, start, end;
    int m;
    int lens[kRpt];
    uintptr_t a0;
    int nvec;
    uint4 v[kMaxV];
    bool lo_set;    // kDeferLens: lens still to be taken from lo
    int64_t lo[5];  // this thread's 4 records' offsets and the next
  };
  auto fetch = [&](int64_t t, Fetch& f) {
    f.t = t;
    f.rb = f.start = f.end = 0;
    f.m = f.nvec = 0;
    f.a0 = 0;
#pragma unroll
    for (int k = 0; k < kMaxV; ++k) f.v[k] = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int q = 0; q < kRpt; ++q) f.lens[q] = 0;
    f.lo_set = false;
    if (t >= n_tiles) return;
    f.rb = tile_first(t);
    f.m = static_cast<int>(min(tile_size(t), a.n - f.rb));
    // the tile's letter range: loaded once per block by grab(), not once per wave (each load of host
    // memory is a PCIe read request of its own)
    f.start = static_cast<int64_t>((static_cast<uint64_t>(static_cast<uint32_t>(misc[9])) << 32) |
                                   static_cast<uint32_t>(misc[8]));
    f.end = static_cast<int64_t>((static_cast<uint64_t>(static_cast<uint32_t>(misc[11])) << 32) |
                                 static_cast<uint32_t>(misc[10]));
#pragma unroll
    for (int h = 0; h < kRpt / 4; ++h) {  // this thread's kRpt records' lengths, 4 per load
      int l4[4];
      const int r0 = tid * kRpt + 4 * h;
      const int nv = min(4, max(0, f.m - r0));
      if constexpr (kDeferLens) {
        if (!a.lengths3 && !a.lengths4 && !a.lengths6 && !a.lengths8 && !a.off_shift) {
          const int64_t i0 = f.rb + r0;
#pragma unroll
          for (int q = 0; q < 5; ++q) f.lo[q] = nv > 0 && q <= nv ? a.offsets[i0 + q] : 0;  // <= offsets[n]
          f.lo_set = true;
          continue;
        }
      }
      record_lengths4(a, f.rb + r0, nv, l4);
#pragma unroll
      for (int q = 0; q < 4; ++q) f.lens[4 * h + q] = l4[q];
    }
    const int64_t b_first = P33 ? (33 * (f.start / 7)) >> 3 : f.start;
    const int64_t b_end = P33 ? (33 * ((f.end + 6) / 7) + 7) >> 3 : f.end;
    f.a0 = reinterpret_cast<uintptr_t>(a.codes + b_first) & ~uintptr_t{15};
    f.nvec = static_cast<int>((reinterpret_cast<uintptr_t>(a.codes + b_end) + 15 - f.a0) >> 4);
    MOC_DCHECK(f.nvec <= kMaxV * kBlock);
#pragma unroll
    for (int k = 0; k < kMaxV; ++k) {
      const int v = tid + k * kBlock;
      if (v < f.nvec) f.v[k] = nt_load16(reinterpret_cast<const uint4*>(f.a0) + v);
    }
  };
  auto grab = [&]() -> int64_t {
    if (tid == 0) {
      const int64_t t = atomicAdd(a.counter, 1u);
      misc[0] = static_cast<int>(t);
      if (t < n_tiles) {  // the tile's letter range [offsets[rb], offsets[rb + m]) for fetch()
        const int64_t rb = tile_first(t);
        const int64_t st = tile_offset(a, rb), en = tile_offset(a, min(rb + tile_size(t), a.n));
        misc[8] = static_cast<int>(static_cast<uint32_t>(st));
        misc[9] = static_cast<int>(static_cast<uint64_t>(st) >> 32);
        misc[10] = static_cast<int>(static_cast<uint32_t>(en));
        misc[11] = static_cast<int>(static_cast<uint64_t>(en) >> 32);
      }
    }
    __syncthreads();
    const int64_t t = misc[0];
    return t;
  };

  Fetch cur, nxt;
  fetch(grab(), cur);  // the first tile's loads are in flight while the block builds its profile

  swipe_build_tables<RK, KB, NOFF, L2W>(smem, pv, tid, kBlock);
  for (;;) {
    if (cur.t >= n_tiles) break;
    const int64_t rb = cur.rb, start = cur.start, end = cur.end;
    const int m = cur.m;
    __syncthreads();  // the previous tile's LDS (loff, letters, results) is free again

    // ---- lengths -> block exclusive scan -> loff[0..m]
    if constexpr (kDeferLens) {
      if (cur.lo_set) {  // the lengths fetch() left as offsets
        const int nv = min(4, max(0, m - tid * kRpt));
#pragma unroll
        for (int q = 0; q < 4; ++q) cur.lens[q] = q < nv ? static_cast<int>(cur.lo[q + 1] - cur.lo[q]) : 0;
      }
    }
    int sum = 0;
#pragma unroll
    for (int q = 0; q < kRpt; ++q) sum += cur.lens[q];
    const int incl = wave_inclusive_sum(sum, lane);
    if (lane == 63) misc[4 + wave] = incl;
    // ---- letters -> LDS. Byte codes: char j at byte j. P33: the fields land in raw_l and are decoded into
    //      bytes below (field f0 = start / 7 -> codes_l[0..]).
    //      shift_b = position of the tile's first char inside the LDS copy.
#pragma unroll
    for (int k = 0; k < kMaxV; ++k) {
      const int v = tid + k * kBlock;
      if (v < cur.nvec) reinterpret_cast<uint4*>(P33 ? raw_l : codes_l)[v] = cur.v[k];
    }
    const uintptr_t p0 = reinterpret_cast<uintptr_t>(a.codes + start);
    const int shift_b = P33 ? static_cast<int>(start - 7 * (start / 7)) : static_cast<int>(p0 - cur.a0);
    if (tid == 0) {
      MOC_DCHECK(a.dbg_codes_end < 0 || cur.a0 + 16 * static_cast<uintptr_t>(cur.nvec) <=
                                            reinterpret_cast<uintptr_t>(a.codes) + a.dbg_codes_end);
      MOC_DCHECK(end >= start && m > 0 && m <= a.tile_records);
      MOC_DCHECK(end - start + 32 <= a.codes_cap);
    }
    __syncthreads();
    int excl = incl - sum;
    for (int w = 0; w < wave; ++w) excl += misc[4 + w];
#pragma unroll
    for (int q = 0; q < kRpt; ++q) {
      const int r = tid * kRpt + q;
      if (r < m) loff[r] = excl;
      excl += cur.lens[q];
    }
    if (tid == kBlock - 1) {
      loff[m] = excl;
      MOC_DCHECK(excl == end - start);  // lengths agree with offsets
    }
    if (P33) {  // 33-bit fields -> byte codes 1..26 (the staged bytes are complete: synchronised above)
      const int64_t f0 = start / 7;
      const int nf = static_cast<int>((end + 6) / 7 - f0);
      const int64_t byte0 = (33 * f0) >> 3;
      const int ro = static_cast<int>(reinterpret_cast<uintptr_t>(a.codes + byte0) - cur.a0);
      const int bit0 = static_cast<int>((33 * f0) & 7);
      for (int f = tid; f < nf; f += kBlock) {
        const int bit = bit0 + 33 * f;
        const uint8_t* r = raw_l + ro + (bit >> 3);
        // 33 bits at a 0..7-bit offset lie in 5 bytes (bits past the field are masked off)
        const uint64_t w = r[0] | (static_cast<uint32_t>(r[1]) << 8) | (static_cast<uint32_t>(r[2]) << 16) |
                           (static_cast<uint32_t>(r[3]) << 24) | (static_cast<uint64_t>(r[4]) << 32);
        const uint64_t x = (w >> (bit & 7)) & 0x1FFFFFFFFull;
        uint32_t v = static_cast<uint32_t>(x >> 1) / 13u;  // x / 26 in 32-bit arithmetic
        uint8_t* d = codes_l + 7 * f;
        d[0] = static_cast<uint8_t>(static_cast<uint32_t>(x) - 26u * v + 1u);  // x - 26q < 26: exact mod 2^32
#pragma unroll
        for (int j = 1; j < 7; ++j) {
          const uint32_t q = v / 26u;
          d[j] = static_cast<uint8_t>(v - 26u * q + 1u);
          v = q;
        }
      }
    }
    // next tile: its loads are in flight while this one is scored
    fetch(grab(), nxt);  // grab() synchronises: loff / letters (decoded P33) are complete

    // ---- one record per lane
    for (int g = wave; g * 64 < m; g += 4) {
      const int rl = g * 64 + lane;
      const bool in = rl < m;
      int L2 = 0, rs = 0;
      if (in) {
        rs = shift_b + loff[rl];  // byte position in LDS
        L2 = loff[rl + 1] - loff[rl];
      }
      const bool mine = in && (L2 < L1 ? L1 - L2 + (spec ? 1 : 0) : 1) <= NOFF;  // others belong to the tile kernel (mixed batches)
      const bool on = mine && L2 <= L1;
      uint32_t wd[NW];
      record_words<NW>(reinterpret_cast<const uint32_t*>(codes_l), rs, L2, on, wd);
      const Result res = swipe_lane<NOFF, L2W, RK>(smem, wd, L2, on, L1, a.max_l2, sem);
      if (mine) store_result(res_l, rl, a.fmt, res, pv.r2);
    }
    __syncthreads();
    copy_results(static_cast<char*>(a.out) + rb * fb, res_l, m * fb, tid, kBlock);
    cur = nxt;
  }
  release_work_counter(a.counter);
}


// Device-resident batches (solve_device, the staged chunks, the rccl transport's batches): each WAVE takes 64
// consecutive records at a time, one per lane, straight from device memory — no block scan and no barrier
// after the block's tables are built. (The block-synchronous tile pipeline of swipe_search_kernel — grab,
// barrier, scan, barrier, copy — held device-resident input6 at ~0.45 of its 0.54 ms even with the hot loop
// removed, round 4's A/B.) Waves walk the tiles t = wave, wave + waves, ... (64 records, or 128 as two
// halves: direct_halves) and load the next tile's offsets (or lengths) while the current one is scored.
//   LF 0: byte letters, dense offsets — a lane loads its record's aligned words itself.
//   LF 2: P33 fields (the wire format: 33 bits per 7 letters) with dense or 64-record sparse offsets and
//         narrow lengths — the wave's tile starts at tile_offset, its lanes' starts come from wave prefix
//         sums of the lengths, lanes decode the tile's fields (field = lane, lane + 64, ...; digit pairs
//         from an LDS table) into 8-byte slots of a wave-private LDS slice (one ds_write_b64 per field:
//         seven byte stores cost +62 % LDS cycles), and each lane gathers its record's words from there
//         (wave-level ordering only: the slice is the wave's own).
constexpr int kBlockD = 512;  // 8 waves share one set of LDS tables
// P33 tiles: one 8-byte slot per field (7 letters + a pad byte) for the fields a tile of records of at most
// max_l2 letters can span, plus the slots a lane's read may run past the last one. Sized by the batch's
// longest record, not by the instance's record words: LDS decides how many blocks share a CU.
constexpr int p33_tile_fields(int records, int max_l2) { return (records * max_l2 + 6) / 7 + 1; }
constexpr int p33_lane_slots(int l2w) { return (4 * l2w + 8 + 6) / 7; }  // the letters of words 0..l2w+1
// 64-record halves per lane-direct tile: P33 records of at most 16 letters with at most 20 offsets per lane
// decode the fields of 128 records at once, so the last, partly idle round of 64 fields comes once per 128
// records (input6: 156 fields in 3 rounds instead of 2 x 78 in 2 + 2). Those instances fit 64 VGPRs (8
// waves per SIMD, amdgpu_waves_per_eu below) without spills; wider ones would spill, and their sweep
// outweighs the decode more.
constexpr int direct_halves(int lf, int l2w, int noff) { return lf == 2 && l2w == 4 && noff <= 20 ? 2 : 1; }
inline SwipeLayout direct_layout(int L1, int noff, int l2w, int lf, int64_t max_l2) {
  SwipeLayout l = swipe_layout(L1, noff, l2w, 0, 0, 0, 0);
  if (lf == 2) {
    const int ml = static_cast<int>(std::min<int64_t>(std::max<int64_t>(max_l2, 1), 4 * l2w));
    l.wave_bytes = 8 * (p33_tile_fields(64 * direct_halves(lf, l2w, noff), ml) + p33_lane_slots(l2w) + 1);
    l.pairs_off = al16(l.s_off + swipe_anchor_bytes(l2w));
    l.codes_off = l.pairs_off + al16(2 * 676);
    l.total = l.codes_off + (kBlockD / 64) * l.wave_bytes;
  }
  return l;
}

// Exclusive prefix sum over the lanes of a wave on the DPP network (row shifts, then row broadcasts).
__device__ __forceinline__ int wave_exclusive_sum_dpp(int v) {
  int x = v;
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return x - v;
}

// P33 field f of a tile (33 bits at bit b0 + 33 f of the 32-bit words from base32): its two words are
// loaded first (p33_field_words, for several fields at once), then decoded to the 7 letter codes 1..26.
// Digits by 24-bit multiplies (full rate) after one 32-bit multiply-high: x < 26^7 splits into
// A = x / 26^4 = (x / 16) / 13^4 (umulhi by ceil(2^46 / 28561), >> 14: exact for x / 16 < 2^29) and
// B = x - 26^4 A < 2^19 (wrapping 32-bit arithmetic); B / 676 and A / 676 by v_mul_hi_u32_u24 with
// ceil(2^32 / 676) (exact below 2^19), and a pair v < 676 -> (v % 26, v / 26) as the two bytes
// v + 230 (v / 26), v / 26 = (2521 v) >> 16 (exact below 676). All constants checked exhaustively over
// their ranges (tools/p33_magic_check.py).
__device__ __forceinline__ void p33_field_words(const uint32_t* base32, int b0, int f, uint32_t& lo, uint32_t& hi) {
  const uint32_t* w = base32 + ((b0 + 33 * f) >> 5);
  lo = __builtin_nontemporal_load(w);
  hi = __builtin_nontemporal_load(w + 1);
}
__device__ __forceinline__ uint32_t mulhi_u24(uint32_t a, uint32_t b) {  // bits 32..47 of the 24 x 24-bit product
  uint32_t r;
  asm("v_mul_hi_u32_u24 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ uint32_t mad_i24(uint32_t a, int b, uint32_t c) {  // a * b + c, a and b signed 24-bit
  // (written out: the compiler folds c - a * 676 into a quarter-rate v_mul_lo_u32 by -676)
  uint32_t r;
  asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(b), "v"(c));
  return r;
}
__device__ __forceinline__ uint32_t p33_pair(uint32_t v) {  // v < 676 -> bytes (v % 26, v / 26)
  return __umul24(__umul24(v, 2521u) >> 16, 230u) + v;
}
__device__ __forceinline__ uint2 decode_p33_field(uint32_t lo, uint32_t hi, int b0, int f) {
  const uint64_t ww = static_cast<uint64_t>(lo) | (static_cast<uint64_t>(hi) << 32);
  const uint64_t x = (ww >> ((b0 + 33 * f) & 31)) & 0x1FFFFFFFFull;
  const uint32_t A = __umulhi(static_cast<uint32_t>(x >> 4), 2463805336u) >> 14;  // digits 4..6
  const uint32_t B = static_cast<uint32_t>(x) - __umul24(A, 456976u);  // digits 0..3
  const uint32_t b32 = mulhi_u24(B, 6353502u), a2 = mulhi_u24(A, 6353502u);
  const uint32_t b10 = mad_i24(b32, -676, B), a10 = mad_i24(a2, -676, A);
  // letter codes are digit + 1; the pad byte stays 0
  return make_uint2((p33_pair(b10) | (p33_pair(b32) << 16)) + 0x01010101u, (p33_pair(a10) | (a2 << 16)) + 0x00010101u);
}

// The lane-direct kernel's decode: the same digits, each pair of them (v < 676) one LDS read of a table of
// 16-bit letter-code pairs (built once per block) instead of three multiply-adds.
__device__ __forceinline__ void build_p33_pair_table(uint16_t* pairs, int tid, int nthreads) {
  for (int v = tid; v < 676; v += nthreads)
    pairs[v] = static_cast<uint16_t>((v % 26 + 1) | ((v / 26 + 1) << 8));
}
__device__ __forceinline__ uint2 decode_p33_field_lut(uint32_t lo, uint32_t hi, int b0, int f, const uint16_t* pairs) {
  const uint64_t ww = static_cast<uint64_t>(lo) | (static_cast<uint64_t>(hi) << 32);
  const uint64_t x = (ww >> ((b0 + 33 * f) & 31)) & 0x1FFFFFFFFull;
  const uint32_t A = __umulhi(static_cast<uint32_t>(x >> 4), 2463805336u) >> 14;  // digits 4..6
  const uint32_t B = static_cast<uint32_t>(x) - __umul24(A, 456976u);  // digits 0..3
  const uint32_t b32 = mulhi_u24(B, 6353502u), a2 = mulhi_u24(A, 6353502u);
  const uint32_t b10 = mad_i24(b32, -676, B), a10 = mad_i24(a2, -676, A);
  return make_uint2(pairs[b10] | (static_cast<uint32_t>(pairs[b32]) << 16), pairs[a10] | ((a2 + 1u) << 16));
}

// The letters of a lane's record from the tile's 8-byte field slots: NS slots from the record's first field
// (ds_read_b64 each), compacted to contiguous words (one v_perm_b32 each: 4 consecutive letters lie in at most
// two of the slots' dwords), then shifted by the record's start within its first field (0..6 letters) and
// masked past its end as record_words does.
template <int NW>
__device__ __forceinline__ void record_words_p33(const uint8_t* slots, int q0, int L2, bool on, uint32_t (&wd)[NW]) {
  constexpr int NS = p33_lane_slots(NW);
  static_assert(NW <= 16, "the 24-bit q0 / 7 below needs q0 < 13110");
  // q0 / 7 by a 24-bit multiply (exact below 13110; q0 <= 6 + 63 * 4 * NW <= 4038 in 64-record tiles,
  // 6 + 127 * 4 * NW <= 4070 in 128-record ones, NW <= 8), q0 % 7 by a 24-bit mad
  const int fa = static_cast<int>(__umul24(static_cast<uint32_t>(q0), 9363u) >> 16);
  const int sh = static_cast<int>(mad_i24(static_cast<uint32_t>(fa), -7, static_cast<uint32_t>(q0)));
  uint32_t dw[2 * NS];
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    uint2 v = make_uint2(0u, 0u);
    if (on) v = *reinterpret_cast<const uint2*>(slots + 8 * (fa + k));
    dw[2 * k] = v.x;
    dw[2 * k + 1] = v.y;
  }
  // compact word c: letters 4c..4c+3 = slot (i / 7) byte (i % 7); byte b of slot k is dw[2k + b / 4] byte b % 4
  constexpr int NC = NW + 2;
  uint32_t cw[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int i0 = 4 * c;
    const int d_first = 2 * (i0 / 7) + (i0 % 7) / 4;  // dword of letter i0
    uint32_t sel = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int i = i0 + b;
      const int dwi = 2 * (i / 7) + (i % 7) / 4, byte = (i % 7) % 4;
      // v_perm_b32(S0 = dw[d_first + 1], S1 = dw[d_first]): selector 0-3 picks S1 bytes, 4-7 S0 bytes
      sel |= static_cast<uint32_t>((dwi == d_first ? 0 : 4) + byte) << (8 * b);
    }
    const uint32_t s1 = d_first < 2 * NS ? dw[d_first] : 0u;
    const uint32_t s0 = d_first + 1 < 2 * NS ? dw[d_first + 1] : 0u;
    cw[c] = __builtin_amdgcn_perm(s0, s1, sel);
  }
  const bool hs = sh >= 4;
  const int bs = (sh & 3) * 8;
  const int rbits = 8 * L2;
#pragma unroll
  for (int k = 0; k < NW; ++k) {
    const uint32_t lo = hs ? cw[k + 1] : cw[k], hi = hs ? cw[k + 2] : cw[k + 1];
    uint32_t w = bs ? ((lo >> bs) | (hi << (32 - bs))) : lo;
    const int left = rbits - 32 * k;  // record bits in this word
    w = left >= 32 ? w : (left <= 0 ? 0u : (w & ((1u << left) - 1u)));
    wd[k] = on ? w : 0u;
  }
}

// Length of record 64 t + lane of a batch with base-6 lengths (three 21-bit octets of 8 digits per 8-byte
// word): the tile's first octet 8 t splits into its word and position once per wave (scalar), a lane adds its
// octet lane / 8 with 24-bit arithmetic, and digit j = lane % 8 of the octet's value v < 2^21 is
// (v / 6^j) - 6 (v / 6^(j+1)), each quotient trunc((v + 0.5) * fl(1 / 6^i)) in f32 — exact for every
// v < 2^21 and i <= 8 (v + 0.5 is exact, one rounding in the product; tools/p33_magic_check.py checks all
// of them). Full-rate ops only: the 32-bit multiply-highs this replaces issue at a quarter of the rate.
struct Len6Digit {
  float r = 1.f, r6 = 1.f;  // fl(1 / 6^j), fl(1 / 6^(j+1)) for j = lane % 8
  uint32_t octet = 0;       // lane / 8
};
__device__ __forceinline__ Len6Digit len6_digit(int lane) {
  constexpr float kR[9] = {1.0f, 1.0f / 6, 1.0f / 36, 1.0f / 216, 1.0f / 1296, 1.0f / 7776, 1.0f / 46656,
                           1.0f / 279936, 1.0f / 1679616};
  Len6Digit d;
  const int j = lane & 7;
#pragma unroll
  for (int k = 0; k < 8; ++k)
    if (j == k) {
      d.r = kR[k];
      d.r6 = kR[k + 1];
    }
  d.octet = static_cast<uint32_t>(lane >> 3);
  return d;
}
__device__ __forceinline__ int lane_length6(const ShortArgs& a, int64_t t, Len6Digit dg) {
  const uint32_t o8 = static_cast<uint32_t>(t) * 8u;  // wave-uniform (t < 2^28)
  const uint32_t sw = o8 / 3u;
  const uint32_t sr = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(o8 - 3u * sw)));
  const uint32_t u = sr + dg.octet;  // <= 9
  const uint32_t dw = __umul24(u, 11u) >> 5, rem = u - __umul24(dw, 3u);  // u / 3, u % 3
  const uint64_t w = *reinterpret_cast<const uint64_t*>(a.lengths6 + 8 * static_cast<uint64_t>(sw + dw));
  const uint32_t v = static_cast<uint32_t>(w >> __umul24(rem, 21u)) & 0x1FFFFFu;
  const float fv = static_cast<float>(v) + 0.5f;
  const int q = static_cast<int>(fv * dg.r), q6 = static_cast<int>(fv * dg.r6);
  return a.len_base + static_cast<int>(mad_i24(static_cast<uint32_t>(q6), -6, static_cast<uint32_t>(q)));
}

template <int NOFF, int L2W, int LF, bool RK>
// (instances of >= 56 offsets per lane and <= 24 record words held to 128 VGPRs: 4 waves per SIMD instead of
// 2, mid 13.6 -> 15.0 T; <64, 24> keeps one 8-byte spill per tile, outside the sweep)
__global__ __launch_bounds__(kBlockD) __attribute__((amdgpu_waves_per_eu(direct_halves(LF, L2W, NOFF) == 2 ? 8 : NOFF >= 56 && L2W <= 24 ? 4 : 1)))
void swipe_direct_kernel(ProblemView pv, ShortArgs a, SwipeLayout lay) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr bool P33 = LF == 2;
  constexpr int KB = RK ? 1 : bounds::swipe_kbits(L2W);
  swipe_build_tables<RK, KB, NOFF, L2W>(smem, pv, threadIdx.x, kBlockD);
  uint16_t* pairs = reinterpret_cast<uint16_t*>(smem + lay.pairs_off);
  if constexpr (P33) build_p33_pair_table(pairs, threadIdx.x, kBlockD);
  __syncthreads();  // the only barrier: tables complete
  const int lane = threadIdx.x & 63;
  const bool spec = pv.semantics == static_cast<int>(Semantics::Spec);
  const int L1 = pv.L1;
  constexpr int H = direct_halves(LF, L2W, NOFF);  // 64-record halves per tile
  const int64_t n = a.n, n_tiles = (n + 64 * H - 1) / (64 * H);
  const int64_t waves = static_cast<int64_t>(gridDim.x) * (kBlockD / 64);
  // the wave's tile index, its tile start (P33) and the loop bounds live in scalar registers
  int64_t t = static_cast<int64_t>(blockIdx.x) * (kBlockD / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const Len6Digit dg = len6_digit(lane);
  uint8_t* wbuf = smem + lay.codes_off + (threadIdx.x >> 6) * lay.wave_bytes;  // P33: this wave's
  // bytes: the record's offsets; P33: the tile's first letter (o0, every lane) and the records' lengths (o1)
  using Len = std::conditional_t<P33, int, int64_t>;  // P33: a length; bytes: the record's end offset
  auto uniform64 = [](int64_t v) {
    return static_cast<int64_t>(
        (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(v >> 32))))
         << 32) |
        static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(v))));
  };
  auto load_meta = [&](int64_t tt, int64_t& o0, Len (&o1)[H]) {
    if constexpr (P33) {
      // tiles of 64 H records: boundaries of sparse (64-record) offsets too
      o0 = uniform64(tt < n_tiles ? tile_offset(a, tt * 64 * H) : 0);
#pragma unroll
      for (int h = 0; h < H; ++h) {
        const int64_t t64 = tt * H + h, r = (t64 << 6) + lane;
        const bool in = tt < n_tiles && r < n;
        o1[h] = !in ? 0
                    : a.lengths6 && t64 < (int64_t{1} << 28) ? lane_length6(a, t64, dg)
                                                              : static_cast<int>(record_length(a, r));
      }
    } else {
      const int64_t r = (tt << 6) + lane;
      const bool in = tt < n_tiles && r < n;
      o0 = in ? a.offsets[r] : 0;
      o1[0] = in ? a.offsets[r + 1] : 0;
    }
  };
  // P33 fields: lanes take fields lane, lane + 64, ... of a tile, the words of up to kBatch fields per lane
  // loaded before any is decoded. (Loading the next tile's words while this one is scored held 18 more
  // VGPRs across the sweep: 4 waves per SIMD instead of 8, and 7 % slower on input6.)
  constexpr int kIters = (p33_tile_fields(64 * H, 4 * L2W) + 63) / 64;  // fields a tile can span / 64
  constexpr int kBatch = kIters < 4 ? kIters : 4;
  int64_t o0;
  Len o1[H];
  load_meta(t, o0, o1);
  for (; t < n_tiles; t += waves) {  // wave-uniform
    uint32_t wd[L2W];
    int L2h[H], excl[H];  // the halves' lengths and (P33) their records' starts within the tile
#pragma unroll
    for (int h = 0; h < H; ++h) L2h[h] = static_cast<int>(P33 ? o1[h] : o1[0] - o0);
    auto searching = [&](int h, int L2) {  // others belong to the tile kernel
      return ((t * H + h) << 6) + lane < n && (L2 < L1 ? L1 - L2 + (spec ? 1 : 0) : 1) <= NOFF;
    };
    int s0 = 0;
    if constexpr (P33) {
      // the tile's first letter and field (wave-uniform: scalar arithmetic), the lanes' starts within the tile
      const int64_t st = uniform64(o0);
      const int64_t f0 = st / 7;
      s0 = static_cast<int>(st - 7 * f0);
      int tot = 0;
#pragma unroll
      for (int h = 0; h < H; ++h) {
        const int e = wave_exclusive_sum_dpp(L2h[h]);
        excl[h] = tot + e;
        tot += __builtin_amdgcn_readlane(e + L2h[h], 63);
      }
      // (a batch whose records exceed its max_l2 gets wrong results, never another wave's slots)
      const int cap = (lay.wave_bytes >> 3) - p33_lane_slots(L2W) - 1;
      MOC_DCHECK((s0 + tot + 6) / 7 <= cap);
      const int nf = min((s0 + tot + 6) / 7, cap);
      const uint32_t* base32 = reinterpret_cast<const uint32_t*>(a.codes) + ((33 * f0) >> 5);
      const int b0 = static_cast<int>((33 * f0) & 31);
      for (int f0b = 0; f0b < nf; f0b += 64 * kBatch) {  // wave-uniform
        uint32_t lo[kBatch], hi[kBatch];
#pragma unroll
        for (int b = 0; b < kBatch; ++b) {  // unconditional (field 0 for lanes past the tile): one wait per batch
          const int f = f0b + 64 * b + lane;
          p33_field_words(base32, b0, f < nf ? f : 0, lo[b], hi[b]);
        }
#pragma unroll
        for (int b = 0; b < kBatch; ++b) asm volatile("" ::"v"(lo[b]), "v"(hi[b]));  // the loads stay ahead
        // of the decode's branches (the compiler would sink each into its branch, one wait per field)
#pragma unroll
        for (int b = 0; b < kBatch; ++b) {
          const int f = f0b + 64 * b + lane;
          if (f < nf) *reinterpret_cast<uint2*>(wbuf + 8 * f) = decode_p33_field_lut(lo[b], hi[b], b0, f, pairs);
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the slice's letters before any lane reads them
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
      // the aligned words holding the record's letters, and only those (never past its last letter's word)
      const int L2 = L2h[0];
      const bool on = searching(0, L2) && L2 <= L1;
      const uintptr_t p = reinterpret_cast<uintptr_t>(a.codes + o0);
      const uint32_t* w32 = reinterpret_cast<const uint32_t*>(p & ~uintptr_t{3});
      const int sh = static_cast<int>(p & 3) * 8;
      const int nwords = on ? ((sh >> 3) + L2 + 3) >> 2 : 0;
      uint32_t raw[L2W + 1];
#pragma unroll
      for (int k = 0; k <= L2W; ++k) raw[k] = k < nwords ? __builtin_nontemporal_load(w32 + k) : 0u;
      const int rbits = 8 * L2;
#pragma unroll
      for (int k = 0; k < L2W; ++k) {
        uint32_t w = sh ? ((raw[k] >> sh) | (raw[k + 1] << (32 - sh))) : raw[k];
        const int left = rbits - 32 * k;  // record bits in this word
        wd[k] = left >= 32 ? w : (left <= 0 ? 0u : (w & ((1u << left) - 1u)));
      }
    }
    int64_t n0;
    Len n1[H];
    load_meta(t + waves, n0, n1);  // in flight while this tile is scored
    // the second half's length and start in one register across the first half's sweep (VGPRs: 8 waves per
    // SIMD at 64)
    const uint32_t later = static_cast<uint32_t>(L2h[H - 1]) | (static_cast<uint32_t>(excl[H - 1]) << 8);
#pragma unroll 1
    for (int h = 0; h < H; ++h) {  // wave-uniform; one copy of the sweep
      const int L2 = h == 0 ? L2h[0] : static_cast<int>(later & 0xffu);
      const bool mine = searching(h, L2);
      const bool on = mine && L2 <= L1;
      MOC_DCHECK(!on || L2 <= a.max_l2);
      if constexpr (P33) {
        const int q0 = s0 + (h == 0 ? excl[0] : static_cast<int>(later >> 8));
        MOC_DCHECK(!on || 8 * (q0 / 7 + p33_lane_slots(L2W)) <= lay.wave_bytes);
        record_words_p33<L2W>(wbuf, q0, L2, on, wd);
      }
      const Result res = swipe_lane<NOFF, L2W, RK>(smem, wd, L2, on, L1, a.max_l2, pv.semantics);
      if (mine) store_result(a.out, ((t * H + h) << 6) + lane, a.fmt, res, pv.r2);
    }
    if constexpr (P33) __builtin_amdgcn_wave_barrier();  // every lane read the slice before the next tile's writes
    o0 = n0;
#pragma unroll
    for (int h = 0; h < H; ++h) o1[h] = n1[h];
  }
}

// Launches the instance of letter form LF with NO offsets per lane that `b` selects (b.rpw = record words,
// b.swipe_rk = RK); false when no instance matches.
// The lane-direct kernel's grid: every block resident at once (the waves stride over the tiles statically,
// so a block that only starts when another ends would run its share after everyone else), sized by the
// occupancy the instance reaches.
inline void launch_direct_instance(void (*kernel)(ProblemView, ShortArgs, SwipeLayout), const ProblemView& pv,
                                   const ShortArgs& b, const SwipeLayout& lay, int num_cus, hipStream_t stream) {
  constexpr int block = kBlockD;
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void*>(kernel), block, lay.total) !=
          hipSuccess ||
      occ < 1) {
    (void)hipGetLastError();
    occ = 1;
  }
  const int64_t tiles = (b.n + 63) >> 6;
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((tiles + block / 64 - 1) / (block / 64),
                                                                static_cast<int64_t>(occ) * num_cus));
  hipLaunchKernelGGL(kernel, dim3(static_cast<unsigned>(blocks)), dim3(block), lay.total, stream, pv, b, lay);
}

template <int NO, int LF>
bool launch_swipe_noff(const ProblemView& pv, const ShortArgs& b, const SwipeLayout& lay, dim3 grid, dim3 block,
                       int num_cus, hipStream_t stream) {
  const int l2w = b.rpw;
  const bool rk = b.swipe_rk != 0;
#define MOC_SWIPE_CASE(LW, RKV)                                                                              \
  if (l2w == LW && rk == RKV) {                                                                            \
    if constexpr (LF == 0 || LW <= 16) { /* P33 records over 64 letters: the block-tiled kernel */        \
      if (b.lane_direct) {                                                                                 \
        launch_direct_instance(&swipe_direct_kernel<NO, LW, LF, RKV>, pv, b, lay, num_cus, stream);       \
        return true;                                                                                       \
      }                                                                                                    \
    }                                                                                                      \
    hipLaunchKernelGGL((swipe_search_kernel<NO, LW, LF, RKV>), grid, block, lay.total, stream, pv, b, lay); \
    return true;                                                                                           \
  }
  MOC_SWIPE_CASE(4, false)
  MOC_SWIPE_CASE(8, false)
  MOC_SWIPE_CASE(4, true)
  MOC_SWIPE_CASE(8, true)
  MOC_SWIPE_CASE(12, true)  // records of 33..128 letters run the RK form only (configure_swipe)
  MOC_SWIPE_CASE(16, true)
  MOC_SWIPE_CASE(24, true)
  MOC_SWIPE_CASE(32, true)
#undef MOC_SWIPE_CASE
  return false;
}

// The instances live in one code object per (letter form, NOFF): swipe_group.inc, compiled once per pair by
// the Makefile and CMakeLists.txt. HIP loads a code object at the first launch of any kernel in it, so a
// job that runs one instance loads ~1/8 of a letter form's kernels (a 2 MB object of 40 kernels took
// 3.4 ms inside a tiny job's first launch on the box, profiles/hip_wall_trace_r4/).
#define MOC_SWIPE_FN_(LF, NO) launch_swipe_lf##LF##_n##NO
#define MOC_SWIPE_FN(LF, NO) MOC_SWIPE_FN_(LF, NO)
#define MOC_SWIPE_PRELOAD_FN_(LF, NO) preload_swipe_lf##LF##_n##NO
#define MOC_SWIPE_PRELOAD_FN(LF, NO) MOC_SWIPE_PRELOAD_FN_(LF, NO)
#define MOC_SWIPE_FOR_NOFF(X, LF)                                                                          \
  X(LF, 4) X(LF, 8) X(LF, 12) X(LF, 16) X(LF, 20) X(LF, 24) X(LF, 28) X(LF, 32) X(LF, 36) X(LF, 40) X(LF, 44) \
  X(LF, 48) X(LF, 52) X(LF, 56) X(LF, 60) X(LF, 64)
#define MOC_SWIPE_DECLARE(LF, NO)                                                                            \
  bool MOC_SWIPE_FN(LF, NO)(const ProblemView& pv, const ShortArgs& b, const SwipeLayout& lay, dim3 grid,    \
                            dim3 block, int num_cus, hipStream_t stream);                                    \
  void MOC_SWIPE_PRELOAD_FN(LF, NO)();
MOC_SWIPE_FOR_NOFF(MOC_SWIPE_DECLARE, 0)
MOC_SWIPE_FOR_NOFF(MOC_SWIPE_DECLARE, 2)
#undef MOC_SWIPE_DECLARE

}  // namespace dev
}  // namespace moc
