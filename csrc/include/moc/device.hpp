// Device (gfx950) launch API for the alignment-search kernels.
//
// Reference: ONE kernel launch per Seq2 record (cudaFunctions.cu:204-220), each followed by
// cudaDeviceSynchronize, launched with grid = ceil(rows*2000/1024) blocks of which at most two hold
// work, with a serial (offset, mutant) loop inside every thread (cudaFunctions.cu:116-167).
//
// Here: one launch per *batch*, three kernels chosen per batch (design: SURVEY.md §7.3):
//   * swipe kernel (swipe_kernels.hip): tiny problems (|Seq1| <= 200, |Seq2| <= 32, int16-exact
//     weights): one LANE per record, all of its offsets' running sums in registers as packed int16
//     pairs — two cells per VALU op, no cross-lane traffic; the headline (input6-shaped) path.
//   For the others parallelism is over offsets (diagonals): every lane owns one offset `o` and streams
//   over the Seq2 positions, keeping its running diagonal prefix sum P_o in a register; the neighbour
//   diagonal's P_{o+1} comes from lane+1 through a DPP wave shift, so a cell costs one LDS gather plus a
//   handful of VALU ops, and no atomics or barriers.
//   * short kernel: records whose offset range fits in a wave (L1-L2+1 <= 64 lanes) are packed
//     several per wave in fixed-width lane slots (the input6-shaped regime). Persistent blocks pull
//     tiles of ~1K records, stage their letters in LDS with 16-byte loads — straight from pinned host
//     memory when the batch lives there (zero-copy streaming: PCIe is the bound, so no staging copy) —
//     and score against a per-block LDS profile S[c][j] = T[c][Seq1[j]].
//   * tile kernel: longer offset ranges are cut into wave tiles of U x 63 offsets (lane 63 of each
//     sub-tile is its helper diagonal), walked by persistent waves in cost-balanced runs planned on the
//     host; partial maxima merge through one 64-bit atomicMax per record run on an order-free packed
//     key (score, -(o*L2+k)) — deterministic tie-break, no races (fixes B9).
//   * tile16 kernel (tile16_kernels.hip): the same kind of plan, two offsets per lane: one ds_read_u16
//     of an LDS-resident int8 difference profile feeds both, summed in the halves of one register
//     (2 SDWA adds + 1 v_pk_max_i16 per two cells, no cross-lane moves); Tot_o from one anchor diagonal
//     per tile + a suffix scan; the k of each record's winning offset recovered afterwards on that one
//     diagonal. Used whenever the weights and Seq1 fit it (T range <= 127, L1 <= 3052).
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>

#include "moc/common.hpp"
#include "moc/kernel_bounds.hpp"
#include "moc/wire.hpp"

namespace moc {

namespace dev {

constexpr int kWave = 64;
constexpr int kTileOffsets = 63;  // owned offsets per tile-kernel wave (lane 63 = helper diagonal)
constexpr int kSeq1Pad = 256;     // zero padding after Seq1 on device (branch-free over-reads)

// Problem resident on the device (uploaded once per problem; tiny).
struct ProblemView {
  const int32_t* lut;   // [32*32] fused pair scores
  const uint8_t* seq1;  // codes, L1 + kSeq1Pad bytes (padding = 0)
  int32_t L1;
  int32_t semantics;    // moc::Semantics
  int32_t key_shift;    // bits reserved for k in the int32 hot-loop key (0 -> 64-bit keys)
  R2Params r2;          // parameters of the R2 result format (when used)
  // tile16 kernel (moc/score_table.hpp Profile16): packed int8 pair D profile, 26 rows of L1 uint16
  // entries + overhang, padded to 16 bytes; null when the problem does not fit it (weights or LDS)
  const uint16_t* prof16 = nullptr;
  int32_t prof16_bytes = 0;
  int32_t max_abs_t = 0;  // max |T| over the table (int16-exactness checks of the packed kernels)
  int32_t mfma_sweep = 0; // 1: long records sweep on the matrix cores (tile_mfma_kernels.hip, MOC_MFMA=1)
  // Windowed tile16 (Seq1 longer than one LDS image holds): prof16 is the whole profile in device memory
  // (26 rows of L1 entries + overhang, prof16_entries in all) and every workgroup stages one window of
  // prof16_window columns of it (its plan's tiles all fall inside that window); prof16_bytes is then the
  // LDS size of a window's rows + overhang. 0 = the whole profile is the LDS image.
  int32_t prof16_window = 0;
  int64_t prof16_entries = 0;
  // 1: the tile16 sweep stages each byte pair widened to two int16 halves (whole images only; the LDS image
  // is then tile16_lds_bytes(2 * prof16_bytes, L1))
  int32_t prof16_wide = 0;
  // tile16: index bits of the 32-bit selection keys (bounds::tile16_key32_bits; 0 = 64-bit keys)
  int32_t t16_key_bits = 0;
  // 1: prof16 holds one int16 Dt per entry (weights past the byte pairs, bounds::profile16_i16_exact), staged
  // into widened images only
  int32_t prof16_i16 = 0;
  int32_t t16_slide = 0;               // tile16: sliding widened windows of prof16_window columns (2: the
                                       // two-workgroups-per-CU instance)
                                       // (tile16_slide_kernel; the plan's items and groups)
};

// Entries after the tile16 profile's last row: reads of wave-tile lanes past the valid offsets reach
// at most L1 + 128*U - 2 (U <= 4) into a row.
#ifndef MOC_PROF16_OVERHANG
#define MOC_PROF16_OVERHANG 512
#endif
constexpr int kProf16Overhang = MOC_PROF16_OVERHANG;  // minimum; >= the widest tile span (128 * U entries)
// LDS budget of one tile16 workgroup (the whole CU: a single workgroup may declare all 160 KiB).
constexpr int kProf16MaxLds = 160 * 1024;
// tile16 LDS image: profile (prof16_bytes, 16-aligned) | int8 LUT T[32][32] | Seq1 codes + pad (for
// the per-tile anchor diagonal). Bytes of the whole image.
constexpr int kProf16Lut8 = 1024;
inline int64_t tile16_lds_bytes(int64_t prof16_bytes, int64_t L1) {
  return prof16_bytes + kProf16Lut8 + ((L1 + 16 + 15) & ~int64_t{15});
}
// Widest window (columns) whose rows + 512-entry overhang + LUT + Seq1 window fit one CU's LDS.
// LDS bytes of a window's byte-pair rows + overhang (pv.prof16_bytes of a windowed view)
inline int64_t tile16_window_bytes(int64_t w) { return ((2 * (26 * w + kProf16Overhang)) + 15) & ~int64_t{15}; }
// The widest window one LDS image holds (wide: the entries widened to int16 pairs, twice the bytes)
inline int64_t tile16_max_window(bool wide = false) {
  const int64_t f = wide ? 2 : 1;
  int64_t w = (kProf16MaxLds - kProf16Lut8 - 32 - 2 * f * kProf16Overhang) / (2 * f * 26 + 1);
  while (w > 0 && tile16_lds_bytes(f * tile16_window_bytes(w), w) > kProf16MaxLds) --w;
  return w & ~int64_t{15};
}
// LDS bytes of the profile part of a tile16 workgroup image (pv.prof16_bytes of a whole-image view): the whole
// profile (26 rows of L1 entries + overhang) when it fits one CU — widened, for int16 entries, which only the
// widened image takes — else one window's rows. Always an LDS size (it never wraps, whatever L1: a long Seq1's
// int16 profile lives in device memory and the sliding windows stage it).
inline int32_t tile16_profile_lds_bytes(int64_t L1, int64_t overhang, bool i16) {
  const int64_t whole = ((2 * (26 * L1 + overhang)) + 15) & ~int64_t{15};
  const bool fits = tile16_lds_bytes(i16 ? 2 * whole : whole, L1) <= kProf16MaxLds;
  return static_cast<int32_t>(fits ? whole : tile16_window_bytes(tile16_max_window()));
}

// One batch of records on the device. Offsets are absolute (int64) and rebased by offsets[0], so
// a chunk of a bigger CSR array can be transferred and launched without host-side rebasing.
struct BatchView {
  const uint8_t* codes;     // codes of this chunk (codes[0] == record 0's first letter)
  const int64_t* offsets;   // n+1 absolute offsets
  int64_t n;
};

// Tile-kernel work decomposition. The long records' offset ranges are cut into wave tiles of
// kTileOffsets * U offsets (U sub-tiles of 63 owned offsets + 1 helper lane, processed together so the
// sub-tiles share each step's Seq2 letter and overlap their dependency chains). The tiles of all long
// records form one record-major list; every wave runs a contiguous, cost-balanced slice of it, from
// starts[w] to starts[w+1] (exclusive), given as (long-record index, tile index within the record).
struct WaveStart {
  int32_t li;
  int32_t t;
};

// Offsets per wave tile: U sub-tiles of 63 (tile kernel) or 128 (tile16: two offsets per lane).
inline int tile_span(bool tile16, int u) { return (tile16 ? 128 : kTileOffsets) * u; }
constexpr int kTile16WavesPerBlock = 16;  // tile16 workgroups: 16 waves
inline int64_t tiles_of(int64_t need, int span) { return (need + span - 1) / span; }

// Host-built plan for the tile kernel of one batch.
struct Plan {
  int64_t n_waves = 0;                 // tile-kernel waves
  const WaveStart* starts = nullptr;   // device, n_waves + 1 entries
  const int32_t* long_recs = nullptr;  // device: records handled by the tile kernel (null = identity)
  int64_t n_long = 0;
  unsigned long long* keys = nullptr;  // device scratch, n_long entries (tile-kernel partial maxima)
  int32_t u = 2;                       // sub-tiles per wave tile (1, 2 or 4)
  int32_t win_tiles = 0;               // windowed tile16: tiles per window stride (the waves of one
                                       // workgroup all walk tiles t in [m*win_tiles, (m+1)*win_tiles))
  R2Params r2;                         // finalize: parameters of the R2 result format
  int64_t slide_items = 0;             // tile16 sliding windows: starts = per-workgroup item offsets, then
  int64_t slide_members = 0;           // items (2 entries each) from slide_items, group members from slide_members
};

// Arguments of the short-record kernel. All pointers must be device-accessible: device memory, or
// pinned host memory (hipHostMalloc / hipHostRegister) for zero-copy streaming.
struct ShortArgs {
  const uint8_t* codes = nullptr;     // base pointer: record i starts at codes + offsets[i]
  const int64_t* offsets = nullptr;   // n+1 absolute offsets, or sparse (off_shift > 0, moc/wire.hpp):
                                      // entry j = offset of record min(j << off_shift, n)
  int32_t off_shift = 0;              // sparse offsets need lengths and tile_records % (1 << off_shift) == 0
  const uint8_t* lengths8 = nullptr;  // optional narrow lengths (saves 7 B/record of reads)
  const uint8_t* lengths4 = nullptr;  // optional nibble lengths: record i = len_base + nibble i (low first)
  const uint8_t* lengths3 = nullptr;  // optional 3-bit lengths: record i = len_base + bits [3i, 3i+3), LSB
                                      // first (one readable slack byte after the last record's)
  const uint8_t* lengths6 = nullptr;  // optional base-6 lengths (moc::kLenBase6): 8-byte words of three 21-bit
                                      // octets, record i = len_base + digit i % 8 of octet i / 8
  int32_t len_base = 0;
  int64_t n = 0;
  void* out = nullptr;                // results, format `fmt`, record i at index i
  int32_t fmt = 0;                    // ResultFormat
  int32_t slot = 0;                   // lanes per record (max lanes_needed over the batch, <= 64)
  int32_t rpw = 0;                    // records per wave = 64 / slot
  int32_t tile_records = 0;           // records per block tile
  int64_t tail_from = INT64_MAX;      // swipe: tiles [tail_from, ...) hold tail_records records each (set
  int32_t tail_records = 0;           // by launch_swipe: the batch's last work is cut finer for the tail)
  int32_t codes_cap = 0;              // LDS bytes for one tile's letters (>= tile_records*max_l2+32)
  int32_t max_l2 = 0;
  int32_t packed5 = 0;                // 1: `codes` is a 5-bit packed stream (char j at bit 5j): staged pipeline only
  int32_t swipe_rk = 0;               // swipe: 1 = keys without k bits, k re-found on the winning diagonal
  int32_t packed33 = 0;               // 1: `codes` holds P33 fields (moc::pack33: char j in field j / 7 at
                                      // bit 33 * (j / 7)); decoded into LDS per tile; swipe only
  int32_t lane_direct = 0;            // swipe: 1 = device-resident byte letters with dense offsets, read by
                                      // each lane straight into registers (swipe_direct_kernel; no counter)
  unsigned* counter = nullptr;        // device work counter {next tile, blocks done}; zero at launch, the
                                      // kernel's last block resets it (no memset between launches)
  int64_t dbg_codes_end = -1;         // debug builds: end of the readable letter bytes (from `codes`)
};

// Copies `bytes` from src to dst on a kernel (copy_kernels.hip); either side may be page-locked host memory
// given by its device address. For small transfers only (kernel_copy_fits): the runtime's SDMA path costs
// 11-34 ms at its first use in a process, this one ~0.3 ms.
constexpr size_t kKernelCopyMaxAligned = size_t{8} << 20;
constexpr size_t kKernelCopyMaxBytes = size_t{1} << 20;
void launch_copy(void* dst, const void* src, size_t bytes, hipStream_t stream);
// A single wave idling `seconds` (clamped to 10 s) on `stream`: the comm-timeout test hook's device stall.
void launch_spin(double seconds, hipStream_t stream);
bool kernel_copy_fits(const void* dst, const void* src, size_t bytes);

// Unpacks n chars of a 5-bit packed stream (device memory) starting at bit `bit0` into byte codes.
void launch_unpack5(const uint8_t* packed, int64_t bit0, int64_t n, uint8_t* out, hipStream_t stream);

// Lanes a record needs in the short kernel (offsets 0..L1-L2 incl. the helper diagonal).
inline int64_t lanes_needed(int64_t L1, int64_t L2) { return L2 <= L1 ? L1 - L2 + 1 : 1; }

// Configures tile size / LDS budget for the short kernel; returns false when the batch cannot run in
// it (a record needs more than 64 lanes). Fills slot/rpw/tile_records/codes_cap.
bool configure_short(int64_t L1, int64_t min_l2, int64_t max_l2, ShortArgs& a);

// Inter-record SIMD kernel (one lane per record, packed int16; swipe_kernels.hip) for tiny problems:
// returns false unless every record fits (|Seq1| <= 200, |Seq2| <= 32, int16-exact weights).
// `hbm`: the records are in device memory (512-record tiles: more blocks per CU, 3.06 vs 2.69 T cells/s on
// input6); host-resident batches stream in 1024-record tiles (fewer PCIe read requests per record).
// `spec`: the batch runs under the spec semantics (one more offset per record, bug B8); the offsets per lane
// follow it (swipe_offsets), the records it accepts do not.
bool configure_swipe(int64_t L1, int64_t min_l2, int64_t max_l2, int32_t max_abs_weight, ShortArgs& a,
                     bool hbm = false, bool spec = true);
// Offsets a record's candidates occupy in the swipe kernel: o < L1 - L2 (the reference's exclusive bound,
// cudaFunctions.cu:116), o <= L1 - L2 under the spec semantics, the single o = 0 when L2 == L1.
inline int64_t swipe_offsets(int64_t L1, int64_t L2, bool spec) { return L2 < L1 ? L1 - L2 + (spec ? 1 : 0) : 1; }
void launch_swipe(const ProblemView& pv, const ShortArgs& a, int num_cus, hipStream_t stream);
// Key form (moc::bounds::kFormSwipe*) the swipe kernel takes for such a batch, 0 when it cannot take it
// by its integer bounds (configure_swipe may still refuse it for the LDS budget).
int32_t swipe_form(int64_t L1, int64_t min_l2, int64_t max_l2, int32_t max_abs_weight);
inline int32_t swipe_launch_form(const ShortArgs& a) {
  return a.swipe_rk ? bounds::kFormSwipeRK : bounds::kFormSwipeKBits;
}

// Short-record kernel (all records with lanes_needed <= a.slot are processed; others are skipped).
void launch_short(const ProblemView& pv, const ShortArgs& a, int num_cus, hipStream_t stream);
// Arithmetic form (moc::bounds::kFormShort*) launch_short runs for these arguments.
int32_t short_form(const ProblemView& pv, const ShortArgs& a);

// Tile kernel + finalize for the long records listed in `plan`; results -> out (format fmt).
// plan.long_recs == nullptr means the identity list (record li of the batch).
void launch_tiles(const ProblemView& pv, const BatchView& bv, const Plan& plan, void* out, int fmt,
                  hipStream_t stream);
// The two halves separately (context-parallel mode: keys are max-reduced across ranks in between).
// launch_tile_keys zeroes plan.keys[0..n_long) and max-accumulates the plan's tiles into them as PASS-1
// keys (score, ~(2o + mutated)); launch_finalize_keys resolves each record's k on its winning diagonal
// (one wave per record, O(L2)) and writes the results — no o*L2 + k index, so L1 * L2 >= 2^32 is fine.
void launch_tile_keys(const ProblemView& pv, const BatchView& bv, const Plan& plan, hipStream_t stream);
// Arithmetic form (moc::bounds::kFormTile16 / kFormMfma / kFormTilesKey32 / kFormTilesKey64) of the sweep
// launch_tile_keys runs for this problem view.
inline int32_t tile_form(const ProblemView& pv) {
  if (pv.prof16)
    return pv.mfma_sweep ? bounds::kFormMfma
                         : bounds::kFormTile16 | (pv.t16_key_bits ? bounds::kFormTile16Key32 : 0) |
                               (pv.prof16_i16 ? bounds::kFormTile16I16 : 0) |
                               (pv.t16_slide ? bounds::kFormTile16Slide : 0);
  return pv.key_shift > 0 ? bounds::kFormTilesKey32 : bounds::kFormTilesKey64;
}
void launch_finalize_keys(const ProblemView& pv, const BatchView& bv, const Plan& plan, void* out, int fmt,
                          hipStream_t stream);
// tile16 variant of launch_tile_keys (pv.prof16 must be set): packed-int16 sweep over the LDS profile.
// mfma_sweep: the matrix-core sweep (tile_mfma_kernels.hip, plan.u <= 2) in place of the packed-int16 one.
void launch_tile16_keys(const ProblemView& pv, const BatchView& bv, const Plan& plan, hipStream_t stream,
                        bool mfma_sweep = false);
void launch_tile_mfma_sweep(const ProblemView& pv, const BatchView& bv, const Plan& plan, hipStream_t stream);
// i8 MFMA operand/accumulator layout self-test: C = A * B (row-major 32x32 int8 -> int32), one wave.
void launch_mfma_i8_probe(const int8_t* d_a, const int8_t* d_b, int* d_c, hipStream_t stream);
// Waves per CU the tile16 kernel keeps resident (16-wave workgroups, as many as the LDS allows).
int tile16_waves_per_cu(int lds_bytes);

// Loads every kernel file's code object onto the current device now (HIP loads them lazily, at the first
// launch from each file: milliseconds inside the first timed search of a job otherwise).
void preload_align_kernels();
void preload_short_kernels();
void preload_swipe_byte_kernels();
void preload_swipe_p33_kernels();
void preload_tile16_kernels();
void preload_mfma_kernels();
// Kernel files by code object, for a preload of only what a job will launch.
enum PreloadSet : unsigned {
  kPreloadAlign = 1,
  kPreloadShort = 2,
  kPreloadSwipeByte = 4,
  kPreloadSwipeP33 = 8,
  kPreloadTile16 = 16,
  kPreloadMfma = 32,  // the measured-slower MFMA variant: only when it is selected (MOC_MFMA=1)
  kPreloadAll = 31,   // all but MFMA
};
inline void preload_kernels(unsigned set) {
  if (set & kPreloadMfma) preload_mfma_kernels();
  if (set & kPreloadAlign) preload_align_kernels();
  if (set & kPreloadShort) preload_short_kernels();
  if (set & kPreloadSwipeByte) preload_swipe_byte_kernels();
  if (set & kPreloadSwipeP33) preload_swipe_p33_kernels();
  if (set & kPreloadTile16) preload_tile16_kernels();
}
// "all", "none", or a comma list of align, short, swipe (both letter forms), swipe8, swipe33, tile16, mfma;
// returns -1 for a name it does not know
int parse_preload_set(const char* s);

// One-wave self-test of the DPP / shuffle primitives (192 ints, see align_kernels.hip).
void launch_dpp_probe(int* d_out, hipStream_t stream);

// Transfer calibration in GB/s (kinds: transfer_probe.hip). Allocates/frees its own buffers.
double transfer_probe(int kind, size_t bytes, int iters);

}  // namespace dev
}  // namespace moc
