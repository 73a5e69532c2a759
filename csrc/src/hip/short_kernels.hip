// Short-record search kernel (records with L1 - L2 + 1 <= 64 offsets; the input6-shaped regime).
//
// Persistent blocks of 4 waves pull tiles of `tile_records` consecutive records from a device work
// counter. Per tile the block:
//   1. reads the tile's lengths (narrow uint8 lengths when available, else offsets) and block-scans
//      them into LDS-local offsets;
//   2. copies the tile's letters into LDS with 16-byte loads — from device memory, or straight from
//      pinned host memory (zero-copy streaming: the batch crosses PCIe exactly once and no staging
//      buffers/copies are needed);
//   3. scores every record: each wave holds 64/slot records in fixed lane slots, lane = offset o,
//      P += S[c][o+i] from the per-block LDS profile S[c][j] = T[c][Seq1[j]] (row 0 = padding = 0, so
//      lanes past their record's end add 0 and need no masking), P_{o+1} via DPP wave_shl:1,
//      best = max over k of pack(P_o(k) - P_{o+1}(k), k);
//   4. reduces each slot with a segmented suffix max of 64-bit keys and writes the tile's results
//      (R4/R8/R12) back with coalesced dword stores.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "kernel_common.hpp"
#include "moc/kernel_bounds.hpp"

namespace moc {
namespace dev {

using namespace kc;

namespace {
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
constexpr int kBlock = 256;
#ifndef MOC_SHORT_GROUP
#define MOC_SHORT_GROUP 8
#endif
constexpr int kShortGroup = MOC_SHORT_GROUP;  // steps whose LDS reads are issued together
constexpr int kMaxTile = 1024;            // records per block tile (4 per thread in the scan)
constexpr int kShortLdsBudget = 60 * 1024;  // stay under the 64 KiB default dynamic-LDS limit
constexpr int kShortLdsOccupancy = 160 * 1024 / 6;  // preferred: 6 blocks per CU

struct ShortLayout {
  int row = 0;          // profile row length (entries), Profile mode
  int table_bytes = 0;  // profile or LUT
  int s1_bytes = 0;     // LUT mode: Seq1 copy
  int loff_off = 0, codes_off = 0, res_off = 0, total = 0;
  bool profile = false;
};

inline int align16(int x) { return (x + 15) & ~15; }
// per-block profile S[c][j] (one int per entry) when it is small, else the LUT + Seq1 in LDS
bool short_profile(int L1) { return kAlphabet * ((L1 + kWave + 3) & ~3) * 4 <= 24 * 1024; }

ShortLayout short_layout(int L1, int tile_records, int codes_cap, int fmt_bytes, bool profile) {
  ShortLayout l;
  l.profile = profile;
  if (profile) {
    l.row = (L1 + kWave + 3) & ~3;
    l.table_bytes = align16(kAlphabet * l.row * 4);
  } else {
    l.table_bytes = kLutInts * 4;
    l.s1_bytes = align16(L1 + kWave + 4);
  }
  l.loff_off = l.table_bytes + l.s1_bytes;
  l.codes_off = l.loff_off + align16((tile_records + 1) * 4 + 64);  // + misc: 16 ints
  l.res_off = l.codes_off + align16(codes_cap);
  l.total = l.res_off + align16(tile_records * fmt_bytes);
  return l;
}
}  // namespace

// Pk (profile mode, int16-exact batches): the profile holds packed pairs (Dt << 16 | S), Dt[c][j] =
// S[c][j] - S[c][j+1], so one v_pk_add_u16 advances both Tot_o (low half) and D_o(k) = P_o(k) - P_{o+1}(k)
// (high half) and the hot key is one v_and_or_b32 of the accumulator with the step's (0xffff - k): no
// DPP neighbour move and no subtraction per cell (3 VALU instead of 5); Tot_{o+1} = Tot_o - D_o(L2).
template <bool Wide, bool Profile, bool Pk>
__global__ __launch_bounds__(kBlock) void short_search_kernel(ProblemView pv, ShortArgs a, ShortLayout lay) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int* table = reinterpret_cast<int*>(smem);
  uint8_t* s1l = smem + lay.table_bytes;
  int* loff = reinterpret_cast<int*>(smem + lay.loff_off);
  int* misc = loff + a.tile_records + 1;  // 8 ints of slack: [0] tile id, [4..7] per-wave scan totals
  uint8_t* codes_l = smem + lay.codes_off;
  uint8_t* res_l = smem + lay.res_off;
  const int L1 = pv.L1;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  // ---- per-block problem tables (built once, reused for every tile this block pulls)
  if (Profile) {
    const int row = lay.row;
    for (int e = tid; e < kAlphabet * row; e += kBlock) {
      const int c = e / row, j = e - c * row;
      const int sj = (c >= 1 && j < L1) ? pv.lut[c * kLutStride + pv.seq1[j]] : 0;
      if (Pk) {
        const int sn = (c >= 1 && j + 1 < L1) ? pv.lut[c * kLutStride + pv.seq1[j + 1]] : 0;
        table[e] = static_cast<int>((static_cast<uint32_t>(sj - sn) << 16) | (static_cast<uint32_t>(sj) & 0xffffu));
      } else {
        table[e] = sj;
      }
    }
  } else {
    for (int e = tid; e < kLutInts; e += kBlock) {
      const int c = e >> 5;
      table[e] = c >= 1 ? pv.lut[e] : 0;  // row 0 = padding -> contributes 0
    }
    stage_bytes(s1l, pv.seq1, L1 + kWave);
  }

  using K = HotKey<Wide>;
  const int slot = a.slot, rpw = a.rpw;
  const int sl = lane / slot;
  const int o = lane - sl * slot;
  const int shift = pv.key_shift, mask = (1 << pv.key_shift) - 1;
  const int fb = fmt_bytes(a.fmt);
  const int64_t n_tiles = (a.n + a.tile_records - 1) / a.tile_records;

  for (;;) {
    __syncthreads();  // previous tile fully consumed (and tables built on the first pass)
    if (tid == 0) {  // tile id, and its letter range (one host-memory read per block, not per wave)
      const int64_t tt = atomicAdd(a.counter, 1u);
      misc[0] = static_cast<int>(tt);
      if (tt < n_tiles) {
        const int64_t r0 = tt * a.tile_records;
        const int64_t st = tile_offset(a, r0), en = tile_offset(a, min(r0 + a.tile_records, a.n));
        misc[8] = static_cast<int>(static_cast<uint32_t>(st));
        misc[9] = static_cast<int>(static_cast<uint64_t>(st) >> 32);
        misc[10] = static_cast<int>(static_cast<uint32_t>(en));
        misc[11] = static_cast<int>(static_cast<uint64_t>(en) >> 32);
      }
    }
    __syncthreads();
    const int64_t t = misc[0];
    if (t >= n_tiles) break;  // block-uniform exit; every wave reaches it
    const int64_t rb = t * a.tile_records;
    const int m = static_cast<int>(min(static_cast<int64_t>(a.tile_records), a.n - rb));
    const int64_t start = static_cast<int64_t>((static_cast<uint64_t>(static_cast<uint32_t>(misc[9])) << 32) |
                                               static_cast<uint32_t>(misc[8]));
    const int64_t end = static_cast<int64_t>((static_cast<uint64_t>(static_cast<uint32_t>(misc[11])) << 32) |
                                             static_cast<uint32_t>(misc[10]));

    // ---- 1. lengths -> block exclusive scan -> loff[0..m]
    int len4[4];
    record_lengths4(a, rb + tid * 4, min(4, max(0, m - tid * 4)), len4);
    const int sum = len4[0] + len4[1] + len4[2] + len4[3];
    const int incl = wave_inclusive_sum(sum, lane);
    if (lane == 63) misc[4 + wave] = incl;
    __syncthreads();
    int excl = incl - sum;
    for (int w = 0; w < wave; ++w) excl += misc[4 + w];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = tid * 4 + q;
      if (r < m) loff[r] = excl;
      excl += len4[q];
    }
    if (tid == kBlock - 1) loff[m] = excl;  // the last thread's running sum is the tile total

    // ---- 2. letters -> LDS (16-byte loads; never crosses a page the tile does not touch)
    const uintptr_t p0 = reinterpret_cast<uintptr_t>(a.codes + start);
    const uintptr_t a0 = p0 & ~uintptr_t{15};
    const int shift_b = static_cast<int>(p0 - a0);
    const int nvec = static_cast<int>((reinterpret_cast<uintptr_t>(a.codes + end) + 15 - a0) >> 4);
    for (int v = tid; v < nvec; v += kBlock)
      reinterpret_cast<uint4*>(codes_l)[v] = reinterpret_cast<const uint4*>(a0)[v];
    __syncthreads();

    // ---- 3. score: each wave takes groups of rpw records
    for (int g = wave; g * rpw < m; g += 4) {
      const int rl = g * rpw + sl;
      const bool in = sl < rpw && rl < m;
      int L2 = 0, roff = 0;
      if (in) {
        roff = loff[rl];
        L2 = loff[rl + 1] - roff;
      }
      const int need = L2 <= L1 ? L1 - L2 + 1 : 1;
      const bool mine = in && need <= slot;
      const bool on = mine && L2 <= L1 && o < need;
      const int steps = wave_max_i32(on ? L2 : 0);
      const uint8_t* rec = codes_l + shift_b + roff;
      int P = 0;
      typename K::T best = K::min();
      uint32_t acc = 0;         // Pk: (D_o, Tot_o) halves
      int32_t best16 = INT32_MIN;  // Pk: max of (D << 16 | 0xffff - k)
      // 8 steps per round: the letter and table reads of the round are issued together (independent
      // LDS reads in flight), then the dependent prefix / neighbour / key chain consumes them
      auto gather = [&](int i) {
        const int c = (on && i < L2) ? rec[i] : 0;
        return Profile ? table[c * lay.row + o + i] : table[(c << 5) | s1l[o + i]];
      };
      auto step = [&](int v, int i) {
        if (Pk) {
          acc = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, acc) + __builtin_bit_cast(u16x2, static_cast<uint32_t>(v)));
          const int32_t key = static_cast<int32_t>((acc & 0xffff0000u) | (0xffffu - static_cast<uint32_t>(i + 1)));
          best16 = key > best16 ? key : best16;
        } else {
          P += v;
          const int Pn = wave_shl1(P);
          const typename K::T key = K::make(P - Pn, i + 1, shift, mask);
          best = key > best ? key : best;
        }
      };
      int i = 0;
      for (; i + kShortGroup <= steps; i += kShortGroup) {
        int v[kShortGroup];
#pragma unroll
        for (int j = 0; j < kShortGroup; ++j) v[j] = gather(i + j);
#pragma unroll
        for (int j = 0; j < kShortGroup; ++j) step(v[j], i + j);
      }
      for (; i < steps; ++i) step(gather(i), i);
      unsigned long long key = 0;
      if (Pk) {
        const int tot = static_cast<int16_t>(acc & 0xffffu), dfin = static_cast<int>(acc) >> 16;
        const int last = L1 - L2;
        if (on) {
          const bool v0 = (o < last) || (o == last && (pv.semantics == static_cast<int>(Semantics::Spec) || L2 == L1));
          if (v0) key = final_key(tot, static_cast<uint32_t>(o) * static_cast<uint32_t>(L2));
          if (o < last && L2 >= 2 && best16 != INT32_MIN) {
            const int k = 0xffff - (best16 & 0xffff);
            key = max_u64(key, final_key((best16 >> 16) + tot - dfin,
                                         static_cast<uint32_t>(o) * static_cast<uint32_t>(L2) + static_cast<uint32_t>(k)));
          }
        }
      } else {
        const int Pn = wave_shl1(P);
        key = lane_candidate<Wide>(on, o, L1, L2, pv.semantics, P, Pn, best, shift, mask);
      }
      for (int d = 1; d < slot; d <<= 1) {  // segmented suffix max within the slot
        const unsigned long long other = shfl_down_u64(key, d);
        if (o + d < slot) key = max_u64(key, other);
      }
      if (mine && o == 0) store_result(res_l, rl, a.fmt, decode_key(key, L2 > 0 ? L2 : 1), pv.r2);
    }
    __syncthreads();

    // ---- 4. results -> out (coalesced dwords; long records are overwritten later by the tile kernel)
    copy_results(static_cast<char*>(a.out) + rb * fb, res_l, m * fb, tid, kBlock);
  }
  release_work_counter(a.counter);
}

// 5-bit packed stream -> byte codes (staged pipeline path for packed batches).
__global__ void unpack5_kernel(const uint8_t* __restrict__ packed, int64_t bit0, int64_t n, uint8_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t bit = bit0 + 5 * i;
    const uint32_t lo = packed[bit >> 3], hi = packed[(bit >> 3) + 1];
    out[i] = static_cast<uint8_t>(((lo | (hi << 8)) >> (bit & 7)) & 31u);
  }
}

void preload_short_kernels() {
  hipFuncAttributes fa;
  (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&unpack5_kernel));
}

void launch_unpack5(const uint8_t* packed, int64_t bit0, int64_t n, uint8_t* out, hipStream_t stream) {
  if (n <= 0) return;
  const int64_t blocks = std::min<int64_t>((n + kBlock - 1) / kBlock, 4096);
  hipLaunchKernelGGL(unpack5_kernel, dim3(static_cast<unsigned>(blocks)), dim3(kBlock), 0, stream, packed, bit0, n,
                     out);
}

bool configure_short(int64_t L1, int64_t min_l2, int64_t max_l2, ShortArgs& a) {
  if (lanes_needed(L1, min_l2) > kWave) return false;
  a.slot = static_cast<int32_t>(std::max<int64_t>(1, lanes_needed(L1, min_l2)));
  a.rpw = kWave / a.slot;
  const int64_t l2cap = std::max<int64_t>(1, std::min(max_l2, L1 + 1));
  const int fb = result_bytes(static_cast<ResultFormat>(a.fmt));
  const bool profile = short_profile(static_cast<int>(L1));
  int max_tile = kMaxTile;  // MOC_SHORT_TILE: cap on records per block tile (A/B runs)
  if (const char* v = std::getenv("MOC_SHORT_TILE")) max_tile = std::max(1, std::min(kMaxTile, std::atoi(v)));
  // Occupancy first: the largest tile whose LDS lets 6 blocks (24 waves) share a CU — the hot loop's
  // two dependent LDS reads per step need that many waves in flight (input1 shape: 1.47 T cells/s at
  // 1024-record tiles / 2 blocks per CU, 2.02 T at 256 / 6 per CU) — else the largest that fits at all.
  for (const int budget : {kShortLdsOccupancy, kShortLdsBudget}) {
    const int min_tile = budget == kShortLdsOccupancy ? std::min(64, max_tile) : 1;  // keep tiles useful
    for (int tr = max_tile; tr >= min_tile; tr /= 2) {
      // worst-case letters of a tile: records longer than L1 are never scored but still staged
      const int64_t cap = static_cast<int64_t>(tr) * std::max(max_l2, int64_t{1}) + 48;
      if (cap > budget) continue;
      ShortLayout l = short_layout(static_cast<int>(L1), tr, static_cast<int>(cap), fb, profile);
      if (l.total <= budget) {
        a.tile_records = tr;
        a.codes_cap = static_cast<int32_t>(cap);
        a.max_l2 = static_cast<int32_t>(l2cap);
        return true;
      }
    }
  }
  return false;
}

int32_t short_form(const ProblemView& pv, const ShortArgs& a) {
  // packed (Dt, S) profile when every partial sum is int16-exact (moc/kernel_bounds.hpp short_pk_exact;
  // MOC_SHORT_PK=0 forces the int32 DPP form, for A/B runs)
  static const bool pk_off = [] {
    const char* v = std::getenv("MOC_SHORT_PK");
    return v && std::atoi(v) == 0;
  }();
  if (short_profile(pv.L1) && !pk_off && bounds::short_pk_exact(pv.max_abs_t, a.max_l2)) return bounds::kFormShortPk;
  return pv.key_shift > 0 ? bounds::kFormShortKey32 : bounds::kFormShortKey64;
}

void launch_short(const ProblemView& pv, const ShortArgs& a, int num_cus, hipStream_t stream) {
  if (a.n <= 0) return;
  const int fb = result_bytes(static_cast<ResultFormat>(a.fmt));
  const bool profile = short_profile(pv.L1);
  const ShortLayout lay = short_layout(pv.L1, a.tile_records, a.codes_cap, fb, profile);
  const int64_t n_tiles = (a.n + a.tile_records - 1) / a.tile_records;
  const int per_cu = std::max(1, std::min(8, 160 * 1024 / std::max(lay.total, 1)));
  const int64_t blocks = std::min<int64_t>(n_tiles, static_cast<int64_t>(num_cus) * per_cu);
  const dim3 grid(static_cast<unsigned>(std::max<int64_t>(blocks, 1))), block(kBlock);
  const int32_t form = short_form(pv, a);
  if (form == bounds::kFormShortPk) {
    hipLaunchKernelGGL((short_search_kernel<false, true, true>), grid, block, lay.total, stream, pv, a, lay);
  } else if (form == bounds::kFormShortKey32) {
    if (profile)
      hipLaunchKernelGGL((short_search_kernel<false, true, false>), grid, block, lay.total, stream, pv, a, lay);
    else
      hipLaunchKernelGGL((short_search_kernel<false, false, false>), grid, block, lay.total, stream, pv, a, lay);
  } else {
    if (profile)
      hipLaunchKernelGGL((short_search_kernel<true, true, false>), grid, block, lay.total, stream, pv, a, lay);
    else
      hipLaunchKernelGGL((short_search_kernel<true, false, false>), grid, block, lay.total, stream, pv, a, lay);
  }
}

}  // namespace dev
}  // namespace moc
