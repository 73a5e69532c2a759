// Long-record search kernel, packed-int16 difference-profile variant ("tile16"; gfx950, wave64).
//
// Work decomposition as tile_search_kernel (align_kernels.hip): persistent waves walk cost-balanced runs
// of wave tiles planned on the host, one record's letters in registers across its tiles, one 64-bit
// atomicMax per record run. The per-cell work is what changes. With the closed form
//     score(o, 0) = Tot_o,   score(o, k >= 1) = D_o(k) + Tot_{o+1},   D_o(k) = P_o(k) - P_{o+1}(k)
//     D_o(k) = sum_{i<k} Dt[c_i][o + i],   Dt[c][j] = T[c][Seq1[j]] - T[c][Seq1[j+1]]
// the hot loop only needs the running sums of Dt along each diagonal and their running maximum. A LANE
// carries a pair of adjacent offsets o, o + 1 as the two int16 halves of one register; LDS holds the
// difference profile (moc/score_table.hpp Profile16), entry [c][j] = (Dt[c][j], Dt[c][j+1]) — the step-i
// terms of both diagonals — in one of three forms:
//   * byte pairs (|Dt| <= 127, 2 bytes per entry): per step and lane one ds_read_u16, then
//       acc.lo += sext(byte0); acc.hi += sext(byte1)   2 x v_add_u16_sdwa
//       best = max(best, acc)                          v_pk_max_i16
//   * widened pairs (Wide: the byte pairs sign-extended to int16 halves while staging, 4 bytes per entry,
//     split by flat-index parity so the lanes' reads are conflict-free): one ds_read_b32, v_pk_add_u16,
//     v_pk_max_i16 — where twice the image fits (whole, or as windows for short records);
//   * an int16 profile (pv.prof16_i16: |Dt| <= 511, weights past the byte pairs): staged straight into the
//     widened form.
//   The U sub-tiles (128 offsets each) of a wave tile sit at immediate LDS offsets, a step's row offset
//   arrives by one DPP row broadcast, and G * U reads issue before a group's adds;
//   * every 64 steps the int16 halves are folded into int32 (|partial sums| <= 64 * 511 < 2^15: exact);
//   * Tot_o is not summed per cell: per tile one anchor diagonal Tot_{oA} (oA = first offset past the
//     tile or past the valid range) is summed alongside the sweep (each chunk's lanes add their step's
//     pair score from the LUT + Seq1 staged next to the profile), and
//     Tot_o = Tot_{oA} + sum_{o <= o' < oA} D_{o'}(L2) comes from a wave scan on the DPP network;
//   * short records take U = 8 sub-tiles (1024-offset tiles: fewer per-tile epilogues).
// Per offset this gives the best score, but not which k: the sweep reduces pass-1 keys (score,
// ~(2o + mutated)) — the reference order: score, then smallest o, then k = 0 first — 32-bit ones where
// bounds::tile16_key32_bits says score and index fit — and resolve_long_kernel (align_kernels.hip)
// re-walks only the winning diagonal of each record (one wave, O(L2)) to find the smallest k with that
// score. Host replay of all of it, ties included: csrc/tests/test_core.cpp test_profile16,
// test_tile16_key32_replay, test_tile16_i16_replay.
//
// Replaces calc_result (cudaFunctions.cu:63-176) for long records when the weights fit the profile
// (byte pairs or int16) and the image fits one CU's LDS (whole, or as windows of Seq1 for longer ones).
#include <hip/hip_runtime.h>

#include <mutex>
#include <set>
#include <type_traits>

#include "kernel_common.hpp"
#include "moc/runtime/hip_check.hpp"

namespace moc {
namespace dev {

using namespace kc;

namespace {
typedef short s16x2 __attribute__((ext_vector_type(2)));

constexpr int kBlock16 = 1024;  // 16 waves: the profile takes most of the CU's LDS, one workgroup holds it
constexpr int kWavesPerBlock16 = kBlock16 / 64;
constexpr int kSub = 128;                    // offsets per sub-tile (2 per lane)
constexpr uint32_t kBestInit = 0x80008000u;  // both halves INT16_MIN

// acc.lo += sext(e.byte0), acc.hi += sext(e.byte1): 16-bit wrapping adds on sub-dword operands (SDWA)
__device__ __forceinline__ void add_pair(uint32_t& acc, uint32_t e) {
  asm("v_add_u16_sdwa %0, %0, sext(%1) dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:BYTE_0"
      : "+v"(acc)
      : "v"(e));
  asm("v_add_u16_sdwa %0, %0, sext(%1) dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:BYTE_1"
      : "+v"(acc)
      : "v"(e));
}
__device__ __forceinline__ uint32_t pk_add(uint32_t a, uint32_t b) {  // v_pk_add_u16: both int16 halves
  return __builtin_bit_cast(uint32_t, __builtin_bit_cast(s16x2, a) + __builtin_bit_cast(s16x2, b));
}
__device__ __forceinline__ uint32_t pk_max(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t,
                            __builtin_elementwise_max(__builtin_bit_cast(s16x2, a), __builtin_bit_cast(s16x2, b)));
}
__device__ __forceinline__ int lo16(uint32_t v) { return static_cast<int16_t>(v & 0xffffu); }
__device__ __forceinline__ int hi16(uint32_t v) { return static_cast<int>(v) >> 16; }

// Pass-1 key of offset o: (score, ~(2o + mutated)); the same packing as final_key.
__device__ __forceinline__ unsigned long long pass1_candidate(int o, int L1, int L2, int sem, int tot, int tot_next,
                                                              int maxD) {
  unsigned long long key = 0;
  const int last = L1 - L2;
  if (L2 > L1 || o > last) return key;
  const bool v0 = (o < last) || (sem == static_cast<int>(Semantics::Spec) || L2 == L1);
  if (v0) key = final_key(tot, 2u * static_cast<uint32_t>(o));
  if (o < last && L2 >= 2) key = max_u64(key, final_key(maxD + tot_next, 2u * static_cast<uint32_t>(o) + 1u));
  return key;
}

// Lane k of each DPP row (16 lanes) broadcast across its row; k a constant once the caller is unrolled
template <int K>
__device__ __forceinline__ int newbcast(int v) {
  return __builtin_amdgcn_update_dpp(0, v, 0x150 + K, 0xf, 0xf, false);
}
__device__ __forceinline__ int row_newbcast(int v, int k) {
  switch (k) {
    case 0: return newbcast<0>(v);
    case 1: return newbcast<1>(v);
    case 2: return newbcast<2>(v);
    case 3: return newbcast<3>(v);
    case 4: return newbcast<4>(v);
    case 5: return newbcast<5>(v);
    case 6: return newbcast<6>(v);
    case 7: return newbcast<7>(v);
    case 8: return newbcast<8>(v);
    case 9: return newbcast<9>(v);
    case 10: return newbcast<10>(v);
    case 11: return newbcast<11>(v);
    case 12: return newbcast<12>(v);
    case 13: return newbcast<13>(v);
    case 14: return newbcast<14>(v);
    default: return newbcast<15>(v);
  }
}

// Inclusive prefix sum over the lanes of a wave on the DPP network: row shifts 1/2/4/8 (zero-filled),
// then lane 15 of each row into the next row and lane 31 into rows 2-3. VALU only — no LDS round trip
// per level as with __shfl (ds_bpermute).
template <int Ctrl, int RowMask>
__device__ __forceinline__ int dpp_or0(int v) {
  return __builtin_amdgcn_update_dpp(0, v, Ctrl, RowMask, 0xf, false);
}
__device__ __forceinline__ int wave_prefix_sum_dpp(int v) {
  v += dpp_or0<0x111, 0xf>(v);  // row_shr:1
  v += dpp_or0<0x112, 0xf>(v);  // row_shr:2
  v += dpp_or0<0x114, 0xf>(v);  // row_shr:4
  v += dpp_or0<0x118, 0xf>(v);  // row_shr:8
  v += dpp_or0<0x142, 0xa>(v);  // row_bcast:15 -> rows 1, 3
  v += dpp_or0<0x143, 0xc>(v);  // row_bcast:31 -> rows 2, 3
  return v;
}
// N independent prefix sums step by step: each DPP add waits two cycles on the previous one of its own
// chain, so the chains interleave instead of stalling on s_nop.
template <int N>
__device__ __forceinline__ void wave_prefix_sums_dpp(int (&v)[N]) {
#pragma unroll
  for (int k = 0; k < N; ++k) v[k] += dpp_or0<0x111, 0xf>(v[k]);
#pragma unroll
  for (int k = 0; k < N; ++k) v[k] += dpp_or0<0x112, 0xf>(v[k]);
#pragma unroll
  for (int k = 0; k < N; ++k) v[k] += dpp_or0<0x114, 0xf>(v[k]);
#pragma unroll
  for (int k = 0; k < N; ++k) v[k] += dpp_or0<0x118, 0xf>(v[k]);
#pragma unroll
  for (int k = 0; k < N; ++k) v[k] += dpp_or0<0x142, 0xa>(v[k]);
#pragma unroll
  for (int k = 0; k < N; ++k) v[k] += dpp_or0<0x143, 0xc>(v[k]);
}
// Maximum over the lanes of a wave (unsigned; 0 is the identity) on the DPP network, in every lane's result
// at lane 63.
__device__ __forceinline__ uint32_t wave_max_u32_dpp(uint32_t v) {
  auto dpp = [](uint32_t x, auto ctrl, auto row_mask) {
    return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), decltype(ctrl)::value,
                                                             decltype(row_mask)::value, 0xf, false));
  };
  using std::integral_constant;
  v = max(v, dpp(v, integral_constant<int, 0x111>(), integral_constant<int, 0xf>()));  // row_shr:1
  v = max(v, dpp(v, integral_constant<int, 0x112>(), integral_constant<int, 0xf>()));  // row_shr:2
  v = max(v, dpp(v, integral_constant<int, 0x114>(), integral_constant<int, 0xf>()));  // row_shr:4
  v = max(v, dpp(v, integral_constant<int, 0x118>(), integral_constant<int, 0xf>()));  // row_shr:8
  v = max(v, dpp(v, integral_constant<int, 0x142>(), integral_constant<int, 0xa>()));  // row_bcast:15
  v = max(v, dpp(v, integral_constant<int, 0x143>(), integral_constant<int, 0xc>()));  // row_bcast:31
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 63));
}

// Runs f with the sub-tile count of a tile: the smallest power of two (<= UU) holding its `act` sub-tiles of
// valid offsets — a record's last, partial tile sweeps only those (a tile of U sub-tiles would spend the
// others' adds and maxima on offsets past the record's range). `act` is wave-uniform.
template <int UU, typename F>
__device__ __forceinline__ void with_subtiles(int act, F&& f) {
  if constexpr (UU == 1) {
    f(std::integral_constant<int, 1>());
  } else {
    if (act > UU / 2)
      f(std::integral_constant<int, UU>());
    else
      with_subtiles<UU / 2>(act, f);
  }
}
}  // namespace

// Stages columns [S, S + W) of every profile row as widened entries split by the parity of their window index
// e = c * W + x (halves of pv.prof16_bytes each; then the overhang, zeros), and Seq1 letters S .. S + W + 16
// (the anchor diagonals) at s1l. All threads of the workgroup take part.
__device__ __forceinline__ void stage_window_wide(unsigned char* smem, uint8_t* s1l, const ProblemView& pv, int S,
                                                  int W) {
  // the window's entries e = c * W + x (x < W: global column S + x of row c; then the overhang, zeros),
  // widened and split by the parity of e as in the whole image (halves of pv.prof16_bytes each)
  uint32_t* even = reinterpret_cast<uint32_t*>(smem);
  uint32_t* odd = reinterpret_cast<uint32_t*>(smem + pv.prof16_bytes);
  const int rows_entries = (kAlphabet - 1) * W;
  const int n_entries = pv.prof16_bytes >> 1;
  auto widen1 = [](uint32_t e) {  // byte pair -> two sign-extended int16 halves
    return (static_cast<uint32_t>(static_cast<int8_t>(e & 0xffu)) & 0xffffu) |
           (static_cast<uint32_t>(static_cast<int8_t>((e >> 8) & 0xffu)) << 16);
  };
  if (pv.prof16_i16 && (pv.L1 & 7) == 0) {
    // int16 Dt per entry, rows 16-byte aligned: 8 entries per load — the even pairs are its dwords, the odd
    // ones straddle them and the next load's first value
    const int w8 = W >> 3;
    for (int e = threadIdx.x; e < (kAlphabet - 1) * w8; e += blockDim.x) {
      const int c = e / w8, x = (e - c * w8) << 3;
      const int64_t g = static_cast<int64_t>(c) * pv.L1 + S + x;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      uint32_t nx = 0u;
      if (g + 9 <= pv.prof16_entries) {
        v = *reinterpret_cast<const uint4*>(pv.prof16 + g);
        nx = pv.prof16[g + 8];
      } else {
        uint32_t h[9];
#pragma unroll
        for (int q = 0; q < 9; ++q) h[q] = g + q < pv.prof16_entries ? pv.prof16[g + q] : 0u;
        v = make_uint4(h[0] | h[1] << 16, h[2] | h[3] << 16, h[4] | h[5] << 16, h[6] | h[7] << 16);
        nx = h[8];
      }
      const int d = (c * W + x) >> 1;
      *reinterpret_cast<uint4*>(even + d) = v;
      *reinterpret_cast<uint4*>(odd + d) =
          make_uint4(__builtin_amdgcn_alignbit(v.y, v.x, 16), __builtin_amdgcn_alignbit(v.z, v.y, 16),
                     __builtin_amdgcn_alignbit(v.w, v.z, 16), __builtin_amdgcn_alignbit(nx, v.w, 16));
    }
    for (int e = rows_entries + threadIdx.x; e < n_entries; e += blockDim.x) ((e & 1) ? odd : even)[e >> 1] = 0u;
  } else if (pv.prof16_i16) {  // int16 Dt per entry: the pair of window entry (c, x) is global (g, g + 1)
    for (int e = threadIdx.x; e < n_entries; e += blockDim.x) {
      uint32_t v = 0;
      if (e < rows_entries) {
        const int c = e / W, x = e - c * W;
        const int64_t g = static_cast<int64_t>(c) * pv.L1 + S + x;
        if (g < pv.prof16_entries) v = pv.prof16[g];
        if (g + 1 < pv.prof16_entries) v |= static_cast<uint32_t>(pv.prof16[g + 1]) << 16;
      }
      ((e & 1) ? odd : even)[e >> 1] = v;
    }
  } else if ((pv.L1 & 7) == 0) {  // rows 16-byte aligned (W and S are multiples of 16): 8 entries per load
    const int w8 = W >> 3;
    for (int e = threadIdx.x; e < (kAlphabet - 1) * w8; e += blockDim.x) {
      const int c = e / w8, x = (e - c * w8) << 3;
      const int64_t g = static_cast<int64_t>(c) * pv.L1 + S + x;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (g + 8 <= pv.prof16_entries) v = *reinterpret_cast<const uint4*>(pv.prof16 + g);
      const int d = (c * W + x) >> 1;  // entries c*W + x .. + 7: 4 even, 4 odd, 16-byte aligned
      *reinterpret_cast<uint4*>(even + d) = make_uint4(widen1(v.x & 0xffffu), widen1(v.y & 0xffffu),
                                                       widen1(v.z & 0xffffu), widen1(v.w & 0xffffu));
      *reinterpret_cast<uint4*>(odd + d) = make_uint4(widen1(v.x >> 16), widen1(v.y >> 16), widen1(v.z >> 16),
                                                      widen1(v.w >> 16));
    }
    for (int e = rows_entries + threadIdx.x; e < n_entries; e += blockDim.x) ((e & 1) ? odd : even)[e >> 1] = 0u;
  } else {
    for (int e = threadIdx.x; e < n_entries; e += blockDim.x) {
      uint32_t v = 0;
      if (e < rows_entries) {
        const int c = e / W, x = e - c * W;
        const int64_t g = static_cast<int64_t>(c) * pv.L1 + S + x;
        if (g < pv.prof16_entries) v = widen1(pv.prof16[g]);
      }
      ((e & 1) ? odd : even)[e >> 1] = v;
    }
  }
  for (int t = threadIdx.x; t < W + 16; t += blockDim.x) s1l[t] = S + t < pv.L1 ? pv.seq1[S + t] : 0;
}

// Win (windowed): Seq1 is longer than one LDS image holds. The workgroup's waves all walk tiles of one
// window m (plan: window-major wave runs, 16-wave aligned, tiles t in [m*T, (m+1)*T) of every record), so it
// stages only columns [S, S + W) of each profile row (S = m*T*span, W = pv.prof16_window) and the Seq1
// letters the anchor diagonals read; profile column j lives at LDS column j - S.
// Wide: the LDS entry of a column is the byte pair widened to two int16 halves (4 bytes,
// expanded while staging), so a step adds both offsets of a lane with one v_pk_add_u16 instead of two SDWA
// byte adds — 2 VALU per lane and step instead of 3, at twice the profile's LDS (pv.prof16_wide). The widened
// entries are split by the parity of their flat index e = row * L1 + column: even e at dword e/2 of the first
// half, odd e at dword e/2 of the second. A step's reads then hit consecutive dwords across the lanes (lane l
// reads e = o0 + 2l + s), one conflict-free ds_read_b32 per lane and sub-tile; with the entries in column
// order the lanes' 8-byte stride put two lanes on every bank (SQ_LDS_BANK_CONFLICT = half the LDS cycles,
// profiles/roofline_r5.md).
template <int U, bool Win, bool Wide = false>
__global__ __launch_bounds__(kBlock16) void tile16_search_kernel(ProblemView pv, BatchView bv,
                                                                 const WaveStart* __restrict__ starts, int64_t n_waves,
                                                                 const int32_t* __restrict__ long_recs, int64_t n_long,
                                                                 unsigned long long* __restrict__ keys, int win_tiles) {
  constexpr int EW = Wide ? 4 : 2;  // LDS bytes per profile column
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // LDS image (tile16_lds_bytes): profile (or its window) | int8 LUT | Seq1 codes (the anchor diagonals)
  const int prof_lds = Wide ? 2 * pv.prof16_bytes : pv.prof16_bytes;
  int8_t* lut8 = reinterpret_cast<int8_t*>(smem + prof_lds);
  uint8_t* s1l = smem + prof_lds + kProf16Lut8;
  constexpr int kSpan = kSub * U;
  const int64_t w0 = static_cast<int64_t>(blockIdx.x) * kWavesPerBlock16;  // the workgroup's first wave: real
  const int t_base = Win ? (starts[w0].t / win_tiles) * win_tiles : 0;     // first tile of the window
  const int S = t_base * kSpan;                                             // first column of the window
  const int W = Win ? pv.prof16_window : pv.L1;                             // columns per LDS row
  if (Win && Wide) {
    stage_window_wide(smem, s1l, pv, S, W);
  } else if (Win) {
    // rows' window columns; entries past the global profile read as 0, then the overhang (zeros)
    uint16_t* dst = reinterpret_cast<uint16_t*>(smem);
    const int rows_entries = (kAlphabet - 1) * W;
    const int n_entries = pv.prof16_bytes >> 1;
    if ((pv.L1 & 7) == 0) {  // rows 16-byte aligned (W and S are multiples of 16): 8 entries per load
      const int w8 = W >> 3;
      for (int e = threadIdx.x; e < (kAlphabet - 1) * w8; e += blockDim.x) {
        const int c = e / w8, x = (e - c * w8) << 3;
        const int64_t g = static_cast<int64_t>(c) * pv.L1 + S + x;
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (g + 8 <= pv.prof16_entries) v = *reinterpret_cast<const uint4*>(pv.prof16 + g);
        *reinterpret_cast<uint4*>(dst + c * W + x) = v;
      }
      for (int e = rows_entries + threadIdx.x; e < n_entries; e += blockDim.x) dst[e] = 0;
    } else {
      for (int e = threadIdx.x; e < n_entries; e += blockDim.x) {
        uint16_t v = 0;
        if (e < rows_entries) {
          const int c = e / W, x = e - c * W;
          const int64_t g = static_cast<int64_t>(c) * pv.L1 + S + x;
          if (g < pv.prof16_entries) v = pv.prof16[g];
        }
        dst[e] = v;
      }
    }
    for (int t = threadIdx.x; t < W + 16; t += blockDim.x) s1l[t] = S + t < pv.L1 ? pv.seq1[S + t] : 0;
  } else if (Wide) {
    // 8 byte pairs per 16-byte load -> 8 sign-extended int16 pairs: the 4 even entries into the first half,
    // the 4 odd ones into the second (pv.prof16_bytes each)
    const uint4* src = reinterpret_cast<const uint4*>(pv.prof16);  // 16-byte padded
    uint4* dst = reinterpret_cast<uint4*>(smem);
    const int n16 = pv.prof16_bytes >> 4;
    auto widen = [](uint32_t pair2) {  // two byte pairs (b0, b1), (b2, b3) -> (sext b0 | sext b1 << 16), ...
      const uint32_t lo = (static_cast<uint32_t>(static_cast<int8_t>(pair2 & 0xff)) & 0xffffu) |
                          (static_cast<uint32_t>(static_cast<int8_t>((pair2 >> 8) & 0xff)) << 16);
      const uint32_t hi = (static_cast<uint32_t>(static_cast<int8_t>((pair2 >> 16) & 0xff)) & 0xffffu) |
                          (static_cast<uint32_t>(static_cast<int8_t>(pair2 >> 24)) << 16);
      return make_uint2(lo, hi);
    };
    if (pv.prof16_i16) {
      // int16 Dt per entry: entry e's pair is (Dt[e], Dt[e+1]) — the even pairs are the loaded dwords, the
      // odd ones straddle them (and the next load's first value)
      for (int t = threadIdx.x; t < n16; t += blockDim.x) {
        const uint4 v = src[t];
        const uint32_t nx = t + 1 < n16 ? reinterpret_cast<const uint32_t*>(src + t + 1)[0] : 0u;
        dst[t] = v;
        dst[n16 + t] = make_uint4(__builtin_amdgcn_alignbit(v.y, v.x, 16), __builtin_amdgcn_alignbit(v.z, v.y, 16),
                                  __builtin_amdgcn_alignbit(v.w, v.z, 16), __builtin_amdgcn_alignbit(nx, v.w, 16));
      }
    } else {
      for (int t = threadIdx.x; t < n16; t += blockDim.x) {
        const uint4 v = src[t];
        const uint2 a = widen(v.x), b = widen(v.y), c = widen(v.z), d = widen(v.w);
        dst[t] = make_uint4(a.x, b.x, c.x, d.x);
        dst[n16 + t] = make_uint4(a.y, b.y, c.y, d.y);
      }
    }
    stage_bytes(s1l, pv.seq1, pv.L1 + 16);  // Seq1 + zero pad (device copy has kSeq1Pad zeros)
  } else {
    const uint4* src = reinterpret_cast<const uint4*>(pv.prof16);  // 16-byte padded
    uint4* dst = reinterpret_cast<uint4*>(smem);
    const int n16 = pv.prof16_bytes >> 4;
    for (int t = threadIdx.x; t < n16; t += blockDim.x) dst[t] = src[t];
    stage_bytes(s1l, pv.seq1, pv.L1 + 16);  // Seq1 + zero pad (device copy has kSeq1Pad zeros)
  }
  for (int t = threadIdx.x; t < kProf16Lut8; t += blockDim.x) lut8[t] = static_cast<int8_t>(pv.lut[t]);  // |T| <= 127
  __syncthreads();
  const int64_t w = w0 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (w >= n_waves) return;  // wave-uniform; no barrier follows
  const int L1 = pv.L1;
  const int lane = threadIdx.x & 63;
  const int kib = pv.t16_key_bits;  // wave-uniform: 32-bit selection keys (0: 64-bit)
  const uint32_t kmask = kib ? (1u << kib) - 1u : 0u;
  const int t_win_end = Win ? t_base + win_tiles : INT32_MAX;

  const WaveStart ws = starts[w], we = starts[w + 1];
  int li = __builtin_amdgcn_readfirstlane(ws.li), t = __builtin_amdgcn_readfirstlane(ws.t);
  const int end_li = __builtin_amdgcn_readfirstlane(we.li), end_t = __builtin_amdgcn_readfirstlane(we.t);
  // The next record's index and letter offsets are loaded one record ahead (scalar loads), and its first 64
  // letters from the current record's last chunk on (vector loads in flight through that chunk's sweep and
  // the tile epilogue): a wave moving to its next record does not wait on memory there. (Windowed plans
  // visit every record once per window, so that wait would come back per window.)
  const int64_t base_off = bv.offsets[0];
  auto rec_index = [&](int lj) { return long_recs ? __builtin_amdgcn_readfirstlane(long_recs[lj]) : lj; };
  int r_cur = li < n_long ? rec_index(li) : 0;
  int64_t off_a = li < n_long ? bv.offsets[r_cur] : 0, off_b = li < n_long ? bv.offsets[r_cur + 1] : 0;
  int c_pref = 0;
  bool pref = false;  // c_pref holds this record's first letters
  while (li < end_li || (li == end_li && t < end_t)) {  // wave-uniform
    const uint8_t* rec = bv.codes + (off_a - base_off);
    const int L2 = __builtin_amdgcn_readfirstlane(static_cast<int>(off_b - off_a));
    const bool more = li + 1 < n_long;  // wave-uniform
    const int r_next = more ? rec_index(li + 1) : 0;
    const int64_t next_a = more ? bv.offsets[r_next] : 0, next_b = more ? bv.offsets[r_next + 1] : 0;
    const int next_steps = more && next_b - next_a <= L1 ? static_cast<int>(next_b - next_a) : 0;
    const int steps = L2 <= L1 ? L2 : 0;
    const int need = L2 <= L1 ? L1 - L2 + 1 : 1;
    const int ntiles = min((need + kSpan - 1) / kSpan, t_win_end);
    const int t_stop = li == end_li ? min(end_t, ntiles) : ntiles;
    const int last = L1 - L2;
    const bool v0_at_last = pv.semantics == static_cast<int>(Semantics::Spec) || L2 == L1;
    // lane j of a chunk holds step i0 + j's letter (0 past the record) and its profile row/step offset
    auto letter = [&](int i) { return i < steps ? static_cast<int>(rec[i]) : 0; };
    auto row_off = [&](int c, int i) {
      const int e = max(c - 1, 0) * W + i;  // flat entry index past the lane's own
      return Wide ? ((e & 1) ? pv.prof16_bytes : 0) + 4 * (e >> 1) : 2 * e;
    };
    const int c_first = pref ? c_pref : letter(lane);
    pref = false;
    unsigned long long acc64 = 0;
    uint32_t acc32 = 0;  // pv.t16_key_bits: the same selection in 32-bit keys
    for (; t < t_stop && L2 <= L1; ++t) {
      const int o0 = t * kSpan;
      MOC_DCHECK(o0 >= 0 && o0 <= L1);
      // sub-tiles with valid offsets: all U but in a record's last tile (wave-uniform; no barrier below)
      const int act = (min(need, o0 + kSpan) - o0 + kSub - 1) / kSub;
      with_subtiles<U>(act, [&](auto uu) {
      constexpr int UU = decltype(uu)::value;  // this tile's sub-tiles
      // sub-tile u: lane owns offsets o0 + 128u + 2*lane (low half) and + 1 (high half); its entries sit at
      // 4 bytes per lane and 256 bytes per sub-tile in both layouts (Wide: o0 and 2*lane even)
      const unsigned char* lbase = smem + 2 * (o0 - S) + 4 * lane;
      uint32_t acc[UU], best[UU];
      int DcA[UU], DcB[UU], mxA[UU], mxB[UU];
#pragma unroll
      for (int u = 0; u < UU; ++u) {
        acc[u] = 0;
        best[u] = kBestInit;
        DcA[u] = DcB[u] = 0;
        mxA[u] = mxB[u] = INT32_MIN;
      }
      auto step = [&](int so, int j, bool key) {
        const int soff = __builtin_amdgcn_readlane(so, j);
        const unsigned char* p = lbase + soff;
        MOC_DCHECK(2 * (o0 - S) + 4 * lane + soff + 2 * kSub * (UU - 1) + EW <= prof_lds);
#pragma unroll
        for (int u = 0; u < UU; ++u) {
          if (Wide) {
            acc[u] = pk_add(acc[u], *reinterpret_cast<const uint32_t*>(p + 2 * kSub * u));
          } else {
            const uint32_t e = *reinterpret_cast<const uint16_t*>(p + 2 * kSub * u);
            add_pair(acc[u], e);
          }
          if (key) best[u] = pk_max(best[u], acc[u]);
        }
      };
      // The step offsets of 16 steps replicated in every DPP row (lane 16r + k: step 16g + k), so a step's
      // address is one row_newbcast add: no v_readlane into an SGPR (and its hazard nop) per step.
      auto replicate = [&](int so, int (&so16)[4]) {
#pragma unroll
        for (int g = 0; g < 4; ++g) so16[g] = __shfl(so, 16 * g + (lane & 15), 64);
      };
      // GG steps from chunk step j (a constant once unrolled), every step a key step: the GG*UU profile reads
      // issue before the first add, so the LDS latency of a group hides under the adds of the group before
      auto group = [&](const int (&so16)[4], int j, auto gg) {
        constexpr int GG = decltype(gg)::value;
        uint32_t e[GG][UU];
#pragma unroll
        for (int q = 0; q < GG; ++q) {
          const unsigned char* p = lbase + row_newbcast(so16[(j + q) >> 4], (j + q) & 15);
#pragma unroll
          for (int u = 0; u < UU; ++u)
            e[q][u] = Wide ? *reinterpret_cast<const uint32_t*>(p + 2 * kSub * u)
                           : *reinterpret_cast<const uint16_t*>(p + 2 * kSub * u);
        }
#pragma unroll
        for (int q = 0; q < GG; ++q)
#pragma unroll
          for (int u = 0; u < UU; ++u) {
            if (Wide)
              acc[u] = pk_add(acc[u], e[q][u]);
            else
              add_pair(acc[u], e[q][u]);
            best[u] = pk_max(best[u], acc[u]);
          }
      };
      // full chunks: G steps per group, G * UU reads in flight (UU = 8 keeps the VGPRs within 4 waves per SIMD)
      constexpr int G = UU >= 8 ? 2 : UU >= 4 ? 4 : 8;
      // every 64-step chunk starts from zero halves and folds them into the int32 state at its end; the
      // record's first chunk sets the state (no adds to zero, no max with INT32_MIN); a chunk of one step
      // has no key step (compile-time forms: no per-lane selects)
      auto flush = [&](auto first_c, auto key_c) {
        constexpr bool First = decltype(first_c)::value, AnyKey = decltype(key_c)::value;
#pragma unroll
        for (int u = 0; u < UU; ++u) {
          if (AnyKey) {
            mxA[u] = First ? lo16(best[u]) : max(mxA[u], DcA[u] + lo16(best[u]));
            mxB[u] = First ? hi16(best[u]) : max(mxB[u], DcB[u] + hi16(best[u]));
          }
          DcA[u] = First ? lo16(acc[u]) : DcA[u] + lo16(acc[u]);
          DcB[u] = First ? hi16(acc[u]) : DcB[u] + hi16(acc[u]);
          acc[u] = 0;
          best[u] = kBestInit;
        }
      };
      using True = std::true_type;
      using False = std::false_type;
      // Tot of the anchor offset oA (first offset past the tile or past the valid range): each chunk's
      // lanes add their step's pair score from LDS while the sweep runs
      const int oA = min(o0 + kSpan, need);
      int anchor = 0;
      auto anchor_add = [&](int c, int i) {  // an int16 profile's weights may pass int8: T from the global LUT
        if (c != 0) anchor += pv.prof16_i16 ? pv.lut[c * kLutStride + s1l[oA - S + i]] : lut8[c * kLutStride + s1l[oA - S + i]];
      };
      int c = c_first;
      int i0 = 0;
      for (; i0 + 64 < steps; i0 += 64) {  // full chunks (the record's last letter lies beyond)
        const int c_next = letter(i0 + 64 + lane);
        const int so = row_off(c, i0 + lane);
        anchor_add(c, i0 + lane);
        int so16[4];
        replicate(so, so16);
#pragma unroll
        for (int j = 0; j < 64; j += G) group(so16, j, std::integral_constant<int, G>());
        flush(False(), True());  // (a first-chunk form here peels the loop: 128 VGPRs and spills)
        c = c_next;
      }
      if (steps > 0) {  // last chunk: 1..64 steps; no hyphen after the final letter
        if (t + 1 == t_stop && more) {  // the record's last tile here: the next record's first letters
          c_pref = lane < next_steps ? static_cast<int>(bv.codes[next_a - base_off + lane]) : 0;
          pref = true;
        }
        const int m = steps - i0;
        const int so = row_off(c, i0 + lane);
        anchor_add(c, i0 + lane);
        int j = 0;
        // groups of 8 steps before the last one (short records live here)
        if constexpr (UU >= 8) {  // 8 sub-tiles: a runtime loop (the unrolled one is too large), v_readlane steps
          for (; j + 4 <= m - 1; j += 4) {
            uint32_t e[4][UU];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const unsigned char* p = lbase + __builtin_amdgcn_readlane(so, j + q);
#pragma unroll
              for (int u = 0; u < UU; ++u)
                e[q][u] = Wide ? *reinterpret_cast<const uint32_t*>(p + 2 * kSub * u)
                               : *reinterpret_cast<const uint16_t*>(p + 2 * kSub * u);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
              for (int u = 0; u < UU; ++u) {
                if (Wide)
                  acc[u] = pk_add(acc[u], e[q][u]);
                else
                  add_pair(acc[u], e[q][u]);
                best[u] = pk_max(best[u], acc[u]);
              }
          }
        } else {
          int so16[4];
          replicate(so, so16);
#pragma unroll
          for (int jj = 0; jj + 8 < 64; jj += 8) {
            if (jj + 8 > m - 1) break;  // wave-uniform
            group(so16, jj, std::integral_constant<int, 8>());
            j = jj + 8;
          }
        }
        for (; j < m - 1; ++j) step(so, j, true);
        step(so, m - 1, false);
        if (i0 == 0 && m > 1)  // wave-uniform: the record's only chunk (short records, input4)
          flush(True(), True());
        else if (m > 1)
          flush(False(), True());
        else if (i0 == 0)
          flush(True(), False());
        else
          flush(False(), False());
      }
      // ---- Tot per offset: anchor diagonal oA, then suffix sums of the D totals (valid offsets only)
      anchor = __builtin_amdgcn_readlane(wave_prefix_sum_dpp(anchor), 63);
      // Full: every candidate of the tile's sub-tiles is valid (all but a record's last tiles) — no per-lane
      // limit tests and no masked D totals (compile-time form)
      auto epilogue = [&](auto full_c, auto key32_c) {
        constexpr bool Full = decltype(full_c)::value, Key32 = decltype(key32_c)::value;
        int carry = anchor;  // Tot at the end of the sub-tile being processed
        int incl[UU];        // the sub-tiles' pair sums, then their inclusive prefix sums over the lanes
#pragma unroll
        for (int u = 0; u < UU; ++u) {
          const int oa = o0 + kSub * u + 2 * lane;
          if (!Full) {
            DcA[u] = oa < oA ? DcA[u] : 0;
            DcB[u] = oa + 1 < oA ? DcB[u] : 0;
          }
          incl[u] = DcA[u] + DcB[u];
        }
        wave_prefix_sums_dpp(incl);
#pragma unroll
        for (int u = UU - 1; u >= 0; --u) {
          const int oa = o0 + kSub * u + 2 * lane;
          const int ca = DcA[u], cb = DcB[u];  // (masked past oA)
          const int sub_total = __builtin_amdgcn_readlane(incl[u], 63);
          const int excl = sub_total - incl[u];  // lanes above this one
          const int totB = carry + excl + cb;    // Tot_{oa+1}
          const int totA = totB + ca;            // Tot_{oa}
          carry += sub_total;
          // every candidate of the sub-tile valid (wave-uniform)
          const bool all_valid = Full || (o0 + kSub * (u + 1) < last && L2 >= 2);
          if constexpr (Key32) {
            // keys ((score + 2^(31 - kib)) << kib) | (2^kib - 1 - idx): the bias and the index term are one
            // per-lane constant, so a key is one shift-add of the score (moc/kernel_bounds.hpp tile16_key32_bits)
            const uint32_t c0 = 0x80000000u + kmask - 2u * static_cast<uint32_t>(oa);  // idx 2 oa
            const uint32_t kA0 = (static_cast<uint32_t>(totA) << kib) + c0;
            const uint32_t kA1 = ((static_cast<uint32_t>(mxA[u]) + static_cast<uint32_t>(totB)) << kib) + (c0 - 1u);
            const uint32_t kB0 = (static_cast<uint32_t>(totB) << kib) + (c0 - 2u);
            const uint32_t kB1 = ((static_cast<uint32_t>(mxB[u]) + static_cast<uint32_t>(totB - cb)) << kib) + (c0 - 3u);
            // validity as pass1_candidate: o <= last (o < last, or L2 == L1 / spec semantics, for the
            // un-mutated one), mutants at o < last with L2 >= 2
            if (all_valid) {
              acc32 = max(max(acc32, max(kA0, kA1)), max(kB0, kB1));
            } else {
              const uint32_t a0 = oa < last || (oa == last && v0_at_last) ? kA0 : 0u;
              const uint32_t a1 = oa < last && L2 >= 2 ? kA1 : 0u;
              const uint32_t b0 = oa + 1 < last || (oa + 1 == last && v0_at_last) ? kB0 : 0u;
              const uint32_t b1 = oa + 1 < last && L2 >= 2 ? kB1 : 0u;
              acc32 = max(max(acc32, max(a0, a1)), max(b0, b1));
            }
          } else {
            if (all_valid) {
              const uint32_t i0 = 2u * static_cast<uint32_t>(oa);
              acc64 = max_u64(acc64, max_u64(max_u64(final_key(totA, i0), final_key(mxA[u] + totB, i0 + 1u)),
                                             max_u64(final_key(totB, i0 + 2u), final_key(mxB[u] + totB - cb, i0 + 3u))));
            } else {
              acc64 = max_u64(acc64, pass1_candidate(oa, L1, L2, pv.semantics, totA, totB, mxA[u]));
              acc64 = max_u64(acc64, pass1_candidate(oa + 1, L1, L2, pv.semantics, totB, totB - cb, mxB[u]));
            }
          }
        }
      };
      // (key width and fullness outside the sub-tile loop: one basic block, the 8 sub-tiles' DPP scans
      // interleave)
      const bool full = o0 + kSub * UU < last && L2 >= 2;  // wave-uniform (then oA >= o0 + kSub * UU too)
      if (kib) {
        if (full)
          epilogue(True(), True());
        else
          epilogue(False(), True());
      } else {
        if (full)
          epilogue(True(), False());
        else
          epilogue(False(), False());
      }
      });
    }
    if (kib) {
      const uint32_t k = wave_max_u32_dpp(acc32);
      if (lane == 0 && k != 0u)
        atomicMax(keys + li, final_key(static_cast<int>(k >> kib) - (1 << (31 - kib)), kmask - (k & kmask)));
    } else {
      const unsigned long long k = wave_max_u64(acc64);
      if (lane == 0 && k != 0ull) atomicMax(keys + li, k);
    }
    ++li;
    t = t_base;
    off_a = next_a;
    off_b = next_b;
  }
}

// Sliding windows: long records on a Seq1 whose widened image does not fit one CU (limits: L1 3000,
// records up to 2000 letters; int16 profiles past L1 ~ 1500). The 16 waves of a workgroup take 16 records of
// similar length (plan: records sorted by length, groups of 16) and sweep the SAME offset tile t of each, in
// lockstep over windows of C steps: for steps [iw, iw + C) every wave reads only columns
// [o0 + iw, o0 + iw + span + C), so the workgroup stages that window (widened, W = span + C columns), runs the
// window's 64-step chunks, and slides on. The per-offset state stays in registers across windows; waves
// whose record ends early (or has fewer tiles) only join the barriers. Items (group, tiles [t0, t1)) are
// LPT-balanced over the workgroups on the host (HipEngine::plan_waves).
//   plan16[0 .. n_wg]: workgroup b takes items [plan16[b].li, plan16[b + 1].li);
//   plan16[items + 2k]     = {group g, t0},  plan16[items + 2k + 1] = {group's longest record, t1};
//   plan16[members + 16g + w] = {li (-1: none), L2} — wave w's record.
template <int U, int WavesPerSimd>
__global__ __launch_bounds__(kBlock16) __attribute__((amdgpu_waves_per_eu(WavesPerSimd)))
void tile16_slide_kernel(ProblemView pv, BatchView bv,
                                                                const WaveStart* __restrict__ plan16, int64_t items,
                                                                int64_t members, const int32_t* __restrict__ long_recs,
                                                                unsigned long long* __restrict__ keys) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int prof_lds = 2 * pv.prof16_bytes;
  int8_t* lut8 = reinterpret_cast<int8_t*>(smem + prof_lds);
  uint8_t* s1l = smem + prof_lds + kProf16Lut8;
  constexpr int kSpan = kSub * U;
  const int W = pv.prof16_window;  // window columns: span + C
  const int C = W - kSpan;         // steps per window (a multiple of 64)
  for (int t = threadIdx.x; t < kProf16Lut8; t += blockDim.x) lut8[t] = static_cast<int8_t>(pv.lut[t]);
  const int L1 = pv.L1;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int kib = pv.t16_key_bits;
  const uint32_t kmask = kib ? (1u << kib) - 1u : 0u;
  const int64_t base_off = bv.offsets[0];
  const int k_end = __builtin_amdgcn_readfirstlane(plan16[blockIdx.x + 1].li);
  for (int k = __builtin_amdgcn_readfirstlane(plan16[blockIdx.x].li); k < k_end; ++k) {  // workgroup-uniform
    const WaveStart ia = plan16[items + 2 * k], ib = plan16[items + 2 * k + 1];
    const int g = __builtin_amdgcn_readfirstlane(ia.li), t0 = __builtin_amdgcn_readfirstlane(ia.t);
    const int lmax = __builtin_amdgcn_readfirstlane(ib.li), t1 = __builtin_amdgcn_readfirstlane(ib.t);
    const WaveStart mem = plan16[members + 16 * static_cast<int64_t>(g) + wave];
    const int li = __builtin_amdgcn_readfirstlane(mem.li);
    const int L2 = __builtin_amdgcn_readfirstlane(mem.t);
    const int r = li < 0 ? 0 : long_recs ? __builtin_amdgcn_readfirstlane(long_recs[li]) : li;
    const uint8_t* rec = bv.codes + (bv.offsets[r] - base_off);
    const int steps = li >= 0 && L2 <= L1 ? L2 : 0;
    const int need = L2 <= L1 ? L1 - L2 + 1 : 1;
    const int own_tiles = steps > 0 ? (need + kSpan - 1) / kSpan : 0;
    const int last = L1 - L2;
    const bool v0_at_last = pv.semantics == static_cast<int>(Semantics::Spec) || L2 == L1;
    auto letter = [&](int i) { return i < steps ? static_cast<int>(rec[i]) : 0; };
    // the record's best candidate key: 64-bit, or a 32-bit selection key in the low half (pv.t16_key_bits)
    unsigned long long acc64 = 0;
    for (int t = t0; t < t1; ++t) {  // workgroup-uniform
      const int o0 = t * kSpan;
      const bool on = t < own_tiles;  // wave-uniform
      uint32_t acc[U], best[U];
      int DcA[U], DcB[U], mxA[U], mxB[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        acc[u] = 0;
        best[u] = kBestInit;
        DcA[u] = DcB[u] = 0;
        mxA[u] = mxB[u] = INT32_MIN;
      }
      const int oA = min(o0 + kSpan, need);
      int anchor = 0;
      int c = letter(lane);
      for (int iw = 0; iw < lmax; iw += C) {  // workgroup-uniform
        const int S = o0 + iw;
        __syncthreads();  // every wave is done with the previous window
        stage_window_wide(smem, s1l, pv, S, W);
        __syncthreads();
        if (!on || iw >= steps) continue;  // wave-uniform: this wave only joins the barriers
        // lane l of a chunk holds step i0 + l's letter; its entry sits at (c - 1) * W + (i - iw) + the
        // lane's own offset within the window (o0 - S = -iw), split by parity (iw is even)
        const unsigned char* lbase = smem - 2 * iw + 4 * lane;
        auto row_off = [&](int cc, int i) {
          const int e = max(cc - 1, 0) * W + i;
          return ((e & 1) ? pv.prof16_bytes : 0) + 4 * (e >> 1);
        };
        auto anchor_add = [&](int cc, int i) {
          if (cc != 0) anchor += pv.prof16_i16 ? pv.lut[cc * kLutStride + s1l[oA - S + i]] : lut8[cc * kLutStride + s1l[oA - S + i]];
        };
        auto step = [&](int so, int j, bool key) {
          const unsigned char* p = lbase + __builtin_amdgcn_readlane(so, j);
#pragma unroll
          for (int u = 0; u < U; ++u) {
            acc[u] = pk_add(acc[u], *reinterpret_cast<const uint32_t*>(p + 2 * kSub * u));
            if (key) best[u] = pk_max(best[u], acc[u]);
          }
        };
        auto group = [&](const int (&so16)[4], int j, auto gg) {
          constexpr int GG = decltype(gg)::value;
          uint32_t e[GG][U];
#pragma unroll
          for (int q = 0; q < GG; ++q) {
            const unsigned char* p = lbase + row_newbcast(so16[(j + q) >> 4], (j + q) & 15);
#pragma unroll
            for (int u = 0; u < U; ++u) e[q][u] = *reinterpret_cast<const uint32_t*>(p + 2 * kSub * u);
          }
#pragma unroll
          for (int q = 0; q < GG; ++q)
#pragma unroll
            for (int u = 0; u < U; ++u) {
              acc[u] = pk_add(acc[u], e[q][u]);
              best[u] = pk_max(best[u], acc[u]);
            }
        };
        auto flush = [&](bool any_key) {
#pragma unroll
          for (int u = 0; u < U; ++u) {
            if (any_key) {
              mxA[u] = max(mxA[u], DcA[u] + lo16(best[u]));
              mxB[u] = max(mxB[u], DcB[u] + hi16(best[u]));
            }
            DcA[u] += lo16(acc[u]);
            DcB[u] += hi16(acc[u]);
            acc[u] = 0;
            best[u] = kBestInit;
          }
        };
        // two workgroups per CU (64 VGPRs): half the reads per group in flight, the other workgroup hides the rest
        constexpr int G = WavesPerSimd >= 8 ? (U >= 4 ? 2 : 4) : (U >= 4 ? 4 : 8);
        const int i_end = min(iw + C, steps);
        int i0 = iw;
        for (; i0 + 64 <= i_end && i0 + 64 < steps; i0 += 64) {  // full chunks (the record goes on past them)
          const int c_next = letter(i0 + 64 + lane);
          const int so = row_off(c, i0 + lane);
          anchor_add(c, i0 + lane);
          int so16[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) so16[q] = __shfl(so, 16 * q + (lane & 15), 64);
#pragma unroll
          for (int j = 0; j < 64; j += G) group(so16, j, std::integral_constant<int, G>());
          flush(true);
          c = c_next;
        }
        if (i0 < i_end) {  // the record's last chunk (1..64 steps) lies in this window
          const int m = steps - i0;
          const int so = row_off(c, i0 + lane);
          anchor_add(c, i0 + lane);
          int j = 0;
          for (; j < m - 1; ++j) step(so, j, true);
          step(so, m - 1, false);
          flush(m > 1);
        }
      }
      if (!on) continue;
      // ---- Tot per offset: anchor diagonal oA, then suffix sums of the D totals (valid offsets only)
      anchor = __builtin_amdgcn_readlane(wave_prefix_sum_dpp(anchor), 63);
      int carry = anchor;
#pragma unroll
      for (int u = U - 1; u >= 0; --u) {
        const int oa = o0 + kSub * u + 2 * lane;
        const int ca = oa < oA ? DcA[u] : 0, cb = oa + 1 < oA ? DcB[u] : 0;
        const int incl = wave_prefix_sum_dpp(ca + cb);
        const int sub_total = __builtin_amdgcn_readlane(incl, 63);
        const int totB = carry + (sub_total - incl) + cb;  // Tot_{oa+1}
        const int totA = totB + ca;                        // Tot_{oa}
        carry += sub_total;
        if (kib) {
          const uint32_t c0 = 0x80000000u + kmask - 2u * static_cast<uint32_t>(oa);
          const uint32_t kA0 = (static_cast<uint32_t>(totA) << kib) + c0;
          const uint32_t kA1 = ((static_cast<uint32_t>(mxA[u]) + static_cast<uint32_t>(totB)) << kib) + (c0 - 1u);
          const uint32_t kB0 = (static_cast<uint32_t>(totB) << kib) + (c0 - 2u);
          const uint32_t kB1 = ((static_cast<uint32_t>(mxB[u]) + static_cast<uint32_t>(totB - cb)) << kib) + (c0 - 3u);
          uint32_t k32 = static_cast<uint32_t>(acc64);
          if (o0 + kSub * (u + 1) < last && L2 >= 2) {  // wave-uniform: every candidate of the sub-tile valid
            k32 = max(max(k32, max(kA0, kA1)), max(kB0, kB1));
          } else {
            const uint32_t a0 = oa < last || (oa == last && v0_at_last) ? kA0 : 0u;
            const uint32_t a1 = oa < last && L2 >= 2 ? kA1 : 0u;
            const uint32_t b0 = oa + 1 < last || (oa + 1 == last && v0_at_last) ? kB0 : 0u;
            const uint32_t b1 = oa + 1 < last && L2 >= 2 ? kB1 : 0u;
            k32 = max(max(k32, max(a0, a1)), max(b0, b1));
          }
          acc64 = k32;
        } else {
          if (o0 + kSub * (u + 1) < last && L2 >= 2) {  // wave-uniform: every candidate of the sub-tile valid
            const uint32_t i0 = 2u * static_cast<uint32_t>(oa);
            acc64 = max_u64(acc64, max_u64(max_u64(final_key(totA, i0), final_key(mxA[u] + totB, i0 + 1u)),
                                           max_u64(final_key(totB, i0 + 2u), final_key(mxB[u] + totB - cb, i0 + 3u))));
          } else {
            acc64 = max_u64(acc64, pass1_candidate(oa, L1, L2, pv.semantics, totA, totB, mxA[u]));
            acc64 = max_u64(acc64, pass1_candidate(oa + 1, L1, L2, pv.semantics, totB, totB - cb, mxB[u]));
          }
        }
      }
    }
    if (li < 0 || L2 > L1) continue;  // wave-uniform; no barrier follows in this item
    if (kib) {
      const uint32_t kk = wave_max_u32_dpp(static_cast<uint32_t>(acc64));
      if (lane == 0 && kk != 0u)
        atomicMax(keys + li, final_key(static_cast<int>(kk >> kib) - (1 << (31 - kib)), kmask - (kk & kmask)));
    } else {
      const unsigned long long kk = wave_max_u64(acc64);
      if (lane == 0 && kk != 0ull) atomicMax(keys + li, kk);
    }
  }
}

int tile16_waves_per_cu(int lds_bytes) {  // lds_bytes: the whole image a workgroup stages
  const int blocks = lds_bytes > 0 ? kProf16MaxLds / lds_bytes : 2;
  return kWavesPerBlock16 * max(1, min(2, blocks));
}

namespace {
template <int U, bool Win, bool Wide = false>
void launch16_t(const ProblemView& pv, const BatchView& bv, const Plan& plan, hipStream_t stream) {
  // dynamic LDS above 64 KiB is declared per kernel and device (engines may live on several devices
  // and threads of one process)
  static std::mutex mu;
  static std::set<int> declared;
  int dev = 0;
  MOC_HIP_CHECK(hipGetDevice(&dev));
  {
    std::lock_guard<std::mutex> lock(mu);
    if (declared.insert(dev).second)
      MOC_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&tile16_search_kernel<U, Win, Wide>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, kProf16MaxLds));
  }
  const int64_t blocks = (plan.n_waves + kWavesPerBlock16 - 1) / kWavesPerBlock16;
  const int64_t s1_len = Win ? pv.prof16_window : pv.L1;
  hipLaunchKernelGGL((tile16_search_kernel<U, Win, Wide>), dim3(static_cast<unsigned>(blocks)), dim3(kBlock16),
                     static_cast<size_t>(tile16_lds_bytes(Wide ? 2 * pv.prof16_bytes : pv.prof16_bytes, s1_len)),
                     stream, pv, bv, plan.starts, plan.n_waves, plan.long_recs, plan.n_long, plan.keys,
                     plan.win_tiles);
}

template <int U, int WavesPerSimd>
void launch16_slide(const ProblemView& pv, const BatchView& bv, const Plan& plan, hipStream_t stream) {
  static std::mutex mu;
  static std::set<int> declared;
  int dev = 0;
  MOC_HIP_CHECK(hipGetDevice(&dev));
  {
    std::lock_guard<std::mutex> lock(mu);
    if (declared.insert(dev).second)
      MOC_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&tile16_slide_kernel<U, WavesPerSimd>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, kProf16MaxLds));
  }
  const int64_t blocks = plan.n_waves / kWavesPerBlock16;
  hipLaunchKernelGGL((tile16_slide_kernel<U, WavesPerSimd>), dim3(static_cast<unsigned>(blocks)), dim3(kBlock16),
                     static_cast<size_t>(tile16_lds_bytes(2 * pv.prof16_bytes, pv.prof16_window)), stream, pv, bv,
                     plan.starts, plan.slide_items, plan.slide_members, plan.long_recs, plan.keys);
}
}  // namespace

void preload_tile16_kernels() {
  hipFuncAttributes fa;
  (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&tile16_search_kernel<2, false>));
}

void launch_tile16_keys(const ProblemView& pv, const BatchView& bv, const Plan& plan, hipStream_t stream,
                        bool mfma_sweep) {
  if (pv.t16_slide) {
    // sliding windows: span + 64k columns, widened, every item's group in lockstep (plan_slide)
    const int span = kSub * plan.u;
    if (!pv.prof16 || mfma_sweep || !pv.prof16_wide || (plan.u != 2 && plan.u != 4 && plan.u != 8) || (pv.t16_slide == 2 && plan.u == 8) ||
        plan.slide_items <= 0 ||
        plan.slide_members <= plan.slide_items || plan.n_waves % kWavesPerBlock16 ||
        pv.prof16_window < span + 64 || (pv.prof16_window - span) % 64 ||
        pv.prof16_bytes != tile16_window_bytes(pv.prof16_window) ||
        tile16_lds_bytes(2 * pv.prof16_bytes, pv.prof16_window) > kProf16MaxLds)
      throw Error("launch_tile16_keys: bad sliding-window plan");
    if (plan.n_long > 0) MOC_HIP_CHECK(hipMemsetAsync(plan.keys, 0, sizeof(unsigned long long) * plan.n_long, stream));
    if (plan.n_waves <= 0) return;
    if (pv.t16_slide == 2) {  // two workgroups per CU: 8 waves per SIMD, 64 VGPRs
      if (plan.u == 2)
        launch16_slide<2, 8>(pv, bv, plan, stream);
      else
        launch16_slide<4, 8>(pv, bv, plan, stream);
    } else {
      switch (plan.u) {
        case 2: launch16_slide<2, 4>(pv, bv, plan, stream); break;
        case 8: launch16_slide<8, 4>(pv, bv, plan, stream); break;
        default: launch16_slide<4, 4>(pv, bv, plan, stream); break;
      }
    }
    return;
  }
  const int64_t s1_len = pv.prof16_window > 0 ? pv.prof16_window : pv.L1;
  const bool wide = pv.prof16_wide && !mfma_sweep;
  if (pv.prof16_i16 && !wide) throw Error("launch_tile16_keys: an int16 profile runs the widened image only");
  if (!pv.prof16 || pv.prof16_bytes <= 0 ||
      tile16_lds_bytes(wide ? 2 * pv.prof16_bytes : pv.prof16_bytes, s1_len) > kProf16MaxLds ||
      (pv.prof16_bytes & 15) ||
      (pv.prof16_window > 0 && (plan.win_tiles <= 0 || mfma_sweep || plan.u > (wide ? 8 : 4))))
    throw Error("launch_tile16_keys: no usable profile");
  if (plan.n_long > 0) MOC_HIP_CHECK(hipMemsetAsync(plan.keys, 0, sizeof(unsigned long long) * plan.n_long, stream));
  if (plan.n_waves <= 0) return;
  if (mfma_sweep) {
    launch_tile_mfma_sweep(pv, bv, plan, stream);
  } else {
    if (pv.prof16_window > 0 && wide) {
      switch (plan.u) {
        case 1: launch16_t<1, true, true>(pv, bv, plan, stream); break;
        case 2: launch16_t<2, true, true>(pv, bv, plan, stream); break;
        case 8: launch16_t<8, true, true>(pv, bv, plan, stream); break;
        default: launch16_t<4, true, true>(pv, bv, plan, stream); break;
      }
    } else if (pv.prof16_window > 0) {
      switch (plan.u) {
        case 1: launch16_t<1, true>(pv, bv, plan, stream); break;
        case 2: launch16_t<2, true>(pv, bv, plan, stream); break;
        default: launch16_t<4, true>(pv, bv, plan, stream); break;
      }
    } else if (wide) {
      switch (plan.u) {
        case 1: launch16_t<1, false, true>(pv, bv, plan, stream); break;
        case 2: launch16_t<2, false, true>(pv, bv, plan, stream); break;
        case 8: launch16_t<8, false, true>(pv, bv, plan, stream); break;
        default: launch16_t<4, false, true>(pv, bv, plan, stream); break;
      }
    } else {
      switch (plan.u) {
        case 1: launch16_t<1, false>(pv, bv, plan, stream); break;
        case 2: launch16_t<2, false>(pv, bv, plan, stream); break;
        case 8: launch16_t<8, false>(pv, bv, plan, stream); break;
        default: launch16_t<4, false>(pv, bv, plan, stream); break;
      }
    }
  }
}

}  // namespace dev
}  // namespace moc
