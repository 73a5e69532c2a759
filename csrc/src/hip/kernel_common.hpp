// Device helpers shared by the gfx950 search kernels (wave64 cross-lane ops, candidate keys, result
// formats). Included only by .hip translation units.
#pragma once

#include <hip/hip_runtime.h>

#include "moc/device.hpp"

// Device-side bounds checks: compiled in with -DMOC_DEBUG_KERNELS (make debug-kernels),
// they print the failing condition and let the kernel continue — a report, never a GPU fault.
#ifdef MOC_DEBUG_KERNELS
#define MOC_DCHECK(cond)                                                                                     \
  do {                                                                                                       \
    if (!(cond)) printf("MOC_DCHECK %s:%d block %d thread %d: %s\n", __FILE__, __LINE__, (int)blockIdx.x,    \
                        (int)threadIdx.x, #cond);                                                            \
  } while (0)
#else
#define MOC_DCHECK(cond) \
  do {                   \
  } while (0)
#endif

namespace moc {
namespace dev {
namespace kc {

constexpr int kLutInts = kLutStride * kLutStride;  // 1024
constexpr int kDppWaveShl1 = 0x130;                // lane i <- lane i+1 (lane 63: bound)

// The result goes through an empty asm so the backend's DPP combiner cannot fold the move into the
// consuming VALU op: on gfx950 / ROCm 7.2 the folded `v_subrev_u32_dpp vD, vP, vP wave_shl:1` computed
// P(lane+1) - P(lane) instead of P(lane) - P(lane+1) (found with tools/debug_tiles.py: every
// tile-kernel candidate came out with the sign of d flipped). One extra v_mov_dpp per cell.
__device__ __forceinline__ int wave_shl1(int v) {
  int r = __builtin_amdgcn_update_dpp(0, v, kDppWaveShl1, 0xf, 0xf, true);
  asm volatile("" : "+v"(r));
  return r;
}
// Same shift, but lane 63 receives `fill` instead of 0.
__device__ __forceinline__ int wave_shl1_fill(int v, int fill) {
  int r = __builtin_amdgcn_update_dpp(fill, v, kDppWaveShl1, 0xf, 0xf, false);
  asm volatile("" : "+v"(r));
  return r;
}

// ---- hot-loop keys: (d = P_o(k) - P_{o+1}(k), k) with "larger d, then smaller k" ordering ----------
template <bool Wide>
struct HotKey;

template <>
struct HotKey<false> {  // int32: d in the high bits, (mask - k) in the low `shift` bits
  using T = int32_t;
  static __device__ __forceinline__ T min() { return INT32_MIN; }
  static __device__ __forceinline__ T make(int d, int k, int shift, int mask) {
    return static_cast<int32_t>((static_cast<uint32_t>(d) << shift) | static_cast<uint32_t>(mask - k));
  }
  static __device__ __forceinline__ int d(T key, int shift) { return key >> shift; }
  static __device__ __forceinline__ int k(T key, int mask) { return mask - (key & mask); }
};

template <>
struct HotKey<true> {  // int64: d in the high word, (0xffffffff - k) in the low word
  using T = int64_t;
  static __device__ __forceinline__ T min() { return INT64_MIN; }
  static __device__ __forceinline__ T make(int d, int k, int, int) {
    return static_cast<int64_t>(d) * 4294967296ll + static_cast<int64_t>(0xffffffffu - static_cast<uint32_t>(k));
  }
  static __device__ __forceinline__ int d(T key, int) { return static_cast<int>(key >> 32); }
  static __device__ __forceinline__ int k(T key, int) {
    return static_cast<int>(0xffffffffu - static_cast<uint32_t>(key & 0xffffffffll));
  }
};

// ---- final 64-bit candidate keys: score high, ~(o*L2 + k) low -> max = best with reference tie-break
__device__ __forceinline__ unsigned long long final_key(int score, uint32_t idx) {
  return (static_cast<unsigned long long>(static_cast<uint32_t>(score) ^ 0x80000000u) << 32) |
         static_cast<unsigned long long>(0xffffffffu - idx);
}

__device__ __forceinline__ Result decode_key(unsigned long long key, int L2) {
  if (key == 0ull) return Result{INT32_MIN, 0, 0};
  const int score = static_cast<int>(static_cast<uint32_t>(key >> 32) ^ 0x80000000u);
  const uint32_t idx = 0xffffffffu - static_cast<uint32_t>(key);
  return Result{score, static_cast<int>(idx / static_cast<uint32_t>(L2)),
                static_cast<int>(idx % static_cast<uint32_t>(L2))};
}

__device__ __forceinline__ unsigned long long max_u64(unsigned long long a, unsigned long long b) {
  return a > b ? a : b;
}

__device__ __forceinline__ unsigned long long shfl_down_u64(unsigned long long v, int d) {
  const int lo = __shfl_down(static_cast<int>(v), d, 64);
  const int hi = __shfl_down(static_cast<int>(v >> 32), d, 64);
  return (static_cast<unsigned long long>(static_cast<uint32_t>(hi)) << 32) | static_cast<uint32_t>(lo);
}

__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const int lo = __shfl_xor(static_cast<int>(v), d, 64);
    const int hi = __shfl_xor(static_cast<int>(v >> 32), d, 64);
    v = max_u64(v, (static_cast<unsigned long long>(static_cast<uint32_t>(hi)) << 32) | static_cast<uint32_t>(lo));
  }
  return v;
}

__device__ __forceinline__ int wave_max_i32(int v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v = max(v, __shfl_xor(v, d, 64));
  return v;
}

// Wave maximum of a value in [0, 256), wave-uniform (an SGPR): eight ballots of a binary search, so branches
// on it are scalar and no lane data moves through LDS (wave_max_i32's shuffles are ds_bpermute operations).
__device__ __forceinline__ int wave_max_small(int v) {
  int m = 0;
#pragma unroll
  for (int b = 128; b >= 1; b >>= 1)
    if (__builtin_amdgcn_ballot_w64(v >= m + b) != 0) m += b;
  return __builtin_amdgcn_readfirstlane(m);
}

// Inclusive prefix sum over the 64 lanes of a wave.
__device__ __forceinline__ int wave_inclusive_sum(int v, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int t = __shfl_up(v, d, 64);
    if (lane >= d) v += t;
  }
  return v;
}

// Lane's best candidate key for offset `o` after the sweep.
//   P = Tot_o, Pn = Tot_{o+1}, best = best hot key over k = 1..steps.
// Hot-loop steps past L2 only repeat k = L2 with d = Tot_o - Tot_{o+1}, whose score equals the
// un-mutated candidate's with a larger index, so they can never win (no masking needed in the loop).
template <bool Wide>
__device__ __forceinline__ unsigned long long lane_candidate(bool own, int o, int L1, int L2, int sem, int P, int Pn,
                                                             typename HotKey<Wide>::T best, int shift, int mask) {
  using K = HotKey<Wide>;
  unsigned long long key = 0;
  if (!own) return key;
  const int last = L1 - L2;  // un-mutated at o == last: spec only (or the equal-length case)
  const bool v0 = (o < last) || (o == last && (sem == static_cast<int>(Semantics::Spec) || L2 == L1));
  if (v0) key = final_key(P, static_cast<uint32_t>(o) * static_cast<uint32_t>(L2));
  if (o < last && L2 >= 2 && best != K::min()) {
    const int s1 = K::d(best, shift) + Pn;
    const int k = K::k(best, mask);
    key = max_u64(key, final_key(s1, static_cast<uint32_t>(o) * static_cast<uint32_t>(L2) + static_cast<uint32_t>(k)));
  }
  return key;
}

// The same candidate as a PASS-1 key (score, ~(2o + mutated)) of the long-record sweeps: which k wins on
// the winning diagonal is resolved afterwards (resolve_long_kernel), so the key never holds o*L2 + k and
// L1 * L2 may exceed 2^32 (o < 2^31 is the only bound). Same order as final keys: score, then the
// smallest o, then the un-mutated candidate first.
template <bool Wide>
__device__ __forceinline__ unsigned long long lane_pass1_candidate(bool own, int o, int L1, int L2, int sem, int P,
                                                                   int Pn, typename HotKey<Wide>::T best, int shift) {
  using K = HotKey<Wide>;
  unsigned long long key = 0;
  if (!own) return key;
  const int last = L1 - L2;
  const bool v0 = (o < last) || (o == last && (sem == static_cast<int>(Semantics::Spec) || L2 == L1));
  if (v0) key = final_key(P, 2u * static_cast<uint32_t>(o));
  if (o < last && L2 >= 2 && best != K::min())
    key = max_u64(key, final_key(K::d(best, shift) + Pn, 2u * static_cast<uint32_t>(o) + 1u));
  return key;
}

// ---- result formats -------------------------------------------------------------------------------
__device__ __forceinline__ void store_result(void* out, int64_t r, int fmt, const Result& v, const R2Params& p) {
  if (fmt == static_cast<int>(ResultFormat::R2)) {
    static_cast<uint16_t*>(out)[r] =
        v.score == INT32_MIN ? kR2None : static_cast<uint16_t>((v.score - p.smin) * p.j + v.n * p.kw + v.k);
  } else if (fmt == static_cast<int>(ResultFormat::R4)) {
    R4 x;
    x.score = static_cast<int16_t>(v.score == INT32_MIN ? INT16_MIN : v.score);
    x.n = static_cast<uint8_t>(v.n);
    x.k = static_cast<uint8_t>(v.k);
    static_cast<R4*>(out)[r] = x;
  } else if (fmt == static_cast<int>(ResultFormat::R8)) {
    R8 x;
    x.score = v.score;
    x.n = static_cast<uint16_t>(v.n);
    x.k = static_cast<uint16_t>(v.k);
    static_cast<R8*>(out)[r] = x;
  } else {
    static_cast<Result*>(out)[r] = v;
  }
}

__device__ __forceinline__ int fmt_bytes(int fmt) {
  return fmt == static_cast<int>(ResultFormat::R12) ? 12
         : fmt == static_cast<int>(ResultFormat::R8) ? 8
         : fmt == static_cast<int>(ResultFormat::R4) ? 4
                                                      : 2;
}

// Persistent-kernel work counter {next tile, blocks done}: the last block to leave resets both to 0, so
// the next launch needs no memset (and a captured hipGraph replays correctly). Call from every block
// after it left its tile loop; stream order makes the reset visible to the next kernel.
__device__ __forceinline__ void release_work_counter(unsigned* counter) {
  if (threadIdx.x == 0) {
    __threadfence();
    if (atomicAdd(counter + 1, 1u) == gridDim.x - 1) {
      atomicExch(counter, 0u);
      atomicExch(counter + 1, 0u);
    }
  }
}

// Letter offset of record r, where r is a tile boundary (a multiple of 1 << off_shift) or the batch end n:
// dense offsets hold every record, sparse ones (the parser's narrow wire format) every 2^off_shift-th
// plus the end, so entry ceil(r / 2^off_shift) is record r's.
__device__ __forceinline__ int64_t tile_offset(const ShortArgs& a, int64_t r) {
  return a.offsets[(r + (int64_t{1} << a.off_shift) - 1) >> a.off_shift];
}

// Length of record `idx` of the batch from the narrowest available source.
__device__ __forceinline__ uint32_t base6_octet(const uint8_t* words, int64_t octet) {
  const uint64_t w = *reinterpret_cast<const uint64_t*>(words + 8 * (octet / 3));
  return static_cast<uint32_t>(w >> (21 * static_cast<int>(octet % 3))) & 0x1FFFFFu;
}

__device__ __forceinline__ int record_length(const ShortArgs& a, int64_t idx) {
  if (a.lengths6) {
    uint32_t v = base6_octet(a.lengths6, idx >> 3);
    for (int j = static_cast<int>(idx & 7); j > 0; --j) v /= 6u;
    return a.len_base + static_cast<int>(v % 6u);
  }
  if (a.lengths3) {
    const int64_t bit = 3 * idx;
    const uint32_t w = a.lengths3[bit >> 3] | (static_cast<uint32_t>(a.lengths3[(bit >> 3) + 1]) << 8);
    return a.len_base + static_cast<int>((w >> (bit & 7)) & 7u);
  }
  if (a.lengths4) return a.len_base + ((a.lengths4[idx >> 1] >> (4 * (idx & 1))) & 15);
  if (a.lengths8) return a.lengths8[idx];
  return static_cast<int>(a.offsets[idx + 1] - a.offsets[idx]);
}

// Lengths of the 4 consecutive records i0 .. i0+3 of a thread (entries past n_valid are 0) with one or
// two loads instead of one or two per record: for host-resident (zero-copy) batches every load instruction
// becomes PCIe read requests, and the length loads outnumber the letter loads otherwise.
__device__ __forceinline__ void record_lengths4(const ShortArgs& a, int64_t i0, int n_valid, int (&L)[4]) {
  if (n_valid >= 4 && (i0 & 3) == 0 &&
      !(a.lengths3 == nullptr && a.lengths4 == nullptr && a.lengths8 == nullptr && a.lengths6 == nullptr)) {
    if (a.lengths6) {  // one aligned 8-byte load; the upper half of an octet starts at digit 4 (6^4 = 1296)
      uint32_t v = base6_octet(a.lengths6, i0 >> 3);
      if (i0 & 4) v /= 1296u;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t d = v / 6u;
        L[q] = a.len_base + static_cast<int>(v - 6u * d);
        v = d;
      }
      return;
    }
    if (a.lengths8) {
      const uint32_t w = *reinterpret_cast<const uint32_t*>(a.lengths8 + i0);
#pragma unroll
      for (int q = 0; q < 4; ++q) L[q] = static_cast<int>((w >> (8 * q)) & 0xffu);
      return;
    }
    if (a.lengths4) {
      const uint32_t w = *reinterpret_cast<const uint16_t*>(a.lengths4 + (i0 >> 1));
#pragma unroll
      for (int q = 0; q < 4; ++q) L[q] = a.len_base + static_cast<int>((w >> (4 * q)) & 15u);
      return;
    }
    const int64_t bit = 3 * i0;  // multiple of 4 records: the 12 bits start at bit 0 or 4 of a byte
    const uint8_t* b = a.lengths3 + (bit >> 3);
    const uint32_t w = (static_cast<uint32_t>(b[0]) | (static_cast<uint32_t>(b[1]) << 8)) >> (bit & 7);
#pragma unroll
    for (int q = 0; q < 4; ++q) L[q] = a.len_base + static_cast<int>((w >> (3 * q)) & 7u);
    return;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) L[q] = q < n_valid ? record_length(a, i0 + q) : 0;
}

// 16-byte non-temporal (streaming) accesses: host memory read or written once over PCIe (zero-copy)
// needs no L2 residency
typedef unsigned int u32x4_nt __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 nt_load16(const void* p) {
  const u32x4_nt v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_nt*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void nt_store16(void* p, uint4 x) {
  const u32x4_nt v = {x.x, x.y, x.z, x.w};
  __builtin_nontemporal_store(v, reinterpret_cast<u32x4_nt*>(p));
}

// Copies a block's staged results (LDS) to the output: dwords, plus a trailing halfword for R2 tiles
// of odd length. `dst` is 4-byte aligned (tiles start at multiples of 64 records).
__device__ __forceinline__ void copy_results(void* dst, const uint8_t* src, int bytes, int tid, int nthreads) {
  // 16-byte stores when the destination allows (tile starts are multiples of 128 bytes): to host memory
  // (zero-copy) fewer, fuller write requests share the link with the tile loads' read requests
  int done = 0;
  if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
    const int n16 = bytes >> 4;
    for (int q = tid; q < n16; q += nthreads)
      nt_store16(static_cast<uint4*>(dst) + q, reinterpret_cast<const uint4*>(src)[q]);
    done = n16 << 4;
  }
  const int nd = (bytes - done) >> 2;
  uint32_t* d32 = reinterpret_cast<uint32_t*>(static_cast<char*>(dst) + done);
  const uint32_t* s32 = reinterpret_cast<const uint32_t*>(src + done);
  for (int q = tid; q < nd; q += nthreads) d32[q] = s32[q];
  if (((bytes - done) & 2) && tid == 0)
    reinterpret_cast<uint16_t*>(d32)[2 * nd] = reinterpret_cast<const uint16_t*>(s32)[2 * nd];
}

__device__ __forceinline__ void stage_lut(int* lut, const int32_t* g) {
  for (int t = threadIdx.x; t < kLutInts; t += blockDim.x) lut[t] = g[t];
}
__device__ __forceinline__ void stage_bytes(uint8_t* dst, const uint8_t* src, int n) {
  // 4-byte copy; both buffers are padded so rounding n up to a multiple of 4 stays in bounds
  const int n4 = (n + 3) >> 2;
  const uint32_t* s = reinterpret_cast<const uint32_t*>(src);
  uint32_t* d = reinterpret_cast<uint32_t*>(dst);
  for (int t = threadIdx.x; t < n4; t += blockDim.x) d[t] = s[t];
}

}  // namespace kc
}  // namespace dev
}  // namespace moc
