// CDNA4 (gfx950) alignment-search kernels. Native HIP, wave64, no CUDA shims.
//
// Replaces calc_result (cudaFunctions.cu:63-176). See moc/device.hpp for the design summary and
// csrc/include/moc/cpu_engine.hpp for the closed form
//     score(o, 0) = Tot_o,   score(o, k>=1) = P_o(k) - P_{o+1}(k) + Tot_{o+1}.
//
// Per lane (= one offset o) and per Seq2 position i:
//     x   = Seq1[o+i]           (LDS; the tile kernel shifts it in from lane+1 with DPP)
//     P  += LUT[Seq2[i]][x]     (one conflict-free ds_read_b32: <= 27 distinct consecutive dwords)
//     Pn  = P of lane+1         (DPP wave_shl:1 — the neighbouring diagonal, no LDS traffic)
//     key = max(key, pack(P - Pn, k = i+1))   (ties -> smallest k, exactly the reference order)
#include <hip/hip_runtime.h>

#include "moc/device.hpp"

namespace moc {
namespace dev {

namespace {

constexpr int kLutInts = kLutStride * kLutStride;  // 1024
constexpr int kDppWaveShl1 = 0x130;                // lane i <- lane i+1 (lane 63: bound)

// The result goes through an empty asm so the backend's DPP combiner cannot fold the move into the
// consuming VALU op: on gfx950 / ROCm 7.2 the folded `v_subrev_u32_dpp vD, vP, vP wave_shl:1` computed
// P(lane+1) - P(lane) instead of P(lane) - P(lane+1) (measured with tools/debug_tiles.py: every
// tile-kernel candidate came out with the sign of d flipped). One extra v_mov_dpp per cell.
__device__ __forceinline__ int wave_shl1(int v) {
  int r = __builtin_amdgcn_update_dpp(0, v, kDppWaveShl1, 0xf, 0xf, true);
  asm volatile("" : "+v"(r));
  return r;
}
// Same shift, but lane 63 receives `fill` instead of 0.
__device__ __forceinline__ int wave_shl1_fill(int v, int fill) {
  return __builtin_amdgcn_update_dpp(fill, v, kDppWaveShl1, 0xf, 0xf, false);
}

// ---- hot-loop keys: (d = P_o(k) - P_{o+1}(k), k) with "larger d, then smaller k" ordering --------
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
  return Result{score, static_cast<int>(idx / static_cast<uint32_t>(L2)), static_cast<int>(idx % static_cast<uint32_t>(L2))};
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

// Lane's best candidate key for offset `o` after the sweep.
//   P = Tot_o, Pn = Tot_{o+1}, best = best hot key over k = 1..L2-1.
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

template <bool Seq1Lds>
struct Seq1Src {
  const uint8_t* p;
  __device__ __forceinline__ int operator[](int i) const { return p[i]; }
};

__device__ __forceinline__ void stage_lut(int* lut, const int32_t* g) {
  for (int t = threadIdx.x; t < kLutInts; t += blockDim.x) lut[t] = g[t];
}
__device__ __forceinline__ void stage_seq1(uint8_t* s1, const uint8_t* g, int n) {
  // 4-byte vectorised copy (n is padded by kSeq1Pad, so a multiple-of-4 round-up stays in bounds)
  const int n4 = (n + 3) >> 2;
  const uint32_t* src = reinterpret_cast<const uint32_t*>(g);
  uint32_t* dst = reinterpret_cast<uint32_t*>(s1);
  for (int t = threadIdx.x; t < n4; t += blockDim.x) dst[t] = src[t];
}

}  // namespace

// =====================================================================================================
// Packed kernel: several short records per wave, one lane slot of `slot` lanes per record.
// =====================================================================================================
template <bool Wide>
__global__ __launch_bounds__(256) void packed_search_kernel(ProblemView pv, BatchView bv, int slot, int rpw,
                                                            Result* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int* lut = reinterpret_cast<int*>(smem);
  uint8_t* s1 = smem + kLutInts * sizeof(int);
  const int L1 = pv.L1;
  stage_lut(lut, pv.lut);
  stage_seq1(s1, pv.seq1, L1 + kSeq1Pad);
  __syncthreads();

  using K = HotKey<Wide>;
  const int lane = threadIdx.x & 63;
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int sl = lane / slot;
  const int o = lane - sl * slot;
  const int64_t r = wave * rpw + sl;
  const bool in = sl < rpw && r < bv.n;
  int L2 = 0;
  int64_t base = 0;
  if (in) {
    base = bv.offsets[r] - bv.offsets[0];
    L2 = static_cast<int>(bv.offsets[r + 1] - bv.offsets[r]);
  }
  const int need = L2 <= L1 ? L1 - L2 + 1 : 1;
  const bool mine = in && need <= slot;  // longer records belong to the tile kernel
  const bool on = mine && L2 <= L1 && o < need;
  const int steps = wave_max_i32(on ? L2 : 0);
  const int shift = pv.key_shift, mask = (1 << pv.key_shift) - 1;

  const uint8_t* rec = bv.codes + base;
  int P = 0;
  typename K::T best = K::min();
  for (int i = 0; i < steps; ++i) {
    const bool live = on && i < L2;
    const int c = live ? rec[i] : 0;
    const int x = s1[o + i];  // o + i < L1 + 64 <= L1 + kSeq1Pad
    const int a = lut[(c << 5) | x];
    P += live ? a : 0;
    const int Pn = wave_shl1(P);
    if (live && i + 1 < L2) {
      const typename K::T key = K::make(P - Pn, i + 1, shift, mask);
      best = key > best ? key : best;
    }
  }
  const int Pn = wave_shl1(P);
  unsigned long long key = lane_candidate<Wide>(on, o, L1, L2, pv.semantics, P, Pn, best, shift, mask);

  // segmented (per-slot) max: suffix max over the slot's lanes, leader = lane with o == 0
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned long long other = shfl_down_u64(key, d);
    if (o + d < slot) key = max_u64(key, other);
  }
  if (mine && o == 0) out[r] = decode_key(key, L2 > 0 ? L2 : 1);
}

// =====================================================================================================
// Tile kernel: one wave = (record, 63 consecutive offsets); lane 63 is the helper diagonal.
// =====================================================================================================
template <bool Wide, bool Seq1Lds>
__global__ __launch_bounds__(256) void tile_search_kernel(ProblemView pv, BatchView bv, const Tile* __restrict__ tiles,
                                                          int64_t n_tiles, const int32_t* __restrict__ long_recs,
                                                          unsigned long long* __restrict__ keys, int* debug) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int* lut = reinterpret_cast<int*>(smem);
  uint8_t* s1l = smem + kLutInts * sizeof(int);
  const int L1 = pv.L1;
  stage_lut(lut, pv.lut);
  if (Seq1Lds) stage_seq1(s1l, pv.seq1, L1 + kSeq1Pad);
  __syncthreads();
  const uint8_t* s1 = Seq1Lds ? s1l : pv.seq1;

  using K = HotKey<Wide>;
  const int lane = threadIdx.x & 63;
  const int64_t wave = __builtin_amdgcn_readfirstlane(
      static_cast<int>((static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6));
  if (wave >= n_tiles) return;  // wave-uniform exit (no barrier follows)
  const Tile tile = tiles[wave];
  const int li = __builtin_amdgcn_readfirstlane(tile.li);
  const int o0 = __builtin_amdgcn_readfirstlane(tile.o0);
  const int r = __builtin_amdgcn_readfirstlane(long_recs[li]);
  const int64_t base = bv.offsets[r] - bv.offsets[0];
  const int L2 = __builtin_amdgcn_readfirstlane(static_cast<int>(bv.offsets[r + 1] - bv.offsets[r]));
  const uint8_t* rec = bv.codes + base;
  const int o = o0 + lane;
  const int shift = pv.key_shift, mask = (1 << pv.key_shift) - 1;

  int x = s1[min(o, L1 + kSeq1Pad - 1)];
  int P = 0;
  typename K::T best = K::min();
  const int feed0 = o0 + 64;  // lane 63's next letter index
  for (int i = 0; i < L2; ++i) {
    const int c = __builtin_amdgcn_readfirstlane(static_cast<int>(rec[i]));
    const int a = lut[(c << 5) | x];
    P += a;
    const int Pn = wave_shl1(P);
    if (i + 1 < L2) {
      const typename K::T key = K::make(P - Pn, i + 1, shift, mask);
      best = key > best ? key : best;
    }
    const int fidx = min(feed0 + i, L1 + kSeq1Pad - 1);
    const int feed = __builtin_amdgcn_readfirstlane(static_cast<int>(s1[fidx]));
    x = wave_shl1_fill(x, feed);
  }
  const int Pn = wave_shl1(P);
  const bool own = lane < kTileOffsets && o <= L1 - L2;
  unsigned long long key = lane_candidate<Wide>(own, o, L1, L2, pv.semantics, P, Pn, best, shift, mask);
  if (debug && wave == debug[0]) {
    debug[64 + lane * 4 + 0] = P;
    debug[64 + lane * 4 + 1] = static_cast<int>(best);
    debug[64 + lane * 4 + 2] = Pn;
    debug[64 + lane * 4 + 3] = x;
    if (lane == 0) {
      debug[1] = L2;
      debug[2] = o0;
      debug[3] = r;
      for (int i = 0; i < 8 && i < L2; ++i) debug[8 + i] = rec[i];
      debug[16] = static_cast<int>(key >> 32);
      debug[17] = static_cast<int>(key);
    }
  }
  key = wave_max_u64(key);
  if (lane == 0 && key != 0ull) atomicMax(keys + li, key);
}

__global__ void finalize_long_kernel(BatchView bv, const int32_t* __restrict__ long_recs,
                                     const unsigned long long* __restrict__ keys, int64_t n_long,
                                     Result* __restrict__ out) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n_long) return;
  const int r = long_recs[i];
  const int L2 = static_cast<int>(bv.offsets[r + 1] - bv.offsets[r]);
  out[r] = decode_key(keys[i], L2);
}

// Self-test of the cross-lane primitives the search kernels rely on (one wave):
//   out[0..63]   = wave_shl1(lane)           expected lane+1, lane 63 -> 0
//   out[64..127] = wave_shl1_fill(lane, 777) expected lane+1, lane 63 -> 777
//   out[128..191]= wave_max_i32(lane*7 % 61)  expected 60 everywhere
__global__ void dpp_probe_kernel(int* out) {
  const int lane = threadIdx.x & 63;
  out[lane] = wave_shl1(lane);
  out[64 + lane] = wave_shl1_fill(lane, 777);
  out[128 + lane] = wave_max_i32((lane * 7) % 61);
}

void launch_dpp_probe(int* d_out, hipStream_t stream) {
  hipLaunchKernelGGL(dpp_probe_kernel, dim3(1), dim3(64), 0, stream, d_out);
}

// =====================================================================================================
// Host launchers
// =====================================================================================================
namespace {
constexpr int kBlock = 256;
constexpr int kMaxSeq1Lds = 56 * 1024;  // Seq1 staged in LDS up to this size (keeps dyn. LDS < 64 KiB)

template <bool Wide>
void launch_all(const ProblemView& pv, const BatchView& bv, const Plan& plan, Result* out, hipStream_t stream) {
  const size_t lds_lut = kLutInts * sizeof(int);
  const size_t lds_s1 = static_cast<size_t>(pv.L1 + kSeq1Pad + 3) & ~size_t{3};
  const bool s1_in_lds = pv.L1 + kSeq1Pad <= kMaxSeq1Lds;
  if (plan.slot > 0 && bv.n > 0) {
    const int64_t waves = (bv.n + plan.rec_per_wave - 1) / plan.rec_per_wave;
    const int64_t blocks = (waves * 64 + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(packed_search_kernel<Wide>, dim3(static_cast<unsigned>(blocks)), dim3(kBlock),
                       lds_lut + lds_s1, stream, pv, bv, plan.slot, plan.rec_per_wave, out);
  }
  if (plan.n_tiles > 0) {
    (void)hipMemsetAsync(plan.keys, 0, sizeof(unsigned long long) * plan.n_long, stream);
    const int64_t blocks = (plan.n_tiles * 64 + kBlock - 1) / kBlock;
    if (s1_in_lds)
      hipLaunchKernelGGL((tile_search_kernel<Wide, true>), dim3(static_cast<unsigned>(blocks)), dim3(kBlock),
                         lds_lut + lds_s1, stream, pv, bv, plan.tiles, plan.n_tiles, plan.long_recs, plan.keys, plan.debug);
    else
      hipLaunchKernelGGL((tile_search_kernel<Wide, false>), dim3(static_cast<unsigned>(blocks)), dim3(kBlock),
                         lds_lut, stream, pv, bv, plan.tiles, plan.n_tiles, plan.long_recs, plan.keys, plan.debug);
    const int64_t fb = (plan.n_long + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(finalize_long_kernel, dim3(static_cast<unsigned>(fb)), dim3(kBlock), 0, stream, bv,
                       plan.long_recs, plan.keys, plan.n_long, out);
  }
}
}  // namespace

void launch_search(const ProblemView& pv, const BatchView& bv, const Plan& plan, Result* out, hipStream_t stream) {
  if (pv.key_shift > 0)
    launch_all<false>(pv, bv, plan, out, stream);
  else
    launch_all<true>(pv, bv, plan, out, stream);
}

}  // namespace dev
}  // namespace moc
