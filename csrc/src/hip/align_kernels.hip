// Long-record search kernels (gfx950, wave64): one wave = (record, 63 consecutive offsets).
//
// Replaces calc_result (cudaFunctions.cu:63-176) for records whose offset range does not fit in one
// wave (L1 - L2 + 1 > 64; input3/input4-shaped). See moc/device.hpp for the design summary and
// csrc/include/moc/cpu_engine.hpp for the closed form
//     score(o, 0) = Tot_o,   score(o, k>=1) = P_o(k) - P_{o+1}(k) + Tot_{o+1}.
// Per lane (= one offset o) and per Seq2 position i:
//     x   = Seq1[o+i]           (shifted in from lane+1 with DPP; lane 63 gets a wave-uniform LDS read)
//     P  += LUT[Seq2[i]][x]     (one conflict-free ds_read_b32: <= 27 distinct consecutive dwords)
//     Pn  = P of lane+1         (DPP wave_shl:1 — the neighbouring diagonal, no LDS traffic)
//     key = max(key, pack(P - Pn, k = i+1))   (ties -> smallest k, exactly the reference order)
// Lane 63 only provides the helper diagonal; the wave's best candidate goes to the record's slot with
// one 64-bit atomicMax (max over unique keys is order-free: deterministic), then a finalize pass
// decodes (score, n, k).
#include <hip/hip_runtime.h>

#include "kernel_common.hpp"

namespace moc {
namespace dev {

using namespace kc;

template <bool Wide, bool Seq1Lds>
__global__ __launch_bounds__(256) void tile_search_kernel(ProblemView pv, BatchView bv, const Tile* __restrict__ tiles,
                                                          int64_t n_tiles, const int32_t* __restrict__ long_recs,
                                                          unsigned long long* __restrict__ keys) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int* lut = reinterpret_cast<int*>(smem);
  uint8_t* s1l = smem + kLutInts * sizeof(int);
  const int L1 = pv.L1;
  stage_lut(lut, pv.lut);
  if (Seq1Lds) stage_bytes(s1l, pv.seq1, L1 + kSeq1Pad);
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
  const int r = long_recs ? __builtin_amdgcn_readfirstlane(long_recs[li]) : li;  // null: identity (CP plans)
  const int64_t base = bv.offsets[r] - bv.offsets[0];
  const int L2 = __builtin_amdgcn_readfirstlane(static_cast<int>(bv.offsets[r + 1] - bv.offsets[r]));
  const uint8_t* rec = bv.codes + base;
  const int o = o0 + lane;
  const int shift = pv.key_shift, mask = (1 << pv.key_shift) - 1;

  int x = s1[min(o, L1 + kSeq1Pad - 1)];
  int P = 0;
  typename K::T best = K::min();
  const int feed0 = o0 + 64;  // lane 63's next letter index
  const int steps = L2 <= L1 ? L2 : 0;
  for (int i = 0; i < steps; ++i) {
    const int c = __builtin_amdgcn_readfirstlane(static_cast<int>(rec[i]));
    P += lut[(c << 5) | x];
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
  const bool own = lane < kTileOffsets && L2 <= L1 && o <= L1 - L2;
  unsigned long long key = lane_candidate<Wide>(own, o, L1, L2, pv.semantics, P, Pn, best, shift, mask);
  key = wave_max_u64(key);
  if (lane == 0 && key != 0ull) atomicMax(keys + li, key);
}

__global__ void finalize_long_kernel(BatchView bv, const int32_t* __restrict__ long_recs,
                                     const unsigned long long* __restrict__ keys, int64_t n_long, void* out, int fmt) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n_long) return;
  const int r = long_recs ? long_recs[i] : static_cast<int>(i);
  const int L2 = static_cast<int>(bv.offsets[r + 1] - bv.offsets[r]);
  store_result(out, r, fmt, decode_key(keys[i], L2 > 0 ? L2 : 1));
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

namespace {
constexpr int kBlock = 256;
constexpr int kMaxSeq1Lds = 56 * 1024;  // Seq1 staged in LDS up to this size (keeps dyn. LDS < 64 KiB)

template <bool Wide>
void launch_search_t(const ProblemView& pv, const BatchView& bv, const Plan& plan, hipStream_t stream) {
  const size_t lds_lut = kLutInts * sizeof(int);
  const size_t lds_s1 = static_cast<size_t>(pv.L1 + kSeq1Pad + 3) & ~size_t{3};
  const bool s1_in_lds = pv.L1 + kSeq1Pad <= kMaxSeq1Lds;
  const int64_t blocks = (plan.n_tiles * 64 + kBlock - 1) / kBlock;
  if (s1_in_lds)
    hipLaunchKernelGGL((tile_search_kernel<Wide, true>), dim3(static_cast<unsigned>(blocks)), dim3(kBlock),
                       lds_lut + lds_s1, stream, pv, bv, plan.tiles, plan.n_tiles, plan.long_recs, plan.keys);
  else
    hipLaunchKernelGGL((tile_search_kernel<Wide, false>), dim3(static_cast<unsigned>(blocks)), dim3(kBlock), lds_lut,
                       stream, pv, bv, plan.tiles, plan.n_tiles, plan.long_recs, plan.keys);
}

void launch_finalize(const BatchView& bv, const Plan& plan, void* out, int fmt, hipStream_t stream) {
  if (plan.n_long <= 0) return;
  const int64_t fb = (plan.n_long + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(finalize_long_kernel, dim3(static_cast<unsigned>(fb)), dim3(kBlock), 0, stream, bv,
                     plan.long_recs, plan.keys, plan.n_long, out, fmt);
}
}  // namespace

void launch_tile_keys(const ProblemView& pv, const BatchView& bv, const Plan& plan, hipStream_t stream) {
  if (plan.n_long > 0) (void)hipMemsetAsync(plan.keys, 0, sizeof(unsigned long long) * plan.n_long, stream);
  if (plan.n_tiles <= 0) return;
  if (pv.key_shift > 0)
    launch_search_t<false>(pv, bv, plan, stream);
  else
    launch_search_t<true>(pv, bv, plan, stream);
}

void launch_finalize_keys(const BatchView& bv, const Plan& plan, void* out, int fmt, hipStream_t stream) {
  launch_finalize(bv, plan, out, fmt, stream);
}

void launch_tiles(const ProblemView& pv, const BatchView& bv, const Plan& plan, void* out, int fmt,
                  hipStream_t stream) {
  if (plan.n_tiles <= 0) return;
  launch_tile_keys(pv, bv, plan, stream);
  launch_finalize(bv, plan, out, fmt, stream);
}

}  // namespace dev
}  // namespace moc
