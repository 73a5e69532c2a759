// Long-record search kernels (gfx950, wave64). Work unit: a wave tile = (record, 63·U consecutive
// offsets) as U sub-tiles of 63 owned offsets + 1 helper lane that advance together (they share each
// Seq2 letter; their dependency chains interleave). Persistent waves walk cost-balanced contiguous runs
// of the record-major tile list (host plan: moc::HipEngine::plan_waves), keeping a record's letters in
// registers and its running best key across the run (one reduction + atomic per record run).
//
// Replaces calc_result (cudaFunctions.cu:63-176) for records whose offset range does not fit in one
// wave (L1 - L2 + 1 > 64; input3/input4-shaped). See moc/device.hpp for the design summary and
// csrc/include/moc/cpu_engine.hpp for the closed form
//     score(o, 0) = Tot_o,   score(o, k>=1) = P_o(k) - P_{o+1}(k) + Tot_{o+1}.
// Per lane (= one offset o) and per Seq2 position i:
//     x   = Seq1[o+i]           (shifted in from lane+1 with DPP; lane 63 gets the next Seq1 letter,
//                                 64 of them fetched per load and pulled out with v_readlane)
//     P  += LUT[Seq2[i]][x]     (one conflict-free ds_read_b32: <= 27 distinct consecutive dwords;
//                                 Seq2[i] arrives 64 letters per load, broadcast with v_readlane)
//     Pn  = P of lane+1         (DPP wave_shl:1 — the neighbouring diagonal, no LDS traffic)
//     key = max(key, pack(P - Pn, k = i+1))   (ties -> smallest k, exactly the reference order)
// Lane 63 only provides the helper diagonal; the wave's best candidate goes to the record's slot with
// one 64-bit atomicMax (max over unique keys is order-free: deterministic), then a finalize pass
// decodes (score, n, k).
#include <hip/hip_runtime.h>

#include "kernel_common.hpp"
#include "moc/runtime/hip_check.hpp"

namespace moc {
namespace dev {

using namespace kc;

template <bool Wide, bool Seq1Lds, int U>
__global__ __launch_bounds__(256) void tile_search_kernel(ProblemView pv, BatchView bv, const WaveStart* __restrict__ starts,
                                                          int64_t n_waves, const int32_t* __restrict__ long_recs,
                                                          unsigned long long* __restrict__ keys) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int* lut = reinterpret_cast<int*>(smem);
  uint8_t* s1l = smem + kLutInts * sizeof(int);
  const int L1 = pv.L1;
  stage_lut(lut, pv.lut);
  if (Seq1Lds) stage_bytes(s1l, pv.seq1, L1 + kSeq1Pad);
  __syncthreads();
  const int64_t w = static_cast<int64_t>(blockIdx.x) * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (w >= n_waves) return;  // wave-uniform; no barrier follows
  const uint8_t* s1 = Seq1Lds ? s1l : pv.seq1;
  const int s1_last = L1 + kSeq1Pad - 1;

  using K = HotKey<Wide>;
  const int lane = threadIdx.x & 63;
  const int shift = pv.key_shift, mask = (1 << pv.key_shift) - 1;
  constexpr int kSpan = kTileOffsets * U;  // offsets per wave tile

  const WaveStart ws = starts[w], we = starts[w + 1];
  int li = __builtin_amdgcn_readfirstlane(ws.li), t = __builtin_amdgcn_readfirstlane(ws.t);
  const int end_li = __builtin_amdgcn_readfirstlane(we.li), end_t = __builtin_amdgcn_readfirstlane(we.t);
  while (li < end_li || (li == end_li && t < end_t)) {  // wave-uniform
    // ---- one record: its letters stay in registers across the run's tiles of it
    const int r = long_recs ? __builtin_amdgcn_readfirstlane(long_recs[li]) : li;  // null: identity (CP plans)
    const uint8_t* rec = bv.codes + (bv.offsets[r] - bv.offsets[0]);
    const int L2 = __builtin_amdgcn_readfirstlane(static_cast<int>(bv.offsets[r + 1] - bv.offsets[r]));
    const int steps = L2 <= L1 ? L2 : 0;
    const int need = L2 <= L1 ? L1 - L2 + 1 : 1;
    const int ntiles = (need + kSpan - 1) / kSpan;
    const int t_stop = li == end_li ? min(end_t, ntiles) : ntiles;
    const int cv_first = lane < steps ? static_cast<int>(rec[lane]) : 0;
    unsigned long long acc = 0;
    for (; t < t_stop; ++t) {
      const int o0 = t * kSpan;
      MOC_DCHECK(o0 >= 0 && o0 <= L1);
      // sub-tile u: lanes 0..62 own offsets o0 + 63u + lane, lane 63 is its helper diagonal
      int x[U], P[U];
      typename K::T best[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        x[u] = s1[min(o0 + kTileOffsets * u + lane, s1_last)];
        P[u] = 0;
        best[u] = K::min();
      }
      // Seq2 letters and the helper lanes' Seq1 feeds arrive 64 steps at a time as one coalesced load
      // per wave (lane j holds step j's value; the next chunk's letters are in flight meanwhile); each
      // step pulls its values out with v_readlane, so only the LDS LUT reads sit on its critical path.
      auto step = [&](int cv, const int (&fv)[U], int j, int k, bool key) {
        const int c = __builtin_amdgcn_readlane(cv, j);
        const int* row = lut + (c << 5);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          P[u] += row[x[u]];
          if (key) {
            const int Pn = wave_shl1(P[u]);
            const typename K::T kk = K::make(P[u] - Pn, k, shift, mask);
            best[u] = kk > best[u] ? kk : best[u];
            x[u] = wave_shl1_fill(x[u], __builtin_amdgcn_readlane(fv[u], j));
          }
        }
      };
      int cv = cv_first;
      int i0 = 0;
      for (; i0 + 64 < steps; i0 += 64) {  // full chunks (the record's last letter lies beyond)
        const int cv_next = i0 + 64 + lane < steps ? static_cast<int>(rec[i0 + 64 + lane]) : 0;
        int fv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) fv[u] = s1[min(o0 + kTileOffsets * u + 64 + i0 + lane, s1_last)];
#pragma unroll 8
        for (int j = 0; j < 64; ++j) step(cv, fv, j, i0 + j + 1, true);
        cv = cv_next;
      }
      if (steps > 0) {  // last chunk: 1..64 steps; no hyphen after the final letter
        const int m = steps - i0;
        int fv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) fv[u] = s1[min(o0 + kTileOffsets * u + 64 + i0 + lane, s1_last)];
        for (int j = 0; j < m - 1; ++j) step(cv, fv, j, i0 + j + 1, true);
        step(cv, fv, m - 1, 0, false);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int o = o0 + kTileOffsets * u + lane;
        const int Pn = wave_shl1(P[u]);
        const bool own = lane < kTileOffsets && L2 <= L1 && o <= L1 - L2;
        acc = max_u64(acc, lane_pass1_candidate<Wide>(own, o, L1, L2, pv.semantics, P[u], Pn, best[u], shift));
      }
    }
    const unsigned long long k = wave_max_u64(acc);
    if (lane == 0 && k != 0ull) atomicMax(keys + li, k);
    ++li;
    t = 0;
  }
}

// One wave per long record: its pass-1 key (score, ~(2o + mutated)) from the sweep (tile, tile16 or
// tile-mfma; or a context-parallel MAX of several) -> the result (score, n = o, k). For a mutated winner
// k is the smallest k in 1..L2-1 with P_o(k) - P_{o+1}(k) + Tot_{o+1} == score, found with a wave prefix
// scan of the diagonal differences (ballot picks the first match): O(L2) per record, and no o*L2 + k
// index anywhere, so L1 * L2 may exceed 2^32.
__global__ __launch_bounds__(256) void resolve_long_kernel(ProblemView pv, BatchView bv,
                                                           const int32_t* __restrict__ long_recs,
                                                           const unsigned long long* __restrict__ keys, int64_t n_long,
                                                           void* out, int fmt) {
  const int64_t li = static_cast<int64_t>(blockIdx.x) * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (li >= n_long) return;
  const int lane = threadIdx.x & 63;
  const int r = long_recs ? long_recs[li] : static_cast<int>(li);
  const unsigned long long key = keys[li];
  if (key == 0ull) {
    if (lane == 0) store_result(out, r, fmt, Result{INT32_MIN, 0, 0}, pv.r2);
    return;
  }
  const int score = static_cast<int>(static_cast<uint32_t>(key >> 32) ^ 0x80000000u);
  const uint32_t idx = 0xffffffffu - static_cast<uint32_t>(key);
  const int o = static_cast<int>(idx >> 1);
  const uint8_t* rec = bv.codes + (bv.offsets[r] - bv.offsets[0]);
  const int L2 = static_cast<int>(bv.offsets[r + 1] - bv.offsets[r]);
  int k = 0;
  if (idx & 1u) {  // mutated: o < L1 - L2, so Seq1[o + 1 + i] stays inside Seq1 for i < L2
    MOC_DCHECK(o + L2 < pv.L1 && L2 >= 2);
    const uint8_t* s1 = pv.seq1 + o;
    int tot1 = 0;
    for (int i = lane; i < L2; i += 64) tot1 += pv.lut[rec[i] * kLutStride + s1[i + 1]];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) tot1 += __shfl_xor(tot1, d, 64);
    const int target = score - tot1;  // D_o(k) of the winning k
    int carry = 0;
    k = -1;
    for (int i0 = 0; i0 < L2 - 1; i0 += 64) {  // candidate k = i + 1, i in [0, L2 - 2]
      const int i = i0 + lane;
      int d = 0;
      if (i < L2 - 1) {
        const int* row = pv.lut + rec[i] * kLutStride;
        d = row[s1[i]] - row[s1[i + 1]];
      }
      const int incl = wave_inclusive_sum(d, lane) + carry;
      const unsigned long long hit = __ballot(i < L2 - 1 && incl == target);
      if (hit) {
        k = i0 + __builtin_ctzll(hit) + 1;
        break;
      }
      carry = __shfl(incl, 63, 64);
    }
    MOC_DCHECK(k >= 1);
    if (k < 1) k = 0;  // unreachable (the sweep saw this score on this diagonal)
  }
  if (lane == 0) store_result(out, r, fmt, Result{score, o, k}, pv.r2);
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

void preload_align_kernels() {
  hipFuncAttributes fa;
  (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&dpp_probe_kernel));
}

void launch_dpp_probe(int* d_out, hipStream_t stream) {
  hipLaunchKernelGGL(dpp_probe_kernel, dim3(1), dim3(64), 0, stream, d_out);
}

namespace {
constexpr int kBlock = 256;
constexpr int kMaxSeq1Lds = 56 * 1024;  // Seq1 staged in LDS up to this size (keeps dyn. LDS < 64 KiB)

template <bool Wide, int U>
void launch_search_t(const ProblemView& pv, const BatchView& bv, const Plan& plan, hipStream_t stream) {
  const size_t lds_lut = kLutInts * sizeof(int);
  const size_t lds_s1 = static_cast<size_t>(pv.L1 + kSeq1Pad + 3) & ~size_t{3};
  const bool s1_in_lds = pv.L1 + kSeq1Pad <= kMaxSeq1Lds;
  const int64_t blocks = (plan.n_waves * 64 + kBlock - 1) / kBlock;
  if (s1_in_lds)
    hipLaunchKernelGGL((tile_search_kernel<Wide, true, U>), dim3(static_cast<unsigned>(blocks)), dim3(kBlock),
                       lds_lut + lds_s1, stream, pv, bv, plan.starts, plan.n_waves, plan.long_recs, plan.keys);
  else
    hipLaunchKernelGGL((tile_search_kernel<Wide, false, U>), dim3(static_cast<unsigned>(blocks)), dim3(kBlock),
                       lds_lut, stream, pv, bv, plan.starts, plan.n_waves, plan.long_recs, plan.keys);
}

template <bool Wide>
void launch_search_u(const ProblemView& pv, const BatchView& bv, const Plan& plan, hipStream_t stream) {
  switch (plan.u) {
    case 1: launch_search_t<Wide, 1>(pv, bv, plan, stream); break;
    case 4: launch_search_t<Wide, 4>(pv, bv, plan, stream); break;
    default: launch_search_t<Wide, 2>(pv, bv, plan, stream); break;
  }
}

void launch_finalize(const ProblemView& pv, const BatchView& bv, const Plan& plan, void* out, int fmt,
                     hipStream_t stream) {
  if (plan.n_long <= 0) return;
  ProblemView p = pv;
  p.r2 = plan.r2;
  const int64_t rb = (plan.n_long + 3) / 4;
  hipLaunchKernelGGL(resolve_long_kernel, dim3(static_cast<unsigned>(rb)), dim3(256), 0, stream, p, bv, plan.long_recs,
                     plan.keys, plan.n_long, out, fmt);
}
}  // namespace

void launch_tile_keys(const ProblemView& pv, const BatchView& bv, const Plan& plan, hipStream_t stream) {
  if (pv.prof16) {  // packed-int16 profile variant (tile16_kernels.hip) when the problem fits it
    launch_tile16_keys(pv, bv, plan, stream, pv.mfma_sweep != 0);
    return;
  }
  if (plan.n_long > 0) MOC_HIP_CHECK(hipMemsetAsync(plan.keys, 0, sizeof(unsigned long long) * plan.n_long, stream));
  if (plan.n_waves <= 0) return;
  if (pv.key_shift > 0)
    launch_search_u<false>(pv, bv, plan, stream);
  else
    launch_search_u<true>(pv, bv, plan, stream);
}

void launch_finalize_keys(const ProblemView& pv, const BatchView& bv, const Plan& plan, void* out, int fmt,
                          hipStream_t stream) {
  launch_finalize(pv, bv, plan, out, fmt, stream);
}

void launch_tiles(const ProblemView& pv, const BatchView& bv, const Plan& plan, void* out, int fmt,
                  hipStream_t stream) {
  if (plan.n_long <= 0) return;
  launch_tile_keys(pv, bv, plan, stream);
  launch_finalize(pv, bv, plan, out, fmt, stream);
}

}  // namespace dev
}  // namespace moc
