// Long-record search sweep on the matrix cores ("tile-mfma"; gfx950 v_mfma_i32_32x32x32_i8), the measured
// MFMA variant of tile16_search_kernel (SURVEY.md §7.3 formulation (b); docs/MFMA_ANALYSIS.md). Selected
// with MOC_MFMA=1 in place of the tile16 sweep; plan, pass-1 keys and resolve_long_kernel are shared.
//
// Per record, wave tile of 128*U offsets and chunk of 32 steps i0 .. i0+31, the running differences
//     D_o(k) = sum_{i<k} Dt[c_i][o + i]      (Dt: the int8 difference profile in LDS, tile16's image)
// advance by a prefix sum over the chunk, which is a product with a lower-triangular ones matrix:
//     C[t][o] = sum_s L[t][s] * X[s][o],   L[t][s] = (s <= t),   X[s][o] = Dt[c_{i0+s}][o + i0 + s]
// so C[t][o] = D_o(i0 + t + 1) - D_o(i0): one i8 MFMA (M = t, N = o, K = s; 32 x 32 x 32) per 32 offsets
// replaces the 32 dependent adds per offset of the VALU kernels. A = L is a constant fragment, B = X is
// gathered per lane from LDS (16 bytes: its offset, 16 steps), C comes back with the offset on the lane
// and 16 of the 32 prefix lengths in its registers (the other 16 in lane ^ 32), so the running maximum
// over k is 15 v_max_i32 + one cross-half max per 32 cells, and the chunk total (row 31) carries on.
// Exactness: |X| <= 127 (i8), |C| <= 32 * 127: int32 throughout.
//
// Cost per 1024 cells and wave: 16 ds_read_u8 + 4 dword packs (B gather), 1 MFMA, ~22 VALU (max, carry,
// masking) — against tile16's 8 ds_read_u16 + 24 packed-int16 VALU. Measured: profiles/mfma_ab.log.
#include <hip/hip_runtime.h>

#include <mutex>
#include <set>

#include "kernel_common.hpp"
#include "moc/common.hpp"
#include "moc/runtime/hip_check.hpp"

namespace moc {
namespace dev {

using namespace kc;

namespace {
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int kBlockM = 1024;  // 16 waves; the profile image takes most of the CU's LDS (as tile16)
constexpr int kWavesPerBlockM = kBlockM / 64;
constexpr int kSubM = 128;  // offsets per sub-tile: the tile16 plan's unit (4 MFMA column blocks)

// C/D row of accumulator register `reg` on a lane of half h (gfx950 32x32 layout; column = lane & 31)
__device__ __forceinline__ constexpr int c_row(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }

// Fragment element j of lane half h <-> logical k = 16h + j (byte j of the 4 dwords). The contraction
// pairs element j of A's lane (m, h) with element j of B's lane (n, h), so any k labelling works as long as
// A and B use the same one: mfma_i8_probe_kernel checks that on the hardware (tests/test_gpu.py).
__device__ __forceinline__ int frag_k(int h, int j) { return 16 * h + j; }

__device__ __forceinline__ unsigned long long pass1_key(int o, int L1, int L2, int sem, int tot, int tot_next,
                                                        int maxD) {
  unsigned long long key = 0;
  const int last = L1 - L2;
  if (L2 > L1 || o > last) return key;
  const bool v0 = (o < last) || (sem == static_cast<int>(Semantics::Spec) || L2 == L1);
  if (v0) key = final_key(tot, 2u * static_cast<uint32_t>(o));
  if (o < last && L2 >= 2) key = max_u64(key, final_key(maxD + tot_next, 2u * static_cast<uint32_t>(o) + 1u));
  return key;
}
}  // namespace

// Self-test of the i8 operand packing + C layout: C = A * B for row-major 32x32 int8 A, B.
__global__ void mfma_i8_probe_kernel(const int8_t* __restrict__ A, const int8_t* __restrict__ B, int* __restrict__ C) {
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  v4i a, b;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t wa = 0, wb = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = frag_k(h, 4 * q + e);
      wa |= static_cast<uint32_t>(static_cast<uint8_t>(A[r * 32 + k])) << (8 * e);
      wb |= static_cast<uint32_t>(static_cast<uint8_t>(B[k * 32 + r])) << (8 * e);
    }
    a[q] = static_cast<int>(wa);
    b[q] = static_cast<int>(wb);
  }
  v16i c = {0};
  c = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) C[c_row(reg, h) * 32 + r] = c[reg];
}

template <int U>
__global__ __launch_bounds__(kBlockM) void tile_mfma_search_kernel(ProblemView pv, BatchView bv,
                                                                   const WaveStart* __restrict__ starts, int64_t n_waves,
                                                                   const int32_t* __restrict__ long_recs,
                                                                   unsigned long long* __restrict__ keys) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int8_t* lut8 = reinterpret_cast<int8_t*>(smem + pv.prof16_bytes);
  uint8_t* s1l = smem + pv.prof16_bytes + kProf16Lut8;
  {
    const uint4* src = reinterpret_cast<const uint4*>(pv.prof16);
    uint4* dst = reinterpret_cast<uint4*>(smem);
    const int n16 = pv.prof16_bytes >> 4;
    for (int t = threadIdx.x; t < n16; t += blockDim.x) dst[t] = src[t];
    for (int t = threadIdx.x; t < kProf16Lut8; t += blockDim.x) lut8[t] = static_cast<int8_t>(pv.lut[t]);
    stage_bytes(s1l, pv.seq1, pv.L1 + 16);
  }
  __syncthreads();
  const int64_t w = static_cast<int64_t>(blockIdx.x) * kWavesPerBlockM + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (w >= n_waves) return;
  const int L1 = pv.L1;
  const int rowb = 2 * L1;
  const int lane = threadIdx.x & 63, n = lane & 31, h = lane >> 5;
  constexpr int kSpan = kSubM * U;
  constexpr int kBlocks = kSpan / 32;  // MFMA column blocks per wave tile

  // A = L: element j of lane (t = n, h) is 1 when its step s = frag_k(h, j) <= t
  v4i lower;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t wv = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) wv |= (frag_k(h, 4 * q + e) <= n ? 1u : 0u) << (8 * e);
    lower[q] = static_cast<int>(wv);
  }

  const WaveStart ws = starts[w], we = starts[w + 1];
  int li = __builtin_amdgcn_readfirstlane(ws.li), t = __builtin_amdgcn_readfirstlane(ws.t);
  const int end_li = __builtin_amdgcn_readfirstlane(we.li), end_t = __builtin_amdgcn_readfirstlane(we.t);
  while (li < end_li || (li == end_li && t < end_t)) {
    const int r = long_recs ? __builtin_amdgcn_readfirstlane(long_recs[li]) : li;
    const uint8_t* rec = bv.codes + (bv.offsets[r] - bv.offsets[0]);
    const int L2 = __builtin_amdgcn_readfirstlane(static_cast<int>(bv.offsets[r + 1] - bv.offsets[r]));
    const int steps = L2 <= L1 ? L2 : 0;
    const int need = L2 <= L1 ? L1 - L2 + 1 : 1;
    const int ntiles = (need + kSpan - 1) / kSpan;
    const int t_stop = li == end_li ? min(end_t, ntiles) : ntiles;
    unsigned long long acc64 = 0;
    for (; t < t_stop && L2 <= L1; ++t) {
      const int o0 = t * kSpan;
      int Dc[kBlocks], mx[kBlocks];  // per column block: D_o(i0) and max_k D_o(k) of this lane's offset
#pragma unroll
      for (int v = 0; v < kBlocks; ++v) {
        Dc[v] = 0;
        mx[v] = INT32_MIN;
      }
      const int oA = min(o0 + kSpan, need);
      int anchor = 0;
      for (int i0 = 0; i0 < steps; i0 += 32) {
        // lane q < 32 holds step i0 + q's letter (0 past the record) and its profile row offset
        const int ci = n < steps - i0 ? static_cast<int>(rec[i0 + n]) : 0;
        const int so = ci != 0 ? (ci - 1) * rowb + 2 * (i0 + n) : -1;  // -1: padding, contributes 0
        if (h == 0 && ci != 0) anchor += lut8[ci * kLutStride + s1l[oA + i0 + n]];
        // this lane's 16 steps (frag_k(h, j) = 16h + j): the row offsets of lanes j and 16 + j, by half
        int sro[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int r0 = __builtin_amdgcn_readlane(so, j), r1 = __builtin_amdgcn_readlane(so, 16 + j);
          sro[j] = h ? r1 : r0;
        }
        const int kmax = min(31, L2 - 2 - i0);  // rows t with k = i0 + t + 1 <= L2 - 1 count for the max
#pragma unroll
        for (int v = 0; v < kBlocks; ++v) {
          const unsigned char* base = smem + 2 * (o0 + 32 * v + n);
          v4i xb;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            uint32_t wv = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int j = 4 * q + e;
              const uint32_t byte = sro[j] >= 0 ? base[sro[j]] : 0u;  // low byte of entry o + i0 + s
              wv |= byte << (8 * e);
            }
            xb[q] = static_cast<int>(wv);
          }
          v16i c = {0};
          c = __builtin_amdgcn_mfma_i32_32x32x32_i8(lower, xb, c, 0, 0, 0);
          int m = INT32_MIN;
          if (kmax >= 31) {  // wave-uniform: every prefix of a full chunk is a candidate k
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) m = max(m, c[reg]);
          } else {
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) m = max(m, c_row(reg, h) <= kmax ? c[reg] : INT32_MIN);
          }
          m = max(m, __shfl_xor(m, 32, 64));
          const int total = __shfl(c[15], n + 32, 64);  // row 31 (t = 31) lives in register 15 of half 1
          if (kmax >= 0) mx[v] = max(mx[v], Dc[v] + m);
          Dc[v] += total;
        }
      }
      // ---- Tot per offset: anchor diagonal oA, then suffix sums of D_o(L2) over the tile's offsets
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) anchor += __shfl_xor(anchor, d, 64);
      int carry = anchor;  // Tot just past the column block being processed
#pragma unroll
      for (int v = kBlocks - 1; v >= 0; --v) {
        const int o = o0 + 32 * v + n;
        const int d = o < oA ? Dc[v] : 0;
        // inclusive suffix sum over the 32 offsets of the block (lanes n .. 31 of this half)
        int suf = d;
#pragma unroll
        for (int s = 1; s < 32; s <<= 1) {
          const int x = __shfl_down(suf, s, 32);
          if (n + s < 32) suf += x;
        }
        const int tot = carry + suf;       // Tot_o
        const int tot_next = tot - d;      // Tot_{o+1}
        if (h == 0) acc64 = max_u64(acc64, pass1_key(o, L1, L2, pv.semantics, tot, tot_next, mx[v]));
        carry += __shfl(suf, 0, 32);
      }
    }
    const unsigned long long k = wave_max_u64(acc64);
    if (lane == 0 && k != 0ull) atomicMax(keys + li, k);
    ++li;
    t = 0;
  }
}

namespace {
template <int U>
void launch_mfma_t(const ProblemView& pv, const BatchView& bv, const Plan& plan, hipStream_t stream) {
  static std::mutex mu;
  static std::set<int> declared;
  int dev = 0;
  MOC_HIP_CHECK(hipGetDevice(&dev));
  {
    std::lock_guard<std::mutex> lock(mu);
    if (declared.insert(dev).second)
      MOC_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&tile_mfma_search_kernel<U>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, kProf16MaxLds));
  }
  const int64_t blocks = (plan.n_waves + kWavesPerBlockM - 1) / kWavesPerBlockM;
  hipLaunchKernelGGL((tile_mfma_search_kernel<U>), dim3(static_cast<unsigned>(blocks)), dim3(kBlockM),
                     static_cast<size_t>(tile16_lds_bytes(pv.prof16_bytes, pv.L1)), stream, pv, bv, plan.starts,
                     plan.n_waves, plan.long_recs, plan.keys);
}
}  // namespace

void preload_mfma_kernels() {
  hipFuncAttributes fa;
  (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&mfma_i8_probe_kernel));
}

void launch_mfma_i8_probe(const int8_t* d_a, const int8_t* d_b, int* d_c, hipStream_t stream) {
  hipLaunchKernelGGL(mfma_i8_probe_kernel, dim3(1), dim3(64), 0, stream, d_a, d_b, d_c);
}

void launch_tile_mfma_sweep(const ProblemView& pv, const BatchView& bv, const Plan& plan, hipStream_t stream) {
  switch (plan.u) {  // the host caps U at 2 for this sweep (register budget of 16-wave blocks)
    case 1: launch_mfma_t<1>(pv, bv, plan, stream); break;
    case 2: launch_mfma_t<2>(pv, bv, plan, stream); break;
    case 4: launch_mfma_t<4>(pv, bv, plan, stream); break;
    default: throw Error("tile-mfma sweep: sub-tiles per wave tile must be 1, 2 or 4");
  }
}

}  // namespace dev
}  // namespace moc
