// Long-record search kernel, packed-int16 profile variant ("tile16"; gfx950, wave64).
//
// Same work decomposition as tile_search_kernel (align_kernels.hip: persistent waves over cost-balanced
// runs of 63*U-offset wave tiles, one lane per offset), but the per-cell work is cut from a LUT gather,
// two DPP moves and five VALU ops to ONE LDS read and THREE VALU ops, by reading a precomputed Seq1
// profile instead of shifting Seq1 letters across lanes:
//
//   profile entry (row c = Seq2 letter, column j = Seq1 position; moc::Profile16, 2 bytes)
//       low byte  S + bias,  S = T[c][Seq1[j]]
//       high byte D (int8),  D = T[c][Seq1[j]] - T[c][Seq1[j+1]]
//   per lane (offset o) and Seq2 position i:
//       e    = prof[c_i][o + i]           ds_read_u16 — lanes read consecutive halfwords: conflict-free;
//                                         the address is lane base + a wave-uniform SGPR term, and the U
//                                         sub-tiles of a wave tile sit at immediate offsets (+126 B)
//       w    = (sext D << 16) | (S+bias)  v_perm_b32
//       acc += w                          v_pk_add_u16: high half = D_o(i+1) = P_o(i+1) - P_{o+1}(i+1),
//                                         low half = P_o(i+1) + bias*(i+1) (both mod 2^16)
//       best = max(best, acc)             v_pk_max_i16: high half = running max of D over k = i+1
//   every 64 steps the int16 halves are flushed into int32 (|partial sums| <= 64*127 < 2^15, exact).
//
// Per offset this yields Tot_o, Tot_{o+1} = Tot_o - D_o(L2) and max_k D_o(k) — the best score of the
// offset, max(Tot_o [k = 0], max_k D_o(k) + Tot_{o+1}), but not WHICH k. So the sweep reduces keys
// (score, ~(2o + mutated)) — same order as the reference (score, then smallest o, then k = 0 first) —
// and a second kernel re-walks only the winning diagonal of each record (one wave, O(L2)) to find the
// smallest k with that score and write the engine's final key (score, ~(o*L2 + k)). Host replay of the
// arithmetic, ties included: csrc/tests/test_core.cpp test_profile16.
//
// Replaces calc_result (cudaFunctions.cu:63-176) for long records when the weights fit the profile
// bytes (|T| range <= 127, i.e. W1 + max(W2,W3,W4) <= 127) and the profile fits one CU's LDS
// (26*L1 + 256 halfwords <= 160 KiB: L1 <= 3140, covering the reference's 3000-letter buffers).
#include <hip/hip_runtime.h>

#include "kernel_common.hpp"
#include "moc/runtime/hip_check.hpp"

namespace moc {
namespace dev {

using namespace kc;

namespace {
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));

constexpr int kBlock16 = 1024;  // 16 waves: the profile takes most of the CU's LDS, one workgroup holds it
constexpr int kWavesPerBlock16 = kBlock16 / 64;
constexpr uint32_t kPermDS = 0x08010c00u;  // bytes: [S+bias, 0x00, D, sign(D)]

__device__ __forceinline__ uint32_t pk_add(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, a) + __builtin_bit_cast(u16x2, b));
}
__device__ __forceinline__ uint32_t pk_max(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t,
                            __builtin_elementwise_max(__builtin_bit_cast(s16x2, a), __builtin_bit_cast(s16x2, b)));
}
constexpr uint32_t kBestInit = 0x80008000u;  // both halves INT16_MIN

// Pass-1 key of an offset: (score, ~(2o + mutated)); the same packing as final_key.
__device__ __forceinline__ unsigned long long pass1_candidate(bool own, int o, int L1, int L2, int sem, int P, int Dfin,
                                                              int maxD) {
  unsigned long long key = 0;
  if (!own) return key;
  const int last = L1 - L2;
  const bool v0 = (o < last) || (o == last && (sem == static_cast<int>(Semantics::Spec) || L2 == L1));
  if (v0) key = final_key(P, 2u * static_cast<uint32_t>(o));
  if (o < last && L2 >= 2) key = max_u64(key, final_key(maxD + P - Dfin, 2u * static_cast<uint32_t>(o) + 1u));
  return key;
}
}  // namespace

template <int U>
__global__ __launch_bounds__(kBlock16) void tile16_search_kernel(ProblemView pv, BatchView bv,
                                                                 const WaveStart* __restrict__ starts, int64_t n_waves,
                                                                 const int32_t* __restrict__ long_recs,
                                                                 unsigned long long* __restrict__ keys) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  {  // stage the profile (16-byte copies; the global buffer is padded to 16 bytes)
    const uint4* src = reinterpret_cast<const uint4*>(pv.prof16);
    uint4* dst = reinterpret_cast<uint4*>(smem);
    const int n16 = pv.prof16_bytes >> 4;
    for (int t = threadIdx.x; t < n16; t += blockDim.x) dst[t] = src[t];
  }
  __syncthreads();
  const int64_t w = static_cast<int64_t>(blockIdx.x) * kWavesPerBlock16 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (w >= n_waves) return;  // wave-uniform; no barrier follows
  const int L1 = pv.L1;
  const int rowb = 2 * L1;  // bytes per profile row
  const int bias = pv.prof16_bias;
  const int lane = threadIdx.x & 63;
  constexpr int kSpan = kTileOffsets * U;

  const WaveStart ws = starts[w], we = starts[w + 1];
  int li = __builtin_amdgcn_readfirstlane(ws.li), t = __builtin_amdgcn_readfirstlane(ws.t);
  const int end_li = __builtin_amdgcn_readfirstlane(we.li), end_t = __builtin_amdgcn_readfirstlane(we.t);
  while (li < end_li || (li == end_li && t < end_t)) {  // wave-uniform
    const int r = long_recs ? __builtin_amdgcn_readfirstlane(long_recs[li]) : li;
    const uint8_t* rec = bv.codes + (bv.offsets[r] - bv.offsets[0]);
    const int L2 = __builtin_amdgcn_readfirstlane(static_cast<int>(bv.offsets[r + 1] - bv.offsets[r]));
    const int steps = L2 <= L1 ? L2 : 0;
    const int need = L2 <= L1 ? L1 - L2 + 1 : 1;
    const int ntiles = (need + kSpan - 1) / kSpan;
    const int t_stop = li == end_li ? min(end_t, ntiles) : ntiles;
    const int cv_first = lane < steps ? static_cast<int>(rec[lane]) : 0;
    unsigned long long acc64 = 0;
    for (; t < t_stop; ++t) {
      const int o0 = t * kSpan;
      MOC_DCHECK(o0 >= 0 && o0 <= L1);
      // sub-tile u: lane owns offset o0 + 63u + lane (lane 63 duplicates the next sub-tile's lane 0)
      const unsigned char* lbase = smem + 2 * (o0 + lane);
      uint32_t acc[U], best[U];
      int Dc[U], Pc[U], maxD[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        acc[u] = 0;
        best[u] = kBestInit;
        Dc[u] = 0;
        Pc[u] = 0;
        maxD[u] = INT32_MIN;
      }
      auto step = [&](int cv, int j, int i, bool key) {
        const int c = __builtin_amdgcn_readlane(cv, j);
        const int soff = __builtin_amdgcn_readfirstlane(max(c - 1, 0) * rowb + 2 * i);
        const unsigned char* p = lbase + soff;
        MOC_DCHECK(2 * (o0 + lane) + soff + 2 * kTileOffsets * (U - 1) + 2 <= pv.prof16_bytes);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t e = *reinterpret_cast<const uint16_t*>(p + 2 * kTileOffsets * u);
          acc[u] = pk_add(acc[u], __builtin_amdgcn_perm(e, e, kPermDS));
          if (key) best[u] = pk_max(best[u], acc[u]);
        }
      };
      // every 64-step chunk starts from zero halves and folds them into the int32 state at its end
      auto flush = [&](int m, bool any_key) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (any_key) maxD[u] = max(maxD[u], Dc[u] + (static_cast<int>(best[u]) >> 16));
          Dc[u] += static_cast<int>(acc[u]) >> 16;
          Pc[u] += static_cast<int16_t>(static_cast<uint16_t>((acc[u] & 0xffffu) - static_cast<uint32_t>(bias * m)));
        }
      };
      int cv = cv_first;
      int i0 = 0;
      for (; i0 + 64 < steps; i0 += 64) {  // full chunks (the record's last letter lies beyond)
        const int cv_next = i0 + 64 + lane < steps ? static_cast<int>(rec[i0 + 64 + lane]) : 0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          acc[u] = 0;
          best[u] = kBestInit;
        }
#pragma unroll 16
        for (int j = 0; j < 64; ++j) step(cv, j, i0 + j, true);
        flush(64, true);
        cv = cv_next;
      }
      if (steps > 0) {  // last chunk: 1..64 steps; no hyphen after the final letter
        const int m = steps - i0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          acc[u] = 0;
          best[u] = kBestInit;
        }
        for (int j = 0; j < m - 1; ++j) step(cv, j, i0 + j, true);
        step(cv, m - 1, i0 + m - 1, false);
        flush(m, m > 1);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int o = o0 + kTileOffsets * u + lane;
        const bool own = lane < kTileOffsets && L2 <= L1 && o <= L1 - L2;
        acc64 = max_u64(acc64, pass1_candidate(own, o, L1, L2, pv.semantics, Pc[u], Dc[u], maxD[u]));
      }
    }
    const unsigned long long k = wave_max_u64(acc64);
    if (lane == 0 && k != 0ull) atomicMax(keys + li, k);
    ++li;
    t = 0;
  }
}

// One wave per long record: pass-1 key (score, ~(2o + m)) -> final key (score, ~(o*L2 + k)). For a
// mutated winner, k is the smallest k in 1..L2-1 with P_o(k) - P_{o+1}(k) + Tot_{o+1} == score, found
// with a wave prefix scan of the diagonal differences (ballot picks the first match).
__global__ __launch_bounds__(256) void resolve16_kernel(ProblemView pv, BatchView bv,
                                                        const int32_t* __restrict__ long_recs,
                                                        unsigned long long* __restrict__ keys, int64_t n_long) {
  const int64_t li = static_cast<int64_t>(blockIdx.x) * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (li >= n_long) return;
  const int lane = threadIdx.x & 63;
  const unsigned long long key = keys[li];
  if (key == 0ull) return;
  const int score = static_cast<int>(static_cast<uint32_t>(key >> 32) ^ 0x80000000u);
  const uint32_t idx = 0xffffffffu - static_cast<uint32_t>(key);
  const int o = static_cast<int>(idx >> 1);
  const int r = long_recs ? long_recs[li] : static_cast<int>(li);
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
  if (lane == 0)
    keys[li] = final_key(score, static_cast<uint32_t>(o) * static_cast<uint32_t>(L2) + static_cast<uint32_t>(k));
}

int tile16_waves_per_cu(int prof16_bytes) {
  const int blocks = prof16_bytes > 0 ? kProf16MaxLds / prof16_bytes : 2;
  return kWavesPerBlock16 * max(1, min(2, blocks));
}

namespace {
template <int U>
void launch16_t(const ProblemView& pv, const BatchView& bv, const Plan& plan, hipStream_t stream) {
  static bool attr_set = false;  // dynamic LDS above 64 KiB must be declared once per kernel
  if (!attr_set) {
    MOC_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&tile16_search_kernel<U>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, kProf16MaxLds));
    attr_set = true;
  }
  const int64_t blocks = (plan.n_waves + kWavesPerBlock16 - 1) / kWavesPerBlock16;
  hipLaunchKernelGGL((tile16_search_kernel<U>), dim3(static_cast<unsigned>(blocks)), dim3(kBlock16),
                     static_cast<size_t>(pv.prof16_bytes), stream, pv, bv, plan.starts, plan.n_waves, plan.long_recs,
                     plan.keys);
}
}  // namespace

void launch_tile16_keys(const ProblemView& pv, const BatchView& bv, const Plan& plan, hipStream_t stream) {
  if (!pv.prof16 || pv.prof16_bytes <= 0 || pv.prof16_bytes > kProf16MaxLds || (pv.prof16_bytes & 15))
    throw Error("launch_tile16_keys: no usable profile");
  if (plan.n_long > 0) MOC_HIP_CHECK(hipMemsetAsync(plan.keys, 0, sizeof(unsigned long long) * plan.n_long, stream));
  if (plan.n_waves <= 0) return;
  switch (plan.u) {
    case 1: launch16_t<1>(pv, bv, plan, stream); break;
    case 4: launch16_t<4>(pv, bv, plan, stream); break;
    default: launch16_t<2>(pv, bv, plan, stream); break;
  }
  const int64_t rb = (plan.n_long + 3) / 4;
  hipLaunchKernelGGL(resolve16_kernel, dim3(static_cast<unsigned>(rb)), dim3(256), 0, stream, pv, bv, plan.long_recs,
                     plan.keys, plan.n_long);
}

}  // namespace dev
}  // namespace moc
