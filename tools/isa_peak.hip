// Issue-rate probe for the instructions the search kernels' hot loops are made of (profiles/roofline_r5.md):
// how many wave64 instructions of each kind one SIMD completes per shader clock when W waves per SIMD issue
// independent streams of it, and the shader clock under that load.
//
//   hipcc -O3 --offload-arch=gfx950 -o build/isa_peak tools/isa_peak.hip && build/isa_peak
//
// Each wave runs `iters` rounds of 64 independent VALU instructions (8 accumulators) or 32 readlanes / LDS
// reads (conflict-free addresses, one s_waitcnt per round), timed with s_memtime
// (shader clock) per wave and with events for the wall clock; grid = 256 CUs x W blocks of 4 waves (one per
// SIMD), so every SIMD holds W waves. Prints one JSON line per (instruction, W):
//   wave_instr_per_cu_clock = all waves' instructions / (CUs x the span from the first wave's start to the last
//   wave's end in shader cycles; s_memrealtime for the span, each wave's s_memtime / s_memrealtime for the clock).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                              \
    }                                                                            \
  } while (0)

enum Op { kPkAdd, kPkMax, kSdwaAdd, kAddU32, kAddDpp, kReadlane, kDsB32, kDsB64, kDsU16, kNumOps };
static const char* kNames[] = {"v_pk_add_u16", "v_pk_max_i16", "v_add_u16_sdwa(sext byte)", "v_add_u32",
                               "v_add_u32_dpp(row_newbcast)", "v_readlane_b32", "ds_read_b32(stride 4B)",
                               "ds_read_b64(stride 8B)", "ds_read_u16(stride 4B)"};

#define R8(S) S S S S S S S S

template <int OP>
__global__ __launch_bounds__(256) void probe(uint32_t* sink, long long* cyc, int iters) {
  // cyc per wave: [shader-clock delta, real-time start, real-time end] (s_memtime, s_memrealtime at 100 MHz)
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < 4096; i += 256) reinterpret_cast<uint32_t*>(lds)[i] = i * 2654435761u;
  __syncthreads();
  uint32_t a0 = tid, a1 = tid + 1, a2 = tid + 2, a3 = tid + 3, a4 = tid + 4, a5 = tid + 5, a6 = tid + 6,
           a7 = tid + 7;
  const uint32_t b = sink[lane] | 0x01010101u;
  uint32_t s = 0;
  const uint32_t la = (tid & 63) * 4, la8 = (tid & 63) * 8;
  const long long r0 = wall_clock64(), t0 = clock64();
  for (int it = 0; it < iters; ++it) {
    if constexpr (OP == kPkAdd) {
      asm volatile(R8("v_pk_add_u16 %0, %0, %8\n v_pk_add_u16 %1, %1, %8\n v_pk_add_u16 %2, %2, %8\n v_pk_add_u16 %3, %3, %8\n"
                      "v_pk_add_u16 %4, %4, %8\n v_pk_add_u16 %5, %5, %8\n v_pk_add_u16 %6, %6, %8\n v_pk_add_u16 %7, %7, %8\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                   : "v"(b));
    } else if constexpr (OP == kPkMax) {
      asm volatile(R8("v_pk_max_i16 %0, %0, %8\n v_pk_max_i16 %1, %1, %8\n v_pk_max_i16 %2, %2, %8\n v_pk_max_i16 %3, %3, %8\n"
                      "v_pk_max_i16 %4, %4, %8\n v_pk_max_i16 %5, %5, %8\n v_pk_max_i16 %6, %6, %8\n v_pk_max_i16 %7, %7, %8\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                   : "v"(b));
    } else if constexpr (OP == kSdwaAdd) {
#define SD(R) "v_add_u16_sdwa " R ", " R ", sext(%8) dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:BYTE_0\n"
      asm volatile(R8(SD("%0") SD("%1") SD("%2") SD("%3") SD("%4") SD("%5") SD("%6") SD("%7"))
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                   : "v"(b));
#undef SD
    } else if constexpr (OP == kAddU32) {
      asm volatile(R8("v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n"
                      "v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                   : "v"(b));
    } else if constexpr (OP == kAddDpp) {
#define DP(R, K) "v_add_u32_dpp " R ", %8, " R " row_newbcast:" K " row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      asm volatile(R8(DP("%0", "0") DP("%1", "1") DP("%2", "2") DP("%3", "3") DP("%4", "4") DP("%5", "5")
                          DP("%6", "6") DP("%7", "7"))
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                   : "v"(b));
#undef DP
    } else if constexpr (OP == kReadlane) {
      uint32_t r0, r1, r2, r3;
      asm volatile(R8("v_readlane_b32 %0, %4, 1\n v_readlane_b32 %1, %4, 2\n v_readlane_b32 %2, %4, 3\n v_readlane_b32 %3, %4, 4\n")
                   : "=s"(r0), "=s"(r1), "=s"(r2), "=s"(r3)
                   : "v"(a0));
      s += r0 ^ r1 ^ r2 ^ r3;
#define DS32(X)                                                                                                 \
  X("%0", "0") X("%1", "256") X("%2", "512") X("%3", "768") X("%4", "1024") X("%5", "1280") X("%6", "1536")     \
  X("%7", "1792") X("%0", "2048") X("%1", "2304") X("%2", "2560") X("%3", "2816") X("%4", "3072") X("%5", "3328") \
  X("%6", "3584") X("%7", "3840") X("%0", "4096") X("%1", "4352") X("%2", "4608") X("%3", "4864") X("%4", "5120") \
  X("%5", "5376") X("%6", "5632") X("%7", "5888") X("%0", "6144") X("%1", "6400") X("%2", "6656") X("%3", "6912") \
  X("%4", "7168") X("%5", "7424") X("%6", "7680") X("%7", "7936") "s_waitcnt lgkmcnt(0)\n"
#define B32(R, O) "ds_read_b32 " R ", %8 offset:" O "\n"
#define U16(R, O) "ds_read_u16 " R ", %8 offset:" O "\n"
    } else if constexpr (OP == kDsB32) {
      asm volatile(DS32(B32)
                   : "=v"(a0), "=v"(a1), "=v"(a2), "=v"(a3), "=v"(a4), "=v"(a5), "=v"(a6), "=v"(a7)
                   : "v"(la));
    } else if constexpr (OP == kDsU16) {
      asm volatile(DS32(U16)
                   : "=v"(a0), "=v"(a1), "=v"(a2), "=v"(a3), "=v"(a4), "=v"(a5), "=v"(a6), "=v"(a7)
                   : "v"(la));
#undef B32
#undef U16
#undef DS32
    } else if constexpr (OP == kDsB64) {
      uint64_t d0, d1, d2, d3;
#define DQ(R, O) "ds_read_b64 " R ", %4 offset:" O "\n"
      asm volatile(DQ("%0", "0") DQ("%1", "512") DQ("%2", "1024") DQ("%3", "1536") DQ("%0", "2048") DQ("%1", "2560")
                       DQ("%2", "3072") DQ("%3", "3584") DQ("%0", "4096") DQ("%1", "4608") DQ("%2", "5120")
                           DQ("%3", "5632") DQ("%0", "6144") DQ("%1", "6656") DQ("%2", "7168") DQ("%3", "7680")
                               DQ("%0", "8192") DQ("%1", "8704") DQ("%2", "9216") DQ("%3", "9728")
                                   DQ("%0", "10240") DQ("%1", "10752") DQ("%2", "11264") DQ("%3", "11776")
                                       DQ("%0", "12288") DQ("%1", "12800") DQ("%2", "13312") DQ("%3", "13824")
                                           DQ("%0", "14336") DQ("%1", "14848") DQ("%2", "15360") DQ("%3", "0")
                                               "s_waitcnt lgkmcnt(0)\n"
                   : "=v"(d0), "=v"(d1), "=v"(d2), "=v"(d3)
                   : "v"(la8));
#undef DQ
      a0 += static_cast<uint32_t>(d0 ^ d1 ^ d2 ^ d3);
    }
  }
  const long long t1 = clock64(), r1 = wall_clock64();
  if (lane == 0) {
    long long* c = cyc + 3 * (blockIdx.x * 4 + (tid >> 6));
    c[0] = t1 - t0;
    c[1] = r0;
    c[2] = r1;
  }
  sink[64 + blockIdx.x * 256 + tid] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ s;
}

template <int OP>
void run(int cus, int w, int iters) {
  const int blocks = cus * w;
  uint32_t* sink;
  long long* cyc;
  CHECK(hipMalloc(&sink, sizeof(uint32_t) * (64 + blocks * 256)));
  CHECK(hipMemset(sink, 0, sizeof(uint32_t) * (64 + blocks * 256)));
  CHECK(hipMalloc(&cyc, sizeof(long long) * blocks * 4 * 3));
  const size_t lds = 16384 + 64;
  hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(256), lds, 0, sink, cyc, 8);  // warm-up
  CHECK(hipDeviceSynchronize());
  hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(256), lds, 0, sink, cyc, iters);
  CHECK(hipDeviceSynchronize());
  std::vector<long long> c(blocks * 4 * 3);
  CHECK(hipMemcpy(c.data(), cyc, sizeof(long long) * c.size(), hipMemcpyDeviceToHost));
  // the span every wave ran in, on the global 100 MHz clock; the shader clock from each wave's two counters
  long long rmin = c[1], rmax = c[2];
  double cyc_sum = 0, real_sum = 0;
  for (size_t w0 = 0; w0 < c.size(); w0 += 3) {
    rmin = std::min(rmin, c[w0 + 1]);
    rmax = std::max(rmax, c[w0 + 2]);
    cyc_sum += static_cast<double>(c[w0]);
    real_sum += static_cast<double>(c[w0 + 2] - c[w0 + 1]);
  }
  const double ghz = cyc_sum / real_sum * 0.1;  // shader cycles per 10 ns tick -> GHz
  const double span_cycles = static_cast<double>(rmax - rmin) * 10.0 * ghz;
  const double per_wave = (OP <= kAddDpp ? 64.0 : 32.0) * iters;  // instructions per wave: 64 VALU or 32 per round
  const double total = per_wave * blocks * 4;
  std::printf(
      "{\"instr\": \"%s\", \"waves_per_simd\": %d, \"iters\": %d, \"clock_ghz\": %.3f, \"span_us\": %.1f, "
      "\"wave_instr_per_cu_clock\": %.3f, \"simd_cycles_per_instr\": %.3f}\n",
      kNames[OP], w, iters, ghz, (rmax - rmin) * 0.01, total / (cus * span_cycles), 4.0 * cus * span_cycles / total);
  CHECK(hipFree(sink));
  CHECK(hipFree(cyc));
}

int main(int argc, char** argv) {
  int dev = 0;
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, dev));
  const int cus = p.multiProcessorCount;
  const int iters = argc > 1 ? std::atoi(argv[1]) : 4000;
  for (int w : {1, 2, 4, 8}) {
    run<kPkAdd>(cus, w, iters);
    run<kPkMax>(cus, w, iters);
    run<kSdwaAdd>(cus, w, iters);
    run<kAddU32>(cus, w, iters);
    run<kAddDpp>(cus, w, iters);
    run<kReadlane>(cus, w, iters / 4);
    run<kDsB32>(cus, w, iters / 4);
    run<kDsB64>(cus, w, iters / 4);
    run<kDsU16>(cus, w, iters / 4);
  }
  return 0;
}
