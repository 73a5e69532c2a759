// Headline-shaped host<->device traffic through the copy engines: IN bytes (letters + lengths) copied H2D
// in K chunks on one stream, OUT bytes (results) copied D2H in K chunks on another, chunk k's D2H ordered
// after chunk k's H2D (standing in for the search kernel, which reads HBM in ~0.1 ms per chunk). Reports
// the wall time of the whole pipeline against the zero-copy streaming kernel's step (~3.62 ms for 184 MB
// in + 67 MB out). Build + run (GPU box):
//   hipcc -O2 -std=c++17 tools/dma_pipeline_probe.cpp -o build/dma_pipeline_probe && build/dma_pipeline_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

int main(int argc, char** argv) {
  const size_t in_bytes = (argc > 1 ? std::atoll(argv[1]) : 184) << 20;
  const size_t out_bytes = (argc > 2 ? std::atoll(argv[2]) : 67) << 20;
  void *h_in, *h_out, *d_in, *d_out;
  CK(hipHostMalloc(&h_in, in_bytes, hipHostMallocDefault));
  CK(hipHostMalloc(&h_out, out_bytes, hipHostMallocDefault));
  CK(hipMalloc(&d_in, in_bytes));
  CK(hipMalloc(&d_out, out_bytes));
  hipStream_t s_in, s_out;
  CK(hipStreamCreateWithFlags(&s_in, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s_out, hipStreamNonBlocking));
  for (int K : {1, 2, 4, 8, 16, 32}) {
    std::vector<hipEvent_t> ev(static_cast<size_t>(K));
    for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    double best = 1e9;
    for (int rep = 0; rep < 6; ++rep) {
      CK(hipDeviceSynchronize());
      const auto t0 = std::chrono::steady_clock::now();
      for (int k = 0; k < K; ++k) {
        const size_t ib = in_bytes * k / K, ie = in_bytes * (k + 1) / K;
        const size_t ob = out_bytes * k / K, oe = out_bytes * (k + 1) / K;
        CK(hipMemcpyAsync(static_cast<char*>(d_in) + ib, static_cast<char*>(h_in) + ib, ie - ib,
                          hipMemcpyHostToDevice, s_in));
        CK(hipEventRecord(ev[k], s_in));
        CK(hipStreamWaitEvent(s_out, ev[k], 0));
        CK(hipMemcpyAsync(static_cast<char*>(h_out) + ob, static_cast<char*>(d_out) + ob, oe - ob,
                          hipMemcpyDeviceToHost, s_out));
      }
      CK(hipStreamSynchronize(s_in));
      CK(hipStreamSynchronize(s_out));
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if (rep > 0 && ms < best) best = ms;
    }
    std::printf("chunks=%2d in=%zu MB out=%zu MB: %.3f ms  (%.1f GB/s in)\n", K, in_bytes >> 20, out_bytes >> 20, best,
                in_bytes / 1e6 / best);
    for (auto& e : ev) CK(hipEventDestroy(e));
  }
  return 0;
}
