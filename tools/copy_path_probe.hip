// Which copy path the HIP runtime takes for a host->device hipMemcpyAsync from page-locked memory, and what its
// first use costs inside a short process: runtime up, one stream, then the first copy of SIZE bytes
// (timed to completion), a second copy of the same size, and a first device->host copy of SIZE. Run once
// per size in a fresh process (the first use of a copy engine is the cost being measured), with and without
// HSA_ENABLE_SDMA=0 (copies on blit kernels only). A small copy kernel of our own is timed as well.
//   build/copy_path_probe <bytes>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      std::exit(1);                                                              \
    }                                                                            \
  } while (0)

__global__ void copy_words(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n) {
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += size_t{gridDim.x} * blockDim.x) dst[i] = src[i];
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const size_t bytes = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 65536;
  const double t0 = now_ms();
  int n = 0;
  CHECK(hipGetDeviceCount(&n));
  const double t_rt = now_ms();
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const double t_q = now_ms();
  void *h = nullptr, *d = nullptr, *d2 = nullptr;
  CHECK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
  CHECK(hipMalloc(&d, bytes));
  CHECK(hipMalloc(&d2, bytes));
  std::memset(h, 1, bytes);
  const double t_alloc = now_ms();
  CHECK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s));
  CHECK(hipStreamSynchronize(s));
  const double t_c1 = now_ms();
  CHECK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s));
  CHECK(hipStreamSynchronize(s));
  const double t_c2 = now_ms();
  CHECK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s));
  CHECK(hipStreamSynchronize(s));
  const double t_d1 = now_ms();
  // the same upload as a kernel reading the page-locked buffer in place (zero-copy)
  void* hd = nullptr;
  CHECK(hipHostGetDevicePointer(&hd, h, 0));
  const size_t words = bytes / 16;
  hipLaunchKernelGGL(copy_words, dim3(static_cast<unsigned>(std::min<size_t>((words + 255) / 256, 1024))), dim3(256), 0, s,
                     static_cast<const uint4*>(hd), static_cast<uint4*>(d2), words);
  CHECK(hipStreamSynchronize(s));
  const double t_k1 = now_ms();
  hipLaunchKernelGGL(copy_words, dim3(static_cast<unsigned>(std::min<size_t>((words + 255) / 256, 1024))), dim3(256), 0, s,
                     static_cast<const uint4*>(hd), static_cast<uint4*>(d2), words);
  CHECK(hipStreamSynchronize(s));
  const double t_k2 = now_ms();
  const char* sdma = std::getenv("HSA_ENABLE_SDMA");
  std::printf("{\"bytes\": %zu, \"HSA_ENABLE_SDMA\": \"%s\", \"runtime_ms\": %.2f, \"stream_ms\": %.2f, \"alloc_ms\": %.2f, "
              "\"h2d_first_ms\": %.3f, \"h2d_second_ms\": %.3f, \"d2h_first_ms\": %.3f, \"kernel_copy_first_ms\": %.3f, "
              "\"kernel_copy_second_ms\": %.3f}\n",
              bytes, sdma ? sdma : "unset", t_rt - t0, t_q - t_rt, t_alloc - t_q, t_c1 - t_alloc, t_c2 - t_c1, t_d1 - t_c2,
              t_k1 - t_d1, t_k2 - t_k1);
  return 0;
}
