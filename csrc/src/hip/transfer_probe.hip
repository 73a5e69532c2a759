// Host<->device transfer calibration (used to pick the pipeline's transfer mode and to document the
// PCIe / DMA ceilings the end-to-end benchmark is bound by).
//   kind 0: H2D hipMemcpyAsync from pinned host     kind 1: D2H hipMemcpyAsync to pinned host
//   kind 2: H2D + D2H concurrently (two streams, reports the sum)
//   kind 3: zero-copy kernel read of pinned host   kind 4: zero-copy kernel write to pinned host
//   kind 5: D2D hipMemcpyAsync (HBM copy, reports read+write bytes)
//   the streaming search's mix (3 bytes in per byte out), reported as bytes IN per second:
//   kind 6: zero-copy read + zero-copy write (one third) concurrently
//   kind 7: H2D hipMemcpyAsync + zero-copy write (one third) concurrently
//   kind 8: H2D + D2H hipMemcpyAsync (one third) concurrently
//   kind 9: zero-copy read + D2H hipMemcpyAsync (one third) concurrently
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstring>

#include "moc/runtime/hip_check.hpp"

namespace moc {
namespace dev {

namespace {
__global__ void zc_read_kernel(const uint4* __restrict__ p, size_t n16, unsigned* sink) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n16;
       i += static_cast<size_t>(gridDim.x) * blockDim.x) {
    const uint4 v = p[i];
    acc.x ^= v.x;
    acc.y ^= v.y;
    acc.z ^= v.z;
    acc.w ^= v.w;
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) *sink = 1;  // keep the loads alive
}
__global__ void zc_write_kernel(uint4* __restrict__ p, size_t n16) {
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n16;
       i += static_cast<size_t>(gridDim.x) * blockDim.x)
    p[i] = make_uint4(static_cast<unsigned>(i), 1, 2, 3);
}
}  // namespace

double transfer_probe(int kind, size_t bytes, int iters) {
  void *h = nullptr, *h2 = nullptr, *d = nullptr, *d2 = nullptr;
  unsigned* sink = nullptr;
  hipStream_t s1, s2;
  MOC_HIP_CHECK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
  MOC_HIP_CHECK(hipHostMalloc(&h2, bytes, hipHostMallocDefault));
  MOC_HIP_CHECK(hipMalloc(&d, bytes));
  MOC_HIP_CHECK(hipMalloc(&d2, bytes));
  MOC_HIP_CHECK(hipMalloc(&sink, sizeof(unsigned)));
  MOC_HIP_CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  MOC_HIP_CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  std::memset(h, 1, bytes);
  const size_t n16 = bytes / 16;
  auto once = [&] {
    switch (kind) {
      case 0: MOC_HIP_CHECK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s1)); break;
      case 1: MOC_HIP_CHECK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s1)); break;
      case 2:
        MOC_HIP_CHECK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s1));
        MOC_HIP_CHECK(hipMemcpyAsync(h2, d2, bytes, hipMemcpyDeviceToHost, s2));
        break;
      case 3: hipLaunchKernelGGL(zc_read_kernel, dim3(2048), dim3(256), 0, s1, static_cast<const uint4*>(h), n16, sink); break;
      case 4: hipLaunchKernelGGL(zc_write_kernel, dim3(2048), dim3(256), 0, s1, static_cast<uint4*>(h), n16); break;
      case 6:
        hipLaunchKernelGGL(zc_read_kernel, dim3(2048), dim3(256), 0, s1, static_cast<const uint4*>(h), n16, sink);
        hipLaunchKernelGGL(zc_write_kernel, dim3(1024), dim3(256), 0, s2, static_cast<uint4*>(h2), n16 / 3);
        break;
      case 7:
        MOC_HIP_CHECK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s1));
        hipLaunchKernelGGL(zc_write_kernel, dim3(1024), dim3(256), 0, s2, static_cast<uint4*>(h2), n16 / 3);
        break;
      case 8:
        MOC_HIP_CHECK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s1));
        MOC_HIP_CHECK(hipMemcpyAsync(h2, d2, (n16 / 3) * 16, hipMemcpyDeviceToHost, s2));
        break;
      case 9:
        hipLaunchKernelGGL(zc_read_kernel, dim3(2048), dim3(256), 0, s1, static_cast<const uint4*>(h), n16, sink);
        MOC_HIP_CHECK(hipMemcpyAsync(h2, d2, (n16 / 3) * 16, hipMemcpyDeviceToHost, s2));
        break;
      default: MOC_HIP_CHECK(hipMemcpyAsync(d2, d, bytes, hipMemcpyDeviceToDevice, s1)); break;
    }
  };
  once();  // warm-up
  MOC_HIP_CHECK(hipDeviceSynchronize());
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < iters; ++i) once();
  MOC_HIP_CHECK(hipDeviceSynchronize());
  const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  const double moved = static_cast<double>(bytes) * iters * ((kind == 2 || kind == 5) ? 2.0 : 1.0);
  (void)hipStreamDestroy(s1);
  (void)hipStreamDestroy(s2);
  (void)hipFree(sink);
  (void)hipFree(d);
  (void)hipFree(d2);
  (void)hipHostFree(h);
  (void)hipHostFree(h2);
  return moved / sec / 1e9;
}

}  // namespace dev
}  // namespace moc
