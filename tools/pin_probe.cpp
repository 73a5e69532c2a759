// Page-locking costs on the box (why the streaming ring's first registrations took ~25 ms each while the
// sliced path's took ~6): hipHostRegister of prefaulted 2 MiB-page regions of several sizes, first call of
// the process vs later ones, with the GPU idle vs busy (a kernel-free busy: a long device memset), and
// hipHostMalloc of the same sizes.
// Build: hipcc -O2 -std=c++17 -fopenmp -Icsrc/include tools/pin_probe.cpp -Lmpi_openmp_cuda_amd/lib -lmoc
//        -Wl,-rpath,$PWD/mpi_openmp_cuda_amd/lib -o build/pin_probe
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstdio>
#include <vector>

#include "moc/runtime/host_region.hpp"

namespace {
double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

int main() {
  (void)hipSetDevice(0);
  void* warm = nullptr;
  (void)hipMalloc(&warm, 1 << 20);
  const size_t sizes[] = {size_t{8} << 20, size_t{32} << 20, size_t{128} << 20, size_t{512} << 20, size_t{1} << 30};
  for (int round = 0; round < 2; ++round) {
    for (size_t sz : sizes) {
      moc::HostRegion r(sz, 0);
      double t0 = now_ms();
      r.prefault();
      double t1 = now_ms();
      const hipError_t e = hipHostRegister(r.data(), sz, hipHostRegisterMapped);
      double t2 = now_ms();
      (void)hipHostUnregister(r.data());
      double t3 = now_ms();
      std::printf("round %d register %5zu MB: prefault %7.2f ms  register %7.2f ms  unregister %7.2f ms  rc=%d\n", round,
                  sz >> 20, t1 - t0, t2 - t1, t3 - t2, static_cast<int>(e));
    }
  }
  // the GPU busy: a stream of large device memsets in flight while registering
  void* big = nullptr;
  (void)hipMalloc(&big, size_t{4} << 30);
  hipStream_t s;
  (void)hipStreamCreate(&s);
  for (size_t sz : sizes) {
    for (int k = 0; k < 8; ++k) (void)hipMemsetAsync(big, k, size_t{4} << 30, s);
    moc::HostRegion r(sz, 0);
    r.prefault();
    double t1 = now_ms();
    (void)hipHostRegister(r.data(), sz, hipHostRegisterMapped);
    double t2 = now_ms();
    (void)hipStreamSynchronize(s);
    double t3 = now_ms();
    (void)hipHostUnregister(r.data());
    std::printf("busy   register %5zu MB: register %7.2f ms  (memsets drained %7.2f ms later)\n", sz >> 20, t2 - t1, t3 - t2);
  }
  for (size_t sz : sizes) {
    void* p = nullptr;
    double t1 = now_ms();
    (void)hipHostMalloc(&p, sz, hipHostMallocDefault);
    double t2 = now_ms();
    (void)hipHostFree(p);
    double t3 = now_ms();
    std::printf("hipHostMalloc %5zu MB: %7.2f ms  free %7.2f ms\n", sz >> 20, t2 - t1, t3 - t2);
  }
  return 0;
}
