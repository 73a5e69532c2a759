// GPU start-up cost breakdown of one rank (what `final`'s setup phase pays): HIP runtime init (device
// count), device context (hipSetDevice + first allocation), kernel code-object preload, the rest of the
// HipEngine constructor, NUMA binding. Build + run (GPU box):
//   hipcc -O2 -std=c++17 -Icsrc/include tools/init_probe.cpp -Lmpi_openmp_cuda_amd/lib -lmoc \
//     -Wl,-rpath,$PWD/mpi_openmp_cuda_amd/lib -o build/init_probe && build/init_probe
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstdio>

#include "moc/device.hpp"
#include "moc/hip_engine.hpp"
#include "moc/runtime/device.hpp"

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  double t = now_ms();
  auto lap = [&t](const char* what) {
    const double n = now_ms();
    std::printf("%-28s %8.1f ms\n", what, n - t);
    t = n;
  };
  int n = 0;
  (void)hipGetDeviceCount(&n);
  lap("hipGetDeviceCount");
  (void)hipSetDevice(0);
  lap("hipSetDevice");
  void* p = nullptr;
  (void)hipMalloc(&p, 256);
  lap("first hipMalloc (context)");
  moc::dev::preload_kernels(moc::dev::kPreloadAll);
  lap("preload_kernels");
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  lap("hipGetDeviceProperties");
  hipStream_t s[3];
  for (auto& x : s) (void)hipStreamCreateWithFlags(&x, hipStreamNonBlocking);
  lap("3 x hipStreamCreate");
  hipEvent_t ev[4];
  for (auto& x : ev) (void)hipEventCreate(&x);
  lap("4 x hipEventCreate");
  void* q = nullptr;
  (void)hipMalloc(&q, 8);
  lap("hipMalloc");
  (void)hipMemset(q, 0, 8);
  lap("first hipMemset");
  (void)hipMemset(q, 0, 8);
  lap("second hipMemset");
  (void)hipMemsetAsync(q, 0, 8, s[0]);
  (void)hipStreamSynchronize(s[0]);
  lap("hipMemsetAsync + sync");
  for (auto& x : s) (void)hipStreamDestroy(x);
  for (auto& x : ev) (void)hipEventDestroy(x);
  (void)hipFree(q);
  lap("destroy");
  {
    moc::EngineOptions eo;
    eo.device = 0;
    moc::HipEngine e(eo);
    lap("HipEngine ctor (warm)");
  }
  lap("HipEngine dtor");
  std::printf("numa node %d\n", moc::bind_numa_to_device(0));
  lap("bind_numa_to_device");
  (void)hipFree(p);
  return n > 0 ? 0 : 1;
}
