// Copies between page-locked host memory and the device on a kernel of our own, for small transfers. The
// runtime hands host->device copies of about 64 KiB and more to an SDMA engine, and the first use of that
// engine in a process costs 11-34 ms on the MI355X box (profiles/copy_path_probe.log) — more than a whole
// tiny job's search. A kernel reading (or writing) the host pages in place over PCIe costs ~0.3 ms the first
// time (this file's code object loading) and microseconds after. Large transfers keep the copy engines.
#include "moc/device.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

namespace moc {
namespace dev {

namespace {
constexpr int kCopyBlock = 256;

__global__ __launch_bounds__(kCopyBlock) void copy16_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                            int64_t n) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    dst[i] = src[i];
}

__global__ __launch_bounds__(kCopyBlock) void copy1_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                           int64_t n) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    dst[i] = src[i];
}

// One wave that idles until the device's constant-rate wall clock has advanced `ticks` (the comm-timeout
// test hook, moc/device_comm.hpp inject_stall): bounded by construction, it stores nothing.
__global__ __launch_bounds__(64) void spin_kernel(uint64_t ticks) {
  const uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

dim3 copy_grid(int64_t n) { return dim3(static_cast<unsigned>(std::clamp<int64_t>((n + kCopyBlock - 1) / kCopyBlock, 1, 2048))); }
}  // namespace

void launch_copy(void* dst, const void* src, size_t bytes, hipStream_t stream) {
  if (!bytes) return;
  const auto a = reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src);
  size_t done = 0;
  if ((a & 15) == 0 && bytes >= 16) {
    const int64_t n16 = static_cast<int64_t>(bytes / 16);
    hipLaunchKernelGGL(copy16_kernel, copy_grid(n16), dim3(kCopyBlock), 0, stream, static_cast<const uint4*>(src),
                       static_cast<uint4*>(dst), n16);
    done = static_cast<size_t>(n16) * 16;
  }
  if (done < bytes) {
    const int64_t n = static_cast<int64_t>(bytes - done);
    hipLaunchKernelGGL(copy1_kernel, copy_grid(n), dim3(kCopyBlock), 0, stream,
                       static_cast<const uint8_t*>(src) + done, static_cast<uint8_t*>(dst) + done, n);
  }
}

void launch_spin(double seconds, hipStream_t stream) {
  seconds = std::clamp(seconds, 0.0, 10.0);  // a test hook never holds the GPU for long
  int device = 0, khz = 0;
  if (hipGetDevice(&device) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) != hipSuccess ||
      khz <= 0)
    khz = 100000;  // the MI355X's 100 MHz constant clock
  const auto ticks = static_cast<uint64_t>(seconds * 1e3 * khz);
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, stream, ticks);
}

bool kernel_copy_fits(const void* dst, const void* src, size_t bytes) {
  const auto a = reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src);
  // 16-byte aligned pairs move whole uint4s; others a byte per lane, kept to small sizes
  return bytes <= ((a & 15) == 0 ? kKernelCopyMaxAligned : kKernelCopyMaxBytes);
}

}  // namespace dev
}  // namespace moc
