// Device selection and properties — native replacement for the CUDA-Samples device helpers
// (inc/helper_cuda.h:627-930: gpuDeviceInit, findCudaDevice, gpuGetMaxGflopsDeviceId,
// _ConvertSMVer2Cores), which the reference includes but never calls: it has no cudaSetDevice at all,
// so every rank on a node shares GPU 0 (bug B14). Here rank -> device = local_rank % device_count.
#pragma once

#include <cstdint>
#include <string>

namespace moc {

struct DeviceInfo {
  int id = -1;
  std::string name;
  std::string arch;  // gcnArchName, e.g. "gfx950:sramecc+:xnack-"
  int compute_units = 0;
  int wave_size = 0;
  int64_t global_mem = 0;
  int64_t lds_per_block = 0;
  int clock_khz = 0;
  std::string pci_bus_id;  // "dddd:bb:dd.f" (lower case), empty when unknown
  std::string json() const;
};

int device_count();  // 0 when no HIP device (or no driver) is present
DeviceInfo device_info(int id);
// Picks local_rank % count (or `requested` when >= 0), calls hipSetDevice, returns the id.
int select_device(int local_rank, int requested = -1);

// NUMA node the device's PCIe function hangs off (sysfs), or -1 when unknown.
int device_numa_node(int device);
// Binds the calling process's CPUs (sched_setaffinity) and its future page allocations
// (set_mempolicy MPOL_PREFERRED) to the device's NUMA node, so host buffers that the GPU streams
// over PCIe live next to its root complex. Returns the node, or -1 if nothing was changed.
int bind_numa_to_device(int device);

}  // namespace moc
