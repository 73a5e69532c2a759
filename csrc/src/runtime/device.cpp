#include "moc/runtime/device.hpp"

#include <hip/hip_runtime_api.h>

#include <sstream>

#include "moc/runtime/hip_check.hpp"

namespace moc {

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

DeviceInfo device_info(int id) {
  hipDeviceProp_t p;
  MOC_HIP_CHECK(hipGetDeviceProperties(&p, id));
  DeviceInfo d;
  d.id = id;
  d.name = p.name;
  d.arch = p.gcnArchName;
  d.compute_units = p.multiProcessorCount;
  d.wave_size = p.warpSize;
  d.global_mem = static_cast<int64_t>(p.totalGlobalMem);
  d.lds_per_block = static_cast<int64_t>(p.sharedMemPerBlock);
  d.clock_khz = p.clockRate;
  return d;
}

std::string DeviceInfo::json() const {
  std::ostringstream os;
  os << "{\"id\": " << id << ", \"name\": \"" << name << "\", \"arch\": \"" << arch << "\", \"cus\": " << compute_units
     << ", \"wave\": " << wave_size << ", \"mem_gb\": " << (global_mem / 1e9) << ", \"lds_per_block\": " << lds_per_block
     << "}";
  return os.str();
}

int select_device(int local_rank, int requested) {
  const int n = device_count();
  if (n == 0) throw Error("no HIP device available");
  const int id = requested >= 0 ? requested : (local_rank % n);
  if (id >= n) throw Error("requested device " + std::to_string(id) + " but only " + std::to_string(n) + " present");
  MOC_HIP_CHECK(hipSetDevice(id));
  return id;
}

}  // namespace moc
