#include "moc/runtime/device.hpp"

#include <hip/hip_runtime_api.h>

#include <cctype>
#include <fstream>
#include <sstream>

#include "moc/runtime/hip_check.hpp"
#include "moc/runtime/kfd_topology.hpp"

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
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof bus, id) == hipSuccess) {
    d.pci_bus_id = bus;
    for (auto& c : d.pci_bus_id) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  } else {
    (void)hipGetLastError();
  }
  return d;
}

std::string DeviceInfo::json() const {
  std::ostringstream os;
  os << "{\"id\": " << id << ", \"name\": \"" << name << "\", \"arch\": \"" << arch << "\", \"cus\": " << compute_units
     << ", \"wave\": " << wave_size << ", \"mem_gb\": " << (global_mem / 1e9) << ", \"lds_per_block\": " << lds_per_block
     << ", \"pci_bus_id\": \"" << pci_bus_id << "\"}";
  return os.str();
}

int device_numa_node(int device) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof bus, device) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  std::string id(bus);
  for (auto& c : id) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  std::ifstream f("/sys/bus/pci/devices/" + id + "/numa_node");
  int node = -1;
  if (!(f >> node)) return -1;
  return node;
}

int bind_numa_to_device(int device) { return bind_numa_node(device_numa_node(device)); }

int select_device(int local_rank, int requested) {
  const int n = device_count();
  if (n == 0) throw Error("no HIP device available");
  const int id = requested >= 0 ? requested : (local_rank % n);
  if (id >= n) throw Error("requested device " + std::to_string(id) + " but only " + std::to_string(n) + " present");
  MOC_HIP_CHECK(hipSetDevice(id));
  return id;
}

}  // namespace moc
