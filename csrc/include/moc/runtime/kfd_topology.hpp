// The GPUs this process can open, read from the amdgpu kernel driver's topology in sysfs, without starting
// the HIP runtime. The runtime's start-up (hipGetDeviceCount) costs 140-220 ms on the MI355X box
// (profiles/hip_init_variants_box.log); `final` needs only "how many GPUs, and which NUMA node is mine"
// to pick its engine, wire formats and device, so a GPU rank decides from here and lets the runtime start
// on a helper thread behind the parse and the encode (csrc/apps/final_gpu.cpp).
//
// A GPU is a topology node (/sys/class/kfd/kfd/topology/nodes/N/properties) with simd_count > 0 whose
// render node /dev/dri/renderD<drm_render_minor> this process may open — the runtime's own filter (a box
// exposes 1 of its host's 8 GPUs that way). Devices are listed in node order, the runtime's device order,
// then re-mapped the way the runtime does by ROCR_VISIBLE_DEVICES and HIP_VISIBLE_DEVICES (or
// CUDA_VISIBLE_DEVICES / GPU_DEVICE_ORDINAL) index lists (the box sets both to "0"). kfd_gpus() answers
// nullopt when only the runtime can tell — UUID lists, indices out of range, an unreadable topology.
#pragma once

#include <cstdint>
#include <optional>
#include <string>
#include <vector>

namespace moc {

struct KfdGpu {
  int node = -1;           // KFD topology node id
  int render_minor = -1;   // /dev/dri/renderD<minor>
  std::string pci_bus_id;  // "dddd:bb:dd.f" (lower case), from the node's domain + location_id
  int numa_node = -1;      // NUMA node of its PCIe function (/sys/bus/pci/devices/<id>/numa_node), -1 unknown
  uint64_t unique_id = 0;  // the driver's unique id (0 unknown): the runtime's UUID is "GPU-" + its 16 hex digits
};

// "GPU-<16 hex digits>" for a GPU with a unique id (the form ROCR_VISIBLE_DEVICES accepts besides indices),
// "" without one.
std::string kfd_uuid(const KfdGpu& g);

struct KfdPaths {
  std::string nodes = "/sys/class/kfd/kfd/topology/nodes";
  std::string kfd = "/dev/kfd";
  std::string dri = "/dev/dri";
  std::string pci = "/sys/bus/pci/devices";
  bool honour_visible_env = true;  // tests point the paths at a fake tree and switch this off
};

std::optional<std::vector<KfdGpu>> kfd_gpus(const KfdPaths& paths = KfdPaths());

// The device a rank takes from that list: `requested` (--device, or the --device-map entry) when >= 0, else
// node-local rank % device count — the runtime's select_device rule. -1 when the list cannot answer (no
// GPUs, an index out of range, a GPU without a PCIe address to find it again in the runtime by).
int kfd_pick(const std::vector<KfdGpu>& gpus, int local_rank, int requested);

// Per-rank GPU isolation: the index, among the GPUs the driver gives this process (`all`: node order, no
// visibility lists applied), of the GPU that node-local rank `local_rank` takes from `visible` (the list
// after them, kfd_gpus()) — the ROCR_VISIBLE_DEVICES value that leaves the runtime that one GPU. -1 when
// `visible` is empty or its GPU is not in `all`.
int kfd_isolation_index(const std::vector<KfdGpu>& all, const std::vector<KfdGpu>& visible, int local_rank);

// Binds the calling thread's CPUs (sched_setaffinity) and its future page allocations (set_mempolicy
// MPOL_PREFERRED) to NUMA node `node`. Returns the node, or -1 if nothing was changed.
int bind_numa_node(int node);

}  // namespace moc
