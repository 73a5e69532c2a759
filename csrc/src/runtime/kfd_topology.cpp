#include "moc/runtime/kfd_topology.hpp"

#include <dirent.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>

namespace moc {

namespace {

// "name value" lines of a topology node's properties file
bool read_properties(const std::string& path, int64_t& simd, int64_t& minor, int64_t& domain, int64_t& location) {
  std::ifstream f(path);
  if (!f) return false;
  std::string key;
  int64_t v = 0;
  simd = 0;
  minor = domain = location = -1;
  while (f >> key >> v) {
    if (key == "simd_count") simd = v;
    else if (key == "drm_render_minor") minor = v;
    else if (key == "domain") domain = v;
    else if (key == "location_id") location = v;
  }
  return true;
}

// "i,j,k" -> indices; nullopt for anything else (GPU UUIDs, empty lists: the runtime's to interpret)
std::optional<std::vector<int>> index_list(const char* v) {
  std::vector<int> out;
  std::stringstream ss(v);
  std::string tok;
  while (std::getline(ss, tok, ',')) {
    if (tok.empty() || tok.find_first_not_of("0123456789") != std::string::npos || tok.size() > 6) return std::nullopt;
    out.push_back(std::stoi(tok));
  }
  if (out.empty()) return std::nullopt;
  return out;
}

// The runtime's re-mapping by index lists: ROCR_VISIBLE_DEVICES picks from the GPUs the driver gives this
// process, then HIP_VISIBLE_DEVICES (or CUDA_VISIBLE_DEVICES, GPU_DEVICE_ORDINAL) from those — each list
// in its own order. Anything else (UUIDs, out-of-range or repeated indices, disagreeing HIP/CUDA lists)
// is left to the runtime: nullopt.
std::optional<std::vector<KfdGpu>> apply_visible_env(std::vector<KfdGpu> gpus) {
  auto pick = [&gpus](const char* var) -> bool {
    const char* v = std::getenv(var);
    if (!v) return true;
    const auto idx = index_list(v);
    if (!idx) return false;
    std::vector<KfdGpu> next;
    std::vector<bool> used(gpus.size(), false);
    for (int i : *idx) {
      if (i >= static_cast<int>(gpus.size()) || used[static_cast<size_t>(i)]) return false;
      used[static_cast<size_t>(i)] = true;
      next.push_back(gpus[static_cast<size_t>(i)]);
    }
    gpus.swap(next);
    return true;
  };
  if (!pick("ROCR_VISIBLE_DEVICES")) return std::nullopt;
  const char* hip_list = nullptr;
  for (const char* var : {"HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "GPU_DEVICE_ORDINAL"}) {
    const char* v = std::getenv(var);
    if (!v) continue;
    if (hip_list && std::string(hip_list) != v) return std::nullopt;
    hip_list = v;
  }
  if (hip_list) {
    if (std::getenv("HIP_VISIBLE_DEVICES")) {
      if (!pick("HIP_VISIBLE_DEVICES")) return std::nullopt;
    } else if (std::getenv("CUDA_VISIBLE_DEVICES")) {
      if (!pick("CUDA_VISIBLE_DEVICES")) return std::nullopt;
    } else if (!pick("GPU_DEVICE_ORDINAL")) {
      return std::nullopt;
    }
  }
  return gpus;
}

}  // namespace

std::optional<std::vector<KfdGpu>> kfd_gpus(const KfdPaths& paths) {
  DIR* d = opendir(paths.nodes.c_str());
  if (!d) return std::nullopt;
  std::vector<int> ids;
  while (const dirent* e = readdir(d)) {
    char* end = nullptr;
    const long id = std::strtol(e->d_name, &end, 10);
    if (end != e->d_name && *end == '\0') ids.push_back(static_cast<int>(id));
  }
  closedir(d);
  std::sort(ids.begin(), ids.end());
  std::vector<KfdGpu> gpus;
  if (access(paths.kfd.c_str(), R_OK | W_OK) != 0) return gpus;  // no driver access: the runtime sees none
  for (int id : ids) {
    int64_t simd = 0, minor = -1, domain = -1, location = -1;
    if (!read_properties(paths.nodes + "/" + std::to_string(id) + "/properties", simd, minor, domain, location))
      return std::nullopt;  // a node that cannot be read: leave the answer to the runtime
    if (simd <= 0) continue;  // a CPU node
    if (minor < 0) return std::nullopt;
    const std::string render = paths.dri + "/renderD" + std::to_string(minor);
    if (access(render.c_str(), R_OK | W_OK) != 0) continue;  // another tenant's GPU
    KfdGpu g;
    g.node = id;
    g.render_minor = static_cast<int>(minor);
    if (domain >= 0 && location >= 0) {
      char bus[32];
      std::snprintf(bus, sizeof bus, "%04x:%02x:%02x.%x", static_cast<unsigned>(domain),
                    static_cast<unsigned>((location >> 8) & 0xff), static_cast<unsigned>((location >> 3) & 0x1f),
                    static_cast<unsigned>(location & 7));
      g.pci_bus_id = bus;
      std::ifstream nf(paths.pci + "/" + g.pci_bus_id + "/numa_node");
      int node = -1;
      if (nf >> node) g.numa_node = node;
    }
    gpus.push_back(std::move(g));
  }
  if (!paths.honour_visible_env) return gpus;
  return apply_visible_env(std::move(gpus));
}

int kfd_pick(const std::vector<KfdGpu>& gpus, int local_rank, int requested) {
  const int n = static_cast<int>(gpus.size());
  if (n == 0) return -1;
  const int id = requested >= 0 ? requested : local_rank % n;
  if (id >= n || gpus[static_cast<size_t>(id)].pci_bus_id.empty()) return -1;
  return id;
}

int kfd_isolation_index(const std::vector<KfdGpu>& all, const std::vector<KfdGpu>& visible, int local_rank) {
  if (visible.empty() || local_rank < 0) return -1;
  const KfdGpu& g = visible[static_cast<size_t>(local_rank) % visible.size()];
  for (size_t i = 0; i < all.size(); ++i)
    if (all[i].node == g.node) return static_cast<int>(i);
  return -1;
}

int bind_numa_node(int node) {
  if (node < 0) return -1;
  std::ifstream f("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist");
  std::string list;
  if (!(f >> list)) return -1;
  cpu_set_t set;
  CPU_ZERO(&set);
  int ncpu = 0;
  std::stringstream ss(list);
  std::string part;
  while (std::getline(ss, part, ',')) {
    const auto dash = part.find('-');
    const int a = std::stoi(part.substr(0, dash));
    const int b = dash == std::string::npos ? a : std::stoi(part.substr(dash + 1));
    for (int c = a; c <= b && c < CPU_SETSIZE; ++c) {
      CPU_SET(c, &set);
      ++ncpu;
    }
  }
  if (ncpu == 0) return -1;
  if (sched_setaffinity(0, sizeof set, &set) != 0) return -1;
  unsigned long mask[16] = {0};
  if (node >= static_cast<int>(sizeof(mask) * 8)) return node;
  mask[node / (8 * sizeof(unsigned long))] |= 1ul << (node % (8 * sizeof(unsigned long)));
  constexpr int kMpolPreferred = 1;
  syscall(SYS_set_mempolicy, kMpolPreferred, mask, sizeof(mask) * 8);  // best effort
  return node;
}

}  // namespace moc
