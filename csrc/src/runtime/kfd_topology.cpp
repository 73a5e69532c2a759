#include "moc/runtime/kfd_topology.hpp"

#include <dirent.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>

namespace moc {

namespace {

// "name value" lines of a topology node's properties file. Values are unsigned 64-bit (hive_id and unique_id
// use all 64 bits), so each line is parsed on its own: one large value must not end the scan.
struct NodeProps {
  int64_t simd = 0, minor = -1, domain = -1, location = -1;
  uint64_t unique_id = 0;
};
bool read_properties(const std::string& path, NodeProps& p) {
  std::ifstream f(path);
  if (!f) return false;
  std::string line;
  while (std::getline(f, line)) {
    const size_t sp = line.find(' ');
    if (sp == std::string::npos) continue;
    const std::string key = line.substr(0, sp);
    const uint64_t v = std::strtoull(line.c_str() + sp + 1, nullptr, 10);
    if (key == "simd_count") p.simd = static_cast<int64_t>(v);
    else if (key == "drm_render_minor") p.minor = static_cast<int64_t>(v);
    else if (key == "domain") p.domain = static_cast<int64_t>(v);
    else if (key == "location_id") p.location = static_cast<int64_t>(v);
    else if (key == "unique_id") p.unique_id = v;
  }
  return true;
}

// "i,j,k" -> indices into `gpus`; a "GPU-<16 hex digits>" entry names a GPU by its UUID (ROCR_VISIBLE_DEVICES
// takes both). nullopt for anything else (unknown UUIDs, empty lists: the runtime's to interpret).
std::optional<std::vector<int>> index_list(const char* v, const std::vector<KfdGpu>& gpus) {
  std::vector<int> out;
  std::stringstream ss(v);
  std::string tok;
  while (std::getline(ss, tok, ',')) {
    if (tok.size() == 20 && (tok.compare(0, 4, "GPU-") == 0 || tok.compare(0, 4, "gpu-") == 0)) {
      std::string want = "GPU-" + tok.substr(4);
      for (size_t c = 4; c < want.size(); ++c) want[c] = static_cast<char>(std::tolower(static_cast<unsigned char>(want[c])));
      int found = -1;
      for (size_t i = 0; i < gpus.size() && found < 0; ++i)
        if (kfd_uuid(gpus[i]) == want) found = static_cast<int>(i);
      if (found < 0) return std::nullopt;
      out.push_back(found);
      continue;
    }
    if (tok.empty() || tok.find_first_not_of("0123456789") != std::string::npos || tok.size() > 6) return std::nullopt;
    out.push_back(std::stoi(tok));
  }
  if (out.empty()) return std::nullopt;
  return out;
}

// The runtime's re-mapping by index lists: ROCR_VISIBLE_DEVICES picks from the GPUs the driver gives this
// process, then HIP_VISIBLE_DEVICES (or CUDA_VISIBLE_DEVICES, GPU_DEVICE_ORDINAL) from those — each list
// in its own order; ROCR_VISIBLE_DEVICES may also name GPUs by UUID. Anything else (unknown UUIDs,
// out-of-range or repeated indices, disagreeing HIP/CUDA lists) is left to the runtime: nullopt.
std::optional<std::vector<KfdGpu>> apply_visible_env(std::vector<KfdGpu> gpus) {
  auto pick = [&gpus](const char* var) -> bool {
    const char* v = std::getenv(var);
    if (!v) return true;
    const auto idx = index_list(v, gpus);
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
    NodeProps np;
    if (!read_properties(paths.nodes + "/" + std::to_string(id) + "/properties", np))
      return std::nullopt;  // a node that cannot be read: leave the answer to the runtime
    const int64_t simd = np.simd, minor = np.minor, domain = np.domain, location = np.location;
    if (simd <= 0) continue;  // a CPU node
    if (minor < 0) return std::nullopt;
    const std::string render = paths.dri + "/renderD" + std::to_string(minor);
    if (access(render.c_str(), R_OK | W_OK) != 0) continue;  // another tenant's GPU
    KfdGpu g;
    g.node = id;
    g.render_minor = static_cast<int>(minor);
    g.unique_id = np.unique_id;
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

std::string kfd_uuid(const KfdGpu& g) {
  if (!g.unique_id) return "";
  char buf[32];
  std::snprintf(buf, sizeof buf, "GPU-%016llx", static_cast<unsigned long long>(g.unique_id));
  return buf;
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
