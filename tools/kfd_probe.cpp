// Cost of reading the driver's GPU topology from sysfs (moc/runtime/kfd_topology.hpp) on the box: the
// whole kfd_gpus() call, then each node's properties file and render-node check on its own.
// Build: g++ -O2 -std=c++17 -Icsrc/include tools/kfd_probe.cpp csrc/src/runtime/kfd_topology.cpp -o build/kfd_probe
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>

#include "moc/runtime/kfd_topology.hpp"

namespace {
double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

int main() {
  for (int r = 0; r < 3; ++r) {
    const double t0 = now_ms();
    const auto g = moc::kfd_gpus();
    const double t1 = now_ms();
    std::printf("kfd_gpus run %d: %.3f ms, %s", r, t1 - t0, g ? "" : "unknown\n");
    if (g) {
      std::printf("%zu GPU(s):", g->size());
      for (const auto& x : *g) std::printf(" node %d renderD%d %s numa %d;", x.node, x.render_minor, x.pci_bus_id.c_str(), x.numa_node);
      std::printf("\n");
    }
  }
  for (int n = 0; n < 16; ++n) {
    const std::string p = "/sys/class/kfd/kfd/topology/nodes/" + std::to_string(n) + "/properties";
    const double t0 = now_ms();
    std::ifstream f(p);
    if (!f) break;
    std::stringstream ss;
    ss << f.rdbuf();
    const double t1 = now_ms();
    std::string text = ss.str();
    const auto at = text.find("drm_render_minor");
    int minor = -1;
    if (at != std::string::npos) std::sscanf(text.c_str() + at, "drm_render_minor %d", &minor);
    const std::string render = "/dev/dri/renderD" + std::to_string(minor);
    const double t2 = now_ms();
    const int acc = access(render.c_str(), R_OK | W_OK);
    const double t3 = now_ms();
    std::printf("node %2d: properties %6.3f ms (%zu bytes), minor %d access %s %.3f ms\n", n, t1 - t0, text.size(), minor,
                acc == 0 ? "ok" : "no", t3 - t2);
  }
  return 0;
}
