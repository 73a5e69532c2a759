// What a GPU job of `final` waits for before its first HIP call returns (gpu_wait): loading the GPU plugin
// (libmoc_final_gpu.so and what it links: libmoc, the HIP runtime, RCCL) and the HIP runtime's start-up,
// each timed on its own. argv[1] = plugin path. No GPU work.
// Build: g++ -O2 -std=c++17 tools/plugin_load_probe.cpp -ldl -o build/plugin_load_probe
#include <dlfcn.h>

#include <chrono>
#include <cstdio>

namespace {
double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

int main(int argc, char** argv) {
  const char* plugin = argc > 1 ? argv[1] : "mpi_openmp_cuda_amd/lib/libmoc_final_gpu.so";
  const bool hip_first = argc > 2;
  double t = now_ms();
  auto lap = [&t](const char* what) {
    const double n = now_ms();
    std::printf("%-44s %8.1f ms\n", what, n - t);
    t = n;
  };
  if (hip_first) {
    void* hip = dlopen("libamdhip64.so.7", RTLD_NOW | RTLD_GLOBAL);
    lap(hip ? "dlopen libamdhip64 (alone)" : "dlopen libamdhip64 FAILED");
    if (hip) {
      using CountFn = int (*)(int*);
      auto count = reinterpret_cast<CountFn>(dlsym(hip, "hipGetDeviceCount"));
      int n = 0;
      if (count) count(&n);
      lap("hipGetDeviceCount (HIP runtime start-up)");
    }
  }
  void* h = dlopen(plugin, RTLD_NOW | RTLD_LOCAL);
  lap(h ? "dlopen plugin" : "dlopen plugin FAILED");
  if (!h) {
    std::printf("%s\n", dlerror());
    return 1;
  }
  using DevFn = int (*)();
  auto dev = reinterpret_cast<DevFn>(dlsym(h, "moc_final_gpu_device_count"));
  const int n = dev ? dev() : -1;
  lap("moc_final_gpu_device_count");
  std::printf("devices: %d\n", n);
  return 0;
}
