// Does the HIP runtime's start-up slow down while the process's other threads fault pages in (what
// `final`'s read / count / encode do while the runtime starts on a helper thread)? hipGetDeviceCount timed
// alone, then with N threads mmapping + touching + unmapping fresh 4 KiB-page or 2 MiB-page memory, then
// with N threads only computing (no page faults), with N threads faulting in a region mapped beforehand (no
// mmap/munmap while the runtime starts: "touch"), and with N threads streaming reads over memory faulted in
// beforehand ("membw": bandwidth, no faults).
// Build: hipcc -O2 -std=c++17 tools/hip_init_contention.cpp -o build/hip_init_contention -lpthread
//        (each mode is its own process: build/hip_init_contention idle|faults4k|faults2m|compute [N])
#include <hip/hip_runtime_api.h>
#include <sys/mman.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "idle";
  const int n = argc > 2 ? std::atoi(argv[2]) : 15;
  std::atomic<bool> stop{false};
  std::atomic<long> faults{0};
  std::vector<std::thread> busy;
  // touch / membw: one big region mapped (and for membw faulted in) before the runtime starts
  const size_t big = size_t{8} << 30;
  char* region = nullptr;
  if (mode == "touch" || mode == "membw") {
    region = static_cast<char*>(mmap(nullptr, big, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0));
    if (region == MAP_FAILED) return 1;
    madvise(region, big, MADV_HUGEPAGE);
    if (mode == "membw") std::memset(region, 1, big);
  }
  if (mode != "idle") {
    for (int t = 0; t < n; ++t)
      busy.emplace_back([&, t] {
        const size_t sz = size_t{64} << 20;
        volatile double x = t;
        while (!stop.load()) {
          if (mode == "compute") {
            for (int i = 0; i < 1000000; ++i) x = x * 1.0000001 + 1e-9;
            continue;
          }
          if (mode == "touch") {  // fresh pages of the premapped region, 4 KiB strides, until it is used up
            const size_t share = big / n;
            for (size_t o = 0; o < share && !stop.load(); o += 4096) region[t * share + o] = 1;
            faults += static_cast<long>(share / 4096);
            while (!stop.load()) std::this_thread::sleep_for(std::chrono::milliseconds(1));
            continue;
          }
          if (mode == "membw") {
            const size_t share = big / n;
            long acc = 0;
            for (size_t o = 0; o < share; o += 64) acc += region[t * share + o];
            x = x + acc;
            continue;
          }
          char* p = static_cast<char*>(mmap(nullptr, sz, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0));
          if (p == MAP_FAILED) continue;
          madvise(p, sz, mode == "faults2m" ? MADV_HUGEPAGE : MADV_NOHUGEPAGE);
          for (size_t o = 0; o < sz; o += 4096) p[o] = 1;
          faults += static_cast<long>(sz / 4096);
          munmap(p, sz);
        }
      });
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
  const auto t0 = std::chrono::steady_clock::now();
  int count = 0;
  (void)hipGetDeviceCount(&count);
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  stop = true;
  for (auto& t : busy) t.join();
  std::printf("%-9s threads=%2d hipGetDeviceCount %7.1f ms  devices %d  pages touched %ld\n", mode.c_str(),
              mode == "idle" ? 0 : n, ms, count, faults.load());
  return 0;
}
