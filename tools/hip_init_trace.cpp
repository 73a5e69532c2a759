// Where the HIP runtime's 140-220 ms start-up goes on the box, without strace/perf (not in the image): a
// helper thread calls hipGetDeviceCount while the main thread samples that thread's /proc/self/task/<tid>
// syscall file every ~50 us — a histogram of the system calls it sits in (and "running" when it is in user
// code), and the paths of the files it opens (read back from its own memory with process_vm_readv, which
// fails instead of faulting when the buffer is gone), each with the time it was first seen.
// Build: hipcc -O2 -std=c++17 tools/hip_init_trace.cpp -o build/hip_init_trace -lpthread
#include <hip/hip_runtime_api.h>
#include <sys/syscall.h>
#include <sys/uio.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

namespace {
double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
std::string read_str(unsigned long addr) {
  char buf[512];
  iovec local{buf, sizeof buf - 1}, remote{reinterpret_cast<void*>(addr), sizeof buf - 1};
  const ssize_t n = process_vm_readv(getpid(), &local, 1, &remote, 1, 0);
  if (n <= 0) return "?";
  buf[n] = 0;
  return std::string(buf, strnlen(buf, static_cast<size_t>(n)));
}
const char* sysname(long nr) {
  switch (nr) {
    case -1: return "running (user code)";
    case 0: return "read";
    case 1: return "write";
    case 2: return "open";
    case 3: return "close";
    case 4: return "stat";
    case 5: return "fstat";
    case 9: return "mmap";
    case 10: return "mprotect";
    case 11: return "munmap";
    case 16: return "ioctl";
    case 17: return "pread64";
    case 21: return "access";
    case 28: return "madvise";
    case 35: return "nanosleep";
    case 59: return "execve";
    case 72: return "fcntl";
    case 89: return "readlink";
    case 202: return "futex";
    case 217: return "getdents64";
    case 257: return "openat";
    case 262: return "newfstatat";
    case 332: return "statx";
    default: return nullptr;
  }
}
}  // namespace

int main() {
  std::atomic<long> tid{0};
  std::atomic<bool> done{false}, started{false};
  double t_start = now_ms(), t_end = 0;
  int count = 0;
  std::thread worker([&] {
    tid = syscall(SYS_gettid);
    while (tid.load() == 0) {
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(5));  // the sampler is up
    t_start = now_ms();
    started = true;
    (void)hipGetDeviceCount(&count);
    t_end = now_ms();
    done = true;
  });
  while (!started.load()) {
  }
  const std::string path = "/proc/self/task/" + std::to_string(tid.load()) + "/syscall";
  std::map<long, int> hist;
  std::map<std::string, double> opened;  // path -> first seen (ms since start)
  std::vector<std::pair<double, std::string>> order;
  int samples = 0;
  while (!done.load()) {
    FILE* f = std::fopen(path.c_str(), "r");
    if (!f) break;
    char line[512] = {0};
    const bool got = std::fgets(line, sizeof line, f) != nullptr;
    std::fclose(f);
    if (!got) continue;
    long nr = -2;
    unsigned long a[6] = {0};
    if (std::strncmp(line, "running", 7) == 0) {
      nr = -1;
    } else {
      std::sscanf(line, "%ld %lx %lx %lx %lx %lx %lx", &nr, &a[0], &a[1], &a[2], &a[3], &a[4], &a[5]);
    }
    ++hist[nr];
    ++samples;
    std::string p;
    if (nr == 257) p = read_str(a[1]);
    else if (nr == 2 || nr == 4 || nr == 21 || nr == 89) p = read_str(a[0]);
    else if (nr == 262 || nr == 332) p = read_str(a[1]);
    if (!p.empty() && !opened.count(p)) {
      opened[p] = now_ms() - t_start;
      order.emplace_back(opened[p], p);
    }
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
  worker.join();
  std::printf("hipGetDeviceCount: %.1f ms, %d device(s), %d samples\n", t_end - t_start, count, samples);
  std::vector<std::pair<int, long>> by;
  for (const auto& [nr, c] : hist) by.emplace_back(c, nr);
  std::sort(by.rbegin(), by.rend());
  for (const auto& [c, nr] : by) {
    const char* n = sysname(nr);
    std::printf("  %5.1f %%  %s (%ld)\n", 100.0 * c / std::max(samples, 1), n ? n : "syscall", nr);
  }
  std::printf("paths, first seen (ms):\n");
  for (const auto& [t, p] : order) std::printf("  %8.2f  %s\n", t, p.c_str());
  return 0;
}
