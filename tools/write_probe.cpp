// Output write-path probe: the same bytes written by T threads with pwrite (one inode lock: serial) vs
// memcpy into a shared file mapping (parallel page faults), 5 MB per thread per block. Build:
//   g++ -O2 -fopenmp tools/write_probe.cpp -o build/write_probe && build/write_probe /tmp/x.out 1400
#include <fcntl.h>
#include <omp.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <vector>

static double now() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const char* path = argc > 1 ? argv[1] : "/dev/shm/wr.out";
  const size_t total = (argc > 2 ? atoll(argv[2]) : 1400) << 20;
  const int T = omp_get_max_threads();
  const size_t part = 5 << 20;  // 5 MB per part per block
  std::vector<std::vector<char>> bufs(T, std::vector<char>(part, 'x'));
  for (int mode = 0; mode < 3; ++mode) {
    unlink(path);
    int fd = open(path, O_RDWR | O_CREAT | O_TRUNC, 0644);
    double t0 = now();
    if (mode == 0) {
      for (size_t b = 0; b < total; b += part * T) {
#pragma omp parallel for num_threads(T)
        for (int t = 0; t < T; ++t) pwrite(fd, bufs[t].data(), part, b + t * part);
      }
    } else {
      ftruncate(fd, total + (size_t(1) << 30));
      char* m = (char*)mmap(nullptr, total + (size_t(1) << 30), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
      if (mode == 2) madvise(m, total, MADV_HUGEPAGE);
      for (size_t b = 0; b < total; b += part * T) {
#pragma omp parallel for num_threads(T)
        for (int t = 0; t < T; ++t) memcpy(m + b + t * part, bufs[t].data(), part);
      }
      munmap(m, total + (size_t(1) << 30));
      ftruncate(fd, total);
    }
    close(fd);
    printf("%s mode %d: %.1f ms (%.2f GB/s)\n", path, mode, now() - t0, total / 1e6 / (now() - t0));
  }
  unlink(path);
}
