// Scanning a page-cached file through a fresh mapping (what the node streaming flow's count pass does on an
// --input file): plain faults (fault-around) vs each thread populating its chunk's page tables first with
// madvise(MADV_POPULATE_READ) vs MAP_POPULATE at map time. 16 threads read it at memory speed in 1 MiB chunks.
// Build: g++ -O3 -march=native -fopenmp tools/populate_probe.cpp -o build/populate_probe; run: build/populate_probe FILE
#include <fcntl.h>
#include <omp.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>

#ifndef MADV_POPULATE_READ
#define MADV_POPULATE_READ 22
#endif

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  if (argc < 2) return 1;
  const int fd = open(argv[1], O_RDONLY);
  struct stat st {};
  if (fd < 0 || fstat(fd, &st) != 0) return 1;
  const size_t len = static_cast<size_t>(st.st_size);
  const size_t chunk = size_t{1} << 20;
  const long nch = static_cast<long>((len + chunk - 1) / chunk);
  for (int round = 0; round < 2; ++round)
    for (int mode = 0; mode < 3; ++mode) {
      const double t0 = now_ms();
      const char* p = static_cast<const char*>(
          mmap(nullptr, len, PROT_READ, MAP_SHARED | (mode == 2 ? MAP_POPULATE : 0), fd, 0));
      if (p == MAP_FAILED) return 1;
      const double t1 = now_ms();
      long lines = 0;
      int madv_err = 0;
#pragma omp parallel for schedule(dynamic, 4) reduction(+ : lines, madv_err)
      for (long c = 0; c < nch; ++c) {
        const size_t b = static_cast<size_t>(c) * chunk, e = std::min(len, b + chunk);
        if (mode == 1 && madvise(const_cast<char*>(p + b), e - b, MADV_POPULATE_READ) != 0) ++madv_err;
        // a memory-speed pass: 8 bytes at a time (every page is read)
        unsigned long k = 0;
        size_t i = b;
        for (; i + 8 <= e; i += 8) {
          unsigned long w;
          std::memcpy(&w, p + i, 8);
          k += w;
        }
        lines += static_cast<long>(k & 0xff);
      }
      const double t2 = now_ms();
      munmap(const_cast<char*>(p), len);
      std::printf("round %d mode %-14s map %7.1f ms  scan %7.1f ms  (%.1f GB/s)  lines %ld  madvise errors %d\n", round,
                  mode == 0 ? "faults" : mode == 1 ? "populate_read" : "map_populate", t1 - t0, t2 - t1,
                  len / ((t2 - t0) * 1e6), lines, madv_err);
    }
  return 0;
}
