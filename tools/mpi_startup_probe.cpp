// Where a tiny job's wall clock goes under `mpiexec -np N`: process start to main, MPI_Init, MPI_Finalize,
// each on the process's own steady clock (process start from /proc/self/stat), next to the launcher's wall
// measured outside (tools/mpi_startup_probe.sh). Build: see that script.
#include <mpi.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <ctime>

namespace {
double mono_ms() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e3 + ts.tv_nsec / 1e6;
}
// process start time (field 22 of /proc/self/stat, clock ticks since boot) on CLOCK_MONOTONIC's scale
double start_ms() {
  FILE* f = std::fopen("/proc/self/stat", "r");
  if (!f) return -1;
  char buf[4096];
  size_t n = std::fread(buf, 1, sizeof buf - 1, f);
  std::fclose(f);
  buf[n] = 0;
  const char* p = std::strrchr(buf, ')');
  if (!p) return -1;
  unsigned long long st = 0;
  int field = 2;
  for (const char* q = p + 1; *q && field < 22; ++q)
    if (*q == ' ' && ++field == 22) std::sscanf(q + 1, "%llu", &st);
  return st * 1e3 / sysconf(_SC_CLK_TCK);
}
}  // namespace

int main(int argc, char** argv) {
  const double t_main = mono_ms();
  const double t_start = start_ms();
  int provided = 0;
  const bool multi = argc > 1 && std::strcmp(argv[1], "multiple") == 0;
  if (multi)
    MPI_Init_thread(&argc, &argv, MPI_THREAD_MULTIPLE, &provided);
  else
    MPI_Init(&argc, &argv);
  const double t_init = mono_ms();
  int rank = 0, size = 1;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  MPI_Barrier(MPI_COMM_WORLD);
  const double t_bar = mono_ms();
  MPI_Finalize();
  const double t_fin = mono_ms();
  std::printf("rank %d/%d%s: exec->main %.1f ms, MPI_Init %.1f ms, first barrier %.1f ms, MPI_Finalize %.1f ms\n", rank,
              size, multi ? " (THREAD_MULTIPLE)" : "", t_start >= 0 ? t_main - t_start : -1.0, t_init - t_main,
              t_bar - t_init, t_fin - t_bar);
  return 0;
}
