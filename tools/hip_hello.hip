// The floor of `mpiexec -np N ./final --backend=hip` on a tiny input: the least a program can do that starts
// MPI and runs one kernel on the GPU — HIP runtime up, one stream (one hardware queue), one empty kernel,
// sync, finalize. The runtime starts on a helper thread while MPI_Init runs, as ./final's early prewarm does
// (csrc/apps/final.cpp), so the two overlap the same way. Prints the in-process split on stderr.
// Build and use: tools/final_walltime.sh (HELLO=1).
#include <hip/hip_runtime.h>
#include <mpi.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>

__global__ void empty_kernel(int* out) {
  if (out && threadIdx.x == 0 && blockIdx.x == 0) out[0] = 1;
}

static double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int main(int argc, char** argv) {
  auto t0 = std::chrono::steady_clock::now();
  double t_rt = 0, t_q = 0, t_k = 0;
  bool ok = true;
  std::thread gpu([&] {
    int n = 0;
    ok = hipGetDeviceCount(&n) == hipSuccess && n > 0;
    t_rt = ms_since(t0);
    if (!ok) return;
    // HELLO_NULL_STREAM=1: the runtime's null stream instead of a stream of our own (does it come with the
    // runtime's start, or cost its own hardware queue at first use?)
    const bool null_stream = std::getenv("HELLO_NULL_STREAM") && std::atoi(std::getenv("HELLO_NULL_STREAM")) != 0;
    hipStream_t s = nullptr;
    ok = hipSetDevice(0) == hipSuccess &&
         (null_stream || hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess);
    t_q = ms_since(t0);
    if (!ok) return;
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, nullptr);
    ok = hipStreamSynchronize(s) == hipSuccess;
    t_k = ms_since(t0);
    if (s) (void)hipStreamDestroy(s);
  });
  MPI_Init(&argc, &argv);
  double t_mpi = ms_since(t0);
  int rank = 0;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  gpu.join();
  if (rank == 0) {
    std::printf("hello\n");
    std::fprintf(stderr, "{\"mpi_init_ms\": %.1f, \"runtime_up_ms\": %.1f, \"queue_up_ms\": %.1f, \"kernel_done_ms\": %.1f, "
                 "\"ok\": %s}\n", t_mpi, t_rt, t_q, t_k, ok ? "true" : "false");
  }
  MPI_Finalize();
  return ok ? 0 : 1;
}
