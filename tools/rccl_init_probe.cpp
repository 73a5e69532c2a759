// RCCL communicator start-up, phase by phase, for one rank on one GPU (VERDICT r2 "root-cause RCCL
// start-up"). Times: loading librccl (dlopen: 573 MB of fat binaries to map and register), the HIP context,
// ncclGetUniqueId (bootstrap network discovery), ncclCommInitRank (topology, channels, device kernels),
// the first collective, and a second communicator (what is one-time per process vs per communicator).
//   --busy=T   a team of T OpenMP threads computes on other threads during the whole start-up (what the
//              parse does in ./final when the connect overlaps it); --passive: the team sleeps between
//              bursts instead of spinning (OMP_WAIT_POLICY-like behaviour, simulated).
//   --dlopen-first   load librccl before the HIP runtime starts (as ./final's plugin does)
//   --warm           a 1-rank communicator on a helper thread first (what ./final can start before MPI is
//                    up), then the timed one
//   --teardown=destroy|abort|none   how the communicators end
// Build (here): hipcc -O2 -std=c++17 -fopenmp tools/rccl_init_probe.cpp -ldl -o build/rccl_init_probe
// Run (box):    build/rccl_init_probe [--busy=16]
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <omp.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {
double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
template <typename F>
F sym(void* h, const char* name) {
  void* p = dlsym(h, name);
  if (!p) {
    std::fprintf(stderr, "missing %s\n", name);
    std::exit(2);
  }
  return reinterpret_cast<F>(p);
}
}  // namespace

int main(int argc, char** argv) {
  int busy = 0;
  bool passive = false, dlopen_first = false, warm = false;
  std::string teardown = "destroy";
  for (int i = 1; i < argc; ++i) {
    if (std::strncmp(argv[i], "--busy=", 7) == 0) busy = std::atoi(argv[i] + 7);
    if (std::strcmp(argv[i], "--passive") == 0) passive = true;
    if (std::strcmp(argv[i], "--dlopen-first") == 0) dlopen_first = true;
    if (std::strcmp(argv[i], "--warm") == 0) warm = true;
    if (std::strncmp(argv[i], "--teardown=", 11) == 0) teardown = argv[i] + 11;
  }
  std::atomic<bool> stop{false};
  std::atomic<long> bursts{0};
  std::thread load;
  if (busy > 0) {
    // a parse-like load: every thread of a team streams over its own 64 MB buffer, repeatedly
    load = std::thread([&] {
      std::vector<std::vector<unsigned char>> bufs(static_cast<size_t>(busy), std::vector<unsigned char>(64u << 20, 1));
      while (!stop.load()) {
#pragma omp parallel for num_threads(busy) schedule(static, 1)
        for (int t = 0; t < busy; ++t) {
          unsigned acc = 0;
          for (size_t i = 0; i < bufs[t].size(); i += 64) acc += bufs[t][i] * 2654435761u;
          bufs[t][0] = static_cast<unsigned char>(acc);
        }
        ++bursts;
        if (passive) std::this_thread::sleep_for(std::chrono::milliseconds(1));
      }
    });
    std::this_thread::sleep_for(std::chrono::milliseconds(200));
  }
  double t = now_ms();
  const double t_start = t;
  auto lap = [&t](const char* what) {
    const double n = now_ms();
    std::printf("%-34s %9.1f ms\n", what, n - t);
    std::fflush(stdout);
    t = n;
  };
  void* h = nullptr;
  if (dlopen_first) {
    h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    lap("dlopen librccl.so.1 (before HIP)");
  }
  int ndev = 0;
  (void)hipGetDeviceCount(&ndev);
  lap("hipGetDeviceCount (HIP runtime)");
  (void)hipSetDevice(0);
  void* p = nullptr;
  (void)hipMalloc(&p, 256);
  lap("hipSetDevice + hipMalloc (context)");
  if (!h) {
    h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    lap("dlopen librccl.so.1");
  }
  if (!h) {
    std::fprintf(stderr, "dlopen librccl: %s\n", dlerror());
    return 2;
  }
  auto get_id = sym<ncclResult_t (*)(ncclUniqueId*)>(h, "ncclGetUniqueId");
  auto init = sym<ncclResult_t (*)(ncclComm_t*, int, ncclUniqueId, int)>(h, "ncclCommInitRank");
  auto allreduce = sym<ncclResult_t (*)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                                        hipStream_t)>(h, "ncclAllReduce");
  auto destroy = sym<ncclResult_t (*)(ncclComm_t)>(h, "ncclCommDestroy");
  auto abort_fn = sym<ncclResult_t (*)(ncclComm_t)>(h, "ncclCommAbort");
  ncclComm_t warm_comm = nullptr;
  if (warm) {  // a helper thread's throw-away communicator: the library's one-time loading happens there
    std::thread t([&] {
      (void)hipSetDevice(0);
      ncclUniqueId wid;
      if (get_id(&wid) == ncclSuccess) (void)init(&warm_comm, 1, wid, 0);
    });
    t.join();
    lap("warm-up communicator (helper thread)");
  }
  ncclUniqueId id;
  if (get_id(&id) != ncclSuccess) return 3;
  lap("ncclGetUniqueId");
  ncclComm_t comm = nullptr;
  if (init(&comm, 1, id, 0) != ncclSuccess) return 4;
  lap("ncclCommInitRank (1st)");
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  void* d = nullptr;
  (void)hipMalloc(&d, 1 << 20);
  if (allreduce(d, d, 1024, ncclUint64, ncclMax, comm, s) != ncclSuccess) return 5;
  (void)hipStreamSynchronize(s);
  lap("first ncclAllReduce + sync");
  if (allreduce(d, d, 1024, ncclUint64, ncclMax, comm, s) != ncclSuccess) return 5;
  (void)hipStreamSynchronize(s);
  lap("second ncclAllReduce + sync");
  ncclUniqueId id2;
  if (get_id(&id2) != ncclSuccess) return 3;
  ncclComm_t comm2 = nullptr;
  if (init(&comm2, 1, id2, 0) != ncclSuccess) return 4;
  lap("getId + ncclCommInitRank (2nd)");
  if (warm_comm) {
    if (teardown == "abort") (void)abort_fn(warm_comm);
    else if (teardown == "destroy") (void)destroy(warm_comm);
  }
  if (teardown == "abort") {
    (void)abort_fn(comm2);
    (void)abort_fn(comm);
    lap("ncclCommAbort x2");
  } else if (teardown == "destroy") {
    (void)destroy(comm2);
    (void)destroy(comm);
    lap("ncclCommDestroy x2");
  } else {
    lap("communicators left to process exit");
  }
  std::printf("%-34s %9.1f ms  (busy=%d%s, %ld bursts)\n", "TOTAL", now_ms() - t_start, busy,
              passive ? " passive" : "", bursts.load());
  stop = true;
  if (load.joinable()) load.join();
  (void)hipFree(d);
  (void)hipFree(p);
  (void)hipStreamDestroy(s);
  return 0;
}
