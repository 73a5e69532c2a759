// GPU side of the `final` CLI, built as a plugin (mpi_openmp_cuda_amd/lib/libmoc_final_gpu.so) and
// loaded with dlopen only when a rank runs the HIP backend. `final` itself links no ROCm library, so
//   * CPU-backend runs (BASELINE.json config 1, small jobs under --backend=auto) start as fast as a plain
//     MPI program and work on hosts without ROCm,
//   * GPU runs pay for the HIP/RCCL runtimes only when they use them.
// The reference links the CUDA runtime statically into every rank (makefile:4).
#pragma once

#include <cstddef>
#include <cstdint>
#include <functional>
#include <string>
#include <vector>

#include "moc/comm.hpp"
#include "moc/device_comm.hpp"
#include "moc/common.hpp"
#include "moc/problem.hpp"
#include "moc/wire.hpp"

namespace moc {

struct GpuRankOptions {
  int device = -1;              // explicit device, or -1: node-local rank (or device_map)
  std::vector<int> device_map;  // node-local rank i -> device_map[i % size]
  int64_t chunk_records = 0;    // 0: engine defaults
  int64_t chunk_bytes = 0;
  std::string log_level = "warn";
  bool preload_kernels = true;  // false: kernel code objects load at their first launch (tiny jobs)
  double comm_timeout_s = 300;  // the RCCL comm's wait deadline (--comm-timeout; <= 0: none)
};

// What the last solve moved and ran (for --timing).
struct GpuSolveStats {
  double kernel_ms = 0;
  int64_t h2d_bytes = 0, d2h_bytes = 0;
  int32_t kernels = 0;  // bitmask: 1 swipe, 2 short, 4 tiles
  int32_t direct = 0;   // 1: streamed zero-copy / DMA from pinned host memory
  R2Params r2{};        // parameters of R2 results
};

class GpuRank {
 public:
  virtual ~GpuRank() = default;
  virtual int device() const = 0;
  virtual void set_problem(const Weights& w, const uint8_t* seq1, int64_t L1, Semantics sem) = 0;
  // Host batch -> host results (record i at codes + offsets[i]); zero-copy when the buffers are pinned.
  virtual void solve(const uint8_t* codes, const int64_t* offsets, int64_t n, Result* out) = 0;
  // Context-parallel share `part` of `parts` of every record -> packed 64-bit keys (host).
  virtual void search_keys(const uint8_t* codes, const int64_t* offsets, int64_t n, int part, int parts,
                           uint64_t* keys) = 0;
  virtual double last_kernel_ms() const = 0;
  // NUMA node of the device's PCIe root complex (-1: unknown); the rank's threads are bound to it.
  virtual int numa_node() const = 0;
  // The HIP runtime has started (page-locking and the engine no longer wait for it); never blocks.
  virtual bool runtime_ready() const = 0;
  // Wire-format batch (moc/wire.hpp) -> results in `fmt` (zero-copy when every buffer is pinned).
  virtual void solve_wire(const WireBatch& b, void* out, ResultFormat fmt) = 0;
  // The same in two halves (HipEngine::begin_wire / finish_wire): begin queues the zero-copy streaming
  // kernel and returns; finish waits for it and returns its stats.
  virtual void begin_wire(const WireBatch& b, void* out, ResultFormat fmt) = 0;
  virtual GpuSolveStats finish_wire() = 0;
  // True when batches of this length range stream packed letters + narrow lengths + sparse offsets.
  virtual bool streams_packed(int64_t min_l2, int64_t max_l2) const = 0;
  // Smallest result format for records of lengths [min_l2, max_l2].
  virtual ResultFormat result_format(int64_t min_l2, int64_t max_l2) const = 0;
  virtual GpuSolveStats last_stats() const = 0;
  virtual void pin(const void* p, size_t bytes) = 0;
  virtual void unpin_all() = 0;
  // Hands over this rank's page-lock registrations: the returned task unregisters them (e.g. on a
  // BackgroundReleaser, ahead of the unmap of the pages); the engine forgets them at once.
  virtual std::function<void()> detach_pins() = 0;
  // Creates the RCCL communicator (collective over ctx.world: every rank must call it). _begin exchanges
  // the unique id over MPI and connects on a helper thread; init_rccl waits for (or does) the connect.
  virtual void init_rccl_begin() = 0;
  virtual void init_rccl() = 0;
  // The rccl transport's device layer (moc/device_comm.hpp): RCCL over xGMI on the engine's stream, and the
  // engine over device-resident wire batches (init_rccl first).
  virtual DeviceComm& device_comm() = 0;
  virtual DeviceSearch& device_search() = 0;
  // The communicator's set-up time on its helper thread, and how long the rank then waited for it (0 before
  // init_rccl; --timing).
  virtual double rccl_init_ms() const = 0;
  virtual double rccl_wait_ms() const = 0;
};

// Plugin entry points (extern "C", resolved with dlsym).
using GpuDeviceCountFn = int (*)();
using GpuRankCreateFn = GpuRank* (*)(const MpiContext& ctx, const GpuRankOptions& opt);
// RCCL's one-time start-up on `device` (moc::rccl_warmup), for a helper thread before MPI starts; 0 = ok.
using GpuRcclWarmupFn = int (*)(int device);
constexpr const char* kGpuDeviceCountSym = "moc_final_gpu_device_count";
constexpr const char* kGpuRankCreateSym = "moc_final_gpu_create";
constexpr const char* kGpuRcclWarmupSym = "moc_final_gpu_rccl_warmup";

}  // namespace moc
