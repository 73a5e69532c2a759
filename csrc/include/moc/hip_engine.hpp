// Per-rank GPU engine: problem upload, launch planning, and the chunked host<->device pipeline.
//
// Reference: send_divided_Seq2_To_Cuda (cudaFunctions.cu:178-242) — cudaMalloc per call and per
// record (leaking all but the last dev_count_signs), a blocking H2D of the whole fixed-stride chunk,
// one launch + cudaDeviceSynchronize per record, three blocking D2H copies, and the problem state in
// __constant__ symbols uploaded by four separate calls (cudaFunctions.cu:35-61).
//
// Here: pooled device buffers (grown, never freed per call), the problem (LUT + Seq1) uploaded once,
// and a double-buffered 3-stream pipeline per chunk of records:
//     copy stream:    H2D codes/offsets/plan of chunk c+1
//     compute stream: packed + tile kernels of chunk c
//     return stream:  D2H results of chunk c-1 straight into the caller's (pinned) result array
// ordered by events only — no device-wide synchronisation inside the loop.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <memory>
#include <vector>

#include "moc/common.hpp"
#include "moc/device.hpp"
#include "moc/score_table.hpp"

namespace moc {

struct EngineOptions {
  int device = -1;                     // -1: keep the current device
  int64_t chunk_records = 1 << 21;     // max records per pipeline chunk
  int64_t chunk_bytes = 64ll << 20;    // max letter bytes per pipeline chunk
  bool pin_host = true;                // hipHostRegister caller buffers for direct DMA
};

struct EngineStats {
  double kernel_ms = 0;  // sum of compute-stream time (events), last solve
  double total_ms = 0;   // wall time of the last solve call
  int64_t h2d_bytes = 0, d2h_bytes = 0, chunks = 0, cells = 0, records = 0;
};

class HipEngine {
 public:
  explicit HipEngine(const EngineOptions& opt = {});
  ~HipEngine();
  HipEngine(const HipEngine&) = delete;
  HipEngine& operator=(const HipEngine&) = delete;

  void set_problem(const Weights& w, const uint8_t* seq1, int64_t L1, Semantics sem);
  // Same, with Seq1 already on this device (e.g. delivered by an RCCL broadcast).
  void set_problem_device(const Weights& w, const uint8_t* d_seq1, int64_t L1, Semantics sem);

  // Host CSR in -> host results out (the pipeline). `offsets` are absolute (n+1 entries).
  void solve(const uint8_t* codes, const int64_t* offsets, int64_t n, Result* out);

  // Device-resident batch: d_codes/d_offsets/d_out on this device; h_offsets is a host copy of the
  // offsets used for planning. Work is queued on `stream` (0 = engine compute stream); no sync.
  void solve_device(const uint8_t* d_codes, const int64_t* d_offsets, const int64_t* h_offsets, int64_t n,
                    Result* d_out, hipStream_t stream);

  const EngineStats& stats() const { return stats_; }
  int device() const { return device_; }
  hipStream_t compute_stream() const { return s_compute_; }
  int64_t L1() const { return L1_; }

 private:
  struct Slot;  // one double-buffer half
  struct HostPlan {
    int32_t slot = 0, rpw = 0;
    std::vector<dev::Tile> tiles;
    std::vector<int32_t> long_recs;
    int64_t max_l2 = 0, cells = 0;
  };
  void plan_chunk(const int64_t* offsets, int64_t n, HostPlan& hp) const;
  dev::ProblemView problem_view(int64_t max_l2) const;
  void ensure(void*& ptr, size_t& cap, size_t bytes);
  void ensure_host(void*& ptr, size_t& cap, size_t bytes);

  EngineOptions opt_;
  int device_ = 0;
  hipStream_t s_copy_ = nullptr, s_compute_ = nullptr, s_return_ = nullptr;
  // problem
  ScoreTable table_{};
  int32_t* d_lut_ = nullptr;
  uint8_t* d_seq1_ = nullptr;
  int64_t L1_ = 0;
  Semantics sem_ = Semantics::Reference;
  bool have_problem_ = false;
  std::vector<std::unique_ptr<Slot>> slots_;
  // scratch for solve_device
  void* d_plan_ = nullptr;
  size_t d_plan_cap_ = 0;
  void* h_plan_ = nullptr;
  size_t h_plan_cap_ = 0;
  hipEvent_t ev_plan_ = nullptr;
  EngineStats stats_;
};

// Picks the int32 hot-loop key width for a problem: bits for k, or 0 (=> 64-bit keys) when
// 2*max|T|*L2 does not fit next to them in an int32.
int32_t choose_key_shift(int32_t max_abs_weight, int64_t max_l2);

}  // namespace moc
