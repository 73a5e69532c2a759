// Per-rank GPU engine: problem upload, launch planning, and host<->device data movement.
//
// Reference: send_divided_Seq2_To_Cuda (cudaFunctions.cu:178-242) — cudaMalloc per call and per
// record (leaking all but the last dev_count_signs), a blocking H2D of the whole fixed-stride chunk,
// one launch + cudaDeviceSynchronize per record, three blocking D2H copies, and the problem state in
// __constant__ symbols uploaded by four separate calls (cudaFunctions.cu:35-61).
//
// Here two data paths, chosen per call:
//   * direct (zero-copy streaming): when the batch lives in pinned host memory (hipHostMalloc /
//     hipHostRegister — e.g. the node-shared input window) and every record fits the short kernel, ONE
//     persistent kernel reads the letters straight over PCIe into LDS and writes packed results straight
//     back. Measured on MI355X: kernel reads of pinned host memory run at the hipMemcpy rate
//     (~56-57 GB/s, tools/probe_transfers.py), so staging copies would only add a second pass.
//   * staged pipeline: pooled device buffers (grown, never freed per call) and a double-buffered
//     3-stream chunk pipeline — copy stream H2D chunk c+1 | compute stream kernels of chunk c | return
//     stream D2H of chunk c-1 — ordered by events only. Used for pageable memory and for batches with
//     long records (tile kernel + host-planned tile lists).
// Results are written in the smallest wire format that fits the problem (R4/R8/R12, moc/device.hpp).
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <memory>
#include <utility>
#include <vector>

#include "moc/common.hpp"
#include "moc/device.hpp"
#include "moc/runtime/timer.hpp"
#include "moc/score_table.hpp"

namespace moc {

struct EngineOptions {
  int device = -1;                   // -1: keep the current device
  int64_t chunk_records = 1 << 21;   // staged pipeline: max records per chunk
  int64_t chunk_bytes = 64ll << 20;  // staged pipeline: max letter bytes per chunk
  bool allow_direct = true;          // use zero-copy streaming when the host buffers are pinned
  bool use_graphs = true;            // replay the direct path's launches as a captured hipGraph
  // kernel files (dev::PreloadSet) whose code objects load when the engine starts, on a helper thread beside
  // the stream set-up, not inside the first timed launch; the rest load at their first launch. MOC_PRELOAD
  // (dev::parse_preload_set) overrides.
  unsigned preload = dev::kPreloadAll;
  // Pinned host batches stream zero-copy: the kernel reads / writes host memory itself. A chunked SDMA
  // pipeline around the HBM-resident kernel was measured slower on the registered node-shared arrays the
  // headline streams from (4.4 vs 4.0 ms/step, profiles/host_stream_ab.log) and was retired in round 4.
};

struct EngineStats {
  double kernel_ms = 0;  // device time of the search kernels (events), last solve
  double total_ms = 0;   // wall time of the last solve call
  int64_t h2d_bytes = 0, d2h_bytes = 0, chunks = 0, cells = 0, records = 0;
  int32_t direct = 0;    // 1 if the last solve streamed from pinned host memory (zero-copy)
  int32_t format = 0;    // ResultFormat of the last solve
  int32_t kernels = 0;   // bitmask of kernels used: 1 swipe (lane/record), 2 short (lane/offset), 4 tiles
                         // (LUT tile kernel), 8 tile16
  int32_t forms = 0;     // bitmask of the arithmetic forms they ran (moc::bounds::FormBits)
  R2Params r2;           // parameters of the R2 results of the last solve (when fmt == R2)
};

// Optional metadata about a batch (e.g. known from parsing / generation) that lets the engine skip its
// own scan over the lengths.
struct BatchHints {
  int64_t min_l2 = -1;
  int64_t max_l2 = -1;
};

// One engine per (rank, device). Not thread-safe: calls on one engine must not overlap (the streams,
// pooled buffers, work counter and cached graph are per engine); use one engine per thread instead.
class HipEngine {
 public:
  explicit HipEngine(const EngineOptions& opt = {});
  ~HipEngine();
  HipEngine(const HipEngine&) = delete;
  HipEngine& operator=(const HipEngine&) = delete;

  void set_problem(const Weights& w, const uint8_t* seq1, int64_t L1, Semantics sem);
  // Same, with Seq1 already on this device (e.g. delivered by an RCCL broadcast).
  void set_problem_device(const Weights& w, const uint8_t* d_seq1, int64_t L1, Semantics sem);

  // Host batch in -> host results out as moc::Result. `codes` is the base pointer (record i starts at
  // codes + offsets[i]); `offsets` has n+1 absolute entries.
  void solve(const uint8_t* codes, const int64_t* offsets, int64_t n, Result* out);
  // General form: optional narrow lengths — len_bits 8 (uint8, max L2 <= 255) or 4 (two per byte, low
  // nibble first, record i = len_base + nibble) — results in `fmt`. `packed`: 1 = `codes` is a 5-bit
  // packed stream (moc::pack5; char j at bit 5j), 3 = P33 fields (moc::pack33; 2 was the retired P24 code)
  // 0 = one byte per letter.
  // R2 results are encoded for the hints' [min_l2, max_l2] (or the batch's own range): stats().r2 holds
  // the parameters.
  void solve_ex(const uint8_t* codes, const int64_t* offsets, const uint8_t* lengths, int64_t n, void* out,
                ResultFormat fmt, const BatchHints& hints = {}, int packed = 0, int len_bits = 8,
                int len_base = 0);
  // Any wire-format batch (moc/wire.hpp): packed or byte letters, dense or sparse offsets, narrow lengths.
  // Sparse offsets stream zero-copy when the buffers are pinned and the swipe kernel takes the batch;
  // otherwise dense offsets are rebuilt from the lengths for the staged pipeline.
  void solve_wire(const WireBatch& b, void* out, ResultFormat fmt);
  // The same in two halves: begin_wire queues the zero-copy streaming kernel and returns (any other path
  // completes inside it); finish_wire waits for it and completes stats(). Every other call on the engine
  // finishes an open solve first. A streaming job encodes batch b+1 on the host while batch b streams.
  void begin_wire(const WireBatch& b, void* out, ResultFormat fmt);
  void finish_wire();
  // True when batches of this length range stream packed letters (the swipe kernel takes them).
  bool streams_packed(int64_t min_l2, int64_t max_l2) const;
  // Smallest result format for this problem given the batch's length range (min_l2 <= 0: unknown,
  // R2 not considered).
  ResultFormat auto_format(int64_t max_l2, int64_t min_l2 = 0) const;
  R2Params r2_params_for(int64_t min_l2, int64_t max_l2) const;

  // Device-resident batch: d_codes/d_offsets/d_out on this device; h_offsets is a host copy of the
  // offsets used for planning. Work is queued on `stream` (0 = engine compute stream); no sync.
  // Device time of the last solve_device's kernels (events recorded around its launches, after the host
  // planning): waits for them. Kernel throughput without the host's per-call planning in the interval.
  double device_kernel_ms();
  void solve_device(const uint8_t* d_codes, const int64_t* d_offsets, const int64_t* h_offsets, int64_t n,
                    Result* d_out, hipStream_t stream);

  // Context-parallel search: this engine evaluates part `part` of `parts` of the batch's
  // global list of offset tiles and writes one packed 64-bit key per record (moc::encode_key; 0 =
  // no candidate in this part). A MAX all-reduce of the keys over the parts + finalize_keys gives the
  // full answer; this splits single huge records across GPUs.
  void search_keys_device(const uint8_t* d_codes, const int64_t* d_offsets, const int64_t* h_offsets, int64_t n,
                          int part, int parts, unsigned long long* d_keys, hipStream_t stream);
  // MAX-combined pass-1 keys -> results (k resolved on each record's winning diagonal: needs the batch).
  void finalize_keys_device(const uint8_t* d_codes, const int64_t* d_offsets, const int64_t* h_offsets, int64_t n,
                            const unsigned long long* d_keys, void* d_out, ResultFormat fmt, hipStream_t stream);
  // Host-memory form of search_keys_device (uploads the batch, returns host keys; synchronous).
  void search_keys(const uint8_t* codes, const int64_t* offsets, int64_t n, int part, int parts, uint64_t* keys);

  // Page-locks a host range for the lifetime of the engine (or until unpin); enables the direct path.
  void pin(const void* p, size_t bytes);
  void unpin_all();
  // The registrations made by pin(), handed over to the caller (pinned::unregister them); forgotten here.
  std::vector<void*> detach_pins() {
    finish_wire();
    return std::exchange(pinned_, {});
  }

  const EngineStats& stats() const { return stats_; }
  int device() const { return device_; }
  hipStream_t compute_stream() const { return s_compute_; }
  int64_t L1() const { return L1_; }
  int num_cus() const { return num_cus_; }

 private:
  struct Slot;  // one double-buffer half
  struct ChunkPlan {
    int64_t min_short = 0, max_l2 = 0, n_short = 0, cells = 0;
    std::vector<int32_t> long_recs;
  };
  void plan_chunk(const int64_t* offsets, int64_t n, ChunkPlan& cp) const;
  struct TilePlan {
    int u = 2;              // sub-tiles per wave tile
    int win_tiles = 0;      // windowed tile16: tiles per window stride
    bool tile16 = false;    // the plan is for the tile16 sweep (else the LUT tile kernel)
    int64_t window = 0;     // tile16: columns per LDS window (0: the whole profile is the image)
    bool wide = false;      // tile16: widened int16-pair entries
    bool slide = false;     // tile16: sliding widened windows (window = their columns; dev::Plan::slide_*)
    int64_t slide_items = 0, slide_members = 0, slide_wgs = 0;
    int slide_per_cu = 1;  // workgroups per CU the slide plan is for (1, or 2 with half-LDS windows)
  };
  std::vector<dev::WaveStart> plan_waves(const int64_t* offsets, const int32_t* long_recs, int64_t n_long, int part,
                                         int parts, TilePlan& tp) const;
  bool plan_slide(const int64_t* offsets, const int32_t* long_recs, int64_t n_long, double min_fill, TilePlan& tp,
                  std::vector<dev::WaveStart>& starts) const;
  dev::Plan device_plan(void* d_plan, size_t n_starts, bool has_long_recs, int64_t n_long, const TilePlan& tp) const;
  // problem view for a plan: without the profile when the plan is for the LUT tile kernel
  dev::ProblemView tile_view(int64_t max_l2, const TilePlan& tp) const {
    dev::ProblemView pv = problem_view(max_l2);
    if (!tp.tile16) {
      pv.prof16 = nullptr;
      pv.mfma_sweep = 0;
    } else {  // the plan's image: whole or windowed, byte pairs or widened
      pv.prof16_window = static_cast<int32_t>(tp.window);
      pv.prof16_bytes = tp.window ? static_cast<int32_t>(dev::tile16_window_bytes(tp.window)) : prof16_bytes_;
      pv.prof16_wide = tp.wide ? 1 : 0;
      pv.t16_slide = tp.slide ? tp.slide_per_cu : 0;
      if (tp.window) pv.mfma_sweep = 0;
      if (!pv.mfma_sweep) pv.t16_key_bits = bounds::tile16_key32_bits(L1_, table_.max_abs(), max_l2);
    }
    return pv;
  }
  dev::ProblemView problem_view(int64_t max_l2) const;
  void ensure(void*& ptr, size_t& cap, size_t bytes);
  void ensure_host(void*& ptr, size_t& cap, size_t bytes);
  bool direct_pointers(const WireBatch& b, void* out, int fb, dev::ShortArgs& a) const;
  bool prepare_direct(const dev::ProblemView& pv, const dev::ShortArgs& a, bool swipe);
  void launch_direct(const dev::ProblemView& pv, const dev::ShortArgs& a, bool swipe, bool graph);
  void run_staged(const uint8_t* codes, const int64_t* offsets, int64_t n, void* out, ResultFormat fmt,
                  bool packed5);
  void solve_wire_impl(const WireBatch& b, void* out, ResultFormat fmt, bool async);

  EngineOptions opt_;
  int device_ = 0;
  int num_cus_ = 256;
  int tile_u_ = 0;              // tile-kernel sub-tiles per wave tile (0 = per batch; MOC_TILE_U = 1|2|4)
  bool tile16_window_wide_ = true;  // widened windows for short records where the widened whole image is too big
  bool short_window_u8_ = true;     // ... with 8 sub-tiles per wave tile (MOC_TILE16_WIN_U8=0: 4)
  bool tile16_slide_ = true;        // long records past the widened image: sliding windows (MOC_TILE16_SLIDE=0: not)
  int slide_wgs_per_cu_ = 2;        // ... two workgroups per CU, half-LDS windows (MOC_TILE16_SLIDE_WG=1: one)
  int tile_waves_per_cu_ = 32;  // tile-kernel waves per CU (MOC_TILE_WAVES_PER_CU)
  hipStream_t s_copy_ = nullptr, s_compute_ = nullptr, s_return_ = nullptr;  // copy / return: made on first use
  void ensure_side_streams();
  // problem
  ScoreTable table_{};
  int32_t min_t_ = 0, max_t_ = 0;  // pair-score range over letters (R2 parameters)
  R2Params r2_{};                  // R2 parameters of the current solve
  void* d_image_ = nullptr;  // problem image: LUT | Seq1 | profile (views below)
  size_t d_image_cap_ = 0;
  // page-locked staging of the image: the upload is one copy kernel on the compute stream (dev::launch_copy;
  // a pageable hipMemcpy, or any copy the runtime gives its SDMA engine, cost 8-34 ms of engine start-up
  // inside a tiny job's first search on the box, profiles/copy_path_probe.log)
  void* h_image_ = nullptr;
  size_t h_image_cap_ = 0;
  std::vector<uint8_t> image_;
  Weights last_w_{};                // the last set_problem's inputs: a repeat returns at once
  std::vector<uint8_t> last_seq1_;
  int32_t* d_lut_ = nullptr;
  uint8_t* d_seq1_ = nullptr;
  uint16_t* d_prof16_ = nullptr;  // tile16 profile (null: the problem does not fit it, or MOC_TILE16=0)
  int32_t prof16_bytes_ = 0;
  int32_t prof16_overhang_ = 0;  // zero profile entries past the last row (bounds the tile span)
  int32_t prof16_window_ = 0;    // > 0: windowed tile16 (columns per workgroup window; Seq1 > one LDS image)
  int64_t prof16_entries_ = 0;   // entries of the device profile (windowed staging bounds)
  int32_t prof16_lds_bytes_ = 0; // LDS bytes of the profile part of a workgroup's image
  bool prof16_wide_ = false;      // the sweep stages widened int16 pairs (dev::ProblemView::prof16_wide)
  bool prof16_i16_ = false;       // the profile holds one int16 Dt per entry (dev::ProblemView::prof16_i16)
  bool tile16_ = true;            // MOC_TILE16 (A/B switch of the long-record kernel)
  bool mfma_ = false;             // MOC_MFMA: tile16 plans swept on the matrix cores (tile_mfma_kernels.hip)
  int64_t L1_ = 0;
  Semantics sem_ = Semantics::Reference;
  bool have_problem_ = false;
  std::vector<std::unique_ptr<Slot>> slots_;
  unsigned* d_counter_ = nullptr;  // direct-path work counter
  hipEvent_t ev_a_ = nullptr, ev_b_ = nullptr;
  // scratch for solve_device
  void* d_plan_ = nullptr;
  size_t d_plan_cap_ = 0;
  void* h_plan_ = nullptr;
  size_t h_plan_cap_ = 0;
  hipEvent_t ev_plan_ = nullptr;
  hipEvent_t ev_d0_ = nullptr, ev_d1_ = nullptr;  // around solve_device's launches (device_kernel_ms)
  std::vector<void*> pinned_;
  struct DirectKey {
    dev::ProblemView pv;
    dev::ShortArgs a;
    int32_t swipe;
  };
  static constexpr int kGraphs = 2;
  DirectKey graph_key_[kGraphs]{};
  hipGraphExec_t graph_exec_[kGraphs] = {nullptr, nullptr};
  int graph_cur_ = 0;
  // the last two argument sets launched without a graph (captured when seen again; a streaming job's ring
  // alternates two)
  DirectKey seen_key_[kGraphs]{};
  bool seen_valid_[kGraphs] = {false, false};
  int seen_next_ = 0;
  bool pending_ = false;  // a begin_wire solve is in flight (ev_a_ .. ev_b_)
  Stopwatch pending_wall_;
  EngineStats stats_;
};

// Picks the int32 hot-loop key width for a problem: bits for k, or 0 (=> 64-bit keys) when
// 2*max|T|*L2 does not fit next to them in an int32.
int32_t choose_key_shift(int32_t max_abs_weight, int64_t max_l2);

}  // namespace moc
