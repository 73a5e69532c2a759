// Device (gfx950) launch API for the alignment-search kernels.
//
// Reference: ONE kernel launch per Seq2 record (cudaFunctions.cu:204-220), each followed by
// cudaDeviceSynchronize, launched with grid = ceil(rows*2000/1024) blocks of which at most two hold
// work, with a serial (offset, mutant) loop inside every thread (cudaFunctions.cu:116-167).
//
// Here: one launch per *batch*. Parallelism is over offsets (diagonals): every lane owns one offset
// `o` and streams over the Seq2 positions, keeping its running diagonal prefix sum P_o in a register;
// the neighbour diagonal's P_{o+1} comes from lane+1 through a DPP wave shift, so a cell costs one LDS
// LUT gather plus a handful of VALU ops and no atomics/barriers (design: SURVEY.md §7.3).
//   * packed kernel: records whose offset range fits in a wave (L1-L2+1 <= 64 lanes) are packed
//     several per wave in fixed-width lane slots (the input6-shaped regime);
//   * tile kernel: longer offset ranges are cut into 63-offset tiles (lane 63 is the helper diagonal)
//     listed by the host planner; partial maxima merge through one 64-bit atomicMax per wave on an
//     order-free packed key (score, -(o*L2+k)) — deterministic tie-break, no races (fixes B9).
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>

#include "moc/common.hpp"

namespace moc {
namespace dev {

constexpr int kWave = 64;
constexpr int kTileOffsets = 63;  // owned offsets per tile-kernel wave (lane 63 = helper diagonal)
constexpr int kSeq1Pad = 256;     // zero padding after Seq1 on device (branch-free over-reads)

// Problem resident on the device (uploaded once per problem; tiny).
struct ProblemView {
  const int32_t* lut;   // [32*32] fused pair scores
  const uint8_t* seq1;  // codes, L1 + kSeq1Pad bytes (padding = 0)
  int32_t L1;
  int32_t semantics;    // moc::Semantics
  int32_t key_shift;    // bits reserved for k in the int32 hot-loop key (0 -> 64-bit keys)
};

// One batch of records on the device. Offsets are absolute (int64) and rebased by offsets[0], so
// a chunk of a bigger CSR array can be transferred and launched without host-side rebasing.
struct BatchView {
  const uint8_t* codes;     // codes of this chunk (codes[0] == record 0's first letter)
  const int64_t* offsets;   // n+1 absolute offsets
  int64_t n;
};

// One tile-kernel work item: index into Plan::long_recs and the tile's first offset.
struct Tile {
  int32_t li;
  int32_t o0;
};

// Host-built launch plan for one batch (see planner in hip_engine.cpp).
struct Plan {
  int32_t slot = 0;           // lanes per record in the packed kernel (0 = no packed records)
  int32_t rec_per_wave = 0;   // floor(64 / slot)
  int64_t n_tiles = 0;        // tile-kernel work items
  const Tile* tiles = nullptr;      // device: (long-record index, first offset) per tile
  const int32_t* long_recs = nullptr;  // device: records handled by the tile kernel
  int64_t n_long = 0;
  unsigned long long* keys = nullptr;  // device scratch, n_long entries (tile-kernel partial maxima)
  int* debug = nullptr;                // optional per-lane dump of one tile (debug builds/tools only)
};

// Lanes a record needs in the packed kernel (offsets 0..L1-L2 incl. the helper diagonal).
inline int64_t lanes_needed(int64_t L1, int64_t L2) { return L2 <= L1 ? L1 - L2 + 1 : 1; }

// Launches packed + tile + finalize kernels for one batch on `stream`; results -> out[0..n).
void launch_search(const ProblemView& pv, const BatchView& bv, const Plan& plan, Result* out,
                   hipStream_t stream);

// One-wave self-test of the DPP / shuffle primitives (192 ints, see align_kernels.hip).
void launch_dpp_probe(int* d_out, hipStream_t stream);

// Transfer calibration in GB/s (kinds: transfer_probe.hip). Allocates/frees its own buffers.
double transfer_probe(int kind, size_t bytes, int iters);

}  // namespace dev
}  // namespace moc
