// Work decomposition across ranks.
//
// Reference (main.c:110-121, 141-146, 183-185): rows = N/p (or 1 when p >= N), the root takes the
// remainder in a second pass. Broken for p > N (scatter over-read + gather heap overflow, bug B5),
// for remain > rows (B6), and badly imbalanced (per-record cost varies 5000x on input3/input4).
//
// Here: contiguous ranges (so the gather is already in input order) balanced by a cost model
// cost_j = cell_w * cells(L1, L2_j) + byte_w * L2_j + record_w. Valid for any p >= 1, including
// p > N (trailing ranks get empty ranges) and N == 0.
#pragma once

#include <cstdint>
#include <vector>

#include "moc/problem.hpp"

namespace moc {

struct CostModel {
  double cell_w = 1.0;     // search work
  double byte_w = 4.0;     // transfer / parse work per letter
  double record_w = 64.0;  // fixed per-record overhead (result write, launch share)
};

double record_cost(int64_t L1, int64_t L2, const CostModel& m);

// Returns parts+1 boundaries b[0]=0 <= ... <= b[parts]=N; rank r owns records [b[r], b[r+1]).
std::vector<int64_t> partition_by_cost(const int64_t* lengths, int64_t n, int64_t L1, int parts,
                                       const CostModel& m = {});
// The same split from CSR offsets (record i = [offsets[i], offsets[i+1])), without a lengths copy.
std::vector<int64_t> partition_by_cost_offsets(const int64_t* offsets, int64_t n, int64_t L1, int parts,
                                               const CostModel& m = {});
std::vector<int64_t> partition_batch(const RecordBatch& batch, int64_t L1, int parts, const CostModel& m = {});

// Equal-count split (reference-like but correct for any p).
std::vector<int64_t> partition_even(int64_t n, int parts);

}  // namespace moc
