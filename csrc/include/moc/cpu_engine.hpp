// CPU (OpenMP) search engine — the "GPU kernel stubbed" backend of BASELINE.json config 1, and the
// C++ test oracle for the HIP kernels.
//
// Reference semantics (cudaFunctions.cu:63-176, race-free reading):
//   score(o, 0)  = sum_i T[s2_i][s1_{i+o}]                                  (no hyphen)
//   score(o, k)  = sum_{i<k} T[s2_i][s1_{i+o}] + sum_{i>=k} T[s2_i][s1_{i+o+1}],  k = 1..L2-1
//   offsets o in [0, L1-L2) (exclusive, :116), ties -> first in offset-major / mutant-minor order
//   (strict `max <` at :161); L2 == L1 -> (0,0) only (:74-106); L2 > L1 -> (INT_MIN, 0, 0).
// Closed form used here: with P_d(k) = sum_{i<k} T[s2_i][s1_{i+d}] and Tot_d = P_d(L2),
//   score(o, k>=1) = P_o(k) - P_{o+1}(k) + Tot_{o+1}  -> O(L1*L2) instead of O(L1*L2^2).
#pragma once

#include <cstdint>

#include "moc/common.hpp"
#include "moc/problem.hpp"
#include "moc/score_table.hpp"

namespace moc {

// Lexicographic "better than" for candidates: higher score, then smaller offset, then smaller k
// (k == 0 is the un-mutated sequence and comes first inside an offset, as in the reference loop).
inline bool better(const Result& a, const Result& b) {
  if (a.score != b.score) return a.score > b.score;
  if (a.n != b.n) return a.n < b.n;
  return a.k < b.k;
}

// Best candidate for one record restricted to offsets [o_begin, o_end) of the full candidate set.
// Returns {kNoCandidateScore, -1, -1} when the range holds no candidate.
Result solve_offsets(const ScoreTable& t, const uint8_t* s1, int64_t L1, const uint8_t* s2, int64_t L2,
                     int64_t o_begin, int64_t o_end, Semantics sem);

// Number of offsets in the candidate set of a record (reference: L1-L2, spec: L1-L2+1; 1 if equal).
int64_t candidate_offsets(int64_t L1, int64_t L2, Semantics sem);

// Full search for one record.
Result solve_record(const ScoreTable& t, const uint8_t* s1, int64_t L1, const uint8_t* s2, int64_t L2,
                    Semantics sem);

// Batch search (OpenMP). Records [0, batch.size()) -> out[0..N). Parallel over records when there are
// many, over offset ranges of each record when there are few (the "context-parallel" split, §5.7).
void solve_batch_cpu(const ScoreTable& t, const uint8_t* s1, int64_t L1, const RecordBatch& batch, Result* out,
                     Semantics sem, int num_threads = 0);

// ---- packed candidate keys: the context-parallel combine
// PASS-1 key = (score ^ 2^31) << 32 | (2^32 - 1 - (2n + mutated)); 0 = "no candidate". The unsigned max
// over keys is the reference's winner up to its k (higher score, then smaller offset, then the un-mutated
// candidate first), so partial searches over disjoint offset ranges combine with one MAX reduction
// (MPI_Allreduce / ncclAllReduce, UINT64); resolve_key then finds k on the winning diagonal (the smallest k
// with that score — the reference's order inside an offset). No o*L2 + k index: L1 * L2 may exceed 2^32.
// Identical to the device encoding (csrc/src/hip/kernel_common.hpp lane_pass1_candidate, resolve_long_kernel).
inline uint64_t encode_key(const Result& r) {
  if (r.n < 0 || r.score == kNoCandidateScore) return 0;
  const uint32_t idx = 2u * static_cast<uint32_t>(r.n) + (r.k > 0 ? 1u : 0u);
  return (static_cast<uint64_t>(static_cast<uint32_t>(r.score) ^ 0x80000000u) << 32) | (0xffffffffu - idx);
}
// The result a MAX-combined key stands for (record s2 of length L2 against Seq1 s1): O(L2).
Result resolve_key(const ScoreTable& t, const uint8_t* s1, int64_t L1, const uint8_t* s2, int64_t L2, uint64_t key);

// Part `part` of `parts` of every record's candidate set (offsets [C*part/parts, C*(part+1)/parts) of
// its C candidate offsets) -> keys[i] (0 where the part holds no candidate). max over all parts of
// keys[i] == encode_key(solve_record(i)).
void solve_keys_cpu(const ScoreTable& t, const uint8_t* s1, int64_t L1, const RecordBatch& batch, int part,
                    int parts, uint64_t* keys, Semantics sem, int num_threads = 0);

// Literal O(L1*L2^2) emulation of calc_result's loops (cudaFunctions.cu:74-172), race-free.
// Test oracle only.
Result brute_force_record(const ScoreTable& t, const uint8_t* s1, int64_t L1, const uint8_t* s2, int64_t L2,
                          Semantics sem);

}  // namespace moc
