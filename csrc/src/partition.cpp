#include "moc/partition.hpp"

#include <omp.h>

#include <algorithm>

namespace moc {

double record_cost(int64_t L1, int64_t L2, const CostModel& m) {
  return m.cell_w * static_cast<double>(record_cells(L1, L2)) + m.byte_w * static_cast<double>(L2) + m.record_w;
}

namespace {
// Cost-balanced split over records whose lengths come from `len(i)`. Small inputs: one serial prefix
// scan. Large ones (a 10^8-record batch costs ~1 s serially): per-thread chunk sums, then each split
// rescans only the chunk that holds its target. Both place split r at the first index whose cost prefix
// reaches total*r/parts, or the index before it when that prefix is closer.
template <class Len>
std::vector<int64_t> partition_cost_impl(Len len, int64_t n, int64_t L1, int parts, const CostModel& m) {
  if (parts < 1) parts = 1;
  std::vector<int64_t> b(static_cast<size_t>(parts) + 1, 0);
  b[parts] = n;
  if (parts == 1 || n <= 0) return b;
  const int nt = n > (int64_t{1} << 20) ? std::max(1, omp_get_max_threads()) : 1;
  std::vector<double> csum(static_cast<size_t>(nt) + 1, 0.0);
  auto chunk_begin = [&](int t) { return n * t / nt; };
#pragma omp parallel for num_threads(nt) schedule(static, 1)
  for (int t = 0; t < nt; ++t) {
    double s = 0.0;
    for (int64_t i = chunk_begin(t); i < chunk_begin(t + 1); ++i) s += record_cost(L1, len(i), m);
    csum[t + 1] = s;
  }
  for (int t = 0; t < nt; ++t) csum[t + 1] += csum[t];  // chunk t starts at prefix csum[t]
  const double total = csum[nt];
  for (int r = 1; r < parts; ++r) {
    const double target = total * r / parts;
    int64_t idx = n;
    if (target <= 0.0) {
      idx = 0;
    } else {
      const int t = static_cast<int>(std::lower_bound(csum.begin() + 1, csum.end(), target) - csum.begin()) - 1;
      if (t < nt) {
        idx = chunk_begin(t + 1);  // rounding: the rescan may end a hair short of the chunk sum
        double acc = csum[t];
        for (int64_t i = chunk_begin(t); i < chunk_begin(t + 1); ++i) {
          const double next = acc + record_cost(L1, len(i), m);
          if (next >= target) {
            idx = (target - acc) < (next - target) ? i : i + 1;
            break;
          }
          acc = next;
        }
      }
    }
    b[r] = std::clamp<int64_t>(idx, b[r - 1], n);
  }
  return b;
}
}  // namespace

std::vector<int64_t> partition_by_cost(const int64_t* lengths, int64_t n, int64_t L1, int parts,
                                       const CostModel& m) {
  return partition_cost_impl([lengths](int64_t i) { return lengths[i]; }, n, L1, parts, m);
}

std::vector<int64_t> partition_by_cost_offsets(const int64_t* offsets, int64_t n, int64_t L1, int parts,
                                               const CostModel& m) {
  return partition_cost_impl([offsets](int64_t i) { return offsets[i + 1] - offsets[i]; }, n, L1, parts, m);
}

std::vector<int64_t> partition_batch(const RecordBatch& batch, int64_t L1, int parts, const CostModel& m) {
  std::vector<int64_t> len(static_cast<size_t>(batch.size()));
  for (int64_t i = 0; i < batch.size(); ++i) len[i] = batch.length(i);
  return partition_by_cost(len.data(), batch.size(), L1, parts, m);
}

std::vector<int64_t> partition_even(int64_t n, int parts) {
  if (parts < 1) parts = 1;
  std::vector<int64_t> b(static_cast<size_t>(parts) + 1);
  for (int r = 0; r <= parts; ++r) b[r] = n * r / parts;
  return b;
}

}  // namespace moc
