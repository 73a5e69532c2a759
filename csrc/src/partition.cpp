#include "moc/partition.hpp"

#include <algorithm>

namespace moc {

double record_cost(int64_t L1, int64_t L2, const CostModel& m) {
  return m.cell_w * static_cast<double>(record_cells(L1, L2)) + m.byte_w * static_cast<double>(L2) + m.record_w;
}

std::vector<int64_t> partition_by_cost(const int64_t* lengths, int64_t n, int64_t L1, int parts,
                                       const CostModel& m) {
  if (parts < 1) parts = 1;
  std::vector<double> prefix(static_cast<size_t>(n) + 1, 0.0);
  for (int64_t i = 0; i < n; ++i) prefix[i + 1] = prefix[i] + record_cost(L1, lengths[i], m);
  const double total = prefix[n];
  std::vector<int64_t> b(static_cast<size_t>(parts) + 1, 0);
  b[parts] = n;
  for (int r = 1; r < parts; ++r) {
    const double target = total * r / parts;
    // first index whose prefix reaches the target; pick the closer of the two neighbours
    int64_t i = std::lower_bound(prefix.begin(), prefix.end(), target) - prefix.begin();
    if (i > 0 && (target - prefix[i - 1]) < (prefix[std::min(i, n)] - target)) --i;
    i = std::clamp<int64_t>(i, b[r - 1], n);
    b[r] = i;
  }
  return b;
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
