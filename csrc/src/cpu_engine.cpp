#include "moc/cpu_engine.hpp"

#include <string>

#include <omp.h>

#include <algorithm>
#include <vector>

namespace moc {

int64_t candidate_offsets(int64_t L1, int64_t L2, Semantics sem) {
  if (L2 > L1 || L2 <= 0) return 0;
  if (L2 == L1) return 1;
  return sem == Semantics::Spec ? L1 - L2 + 1 : L1 - L2;
}

namespace {

inline void consider(Result& best, int32_t score, int64_t o, int64_t k) {
  Result c{score, static_cast<int32_t>(o), static_cast<int32_t>(k)};
  if (best.n < 0 || better(c, best)) best = c;
}

}  // namespace

Result solve_offsets(const ScoreTable& t, const uint8_t* s1, int64_t L1, const uint8_t* s2, int64_t L2,
                     int64_t o_begin, int64_t o_end, Semantics sem) {
  Result best{kNoCandidateScore, -1, -1};
  const int64_t n_off = candidate_offsets(L1, L2, sem);
  o_end = std::min(o_end, n_off);
  if (o_begin >= o_end) return best;
  if (L2 == L1) {  // equal lengths: un-shifted, un-mutated only (cudaFunctions.cu:74-106)
    int32_t s = 0;
    for (int64_t i = 0; i < L2; ++i) s += t.lut[s2[i] * kLutStride + s1[i]];
    consider(best, s, 0, 0);
    return best;
  }
  const int64_t last_mut_off = L1 - L2;  // offsets with a hyphen need o + L2 + 1 <= L1
  // per-thread scratch (no allocation per record): LUT row of every Seq2 letter, and P_o(1..L2) of the
  // current diagonal; each offset then takes ONE fused pass over its neighbour diagonal: prefix
  // P_{o+1}(i+1), difference D_o(i+1) = P_o(i+1) - P_{o+1}(i+1) and its running max (strict '>': the
  // smallest k wins ties, as the reference loop order does)
  thread_local std::vector<const int32_t*> rows;
  thread_local std::vector<int32_t> cur;
  if (static_cast<int64_t>(rows.size()) < L2) rows.resize(static_cast<size_t>(L2));
  if (static_cast<int64_t>(cur.size()) < L2 + 1) cur.resize(static_cast<size_t>(L2) + 1);
  for (int64_t i = 0; i < L2; ++i) rows[i] = t.lut.data() + s2[i] * kLutStride;
  const int32_t* const* rw = rows.data();
  int32_t* P = cur.data();
  {
    int32_t acc = 0;
    const uint8_t* a = s1 + o_begin;
    for (int64_t i = 0; i < L2; ++i) P[i + 1] = acc += rw[i][a[i]];
  }
  for (int64_t o = o_begin; o < o_end; ++o) {
    consider(best, P[L2], o, 0);
    if (o >= last_mut_off) continue;
    const uint8_t* a = s1 + o + 1;
    int32_t q = 0, bd = INT32_MIN;
    int64_t bk = 0;
    for (int64_t i = 0; i + 1 < L2; ++i) {  // candidates k = i + 1 = 1 .. L2-1
      q += rw[i][a[i]];
      const int32_t d = P[i + 1] - q;
      P[i + 1] = q;  // becomes P_{o+1}(i+1) for the next offset
      if (d > bd) {
        bd = d;
        bk = i + 1;
      }
    }
    q += rw[L2 - 1][a[L2 - 1]];
    P[L2] = q;  // Tot_{o+1}
    if (L2 >= 2) consider(best, bd + q, o, bk);
  }
  return best;
}

Result solve_record(const ScoreTable& t, const uint8_t* s1, int64_t L1, const uint8_t* s2, int64_t L2,
                    Semantics sem) {
  Result r = solve_offsets(t, s1, L1, s2, L2, 0, L1 + 1, sem);
  return r.n < 0 ? no_candidate() : r;
}

namespace {
// Threads worth waking for `cells` of search work: a thread per ~0.25 M cells (~0.5 ms at the engine's
// rate), so a reference-sized job (input6: 730 cells) runs on the calling thread without forking a team —
// the team's start-up and spin-down cost more than the whole search (49-63 ms vs 26 ms).
int threads_for(const RecordBatch& batch, int64_t L1, Semantics sem, int nt) {
  if (nt <= 1) return 1;
  const int64_t n = batch.size();
  int64_t cells = 0;
  for (int64_t i = 0; i < n && cells < int64_t{nt} << 18; ++i)
    cells += candidate_offsets(L1, batch.length(i), sem) * std::max<int64_t>(batch.length(i), 1);
  return static_cast<int>(std::clamp<int64_t>(cells >> 18, 1, nt));
}
}  // namespace

void solve_batch_cpu(const ScoreTable& t, const uint8_t* s1, int64_t L1, const RecordBatch& batch, Result* out,
                     Semantics sem, int num_threads) {
  const int64_t n = batch.size();
  const int nt = threads_for(batch, L1, sem, num_threads > 0 ? num_threads : omp_get_max_threads());
  if (n >= 4 * nt || nt == 1) {
    // dynamic balance in chunks: per-record dispatch would dominate tiny records (input6: ~150 cells)
    const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(1024, n / (64 * nt)));
#pragma omp parallel for schedule(dynamic, chunk) num_threads(nt) if (nt > 1)
    for (int64_t i = 0; i < n; ++i) out[i] = solve_record(t, s1, L1, batch.record(i), batch.length(i), sem);
    return;
  }
  // Few records: split every record's offset range into chunks and run all (record, chunk) items in ONE
  // parallel loop (one fork/join for the batch, dynamic balance), then merge per record — max is
  // order-free, so the result does not depend on the thread count.
  struct Item {
    int64_t rec, ob, oe;
  };
  std::vector<Item> items;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t n_off = candidate_offsets(L1, batch.length(i), sem);
    const int64_t chunk = std::max<int64_t>(16, (n_off + 4 * nt - 1) / (4 * nt));
    if (n_off <= 1) {
      items.push_back(Item{i, 0, L1 + 1});
      continue;
    }
    for (int64_t ob = 0; ob < n_off; ob += chunk) items.push_back(Item{i, ob, std::min(n_off, ob + chunk)});
  }
  std::vector<Result> part(items.size());
#pragma omp parallel for schedule(dynamic, 1) num_threads(nt) if (nt > 1)
  for (int64_t j = 0; j < static_cast<int64_t>(items.size()); ++j) {
    const Item& it = items[j];
    part[j] = solve_offsets(t, s1, L1, batch.record(it.rec), batch.length(it.rec), it.ob, it.oe, sem);
  }
  for (int64_t i = 0; i < n; ++i) out[i] = Result{kNoCandidateScore, -1, -1};
  for (size_t j = 0; j < items.size(); ++j) {
    Result& b = out[items[j].rec];
    const Result& p = part[j];
    if (p.n >= 0 && (b.n < 0 || better(p, b))) b = p;
  }
  for (int64_t i = 0; i < n; ++i)
    if (out[i].n < 0) out[i] = no_candidate();
}

void solve_keys_cpu(const ScoreTable& t, const uint8_t* s1, int64_t L1, const RecordBatch& batch, int part,
                    int parts, uint64_t* keys, Semantics sem, int num_threads) {
  if (parts < 1 || part < 0 || part >= parts) throw Error("solve_keys_cpu: bad part");
  const int64_t n = batch.size();
  const int nt = threads_for(batch, L1, sem, num_threads > 0 ? num_threads : omp_get_max_threads());
  auto range = [&](int64_t i, int64_t& b, int64_t& e) {
    const int64_t c = candidate_offsets(L1, batch.length(i), sem);
    b = c * part / parts;
    e = c * (part + 1) / parts;
  };
  if (n >= 4 * nt || nt == 1) {
    const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(1024, n / (64 * nt)));
#pragma omp parallel for schedule(dynamic, chunk) num_threads(nt) if (nt > 1)
    for (int64_t i = 0; i < n; ++i) {
      int64_t b, e;
      range(i, b, e);
      const int64_t L2 = batch.length(i);
      keys[i] = encode_key(solve_offsets(t, s1, L1, batch.record(i), L2, b, e, sem));
    }
    return;
  }
  // few records: this part's range of every record in chunks, one parallel loop for the batch
  struct Item {
    int64_t rec, ob, oe;
  };
  std::vector<Item> items;
  for (int64_t i = 0; i < n; ++i) {
    int64_t b, e;
    range(i, b, e);
    const int64_t chunk = std::max<int64_t>(16, (e - b + 4 * nt - 1) / (4 * nt));
    for (int64_t ob = b; ob < e; ob += chunk) items.push_back(Item{i, ob, std::min(e, ob + chunk)});
  }
  std::vector<uint64_t> pk(items.size());
#pragma omp parallel for schedule(dynamic, 1) num_threads(nt) if (nt > 1)
  for (int64_t j = 0; j < static_cast<int64_t>(items.size()); ++j) {
    const Item& it = items[j];
    const int64_t L2 = batch.length(it.rec);
    pk[j] = encode_key(solve_offsets(t, s1, L1, batch.record(it.rec), L2, it.ob, it.oe, sem));
  }
  for (int64_t i = 0; i < n; ++i) keys[i] = 0;
  for (size_t j = 0; j < items.size(); ++j) keys[items[j].rec] = std::max(keys[items[j].rec], pk[j]);
}

Result brute_force_record(const ScoreTable& t, const uint8_t* s1, int64_t L1, const uint8_t* s2, int64_t L2,
                          Semantics sem) {
  if (L2 > L1) return no_candidate();
  if (L2 == L1) {
    int32_t s = 0;
    for (int64_t i = 0; i < L2; ++i) s += t.lut[s2[i] * kLutStride + s1[i]];
    return Result{s, 0, 0};
  }
  Result best{kNoCandidateScore, 0, 0};
  bool have = false;
  for (int64_t o = 0; o < L1 - L2; ++o) {
    for (int64_t m = 0; m < L2; ++m) {
      int32_t s = 0;
      for (int64_t i = 0; i < L2; ++i) {
        const int64_t j = (i < m || m == 0) ? i + o : i + o + 1;
        s += t.lut[s2[i] * kLutStride + s1[j]];
      }
      if (!have || best.score < s) {
        best = Result{s, static_cast<int32_t>(o), static_cast<int32_t>(m)};
        have = true;
      }
    }
  }
  if (sem == Semantics::Spec) {
    int32_t s = 0;
    const int64_t o = L1 - L2;
    for (int64_t i = 0; i < L2; ++i) s += t.lut[s2[i] * kLutStride + s1[i + o]];
    if (!have || best.score < s) best = Result{s, static_cast<int32_t>(o), 0};
  }
  return best;
}

Result resolve_key(const ScoreTable& t, const uint8_t* s1, int64_t L1, const uint8_t* s2, int64_t L2, uint64_t key) {
  if (key == 0) return no_candidate();
  const int32_t score = static_cast<int32_t>(static_cast<uint32_t>(key >> 32) ^ 0x80000000u);
  const uint32_t idx = 0xffffffffu - static_cast<uint32_t>(key);
  const int64_t o = idx >> 1;
  if (!(idx & 1u)) return Result{score, static_cast<int32_t>(o), 0};
  if (o + L2 >= L1) throw Error("resolve_key: a mutated candidate needs o + L2 < L1");
  // score = D_o(k) + Tot_{o+1}; the smallest k in 1..L2-1 with that value
  int64_t tot1 = 0;
  for (int64_t i = 0; i < L2; ++i) tot1 += t.score(s2[i], s1[o + 1 + i]);
  int64_t d = 0;
  for (int64_t k = 1; k < L2; ++k) {
    d += t.score(s2[k - 1], s1[o + k - 1]) - t.score(s2[k - 1], s1[o + k]);
    if (d + tot1 == score) return Result{score, static_cast<int32_t>(o), static_cast<int32_t>(k)};
  }
  throw Error("resolve_key: no k on diagonal " + std::to_string(o) + " reaches the key's score");
}

}  // namespace moc
