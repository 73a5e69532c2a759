// Native unit tests of the host core (SURVEY.md §4.3 "unit (C++)"): score table vs the spec groups,
// parser and streaming reader edge cases, partitioner, packed-key ordering, 5-bit packing, CPU engine vs
// the brute-force replay of the reference loops. No GPU, no MPI. Run: `make unit` or `ctest`.
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <memory>
#include <random>
#include <string>
#include <vector>

#include "moc/cpu_engine.hpp"
#include "moc/device.hpp"
#include "moc/io.hpp"
#include "moc/kernel_bounds.hpp"
#include "moc/partition.hpp"
#include "moc/problem.hpp"
#include "moc/runtime/kfd_topology.hpp"
#include "moc/runtime/releaser.hpp"
#include "moc/runtime/watchdog.hpp"
#include "moc/score_table.hpp"
#include "moc/wire.hpp"
#include "../apps/text_cut.hpp"

using namespace moc;

namespace {
int g_failed = 0, g_checks = 0;

#define CHECK(cond)                                                              \
  do {                                                                           \
    ++g_checks;                                                                  \
    if (!(cond)) {                                                               \
      ++g_failed;                                                                \
      std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #cond); \
    }                                                                            \
  } while (0)

template <typename F>
bool throws(F f, const char* needle) {
  try {
    f();
  } catch (const Error& e) {
    return std::strstr(e.what(), needle) != nullptr;
  }
  return false;
}

bool in_any_group(const std::vector<std::string>& groups, char a, char b) {
  for (const auto& g : groups)
    if (g.find(a) != std::string::npos && g.find(b) != std::string::npos) return true;
  return false;
}

void test_score_table() {
  const Weights w{{10, 2, 3, 4}};
  const ScoreTable t = ScoreTable::build(w);
  for (char a = 'A'; a <= 'Z'; ++a)
    for (char b = 'A'; b <= 'Z'; ++b) {
      const int x = a - 'A' + 1, y = b - 'A' + 1;
      PairClass want = kSpace;
      if (a == b) want = kDollar;
      else if (in_any_group(first_type_groups(), a, b)) want = kPercent;
      else if (in_any_group(second_type_groups(), a, b)) want = kHash;
      CHECK(t.pair_class(x, y) == want);
      CHECK(t.pair_class(x, y) == t.pair_class(y, x));
      const int32_t s = t.lut[x * kLutStride + y];
      CHECK(s == (want == kDollar ? 10 : want == kPercent ? -2 : want == kHash ? -3 : -4));
    }
  CHECK(t.max_abs() == 10);
}

void test_parser() {
  const std::string text = "10 2 3 4\r\napqrsbatav\r\n  2\r\n asqreavsl \r\n\tHELLO\r\nEXTRA\n";
  Problem p = parse_problem(text.data(), text.size());
  CHECK(p.weights.w[0] == 10 && p.weights.w[3] == 4);
  CHECK(p.L1() == 10 && p.seq2.size() == 2);
  CHECK(p.seq2.length(0) == 9 && p.seq2.length(1) == 5);
  CHECK(p.seq2.record(1)[0] == letter_code('H'));
  CHECK(throws([] { parse_problem("1 2 3", 5); }, "W4"));
  CHECK(throws([] { std::string s = "1 2 3 4\nAB1C\n1\nAB\n"; parse_problem(s.data(), s.size()); }, "non-letter"));
  CHECK(throws([] { std::string s = "1 2 3 4\nABC\n3\nAB\nCD\n"; parse_problem(s.data(), s.size()); }, "expected 3"));
  CHECK(throws([] { std::string s = "1 -2 3 4\nABC\n1\nAB\n"; parse_problem(s.data(), s.size()); }, "out of range"));
  ParseOptions lim;
  lim.max_l2 = 3;
  CHECK(throws([&] { std::string s = "1 2 3 4\nABCDE\n1\nABCD\n"; parse_problem(s.data(), s.size(), lim); },
               "limit is 3"));
  std::string empty = "1 1 1 1\nABCD\n0\n";
  CHECK(parse_problem(empty.data(), empty.size()).seq2.size() == 0);
}

void test_stream_reader() {
  // records spanning refills of a tiny buffer, batches, skip, limits
  std::string text = "4 3 2 10\nABCDEFGHIJKLMNOPQRSTUVWXYZ\n7\n";
  std::vector<std::string> recs = {"ABCDEF", "xyz", "QRSTUVWXYZAB", "M", "LONGERRECORDABCDEFGHIJ", "AA", "ZZZ"};
  for (auto& r : recs) text += r + "\n";
  FILE* f = fmemopen(text.data(), text.size(), "rb");
  StreamReader rd(f, {}, 4096);
  CHECK(rd.count() == 7 && rd.seq1().size() == 26 && rd.weights().w[3] == 10);
  CHECK(rd.skip(1) == 1 && rd.next_index() == 1);
  RecordBatch b;
  CHECK(rd.next_batch(2, b) == 2);
  CHECK(b.size() == 2 && b.length(0) == 3 && b.length(1) == 12 && b.record(0)[0] == letter_code('X'));
  CHECK(rd.next_batch(100, b, 10) == 2);  // letter cap: stops after the batch reaches 10 letters
  CHECK(b.length(0) == 1 && b.length(1) == 22);
  CHECK(rd.next_batch(100, b) == 2);
  CHECK(rd.next_batch(100, b) == 0);
  std::fclose(f);
  std::string bad = "1 1 1 1\nABC\n3\nAB\nA1\nC\n";
  FILE* g = fmemopen(bad.data(), bad.size(), "rb");
  StreamReader rb(g);
  RecordBatch x;
  CHECK(rb.next_batch(1, x) == 1);
  CHECK(throws([&] { rb.next_batch(5, x); }, "record #1"));
  std::fclose(g);

  // multi-MB regions take the chunked OpenMP path: batches (record and letter caps, buffers smaller and
  // larger than a batch) must concatenate to exactly what the bulk parser produces
  std::mt19937 rng(3);
  std::string big = "5 1 2 3\nHELLOWORLD\n150000\n";
  const char* ws[5] = {"\n", " ", "\r\n", "  \t", "\n\n"};
  std::vector<size_t> rec_start;
  for (int i = 0; i < 150000; ++i) {
    rec_start.push_back(big.size());
    const int L = 1 + static_cast<int>(rng() % (i % 5000 == 0 ? 900 : 40));
    for (int j = 0; j < L; ++j) big += static_cast<char>((rng() % 2 ? 'A' : 'a') + rng() % 26);
    big += ws[rng() % 5];
  }
  big += "EXTRA TOKENS\n";
  const Problem ref = parse_problem(big.data(), big.size());
  for (const auto& cfg : std::vector<std::array<int64_t, 3>>{{int64_t{1} << 20, 1000, INT64_MAX},
                                                             {int64_t{4} << 20, 77777, INT64_MAX},
                                                             {int64_t{4} << 20, INT64_MAX, 500000},
                                                             {int64_t{2} << 20, 150000, 2000000},
                                                             {int64_t{8} << 20, INT64_MAX, INT64_MAX}}) {
    FILE* h = fmemopen(big.data(), big.size(), "rb");
    StreamReader sr(h, {}, static_cast<size_t>(cfg[0]));
    std::vector<uint8_t> codes;
    std::vector<int64_t> offs = {0};
    RecordBatch bb;
    int64_t batches = 0;
    bool caps_ok = true;
    while (int64_t k = sr.next_batch(cfg[1], bb, cfg[2])) {
      ++batches;
      caps_ok &= k <= cfg[1] && bb.size() == k;
      // the letter cap: every record but the first starts below it
      caps_ok &= bb.offsets[k - 1] < cfg[2] || k == 1;
      for (int64_t r = 0; r < k; ++r) offs.push_back(static_cast<int64_t>(codes.size()) + bb.offsets[r + 1]);
      codes.insert(codes.end(), bb.codes.begin(), bb.codes.end());
    }
    CHECK(caps_ok && batches >= 1);
    CHECK(std::equal(offs.begin(), offs.end(), ref.seq2.offsets.begin(), ref.seq2.offsets.end()) &&
          std::equal(codes.begin(), codes.end(), ref.seq2.codes.begin(), ref.seq2.codes.end()));
    std::fclose(h);
  }
  // a bad letter / an over-long record deep inside a chunked region: the smallest record is named,
  // and a length-limit violation in an earlier record wins over a later bad letter
  auto run_all = [&](std::string& text, int64_t cap) {
    FILE* h = fmemopen(text.data(), text.size(), "rb");
    ParseOptions o;
    o.max_l2 = cap;
    StreamReader sr(h, o, size_t{2} << 20);
    RecordBatch bb;
    std::string msg;
    try {
      while (sr.next_batch(40000, bb)) {
      }
    } catch (const Error& e) {
      msg = e.what();
    }
    std::fclose(h);
    return msg;
  };
  std::string bad2 = big;
  bad2[rec_start[123457]] = '7';
  CHECK(run_all(bad2, 0).find("record #123457 contains a non-letter") != std::string::npos);
  bad2[rec_start[70001]] = '#';
  CHECK(run_all(bad2, 0).find("record #70001 contains a non-letter") != std::string::npos);
  // records i % 5000 == 0 may be up to 900 letters long: with a cap of 45 the first such record over it
  int64_t first_long = -1;
  for (int64_t r = 0; r < 150000 && first_long < 0; ++r)
    if (ref.seq2.offsets[r + 1] - ref.seq2.offsets[r] > 45) first_long = r;
  CHECK(first_long >= 0);
  CHECK(run_all(big, 45).find("record #" + std::to_string(first_long) + " has") != std::string::npos);
}

void test_partition() {
  std::vector<int64_t> len = {10, 20, 5, 7, 1000, 3, 3, 3};
  for (int p : {1, 2, 3, 8, 13}) {
    auto b = partition_by_cost(len.data(), static_cast<int64_t>(len.size()), 1200, p);
    CHECK(static_cast<int>(b.size()) == p + 1 && b.front() == 0 && b.back() == static_cast<int64_t>(len.size()));
    for (int r = 0; r < p; ++r) CHECK(b[r] <= b[r + 1]);
    auto e = partition_even(static_cast<int64_t>(len.size()), p);
    CHECK(e.back() == static_cast<int64_t>(len.size()));
  }
  auto z = partition_by_cost(nullptr, 0, 10, 4);
  CHECK(z.size() == 5 && z.back() == 0);
  // large batches take the chunked OpenMP path: same splits as one serial prefix scan (+-1 for rounding)
  std::mt19937 rng(5);
  const int64_t n = 3000000, L1 = 1500;
  std::vector<int64_t> big(static_cast<size_t>(n)), offs(static_cast<size_t>(n) + 1, 0);
  for (int64_t i = 0; i < n; ++i) {
    big[i] = 1 + static_cast<int64_t>(rng() % (i % 1000 == 0 ? 1400 : 30));
    offs[i + 1] = offs[i] + big[i];
  }
  const CostModel cm{1.0, 200.0, 2400.0};
  std::vector<double> prefix(static_cast<size_t>(n) + 1, 0.0);
  for (int64_t i = 0; i < n; ++i) prefix[i + 1] = prefix[i] + record_cost(L1, big[i], cm);
  for (int p : {2, 3, 8, 13}) {
    auto b1 = partition_by_cost(big.data(), n, L1, p, cm);
    auto b2 = partition_by_cost_offsets(offs.data(), n, L1, p, cm);
    CHECK(b1 == b2);
    for (int r = 1; r < p; ++r) {
      const double target = prefix[n] * r / p;
      int64_t i = std::lower_bound(prefix.begin(), prefix.end(), target) - prefix.begin();
      if (i > 0 && (target - prefix[i - 1]) < (prefix[std::min(i, n)] - target)) --i;
      CHECK(std::llabs(b1[r] - i) <= 1);
    }
  }
}

void test_keys() {
  // pass-1 keys: higher score wins; then the smaller offset; then the un-mutated candidate (k = 0) first
  const uint64_t a = encode_key(Result{5, 2, 0}), b = encode_key(Result{5, 2, 4}), c = encode_key(Result{5, 1, 6}),
                 d = encode_key(Result{6, 9, 6}), e = encode_key(Result{-100, 0, 0});
  CHECK(a > b && c > a && d > c && e < a && e > 0);
  CHECK(encode_key(Result{5, 2, 3}) == encode_key(Result{5, 2, 4}));  // k is resolved afterwards
  CHECK(encode_key(no_candidate()) == 0);
  // resolve_key recovers the smallest k on the winning diagonal, also where o*L2 + k exceeds 32 bits
  const ScoreTable t = ScoreTable::build(Weights{{4, 3, 2, 10}});
  const Result none = resolve_key(t, nullptr, 10, nullptr, 3, 0);
  CHECK(none.score == kNoCandidateScore && none.n == 0 && none.k == 0);
  std::mt19937 rng(5);
  for (int trial = 0; trial < 4; ++trial) {
    const int64_t L1 = trial < 2 ? 60 : 70000, L2 = trial < 2 ? 17 : 65000;  // 70000 * 65000 > 2^32
    std::vector<uint8_t> s1(static_cast<size_t>(L1)), s2(static_cast<size_t>(L2));
    for (auto& x : s1) x = static_cast<uint8_t>(1 + rng() % 26);
    for (auto& x : s2) x = static_cast<uint8_t>(1 + rng() % 26);
    const Result full = solve_record(t, s1.data(), L1, s2.data(), L2, Semantics::Reference);
    const Result r = resolve_key(t, s1.data(), L1, s2.data(), L2, encode_key(full));
    CHECK(r.score == full.score && r.n == full.n && r.k == full.k);
  }
}

void test_pack5() {
  std::mt19937 rng(1);
  for (int64_t n : {0, 1, 7, 8, 9, 1000, 70000}) {
    std::vector<uint8_t> c(static_cast<size_t>(n));
    for (auto& x : c) x = static_cast<uint8_t>(1 + rng() % 26);
    std::vector<uint8_t> p(static_cast<size_t>(packed5_bytes(n)));
    pack5(c.data(), n, p.data());
    std::vector<uint8_t> u(static_cast<size_t>(n));
    unpack5(p.data(), 0, n, u.data());
    CHECK(u == c);
  }
}

void test_engine_vs_brute_force() {
  std::mt19937 rng(7);
  for (int trial = 0; trial < 60; ++trial) {
    const int64_t L1 = 1 + rng() % 40;
    Weights w{{static_cast<int32_t>(rng() % 12), static_cast<int32_t>(rng() % 12), static_cast<int32_t>(rng() % 12),
               static_cast<int32_t>(rng() % 12)}};
    const ScoreTable t = ScoreTable::build(w);
    std::vector<uint8_t> s1(static_cast<size_t>(L1));
    for (auto& x : s1) x = static_cast<uint8_t>(1 + rng() % 26);
    RecordBatch batch;
    for (int r = 0; r < 12; ++r) {
      const int64_t L2 = 1 + rng() % (L1 + 2);
      std::vector<uint8_t> s2(static_cast<size_t>(L2));
      for (auto& x : s2) x = static_cast<uint8_t>(1 + rng() % 26);
      batch.push_back(s2.data(), L2);
    }
    for (Semantics sem : {Semantics::Reference, Semantics::Spec}) {
      std::vector<Result> out(static_cast<size_t>(batch.size()));
      solve_batch_cpu(t, s1.data(), L1, batch, out.data(), sem, 2);
      for (int64_t i = 0; i < batch.size(); ++i) {
        const Result bf = brute_force_record(t, s1.data(), L1, batch.record(i), batch.length(i), sem);
        CHECK(out[i].score == bf.score && out[i].n == bf.n && out[i].k == bf.k);
      }
      // context-parallel shares combine to the same answers
      std::vector<uint64_t> keys(static_cast<size_t>(batch.size()), 0), part(keys.size());
      for (int p = 0; p < 3; ++p) {
        solve_keys_cpu(t, s1.data(), L1, batch, p, 3, part.data(), sem, 2);
        for (size_t i = 0; i < keys.size(); ++i) keys[i] = std::max(keys[i], part[i]);
      }
      for (int64_t i = 0; i < batch.size(); ++i) {
        const Result r = resolve_key(t, s1.data(), L1, batch.record(i), batch.length(i), keys[i]);
        CHECK(r.score == out[i].score && r.n == out[i].n && r.k == out[i].k);
      }
    }
  }
}

void test_pack33() {
  std::mt19937 rng(33);
  for (int64_t n : {0, 1, 6, 7, 8, 55, 56, 57, 112, 1000, 70001}) {
    std::vector<uint8_t> codes(static_cast<size_t>(n));
    for (auto& c : codes) c = static_cast<uint8_t>(1 + rng() % 26);
    if (n > 20) std::fill(codes.begin() + 7, codes.begin() + 21, uint8_t{26});  // largest fields
    std::vector<uint8_t> p(static_cast<size_t>(packed33_bytes(n)), 0xAB);
    pack33(codes.data(), n, p.data());
    bool slack_zero = true;
    for (size_t i = static_cast<size_t>(33 * ((n + 55) / 56)); i < p.size(); ++i) slack_zero &= p[i] == 0;
    CHECK(slack_zero);
    for (int64_t b : {int64_t{0}, int64_t{1}, int64_t{6}, int64_t{7}, int64_t{57}, n / 3}) {
      if (b > n) continue;
      std::vector<uint8_t> back(static_cast<size_t>(n - b));
      unpack33(p.data(), b, n - b, back.data());
      CHECK(std::equal(back.begin(), back.end(), codes.begin() + b));
    }
    // byte ranges of any letter range cover exactly its fields
    for (int64_t c0 : {int64_t{0}, int64_t{3}, int64_t{7}, int64_t{50}}) {
      if (c0 >= n) continue;
      CHECK(p33_first_byte(c0) == (33 * (c0 / 7)) / 8);
      CHECK(p33_end_byte(n) <= 33 * ((n + 55) / 56) + 1);
    }
  }
  const uint8_t seven[7] = {26, 26, 26, 26, 26, 26, 26};
  CHECK(p33_field(seven) == 8031810175ull);  // 26^7 - 1 < 2^33
  // the straight-line whole-block encoder equals the generic field path (m = 55 counts letter 55 as 1)
  for (int rep = 0; rep < 200; ++rep) {
    uint8_t c[56], a[33], b[33];
    for (auto& x : c) x = static_cast<uint8_t>(1 + rng() % 26);
    if (rep % 3 == 0) std::fill(c, c + 56, uint8_t{26});
    c[55] = 1;
    p33_block(c, a);
    p33_block(c, b, 55);
    CHECK(std::equal(a, a + 33, b));
  }
  // the kernel's first digit: (x >> 1) / 13 == x / 26 for every field value class
  const uint64_t probes[] = {0, 25, 26, 51, 52, 8031810175ull, 8031810150ull, 4294967295ull, 4294967296ull,
                             4294967297ull};
  for (uint64_t x : probes)
    CHECK(static_cast<uint32_t>(x >> 1) / 13u == x / 26u);
}

void test_profile16() {
  std::mt19937 rng(11);
  for (int trial = 0; trial < 40; ++trial) {
    const int64_t L1 = 1 + rng() % 400;
    const int32_t wmax = trial % 2 ? 100 : 12;
    Weights w{{static_cast<int32_t>(rng() % wmax), static_cast<int32_t>(rng() % 27),
               static_cast<int32_t>(rng() % 27), static_cast<int32_t>(rng() % 27)}};
    const ScoreTable t = ScoreTable::build(w);
    std::vector<uint8_t> s1(static_cast<size_t>(L1));
    for (auto& x : s1) x = static_cast<uint8_t>(1 + rng() % (trial % 3 ? 26 : 3));  // few letters: many ties
    Profile16 prof;
    const int64_t span = trial % 4 < 2 ? 512 : 1024;  // tile span = 128*U offsets (U = 4 or 8) = overhang
    if (!build_profile16(t, s1.data(), L1, span, prof)) {
      CHECK(w.w[0] + std::max({w.w[1], w.w[2], w.w[3]}) > 127);
      continue;
    }
    CHECK(prof.entries.size() == static_cast<size_t>(26 * L1 + span));
    auto entry = [&](int c, int64_t j) { return prof.entries[static_cast<size_t>((c - 1) * L1 + j)]; };
    RecordBatch batch;
    for (int r = 0; r < 6; ++r) {
      const int64_t L2 = 1 + rng() % (L1 + 2);
      std::vector<uint8_t> s2(static_cast<size_t>(L2));
      for (auto& x : s2) x = static_cast<uint8_t>(1 + rng() % (trial % 3 ? 26 : 3));
      batch.push_back(s2.data(), L2);
    }
    for (Semantics sem : {Semantics::Reference, Semantics::Spec}) {
      std::vector<Result> out(static_cast<size_t>(batch.size()));
      solve_batch_cpu(t, s1.data(), L1, batch, out.data(), sem, 1);
      for (int64_t r = 0; r < batch.size(); ++r) {
        const uint8_t* s2 = batch.record(r);
        const int64_t L2 = batch.length(r);
        uint64_t best_key = 0;
        const int64_t need = L2 <= L1 ? L1 - L2 + 1 : 0;
        std::vector<int32_t> Dc(static_cast<size_t>(need) + 1, 0), maxD(static_cast<size_t>(need) + 1, INT32_MIN);
        for (int64_t o = 0; o < need; ++o) {
          for (int64_t i0 = 0; i0 < L2; i0 += 64) {
            const int64_t m = std::min<int64_t>(64, L2 - i0);
            uint16_t accD = 0;
            int16_t bestD = INT16_MIN;
            bool any = false;
            for (int64_t j = 0; j < m; ++j) {  // lane pair (o & ~1, o | 1): byte (o & 1) of one entry
              const uint16_t e = entry(s2[i0 + j], (o & ~int64_t{1}) + i0 + j);
              const int8_t d = static_cast<int8_t>(o & 1 ? e >> 8 : e & 0xff);
              accD = static_cast<uint16_t>(accD + static_cast<uint16_t>(static_cast<int16_t>(d)));
              if (i0 + j + 1 < L2) {  // k = i+1 <= L2-1 is a candidate
                bestD = std::max(bestD, static_cast<int16_t>(accD));
                any = true;
              }
            }
            if (any) maxD[o] = std::max(maxD[o], Dc[o] + bestD);
            Dc[o] += static_cast<int16_t>(accD);
          }
        }
        // Tot per tile: anchor diagonal at min(tile end, L1 - L2 + 1), then suffix sums of D totals
        std::vector<int32_t> tot(static_cast<size_t>(need) + 1, 0);
        for (int64_t o0 = 0; o0 < need; o0 += span) {
          const int64_t oA = std::min<int64_t>(o0 + span, need);
          int32_t acc = 0;
          for (int64_t i = 0; i < L2; ++i) acc += t.score(s2[i], oA + i < L1 ? s1[oA + i] : 0);
          for (int64_t o = oA - 1; o >= o0; --o) {
            acc += Dc[o];
            tot[o] = acc;
          }
        }
        for (int64_t o = 0; o < need; ++o) {
          const int32_t Pc = tot[o], Tn = tot[o] - Dc[o];  // Tot_o, Tot_{o+1}
          const int64_t last = L1 - L2;
          const bool v0 = o < last || (o == last && (sem == Semantics::Spec || L2 == L1));
          auto key1 = [](int32_t s, uint32_t idx) {
            return (static_cast<uint64_t>(static_cast<uint32_t>(s) ^ 0x80000000u) << 32) | (0xffffffffu - idx);
          };
          if (v0) best_key = std::max(best_key, key1(Pc, static_cast<uint32_t>(2 * o)));
          if (o < last && L2 >= 2) best_key = std::max(best_key, key1(maxD[o] + Tn, static_cast<uint32_t>(2 * o + 1)));
        }
        Result got{kNoCandidateScore, 0, 0};
        if (best_key) {
          const int32_t score = static_cast<int32_t>(static_cast<uint32_t>(best_key >> 32) ^ 0x80000000u);
          const uint32_t idx = 0xffffffffu - static_cast<uint32_t>(best_key);
          got = Result{score, static_cast<int32_t>(idx >> 1), 0};
          if (idx & 1) {  // pass 2: smallest k >= 1 on the winning diagonal
            int32_t tot1 = 0, d = 0;
            for (int64_t i = 0; i < L2; ++i) tot1 += t.score(s2[i], s1[got.n + 1 + i]);
            got.k = -1;
            for (int64_t i = 0; i + 1 < L2 && got.k < 0; ++i) {
              d += t.score(s2[i], s1[got.n + i]) - t.score(s2[i], s1[got.n + i + 1]);
              if (d + tot1 == score) got.k = static_cast<int32_t>(i + 1);
            }
          }
        }
        CHECK(got.score == out[r].score && got.n == out[r].n && got.k == out[r].k);
      }
    }
  }
}

// pv.prof16_bytes of a whole-image view is an LDS size for every Seq1 length the engine accepts (up to 2^30):
// an int16 profile of a long Seq1 (|Dt| 128..511) used to be sized in int32 from the whole profile, which
// wrapped past L1 ~ 43 M and could pass the widened-image check with a negative size.
void test_profile16_lds_bytes() {
  const int64_t lengths[] = {1, 26, 1489, 2976, 3052, 3100, 20000, 150000, 43'000'000, 60'000'000, 86'000'000,
                             100'000'000, int64_t{1} << 30};
  for (int64_t L1 : lengths)
    for (int64_t oh : {int64_t{dev::kProf16Overhang}, int64_t{2 * dev::kProf16Overhang}})
      for (bool i16 : {false, true}) {
        const int32_t b = dev::tile16_profile_lds_bytes(L1, oh, i16);
        CHECK(b > 0 && b <= dev::kProf16MaxLds && b % 16 == 0);
        // the widened-image check of HipEngine::set_problem only passes where the doubled image fits
        const bool wide = dev::tile16_lds_bytes(2 * static_cast<int64_t>(b), L1) <= dev::kProf16MaxLds;
        if (wide) CHECK(2 * (26 * L1 + oh) <= dev::kProf16MaxLds);
      }
  // input3's Seq1: the whole byte-pair profile is the image; an int16 one needs the widened image to fit
  CHECK(dev::tile16_profile_lds_bytes(1489, 512, false) == ((2 * (26 * 1489 + 512)) + 15) / 16 * 16);
}

// The comm deadline: a wait that completes returns; one that does not throws CommTimeout naming the
// operation, what is outstanding, and the phase; expire runs first; 0 disables the deadline.
void test_watchdog() {
  watchdog::set_timeout_s(0.05);
  watchdog::set_rank(3);
  watchdog::set_phase("gather");
  int n = 0;
  watchdog::WaitSpec spec;
  spec.what = "test op";
  watchdog::wait([&] { return ++n > 100; }, spec);
  CHECK(n == 101);
  bool expired = false;
  spec.outstanding = [] { return std::string("recv 24 B from rank 2"); };
  spec.expire = [&] { expired = true; };
  for (watchdog::Poll poll : {watchdog::Poll::Busy, watchdog::Poll::Backoff}) {
    spec.poll = poll;
    expired = false;
    std::string msg;
    try {
      watchdog::wait([] { return false; }, spec);
    } catch (const CommTimeout& e) {
      msg = e.what();
    }
    CHECK(expired);
    CHECK(msg.find("rank 3") != std::string::npos && msg.find("phase 'gather'") != std::string::npos &&
          msg.find("test op") != std::string::npos && msg.find("from rank 2") != std::string::npos);
  }
  int checks = 0;
  spec.check = [&] {
    if (++checks == 3) throw Error("async error");
  };
  spec.poll = watchdog::Poll::Backoff;
  watchdog::set_timeout_s(10);
  std::string msg;
  try {
    watchdog::wait([] { return false; }, spec);
  } catch (const Error& e) {
    msg = e.what();
  }
  CHECK(msg == "async error");
  watchdog::set_timeout_s(0);  // disabled: a slow wait completes
  int m = 0;
  watchdog::WaitSpec plain;
  watchdog::wait([&] { return ++m > 200000; }, plain);
  CHECK(m == 200001);
  CHECK(watchdog::human_bytes(24) == "24 B" && watchdog::human_bytes(3 << 20) == "3.0 MiB");
  watchdog::set_timeout_s(watchdog::kDefaultTimeoutS);
  watchdog::set_phase("");
}

void test_formatter() {
  const Result r[3] = {{1, 2, 3}, {kNoCandidateScore, 0, 0}, {-5, 10, 0}};
  CHECK(format_results(r, 3, 7) == "#7: score: 1, n: 2, k: 3\n#8: score: -2147483648, n: 0, k: 0\n"
                                   "#9: score: -5, n: 10, k: 0\n");
  // the row counter carries across digit counts; numbers of every width
  const Result q[3] = {{2147483647, 123456789, 99}, {-100, 0, 1}, {10, 100, 1000}};
  CHECK(format_results(q, 3, 998) == "#998: score: 2147483647, n: 123456789, k: 99\n"
                                     "#999: score: -100, n: 0, k: 1\n#1000: score: 10, n: 100, k: 1000\n");
  CHECK(format_results(q, 1, 0) == "#0: score: 2147483647, n: 123456789, k: 99\n");
}
}  // namespace

// BackgroundReleaser: FIFO order on one worker, drain() waits for everything queued, captured owners are
// released on the worker, and stop() after drain is idempotent.
void test_releaser() {
  std::vector<int> order;
  auto owned = std::make_shared<int>(7);
  std::weak_ptr<int> watch = owned;
  {
    BackgroundReleaser rel;
    for (int i = 0; i < 100; ++i) rel.defer([&order, i] { order.push_back(i); });
    rel.defer([o = std::move(owned)]() mutable { o.reset(); });
    rel.drain();
    CHECK(order.size() == 100);
    bool sorted = true;
    for (int i = 0; i < 100; ++i) sorted = sorted && order[i] == i;
    CHECK(sorted);
    CHECK(watch.expired());
    rel.defer([&order] { order.push_back(100); });  // queued, then run by the destructor's stop()
  }
  CHECK(order.size() == 101 && order.back() == 100);
  BackgroundReleaser idle;  // never started: stop() is a no-op
  idle.drain();
  idle.stop();
}

// Cooperative pass 1 + slice fills (the node-parallel parse of `final`): any chunk count, any slice,
// byte and 5-bit packed output (incl. letters of one group split over pieces) equal a sequential parse.
void test_slices() {
  std::mt19937 rng(7);
  for (int trial = 0; trial < 40; ++trial) {
    const int n = 1 + static_cast<int>(rng() % 400);
    const int maxlen = trial % 3 == 0 ? 40 : (trial % 3 == 1 ? 3 : 300);
    std::string text = "1 2 3 4\nABCDEFGHIJKLMNOPQRSTUVWXYZABCDEFGHIJKLMNOPQRSTUVWXYZ\n" + std::to_string(n) + "\n";
    std::vector<std::string> recs;
    for (int i = 0; i < n; ++i) {
      std::string r;
      const int L = 1 + static_cast<int>(rng() % maxlen);
      for (int j = 0; j < L; ++j) r += static_cast<char>((rng() & 1 ? 'A' : 'a') + rng() % 26);
      recs.push_back(r);
      text += r;
      const int sep = static_cast<int>(rng() % 6);
      text += sep == 0 ? "\n" : sep == 1 ? " \r\n" : sep == 2 ? "\t" : sep == 3 ? "\n\n  " : sep == 4 ? "\v" : "\f \n";
    }
    if (trial % 5 == 0) text += "EXTRA TRAILING TOKENS\n";
    const Problem ref = parse_problem(text.data(), text.size());
    {  // the reference parse (same encoder as below: SIMD or scalar, MOC_FILL_SIMD) against the records
      bool same = ref.seq2.size() == n;
      for (int i = 0; same && i < n; ++i) {
        same = ref.seq2.length(i) == static_cast<int64_t>(recs[i].size());
        for (size_t j = 0; same && j < recs[i].size(); ++j)
          same = ref.seq2.record(i)[j] == letter_code(static_cast<unsigned char>(recs[i][j]));
      }
      CHECK(same);
    }
    BulkParser p(text.data(), text.size(), ParseOptions{}, false);
    CHECK(p.total_chars() < 0);
    const int nch = 1 + static_cast<int>(rng() % 97);
    std::vector<int64_t> st = p.chunk_starts(nch), tk(static_cast<size_t>(nch)), ch(static_cast<size_t>(nch));
    // counted in two "ranks'" shares, like the distributed pass 1
    const int mid = nch / 2;
    p.count_chunks(st, 0, mid, tk.data(), ch.data());
    p.count_chunks(st, mid, nch, tk.data() + mid, ch.data() + mid);
    p.set_chunks(st, tk.data(), ch.data());
    CHECK(p.total_chars() == ref.seq2.total_chars());
    CHECK(p.chunk_first_record(0) == 0 && p.chunk_first_record(nch) == n);
    // rank bounds from the chunk table: estimated splits are monotone and cover [first, n); with exact
    // chunk costs they equal the lengths-based cost partition of the same records
    {
      const CostModel cm{1.0, 200.0, 2400.0};
      const int parts = 1 + static_cast<int>(rng() % 9);
      const int64_t first = trial % 4 == 0 ? static_cast<int64_t>(rng() % (n + 1)) : 0;
      int64_t prev = first;
      bool mono = p.cost_split(first, 0, parts, cm) == first && p.cost_split(first, parts, parts, cm) == n;
      for (int q = 1; q <= parts; ++q) {
        const int64_t x = p.cost_split(first, q, parts, cm);
        mono = mono && x >= prev && x <= n;
        prev = x;
      }
      CHECK(mono);
      std::vector<double> costs(static_cast<size_t>(nch));
      p.chunk_costs(st, 0, nch, cm, costs.data());
      p.set_chunk_costs(costs);
      const std::vector<int64_t> want =
          partition_by_cost_offsets(ref.seq2.offsets.data() + first, n - first, 52, parts, cm);
      bool same = true;
      for (int q = 0; q <= parts; ++q) same = same && p.cost_split(first, q, parts, cm) == first + want[q];
      CHECK(same);
    }
    for (int rep = 0; rep < 6; ++rep) {
      int64_t b = rng() % (n + 1), e = rng() % (n + 1);
      if (b > e) std::swap(b, e);
      if (rep == 0) { b = 0; e = n; }
      const AreaSlice s = p.slice(b, e);
      CHECK(s.records == e - b);
      CHECK(s.letters == ref.seq2.offsets[e] - ref.seq2.offsets[b]);
      std::vector<uint8_t> codes(static_cast<size_t>(s.letters) + 1, 0xEE), packed(packed5_bytes(s.letters), 0xEE);
      std::vector<int64_t> offs(static_cast<size_t>(s.records) + 1, -7);
      const FillReport r = p.fill_slice(s, codes.data(), packed.data(), offs.data());
      CHECK(r.bad_record < 0 && r.long_record < 0);
      bool ok = true;
      for (int64_t i = 0; i <= s.records; ++i) ok = ok && offs[i] == ref.seq2.offsets[b + i] - ref.seq2.offsets[b];
      for (int64_t i = 0; i < s.letters; ++i) ok = ok && codes[i] == ref.seq2.codes[ref.seq2.offsets[b] + i];
      CHECK(ok);
      std::vector<uint8_t> want(packed5_bytes(s.letters));
      pack5(ref.seq2.codes.data() + ref.seq2.offsets[b], s.letters, want.data());
      CHECK(want == packed);
      if (s.records) {
        int64_t mn = INT64_MAX, mx = 0;
        for (int64_t i = b; i < e; ++i) {
          mn = std::min(mn, ref.seq2.length(i));
          mx = std::max(mx, ref.seq2.length(i));
        }
        CHECK(r.min_len == mn && r.max_len == mx);
        // packed-only fill (no byte codes) gives the same stream
        std::vector<uint8_t> p2(packed5_bytes(s.letters), 0x55);
        p.fill_slice(s, nullptr, p2.data(), offs.data());
        CHECK(p2 == want);
      }
      // the narrow wire form: packed letters + sparse offsets + uint16 lengths, no dense offsets
      std::vector<int64_t> sp(static_cast<size_t>(sparse_count(s.records, kSparseShift)), -9);
      std::vector<uint16_t> l16(static_cast<size_t>(s.records) + 1, 0xBEEF);
      std::vector<uint8_t> p3(packed5_bytes(s.letters), 0x33);
      const FillReport r3 = p.fill_slice(s, nullptr, p3.data(), nullptr, sp.data(), l16.data());
      CHECK(r3.min_len == r.min_len && r3.max_len == r.max_len && r3.cells == r.cells && p3 == want);
      // ... and with P33 fields (56-letter blocks straddling the pieces assembled afterwards)
      std::vector<uint8_t> p33(static_cast<size_t>(packed33_bytes(s.letters)), 0x33),
          want33(static_cast<size_t>(packed33_bytes(s.letters)));
      pack33(ref.seq2.codes.data() + ref.seq2.offsets[b], s.letters, want33.data());
      const FillReport r33 = p.fill_slice(s, nullptr, p33.data(), nullptr, sp.data(), l16.data(), 33);
      CHECK(r33.min_len == r.min_len && r33.max_len == r.max_len && r33.cells == r.cells && p33 == want33);
      ok = true;
      for (size_t j = 0; j < sp.size(); ++j)
        ok = ok && sp[j] == offs[std::min<int64_t>(static_cast<int64_t>(j) << kSparseShift, s.records)];
      for (int64_t i = 0; i < s.records; ++i) ok = ok && l16[i] == offs[i + 1] - offs[i];
      CHECK(ok);
      if (s.records && r3.max_len <= 255) {  // -> narrow lengths -> dense offsets again
        const int bits = narrow_length_bits(r3.min_len, r3.max_len);
        std::vector<uint8_t> nl(static_cast<size_t>(narrow_lengths_bytes(s.records, bits)) + 1);
        pack_lengths16(l16.data(), s.records, bits, r3.min_len, nl.data());
        std::vector<int64_t> dense(static_cast<size_t>(s.records) + 1, -1);
        expand_offsets(sp.data(), kSparseShift, nl.data(), bits, r3.min_len, s.records, dense.data());
        CHECK(dense == offs);
      }
    }
  }
  // errors name the first offending record of the slice, in global numbering
  const std::string bad = "1 2 3 4\nABCDEFGH\n5\nAB\nCD\nE1\nFG\nHIJKLMNOP\n";
  BulkParser p(bad.data(), bad.size(), ParseOptions{false, 0, 4}, true);
  FillReport r = p.fill_slice(p.slice(1, 5), nullptr, std::vector<uint8_t>(64).data(), std::vector<int64_t>(8).data());
  CHECK(r.bad_record == 2 && r.long_record == 4 && r.long_len == 9);
  CHECK(throws([&] { p.check(r); }, "record #2 contains a non-letter"));
  r = p.fill_slice(p.slice(3, 5), nullptr, std::vector<uint8_t>(64).data(), std::vector<int64_t>(8).data());
  CHECK(throws([&] { p.check(r); }, "record #4 has 9 letters"));
}

// Narrow record lengths (3 / 4 / 8 bits) round-trip through the host decoder.
void test_narrow_lengths() {
  std::mt19937 rng(3);
  for (int bits : {3, 4, 8, kLenBase6})
    for (int n : {0, 1, 7, 8, 9, 23, 24, 25, 1000, 100003}) {
      const int span = bits == 3 ? 8 : bits == 4 ? 16 : bits == kLenBase6 ? 6 : 200;
      std::vector<int64_t> offs(static_cast<size_t>(n) + 1, 0);
      for (int i = 0; i < n; ++i) offs[i + 1] = offs[i] + 6 + static_cast<int64_t>(rng() % span);
      std::vector<uint8_t> out(static_cast<size_t>(narrow_lengths_bytes(n, bits)) + 1, 0xAB);
      pack_lengths(offs.data(), n, bits, 6, out.data());
      bool ok = true;
      for (int i = 0; i < n; ++i) ok = ok && narrow_length(out.data(), bits, 6, i) == offs[i + 1] - offs[i];
      CHECK(ok);
      if (bits == 3) CHECK(out[narrow_lengths_bytes(n, 3) - 1] == 0);
      // the same packing from uint16 lengths
      std::vector<uint16_t> l16(static_cast<size_t>(n) + 1);
      for (int i = 0; i < n; ++i) l16[i] = static_cast<uint16_t>(offs[i + 1] - offs[i]);
      std::vector<uint8_t> out16(out.size(), 0xAB);
      pack_lengths16(l16.data(), n, bits, 6, out16.data());
      CHECK(std::equal(out.begin(), out.begin() + narrow_lengths_bytes(n, bits), out16.begin()));
      // sparse offsets + narrow lengths -> dense offsets
      if (n > 0) {
        std::vector<int64_t> sp(static_cast<size_t>(sparse_count(n, kSparseShift)));
        for (size_t j = 0; j < sp.size(); ++j) sp[j] = offs[std::min<int64_t>(static_cast<int64_t>(j) << kSparseShift, n)];
        std::vector<int64_t> dense(static_cast<size_t>(n) + 1, -1);
        expand_offsets(sp.data(), kSparseShift, out.data(), bits, bits == 8 ? 0 : 6, n, dense.data());
        if (bits != 8) CHECK(dense == offs);
      }
    }
  if (true) {  // base 6: 8 lengths per 21-bit octet, 3 octets per little-endian word
    const int64_t offs[9] = {0, 11, 17, 23, 29, 35, 41, 47, 58};  // lengths 11, 6, 6, 6, 6, 6, 6, 11
    uint8_t w[8];
    pack_lengths(offs, 8, kLenBase6, 6, w);
    uint64_t word;
    std::memcpy(&word, w, 8);
    CHECK(word == 5ull + 5ull * 279936ull);  // digit 0 and digit 7 (6^7) hold 5
  }
  CHECK(narrow_lengths_bytes(25, kLenBase6) == 16);
  CHECK(narrow_length_bits(6, 11) == kLenBase6 && narrow_length_bits(6, 13) == 3 && narrow_length_bits(6, 21) == 4 &&
        narrow_length_bits(1, 255) == 8);
  CHECK(narrow_length_bits(1, 256) == 0);
}

// Every result wire format decodes back to the rows it encodes.
void test_result_formats() {
  R2Params p;
  CHECK(r2_params(26, 6, 11, -10, 4, p));
  const Result rows[3] = {{-20, 3, 5}, {44, 0, 0}, no_candidate()};
  uint16_t r2[3];
  for (int i = 0; i < 2; ++i)
    r2[i] = static_cast<uint16_t>((rows[i].score - p.smin) * p.j + rows[i].n * p.kw + rows[i].k);
  r2[2] = kR2None;
  R4 r4[3];
  R8 r8[3];
  for (int i = 0; i < 3; ++i) {
    r4[i] = R4{static_cast<int16_t>(i == 2 ? INT16_MIN : rows[i].score), static_cast<uint8_t>(rows[i].n),
               static_cast<uint8_t>(rows[i].k)};
    r8[i] = R8{rows[i].score, static_cast<uint16_t>(rows[i].n), static_cast<uint16_t>(rows[i].k)};
  }
  bool ok = true;
  for (int i = 0; i < 3; ++i) {
    const Result a = decode_result(r2, ResultFormat::R2, p, i), b = decode_result(r4, ResultFormat::R4, p, i),
                 c = decode_result(r8, ResultFormat::R8, p, i), d = decode_result(rows, ResultFormat::R12, p, i);
    for (const Result& x : {a, b, c, d}) ok = ok && x.score == rows[i].score && x.n == rows[i].n && x.k == rows[i].k;
  }
  CHECK(ok);
}

// write_results over mixed runs (two large R2 runs with different parameters -> the row-tail tables, one
// small R4 run -> the direct path) equals format_results of the expanded rows, with both file writers.
void test_write_runs() {
  R2Params pa, pb;
  CHECK(r2_params(26, 6, 11, -10, 4, pa));
  CHECK(r2_params(20, 1, 8, -3, 5, pb));
  const int64_t na = 300000, nb = 4, nc = 270001;
  std::vector<uint16_t> a(na), c(nc);
  std::vector<R4> b(nb);
  std::vector<Result> all;
  uint32_t x = 12345;
  auto rnd = [&x] { return x = x * 1664525u + 1013904223u; };
  auto fill_r2 = [&](std::vector<uint16_t>& v, const R2Params& p, int max_l2) {
    for (auto& code : v) {
      const int r = static_cast<int>(rnd() >> 8);
      if (r % 97 == 0) {
        code = kR2None;
      } else {
        const int k = r % (max_l2 + 1), n = (r >> 5) % 16, s = (r >> 10) % 200;
        code = static_cast<uint16_t>(s * p.j + n * p.kw + k);
      }
      all.push_back(decode_result(&code, ResultFormat::R2, p, 0));
    }
  };
  fill_r2(a, pa, 11);
  for (int i = 0; i < nb; ++i) {
    b[i] = R4{static_cast<int16_t>(i == 1 ? INT16_MIN : -i * 7), static_cast<uint8_t>(i), static_cast<uint8_t>(2 * i)};
    all.push_back(decode_result(b.data(), ResultFormat::R4, pa, i));
  }
  fill_r2(c, pb, 8);
  const std::string want = format_results(all.data(), static_cast<int64_t>(all.size()), 41);
  const std::vector<ResultRun> runs = {ResultRun{a.data(), ResultFormat::R2, pa, na},
                                       ResultRun{b.data(), ResultFormat::R4, pa, nb},
                                       ResultRun{c.data(), ResultFormat::R2, pb, nc}};
  for (const char* writer : {"", "ordered"}) {
    setenv("MOC_WRITER", writer, 1);
    FILE* f = std::tmpfile();
    std::fputs("head\n", f);
    write_results(f, runs, 41);
    std::fputs("tail\n", f);
    std::fflush(f);
    std::string got(static_cast<size_t>(std::ftell(f)), '\0');
    std::rewind(f);
    CHECK(std::fread(got.data(), 1, got.size(), f) == got.size());
    std::fclose(f);
    CHECK(got == "head\n" + want + "tail\n");
  }
  unsetenv("MOC_WRITER");
  // the sizing pass and the offset writer (ranks writing their own rows of one file), also across
  // index digit boundaries
  for (int64_t first : {int64_t{41}, int64_t{999990}, int64_t{99999999999}}) {
    const std::string w2 = format_results(all.data(), static_cast<int64_t>(all.size()), first);
    CHECK(formatted_bytes(runs, first) == static_cast<int64_t>(w2.size()));
    FILE* f = std::tmpfile();
    const int64_t at = 7;
    CHECK(write_results_at(fileno(f), at, runs, first) == static_cast<int64_t>(w2.size()));
    std::string got(w2.size(), '\0');
    CHECK(pread(fileno(f), got.data(), got.size(), at) == static_cast<ssize_t>(got.size()));
    std::fclose(f);
    CHECK(got == w2);
  }
}

// GPUs from a fake driver topology: CPU nodes skipped, render nodes this process cannot open skipped,
// nodes in numeric order (10 after 2), PCIe address and NUMA node from domain + location_id
void test_kfd_topology() {
  char tmpl[] = "/tmp/moc_kfd_XXXXXX";
  const char* root_c = mkdtemp(tmpl);
  CHECK(root_c != nullptr);
  if (!root_c) return;
  const std::string root = root_c;
  auto put = [](const std::string& path, const std::string& text) {
    FILE* f = std::fopen(path.c_str(), "w");
    if (!f) return;
    std::fputs(text.c_str(), f);
    std::fclose(f);
  };
  auto node = [&](int id, const std::string& props) {
    const std::string d = root + "/nodes/" + std::to_string(id);
    mkdir(d.c_str(), 0755);
    put(d + "/properties", props);
  };
  mkdir((root + "/nodes").c_str(), 0755);
  mkdir((root + "/dri").c_str(), 0755);
  mkdir((root + "/pci").c_str(), 0755);
  mkdir((root + "/pci/0000:0d:00.0").c_str(), 0755);
  put(root + "/pci/0000:0d:00.0/numa_node", "1\n");
  node(0, "cpu_cores_count 64\nsimd_count 0\nlocation_id 0\ndomain 0\n");
  node(2, "simd_count 1024\ndrm_render_minor 129\nlocation_id 7424\ndomain 0\n");   // 1d:00.0, not ours
  node(10, "simd_count 1024\ndrm_render_minor 130\nlocation_id 34816\ndomain 1\n");  // 0001:88:00.0
  node(3, "simd_count 1024\ndrm_render_minor 128\nlocation_id 3328\ndomain 0\n");   // 0000:0d:00.0
  put(root + "/dri/renderD128", "");
  put(root + "/dri/renderD130", "");
  put(root + "/kfd", "");
  KfdPaths p;
  p.nodes = root + "/nodes";
  p.kfd = root + "/kfd";
  p.dri = root + "/dri";
  p.pci = root + "/pci";
  p.honour_visible_env = false;
  auto g = kfd_gpus(p);
  CHECK(g.has_value() && g->size() == 2);
  if (g && g->size() == 2) {
    CHECK((*g)[0].node == 3 && (*g)[0].render_minor == 128 && (*g)[0].pci_bus_id == "0000:0d:00.0" &&
          (*g)[0].numa_node == 1);
    CHECK((*g)[1].node == 10 && (*g)[1].pci_bus_id == "0001:88:00.0" && (*g)[1].numa_node == -1);
  }
  // the runtime's re-mapping by index lists: ROCR_ first, then HIP_ (or CUDA_) on top; UUIDs, indices out
  // of range and disagreeing HIP/CUDA lists are left to the runtime
  p.honour_visible_env = true;
  for (const char* v : {"ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "GPU_DEVICE_ORDINAL"})
    unsetenv(v);
  g = kfd_gpus(p);
  CHECK(g && g->size() == 2);
  setenv("HIP_VISIBLE_DEVICES", "1", 1);
  g = kfd_gpus(p);
  CHECK(g && g->size() == 1 && (*g)[0].node == 10);
  setenv("ROCR_VISIBLE_DEVICES", "1,0", 1);
  g = kfd_gpus(p);
  CHECK(g && g->size() == 1 && (*g)[0].node == 3);
  setenv("HIP_VISIBLE_DEVICES", "0", 1);
  setenv("ROCR_VISIBLE_DEVICES", "0", 1);
  g = kfd_gpus(p);
  CHECK(g && g->size() == 1 && (*g)[0].node == 3);
  setenv("CUDA_VISIBLE_DEVICES", "1", 1);
  CHECK(!kfd_gpus(p).has_value());
  unsetenv("CUDA_VISIBLE_DEVICES");
  setenv("HIP_VISIBLE_DEVICES", "2", 1);
  CHECK(!kfd_gpus(p).has_value());
  setenv("HIP_VISIBLE_DEVICES", "GPU-4c3a2b1d00000000", 1);
  CHECK(!kfd_gpus(p).has_value());
  setenv("HIP_VISIBLE_DEVICES", "", 1);
  CHECK(!kfd_gpus(p).has_value());
  unsetenv("HIP_VISIBLE_DEVICES");
  unsetenv("ROCR_VISIBLE_DEVICES");
  p.honour_visible_env = false;
  // no access to the driver: none; no topology: unknown; a GPU node without a render minor: unknown
  p.kfd = root + "/no_kfd";
  g = kfd_gpus(p);
  CHECK(g.has_value() && g->empty());
  p.kfd = root + "/kfd";
  p.nodes = root + "/no_nodes";
  CHECK(!kfd_gpus(p).has_value());
  p.nodes = root + "/nodes";
  node(11, "simd_count 1024\n");
  CHECK(!kfd_gpus(p).has_value());
  CHECK(std::system(("rm -rf " + root).c_str()) == 0);
}

// An 8-GPU, two-socket node as the driver describes it (two CPU nodes, then eight GPU nodes; GPUs 0-3 on
// NUMA node 0, 4-7 on node 1): every node-local rank of an 8- or 16-rank job gets device rank % 8 and that
// device's NUMA node, also under ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES permutations, with --device,
// and on a box that exposes one of the eight render nodes (the gpurun box: HIP_/ROCR_VISIBLE_DEVICES=0).
void test_kfd_topology_8gpu() {
  char tmpl[] = "/tmp/moc_kfd8_XXXXXX";
  const char* root_c = mkdtemp(tmpl);
  CHECK(root_c != nullptr);
  if (!root_c) return;
  const std::string root = root_c;
  auto put = [](const std::string& path, const std::string& text) {
    FILE* f = std::fopen(path.c_str(), "w");
    if (!f) return;
    std::fputs(text.c_str(), f);
    std::fclose(f);
  };
  for (const char* d : {"/nodes", "/dri", "/pci"}) mkdir((root + d).c_str(), 0755);
  const int bus[8] = {0x05, 0x15, 0x5d, 0x75, 0x85, 0x95, 0xe5, 0xf1};
  auto bus_id = [&](int g) {
    char b[16];
    std::snprintf(b, sizeof b, "0000:%02x:00.0", bus[g]);
    return std::string(b);
  };
  for (int cpu = 0; cpu < 2; ++cpu) {
    mkdir((root + "/nodes/" + std::to_string(cpu)).c_str(), 0755);
    put(root + "/nodes/" + std::to_string(cpu) + "/properties", "cpu_cores_count 64\nsimd_count 0\n");
  }
  for (int g = 0; g < 8; ++g) {
    const std::string d = root + "/nodes/" + std::to_string(2 + g);
    mkdir(d.c_str(), 0755);
    // 64-bit values (hive_id, unique_id) anywhere in the file: one of them must not end the scan
    const unsigned long long uid = 0xfedcba9876543210ull + static_cast<unsigned long long>(g);
    put(d + "/properties", "simd_count 1024\nhive_id 18446744073709551615\ndrm_render_minor " +
                               std::to_string(128 + g) + "\nlocation_id " + std::to_string(bus[g] << 8) +
                               "\ndomain 0\nunique_id " + std::to_string(uid) + "\n");
    put(root + "/dri/renderD" + std::to_string(128 + g), "");
    mkdir((root + "/pci/" + bus_id(g)).c_str(), 0755);
    put(root + "/pci/" + bus_id(g) + "/numa_node", g < 4 ? "0\n" : "1\n");
  }
  put(root + "/kfd", "");
  KfdPaths p;
  p.nodes = root + "/nodes";
  p.kfd = root + "/kfd";
  p.dri = root + "/dri";
  p.pci = root + "/pci";
  for (const char* v : {"ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "GPU_DEVICE_ORDINAL"})
    unsetenv(v);
  auto g = kfd_gpus(p);
  CHECK(g && g->size() == 8);
  if (!g || g->size() != 8) return;
  // unique ids -> the runtime's UUIDs; ROCR_VISIBLE_DEVICES by UUID (any case), mixed with indices
  CHECK(kfd_uuid((*g)[3]) == "GPU-fedcba9876543213" && (*g)[0].pci_bus_id == bus_id(0));
  setenv("ROCR_VISIBLE_DEVICES", "GPU-FEDCBA9876543215,2", 1);
  {
    const auto u = kfd_gpus(p);
    CHECK(u && u->size() == 2 && (*u)[0].pci_bus_id == bus_id(5) && (*u)[1].pci_bus_id == bus_id(2));
  }
  setenv("ROCR_VISIBLE_DEVICES", "GPU-0000000000000001", 1);  // unknown: the runtime's to interpret
  CHECK(!kfd_gpus(p));
  unsetenv("ROCR_VISIBLE_DEVICES");
  // rank -> device -> NUMA node, 8 and 16 ranks per node
  for (int r = 0; r < 16; ++r) {
    const int id = kfd_pick(*g, r, -1);
    CHECK(id == r % 8);
    CHECK((*g)[static_cast<size_t>(id)].pci_bus_id == bus_id(r % 8));
    CHECK((*g)[static_cast<size_t>(id)].numa_node == (r % 8 < 4 ? 0 : 1));
  }
  CHECK(kfd_pick(*g, 3, 6) == 6 && kfd_pick(*g, 0, 8) == -1);
  // the sockets swapped: device 0 is the first GPU of NUMA node 1
  setenv("ROCR_VISIBLE_DEVICES", "4,5,6,7,0,1,2,3", 1);
  g = kfd_gpus(p);
  CHECK(g && g->size() == 8);
  if (g && g->size() == 8)
    for (int r = 0; r < 8; ++r) {
      const KfdGpu& x = (*g)[static_cast<size_t>(kfd_pick(*g, r, -1))];
      CHECK(x.pci_bus_id == bus_id((r + 4) % 8) && x.numa_node == (r < 4 ? 1 : 0));
    }
  // reversed, then every second one on top: [7, 5, 3, 1]
  setenv("ROCR_VISIBLE_DEVICES", "7,6,5,4,3,2,1,0", 1);
  setenv("HIP_VISIBLE_DEVICES", "0,2,4,6", 1);
  g = kfd_gpus(p);
  CHECK(g && g->size() == 4);
  if (g && g->size() == 4)
    for (int r = 0; r < 8; ++r) {
      const KfdGpu& x = (*g)[static_cast<size_t>(kfd_pick(*g, r, -1))];
      const int phys = 7 - 2 * (r % 4);
      CHECK(x.pci_bus_id == bus_id(phys) && x.numa_node == (phys < 4 ? 0 : 1));
    }
  // per-rank isolation (final --gpu-isolate): the rank's GPU by its index among all the driver's GPUs; with
  // ROCR_VISIBLE_DEVICES set to it and HIP_VISIBLE_DEVICES to 0 the runtime's view is that one GPU
  {
    KfdPaths raw = p;
    raw.honour_visible_env = false;
    const auto all = kfd_gpus(raw);
    const auto vis = kfd_gpus(p);
    CHECK(all && all->size() == 8 && vis && vis->size() == 4);
    if (all && vis && vis->size() == 4)
      for (int r = 0; r < 8; ++r) {
        const int idx = kfd_isolation_index(*all, *vis, r);
        CHECK(idx == 7 - 2 * (r % 4));
        for (const std::string& v : {std::to_string(idx), kfd_uuid((*all)[static_cast<size_t>(idx)])}) {
          setenv("ROCR_VISIBLE_DEVICES", v.c_str(), 1);  // by index, and by UUID (what final sets)
          setenv("HIP_VISIBLE_DEVICES", "0", 1);
          const auto one = kfd_gpus(p);
          CHECK(one && one->size() == 1 && kfd_pick(*one, r, -1) == 0 && (*one)[0].pci_bus_id == bus_id(idx));
        }
        setenv("ROCR_VISIBLE_DEVICES", "7,6,5,4,3,2,1,0", 1);
        setenv("HIP_VISIBLE_DEVICES", "0,2,4,6", 1);
      }
    CHECK(all && kfd_isolation_index(*all, {}, 0) == -1 && kfd_isolation_index(*all, *all, -1) == -1);
  }
  unsetenv("HIP_VISIBLE_DEVICES");
  unsetenv("ROCR_VISIBLE_DEVICES");
  // a box that may open one of the host's eight GPUs (render node access), indexed 0 by both lists
  for (int x = 0; x < 8; ++x)
    if (x != 5) std::remove((root + "/dri/renderD" + std::to_string(128 + x)).c_str());
  setenv("ROCR_VISIBLE_DEVICES", "0", 1);
  setenv("HIP_VISIBLE_DEVICES", "0", 1);
  g = kfd_gpus(p);
  CHECK(g && g->size() == 1 && (*g)[0].pci_bus_id == bus_id(5) && (*g)[0].numa_node == 1);
  if (g && g->size() == 1) CHECK(kfd_pick(*g, 0, -1) == 0 && kfd_pick(*g, 3, -1) == 0);
  unsetenv("HIP_VISIBLE_DEVICES");
  unsetenv("ROCR_VISIBLE_DEVICES");
  CHECK(std::system(("rm -rf " + root).c_str()) == 0);
}

// The streaming root's cutter: batches cut after counting ahead (while a GPU's runtime starts) are the
// batches cut without it, by record count and by letter count; count_ahead stops at its batch bound
void test_cutter_count_ahead() {
  std::mt19937_64 rng(5);
  std::string text;
  int64_t records = 0;
  while (text.size() < (size_t{9} << 20)) {
    const int len = 1 + static_cast<int>(rng() % 24);
    for (int i = 0; i < len; ++i) text.push_back(static_cast<char>('A' + rng() % 26));
    text.push_back(rng() % 7 == 0 ? ' ' : '\n');
    ++records;
  }
  auto cuts = [&](int64_t max_rec, int64_t max_chr, int ahead_at_start) {
    AreaText t(text.data(), static_cast<int64_t>(text.size()));
    Cutter c(t);
    if (ahead_at_start > 0) {
      int steps = 0;
      while (c.count_ahead(max_rec, max_chr, ahead_at_start)) ++steps;
      CHECK(steps > 0);
      CHECK(!c.count_ahead(max_rec, max_chr, ahead_at_start));  // bound reached (or the text counted)
    }
    std::vector<std::vector<int64_t>> out;
    int64_t taken = 0;
    while (taken < records) {
      const BatchCut b = c.take(max_rec, max_chr);
      if (b.n == 0) break;
      taken += b.n;
      out.push_back({b.n, b.letters, b.begin, b.end, b.next, static_cast<int64_t>(b.chunks.size())});
    }
    CHECK(taken == records);
    return out;
  };
  for (int64_t max_rec : {int64_t{50000}, int64_t{1} << 40}) {
    const int64_t max_chr = max_rec == (int64_t{1} << 40) ? 700000 : INT64_MAX;
    const auto plain = cuts(max_rec, max_chr, 0);
    CHECK(plain.size() > 3);
    for (int ahead : {1, 3, 64}) {
      const auto early = cuts(max_rec, max_chr, ahead);
      CHECK(early.size() == plain.size());
      for (size_t i = 0; i < std::min(early.size(), plain.size()); ++i)  // n, letters, begin, next agree
        CHECK(early[i][0] == plain[i][0] && early[i][1] == plain[i][1] && early[i][2] == plain[i][2] &&
              early[i][4] == plain[i][4]);
    }
  }
}


// ---- narrow-integer forms at their exactness bounds (moc/kernel_bounds.hpp) ------------------------------
// Host replays of the kernels' integer arithmetic, with the same wrap-around (int16 / int32 / int8 casts),
// driven by the product's own rules: at the bound the rule picks the form and the replay equals brute force;
// one step past it the rule refuses the form, and the replay of the refused form goes wrong on the same
// input (so the bound is tight, not just safe). The adversarial input: Seq1 = "AZAZ...", records that are
// pieces of Seq1 at even offsets (every step Dt = +(W1 + W4)) and odd ones (-(W1 + W4)), constant records,
// and a periodic Seq1 that makes most offsets tie.
namespace xv {
constexpr uint8_t kA = 1, kZ = 26;

struct Fixture {
  std::vector<uint8_t> s1;
  RecordBatch batch;
  int64_t min_l2 = INT64_MAX, max_l2 = 0;
};

Fixture azaz(int64_t L1, int64_t lo, int64_t hi, uint32_t seed) {
  Fixture f;
  f.s1.resize(static_cast<size_t>(L1));
  for (int64_t j = 0; j < L1; ++j) f.s1[j] = (j & 1) ? kZ : kA;
  std::mt19937 rng(seed);
  auto add = [&](std::vector<uint8_t> r) {
    f.min_l2 = std::min<int64_t>(f.min_l2, static_cast<int64_t>(r.size()));
    f.max_l2 = std::max<int64_t>(f.max_l2, static_cast<int64_t>(r.size()));
    f.batch.push_back(r.data(), static_cast<int64_t>(r.size()));
  };
  for (int64_t L2 : {lo, hi, (lo + hi) / 2, hi - 1}) {
    if (L2 < lo || L2 > hi || L2 < 1) continue;
    for (int64_t at : {int64_t{0}, int64_t{1}, L1 - L2, L1 - L2 - 1}) {  // even / odd pieces of Seq1, both ends
      if (at < 0 || at + L2 > L1) continue;
      add(std::vector<uint8_t>(f.s1.begin() + at, f.s1.begin() + at + L2));
    }
    add(std::vector<uint8_t>(static_cast<size_t>(L2), kA));
    add(std::vector<uint8_t>(static_cast<size_t>(L2), kZ));
    std::vector<uint8_t> r(static_cast<size_t>(L2));
    for (auto& x : r) x = rng() % 2 ? kA : kZ;  // A/Z noise: large |D| on most diagonals
    add(r);
    for (auto& x : r) x = static_cast<uint8_t>(1 + rng() % 26);
    add(r);
  }
  return f;
}

bool same(const Result& a, const Result& b) { return a.score == b.score && a.n == b.n && a.k == b.k; }

uint64_t final_key(int32_t score, uint32_t idx) {
  return (static_cast<uint64_t>(static_cast<uint32_t>(score) ^ 0x80000000u) << 32) | (0xffffffffu - idx);
}
Result decode_key(uint64_t key, int64_t L2) {
  if (key == 0) return Result{kNoCandidateScore, 0, 0};
  const int32_t score = static_cast<int32_t>(static_cast<uint32_t>(key >> 32) ^ 0x80000000u);
  const uint32_t idx = 0xffffffffu - static_cast<uint32_t>(key);
  return Result{score, static_cast<int32_t>(idx / static_cast<uint32_t>(L2)),
                static_cast<int32_t>(idx % static_cast<uint32_t>(L2))};
}
int32_t S(const ScoreTable& t, const std::vector<uint8_t>& s1, int c, int64_t j) {
  return (c >= 1 && j < static_cast<int64_t>(s1.size())) ? t.score(c, s1[j]) : 0;
}

// swipe_search_kernel (swipe_impl.hpp) for one record: NOFF offsets per lane, KB k bits or the RK form,
// `steps` = its wave's longest record, `max_l2` = the batch's.
Result swipe_record(const ScoreTable& t, const std::vector<uint8_t>& s1, const uint8_t* s2, int64_t L2, int noff,
                    int kb, bool rk, int steps, int64_t max_l2, Semantics sem) {
  const int64_t L1 = static_cast<int64_t>(s1.size());
  const int KB = rk ? 1 : kb, KMASK = (1 << KB) - 1;
  const bool on = L2 <= L1;
  auto pf = [&](int c, int64_t j) {  // the LDS profile entry (int16)
    const int d = S(t, s1, c, j) - S(t, s1, c, j + 1);
    return static_cast<int16_t>(rk ? d : d * (1 << KB) - 1);
  };
  std::vector<int16_t> E(static_cast<size_t>(noff), static_cast<int16_t>(rk ? 0 : KMASK)),
      B(static_cast<size_t>(noff), INT16_MIN);
  int anchor = 0;
  for (int i = 0; i < steps; ++i) {
    const int c = on && i < L2 ? s2[i] : 0;
    for (int o = 0; o < noff; ++o) {
      E[o] = static_cast<int16_t>(E[o] + pf(c, i + o));
      B[o] = std::max(B[o], E[o]);
    }
    const int64_t j = noff + i;
    const int y = j < L1 ? s1[j] : 31;
    anchor += (y == 31 || c == 0) ? 0 : t.score(c, y);  // the int32 anchor table (swipe_build_tables)
  }
  const int64_t last = L1 - L2;
  const int64_t lim0 = on ? last + ((sem == Semantics::Spec || L2 == L1) ? 1 : 0) : 0;
  const int64_t lim1 = on && L2 >= 2 ? last : 0;
  (void)max_l2;
  // the selection's chain value C_o = (Tot_o + 2^15) << 16 + ~(o << KB), from the anchor diagonal down
  // (swipe_lane): the un-mutated key is C_o, the best mutant's C_{o+1} + ((d << 16) | (KMASK - k)) + 1. The
  // kernel skips the limit tests where they hold for its whole wave; applying them everywhere is the same.
  const uint32_t kStep = 1u << KB;
  uint32_t C = (static_cast<uint32_t>(anchor + 32768) << 16) + (0xffffu - (static_cast<uint32_t>(noff) << KB));
  uint32_t best = 0;
  for (int o = noff - 1; o >= 0; --o) {
    // D_o(L2) = E >> KB (E = D * 2^KB + KMASK - steps, steps <= KMASK); RK: E itself
    const int16_t dq = rk ? E[o] : static_cast<int16_t>(E[o] >> KB);
    const int16_t bd = rk ? B[o] : static_cast<int16_t>(B[o] >> KB);
    const uint32_t ds = (static_cast<uint32_t>(static_cast<uint16_t>(dq)) << 16) | kStep;
    const uint32_t m = (static_cast<uint32_t>(static_cast<uint16_t>(bd)) << 16) |
                       (rk ? 0u : static_cast<uint32_t>(static_cast<uint16_t>(B[o])) & static_cast<uint32_t>(KMASK));
    uint32_t k1 = C + m + 1u;
    C += ds;
    uint32_t k0 = C;
    k0 = o < lim0 ? k0 : 0u;
    k1 = o < lim1 ? k1 : 0u;
    best = std::max(best, std::max(k0, k1));
  }
  if (!on || best == 0u) return Result{kNoCandidateScore, 0, 0};
  const uint32_t idx = 0xffffu - (best & 0xffffu);
  if (!rk) return Result{static_cast<int>(best >> 16) - 32768, static_cast<int>(idx >> KB), static_cast<int>(idx & KMASK)};
  int kw = 0;
  if (idx & 1u) {  // the k re-walk on the winning diagonal (copy 0 of the profile, int sums): the first argmax
    const int ow = static_cast<int>(idx >> 1);
    int run = 0, top = INT32_MIN;
    for (int i = 0; i < steps; ++i) {
      run += pf(i < L2 ? s2[i] : 0, ow + i);
      if (run > top) {
        top = run;
        kw = i + 1;
      }
    }
  }
  return Result{static_cast<int>(best >> 16) - 32768, static_cast<int>(idx >> 1), (idx & 1u) ? kw : 0};
}

// short_search_kernel's packed form (Pk): (Dt << 16 | S) entries, one packed int16 add per cell.
Result short_pk_record(const ScoreTable& t, const std::vector<uint8_t>& s1, const uint8_t* s2, int64_t L2, int steps,
                       Semantics sem) {
  const int64_t L1 = static_cast<int64_t>(s1.size());
  if (L2 > L1) return Result{kNoCandidateScore, 0, 0};
  uint64_t best_key = 0;
  for (int64_t o = 0; o <= L1 - L2; ++o) {
    uint32_t acc = 0;
    int32_t best16 = INT32_MIN;
    for (int i = 0; i < steps; ++i) {
      const int c = i < L2 ? s2[i] : 0;
      const int sj = S(t, s1, c, o + i), sn = S(t, s1, c, o + i + 1);
      const uint32_t v = c ? ((static_cast<uint32_t>(sj - sn) << 16) | (static_cast<uint32_t>(sj) & 0xffffu)) : 0u;
      acc = ((acc + (v & 0xffffu)) & 0xffffu) | (((acc >> 16) + (v >> 16)) << 16);  // v_pk_add_u16
      best16 = std::max(best16, static_cast<int32_t>((acc & 0xffff0000u) | (0xffffu - static_cast<uint32_t>(i + 1))));
    }
    const int tot = static_cast<int16_t>(acc & 0xffffu), dfin = static_cast<int32_t>(acc) >> 16;
    const int64_t last = L1 - L2;
    uint64_t key = 0;
    if (o < last || (sem == Semantics::Spec || L2 == L1)) key = final_key(tot, static_cast<uint32_t>(o * L2));
    if (o < last && L2 >= 2 && best16 != INT32_MIN) {
      const int k = 0xffff - (best16 & 0xffff);
      key = std::max(key, final_key((best16 >> 16) + tot - dfin, static_cast<uint32_t>(o * L2 + k)));
    }
    best_key = std::max(best_key, key);
  }
  return decode_key(best_key, std::max<int64_t>(L2, 1));
}

// The int32 hot keys of the short (non-Pk) and LUT tile kernels (HotKey<false>, kernel_common.hpp).
Result key32_record(const ScoreTable& t, const std::vector<uint8_t>& s1, const uint8_t* s2, int64_t L2, int shift,
                    Semantics sem) {
  const int64_t L1 = static_cast<int64_t>(s1.size());
  if (L2 > L1) return Result{kNoCandidateScore, 0, 0};
  const int mask = (1 << shift) - 1;
  uint64_t best_key = 0;
  for (int64_t o = 0; o <= L1 - L2; ++o) {
    int P = 0, Pn = 0;
    int32_t best = INT32_MIN;
    for (int64_t i = 0; i < L2; ++i) {
      P += S(t, s1, s2[i], o + i);
      Pn += S(t, s1, s2[i], o + i + 1);
      const int32_t key = static_cast<int32_t>((static_cast<uint32_t>(P - Pn) << shift) | static_cast<uint32_t>(mask - (i + 1)));
      best = std::max(best, key);
    }
    const int64_t last = L1 - L2;
    uint64_t key = 0;
    if (o < last || (sem == Semantics::Spec || L2 == L1)) key = final_key(P, static_cast<uint32_t>(o * L2));
    if (o < last && L2 >= 2)
      key = std::max(key, final_key((best >> shift) + Pn, static_cast<uint32_t>(o * L2 + (mask - (best & mask)))));
    best_key = std::max(best_key, key);
  }
  return decode_key(best_key, L2);
}

// tile16_search_kernel + resolve_long_kernel (tile16_kernels.hip, align_kernels.hip) over a Profile16 whose
// bytes are taken as given (so a profile built past the bound wraps as the kernel would see it).
// kib > 0: the per-lane selection in 32-bit keys ((score << kib) + 2^31 + 2^kib - 1 - idx, kernel_bounds.hpp
// tile16_key32_bits), converted back to the 64-bit key at the end as the kernel does.
// i16: prof holds one int16 Dt per entry (the widened images' int16 profile): a lane's pair at column j is
// entries j and j + 1, read as int16.
Result tile16_record(const ScoreTable& t, const std::vector<uint8_t>& s1, const std::vector<uint16_t>& prof,
                     const uint8_t* s2, int64_t L2, int64_t span, Semantics sem, int kib = 0, bool i16 = false) {
  const int64_t L1 = static_cast<int64_t>(s1.size());
  auto entry = [&](int c, int64_t j) { return prof[static_cast<size_t>((c - 1) * L1 + j)]; };
  auto step_d = [&](int c, int64_t o, int64_t i) -> int16_t {  // Dt of offset o at step i as the kernel adds it
    if (i16) {
      const size_t e = static_cast<size_t>((c - 1) * L1 + (o & ~int64_t{1}) + i + (o & 1));
      return static_cast<int16_t>(prof[e]);
    }
    const uint16_t p = entry(c, (o & ~int64_t{1}) + i);
    return static_cast<int16_t>(static_cast<int8_t>(o & 1 ? p >> 8 : p & 0xff));
  };
  const int64_t need = L2 <= L1 ? L1 - L2 + 1 : 0;
  if (!need) return Result{kNoCandidateScore, 0, 0};
  std::vector<int32_t> Dc(static_cast<size_t>(need) + 1, 0), maxD(static_cast<size_t>(need) + 1, INT32_MIN);
  for (int64_t o = 0; o < need; ++o)
    for (int64_t i0 = 0; i0 < L2; i0 += bounds::kProf16Fold) {
      const int64_t m = std::min<int64_t>(bounds::kProf16Fold, L2 - i0);
      uint16_t accD = 0;
      int16_t bestD = INT16_MIN;
      bool any = false;
      for (int64_t j = 0; j < m; ++j) {
        const int16_t d = step_d(s2[i0 + j], o, i0 + j);
        accD = static_cast<uint16_t>(accD + static_cast<uint16_t>(d));
        if (i0 + j + 1 < L2) {
          bestD = std::max(bestD, static_cast<int16_t>(accD));
          any = true;
        }
      }
      if (any) maxD[o] = std::max(maxD[o], Dc[o] + bestD);
      Dc[o] += static_cast<int16_t>(accD);
    }
  std::vector<int32_t> tot(static_cast<size_t>(need) + 1, 0);
  for (int64_t o0 = 0; o0 < need; o0 += span) {
    const int64_t oA = std::min<int64_t>(o0 + span, need);
    int32_t acc = 0;
    for (int64_t i = 0; i < L2; ++i) {
      const int32_t tv = t.score(s2[i], oA + i < L1 ? s1[oA + i] : 0);
      acc += i16 ? tv : static_cast<int8_t>(tv);  // the int16 profile's anchors read the int32 LUT
    }
    for (int64_t o = oA - 1; o >= o0; --o) tot[o] = (acc += Dc[o]);
  }
  uint64_t best_key = 0;
  uint32_t best32 = 0;
  const uint32_t kmask = kib ? (1u << kib) - 1u : 0u;
  auto offer = [&](int32_t score, uint32_t idx) {
    if (kib)
      best32 = std::max(best32, (static_cast<uint32_t>(score) << kib) + (0x80000000u + kmask - idx));
    else
      best_key = std::max(best_key, final_key(score, idx));
  };
  const int64_t last = L1 - L2;
  for (int64_t o = 0; o < need; ++o) {
    if (o < last || (o == last && (sem == Semantics::Spec || L2 == L1))) offer(tot[o], static_cast<uint32_t>(2 * o));
    if (o < last && L2 >= 2) offer(maxD[o] + tot[o] - Dc[o], static_cast<uint32_t>(2 * o + 1));
  }
  if (kib && best32)
    best_key = final_key(static_cast<int32_t>(best32 >> kib) - (1 << (31 - kib)), kmask - (best32 & kmask));
  if (!best_key) return Result{kNoCandidateScore, 0, 0};
  const int32_t score = static_cast<int32_t>(static_cast<uint32_t>(best_key >> 32) ^ 0x80000000u);
  const uint32_t idx = 0xffffffffu - static_cast<uint32_t>(best_key);
  Result got{score, static_cast<int32_t>(idx >> 1), 0};
  if (idx & 1) {  // pass 2: smallest k >= 1 on the winning diagonal
    int32_t tot1 = 0, d = 0;
    for (int64_t i = 0; i < L2; ++i) tot1 += t.score(s2[i], s1[got.n + 1 + i]);
    got.k = -1;
    for (int64_t i = 0; i + 1 < L2 && got.k < 0; ++i) {
      d += t.score(s2[i], s1[got.n + i]) - t.score(s2[i], s1[got.n + i + 1]);
      if (d + tot1 == score) got.k = static_cast<int32_t>(i + 1);
    }
  }
  return got;
}

// Profile16 bytes without the range check (past the bound: the bytes wrap as a kernel would read them).
std::vector<uint16_t> raw_profile16(const ScoreTable& t, const std::vector<uint8_t>& s1, int64_t overhang) {
  const int64_t L1 = static_cast<int64_t>(s1.size());
  std::vector<uint16_t> e(static_cast<size_t>(26 * L1 + overhang), 0);
  for (int c = 1; c < kAlphabet; ++c)
    for (int64_t j = 0; j < L1; ++j) {
      auto d = [&](int64_t x) { return x < L1 ? t.score(c, s1[x]) - t.score(c, x + 1 < L1 ? s1[x + 1] : 0) : 0; };
      e[static_cast<size_t>((c - 1) * L1 + j)] =
          static_cast<uint16_t>((static_cast<uint32_t>(d(j + 1) & 0xff) << 8) | static_cast<uint32_t>(d(j) & 0xff));
    }
  return e;
}

// Counts the records whose replay differs from brute force.
template <typename F>
int mismatches(const ScoreTable& t, const Fixture& f, Semantics sem, F replay) {
  int bad = 0;
  for (int64_t r = 0; r < f.batch.size(); ++r) {
    const Result bf = brute_force_record(t, f.s1.data(), static_cast<int64_t>(f.s1.size()), f.batch.record(r),
                                         f.batch.length(r), sem);
    bad += same(replay(f.batch.record(r), f.batch.length(r)), bf) ? 0 : 1;
  }
  return bad;
}
}  // namespace xv

void test_swipe_replay_bounds() {
  using namespace xv;
  // (L1, record lengths): records <= 16 letters (4 record words, 5 k bits), <= 32 (8 words, 6 k bits),
  // 33..64 (16 words: RK only). W1 = W4 = w, W2 = W3 = 0: Dt = 2w at every step of an even-offset piece.
  struct Case {
    int64_t L1, lo, hi;
  };
  for (const Case cs : {Case{40, 6, 16}, Case{60, 20, 32}, Case{70, 40, 64}, Case{100, 40, 64}, Case{130, 67, 96},
                        Case{190, 127, 128}}) {
    const Fixture f = azaz(cs.L1, cs.lo, cs.hi, static_cast<uint32_t>(cs.L1));
    const int l2w = bounds::swipe_record_words(f.max_l2), kb = bounds::swipe_kbits(l2w);
    // offsets per lane as swipe_choice sizes them: the semantics' widest range, a multiple of 4
    auto noff_of = [&](Semantics sem) {
      const int64_t need = dev::swipe_offsets(cs.L1, std::min(f.min_l2, cs.L1), sem == Semantics::Spec);
      return static_cast<int>(((std::max<int64_t>(need, 4) + 3) / 4) * 4);
    };
    const int steps = static_cast<int>(f.max_l2);
    // the largest w of each form, from the rule itself
    int w_kbits = 0, w_rk = 0;
    for (int w = 1; w <= 1100; ++w) {
      const bounds::SwipeKeys k = bounds::swipe_keys(w, f.max_l2);
      if (k == bounds::SwipeKeys::KBits) w_kbits = w;
      if (k == bounds::SwipeKeys::RK) w_rk = w;
    }
    CHECK(2 * w_rk * f.max_l2 < 32767 && 2 * (w_rk + 1) * f.max_l2 >= 32767);  // int16 sums end the RK form
    if (l2w >= 16) CHECK(w_kbits == 0);      // 33..128-letter records: RK only
    if (l2w == 4) CHECK(w_kbits == 31);      // 2*31*16*32 + 32 < 32767 <= 2*32*16*32 + 32
    if (l2w == 8) CHECK(w_kbits == 7);       // 2*7*32*64 + 64 < 32767 <= 2*8*32*64 + 64
    for (Semantics sem : {Semantics::Reference, Semantics::Spec}) {
      const int noff = noff_of(sem);
      if (w_kbits > 0) {
        const ScoreTable at = ScoreTable::build(Weights{{w_kbits, 0, 0, w_kbits}});
        CHECK(mismatches(at, f, sem, [&](const uint8_t* s2, int64_t L2) {
                return swipe_record(at, f.s1, s2, L2, noff, kb, false, steps, f.max_l2, sem);
              }) == 0);
        // one past: the rule takes the RK form, which is exact there, and the k-bit keys would wrap
        const ScoreTable past = ScoreTable::build(Weights{{w_kbits + 1, 0, 0, w_kbits + 1}});
        CHECK(bounds::swipe_keys(w_kbits + 1, f.max_l2) == bounds::SwipeKeys::RK);
        CHECK(mismatches(past, f, sem, [&](const uint8_t* s2, int64_t L2) {
                return swipe_record(past, f.s1, s2, L2, noff, kb, true, steps, f.max_l2, sem);
              }) == 0);
        CHECK(mismatches(past, f, sem, [&](const uint8_t* s2, int64_t L2) {
                return swipe_record(past, f.s1, s2, L2, noff, kb, false, steps, f.max_l2, sem);
              }) > 0);
      }
      const ScoreTable at = ScoreTable::build(Weights{{w_rk, 0, 0, w_rk}});
      CHECK(mismatches(at, f, sem, [&](const uint8_t* s2, int64_t L2) {
              return swipe_record(at, f.s1, s2, L2, noff, kb, true, steps, f.max_l2, sem);
            }) == 0);
      // one past: no swipe form. The rule is conservative by a step there (this fixture's sums stay exact
      // up to 2 w (L2 - 1)), but where w L2 reaches 2^15 the keys' 16-bit score wraps and the RK form is wrong
      CHECK(bounds::swipe_keys(w_rk + 1, f.max_l2) == bounds::SwipeKeys::None);
      const int w_wrap = static_cast<int>((32768 + f.max_l2 - 1) / f.max_l2);
      const ScoreTable wrap = ScoreTable::build(Weights{{w_wrap, 0, 0, w_wrap}});
      CHECK(mismatches(wrap, f, sem, [&](const uint8_t* s2, int64_t L2) {
              return swipe_record(wrap, f.s1, s2, L2, noff, kb, true, steps, f.max_l2, sem);
            }) > 0);
    }
  }
}

void test_short_replay_bounds() {
  using namespace xv;
  // records of 67..85 letters under a 130-letter Seq1: <= 64 lanes per record, too long for the swipe kernel
  const Fixture f = azaz(130, 67, 85, 5);
  const int steps = static_cast<int>(f.max_l2);
  int w_pk = 0;
  for (int w = 1; w <= 400; ++w)
    if (bounds::short_pk_exact(w, f.max_l2)) w_pk = w;
  CHECK(w_pk == 192);  // 2*192*85 = 32640 < 32767 <= 2*193*85
  for (Semantics sem : {Semantics::Reference, Semantics::Spec}) {
    const ScoreTable at = ScoreTable::build(Weights{{w_pk, 0, 0, w_pk}});
    CHECK(mismatches(at, f, sem, [&](const uint8_t* s2, int64_t L2) { return short_pk_record(at, f.s1, s2, L2, steps, sem); }) == 0);
    const ScoreTable past = ScoreTable::build(Weights{{w_pk + 1, 0, 0, w_pk + 1}});
    CHECK(mismatches(past, f, sem, [&](const uint8_t* s2, int64_t L2) { return short_pk_record(past, f.s1, s2, L2, steps, sem); }) > 0);
    // past the packed form: int32 keys, exact up to their own bound and wrapping one past it
    const int shift = bounds::key_shift(w_pk + 1, f.max_l2);
    CHECK(shift == 7);
    CHECK(mismatches(past, f, sem, [&](const uint8_t* s2, int64_t L2) { return key32_record(past, f.s1, s2, L2, shift, sem); }) == 0);
    int w32 = 0;
    for (int w = 98000; w <= 99000; ++w)
      if (bounds::key_shift(w, f.max_l2) == shift) w32 = w;
    CHECK(w32 == 98689);  // 2*98689*85 << 7 < 2^31 <= 2*98690*85 << 7
    CHECK(bounds::key_shift(w32 + 1, f.max_l2) == 0);
    const ScoreTable at32 = ScoreTable::build(Weights{{w32, 0, 0, w32}});
    CHECK(mismatches(at32, f, sem, [&](const uint8_t* s2, int64_t L2) { return key32_record(at32, f.s1, s2, L2, shift, sem); }) == 0);
    const ScoreTable past32 = ScoreTable::build(Weights{{w32 + 1, 0, 0, w32 + 1}});
    CHECK(mismatches(past32, f, sem, [&](const uint8_t* s2, int64_t L2) { return key32_record(past32, f.s1, s2, L2, shift, sem); }) > 0);
  }
}

void test_tile16_replay_bounds() {
  using namespace xv;
  // long records (several 64-step folds) under a 600-letter Seq1; W1 + W4 = 127 is the largest Dt a byte holds
  const Fixture f = azaz(600, 150, 400, 9);
  for (Semantics sem : {Semantics::Reference, Semantics::Spec}) {
    for (int64_t span : {512, 1024}) {
      const ScoreTable at = ScoreTable::build(Weights{{63, 0, 0, 64}});
      CHECK(profile16_fits(at));
      Profile16 prof;
      CHECK(build_profile16(at, f.s1.data(), 600, span, prof));
      CHECK(mismatches(at, f, sem, [&](const uint8_t* s2, int64_t L2) {
              return tile16_record(at, f.s1, prof.entries, s2, L2, span, sem);
            }) == 0);
      const ScoreTable past = ScoreTable::build(Weights{{64, 0, 0, 64}});
      CHECK(!profile16_fits(past) && !build_profile16(past, f.s1.data(), 600, span, prof));
      const std::vector<uint16_t> wrapped = raw_profile16(past, f.s1, span);
      CHECK(mismatches(past, f, sem, [&](const uint8_t* s2, int64_t L2) {
              return tile16_record(past, f.s1, wrapped, s2, L2, span, sem);
            }) > 0);
    }
  }
}

void test_tile16_i16_replay() {
  using namespace xv;
  // weights past the byte pairs: |Dt| = W1 + W4 = 511 in the int16 profile (exact: 64-step partial sums stay
  // within 64 * 511 < 2^15), and 512 refused by the rule; the profile wrapped to int16 past it replays wrong
  const Fixture f = azaz(600, 150, 400, 13);
  for (Semantics sem : {Semantics::Reference, Semantics::Spec}) {
    const ScoreTable at = ScoreTable::build(Weights{{255, 0, 0, 256}});
    CHECK(!profile16_fits(at) && profile16_i16_fits(at));
    Profile16 prof;
    CHECK(!build_profile16(at, f.s1.data(), 600, 512, prof) && build_profile16(at, f.s1.data(), 600, 512, prof, true));
    CHECK(prof.i16);
    CHECK(mismatches(at, f, sem, [&](const uint8_t* s2, int64_t L2) {
            return tile16_record(at, f.s1, prof.entries, s2, L2, 512, sem, 0, true);
          }) == 0);
    const ScoreTable past = ScoreTable::build(Weights{{256, 0, 0, 256}});
    CHECK(!profile16_i16_fits(past) && !build_profile16(past, f.s1.data(), 600, 512, prof, true));
  }
}

void test_tile16_key32_replay() {
  using namespace xv;
  // tile16's 32-bit selection keys against its 64-bit ones (the latter pinned to brute force above): W1 = 127,
  // L1 = 2600 (13 index bits): even pieces of Seq1 score 127 * L2, inside 2^18 up to L2 = 2064
  const ScoreTable tt = ScoreTable::build(Weights{{127, 0, 0, 0}});
  CHECK(profile16_fits(tt));
  CHECK(bounds::tile16_key32_bits(2600, tt.max_abs(), 2064) == 13 && bounds::tile16_key32_bits(2600, tt.max_abs(), 2065) == 0);
  for (int64_t hi : {2064, 2065}) {
    const Fixture f = azaz(2600, hi - 3, hi, 11);
    Profile16 prof;
    CHECK(build_profile16(tt, f.s1.data(), 2600, 512, prof));
    int differ = 0;
    for (int64_t r = 0; r < f.batch.size(); ++r) {
      const Result a = tile16_record(tt, f.s1, prof.entries, f.batch.record(r), f.batch.length(r), 512, Semantics::Reference, 13);
      const Result b = tile16_record(tt, f.s1, prof.entries, f.batch.record(r), f.batch.length(r), 512, Semantics::Reference, 0);
      differ += same(a, b) ? 0 : 1;
    }
    CHECK(hi == 2064 ? differ == 0 : differ > 0);  // one past the bound the 32-bit keys wrap
  }
}

int main() {
  const std::vector<std::pair<const char*, std::function<void()>>> tests = {
      {"score_table", test_score_table}, {"parser", test_parser},     {"stream_reader", test_stream_reader},
      {"partition", test_partition},     {"keys", test_keys},         {"pack5", test_pack5},
      {"engine_vs_brute_force", test_engine_vs_brute_force},          {"formatter", test_formatter},
      {"profile16", test_profile16},     {"releaser", test_releaser},   {"slices", test_slices},
      {"narrow_lengths", test_narrow_lengths}, {"result_formats", test_result_formats},
      {"write_runs", test_write_runs},   {"pack33", test_pack33},
      {"kfd_topology", test_kfd_topology}, {"kfd_topology_8gpu", test_kfd_topology_8gpu},
      {"cutter_count_ahead", test_cutter_count_ahead}, {"swipe_replay_bounds", test_swipe_replay_bounds},
      {"short_replay_bounds", test_short_replay_bounds}, {"tile16_replay_bounds", test_tile16_replay_bounds},
      {"tile16_key32_replay", test_tile16_key32_replay}, {"tile16_i16_replay", test_tile16_i16_replay},
      {"profile16_lds_bytes", test_profile16_lds_bytes}, {"watchdog", test_watchdog}};
  for (const auto& t : tests) {
    const int before = g_failed;
    t.second();
    std::printf("%-24s %s\n", t.first, g_failed == before ? "ok" : "FAILED");
  }
  std::printf("%d checks, %d failed\n", g_checks, g_failed);
  return g_failed ? 1 : 0;
}
