// Parser fill throughput by letter code: BulkParser::fill_slice into the GPU wire form (packed letters +
// sparse offsets + uint16 lengths) for 5-bit / P24 / P33 letters on an input6-shaped text (CPU only).
// Build: g++ -O3 -std=c++17 -fopenmp -Icsrc/include tools/fill_bench.cpp build/obj/io.o build/obj/problem.o \
//          build/obj/score_table.o build/obj/partition.o build/obj/runtime/runtime.o -ldl -o build/fill_bench
#include <chrono>
#include <cstdio>
#include <random>
#include <string>
#include <vector>

#include "moc/io.hpp"
#include "moc/problem.hpp"
#include "moc/wire.hpp"

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? std::atoll(argv[1]) : 20000000;
  std::mt19937_64 rng(1);
  std::string text = "4 3 2 10\nABCDEFGHIJKLMNOPQRSTUVWXYZ\n" + std::to_string(n) + "\n";
  text.reserve(static_cast<size_t>(n) * 10 + 64);
  for (int64_t i = 0; i < n; ++i) {
    const int L = 6 + static_cast<int>(rng() % 6);
    for (int j = 0; j < L; ++j) text += static_cast<char>('A' + rng() % 26);
    text += '\n';
  }
  moc::BulkParser p(text.data(), text.size());
  const moc::AreaSlice s = p.slice(0, p.count());
  std::vector<int64_t> sp(static_cast<size_t>(moc::sparse_count(s.records, moc::kSparseShift)));
  std::vector<uint16_t> l16(static_cast<size_t>(s.records));
  std::vector<uint8_t> out(static_cast<size_t>(moc::packed5_bytes(s.letters)) + 64);
  for (int rep = 0; rep < 3; ++rep)
    for (int pack : {5, 24, 33}) {
      const auto t0 = std::chrono::steady_clock::now();
      p.fill_slice(s, nullptr, out.data(), nullptr, sp.data(), l16.data(), pack);
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      std::printf("pack=%d letters=%lld fill_ms=%.1f\n", pack, static_cast<long long>(s.letters), ms);
    }
  return 0;
}
