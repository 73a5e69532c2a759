// Parser throughput on an input6-shaped text (CPU only): pass 1 (count_tokens over thread chunks) against
// pass 2 (BulkParser::fill_slice into the GPU wire form: packed letters + sparse offsets + uint16 lengths)
// for 5-bit / P33 letters, and the byte form the CPU engine takes. MOC_FILL_SIMD=0 forces the
// portable SSE2 encoder (A/B against the AVX-512 one).
// Build: make build/fill_bench   (or see the Makefile rule)   Run: build/fill_bench [records]
#include <omp.h>

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
  const double gb = text.size() / 1e9;
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto ms_since = [](auto t0) { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
  moc::BulkParser p(text.data(), text.size(), {}, false);
  const int nch = 4 * omp_get_max_threads();
  std::vector<int64_t> st = p.chunk_starts(nch), tk(nch), ch(nch);
  for (int rep = 0; rep < 3; ++rep) {
    const auto t0 = now();
    p.count_chunks(st, 0, nch, tk.data(), ch.data());
    const double ms = ms_since(t0);
    std::printf("count threads=%d ms=%.1f GB/s=%.1f\n", omp_get_max_threads(), ms, gb / (ms / 1e3));
  }
  p.set_chunks(st, tk.data(), ch.data());
  const moc::AreaSlice s = p.slice(0, p.count());
  std::vector<int64_t> sp(static_cast<size_t>(moc::sparse_count(s.records, moc::kSparseShift)));
  std::vector<uint16_t> l16(static_cast<size_t>(s.records));
  std::vector<uint8_t> out(static_cast<size_t>(moc::packed5_bytes(s.letters)) + 64);
  std::vector<uint8_t> codes(static_cast<size_t>(s.letters) + 64);
  std::vector<int64_t> offs(static_cast<size_t>(s.records) + 1);
  for (int rep = 0; rep < 3; ++rep) {
    for (int pack : {5, 33}) {
      const auto t0 = now();
      p.fill_slice(s, nullptr, out.data(), nullptr, sp.data(), l16.data(), pack);
      const double ms = ms_since(t0);
      std::printf("fill pack=%d letters=%lld ms=%.1f GB/s=%.1f\n", pack, static_cast<long long>(s.letters), ms,
                  gb / (ms / 1e3));
    }
    {  // the sliced path's "wire" step: uint16 lengths -> base-6 narrow lengths
      std::vector<uint8_t> lens(static_cast<size_t>(moc::narrow_lengths_bytes(s.records, moc::kLenBase6)) + 8);
      const auto tl = now();
      moc::pack_lengths16(l16.data(), s.records, moc::kLenBase6, 6, lens.data());
      std::printf("pack_lengths16 base6 records=%lld ms=%.1f\n", static_cast<long long>(s.records), ms_since(tl));
    }
    const auto t0 = now();
    p.fill_slice(s, codes.data(), nullptr, offs.data());
    const double ms = ms_since(t0);
    std::printf("fill bytes+offsets ms=%.1f GB/s=%.1f\n", ms, gb / (ms / 1e3));
    // the rccl transport's root packs byte codes into P33 per rank piece (pack33: whole blocks in parallel)
    const auto t1 = now();
    moc::pack33(codes.data(), s.letters, out.data());
    const double ms1 = ms_since(t1);
    std::printf("pack33 from bytes ms=%.1f G letters/s=%.2f out GB/s=%.1f\n", ms1, s.letters / 1e6 / ms1,
                moc::packed33_bytes(s.letters) / 1e6 / ms1);
  }
  return 0;
}
