// Fused pair-score lookup table.
//
// The reference builds two 27x27 char membership matrices (build_mat, main.c:14-44, groups at
// main.c:59-60), uploads them plus the weights into __constant__ memory (cudaFunctions.cu:9-13,35-61)
// and, per character pair, walks an if/else chain ($ -> % -> # -> ' ', cudaFunctions.cu:132-153)
// followed by a 4-bin atomic histogram and a weight dot product.
//
// Here the whole chain collapses into ONE int32 table T[a][b] = +W1 / -W2 / -W3 / -W4 (fully
// initialised — fixes bug B1, main.c:24), so the device inner loop is a single LDS gather + add.
#pragma once

#include <array>
#include <cstdint>
#include <string>
#include <vector>

#include "moc/common.hpp"

namespace moc {

enum PairClass : uint8_t { kDollar = 0, kPercent = 1, kHash = 2, kSpace = 3 };

// First-type ("%") groups: PDF p.1-2, main.c:59 (9 groups; the reference pads with two "").
const std::vector<std::string>& first_type_groups();
// Second-type ("#") groups: PDF p.2, main.c:60 (11 groups).
const std::vector<std::string>& second_type_groups();

struct ScoreTable {
  Weights weights;
  // cls[a*32+b]: PairClass of (Seq2 letter a, Seq1 letter b), codes 1..26; row/col 0 and 27..31 = kSpace.
  std::array<uint8_t, kLutStride * kLutStride> cls{};
  // lut[a*32+b]: signed score contribution of that pair.
  std::array<int32_t, kLutStride * kLutStride> lut{};

  static ScoreTable build(const Weights& w);

  int32_t score(int a, int b) const { return lut[a * kLutStride + b]; }
  PairClass pair_class(int a, int b) const { return static_cast<PairClass>(cls[a * kLutStride + b]); }

  int32_t max_abs() const;  // max |T| — used to pick safe device key widths
  // The reference's display character for a pair class ('$', '%', '#', ' ').
  static char class_char(PairClass c);
};

// Packed Seq1 difference profile of the tile16 kernel (csrc/src/hip/tile16_kernels.hip). With
//     D[c][j] = T[c][Seq1[j]] - T[c][Seq1[j+1]]   (Seq1[L1] = pad code 0; D[c][j >= L1] = 0)
// the entry for Seq2 letter c = 1..26 (row c-1) and Seq1 position j is the uint16
//     low byte = D[c][j] (int8),  high byte = D[c][j+1] (int8)
// i.e. the step-i terms of the two adjacent diagonals o = j - i and o + 1 that one lane carries: one
// LDS read feeds two cells, whose running sums are D_o(k) = P_o(k) - P_{o+1}(k). Rows are L1 entries
// long and packed back to back; `overhang` zero entries follow the last row (reads of tiles past the
// valid offsets). Returns false (out untouched) when some D does not fit a signed byte.
struct Profile16 {
  std::vector<uint16_t> entries;
  int64_t row = 0;   // entries per row (= L1)
  bool i16 = false;  // entries are int16 Dt[c][j] (build_profile16 with allow_i16), not byte pairs
};
// True when every Dt and T of the table fit the profile bytes (moc/kernel_bounds.hpp profile16_exact).
bool profile16_fits(const ScoreTable& t);
// True when every Dt fits the int16 profile (moc/kernel_bounds.hpp profile16_i16_exact).
bool profile16_i16_fits(const ScoreTable& t);
// Byte pairs when the table fits them; otherwise, with allow_i16, one int16 Dt per entry when it fits that.
bool build_profile16(const ScoreTable& t, const uint8_t* seq1, int64_t L1, int64_t overhang, Profile16& out,
                     bool allow_i16 = false);

}  // namespace moc
