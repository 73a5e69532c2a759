#include "moc/score_table.hpp"

#include <algorithm>
#include <cstdlib>

namespace moc {

const std::vector<std::string>& first_type_groups() {
  static const std::vector<std::string> g = {"NDEQ", "NEQK", "STA", "MILV", "QHRK",
                                             "NHQK", "FYW",  "HY",  "MILF"};
  return g;
}

const std::vector<std::string>& second_type_groups() {
  static const std::vector<std::string> g = {"SAG",  "ATV",    "CSA",    "SGND",   "STPA", "STNK",
                                             "NEQHRK", "NDEQHK", "SNDEQK", "HFY", "FVLIM"};
  return g;
}

namespace {
// Marks every ordered pair inside each group word (symmetric, diagonal included).
void mark_groups(const std::vector<std::string>& groups, std::array<uint8_t, kLutStride * kLutStride>& m) {
  for (const auto& word : groups) {
    for (char x : word) {
      for (char y : word) {
        int a = letter_code(static_cast<unsigned char>(x));
        int b = letter_code(static_cast<unsigned char>(y));
        m[a * kLutStride + b] = 1;
        m[b * kLutStride + a] = 1;
      }
    }
  }
}
}  // namespace

ScoreTable ScoreTable::build(const Weights& w) {
  ScoreTable t;
  t.weights = w;
  std::array<uint8_t, kLutStride * kLutStride> g1{}, g2{};
  mark_groups(first_type_groups(), g1);
  mark_groups(second_type_groups(), g2);
  const int32_t value[4] = {w.w[0], -w.w[1], -w.w[2], -w.w[3]};
  for (int a = 0; a < kLutStride; ++a) {
    for (int b = 0; b < kLutStride; ++b) {
      const int idx = a * kLutStride + b;
      PairClass c = kSpace;
      const bool letters = a >= 1 && a <= 26 && b >= 1 && b <= 26;
      if (letters) {
        if (a == b)
          c = kDollar;
        else if (g1[idx])
          c = kPercent;
        else if (g2[idx])
          c = kHash;
      }
      t.cls[idx] = c;
      t.lut[idx] = value[c];
    }
  }
  return t;
}

int32_t ScoreTable::max_abs() const {
  int32_t m = 0;
  for (int i = 0; i < 4; ++i) m = std::max<int32_t>(m, std::abs(weights.w[i]));
  return m;
}

char ScoreTable::class_char(PairClass c) {
  static const char chars[4] = {'$', '%', '#', ' '};
  return chars[c];
}

}  // namespace moc
