#include "moc/score_table.hpp"

#include <algorithm>
#include <cstdlib>

#include "moc/kernel_bounds.hpp"

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

bool profile16_fits(const ScoreTable& t) {
  int32_t dmin = INT32_MAX, dmax = INT32_MIN, tabs = 0;
  for (int c = 1; c < kAlphabet; ++c)
    for (int x = 0; x < kAlphabet; ++x) {  // 0: the pad code after Seq1
      tabs = std::max(tabs, std::abs(t.score(c, x)));
      for (int y = 0; y < kAlphabet; ++y) {
        const int32_t d = t.score(c, x) - t.score(c, y);
        dmin = std::min(dmin, d);
        dmax = std::max(dmax, d);
      }
    }
  // the kernel's anchor diagonals read T itself as int8 too (negative weights through the API could give
  // a narrow range of large values)
  return bounds::profile16_exact(dmin, dmax, tabs);
}

bool profile16_i16_fits(const ScoreTable& t) {
  int32_t dmin = INT32_MAX, dmax = INT32_MIN;
  for (int c = 1; c < kAlphabet; ++c)
    for (int x = 0; x < kAlphabet; ++x)
      for (int y = 0; y < kAlphabet; ++y) {
        const int32_t d = t.score(c, x) - t.score(c, y);
        dmin = std::min(dmin, d);
        dmax = std::max(dmax, d);
      }
  return bounds::profile16_i16_exact(dmin, dmax);
}

bool build_profile16(const ScoreTable& t, const uint8_t* seq1, int64_t L1, int64_t overhang, Profile16& out,
                     bool allow_i16) {
  if (L1 <= 0 || overhang < 0) return false;
  const bool pairs = profile16_fits(t);
  if (!pairs && !(allow_i16 && profile16_i16_fits(t))) return false;
  out.row = L1;
  out.i16 = !pairs;
  out.entries.assign(static_cast<size_t>((kAlphabet - 1) * L1 + overhang), 0);
  std::vector<int32_t> d(static_cast<size_t>(L1) + 1, 0);
  for (int c = 1; c < kAlphabet; ++c) {
    for (int64_t j = 0; j < L1; ++j) d[j] = t.score(c, seq1[j]) - t.score(c, j + 1 < L1 ? seq1[j + 1] : 0);
    uint16_t* r = out.entries.data() + static_cast<size_t>(c - 1) * static_cast<size_t>(L1);
    for (int64_t j = 0; j < L1; ++j)
      r[j] = pairs ? static_cast<uint16_t>((static_cast<uint32_t>(d[j + 1] & 0xff) << 8) | static_cast<uint32_t>(d[j] & 0xff))
                   : static_cast<uint16_t>(static_cast<int16_t>(d[j]));
  }
  return true;
}

char ScoreTable::class_char(PairClass c) {
  static const char chars[4] = {'$', '%', '#', ' '};
  return chars[c];
}

}  // namespace moc
