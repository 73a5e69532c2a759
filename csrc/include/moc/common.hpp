// Core types shared by every layer of the framework (host, device launchers, comm, CLI).
//
// Parity map (reference = /root/reference):
//   * problem contract ............ parallel_finalEx2021_summer.pdf p.1-6, SURVEY.md §0.3-0.4
//   * buffer limits (3000/2000) ... myProto.h:3-4  -> runtime Limits (defaults: unlimited)
//   * result triple (score,n,k) ... main.c:123-125, main.c:204
//   * ROOT rank enum .............. main.c:9-12    -> kRoot
#pragma once

#include <cstddef>
#include <cstdint>
#include <limits>
#include <stdexcept>
#include <string>

namespace moc {

// Letters are encoded 1..26 ('A'..'Z'); 0 is never a valid letter (padding / "no letter").
// The reference indexes its 27x27 tables with c - 'A' + 1 (main.c:40-41) — same alphabet.
constexpr int kAlphabet = 27;
constexpr int kLutStride = 32;  // LUT rows padded to 32 ints (one LDS bank row half)

constexpr int kRoot = 0;  // main.c:9-12: the reader / printer / scatter-gather root

// Reference-compatible limits (myProto.h:3-4 hold 3000/2000 *bytes incl. NUL*). The new framework
// allocates dynamically; these are only enforced with --strict-limits.
constexpr int64_t kSpecMaxSeq1 = 3000;
constexpr int64_t kSpecMaxSeq2 = 2000;

struct Weights {
  int32_t w[4] = {0, 0, 0, 0};  // W1 ($), W2 (%), W3 (#), W4 (' ')
};

// Which (offset, mutant) candidates are searched (bug B8).
//   Reference: offsets [0, L1-L2) x mutants [0, L2) (mutant 0 = no hyphen), L2 == L1 -> (0,0) only.
//   Spec:      Reference + the un-mutated sequence at the final offset n = L1-L2.
enum class Semantics : int32_t { Reference = 0, Spec = 1 };

// One output row "#i: score: S, n: N, k: K" (main.c:204).
struct Result {
  int32_t score;
  int32_t n;
  int32_t k;
};
static_assert(sizeof(Result) == 12, "Result must stay a packed 12-byte POD (device + MPI wire format)");

constexpr int32_t kNoCandidateScore = std::numeric_limits<int32_t>::min();  // L2 > L1 (cudaFunctions.cu:113)

inline Result no_candidate() { return Result{kNoCandidateScore, 0, 0}; }

class Error : public std::runtime_error {
 public:
  explicit Error(const std::string& what) : std::runtime_error(what) {}
};

// Encodes a byte as a letter code (1..26) or returns 0 for a non-letter.
inline int letter_code(unsigned char c) {
  if (c >= 'a' && c <= 'z') return c - 'a' + 1;
  if (c >= 'A' && c <= 'Z') return c - 'A' + 1;
  return 0;
}

inline char code_letter(int code) { return static_cast<char>('A' + code - 1); }

}  // namespace moc
