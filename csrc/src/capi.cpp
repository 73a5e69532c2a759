// C ABI implementation (see moc/capi.h).
#include "moc/capi.h"

#include <cstring>
#include <exception>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "moc/cpu_engine.hpp"
#include "moc/device.hpp"
#include "moc/hip_engine.hpp"
#include "moc/io.hpp"
#include "moc/partition.hpp"
#include "moc/problem.hpp"
#include "moc/runtime/device.hpp"
#include "moc/runtime/hip_check.hpp"
#include "moc/runtime/log.hpp"
#include "moc/runtime/pinned.hpp"
#include "moc/score_table.hpp"

static_assert(sizeof(moc_result) == sizeof(moc::Result), "ABI result layout");

namespace {
thread_local std::string g_err;

template <class F>
int guard(F&& f) {
  try {
    f();
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
  } catch (...) {
    g_err = "unknown error";
  }
  return -1;
}

moc::Weights weights_of(const int32_t* w4) {
  moc::Weights w;
  for (int i = 0; i < 4; ++i) w.w[i] = w4[i];
  return w;
}

// moc_host_register calls -> the registrations each made (released together by moc_host_unregister)
std::mutex g_host_regs_mu;
std::map<void*, std::vector<void*>> g_host_regs;

moc::RecordBatch view_batch(const uint8_t* codes, const int64_t* offsets, int64_t n) {
  moc::RecordBatch b;
  const int64_t base = offsets[0];
  b.codes.assign(codes + base, codes + offsets[n]);
  b.offsets.resize(static_cast<size_t>(n) + 1);
  for (int64_t i = 0; i <= n; ++i) b.offsets[i] = offsets[i] - base;
  return b;
}
}  // namespace

extern "C" {

const char* moc_last_error(void) { return g_err.c_str(); }
int moc_abi_version(void) { return 1; }
int moc_set_log_level(const char* level) {
  return guard([&] { moc::log_set_level(std::string(level)); });
}

void* moc_parse(const char* data, size_t len, int strict_limits) {
  moc::Problem* p = nullptr;
  int rc = guard([&] {
    moc::ParseOptions opt;
    opt.strict_limits = strict_limits != 0;
    p = new moc::Problem(moc::parse_problem(data, len, opt));
  });
  return rc == 0 ? p : nullptr;
}

void moc_problem_free(void* p) { delete static_cast<moc::Problem*>(p); }

int moc_problem_info(void* p, int32_t* weights4, int64_t* L1, int64_t* n, int64_t* total_chars) {
  return guard([&] {
    auto* pr = static_cast<moc::Problem*>(p);
    for (int i = 0; i < 4; ++i) weights4[i] = pr->weights.w[i];
    *L1 = pr->L1();
    *n = pr->seq2.size();
    *total_chars = pr->seq2.total_chars();
  });
}
const uint8_t* moc_problem_seq1(void* p) { return static_cast<moc::Problem*>(p)->seq1.data(); }
const uint8_t* moc_problem_codes(void* p) { return static_cast<moc::Problem*>(p)->seq2.codes.data(); }
const int64_t* moc_problem_offsets(void* p) { return static_cast<moc::Problem*>(p)->seq2.offsets.data(); }

int64_t moc_format_results(const moc_result* r, int64_t n, int64_t first_index, char* buf, int64_t cap) {
  int64_t written = -1;
  guard([&] {
    std::string s = moc::format_results(reinterpret_cast<const moc::Result*>(r), n, first_index);
    if (static_cast<int64_t>(s.size()) > cap) throw moc::Error("format buffer too small");
    std::memcpy(buf, s.data(), s.size());
    written = static_cast<int64_t>(s.size());
  });
  return written;
}

int64_t moc_packed5_bytes(int64_t n_chars) { return moc::packed5_bytes(n_chars); }
int moc_pack5(const uint8_t* codes, int64_t n, uint8_t* out) {
  return guard([&] { moc::pack5(codes, n, out); });
}
int moc_unpack5(const uint8_t* packed, int64_t begin, int64_t n, uint8_t* out) {
  return guard([&] { moc::unpack5(packed, begin, n, out); });
}
int64_t moc_packed33_bytes(int64_t n_chars) { return moc::packed33_bytes(n_chars); }
int moc_pack33(const uint8_t* codes, int64_t n, uint8_t* out) {
  return guard([&] { moc::pack33(codes, n, out); });
}
int moc_unpack33(const uint8_t* packed, int64_t begin, int64_t n, uint8_t* out) {
  return guard([&] { moc::unpack33(packed, begin, n, out); });
}
int moc_pack_lengths(const int64_t* offsets, int64_t n, int bits, int64_t base, uint8_t* out) {
  return guard([&] { moc::pack_lengths(offsets, n, bits, base, out); });
}

int moc_score_table(const int32_t* weights4, int32_t* lut1024, uint8_t* cls1024) {
  return guard([&] {
    moc::ScoreTable t = moc::ScoreTable::build(weights_of(weights4));
    if (lut1024) std::memcpy(lut1024, t.lut.data(), sizeof(int32_t) * t.lut.size());
    if (cls1024) std::memcpy(cls1024, t.cls.data(), t.cls.size());
  });
}

int moc_kernel_bounds(const int32_t* weights4, int64_t L1, int64_t min_l2, int64_t max_l2, int32_t* out6) {
  return guard([&] {
    const moc::ScoreTable t = moc::ScoreTable::build(weights_of(weights4));
    const int32_t w = t.max_abs();
    const int64_t searched = std::max<int64_t>(1, std::min(max_l2, L1 + 1));  // longer records are not searched
    out6[0] = moc::dev::swipe_form(L1, min_l2, max_l2, w);
    out6[1] = moc::bounds::short_pk_exact(w, searched) ? 1 : 0;
    out6[2] = moc::bounds::key_shift(w, searched);
    out6[3] = moc::profile16_fits(t) ? 1 : 0;
    out6[4] = moc::bounds::tile16_key32_bits(L1, w, searched);
    out6[5] = moc::profile16_i16_fits(t) ? 1 : 0;
  });
}

int moc_cpu_solve(const int32_t* weights4, const uint8_t* seq1, int64_t L1, const uint8_t* codes,
                  const int64_t* offsets, int64_t n, int semantics, int threads, moc_result* out) {
  return guard([&] {
    moc::Weights w = weights_of(weights4);
    moc::RecordBatch b = view_batch(codes, offsets, n);
    moc::validate_score_range(w, std::max<int64_t>(b.max_length(), 1));
    moc::ScoreTable t = moc::ScoreTable::build(w);
    moc::solve_batch_cpu(t, seq1, L1, b, reinterpret_cast<moc::Result*>(out), static_cast<moc::Semantics>(semantics),
                         threads);
  });
}

int moc_cpu_solve_keys(const int32_t* weights4, const uint8_t* seq1, int64_t L1, const uint8_t* codes,
                       const int64_t* offsets, int64_t n, int semantics, int part, int parts, int threads,
                       uint64_t* keys) {
  return guard([&] {
    moc::Weights w = weights_of(weights4);
    moc::RecordBatch b = view_batch(codes, offsets, n);
    moc::validate_score_range(w, std::max<int64_t>(b.max_length(), 1));
    moc::ScoreTable t = moc::ScoreTable::build(w);
    moc::solve_keys_cpu(t, seq1, L1, b, part, parts, keys, static_cast<moc::Semantics>(semantics), threads);
  });
}

int moc_resolve_keys(const int32_t* weights4, const uint8_t* seq1, int64_t L1, const uint8_t* codes,
                     const int64_t* offsets, int64_t n, const uint64_t* keys, moc_result* out) {
  return guard([&] {
    const moc::ScoreTable t = moc::ScoreTable::build(weights_of(weights4));
    for (int64_t i = 0; i < n; ++i) {
      const moc::Result r = moc::resolve_key(t, seq1, L1, codes + offsets[i], offsets[i + 1] - offsets[i], keys[i]);
      std::memcpy(out + i, &r, sizeof r);
    }
  });
}

int moc_brute_force(const int32_t* weights4, const uint8_t* seq1, int64_t L1, const uint8_t* codes,
                    const int64_t* offsets, int64_t n, int semantics, moc_result* out) {
  return guard([&] {
    moc::ScoreTable t = moc::ScoreTable::build(weights_of(weights4));
    for (int64_t i = 0; i < n; ++i) {
      moc::Result r = moc::brute_force_record(t, seq1, L1, codes + offsets[i], offsets[i + 1] - offsets[i],
                                              static_cast<moc::Semantics>(semantics));
      std::memcpy(out + i, &r, sizeof r);
    }
  });
}

int moc_partition(const int64_t* lengths, int64_t n, int64_t L1, int parts, double cell_w, double byte_w,
                  double record_w, int64_t* bounds_out) {
  return guard([&] {
    moc::CostModel m{cell_w, byte_w, record_w};
    auto b = moc::partition_by_cost(lengths, n, L1, parts, m);
    std::memcpy(bounds_out, b.data(), sizeof(int64_t) * b.size());
  });
}

int moc_device_count(void) { return moc::device_count(); }

int moc_dpp_probe(int32_t* out192) {
  return guard([&] {
    int* d = nullptr;
    MOC_HIP_CHECK(hipMalloc(&d, 192 * sizeof(int)));
    moc::dev::launch_dpp_probe(d, nullptr);
    MOC_HIP_CHECK(hipGetLastError());
    MOC_HIP_CHECK(hipMemcpy(out192, d, 192 * sizeof(int), hipMemcpyDeviceToHost));
    MOC_HIP_CHECK(hipFree(d));
  });
}

int moc_mfma_i8_probe(const int8_t* a32x32, const int8_t* b32x32, int32_t* c32x32) {
  return guard([&] {
    char* d = nullptr;
    MOC_HIP_CHECK(hipMalloc(&d, 2 * 1024 + 4 * 1024));
    MOC_HIP_CHECK(hipMemcpy(d, a32x32, 1024, hipMemcpyHostToDevice));
    MOC_HIP_CHECK(hipMemcpy(d + 1024, b32x32, 1024, hipMemcpyHostToDevice));
    moc::dev::launch_mfma_i8_probe(reinterpret_cast<const int8_t*>(d), reinterpret_cast<const int8_t*>(d + 1024),
                                   reinterpret_cast<int*>(d + 2048), nullptr);
    MOC_HIP_CHECK(hipGetLastError());
    MOC_HIP_CHECK(hipMemcpy(c32x32, d + 2048, 4 * 1024, hipMemcpyDeviceToHost));
    MOC_HIP_CHECK(hipFree(d));
  });
}

double moc_transfer_probe(int kind, size_t bytes, int iters) {
  double gbs = -1;
  guard([&] { gbs = moc::dev::transfer_probe(kind, bytes, iters); });
  return gbs;
}

int moc_bind_numa(int device) { return moc::bind_numa_to_device(device); }
int moc_device_numa_node(int device) { return moc::device_numa_node(device); }

void* moc_host_alloc(size_t bytes) {
  void* p = nullptr;
  if (guard([&] { p = moc::pinned::alloc_host(bytes); }) != 0) return nullptr;
  return p;
}

int moc_host_free(void* p) {
  return guard([&] { moc::pinned::free_host(p); });
}

int moc_host_register(void* p, size_t bytes) {
  return guard([&] {
    std::vector<void*> made = moc::pinned::register_range(p, bytes);
    std::lock_guard<std::mutex> lock(g_host_regs_mu);
    auto& v = g_host_regs[p];
    v.insert(v.end(), made.begin(), made.end());
  });
}

/* Diagnostics: device address of a pinned host range (0 when the range is not page-locked as one
 * registration), and the runtime's view of the pointer (type, host and device pointers). */
int moc_pointer_info(const void* p, size_t bytes, uint64_t* out4) {
  return guard([&] {
    out4[0] = out4[1] = out4[2] = out4[3] = out4[4] = out4[5] = 0;
    {
      hipDeviceptr_t base = nullptr;
      size_t size = 0;
      if (hipMemGetAddressRange(&base, &size, reinterpret_cast<hipDeviceptr_t>(const_cast<void*>(p))) == hipSuccess) {
        out4[4] = reinterpret_cast<uint64_t>(base);
        out4[5] = size;
      } else {
        (void)hipGetLastError();
      }
    }
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
      (void)hipGetLastError();
      return;
    }
    out4[0] = static_cast<uint64_t>(a.type);
    out4[1] = reinterpret_cast<uint64_t>(a.hostPointer);
    out4[2] = reinterpret_cast<uint64_t>(a.devicePointer);
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, const_cast<void*>(p), 0) == hipSuccess) out4[3] = reinterpret_cast<uint64_t>(d);
    else (void)hipGetLastError();
    (void)bytes;
  });
}

int moc_pinned_covers(const void* p, size_t bytes) { return moc::pinned::covers(p, bytes) ? 1 : 0; }

int moc_host_unregister(void* p) {
  return guard([&] {
    std::vector<void*> bases;
    {
      std::lock_guard<std::mutex> lock(g_host_regs_mu);
      auto it = g_host_regs.find(p);
      if (it == g_host_regs.end()) return;
      bases = std::move(it->second);
      g_host_regs.erase(it);
    }
    moc::pinned::unregister(bases);
  });
}

int moc_device_info_json(int device, char* buf, int64_t cap) {
  return guard([&] {
    std::string s = moc::device_info(device).json();
    if (static_cast<int64_t>(s.size()) + 1 > cap) throw moc::Error("buffer too small");
    std::memcpy(buf, s.c_str(), s.size() + 1);
  });
}

void* moc_engine_create(int device, int64_t chunk_records, int64_t chunk_bytes, int allow_direct) {
  moc::HipEngine* e = nullptr;
  int rc = guard([&] {
    moc::EngineOptions o;
    o.device = device;
    if (chunk_records > 0) o.chunk_records = chunk_records;
    if (chunk_bytes > 0) o.chunk_bytes = chunk_bytes;
    o.allow_direct = allow_direct != 0;
    e = new moc::HipEngine(o);
  });
  return rc == 0 ? e : nullptr;
}

void moc_engine_destroy(void* e) { delete static_cast<moc::HipEngine*>(e); }

int moc_engine_set_problem(void* e, const int32_t* weights4, const uint8_t* seq1, int64_t L1, int semantics) {
  return guard([&] {
    static_cast<moc::HipEngine*>(e)->set_problem(weights_of(weights4), seq1, L1, static_cast<moc::Semantics>(semantics));
  });
}

int moc_engine_solve(void* e, const uint8_t* codes, const int64_t* offsets, int64_t n, moc_result* out) {
  return guard([&] {
    static_cast<moc::HipEngine*>(e)->solve(codes, offsets, n, reinterpret_cast<moc::Result*>(out));
  });
}

int moc_engine_solve_ex(void* e, const uint8_t* codes, const int64_t* offsets, const uint8_t* lengths, int len_bits,
                        int len_base, int64_t n, void* out, int fmt, int64_t min_l2, int64_t max_l2, int packed) {
  return guard([&] {
    moc::BatchHints h;
    h.min_l2 = min_l2;
    h.max_l2 = max_l2;
    static_cast<moc::HipEngine*>(e)->solve_ex(codes, offsets, lengths, n, out, static_cast<moc::ResultFormat>(fmt), h,
                                              packed, len_bits, len_base);
  });
}

int moc_engine_solve_wire_device(void* e, const uint8_t* d_letters, const int64_t* d_offsets, const uint8_t* d_lengths,
                                 int len_bits, int len_base, int64_t n, void* d_out, int fmt, int64_t min_l2,
                                 int64_t max_l2, int packed) {
  return guard([&] {
    if (packed != 0 && packed != 3) throw moc::Error("device-resident letters: 0 bytes or 3 P33 fields");
    moc::WireBatch b;
    b.letters = d_letters;
    b.packed33 = packed == 3;
    b.offsets = d_offsets;
    b.lengths = d_lengths;
    b.len_bits = len_bits;
    b.len_base = len_base;
    b.n = n;
    b.min_l2 = min_l2;
    b.max_l2 = max_l2;
    b.device = true;
    static_cast<moc::HipEngine*>(e)->solve_wire(b, d_out, static_cast<moc::ResultFormat>(fmt));
  });
}

int moc_engine_auto_format(void* e, int64_t max_l2, int64_t min_l2) {
  return static_cast<int>(static_cast<moc::HipEngine*>(e)->auto_format(max_l2, min_l2));
}

int moc_engine_r2_params(void* e, int64_t min_l2, int64_t max_l2, int32_t* out3) {
  return guard([&] {
    const moc::R2Params p = static_cast<moc::HipEngine*>(e)->r2_params_for(min_l2, max_l2);
    out3[0] = p.smin;
    out3[1] = p.kw;
    out3[2] = p.j;
  });
}

int moc_engine_pin(void* e, const void* p, size_t bytes) {
  return guard([&] { static_cast<moc::HipEngine*>(e)->pin(p, bytes); });
}

int moc_engine_device_kernel_ms(void* e, double* ms) {
  return guard([&] { *ms = static_cast<moc::HipEngine*>(e)->device_kernel_ms(); });
}

int moc_engine_solve_device(void* e, const uint8_t* d_codes, const int64_t* d_offsets, const int64_t* h_offsets,
                            int64_t n, moc_result* d_out, void* stream) {
  return guard([&] {
    static_cast<moc::HipEngine*>(e)->solve_device(d_codes, d_offsets, h_offsets, n,
                                                  reinterpret_cast<moc::Result*>(d_out),
                                                  static_cast<hipStream_t>(stream));
  });
}

int moc_engine_search_keys(void* e, const uint8_t* codes, const int64_t* offsets, int64_t n, int part, int parts,
                           uint64_t* keys) {
  return guard([&] { static_cast<moc::HipEngine*>(e)->search_keys(codes, offsets, n, part, parts, keys); });
}

int moc_engine_search_keys_device(void* e, const uint8_t* d_codes, const int64_t* d_offsets, const int64_t* h_offsets,
                                  int64_t n, int part, int parts, uint64_t* d_keys, void* stream) {
  return guard([&] {
    static_cast<moc::HipEngine*>(e)->search_keys_device(d_codes, d_offsets, h_offsets, n, part, parts,
                                                        reinterpret_cast<unsigned long long*>(d_keys),
                                                        static_cast<hipStream_t>(stream));
  });
}

int moc_engine_finalize_keys_device(void* e, const uint8_t* d_codes, const int64_t* d_offsets, const int64_t* h_offsets,
                                    int64_t n, const uint64_t* d_keys, void* d_out,
                                    int fmt, void* stream) {
  return guard([&] {
    static_cast<moc::HipEngine*>(e)->finalize_keys_device(d_codes, d_offsets, h_offsets, n,
                                                          reinterpret_cast<const unsigned long long*>(d_keys), d_out,
                                                          static_cast<moc::ResultFormat>(fmt),
                                                          static_cast<hipStream_t>(stream));
  });
}

int moc_engine_stats(void* e, double* out14) {
  return guard([&] {
    double* out13 = out14;
    double* out10 = out14;
    out14[13] = static_cast<double>(static_cast<moc::HipEngine*>(e)->stats().forms);
    const auto& s = static_cast<moc::HipEngine*>(e)->stats();
    out13[10] = s.r2.smin;
    out13[11] = s.r2.kw;
    out13[12] = s.r2.j;
    out10[0] = s.kernel_ms;
    out10[1] = s.total_ms;
    out10[2] = static_cast<double>(s.h2d_bytes);
    out10[3] = static_cast<double>(s.d2h_bytes);
    out10[4] = static_cast<double>(s.chunks);
    out10[5] = static_cast<double>(s.cells);
    out10[6] = static_cast<double>(s.records);
    out10[7] = static_cast<double>(s.direct);
    out10[8] = static_cast<double>(s.format);
    out10[9] = static_cast<double>(s.kernels);
  });
}

int moc_expand_results(const void* in, int fmt, int64_t n, const int32_t* r2_3, moc_result* out) {
  return guard([&] {
    moc::R2Params p;
    if (r2_3) {
      p.smin = r2_3[0];
      p.kw = r2_3[1];
      p.j = r2_3[2];
    }
    moc::expand_results(in, static_cast<moc::ResultFormat>(fmt), n, reinterpret_cast<moc::Result*>(out),
                        r2_3 ? &p : nullptr);
  });
}

}  // extern "C"
