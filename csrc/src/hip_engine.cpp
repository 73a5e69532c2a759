#include "moc/hip_engine.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "moc/problem.hpp"
#include "moc/runtime/hip_check.hpp"
#include "moc/runtime/log.hpp"
#include "moc/runtime/timer.hpp"

namespace moc {

int32_t choose_key_shift(int32_t max_abs_weight, int64_t max_l2) {
  int shift = 1;
  while ((int64_t{1} << shift) < max_l2) ++shift;  // mask = 2^shift - 1 >= L2 - 1
  const int64_t dmax = 2 * static_cast<int64_t>(std::max(max_abs_weight, 1)) * std::max<int64_t>(max_l2, 1);
  if (shift > 24 || (dmax << shift) >= (int64_t{1} << 31)) return 0;  // 64-bit hot keys
  return shift;
}

// ------------------------------------------------------------------------------------------------
// Host-memory pinning for direct DMA: registers the page range of a caller buffer for the duration
// of one solve() (skipped when the memory is already pinned, e.g. hipHostMalloc or registered).
namespace {
class PinGuard {
 public:
  PinGuard(const void* p, size_t bytes) {
    // Small buffers may share pages with unrelated allocations: leave them pageable (HIP stages them).
    if (!p || bytes < (size_t{64} << 20)) return;
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) == hipSuccess && attr.type != hipMemoryTypeUnregistered) return;
    (void)hipGetLastError();
    const uintptr_t page = 4096;
    uintptr_t b = reinterpret_cast<uintptr_t>(p) & ~(page - 1);
    uintptr_t e = (reinterpret_cast<uintptr_t>(p) + bytes + page - 1) & ~(page - 1);
    hipError_t err = hipHostRegister(reinterpret_cast<void*>(b), e - b, hipHostRegisterDefault);
    if (err == hipSuccess) {
      base_ = reinterpret_cast<void*>(b);
    } else {
      (void)hipGetLastError();  // fall back to pageable DMA (slower, still correct)
      MOC_LOG_DEBUG("hipHostRegister(%zu bytes) failed: %s", static_cast<size_t>(e - b), hipGetErrorString(err));
    }
  }
  ~PinGuard() {
    if (base_) (void)hipHostUnregister(base_);
  }
  PinGuard(const PinGuard&) = delete;
  PinGuard& operator=(const PinGuard&) = delete;

 private:
  void* base_ = nullptr;
};
}  // namespace

// One half of the double buffer: device buffers + pinned plan staging + events.
struct HipEngine::Slot {
  void* d_codes = nullptr;
  size_t d_codes_cap = 0;
  void* d_offsets = nullptr;
  size_t d_offsets_cap = 0;
  void* d_out = nullptr;
  size_t d_out_cap = 0;
  void* d_plan = nullptr;  // tiles | long_recs | keys
  size_t d_plan_cap = 0;
  void* h_plan = nullptr;  // pinned staging for tiles | long_recs
  size_t h_plan_cap = 0;
  hipEvent_t ev_h2d = nullptr, ev_k0 = nullptr, ev_k1 = nullptr, ev_done = nullptr;
  bool busy = false;
};

HipEngine::HipEngine(const EngineOptions& opt) : opt_(opt) {
  if (opt_.device >= 0) MOC_HIP_CHECK(hipSetDevice(opt_.device));
  MOC_HIP_CHECK(hipGetDevice(&device_));
  MOC_HIP_CHECK(hipStreamCreateWithFlags(&s_copy_, hipStreamNonBlocking));
  MOC_HIP_CHECK(hipStreamCreateWithFlags(&s_compute_, hipStreamNonBlocking));
  MOC_HIP_CHECK(hipStreamCreateWithFlags(&s_return_, hipStreamNonBlocking));
  for (int i = 0; i < 2; ++i) {
    auto s = std::make_unique<Slot>();
    MOC_HIP_CHECK(hipEventCreateWithFlags(&s->ev_h2d, hipEventDisableTiming));
    MOC_HIP_CHECK(hipEventCreate(&s->ev_k0));
    MOC_HIP_CHECK(hipEventCreate(&s->ev_k1));
    MOC_HIP_CHECK(hipEventCreateWithFlags(&s->ev_done, hipEventDisableTiming));
    slots_.push_back(std::move(s));
  }
  MOC_HIP_CHECK(hipEventCreateWithFlags(&ev_plan_, hipEventDisableTiming));
}

HipEngine::~HipEngine() {
  (void)hipSetDevice(device_);
  (void)hipDeviceSynchronize();
  for (auto& s : slots_) {
    (void)hipFree(s->d_codes);
    (void)hipFree(s->d_offsets);
    (void)hipFree(s->d_out);
    (void)hipFree(s->d_plan);
    (void)hipHostFree(s->h_plan);
    (void)hipEventDestroy(s->ev_h2d);
    (void)hipEventDestroy(s->ev_k0);
    (void)hipEventDestroy(s->ev_k1);
    (void)hipEventDestroy(s->ev_done);
  }
  (void)hipFree(d_plan_);
  (void)hipHostFree(h_plan_);
  (void)hipEventDestroy(ev_plan_);
  (void)hipFree(d_lut_);
  (void)hipFree(d_seq1_);
  (void)hipStreamDestroy(s_copy_);
  (void)hipStreamDestroy(s_compute_);
  (void)hipStreamDestroy(s_return_);
}

void HipEngine::ensure(void*& ptr, size_t& cap, size_t bytes) {
  if (bytes <= cap) return;
  size_t want = std::max<size_t>(bytes + bytes / 4, 4096);
  if (ptr) {
    MOC_HIP_CHECK(hipDeviceSynchronize());  // growth is rare (first chunks); keep it simple and safe
    MOC_HIP_CHECK(hipFree(ptr));
  }
  MOC_HIP_CHECK(hipMalloc(&ptr, want));
  cap = want;
}

void HipEngine::ensure_host(void*& ptr, size_t& cap, size_t bytes) {
  if (bytes <= cap) return;
  size_t want = std::max<size_t>(bytes + bytes / 4, 4096);
  if (ptr) MOC_HIP_CHECK(hipHostFree(ptr));
  MOC_HIP_CHECK(hipHostMalloc(&ptr, want, hipHostMallocDefault));
  cap = want;
}

void HipEngine::set_problem(const Weights& w, const uint8_t* seq1, int64_t L1, Semantics sem) {
  MOC_HIP_CHECK(hipSetDevice(device_));
  if (L1 > (int64_t{1} << 30)) throw Error("Seq1 too long for the device engine");
  MOC_HIP_CHECK(hipDeviceSynchronize());  // previous problem's launches may still read the buffers
  table_ = ScoreTable::build(w);
  L1_ = L1;
  sem_ = sem;
  if (!d_lut_) MOC_HIP_CHECK(hipMalloc(&d_lut_, sizeof(int32_t) * kLutStride * kLutStride));
  MOC_HIP_CHECK(hipFree(d_seq1_));
  d_seq1_ = nullptr;
  const size_t s1bytes = static_cast<size_t>(L1) + dev::kSeq1Pad;
  MOC_HIP_CHECK(hipMalloc(&d_seq1_, s1bytes));
  std::vector<uint8_t> padded(s1bytes, 0);
  if (L1) std::memcpy(padded.data(), seq1, static_cast<size_t>(L1));
  MOC_HIP_CHECK(hipMemcpy(d_lut_, table_.lut.data(), sizeof(int32_t) * table_.lut.size(), hipMemcpyHostToDevice));
  MOC_HIP_CHECK(hipMemcpy(d_seq1_, padded.data(), s1bytes, hipMemcpyHostToDevice));
  have_problem_ = true;
}

void HipEngine::set_problem_device(const Weights& w, const uint8_t* d_seq1, int64_t L1, Semantics sem) {
  std::vector<uint8_t> host(static_cast<size_t>(L1));
  if (L1) MOC_HIP_CHECK(hipMemcpy(host.data(), d_seq1, static_cast<size_t>(L1), hipMemcpyDeviceToHost));
  set_problem(w, host.data(), L1, sem);
}

dev::ProblemView HipEngine::problem_view(int64_t max_l2) const {
  dev::ProblemView pv;
  pv.lut = d_lut_;
  pv.seq1 = d_seq1_;
  pv.L1 = static_cast<int32_t>(L1_);
  pv.semantics = static_cast<int32_t>(sem_);
  pv.key_shift = choose_key_shift(table_.max_abs(), max_l2);
  return pv;
}

void HipEngine::plan_chunk(const int64_t* offsets, int64_t n, HostPlan& hp) const {
  hp.slot = 0;
  hp.tiles.clear();
  hp.long_recs.clear();
  hp.max_l2 = 0;
  hp.cells = 0;
  int64_t slot = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t L2 = offsets[i + 1] - offsets[i];
    hp.max_l2 = std::max(hp.max_l2, L2);
    hp.cells += record_cells(L1_, L2);
    const int64_t need = dev::lanes_needed(L1_, L2);
    if (need <= dev::kWave) {
      slot = std::max(slot, need);
    } else {
      const int32_t li = static_cast<int32_t>(hp.long_recs.size());
      hp.long_recs.push_back(static_cast<int32_t>(i));
      for (int64_t o0 = 0; o0 < need; o0 += dev::kTileOffsets)
        hp.tiles.push_back(dev::Tile{li, static_cast<int32_t>(o0)});
    }
  }
  hp.slot = static_cast<int32_t>(slot);
  hp.rpw = slot > 0 ? static_cast<int32_t>(dev::kWave / slot) : 0;
  if (hp.max_l2 * L1_ >= (int64_t{1} << 32))
    throw Error("L1 * max L2 exceeds the 32-bit candidate index of the device engine");
}

namespace {
// Layout of one chunk's plan in a single buffer: tiles | long_recs | keys(8-aligned).
struct PlanLayout {
  size_t tiles_off = 0, long_off = 0, keys_off = 0, upload_bytes = 0, total = 0;
  PlanLayout(size_t n_tiles, size_t n_long) {
    long_off = n_tiles * sizeof(dev::Tile);
    keys_off = (long_off + n_long * sizeof(int32_t) + 7) & ~size_t{7};
    upload_bytes = long_off + n_long * sizeof(int32_t);
    total = keys_off + n_long * sizeof(unsigned long long);
  }
};
}  // namespace

void HipEngine::solve(const uint8_t* codes, const int64_t* offsets, int64_t n, Result* out) {
  if (!have_problem_) throw Error("HipEngine::solve before set_problem");
  MOC_HIP_CHECK(hipSetDevice(device_));
  Stopwatch wall;
  wall.start();
  stats_ = EngineStats{};
  if (n <= 0) return;
  const int64_t total_chars = offsets[n] - offsets[0];
  std::unique_ptr<PinGuard> pin_codes, pin_offs, pin_out;
  if (opt_.pin_host) {
    pin_codes = std::make_unique<PinGuard>(codes + offsets[0], static_cast<size_t>(total_chars));
    pin_offs = std::make_unique<PinGuard>(offsets, sizeof(int64_t) * static_cast<size_t>(n + 1));
    pin_out = std::make_unique<PinGuard>(out, sizeof(Result) * static_cast<size_t>(n));
  }
  HostPlan hp;
  double kernel_ms = 0;
  auto retire = [&](Slot& s) {
    if (!s.busy) return;
    MOC_HIP_CHECK(hipEventSynchronize(s.ev_done));
    float ms = 0;
    MOC_HIP_CHECK(hipEventElapsedTime(&ms, s.ev_k0, s.ev_k1));
    kernel_ms += ms;
    s.busy = false;
  };
  int64_t chunk = 0;
  for (int64_t rb = 0; rb < n; ++chunk) {
    // chunk end: at most chunk_records records and chunk_bytes letters (at least one record)
    int64_t re = std::min(n, rb + opt_.chunk_records);
    const int64_t byte_cap = offsets[rb] + opt_.chunk_bytes;
    if (offsets[re] > byte_cap) {
      re = std::upper_bound(offsets + rb + 1, offsets + re + 1, byte_cap) - offsets - 1;
      re = std::max(re, rb + 1);
    }
    const int64_t cn = re - rb;
    Slot& s = *slots_[chunk % 2];
    retire(s);
    plan_chunk(offsets + rb, cn, hp);
    stats_.cells += hp.cells;
    const PlanLayout lay(hp.tiles.size(), hp.long_recs.size());
    const size_t cbytes = static_cast<size_t>(offsets[re] - offsets[rb]);
    ensure(s.d_codes, s.d_codes_cap, std::max<size_t>(cbytes, 4));
    ensure(s.d_offsets, s.d_offsets_cap, sizeof(int64_t) * static_cast<size_t>(cn + 1));
    ensure(s.d_out, s.d_out_cap, sizeof(Result) * static_cast<size_t>(cn));
    if (lay.total) {
      ensure(s.d_plan, s.d_plan_cap, lay.total);
      ensure_host(s.h_plan, s.h_plan_cap, lay.upload_bytes);
      std::memcpy(static_cast<char*>(s.h_plan) + lay.tiles_off, hp.tiles.data(), hp.tiles.size() * sizeof(dev::Tile));
      std::memcpy(static_cast<char*>(s.h_plan) + lay.long_off, hp.long_recs.data(), hp.long_recs.size() * sizeof(int32_t));
    }
    // ---- copy stream: H2D
    if (cbytes) MOC_HIP_CHECK(hipMemcpyAsync(s.d_codes, codes + offsets[rb], cbytes, hipMemcpyHostToDevice, s_copy_));
    MOC_HIP_CHECK(hipMemcpyAsync(s.d_offsets, offsets + rb, sizeof(int64_t) * (cn + 1), hipMemcpyHostToDevice, s_copy_));
    if (lay.upload_bytes)
      MOC_HIP_CHECK(hipMemcpyAsync(s.d_plan, s.h_plan, lay.upload_bytes, hipMemcpyHostToDevice, s_copy_));
    MOC_HIP_CHECK(hipEventRecord(s.ev_h2d, s_copy_));
    stats_.h2d_bytes += static_cast<int64_t>(cbytes + sizeof(int64_t) * (cn + 1) + lay.upload_bytes);
    // ---- compute stream
    MOC_HIP_CHECK(hipStreamWaitEvent(s_compute_, s.ev_h2d, 0));
    dev::Plan plan;
    plan.slot = hp.slot;
    plan.rec_per_wave = hp.rpw;
    plan.n_tiles = static_cast<int64_t>(hp.tiles.size());
    plan.n_long = static_cast<int64_t>(hp.long_recs.size());
    plan.tiles = reinterpret_cast<const dev::Tile*>(static_cast<char*>(s.d_plan) + lay.tiles_off);
    plan.long_recs = reinterpret_cast<const int32_t*>(static_cast<char*>(s.d_plan) + lay.long_off);
    plan.keys = reinterpret_cast<unsigned long long*>(static_cast<char*>(s.d_plan) + lay.keys_off);
    dev::BatchView bv{static_cast<const uint8_t*>(s.d_codes), static_cast<const int64_t*>(s.d_offsets), cn};
    int* d_dbg = nullptr;
    const char* dbg_env = std::getenv("MOC_DEBUG_TILE");
    if (dbg_env) {
      MOC_HIP_CHECK(hipMalloc(&d_dbg, 4096));
      std::vector<int> init(1024, 0);
      init[0] = std::atoi(dbg_env);
      MOC_HIP_CHECK(hipMemcpy(d_dbg, init.data(), 4096, hipMemcpyHostToDevice));
      plan.debug = d_dbg;
    }
    MOC_HIP_CHECK(hipEventRecord(s.ev_k0, s_compute_));
    dev::launch_search(problem_view(hp.max_l2), bv, plan, static_cast<Result*>(s.d_out), s_compute_);
    if (d_dbg) {
      std::vector<int> h(1024);
      MOC_HIP_CHECK(hipStreamSynchronize(s_compute_));
      MOC_HIP_CHECK(hipMemcpy(h.data(), d_dbg, 4096, hipMemcpyDeviceToHost));
      std::fprintf(stderr, "DBG tile=%d L2=%d o0=%d r=%d codes=%d,%d,%d,%d,%d,%d,%d,%d key0=%08x%08x\n", h[0], h[1], h[2],
                   h[3], h[8], h[9], h[10], h[11], h[12], h[13], h[14], h[15], h[16], h[17]);
      for (int l = 0; l < 64; ++l)
        std::fprintf(stderr, "DBG lane %d P=%d best=%d Pn=%d x=%d\n", l, h[64 + 4 * l], h[65 + 4 * l], h[66 + 4 * l],
                     h[67 + 4 * l]);
      (void)hipFree(d_dbg);
    }
    MOC_HIP_CHECK(hipGetLastError());
    MOC_HIP_CHECK(hipEventRecord(s.ev_k1, s_compute_));
    // ---- return stream: D2H straight into the caller's result array
    MOC_HIP_CHECK(hipStreamWaitEvent(s_return_, s.ev_k1, 0));
    MOC_HIP_CHECK(hipMemcpyAsync(out + rb, s.d_out, sizeof(Result) * cn, hipMemcpyDeviceToHost, s_return_));
    MOC_HIP_CHECK(hipEventRecord(s.ev_done, s_return_));
    stats_.d2h_bytes += static_cast<int64_t>(sizeof(Result) * cn);
    s.busy = true;
    rb = re;
  }
  for (auto& s : slots_) retire(*s);
  wall.stop();
  stats_.kernel_ms = kernel_ms;
  stats_.total_ms = wall.total_ms();
  stats_.chunks = chunk;
  stats_.records = n;
}

void HipEngine::solve_device(const uint8_t* d_codes, const int64_t* d_offsets, const int64_t* h_offsets, int64_t n,
                             Result* d_out, hipStream_t stream) {
  if (!have_problem_) throw Error("HipEngine::solve_device before set_problem");
  MOC_HIP_CHECK(hipSetDevice(device_));
  if (n <= 0) return;
  if (!stream) stream = s_compute_;
  HostPlan hp;
  plan_chunk(h_offsets, n, hp);
  const PlanLayout lay(hp.tiles.size(), hp.long_recs.size());
  MOC_HIP_CHECK(hipEventSynchronize(ev_plan_));  // previous call's plan buffers are free again
  if (lay.total) {
    ensure(d_plan_, d_plan_cap_, lay.total);
    ensure_host(h_plan_, h_plan_cap_, lay.upload_bytes);
    std::memcpy(static_cast<char*>(h_plan_) + lay.tiles_off, hp.tiles.data(), hp.tiles.size() * sizeof(dev::Tile));
    std::memcpy(static_cast<char*>(h_plan_) + lay.long_off, hp.long_recs.data(), hp.long_recs.size() * sizeof(int32_t));
    MOC_HIP_CHECK(hipMemcpyAsync(d_plan_, h_plan_, lay.upload_bytes, hipMemcpyHostToDevice, stream));
  }
  dev::Plan plan;
  plan.slot = hp.slot;
  plan.rec_per_wave = hp.rpw;
  plan.n_tiles = static_cast<int64_t>(hp.tiles.size());
  plan.n_long = static_cast<int64_t>(hp.long_recs.size());
  plan.tiles = reinterpret_cast<const dev::Tile*>(static_cast<char*>(d_plan_) + lay.tiles_off);
  plan.long_recs = reinterpret_cast<const int32_t*>(static_cast<char*>(d_plan_) + lay.long_off);
  plan.keys = reinterpret_cast<unsigned long long*>(static_cast<char*>(d_plan_) + lay.keys_off);
  dev::BatchView bv{d_codes + h_offsets[0], d_offsets, n};
  dev::launch_search(problem_view(hp.max_l2), bv, plan, d_out, stream);
  MOC_HIP_CHECK(hipGetLastError());
  MOC_HIP_CHECK(hipEventRecord(ev_plan_, stream));
  stats_.cells = hp.cells;
  stats_.records = n;
}

}  // namespace moc
