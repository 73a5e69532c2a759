#include "moc/hip_engine.hpp"

#include <omp.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <future>
#include <queue>
#include <string>

#include "moc/problem.hpp"
#include "moc/runtime/hip_check.hpp"
#include "moc/runtime/log.hpp"
#include "moc/runtime/pinned.hpp"
#include "moc/runtime/timer.hpp"
#include "moc/runtime/trace.hpp"

namespace moc {

int32_t choose_key_shift(int32_t max_abs_weight, int64_t max_l2) { return bounds::key_shift(max_abs_weight, max_l2); }

namespace {
// Copies between device memory and a caller's host range, one per piece of the range that lies within a
// single page-locked registration (or outside all): see pinned::segments. A small registered piece moves on
// a copy kernel through its device address (dev::launch_copy: no SDMA start-up inside a short job), the
// rest with hipMemcpyAsync.
void copy_h2d(void* dst, const void* src, size_t bytes, hipStream_t s) {
  for (const auto& seg : pinned::segments(src, bytes)) {
    char* d = static_cast<char*>(dst) + seg.first;
    const char* h = static_cast<const char*>(src) + seg.first;
    const void* hd = nullptr;
    if (dev::kernel_copy_fits(d, h, seg.second) && (hd = pinned::device_address(h, seg.second)))
      dev::launch_copy(d, hd, seg.second, s);
    else
      MOC_HIP_CHECK(hipMemcpyAsync(d, h, seg.second, hipMemcpyHostToDevice, s));
  }
}
void copy_d2h(void* dst, const void* src, size_t bytes, hipStream_t s) {
  for (const auto& seg : pinned::segments(dst, bytes)) {
    char* h = static_cast<char*>(dst) + seg.first;
    const char* d = static_cast<const char*>(src) + seg.first;
    const void* hd = nullptr;
    if (dev::kernel_copy_fits(h, d, seg.second) && (hd = pinned::device_address(h, seg.second)))
      dev::launch_copy(const_cast<void*>(hd), d, seg.second, s);
    else
      MOC_HIP_CHECK(hipMemcpyAsync(h, d, seg.second, hipMemcpyDeviceToHost, s));
  }
}
// host -> device from a hipHostMalloc allocation of the engine's own (h_image_, plan staging)
void upload_staged(void* dst, const void* h, size_t bytes, hipStream_t s) {
  void* hd = nullptr;
  if (dev::kernel_copy_fits(dst, h, bytes)) {
    if (hipHostGetDevicePointer(&hd, const_cast<void*>(h), 0) != hipSuccess) {
      (void)hipGetLastError();  // clear the sticky error: the next launch check must not report this lookup
      hd = nullptr;
    }
  }
  if (hd)
    dev::launch_copy(dst, hd, bytes, s);
  else
    MOC_HIP_CHECK(hipMemcpyAsync(dst, h, bytes, hipMemcpyHostToDevice, s));
}

// Device-resident byte batches with dense offsets run the wave-autonomous swipe kernel (swipe_direct_kernel);
// MOC_SWIPE_DIRECT=0 keeps them on the block-tiled one (A/B runs; both give the same results).
bool lane_direct_enabled() {
  static const bool on = [] {
    const char* v = std::getenv("MOC_SWIPE_DIRECT");
    return !(v && std::atoi(v) == 0);
  }();
  return on;
}

// True when every byte of [p, p+bytes) is page-locked through the registry (moc/runtime/pinned.hpp);
// *dev gets the device-side address of p.
bool pinned_range(const void* p, size_t bytes, const void** dev) {
  const void* d = pinned::device_address(p, bytes);
  if (!d) return false;
  *dev = d;
  return true;
}
}  // namespace

// One half of the double buffer of the staged pipeline.
struct HipEngine::Slot {
  void* d_codes = nullptr;
  size_t d_codes_cap = 0;
  void* d_offsets = nullptr;
  size_t d_offsets_cap = 0;
  void* d_packed = nullptr;  // 5-bit packed letters of the chunk (packed batches)
  size_t d_packed_cap = 0;
  void* d_out = nullptr;
  size_t d_out_cap = 0;
  void* d_plan = nullptr;  // tiles | long_recs | keys
  size_t d_plan_cap = 0;
  void* h_plan = nullptr;  // pinned staging for tiles | long_recs
  size_t h_plan_cap = 0;
  unsigned* d_counter = nullptr;
  hipEvent_t ev_h2d = nullptr, ev_k0 = nullptr, ev_k1 = nullptr, ev_done = nullptr;
  bool busy = false;
};

namespace dev {
int parse_preload_set(const char* s) {
  static const struct {
    const char* name;
    unsigned set;
  } names[] = {{"all", kPreloadAll}, {"none", 0}, {"align", kPreloadAlign}, {"short", kPreloadShort},
               {"swipe", kPreloadSwipeByte | kPreloadSwipeP33}, {"swipe8", kPreloadSwipeByte},
               {"swipe33", kPreloadSwipeP33}, {"tile16", kPreloadTile16}, {"mfma", kPreloadMfma}};
  unsigned set = 0;
  std::string list(s);
  size_t at = 0;
  while (at <= list.size()) {
    const size_t end = std::min(list.find(',', at), list.size());
    const std::string item = list.substr(at, end - at);
    bool known = item.empty();
    for (const auto& n : names)
      if (item == n.name) {
        set |= n.set;
        known = true;
      }
    if (!known) return -1;
    at = end + 1;
  }
  return static_cast<int>(set);
}
}  // namespace dev

HipEngine::HipEngine(const EngineOptions& opt) : opt_(opt) {
  Stopwatch init_sw;
  init_sw.start();
  if (opt_.device >= 0) MOC_HIP_CHECK(hipSetDevice(opt_.device));
  MOC_HIP_CHECK(hipGetDevice(&device_));
  MOC_HIP_CHECK(hipDeviceGetAttribute(&num_cus_, hipDeviceAttributeMultiprocessorCount, device_));
  const double t_dev = init_sw.total_ms();
  if (const char* m = std::getenv("MOC_MFMA")) mfma_ = std::atoi(m) != 0;
  unsigned set = opt_.preload;
  if (const char* p = std::getenv("MOC_PRELOAD")) {
    const int v = dev::parse_preload_set(p);
    if (v < 0) throw Error(std::string("MOC_PRELOAD: unknown kernel file in '") + p + "'");
    set = static_cast<unsigned>(v);
  }
  if (mfma_ && (set & dev::kPreloadTile16)) set |= dev::kPreloadMfma;
  // code objects on the device now, not inside the first timed launch, and the image's page-locked staging
  // — on a helper thread, while this one sets up the compute stream and buffers (independent runtime work,
  // ~13 and ~20 ms on the MI355X box)
  std::future<void> preload = std::async(std::launch::async, [this, set] {
    MOC_HIP_CHECK(hipSetDevice(device_));
    if (set) dev::preload_kernels(set);
    MOC_HIP_CHECK(hipHostMalloc(&h_image_, size_t{256} << 10, hipHostMallocDefault));  // Seq1 up to ~5000 letters
    h_image_cap_ = size_t{256} << 10;
  });
  const double t_preload = init_sw.total_ms();
  if (const char* g = std::getenv("MOC_GRAPHS")) opt_.use_graphs = std::atoi(g) != 0;
  if (const char* u = std::getenv("MOC_TILE_U")) {  // tuning override of the per-batch choice
    const int v = std::atoi(u);
    if (v == 1 || v == 2 || v == 4 || v == 8) tile_u_ = v;
  }
  if (const char* t16 = std::getenv("MOC_TILE16")) tile16_ = std::atoi(t16) != 0;
  // MOC_TILE16_WINWIDE=0: short records on an L1 ~ 1500..3050 problem keep the whole byte-pair image (A/B)
  if (const char* ww = std::getenv("MOC_TILE16_WINWIDE")) tile16_window_wide_ = std::atoi(ww) != 0;
  if (const char* w8 = std::getenv("MOC_TILE16_WIN_U8")) short_window_u8_ = std::atoi(w8) != 0;
  if (const char* sl = std::getenv("MOC_TILE16_SLIDE")) tile16_slide_ = std::atoi(sl) != 0;
  if (const char* sw = std::getenv("MOC_TILE16_SLIDE_WG")) slide_wgs_per_cu_ = std::atoi(sw) == 1 ? 1 : 2;
  if (const char* w = std::getenv("MOC_TILE_WAVES_PER_CU")) {
    const int v = std::atoi(w);
    if (v >= 1 && v <= 32) tile_waves_per_cu_ = v;
  }
  // the compute stream only: each stream costs ~10 ms of hardware-queue set-up on the MI355X box
  // (profiles/hip_init_variants_box.log), and the streaming kernels need no other; the staged pipeline
  // makes its copy and return streams on first use (ensure_side_streams)
  MOC_HIP_CHECK(hipStreamCreateWithFlags(&s_compute_, hipStreamNonBlocking));
  const double t_streams = init_sw.total_ms();
  for (int i = 0; i < 2; ++i) {  // run_staged cycles two
    auto s = std::make_unique<Slot>();
    MOC_HIP_CHECK(hipEventCreateWithFlags(&s->ev_h2d, hipEventDisableTiming));
    MOC_HIP_CHECK(hipEventCreate(&s->ev_k0));
    MOC_HIP_CHECK(hipEventCreate(&s->ev_k1));
    MOC_HIP_CHECK(hipEventCreateWithFlags(&s->ev_done, hipEventDisableTiming));
    MOC_HIP_CHECK(hipMalloc(&s->d_counter, 2 * sizeof(unsigned)));
    MOC_HIP_CHECK(hipMemsetAsync(s->d_counter, 0, 2 * sizeof(unsigned), s_compute_));  // before any kernel
    slots_.push_back(std::move(s));
  }
  MOC_HIP_CHECK(hipMalloc(&d_counter_, 2 * sizeof(unsigned)));  // {next tile, blocks done}, self-resetting
  MOC_HIP_CHECK(hipMemsetAsync(d_counter_, 0, 2 * sizeof(unsigned), s_compute_));
  MOC_HIP_CHECK(hipEventCreate(&ev_a_));
  MOC_HIP_CHECK(hipEventCreate(&ev_b_));
  MOC_HIP_CHECK(hipEventCreateWithFlags(&ev_plan_, hipEventDisableTiming));
  preload.get();  // rethrows a load error
  MOC_LOG_DEBUG("engine on device %d up in %.1f ms (device %.1f, kernel preload started %.1f, streams %.1f, buffers + preload %.1f)", device_,
                init_sw.total_ms(), t_dev, t_preload - t_dev, t_streams - t_preload, init_sw.total_ms() - t_streams);
}

HipEngine::~HipEngine() {
  (void)hipSetDevice(device_);
  (void)hipDeviceSynchronize();
  for (auto& s : slots_) {
    (void)hipFree(s->d_codes);
    (void)hipFree(s->d_offsets);
    (void)hipFree(s->d_packed);
    (void)hipFree(s->d_out);
    (void)hipFree(s->d_plan);
    (void)hipFree(s->d_counter);
    (void)hipHostFree(s->h_plan);
    (void)hipEventDestroy(s->ev_h2d);
    (void)hipEventDestroy(s->ev_k0);
    (void)hipEventDestroy(s->ev_k1);
    (void)hipEventDestroy(s->ev_done);
  }
  unpin_all();
  for (hipGraphExec_t g : graph_exec_)
    if (g) (void)hipGraphExecDestroy(g);
  (void)hipFree(d_counter_);
  (void)hipFree(d_plan_);
  (void)hipHostFree(h_plan_);
  (void)hipEventDestroy(ev_plan_);
  if (ev_d0_) (void)hipEventDestroy(ev_d0_);
  if (ev_d1_) (void)hipEventDestroy(ev_d1_);
  (void)hipEventDestroy(ev_a_);
  (void)hipEventDestroy(ev_b_);
  (void)hipFree(d_image_);
  (void)hipHostFree(h_image_);
  if (s_copy_) (void)hipStreamDestroy(s_copy_);
  (void)hipStreamDestroy(s_compute_);
  if (s_return_) (void)hipStreamDestroy(s_return_);
}

void HipEngine::ensure_side_streams() {
  if (!s_copy_) MOC_HIP_CHECK(hipStreamCreateWithFlags(&s_copy_, hipStreamNonBlocking));
  if (!s_return_) MOC_HIP_CHECK(hipStreamCreateWithFlags(&s_return_, hipStreamNonBlocking));
}

void HipEngine::pin(const void* p, size_t bytes) {
  const std::vector<void*> made = pinned::register_range(p, bytes);  // only pages not yet locked
  pinned_.insert(pinned_.end(), made.begin(), made.end());
}

void HipEngine::unpin_all() {
  finish_wire();
  pinned::unregister(pinned_);
  pinned_.clear();
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
  finish_wire();
  // the same problem again (every step of a repeated job): nothing to rebuild or upload
  if (have_problem_ && sem == sem_ && L1 == L1_ && std::equal(w.w, w.w + 4, last_w_.w) &&
      (L1 == 0 || std::memcmp(seq1, last_seq1_.data(), static_cast<size_t>(L1)) == 0))
    return;
  MOC_HIP_CHECK(hipSetDevice(device_));
  if (L1 > (int64_t{1} << 30)) throw Error("Seq1 too long for the device engine");
  // the inputs are recorded as current only once the device image holds them (below): a set_problem that
  // throws half-way cannot be skipped by the next call for the same problem
  have_problem_ = false;
  table_ = ScoreTable::build(w);
  min_t_ = INT32_MAX;
  max_t_ = INT32_MIN;
  for (int x = 1; x < kAlphabet; ++x)
    for (int y = 1; y < kAlphabet; ++y) {
      min_t_ = std::min(min_t_, table_.lut[x * kLutStride + y]);
      max_t_ = std::max(max_t_, table_.lut[x * kLutStride + y]);
    }
  L1_ = L1;
  sem_ = sem;
  // One device image per problem, uploaded with one copy: LUT | Seq1 + zero pad | tile16 profile. The
  // buffer only grows, so repeated problems (one per job step) cost no allocation, and kernel arguments
  // (and a captured direct-path graph) keep pointing at the same addresses.
  const size_t s1bytes = static_cast<size_t>(L1) + dev::kSeq1Pad;
  const size_t lut_bytes = sizeof(int32_t) * table_.lut.size();
  const size_t s1_off = (lut_bytes + 255) & ~size_t{255};
  const size_t prof_off = (s1_off + s1bytes + 255) & ~size_t{255};
  Profile16 prof;
  // the overhang (zero entries past the last row) must cover the widest tile span, 128*U entries: 1024
  // when that still fits the LDS (U = 8 for short records), else 512 (U <= 4, L1 up to 3052)
  auto prof_bytes = [&](int64_t oh) { return ((2 * ((kAlphabet - 1) * L1 + oh)) + 15) & ~int64_t{15}; };
  // Occupancy first: a CU holds two 16-wave workgroups when the image fits half its LDS, and the sweep is
  // latency-bound, so the wide overhang (U = 8 tiles, for short records only) is kept only where it costs no
  // workgroup: input3's 1489-letter Seq1 fits twice with 512 (32 waves per CU), once with 1024 (16).
  int64_t overhang = 2 * dev::kProf16Overhang;
  const int64_t half = dev::kProf16MaxLds / 2;
  if (dev::tile16_lds_bytes(prof_bytes(overhang), L1) > dev::kProf16MaxLds ||
      (dev::tile16_lds_bytes(prof_bytes(overhang), L1) > half &&
       dev::tile16_lds_bytes(prof_bytes(dev::kProf16Overhang), L1) <= half))
    overhang = dev::kProf16Overhang;
  int64_t pbytes = prof_bytes(overhang);
  // Seq1 too long for one LDS image: the whole profile lives in device memory and each workgroup stages
  // a window of it (tile16_search_kernel<U, true>); records must then fit a window with two tiles' slack
  const bool whole = dev::tile16_lds_bytes(pbytes, L1) <= dev::kProf16MaxLds;
  const int64_t window = whole ? 0 : dev::tile16_max_window();
  // weights past the byte pairs (|Dt| > 127) up to |Dt| <= 511: one int16 Dt per entry, which only the widened
  // images take (whole where it fits, windows for short records; otherwise the LUT tile kernel)
  const bool t16 = tile16_ && L1 > 0 && build_profile16(table_, seq1, L1, overhang, prof, /*allow_i16=*/true);
  prof16_i16_ = t16 && prof.i16;
  prof16_window_ = t16 && !prof16_i16_ ? static_cast<int32_t>(window) : 0;
  prof16_entries_ = t16 ? static_cast<int64_t>(prof.entries.size()) : 0;
  prof16_lds_bytes_ = t16 ? dev::tile16_profile_lds_bytes(L1, overhang, prof16_i16_) : 0;
  pbytes = (2 * static_cast<int64_t>(prof.entries.size()) + 15) & ~int64_t{15};
  prof16_overhang_ = t16 ? static_cast<int>(overhang) : 0;
  // widened entries (two int16 halves per column: one packed add per lane and step) where the doubled image
  // still fits one CU; MOC_TILE16_WIDE=0 keeps the byte pairs (A/B runs, same results)
  static const bool wide_env = [] {
    const char* v = std::getenv("MOC_TILE16_WIDE");
    return !(v && std::atoi(v) == 0);
  }();
  prof16_wide_ = t16 && (whole || prof16_i16_) && (wide_env || prof16_i16_) &&
                 dev::tile16_lds_bytes(2 * static_cast<int64_t>(prof16_lds_bytes_), L1) <= dev::kProf16MaxLds;
  const size_t total = t16 ? prof_off + static_cast<size_t>(pbytes) : prof_off;
  std::vector<uint8_t> next(total, 0);
  std::memcpy(next.data(), table_.lut.data(), lut_bytes);
  if (L1) std::memcpy(next.data() + s1_off, seq1, static_cast<size_t>(L1));
  if (t16) std::memcpy(next.data() + prof_off, prof.entries.data(), sizeof(uint16_t) * prof.entries.size());
  // the same problem again (one per job step of a repeated job): the device image is already current —
  // no device-wide synchronisation, no copy
  if (!image_.empty() && next == image_ && d_image_) {
    prof16_bytes_ = prof16_lds_bytes_;
    last_w_ = w;
    last_seq1_.assign(seq1, seq1 + L1);
    have_problem_ = true;
    return;
  }
  image_.clear();  // the device image is about to change: not current until the upload completes
  // Kernels of the previous problem may still be queued — on our streams or on a solve_device caller's —
  // and read the image in place: let them finish before it is overwritten.
  MOC_HIP_CHECK(hipDeviceSynchronize());
  if (total > d_image_cap_) {
    void* old = std::exchange(d_image_, nullptr);
    d_image_cap_ = 0;
    MOC_HIP_CHECK(hipFree(old));
    MOC_HIP_CHECK(hipMalloc(&d_image_, std::max(total, size_t{64} << 10)));
    d_image_cap_ = std::max(total, size_t{64} << 10);
  }
  if (total > h_image_cap_) {
    void* old = std::exchange(h_image_, nullptr);
    h_image_cap_ = 0;
    MOC_HIP_CHECK(hipHostFree(old));
    MOC_HIP_CHECK(hipHostMalloc(&h_image_, total, hipHostMallocDefault));
    h_image_cap_ = total;
  }
  std::memcpy(h_image_, next.data(), total);
  upload_staged(d_image_, h_image_, total, s_compute_);
  // complete before any stream's kernel reads it (solve_device callers launch on streams of their own)
  MOC_HIP_CHECK(hipStreamSynchronize(s_compute_));
  image_.swap(next);
  char* base = static_cast<char*>(d_image_);
  d_lut_ = reinterpret_cast<int32_t*>(base);
  d_seq1_ = reinterpret_cast<uint8_t*>(base + s1_off);
  d_prof16_ = t16 ? reinterpret_cast<uint16_t*>(base + prof_off) : nullptr;
  prof16_bytes_ = prof16_lds_bytes_;
  last_w_ = w;
  last_seq1_.assign(seq1, seq1 + L1);
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
  pv.key_shift = choose_key_shift(table_.max_abs(), std::min<int64_t>(std::max<int64_t>(max_l2, 1), L1_ + 1));
  pv.r2 = r2_;
  pv.prof16 = d_prof16_;
  pv.prof16_bytes = prof16_bytes_;
  pv.prof16_window = prof16_window_;
  pv.prof16_entries = prof16_entries_;
  pv.prof16_wide = prof16_wide_ && !mfma_ ? 1 : 0;
  pv.prof16_i16 = prof16_i16_ ? 1 : 0;
  pv.max_abs_t = table_.max_abs();
  pv.mfma_sweep = mfma_ && d_prof16_ && !prof16_window_ && !prof16_i16_ ? 1 : 0;
  return pv;
}

ResultFormat HipEngine::auto_format(int64_t max_l2, int64_t min_l2) const {
  R2Params p;
  if (min_l2 > 0 && r2_params(L1_, min_l2, max_l2, min_t_, max_t_, p)) return ResultFormat::R2;
  return pick_result_format(L1_, max_l2, table_.max_abs());
}

R2Params HipEngine::r2_params_for(int64_t min_l2, int64_t max_l2) const {
  R2Params p;
  if (!r2_params(L1_, min_l2, max_l2, min_t_, max_t_, p)) throw Error("R2 cannot hold records of these lengths");
  return p;
}

// Splits a chunk's records into the short-kernel set (<= 64 lanes) and the long list (tile kernel).
// OpenMP: per-thread partial lists are concatenated in thread order, so long_recs stays sorted.
void HipEngine::plan_chunk(const int64_t* offsets, int64_t n, ChunkPlan& cp) const {
  cp.long_recs.clear();
  const int64_t short_min_len = std::max<int64_t>(L1_ - (dev::kWave - 1), 0);  // lanes_needed <= 64
  const int nt = n > (1 << 16) ? omp_get_max_threads() : 1;
  std::vector<std::vector<int32_t>> part(nt);
  std::vector<int64_t> mins(nt, INT64_MAX), maxs(nt, 0), nshort(nt, 0), cells(nt, 0);
#pragma omp parallel for schedule(static, 1) num_threads(nt)  // parts, not thread ids (any team size)
  for (int t = 0; t < nt; ++t) {
    const int64_t b = n * t / nt, e = n * (t + 1) / nt;
    int64_t mn = INT64_MAX, mx = 0, ns = 0, cl = 0;
    for (int64_t i = b; i < e; ++i) {
      const int64_t L2 = offsets[i + 1] - offsets[i];
      mx = std::max(mx, L2);
      cl += record_cells(L1_, L2);
      if (L2 >= short_min_len) {
        mn = std::min(mn, L2);
        ++ns;
      } else {
        part[t].push_back(static_cast<int32_t>(i));
      }
    }
    mins[t] = mn;
    maxs[t] = mx;
    nshort[t] = ns;
    cells[t] = cl;
  }
  cp.min_short = INT64_MAX;
  cp.max_l2 = 0;
  cp.n_short = 0;
  cp.cells = 0;
  for (int t = 0; t < nt; ++t) {
    cp.min_short = std::min(cp.min_short, mins[t]);
    cp.max_l2 = std::max(cp.max_l2, maxs[t]);
    cp.n_short += nshort[t];
    cp.cells += cells[t];
    cp.long_recs.insert(cp.long_recs.end(), part[t].begin(), part[t].end());
  }
  if (L1_ >= (int64_t{1} << 30) || cp.max_l2 >= (int64_t{1} << 30))
    throw Error("Seq1 / Seq2 lengths beyond 2^30 exceed the device engine's offset range");
}

namespace {
// Layout of one chunk's tile plan in a single buffer: wave starts | long_recs | keys (8-aligned).
struct PlanLayout {
  size_t starts_off = 0, long_off = 0, keys_off = 0, upload_bytes = 0, total = 0;
  PlanLayout(size_t n_starts, size_t n_long) {
    long_off = n_starts * sizeof(dev::WaveStart);
    keys_off = (long_off + n_long * sizeof(int32_t) + 7) & ~size_t{7};
    upload_bytes = long_off + n_long * sizeof(int32_t);
    total = keys_off + n_long * sizeof(unsigned long long);
  }
};

// Per-tile fixed cost in step units (record/tile setup, the wave reduction), for load balancing.
constexpr int64_t kTileOverheadSteps = 24;
// Staging one sliding window (tile16_slide_kernel), per wave, in step units.
constexpr int64_t kSlideStageSteps = 96;
}  // namespace

// Device view of an uploaded plan buffer (starts | long_recs | keys). Identity record lists upload no
// long_recs (PlanLayout built with n_long = 0): their keys follow the starts.
dev::Plan HipEngine::device_plan(void* d_plan, size_t n_starts, bool has_long_recs, int64_t n_long,
                                 const TilePlan& tp) const {
  const PlanLayout lay(n_starts, has_long_recs ? static_cast<size_t>(n_long) : 0);
  char* base = static_cast<char*>(d_plan);
  dev::Plan plan;
  plan.u = tp.u;
  plan.win_tiles = tp.win_tiles;
  plan.n_waves = tp.slide ? tp.slide_wgs * dev::kTile16WavesPerBlock : static_cast<int64_t>(n_starts) - 1;
  plan.slide_items = tp.slide_items;
  plan.slide_members = tp.slide_members;
  plan.starts = reinterpret_cast<const dev::WaveStart*>(base + lay.starts_off);
  plan.long_recs = has_long_recs ? reinterpret_cast<const int32_t*>(base + lay.long_off) : nullptr;
  plan.n_long = n_long;
  plan.keys = reinterpret_cast<unsigned long long*>(base + lay.keys_off);
  plan.r2 = r2_;
  return plan;
}

// Sliding-window plan (tile16_slide_kernel): the long records sorted by length (longest first) in groups of 16,
// one per wave of a workgroup; a group's tiles split into items of at most half a workgroup's share, the
// items assigned largest first to the least-loaded workgroup (one 16-wave workgroup per CU: the window takes
// most of the LDS). Encoding in `starts` (dev::Plan::slide_items / slide_members). False: no window fits, or
// the groups would run less than min_fill of their waves (a few huge records: the other plans give every wave
// a tile of its own; an int16 profile's other plan is the LUT tile kernel, so it takes emptier groups).
bool HipEngine::plan_slide(const int64_t* offsets, const int32_t* long_recs, int64_t n_long, double min_fill,
                           TilePlan& tp, std::vector<dev::WaveStart>& starts) const {
  // 4 sub-tiles by default: limits 14.9 (U = 2) -> 16.7 T cells/s, the int16 profile on limits' lengths
  // 10.6 -> 13.8 (profiles/tile16_r5/README.txt)
  const int u = tile_u_ == 2 || (tile_u_ == 8 && slide_wgs_per_cu_ == 1) ? tile_u_ : 4;
  const int span = dev::tile_span(true, u);
  // two workgroups per CU with half the LDS each (8 waves per SIMD hide the sweep's LDS waits: limits 16.8 ->
  // 17.6 T cells/s, the int16 profile 16.9 -> 18.0), or one with the widest window (MOC_TILE16_SLIDE_WG=1)
  int64_t wmax = dev::tile16_max_window(true);
  if (slide_wgs_per_cu_ == 2)
    while (wmax > 0 && dev::tile16_lds_bytes(2 * dev::tile16_window_bytes(wmax), wmax) > dev::kProf16MaxLds / 2) --wmax;
  const int64_t C = (wmax - span) / 64 * 64;  // steps per window
  if (C < 64) return false;
  constexpr int G = dev::kTile16WavesPerBlock;
  if (static_cast<double>(n_long) < min_fill * static_cast<double>(G * ((n_long + G - 1) / G))) return false;
  std::vector<int32_t> order(static_cast<size_t>(n_long));
  std::vector<int32_t> steps(static_cast<size_t>(n_long));
  for (int64_t li = 0; li < n_long; ++li) {
    const int64_t r = long_recs ? long_recs[li] : li;
    const int64_t L2 = offsets[r + 1] - offsets[r];
    order[li] = static_cast<int32_t>(li);
    steps[li] = static_cast<int32_t>(L2 <= L1_ ? L2 : 0);
  }
  std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return steps[a] > steps[b]; });
  const int64_t n_groups = (n_long + G - 1) / G;
  struct Item {
    int64_t cost;
    int32_t g, t0, t1;
  };
  std::vector<Item> items;
  std::vector<int32_t> glmax(static_cast<size_t>(n_groups), 0);
  int64_t total = 0;
  std::vector<int64_t> gcost(static_cast<size_t>(n_groups), 0);
  std::vector<int32_t> gtiles(static_cast<size_t>(n_groups), 0);
  for (int64_t g = 0; g < n_groups; ++g) {
    int32_t lmax = 0, nt = 0;
    for (int64_t k = g * G; k < std::min<int64_t>(n_long, (g + 1) * G); ++k) {
      const int32_t st = steps[order[k]];
      if (st <= 0) continue;
      lmax = std::max(lmax, st);
      nt = std::max<int32_t>(nt, static_cast<int32_t>(dev::tiles_of(L1_ - st + 1, span)));
    }
    glmax[g] = lmax;
    gtiles[g] = nt;
    // a tile: every wave in lockstep for the group's longest record, plus the staging of each window
    gcost[g] = G * (lmax + kTileOverheadSteps + kSlideStageSteps * ((lmax + C - 1) / C));
    total += gcost[g] * nt;
  }
  if (total <= 0) return false;
  int64_t all_tiles = 0;
  for (int64_t g = 0; g < n_groups; ++g) all_tiles += gtiles[g];
  const int64_t n_wg = std::min<int64_t>(static_cast<int64_t>(num_cus_) * slide_wgs_per_cu_, all_tiles);
  const double share = static_cast<double>(total) / static_cast<double>(n_wg);
  for (int64_t g = 0; g < n_groups; ++g) {
    if (gtiles[g] <= 0) continue;
    const int32_t per = static_cast<int32_t>(std::max<int64_t>(1, static_cast<int64_t>(share / 2) / gcost[g]));
    for (int32_t t0 = 0; t0 < gtiles[g]; t0 += per) {
      const int32_t t1 = std::min(gtiles[g], t0 + per);
      items.push_back(Item{gcost[g] * (t1 - t0), static_cast<int32_t>(g), t0, t1});
    }
  }
  std::stable_sort(items.begin(), items.end(), [](const Item& a, const Item& b) { return a.cost > b.cost; });
  std::vector<std::vector<int32_t>> of(static_cast<size_t>(n_wg));
  std::priority_queue<std::pair<int64_t, int64_t>, std::vector<std::pair<int64_t, int64_t>>, std::greater<>> load;
  for (int64_t b = 0; b < n_wg; ++b) load.emplace(0, b);
  for (size_t k = 0; k < items.size(); ++k) {
    auto [l, b] = load.top();
    load.pop();
    of[static_cast<size_t>(b)].push_back(static_cast<int32_t>(k));
    load.emplace(l + items[k].cost, b);
  }
  starts.clear();
  starts.reserve(static_cast<size_t>(n_wg + 1 + 2 * static_cast<int64_t>(items.size()) + n_groups * G));
  int32_t n_it = 0;
  for (int64_t b = 0; b < n_wg; ++b) {
    starts.push_back(dev::WaveStart{n_it, 0});
    n_it += static_cast<int32_t>(of[b].size());
  }
  starts.push_back(dev::WaveStart{n_it, 0});
  tp.slide_items = static_cast<int64_t>(starts.size());
  for (int64_t b = 0; b < n_wg; ++b)
    for (const int32_t k : of[b]) {
      const Item& it = items[k];
      starts.push_back(dev::WaveStart{it.g, it.t0});
      starts.push_back(dev::WaveStart{glmax[it.g], it.t1});
    }
  tp.slide_members = static_cast<int64_t>(starts.size());
  for (int64_t k = 0; k < n_groups * G; ++k) {
    if (k < n_long) {
      const int32_t li = order[k];
      const int64_t r = long_recs ? long_recs[li] : li;
      starts.push_back(dev::WaveStart{li, static_cast<int32_t>(offsets[r + 1] - offsets[r])});
    } else {
      starts.push_back(dev::WaveStart{-1, 0});
    }
  }
  tp.slide_wgs = n_wg;
  tp.slide_per_cu = slide_wgs_per_cu_;
  tp.tile16 = true;
  tp.wide = true;
  tp.slide = true;
  tp.u = u;
  tp.window = span + C;
  tp.win_tiles = 0;
  return true;
}

// Cost-balanced contiguous wave runs over the record-major tile list of the long records (record li =
// offsets-relative index long_recs[li], or li when long_recs is null), restricted to part `part` of
// `parts` of the total cost (context-parallel shares). Returns n_waves + 1 starts (empty: no work).
// tp: sub-tiles per wave tile, and which sweep the plan is for (tile16 when the problem has a profile and,
// for a windowed one, the records fit a window — else the LUT tile kernel).
// Windowed tile16 (Seq1 longer than one LDS image): the list is window-major — window m holds the tiles
// t in [m*T, (m+1)*T) of every record, T = (W - span - max L2) / span so that their profile columns
// [t*span, t*span + span + L2) all lie in [m*T*span, m*T*span + W) — and every window gets whole
// workgroups of waves (16-aligned; its last wave is an empty marker ending at (n_long, m*T)), each
// workgroup staging its window once.
std::vector<dev::WaveStart> HipEngine::plan_waves(const int64_t* offsets, const int32_t* long_recs, int64_t n_long,
                                                  int part, int parts, TilePlan& tp) const {
  std::vector<dev::WaveStart> starts;
  tp = TilePlan{};
  if (n_long <= 0) return starts;
  int64_t sum_l2 = 0, max_l2 = 0;
  for (int64_t li = 0; li < n_long; ++li) {
    const int64_t r = long_recs ? long_recs[li] : li;
    const int64_t L2 = offsets[r + 1] - offsets[r];
    sum_l2 += L2;
    max_l2 = std::max(max_l2, L2 <= L1_ ? L2 : 0);
  }
  int64_t W = prof16_window_;
  bool wide = prof16_wide_ && !mfma_ && W == 0;
  // a whole byte-pair image whose widened form does not fit (L1 ~ 1500..3050): short records take a widened
  // WINDOW instead (one packed add per lane and step; the window holds U = 4 tiles plus the longest record)
  if (W == 0 && d_prof16_ && !prof16_wide_ && !mfma_ && tile16_window_wide_ && tile_u_ <= 0 &&
      max_l2 + 2 * 128 * 4 <= dev::tile16_max_window(true)) {
    W = dev::tile16_max_window(true);
    wide = true;
  }
  // records too long for a widened window on a Seq1 whose widened image exceeds the LDS — with the byte pairs
  // whole (limits: L1 3000, records up to 2000 letters), as windows (L1 past ~3050), or an int16 profile:
  // sliding widened windows (limits 12.9 -> 16.8 T cells/s, L1 20 000 with input3's records 17.3 -> 20.7,
  // L1 150 000 9.6 -> 15.9; profiles/tile16_r5/README.txt)
  if ((W == 0 || max_l2 + 2 * 128 * 4 > dev::tile16_max_window(true)) && !wide && d_prof16_ && !mfma_ &&
      tile16_slide_ && parts == 1 &&
      (tile_u_ <= 0 || tile_u_ == 2 || tile_u_ == 4 || tile_u_ == 8))
    if (plan_slide(offsets, long_recs, n_long, prof16_i16_ ? 0.25 : 0.8, tp, starts)) return starts;
  tp.window = W;
  tp.wide = wide;
  tp.tile16 = d_prof16_ != nullptr && (W == 0 || max_l2 + 2 * 128 <= W) && (wide || !prof16_i16_);
  // sub-tiles per wave tile: 4 amortises the per-tile setup over short records, 2 keeps more waves busy
  // on long ones (measured, both kernels: profiles/tile_variants.log, profiles/tile16_variants.log) — unless
  // the batch gives every resident wave >= 8 tiles of 4 sub-tiles: with a record's last tile cut to its
  // valid sub-tiles (tile16_search_kernel) 4 then wins on long records too (input3: 17.2 -> 17.7 T cells/s;
  // 4 tiles per wave, heavy3's bench batch, stays on 2: 14.8 vs 14.3; profiles/r6/README.txt)
  int u = tile_u_ > 0 ? tile_u_ : (sum_l2 < 96 * n_long ? 4 : 2);
  if (tile_u_ <= 0 && u == 2 && W == 0 && tp.tile16) {
    int64_t tiles4 = 0;
    for (int64_t li = 0; li < n_long; ++li) {
      const int64_t r = long_recs ? long_recs[li] : li;
      tiles4 += dev::tiles_of(dev::lanes_needed(L1_, offsets[r + 1] - offsets[r]), dev::tile_span(true, 4));
    }
    const int64_t lds = dev::tile16_lds_bytes((wide ? 2 : 1) * static_cast<int64_t>(prof16_bytes_), L1_);
    const int64_t resident = static_cast<int64_t>(num_cus_) * dev::tile16_waves_per_cu(static_cast<int>(lds));
    if (tiles4 >= 8 * resident * parts) u = 4;
  }
  if (tile_u_ <= 0 && u == 4 && tp.tile16 && W == 0 && 128 * 8 <= prof16_overhang_) u = 8;  // tile16: wider tiles
  if (u > 4 && !(tp.tile16 && W == 0 && 128 * u <= prof16_overhang_)) u = 4;  // the overhang bounds the span
  if (u > 2 && mfma_ && tp.tile16 && W == 0) u = 2;  // the matrix-core sweep's register budget (U = 4 spills)
  if (tp.tile16 && W > 0) {
    // windowed: the widest tiles a window holds twice (L1 = 20 000, input3 records: U = 4 -> 9.3 T cells/s,
    // U = 2 -> 8.4, U = 1 -> 7.0; profiles/kernel_bench_long.log)
    if (tile_u_ <= 0) u = 4;
    while (u > 1 && max_l2 + 2 * 128 * u > W) u /= 2;
    // widened windows (short records): 8 sub-tiles when one tile and the longest record fit the window
    if (wide && tile_u_ <= 0 && short_window_u8_ && max_l2 + 128 * 8 <= W) u = 8;
  }
  tp.u = u;
  const int span = dev::tile_span(tp.tile16, u);
  std::vector<int64_t> tcost(static_cast<size_t>(n_long));
  std::vector<int32_t> ntiles(static_cast<size_t>(n_long));
  int64_t total_tiles = 0;
  for (int64_t li = 0; li < n_long; ++li) {
    const int64_t r = long_recs ? long_recs[li] : li;
    const int64_t L2 = offsets[r + 1] - offsets[r];
    ntiles[li] = static_cast<int32_t>(dev::tiles_of(dev::lanes_needed(L1_, L2), span));
    tcost[li] = (L2 <= L1_ ? L2 : 0) + kTileOverheadSteps;
    total_tiles += ntiles[li];
  }
  const int s1_len = tp.tile16 && W > 0 ? static_cast<int>(W) : static_cast<int>(L1_);
  const int64_t prof_lds = (wide ? 2 : 1) * (W ? dev::tile16_window_bytes(W) : static_cast<int64_t>(prof16_bytes_));
  const int waves_per_cu = tp.tile16 ? dev::tile16_waves_per_cu(static_cast<int>(dev::tile16_lds_bytes(prof_lds, s1_len)))
                                     : tile_waves_per_cu_;
  if (!(tp.tile16 && W > 0)) {
    std::vector<int64_t> pre(static_cast<size_t>(n_long) + 1, 0);
    for (int64_t li = 0; li < n_long; ++li) pre[li + 1] = pre[li] + ntiles[li] * tcost[li];
    const int64_t C = pre[n_long];
    const int64_t lo = C * part / parts, hi = C * (part + 1) / parts;
    // position of cost threshold X in (li, t): first tile whose start cost is >= X
    auto locate = [&](int64_t X) {
      if (X >= C) return dev::WaveStart{static_cast<int32_t>(n_long), 0};
      const int64_t li = std::upper_bound(pre.begin(), pre.end(), X) - pre.begin() - 1;
      const int64_t t = (X - pre[li] + tcost[li] - 1) / tcost[li];
      if (t >= ntiles[li]) return dev::WaveStart{static_cast<int32_t>(li + 1), 0};
      return dev::WaveStart{static_cast<int32_t>(li), static_cast<int32_t>(t)};
    };
    const int64_t part_tiles = std::max<int64_t>(1, total_tiles * (hi - lo) / std::max<int64_t>(C, 1));
    const int64_t n_waves = std::min<int64_t>(part_tiles, static_cast<int64_t>(num_cus_) * waves_per_cu);
    starts.resize(static_cast<size_t>(n_waves) + 1);
    for (int64_t w = 0; w <= n_waves; ++w) starts[w] = locate(lo + (hi - lo) * w / n_waves);
    return starts;
  }
  // ---- windowed tile16: window-major runs, whole workgroups per window
  // (a widened window, chosen for short records only, packs one more tile: its columns
  // [0, T * span + max L2) still lie inside the window)
  const int64_t T = std::max<int64_t>(1, (W - (wide ? 0 : span) - max_l2) / span);
  tp.win_tiles = static_cast<int32_t>(T);
  int32_t max_nt = 0;
  for (int64_t li = 0; li < n_long; ++li) max_nt = std::max(max_nt, ntiles[li]);
  const int64_t M = (max_nt + T - 1) / T;
  auto count = [&](int64_t li, int64_t m) { return std::clamp<int64_t>(ntiles[li] - m * T, 0, T); };
  std::vector<int64_t> wcost(static_cast<size_t>(M), 0);
  for (int64_t li = 0; li < n_long; ++li)
    for (int64_t m = 0; m * T < ntiles[li]; ++m) wcost[m] += count(li, m) * tcost[li];
  std::vector<int64_t> wstart(static_cast<size_t>(M) + 1, 0);
  for (int64_t m = 0; m < M; ++m) wstart[m + 1] = wstart[m] + wcost[m];
  const int64_t C = wstart[M];
  const int64_t lo = C * part / parts, hi = C * (part + 1) / parts;
  constexpr int kWg = 16;  // waves per tile16 workgroup
  const int64_t target_wgs = std::max<int64_t>(1, static_cast<int64_t>(num_cus_) * waves_per_cu / kWg);
  // workgroups per window in proportion to its cost, largest remainders first, so that they add up to
  // target_wgs: one workgroup over the resident count waits for a second round (ceil per window put input4's
  // 3 windows at 3 x 86 = 258 on 256 CUs: 2.4 ms instead of 1.3)
  std::vector<int64_t> wgs_of(static_cast<size_t>(M), 0);
  {
    std::vector<std::pair<double, int64_t>> frac;
    int64_t used = 0;
    for (int64_t m = 0; m < M; ++m) {
      const int64_t a = std::max(lo, wstart[m]) - wstart[m], b = std::min(hi, wstart[m + 1]) - wstart[m];
      if (b <= a) continue;
      const double ideal = static_cast<double>(target_wgs) * static_cast<double>(b - a) /
                           static_cast<double>(std::max<int64_t>(hi - lo, 1));
      const int64_t share_tiles = std::max<int64_t>(1, (b - a) / std::max<int64_t>(1, C / std::max<int64_t>(total_tiles, 1)));
      const int64_t cap = std::max<int64_t>(1, (share_tiles + kWg - 2) / (kWg - 1));
      wgs_of[m] = std::clamp<int64_t>(static_cast<int64_t>(ideal), 1, cap);
      used += wgs_of[m];
      if (wgs_of[m] < cap) frac.emplace_back(ideal - static_cast<double>(wgs_of[m]), m);
    }
    std::sort(frac.begin(), frac.end(), [](const auto& x, const auto& y) { return x.first > y.first; });
    for (const auto& f : frac) {
      if (used >= target_wgs) break;
      ++wgs_of[f.second];
      ++used;
    }
  }
  std::vector<int64_t> pre(static_cast<size_t>(n_long) + 1);
  for (int64_t m = 0; m < M; ++m) {
    const int64_t a = std::max(lo, wstart[m]) - wstart[m], b = std::min(hi, wstart[m + 1]) - wstart[m];
    if (b <= a) continue;
    pre[0] = 0;
    for (int64_t li = 0; li < n_long; ++li) pre[li + 1] = pre[li] + count(li, m) * tcost[li];
    const dev::WaveStart end_marker{static_cast<int32_t>(n_long), static_cast<int32_t>(m * T)};
    auto locate = [&](int64_t X) {
      if (X >= pre[n_long]) return end_marker;
      const int64_t li = std::upper_bound(pre.begin(), pre.end(), X) - pre.begin() - 1;
      const int64_t t = (X - pre[li] + tcost[li] - 1) / tcost[li];
      if (t >= count(li, m)) return dev::WaveStart{static_cast<int32_t>(li + 1), static_cast<int32_t>(m * T)};
      return dev::WaveStart{static_cast<int32_t>(li), static_cast<int32_t>(m * T + t)};
    };
    const int64_t wgs = wgs_of[m];
    const int64_t real = wgs * kWg - 1;  // + one empty marker wave that ends the window's list
    for (int64_t q = 0; q < real; ++q) starts.push_back(locate(a + (b - a) * q / real));
    starts.push_back(locate(b));  // the last real wave ends at the share's end ...
    starts.back() = b >= pre[n_long] ? end_marker : starts.back();
    // ... and the marker wave [end, next window's first start) is empty: its start is the end of this window
  }
  if (starts.empty()) return starts;
  // every window contributed wgs*16 entries: the real waves' starts + its end; the final entry ends the list
  starts.push_back(starts.back());
  return starts;
}

namespace {
struct LenStats {
  int64_t mn = INT64_MAX, mx = 0;
};
LenStats scan_lengths(const int64_t* offsets, const uint8_t* lengths8, int64_t n) {
  const int nt = n > (1 << 16) ? omp_get_max_threads() : 1;
  std::vector<int64_t> mins(nt, INT64_MAX), maxs(nt, 0);
#pragma omp parallel for schedule(static, 1) num_threads(nt)  // parts, not thread ids (any team size)
  for (int t = 0; t < nt; ++t) {
    const int64_t b = n * t / nt, e = n * (t + 1) / nt;
    int64_t mn = INT64_MAX, mx = 0;
    if (lengths8) {
      for (int64_t i = b; i < e; ++i) {
        const int64_t L = lengths8[i];
        mn = std::min(mn, L);
        mx = std::max(mx, L);
      }
    } else {
      for (int64_t i = b; i < e; ++i) {
        const int64_t L = offsets[i + 1] - offsets[i];
        mn = std::min(mn, L);
        mx = std::max(mx, L);
      }
    }
    mins[t] = mn;
    maxs[t] = mx;
  }
  LenStats s;
  for (int t = 0; t < nt; ++t) {
    s.mn = std::min(s.mn, mins[t]);
    s.mx = std::max(s.mx, maxs[t]);
  }
  return s;
}
}  // namespace

bool HipEngine::direct_pointers(const WireBatch& b, void* out, int fb, dev::ShortArgs& a) const {
  const void *dc = nullptr, *doff = nullptr, *dlen = nullptr, *dout = nullptr;
  const int64_t c0 = b.first_letter(), c1 = b.end_letter(), n = b.n;
  // byte range of the letters: [b0, b1)
  const int64_t b0 = b.packed33 ? p33_first_byte(c0) : b.packed5 ? (5 * c0) >> 3 : c0;
  const int64_t b1 = b.packed33 ? p33_end_byte(c1) : b.packed5 ? ((5 * c1 + 7) >> 3) + 1 : c1;
  if (b.device) {  // device-resident (e.g. received over RCCL): the pointers are the kernel's already
    dc = b.letters + b0;
    doff = b.offsets;
    dlen = b.lengths;
    dout = out;
  } else {
    // the kernels stage letters with 16-byte loads of the aligned granules covering [b0, b1): a granule
    // never crosses a page, so the pages of [b0, b1) are all that must be mapped
    if (c1 > c0 && !pinned_range(b.letters + b0, static_cast<size_t>(b1 - b0), &dc)) return false;
    if (!pinned_range(b.offsets, sizeof(int64_t) * static_cast<size_t>(b.offset_entries()), &doff)) return false;
    if (b.lengths && !pinned_range(b.lengths, static_cast<size_t>(b.length_bytes()), &dlen)) return false;
    if (!pinned_range(out, static_cast<size_t>(fb) * static_cast<size_t>(n), &dout)) return false;
  }
  // device view of the codes base pointer (record i at base + offsets[i], or at bit 5*offsets[i])
  a.codes = c1 > c0 ? static_cast<const uint8_t*>(dc) - b0 : nullptr;
  a.dbg_codes_end = b1 + 15;  // the last granule may extend up to 15 bytes past b1
  a.offsets = static_cast<const int64_t*>(doff);
  a.off_shift = b.off_shift;
  a.lengths8 = b.lengths && b.len_bits == 8 ? static_cast<const uint8_t*>(dlen) : nullptr;
  a.lengths4 = b.lengths && b.len_bits == 4 ? static_cast<const uint8_t*>(dlen) : nullptr;
  a.lengths3 = b.lengths && b.len_bits == 3 ? static_cast<const uint8_t*>(dlen) : nullptr;
  a.lengths6 = b.lengths && b.len_bits == kLenBase6 ? static_cast<const uint8_t*>(dlen) : nullptr;
  a.len_base = static_cast<int32_t>(b.len_base);
  a.out = const_cast<void*>(dout);
  return c1 > c0;
}

void HipEngine::solve(const uint8_t* codes, const int64_t* offsets, int64_t n, Result* out) {
  solve_ex(codes, offsets, nullptr, n, out, ResultFormat::R12);
}

void HipEngine::solve_ex(const uint8_t* codes, const int64_t* offsets, const uint8_t* lengths, int64_t n, void* out,
                         ResultFormat fmt, const BatchHints& hints, int packed, int len_bits, int len_base) {
  WireBatch b;
  b.letters = codes;
  if (packed < 0 || packed > 3 || packed == 2) throw Error("letters: 0 bytes, 1 5-bit packed or 3 P33 fields");
  b.packed5 = packed == 1;
  b.packed33 = packed == 3;
  b.offsets = offsets;
  b.lengths = lengths;
  b.len_bits = len_bits;
  b.len_base = len_base;
  b.n = n;
  b.min_l2 = hints.min_l2;
  b.max_l2 = hints.max_l2;
  solve_wire(b, out, fmt);
}

bool HipEngine::streams_packed(int64_t min_l2, int64_t max_l2) const {
  dev::ShortArgs a;
  a.packed33 = 1;  // the widest LDS layout of the letter forms
  return have_problem_ && dev::configure_swipe(L1_, min_l2, max_l2, table_.max_abs(), a);
}

void HipEngine::solve_wire(const WireBatch& batch, void* out, ResultFormat fmt) { solve_wire_impl(batch, out, fmt, false); }

void HipEngine::begin_wire(const WireBatch& batch, void* out, ResultFormat fmt) { solve_wire_impl(batch, out, fmt, true); }

void HipEngine::finish_wire() {
  if (!pending_) return;
  pending_ = false;
  MOC_HIP_CHECK(hipEventSynchronize(ev_b_));
  float ms = 0;
  MOC_HIP_CHECK(hipEventElapsedTime(&ms, ev_a_, ev_b_));
  stats_.kernel_ms = ms;
  pending_wall_.stop();
  stats_.total_ms = pending_wall_.total_ms();
}

void HipEngine::solve_wire_impl(const WireBatch& batch, void* out, ResultFormat fmt, bool async) {
  finish_wire();  // a solve still in flight completes first (its stats are replaced below)
  WireBatch b = batch;
  const int64_t n = b.n;
  if (b.lengths && b.len_bits != 8 && b.len_bits != 4 && b.len_bits != 3 && b.len_bits != kLenBase6)
    throw Error("lengths must be 8-, 4-, 3-bit or base-6");
  if (b.lengths && b.len_bits == kLenBase6 && (reinterpret_cast<uintptr_t>(b.lengths) & 7))
    throw Error("base-6 lengths must be 8-byte aligned (the kernels load whole words)");
  if (b.off_shift && (!b.lengths || b.min_l2 < 0 || b.max_l2 < 0 || b.off_shift > 6))
    throw Error("sparse offsets need narrow lengths, the length range and a stride of at most 64 records");
  if (b.device && (b.min_l2 < 0 || b.max_l2 < 0)) throw Error("a device-resident batch needs its length range");
  if (!have_problem_) throw Error("HipEngine::solve before set_problem");
  MOC_HIP_CHECK(hipSetDevice(device_));
  TraceRange tr("moc.solve");
  Stopwatch wall;
  wall.start();
  stats_ = EngineStats{};
  stats_.format = static_cast<int32_t>(fmt);
  stats_.records = n;
  if (n <= 0) return;
  const int fb = result_bytes(fmt);

  // ---- batch bounds (hints, or one parallel pass over the lengths)
  LenStats ls;
  if (b.min_l2 >= 0 && b.max_l2 >= 0) {
    ls.mn = b.min_l2;
    ls.mx = b.max_l2;
  } else {
    ls = scan_lengths(b.offsets, b.len_bits == 8 ? b.lengths : nullptr, n);
  }
  if (b.len_bits == 8 && b.lengths && ls.mx > 255 && !b.off_shift) b.lengths = nullptr;
  if (b.len_bits == 8 && b.lengths && ls.mx > 255) throw Error("8-bit lengths cannot hold this batch's lengths");
  if (b.len_bits == 4 && b.lengths && (ls.mn < b.len_base || ls.mx > b.len_base + 15))
    throw Error("nibble lengths cannot hold this batch's lengths");
  if (b.len_bits == 3 && b.lengths && (ls.mn < b.len_base || ls.mx > b.len_base + 7))
    throw Error("3-bit lengths cannot hold this batch's lengths");
  if (b.len_bits == kLenBase6 && b.lengths && (ls.mn < b.len_base || ls.mx > b.len_base + 5))
    throw Error("base-6 lengths cannot hold this batch's lengths");
  if (fmt == ResultFormat::R4 && (L1_ > 255 || ls.mx > 255 || table_.max_abs() * ls.mx >= 32767))
    throw Error("result format R4 cannot hold this batch");
  if (fmt == ResultFormat::R8 && (L1_ > 65535 || ls.mx > 65535)) throw Error("result format R8 cannot hold this batch");
  r2_ = R2Params{};
  if (fmt == ResultFormat::R2 && !r2_params(L1_, ls.mn, ls.mx, min_t_, max_t_, r2_))
    throw Error("result format R2 cannot hold this batch");
  stats_.r2 = r2_;

  // ---- direct zero-copy streaming path
  dev::ShortArgs a;
  a.n = n;
  a.fmt = static_cast<int32_t>(fmt);
  a.counter = d_counter_;
  a.packed5 = b.packed5 ? 1 : 0;
  a.packed33 = b.packed33 ? 1 : 0;
  const bool swipe = dev::configure_swipe(L1_, ls.mn, ls.mx, table_.max_abs(), a, b.device, sem_ == Semantics::Spec);
  // packed letters stream straight into the swipe kernel only; other kernels read unpacked bytes. Sparse
  // offsets need whole tiles of 2^off_shift records (the swipe tiles are powers of two >= 64).
  const bool kernel_ok = (swipe || (!b.packed5 && !b.packed33 &&
                                    dev::configure_short(L1_, ls.mn, ls.mx, a))) &&
                         (a.tile_records % (1 << b.off_shift)) == 0;
  if ((opt_.allow_direct || b.device) && kernel_ok && direct_pointers(b, out, fb, a)) {
    // device-resident: the wave-autonomous swipe kernel (byte letters with dense offsets, or P33 letters with
    // dense or 64-record sparse offsets)
    a.lane_direct =
        swipe && b.device && (b.packed33 || !b.off_shift) && (!b.packed33 || a.rpw <= 16) && lane_direct_enabled()
            ? 1
            : 0;
    const dev::ProblemView pv = problem_view(ls.mx);
    const bool graph = prepare_direct(pv, a, swipe);  // capture / instantiation stays outside the timed span
    MOC_HIP_CHECK(hipEventRecord(ev_a_, s_compute_));
    launch_direct(pv, a, swipe, graph);
    stats_.kernels = swipe ? 1 : 2;
    stats_.forms = swipe ? dev::swipe_launch_form(a) : dev::short_form(pv, a);
    MOC_HIP_CHECK(hipEventRecord(ev_b_, s_compute_));
    stats_.direct = 1;
    stats_.chunks = 1;
    stats_.h2d_bytes = b.device ? 0 : b.letter_bytes() + (a.lengths3 || a.lengths4 || a.lengths6 || a.lengths8 ? b.length_bytes() : 8 * n);
    stats_.d2h_bytes = b.device ? 0 : static_cast<int64_t>(fb) * n;
    pending_ = true;
    pending_wall_ = wall;
    if (!async) finish_wire();
    return;
  }
  if (b.device) throw Error("device-resident wire batches stream through the swipe kernel only");
  uvector<uint8_t> bytes;  // P33 letters: the staged pipeline takes bytes (or 5-bit packing)
  if (b.packed33) {
    const int64_t c0 = b.first_letter(), c1 = b.end_letter();
    bytes.resize(static_cast<size_t>(c1) + 16);
    unpack33(b.letters, c0, c1 - c0, bytes.data() + c0);
    b.letters = bytes.data();
    b.packed33 = false;
  }
  if (b.off_shift) {  // the staged pipeline plans from dense offsets: rebuild them from the lengths
    uvector<int64_t> dense(static_cast<size_t>(n) + 1);
    expand_offsets(b.offsets, b.off_shift, b.lengths, b.len_bits, b.len_base, n, dense.data());
    run_staged(b.letters, dense.data(), n, out, fmt, b.packed5);
  } else {
    run_staged(b.letters, b.offsets, n, out, fmt, b.packed5);
  }
  wall.stop();
  stats_.total_ms = wall.total_ms();
}

// The direct path's launch sequence (work-counter reset + persistent streaming kernel) as a hipGraph:
// captured once per distinct argument set, replayed for repeated solves over the same buffers (a
// bench loop, a service re-scoring a resident batch) — one graph launch instead of re-validating and
// re-encoding two launches. Arguments are plain structs, compared bytewise.
bool HipEngine::prepare_direct(const dev::ProblemView& pv, const dev::ShortArgs& a, bool swipe) {
  if (!opt_.use_graphs) return false;
  DirectKey key;
  std::memset(static_cast<void*>(&key), 0, sizeof key);  // padding too: keys are compared bytewise
  key.pv = pv;
  key.a = a;
  key.swipe = swipe ? 1 : 0;
  for (int i = 0; i < kGraphs; ++i)
    if (graph_exec_[i] && std::memcmp(&key, &graph_key_[i], sizeof key) == 0) {
      graph_cur_ = i;
      return true;
    }
  // an argument set seen for the first time launches plainly: a one-shot job (./final on a reference
  // input) pays no capture and instantiation; a repeated solve captures at its second launch
  bool seen = false;
  for (int i = 0; i < kGraphs; ++i) seen = seen || (seen_valid_[i] && std::memcmp(&key, &seen_key_[i], sizeof key) == 0);
  if (!seen) {
    std::memcpy(static_cast<void*>(&seen_key_[seen_next_]), &key, sizeof key);
    seen_valid_[seen_next_] = true;
    seen_next_ = (seen_next_ + 1) % kGraphs;
    return false;
  }
  // two argument sets stay instantiated (a streaming job alternates between the two slots of its ring):
  // the one not used last is replaced
  const int slot = graph_exec_[graph_cur_] ? 1 - graph_cur_ : graph_cur_;
  if (graph_exec_[slot]) {
    MOC_HIP_CHECK(hipGraphExecDestroy(graph_exec_[slot]));
    graph_exec_[slot] = nullptr;
  }
  hipGraph_t g = nullptr;
  MOC_HIP_CHECK(hipStreamBeginCapture(s_compute_, hipStreamCaptureModeThreadLocal));
  if (swipe)
    dev::launch_swipe(pv, a, num_cus_, s_compute_);
  else
    dev::launch_short(pv, a, num_cus_, s_compute_);
  const hipError_t launch_err = hipGetLastError();
  MOC_HIP_CHECK(hipStreamEndCapture(s_compute_, &g));
  MOC_HIP_CHECK(launch_err);
  const hipError_t inst = hipGraphInstantiate(&graph_exec_[slot], g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  MOC_HIP_CHECK(inst);
  std::memcpy(static_cast<void*>(&graph_key_[slot]), &key, sizeof key);
  graph_cur_ = slot;
  return true;
}

// The direct path's launch (work-counter reset + persistent streaming kernel): the hipGraph captured
// by prepare_direct for this argument set — one graph launch for repeated solves over the same buffers
// (a bench loop, a service re-scoring a resident batch) — or a plain launch without graphs.
void HipEngine::launch_direct(const dev::ProblemView& pv, const dev::ShortArgs& a, bool swipe, bool graph) {
  if (!graph) {
    if (swipe)
      dev::launch_swipe(pv, a, num_cus_, s_compute_);
    else
      dev::launch_short(pv, a, num_cus_, s_compute_);
    MOC_HIP_CHECK(hipGetLastError());
    return;
  }
  MOC_HIP_CHECK(hipGraphLaunch(graph_exec_[graph_cur_], s_compute_));
}

void HipEngine::run_staged(const uint8_t* codes, const int64_t* offsets, int64_t n, void* out, ResultFormat fmt,
                           bool packed5) {
  // a batch of one chunk has nothing to overlap: its copies go on the compute stream, and a job that only
  // ever runs such batches (every tiny --backend=hip job) never pays the two side streams' hardware queues
  // (~10-20 ms each to set up on the MI355X box)
  const bool one_chunk = n <= opt_.chunk_records && offsets[n] - offsets[0] <= opt_.chunk_bytes;
  if (!one_chunk) ensure_side_streams();
  hipStream_t s_in = one_chunk ? s_compute_ : s_copy_, s_back = one_chunk ? s_compute_ : s_return_;
  const int fb = result_bytes(fmt);
  ChunkPlan cp;
  double kernel_ms = 0;
  auto retire = [&](Slot& s) {
    if (!s.busy) return;
    MOC_HIP_CHECK(hipEventSynchronize(s.ev_done));
    MOC_HIP_CHECK(hipEventSynchronize(s.ev_k1));  // complete itself before it is read (not only what it marks)
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
    TraceRange tr_chunk("moc.chunk");
    plan_chunk(offsets + rb, cn, cp);
    stats_.cells += cp.cells;
    // records that the short kernel cannot hold (LDS budget) go to the tile kernel too
    dev::ShortArgs a;
    a.fmt = static_cast<int32_t>(fmt);
    const bool swipe = cp.n_short > 0 && cp.long_recs.empty() &&
                       dev::configure_swipe(L1_, cp.min_short, cp.max_l2, table_.max_abs(), a, true, sem_ == Semantics::Spec);
    bool short_ok = swipe || (cp.n_short > 0 && dev::configure_short(L1_, cp.min_short, cp.max_l2, a));
    // everything through the tile kernel (identity record list) when the short kernel cannot hold it
    const bool all_tiles = cp.n_short > 0 && !short_ok;
    const int32_t* lrecs = all_tiles ? nullptr : cp.long_recs.data();
    const int64_t n_long = all_tiles ? cn : static_cast<int64_t>(cp.long_recs.size());
    TilePlan tp;
    const std::vector<dev::WaveStart> starts = plan_waves(offsets + rb, lrecs, n_long, 0, 1, tp);
    const PlanLayout lay(starts.size(), lrecs ? static_cast<size_t>(n_long) : 0);
    const size_t keys_extra = lrecs ? 0 : sizeof(unsigned long long) * static_cast<size_t>(n_long);
    const size_t cbytes = static_cast<size_t>(offsets[re] - offsets[rb]);
    ensure(s.d_codes, s.d_codes_cap, std::max<size_t>(cbytes, 16) + 32);
    // packed chunk: bytes [pb0, pb1) of the 5-bit stream, char offsets[rb] at bit pbit within it
    const int64_t pb0 = (5 * offsets[rb]) >> 3, pb1 = ((5 * offsets[re] + 7) >> 3) + 1;
    const int64_t pbit = 5 * offsets[rb] - 8 * pb0;
    if (packed5) ensure(s.d_packed, s.d_packed_cap, static_cast<size_t>(pb1 - pb0) + 16);
    ensure(s.d_offsets, s.d_offsets_cap, sizeof(int64_t) * static_cast<size_t>(cn + 1));
    ensure(s.d_out, s.d_out_cap, static_cast<size_t>(fb) * static_cast<size_t>(cn));
    if (!starts.empty()) {
      ensure(s.d_plan, s.d_plan_cap, lay.total + keys_extra);
      ensure_host(s.h_plan, s.h_plan_cap, std::max<size_t>(lay.upload_bytes, 8));
      std::memcpy(static_cast<char*>(s.h_plan) + lay.starts_off, starts.data(), starts.size() * sizeof(dev::WaveStart));
      if (lrecs)
        std::memcpy(static_cast<char*>(s.h_plan) + lay.long_off, lrecs, static_cast<size_t>(n_long) * sizeof(int32_t));
    }
    // ---- copy stream: H2D
    size_t letter_bytes = cbytes;
    if (packed5) {
      letter_bytes = static_cast<size_t>(pb1 - pb0);
      if (cbytes)
        copy_h2d(s.d_packed, codes + pb0, letter_bytes, s_in);
    } else if (cbytes) {
      copy_h2d(s.d_codes, codes + offsets[rb], cbytes, s_in);
    }
    copy_h2d(s.d_offsets, offsets + rb, sizeof(int64_t) * (cn + 1), s_in);
    if (!starts.empty())
      upload_staged(s.d_plan, s.h_plan, lay.upload_bytes, s_in);
    MOC_HIP_CHECK(hipEventRecord(s.ev_h2d, s_in));
    stats_.h2d_bytes += static_cast<int64_t>(letter_bytes + sizeof(int64_t) * (cn + 1) + lay.upload_bytes);
    // ---- compute stream
    MOC_HIP_CHECK(hipStreamWaitEvent(s_compute_, s.ev_h2d, 0));
    if (packed5)
      dev::launch_unpack5(static_cast<const uint8_t*>(s.d_packed), pbit, static_cast<int64_t>(cbytes),
                          static_cast<uint8_t*>(s.d_codes), s_compute_);
    MOC_HIP_CHECK(hipEventRecord(s.ev_k0, s_compute_));
    const dev::ProblemView pv = problem_view(cp.max_l2);
    const uint8_t* dcodes = static_cast<const uint8_t*>(s.d_codes);
    const int64_t* doffs = static_cast<const int64_t*>(s.d_offsets);
    if (short_ok) {
      a.codes = dcodes - offsets[rb];  // base: record i at base + offsets[i] (absolute offsets)
      a.offsets = doffs;
      a.lengths8 = nullptr;
      a.lengths4 = nullptr;
      a.lengths3 = nullptr;
      a.n = cn;
      a.out = s.d_out;
      a.counter = s.d_counter;
      a.lane_direct = swipe && lane_direct_enabled() ? 1 : 0;
      if (swipe)
        dev::launch_swipe(pv, a, num_cus_, s_compute_);
      else
        dev::launch_short(pv, a, num_cus_, s_compute_);
      stats_.kernels |= swipe ? 1 : 2;
      stats_.forms |= swipe ? dev::swipe_launch_form(a) : dev::short_form(pv, a);
    }
    if (!starts.empty()) {
      dev::Plan plan = device_plan(s.d_plan, starts.size(), lrecs != nullptr, n_long, tp);
      dev::BatchView bv{dcodes, doffs, cn};
      const dev::ProblemView tpv = tile_view(cp.max_l2, tp);  // the plan's image: whole / windowed, widened
      dev::launch_tiles(tpv, bv, plan, s.d_out, static_cast<int>(fmt), s_compute_);
      stats_.kernels |= tp.tile16 ? 8 : 4;
      stats_.forms |= dev::tile_form(tpv);
    }
    MOC_HIP_CHECK(hipGetLastError());
    MOC_HIP_CHECK(hipEventRecord(s.ev_k1, s_compute_));
    // ---- return stream: D2H straight into the caller's result array
    MOC_HIP_CHECK(hipStreamWaitEvent(s_back, s.ev_k1, 0));
    copy_d2h(static_cast<char*>(out) + rb * fb, s.d_out, static_cast<size_t>(fb) * cn, s_back);
    MOC_HIP_CHECK(hipEventRecord(s.ev_done, s_back));
    stats_.d2h_bytes += static_cast<int64_t>(fb) * cn;
    s.busy = true;
    rb = re;
  }
  for (auto& s : slots_) retire(*s);
  stats_.kernel_ms = kernel_ms;
  stats_.chunks = chunk;
}

double HipEngine::device_kernel_ms() {
  if (!ev_d1_) return 0;
  MOC_HIP_CHECK(hipEventSynchronize(ev_d1_));
  float ms = 0;
  MOC_HIP_CHECK(hipEventElapsedTime(&ms, ev_d0_, ev_d1_));
  return ms;
}

void HipEngine::solve_device(const uint8_t* d_codes, const int64_t* d_offsets, const int64_t* h_offsets, int64_t n,
                             Result* d_out, hipStream_t stream) {
  if (!have_problem_) throw Error("HipEngine::solve_device before set_problem");
  finish_wire();
  MOC_HIP_CHECK(hipSetDevice(device_));
  if (n <= 0) return;
  if (!stream) stream = s_compute_;
  TraceRange tr("moc.solve_device");
  ChunkPlan cp;
  plan_chunk(h_offsets, n, cp);
  dev::ShortArgs a;
  a.fmt = static_cast<int32_t>(ResultFormat::R12);
  const bool swipe = cp.n_short > 0 && cp.long_recs.empty() &&
                     dev::configure_swipe(L1_, cp.min_short, cp.max_l2, table_.max_abs(), a, true, sem_ == Semantics::Spec);
  bool short_ok = swipe || (cp.n_short > 0 && dev::configure_short(L1_, cp.min_short, cp.max_l2, a));
  const bool all_tiles = cp.n_short > 0 && !short_ok;  // everything through the tile kernel
  const int32_t* lrecs = all_tiles ? nullptr : cp.long_recs.data();
  const int64_t n_long = all_tiles ? n : static_cast<int64_t>(cp.long_recs.size());
  TilePlan tp;
  const std::vector<dev::WaveStart> starts = plan_waves(h_offsets, lrecs, n_long, 0, 1, tp);
  const PlanLayout lay(starts.size(), lrecs ? static_cast<size_t>(n_long) : 0);
  const size_t keys_extra = lrecs ? 0 : sizeof(unsigned long long) * static_cast<size_t>(n_long);
  MOC_HIP_CHECK(hipEventSynchronize(ev_plan_));  // previous call's plan buffers are free again
  if (!starts.empty()) {
    ensure(d_plan_, d_plan_cap_, lay.total + keys_extra);
    ensure_host(h_plan_, h_plan_cap_, std::max<size_t>(lay.upload_bytes, 8));
    std::memcpy(static_cast<char*>(h_plan_) + lay.starts_off, starts.data(), starts.size() * sizeof(dev::WaveStart));
    if (lrecs)
      std::memcpy(static_cast<char*>(h_plan_) + lay.long_off, lrecs, static_cast<size_t>(n_long) * sizeof(int32_t));
    upload_staged(d_plan_, h_plan_, lay.upload_bytes, stream);
  }
  const dev::ProblemView pv = problem_view(cp.max_l2);
  if (!ev_d0_) {
    MOC_HIP_CHECK(hipEventCreate(&ev_d0_));
    MOC_HIP_CHECK(hipEventCreate(&ev_d1_));
  }
  MOC_HIP_CHECK(hipEventRecord(ev_d0_, stream));
  if (short_ok) {
    a.codes = d_codes;
    a.offsets = d_offsets;
    a.n = n;
    a.out = d_out;
    a.counter = d_counter_;
    a.lane_direct = swipe && lane_direct_enabled() ? 1 : 0;
    if (swipe)
      dev::launch_swipe(pv, a, num_cus_, stream);
    else
      dev::launch_short(pv, a, num_cus_, stream);
  }
  if (!starts.empty()) {
    dev::Plan plan = device_plan(d_plan_, starts.size(), lrecs != nullptr, n_long, tp);
    dev::BatchView bv{d_codes + h_offsets[0], d_offsets, n};
    dev::launch_tiles(tile_view(cp.max_l2, tp), bv, plan, d_out, static_cast<int>(ResultFormat::R12), stream);
  }
  MOC_HIP_CHECK(hipGetLastError());
  MOC_HIP_CHECK(hipEventRecord(ev_d1_, stream));
  MOC_HIP_CHECK(hipEventRecord(ev_plan_, stream));
  stats_ = EngineStats{};
  stats_.cells = cp.cells;
  stats_.records = n;
  stats_.kernels = (short_ok ? (swipe ? 1 : 2) : 0) | (starts.empty() ? 0 : (tp.tile16 ? 8 : 4));
  stats_.forms = (short_ok ? (swipe ? dev::swipe_launch_form(a) : dev::short_form(pv, a)) : 0) |
                 (starts.empty() ? 0 : dev::tile_form(tile_view(cp.max_l2, tp)));
}

}  // namespace moc

namespace moc {

void HipEngine::search_keys_device(const uint8_t* d_codes, const int64_t* d_offsets, const int64_t* h_offsets,
                                   int64_t n, int part, int parts, unsigned long long* d_keys, hipStream_t stream) {
  finish_wire();
  if (!have_problem_) throw Error("HipEngine::search_keys before set_problem");
  if (parts < 1 || part < 0 || part >= parts) throw Error("search_keys: bad part");
  MOC_HIP_CHECK(hipSetDevice(device_));
  if (n <= 0) return;
  if (!stream) stream = s_compute_;
  TraceRange tr("moc.search_keys");
  int64_t max_l2 = 0;
  for (int64_t i = 0; i < n; ++i) max_l2 = std::max(max_l2, h_offsets[i + 1] - h_offsets[i]);
  if (max_l2 >= (int64_t{1} << 30)) throw Error("Seq2 lengths beyond 2^30 exceed the device engine's offset range");
  // the record-major tile list of all records; this part takes a contiguous, cost-balanced share of it
  TilePlan tp;
  const std::vector<dev::WaveStart> starts = plan_waves(h_offsets, nullptr, n, part, parts, tp);
  MOC_HIP_CHECK(hipEventSynchronize(ev_plan_));  // previous call's plan buffers are free again
  const size_t bytes = std::max<size_t>(starts.size() * sizeof(dev::WaveStart), 8);
  ensure(d_plan_, d_plan_cap_, bytes);
  ensure_host(h_plan_, h_plan_cap_, bytes);
  if (!starts.empty()) {
    std::memcpy(h_plan_, starts.data(), starts.size() * sizeof(dev::WaveStart));
    upload_staged(d_plan_, h_plan_, starts.size() * sizeof(dev::WaveStart), stream);
  }
  dev::Plan plan;
  plan.u = tp.u;
  plan.win_tiles = tp.win_tiles;
  plan.n_waves = starts.empty() ? 0
                 : tp.slide   ? tp.slide_wgs * dev::kTile16WavesPerBlock
                              : static_cast<int64_t>(starts.size()) - 1;
  plan.slide_items = tp.slide_items;
  plan.slide_members = tp.slide_members;
  plan.starts = static_cast<const dev::WaveStart*>(d_plan_);
  plan.long_recs = nullptr;
  plan.n_long = n;
  plan.keys = d_keys;
  dev::BatchView bv{d_codes + h_offsets[0], d_offsets, n};
  dev::launch_tile_keys(tile_view(max_l2, tp), bv, plan, stream);
  MOC_HIP_CHECK(hipGetLastError());
  MOC_HIP_CHECK(hipEventRecord(ev_plan_, stream));
  stats_ = EngineStats{};
  stats_.records = n;
  stats_.kernels = plan.n_waves ? (tp.tile16 ? 8 : 4) : 0;
  stats_.forms = plan.n_waves ? dev::tile_form(tile_view(max_l2, tp)) : 0;
}

void HipEngine::finalize_keys_device(const uint8_t* d_codes, const int64_t* d_offsets, const int64_t* h_offsets,
                                     int64_t n, const unsigned long long* d_keys, void* d_out, ResultFormat fmt,
                                     hipStream_t stream) {
  finish_wire();
  MOC_HIP_CHECK(hipSetDevice(device_));
  if (n <= 0) return;
  if (!stream) stream = s_compute_;
  int64_t max_l2 = 0;
  for (int64_t i = 0; i < n; ++i) max_l2 = std::max(max_l2, h_offsets[i + 1] - h_offsets[i]);
  dev::Plan plan;
  plan.long_recs = nullptr;
  plan.n_long = n;
  plan.keys = const_cast<unsigned long long*>(d_keys);
  if (fmt == ResultFormat::R2) throw Error("finalize_keys_device: R2 needs the batch's parameters; use R4/R8/R12");
  dev::BatchView bv{d_codes + h_offsets[0], d_offsets, n};
  dev::launch_finalize_keys(problem_view(max_l2), bv, plan, d_out, static_cast<int>(fmt), stream);
  MOC_HIP_CHECK(hipGetLastError());
}

void HipEngine::search_keys(const uint8_t* codes, const int64_t* offsets, int64_t n, int part, int parts,
                            uint64_t* keys) {
  finish_wire();
  MOC_HIP_CHECK(hipSetDevice(device_));
  if (n <= 0) return;
  Stopwatch wall;
  wall.start();
  Slot& s = *slots_[0];
  const size_t cbytes = static_cast<size_t>(offsets[n] - offsets[0]);
  ensure(s.d_codes, s.d_codes_cap, std::max<size_t>(cbytes, 16) + 32);
  ensure(s.d_offsets, s.d_offsets_cap, sizeof(int64_t) * static_cast<size_t>(n + 1));
  ensure(s.d_out, s.d_out_cap, sizeof(uint64_t) * static_cast<size_t>(n));
  // offsets rebased to 0, so the device base pointer is the buffer itself (record i at d_codes + rebased[i])
  std::vector<int64_t> rebased(static_cast<size_t>(n) + 1);
  for (int64_t i = 0; i <= n; ++i) rebased[i] = offsets[i] - offsets[0];
  if (cbytes)
    copy_h2d(s.d_codes, codes + offsets[0], cbytes, s_compute_);
  MOC_HIP_CHECK(hipMemcpyAsync(s.d_offsets, rebased.data(), sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice,
                               s_compute_));
  MOC_HIP_CHECK(hipEventRecord(ev_a_, s_compute_));
  search_keys_device(static_cast<const uint8_t*>(s.d_codes), static_cast<const int64_t*>(s.d_offsets), rebased.data(),
                     n, part, parts, static_cast<unsigned long long*>(s.d_out), s_compute_);
  MOC_HIP_CHECK(hipEventRecord(ev_b_, s_compute_));
  copy_d2h(keys, s.d_out, sizeof(uint64_t) * n, s_compute_);
  MOC_HIP_CHECK(hipStreamSynchronize(s_compute_));
  float ms = 0;
  MOC_HIP_CHECK(hipEventElapsedTime(&ms, ev_a_, ev_b_));
  stats_.kernel_ms = ms;
  stats_.h2d_bytes = static_cast<int64_t>(cbytes + sizeof(int64_t) * (n + 1));
  stats_.d2h_bytes = static_cast<int64_t>(sizeof(uint64_t) * n);
  wall.stop();
  stats_.total_ms = wall.total_ms();
}

}  // namespace moc
