// GPU side of `final` (plugin, see moc/gpu_rank.hpp): HIP engine per rank, RCCL communicator, and the
// rccl transport's batch (root upload, grouped send/recv scatter over xGMI, gather of packed results; or
// in context-parallel mode a broadcast of the batch and a MAX all-reduce of packed keys).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <memory>
#include <vector>

#include "moc/comm.hpp"
#include "moc/gpu_rank.hpp"
#include "moc/hip_engine.hpp"
#include "moc/rccl_comm.hpp"
#include "moc/runtime/device.hpp"
#include "moc/runtime/hip_check.hpp"
#include "moc/runtime/log.hpp"
#include "moc/runtime/pinned.hpp"
#include "moc/runtime/timer.hpp"

namespace moc {
namespace {

class GpuRankImpl final : public GpuRank {
 public:
  GpuRankImpl(const MpiContext& ctx, const GpuRankOptions& opt) : ctx_(ctx) {
    log_set_level(opt.log_level);
    log_set_rank(ctx.rank);
    int requested = opt.device;
    if (requested < 0 && !opt.device_map.empty())
      requested = opt.device_map[static_cast<size_t>(ctx.local_rank) % opt.device_map.size()];
    device_ = select_device(ctx.local_rank, requested);
    EngineOptions eo;
    eo.device = device_;
    if (opt.chunk_records > 0) eo.chunk_records = opt.chunk_records;
    if (opt.chunk_bytes > 0) eo.chunk_bytes = opt.chunk_bytes;
    engine_ = std::make_unique<HipEngine>(eo);
    // host buffers this rank's GPU streams over PCIe, and the threads that fill them, on the NUMA node
    // of the GPU's root complex
    numa_ = bind_numa_to_device(device_);
  }
  void init_rccl() override {
    if (!nccl_) nccl_ = std::make_unique<RcclComm>(ctx_, device_);
  }
  int device() const override { return device_; }
  void set_problem(const Weights& w, const uint8_t* seq1, int64_t L1, Semantics sem) override {
    engine_->set_problem(w, seq1, L1, sem);
  }
  void solve(const uint8_t* codes, const int64_t* offsets, int64_t n, Result* out) override {
    engine_->solve(codes, offsets, n, out);
  }
  void search_keys(const uint8_t* codes, const int64_t* offsets, int64_t n, int part, int parts,
                   uint64_t* keys) override {
    engine_->search_keys(codes, offsets, n, part, parts, keys);
  }
  double last_kernel_ms() const override { return engine_->stats().kernel_ms; }
  int numa_node() const override { return numa_; }
  void solve_wire(const WireBatch& b, void* out, ResultFormat fmt) override { engine_->solve_wire(b, out, fmt); }
  bool streams_packed(int64_t min_l2, int64_t max_l2) const override {
    return engine_->streams_packed(min_l2, max_l2);
  }
  ResultFormat result_format(int64_t min_l2, int64_t max_l2) const override {
    return engine_->auto_format(max_l2, min_l2);
  }
  GpuSolveStats last_stats() const override {
    const EngineStats& st = engine_->stats();
    GpuSolveStats g;
    g.kernel_ms = st.kernel_ms;
    g.h2d_bytes = st.h2d_bytes;
    g.d2h_bytes = st.d2h_bytes;
    g.kernels = st.kernels;
    g.direct = st.direct;
    g.r2 = st.r2;
    return g;
  }
  void pin(const void* p, size_t bytes) override { engine_->pin(p, bytes); }
  void unpin_all() override { engine_->unpin_all(); }
  std::function<void()> detach_pins() override {
    auto regs = std::make_shared<std::vector<void*>>(engine_->detach_pins());
    const int dev = device_;
    return [regs, dev] {
      (void)hipSetDevice(dev);
      pinned::unregister(*regs);
    };
  }
  double rccl_batch(const RecordBatch* rb, int64_t n, int64_t total_chars, const std::vector<int64_t>& bounds, bool cp,
                    Result* out, const PhaseHooks& hooks) override;

 private:
  const MpiContext& ctx_;
  int device_ = -1;
  int numa_ = -1;
  std::unique_ptr<HipEngine> engine_;
  std::unique_ptr<RcclComm> nccl_;
};

// Device buffers of one rccl batch (freed on scope exit, also when unwinding).
struct DeviceBufs {
  std::vector<void*> ptrs;
  template <typename T>
  T* alloc(int64_t bytes) {
    void* p = nullptr;
    MOC_HIP_CHECK(hipMalloc(&p, static_cast<size_t>(std::max<int64_t>(bytes, 16))));
    ptrs.push_back(p);
    return static_cast<T*>(p);
  }
  ~DeviceBufs() {
    for (void* p : ptrs) (void)hipFree(p);
  }
};

double GpuRankImpl::rccl_batch(const RecordBatch* rb, int64_t n, int64_t total_chars,
                               const std::vector<int64_t>& bounds, bool cp, Result* out, const PhaseHooks& hooks) {
  if (!nccl_) throw Error("rccl_batch: the RCCL communicator was not created");
  RcclComm& nccl = *nccl_;
  hipStream_t s = engine_->compute_stream();
  double compute_ms = 0;
  const int p = ctx_.size;
  DeviceBufs bufs;
  hooks.begin("distribute");
  if (cp) {
    // root uploads the batch once; RCCL broadcasts it to every device over xGMI; each GPU searches its
    // share of every record's offset tiles; ncclAllReduce(MAX, uint64) combines the packed keys.
    uint8_t* d_codes = bufs.alloc<uint8_t>(total_chars);
    int64_t* d_offs = bufs.alloc<int64_t>(8 * (n + 1));
    std::vector<int64_t> h_offs(static_cast<size_t>(n) + 1);
    if (ctx_.rank == kRoot) {
      h_offs.assign(rb->offsets.begin(), rb->offsets.end());
      MOC_HIP_CHECK(hipMemcpyAsync(d_codes, rb->codes.data(), total_chars, hipMemcpyHostToDevice, s));
      MOC_HIP_CHECK(hipMemcpyAsync(d_offs, rb->offsets.data(), 8 * (n + 1), hipMemcpyHostToDevice, s));
    }
    nccl.bcast(d_codes, total_chars, kRoot, s);
    nccl.bcast(d_offs, 8 * (n + 1), kRoot, s);
    bcast_bytes(h_offs.data(), 8 * (n + 1), kRoot, ctx_.world);  // host copy for tile planning
    MOC_HIP_CHECK(hipStreamSynchronize(s));
    nccl.check_async();
    hooks.end();
    hooks.begin("compute");
    Stopwatch sw;
    sw.start();
    auto* d_keys = bufs.alloc<unsigned long long>(8 * n);
    engine_->search_keys_device(d_codes, d_offs, h_offs.data(), n, ctx_.rank, ctx_.size, d_keys, s);
    MOC_HIP_CHECK(hipStreamSynchronize(s));
    sw.stop();
    compute_ms += sw.total_ms();
    hooks.end();
    hooks.begin("gather");
    nccl.allreduce_max_u64(d_keys, n, s);
    if (ctx_.rank == kRoot) {
      auto* d_res = bufs.alloc<Result>(12 * n);
      engine_->finalize_keys_device(d_offs, n, d_keys, d_res, ResultFormat::R12, s);
      MOC_HIP_CHECK(hipMemcpyAsync(out, d_res, 12 * n, hipMemcpyDeviceToHost, s));
    }
    MOC_HIP_CHECK(hipStreamSynchronize(s));
    nccl.check_async();
    hooks.end();
    return compute_ms;
  }
  const int64_t my_b = bounds[ctx_.rank], my_n = bounds[ctx_.rank + 1] - my_b;
  // counts in bytes for codes and (absolute) offsets; each rank receives n_r+1 offsets
  std::vector<int64_t> ccount(p), cdispl(p), ocount(p), odispl(p);
  if (ctx_.rank == kRoot) {
    for (int r = 0; r < p; ++r) {
      ccount[r] = rb->offsets[bounds[r + 1]] - rb->offsets[bounds[r]];
      cdispl[r] = rb->offsets[bounds[r]];
    }
  }
  bcast_bytes(ccount.data(), 8 * p, kRoot, ctx_.world);
  bcast_bytes(cdispl.data(), 8 * p, kRoot, ctx_.world);
  for (int r = 0; r < p; ++r) {
    ocount[r] = 8 * (bounds[r + 1] - bounds[r] + 1);
    odispl[r] = 8 * bounds[r];
  }
  uint8_t* d_all_codes = nullptr;
  int64_t* d_all_offs = nullptr;
  Result* d_all_out = nullptr;
  if (ctx_.rank == kRoot) {
    d_all_codes = bufs.alloc<uint8_t>(total_chars);
    d_all_offs = bufs.alloc<int64_t>(8 * (n + 1));
    d_all_out = bufs.alloc<Result>(12 * n);
    MOC_HIP_CHECK(hipMemcpyAsync(d_all_codes, rb->codes.data(), total_chars, hipMemcpyHostToDevice, s));
    MOC_HIP_CHECK(hipMemcpyAsync(d_all_offs, rb->offsets.data(), 8 * (n + 1), hipMemcpyHostToDevice, s));
  }
  uint8_t* d_codes = bufs.alloc<uint8_t>(ccount[ctx_.rank]);
  int64_t* d_offs = bufs.alloc<int64_t>(8 * (my_n + 1));
  Result* d_out = bufs.alloc<Result>(12 * my_n);
  nccl.scatterv(d_all_codes, ccount, cdispl, d_codes, kRoot, s);
  nccl.scatterv(d_all_offs, ocount, odispl, d_offs, kRoot, s);
  std::vector<int64_t> h_offs(static_cast<size_t>(my_n) + 1);
  MOC_HIP_CHECK(hipMemcpyAsync(h_offs.data(), d_offs, 8 * (my_n + 1), hipMemcpyDeviceToHost, s));
  MOC_HIP_CHECK(hipStreamSynchronize(s));
  nccl.check_async();
  hooks.end();
  hooks.begin("compute");
  Stopwatch sw;
  sw.start();
  // d_codes holds this rank's letters starting at absolute offset h_offs[0]
  if (my_n > 0) engine_->solve_device(d_codes - h_offs[0], d_offs, h_offs.data(), my_n, d_out, s);
  MOC_HIP_CHECK(hipStreamSynchronize(s));
  sw.stop();
  compute_ms += sw.total_ms();
  hooks.end();
  hooks.begin("gather");
  std::vector<int64_t> rcount(p), rdispl(p);
  for (int r = 0; r < p; ++r) {
    rcount[r] = 12 * (bounds[r + 1] - bounds[r]);
    rdispl[r] = 12 * bounds[r];
  }
  nccl.gatherv(d_out, 12 * my_n, d_all_out, rcount, rdispl, kRoot, s);
  if (ctx_.rank == kRoot) {
    MOC_HIP_CHECK(hipMemcpyAsync(out, d_all_out, 12 * n, hipMemcpyDeviceToHost, s));
  }
  MOC_HIP_CHECK(hipStreamSynchronize(s));
  nccl.check_async();
  hooks.end();
  return compute_ms;
}

}  // namespace
}  // namespace moc

extern "C" {
int moc_final_gpu_device_count() {
  try {
    return moc::device_count();
  } catch (...) {
    return 0;
  }
}
moc::GpuRank* moc_final_gpu_create(const moc::MpiContext& ctx, const moc::GpuRankOptions& opt) {
  return new moc::GpuRankImpl(ctx, opt);
}
}
