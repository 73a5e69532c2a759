// GPU side of `final` (plugin, see moc/gpu_rank.hpp): HIP engine per rank, and the rccl transport's device
// layer (moc/device_comm.hpp): RCCL over xGMI + the engine over device-resident wire batches. The batch
// driver itself (device_batch.cpp) is shared with the MPI-emulated device layer of CPU ranks.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <deque>
#include <exception>
#include <future>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "moc/comm.hpp"
#include "moc/device.hpp"
#include "moc/device_comm.hpp"
#include "moc/gpu_rank.hpp"
#include "moc/hip_engine.hpp"
#include "moc/rccl_comm.hpp"
#include "moc/runtime/device.hpp"
#include "moc/runtime/hip_check.hpp"
#include "moc/runtime/host_region.hpp"
#include "moc/runtime/kfd_topology.hpp"
#include "moc/runtime/log.hpp"
#include "moc/runtime/pinned.hpp"
#include "moc/runtime/timer.hpp"
#include "moc/runtime/watchdog.hpp"
#include "moc/score_table.hpp"
#include "moc/wire.hpp"

namespace moc {
namespace {

// RCCL over xGMI as the rccl transport's device layer: comm lane = the engine's compute stream (so the
// searches and the collectives are ordered without host waits), copy lane = a stream of its own.
//
// Every host wait polls (hipEventQuery / hipStreamQuery, ncclCommGetAsyncError every ~1 ms) against the job's
// comm deadline; past it the communicator is aborted and CommTimeout names the wait and the comm-lane
// transfers not yet known complete (moc/runtime/watchdog.hpp). The reference's ranks instead exit(1) or block
// forever (/root/reference/cudaFunctions.cu:15-33, main.c:174,195-197).
//
// Completion events are pooled: a ticket is a sequence number; an event goes back to the pool once it has
// completed (checked in ticket order at the next record), and a ticket whose event was recycled is known
// complete, so the pool is bounded by what is in flight (the pipelines' depth), not by the job's length
// (the reference allocated, and leaked, per record: cudaFunctions.cu:206).
class RcclDeviceComm final : public DeviceComm {
 public:
  RcclDeviceComm(const MpiContext& ctx, int device, hipStream_t comm_lane, const ncclUniqueId& id)
      : ctx_(ctx), device_(device), s_(comm_lane), nccl_(ctx, device, id) {
    nccl_.keep_until_exit();  // the rank's communicator: released by the process exit, not a 0.45 s destroy
    MOC_HIP_CHECK(hipStreamCreateWithFlags(&copy_, hipStreamNonBlocking));
  }
  ~RcclDeviceComm() override {
    if (std::uncaught_exceptions() == 0) (void)hipStreamSynchronize(copy_);
    for (const Live& l : live_) (void)hipEventDestroy(l.e);
    for (hipEvent_t e : free_) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(copy_);
  }
  int rank() const override { return ctx_.rank; }
  int size() const override { return ctx_.size; }
  const char* name() const override { return "rccl"; }
  void* dev_alloc(int64_t bytes) override {
    void* p = nullptr;
    MOC_HIP_CHECK(hipMalloc(&p, static_cast<size_t>(std::max<int64_t>(bytes, 16))));
    return p;
  }
  void dev_free(void* p) override { (void)hipFree(p); }
  // Page-locked staging. Large buffers are 2 MiB pages on the device's NUMA node, registered with the
  // runtime (the sliced path's registration rate, profiles/final_scale_1.1G_r3_stream.log pin_ms); small
  // ones come from hipHostMalloc.
  void* host_alloc(int64_t bytes) override {
    bytes = std::max<int64_t>(bytes, 16);
    if (bytes >= kBigHost) {
      Big b;
      b.region = HostRegion(static_cast<size_t>(bytes), device_numa_node(device_));
      b.region.prefault();
      b.bases = pinned::register_range(b.region.data(), static_cast<size_t>(bytes));
      void* p = b.region.data();
      big_.emplace(p, std::move(b));
      return p;
    }
    void* p = nullptr;
    MOC_HIP_CHECK(hipHostMalloc(&p, static_cast<size_t>(bytes), hipHostMallocDefault));
    return p;
  }
  void host_free(void* p) override {
    auto it = big_.find(p);
    if (it == big_.end()) {
      (void)hipHostFree(p);
      return;
    }
    pinned::unregister(it->second.bases);
    big_.erase(it);
  }
  int upload(void* d, const void* h, int64_t bytes) override {
    if (bytes > 0) MOC_HIP_CHECK(hipMemcpyAsync(d, h, static_cast<size_t>(bytes), hipMemcpyHostToDevice, copy_));
    return record(copy_);
  }
  void wait_upload(int ticket) override {
    if (hipEvent_t e = pending_event(ticket)) MOC_HIP_CHECK(hipStreamWaitEvent(s_, e, 0));
  }
  int upload_after(void* d, const void* h, int64_t bytes, int after) override {
    if (after >= 0)
      if (hipEvent_t e = pending_event(after)) MOC_HIP_CHECK(hipStreamWaitEvent(copy_, e, 0));
    return upload(d, h, bytes);
  }
  void wait_upload_host(int ticket) override { host_wait(ticket, "an upload to finish reading its staging buffer"); }
  void download(void* h, const void* d, int64_t bytes) override {
    if (bytes > 0) MOC_HIP_CHECK(hipMemcpyAsync(h, d, static_cast<size_t>(bytes), hipMemcpyDeviceToHost, s_));
    sync();
  }
  void group_start() override { nccl_.settle(ncclGroupStart(), "ncclGroupStart"); }
  void group_end() override { nccl_.settle(ncclGroupEnd(), "ncclGroupEnd"); }
  void send(const void* d, int64_t bytes, int peer) override {
    if (bytes <= 0) return;
    nccl_.settle(ncclSend(d, static_cast<size_t>(bytes), ncclUint8, peer, nccl_.comm(), s_), "ncclSend");
    ops_.push_back(Op{++op_seq_, peer, bytes, "send"});
  }
  void recv(void* d, int64_t bytes, int peer) override {
    if (bytes <= 0) return;
    nccl_.settle(ncclRecv(d, static_cast<size_t>(bytes), ncclUint8, peer, nccl_.comm(), s_), "ncclRecv");
    ops_.push_back(Op{++op_seq_, peer, bytes, "recv"});
  }
  void bcast(void* d, int64_t bytes, int root) override {
    nccl_.bcast(d, bytes, root, s_);
    if (bytes > 0) ops_.push_back(Op{++op_seq_, root, bytes, "bcast"});
  }
  void allgather(const void* d_send, void* d_recv, int64_t bytes_each) override {
    nccl_.allgather(d_send, d_recv, bytes_each, s_);
    if (bytes_each > 0) ops_.push_back(Op{++op_seq_, -1, bytes_each * ctx_.size, "allgather"});
  }
  void allreduce_max_u64(uint64_t* d, int64_t n) override {
    nccl_.allreduce_max_u64(d, n, s_);
    if (n > 0) ops_.push_back(Op{++op_seq_, -1, 8 * n, "allreduce"});
  }
  void sync() override {
    poll([this] { return query(hipStreamQuery(s_)); }, "the comm lane to drain");
    ops_.clear();  // everything queued on the lane is complete
  }
  int mark() override {
    const int t = record(s_);
    mark_ops_.emplace_back(t, op_seq_);
    return t;
  }
  void wait_mark(int m) override {
    host_wait(m, "a comm-lane point (a staging buffer's last send)");
    // the transfers queued before that point are complete
    uint64_t upto = 0;
    while (!mark_ops_.empty() && mark_ops_.front().first <= m) {
      upto = mark_ops_.front().second;
      mark_ops_.pop_front();
    }
    while (!ops_.empty() && ops_.front().seq <= upto) ops_.pop_front();
  }
  void inject_stall(double seconds) override {
    dev::launch_spin(seconds, s_);
    MOC_HIP_CHECK(hipGetLastError());
  }
  int64_t events_live() const override { return static_cast<int64_t>(live_.size() + free_.size()); }

 private:
  struct Live {
    int64_t ticket;
    hipEvent_t e;
  };
  struct Op {
    uint64_t seq;
    int peer;
    int64_t bytes;
    const char* kind;
  };
  static bool query(hipError_t r) {
    if (r == hipSuccess) return true;
    if (r != hipErrorNotReady) MOC_HIP_CHECK(r);
    return false;
  }
  // the ticket's event while it may still be pending; nullptr once it is known complete (recycled)
  hipEvent_t pending_event(int ticket) const {
    if (live_.empty() || ticket < live_.front().ticket) return nullptr;
    const size_t i = static_cast<size_t>(ticket - live_.front().ticket);
    if (i >= live_.size()) throw Error("RcclDeviceComm: unknown ticket " + std::to_string(ticket));
    return live_[i].e;
  }
  void host_wait(int ticket, const char* what) {
    if (hipEvent_t e = pending_event(ticket)) poll([e] { return query(hipEventQuery(e)); }, what);
  }
  template <typename Done>
  void poll(Done done, const char* what) {
    watchdog::WaitSpec spec;
    spec.what = what;
    spec.poll = watchdog::Poll::Backoff;
    spec.check = [this] { nccl_.check_async(); };
    spec.expire = [this] { nccl_.abort(); };
    spec.outstanding = [this] { return describe_ops(); };
    watchdog::wait(done, spec);
    nccl_.check_async();  // an error the communicator hit while the lane drained
  }
  std::string describe_ops() const {
    std::string o;
    size_t k = 0;
    for (const Op& op : ops_) {
      if (++k > 8) break;
      if (!o.empty()) o += ", ";
      o += std::string(op.kind) + " " + watchdog::human_bytes(op.bytes);
      if (op.peer >= 0)
        o += std::string(op.kind[0] == 's' ? " to" : op.kind[0] == 'r' ? " from" : " root") + " rank " +
             std::to_string(op.peer);
    }
    if (ops_.size() > 8) o += " (+" + std::to_string(ops_.size() - 8) + " more)";
    return o.empty() ? "no transfer queued (device work on the comm lane)" : "comm-lane transfers " + o;
  }
  int record(hipStream_t st) {
    // completed events (in ticket order) go back to the pool
    while (!live_.empty() && hipEventQuery(live_.front().e) == hipSuccess) {
      free_.push_back(live_.front().e);
      live_.pop_front();
    }
    hipEvent_t e = nullptr;
    if (free_.empty()) {
      MOC_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    } else {
      e = free_.back();
      free_.pop_back();
    }
    MOC_HIP_CHECK(hipEventRecord(e, st));
    live_.push_back(Live{next_ticket_, e});
    return static_cast<int>(next_ticket_++);
  }
  static constexpr int64_t kBigHost = int64_t{4} << 20;
  struct Big {
    HostRegion region;
    std::vector<void*> bases;
  };
  const MpiContext& ctx_;
  int device_;
  hipStream_t s_, copy_ = nullptr;
  RcclComm nccl_;
  std::deque<Live> live_;         // recorded, not yet seen complete (ticket order)
  std::vector<hipEvent_t> free_;  // completed, reusable
  int64_t next_ticket_ = 0;
  std::deque<Op> ops_;            // comm-lane transfers not yet known complete (for a timeout's message)
  uint64_t op_seq_ = 0;
  std::deque<std::pair<int, uint64_t>> mark_ops_;  // mark ticket -> the last transfer queued before it
  std::unordered_map<void*, Big> big_;
};

// The HIP engine over device-resident wire batches: the packed narrow form streams through the swipe
// kernel straight from device memory; the dense form is unpacked on the device and searched by the
// record/tile kernels (R12 results).
class HipDeviceSearch final : public DeviceSearch {
 public:
  explicit HipDeviceSearch(HipEngine& e) : e_(e) {}
  ~HipDeviceSearch() override { (void)hipFree(scratch_); }
  bool streams_packed(int64_t min_l2, int64_t max_l2) const override { return e_.streams_packed(min_l2, max_l2); }
  ResultFormat result_format(int64_t min_l2, int64_t max_l2, bool packed_form) const override {
    return packed_form ? e_.auto_format(max_l2, min_l2) : ResultFormat::R12;
  }
  void solve(const WireBatch& b, void* d_out, ResultFormat fmt) override {
    kernel_ms_ = 0;
    r2_ = R2Params{};
    if (b.off_shift) {
      e_.solve_wire(b, d_out, fmt);
      kernel_ms_ = e_.stats().kernel_ms;
      r2_ = e_.stats().r2;
      return;
    }
    if (fmt != ResultFormat::R12) throw Error("the dense device form returns R12 results");
    hipStream_t s = e_.compute_stream();
    std::vector<int64_t> h_offs(static_cast<size_t>(b.n) + 1);
    MOC_HIP_CHECK(hipMemcpyAsync(h_offs.data(), b.offsets, 8 * h_offs.size(), hipMemcpyDeviceToHost, s));
    MOC_HIP_CHECK(hipStreamSynchronize(s));
    const int64_t letters = h_offs[b.n] - h_offs[0];
    if (b.packed5) {
      if (static_cast<size_t>(letters) + 64 > scratch_cap_) {
        (void)hipFree(scratch_);
        scratch_cap_ = static_cast<size_t>(letters) + 64;
        MOC_HIP_CHECK(hipMalloc(&scratch_, scratch_cap_));
      }
      dev::launch_unpack5(b.letters, 5 * h_offs[0], letters, static_cast<uint8_t*>(scratch_), s);
      MOC_HIP_CHECK(hipGetLastError());
      // record i of the unpacked copy at scratch + offsets[i] - offsets[0]: offsets start at 0 here
      e_.solve_device(static_cast<const uint8_t*>(scratch_), b.offsets, h_offs.data(), b.n, static_cast<Result*>(d_out), s);
    } else {
      e_.solve_device(b.letters, b.offsets, h_offs.data(), b.n, static_cast<Result*>(d_out), s);
    }
    MOC_HIP_CHECK(hipStreamSynchronize(s));
  }
  void search_keys(const uint8_t* d_codes, const int64_t* d_offsets, const int64_t* h_offsets, int64_t n, int part,
                   int parts, uint64_t* d_keys) override {
    e_.search_keys_device(d_codes, d_offsets, h_offsets, n, part, parts, reinterpret_cast<unsigned long long*>(d_keys),
                          e_.compute_stream());
  }
  void finalize_keys(const uint8_t* d_codes, const int64_t* d_offsets, const int64_t* h_offsets, int64_t n,
                     const uint64_t* d_keys, Result* d_out) override {
    e_.finalize_keys_device(d_codes, d_offsets, h_offsets, n, reinterpret_cast<const unsigned long long*>(d_keys), d_out,
                            ResultFormat::R12, e_.compute_stream());
  }
  double last_kernel_ms() const override { return kernel_ms_; }
  R2Params last_r2() const override { return r2_; }

 private:
  HipEngine& e_;
  void* scratch_ = nullptr;
  size_t scratch_cap_ = 0;
  double kernel_ms_ = 0;
  R2Params r2_{};
};

// The HIP engine's construction (streams, events, device buffers, kernel code objects: 0.1-0.2 s on the
// MI355X box, tools/init_probe.cpp) runs on a helper thread started by the constructor, so it overlaps the
// rank's pass 1 and slice encoding; the first call that needs the engine waits for it. set_problem before
// that point is kept and applied when the engine is ready. When the driver's topology names the rank's
// GPU (moc/runtime/kfd_topology.hpp) the HIP runtime's own start-up (140-220 ms,
// profiles/hip_init_variants_box.log) moves onto that thread too: the device and its NUMA node come from
// sysfs, and the helper finds the same device in the runtime by its PCIe address.
class GpuRankImpl final : public GpuRank {
 public:
  GpuRankImpl(const MpiContext& ctx, const GpuRankOptions& opt) : ctx_(ctx) {
    log_set_level(opt.log_level);
    log_set_rank(ctx.rank);
    watchdog::set_timeout_s(opt.comm_timeout_s);  // this library's copy of the job's deadline
    int requested = opt.device;
    if (requested < 0 && !opt.device_map.empty())
      requested = opt.device_map[static_cast<size_t>(ctx.local_rank) % opt.device_map.size()];
    EngineOptions eo;
    if (opt.chunk_records > 0) eo.chunk_records = opt.chunk_records;
    if (opt.chunk_bytes > 0) eo.chunk_bytes = opt.chunk_bytes;
    eo.preload = opt.preload_kernels ? dev::kPreloadAll : 0u;
    std::string bus;  // the PCIe address of the device chosen from the topology
    if (const auto kfd = kfd_gpus(); kfd && !kfd->empty()) {
      const int id = kfd_pick(*kfd, ctx.local_rank, requested);
      if (id >= 0) {  // found again in the runtime by its PCIe address
        device_ = id;
        bus = (*kfd)[static_cast<size_t>(id)].pci_bus_id;
        // host buffers this rank's GPU streams over PCIe, and the threads that fill them, on the NUMA node
        // of the GPU's root complex (this, the calling thread)
        numa_ = bind_numa_node((*kfd)[static_cast<size_t>(id)].numa_node);
      }
    }
    if (device_ < 0) {  // the runtime's answer, on this thread
      device_ = select_device(ctx.local_rank, requested);
      numa_ = bind_numa_to_device(device_);
      bus.clear();
      runtime_up_.store(true);
    }
    eo.device = device_;
    const int local = ctx.local_rank;
    pending_engine_ = std::async(std::launch::async, [this, eo, bus, local, requested]() mutable {
      if (!bus.empty()) {
        // --device / --device-map name the runtime's index; otherwise the device the topology chose, found
        // by its PCIe address (the same GPU whatever order the runtime lists them in)
        int id = -1;
        const int n = device_count();  // the runtime's start-up (or the wait for the prewarm thread's)
        runtime_up_.store(true);
        if (requested < 0) {
          for (int i = 0; i < n && id < 0; ++i)
            if (device_info(i).pci_bus_id == bus) id = i;
        }
        if (id < 0) id = select_device(local, requested);
        if (id != eo.device) {
          MOC_LOG_INFO("device %s is the runtime's %d, the driver topology's %d: using %d", bus.c_str(), id, eo.device,
                       id);
          // the NUMA node was taken from the topology's device: take the one the runtime resolved, and let
          // the rank's main thread re-bind at its next device call (bind_thread)
          const int node = device_numa_node(id);
          if (node >= 0 && node != numa_.load()) {
            numa_.store(node);
            rebind_.store(true);
          }
        }
        eo.device = id;
        device_.store(id);
      }
      return std::make_unique<HipEngine>(eo);
    });
  }
  ~GpuRankImpl() override {
    ds_.reset();
    dc_.reset();
    if (pending_engine_.valid()) pending_engine_.wait();
  }
  void init_rccl_begin() override {
    if (dc_ || pending_.valid()) return;
    const ncclUniqueId id = RcclComm::exchange_id(ctx_);  // MPI: this (the main) thread
    pending_ = std::async(std::launch::async, [this, id] {
      HipEngine& e = engine();  // resolves the device first
      Stopwatch sw;
      sw.start();
      auto dc = std::make_unique<RcclDeviceComm>(ctx_, device_.load(), e.compute_stream(), id);
      sw.stop();
      rccl_init_ms_.store(sw.total_ms());
      return dc;
    });
  }
  void init_rccl() override {
    if (!dc_) {
      init_rccl_begin();
      Stopwatch sw;
      sw.start();
      dc_ = pending_.get();
      sw.stop();
      rccl_wait_ms_ = sw.total_ms();
    }
    if (!ds_) ds_ = std::make_unique<HipDeviceSearch>(engine());
  }
  DeviceComm& device_comm() override {
    init_rccl();
    bind_thread();
    return *dc_;
  }
  DeviceSearch& device_search() override {
    init_rccl();
    bind_thread();
    return *ds_;
  }
  int device() const override { return device_.load(); }
  double rccl_init_ms() const override { return rccl_init_ms_.load(); }
  double rccl_wait_ms() const override { return rccl_wait_ms_; }
  void set_problem(const Weights& w, const uint8_t* seq1, int64_t L1, Semantics sem) override {
    std::lock_guard<std::mutex> lock(mu_);
    facts_ = ProblemFacts::of(w, L1);
    if (engine_) {
      engine_->set_problem(w, seq1, L1, sem);
      return;
    }
    problem_ = Problem{w, std::vector<uint8_t>(seq1, seq1 + L1), sem, true};
  }
  void solve(const uint8_t* codes, const int64_t* offsets, int64_t n, Result* out) override {
    engine().solve(codes, offsets, n, out);
  }
  void search_keys(const uint8_t* codes, const int64_t* offsets, int64_t n, int part, int parts,
                   uint64_t* keys) override {
    engine().search_keys(codes, offsets, n, part, parts, keys);
  }
  double last_kernel_ms() const override { return engine().stats().kernel_ms; }
  int numa_node() const override { return numa_.load(); }
  bool runtime_ready() const override { return runtime_up_.load(); }
  void solve_wire(const WireBatch& b, void* out, ResultFormat fmt) override { engine().solve_wire(b, out, fmt); }
  void begin_wire(const WireBatch& b, void* out, ResultFormat fmt) override { engine().begin_wire(b, out, fmt); }
  GpuSolveStats finish_wire() override {
    engine().finish_wire();
    return last_stats();
  }
  // answered from the problem alone (the engine's own rules, dev::configure_swipe / r2_params /
  // pick_result_format), so the encode does not wait for the engine's start-up
  bool streams_packed(int64_t min_l2, int64_t max_l2) const override {
    const ProblemFacts f = facts();
    if (!f.set) return engine().streams_packed(min_l2, max_l2);
    dev::ShortArgs a;
    a.packed33 = 1;  // the widest LDS layout of the letter forms (HipEngine::streams_packed)
    return dev::configure_swipe(f.L1, min_l2, max_l2, f.max_abs, a);
  }
  ResultFormat result_format(int64_t min_l2, int64_t max_l2) const override {
    const ProblemFacts f = facts();
    if (!f.set) return engine().auto_format(max_l2, min_l2);
    R2Params r2;
    if (min_l2 > 0 && r2_params(f.L1, min_l2, max_l2, f.min_t, f.max_t, r2)) return ResultFormat::R2;
    return pick_result_format(f.L1, max_l2, f.max_abs);
  }
  GpuSolveStats last_stats() const override {
    const EngineStats& st = engine().stats();
    GpuSolveStats g;
    g.kernel_ms = st.kernel_ms;
    g.h2d_bytes = st.h2d_bytes;
    g.d2h_bytes = st.d2h_bytes;
    g.kernels = st.kernels;
    g.direct = st.direct;
    g.r2 = st.r2;
    return g;
  }
  // Page-locking needs the HIP runtime, not the engine: a rank registers its buffers while the engine's
  // streams and buffers are still being made. The registrations are this rank's until detached.
  void pin(const void* p, size_t bytes) override {
    bind_thread();  // waits for the runtime's start-up (on the helper thread since process start)
    const std::vector<void*> made = pinned::register_range(p, bytes);
    std::lock_guard<std::mutex> lock(pin_mu_);
    pins_.insert(pins_.end(), made.begin(), made.end());
  }
  void unpin_all() override {
    quiesce();
    std::lock_guard<std::mutex> lock(pin_mu_);
    pinned::unregister(pins_);
    pins_.clear();
  }
  std::function<void()> detach_pins() override {
    quiesce();  // no kernel in flight reads them any more
    std::shared_ptr<std::vector<void*>> regs;
    {
      std::lock_guard<std::mutex> lock(pin_mu_);
      regs = std::make_shared<std::vector<void*>>(std::exchange(pins_, {}));
    }
    const int dev = device_.load();
    return [regs, dev] {
      (void)hipSetDevice(dev);
      pinned::unregister(*regs);
    };
  }

 private:
  // What the engine's format rules read from a problem: Seq1's length and the score table's range.
  struct ProblemFacts {
    int64_t L1 = 0;
    int32_t max_abs = 0, min_t = 0, max_t = 0;
    bool set = false;
    static ProblemFacts of(const Weights& w, int64_t L1) {
      ProblemFacts f;
      const ScoreTable t = ScoreTable::build(w);
      f.L1 = L1;
      f.max_abs = t.max_abs();
      f.min_t = INT32_MAX;
      f.max_t = INT32_MIN;
      for (int x = 1; x < kAlphabet; ++x)  // HipEngine::set_problem's min_t_ / max_t_
        for (int y = 1; y < kAlphabet; ++y) {
          f.min_t = std::min(f.min_t, t.lut[x * kLutStride + y]);
          f.max_t = std::max(f.max_t, t.lut[x * kLutStride + y]);
        }
      f.set = true;
      return f;
    }
  };
  ProblemFacts facts() const {
    std::lock_guard<std::mutex> lock(mu_);
    return facts_;
  }
  // the engine's wire kernel finished (when there is an engine: none started one before it was up)
  void quiesce() const {
    if (engine_up_.load()) engine().finish_wire();
  }

  struct Problem {
    Weights w{};
    std::vector<uint8_t> seq1;
    Semantics sem = Semantics::Reference;
    bool set = false;
  };
  // the engine, once its construction has finished (any thread; the first caller applies a kept problem)
  HipEngine& engine() const {
    std::call_once(ready_, [this] {
      std::unique_ptr<HipEngine> e;
      try {
        e = pending_engine_.get();  // rethrows a construction error: kept for every caller
      } catch (const std::exception& ex) {
        start_error_ = ex.what();
        return;
      }
      std::lock_guard<std::mutex> lock(mu_);
      if (problem_.set) e->set_problem(problem_.w, problem_.seq1.data(), static_cast<int64_t>(problem_.seq1.size()),
                                       problem_.sem);
      problem_ = Problem{};
      engine_ = std::move(e);
      engine_up_.store(true);
    });
    if (!engine_) throw Error("the HIP engine failed to start: " + start_error_);
    bind_thread();
    return *engine_;
  }

  // the calling thread's current HIP device = this rank's (the runtime keeps one per thread; the engine
  // may have started on another thread)
  void bind_thread() const {
    if (rebind_.load() && std::this_thread::get_id() == main_thread_ && rebind_.exchange(false))
      (void)bind_numa_node(numa_.load());
    thread_local int current = -1;
    const int d = device_.load();
    if (current != d) {
      MOC_HIP_CHECK(hipSetDevice(d));
      current = d;
    }
  }

  const MpiContext& ctx_;
  std::atomic<int> device_{-1};
  std::atomic<int> numa_{-1};
  mutable std::atomic<bool> rebind_{false};  // numa_ changed after the main thread was bound to the old node
  const std::thread::id main_thread_ = std::this_thread::get_id();
  mutable std::future<std::unique_ptr<HipEngine>> pending_engine_;
  mutable std::once_flag ready_;
  mutable std::mutex mu_;
  mutable Problem problem_;
  mutable std::unique_ptr<HipEngine> engine_;
  mutable std::string start_error_;
  std::atomic<bool> runtime_up_{false};
  mutable std::atomic<bool> engine_up_{false};  // engine_ is set (kernels can only run after that)
  ProblemFacts facts_;  // under mu_
  std::mutex pin_mu_;
  std::vector<void*> pins_;  // this rank's page-locked ranges (pinned registry bases)
  std::unique_ptr<DeviceSearch> ds_;  // destroyed after dc_ (declared before it)
  std::unique_ptr<DeviceComm> dc_;
  std::future<std::unique_ptr<RcclDeviceComm>> pending_;  // connect in flight (init_rccl_begin)
  std::atomic<double> rccl_init_ms_{0.0};                 // the connect, on its helper thread
  double rccl_wait_ms_ = 0;                               // init_rccl's wait for it
};

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
int moc_final_gpu_rccl_warmup(int device) {
  try {
    return moc::rccl_warmup(device) ? 0 : 1;
  } catch (...) {
    return 1;
  }
}
}
