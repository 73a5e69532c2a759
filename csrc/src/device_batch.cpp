// device_batch (moc/device_comm.hpp): the rccl transport's batch — slices packed into wire formats and
// pipelined to the ranks' devices, device-resident search, narrow results gathered; or the
// context-parallel broadcast + MAX all-reduce of packed keys.
#include <omp.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <thread>

#include "moc/device_comm.hpp"
#include "moc/io.hpp"
#include "moc/runtime/timer.hpp"

namespace moc {

namespace {

// send/recv pieces: the pipeline's xGMI stage (MOC_SEND_CHUNK overrides it, e.g. for tests of the
// multi-piece path on small batches)
int64_t send_chunk() {
  static const int64_t c = [] {
    const char* v = std::getenv("MOC_SEND_CHUNK");
    return v && std::atoll(v) > 0 ? static_cast<int64_t>(std::atoll(v)) : int64_t{64} << 20;
  }();
  return c;
}
inline int64_t al16(int64_t x) { return (x + 15) & ~int64_t{15}; }

// Per-rank plan, decided by the root (every rank runs the same engine type on the same problem, so the
// root's DeviceSearch answers for all of them) and broadcast through the device layer.
struct RankPlan {
  int64_t n = 0, first = 0, letters = 0, min_l2 = 0, max_l2 = 0;
  int64_t narrow = 0;  // 1: P33 letters + narrow lengths + sparse offsets; 0: 5-bit letters + dense offsets
  int64_t bits = 0, fmt = 0;
  int64_t off_letters = 0, off_offsets = 0, off_lengths = 0, block = 0;  // block layout (bytes)
};
static_assert(sizeof(RankPlan) == 12 * sizeof(int64_t), "plan table entries are int64");

void layout(RankPlan& pl) {
  pl.off_letters = 0;
  pl.off_offsets = al16(pl.narrow ? packed33_bytes(pl.letters) : packed5_bytes(pl.letters));
  const int64_t offs = pl.narrow ? sparse_count(pl.n, kSparseShift) : pl.n + 1;
  pl.off_lengths = pl.off_offsets + al16(8 * offs);
  pl.block = pl.off_lengths + (pl.narrow ? al16(narrow_lengths_bytes(pl.n, static_cast<int>(pl.bits))) : 0);
  if (pl.n == 0) pl.block = 0;
}

// A piece of a rank's block: bytes [b0, b1) of one region (0 letters, 1 offsets, 2 lengths).
struct Piece {
  int rank = 0, region = 0;
  int64_t b0 = 0, b1 = 0;
};

// The pieces of rank r's block: letter blocks and offsets in chunks of `chunk` bytes (a multiple of 33, 5
// and 16: P33 blocks, 5-bit groups and int64 entries never straddle two pieces), the narrow lengths whole.
std::vector<Piece> pieces_of(const RankPlan& pl, int r, int64_t chunk) {
  std::vector<Piece> v;
  if (pl.block == 0) return v;
  const int64_t lb = pl.narrow ? packed33_bytes(pl.letters) : packed5_bytes(pl.letters);
  for (int64_t b = 0; b < lb; b += chunk) v.push_back(Piece{r, 0, b, std::min(lb, b + chunk)});
  const int64_t ob = 8 * (pl.narrow ? sparse_count(pl.n, kSparseShift) : pl.n + 1);
  for (int64_t b = 0; b < ob; b += chunk) v.push_back(Piece{r, 1, pl.off_offsets + b, pl.off_offsets + std::min(ob, b + chunk)});
  if (pl.narrow) {
    const int64_t nb = narrow_lengths_bytes(pl.n, static_cast<int>(pl.bits));
    v.push_back(Piece{r, 2, pl.off_lengths, pl.off_lengths + nb});
  }
  return v;
}

// The text batch's pieces: its blocks are encoded whole before they move, so plain byte ranges of <= chunk.
std::vector<Piece> byte_pieces(const RankPlan& pl, int r, int64_t chunk) {
  std::vector<Piece> v;
  for (int64_t b = 0; b < pl.block; b += chunk) v.push_back(Piece{r, 0, b, std::min(pl.block, b + chunk)});
  return v;
}

// Root: piece `pc` of the plan's wire form of rank slice [first, first + n) of rb -> dst (host staging with
// 64 bytes of slack: the packers write a piece's read slack past its end).
void pack_piece(const RecordBatch& rb, const RankPlan& pl, const Piece& pc, char* dst) {
  const int64_t b = pl.first, c0 = rb.offsets[b];
  if (pc.region == 0) {
    const int64_t lb = pl.narrow ? packed33_bytes(pl.letters) : packed5_bytes(pl.letters);
    const bool last = pc.b1 == lb;
    const int64_t L0 = pl.narrow ? kP33Letters * (pc.b0 / kP33Bytes) : 8 * (pc.b0 / 5);
    const int64_t n = last ? pl.letters - L0 : (pl.narrow ? kP33Letters * ((pc.b1 - pc.b0) / kP33Bytes) : 8 * ((pc.b1 - pc.b0) / 5));
    if (pl.narrow)  // the streaming kernel's form: P33 letter fields
      pack33(rb.codes.data() + c0 + L0, n, reinterpret_cast<uint8_t*>(dst));
    else  // the record/tile kernels' form: unpacked on the device
      pack5(rb.codes.data() + c0 + L0, n, reinterpret_cast<uint8_t*>(dst));
    return;
  }
  if (pc.region == 1) {
    int64_t* offs = reinterpret_cast<int64_t*>(dst);
    const int64_t e0 = (pc.b0 - pl.off_offsets) / 8, e1 = (pc.b1 - pl.off_offsets) / 8;
    if (pl.narrow) {
      for (int64_t j = e0; j < e1; ++j) offs[j - e0] = rb.offsets[b + std::min(j << kSparseShift, pl.n)] - c0;
    } else {
#pragma omp parallel for schedule(static) if (e1 - e0 > 65536)
      for (int64_t i = e0; i < e1; ++i) offs[i - e0] = rb.offsets[b + i] - c0;
    }
    return;
  }
  pack_lengths(rb.offsets.data() + b, pl.n, static_cast<int>(pl.bits), pl.bits == 8 ? 0 : pl.min_l2,
               reinterpret_cast<uint8_t*>(dst));
}

WireBatch device_view(const RankPlan& pl, char* d_block) {
  WireBatch w;
  w.letters = reinterpret_cast<const uint8_t*>(d_block + pl.off_letters);
  w.packed33 = pl.narrow != 0;
  w.packed5 = pl.narrow == 0;
  w.offsets = reinterpret_cast<const int64_t*>(d_block + pl.off_offsets);
  w.off_shift = pl.narrow ? kSparseShift : 0;
  w.lengths = pl.narrow ? reinterpret_cast<const uint8_t*>(d_block + pl.off_lengths) : nullptr;
  w.len_bits = static_cast<int>(pl.narrow ? pl.bits : 8);
  w.len_base = pl.bits == 8 ? 0 : pl.min_l2;
  w.n = pl.n;
  w.min_l2 = pl.min_l2;
  w.max_l2 = pl.max_l2;
  w.device = true;
  return w;
}

// Device buffers of one batch, freed on scope exit (also when unwinding).
struct DevBufs {
  DeviceComm& dc;
  std::vector<void*> dev, host;
  explicit DevBufs(DeviceComm& c) : dc(c) {}
  template <typename T>
  T* d(int64_t bytes) {
    void* p = dc.dev_alloc(std::max<int64_t>(bytes, 16));
    dev.push_back(p);
    return static_cast<T*>(p);
  }
  char* h(int64_t bytes) {
    void* p = dc.host_alloc(std::max<int64_t>(bytes, 16));
    host.push_back(p);
    return static_cast<char*>(p);
  }
  ~DevBufs() {
    for (void* p : dev) dc.dev_free(p);
    for (void* p : host) dc.host_free(p);
  }
};

DeviceBatchOut batch_cp(DeviceComm& dc, DeviceSearch& ds, const RecordBatch* rb, int64_t n, int64_t total_chars,
                        const PhaseHooks& hooks) {
  DeviceBatchOut out;
  DevBufs bufs(dc);
  const int rank = dc.rank(), p = dc.size();
  hooks.begin("distribute");
  // the root uploads the batch once; the device layer broadcasts it; every rank needs a host copy of the
  // offsets for its tile planning
  uint8_t* d_codes = bufs.d<uint8_t>(total_chars + 16);
  int64_t* d_offs = bufs.d<int64_t>(8 * (n + 1));
  if (rank == 0) {
    dc.wait_upload(dc.upload(d_codes, rb->codes.data(), total_chars));
    dc.wait_upload(dc.upload(d_offs, rb->offsets.data(), 8 * (n + 1)));
  }
  dc.bcast(d_codes, total_chars, 0);
  dc.bcast(d_offs, 8 * (n + 1), 0);
  std::vector<int64_t> h_offs(static_cast<size_t>(n) + 1);
  dc.download(h_offs.data(), d_offs, 8 * (n + 1));
  hooks.end();
  hooks.begin("compute");
  Stopwatch sw;
  sw.start();
  uint64_t* d_keys = bufs.d<uint64_t>(8 * n);
  ds.search_keys(d_codes, d_offs, h_offs.data(), n, rank, p, d_keys);
  dc.sync();
  sw.stop();
  out.compute_ms = sw.total_ms();
  out.kernel_ms = ds.last_kernel_ms();
  hooks.end();
  hooks.begin("gather");
  dc.allreduce_max_u64(d_keys, n);
  if (rank == 0) {
    Result* d_res = bufs.d<Result>(12 * n);
    ds.finalize_keys(d_codes, d_offs, h_offs.data(), n, d_keys, d_res);
    out.storage.emplace_back(static_cast<size_t>(12 * n));
    dc.download(out.storage.back().data(), d_res, 12 * n);
    out.runs.push_back(ResultRun{out.storage.back().data(), ResultFormat::R12, R2Params{}, n});
  }
  dc.sync();
  hooks.end();
  return out;
}

}  // namespace

void DeviceComm::inject_stall(double seconds) {
  std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
}

DeviceScratch::~DeviceScratch() {
  for (Buf& b : dev_)
    if (b.p) dc_.dev_free(b.p);
  for (Buf& b : host_)
    if (b.p) dc_.host_free(b.p);
}

char* DeviceScratch::get(std::vector<Buf>& v, int slot, int64_t bytes, bool host) {
  if (static_cast<size_t>(slot) >= v.size()) v.resize(static_cast<size_t>(slot) + 1);
  Buf& b = v[static_cast<size_t>(slot)];
  bytes = std::max<int64_t>(bytes, 64);
  if (bytes > b.cap) {
    if (b.p) host ? dc_.host_free(b.p) : dc_.dev_free(b.p);
    b.p = nullptr;
    b.cap = 0;
    const int64_t cap = bytes + bytes / 8;
    b.p = host ? dc_.host_alloc(cap) : dc_.dev_alloc(cap);
    b.cap = cap;
  }
  return static_cast<char*>(b.p);
}

namespace {
enum Slot { kPlanBuf, kBlock, kOut, kR2, kMineR2, kGather, kStage0, kStageEnd = kStage0 + 3, kStatus = kStageEnd,
            kHostResults = 0, kHostStage0 = 1, kHostPlan = kHostStage0 + 3, kHostStatus,
            kHostBlock0, kHostResults1 = kHostBlock0 + 2 };
}  // namespace

namespace {
// ---- search this rank's slice on its device, then its narrow results -> root (+ each rank's R2
// parameters, 3 ints, through the device layer). `plan` is complete on the root; other ranks read `mine`.
// Bytes of every rank's narrow results, 16-aligned runs in rank order (the root's gather buffer).
int64_t results_bytes(const std::vector<RankPlan>& plan) {
  int64_t b = 0;
  for (const RankPlan& pl : plan) b += al16(result_bytes(static_cast<ResultFormat>(pl.fmt)) * pl.n);
  return b;
}

void solve_gather(DeviceComm& dc, DeviceSearch& ds, DeviceScratch& sc, const std::vector<RankPlan>& plan,
                  const RankPlan& mine, char* d_block, const PhaseHooks& hooks, DeviceBatchOut& out,
                  int host_results = kHostResults) {
  const int rank = dc.rank(), p = dc.size();
  hooks.begin("compute");
  Stopwatch sw;
  sw.start();
  const ResultFormat fmt = static_cast<ResultFormat>(mine.fmt);
  const int fb = result_bytes(fmt);
  char* d_out = sc.dev(kOut, fb * mine.n + 16);
  if (mine.n > 0) ds.solve(device_view(mine, d_block), d_out, fmt);
  dc.sync();
  sw.stop();
  out.compute_ms = sw.total_ms();
  out.kernel_ms = ds.last_kernel_ms();
  const R2Params r2 = ds.last_r2();
  hooks.end();

  hooks.begin("gather");
  std::vector<int64_t> rstart(static_cast<size_t>(p) + 1, 0);
  for (int r = 0; r < p; ++r) rstart[r + 1] = rstart[r] + al16(result_bytes(static_cast<ResultFormat>(plan[r].fmt)) * plan[r].n);
  std::vector<int64_t> r2v(static_cast<size_t>(3 * p), 0);
  char* d_r2 = sc.dev(kR2, 24 * p);
  {
    const int64_t mine_r2[3] = {r2.smin, r2.kw, r2.j};
    // every rank's parameters land at its slot of the root's table
    char* d_mine_r2 = sc.dev(kMineR2, 24);
    dc.wait_upload(dc.upload(d_mine_r2, mine_r2, 24));
    dc.group_start();
    if (rank == 0) {
      for (int r = 1; r < p; ++r) dc.recv(d_r2 + 24 * r, 24, r);
    } else {
      dc.send(d_mine_r2, 24, 0);
      out.sent_bytes += 24;
    }
    dc.group_end();
    if (rank == 0) {
      r2v[0] = r2.smin;
      r2v[1] = r2.kw;
      r2v[2] = r2.j;
    }
  }
  char* d_gather = rank == 0 ? sc.dev(kGather, rstart[p] + 16) : nullptr;
  dc.group_start();
  if (rank == 0) {
    for (int r = 1; r < p; ++r) {
      const int64_t bytes = result_bytes(static_cast<ResultFormat>(plan[r].fmt)) * plan[r].n;
      if (bytes > 0) dc.recv(d_gather + rstart[r], bytes, r);
    }
  } else if (fb * mine.n > 0) {
    dc.send(d_out, fb * mine.n, 0);
    out.sent_bytes += fb * mine.n;
  }
  dc.group_end();
  if (rank == 0) {
    char* h = sc.host(host_results, rstart[p] + 16);  // page-locked: the downloads are plain DMA
    if (p > 1) dc.download(r2v.data() + 3, d_r2 + 24, 24 * (p - 1));
    if (fb * mine.n > 0) dc.download(h, d_out, fb * mine.n);
    if (rstart[p] > rstart[1]) dc.download(h + rstart[1], d_gather + rstart[1], rstart[p] - rstart[1]);
    out.rank_records.resize(static_cast<size_t>(p));
    for (int r = 0; r < p; ++r) {
      ResultRun run;
      run.data = h + rstart[r];
      run.fmt = static_cast<ResultFormat>(plan[r].fmt);
      run.r2 = R2Params{static_cast<int32_t>(r2v[3 * r]), static_cast<int32_t>(r2v[3 * r + 1]),
                        static_cast<int32_t>(r2v[3 * r + 2])};
      run.n = plan[r].n;
      out.runs.push_back(run);
      out.rank_records[r] = plan[r].n;
    }
  }
  dc.sync();
  hooks.end();
}
}  // namespace

DeviceBatchOut device_batch(DeviceComm& dc, DeviceSearch& ds, const RecordBatch* rb, int64_t n, int64_t total_chars,
                            const std::vector<int64_t>& bounds, bool cp, const PhaseHooks& hooks,
                            DeviceScratch* scratch) {
  if (cp) return batch_cp(dc, ds, rb, n, total_chars, hooks);
  std::unique_ptr<DeviceScratch> own;
  if (!scratch) {
    own = std::make_unique<DeviceScratch>(dc);
    scratch = own.get();
  }
  DeviceScratch& sc = *scratch;
  DeviceBatchOut out;
  Stopwatch dist;  // root: first piece sent -> the last one delivered
  const int rank = dc.rank(), p = dc.size();

  // ---- plan (root) -> every rank, through the device layer
  hooks.begin("distribute");
  std::vector<RankPlan> plan(static_cast<size_t>(p));
  if (rank == 0) {
    for (int r = 0; r < p; ++r) {
      RankPlan& pl = plan[r];
      pl.first = bounds[r];
      pl.n = bounds[r + 1] - bounds[r];
      pl.letters = rb->offsets[bounds[r + 1]] - rb->offsets[bounds[r]];
      int64_t mn = INT64_MAX, mx = 0;
#pragma omp parallel for reduction(min : mn) reduction(max : mx) schedule(static) if (pl.n > 65536)
      for (int64_t i = bounds[r]; i < bounds[r + 1]; ++i) {
        const int64_t L = rb->offsets[i + 1] - rb->offsets[i];
        mn = std::min(mn, L);
        mx = std::max(mx, L);
      }
      pl.min_l2 = pl.n ? mn : 0;
      pl.max_l2 = mx;
      pl.narrow = pl.n > 0 && mx <= 255 && ds.streams_packed(mn, mx) ? 1 : 0;
      pl.bits = pl.narrow ? narrow_length_bits(mn, mx) : 0;
      pl.fmt = pl.n ? static_cast<int64_t>(ds.result_format(mn, mx, pl.narrow != 0)) : 0;
      layout(pl);
    }
  }
  {
    const int64_t bytes = static_cast<int64_t>(sizeof(RankPlan)) * p;
    char* d_plan = sc.dev(kPlanBuf, bytes);
    if (rank == 0) dc.wait_upload(dc.upload(d_plan, plan.data(), bytes));
    dc.bcast(d_plan, bytes, 0);
    dc.download(plan.data(), d_plan, bytes);
    if (rank == 0) {  // the plan table reaches every peer (counted like device_batch_text's per-peer plans)
      out.peer_bytes.assign(static_cast<size_t>(p), 0);
      for (int r = 1; r < p; ++r) out.peer_bytes[r] += bytes;
      out.sent_bytes += bytes * (p - 1);
    }
  }
  const RankPlan& mine = plan[rank];
  char* d_block = sc.dev(kBlock, mine.block + 16);

  // ---- root: pack piece i+1 (host threads) | upload piece i (copy lane) | send piece i-1 (comm lane).
  // Pieces go round-robin over the ranks (the root's own, uploaded straight into its block, among them), so
  // every rank's transfer starts at once and the root's slice is not the last to arrive.
  const int64_t chunk = std::max<int64_t>(2640, send_chunk() / 2640 * 2640);  // lcm(33, 5, 16) = 2640
  if (rank == 0) {
    std::vector<std::vector<Piece>> per(static_cast<size_t>(p));
    int64_t stage_bytes = 0;
    size_t rounds = 0;
    for (int r = 0; r < p; ++r) {
      per[r] = pieces_of(plan[r], r, chunk);
      rounds = std::max(rounds, per[r].size());
      for (const Piece& pc : per[r]) stage_bytes = std::max(stage_bytes, pc.b1 - pc.b0);
    }
    constexpr int kSlots = 3;
    char* stage[kSlots];
    char* d_stage[kSlots];
    int up[kSlots], sent[kSlots];
    for (int q = 0; q < kSlots; ++q) {
      stage[q] = sc.host(kHostStage0 + q, stage_bytes + 64);
      d_stage[q] = p > 1 ? sc.dev(kStage0 + q, stage_bytes + 64) : nullptr;
      up[q] = sent[q] = -1;
    }
    sc.host(kHostResults, results_bytes(plan) + 16);  // the gather's page-locked buffer, ahead of the search
    hooks.begin("pack");  // host packing, and the waits for staging slots (a packing-bound distribution)
    dist.start();
    int64_t i = 0;
    for (size_t k = 0; k < rounds; ++k)
      for (int step = 1; step <= p; ++step) {
        const int r = step % p;  // peers 1..p-1, then the root
        if (k >= per[r].size()) continue;
        const Piece& pc = per[r][k];
        const int q = static_cast<int>(i++ % kSlots);
        if (up[q] >= 0) dc.wait_upload_host(up[q]);  // the staging's previous piece has left the host
        pack_piece(*rb, plan[r], pc, stage[q]);
        const int64_t len = pc.b1 - pc.b0;
        if (r == 0) {
          up[q] = dc.upload_after(d_block + pc.b0, stage[q], len, -1);
          dc.wait_upload(up[q]);
          continue;
        }
        up[q] = dc.upload_after(d_stage[q], stage[q], len, sent[q]);  // after that buffer's last send
        dc.wait_upload(up[q]);
        dc.group_start();
        dc.send(d_stage[q], len, r);
        dc.group_end();
        sent[q] = dc.mark();
        out.scattered_bytes += len;
        out.peer_bytes[r] += len;
      }
    hooks.begin("distribute");
  } else {
    for (const Piece& pc : pieces_of(mine, rank, chunk)) {  // the root's order of this rank's pieces
      dc.group_start();
      dc.recv(d_block + pc.b0, pc.b1 - pc.b0, 0);
      dc.group_end();
    }
  }
  dc.sync();
  if (rank == 0) {
    dist.stop();
    out.distribute_ms = dist.total_ms();
    out.sent_bytes += out.scattered_bytes;
  }
  hooks.end();

  solve_gather(dc, ds, sc, plan, mine, d_block, hooks, out);
  return out;
}

// ---- text batch: the root encodes every rank's slice straight from the input text into that rank's wire
// block (page-locked, two blocks in turn), its own first, then the peers'; a block's pieces upload and leave
// over the comm lane while the next rank's slice is encoded. Each peer learns its plan from a 96-byte
// message ahead of its pieces (the plan depends on the slice's length range, known after its encode).
DeviceBatchOut device_batch_text(DeviceComm& dc, DeviceSearch& ds, const BulkParser* parser,
                                 const std::vector<int64_t>& bounds, const PhaseHooks& hooks, DeviceScratch* scratch,
                                 int64_t record_base, int results_slot) {
  const int host_results = results_slot ? kHostResults1 : kHostResults;
  std::unique_ptr<DeviceScratch> own;
  if (!scratch) {
    own = std::make_unique<DeviceScratch>(dc);
    scratch = own.get();
  }
  DeviceScratch& sc = *scratch;
  DeviceBatchOut out;
  Stopwatch dist;  // root: first piece sent -> the last one delivered
  const int rank = dc.rank(), p = dc.size();
  constexpr int64_t kPlanBytes = static_cast<int64_t>(sizeof(RankPlan));
  const int64_t chunk = std::max<int64_t>(2640, send_chunk() / 2640 * 2640);
  std::vector<RankPlan> plan(static_cast<size_t>(p));
  char* d_block = nullptr;
  char* d_status = sc.dev(kStatus, 16);
  int64_t status = 0;
  if (rank == 0) {
    hooks.begin("fill");  // encode (host threads), and the waits for a block to be free again
    out.peer_bytes.assign(static_cast<size_t>(p), 0);
    const int64_t L1 = static_cast<int64_t>(parser->seq1().size());
    char* d_plan = sc.dev(kPlanBuf, kPlanBytes * p);
    RankPlan* h_plan = reinterpret_cast<RankPlan*>(sc.host(kHostPlan, kPlanBytes * p));
    // every slice's extent first (cheap: pass 1's chunk table): staging and host blocks at their final size
    std::vector<AreaSlice> slices(static_cast<size_t>(p));
    // a block's size in the narrow form (P33 + sparse offsets + lengths) or the dense one (5-bit + offsets)
    auto wire_cap = [](const AreaSlice& sl, bool narrow) {
      const int64_t n = sl.records;
      return narrow ? al16(packed33_bytes(sl.letters)) + al16(8 * sparse_count(n, kSparseShift)) + al16(n + 16) + 64
                    : al16(packed5_bytes(sl.letters)) + al16(8 * (n + 1)) + 64;
    };
    // the narrow form when the mean length says it can hold the slice (checked against the slice's range)
    auto guess_narrow = [L1](const AreaSlice& sl) { return sl.records > 0 && L1 <= 200 && sl.letters <= 64 * sl.records; };
    int64_t block_cap = 64, stage_bytes = 64;
    for (int r = 0; r < p; ++r) {
      slices[r] = parser->slice(bounds[r], bounds[r + 1]);
      const int64_t cap = wire_cap(slices[r], guess_narrow(slices[r]));
      block_cap = std::max(block_cap, cap);
      if (r != 0) stage_bytes = std::max(stage_bytes, std::min(chunk, std::max(cap, wire_cap(slices[r], false))));
    }
    constexpr int kSlots = 3;
    char* d_stage[kSlots];
    int sent[kSlots] = {-1, -1, -1};
    for (int q = 0; q < kSlots; ++q) d_stage[q] = p > 1 ? sc.dev(kStage0 + q, stage_bytes + 64) : nullptr;
    int block_up[2] = {-1, -1};  // the last upload out of each host block
    int own_up = -1;
    int64_t qi = 0;
    FillReport whole;
    uvector<uint16_t> len16;
    for (int k = 0; k < p; ++k) {
      // the root's own slice first: its block uploads (copy lane) while the peers' slices are encoded and
      // sent, so the root's search waits for no encode or upload of its own once the last piece is out
      // (before: peers first, the root's slice encoded and uploaded after all of them, the critical path)
      const int r = k;
      out.fill_order.push_back(r);
      const int hb = k % 2;
      if (block_up[hb] >= 0) dc.wait_upload_host(block_up[hb]);
      const AreaSlice& sl = slices[r];
      RankPlan& pl = plan[r];
      pl.first = bounds[r];
      pl.n = sl.records;
      pl.letters = sl.letters;
      const int64_t n = pl.n;
      char* h = sc.host(kHostBlock0 + hb, block_cap);
      FillReport rep;
      if (n > 0) {
        pl.narrow = guess_narrow(sl) ? 1 : 0;
        if (pl.narrow) {
          layout(pl);
          if (static_cast<int64_t>(len16.size()) < n) len16 = uvector<uint16_t>(static_cast<size_t>(n));
          rep = parser->fill_slice(sl, nullptr, reinterpret_cast<uint8_t*>(h), nullptr,
                                   reinterpret_cast<int64_t*>(h + pl.off_offsets), len16.data(), 33);
          if (!(rep.max_len <= 255 && ds.streams_packed(rep.min_len, rep.max_len))) pl.narrow = 0;
        }
        if (!pl.narrow) {
          layout(pl);
          h = sc.host(kHostBlock0 + hb, std::max(block_cap, wire_cap(sl, false)));  // grows when it must
          rep = parser->fill_slice(sl, nullptr, reinterpret_cast<uint8_t*>(h),
                                   reinterpret_cast<int64_t*>(h + pl.off_offsets), nullptr, nullptr, 5);
        }
        pl.min_l2 = rep.min_len;
        pl.max_l2 = rep.max_len;
        pl.bits = pl.narrow ? narrow_length_bits(rep.min_len, rep.max_len) : 0;
        layout(pl);
        if (pl.narrow)
          pack_lengths16(len16.data(), n, static_cast<int>(pl.bits), pl.bits == 8 ? 0 : pl.min_l2,
                         reinterpret_cast<uint8_t*>(h + pl.off_lengths));
        pl.fmt = static_cast<int64_t>(ds.result_format(rep.min_len, rep.max_len, pl.narrow != 0));
      } else {
        layout(pl);
      }
      whole.min_len = std::min(whole.min_len, rep.min_len);
      whole.max_len = std::max(whole.max_len, rep.max_len);
      if (rep.bad_record >= 0 && (whole.bad_record < 0 || rep.bad_record < whole.bad_record)) whole.bad_record = rep.bad_record;
      if (rep.long_record >= 0 && (whole.long_record < 0 || rep.long_record < whole.long_record)) {
        whole.long_record = rep.long_record;
        whole.long_len = rep.long_len;
      }
      whole.cells += rep.cells;
      out.letters += sl.letters;
      int last = -1;
      if (r != 0) {
        h_plan[r] = pl;
        // the distribution time runs from the first byte on the wire (the first slice's encode is before it)
        if (r == 1) dist.start();
        const int t = dc.upload(d_plan + kPlanBytes * r, h_plan + r, kPlanBytes);
        dc.wait_upload(t);
        dc.group_start();
        dc.send(d_plan + kPlanBytes * r, kPlanBytes, r);
        dc.group_end();
        out.peer_bytes[r] += kPlanBytes;
        out.sent_bytes += kPlanBytes;
        for (const Piece& pc : byte_pieces(pl, r, chunk)) {
          const int q = static_cast<int>(qi++ % kSlots);
          const int64_t len = pc.b1 - pc.b0;
          last = dc.upload_after(d_stage[q], h + pc.b0, len, sent[q]);  // after that buffer's last send
          dc.wait_upload(last);
          dc.group_start();
          dc.send(d_stage[q], len, r);
          dc.group_end();
          sent[q] = dc.mark();
          out.scattered_bytes += len;
          out.peer_bytes[r] += len;
        }
      } else {
        d_block = sc.dev(kBlock, pl.block + 16);
        for (const Piece& pc : byte_pieces(pl, r, chunk)) last = dc.upload(d_block + pc.b0, h + pc.b0, pc.b1 - pc.b0);
        own_up = last;
      }
      block_up[hb] = last;
    }
    hooks.begin("distribute");
    sc.host(host_results, results_bytes(plan) + 16);  // the gather's page-locked buffer, while the blocks move
    if (own_up >= 0) dc.wait_upload(own_up);  // the root's search waits for its own block on the device
    if (whole.bad_record >= 0) whole.bad_record += record_base;
    if (whole.long_record >= 0) whole.long_record += record_base;
    try {
      parser->check(whole);
    } catch (const std::exception& e) {
      status = 1;
      out.error = e.what();
    }
    out.cells = whole.cells;
    int64_t* h_status = reinterpret_cast<int64_t*>(sc.host(kHostStatus, 16));
    h_status[0] = status;
    dc.wait_upload(dc.upload(d_status, h_status, 8));
  } else {
    hooks.begin("distribute");
    char* d_plan = sc.dev(kPlanBuf, kPlanBytes);
    dc.group_start();
    dc.recv(d_plan, kPlanBytes, 0);
    dc.group_end();
    dc.download(&plan[rank], d_plan, kPlanBytes);
    const RankPlan& mine = plan[rank];
    d_block = sc.dev(kBlock, mine.block + 16);
    for (const Piece& pc : byte_pieces(mine, rank, chunk)) {  // the root's order of this rank's pieces
      dc.group_start();
      dc.recv(d_block + pc.b0, pc.b1 - pc.b0, 0);
      dc.group_end();
    }
  }
  // the input's verdict (the error a sequential reader meets first) on every rank
  dc.bcast(d_status, 8, 0);
  dc.download(&status, d_status, 8);
  if (rank == 0) {
    dist.stop();  // the bcast is ordered after every piece on the comm lane: all of them have arrived
    out.distribute_ms = dist.total_ms();
    out.sent_bytes += out.scattered_bytes;
  }
  hooks.end();
  if (status != 0) {
    out.input_error = true;
    return out;
  }
  solve_gather(dc, ds, sc, plan, plan[rank], d_block, hooks, out, host_results);
  return out;
}

}  // namespace moc
