// Streaming job on one node (`final --batch-records=B [--batch-chars=C]`, transport shm, record slices):
// the input is searched and printed in batches, with host memory bounded by the batch, through a
// software pipeline whose buffers are allocated and page-locked once.
//
// Reference: read everything, then one blocking scatter and one kernel launch per record
// (/root/reference/main.c:90-108,174; cudaFunctions.cu:201-218) — no overlap, memory O(input).
//
// Per batch b (every rank of the node):
//   A  root: cut batch b from the input text — pass 1 (token/letter counts) in parallel chunks, kept for
//      the next batch past the cut — and broadcast its chunk table (a few KB). The text is an --input file
//      mapped by every rank, or the root's stream buffer (copied into a node-shared slot when the node has
//      several ranks).
//   B  every rank encodes its cost-balanced slice of batch b straight from the text into its ring slot
//      b % 2: P33 letters + sparse offsets + narrow lengths in NUMA-local, page-locked memory (GPU ranks),
//      or byte letters + CSR offsets (CPU ranks). The slot is the kernel's zero-copy input: no copy, no
//      per-batch allocation, registration or unmap.
//   C  fill reports are all-gathered (first input error of the batch, on every rank; result-ring growth).
//   F  batch b-1's kernel is waited for and the ranks' result descriptors are all-gathered.
//   D  batch b's kernel is queued on the GPU (it streams slot b % 2 while the host goes on).
//   E  root prints batch b-1 from the ranks' node-shared result slots (b-1) % 2, while batch b streams
//      (on this thread: printing beside the next batch's encode on a helper thread was measured no faster
//      on the box's 16-CPU share, 0.63-0.72 vs 0.60 s at 1.14 G letters — both use every core,
//      profiles/final_modes_1.1G_r3f_async_print.log).
// So the host encodes batch b+1 while the kernel streams batch b, and prints batch b while batch b+1
// streams. Ordering makes the rings safe without extra barriers: a rank writes slot s again only after
// the root's broadcast of a later batch, which the root sends after printing the batch that used slot s.
#include <omp.h>

#include <algorithm>
#include <cstring>
#include <deque>

#include "job.hpp"
#include "text_cut.hpp"
#include "moc/runtime/host_region.hpp"
#include "moc/runtime/log.hpp"

namespace moc {

namespace {

// The fixed part of a batch's broadcast (the chunk table follows).
struct BatchMsg {
  int64_t n = 0, letters = 0, begin = 0, end = 0, nchunks = 0, status = 0;
};

// A host buffer of a ring slot: grows (rarely) and stays page-locked for the GPU between batches.
struct RingBuf {
  HostRegion region;
  int64_t cap = 0;
  std::function<void()> unpin;  // the buffer's registrations (GPU ranks)
  template <typename T>
  T* as() const {
    return region.as<T>();
  }
};

class StreamFlow {
 public:
  StreamFlow(JobCore& j, const Header& h, StreamSource& src, int64_t batch_records, int64_t batch_chars,
             const ParseOptions& po)
      : j_(j), h_(h), src_(src), max_rec_(batch_records > 0 ? batch_records : INT64_MAX),
        max_chr_(batch_chars > 0 ? batch_chars : INT64_MAX), l2_cap_(po.strict_limits ? kSpecMaxSeq2 : po.max_l2) {
    w_ = Weights{};
    for (int i = 0; i < 4; ++i) w_.w[i] = h.w[i];
    gpu_ = j_.eng.gpu ? j_.eng.hip.get() : nullptr;
    numa_ = gpu_ ? gpu_->numa_node() : -1;
    pin_ = gpu_ && j_.pin_window;
  }
  ~StreamFlow() {
    if (gpu_) (void)safe_finish();
    for (auto& s : in_)
      for (RingBuf* b : {&s.arena, &s.len16, &s.dense, &s.codes})
        if (b->unpin) b->unpin();
    for (auto& u : res_unpin_)
      if (u) u();
  }
  int run();

 private:
  struct InSlot {
    RingBuf arena;         // GPU ranks: the wire batch (page-locked)
    RingBuf len16;         // GPU ranks: the encoder's uint16 lengths
    RingBuf codes, dense;  // CPU ranks: byte letters + CSR offsets
  };
  // what one rank did with batch b (kept until its results are printed)
  struct Done {
    int64_t n = 0, first = 0;  // this rank's records; the batch's first global index
    ResultFormat fmt = ResultFormat::R12;
    WireBatch wb;
    bool launched = false;
  };
  bool safe_finish() {
    try {
      if (gpu_) gpu_->finish_wire();
      return true;
    } catch (...) {
      return false;
    }
  }
  void ensure(RingBuf& b, int64_t bytes, bool pin);
  char* ensure_results(int s, const std::vector<int64_t>& need, const std::vector<int64_t>& caps);
  BatchMsg next_batch(std::vector<int64_t>& table);   // A (root cuts, everyone receives)
  const char* batch_area(const BatchMsg& m, int s);    // the batch's text on this rank
  bool fill(const BatchMsg& m, const std::vector<int64_t>& table, int s, Done& d);  // B + C; false: input error
  void launch(int s, Done& d);                         // D
  void finish(int s, Done& d);                         // F
  void print(int s);                                   // E (root)

  JobCore& j_;
  const Header& h_;
  StreamSource& src_;
  const int64_t max_rec_, max_chr_, l2_cap_;
  Weights w_{};
  GpuRank* gpu_ = nullptr;
  int numa_ = -1;
  bool pin_ = false;
  std::unique_ptr<AreaText> text_;  // root
  std::unique_ptr<Cutter> cutter_;  // root
  int64_t next_index_ = 0;          // global index of the next batch's first record
  int64_t drop_at_ = 0;             // root, stream input: text before this may go once the batch is encoded
  InSlot in_[2];
  std::unique_ptr<SegmentWindow> res_[2];
  int64_t res_cap_[2] = {0, 0};  // this rank's segment bytes
  std::function<void()> res_unpin_[2];
  std::unique_ptr<SharedWindow> text_slot_[2];  // stream input, several ranks: the batch's text
  int64_t text_cap_[2] = {0, 0};
  // every rank's result run of the batch waiting to be printed (root)
  std::vector<ResultRun> runs_[2];
  int64_t runs_first_[2] = {0, 0};
  std::string error_;
  std::vector<double> kernel_ms_;  // per batch (this rank)
  double hidden_ms_ = 0;           // kernel time the host spent on other work (not waiting for it)
  double ring_ms_ = 0, encode_ms_ = 0, lengths_ms_ = 0;  // this rank's fill phase, split (--timing)
  double ring_fault_ms_ = 0, ring_pin_ms_ = 0;            // ... and the ring allocation's page faults / pins
  double count_ahead_ms_ = 0;  // root: batches counted while the GPU's runtime started
};

void StreamFlow::ensure(RingBuf& b, int64_t bytes, bool pin) {
  bytes = std::max<int64_t>(bytes, 64);
  if (bytes <= b.cap) return;
  if (b.unpin) {
    b.unpin();
    b.unpin = nullptr;
  }
  Stopwatch sw;
  sw.start();
  struct Stop {  // the allocation's time, whichever way it ends
    Stopwatch& sw;
    double& acc;
    ~Stop() {
      sw.stop();
      acc += sw.total_ms();
    }
  } stop{sw, ring_ms_};
  const int64_t cap = bytes + bytes / 4;
  b.region = HostRegion(static_cast<size_t>(cap), numa_);
  b.region.set_releaser(&j_.rel);
  b.cap = cap;
  if (pin && pin_) {
    try {
      Stopwatch t;
      t.start();
      b.region.prefault();  // OpenMP threads fault the pages in; the registration would on one thread
      t.stop();
      ring_fault_ms_ += t.total_ms();
      Stopwatch t2;
      t2.start();
      gpu_->pin(b.region.data(), static_cast<size_t>(cap));
      t2.stop();
      ring_pin_ms_ += t2.total_ms();
      b.unpin = gpu_->detach_pins();
      j_.pinned_bytes += cap;
    } catch (const std::exception& e) {
      MOC_LOG_WARN("could not page-lock a ring slot (%s); using the staged pipeline", e.what());
    }
  }
}

// Result slot s: every rank's segment holds at least need[q] bytes. Every rank knows every rank's need and
// capacity (exchanged with the fill reports), so all of them decide alike whether the collective
// re-allocation runs.
char* StreamFlow::ensure_results(int s, const std::vector<int64_t>& need, const std::vector<int64_t>& caps) {
  const int me = j_.ctx.rank;
  bool grow = !res_[s];
  for (size_t q = 0; q < need.size(); ++q) grow = grow || need[q] > caps[q];
  if (grow) {
    if (res_unpin_[s]) {
      res_unpin_[s]();
      res_unpin_[s] = nullptr;
    }
    res_[s].reset();  // collective
    const int64_t cap = std::max<int64_t>(std::max(need[me] + need[me] / 4, res_cap_[s]), 64);
    res_[s] = std::make_unique<SegmentWindow>(j_.ctx, cap, numa_);
    res_[s]->set_releaser(&j_.rel);
    res_cap_[s] = cap;
    if (pin_) {
      try {
        gpu_->pin(res_[s]->mine(), static_cast<size_t>(cap));
        res_unpin_[s] = gpu_->detach_pins();
        j_.pinned_bytes += cap;
      } catch (const std::exception& e) {
        MOC_LOG_WARN("could not page-lock a result slot (%s)", e.what());
      }
    }
  }
  return res_[s]->mine();
}

BatchMsg StreamFlow::next_batch(std::vector<int64_t>& table) {
  BatchMsg m;
  BatchCut cut;
  if (j_.ctx.rank == kRoot) {
    j_.pt.begin("count");
    try {
      const int64_t left = h_.n_total - next_index_;
      cut = cutter_->take(std::min(max_rec_, left), max_chr_);
      if (cut.n < std::min(max_rec_, left) && !(max_chr_ < INT64_MAX && cut.letters >= max_chr_))
        throw Error("expected " + std::to_string(h_.n_total) + " Seq2 records, found only " +
                    std::to_string(next_index_ + cut.n));
      m.n = cut.n;
      m.letters = cut.letters;
      m.begin = cut.begin;
      m.end = cut.end;
      m.nchunks = static_cast<int64_t>(cut.chunks.size());
    } catch (const std::exception& e) {
      m = BatchMsg{};
      m.status = 1;
      error_ = e.what();
    }
    j_.pt.end();
  }
  j_.pt.begin("bcast");
  bcast_bytes(&m, sizeof m, kRoot, j_.ctx.world);
  table.assign(static_cast<size_t>(3 * m.nchunks + 1), 0);
  if (j_.ctx.rank == kRoot) {
    for (int64_t c = 0; c < m.nchunks; ++c) {
      const Chunk& ch = cut.chunks[c];
      table[c] = ch.begin - m.begin;
      table[m.nchunks + 1 + c] = ch.toks;
      table[2 * m.nchunks + 1 + c] = ch.chars;
    }
    table[m.nchunks] = m.end - m.begin;
    // A stream's text before cut.next is dropped only after this batch is encoded (run): fill() may load
    // more text (count_ahead) while batch_area() still points into the buffer, and a load may move or
    // free the text it has been told it can drop.
    drop_at_ = cut.next;
  }
  if (m.nchunks > 0) bcast_bytes(table.data(), 8 * static_cast<int64_t>(table.size()), kRoot, j_.ctx.world);
  j_.pt.end();
  return m;
}

const char* StreamFlow::batch_area(const BatchMsg& m, int s) {
  if (src_.mapped) return src_.mapped + src_.area_begin + m.begin;
  if (j_.ctx.size == 1) return text_->at(m.begin);
  // several ranks, stream input: the root copies the batch's text into the node-shared slot s
  const int64_t len = m.end - m.begin;
  j_.pt.begin("share");
  if (len + 64 > text_cap_[s]) {
    text_slot_[s].reset();  // collective
    text_cap_[s] = (len + 64) + (len + 64) / 4;
    text_slot_[s] = std::make_unique<SharedWindow>(j_.ctx, text_cap_[s]);
  }
  if (j_.ctx.rank == kRoot) {
    const char* src = text_->at(m.begin);
    char* dst = text_slot_[s]->base();
    const int nt = len > (int64_t{1} << 24) ? omp_get_max_threads() : 1;
#pragma omp parallel for schedule(static, 1) num_threads(nt) if (nt > 1)
    for (int t = 0; t < nt; ++t) {
      const int64_t b = len * t / nt, e = len * (t + 1) / nt;
      std::memcpy(dst + b, src + b, static_cast<size_t>(e - b));
    }
  }
  text_slot_[s]->fence();
  j_.pt.end();
  return text_slot_[s]->base();
}

bool StreamFlow::fill(const BatchMsg& m, const std::vector<int64_t>& table, int s, Done& d) {
  const MpiContext& ctx = j_.ctx;
  const int p = ctx.size, r = ctx.rank;
  // A GPU job's first ring slot is page-locked only once the HIP runtime is up: the root counts later batches
  // meanwhile (mapped input: up to 32 batches ahead, ~3 ms of counting each; a stream holds what it counts,
  // so 2). This runs before the batch's text is located (batch_area): counting a stream loads more text,
  // and a load may move the buffer's text (dropping what earlier batches used) or reallocate the buffer.
  if (gpu_ && cutter_ && in_[s].arena.cap == 0 && !gpu_->runtime_ready()) {
    Stopwatch ca;
    ca.start();
    const int64_t ahead = src_.mapped ? 32 : 2;
    try {
      while (!gpu_->runtime_ready() && cutter_->count_ahead(max_rec_, max_chr_, ahead)) {
      }
    } catch (const std::exception&) {
      // a read error ahead of the batches: the batch that reaches it reports it (next_batch)
    }
    ca.stop();
    count_ahead_ms_ += ca.total_ms();
  }
  const char* area = batch_area(m, s);
  j_.pt.begin("fill");
  j_.fault.at("distribute", r);
  const int64_t nch = m.nchunks;
  BulkParser bp(area, static_cast<size_t>(m.end - m.begin), w_, j_.eng.seq1, l2_cap_, m.n);
  bp.set_chunks(std::vector<int64_t>(table.begin(), table.begin() + nch + 1), table.data() + nch + 1,
                table.data() + 2 * nch + 1);
  int64_t b0, b1;
  if (j_.partition == "even") {
    b0 = m.n * r / p;
    b1 = m.n * (r + 1) / p;
  } else {
    b0 = bp.cost_split(0, r, p, j_.cost_model());
    b1 = std::max(b0, bp.cost_split(0, r + 1, p, j_.cost_model()));
  }
  const AreaSlice slice = bp.slice(b0, b1);
  const int64_t n = slice.records;
  const int64_t L1 = static_cast<int64_t>(j_.eng.seq1.size());
  InSlot& in = in_[s];
  FillReport rep;
  d = Done{};
  d.n = n;
  d.first = next_index_ + b0;
  if (n > 0 && !gpu_) {
    ensure(in.codes, slice.letters + 16, false);
    ensure(in.dense, 8 * (n + 1), false);
    rep = bp.fill_slice(slice, in.codes.as<uint8_t>(), nullptr, in.dense.as<int64_t>());
  } else if (n > 0) {
    // one page-locked arena per slot, carved into letters | offsets | lengths: one registration per slot
    // (each registration costs milliseconds, whatever its size)
    auto al64 = [](int64_t x) { return (x + 63) & ~int64_t{63}; };
    bool narrow = L1 <= 200 && slice.letters <= 64 * n;
    const int pack = narrow ? 33 : 5;
    uint8_t* letters = nullptr;
    int64_t* offsets = nullptr;
    uint8_t* lens = nullptr;
    if (narrow) {
      const int64_t lb = al64(packed33_bytes(slice.letters) + 16);
      const int64_t sb = al64(8 * sparse_count(n, kSparseShift));
      ensure(in.arena, lb + sb + al64(n + 16), true);  // lengths: at most one byte each (+ slack)
      letters = in.arena.as<uint8_t>();
      offsets = reinterpret_cast<int64_t*>(in.arena.as<char>() + lb);
      lens = in.arena.as<uint8_t>() + lb + sb;
      ensure(in.len16, 2 * n, false);
      Stopwatch esw;
      esw.start();
      rep = bp.fill_slice(slice, nullptr, letters, nullptr, offsets, in.len16.as<uint16_t>(), pack);
      esw.stop();
      encode_ms_ += esw.total_ms();
      j_.pt.begin("engine_wait");  // the first batch: the engine's start-up, overlapped with the encode
      if (!(rep.max_len <= 255 && gpu_->streams_packed(rep.min_len, rep.max_len))) narrow = false;
      j_.pt.begin("fill");
    }
    if (!narrow) {  // 5-bit letters + CSR offsets (the staged pipeline's form)
      const int64_t lb = al64(packed5_bytes(slice.letters) + 16);
      ensure(in.arena, lb + 8 * (n + 1), true);
      letters = in.arena.as<uint8_t>();
      offsets = reinterpret_cast<int64_t*>(in.arena.as<char>() + lb);
      rep = bp.fill_slice(slice, nullptr, letters, offsets);
    }
    WireBatch& wb = d.wb;
    wb.letters = letters;
    wb.packed33 = narrow && pack == 33;
    wb.packed5 = !narrow;
    wb.n = n;
    wb.min_l2 = rep.min_len;
    wb.max_l2 = rep.max_len;
    wb.offsets = offsets;
    if (narrow) {
      const int bits = narrow_length_bits(rep.min_len, rep.max_len);
      Stopwatch lsw;
      lsw.start();
      pack_lengths16(in.len16.as<uint16_t>(), n, bits, rep.min_len, lens);
      lsw.stop();
      lengths_ms_ += lsw.total_ms();
      wb.off_shift = kSparseShift;
      wb.lengths = lens;
      wb.len_bits = bits;
      wb.len_base = bits == 8 ? 0 : rep.min_len;
    }
    d.fmt = gpu_->result_format(rep.min_len, rep.max_len);
  }
  j_.pt.end();
  // ---- C: the batch's first input error, on every rank; result-slot sizes
  j_.pt.begin("report");
  const int fb = result_bytes(d.fmt);
  int64_t mine[9] = {rep.min_len, rep.max_len, rep.bad_record, rep.long_record, rep.long_len, rep.cells,
                     slice.letters, fb * n, res_[s] ? res_cap_[s] : -1};
  std::vector<int64_t> all(static_cast<size_t>(9 * p));
  j_.allgather_i64(mine, 9, all.data());
  FillReport whole;
  std::vector<int64_t> need(static_cast<size_t>(p)), caps(static_cast<size_t>(p));
  for (int q = 0; q < p; ++q) {
    const int64_t* x = all.data() + 9 * q;
    caps[q] = x[8];
    whole.min_len = std::min(whole.min_len, x[0]);
    whole.max_len = std::max(whole.max_len, x[1]);
    if (x[2] >= 0 && (whole.bad_record < 0 || x[2] < whole.bad_record)) whole.bad_record = x[2];
    if (x[3] >= 0 && (whole.long_record < 0 || x[3] < whole.long_record)) {
      whole.long_record = x[3];
      whole.long_len = x[4];
    }
    whole.cells += x[5];
    need[q] = x[7];
  }
  // batch-relative record indices -> the job's
  if (whole.bad_record >= 0) whole.bad_record += next_index_;
  if (whole.long_record >= 0) whole.long_record += next_index_;
  try {
    bp.check(whole);
  } catch (const std::exception& e) {
    error_ = e.what();
    j_.pt.end();
    return false;
  }
  j_.cells += whole.cells;
  j_.chars += m.letters;
  j_.records += m.n;
  ++j_.batches;
  ensure_results(s, need, caps);
  j_.pt.end();
  return true;
}

void StreamFlow::launch(int s, Done& d) {
  if (d.n <= 0) return;
  j_.pt.begin("compute");
  j_.fault.at("compute", j_.ctx.rank);
  Stopwatch sw;
  sw.start();
  char* out = res_[s]->mine();
  if (gpu_) {
    gpu_->begin_wire(d.wb, out, d.fmt);
    d.launched = true;
  } else {
    RecordBatch b;  // the CPU engine reads a RecordBatch: the slot's codes/offsets, viewed (no copy needed
                    // for correctness; one copy of a batch is cheap next to its O(L1*L2) search)
    const InSlot& in = in_[s];
    b.codes.assign(in.codes.as<uint8_t>(), in.codes.as<uint8_t>() + in.dense.as<int64_t>()[d.n]);
    b.offsets.assign(in.dense.as<int64_t>(), in.dense.as<int64_t>() + d.n + 1);
    solve_batch_cpu(j_.eng.table, j_.eng.seq1.data(), static_cast<int64_t>(j_.eng.seq1.size()), b,
                    reinterpret_cast<Result*>(out), j_.eng.sem, j_.eng.threads);
  }
  sw.stop();
  j_.compute_ms += sw.total_ms();
  j_.pt.end();
}

void StreamFlow::finish(int s, Done& d) {
  GpuSolveStats gs;
  if (d.launched) {
    j_.pt.begin("compute");
    Stopwatch sw;
    sw.start();
    gs = gpu_->finish_wire();
    sw.stop();
    j_.compute_ms += sw.total_ms();
    hidden_ms_ += std::max(0.0, gs.kernel_ms - sw.total_ms());
    j_.eng.kernel_ms += gs.kernel_ms;
    j_.h2d_bytes += gs.h2d_bytes;
    j_.d2h_bytes += gs.d2h_bytes;
    kernel_ms_.push_back(gs.kernel_ms);
    d.launched = false;
    j_.pt.end();
  }
  j_.pt.begin("gather");
  j_.fault.at("gather", j_.ctx.rank);
  const int p = j_.ctx.size;
  int64_t info[5] = {d.n, static_cast<int64_t>(d.fmt), gs.r2.smin, gs.r2.kw, gs.r2.j};
  std::vector<int64_t> infos(static_cast<size_t>(5 * p));
  j_.allgather_i64(info, 5, infos.data());
  res_[s]->fence();
  if (j_.ctx.rank == kRoot) {
    runs_[s].assign(static_cast<size_t>(p), ResultRun{});
    if (j_.rank_records.size() != static_cast<size_t>(p)) j_.rank_records.assign(static_cast<size_t>(p), 0);
    for (int q = 0; q < p; ++q) {
      const int64_t* x = infos.data() + 5 * q;
      runs_[s][q] = ResultRun{res_[s]->segment(q), static_cast<ResultFormat>(x[1]),
                              R2Params{static_cast<int32_t>(x[2]), static_cast<int32_t>(x[3]), static_cast<int32_t>(x[4])},
                              x[0]};
      j_.rank_records[q] += x[0];
    }
    runs_first_[s] = d.first;
  }
  j_.pt.end();
}

void StreamFlow::print(int s) {
  if (j_.ctx.rank != kRoot || runs_[s].empty()) return;
  j_.pt.begin("print");
  ScopedOmpThreads team(j_.print_threads);  // the other ranks wait for the next batch's broadcast
  write_results(j_.out, runs_[s], runs_first_[s]);
  runs_[s].clear();
  j_.pt.end();
}

int StreamFlow::run() {
  const MpiContext& ctx = j_.ctx;
  if (src_.mapped) bcast_bytes(&src_.area_begin, sizeof src_.area_begin, kRoot, ctx.world);
  if (ctx.rank == kRoot) {
    if (src_.mapped)
      text_ = std::make_unique<AreaText>(src_.mapped + src_.area_begin, src_.mapped_bytes - src_.area_begin);
    else
      text_ = std::make_unique<AreaText>(std::move(src_.head), src_.eof, src_.in);
    cutter_ = std::make_unique<Cutter>(*text_);
  }
  // --skip-records: the root cuts the skipped records like a batch that nobody encodes
  next_index_ = h_.first_index;
  if (ctx.rank == kRoot && h_.first_index > 0) {
    j_.pt.begin("skip");
    const BatchCut skipped = cutter_->take(h_.first_index, INT64_MAX);
    if (!text_->mapped()) text_->drop_before(skipped.next);
    j_.pt.end();
  }
  j_.first_index = next_index_;
  std::vector<int64_t> table;
  Done done[2];
  int b = 0;
  int rc = 0;
  bool have_prev = false;  // batch b-1 is launched and not yet finished / printed
  while (true) {
    const int s = b & 1;
    BatchMsg m = next_batch(table);
    bool ok = m.status == 0;
    if (ok && m.n > 0) ok = fill(m, table, s, done[s]);  // while the kernel of batch b-1 streams
    if (ctx.rank == kRoot && !text_->mapped()) text_->drop_before(drop_at_);  // batch b's text is encoded
    if (have_prev) {  // F + E of batch b-1 (also before leaving on an input error of batch b)
      finish(s ^ 1, done[s ^ 1]);
      if (ok && m.n > 0) launch(s, done[s]);
      print(s ^ 1);
      have_prev = false;
    } else if (ok && m.n > 0) {
      launch(s, done[s]);
    }
    if (!ok) {
      if (ctx.rank == kRoot) std::fprintf(stderr, "input error: %s\n", error_.c_str());
      rc = 1;
      break;
    }
    if (m.n == 0) break;
    next_index_ += m.n;
    have_prev = true;
    ++b;
  }
  if (rc == 0 && ctx.rank == kRoot && next_index_ < h_.n_total) {
    // unreachable: next_batch reports a short input (kept as a guard)
    std::fprintf(stderr, "input error: expected %lld Seq2 records\n", static_cast<long long>(h_.n_total));
    rc = 1;
  }
  if (!kernel_ms_.empty()) {
    std::vector<double> k = kernel_ms_;
    std::sort(k.begin(), k.end());
    char buf[160];
    std::snprintf(buf, sizeof buf, "{\"p50\": %.4f, \"max\": %.4f, \"batches\": %zu}", k[k.size() / 2], k.back(), k.size());
    j_.extra_timing.emplace_back("rank0_batch_kernel_ms", buf);
  }
  {
    char buf[64];
    std::snprintf(buf, sizeof buf, "%.3f", hidden_ms_);
    j_.extra_timing.emplace_back("rank0_kernel_hidden_ms", buf);
  }
  {
    char buf[240];
    std::snprintf(buf, sizeof buf,
                  "{\"ring_alloc\": %.3f, \"ring_fault\": %.3f, \"ring_pin\": %.3f, \"encode\": %.3f, \"lengths\": %.3f, "
                  "\"count_ahead\": %.3f}",
                  ring_ms_, ring_fault_ms_, ring_pin_ms_, encode_ms_, lengths_ms_, count_ahead_ms_);
    j_.extra_timing.emplace_back("rank0_fill_split_ms", buf);
  }
  return rc;
}

}  // namespace

int run_streaming(JobCore& job, const Header& h, StreamSource& src, int64_t batch_records, int64_t batch_chars,
                  const ParseOptions& po) {
  StreamFlow f(job, h, src, batch_records, batch_chars, po);
  return f.run();
}

}  // namespace moc
