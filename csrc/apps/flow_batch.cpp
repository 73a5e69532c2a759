// One in-memory batch of records over the job's transport (job.hpp): the path of multi-node jobs (mpi,
// rccl), of the context-parallel decomposition, of --transport=rccl-emul and of the StreamReader-fed
// streaming mode on those transports. Decomposition + distribution + search + combine + print.
// Reference: MPI_Scatter of fixed 2000-byte records (main.c:174), one kernel launch per record per rank
// (cudaFunctions.cu:204-218), MPI_Gather x3 (main.c:195-197).
#include <omp.h>

#include <algorithm>
#include <cstring>

#include "job.hpp"
#include "moc/device_comm.hpp"

namespace moc {

namespace {

class BatchFlow {
 public:
  BatchFlow(JobCore& j, std::unique_ptr<BulkParser>* parser, uvector<char>* text)
      : j_(j), parser_(parser), text_(text) {}
  void run(RecordBatch* rb, int64_t n, int64_t total_chars);
  void release_input_now() { release_input(); }

 private:
  std::vector<int64_t> make_bounds(const int64_t* offsets, int64_t n, bool cp);
  void batch_shm(RecordBatch* rb, int64_t n, int64_t total_chars);
  void batch_mpi(RecordBatch* rb, int64_t n, int64_t total_chars, const std::vector<int64_t>& bounds, bool cp);
  void batch_rccl(RecordBatch* rb, int64_t n, int64_t total_chars, const std::vector<int64_t>& bounds, bool cp);
  // the input (deferred parser + text) goes back to the OS on the releaser
  void release_input();

  JobCore& j_;
  std::unique_ptr<BulkParser>* parser_;  // root: the parser of a text batch (or null), released with the text
  uvector<char>* text_;                  // root: the text that parser reads
};

void BatchFlow::release_input() {
  std::shared_ptr<BulkParser> p(parser_ && *parser_ ? std::move(*parser_) : nullptr);
  std::shared_ptr<uvector<char>> t;
  if (text_ && !text_->empty()) {
    t = std::make_shared<uvector<char>>(std::move(*text_));
    *text_ = uvector<char>();
  }
  if (p || t)
    j_.rel.defer([p, t]() mutable {
      p.reset();
      t.reset();
    });
}

void BatchFlow::run(RecordBatch* rb, int64_t n, int64_t total_chars) {
  const bool cp = j_.partition == "offsets";
  if (j_.transport == "shm") {  // the window is filled first; the bounds come from it
    if (!cp) throw Error("record-slice batches on the shm transport run sliced or streamed");
    batch_shm(rb, n, total_chars);
    return;
  }
  const std::vector<int64_t> bounds = make_bounds(j_.ctx.rank == kRoot ? rb->offsets.data() : nullptr, n, cp);
  if (j_.transport == "mpi")
    batch_mpi(rb, n, total_chars, bounds, cp);
  else
    batch_rccl(rb, n, total_chars, bounds, cp);
}

// Root: record lengths -> search cells (for --timing) and the cost-balanced rank bounds; broadcast.
std::vector<int64_t> BatchFlow::make_bounds(const int64_t* offsets, int64_t n, bool cp) {
  const int p = j_.ctx.size;
  std::vector<int64_t> bounds(static_cast<size_t>(p) + 1, 0);
  if (j_.ctx.rank == kRoot) {
    const int64_t L1 = static_cast<int64_t>(j_.eng.seq1.size());
    int64_t cells = 0;
#pragma omp parallel for reduction(+ : cells) schedule(static) if (n > 65536)
    for (int64_t i = 0; i < n; ++i) cells += record_cells(L1, offsets[i + 1] - offsets[i]);
    j_.cells += cells;
    if (!cp)
      bounds = j_.partition == "even" ? partition_even(n, p) : partition_by_cost_offsets(offsets, n, L1, p, j_.cost_model());
  }
  if (!cp) bcast_bytes(bounds.data(), sizeof(int64_t) * (p + 1), kRoot, j_.ctx.world);
  return bounds;
}

// Context parallel on one node (shm transport, --partition=offsets; the record-slice jobs of the node run
// sliced or streamed): the batch in a node-shared window, every rank searches its share of every record's
// offsets, packed keys MAX-all-reduced, the root resolves and prints.
void BatchFlow::batch_shm(RecordBatch* rb, int64_t n, int64_t total_chars) {
  PhaseTimer& pt = j_.pt;
  const MpiContext& ctx = j_.ctx;
  // layout: offsets[(N+1)] | results[N] | codes[total]   (8-byte aligned sections)
  const int64_t off_bytes = 8 * (n + 1);
  const int64_t res_bytes = ((12 * n) + 7) & ~int64_t{7};
  pt.begin("distribute");
  auto win = std::make_unique<SharedWindow>(ctx, off_bytes + res_bytes + total_chars);
  win->set_releaser(&j_.rel);
  int64_t* w_offs = reinterpret_cast<int64_t*>(win->base());
  Result* w_res = reinterpret_cast<Result*>(win->base() + off_bytes);
  uint8_t* w_codes = reinterpret_cast<uint8_t*>(win->base() + off_bytes + res_bytes);
  if (ctx.rank == kRoot) {
    const int64_t* src_off = rb->offsets.data();
    const uint8_t* src_codes = rb->codes.data();
    const int nt = total_chars > (1 << 20) ? omp_get_max_threads() : 1;
#pragma omp parallel for schedule(static, 1) num_threads(nt)
    for (int t = 0; t < nt; ++t) {
      const int64_t cb = total_chars * t / nt, ce = total_chars * (t + 1) / nt;
      std::memcpy(w_codes + cb, src_codes + cb, static_cast<size_t>(ce - cb));
      const int64_t ob = (n + 1) * t / nt, oe = (n + 1) * (t + 1) / nt;
      std::memcpy(w_offs + ob, src_off + ob, static_cast<size_t>(oe - ob) * 8);
    }
    *rb = RecordBatch{};  // the window is now the only copy
  }
  j_.fault.at("distribute", ctx.rank);
  win->fence();
  pt.end();
  pt.begin("bounds");
  make_bounds(ctx.rank == kRoot ? w_offs : nullptr, n, true);  // the search cells (--timing)
  pt.end();
  pt.begin("compute");
  j_.fault.at("compute", ctx.rank);
  Stopwatch sw;
  sw.start();
  std::vector<uint64_t> keys(static_cast<size_t>(n), 0);
  j_.eng.solve_keys(w_codes, w_offs, n, ctx.rank, ctx.size, keys.data());
  sw.stop();
  pt.end();
  pt.begin("gather");
  j_.fault.at("gather", ctx.rank);
  j_.allreduce_keys(keys.data(), n);
  if (ctx.rank == kRoot) j_.resolve_keys(keys.data(), w_codes, w_offs, n, w_res);
  pt.end();
  j_.compute_ms += sw.total_ms();
  // printing reads only the results: the input, offsets and letters go back to the OS while it runs
  release_input();
  win->discard(0, off_bytes);
  win->discard(off_bytes + res_bytes, total_chars);
  j_.print(w_res, n, 0);
  pt.begin("release");
  win.reset();  // collective: unmaps the node-shared window
  pt.end();
}

void BatchFlow::batch_mpi(RecordBatch* rb, int64_t n, int64_t total_chars, const std::vector<int64_t>& bounds,
                          bool cp) {
  PhaseTimer& pt = j_.pt;
  const MpiContext& ctx = j_.ctx;
  const int p = ctx.size;
  pt.begin("distribute");
  j_.fault.at("distribute", ctx.rank);
  std::vector<Result> results;
  if (cp) {  // every rank needs every record
    RecordBatch all;
    if (ctx.rank == kRoot) all = std::move(*rb);
    all.offsets.resize(static_cast<size_t>(n) + 1);
    all.codes.resize(static_cast<size_t>(total_chars));
    bcast_bytes(all.offsets.data(), 8 * (n + 1), kRoot, ctx.world);
    bcast_bytes(all.codes.data(), total_chars, kRoot, ctx.world);
    pt.end();
    pt.begin("compute");
    j_.fault.at("compute", ctx.rank);
    Stopwatch sw;
    sw.start();
    std::vector<uint64_t> keys(static_cast<size_t>(n), 0);
    j_.eng.solve_keys(all.codes.data(), all.offsets.data(), n, ctx.rank, ctx.size, keys.data());
    sw.stop();
    j_.compute_ms += sw.total_ms();
    pt.end();
    pt.begin("gather");
    j_.fault.at("gather", ctx.rank);
    allreduce_max_u64(keys.data(), n, ctx.world);
    pt.end();
    if (ctx.rank == kRoot) {
      results.resize(static_cast<size_t>(n));
      j_.resolve_keys(keys.data(), all.codes.data(), all.offsets.data(), n, results.data());
    }
    j_.print(results.data(), n, 0);
    return;
  }
  const int64_t my_b = bounds[ctx.rank], my_n = bounds[ctx.rank + 1] - my_b;
  std::vector<int64_t> lcount(p), ldispl(p), ccount(p), cdispl(p);
  for (int r = 0; r < p; ++r) {
    lcount[r] = 8 * (bounds[r + 1] - bounds[r]);
    ldispl[r] = 8 * bounds[r];
  }
  std::vector<int64_t> lengths;
  if (ctx.rank == kRoot) {
    lengths.resize(static_cast<size_t>(n));
    for (int64_t i = 0; i < n; ++i) lengths[i] = rb->length(i);
    for (int r = 0; r < p; ++r) {
      ccount[r] = rb->offsets[bounds[r + 1]] - rb->offsets[bounds[r]];
      cdispl[r] = rb->offsets[bounds[r]];
    }
  }
  bcast_bytes(ccount.data(), 8 * p, kRoot, ctx.world);
  std::vector<int64_t> my_len(static_cast<size_t>(my_n));
  scatterv_bytes(lengths.data(), lcount, ldispl, my_len.data(), kRoot, ctx.world);
  std::vector<uint8_t> my_codes(static_cast<size_t>(ccount[ctx.rank]));
  scatterv_bytes(ctx.rank == kRoot ? rb->codes.data() : nullptr, ccount, cdispl, my_codes.data(), kRoot, ctx.world);
  std::vector<int64_t> my_off(static_cast<size_t>(my_n) + 1, 0);
  for (int64_t i = 0; i < my_n; ++i) my_off[i + 1] = my_off[i] + my_len[i];
  pt.end();
  pt.begin("compute");
  j_.fault.at("compute", ctx.rank);
  std::vector<Result> mine(static_cast<size_t>(my_n));
  Stopwatch sw;
  sw.start();
  j_.eng.solve(my_codes.data(), my_off.data(), my_n, mine.data());
  sw.stop();
  j_.compute_ms += sw.total_ms();
  pt.end();
  pt.begin("gather");
  j_.fault.at("gather", ctx.rank);
  std::vector<int64_t> rcount(p), rdispl(p);
  for (int r = 0; r < p; ++r) {
    rcount[r] = 12 * (bounds[r + 1] - bounds[r]);
    rdispl[r] = 12 * bounds[r];
  }
  if (ctx.rank == kRoot) results.resize(static_cast<size_t>(n));
  gatherv_bytes(mine.data(), 12 * my_n, results.data(), rcount, rdispl, kRoot, ctx.world);
  pt.end();
  j_.print(results.data(), n, 0);
}

void BatchFlow::batch_rccl(RecordBatch* rb, int64_t n, int64_t total_chars, const std::vector<int64_t>& bounds,
                           bool cp) {
  PhaseHooks hooks;
  DeviceComm& dc = j_.emul_comm ? static_cast<DeviceComm&>(*j_.emul_comm) : j_.eng.hip->device_comm();
  hooks.begin = [this, &dc](const char* phase) {
    j_.pt.begin(phase);
    j_.fault.at(phase, j_.ctx.rank, &dc);
  };
  hooks.end = [this] { j_.pt.end(); };
  DeviceBatchOut out;
  if (!j_.scratch) j_.scratch = std::make_unique<DeviceScratch>(dc);
  if (j_.emul_comm) {
    CpuDeviceSearch ds(j_.eng.table, j_.eng.seq1, j_.eng.sem, j_.eng.threads);
    out = device_batch(dc, ds, rb, n, total_chars, bounds, cp, hooks, j_.scratch.get());
  } else {
    out = device_batch(dc, j_.eng.hip->device_search(), rb, n, total_chars, bounds, cp, hooks, j_.scratch.get());
  }
  j_.compute_ms += out.compute_ms;
  j_.eng.kernel_ms += out.kernel_ms;
  j_.account_comm(out);
  if (j_.ctx.rank == kRoot) {
    if (!out.rank_records.empty()) j_.rank_records = out.rank_records;
    j_.pt.begin("print");
    write_results(j_.out, out.runs, j_.first_index);
    j_.pt.end();
  }
}

}  // namespace

void run_text_batch(JobCore& job, std::unique_ptr<BulkParser>& parser, int64_t first_index, uvector<char>* text) {
  const MpiContext& ctx = job.ctx;
  const int p = ctx.size;
  const bool device = job.transport == "rccl" || job.transport == "rccl-emul";
  // ---- root: pass 1 over the whole text in ~1 MiB chunks (the encode's unit of parallel work), the rank
  // bounds; or, on the mpi transport, the whole batch as byte codes
  std::vector<int64_t> bounds(static_cast<size_t>(p) + 1, 0);
  RecordBatch bulk;
  int64_t st[3] = {0, 0, 0};  // status, records, letters
  std::string error;
  if (ctx.rank == kRoot) {
    job.pt.begin("count");
    try {
      const int64_t area = parser->area_bytes();
      const int nch = static_cast<int>(std::clamp<int64_t>(area >> 20, std::min<int64_t>(64, std::max<int64_t>(area >> 16, 1)),
                                                           int64_t{1} << 14));
      std::vector<int64_t> starts = parser->chunk_starts(nch);
      std::vector<int64_t> tk(static_cast<size_t>(nch)), ch(static_cast<size_t>(nch));
      parser->count_chunks(starts, 0, nch, tk.data(), ch.data());
      const CostModel m = job.cost_model();
      if (device && job.partition != "even" && p > 1 && area <= (int64_t{256} << 20)) {
        std::vector<double> costs(static_cast<size_t>(nch));
        parser->chunk_costs(starts, 0, nch, m, costs.data());
        parser->set_chunk_costs(std::move(costs));
      }
      parser->set_chunks(std::move(starts), tk.data(), ch.data());
      const int64_t n_all = parser->count();
      first_index = std::min(first_index, n_all);
      st[1] = n_all - first_index;
      if (device) {
        for (int r = 0; r <= p; ++r)
          bounds[r] = job.partition == "even" ? first_index + st[1] * r / p : parser->cost_split(first_index, r, p, m);
        for (int r = 1; r <= p; ++r) bounds[r] = std::max(bounds[r], bounds[r - 1]);
      } else {
        const AreaSlice s = parser->slice(first_index, n_all);
        bulk.codes.resize(static_cast<size_t>(s.letters));
        bulk.offsets.resize(static_cast<size_t>(s.records) + 1);
        parser->check(parser->fill_slice(s, bulk.codes.data(), nullptr, bulk.offsets.data()));
        st[2] = s.letters;
      }
    } catch (const std::exception& e) {
      st[0] = 1;
      error = e.what();
    }
    job.pt.end();
  }
  bcast_bytes(st, sizeof st, kRoot, ctx.world);
  if (st[0] != 0) throw InputError(error);
  if (!device) {
    parser.reset();
    if (text) *text = uvector<char>();
    run_record_batch(job, ctx.rank == kRoot ? &bulk : nullptr, st[1], st[2], first_index);
    return;
  }
  ++job.batches;
  job.first_index = first_index;
  job.records += st[1];
  PhaseHooks hooks;
  DeviceComm& dc = job.emul_comm ? static_cast<DeviceComm&>(*job.emul_comm) : job.eng.hip->device_comm();
  hooks.begin = [&job, &dc](const char* phase) {
    job.pt.begin(phase);
    job.fault.at(phase, job.ctx.rank, &dc);
  };
  hooks.end = [&job] { job.pt.end(); };
  if (!job.scratch) job.scratch = std::make_unique<DeviceScratch>(dc);
  DeviceBatchOut out;
  if (job.emul_comm) {
    CpuDeviceSearch ds(job.eng.table, job.eng.seq1, job.eng.sem, job.eng.threads);
    out = device_batch_text(dc, ds, parser.get(), bounds, hooks, job.scratch.get());
  } else {
    out = device_batch_text(dc, job.eng.hip->device_search(), parser.get(), bounds, hooks, job.scratch.get());
  }
  if (out.input_error) throw InputError(out.error);
  // the input text and the parser's tables go back to the OS while the results print
  BatchFlow(job, &parser, text).release_input_now();
  job.compute_ms += out.compute_ms;
  job.eng.kernel_ms += out.kernel_ms;
  job.account_comm(out);
  if (ctx.rank == kRoot) {
    job.cells += out.cells;
    job.chars += out.letters;
    if (!out.rank_records.empty()) job.rank_records = out.rank_records;
    job.pt.begin("print");
    write_results(job.out, out.runs, first_index);
    job.pt.end();
  }
}

void run_record_batch(JobCore& job, RecordBatch* rb, int64_t n, int64_t total_chars, int64_t first_index,
                      std::unique_ptr<BulkParser>* parser, uvector<char>* text) {
  ++job.batches;
  job.first_index = first_index;
  job.records += n;
  job.chars += total_chars;
  BatchFlow(job, parser, text).run(rb, n, total_chars);
}

}  // namespace moc
