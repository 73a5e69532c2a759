// Streaming job off the node's shm transport (`final --batch-records=B [--batch-chars=C]` with
// --transport=rccl | rccl-emul | mpi, record slices): host memory bounded by the batch, every batch
// cut by the root from the input text and sent to the ranks.
//
// Reference: read everything, then one blocking scatter (/root/reference/main.c:90-108,174).
//
// Per batch b: the root cuts it (text_cut.hpp: pass 1 in ~1 MiB chunks kept past the cut, no re-count),
// splits it by cost and, on the device transports, encodes every rank's slice straight from the text into
// that rank's wire block while the previous rank's block is on its way (device_batch_text); the ranks
// search from device memory and the narrow results are gathered into one of two page-locked buffers. The
// root writes batch b's rows on a helper thread while batch b+1 is cut, encoded, sent and searched. On the
// mpi transport the root encodes the batch's byte codes for the Scatterv flow (run_record_batch).
#include <future>

#include "job.hpp"
#include "moc/device_comm.hpp"
#include "moc/runtime/timer.hpp"
#include "text_cut.hpp"

namespace moc {

int run_device_streaming(JobCore& job, const Header& h, StreamSource& src, int64_t batch_records,
                         int64_t batch_chars, const ParseOptions& po) {
  const MpiContext& ctx = job.ctx;
  const int p = ctx.size;
  const bool root = ctx.rank == kRoot;
  const bool device = job.transport == "rccl" || job.transport == "rccl-emul";
  const int64_t max_rec = batch_records > 0 ? batch_records : INT64_MAX;
  const int64_t max_chr = batch_chars > 0 ? batch_chars : INT64_MAX;
  const int64_t l2_cap = po.strict_limits ? kSpecMaxSeq2 : po.max_l2;
  Weights w{};
  for (int i = 0; i < 4; ++i) w.w[i] = h.w[i];
  std::unique_ptr<AreaText> text;
  std::unique_ptr<Cutter> cutter;
  if (root) {
    if (src.mapped)
      text = std::make_unique<AreaText>(src.mapped + src.area_begin, src.mapped_bytes - src.area_begin);
    else
      text = std::make_unique<AreaText>(std::move(src.head), src.eof, src.in);
    cutter = std::make_unique<Cutter>(*text);
  }
  int64_t next = h.first_index;  // global index of the next batch's first record
  if (root && next > 0) {        // --skip-records: cut like a batch nobody encodes
    job.pt.begin("skip");
    const BatchCut skipped = cutter->take(next, INT64_MAX);
    if (!text->mapped()) text->drop_before(skipped.next);
    job.pt.end();
  }
  job.first_index = next;

  DeviceComm* dc = nullptr;
  PhaseHooks hooks;
  hooks.begin = [&job, &dc](const char* phase) {
    job.pt.begin(phase);
    job.fault.at(phase, job.ctx.rank, dc);
  };
  hooks.end = [&job] { job.pt.end(); };
  std::unique_ptr<CpuDeviceSearch> cpu_search;
  DeviceSearch* ds = nullptr;
  if (device) {
    dc = job.emul_comm ? static_cast<DeviceComm*>(job.emul_comm.get()) : &job.eng.hip->device_comm();
    if (!job.scratch) job.scratch = std::make_unique<DeviceScratch>(*dc);
    if (job.emul_comm) {
      cpu_search = std::make_unique<CpuDeviceSearch>(job.eng.table, job.eng.seq1, job.eng.sem, job.eng.threads);
      ds = cpu_search.get();
    } else {
      ds = &job.eng.hip->device_search();
    }
  }

  std::future<double> printing;  // root: the previous batch's rows (returns the ms it took)
  double print_ms = 0;
  auto wait_print = [&] {
    if (printing.valid()) print_ms += printing.get();
  };
  std::string error;
  int rc = 0;
  for (int b = 0;; ++b) {
    int64_t msg[2] = {0, 0};  // records of the batch, status
    BatchCut cut;
    if (root) {
      job.pt.begin("count");
      try {
        const int64_t left = h.n_total - next;
        cut = cutter->take(std::min(max_rec, left), max_chr);
        if (cut.n < std::min(max_rec, left) && !(max_chr < INT64_MAX && cut.letters >= max_chr))
          throw Error("expected " + std::to_string(h.n_total) + " Seq2 records, found only " +
                      std::to_string(next + cut.n));
        msg[0] = cut.n;
      } catch (const std::exception& e) {
        msg[1] = 1;
        error = e.what();
      }
      job.pt.end();
    }
    bcast_bytes(msg, sizeof msg, kRoot, ctx.world);
    if (msg[1] != 0) {
      rc = 1;
      break;
    }
    const int64_t n = msg[0];
    if (n == 0) break;
    // root: a parser over the batch's text with the cutter's chunk table (pass 1 is done)
    std::unique_ptr<BulkParser> bp;
    std::vector<int64_t> bounds(static_cast<size_t>(p) + 1, 0);
    if (root) {
      bp = std::make_unique<BulkParser>(text->at(cut.begin), static_cast<size_t>(cut.end - cut.begin), w, job.eng.seq1,
                                        l2_cap, n);
      const size_t nc = cut.chunks.size();
      std::vector<int64_t> starts(nc + 1), tk(nc), ch(nc);
      for (size_t c = 0; c < nc; ++c) {
        starts[c] = cut.chunks[c].begin - cut.begin;
        tk[c] = cut.chunks[c].toks;
        ch[c] = cut.chunks[c].chars;
      }
      starts[nc] = cut.end - cut.begin;
      bp->set_chunks(std::move(starts), tk.data(), ch.data());
      const CostModel m = job.cost_model();
      for (int r = 0; r <= p; ++r) bounds[r] = job.partition == "even" ? n * r / p : bp->cost_split(0, r, p, m);
      for (int r = 1; r <= p; ++r) bounds[r] = std::max(bounds[r], bounds[r - 1]);
    }
    if (!device) {  // mpi: the batch as byte codes for the Scatterv flow (printed in order, on this thread)
      RecordBatch rb;
      int64_t st[2] = {0, 0};  // status, letters
      if (root) {
        job.pt.begin("fill");
        try {
          const AreaSlice s = bp->slice(0, n);
          rb.codes.resize(static_cast<size_t>(s.letters));
          rb.offsets.resize(static_cast<size_t>(n) + 1);
          FillReport rep = bp->fill_slice(s, rb.codes.data(), nullptr, rb.offsets.data());
          if (rep.bad_record >= 0) rep.bad_record += next;
          if (rep.long_record >= 0) rep.long_record += next;
          bp->check(rep);
          st[1] = s.letters;
        } catch (const std::exception& e) {
          st[0] = 1;
          error = e.what();
        }
        if (!text->mapped()) text->drop_before(cut.next);
        job.pt.end();
      }
      bcast_bytes(st, sizeof st, kRoot, ctx.world);
      if (st[0] != 0) {
        rc = 1;
        break;
      }
      run_record_batch(job, root ? &rb : nullptr, n, st[1], next);
      next += n;
      continue;
    }
    DeviceBatchOut out = device_batch_text(*dc, *ds, bp.get(), bounds, hooks, job.scratch.get(), next, b & 1);
    if (root && !text->mapped()) text->drop_before(cut.next);  // encoded: the stream buffer may reuse it
    if (out.input_error) {
      error = out.error;
      rc = 1;
      break;
    }
    job.compute_ms += out.compute_ms;
    job.eng.kernel_ms += out.kernel_ms;
    job.account_comm(out);
    ++job.batches;
    if (root) {
      job.records += n;
      job.cells += out.cells;
      job.chars += out.letters;
      if (job.rank_records.size() != static_cast<size_t>(p)) job.rank_records.assign(static_cast<size_t>(p), 0);
      for (int q = 0; q < p && q < static_cast<int>(out.rank_records.size()); ++q) job.rank_records[q] += out.rank_records[q];
      // batch b's rows, while batch b+1 is cut, encoded and searched (its results go to the other buffer)
      wait_print();
      printing = std::async(std::launch::async, [&job, runs = std::move(out.runs), first = next]() {
        Stopwatch sw;
        sw.start();
        write_results(job.out, runs, first);
        sw.stop();
        return sw.total_ms();
      });
    }
    next += n;
  }
  if (root) {
    job.pt.begin("print");  // the last batch's rows (and the rows before an input error)
    wait_print();
    job.pt.end();
    if (device) {
      char buf[32];
      std::snprintf(buf, sizeof buf, "%.3f", print_ms);
      job.extra_timing.emplace_back("print_overlapped_ms", buf);
    }
    if (rc != 0) std::fprintf(stderr, "input error: %s\n", error.c_str());
  }
  return rc;
}

}  // namespace moc
