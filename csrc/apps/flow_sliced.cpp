// Bulk job on one node, records split into contiguous rank slices (transport shm, partition cost|even).
// Every rank encodes its OWN slice straight from the node-shared input text into its own buffers, in the
// wire formats its engine streams (SURVEY.md §7.3 / moc/wire.hpp):
//   GPU rank: P33 letters (56 per 33 bytes) + 3/4/8-bit or base-6 lengths + sparse offsets (1 per 64
//             records) in private, huge-page memory on its GPU's NUMA node, page-locked (only this slice),
//             results in the narrowest format (R2/R4/R8/R12) in this rank's segment of a node-shared window;
//   CPU rank: byte letters + CSR offsets, results as R12.
// Pass 1 (token/letter counts) is cooperative: each rank counts a share of the text's chunks and the
// counts are all-gathered, so every rank holds the same chunk table and computes its own bounds from it
// (BulkParser::cost_split) without a further collective. The root prints from every rank's result segment
// in place (reference: MPI_Scatter of 2000-byte records + 3 MPI_Gathers, main.c:174,195-197).
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>

#include "job.hpp"
#include "moc/runtime/host_region.hpp"
#include "moc/runtime/log.hpp"

namespace moc {

void run_sliced(JobCore& job, BulkParser& parser, int64_t first_index, SharedWindow* text_win, uvector<char>* text) {
  const MpiContext& ctx = job.ctx;
  PhaseTimer& pt = job.pt;
  RankEngine& eng = job.eng;
  const int p = ctx.size, r = ctx.rank;
  ++job.batches;
  job.first_index = first_index;
  const int64_t L1 = static_cast<int64_t>(eng.seq1.size());
  const bool gpu = eng.gpu;
  const int numa = gpu ? eng.hip->numa_node() : -1;

  const CostModel cost_model = job.cost_model();
  // ---- pass 1, cooperative
  pt.begin("count");
  const int64_t area = parser.area_bytes();
  const int nch = static_cast<int>(std::clamp<int64_t>(std::max(area >> 20, std::min<int64_t>(area >> 16, 64 * p)), 1,
                                                       int64_t{1} << 14));
  std::vector<int64_t> starts = parser.chunk_starts(nch);
  std::vector<int64_t> tk(static_cast<size_t>(nch)), ch(static_cast<size_t>(nch));
  {
    std::vector<int> cnt(p), dsp(p);
    for (int q = 0; q < p; ++q) {
      dsp[q] = static_cast<int>(int64_t{nch} * q / p);
      cnt[q] = static_cast<int>(int64_t{nch} * (q + 1) / p) - dsp[q];
    }
    parser.count_chunks(starts, dsp[r], dsp[r] + cnt[r], tk.data() + dsp[r], ch.data() + dsp[r]);
    MPI_Request rq[2];
    mpi_check(MPI_Iallgatherv(MPI_IN_PLACE, 0, MPI_DATATYPE_NULL, tk.data(), cnt.data(), dsp.data(), MPI_INT64_T,
                              ctx.world, &rq[0]),
              "MPI_Iallgatherv");
    mpi_check(MPI_Iallgatherv(MPI_IN_PLACE, 0, MPI_DATATYPE_NULL, ch.data(), cnt.data(), dsp.data(), MPI_INT64_T,
                              ctx.world, &rq[1]),
              "MPI_Iallgatherv");
    std::vector<MPI_Request> reqs(rq, rq + 2);
    mpi_wait_all(reqs, "MPI_Iallgatherv (pass-1 chunk counts)");
    // inputs up to 256 MiB also get exact chunk costs (a token walk) for the bounds: few, coarse chunks
    // of records of very different lengths are what the mean-length estimate gets wrong
    if (job.partition != "even" && p > 1 && area <= (int64_t{256} << 20)) {
      std::vector<double> costs(static_cast<size_t>(nch));
      parser.chunk_costs(starts, dsp[r], dsp[r] + cnt[r], cost_model, costs.data() + dsp[r]);
      MPI_Request r;
      mpi_check(MPI_Iallgatherv(MPI_IN_PLACE, 0, MPI_DATATYPE_NULL, costs.data(), cnt.data(), dsp.data(), MPI_DOUBLE,
                                ctx.world, &r),
                "MPI_Iallgatherv");
      mpi_wait(r, "MPI_Iallgatherv (chunk costs)");
      parser.set_chunk_costs(std::move(costs));
    }
  }
  try {
    parser.set_chunks(std::move(starts), tk.data(), ch.data());
  } catch (const std::exception& e) {
    throw InputError(e.what());
  }
  const int64_t n_all = parser.count();
  first_index = std::min(first_index, n_all);
  job.records += n_all - first_index;
  pt.end();

  // ---- this rank's slice
  pt.begin("bounds");
  int64_t b0, b1;
  if (job.partition == "even") {
    b0 = first_index + (n_all - first_index) * r / p;
    b1 = first_index + (n_all - first_index) * (r + 1) / p;
  } else {
    b0 = parser.cost_split(first_index, r, p, cost_model);
    b1 = std::max(b0, parser.cost_split(first_index, r + 1, p, cost_model));
  }
  const AreaSlice slice = parser.slice(b0, b1);
  const int64_t n = slice.records;
  pt.end();

  // ---- fill: every rank encodes its slice (GPU ranks guess the narrow form from the mean length)
  pt.begin("fill");
  job.fault.at("distribute", r);
  bool narrow = gpu && n > 0 && L1 <= 200 && slice.letters <= 64 * n;
  // GPU ranks: one NUMA-local region for the wire batch, letters | offsets | lengths (one page-lock
  // registration for the slice: each costs milliseconds whatever its size)
  HostRegion wire, len16;
  auto al64 = [](int64_t x) { return (x + 63) & ~int64_t{63}; };
  int64_t off_bytes = 0, len_at = 0;  // the offsets' and the lengths' byte offsets in `wire`
  int letters_pack = 5;  // GPU ranks: 33 = P33 fields, 5 = 5-bit packed
  int64_t letter_bytes = 0;
  RecordBatch cpu_batch;
  FillReport rep;
  if (n > 0) {
    if (!gpu) {
      cpu_batch.codes.resize(static_cast<size_t>(slice.letters));
      cpu_batch.offsets.resize(static_cast<size_t>(n) + 1);
      rep = parser.fill_slice(slice, cpu_batch.codes.data(), nullptr, cpu_batch.offsets.data());
    } else {
      // letters as P33 fields (4.714 bits each) for the streaming kernel, else 5-bit packed
      auto dense_form = [&] {
        letters_pack = 5;
        letter_bytes = packed5_bytes(slice.letters);
        off_bytes = al64(letter_bytes + 16);
        wire = HostRegion(static_cast<size_t>(off_bytes + 8 * (n + 1)), numa);
        rep = parser.fill_slice(slice, nullptr, wire.as<uint8_t>(), reinterpret_cast<int64_t*>(wire.data() + off_bytes));
      };
      if (narrow) {
        const int pack = 33;
        letters_pack = pack;
        letter_bytes = packed33_bytes(slice.letters);
        off_bytes = al64(letter_bytes + 16);
        len_at = off_bytes + al64(8 * sparse_count(n, kSparseShift));
        wire = HostRegion(static_cast<size_t>(len_at + al64(n + 16)), numa);  // lengths: <= 1 byte each
        len16 = HostRegion(2 * static_cast<size_t>(n), numa);
        rep = parser.fill_slice(slice, nullptr, wire.as<uint8_t>(), nullptr,
                                reinterpret_cast<int64_t*>(wire.data() + off_bytes), len16.as<uint16_t>(), pack);
        // the engine's answer for the lengths seen (waits for its start-up, its own phase): a wrong guess
        // re-encodes the slice as 5-bit letters + CSR offsets NOW, while the input text is still mapped —
        // every rank releases its share of the node-shared text after the report exchange below
        pt.begin("engine_wait");
        const bool streams = rep.max_len <= 255 && eng.hip->streams_packed(rep.min_len, rep.max_len);
        pt.begin("fill");
        if (!streams) {
          narrow = false;
          len16 = HostRegion();
          dense_form();
        }
      } else {
        dense_form();
      }
    }
  }
  // the job's first input error (the one a sequential reader meets first) on every rank
  {
    int64_t mine[7] = {rep.min_len, rep.max_len, rep.bad_record, rep.long_record, rep.long_len, rep.cells,
                       slice.letters};
    std::vector<int64_t> all(static_cast<size_t>(7 * p));
    job.allgather_i64(mine, 7, all.data());
    FillReport whole;
    for (int q = 0; q < p; ++q) {
      const int64_t* x = all.data() + 7 * q;
      job.chars += x[6];
      whole.min_len = std::min(whole.min_len, x[0]);
      whole.max_len = std::max(whole.max_len, x[1]);
      if (x[2] >= 0 && (whole.bad_record < 0 || x[2] < whole.bad_record)) whole.bad_record = x[2];
      if (x[3] >= 0 && (whole.long_record < 0 || x[3] < whole.long_record)) {
        whole.long_record = x[3];
        whole.long_len = x[4];
      }
      whole.cells += x[5];
    }
    job.cells += whole.cells;
    // every slice is encoded in its final form: the helpers return the node-shared input text's pages to
    // the OS while their GPUs search and the root prints
    if (text_win) text_win->release_shares(ctx);
    try {
      parser.check(whole);
    } catch (const std::exception& e) {
      throw InputError(e.what());
    }
  }
  pt.end();
  // GPU ranks: the wire form the engine streams
  pt.begin("wire");
  WireBatch wb;
  ResultFormat fmt = ResultFormat::R12;
  if (gpu && n > 0) {
    wb.letters = wire.as<uint8_t>();
    wb.packed33 = letters_pack == 33;
    wb.packed5 = letters_pack == 5;
    wb.n = n;
    wb.min_l2 = rep.min_len;
    wb.max_l2 = rep.max_len;
    wb.offsets = reinterpret_cast<const int64_t*>(wire.data() + off_bytes);
    if (narrow) {
      const int bits = narrow_length_bits(rep.min_len, rep.max_len);
      pack_lengths16(len16.as<uint16_t>(), n, bits, rep.min_len, wire.as<uint8_t>() + len_at);
      len16.set_releaser(&job.rel);  // its pages go back to the OS on the releaser thread
      len16 = HostRegion();
      wb.off_shift = kSparseShift;
      wb.lengths = wire.as<uint8_t>() + len_at;
      wb.len_bits = bits;
      wb.len_base = bits == 8 ? 0 : rep.min_len;
    }
    fmt = eng.hip->result_format(rep.min_len, rep.max_len);
  }
  pt.end();

  // ---- results: this rank's segment of a node-shared window, printed by the root; or, with
  // --parallel-print, several ranks and an --output file, every rank prints its own rows into the file
  // (formatting split over the ranks, no result window). Measured on one MI355X box at 2 ranks the root
  // print was faster (0.52 vs 0.76 s for 4.6 GB: the ranks' writes contend for the one file and their
  // threads for the cores), so it is opt-in.
  const int fb = result_bytes(fmt);
  pt.begin("results");
  int64_t dp[2] = {0, 0};  // {distributed print, the file offset of the first row}
  if (r == kRoot && p > 1 && job.out != stdout && job.flags.get_bool("parallel-print", false)) {
    struct stat st {};
    const int fd = fileno(job.out);
    const int fl = fcntl(fd, F_GETFL);
    std::fflush(job.out);
    if (fl >= 0 && !(fl & O_APPEND) && fstat(fd, &st) == 0 && S_ISREG(st.st_mode)) {
      dp[0] = 1;
      dp[1] = static_cast<int64_t>(std::ftell(job.out));
    }
  }
  bcast_bytes(dp, sizeof dp, kRoot, ctx.world);
  std::unique_ptr<SegmentWindow> seg;
  HostRegion own;
  char* res_mine = nullptr;
  if (dp[0]) {
    own = HostRegion(static_cast<size_t>(std::max<int64_t>(fb * n, 16)), numa);
    own.set_releaser(&job.rel);
    res_mine = own.data();
  } else {
    seg = std::make_unique<SegmentWindow>(ctx, fb * n, numa);
    seg->set_releaser(&job.rel);
    res_mine = seg->mine();
  }
  pt.end();
  // GPU ranks page-lock this slice's pieces only (the registration faults in and locks every page)
  pt.begin("pin");
  Stopwatch pin_sw;
  pin_sw.start();
  if (gpu && n > 0 && job.pin_window) {
    try {
      auto pin = [&](const void* ptr, int64_t bytes) {
        if (ptr && bytes > 0) {
          eng.hip->pin(ptr, static_cast<size_t>(bytes));
          job.pinned_bytes += bytes;
        }
      };
      // letters, offsets and lengths at once: the region's used prefix (the lengths took their narrow size)
      pin(wire.data(), narrow ? len_at + wb.length_bytes() : off_bytes + 8 * (n + 1));
      pin(res_mine, fb * n);
    } catch (const std::exception& e) {
      MOC_LOG_WARN("could not page-lock this rank's slice (%s); using the staged pipeline", e.what());
    }
  }
  pin_sw.stop();
  pt.end();
  pt.begin("compute");
  job.fault.at("compute", r);
  Stopwatch sw;
  sw.start();
  GpuSolveStats gs;
  if (n > 0) {
    if (gpu) {
      eng.hip->solve_wire(wb, res_mine, fmt);
      gs = eng.hip->last_stats();
      eng.kernel_ms += gs.kernel_ms;
      job.h2d_bytes += gs.h2d_bytes;
      job.d2h_bytes += gs.d2h_bytes;
    } else {
      solve_batch_cpu(eng.table, eng.seq1.data(), L1, cpu_batch, reinterpret_cast<Result*>(res_mine), eng.sem,
                      eng.threads);
    }
  }
  sw.stop();
  job.compute_ms += sw.total_ms();
  pt.end();
  // inputs nobody reads any more go back to the OS while the root prints: their registrations are
  // dropped first (the releaser runs its tasks in order), then the pages
  pt.begin("drop");
  if (gpu) job.rel.defer(eng.hip->detach_pins());
  wire.set_releaser(&job.rel);
  { HostRegion drop = std::move(wire); }
  if (!cpu_batch.codes.empty()) {
    auto spent = std::make_shared<RecordBatch>(std::move(cpu_batch));
    job.rel.defer([spent]() mutable { spent.reset(); });
  }
  pt.end();

  // ---- every rank's result run -> root, which prints them in order straight from the segments
  pt.begin("gather");
  job.fault.at("gather", r);
  int64_t info[8] = {n,           static_cast<int64_t>(fmt), gs.r2.smin, gs.r2.kw, gs.r2.j, job.pinned_bytes, job.h2d_bytes,
                     static_cast<int64_t>(pin_sw.total_ms() * 1000.0)};
  std::vector<int64_t> infos(static_cast<size_t>(8 * p));
  job.allgather_i64(info, 8, infos.data());
  if (seg) seg->fence();
  pt.end();
  if (r == kRoot) {  // --timing: what every rank owned, page-locked and moved
    job.rank_pinned.assign(static_cast<size_t>(p), 0);
    job.rank_h2d.assign(static_cast<size_t>(p), 0);
    job.rank_records.assign(static_cast<size_t>(p), 0);
    job.rank_pin_us.assign(static_cast<size_t>(p), 0);
    for (int q = 0; q < p; ++q) {
      const int64_t* x = infos.data() + 8 * q;
      job.rank_records[q] = x[0];
      job.rank_pinned[q] = x[5];
      job.rank_h2d[q] = x[6];
      job.rank_pin_us[q] = x[7];
    }
    // a private input text goes back to the OS while the results print
    if (text && !text->empty()) {
      auto t = std::make_shared<uvector<char>>(std::move(*text));
      job.rel.defer([t]() mutable { t.reset(); });
      *text = uvector<char>();
    }
  }
  if (dp[0]) {  // every rank: its rows at its offset of the output file (sizes all-gathered first)
    pt.begin("print");
    const std::vector<ResultRun> mine = {ResultRun{res_mine, fmt, gs.r2, n}};
    int64_t bytes = formatted_bytes(mine, b0);
    std::vector<int64_t> sizes(static_cast<size_t>(p));
    job.allgather_i64(&bytes, 1, sizes.data());
    int64_t at = dp[1], total = 0;
    for (int q = 0; q < p; ++q) {
      if (q < r) at += sizes[q];
      total += sizes[q];
    }
    int fd = r == kRoot ? fileno(job.out) : -1;
    if (r != kRoot && n > 0) {
      fd = ::open(job.flags.get("output", "").c_str(), O_WRONLY | O_CLOEXEC);
      if (fd < 0) throw Error("cannot open --output " + job.flags.get("output", "") + " on rank " + std::to_string(r));
    }
    if (n > 0) write_results_at(fd, at, mine, b0);
    if (r != kRoot && fd >= 0) ::close(fd);
    barrier(ctx.world, "MPI_Ibarrier (parallel print)");  // every row is in the file
    if (r == kRoot) std::fseek(job.out, static_cast<long>(dp[1] + total), SEEK_SET);
    pt.end();
    return;
  }
  if (r == kRoot) {
    std::vector<ResultRun> runs(static_cast<size_t>(p));
    for (int q = 0; q < p; ++q) {
      const int64_t* x = infos.data() + 8 * q;
      runs[q].data = seg->segment(q);
      runs[q].n = x[0];
      runs[q].fmt = static_cast<ResultFormat>(x[1]);
      runs[q].r2 = R2Params{static_cast<int32_t>(x[2]), static_cast<int32_t>(x[3]), static_cast<int32_t>(x[4])};
    }
    pt.begin("print");
    ScopedOmpThreads team(job.print_threads);  // the other ranks wait at the segments' fence
    write_results(job.out, runs, first_index);
    pt.end();
  }
  pt.begin("release");
  seg->fence();  // nobody unmaps a segment the root still prints from
  pt.end();
}

}  // namespace moc
