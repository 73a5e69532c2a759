// `final` — the CLI, behaviour-compatible with the reference binary (main.c:46-244):
//     mpiexec -np N ./final < inputX.txt   ->   "#i: score: S, n: N, k: K" per Seq2, input order.
//
// Flow (reference call stacks E2/E3), re-designed:
//   1. MPI bootstrap; rank -> GPU by node-local rank (reference: every rank on GPU 0, B14).
//   2. Root reads + parses stdin in bulk (OpenMP tokeniser; reference: racy parallel fscanf, B2).
//   3. Exact-count header/Seq1 broadcast (reference: 16 ints into int[4], B3).
//   4. Cost-balanced contiguous partition, valid for any -np (reference: B4/B5/B6).
//   5. Distribution by transport:
//        shm  — root parses once into an MPI shared window; each rank DMAs its own slice over its own
//               PCIe link and writes results back in place (single node; no payload copies at all);
//        rccl — root uploads, RCCL grouped send/recv scatters slices over xGMI, results gathered back;
//        mpi  — host Scatterv/Gatherv (CPU backend, or GPU ranks without a shared window).
//   6. Every rank runs its engine (HIP kernels, or the OpenMP CPU engine), root prints in order.
// Any error on any rank -> message + MPI_Abort (reference: exit(1) without abort, peers hang, B11).
#include <hip/hip_runtime_api.h>
#include <omp.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "moc/comm.hpp"
#include "moc/cpu_engine.hpp"
#include "moc/hip_engine.hpp"
#include "moc/io.hpp"
#include "moc/partition.hpp"
#include "moc/problem.hpp"
#include "moc/runtime/device.hpp"
#include "moc/runtime/flags.hpp"
#include "moc/runtime/hip_check.hpp"
#include "moc/runtime/log.hpp"
#include "moc/runtime/timer.hpp"
#include "moc/score_table.hpp"

using namespace moc;

namespace {

const char* kUsage =
    "usage: mpiexec -np N ./final [options] < input.txt\n"
    "  --backend=auto|hip|cpu      compute engine (auto: hip when a GPU is visible)\n"
    "  --transport=auto|shm|rccl|mpi   record distribution (auto: shm on one node, else rccl/mpi)\n"
    "  --semantics=reference|spec  candidate set (spec adds the un-mutated final offset, bug B8)\n"
    "  --partition=cost|even       rank decomposition\n"
    "  --timing                    per-phase JSON on stderr (root)\n"
    "  --strict-limits             enforce |Seq1|<=3000, |Seq2|<=2000 (PDF p.5-6)\n"
    "  --device=K                  force device K (default: node-local rank %% devices)\n"
    "  --chunk-records=R --chunk-bytes=B   pipeline chunk sizes\n"
    "  --threads=T                 OpenMP threads (default: OMP_NUM_THREADS / all)\n"
    "  --log-level=error|warn|info|debug\n"
    "  --inject-fault=PHASE[:RANK] test hook: fail at parse|bcast|distribute|compute|gather\n"
    "every flag can also be given as environment variable MOC_<FLAG> (e.g. MOC_BACKEND=cpu)\n";

const std::vector<std::string> kKnown = {"backend", "transport", "semantics", "partition", "timing",
                                         "strict-limits", "device", "chunk-records", "chunk-bytes", "threads",
                                         "log-level", "inject-fault", "help"};

struct Header {
  int32_t w[4];
  int32_t semantics;
  int32_t status;  // 0 ok, else parse error on root
  int64_t L1;
  int64_t n;
  int64_t total_chars;
};

struct FaultHook {
  std::string phase;
  int rank = 0;
  void at(const char* p, int my_rank) const {
    if (!phase.empty() && phase == p && my_rank == rank)
      throw Error(std::string("injected fault at phase '") + p + "'");
  }
};

std::string to_lower(std::string s) {
  for (auto& c : s) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  return s;
}

// Runs the selected engine on one contiguous slice (host buffers).
struct RankEngine {
  bool gpu = false;
  std::unique_ptr<HipEngine> hip;
  ScoreTable table{};
  std::vector<uint8_t> seq1;
  Semantics sem = Semantics::Reference;
  int threads = 0;

  void set_problem(const Weights& w, const std::vector<uint8_t>& s1, Semantics s) {
    sem = s;
    seq1 = s1;
    table = ScoreTable::build(w);
    if (gpu) hip->set_problem(w, s1.data(), static_cast<int64_t>(s1.size()), s);
  }
  void solve(const uint8_t* codes, const int64_t* offsets, int64_t n, Result* out) {
    if (n <= 0) return;
    if (gpu) {
      hip->solve(codes, offsets, n, out);
      return;
    }
    RecordBatch b;
    b.codes.assign(codes + offsets[0], codes + offsets[n]);
    b.offsets.resize(static_cast<size_t>(n) + 1);
    for (int64_t i = 0; i <= n; ++i) b.offsets[i] = offsets[i] - offsets[0];
    solve_batch_cpu(table, seq1.data(), static_cast<int64_t>(seq1.size()), b, out, sem, threads);
  }
};

int run(MpiContext& ctx, int argc, char** argv) {
  Flags flags(argc, argv);
  if (flags.get_bool("help", false)) {
    if (ctx.rank == kRoot) std::fputs(kUsage, stdout);
    return 0;
  }
  auto unknown = flags.unknown(kKnown);
  if (!unknown.empty()) {
    if (ctx.rank == kRoot) std::fprintf(stderr, "unknown flag --%s\n%s", unknown[0].c_str(), kUsage);
    return 2;
  }
  log_set_level(flags.get("log-level", "warn"));
  const int threads = static_cast<int>(flags.get_int("threads", 0));
  if (threads > 0) omp_set_num_threads(threads);
  FaultHook fault;
  {
    std::string f = flags.get("inject-fault", "");
    auto colon = f.find(':');
    fault.phase = f.substr(0, colon);
    if (colon != std::string::npos) fault.rank = std::stoi(f.substr(colon + 1));
  }
  const bool timing = flags.get_bool("timing", false);
  const std::string sem_s = to_lower(flags.get("semantics", "reference"));
  if (sem_s != "reference" && sem_s != "spec") throw Error("--semantics must be reference|spec");
  const Semantics sem = sem_s == "spec" ? Semantics::Spec : Semantics::Reference;

  // ---- 1. engine / device selection (per rank), transport agreement (collective)
  std::string backend = to_lower(flags.get("backend", "auto"));
  const int ndev = (backend == "cpu") ? 0 : device_count();
  if (backend == "hip" && ndev == 0) throw Error("--backend=hip but no HIP device is visible");
  RankEngine eng;
  eng.threads = threads;
  eng.gpu = ndev > 0;
  int device = -1;
  if (eng.gpu) {
    device = select_device(ctx.local_rank, static_cast<int>(flags.get_int("device", -1)));
    EngineOptions eo;
    eo.device = device;
    eo.chunk_records = flags.get_int("chunk-records", eo.chunk_records);
    eo.chunk_bytes = flags.get_int("chunk-bytes", eo.chunk_bytes);
    eng.hip = std::make_unique<HipEngine>(eo);
  }
  int all_gpu = eng.gpu ? 1 : 0;
  MPI_Allreduce(MPI_IN_PLACE, &all_gpu, 1, MPI_INT, MPI_MIN, ctx.world);
  std::string transport = to_lower(flags.get("transport", "auto"));
  if (transport == "auto") transport = ctx.single_node() ? "shm" : (all_gpu ? "rccl" : "mpi");
  if (transport == "shm" && !ctx.single_node()) throw Error("--transport=shm needs all ranks on one node");
  if (transport == "rccl" && !all_gpu) throw Error("--transport=rccl needs a GPU on every rank");
  if (transport != "shm" && transport != "rccl" && transport != "mpi") throw Error("unknown --transport " + transport);
  MOC_LOG_INFO("rank %d/%d host %s local %d/%d engine=%s device=%d transport=%s", ctx.rank, ctx.size,
               ctx.hostname.c_str(), ctx.local_rank, ctx.local_size, eng.gpu ? "hip" : "cpu", device,
               transport.c_str());

  PhaseTimer pt;
  Stopwatch total;
  total.start();

  // ---- 2. root reads + parses
  Problem prob;
  Header h{};
  std::string parse_error;
  if (ctx.rank == kRoot) {
    pt.begin("parse");
    try {
      fault.at("parse", ctx.rank);
      std::vector<char> text = read_stream(stdin);
      ParseOptions po;
      po.strict_limits = flags.get_bool("strict-limits", false);
      prob = parse_problem(text.data(), text.size(), po);
    } catch (const std::exception& e) {
      parse_error = e.what();
      h.status = 1;
    }
    pt.end();
    for (int i = 0; i < 4; ++i) h.w[i] = prob.weights.w[i];
    h.semantics = static_cast<int32_t>(sem);
    h.L1 = prob.L1();
    h.n = prob.seq2.size();
    h.total_chars = prob.seq2.total_chars();
  }

  // ---- 3. header + Seq1 broadcast (exact counts)
  pt.begin("bcast");
  fault.at("bcast", ctx.rank);
  bcast_bytes(&h, sizeof h, kRoot, ctx.world);
  if (h.status != 0) {
    if (ctx.rank == kRoot) std::fprintf(stderr, "input error: %s\n", parse_error.c_str());
    return 1;
  }
  for (int i = 0; i < 4; ++i) prob.weights.w[i] = h.w[i];
  prob.seq1.resize(static_cast<size_t>(h.L1));
  bcast_bytes(prob.seq1.data(), h.L1, kRoot, ctx.world);
  eng.set_problem(prob.weights, prob.seq1, sem);
  pt.end();

  // ---- 4. partition (root computes, everybody gets the bounds)
  const int p = ctx.size;
  std::vector<int64_t> bounds(static_cast<size_t>(p) + 1, 0);
  if (ctx.rank == kRoot) {
    std::vector<int64_t> len(static_cast<size_t>(h.n));
    for (int64_t i = 0; i < h.n; ++i) len[i] = prob.seq2.length(i);
    const std::string mode = to_lower(flags.get("partition", "cost"));
    CostModel cm = all_gpu ? CostModel{1.0, 200.0, 2400.0} : CostModel{1.0, 4.0, 64.0};
    bounds = mode == "even" ? partition_even(h.n, p) : partition_by_cost(len.data(), h.n, h.L1, p, cm);
  }
  bcast_bytes(bounds.data(), sizeof(int64_t) * (p + 1), kRoot, ctx.world);
  const int64_t my_b = bounds[ctx.rank], my_n = bounds[ctx.rank + 1] - my_b;

  // ---- 5/6. distribute + compute (+ gather)
  std::vector<Result> results;  // root: all N (mpi/rccl transports)
  const Result* print_from = nullptr;
  std::unique_ptr<SharedWindow> win;
  double compute_ms = 0;

  if (transport == "shm") {
    // layout: offsets[(N+1)] | results[N] | codes[total]   (8-byte aligned sections)
    const int64_t off_bytes = 8 * (h.n + 1);
    const int64_t res_bytes = ((12 * h.n) + 7) & ~int64_t{7};
    pt.begin("distribute");
    win = std::make_unique<SharedWindow>(ctx, off_bytes + res_bytes + h.total_chars);
    int64_t* w_offs = reinterpret_cast<int64_t*>(win->base());
    Result* w_res = reinterpret_cast<Result*>(win->base() + off_bytes);
    uint8_t* w_codes = reinterpret_cast<uint8_t*>(win->base() + off_bytes + res_bytes);
    if (ctx.rank == kRoot) {
      const int64_t* src_off = prob.seq2.offsets.data();
      const uint8_t* src_codes = prob.seq2.codes.data();
#pragma omp parallel
      {
        const int t = omp_get_thread_num(), nt = omp_get_num_threads();
        const int64_t cb = h.total_chars * t / nt, ce = h.total_chars * (t + 1) / nt;
        std::memcpy(w_codes + cb, src_codes + cb, static_cast<size_t>(ce - cb));
        const int64_t ob = (h.n + 1) * t / nt, oe = (h.n + 1) * (t + 1) / nt;
        std::memcpy(w_offs + ob, src_off + ob, static_cast<size_t>(oe - ob) * 8);
      }
      prob.seq2 = RecordBatch{};  // the window is now the only copy
    }
    fault.at("distribute", ctx.rank);
    win->fence();
    pt.end();
    pt.begin("compute");
    fault.at("compute", ctx.rank);
    Stopwatch sw;
    sw.start();
    eng.solve(w_codes, w_offs + my_b, my_n, w_res + my_b);
    sw.stop();
    compute_ms = sw.total_ms();
    pt.end();
    pt.begin("gather");
    fault.at("gather", ctx.rank);
    win->fence();
    pt.end();
    print_from = w_res;
  } else if (transport == "mpi") {
    pt.begin("distribute");
    fault.at("distribute", ctx.rank);
    std::vector<int64_t> lcount(p), ldispl(p), ccount(p), cdispl(p);
    for (int r = 0; r < p; ++r) {
      lcount[r] = 8 * (bounds[r + 1] - bounds[r]);
      ldispl[r] = 8 * bounds[r];
    }
    std::vector<int64_t> lengths;
    if (ctx.rank == kRoot) {
      lengths.resize(static_cast<size_t>(h.n));
      for (int64_t i = 0; i < h.n; ++i) lengths[i] = prob.seq2.length(i);
      for (int r = 0; r < p; ++r) {
        ccount[r] = prob.seq2.offsets[bounds[r + 1]] - prob.seq2.offsets[bounds[r]];
        cdispl[r] = prob.seq2.offsets[bounds[r]];
      }
    }
    bcast_bytes(ccount.data(), 8 * p, kRoot, ctx.world);
    std::vector<int64_t> my_len(static_cast<size_t>(my_n));
    scatterv_bytes(lengths.data(), lcount, ldispl, my_len.data(), kRoot, ctx.world);
    std::vector<uint8_t> my_codes(static_cast<size_t>(ccount[ctx.rank]));
    scatterv_bytes(prob.seq2.codes.data(), ccount, cdispl, my_codes.data(), kRoot, ctx.world);
    std::vector<int64_t> my_off(static_cast<size_t>(my_n) + 1, 0);
    for (int64_t i = 0; i < my_n; ++i) my_off[i + 1] = my_off[i] + my_len[i];
    pt.end();
    pt.begin("compute");
    fault.at("compute", ctx.rank);
    std::vector<Result> mine(static_cast<size_t>(my_n));
    Stopwatch sw;
    sw.start();
    eng.solve(my_codes.data(), my_off.data(), my_n, mine.data());
    sw.stop();
    compute_ms = sw.total_ms();
    pt.end();
    pt.begin("gather");
    fault.at("gather", ctx.rank);
    std::vector<int64_t> rcount(p), rdispl(p);
    for (int r = 0; r < p; ++r) {
      rcount[r] = 12 * (bounds[r + 1] - bounds[r]);
      rdispl[r] = 12 * bounds[r];
    }
    if (ctx.rank == kRoot) results.resize(static_cast<size_t>(h.n));
    gatherv_bytes(mine.data(), 12 * my_n, results.data(), rcount, rdispl, kRoot, ctx.world);
    pt.end();
    print_from = results.data();
  } else {  // rccl
    RcclComm nccl(ctx, device);
    hipStream_t s = eng.hip->compute_stream();
    pt.begin("distribute");
    fault.at("distribute", ctx.rank);
    // counts in bytes for codes and (absolute) offsets; each rank receives n_r+1 offsets
    std::vector<int64_t> ccount(p), cdispl(p), ocount(p), odispl(p);
    if (ctx.rank == kRoot) {
      for (int r = 0; r < p; ++r) {
        ccount[r] = prob.seq2.offsets[bounds[r + 1]] - prob.seq2.offsets[bounds[r]];
        cdispl[r] = prob.seq2.offsets[bounds[r]];
      }
    }
    bcast_bytes(ccount.data(), 8 * p, kRoot, ctx.world);
    bcast_bytes(cdispl.data(), 8 * p, kRoot, ctx.world);
    for (int r = 0; r < p; ++r) {
      ocount[r] = 8 * (bounds[r + 1] - bounds[r] + 1);
      odispl[r] = 8 * bounds[r];
    }
    uint8_t *d_all_codes = nullptr, *d_codes = nullptr;
    int64_t *d_all_offs = nullptr, *d_offs = nullptr;
    Result *d_out = nullptr, *d_all_out = nullptr;
    if (ctx.rank == kRoot) {
      MOC_HIP_CHECK(hipMalloc(&d_all_codes, std::max<int64_t>(h.total_chars, 1)));
      MOC_HIP_CHECK(hipMalloc(&d_all_offs, 8 * (h.n + 1)));
      MOC_HIP_CHECK(hipMalloc(&d_all_out, std::max<int64_t>(12 * h.n, 4)));
      MOC_HIP_CHECK(hipMemcpyAsync(d_all_codes, prob.seq2.codes.data(), h.total_chars, hipMemcpyHostToDevice, s));
      MOC_HIP_CHECK(hipMemcpyAsync(d_all_offs, prob.seq2.offsets.data(), 8 * (h.n + 1), hipMemcpyHostToDevice, s));
    }
    MOC_HIP_CHECK(hipMalloc(&d_codes, std::max<int64_t>(ccount[ctx.rank], 1)));
    MOC_HIP_CHECK(hipMalloc(&d_offs, 8 * (my_n + 1)));
    MOC_HIP_CHECK(hipMalloc(&d_out, std::max<int64_t>(12 * my_n, 4)));
    nccl.scatterv(d_all_codes, ccount, cdispl, d_codes, kRoot, s);
    nccl.scatterv(d_all_offs, ocount, odispl, d_offs, kRoot, s);
    std::vector<int64_t> h_offs(static_cast<size_t>(my_n) + 1);
    MOC_HIP_CHECK(hipMemcpyAsync(h_offs.data(), d_offs, 8 * (my_n + 1), hipMemcpyDeviceToHost, s));
    MOC_HIP_CHECK(hipStreamSynchronize(s));
    nccl.check_async();
    pt.end();
    pt.begin("compute");
    fault.at("compute", ctx.rank);
    Stopwatch sw;
    sw.start();
    // d_codes holds this rank's letters starting at absolute offset h_offs[0]
    if (my_n > 0) eng.hip->solve_device(d_codes - h_offs[0], d_offs, h_offs.data(), my_n, d_out, s);
    MOC_HIP_CHECK(hipStreamSynchronize(s));
    sw.stop();
    compute_ms = sw.total_ms();
    pt.end();
    pt.begin("gather");
    fault.at("gather", ctx.rank);
    std::vector<int64_t> rcount(p), rdispl(p);
    for (int r = 0; r < p; ++r) {
      rcount[r] = 12 * (bounds[r + 1] - bounds[r]);
      rdispl[r] = 12 * bounds[r];
    }
    nccl.gatherv(d_out, 12 * my_n, d_all_out, rcount, rdispl, kRoot, s);
    if (ctx.rank == kRoot) {
      results.resize(static_cast<size_t>(h.n));
      MOC_HIP_CHECK(hipMemcpyAsync(results.data(), d_all_out, 12 * h.n, hipMemcpyDeviceToHost, s));
    }
    MOC_HIP_CHECK(hipStreamSynchronize(s));
    nccl.check_async();
    pt.end();
    (void)hipFree(d_all_codes);
    (void)hipFree(d_all_offs);
    (void)hipFree(d_all_out);
    (void)hipFree(d_codes);
    (void)hipFree(d_offs);
    (void)hipFree(d_out);
    print_from = results.data();
  }

  // ---- print (root) + timing
  double max_compute = compute_ms;
  MPI_Reduce(ctx.rank == kRoot ? MPI_IN_PLACE : &max_compute, &max_compute, 1, MPI_DOUBLE, MPI_MAX, kRoot, ctx.world);
  if (ctx.rank == kRoot) {
    pt.begin("print");
    write_results(stdout, print_from, h.n, 0);
    pt.end();
    total.stop();
    if (timing) {
      const double wall_s = total.total_ms() / 1e3;
      std::fprintf(stderr,
                   "{\"timing\": %s, \"ranks\": %d, \"nodes\": %d, \"engine\": \"%s\", \"transport\": \"%s\", "
                   "\"records\": %lld, \"elements\": %lld, \"max_rank_compute_ms\": %.3f, \"wall_s\": %.6f, "
                   "\"elements_per_s\": %.1f}\n",
                   pt.json().c_str(), ctx.size, ctx.node_count, eng.gpu ? "hip" : "cpu", transport.c_str(),
                   static_cast<long long>(h.n), static_cast<long long>(h.total_chars), max_compute, wall_s,
                   wall_s > 0 ? h.total_chars / wall_s : 0.0);
    }
  }
  MPI_Barrier(ctx.world);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  MpiContext ctx(&argc, &argv);
  int rc = 0;
  try {
    rc = run(ctx, argc, argv);
  } catch (const std::exception& e) {
    ctx.abort(3, e.what());
  }
  return rc;
}
