// `final` — the CLI, behaviour-compatible with the reference binary (main.c:46-244):
//     mpiexec -np N ./final < inputX.txt   ->   "#i: score: S, n: N, k: K" per Seq2, input order.
//
// Flow (reference call stacks E2/E3), re-designed:
//   1. MPI bootstrap; rank -> GPU by node-local rank or --device-map (reference: all ranks on GPU 0, B14).
//   2. Root reads + parses the input: in bulk (OpenMP tokeniser; reference: racy parallel fscanf, B2), or
//      in bounded batches (--batch-records, parse of batch b+1 overlapped with the search of batch b).
//   3. Exact-count header/Seq1 broadcast (reference: 16 ints into int[4], B3).
//   4. Decomposition (--partition):
//        cost/even — contiguous record ranges, cost-balanced by default, valid for any -np (B4/B5/B6);
//        offsets   — context parallel: every rank searches a share of EVERY record's
//                    offset range; one MAX all-reduce of packed 64-bit keys combines them (the Reduce the
//                    reference never had). For few huge records, or fewer records than GPUs.
//   5. Distribution by transport:
//        shm  — root parses once into an MPI shared window; each rank reads its slice over its own PCIe
//               link (zero-copy when the window is pinned) and writes results back in place;
//        rccl — root packs each rank's slice into its wire form, a pipeline overlaps packing, upload and
//               the RCCL send over xGMI, every rank searches in device memory, narrow results are gathered
//               (device_batch.cpp); rccl-emul runs that same driver over MPI on CPU ranks;
//        mpi  — host Scatterv/Gatherv (CPU backend, or GPU ranks without a shared window).
//   6. Every rank runs its engine (HIP kernels, or the OpenMP CPU engine), root prints in order.
// Any error on any rank -> message + MPI_Abort (reference: exit(1) without abort, peers hang, B11).
#include <dlfcn.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <omp.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <future>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "moc/comm.hpp"
#include "moc/cpu_engine.hpp"
#include "moc/device_comm.hpp"
#include "moc/mpi_device_comm.hpp"
#include "moc/gpu_rank.hpp"
#include "moc/io.hpp"
#include "moc/partition.hpp"
#include "moc/problem.hpp"
#include "moc/runtime/flags.hpp"
#include "moc/runtime/host_region.hpp"
#include "moc/runtime/log.hpp"
#include "moc/runtime/timer.hpp"
#include "moc/runtime/trace.hpp"
#include "moc/score_table.hpp"

using namespace moc;

namespace {

// --output is opened without O_TRUNC and cut to the written length at the end: truncating a non-empty file
// on ext4 (auto_da_alloc) makes its close start writeback of every page written since (0.23 s for 0.7 GB
// here), where a plain close returns at once.
FILE* open_output(const std::string& path) {
  const int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_CLOEXEC, 0666);
  if (fd < 0) return nullptr;
  FILE* f = fdopen(fd, "wb");
  if (!f) ::close(fd);
  return f;
}
int close_output(FILE* f) {
  int rc = std::fflush(f);
  struct stat st {};
  const long end = std::ftell(f);
  if (rc == 0 && end >= 0 && fstat(fileno(f), &st) == 0 && S_ISREG(st.st_mode) && st.st_size > end &&
      ftruncate(fileno(f), end) != 0)
    rc = -1;
  return std::fclose(f) != 0 || rc != 0 ? -1 : 0;
}

#ifndef MOC_BUILD_ID
#define MOC_BUILD_ID "src=unknown git=unknown"
#endif
// The sources this binary was built from (Makefile: a hash over csrc/ + Makefile, and the git commit):
// printed by --help and --timing so a test can tell a stale prebuilt binary from the checked-out source.
const char* kBuildId = MOC_BUILD_ID;

const char* kUsage =
    "usage: mpiexec -np N ./final [options] < input.txt\n"
    "  --backend=auto|hip|cpu      compute engine (auto: hip when a GPU is visible and the job has\n"
    "                              >= --gpu-min-cells cells per rank; default: 0.2 s of OpenMP work, i.e.\n"
    "                              0.08 G (records <= 32 letters) / 0.28 G (longer) cells per thread)\n"
    "  --gpu-prewarm-bytes=B       start the HIP runtime during the parse when the input file has >= B bytes\n"
    "                              (default 64 MiB; 0 = never)\n"
    "  --transport=auto|shm|rccl|rccl-emul|mpi   record distribution (auto: shm on one node, else rccl/mpi;\n"
    "                              rccl-emul: the rccl driver over MPI on CPU ranks)\n"
    "  --semantics=reference|spec  candidate set (spec adds the un-mutated final offset, bug B8)\n"
    "  --partition=cost|even|offsets   rank decomposition (offsets: split every record's offset range)\n"
    "  --collectives=auto|mpi|rccl the ranks' host-table collectives on the shm transport (auto = mpi: a few\n"
    "                              int64 per rank, where RCCL's communicator set-up costs 1.7-5.8 s; rccl:\n"
    "                              over xGMI, needs one GPU per rank)\n"
    "  --batch-records=B           streaming mode: parse/search/print B records at a time (0 = all at once)\n"
    "  --batch-chars=C             streaming mode: also cap a batch at C letters\n"
    "  --skip-records=S            start at record #S (resume a partially printed run)\n"
    "  --input=PATH                read PATH instead of stdin\n"
    "  --output=PATH               root writes the result lines to PATH (in parallel) instead of stdout,\n"
    "                              which mpiexec's proxies forward through a pipe\n"
    "  --parallel-print            with several ranks and --output: every rank writes its own rows\n"
    "  --timing                    per-phase JSON on stderr (root)\n"
    "  --strict-limits             enforce |Seq1|<=3000, |Seq2|<=2000 (PDF p.5-6)\n"
    "  --max-l1=L --max-l2=L       explicit length limits (0 = unlimited)\n"
    "  --device=K                  force device K (default: node-local rank %% devices)\n"
    "  --device-map=a,b,...        node-local rank i -> device map[i %% len]\n"
    "  --letters=p33|p24           letter code of GPU slices (p33: 7 letters per 33 bits; p24: 5 per 3 bytes)\n"
    "  --pin-window=0|1            page-lock the shm window so GPU ranks stream it zero-copy (default 1)\n"
    "  --chunk-records=R --chunk-bytes=B   pipeline chunk sizes\n"
    "  --threads=T                 OpenMP threads (default: OMP_NUM_THREADS / all)\n"
    "  --log-level=error|warn|info|debug\n"
    "  --inject-fault=PHASE[:RANK] test hook: fail at parse|bcast|distribute|compute|gather\n"
    "every flag can also be given as environment variable MOC_<FLAG> (e.g. MOC_BACKEND=cpu)\n";

const std::vector<std::string> kKnown = {
    "backend", "collectives", "parallel-print", "gpu-min-cells", "gpu-prewarm-bytes", "transport", "semantics", "partition", "batch-records", "batch-chars", "skip-records", "input",
    "output", "timing", "strict-limits", "max-l1", "max-l2", "device", "device-map", "letters", "pin-window", "chunk-records",
    "chunk-bytes", "threads", "log-level", "inject-fault", "help"};

struct Header {
  int32_t w[4];
  int32_t semantics;
  int32_t status;  // 0 ok, else input error on root
  int64_t L1;
  int64_t n_total;      // number_of_sequences
  int64_t first_index;  // --skip-records actually applied
  int64_t cells;        // search cells of the job (-1: unknown, streaming)
  int64_t text_bytes;   // bytes of the input text (sliced mode)
  int64_t mean_l2;      // mean record length (estimate; 0: unknown)
};

struct BatchHeader {
  int64_t n;
  int64_t total_chars;
  int32_t status;  // 0 ok, else input error on root
  int32_t pad;
};

// An input problem found after the header went out (deferred parsing into the shared window); raised on
// every rank after a status broadcast, so all of them leave the job the same way (exit code 1).
struct InputError : Error {
  using Error::Error;
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

std::vector<int> parse_int_list(const std::string& s) {
  std::vector<int> v;
  std::stringstream ss(s);
  std::string tok;
  while (std::getline(ss, tok, ','))
    if (!tok.empty()) v.push_back(std::stoi(tok));
  return v;
}

// Drops the first s records of a batch (bulk mode + --skip-records).
void drop_front(RecordBatch& b, int64_t s) {
  s = std::min<int64_t>(s, b.size());
  if (s <= 0) return;
  const int64_t c0 = b.offsets[s];
  b.codes.erase(b.codes.begin(), b.codes.begin() + c0);
  b.offsets.erase(b.offsets.begin(), b.offsets.begin() + s);
  for (auto& o : b.offsets) o -= c0;
}

// The GPU plugin (moc/gpu_rank.hpp): mpi_openmp_cuda_amd/lib/libmoc_final_gpu.so next to this binary,
// or $MOC_GPU_PLUGIN. Loaded once, on the first question about GPUs; never for CPU-backend runs.
struct GpuPlugin {
  GpuDeviceCountFn device_count = nullptr;
  GpuRankCreateFn create = nullptr;
  std::string error;
};

const GpuPlugin& gpu_plugin() {
  static const GpuPlugin p = [] {
    GpuPlugin g;
    std::string path;
    if (const char* env = std::getenv("MOC_GPU_PLUGIN")) {
      path = env;
    } else {
      char exe[4096];
      const ssize_t len = readlink("/proc/self/exe", exe, sizeof exe - 1);
      std::string dir = ".";
      if (len > 0) {
        exe[len] = 0;
        dir = std::string(exe);
        dir = dir.substr(0, dir.rfind('/'));
      }
      path = dir + "/mpi_openmp_cuda_amd/lib/libmoc_final_gpu.so";
    }
    void* h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      const char* e = dlerror();
      g.error = e ? e : ("cannot load " + path);
      return g;
    }
    g.device_count = reinterpret_cast<GpuDeviceCountFn>(dlsym(h, kGpuDeviceCountSym));
    g.create = reinterpret_cast<GpuRankCreateFn>(dlsym(h, kGpuRankCreateSym));
    if (!g.device_count || !g.create) g.error = "GPU plugin " + path + " lacks its entry points";
    return g;
  }();
  return p;
}

int gpu_device_count() {
  const GpuPlugin& g = gpu_plugin();
  return g.device_count && g.create ? g.device_count() : 0;
}

// Runs the selected engine on one contiguous slice (host buffers).
struct RankEngine {
  bool gpu = false;
  std::unique_ptr<GpuRank> hip;
  ScoreTable table{};
  std::vector<uint8_t> seq1;
  Semantics sem = Semantics::Reference;
  int threads = 0;
  double kernel_ms = 0;  // accumulated device time of the search kernels

  void set_problem(const Weights& w, const std::vector<uint8_t>& s1, Semantics s) {
    sem = s;
    seq1 = s1;
    table = ScoreTable::build(w);
    if (gpu) hip->set_problem(w, s1.data(), static_cast<int64_t>(s1.size()), s);
  }
  static RecordBatch copy_slice(const uint8_t* codes, const int64_t* offsets, int64_t n) {
    RecordBatch b;
    b.codes.assign(codes + offsets[0], codes + offsets[n]);
    b.offsets.resize(static_cast<size_t>(n) + 1);
    for (int64_t i = 0; i <= n; ++i) b.offsets[i] = offsets[i] - offsets[0];
    return b;
  }
  void solve(const uint8_t* codes, const int64_t* offsets, int64_t n, Result* out) {
    if (n <= 0) return;
    if (gpu) {
      hip->solve(codes, offsets, n, out);
      kernel_ms += hip->last_kernel_ms();
      return;
    }
    solve_batch_cpu(table, seq1.data(), static_cast<int64_t>(seq1.size()), copy_slice(codes, offsets, n), out, sem,
                    threads);
  }
  // Context-parallel share `part` of `parts` of every record -> packed keys.
  void solve_keys(const uint8_t* codes, const int64_t* offsets, int64_t n, int part, int parts, uint64_t* keys) {
    if (n <= 0) return;
    if (gpu) {
      hip->search_keys(codes, offsets, n, part, parts, keys);
      kernel_ms += hip->last_kernel_ms();
      return;
    }
    solve_keys_cpu(table, seq1.data(), static_cast<int64_t>(seq1.size()), copy_slice(codes, offsets, n), part, parts,
                   keys, sem, threads);
  }
};

class Job {
 public:
  Job(MpiContext& ctx, const Flags& flags, BackgroundReleaser& rel, std::future<void> prewarm)
      : ctx_(ctx), flags_(flags), rel_(rel), prewarm_(std::move(prewarm)) {}
  int run();

 private:
  void setup_engine(int64_t cells, int64_t mean_l2);
  void run_batch(RecordBatch* rb, int64_t n, int64_t total_chars, int64_t first_index);
  void run_sliced(BulkParser& parser, int64_t first_index);
  void batch_shm(RecordBatch* rb, int64_t n, int64_t total_chars, bool cp);
  // group letter code of GPU slices for the streaming kernel: 33 (P33 fields, default) or 24 (--letters=p24)
  int group_pack() const {
    const std::string v = to_lower(flags_.get("letters", "p33"));
    if (v != "p33" && v != "p24") throw Error("--letters must be p33|p24");
    return v == "p24" ? 24 : 33;
  }
  void gpu_window_slice(const uint8_t* w_codes, const int64_t* offs, int64_t n, Result* res, ResultFormat& fmt,
                        R2Params& r2);
  std::vector<int64_t> make_bounds(const int64_t* offsets, int64_t n, bool cp);
  void batch_mpi(RecordBatch* rb, int64_t n, int64_t total_chars, const std::vector<int64_t>& bounds, bool cp);
  void batch_rccl(RecordBatch* rb, int64_t n, int64_t total_chars, const std::vector<int64_t>& bounds, bool cp);
  void print(const Result* r, int64_t n, int64_t first_index);  // first_index relative to the batch
  void report(const Header& h);

  MpiContext& ctx_;
  const Flags& flags_;
  BackgroundReleaser& rel_;  // large frees off the critical path (outlives the job: drained after finalize)
  FaultHook fault_;
  RankEngine eng_;
  int device_ = -1;
  bool all_gpu_ = false;
  std::string transport_, partition_;
  bool pin_window_ = true;
  PhaseTimer pt_;
  Stopwatch total_;
  double compute_ms_ = 0;
  int64_t cells_ = 0, chars_ = 0, records_ = 0, batches_ = 0;
  int64_t first_index_ = 0;      // global index of the current batch's first record
  uvector<char> text_;                 // root: the input (kept for deferred parsing)
  FILE* out_ = stdout;                 // root: --output file, else stdout
  std::unique_ptr<BulkParser> parser_;  // root: pass 1 done, letters encoded straight into the window
  std::unique_ptr<SharedWindow> text_win_;  // sliced mode, several ranks on the node: the input text
  std::unique_ptr<MappedFile> text_map_;    // ... or, for an --input file, every rank's mapping of it
  int64_t pinned_bytes_ = 0, h2d_bytes_ = 0, d2h_bytes_ = 0;  // this rank (--timing)
  std::vector<int64_t> rank_pinned_, rank_h2d_, rank_records_, rank_pin_us_;  // root: per rank (--timing)
  std::shared_ptr<BulkParser> spent_parser_;     // root: filled into the window, freed while printing
  std::shared_ptr<uvector<char>> spent_text_;
  std::vector<Result> results_;  // root: results of the current batch (mpi transport)
  std::unique_ptr<MpiDeviceComm> emul_comm_;  // --transport=rccl-emul
  bool coll_rccl_ = false;                     // shm transport: collectives over RCCL (--collectives)
  void allgather_i64(const int64_t* mine, int count, int64_t* all);
  void allreduce_keys(uint64_t* keys, int64_t n);
  // root: MAX-combined pass-1 keys -> results (k resolved on the winning diagonals)
  void resolve_keys(const uint64_t* keys, const uint8_t* codes, const int64_t* offsets, int64_t n, Result* out) {
    const int64_t L1 = static_cast<int64_t>(eng_.seq1.size());
#pragma omp parallel for schedule(dynamic, 64) if (n > 4096)
    for (int64_t i = 0; i < n; ++i)
      out[i] = resolve_key(eng_.table, eng_.seq1.data(), L1, codes + offsets[i], offsets[i + 1] - offsets[i], keys[i]);
  }
  std::future<void> prewarm_;     // HIP runtime start-up overlapped with the parse (large inputs)
};

void Job::setup_engine(int64_t cells, int64_t mean_l2) {
  if (prewarm_.valid()) prewarm_.get();
  const int threads = static_cast<int>(flags_.get_int("threads", 0));
  std::string backend = to_lower(flags_.get("backend", "auto"));
  if (backend != "auto" && backend != "hip" && backend != "cpu") throw Error("--backend must be auto|hip|cpu");
  // auto: a job the OpenMP engine finishes faster than the GPU starts runs on the CPU. The GPU's start-up
  // (HIP runtime + engine) is 0.05-0.25 s; the OpenMP engine on the MI355X box's host cores searches
  // ~0.4 G cells/s per thread for records of <= 32 letters and ~1.4 G for longer ones, so the crossover is
  // ~0.2 s of CPU work (tools/gpu_crossover.sh, profiles/gpu_crossover.log: input6 shape between 0.6 and
  // 2.5 G cells at 16 threads, input3 shape above 1.7 G). `cells` < 0 means unknown (streaming): large.
  const double per_thread = mean_l2 > 32 ? 1.4e9 : 0.4e9;
  const int64_t model_min = static_cast<int64_t>(0.2 * per_thread * std::max(1, omp_get_max_threads()));
  const int64_t min_cells = flags_.get_int("gpu-min-cells", model_min);
  if (backend == "auto" && cells >= 0 && cells < min_cells * ctx_.size) backend = "cpu";
  const int ndev = (backend == "cpu") ? 0 : gpu_device_count();
  if (backend == "hip" && ndev == 0)
    throw Error("--backend=hip but no HIP device is visible" +
                (gpu_plugin().error.empty() ? std::string() : " (" + gpu_plugin().error + ")"));
  eng_.threads = threads;
  eng_.gpu = ndev > 0;
  if (eng_.gpu) {
    GpuRankOptions go;
    go.device = static_cast<int>(flags_.get_int("device", -1));
    go.device_map = parse_int_list(flags_.get("device-map", ""));
    go.chunk_records = flags_.get_int("chunk-records", 0);
    go.chunk_bytes = flags_.get_int("chunk-bytes", 0);
    go.log_level = flags_.get("log-level", "warn");
    eng_.hip.reset(gpu_plugin().create(ctx_, go));
    device_ = eng_.hip->device();
  }
  int gpu_minmax[2] = {eng_.gpu ? 1 : 0, eng_.gpu ? -1 : 0};  // MIN -> {min gpu, -max gpu}
  MPI_Allreduce(MPI_IN_PLACE, gpu_minmax, 2, MPI_INT, MPI_MIN, ctx_.world);
  all_gpu_ = gpu_minmax[0] != 0;
  const bool any_gpu = gpu_minmax[1] != 0;
  transport_ = to_lower(flags_.get("transport", "auto"));
  if (transport_ == "auto") transport_ = ctx_.single_node() ? "shm" : (all_gpu_ ? "rccl" : "mpi");
  if (transport_ == "shm" && !ctx_.single_node()) throw Error("--transport=shm needs all ranks on one node");
  if (transport_ == "rccl" && !all_gpu_) throw Error("--transport=rccl needs a GPU on every rank");
  if (transport_ == "rccl-emul" && any_gpu) throw Error("--transport=rccl-emul runs on CPU ranks (--backend=cpu)");
  if (transport_ != "shm" && transport_ != "rccl" && transport_ != "rccl-emul" && transport_ != "mpi")
    throw Error("unknown --transport " + transport_);
  partition_ = to_lower(flags_.get("partition", "cost"));
  if (partition_ != "cost" && partition_ != "even" && partition_ != "offsets")
    throw Error("--partition must be cost|even|offsets");
  // GPU ranks split by shares of the tile list, CPU ranks by shares of each record's offsets: the two
  // decompositions do not tile each other, so the context-parallel mode needs one engine kind
  if (partition_ == "offsets" && any_gpu && !all_gpu_)
    throw Error("--partition=offsets needs the same backend on every rank (use --backend=hip or --backend=cpu)");
  pin_window_ = flags_.get_bool("pin-window", true);
  if (transport_ == "rccl") eng_.hip->init_rccl();
  // the shm transport moves no record data between ranks; its collectives (the slices' fill reports and
  // result descriptors, the context-parallel key reduction) are a few host int64 per rank (or one key per
  // record), so they stay on MPI unless --collectives=rccl: setting up an RCCL communicator took 1.7-5.8 s
  // on the MI355X box even for one rank (profiles/final_scale_collrccl.log), microseconds of MPI work
  // would wait for it. With rccl the connect runs on a helper thread while the ranks parse their slices.
  const std::string coll = to_lower(flags_.get("collectives", "auto"));
  if (coll != "auto" && coll != "mpi" && coll != "rccl") throw Error("--collectives must be auto|mpi|rccl");
  if (coll == "rccl" && !all_gpu_) throw Error("--collectives=rccl needs a GPU on every rank");
  bool shared_gpu = false;  // RCCL needs one rank per GPU
  if (all_gpu_ && coll == "rccl") {
    const int64_t mine = static_cast<int64_t>(std::hash<std::string>{}(ctx_.hostname) & 0xffffffffffffull) * 4096 + device_;
    std::vector<int64_t> all(static_cast<size_t>(ctx_.size));
    MPI_Allgather(&mine, 1, MPI_INT64_T, all.data(), 1, MPI_INT64_T, ctx_.world);
    std::sort(all.begin(), all.end());
    shared_gpu = std::adjacent_find(all.begin(), all.end()) != all.end();
  }
  if (coll == "rccl" && shared_gpu) throw Error("--collectives=rccl needs one rank per GPU");
  coll_rccl_ = transport_ == "shm" && all_gpu_ && !shared_gpu && coll == "rccl";
  if (coll_rccl_) eng_.hip->init_rccl_begin();
  if (transport_ == "rccl-emul") emul_comm_ = std::make_unique<MpiDeviceComm>(ctx_);
  MOC_LOG_INFO("rank %d/%d host %s local %d/%d engine=%s device=%d transport=%s partition=%s", ctx_.rank, ctx_.size,
               ctx_.hostname.c_str(), ctx_.local_rank, ctx_.local_size, eng_.gpu ? "hip" : "cpu", device_,
               transport_.c_str(), partition_.c_str());
}

// MPI_Allgather of `count` int64 per rank, or the same over RCCL (--collectives).
void Job::allgather_i64(const int64_t* mine, int count, int64_t* all) {
  if (!coll_rccl_) {
    MPI_Allgather(mine, count, MPI_INT64_T, all, count, MPI_INT64_T, ctx_.world);
    return;
  }
  DeviceComm& dc = eng_.hip->device_comm();  // waits for the connect
  const int64_t bytes = 8 * static_cast<int64_t>(count);
  char* d = static_cast<char*>(dc.dev_alloc(bytes * (ctx_.size + 1)));
  try {
    dc.wait_upload(dc.upload(d, mine, bytes));
    dc.allgather(d, d + bytes, bytes);
    dc.download(all, d + bytes, bytes * ctx_.size);
  } catch (...) {
    dc.dev_free(d);
    throw;
  }
  dc.dev_free(d);
}

// In-place MAX of packed keys over the ranks (context-parallel combine), MPI or RCCL.
void Job::allreduce_keys(uint64_t* keys, int64_t n) {
  if (!coll_rccl_) {
    allreduce_max_u64(keys, n, ctx_.world);
    return;
  }
  DeviceComm& dc = eng_.hip->device_comm();
  uint64_t* d = static_cast<uint64_t*>(dc.dev_alloc(8 * n));
  try {
    dc.wait_upload(dc.upload(d, keys, 8 * n));
    dc.allreduce_max_u64(d, n);
    dc.download(keys, d, 8 * n);
  } catch (...) {
    dc.dev_free(d);
    throw;
  }
  dc.dev_free(d);
}

void Job::print(const Result* r, int64_t n, int64_t first_index) {
  if (ctx_.rank != kRoot) return;
  pt_.begin("print");
  write_results(out_, r, n, first_index_ + first_index);
  pt_.end();
}

// One batch of records: decomposition + distribution + search + combine + print.
// rb: the batch (root only; offsets rebased to 0), n / total_chars known on every rank.
void Job::run_batch(RecordBatch* rb, int64_t n, int64_t total_chars, int64_t first_index) {
  ++batches_;
  first_index_ = first_index;
  records_ += n;
  chars_ += total_chars;
  const bool cp = partition_ == "offsets";
  if (transport_ == "shm") {  // the window is filled first; the bounds come from it
    batch_shm(rb, n, total_chars, cp);
    return;
  }
  const std::vector<int64_t> bounds = make_bounds(ctx_.rank == kRoot ? rb->offsets.data() : nullptr, n, cp);
  if (transport_ == "mpi")
    batch_mpi(rb, n, total_chars, bounds, cp);
  else
    batch_rccl(rb, n, total_chars, bounds, cp);
}

// Root: record lengths -> search cells (for --timing) and the cost-balanced rank bounds; broadcast.
std::vector<int64_t> Job::make_bounds(const int64_t* offsets, int64_t n, bool cp) {
  const int p = ctx_.size;
  std::vector<int64_t> bounds(static_cast<size_t>(p) + 1, 0);
  if (ctx_.rank == kRoot) {
    const int64_t L1 = static_cast<int64_t>(eng_.seq1.size());
    int64_t cells = 0;
#pragma omp parallel for reduction(+ : cells) schedule(static) if (n > 65536)
    for (int64_t i = 0; i < n; ++i) cells += record_cells(L1, offsets[i + 1] - offsets[i]);
    cells_ += cells;
    if (!cp) {
      CostModel cm = all_gpu_ ? CostModel{1.0, 200.0, 2400.0} : CostModel{1.0, 4.0, 64.0};
      bounds = partition_ == "even" ? partition_even(n, p) : partition_by_cost_offsets(offsets, n, L1, p, cm);
    }
  }
  if (!cp) bcast_bytes(bounds.data(), sizeof(int64_t) * (p + 1), kRoot, ctx_.world);
  return bounds;
}

void Job::batch_shm(RecordBatch* rb, int64_t n, int64_t total_chars, bool cp) {
  if (ctx_.size == 1 && !cp && rb && !parser_) {  // one rank: no window to share, search the batch in place
    const int64_t* offs = rb->offsets.data();
    const int64_t L1 = static_cast<int64_t>(eng_.seq1.size());
    int64_t cells = 0;
#pragma omp parallel for reduction(+ : cells) schedule(static) if (n > 65536)
    for (int64_t i = 0; i < n; ++i) cells += record_cells(L1, offs[i + 1] - offs[i]);
    cells_ += cells;
    pt_.begin("compute");
    fault_.at("compute", 0);
    Stopwatch sw;
    sw.start();
    HostRegion res(12 * static_cast<size_t>(std::max<int64_t>(n, 1)), eng_.gpu ? eng_.hip->numa_node() : -1);
    ResultFormat fmt = ResultFormat::R12;
    R2Params r2{};
    Result* out = res.as<Result>();
    if (eng_.gpu && n > 0)
      gpu_window_slice(rb->codes.data(), offs, n, out, fmt, r2);
    else if (n > 0)
      eng_.solve(rb->codes.data(), offs, n, out);
    sw.stop();
    compute_ms_ += sw.total_ms();
    pt_.end();
    {  // the batch's letters go back to the OS while its results print
      auto spent = std::make_shared<RecordBatch>(std::move(*rb));
      rel_.defer([spent]() mutable { spent.reset(); });
      *rb = RecordBatch{};
    }
    pt_.begin("print");
    write_results(out_, std::vector<ResultRun>{ResultRun{out, fmt, r2, n}}, first_index_);
    pt_.end();
    res.set_releaser(&rel_);
    return;
  }
  // layout: offsets[(N+1)] | results[N] (or keys[N] in cp mode) | codes[total]   (8-byte aligned sections)
  const int64_t off_bytes = 8 * (n + 1);
  const int64_t res_bytes = ((12 * n) + 7) & ~int64_t{7};
  pt_.begin("distribute");
  auto win = std::make_unique<SharedWindow>(ctx_, off_bytes + res_bytes + total_chars);
  win->set_releaser(&rel_);
  int64_t* w_offs = reinterpret_cast<int64_t*>(win->base());
  Result* w_res = reinterpret_cast<Result*>(win->base() + off_bytes);
  uint8_t* w_codes = reinterpret_cast<uint8_t*>(win->base() + off_bytes + res_bytes);
  int32_t status = 0;
  std::string error;
  if (ctx_.rank == kRoot) {
    if (parser_) {  // deferred pass 2: letters encoded straight into the window, no intermediate copy
      try {
        parser_->fill(w_codes, w_offs);
      } catch (const std::exception& e) {
        status = 1;
        error = e.what();
      }
      // the input buffers (≈1 GB per 10^9 letters) are freed by the background releaser while the
      // results print (not now: unmapping them while the engine page-locks the window slows both)
      spent_parser_ = std::move(parser_);
      spent_text_ = std::make_shared<uvector<char>>(std::move(text_));
      text_ = uvector<char>();
    } else {
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
  }
  bcast_bytes(&status, sizeof status, kRoot, ctx_.world);
  if (status != 0) {
    win.reset();  // collective, on every rank, before leaving
    throw InputError(error);
  }
  fault_.at("distribute", ctx_.rank);
  win->fence();
  pt_.end();
  pt_.begin("bounds");
  const std::vector<int64_t> bounds = make_bounds(ctx_.rank == kRoot ? w_offs : nullptr, n, cp);
  pt_.end();
  pt_.begin("compute");
  fault_.at("compute", ctx_.rank);
  Stopwatch sw;
  sw.start();
  if (cp) {
    std::vector<uint64_t> keys(static_cast<size_t>(n), 0);
    eng_.solve_keys(w_codes, w_offs, n, ctx_.rank, ctx_.size, keys.data());
    sw.stop();
    pt_.end();
    pt_.begin("gather");
    fault_.at("gather", ctx_.rank);
    allreduce_keys(keys.data(), n);
    if (ctx_.rank == kRoot)
      resolve_keys(keys.data(), w_codes, w_offs, n, w_res);
    pt_.end();
  } else {
    const int64_t my_b = bounds[ctx_.rank], my_n = bounds[ctx_.rank + 1] - my_b;
    // this rank's results go to the start of its R12 region of the window, in the format it chose
    ResultFormat fmt = ResultFormat::R12;
    R2Params r2{};
    if (eng_.gpu && my_n > 0) {
      gpu_window_slice(w_codes, w_offs + my_b, my_n, w_res + my_b, fmt, r2);
    } else if (my_n > 0) {
      eng_.solve(w_codes, w_offs + my_b, my_n, w_res + my_b);
    }
    sw.stop();
    pt_.end();
    pt_.begin("gather");
    fault_.at("gather", ctx_.rank);
    int64_t info[4] = {static_cast<int64_t>(fmt), r2.smin, r2.kw, r2.j};
    std::vector<int64_t> infos(static_cast<size_t>(4 * ctx_.size));
    allgather_i64(info, 4, infos.data());
    win->fence();
    pt_.end();
    compute_ms_ += sw.total_ms();
    if (spent_parser_ || spent_text_)
      rel_.defer([parser = std::move(spent_parser_), text = std::move(spent_text_)]() mutable {
        parser.reset();
        text.reset();
      });
    win->discard(0, off_bytes);
    win->discard(off_bytes + res_bytes, total_chars);
    if (ctx_.rank == kRoot) {
      std::vector<ResultRun> runs(static_cast<size_t>(ctx_.size));
      for (int q = 0; q < ctx_.size; ++q) {
        const int64_t* x = infos.data() + 4 * q;
        runs[q] = ResultRun{w_res + bounds[q], static_cast<ResultFormat>(x[0]),
                            R2Params{static_cast<int32_t>(x[1]), static_cast<int32_t>(x[2]), static_cast<int32_t>(x[3])},
                            bounds[q + 1] - bounds[q]};
      }
      pt_.begin("print");
      write_results(out_, runs, first_index_);
      pt_.end();
    }
    pt_.begin("release");
    win.reset();  // collective: unmaps the node-shared window
    pt_.end();
    return;
  }
  compute_ms_ += sw.total_ms();
  // printing reads only the results: the input, offsets and letters go back to the OS while it runs
  if (spent_parser_ || spent_text_)
    rel_.defer([parser = std::move(spent_parser_), text = std::move(spent_text_)]() mutable {
      parser.reset();
      text.reset();
    });
  win->discard(0, off_bytes);
  win->discard(off_bytes + res_bytes, total_chars);
  print(w_res, n, 0);
  pt_.begin("release");
  win.reset();  // collective: unmaps the node-shared window
  pt_.end();
}

// A GPU rank's slice of a node-shared CSR window (streaming batches): encoded into the headline's wire
// formats in NUMA-local memory when the streaming kernel takes the batch (P33 letters, narrow lengths,
// sparse offsets; narrow results written to the start of `res`), else the window's own bytes and offsets.
// Either way only this slice's pieces are page-locked — never the whole window.
void Job::gpu_window_slice(const uint8_t* w_codes, const int64_t* offs, int64_t n, Result* res, ResultFormat& fmt,
                           R2Params& r2) {
  const int64_t c0 = offs[0], c1 = offs[n];
  int64_t mn = INT64_MAX, mx = 0;
#pragma omp parallel for reduction(min : mn) reduction(max : mx) schedule(static) if (n > 65536)
  for (int64_t i = 0; i < n; ++i) {
    const int64_t L = offs[i + 1] - offs[i];
    mn = std::min(mn, L);
    mx = std::max(mx, L);
  }
  const int numa = eng_.hip->numa_node();
  auto pin = [&](const void* ptr, int64_t bytes) {
    if (!pin_window_ || !ptr || bytes <= 0) return;
    try {
      eng_.hip->pin(ptr, static_cast<size_t>(bytes));
      pinned_bytes_ += bytes;
    } catch (const std::exception& e) {
      MOC_LOG_WARN("could not page-lock this rank's slice (%s); using the staged pipeline", e.what());
    }
  };
  GpuSolveStats gs;
  if (mx <= 255 && eng_.hip->streams_packed(mn, mx)) {
    const int64_t letters = c1 - c0;
    const bool p33 = group_pack() == 33;
    HostRegion pk(static_cast<size_t>(p33 ? packed33_bytes(letters) : packed24_bytes(letters)) + 16, numa);
    if (p33)
      pack33(w_codes + c0, letters, pk.as<uint8_t>());
    else
      pack24(w_codes + c0, letters, pk.as<uint8_t>());
    const int bits = narrow_length_bits(mn, mx);
    const int64_t base = bits == 8 ? 0 : mn;
    HostRegion lens(static_cast<size_t>(narrow_lengths_bytes(n, bits)) + 8, numa);
    pack_lengths(offs, n, bits, base, lens.as<uint8_t>());
    const int64_t ns = sparse_count(n, kSparseShift);
    HostRegion sparse(8 * static_cast<size_t>(ns), numa);
    int64_t* sp = sparse.as<int64_t>();
    for (int64_t j = 0; j < ns; ++j) sp[j] = offs[std::min(j << kSparseShift, n)] - c0;
    WireBatch wb;
    wb.letters = pk.as<uint8_t>();
    wb.packed24 = !p33;
    wb.packed33 = p33;
    wb.offsets = sp;
    wb.off_shift = kSparseShift;
    wb.lengths = lens.as<uint8_t>();
    wb.len_bits = bits;
    wb.len_base = base;
    wb.n = n;
    wb.min_l2 = mn;
    wb.max_l2 = mx;
    fmt = eng_.hip->result_format(mn, mx);
    pin(wb.letters, wb.letter_bytes());
    pin(sp, 8 * ns);
    pin(wb.lengths, wb.length_bytes());
    pin(res, static_cast<int64_t>(result_bytes(fmt)) * n);
    eng_.hip->solve_wire(wb, res, fmt);
    gs = eng_.hip->last_stats();
    r2 = gs.r2;
    // unregistered now: the window's memory (the results' pages) is freed by its collective teardown
    eng_.hip->unpin_all();
    pk.set_releaser(&rel_);
    lens.set_releaser(&rel_);
    sparse.set_releaser(&rel_);
  } else {
    pin(w_codes + c0, c1 - c0);
    pin(offs, 8 * (n + 1));
    pin(res, 12 * n);
    eng_.hip->solve(w_codes, offs, n, res);
    gs.kernel_ms = eng_.hip->last_kernel_ms();
    eng_.hip->unpin_all();
    fmt = ResultFormat::R12;
  }
  eng_.kernel_ms += gs.kernel_ms;
  h2d_bytes_ += gs.h2d_bytes;
  d2h_bytes_ += gs.d2h_bytes;
}

// Bulk job on one node, records split into contiguous rank slices (transport shm, partition cost|even).
// Every rank encodes its OWN slice straight from the node-shared input text into its own buffers, in the
// wire formats its engine streams (SURVEY.md §7.3 / moc/wire.hpp):
//   GPU rank: P33 letters (56 per 33 bytes) + 3/4/8-bit lengths + sparse offsets (1 per 64 records) in private,
//             huge-page memory on its GPU's NUMA node, page-locked (only this slice), results in the
//             narrowest format (R2/R4/R8/R12) in this rank's segment of a node-shared result window;
//   CPU rank: byte letters + CSR offsets, results as R12.
// Pass 1 (token/letter counts) is cooperative: each rank counts a share of the text's chunks and the
// counts are all-gathered, so every rank holds the same chunk table and computes its own bounds from it
// (BulkParser::cost_split) without a further collective. The root prints from every rank's result segment
// in place (reference: MPI_Scatter of 2000-byte records + 3 MPI_Gathers, main.c:174,195-197).
void Job::run_sliced(BulkParser& parser, int64_t first_index) {
  const int p = ctx_.size, r = ctx_.rank;
  ++batches_;
  first_index_ = first_index;
  const int64_t L1 = static_cast<int64_t>(eng_.seq1.size());
  const bool gpu = eng_.gpu;
  const int numa = gpu ? eng_.hip->numa_node() : -1;

  const CostModel cost_model = all_gpu_ ? CostModel{1.0, 200.0, 2400.0} : CostModel{1.0, 4.0, 64.0};
  // ---- pass 1, cooperative
  pt_.begin("count");
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
    MPI_Allgatherv(MPI_IN_PLACE, 0, MPI_DATATYPE_NULL, tk.data(), cnt.data(), dsp.data(), MPI_INT64_T, ctx_.world);
    MPI_Allgatherv(MPI_IN_PLACE, 0, MPI_DATATYPE_NULL, ch.data(), cnt.data(), dsp.data(), MPI_INT64_T, ctx_.world);
    // inputs up to 256 MiB also get exact chunk costs (a token walk) for the bounds: few, coarse chunks
    // of records of very different lengths are what the mean-length estimate gets wrong
    if (partition_ != "even" && p > 1 && area <= (int64_t{256} << 20)) {
      std::vector<double> costs(static_cast<size_t>(nch));
      parser.chunk_costs(starts, dsp[r], dsp[r] + cnt[r], cost_model, costs.data() + dsp[r]);
      MPI_Allgatherv(MPI_IN_PLACE, 0, MPI_DATATYPE_NULL, costs.data(), cnt.data(), dsp.data(), MPI_DOUBLE, ctx_.world);
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
  records_ += n_all - first_index;
  pt_.end();

  // ---- this rank's slice
  pt_.begin("bounds");
  int64_t b0, b1;
  if (partition_ == "even") {
    b0 = first_index + (n_all - first_index) * r / p;
    b1 = first_index + (n_all - first_index) * (r + 1) / p;
  } else {
    b0 = parser.cost_split(first_index, r, p, cost_model);
    b1 = std::max(b0, parser.cost_split(first_index, r + 1, p, cost_model));
  }
  const AreaSlice slice = parser.slice(b0, b1);
  const int64_t n = slice.records;
  pt_.end();

  // ---- fill: every rank encodes its slice (GPU ranks guess the narrow form from the mean length)
  pt_.begin("fill");
  fault_.at("distribute", r);
  const bool narrow_guess = gpu && n > 0 && L1 <= 200 && slice.letters <= 32 * n;
  HostRegion letters, sparse, len16, dense, lens;
  int letters_pack = 5;      // GPU ranks: 33 = P33 fields, 24 = P24 groups, 5 = 5-bit packed
  int64_t letter_bytes = 0;
  RecordBatch cpu_batch;
  FillReport rep;
  if (n > 0) {
    if (!gpu) {
      cpu_batch.codes.resize(static_cast<size_t>(slice.letters));
      cpu_batch.offsets.resize(static_cast<size_t>(n) + 1);
      rep = parser.fill_slice(slice, cpu_batch.codes.data(), nullptr, cpu_batch.offsets.data());
    } else {
      // letters as P33 fields (4.714 bits each; --letters=p24: P24 groups, 4.8) for the streaming kernel,
      // else 5-bit packed
      const int pack = narrow_guess ? group_pack() : 5;
      const int64_t lbytes = pack == 33   ? packed33_bytes(slice.letters)
                             : pack == 24 ? packed24_bytes(slice.letters)
                                          : packed5_bytes(slice.letters);
      letters = HostRegion(static_cast<size_t>(lbytes) + 16, numa);
      letters_pack = pack;
      letter_bytes = lbytes;
      if (narrow_guess) {
        sparse = HostRegion(8 * static_cast<size_t>(sparse_count(n, kSparseShift)), numa);
        len16 = HostRegion(2 * static_cast<size_t>(n), numa);
        rep = parser.fill_slice(slice, nullptr, letters.as<uint8_t>(), nullptr, sparse.as<int64_t>(),
                                len16.as<uint16_t>(), pack);
      } else {
        dense = HostRegion(8 * (static_cast<size_t>(n) + 1), numa);
        rep = parser.fill_slice(slice, nullptr, letters.as<uint8_t>(), dense.as<int64_t>(), nullptr, nullptr, pack);
      }
    }
  }
  // the job's first input error (the one a sequential reader meets first) on every rank
  {
    int64_t mine[7] = {rep.min_len, rep.max_len, rep.bad_record, rep.long_record, rep.long_len, rep.cells,
                       slice.letters};
    std::vector<int64_t> all(static_cast<size_t>(7 * p));
    allgather_i64(mine, 7, all.data());
    FillReport job;
    for (int q = 0; q < p; ++q) {
      const int64_t* x = all.data() + 7 * q;
      chars_ += x[6];
      job.min_len = std::min(job.min_len, x[0]);
      job.max_len = std::max(job.max_len, x[1]);
      if (x[2] >= 0 && (job.bad_record < 0 || x[2] < job.bad_record)) job.bad_record = x[2];
      if (x[3] >= 0 && (job.long_record < 0 || x[3] < job.long_record)) {
        job.long_record = x[3];
        job.long_len = x[4];
      }
      job.cells += x[5];
    }
    cells_ += job.cells;
    // every slice is encoded: the helpers return the node-shared input text's pages to the OS while
    // their GPUs search and the root prints
    if (text_win_) text_win_->release_shares(ctx_);
    try {
      parser.check(job);
    } catch (const std::exception& e) {
      throw InputError(e.what());
    }
  }
  pt_.end();
  // GPU ranks: the wire form the engine streams (the first question to the engine: waits for its start-up)
  pt_.begin("wire");
  WireBatch wb;
  ResultFormat fmt = ResultFormat::R12;
  if (gpu && n > 0) {
    wb.letters = letters.as<uint8_t>();
    wb.packed24 = letters_pack == 24;
    wb.packed33 = letters_pack == 33;
    wb.packed5 = letters_pack == 5;
    wb.n = n;
    wb.min_l2 = rep.min_len;
    wb.max_l2 = rep.max_len;
    if (narrow_guess && rep.max_len <= 255 && eng_.hip->streams_packed(rep.min_len, rep.max_len)) {
      const int bits = narrow_length_bits(rep.min_len, rep.max_len);
      lens = HostRegion(static_cast<size_t>(narrow_lengths_bytes(n, bits)), numa);
      pack_lengths16(len16.as<uint16_t>(), n, bits, rep.min_len, lens.as<uint8_t>());
      len16 = HostRegion();
      wb.offsets = sparse.as<int64_t>();
      wb.off_shift = kSparseShift;
      wb.lengths = lens.as<uint8_t>();
      wb.len_bits = bits;
      wb.len_base = bits == 8 ? 0 : rep.min_len;
    } else {
      if (narrow_guess) {  // guessed wrong: CSR offsets and 5-bit letters after all (staged pipeline)
        sparse = HostRegion();
        len16 = HostRegion();
        dense = HostRegion(8 * (static_cast<size_t>(n) + 1), numa);
        letter_bytes = packed5_bytes(slice.letters);
        letters = HostRegion(static_cast<size_t>(letter_bytes) + 16, numa);
        parser.fill_slice(slice, nullptr, letters.as<uint8_t>(), dense.as<int64_t>());
        wb.letters = letters.as<uint8_t>();
        wb.packed24 = wb.packed33 = false;
        wb.packed5 = true;
      }
      wb.offsets = dense.as<int64_t>();
    }
    fmt = eng_.hip->result_format(rep.min_len, rep.max_len);
  }
  pt_.end();

  // ---- results: this rank's segment of a node-shared window, printed by the root; or, with
  // --parallel-print, several ranks and an --output file, every rank prints its own rows into the file
  // (formatting split over the ranks, no result window). Measured on one MI355X box at 2 ranks the root
  // print was faster (0.52 vs 0.76 s for 4.6 GB: the ranks' writes contend for the one file and their
  // threads for the cores), so it is opt-in.
  const int fb = result_bytes(fmt);
  pt_.begin("results");
  int64_t dp[2] = {0, 0};  // {distributed print, the file offset of the first row}
  if (r == kRoot && p > 1 && out_ != stdout && flags_.get_bool("parallel-print", false)) {
    struct stat st {};
    const int fd = fileno(out_);
    const int fl = fcntl(fd, F_GETFL);
    std::fflush(out_);
    if (fl >= 0 && !(fl & O_APPEND) && fstat(fd, &st) == 0 && S_ISREG(st.st_mode)) {
      dp[0] = 1;
      dp[1] = static_cast<int64_t>(std::ftell(out_));
    }
  }
  bcast_bytes(dp, sizeof dp, kRoot, ctx_.world);
  std::unique_ptr<SegmentWindow> seg;
  HostRegion own;
  char* res_mine = nullptr;
  if (dp[0]) {
    own = HostRegion(static_cast<size_t>(std::max<int64_t>(fb * n, 16)), numa);
    own.set_releaser(&rel_);
    res_mine = own.data();
  } else {
    seg = std::make_unique<SegmentWindow>(ctx_, fb * n, numa);
    seg->set_releaser(&rel_);
    res_mine = seg->mine();
  }
  pt_.end();
  // GPU ranks page-lock this slice's pieces only (the registration faults in and locks every page)
  pt_.begin("pin");
  Stopwatch pin_sw;
  pin_sw.start();
  if (gpu && n > 0 && pin_window_) {
    try {
      auto pin = [&](const void* ptr, int64_t bytes) {
        if (ptr && bytes > 0) {
          eng_.hip->pin(ptr, static_cast<size_t>(bytes));
          pinned_bytes_ += bytes;
        }
      };
      pin(wb.letters, letter_bytes);
      pin(wb.offsets, 8 * wb.offset_entries());
      pin(wb.lengths, wb.length_bytes());
      pin(res_mine, fb * n);
    } catch (const std::exception& e) {
      MOC_LOG_WARN("could not page-lock this rank's slice (%s); using the staged pipeline", e.what());
    }
  }
  pin_sw.stop();
  pt_.end();
  pt_.begin("compute");
  fault_.at("compute", r);
  Stopwatch sw;
  sw.start();
  GpuSolveStats gs;
  if (n > 0) {
    if (gpu) {
      eng_.hip->solve_wire(wb, res_mine, fmt);
      gs = eng_.hip->last_stats();
      eng_.kernel_ms += gs.kernel_ms;
      h2d_bytes_ += gs.h2d_bytes;
      d2h_bytes_ += gs.d2h_bytes;
    } else {
      solve_batch_cpu(eng_.table, eng_.seq1.data(), L1, cpu_batch, reinterpret_cast<Result*>(res_mine), eng_.sem,
                      eng_.threads);
    }
  }
  sw.stop();
  compute_ms_ += sw.total_ms();
  pt_.end();
  // inputs nobody reads any more go back to the OS while the root prints: their registrations are
  // dropped first (the releaser runs its tasks in order), then the pages
  pt_.begin("drop");
  if (gpu) rel_.defer(eng_.hip->detach_pins());
  letters.set_releaser(&rel_);
  sparse.set_releaser(&rel_);
  dense.set_releaser(&rel_);
  lens.set_releaser(&rel_);
  { HostRegion drop[4] = {std::move(letters), std::move(sparse), std::move(dense), std::move(lens)}; }
  if (!cpu_batch.codes.empty()) {
    auto spent = std::make_shared<RecordBatch>(std::move(cpu_batch));
    rel_.defer([spent]() mutable { spent.reset(); });
  }
  pt_.end();

  // ---- every rank's result run -> root, which prints them in order straight from the segments
  pt_.begin("gather");
  fault_.at("gather", r);
  int64_t info[8] = {n,           static_cast<int64_t>(fmt), gs.r2.smin, gs.r2.kw, gs.r2.j, pinned_bytes_, h2d_bytes_,
                     static_cast<int64_t>(pin_sw.total_ms() * 1000.0)};
  std::vector<int64_t> infos(static_cast<size_t>(8 * p));
  allgather_i64(info, 8, infos.data());
  if (seg) seg->fence();
  pt_.end();
  if (r == kRoot) {  // --timing: what every rank owned, page-locked and moved
    rank_pinned_.assign(static_cast<size_t>(p), 0);
    rank_h2d_.assign(static_cast<size_t>(p), 0);
    rank_records_.assign(static_cast<size_t>(p), 0);
    rank_pin_us_.assign(static_cast<size_t>(p), 0);
    for (int q = 0; q < p; ++q) {
      const int64_t* x = infos.data() + 8 * q;
      rank_records_[q] = x[0];
      rank_pinned_[q] = x[5];
      rank_h2d_[q] = x[6];
      rank_pin_us_[q] = x[7];
    }
    // a private input text goes back to the OS while the results print
    if (!text_.empty()) {
      auto t = std::make_shared<uvector<char>>(std::move(text_));
      rel_.defer([t]() mutable { t.reset(); });
      text_ = uvector<char>();
    }
  }
  if (dp[0]) {  // every rank: its rows at its offset of the output file (sizes all-gathered first)
    pt_.begin("print");
    const std::vector<ResultRun> mine = {ResultRun{res_mine, fmt, gs.r2, n}};
    int64_t bytes = formatted_bytes(mine, b0);
    std::vector<int64_t> sizes(static_cast<size_t>(p));
    allgather_i64(&bytes, 1, sizes.data());
    int64_t at = dp[1], total = 0;
    for (int q = 0; q < p; ++q) {
      if (q < r) at += sizes[q];
      total += sizes[q];
    }
    int fd = r == kRoot ? fileno(out_) : -1;
    if (r != kRoot && n > 0) {
      fd = ::open(flags_.get("output", "").c_str(), O_WRONLY | O_CLOEXEC);
      if (fd < 0) throw Error("cannot open --output " + flags_.get("output", "") + " on rank " + std::to_string(r));
    }
    if (n > 0) write_results_at(fd, at, mine, b0);
    if (r != kRoot && fd >= 0) ::close(fd);
    MPI_Barrier(ctx_.world);  // every row is in the file
    if (r == kRoot) std::fseek(out_, static_cast<long>(dp[1] + total), SEEK_SET);
    pt_.end();
    pt_.begin("release");
    text_win_.reset();  // collective (node-shared input text)
    pt_.end();
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
    pt_.begin("print");
    write_results(out_, runs, first_index);
    pt_.end();
  }
  pt_.begin("release");
  seg->fence();  // nobody unmaps a segment the root still prints from
  text_win_.reset();  // collective (node-shared input text)
  pt_.end();
}

void Job::batch_mpi(RecordBatch* rb, int64_t n, int64_t total_chars, const std::vector<int64_t>& bounds, bool cp) {
  const int p = ctx_.size;
  pt_.begin("distribute");
  fault_.at("distribute", ctx_.rank);
  if (cp) {  // every rank needs every record
    RecordBatch all;
    if (ctx_.rank == kRoot) all = std::move(*rb);
    all.offsets.resize(static_cast<size_t>(n) + 1);
    all.codes.resize(static_cast<size_t>(total_chars));
    bcast_bytes(all.offsets.data(), 8 * (n + 1), kRoot, ctx_.world);
    bcast_bytes(all.codes.data(), total_chars, kRoot, ctx_.world);
    pt_.end();
    pt_.begin("compute");
    fault_.at("compute", ctx_.rank);
    Stopwatch sw;
    sw.start();
    std::vector<uint64_t> keys(static_cast<size_t>(n), 0);
    eng_.solve_keys(all.codes.data(), all.offsets.data(), n, ctx_.rank, ctx_.size, keys.data());
    sw.stop();
    compute_ms_ += sw.total_ms();
    pt_.end();
    pt_.begin("gather");
    fault_.at("gather", ctx_.rank);
    allreduce_max_u64(keys.data(), n, ctx_.world);
    pt_.end();
    if (ctx_.rank == kRoot) {
      results_.resize(static_cast<size_t>(n));
      resolve_keys(keys.data(), all.codes.data(), all.offsets.data(), n, results_.data());
    }
    print(results_.data(), n, 0);
    return;
  }
  const int64_t my_b = bounds[ctx_.rank], my_n = bounds[ctx_.rank + 1] - my_b;
  std::vector<int64_t> lcount(p), ldispl(p), ccount(p), cdispl(p);
  for (int r = 0; r < p; ++r) {
    lcount[r] = 8 * (bounds[r + 1] - bounds[r]);
    ldispl[r] = 8 * bounds[r];
  }
  std::vector<int64_t> lengths;
  if (ctx_.rank == kRoot) {
    lengths.resize(static_cast<size_t>(n));
    for (int64_t i = 0; i < n; ++i) lengths[i] = rb->length(i);
    for (int r = 0; r < p; ++r) {
      ccount[r] = rb->offsets[bounds[r + 1]] - rb->offsets[bounds[r]];
      cdispl[r] = rb->offsets[bounds[r]];
    }
  }
  bcast_bytes(ccount.data(), 8 * p, kRoot, ctx_.world);
  std::vector<int64_t> my_len(static_cast<size_t>(my_n));
  scatterv_bytes(lengths.data(), lcount, ldispl, my_len.data(), kRoot, ctx_.world);
  std::vector<uint8_t> my_codes(static_cast<size_t>(ccount[ctx_.rank]));
  scatterv_bytes(ctx_.rank == kRoot ? rb->codes.data() : nullptr, ccount, cdispl, my_codes.data(), kRoot, ctx_.world);
  std::vector<int64_t> my_off(static_cast<size_t>(my_n) + 1, 0);
  for (int64_t i = 0; i < my_n; ++i) my_off[i + 1] = my_off[i] + my_len[i];
  pt_.end();
  pt_.begin("compute");
  fault_.at("compute", ctx_.rank);
  std::vector<Result> mine(static_cast<size_t>(my_n));
  Stopwatch sw;
  sw.start();
  eng_.solve(my_codes.data(), my_off.data(), my_n, mine.data());
  sw.stop();
  compute_ms_ += sw.total_ms();
  pt_.end();
  pt_.begin("gather");
  fault_.at("gather", ctx_.rank);
  std::vector<int64_t> rcount(p), rdispl(p);
  for (int r = 0; r < p; ++r) {
    rcount[r] = 12 * (bounds[r + 1] - bounds[r]);
    rdispl[r] = 12 * bounds[r];
  }
  if (ctx_.rank == kRoot) results_.resize(static_cast<size_t>(n));
  gatherv_bytes(mine.data(), 12 * my_n, results_.data(), rcount, rdispl, kRoot, ctx_.world);
  pt_.end();
  print(results_.data(), n, 0);
}

void Job::batch_rccl(RecordBatch* rb, int64_t n, int64_t total_chars, const std::vector<int64_t>& bounds, bool cp) {
  PhaseHooks hooks;
  hooks.begin = [this](const char* phase) {
    pt_.begin(phase);
    fault_.at(phase, ctx_.rank);
  };
  hooks.end = [this] { pt_.end(); };
  DeviceBatchOut out;
  if (emul_comm_) {
    CpuDeviceSearch ds(eng_.table, eng_.seq1, eng_.sem, eng_.threads);
    out = device_batch(*emul_comm_, ds, rb, n, total_chars, bounds, cp, hooks);
  } else {
    out = device_batch(eng_.hip->device_comm(), eng_.hip->device_search(), rb, n, total_chars, bounds, cp, hooks);
  }
  compute_ms_ += out.compute_ms;
  eng_.kernel_ms += out.kernel_ms;
  if (ctx_.rank == kRoot) {
    if (!out.rank_records.empty()) rank_records_ = out.rank_records;
    pt_.begin("print");
    write_results(out_, out.runs, first_index_);
    pt_.end();
  }
}

void Job::report(const Header& h) {
  double mx[2] = {compute_ms_, eng_.kernel_ms};
  MPI_Reduce(ctx_.rank == kRoot ? MPI_IN_PLACE : mx, mx, 2, MPI_DOUBLE, MPI_MAX, kRoot, ctx_.world);
  // every mode: what each rank page-locked and moved host->device over the job (sliced mode also has
  // its per-rank records and pin times, gathered with its results)
  int64_t moved[2] = {pinned_bytes_, h2d_bytes_};
  std::vector<int64_t> all_moved(static_cast<size_t>(2 * ctx_.size));
  MPI_Gather(moved, 2, MPI_INT64_T, all_moved.data(), 2, MPI_INT64_T, kRoot, ctx_.world);
  if (ctx_.rank != kRoot || !flags_.get_bool("timing", false)) return;
  const double wall_s = total_.total_ms() / 1e3;
  auto list = [](const std::vector<int64_t>& v) {
    std::string s = "[";
    for (size_t i = 0; i < v.size(); ++i) s += (i ? ", " : "") + std::to_string(v[i]);
    return s + "]";
  };
  std::string per_rank;
  if (!rank_records_.empty()) {  // sliced mode: what each rank owned, page-locked and moved host->device
    per_rank = ", \"rank_records\": " + list(rank_records_) + ", \"rank_pinned_bytes\": " + list(rank_pinned_) +
               ", \"rank_h2d_bytes\": " + list(rank_h2d_) + ", \"rank_pin_us\": " + list(rank_pin_us_);
  } else {
    std::vector<int64_t> pinned(static_cast<size_t>(ctx_.size)), h2d(static_cast<size_t>(ctx_.size));
    for (int q = 0; q < ctx_.size; ++q) {
      pinned[q] = all_moved[2 * q];
      h2d[q] = all_moved[2 * q + 1];
    }
    per_rank = ", \"rank_pinned_bytes\": " + list(pinned) + ", \"rank_h2d_bytes\": " + list(h2d);
  }
  std::fprintf(stderr,
               "{\"timing\": %s, \"ranks\": %d, \"nodes\": %d, \"engine\": \"%s\", \"transport\": \"%s\", "
               "\"partition\": \"%s\", \"collectives\": \"%s\", \"sliced\": %s, \"batches\": %lld, \"first_index\": %lld, \"records\": %lld, "
               "\"elements\": %lld, \"cells\": %lld, \"max_rank_compute_ms\": %.3f, \"max_rank_kernel_ms\": %.3f, "
               "\"wall_s\": %.6f, \"elements_per_s\": %.1f, \"cells_per_s\": %.1f%s, \"build\": \"%s\"}\n",
               pt_.json().c_str(), ctx_.size, ctx_.node_count, eng_.gpu ? "hip" : "cpu", transport_.c_str(),
               partition_.c_str(), coll_rccl_ || transport_ == "rccl" ? "rccl" : "mpi", rank_records_.empty() ? "false" : "true", static_cast<long long>(batches_),
               static_cast<long long>(h.first_index), static_cast<long long>(records_), static_cast<long long>(chars_),
               static_cast<long long>(cells_), mx[0], mx[1], wall_s, wall_s > 0 ? chars_ / wall_s : 0.0,
               wall_s > 0 ? cells_ / wall_s : 0.0, per_rank.c_str(), kBuildId);
}

int Job::run() {
  log_set_level(flags_.get("log-level", "warn"));
  {
    std::string f = flags_.get("inject-fault", "");
    auto colon = f.find(':');
    fault_.phase = f.substr(0, colon);
    if (colon != std::string::npos) fault_.rank = std::stoi(f.substr(colon + 1));
  }
  const std::string sem_s = to_lower(flags_.get("semantics", "reference"));
  if (sem_s != "reference" && sem_s != "spec") throw Error("--semantics must be reference|spec");
  const Semantics sem = sem_s == "spec" ? Semantics::Spec : Semantics::Reference;
  const int64_t batch_records = flags_.get_int("batch-records", 0);
  const int64_t batch_chars = flags_.get_int("batch-chars", 0);
  const int64_t skip = flags_.get_int("skip-records", 0);
  if (batch_records < 0 || batch_chars < 0 || skip < 0) throw Error("--batch-records/--batch-chars/--skip-records >= 0");
  const bool streaming = batch_records > 0 || batch_chars > 0;
  ParseOptions po;
  po.strict_limits = flags_.get_bool("strict-limits", false);
  po.max_l1 = flags_.get_int("max-l1", 0);
  po.max_l2 = flags_.get_int("max-l2", 0);

  // OpenMP threads: --threads, else OMP_NUM_THREADS, else the node's cores shared by its ranks
  int threads = static_cast<int>(flags_.get_int("threads", 0));
  if (threads <= 0 && !std::getenv("OMP_NUM_THREADS")) threads = std::max(1, omp_get_num_procs() / ctx_.local_size);
  if (threads > 0) omp_set_num_threads(threads);
  total_.start();

  // ---- a large input (a regular file of >= --gpu-prewarm-bytes) will run on the GPU: every rank brings the
  // HIP runtime up on a helper thread while the root reads and parses, instead of after the header bcast
  {
    int64_t hint = 0;
    if (ctx_.rank == kRoot && to_lower(flags_.get("backend", "auto")) != "cpu") {
      const std::string path = flags_.get("input", "");
      struct stat st {};
      const int rc = path.empty() ? fstat(STDIN_FILENO, &st) : stat(path.c_str(), &st);
      const int64_t min_bytes = flags_.get_int("gpu-prewarm-bytes", int64_t{64} << 20);
      hint = rc == 0 && S_ISREG(st.st_mode) && min_bytes > 0 && st.st_size >= min_bytes;
    }
    bcast_bytes(&hint, sizeof hint, kRoot, ctx_.world);
    if (hint && !prewarm_.valid()) prewarm_ = std::async(std::launch::async, [] { (void)gpu_device_count(); });
  }

  // ---- root opens the input; parses it whole (bulk) or just its header (streaming). A bulk job on one
  // node (shm transport) with record slices runs "sliced": every rank encodes its own slice from the
  // input text, which is then read into a node-shared window when the node has several ranks.
  const std::string tr_flag = to_lower(flags_.get("transport", "auto"));
  const bool sliced = !streaming && to_lower(flags_.get("partition", "cost")) != "offsets" &&
                      (tr_flag == "shm" || (tr_flag == "auto" && ctx_.single_node()));
  Header h{};
  std::string error;
  FILE* in = stdin;
  std::unique_ptr<StreamReader> reader;
  RecordBatch bulk;
  std::vector<uint8_t> seq1;
  const char* text = nullptr;  // sliced: the input text (every rank)
  int64_t text_len = 0;
  if (ctx_.rank == kRoot) {
    pt_.begin("read");
    try {
      fault_.at("parse", ctx_.rank);
      const std::string path = flags_.get("input", "");
      if (!path.empty() && !(in = std::fopen(path.c_str(), "rb"))) throw Error("cannot open --input " + path);
      const std::string opath = flags_.get("output", "");
      if (!opath.empty() && !(out_ = open_output(opath))) {
        out_ = stdout;
        throw Error("cannot open --output " + opath);
      }
      if (sliced && ctx_.local_size > 1) {
        text_len = regular_input_bytes(in);  // read straight into the shared window below
        if (text_len < 0) {                  // a pipe: read it all first
          text_ = read_stream(in);
          text_len = static_cast<int64_t>(text_.size());
        }
      } else if (!streaming) {
        text_ = read_stream(in);
        text_len = static_cast<int64_t>(text_.size());
        text = text_.data();
      }
    } catch (const std::exception& e) {
      error = e.what();
      h.status = 1;
    }
    pt_.end();
  }
  if (sliced && ctx_.local_size > 1) {
    // an --input file read from its start: every rank maps it (page cache, nothing copied); otherwise the
    // root reads the input into a node-shared window
    const std::string path = flags_.get("input", "");
    int64_t sz[3] = {h.status, text_len,
                     ctx_.rank == kRoot && !path.empty() && text_.empty() && text_len > 0 && in && std::ftell(in) == 0};
    bcast_bytes(sz, sizeof sz, kRoot, ctx_.world);
    if (sz[0] != 0) {
      if (ctx_.rank == kRoot) std::fprintf(stderr, "input error: %s\n", error.c_str());
      if (in != stdin && in) std::fclose(in);
      return 1;
    }
    text_len = sz[1];
    if (sz[2]) {
      pt_.begin("map");
      text_map_ = std::make_unique<MappedFile>(path.c_str(), static_cast<size_t>(text_len));
      text_map_->set_releaser(&rel_);
      text = text_map_->data();
      pt_.end();
    } else {
      pt_.begin("window");
      text_win_ = std::make_unique<SharedWindow>(ctx_, text_len + 64);
      text_win_->prefault_shares(ctx_);  // every rank faults in a share of the pages the root reads into
      pt_.end();
      text = text_win_->base();
      if (ctx_.rank == kRoot) {
        pt_.begin("read");
        try {
          if (!text_.empty()) {
            const int64_t nt = text_len > (int64_t{1} << 24) ? omp_get_max_threads() : 1;
#pragma omp parallel for schedule(static, 1) num_threads(static_cast<int>(nt))
            for (int64_t t = 0; t < nt; ++t) {
              const int64_t b = text_len * t / nt, e = text_len * (t + 1) / nt;
              std::memcpy(text_win_->base() + b, text_.data() + b, static_cast<size_t>(e - b));
            }
            text_ = uvector<char>();
          } else {
            text_len = static_cast<int64_t>(read_regular_into(in, text_win_->base(), static_cast<size_t>(text_len)));
          }
        } catch (const std::exception& e) {
          error = e.what();
          h.status = 1;
        }
        pt_.end();
      }
    }
  }
  if (ctx_.rank == kRoot && h.status == 0) {
    pt_.begin("parse");
    try {
      Weights w{};
      if (streaming) {
        reader = std::make_unique<StreamReader>(in, po);
        w = reader->weights();
        seq1 = reader->seq1();
        h.n_total = reader->count();
        h.first_index = reader->skip(skip);
        h.cells = -1;
      } else {
        // header (+ pass 1 unless sliced: the ranks count their shares of the text then)
        auto parser = std::make_unique<BulkParser>(text, static_cast<size_t>(text_len), po, !sliced);
        w = parser->weights();
        seq1 = parser->seq1();
        h.n_total = parser->count();
        h.first_index = std::min<int64_t>(skip, h.n_total);
        h.cells = parser->cells_estimate();
        h.mean_l2 = parser->mean_length_estimate();
        // shm transport without a skip: pass 2 later writes straight into the node-shared window (sliced:
        // into every rank's own buffers); otherwise encode now into a private batch
        const bool into_window = sliced || (h.first_index == 0 && (tr_flag == "shm" || (tr_flag == "auto" && ctx_.single_node())));
        if (into_window) {
          parser_ = std::move(parser);
        } else {
          bulk.codes.resize(static_cast<size_t>(parser->total_chars()));
          bulk.offsets.resize(static_cast<size_t>(parser->count()) + 1);
          parser->fill(bulk.codes.data(), bulk.offsets.data());
          text_ = uvector<char>();
          drop_front(bulk, h.first_index);
        }
      }
      for (int i = 0; i < 4; ++i) h.w[i] = w.w[i];
      h.text_bytes = text_len;
    } catch (const std::exception& e) {
      error = e.what();
      h.status = 1;
    }
    pt_.end();
    h.semantics = static_cast<int32_t>(sem);
    h.L1 = static_cast<int64_t>(seq1.size());
  }

  // ---- header + Seq1 broadcast (exact counts)
  pt_.begin("bcast");
  fault_.at("bcast", ctx_.rank);
  bcast_bytes(&h, sizeof h, kRoot, ctx_.world);
  if (h.status != 0) {
    if (ctx_.rank == kRoot) std::fprintf(stderr, "input error: %s\n", error.c_str());
    if (in != stdin && in) std::fclose(in);
    return 1;
  }
  Weights w{};
  for (int i = 0; i < 4; ++i) w.w[i] = h.w[i];
  seq1.resize(static_cast<size_t>(h.L1));
  bcast_bytes(seq1.data(), h.L1, kRoot, ctx_.world);
  pt_.end();
  pt_.begin("gpu_wait");  // the HIP runtime's start-up, when a helper thread began it during the read
  if (prewarm_.valid()) prewarm_.get();
  pt_.end();
  pt_.begin("setup");
  setup_engine(h.cells, h.mean_l2);  // collective: engine kind, transport, RCCL communicator
  pt_.end();
  pt_.begin("problem");
  eng_.set_problem(w, seq1, sem);
  pt_.end();

  int rc = 0;
  if (sliced) {
    std::unique_ptr<BulkParser> own;
    if (ctx_.rank != kRoot) {  // the header again, from the shared text (no pass 1: counted together)
      if (text_win_) text_win_->fence();
      own = std::make_unique<BulkParser>(text, static_cast<size_t>(h.text_bytes), po, false);
    } else if (text_win_) {
      text_win_->fence();
    }
    try {
      run_sliced(ctx_.rank == kRoot ? *parser_ : *own, h.first_index);
    } catch (const InputError& e) {
      if (ctx_.rank == kRoot) std::fprintf(stderr, "input error: %s\n", e.what());
      if (in != stdin && in) std::fclose(in);
      return 1;
    }
    pt_.begin("teardown");
    // the parser's per-chunk tables go back to the OS on the releaser
    rel_.defer([p = std::shared_ptr<BulkParser>(parser_ ? std::move(parser_) : std::move(own))]() mutable { p.reset(); });
    pt_.end();
  } else if (!streaming) {
    int64_t sizes[2] = {bulk.size(), bulk.total_chars()};
    if (parser_) {
      sizes[0] = parser_->count();
      sizes[1] = parser_->total_chars();
    }
    bcast_bytes(sizes, sizeof sizes, kRoot, ctx_.world);
    try {
      run_batch(ctx_.rank == kRoot ? &bulk : nullptr, sizes[0], sizes[1], h.first_index);
    } catch (const InputError& e) {
      if (ctx_.rank == kRoot) std::fprintf(stderr, "input error: %s\n", e.what());
      if (in != stdin && in) std::fclose(in);
      return 1;
    }
  } else {
    // root: parse of batch b+1 runs on a helper thread while batch b is searched and printed
    const int64_t max_rec = batch_records > 0 ? batch_records : INT64_MAX;
    const int64_t max_chr = batch_chars > 0 ? batch_chars : INT64_MAX;
    auto parse_next = [&reader, max_rec, max_chr]() {
      auto b = std::make_unique<RecordBatch>();
      reader->next_batch(max_rec, *b, max_chr);
      return b;
    };
    std::future<std::unique_ptr<RecordBatch>> next;
    if (ctx_.rank == kRoot) next = std::async(std::launch::async, parse_next);
    int64_t first = h.first_index;
    while (true) {
      BatchHeader bh{};
      std::unique_ptr<RecordBatch> cur;
      if (ctx_.rank == kRoot) {
        pt_.begin("parse");
        try {
          cur = next.get();
          bh.n = cur->size();
          bh.total_chars = cur->total_chars();
          if (bh.n > 0) next = std::async(std::launch::async, parse_next);
        } catch (const std::exception& e) {
          error = e.what();
          bh.status = 1;
        }
        pt_.end();
      }
      bcast_bytes(&bh, sizeof bh, kRoot, ctx_.world);
      if (bh.status != 0) {
        if (ctx_.rank == kRoot) std::fprintf(stderr, "input error: %s\n", error.c_str());
        rc = 1;
        break;
      }
      if (bh.n == 0) break;
      run_batch(cur.get(), bh.n, bh.total_chars, first);
      first += bh.n;
    }
  }
  pt_.begin("close");
  if (in != stdin && in) std::fclose(in);
  const int close_rc = out_ != stdout ? close_output(out_) : 0;
  pt_.end();
  if (close_rc != 0 && rc == 0) {
    std::fprintf(stderr, "error while writing --output\n");
    rc = 1;
  }
  out_ = stdout;
  total_.stop();
  report(h);
  MPI_Barrier(ctx_.world);
  return rc;
}

}  // namespace

// An --input file of >= --gpu-prewarm-bytes will run on the GPU (unless --backend=cpu): the HIP runtime
// starts on a helper thread before MPI_Init, every rank deciding from the same flags and file.
std::future<void> early_prewarm(int argc, char** argv) {
  try {
    Flags flags(argc, argv);
    const std::string path = flags.get("input", "");
    if (path.empty() || to_lower(flags.get("backend", "auto")) == "cpu" || flags.get_bool("help", false)) return {};
    struct stat st {};
    const int64_t min_bytes = flags.get_int("gpu-prewarm-bytes", int64_t{64} << 20);
    if (stat(path.c_str(), &st) != 0 || !S_ISREG(st.st_mode) || min_bytes <= 0 || st.st_size < min_bytes) return {};
    return std::async(std::launch::async, [] { (void)gpu_device_count(); });
  } catch (const std::exception&) {
    return {};  // bad flags are reported after MPI_Init
  }
}

int main(int argc, char** argv) {
  // declared before the MPI context: its queued unmaps overlap the job's teardown and MPI_Finalize
  BackgroundReleaser releaser;
  std::future<void> prewarm = early_prewarm(argc, argv);
  MpiContext ctx(&argc, &argv);
  int rc = 0;
  try {
    Flags flags(argc, argv);
    if (flags.get_bool("help", false)) {
      if (ctx.rank == kRoot) std::printf("%sbuild: %s\n", kUsage, kBuildId);
      return 0;
    }
    auto unknown = flags.unknown(kKnown);
    if (!unknown.empty()) {
      if (ctx.rank == kRoot) std::fprintf(stderr, "unknown flag --%s\n%s", unknown[0].c_str(), kUsage);
      return 2;
    }
    Job job(ctx, flags, releaser, std::move(prewarm));
    rc = job.run();
  } catch (const std::exception& e) {
    ctx.abort(3, e.what());
  }
  return rc;
}
