// `final` — the CLI, behaviour-compatible with the reference binary (main.c:46-244):
//     mpiexec -np N ./final < inputX.txt   ->   "#i: score: S, n: N, k: K" per Seq2, input order.
//
// Flow (reference call stacks E2/E3), re-designed; the flows live in their own translation
// units (job.hpp):
//   1. MPI bootstrap; rank -> GPU by node-local rank or --device-map (reference: all ranks on GPU 0, B14).
//   2. Root reads the input header; the records are parsed later, in parallel, by the flow that uses them
//      (reference: racy parallel fscanf, B2).
//   3. Exact-count header/Seq1 broadcast (reference: 16 ints into int[4], B3).
//   4. The job runs one flow:
//        sliced  (bulk, one node)      every rank encodes its own slice of the node-shared text;
//        stream  (--batch-records/-chars, one node)  batch by batch through persistent page-locked rings,
//                                      encode / kernel / print overlapped;
//        text    (transports rccl / rccl-emul / mpi: multi-node, or chosen)  the root cuts bulk or streamed
//                batches from the text and encodes every rank's slice straight into its wire block
//                (device transports) or a byte-code batch (mpi);
//        batch   (--partition=offsets on any transport)  in-memory record batches, context parallel.
//      Decomposition: cost-balanced contiguous record ranges (valid for any -np, B4/B5/B6), or context
//      parallel (--partition=offsets: every rank searches a share of EVERY record's offsets, one MAX
//      all-reduce of packed 64-bit keys combines them — the Reduce the reference never had).
//   5. Root prints in input order.
// Any error on any rank -> message + MPI_Abort (reference: exit(1) without abort, peers hang, B11).
#include <fcntl.h>
#include <omp.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <future>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "job.hpp"
#include "moc/runtime/host_region.hpp"
#include "moc/runtime/kfd_topology.hpp"
#include "moc/runtime/log.hpp"
#include "moc/runtime/watchdog.hpp"

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

// The process's age in ms (CLOCK_MONOTONIC minus the start time in /proc/self/stat), -1 when unknown.
double ms_since_process_start() {
  static const double start = [] {
    FILE* f = std::fopen("/proc/self/stat", "r");
    if (!f) return -1.0;
    char buf[1024];
    const size_t n = std::fread(buf, 1, sizeof buf - 1, f);
    std::fclose(f);
    buf[n] = 0;
    const char* p = std::strrchr(buf, ')');
    unsigned long long st = 0;
    int field = 2;
    for (const char* q = p ? p + 1 : buf + n; *q && field < 22; ++q)
      if (*q == ' ' && ++field == 22) std::sscanf(q + 1, "%llu", &st);
    return st ? st * 1e3 / static_cast<double>(sysconf(_SC_CLK_TCK)) : -1.0;
  }();
  if (start < 0) return -1;
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e3 + ts.tv_nsec / 1e6 - start;
}
std::atomic<double> g_runtime_up_ms{-1};  // set by the prewarm thread once the HIP runtime answered
std::string g_gpu_isolation;  // set by isolate_gpu before MPI_Init: the one GPU this rank's runtime sees

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
    "  --timing-exit               a last stderr line: the teardown after the job (engine, MPI_Finalize,\n"
    "                              releaser) and the time since the process started\n"
    "  --gpu-isolate=auto|0|1      a rank taking its GPU by node-local rank shows the HIP runtime that GPU only\n"
    "                              (auto: several GPUs on the node, no --device/--device-map, no RCCL)\n"
    "  --quick-exit=0|1            1 (default): end with _Exit once outputs are closed and MPI is finalized,\n"
    "                              leaving the runtimes' static teardown to the kernel\n"
    "  --strict-limits             enforce |Seq1|<=3000, |Seq2|<=2000 (PDF p.5-6)\n"
    "  --max-l1=L --max-l2=L       explicit length limits (0 = unlimited)\n"
    "  --device=K                  force device K (default: node-local rank %% devices)\n"
    "  --device-map=a,b,...        node-local rank i -> device map[i %% len]\n"
    "  --pin-window=0|1            page-lock the GPU ranks' slices so they stream zero-copy (default 1)\n"
    "  --chunk-records=R --chunk-bytes=B   pipeline chunk sizes\n"
    "  --threads=T                 OpenMP threads (default: OMP_NUM_THREADS / all)\n"
    "  --mpi-topology=lean|full    lean (default): MPI_Init skips the host's hardware discovery (CPUs, caches,\n"
    "                              PCI devices: 0.2-0.35 s of a tiny job on a 256-CPU node); full: MPI's own\n"
    "  --log-level=error|warn|info|debug\n"
    "  --comm-timeout=SECONDS      deadline of every wait on another rank or on the RCCL comm lane (default 300;\n"
    "                              0 = none): past it the rank aborts the job naming its phase and the peers\n"
    "                              and bytes still outstanding\n"
    "  --inject-fault=[stall:|stall-device:]PHASE[:RANK]   test hook: fail (or stall) at\n"
    "                              parse|bcast|distribute|fill|pack|compute|gather\n"
    "every flag can also be given as environment variable MOC_<FLAG> (e.g. MOC_BACKEND=cpu)\n";

const std::vector<std::string> kKnown = {
    "backend", "collectives", "parallel-print", "gpu-min-cells", "gpu-prewarm-bytes", "transport", "semantics",
    "partition", "batch-records", "batch-chars", "skip-records", "input", "output", "timing", "strict-limits",
    "max-l1", "max-l2", "device", "device-map", "pin-window", "chunk-records", "chunk-bytes", "threads",
    "log-level", "inject-fault", "mpi-topology", "timing-exit", "quick-exit", "gpu-isolate", "comm-timeout", "help"};

struct BatchHeader {
  int64_t n;
  int64_t total_chars;
  int32_t status;  // 0 ok, else input error on root
  int32_t pad;
};

// Drops the first s records of a batch (bulk mode + --skip-records).
void drop_front(RecordBatch& b, int64_t s) {
  s = std::min<int64_t>(s, b.size());
  if (s <= 0) return;
  const int64_t c0 = b.offsets[s];
  b.codes.erase(b.codes.begin(), b.codes.begin() + c0);
  b.offsets.erase(b.offsets.begin(), b.offsets.begin() + s);
  for (auto& o : b.offsets) o -= c0;
}

class Job {
 public:
  Job(MpiContext& ctx, const Flags& flags, BackgroundReleaser& rel, std::future<void> prewarm)
      : job_(ctx, flags, rel), prewarm_(std::move(prewarm)) {
    job_.build_id = kBuildId;
  }
  int run();
  // A process that ends with _Exit (--quick-exit) leaves its GPU engine — streams, device buffers, page-locked
  // ranges — to the kernel driver instead of tearing it down first (17-27 ms on the MI355X box,
  // profiles/final_exit_1.1G_r3b_quick.log).
  void leave_engine_to_exit() { (void)job_.eng.hip.release(); }

 private:
  int fail(const std::string& e) {  // an input error every rank saw: message on root, exit code 1
    if (job_.ctx.rank == kRoot) std::fprintf(stderr, "input error: %s\n", e.c_str());
    if (in_ != stdin && in_) std::fclose(in_);
    in_ = nullptr;
    return 1;
  }
  void prewarm_gpu();
  bool open_io(std::string& error);
  int run_streamed(const Header& h, bool shm_flow, int64_t batch_records, int64_t batch_chars, const ParseOptions& po);

  JobCore job_;
  std::future<void> prewarm_;  // HIP runtime start-up overlapped with the read (large inputs)
  FILE* in_ = stdin;
  uvector<char> text_;                      // root: the input (kept for deferred parsing)
  std::unique_ptr<BulkParser> parser_;      // root: header read, pass 2 deferred
  std::unique_ptr<SharedWindow> text_win_;  // sliced mode, several ranks on the node: the input text
  std::unique_ptr<MappedFile> text_map_;    // ... or, for an --input file, every rank's mapping of it
  std::unique_ptr<StreamReader> reader_;    // root: streaming over a non-shm transport
  StreamSource stream_;                     // streaming on one node
};

// A large input (a regular file of >= --gpu-prewarm-bytes) will run on the GPU: every rank brings the HIP
// runtime up on a helper thread while the root reads and parses, instead of after the header bcast.
void Job::prewarm_gpu() {
  const Flags& flags = job_.flags;
  int64_t hint = 0;
  if (job_.ctx.rank == kRoot && to_lower(flags.get("backend", "auto")) != "cpu") {
    const std::string path = flags.get("input", "");
    struct stat st {};
    const int rc = path.empty() ? fstat(STDIN_FILENO, &st) : stat(path.c_str(), &st);
    const int64_t min_bytes = flags.get_int("gpu-prewarm-bytes", int64_t{64} << 20);
    hint = rc == 0 && S_ISREG(st.st_mode) && min_bytes > 0 && st.st_size >= min_bytes;
  }
  bcast_bytes(&hint, sizeof hint, kRoot, job_.ctx.world);
  if (hint && !prewarm_.valid())
    prewarm_ = std::async(std::launch::async, [] {
      (void)gpu_device_count();
      g_runtime_up_ms.store(ms_since_process_start());
    });
}

bool Job::open_io(std::string& error) {
  try {
    const std::string path = job_.flags.get("input", "");
    if (!path.empty() && !(in_ = std::fopen(path.c_str(), "rb"))) throw Error("cannot open --input " + path);
    const std::string opath = job_.flags.get("output", "");
    if (!opath.empty() && !(job_.out = open_output(opath))) {
      job_.out = stdout;
      throw Error("cannot open --output " + opath);
    }
    return true;
  } catch (const std::exception& e) {
    error = e.what();
    return false;
  }
}

// Streaming with record slices on one node (the node's streaming flow), or context-parallel streaming
// (--partition=offsets): batches from a StreamReader over the job's transport.
int Job::run_streamed(const Header& h0, bool shm_flow, int64_t batch_records, int64_t batch_chars,
                      const ParseOptions& po) {
  const MpiContext& ctx = job_.ctx;
  if (shm_flow) return run_streaming(job_, h0, stream_, batch_records, batch_chars, po);
  // root: parse of batch b+1 runs on a helper thread while batch b is searched and printed
  const int64_t max_rec = batch_records > 0 ? batch_records : INT64_MAX;
  const int64_t max_chr = batch_chars > 0 ? batch_chars : INT64_MAX;
  StreamReader* reader = reader_.get();
  auto parse_next = [reader, max_rec, max_chr]() {
    auto b = std::make_unique<RecordBatch>();
    reader->next_batch(max_rec, *b, max_chr);
    return b;
  };
  std::future<std::unique_ptr<RecordBatch>> next;
  if (ctx.rank == kRoot) next = std::async(std::launch::async, parse_next);
  int64_t first = h0.first_index;
  std::string error;
  while (true) {
    BatchHeader bh{};
    std::unique_ptr<RecordBatch> cur;
    if (ctx.rank == kRoot) {
      job_.pt.begin("parse");
      try {
        cur = next.get();
        bh.n = cur->size();
        bh.total_chars = cur->total_chars();
        if (bh.n > 0) next = std::async(std::launch::async, parse_next);
      } catch (const std::exception& e) {
        error = e.what();
        bh.status = 1;
      }
      job_.pt.end();
    }
    bcast_bytes(&bh, sizeof bh, kRoot, ctx.world);
    if (bh.status != 0) return fail(error);
    if (bh.n == 0) return 0;
    run_record_batch(job_, cur.get(), bh.n, bh.total_chars, first);
    first += bh.n;
  }
}

int Job::run() {
  MpiContext& ctx = job_.ctx;
  const Flags& flags = job_.flags;
  PhaseTimer& pt = job_.pt;
  log_set_level(flags.get("log-level", "warn"));
  log_set_rank(ctx.rank);
  if (!g_gpu_isolation.empty()) MOC_LOG_INFO("runtime isolated to %s", g_gpu_isolation.c_str());
  job_.fault.parse(flags.get("inject-fault", ""));
  const std::string sem_s = to_lower(flags.get("semantics", "reference"));
  if (sem_s != "reference" && sem_s != "spec") throw Error("--semantics must be reference|spec");
  const Semantics sem = sem_s == "spec" ? Semantics::Spec : Semantics::Reference;
  const int64_t batch_records = flags.get_int("batch-records", 0);
  const int64_t batch_chars = flags.get_int("batch-chars", 0);
  const int64_t skip = flags.get_int("skip-records", 0);
  if (batch_records < 0 || batch_chars < 0 || skip < 0) throw Error("--batch-records/--batch-chars/--skip-records >= 0");
  const bool streaming = batch_records > 0 || batch_chars > 0;
  ParseOptions po;
  po.strict_limits = flags.get_bool("strict-limits", false);
  po.max_l1 = flags.get_int("max-l1", 0);
  po.max_l2 = flags.get_int("max-l2", 0);

  // OpenMP threads: --threads, else OMP_NUM_THREADS, else the node's cores shared by its ranks
  int threads = static_cast<int>(flags.get_int("threads", 0));
  if (threads <= 0 && !std::getenv("OMP_NUM_THREADS")) threads = std::max(1, omp_get_num_procs() / ctx.local_size);
  if (threads > 0) omp_set_num_threads(threads);
  // the root formats the rows while the node's other ranks wait for it: it may use their threads too
  // (not when OMP_NUM_THREADS fixes every process's team by itself)
  if (threads > 0 && ctx.local_size > 1)
    job_.print_threads = std::min(omp_get_num_procs(), threads * ctx.local_size);
  job_.total.start();
  prewarm_gpu();

  // One node with record slices (shm transport): a bulk job runs "sliced" (every rank encodes its own slice
  // from the input text, read into a node-shared window when the node has several ranks), a streaming job
  // runs the node's streaming flow. Anything else parses on the root into record batches.
  const std::string tr_flag = to_lower(flags.get("transport", "auto"));
  const bool one_node_slices = to_lower(flags.get("partition", "cost")) != "offsets" &&
                               (tr_flag == "shm" || (tr_flag == "auto" && ctx.single_node()));
  const bool sliced = !streaming && one_node_slices;
  const bool shm_stream = streaming && one_node_slices;
  // a bulk record-slice job off the node's shm transport: the root encodes the ranks' slices straight from
  // the text after the engines are up (run_text_batch)
  const bool text_batch = !streaming && !one_node_slices && to_lower(flags.get("partition", "cost")) != "offsets";
  // ... and a streamed one: the root cuts the batches from the text (run_device_streaming)
  const bool dev_stream = streaming && !one_node_slices && to_lower(flags.get("partition", "cost")) != "offsets";
  const std::string in_path = flags.get("input", "");
  Header h{};
  std::string error;
  RecordBatch bulk;
  std::vector<uint8_t> seq1;
  const char* text = nullptr;  // sliced / mapped streaming: the input text (every rank)
  int64_t text_len = 0;
  if (ctx.rank == kRoot) {
    pt.begin("read");
    try {
      job_.fault.at("parse", ctx.rank);
      if (!open_io(error)) throw Error(error);
      if ((sliced && ctx.local_size > 1) || (shm_stream && !in_path.empty())) {
        text_len = regular_input_bytes(in_);  // mapped, or read straight into the shared window below
        if (text_len < 0 && sliced) {         // a pipe: read it all first
          text_ = read_stream(in_);
          text_len = static_cast<int64_t>(text_.size());
        }
      } else if (dev_stream && !in_path.empty()) {  // the root maps an --input file read from its start
        text_len = regular_input_bytes(in_);
        if (text_len > 0 && std::ftell(in_) == 0) {
          text_map_ = std::make_unique<MappedFile>(in_path.c_str(), static_cast<size_t>(text_len));
          text_map_->set_releaser(&job_.rel);
          text = text_map_->data();
        }
      } else if (!streaming) {
        text_ = read_stream(in_);
        text_len = static_cast<int64_t>(text_.size());
        text = text_.data();
      }
    } catch (const std::exception& e) {
      error = e.what();
      h.status = 1;
    }
    pt.end();
  }
  if ((sliced && ctx.local_size > 1) || (shm_stream && !in_path.empty())) {
    // an --input file read from its start: every rank maps it (page cache, nothing copied); otherwise the
    // root reads the input into a node-shared window
    int64_t sz[3] = {h.status, text_len,
                     ctx.rank == kRoot && !in_path.empty() && text_.empty() && text_len > 0 && in_ && std::ftell(in_) == 0};
    bcast_bytes(sz, sizeof sz, kRoot, ctx.world);
    if (sz[0] != 0) return fail(error);
    text_len = sz[1];
    if (sz[2]) {
      pt.begin("map");
      text_map_ = std::make_unique<MappedFile>(in_path.c_str(), static_cast<size_t>(text_len));
      text_map_->set_releaser(&job_.rel);
      text = text_map_->data();
      pt.end();
    } else if (sliced) {
      pt.begin("window");
      text_win_ = std::make_unique<SharedWindow>(ctx, text_len + 64);
      text_win_->prefault_shares(ctx);  // every rank faults in a share of the pages the root reads into
      pt.end();
      text = text_win_->base();
      if (ctx.rank == kRoot) {
        pt.begin("read");
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
            text_len = static_cast<int64_t>(read_regular_into(in_, text_win_->base(), static_cast<size_t>(text_len)));
          }
        } catch (const std::exception& e) {
          error = e.what();
          h.status = 1;
        }
        pt.end();
      }
    }
  }
  if (ctx.rank == kRoot && h.status == 0) {
    pt.begin("parse");
    try {
      Weights w{};
      if ((shm_stream || dev_stream) && text) {  // mapped: the header from the mapping, the records by the flow
        BulkParser hdr(text, static_cast<size_t>(text_len), po, false);
        w = hdr.weights();
        seq1 = hdr.seq1();
        h.n_total = hdr.count();
        h.first_index = std::min<int64_t>(skip, h.n_total);
        h.cells = -1;
        stream_.mapped = text;
        stream_.mapped_bytes = text_len;
        stream_.area_begin = text_len - hdr.area_bytes();
      } else if (streaming) {
        reader_ = std::make_unique<StreamReader>(in_, po);
        w = reader_->weights();
        seq1 = reader_->seq1();
        h.n_total = reader_->count();
        h.cells = -1;
        if (shm_stream || dev_stream) {  // the flow reads the rest of the stream itself
          h.first_index = std::min<int64_t>(skip, h.n_total);
          stream_.in = in_;
          stream_.eof = reader_->take_rest(stream_.head);
        } else {
          h.first_index = reader_->skip(skip);
        }
      } else {
        // header (+ pass 1 unless sliced: the ranks count their shares of the text then)
        auto parser = std::make_unique<BulkParser>(text, static_cast<size_t>(text_len), po, !sliced && !text_batch);
        w = parser->weights();
        seq1 = parser->seq1();
        h.n_total = parser->count();
        h.first_index = std::min<int64_t>(skip, h.n_total);
        h.cells = parser->cells_estimate();
        h.mean_l2 = parser->mean_length_estimate();
        // shm transport without a skip: pass 2 later writes straight into the node-shared window (sliced:
        // into every rank's own buffers); otherwise encode now into a private batch
        if (sliced || text_batch) {
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
    pt.end();
    h.semantics = static_cast<int32_t>(sem);
    h.L1 = static_cast<int64_t>(seq1.size());
  }

  // ---- header + Seq1 broadcast (exact counts)
  pt.begin("bcast");
  job_.fault.at("bcast", ctx.rank);
  bcast_bytes(&h, sizeof h, kRoot, ctx.world);
  if (h.status != 0) return fail(error);
  Weights w{};
  for (int i = 0; i < 4; ++i) w.w[i] = h.w[i];
  seq1.resize(static_cast<size_t>(h.L1));
  bcast_bytes(seq1.data(), h.L1, kRoot, ctx.world);
  pt.end();
  // A job that connects RCCL first lets the warm-up communicator of early_prewarm finish. Other GPU jobs do
  // not wait here: the HIP runtime keeps starting on the helper thread while the ranks count and encode,
  // and the engine's own helper thread is the first to need it.
  pt.begin("gpu_wait");
  {
    const std::string tr = to_lower(flags.get("transport", "auto"));
    const bool rccl_job = tr == "rccl" || to_lower(flags.get("collectives", "auto")) == "rccl" ||
                          (tr == "auto" && !ctx.single_node());
    if (prewarm_.valid() && rccl_job) prewarm_.get();
  }
  pt.end();
  pt.begin("setup");
  job_.setup_engine(h.cells, h.mean_l2);  // collective: engine kind, transport, RCCL communicator
  pt.end();
  pt.begin("problem");
  job_.eng.set_problem(w, seq1, sem);
  pt.end();
  if (shm_stream && ctx.rank != kRoot && text) {  // every rank streams from its mapping of the file
    stream_.mapped = text;
    stream_.mapped_bytes = text_len;
  }

  int rc = 0;
  try {
    if (sliced) {
      std::unique_ptr<BulkParser> own;
      if (ctx.rank != kRoot) {  // the header again, from the shared text (no pass 1: counted together)
        if (text_win_) text_win_->fence();
        own = std::make_unique<BulkParser>(text, static_cast<size_t>(h.text_bytes), po, false);
      } else if (text_win_) {
        text_win_->fence();
      }
      run_sliced(job_, ctx.rank == kRoot ? *parser_ : *own, h.first_index, text_win_.get(), &text_);
      pt.begin("release");
      text_win_.reset();  // collective (node-shared input text)
      // the parser's per-chunk tables go back to the OS on the releaser
      job_.rel.defer([p = std::shared_ptr<BulkParser>(parser_ ? std::move(parser_) : std::move(own))]() mutable { p.reset(); });
      pt.end();
    } else if (text_batch) {
      run_text_batch(job_, parser_, h.first_index, &text_);
    } else if (!streaming) {
      int64_t sizes[2] = {bulk.size(), bulk.total_chars()};
      if (parser_) {
        sizes[0] = parser_->count();
        sizes[1] = parser_->total_chars();
      }
      bcast_bytes(sizes, sizeof sizes, kRoot, ctx.world);
      run_record_batch(job_, ctx.rank == kRoot ? &bulk : nullptr, sizes[0], sizes[1], h.first_index, &parser_, &text_);
    } else {
      rc = dev_stream ? run_device_streaming(job_, h, stream_, batch_records, batch_chars, po)
                      : run_streamed(h, shm_stream, batch_records, batch_chars, po);
    }
  } catch (const InputError& e) {
    return fail(e.what());
  }
  pt.begin("close");
  if (in_ != stdin && in_) std::fclose(in_);
  in_ = nullptr;
  const int close_rc = job_.out != stdout ? close_output(job_.out) : 0;
  pt.end();
  if (close_rc != 0 && rc == 0) {
    std::fprintf(stderr, "error while writing --output\n");
    rc = 1;
  }
  job_.out = stdout;
  job_.total.stop();
  if (const double up = g_runtime_up_ms.load(); up >= 0) {  // --timing: when the prewarm saw the HIP runtime up
    char buf[32];
    std::snprintf(buf, sizeof buf, "%.3f", up);
    job_.extra_timing.emplace_back("runtime_up_since_start_ms", buf);
  }
  job_.report(h);
  barrier(ctx.world, "MPI_Ibarrier (job end)");
  return rc;
}

}  // namespace

// Start-up work for a helper thread, decided before MPI_Init from the same flags and environment on every
// rank:
//   * an --input file of >= --gpu-prewarm-bytes will run on the GPU (unless --backend=cpu), and so will any
//     job with --backend=hip: the HIP runtime starts;
//   * a job that will use RCCL (--transport=rccl, --collectives=rccl, or the auto transport across nodes)
//     also pays RCCL's one-time start-up there — 1.7 s of library registration and code-object loading,
//     profiles/rccl_init_rootcause.log — on the rank's device (node-local rank from the launcher's
//     environment), so the communicator set-up after the header broadcast takes ~60 ms.
int env_int(const char* name, int fallback) {
  const char* v = std::getenv(name);
  return v && *v ? std::atoi(v) : fallback;
}

std::future<void> early_prewarm(int argc, char** argv) {
  try {
    Flags flags(argc, argv);
    if (to_lower(flags.get("backend", "auto")) == "cpu" || flags.get_bool("help", false)) return {};
    const std::string tr = to_lower(flags.get("transport", "auto"));
    // MPICH's hydra exports the node-local rank and size, Open MPI its own names
    const int local = env_int("MPI_LOCALRANKID", env_int("OMPI_COMM_WORLD_LOCAL_RANK", 0));
    const int local_n = env_int("MPI_LOCALNRANKS", env_int("OMPI_COMM_WORLD_LOCAL_SIZE", 1));
    const int world = env_int("PMI_SIZE", env_int("OMPI_COMM_WORLD_SIZE", 1));
    const bool rccl = tr == "rccl" || to_lower(flags.get("collectives", "auto")) == "rccl" ||
                      (tr == "auto" && world > local_n);
    const std::string path = flags.get("input", "");
    struct stat st {};
    const int64_t min_bytes = flags.get_int("gpu-prewarm-bytes", int64_t{64} << 20);
    const bool big = !path.empty() && stat(path.c_str(), &st) == 0 && S_ISREG(st.st_mode) && min_bytes > 0 &&
                     st.st_size >= min_bytes;
    // --backend=hip: the job will use the GPU whatever its size, so its runtime starts now, beside MPI_Init,
    // the read and the header broadcast, instead of at the engine's set-up
    const bool hip = to_lower(flags.get("backend", "auto")) == "hip";
    if (!big && !rccl && !hip) return {};
    int device = static_cast<int>(flags.get_int("device", -1));
    const std::vector<int> map = parse_int_list(flags.get("device-map", ""));
    if (device < 0 && !map.empty()) device = map[static_cast<size_t>(local) % map.size()];
    return std::async(std::launch::async, [rccl, device, local] {
      const int n = gpu_device_count();
      g_runtime_up_ms.store(ms_since_process_start());
      if (rccl && n > 0) (void)gpu_rccl_warmup(device >= 0 ? device : local % n);
    });
  } catch (const std::exception&) {
    return {};  // bad flags are reported after MPI_Init
  }
}

// --gpu-isolate=auto|0|1: a GPU rank that takes its device by node-local rank lets the HIP runtime see that
// one GPU (ROCR_VISIBLE_DEVICES = its index among the GPUs the driver gives the process; HIP_/CUDA_
// VISIBLE_DEVICES and GPU_DEVICE_ORDINAL, when set, become 0): on an 8-GPU node each rank's runtime would
// otherwise start all 8 devices, 8 processes at once. auto isolates when the node shows more than one GPU,
// no --device / --device-map names one, the launcher exported the node-local rank, and the job uses no
// RCCL (its peer-to-peer transport maps the peers' GPUs); 1 isolates whenever the topology answers (tests).
// Runs before any thread starts (setenv); what it did goes to g_gpu_isolation, for the rank's log.
void isolate_gpu(int argc, char** argv) {
  try {
    Flags flags(argc, argv);
    const std::string mode = to_lower(flags.get("gpu-isolate", "auto"));
    if (mode == "0" || to_lower(flags.get("backend", "auto")) == "cpu" || flags.get_bool("help", false)) return;
    if (flags.get_int("device", -1) >= 0 || !flags.get("device-map", "").empty()) return;
    const char* local_env = std::getenv("MPI_LOCALRANKID");
    if (!local_env) local_env = std::getenv("OMPI_COMM_WORLD_LOCAL_RANK");
    const int world = env_int("PMI_SIZE", env_int("OMPI_COMM_WORLD_SIZE", 1));
    if (!local_env && world > 1) return;  // the node-local rank is only known after MPI_Init
    const int local = local_env ? std::atoi(local_env) : 0;
    const int local_n = env_int("MPI_LOCALNRANKS", env_int("OMPI_COMM_WORLD_LOCAL_SIZE", 1));
    const std::string tr = to_lower(flags.get("transport", "auto"));
    if (tr == "rccl" || to_lower(flags.get("collectives", "auto")) == "rccl" || (tr == "auto" && world > local_n))
      return;
    KfdPaths raw_paths;
    raw_paths.honour_visible_env = false;
    const auto all = kfd_gpus(raw_paths);
    const auto visible = kfd_gpus();
    if (!all || !visible || visible->empty() || (mode == "auto" && visible->size() < 2)) return;
    const int idx = kfd_isolation_index(*all, *visible, local);
    if (idx < 0) return;
    // by the GPU's UUID when the driver gives one: an index counts the GPUs the runtime can open, which
    // a device cgroup can narrow without the topology (or the render nodes' permissions) showing it
    const KfdGpu& g = (*all)[static_cast<size_t>(idx)];
    std::string uuid = kfd_uuid(g);
    for (const KfdGpu& o : *all)  // partitions of one device may share its id: an index is exact then
      if (o.node != g.node && o.unique_id == g.unique_id) uuid.clear();
    const std::string value = uuid.empty() ? std::to_string(idx) : uuid;
    setenv("ROCR_VISIBLE_DEVICES", value.c_str(), 1);
    for (const char* v : {"HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "GPU_DEVICE_ORDINAL"})
      if (std::getenv(v)) setenv(v, "0", 1);
    g_gpu_isolation = "gpu " + g.pci_bus_id + " (ROCR_VISIBLE_DEVICES=" + value + ", " + std::to_string(idx + 1) +
                      " of " + std::to_string(visible->size()) + " visible)";
  } catch (const std::exception&) {
    // bad flags are reported after MPI_Init
  }
}

// --mpi-topology, read before MPI_Init (and before any helper thread: setenv)
void prepare_mpi(int argc, char** argv) {
  bool lean = true;
  try {
    lean = to_lower(Flags(argc, argv).get("mpi-topology", "lean")) != "full";
  } catch (const std::exception&) {
  }
  mpi_prepare_env(lean);
}

// --timing-exit on the root: where the process's teardown goes after the job's report (the Job's destructor —
// engine, pinned ranges, rings —, MPI_Finalize, the helper threads, the releaser's queued unmaps), printed
// as the last stderr line with each mark's time since the process started (/proc/self/stat), so the
// launcher's wall clock minus the last mark is the exit after main (static destructors, the kernel).
class ExitClock {
 public:
  void enable() { on_ = true; }
  void mark(const char* what) {
    if (on_) marks_.emplace_back(what, now_ms());
  }
  ~ExitClock() { print(); }
  void print() {
    if (!on_ || marks_.empty()) return;
    on_ = false;
    const double t0 = process_start_ms();
    std::string out = "{\"exit_timing_ms\": {";
    char buf[96];
    for (size_t i = 0; i < marks_.size(); ++i) {
      std::snprintf(buf, sizeof buf, "%s\"%s\": %.3f", i ? ", " : "", marks_[i].first,
                    i ? marks_[i].second - marks_[i - 1].second : 0.0);
      out += buf;
    }
    std::snprintf(buf, sizeof buf, "}, \"since_process_start_ms\": %.3f}\n", t0 >= 0 ? marks_.back().second - t0 : -1.0);
    out += buf;
    std::fputs(out.c_str(), stderr);
  }

 private:
  static double now_ms() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec / 1e6;
  }
  // the process's start on CLOCK_MONOTONIC's scale (boot-relative, field 22 of /proc/self/stat), -1 unknown
  static double process_start_ms() {
    FILE* f = std::fopen("/proc/self/stat", "r");
    if (!f) return -1;
    char buf[1024];
    const size_t n = std::fread(buf, 1, sizeof buf - 1, f);
    std::fclose(f);
    buf[n] = 0;
    const char* p = std::strrchr(buf, ')');
    unsigned long long st = 0;
    int field = 2;
    for (const char* q = p ? p + 1 : buf + n; *q && field < 22; ++q)
      if (*q == ' ' && ++field == 22) std::sscanf(q + 1, "%llu", &st);
    return st ? st * 1e3 / static_cast<double>(sysconf(_SC_CLK_TCK)) : -1;
  }
  bool on_ = false;
  std::vector<std::pair<const char*, double>> marks_;
};

// Ends the process with _Exit after main's own teardown (--quick-exit=1, the default): not under the host
// sanitizers, whose leak check runs at exit.
bool quick_exit_enabled(bool flag) {
#if defined(__SANITIZE_ADDRESS__) || defined(__SANITIZE_THREAD__)
  return false;
#elif defined(__has_feature)
#if __has_feature(address_sanitizer) || __has_feature(thread_sanitizer)
  return false;
#endif
#endif
  return flag;
}

int main(int argc, char** argv) {
  prepare_mpi(argc, argv);
  isolate_gpu(argc, argv);
  ExitClock exit_clock;  // destroyed last
  // declared before the MPI context: its queued unmaps overlap the job's teardown and MPI_Finalize
  BackgroundReleaser releaser;
  std::future<void> prewarm = early_prewarm(argc, argv);
  auto ctx = std::make_unique<MpiContext>(&argc, &argv);
  int rc = 0;
  bool quick_exit = true;
  try {
    Flags flags(argc, argv);
    if (flags.get_bool("help", false)) {
      if (ctx->rank == kRoot) std::printf("%sbuild: %s\n", kUsage, kBuildId);
      return 0;
    }
    auto unknown = flags.unknown(kKnown);
    if (!unknown.empty()) {
      if (ctx->rank == kRoot) std::fprintf(stderr, "unknown flag --%s\n%s", unknown[0].c_str(), kUsage);
      return 2;
    }
    const std::string topo = to_lower(flags.get("mpi-topology", "lean"));
    if (topo != "lean" && topo != "full") {
      if (ctx->rank == kRoot) std::fprintf(stderr, "--mpi-topology must be lean|full\n");
      return 2;
    }
    if (ctx->rank == kRoot && flags.get_bool("timing-exit", false)) exit_clock.enable();
    watchdog::set_timeout_s(flags.get_double("comm-timeout", watchdog::kDefaultTimeoutS));
    quick_exit = flags.get_bool("quick-exit", true);
    {
      Job job(*ctx, flags, releaser, std::move(prewarm));
      rc = job.run();
      exit_clock.mark("job_done");
      if (quick_exit_enabled(quick_exit)) job.leave_engine_to_exit();
    }
    exit_clock.mark("job_teardown");
  } catch (const std::exception& e) {
    // the phase the rank was in (a comm timeout names it already)
    const std::string ph = watchdog::phase();
    const std::string msg = e.what();
    ctx->abort(3, ph.empty() || msg.find("in phase '") != std::string::npos ? msg : msg + " (phase '" + ph + "')");
  }
  ctx.reset();
  exit_clock.mark("mpi_finalize");
  if (prewarm.valid()) prewarm.wait();
  releaser.stop();
  exit_clock.mark("releaser_drain");
  if (quick_exit_enabled(quick_exit)) {
    // every output is flushed and closed and MPI is finalized: the rest of a normal exit is the runtimes'
    // static teardown (the HIP runtime's queues, streams and device memory), which the kernel driver
    // does anyway when the process goes
    exit_clock.print();
    std::fflush(nullptr);
    std::_Exit(rc);
  }
  return rc;
}
