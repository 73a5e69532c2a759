// The `final` CLI's job state and its flows, one translation unit per flow (reference: the whole flow is
// main() in /root/reference/main.c:46-244):
//   final.cpp        CLI, flags, read + header broadcast, engine set-up, dispatch, --timing report
//   job_common.cpp   engine selection (GPU plugin), transports' small collectives, print, report
//   flow_sliced.cpp  bulk job on one node: every rank encodes its own slice of the node-shared text
//   flow_stream.cpp  streaming job on one node: batch by batch through persistent page-locked rings
//   flow_batch.cpp   one in-memory batch over the shm / mpi / rccl(-emul) transports (multi-node jobs,
//                    context-parallel jobs, the StreamReader path)
#pragma once

#include <omp.h>

#include <cstdio>
#include <functional>
#include <future>
#include <memory>
#include <string>
#include <vector>

#include "moc/comm.hpp"
#include "moc/cpu_engine.hpp"
#include "moc/gpu_rank.hpp"
#include "moc/io.hpp"
#include "moc/mpi_device_comm.hpp"
#include "moc/partition.hpp"
#include "moc/problem.hpp"
#include "moc/runtime/flags.hpp"
#include "moc/runtime/releaser.hpp"
#include "moc/runtime/timer.hpp"
#include "moc/score_table.hpp"
#include "moc/wire.hpp"

namespace moc {

// Exact-size job header, broadcast once (reference: 16 ints into int[4], main.c:150, bug B3).
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

// An input problem found after the header went out; raised on every rank after a status exchange, so all
// of them leave the job the same way (exit code 1).
struct InputError : Error {
  using Error::Error;
};

// --inject-fault=[stall:|stall-device:]PHASE[:RANK] (test hooks, rank 0 by default). Plain: the rank throws
// at the start of PHASE (the fail-fast path: message + MPI_Abort). stall: the rank's thread sleeps there
// for MOC_STALL_S seconds (default 120) — a peer that is alive but stuck, which the other ranks' comm
// deadline must name. stall-device: the rank's device comm lane is held busy instead (a bounded spin
// kernel on a GPU rank; MOC_STALL_S default 3), so its own deadline-polled waits expire.
struct FaultHook {
  enum class Kind { Fail, Stall, StallDevice };
  Kind kind = Kind::Fail;
  std::string phase;
  int rank = 0;
  double stall_s = 0;  // 0: the kind's default
  void parse(const std::string& spec);
  // `dc`: the flow's device comm, the target of stall-device (nullptr: the thread sleeps instead)
  void at(const char* p, int my_rank, DeviceComm* dc = nullptr) const;
};

std::string to_lower(std::string s);
std::vector<int> parse_int_list(const std::string& s);

// The GPU plugin (moc/gpu_rank.hpp), loaded on the first question about GPUs.
int gpu_device_count();
// GPUs this rank may open, from the driver's topology when it is readable (no HIP runtime start-up), else
// gpu_device_count()
int gpu_device_count_fast();
std::string gpu_plugin_error();
// RCCL's one-time start-up (library load + code objects) on `device`, for a helper thread (false: none).
bool gpu_rccl_warmup(int device);
GpuRank* gpu_rank_create(const MpiContext& ctx, const GpuRankOptions& opt);

// The selected engine of this rank over contiguous host slices.
struct RankEngine {
  bool gpu = false;
  std::unique_ptr<GpuRank> hip;
  ScoreTable table{};
  std::vector<uint8_t> seq1;
  Semantics sem = Semantics::Reference;
  int threads = 0;
  double kernel_ms = 0;  // accumulated device time of the search kernels

  void set_problem(const Weights& w, const std::vector<uint8_t>& s1, Semantics s);
  void solve(const uint8_t* codes, const int64_t* offsets, int64_t n, Result* out);
  // context-parallel share `part` of `parts` of every record -> packed keys
  void solve_keys(const uint8_t* codes, const int64_t* offsets, int64_t n, int part, int parts, uint64_t* keys);
};

// What every flow shares: the rank's context, its engine, the transport choice, timers and counters.
struct JobCore {
  JobCore(MpiContext& c, const Flags& f, BackgroundReleaser& r) : ctx(c), flags(f), rel(r) {}
  MpiContext& ctx;
  const Flags& flags;
  BackgroundReleaser& rel;  // large frees off the critical path (drained after MPI_Finalize)
  FaultHook fault;
  RankEngine eng;
  int device = -1;
  bool all_gpu = false;
  std::string transport, partition;
  bool pin_window = true;
  bool coll_rccl = false;  // shm transport: host-table collectives over RCCL (--collectives=rccl)
  std::unique_ptr<MpiDeviceComm> emul_comm;  // --transport=rccl-emul
  std::unique_ptr<DeviceScratch> scratch;    // rccl(-emul) batches: device / page-locked buffers kept across batches
  PhaseTimer pt;
  Stopwatch total;
  FILE* out = stdout;  // root: --output file, else stdout
  double compute_ms = 0;
  int64_t cells = 0, chars = 0, records = 0, batches = 0;
  int64_t first_index = 0;  // global index of the current batch's first record
  int64_t pinned_bytes = 0, h2d_bytes = 0, d2h_bytes = 0;  // this rank (--timing)
  // rccl(-emul) transport (--timing): bytes this rank sent over the comm, the root's bytes to each rank and
  // its distribution time (per-peer rate = bytes / time)
  int64_t comm_sent_bytes = 0;
  std::vector<int64_t> peer_sent;
  double distribute_ms = 0;
  std::vector<int> fill_order;  // root, text batches: the order the slices were encoded (the first batch's)
  std::vector<int64_t> rank_pinned, rank_h2d, rank_records, rank_pin_us;  // root: per rank (--timing)
  std::vector<std::pair<std::string, std::string>> extra_timing;          // flow-specific --timing fields
  const char* build_id = "";  // the sources of this binary (--timing)
  // root: OpenMP threads for formatting the rows, which the other ranks of the node wait for (0: the
  // rank's own count). The node's thread budget, when the ranks' counts were divided from it.
  int print_threads = 0;

  // collective: engine kind, transport, RCCL communicator (cells < 0: unknown)
  void setup_engine(int64_t job_cells, int64_t mean_l2);
  // MPI_Allgather of `count` int64 per rank, or the same over RCCL (--collectives=rccl)
  void allgather_i64(const int64_t* mine, int count, int64_t* all);
  // in-place MAX of packed keys over the ranks (context-parallel combine), MPI or RCCL
  void allreduce_keys(uint64_t* keys, int64_t n);
  // root: MAX-combined pass-1 keys -> results (k resolved on the winning diagonals)
  void resolve_keys(const uint64_t* keys, const uint8_t* codes, const int64_t* offsets, int64_t n, Result* res);
  // root: rows of the current batch (first = index relative to the batch)
  void print(const Result* r, int64_t n, int64_t first);
  CostModel cost_model() const { return all_gpu ? CostModel{1.0, 200.0, 2400.0} : CostModel{1.0, 4.0, 64.0}; }
  // adds a device batch's comm traffic to the job's (--timing)
  void account_comm(const DeviceBatchOut& out);
  // collective: the --timing JSON line on root's stderr
  void report(const Header& h);
};

// Sets the calling thread's OpenMP team size for a scope (n <= 0: unchanged).
class ScopedOmpThreads {
 public:
  explicit ScopedOmpThreads(int n) : prev_(omp_get_max_threads()) {
    if (n > 0) omp_set_num_threads(n);
  }
  ~ScopedOmpThreads() { omp_set_num_threads(prev_); }

 private:
  int prev_;
};

// ---- flows
// Bulk job on one node in record slices (flow_sliced.cpp). `text_win`: the node-shared input text, when
// the root read the input into one (released in shares once every slice is encoded); `text`: root's
// private copy of it, if any (released while the results print).
void run_sliced(JobCore& job, BulkParser& parser, int64_t first_index, SharedWindow* text_win, uvector<char>* text);
// One in-memory batch (root: rb with offsets from 0) over the job's transport (flow_batch.cpp).
// `parser`: root, shm transport, bulk job without a skip — the records are encoded straight into the
// shared window (deferred pass 2) instead of from rb.
// A bulk job over the rccl / rccl-emul transport straight from the input text (device_batch_text: the root
// counts, splits and encodes every rank's slice into its wire block, no byte-code batch); on the mpi
// transport the root encodes one byte-code batch for run_record_batch. `parser` (root: header read, no
// pass 1 yet) and `text` go back to the OS once encoded.
void run_text_batch(JobCore& job, std::unique_ptr<BulkParser>& parser, int64_t first_index, uvector<char>* text);
void run_record_batch(JobCore& job, RecordBatch* rb, int64_t n, int64_t total_chars, int64_t first_index,
                      std::unique_ptr<BulkParser>* parser = nullptr, uvector<char>* text = nullptr);

// Streaming job on one node (flow_stream.cpp): batches of --batch-records / --batch-chars records, each
// encoded by every rank straight into its persistent page-locked ring slot while the previous batch's
// kernel streams, printed by the root while the next one is searched.
struct StreamSource {
  const char* mapped = nullptr;  // every rank: the whole --input file (nullptr: the root reads `in`)
  int64_t mapped_bytes = 0;
  FILE* in = nullptr;            // root, when not mapped
  int64_t area_begin = 0;        // mapped: file offset of the record area (after the header)
  uvector<char> head;            // root, stream input: the bytes read past the header
  bool eof = false;              // root, stream input: nothing follows `head`
};
// Returns 0, or 1 after an input error (reported on root's stderr).
int run_streaming(JobCore& job, const Header& h, StreamSource& src, int64_t batch_records, int64_t batch_chars,
                  const ParseOptions& po);
// Streaming job off the shm transport (flow_device_stream.cpp): the root cuts each batch from the text
// (StreamSource on the root only) and sends it — device_batch_text on rccl / rccl-emul, byte-code batches on
// mpi; batch b prints while batch b+1 is encoded and searched. Returns 0, or 1 after an input error.
int run_device_streaming(JobCore& job, const Header& h, StreamSource& src, int64_t batch_records,
                         int64_t batch_chars, const ParseOptions& po);

}  // namespace moc
