// Shared parts of `final`'s job (moc job.hpp): engine selection through the dlopen'ed GPU plugin, the
// transports' small collectives (MPI or RCCL), the root's printer and the --timing report.
#include <dlfcn.h>
#include <omp.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cctype>
#include <cstdio>
#include <cstring>
#include <sstream>
#include <thread>

#include "job.hpp"
#include "moc/runtime/kfd_topology.hpp"
#include "moc/runtime/log.hpp"
#include "moc/runtime/watchdog.hpp"

namespace moc {

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

namespace {
// The GPU plugin (moc/gpu_rank.hpp): mpi_openmp_cuda_amd/lib/libmoc_final_gpu.so next to the binary, or
// $MOC_GPU_PLUGIN. Loaded once, on the first question about GPUs; never for CPU-backend runs, so `final`
// starts like a plain MPI program (the reference links cudart statically into every rank, makefile:4).
struct GpuPlugin {
  GpuDeviceCountFn device_count = nullptr;
  GpuRankCreateFn create = nullptr;
  GpuRcclWarmupFn rccl_warmup = nullptr;
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
    g.rccl_warmup = reinterpret_cast<GpuRcclWarmupFn>(dlsym(h, kGpuRcclWarmupSym));
    if (!g.device_count || !g.create) g.error = "GPU plugin " + path + " lacks its entry points";
    return g;
  }();
  return p;
}
}  // namespace

int gpu_device_count() {
  const GpuPlugin& g = gpu_plugin();
  return g.device_count && g.create ? g.device_count() : 0;
}
int gpu_device_count_fast() {
  if (const auto kfd = kfd_gpus()) {
    if (kfd->empty()) return 0;
    const GpuPlugin& g = gpu_plugin();  // loads the plugin (~13 ms), not the runtime
    return g.device_count && g.create ? static_cast<int>(kfd->size()) : 0;
  }
  return gpu_device_count();
}
std::string gpu_plugin_error() { return gpu_plugin().error; }
bool gpu_rccl_warmup(int device) {
  const GpuPlugin& g = gpu_plugin();
  return g.rccl_warmup && g.rccl_warmup(device) == 0;
}
GpuRank* gpu_rank_create(const MpiContext& ctx, const GpuRankOptions& opt) { return gpu_plugin().create(ctx, opt); }

// ---- FaultHook

void FaultHook::parse(const std::string& spec) {
  std::string f = spec;
  kind = Kind::Fail;
  if (f.rfind("stall-device:", 0) == 0) {
    kind = Kind::StallDevice;
    f = f.substr(13);
  } else if (f.rfind("stall:", 0) == 0) {
    kind = Kind::Stall;
    f = f.substr(6);
  }
  const auto colon = f.find(':');
  phase = f.substr(0, colon);
  rank = colon != std::string::npos ? std::stoi(f.substr(colon + 1)) : 0;
  if (const char* v = std::getenv("MOC_STALL_S")) stall_s = std::atof(v);
}

void FaultHook::at(const char* p, int my_rank, DeviceComm* dc) const {
  if (phase.empty() || phase != p || my_rank != rank) return;
  if (kind == Kind::Fail) throw Error(std::string("injected fault at phase '") + p + "'");
  const double s = stall_s > 0 ? stall_s : (kind == Kind::Stall ? 120.0 : 3.0);
  MOC_LOG_WARN("injected %s stall of %.1f s at phase '%s'", kind == Kind::Stall ? "rank" : "device comm lane", s, p);
  if (kind == Kind::StallDevice && dc) {
    dc->inject_stall(s);
    return;
  }
  std::this_thread::sleep_for(std::chrono::duration<double>(s));
}

// ---- RankEngine

namespace {
RecordBatch copy_slice(const uint8_t* codes, const int64_t* offsets, int64_t n) {
  RecordBatch b;
  b.codes.assign(codes + offsets[0], codes + offsets[n]);
  b.offsets.resize(static_cast<size_t>(n) + 1);
  for (int64_t i = 0; i <= n; ++i) b.offsets[i] = offsets[i] - offsets[0];
  return b;
}
}  // namespace

void RankEngine::set_problem(const Weights& w, const std::vector<uint8_t>& s1, Semantics s) {
  sem = s;
  seq1 = s1;
  table = ScoreTable::build(w);
  if (gpu) hip->set_problem(w, s1.data(), static_cast<int64_t>(s1.size()), s);
}

void RankEngine::solve(const uint8_t* codes, const int64_t* offsets, int64_t n, Result* out) {
  if (n <= 0) return;
  if (gpu) {
    hip->solve(codes, offsets, n, out);
    kernel_ms += hip->last_kernel_ms();
    return;
  }
  solve_batch_cpu(table, seq1.data(), static_cast<int64_t>(seq1.size()), copy_slice(codes, offsets, n), out, sem,
                  threads);
}

void RankEngine::solve_keys(const uint8_t* codes, const int64_t* offsets, int64_t n, int part, int parts,
                            uint64_t* keys) {
  if (n <= 0) return;
  if (gpu) {
    hip->search_keys(codes, offsets, n, part, parts, keys);
    kernel_ms += hip->last_kernel_ms();
    return;
  }
  solve_keys_cpu(table, seq1.data(), static_cast<int64_t>(seq1.size()), copy_slice(codes, offsets, n), part, parts,
                 keys, sem, threads);
}

// ---- JobCore

void JobCore::setup_engine(int64_t job_cells, int64_t mean_l2) {
  const int threads = static_cast<int>(flags.get_int("threads", 0));
  std::string backend = to_lower(flags.get("backend", "auto"));
  if (backend != "auto" && backend != "hip" && backend != "cpu") throw Error("--backend must be auto|hip|cpu");
  // auto: a job the OpenMP engine finishes faster than the GPU starts runs on the CPU. The GPU's start-up
  // (HIP runtime + engine) is 0.05-0.25 s; the OpenMP engine on the MI355X box's host cores searches
  // ~0.4 G cells/s per thread for records of <= 32 letters and ~1.4 G for longer ones, so the crossover is
  // ~0.2 s of CPU work (tools/gpu_crossover.sh, profiles/gpu_crossover.log: input6 shape between 0.6 and
  // 2.5 G cells at 16 threads, input3 shape above 1.7 G). `job_cells` < 0 means unknown (streaming): large.
  const double per_thread = mean_l2 > 32 ? 1.4e9 : 0.4e9;
  const int64_t model_min = static_cast<int64_t>(0.2 * per_thread * std::max(1, omp_get_max_threads()));
  const int64_t min_cells = flags.get_int("gpu-min-cells", model_min);
  if (backend == "auto" && job_cells >= 0 && job_cells < min_cells * ctx.size) backend = "cpu";
  // the driver's topology answers without waiting for the HIP runtime, which starts on the engine's helper
  // thread behind the parse and the encode (moc/runtime/kfd_topology.hpp)
  Stopwatch sw_count, sw_create, sw_reduce;
  sw_count.start();
  const int ndev = (backend == "cpu") ? 0 : gpu_device_count_fast();
  sw_count.stop();
  if (backend == "hip" && ndev == 0)
    throw Error("--backend=hip but no HIP device is visible" +
                (gpu_plugin_error().empty() ? std::string() : " (" + gpu_plugin_error() + ")"));
  eng.threads = threads;
  eng.gpu = ndev > 0;
  if (eng.gpu) {
    GpuRankOptions go;
    go.device = static_cast<int>(flags.get_int("device", -1));
    go.device_map = parse_int_list(flags.get("device-map", ""));
    go.chunk_records = flags.get_int("chunk-records", 0);
    go.chunk_bytes = flags.get_int("chunk-bytes", 0);
    go.log_level = flags.get("log-level", "warn");
    go.comm_timeout_s = watchdog::timeout_s();
    // a job below the GPU crossover (forced with --backend=hip) runs one kernel once: loading every code
    // object up front would cost more than that kernel's own load at its launch
    go.preload_kernels = job_cells < 0 || job_cells >= min_cells * ctx.size;
    sw_create.start();
    eng.hip.reset(gpu_rank_create(ctx, go));
    device = eng.hip->device();
    sw_create.stop();
  }
  int gpu_minmax[2] = {eng.gpu ? 1 : 0, eng.gpu ? -1 : 0};  // MIN -> {min gpu, -max gpu}
  sw_reduce.start();
  {
    MPI_Request r;
    mpi_check(MPI_Iallreduce(MPI_IN_PLACE, gpu_minmax, 2, MPI_INT, MPI_MIN, ctx.world, &r), "MPI_Iallreduce");
    mpi_wait(r, "MPI_Iallreduce (engine kinds)");
  }
  sw_reduce.stop();
  {
    char buf[160];
    std::snprintf(buf, sizeof buf, "{\"gpu_count\": %.3f, \"rank_create\": %.3f, \"engine_reduce\": %.3f}",
                  sw_count.total_ms(), sw_create.total_ms(), sw_reduce.total_ms());
    extra_timing.emplace_back("rank0_setup_split_ms", buf);
  }
  all_gpu = gpu_minmax[0] != 0;
  const bool any_gpu = gpu_minmax[1] != 0;
  transport = to_lower(flags.get("transport", "auto"));
  if (transport == "auto") transport = ctx.single_node() ? "shm" : (all_gpu ? "rccl" : "mpi");
  if (transport == "shm" && !ctx.single_node()) throw Error("--transport=shm needs all ranks on one node");
  if (transport == "rccl" && !all_gpu) throw Error("--transport=rccl needs a GPU on every rank");
  if (transport == "rccl-emul" && any_gpu) throw Error("--transport=rccl-emul runs on CPU ranks (--backend=cpu)");
  if (transport != "shm" && transport != "rccl" && transport != "rccl-emul" && transport != "mpi")
    throw Error("unknown --transport " + transport);
  partition = to_lower(flags.get("partition", "cost"));
  if (partition != "cost" && partition != "even" && partition != "offsets")
    throw Error("--partition must be cost|even|offsets");
  // GPU ranks split by shares of the tile list, CPU ranks by shares of each record's offsets: the two
  // decompositions do not tile each other, so the context-parallel mode needs one engine kind
  if (partition == "offsets" && any_gpu && !all_gpu)
    throw Error("--partition=offsets needs the same backend on every rank (use --backend=hip or --backend=cpu)");
  pin_window = flags.get_bool("pin-window", true);
  if (transport == "rccl") eng.hip->init_rccl();
  // the shm transport moves no record data between ranks; its collectives (the slices' fill reports and
  // result descriptors, the context-parallel key reduction) are a few host int64 per rank (or one key per
  // record), so they stay on MPI unless --collectives=rccl: setting up an RCCL communicator took 1.7-5.8 s
  // on the MI355X box even for one rank (profiles/final_scale_collrccl.log), microseconds of MPI work
  // would wait for it. With rccl the connect runs on a helper thread while the ranks parse their slices.
  const std::string coll = to_lower(flags.get("collectives", "auto"));
  if (coll != "auto" && coll != "mpi" && coll != "rccl") throw Error("--collectives must be auto|mpi|rccl");
  if (coll == "rccl" && !all_gpu) throw Error("--collectives=rccl needs a GPU on every rank");
  bool shared_gpu = false;  // RCCL needs one rank per GPU
  if (all_gpu && coll == "rccl") {
    const int64_t mine = static_cast<int64_t>(std::hash<std::string>{}(ctx.hostname) & 0xffffffffffffull) * 4096 + device;
    std::vector<int64_t> all(static_cast<size_t>(ctx.size));
    MPI_Request r;
    mpi_check(MPI_Iallgather(&mine, 1, MPI_INT64_T, all.data(), 1, MPI_INT64_T, ctx.world, &r), "MPI_Iallgather");
    mpi_wait(r, "MPI_Iallgather (rank devices)");
    std::sort(all.begin(), all.end());
    shared_gpu = std::adjacent_find(all.begin(), all.end()) != all.end();
  }
  if (coll == "rccl" && shared_gpu) throw Error("--collectives=rccl needs one rank per GPU");
  coll_rccl = transport == "shm" && all_gpu && !shared_gpu && coll == "rccl";
  if (coll_rccl) eng.hip->init_rccl_begin();
  if (transport == "rccl-emul") emul_comm = std::make_unique<MpiDeviceComm>(ctx);
  MOC_LOG_INFO("rank %d/%d host %s local %d/%d engine=%s device=%d transport=%s partition=%s", ctx.rank, ctx.size,
               ctx.hostname.c_str(), ctx.local_rank, ctx.local_size, eng.gpu ? "hip" : "cpu", device,
               transport.c_str(), partition.c_str());
}

void JobCore::allgather_i64(const int64_t* mine, int count, int64_t* all) {
  if (!coll_rccl) {
    MPI_Request r;
    mpi_check(MPI_Iallgather(mine, count, MPI_INT64_T, all, count, MPI_INT64_T, ctx.world, &r), "MPI_Iallgather");
    mpi_wait(r, "MPI_Iallgather");
    return;
  }
  DeviceComm& dc = eng.hip->device_comm();  // waits for the connect
  const int64_t bytes = 8 * static_cast<int64_t>(count);
  char* d = static_cast<char*>(dc.dev_alloc(bytes * (ctx.size + 1)));
  try {
    dc.wait_upload(dc.upload(d, mine, bytes));
    dc.allgather(d, d + bytes, bytes);
    dc.download(all, d + bytes, bytes * ctx.size);
  } catch (...) {
    dc.dev_free(d);
    throw;
  }
  dc.dev_free(d);
}

void JobCore::allreduce_keys(uint64_t* keys, int64_t n) {
  if (!coll_rccl) {
    allreduce_max_u64(keys, n, ctx.world);
    return;
  }
  DeviceComm& dc = eng.hip->device_comm();
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

void JobCore::resolve_keys(const uint64_t* keys, const uint8_t* codes, const int64_t* offsets, int64_t n,
                           Result* res) {
  const int64_t L1 = static_cast<int64_t>(eng.seq1.size());
#pragma omp parallel for schedule(dynamic, 64) if (n > 4096)
  for (int64_t i = 0; i < n; ++i)
    res[i] = resolve_key(eng.table, eng.seq1.data(), L1, codes + offsets[i], offsets[i + 1] - offsets[i], keys[i]);
}

void JobCore::print(const Result* r, int64_t n, int64_t first) {
  if (ctx.rank != kRoot) return;
  pt.begin("print");
  write_results(out, r, n, first_index + first);
  pt.end();
}

void JobCore::account_comm(const DeviceBatchOut& out) {
  comm_sent_bytes += out.sent_bytes;
  distribute_ms += out.distribute_ms;
  if (peer_sent.size() < out.peer_bytes.size()) peer_sent.resize(out.peer_bytes.size(), 0);
  for (size_t q = 0; q < out.peer_bytes.size(); ++q) peer_sent[q] += out.peer_bytes[q];
  if (fill_order.empty()) fill_order = out.fill_order;
}

void JobCore::report(const Header& h) {
  // the RCCL communicator's set-up (connect on its helper thread) and the time the rank then waited for it
  const bool device_transport = transport == "rccl" || transport == "rccl-emul";
  const double comm_init = eng.hip && (device_transport || coll_rccl) ? eng.hip->rccl_init_ms() : 0.0;
  const double comm_wait = eng.hip && (device_transport || coll_rccl) ? eng.hip->rccl_wait_ms() : 0.0;
  double mx[4] = {compute_ms, eng.kernel_ms, comm_init, comm_wait};
  {
    MPI_Request r;
    mpi_check(MPI_Ireduce(ctx.rank == kRoot ? MPI_IN_PLACE : mx, mx, 4, MPI_DOUBLE, MPI_MAX, kRoot, ctx.world, &r),
              "MPI_Ireduce");
    mpi_wait(r, "MPI_Ireduce (--timing)");
  }
  // every mode: what each rank page-locked and moved host->device over the job (sliced mode also has
  // its per-rank records and pin times, gathered with its results), and what it sent over the comm
  int64_t moved[3] = {pinned_bytes, h2d_bytes, comm_sent_bytes};
  std::vector<int64_t> all_moved(static_cast<size_t>(3 * ctx.size));
  {
    MPI_Request r;
    mpi_check(MPI_Igather(moved, 3, MPI_INT64_T, all_moved.data(), 3, MPI_INT64_T, kRoot, ctx.world, &r), "MPI_Igather");
    mpi_wait(r, "MPI_Igather (--timing)");
  }
  if (ctx.rank != kRoot || !flags.get_bool("timing", false)) return;
  const double wall_s = total.total_ms() / 1e3;
  auto list = [](const std::vector<int64_t>& v) {
    std::string s = "[";
    for (size_t i = 0; i < v.size(); ++i) s += (i ? ", " : "") + std::to_string(v[i]);
    return s + "]";
  };
  std::string per_rank;
  if (!rank_records.empty()) per_rank = ", \"rank_records\": " + list(rank_records);
  if (!rank_pin_us.empty()) {  // sliced mode: what each rank page-locked and moved, and its pin time
    per_rank += ", \"rank_pinned_bytes\": " + list(rank_pinned) + ", \"rank_h2d_bytes\": " + list(rank_h2d) +
                ", \"rank_pin_us\": " + list(rank_pin_us);
  } else {
    std::vector<int64_t> pinned(static_cast<size_t>(ctx.size)), h2d(static_cast<size_t>(ctx.size));
    for (int q = 0; q < ctx.size; ++q) {
      pinned[q] = all_moved[3 * q];
      h2d[q] = all_moved[3 * q + 1];
    }
    per_rank += ", \"rank_pinned_bytes\": " + list(pinned) + ", \"rank_h2d_bytes\": " + list(h2d);
  }
  if (device_transport || coll_rccl) {
    // the numbers a first multi-GPU run reads: communicator set-up, bytes each rank put on the comm, and the
    // root's rate to each peer over the distribution (bytes to that rank / the root's distribution time)
    std::vector<int64_t> sent(static_cast<size_t>(ctx.size));
    for (int q = 0; q < ctx.size; ++q) sent[q] = all_moved[3 * q + 2];
    char buf[96];
    std::snprintf(buf, sizeof buf, "%.3f, \"rccl_comm_wait_ms\": %.3f, \"distribute_ms\": %.3f", mx[2], mx[3],
                  distribute_ms);
    per_rank += ", \"rccl_comm_init_ms\": " + std::string(buf) + ", \"rank_sent_bytes\": " + list(sent);
    std::string gbps = "[";
    for (int q = 0; q < ctx.size; ++q) {
      const int64_t b = q < static_cast<int>(peer_sent.size()) ? peer_sent[q] : 0;
      std::snprintf(buf, sizeof buf, "%s%.4g", q ? ", " : "", distribute_ms > 0 ? b / (distribute_ms * 1e6) : 0.0);
      gbps += buf;
    }
    per_rank += ", \"peer_sent_bytes\": " + list(peer_sent.empty() ? std::vector<int64_t>(ctx.size, 0) : peer_sent) +
                ", \"peer_distribute_gbps\": " + gbps + "]";
    if (!fill_order.empty()) per_rank += ", \"fill_order\": " + list(std::vector<int64_t>(fill_order.begin(), fill_order.end()));
  }
  if (device_transport) {  // completion events the device comm holds (pooled: bounded by the pipeline depth)
    const DeviceComm* dc = emul_comm ? static_cast<const DeviceComm*>(emul_comm.get())
                                     : (eng.hip ? &eng.hip->device_comm() : nullptr);
    if (dc) per_rank += ", \"comm_events_live\": " + std::to_string(dc->events_live());
  }
  for (const auto& kv : extra_timing) per_rank += ", \"" + kv.first + "\": " + kv.second;
  std::fprintf(stderr,
               "{\"timing\": %s, \"ranks\": %d, \"nodes\": %d, \"engine\": \"%s\", \"transport\": \"%s\", "
               "\"partition\": \"%s\", \"collectives\": \"%s\", \"sliced\": %s, \"batches\": %lld, \"first_index\": %lld, "
               "\"records\": %lld, \"elements\": %lld, \"cells\": %lld, \"max_rank_compute_ms\": %.3f, "
               "\"max_rank_kernel_ms\": %.3f, \"wall_s\": %.6f, \"elements_per_s\": %.1f, \"cells_per_s\": %.1f%s, "
               "\"build\": \"%s\"}\n",
               pt.json().c_str(), ctx.size, ctx.node_count, eng.gpu ? "hip" : "cpu", transport.c_str(),
               partition.c_str(), coll_rccl || transport == "rccl" ? "rccl" : "mpi",
               rank_pin_us.empty() ? "false" : "true", static_cast<long long>(batches),
               static_cast<long long>(h.first_index), static_cast<long long>(records), static_cast<long long>(chars),
               static_cast<long long>(cells), mx[0], mx[1], wall_s, wall_s > 0 ? chars / wall_s : 0.0,
               wall_s > 0 ? cells / wall_s : 0.0, per_rank.c_str(), build_id);
}

}  // namespace moc
