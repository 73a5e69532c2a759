#include "moc/comm.hpp"

#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>

#include "moc/runtime/log.hpp"
#include "moc/runtime/watchdog.hpp"

namespace moc {

namespace {
constexpr int64_t kMpiChunk = int64_t{1} << 30;  // keep every MPI count < 2^31
}

void mpi_check(int rc, const char* what) {
  if (rc == MPI_SUCCESS) return;
  char msg[MPI_MAX_ERROR_STRING];
  int len = 0;
  MPI_Error_string(rc, msg, &len);
  throw Error(std::string(what) + ": " + std::string(msg, len));
}

#define MOC_MPI_CHECK(call) ::moc::mpi_check((call), #call)

void mpi_wait_all(std::vector<MPI_Request>& reqs, const char* what, const std::vector<ReqInfo>* infos) {
  if (reqs.empty()) return;
  watchdog::WaitSpec spec;
  spec.what = what;
  spec.outstanding = [&reqs, infos]() {
    std::string o;
    int pending = 0;
    for (size_t i = 0; i < reqs.size(); ++i) {
      int f = 1;
      if (reqs[i] != MPI_REQUEST_NULL) MPI_Test(&reqs[i], &f, MPI_STATUS_IGNORE);
      if (f) continue;
      if (++pending > 8) continue;
      if (!o.empty()) o += ", ";
      if (infos && i < infos->size()) {
        const ReqInfo& r = (*infos)[i];
        o += std::string(r.send ? "send " : "recv ") + watchdog::human_bytes(r.bytes) + (r.send ? " to rank " : " from rank ") +
             std::to_string(r.peer);
      } else {
        o += "request " + std::to_string(i);
      }
    }
    if (pending > 8) o += " (+" + std::to_string(pending - 8) + " more)";
    return o;
  };
  int flag = 0;
  const int n = static_cast<int>(reqs.size());
  watchdog::wait(
      [&] {
        mpi_check(MPI_Testall(n, reqs.data(), &flag, MPI_STATUSES_IGNORE), what);
        return flag != 0;
      },
      spec);
  reqs.clear();
}

void mpi_wait(MPI_Request& req, const char* what, const std::string& detail) {
  watchdog::WaitSpec spec;
  spec.what = what;
  if (!detail.empty()) spec.outstanding = [&detail] { return detail; };
  int flag = 0;
  watchdog::wait(
      [&] {
        mpi_check(MPI_Test(&req, &flag, MPI_STATUS_IGNORE), what);
        return flag != 0;
      },
      spec);
}

void barrier(MPI_Comm comm, const char* what) {
  MPI_Request r;
  MOC_MPI_CHECK(MPI_Ibarrier(comm, &r));
  mpi_wait(r, what, "a rank that has not reached the barrier");
}

void mpi_prepare_env(bool lean_topology) {
  if (lean_topology) setenv("HWLOC_COMPONENTS", "no_os,stop", 0);
}

MpiContext::MpiContext(int* argc, char*** argv) {
  int provided = 0;
  MPI_Init_thread(argc, argv, MPI_THREAD_FUNNELED, &provided);
  MPI_Comm_set_errhandler(MPI_COMM_WORLD, MPI_ERRORS_RETURN);
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  MPI_Comm_split_type(MPI_COMM_WORLD, MPI_COMM_TYPE_SHARED, rank, MPI_INFO_NULL, &node);
  MPI_Comm_rank(node, &local_rank);
  MPI_Comm_size(node, &local_size);
  int leader = local_rank == 0 ? 1 : 0;
  MPI_Allreduce(&leader, &node_count, 1, MPI_INT, MPI_SUM, MPI_COMM_WORLD);
  char host[256] = {0};
  gethostname(host, sizeof host - 1);
  hostname = host;
  log_set_rank(rank);
}

MpiContext::~MpiContext() {
  if (node != MPI_COMM_NULL) MPI_Comm_free(&node);
  int fin = 0;
  MPI_Finalized(&fin);
  if (!fin) MPI_Finalize();
}

void MpiContext::abort(int code, const std::string& msg) const {
  std::fprintf(stderr, "[moc rank %d] fatal: %s\n", rank, msg.c_str());
  std::fflush(stderr);
  // the launcher forwards stderr through its proxy, which the abort tears down: give it a moment to
  // forward the message first (under load the line was sometimes lost)
  std::this_thread::sleep_for(std::chrono::milliseconds(100));
  MPI_Abort(MPI_COMM_WORLD, code);
  std::_Exit(code);
}

void bcast_bytes(void* buf, int64_t bytes, int root, MPI_Comm comm) {
  char* p = static_cast<char*>(buf);
  for (int64_t off = 0; off < bytes; off += kMpiChunk) {
    const int n = static_cast<int>(std::min(kMpiChunk, bytes - off));
    MPI_Request r;
    MOC_MPI_CHECK(MPI_Ibcast(p + off, n, MPI_BYTE, root, comm, &r));
    mpi_wait(r, "MPI_Ibcast", "broadcast of " + watchdog::human_bytes(n) + " from rank " + std::to_string(root));
  }
}

void allreduce_max_u64(uint64_t* buf, int64_t n, MPI_Comm comm) {
  const int64_t step = kMpiChunk / 8;
  for (int64_t off = 0; off < n; off += step) {
    const int c = static_cast<int>(std::min(step, n - off));
    MPI_Request r;
    MOC_MPI_CHECK(MPI_Iallreduce(MPI_IN_PLACE, buf + off, c, MPI_UINT64_T, MPI_MAX, comm, &r));
    mpi_wait(r, "MPI_Iallreduce", "MAX all-reduce of " + std::to_string(c) + " keys");
  }
}

namespace {
// Point-to-point transfer of a byte range in < 2^31 pieces (posted as non-blocking requests).
void post_send(std::vector<MPI_Request>& reqs, std::vector<ReqInfo>& infos, const char* p, int64_t bytes, int peer,
               int tag, MPI_Comm comm) {
  for (int64_t off = 0; off < bytes; off += kMpiChunk) {
    MPI_Request r;
    const int64_t n = std::min(kMpiChunk, bytes - off);
    MOC_MPI_CHECK(MPI_Isend(p + off, static_cast<int>(n), MPI_BYTE, peer, tag, comm, &r));
    reqs.push_back(r);
    infos.push_back(ReqInfo{peer, n, true});
  }
}
void post_recv(std::vector<MPI_Request>& reqs, std::vector<ReqInfo>& infos, char* p, int64_t bytes, int peer, int tag,
               MPI_Comm comm) {
  for (int64_t off = 0; off < bytes; off += kMpiChunk) {
    MPI_Request r;
    const int64_t n = std::min(kMpiChunk, bytes - off);
    MOC_MPI_CHECK(MPI_Irecv(p + off, static_cast<int>(n), MPI_BYTE, peer, tag, comm, &r));
    reqs.push_back(r);
    infos.push_back(ReqInfo{peer, n, false});
  }
}
}  // namespace

void scatterv_bytes(const void* sendbuf, const std::vector<int64_t>& counts, const std::vector<int64_t>& displs,
                    void* recvbuf, int root, MPI_Comm comm) {
  int rank = 0, size = 1;
  MPI_Comm_rank(comm, &rank);
  MPI_Comm_size(comm, &size);
  std::vector<MPI_Request> reqs;
  std::vector<ReqInfo> infos;
  if (rank == root) {
    const char* s = static_cast<const char*>(sendbuf);
    for (int r = 0; r < size; ++r) {
      if (r == root) {
        if (counts[r] && recvbuf != s + displs[r]) std::memmove(recvbuf, s + displs[r], static_cast<size_t>(counts[r]));
      } else {
        post_send(reqs, infos, s + displs[r], counts[r], r, 11, comm);
      }
    }
  } else {
    post_recv(reqs, infos, static_cast<char*>(recvbuf), counts[rank], root, 11, comm);
  }
  mpi_wait_all(reqs, "scatterv", &infos);
}

void gatherv_bytes(const void* sendbuf, int64_t count, void* recvbuf, const std::vector<int64_t>& counts,
                   const std::vector<int64_t>& displs, int root, MPI_Comm comm) {
  int rank = 0, size = 1;
  MPI_Comm_rank(comm, &rank);
  MPI_Comm_size(comm, &size);
  std::vector<MPI_Request> reqs;
  std::vector<ReqInfo> infos;
  if (rank == root) {
    char* d = static_cast<char*>(recvbuf);
    for (int r = 0; r < size; ++r) {
      if (r == root) {
        if (count && d + displs[r] != sendbuf) std::memmove(d + displs[r], sendbuf, static_cast<size_t>(count));
      } else {
        post_recv(reqs, infos, d + displs[r], counts[r], r, 12, comm);
      }
    }
  } else {
    post_send(reqs, infos, static_cast<const char*>(sendbuf), count, root, 12, comm);
  }
  mpi_wait_all(reqs, "gatherv", &infos);
}

// ------------------------------------------------------------------------------------------------
SharedWindow::SharedWindow(const MpiContext& ctx, int64_t bytes) : comm_(ctx.node) {
  if (ctx.local_size == 1) {
    // huge pages from 1 MiB up (a small window's first touch would zero a whole 2 MiB page)
    const bool huge = bytes >= (int64_t{1} << 20);
    const size_t align = huge ? size_t{2} << 20 : size_t{4096};
    const size_t want = (static_cast<size_t>(std::max<int64_t>(bytes, 8)) + align - 1) & ~(align - 1);
    map_bytes_ = huge ? want + align : want;  // slack to start on a 2 MiB boundary
    map_ = mmap(nullptr, map_bytes_, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (map_ == MAP_FAILED) {
      map_ = nullptr;
      throw Error("SharedWindow: cannot map " + std::to_string(map_bytes_) + " bytes");
    }
    base_ = reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(map_) + align - 1) & ~(align - 1));
    if (huge) (void)madvise(base_, want, MADV_HUGEPAGE);  // advisory: 4 KiB pages if THP is off
    bytes_ = bytes;
    return;
  }
  const MPI_Aint mine = ctx.local_rank == 0 ? static_cast<MPI_Aint>(std::max<int64_t>(bytes, 8)) : 0;
  void* base = nullptr;
  MOC_MPI_CHECK(MPI_Win_allocate_shared(mine, 1, MPI_INFO_NULL, comm_, &base, &win_));
  MPI_Aint sz = 0;
  int disp = 0;
  void* owner = nullptr;
  MOC_MPI_CHECK(MPI_Win_shared_query(win_, 0, &sz, &disp, &owner));
  base_ = static_cast<char*>(owner);
  bytes_ = bytes;
  MOC_MPI_CHECK(MPI_Win_lock_all(MPI_MODE_NOCHECK, win_));
}

SharedWindow::~SharedWindow() {
  if (map_) {
    if (releaser_) {
      void* m = map_;
      const size_t len = map_bytes_;
      releaser_->defer([m, len] { munmap(m, len); });
    } else {
      munmap(map_, map_bytes_);
    }
    return;
  }
  // Never enter a collective while an exception unwinds: peers may be blocked elsewhere and the caller
  // is about to MPI_Abort (freeing here would deadlock the failing rank).
  if (std::uncaught_exceptions() > 0) return;
  if (win_ != MPI_WIN_NULL) {
    MPI_Win_unlock_all(win_);
    MPI_Win_free(&win_);
  }
}

void SharedWindow::discard(int64_t off, int64_t len) {
  if (!map_ || len <= 0) return;
  constexpr uintptr_t kHuge = uintptr_t{2} << 20;  // whole huge pages only: a partial one would be split
  const uintptr_t lo = (reinterpret_cast<uintptr_t>(base_) + static_cast<uintptr_t>(off) + kHuge - 1) & ~(kHuge - 1);
  const uintptr_t hi = (reinterpret_cast<uintptr_t>(base_) + static_cast<uintptr_t>(off + len)) & ~(kHuge - 1);
  if (hi <= lo) return;
  // MADV_DONTNEED keeps the range mapped (zero-fill on a stray touch instead of a fault) and leaves the
  // mapping whole for the final munmap.
  void* p = reinterpret_cast<void*>(lo);
  const size_t n = hi - lo;
  if (releaser_)
    releaser_->defer([p, n] { (void)madvise(p, n, MADV_DONTNEED); });
  else
    (void)madvise(p, n, MADV_DONTNEED);
}

void SharedWindow::prefault_shares(const MpiContext& ctx) {
  if (map_) return;  // private mapping: huge pages, faulted by the fill
  const int64_t pages = (bytes_ + 4095) / 4096;
  const int64_t b = pages * ctx.local_rank / ctx.local_size, e = pages * (ctx.local_rank + 1) / ctx.local_size;
  prefault_pages(base_ + 4096 * b, static_cast<size_t>(std::min(bytes_, 4096 * e) - std::min(bytes_, 4096 * b)));
  fence();
}

void SharedWindow::release_shares(const MpiContext& ctx) {
  if (map_ || ctx.local_size < 2 || ctx.local_rank == 0) return;
  const int64_t pages = bytes_ / 4096;  // whole pages inside the window only
  const uintptr_t first = (reinterpret_cast<uintptr_t>(base_) + 4095) & ~uintptr_t{4095};
  const int64_t helpers = ctx.local_size - 1, q = ctx.local_rank - 1;
  const int64_t b = pages * q / helpers, e = pages * (q + 1) / helpers;
  if (e > b) (void)madvise(reinterpret_cast<void*>(first + 4096 * b), static_cast<size_t>(4096 * (e - b)), MADV_REMOVE);
}

void SharedWindow::fence() const {
  if (map_) return;  // one rank on the node
  MOC_MPI_CHECK(MPI_Win_sync(win_));
  barrier(comm_, "node window fence");
  MOC_MPI_CHECK(MPI_Win_sync(win_));
}

// ------------------------------------------------------------------------------------------------
SegmentWindow::SegmentWindow(const MpiContext& ctx, int64_t my_bytes, int numa_node)
    : comm_(ctx.node), local_rank_(ctx.local_rank) {
  seg_.assign(static_cast<size_t>(ctx.local_size), nullptr);
  if (ctx.local_size == 1) {
    region_ = HostRegion(static_cast<size_t>(std::max<int64_t>(my_bytes, 8)), numa_node);
    seg_[0] = region_.data();
    return;
  }
  MPI_Info info;
  MPI_Info_create(&info);
  MPI_Info_set(info, "alloc_shared_noncontig", "true");  // each segment page-aligned on its own
  void* base = nullptr;
  const int rc = MPI_Win_allocate_shared(static_cast<MPI_Aint>(std::max<int64_t>(my_bytes, 8)), 1, info, comm_, &base,
                                         &win_);
  MPI_Info_free(&info);
  MOC_MPI_CHECK(rc);
  if (numa_node >= 0) (void)bind_range_to_node(base, static_cast<size_t>(std::max<int64_t>(my_bytes, 8)), numa_node);
  prefault_pages(static_cast<char*>(base), static_cast<size_t>(my_bytes));  // this rank's threads, in parallel
  for (int r = 0; r < ctx.local_size; ++r) {
    MPI_Aint sz = 0;
    int disp = 0;
    void* p = nullptr;
    MOC_MPI_CHECK(MPI_Win_shared_query(win_, r, &sz, &disp, &p));
    seg_[static_cast<size_t>(r)] = static_cast<char*>(p);
  }
  MOC_MPI_CHECK(MPI_Win_lock_all(MPI_MODE_NOCHECK, win_));
}

SegmentWindow::~SegmentWindow() {
  if (win_ == MPI_WIN_NULL || std::uncaught_exceptions() > 0) return;  // see ~SharedWindow
  MPI_Win_unlock_all(win_);
  MPI_Win_free(&win_);
}

void SegmentWindow::fence() const {
  if (win_ == MPI_WIN_NULL) return;
  MOC_MPI_CHECK(MPI_Win_sync(win_));
  barrier(comm_, "node window fence");
  MOC_MPI_CHECK(MPI_Win_sync(win_));
}

}  // namespace moc
