#include "moc/comm.hpp"

#include <hip/hip_runtime_api.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstring>

#include "moc/runtime/hip_check.hpp"
#include "moc/runtime/log.hpp"

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
  MPI_Abort(MPI_COMM_WORLD, code);
  std::_Exit(code);
}

void bcast_bytes(void* buf, int64_t bytes, int root, MPI_Comm comm) {
  char* p = static_cast<char*>(buf);
  for (int64_t off = 0; off < bytes; off += kMpiChunk) {
    const int n = static_cast<int>(std::min(kMpiChunk, bytes - off));
    MOC_MPI_CHECK(MPI_Bcast(p + off, n, MPI_BYTE, root, comm));
  }
}

void allreduce_max_u64(uint64_t* buf, int64_t n, MPI_Comm comm) {
  const int64_t step = kMpiChunk / 8;
  for (int64_t off = 0; off < n; off += step) {
    const int c = static_cast<int>(std::min(step, n - off));
    MOC_MPI_CHECK(MPI_Allreduce(MPI_IN_PLACE, buf + off, c, MPI_UINT64_T, MPI_MAX, comm));
  }
}

namespace {
// Point-to-point transfer of a byte range in < 2^31 pieces (posted as non-blocking requests).
void post_send(std::vector<MPI_Request>& reqs, const char* p, int64_t bytes, int peer, int tag, MPI_Comm comm) {
  for (int64_t off = 0; off < bytes; off += kMpiChunk) {
    MPI_Request r;
    MOC_MPI_CHECK(MPI_Isend(p + off, static_cast<int>(std::min(kMpiChunk, bytes - off)), MPI_BYTE, peer, tag, comm, &r));
    reqs.push_back(r);
  }
}
void post_recv(std::vector<MPI_Request>& reqs, char* p, int64_t bytes, int peer, int tag, MPI_Comm comm) {
  for (int64_t off = 0; off < bytes; off += kMpiChunk) {
    MPI_Request r;
    MOC_MPI_CHECK(MPI_Irecv(p + off, static_cast<int>(std::min(kMpiChunk, bytes - off)), MPI_BYTE, peer, tag, comm, &r));
    reqs.push_back(r);
  }
}
}  // namespace

void scatterv_bytes(const void* sendbuf, const std::vector<int64_t>& counts, const std::vector<int64_t>& displs,
                    void* recvbuf, int root, MPI_Comm comm) {
  int rank = 0, size = 1;
  MPI_Comm_rank(comm, &rank);
  MPI_Comm_size(comm, &size);
  std::vector<MPI_Request> reqs;
  if (rank == root) {
    const char* s = static_cast<const char*>(sendbuf);
    for (int r = 0; r < size; ++r) {
      if (r == root) {
        if (counts[r] && recvbuf != s + displs[r]) std::memmove(recvbuf, s + displs[r], static_cast<size_t>(counts[r]));
      } else {
        post_send(reqs, s + displs[r], counts[r], r, 11, comm);
      }
    }
  } else {
    post_recv(reqs, static_cast<char*>(recvbuf), counts[rank], root, 11, comm);
  }
  if (!reqs.empty()) MOC_MPI_CHECK(MPI_Waitall(static_cast<int>(reqs.size()), reqs.data(), MPI_STATUSES_IGNORE));
}

void gatherv_bytes(const void* sendbuf, int64_t count, void* recvbuf, const std::vector<int64_t>& counts,
                   const std::vector<int64_t>& displs, int root, MPI_Comm comm) {
  int rank = 0, size = 1;
  MPI_Comm_rank(comm, &rank);
  MPI_Comm_size(comm, &size);
  std::vector<MPI_Request> reqs;
  if (rank == root) {
    char* d = static_cast<char*>(recvbuf);
    for (int r = 0; r < size; ++r) {
      if (r == root) {
        if (count && d + displs[r] != sendbuf) std::memmove(d + displs[r], sendbuf, static_cast<size_t>(count));
      } else {
        post_recv(reqs, d + displs[r], counts[r], r, 12, comm);
      }
    }
  } else {
    post_send(reqs, static_cast<const char*>(sendbuf), count, root, 12, comm);
  }
  if (!reqs.empty()) MOC_MPI_CHECK(MPI_Waitall(static_cast<int>(reqs.size()), reqs.data(), MPI_STATUSES_IGNORE));
}

// ------------------------------------------------------------------------------------------------
SharedWindow::SharedWindow(const MpiContext& ctx, int64_t bytes) : comm_(ctx.node) {
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
  // Never enter a collective while an exception unwinds: peers may be blocked elsewhere and the caller
  // is about to MPI_Abort (freeing here would deadlock the failing rank).
  if (std::uncaught_exceptions() > 0) return;
  if (win_ != MPI_WIN_NULL) {
    MPI_Win_unlock_all(win_);
    MPI_Win_free(&win_);
  }
}

void SharedWindow::fence() const {
  MOC_MPI_CHECK(MPI_Win_sync(win_));
  MOC_MPI_CHECK(MPI_Barrier(comm_));
  MOC_MPI_CHECK(MPI_Win_sync(win_));
}

// ------------------------------------------------------------------------------------------------
namespace {
void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw Error(std::string(what) + ": " + ncclGetErrorString(r));
}
#define MOC_NCCL_CHECK(call) nccl_check((call), #call)
}  // namespace

RcclComm::RcclComm(const MpiContext& ctx, int device) : ctx_(ctx) {
  MOC_HIP_CHECK(hipSetDevice(device));
  ncclUniqueId id;
  if (ctx.rank == 0) MOC_NCCL_CHECK(ncclGetUniqueId(&id));
  MOC_MPI_CHECK(MPI_Bcast(&id, sizeof id, MPI_BYTE, 0, ctx.world));
  // RCCL prints a version banner on stdout during init; stdout carries results only (main.c:204).
  std::fflush(stdout);
  const int saved = dup(1);
  dup2(2, 1);
  const ncclResult_t rc = ncclCommInitRank(&comm_, ctx.size, id, ctx.rank);
  std::fflush(stdout);
  dup2(saved, 1);
  close(saved);
  MOC_NCCL_CHECK(rc);
}

RcclComm::~RcclComm() {
  if (std::uncaught_exceptions() > 0) {  // see ~SharedWindow; abort the communicator instead
    if (comm_) ncclCommAbort(comm_);
    return;
  }
  if (comm_) ncclCommDestroy(comm_);
}

void RcclComm::check_async() const {
  ncclResult_t st = ncclSuccess;
  MOC_NCCL_CHECK(ncclCommGetAsyncError(comm_, &st));
  if (st != ncclSuccess) throw Error(std::string("RCCL async error: ") + ncclGetErrorString(st));
}

void RcclComm::allreduce_max_u64(void* dbuf, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  MOC_NCCL_CHECK(ncclAllReduce(dbuf, dbuf, static_cast<size_t>(n), ncclUint64, ncclMax, comm_, s));
}

void RcclComm::bcast(void* dbuf, int64_t bytes, int root, hipStream_t s) {
  if (bytes <= 0) return;
  MOC_NCCL_CHECK(ncclBroadcast(dbuf, dbuf, static_cast<size_t>(bytes), ncclUint8, root, comm_, s));
}

void RcclComm::scatterv(const void* d_send, const std::vector<int64_t>& counts, const std::vector<int64_t>& displs,
                        void* d_recv, int root, hipStream_t s) {
  const int rank = ctx_.rank;
  MOC_NCCL_CHECK(ncclGroupStart());
  if (rank == root) {
    for (int r = 0; r < ctx_.size; ++r)
      if (r != root && counts[r] > 0)
        MOC_NCCL_CHECK(ncclSend(static_cast<const char*>(d_send) + displs[r], static_cast<size_t>(counts[r]), ncclUint8,
                                r, comm_, s));
  } else if (counts[rank] > 0) {
    MOC_NCCL_CHECK(ncclRecv(d_recv, static_cast<size_t>(counts[rank]), ncclUint8, root, comm_, s));
  }
  MOC_NCCL_CHECK(ncclGroupEnd());
  if (rank == root && counts[root] > 0 && d_recv != static_cast<const char*>(d_send) + displs[root])
    MOC_HIP_CHECK(hipMemcpyAsync(d_recv, static_cast<const char*>(d_send) + displs[root],
                                 static_cast<size_t>(counts[root]), hipMemcpyDeviceToDevice, s));
}

void RcclComm::gatherv(const void* d_send, int64_t count, void* d_recv, const std::vector<int64_t>& counts,
                       const std::vector<int64_t>& displs, int root, hipStream_t s) {
  const int rank = ctx_.rank;
  MOC_NCCL_CHECK(ncclGroupStart());
  if (rank == root) {
    for (int r = 0; r < ctx_.size; ++r)
      if (r != root && counts[r] > 0)
        MOC_NCCL_CHECK(ncclRecv(static_cast<char*>(d_recv) + displs[r], static_cast<size_t>(counts[r]), ncclUint8, r,
                                comm_, s));
  } else if (count > 0) {
    MOC_NCCL_CHECK(ncclSend(d_send, static_cast<size_t>(count), ncclUint8, root, comm_, s));
  }
  MOC_NCCL_CHECK(ncclGroupEnd());
  if (rank == root && count > 0 && static_cast<char*>(d_recv) + displs[root] != d_send)
    MOC_HIP_CHECK(hipMemcpyAsync(static_cast<char*>(d_recv) + displs[root], d_send, static_cast<size_t>(count),
                                 hipMemcpyDeviceToDevice, s));
}

}  // namespace moc
