#include "moc/rccl_comm.hpp"

#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <string>

#include "moc/runtime/hip_check.hpp"

#define MOC_MPI_CHECK(call) ::moc::mpi_check((call), #call)

namespace moc {

// ------------------------------------------------------------------------------------------------
namespace {
void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw Error(std::string(what) + ": " + ncclGetErrorString(r));
}
#define MOC_NCCL_CHECK(call) nccl_check((call), #call)
}  // namespace

ncclUniqueId RcclComm::exchange_id(const MpiContext& ctx) {
  ncclUniqueId id;
  if (ctx.rank == 0) MOC_NCCL_CHECK(ncclGetUniqueId(&id));
  MOC_MPI_CHECK(MPI_Bcast(&id, sizeof id, MPI_BYTE, 0, ctx.world));
  return id;
}

RcclComm::RcclComm(const MpiContext& ctx, int device, const ncclUniqueId& id) : ctx_(ctx) {
  MOC_HIP_CHECK(hipSetDevice(device));
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
  const char* d = std::getenv("MOC_RCCL_DESTROY");
  if (keep_ && !(d && std::strcmp(d, "1") == 0)) return;  // the process exit releases it
  if (comm_) ncclCommDestroy(comm_);
}

bool rccl_warmup(int device) {
  static ncclComm_t warm = nullptr;  // kept: destroying it would cost as much as it saves
  if (warm) return true;
  if (hipSetDevice(device) != hipSuccess) return false;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return false;
  // RCCL prints a version banner on stdout during init; stdout carries results only (main.c:204)
  std::fflush(stdout);
  const int saved = dup(1);
  dup2(2, 1);
  const ncclResult_t rc = ncclCommInitRank(&warm, 1, id, 0);
  std::fflush(stdout);
  dup2(saved, 1);
  close(saved);
  if (rc != ncclSuccess) warm = nullptr;
  return rc == ncclSuccess;
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

void RcclComm::allgather(const void* d_send, void* d_recv, int64_t bytes_each, hipStream_t s) {
  if (bytes_each <= 0) return;
  MOC_NCCL_CHECK(ncclAllGather(d_send, d_recv, static_cast<size_t>(bytes_each), ncclUint8, comm_, s));
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
