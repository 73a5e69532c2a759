#include "moc/rccl_comm.hpp"

#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <string>

#include "moc/runtime/hip_check.hpp"
#include "moc/runtime/watchdog.hpp"

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
  bcast_bytes(&id, sizeof id, 0, ctx.world);
  return id;
}

RcclComm::RcclComm(const MpiContext& ctx, int device, const ncclUniqueId& id) : ctx_(ctx) {
  MOC_HIP_CHECK(hipSetDevice(device));
  ncclConfig_t config = NCCL_CONFIG_INITIALIZER;
  const char* b = std::getenv("MOC_RCCL_BLOCKING");
  config.blocking = b && std::strcmp(b, "1") == 0 ? 1 : 0;
  // RCCL prints a version banner on stdout during init; stdout carries results only (main.c:204). The
  // redirect holds until the (non-blocking) init has settled.
  std::fflush(stdout);
  const int saved = dup(1);
  dup2(2, 1);
  try {
    settle(ncclCommInitRankConfig(&comm_, ctx.size, id, ctx.rank, &config), "ncclCommInitRankConfig");
  } catch (...) {
    std::fflush(stdout);
    dup2(saved, 1);
    close(saved);
    throw;
  }
  std::fflush(stdout);
  dup2(saved, 1);
  close(saved);
}

void RcclComm::settle(ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return;
  if (r != ncclInProgress || !comm_) throw Error(std::string(what) + ": " + ncclGetErrorString(r));
  ncclResult_t st = ncclInProgress;
  watchdog::WaitSpec spec;
  spec.what = what;
  spec.poll = watchdog::Poll::Backoff;
  spec.outstanding = [this] { return "RCCL communicator of " + std::to_string(ctx_.size) + " ranks still in progress"; };
  spec.expire = [this] { abort(); };
  watchdog::wait(
      [&] {
        const ncclResult_t q = ncclCommGetAsyncError(comm_, &st);
        if (q != ncclSuccess) throw Error(std::string("ncclCommGetAsyncError: ") + ncclGetErrorString(q));
        return st != ncclInProgress;
      },
      spec);
  if (st != ncclSuccess) throw Error(std::string(what) + ": " + ncclGetErrorString(st));
}

void RcclComm::abort() {
  if (comm_) ncclCommAbort(comm_);
  comm_ = nullptr;
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
  if (!comm_) throw Error("RCCL communicator aborted");
  ncclResult_t st = ncclSuccess;
  MOC_NCCL_CHECK(ncclCommGetAsyncError(comm_, &st));
  if (st != ncclSuccess && st != ncclInProgress) throw Error(std::string("RCCL async error: ") + ncclGetErrorString(st));
}

void RcclComm::allreduce_max_u64(void* dbuf, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  settle(ncclAllReduce(dbuf, dbuf, static_cast<size_t>(n), ncclUint64, ncclMax, comm_, s), "ncclAllReduce");
}

void RcclComm::allgather(const void* d_send, void* d_recv, int64_t bytes_each, hipStream_t s) {
  if (bytes_each <= 0) return;
  settle(ncclAllGather(d_send, d_recv, static_cast<size_t>(bytes_each), ncclUint8, comm_, s), "ncclAllGather");
}

void RcclComm::bcast(void* dbuf, int64_t bytes, int root, hipStream_t s) {
  if (bytes <= 0) return;
  settle(ncclBroadcast(dbuf, dbuf, static_cast<size_t>(bytes), ncclUint8, root, comm_, s), "ncclBroadcast");
}

void RcclComm::scatterv(const void* d_send, const std::vector<int64_t>& counts, const std::vector<int64_t>& displs,
                        void* d_recv, int root, hipStream_t s) {
  const int rank = ctx_.rank;
  MOC_NCCL_CHECK(ncclGroupStart());
  if (rank == root) {
    for (int r = 0; r < ctx_.size; ++r)
      if (r != root && counts[r] > 0)
        settle(ncclSend(static_cast<const char*>(d_send) + displs[r], static_cast<size_t>(counts[r]), ncclUint8, r,
                        comm_, s),
               "ncclSend");
  } else if (counts[rank] > 0) {
    settle(ncclRecv(d_recv, static_cast<size_t>(counts[rank]), ncclUint8, root, comm_, s), "ncclRecv");
  }
  settle(ncclGroupEnd(), "ncclGroupEnd (scatterv)");
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
        settle(ncclRecv(static_cast<char*>(d_recv) + displs[r], static_cast<size_t>(counts[r]), ncclUint8, r, comm_, s),
               "ncclRecv");
  } else if (count > 0) {
    settle(ncclSend(d_send, static_cast<size_t>(count), ncclUint8, root, comm_, s), "ncclSend");
  }
  settle(ncclGroupEnd(), "ncclGroupEnd (gatherv)");
  if (rank == root && count > 0 && static_cast<char*>(d_recv) + displs[root] != d_send)
    MOC_HIP_CHECK(hipMemcpyAsync(static_cast<char*>(d_recv) + displs[root], d_send, static_cast<size_t>(count),
                                 hipMemcpyDeviceToDevice, s));
}

}  // namespace moc
