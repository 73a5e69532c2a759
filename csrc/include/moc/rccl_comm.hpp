// RCCL communicator for GPU ranks: ncclCommInitRank with the unique id broadcast over MPI; device
// broadcast, grouped variable-size send/recv (the scatter/gather of records over xGMI) and the MAX
// all-reduce of packed candidate keys (context-parallel mode). Reference collectives: SURVEY.md §2.3.
#pragma once

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <vector>

#include "moc/comm.hpp"

namespace moc {

class RcclComm {
 public:
  // The unique id travels over MPI (the bootstrap): collective, on the thread that calls MPI.
  static ncclUniqueId exchange_id(const MpiContext& ctx);
  // ncclCommInitRank on `device` (collective over the ranks, any thread: e.g. a helper overlapping the
  // connect with the parse).
  RcclComm(const MpiContext& ctx, int device, const ncclUniqueId& id);
  RcclComm(const MpiContext& ctx, int device) : RcclComm(ctx, device, exchange_id(ctx)) {}
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  void bcast(void* dbuf, int64_t bytes, int root, hipStream_t s);
  // Root: sends slices [displs[r], displs[r]+counts[r]) of d_send to every rank r != root.
  // Others: receive counts[rank] bytes into d_recv. One ncclGroup, variable sizes.
  void scatterv(const void* d_send, const std::vector<int64_t>& counts, const std::vector<int64_t>& displs,
                void* d_recv, int root, hipStream_t s);
  // Inverse: every rank != root sends its slice to root, which receives it at displs[r].
  void gatherv(const void* d_send, int64_t count, void* d_recv, const std::vector<int64_t>& counts,
               const std::vector<int64_t>& displs, int root, hipStream_t s);
  void allgather(const void* d_send, void* d_recv, int64_t bytes_each, hipStream_t s);
  // In-place element-wise MAX of n uint64 device values over all ranks (packed candidate keys).
  void allreduce_max_u64(void* dbuf, int64_t n, hipStream_t s);
  void check_async() const;  // ncclCommGetAsyncError -> throw
  ncclComm_t comm() const { return comm_; }
  // The communicator is non-blocking (ncclConfig_t::blocking = 0; MOC_RCCL_BLOCKING=1 makes it blocking):
  // a call that RCCL leaves in progress — the init's exchange with the peers, a group's lazy p2p connect —
  // returns at once and `settle` polls ncclCommGetAsyncError under the job's comm deadline
  // (moc/runtime/watchdog.hpp), so a peer that never arrives is named instead of hanging the rank.
  // Every call of this class goes through it; callers issuing their own ncclSend/ncclRecv/ncclGroupEnd on
  // comm() pass the result here.
  void settle(ncclResult_t r, const char* what);
  // ncclCommAbort (a timed-out or failed rank, before MPI_Abort): the communicator is gone afterwards.
  void abort();
  // A communicator that lives until the process ends (the `final` CLI's): its destructor leaves it to the
  // process exit instead of ncclCommDestroy, which costs ~0.45 s per communicator on the MI355X box
  // (profiles/rccl_init_variants.log). MOC_RCCL_DESTROY=1 destroys it anyway.
  void keep_until_exit() { keep_ = true; }

 private:
  const MpiContext& ctx_;
  ncclComm_t comm_ = nullptr;
  bool keep_ = false;
};

// A one-rank communicator on `device`, created and kept until the process ends: RCCL's one-time cost —
// registering librccl's 569 MB fat binary, loading its 108 MB gfx950 code object — is paid here, on a
// helper thread that can start before MPI does (profiles/rccl_init_rootcause.log); later communicators of
// the process then start in ~60 ms. Returns false when RCCL cannot start.
bool rccl_warmup(int device);

}  // namespace moc
