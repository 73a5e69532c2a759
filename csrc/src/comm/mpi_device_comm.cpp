// MpiDeviceComm / CpuDeviceSearch (moc/mpi_device_comm.hpp).
#include "moc/mpi_device_comm.hpp"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <exception>

#include "moc/cpu_engine.hpp"
#include "moc/runtime/watchdog.hpp"

namespace moc {

namespace {
constexpr int64_t kMpiChunk = int64_t{1} << 30;  // every MPI count < 2^31
constexpr int kTag = 21;
}  // namespace

MpiDeviceComm::~MpiDeviceComm() {
  // never wait while an error unwinds: a peer may be the stuck party, and the caller is about to abort
  if (!reqs_.empty() && std::uncaught_exceptions() == 0) {
    try {
      mpi_wait_all(reqs_, "MpiDeviceComm teardown", &infos_);
    } catch (...) {
    }
  }
}

void* MpiDeviceComm::dev_alloc(int64_t bytes) {
  void* p = std::aligned_alloc(64, static_cast<size_t>((std::max<int64_t>(bytes, 1) + 63) & ~int64_t{63}));
  if (!p) throw Error("MpiDeviceComm: out of memory");
  return p;
}
void MpiDeviceComm::dev_free(void* p) { std::free(p); }

int MpiDeviceComm::upload(void* d, const void* h, int64_t bytes) {
  if (bytes > 0 && d != h) std::memcpy(d, h, static_cast<size_t>(bytes));
  return 0;
}
void MpiDeviceComm::download(void* h, const void* d, int64_t bytes) {
  if (bytes > 0 && d != h) std::memcpy(h, d, static_cast<size_t>(bytes));
}

void MpiDeviceComm::group_start() { ++depth_; }
void MpiDeviceComm::group_end() {
  if (--depth_ > 0 || reqs_.empty()) return;
  mpi_wait_all(reqs_, "the device comm's send/recv group", &infos_);
  infos_.clear();
}

void MpiDeviceComm::send(const void* d, int64_t bytes, int peer) {
  const char* p = static_cast<const char*>(d);
  for (int64_t off = 0; off < bytes; off += kMpiChunk) {
    MPI_Request r;
    const int64_t n = std::min(kMpiChunk, bytes - off);
    mpi_check(MPI_Isend(p + off, static_cast<int>(n), MPI_BYTE, peer, kTag, ctx_.world, &r), "MPI_Isend");
    reqs_.push_back(r);
    infos_.push_back(ReqInfo{peer, n, true});
  }
  if (depth_ == 0) group_end();
}
void MpiDeviceComm::recv(void* d, int64_t bytes, int peer) {
  char* p = static_cast<char*>(d);
  for (int64_t off = 0; off < bytes; off += kMpiChunk) {
    MPI_Request r;
    const int64_t n = std::min(kMpiChunk, bytes - off);
    mpi_check(MPI_Irecv(p + off, static_cast<int>(n), MPI_BYTE, peer, kTag, ctx_.world, &r), "MPI_Irecv");
    reqs_.push_back(r);
    infos_.push_back(ReqInfo{peer, n, false});
  }
  if (depth_ == 0) group_end();
}

void MpiDeviceComm::bcast(void* d, int64_t bytes, int root) { bcast_bytes(d, bytes, root, ctx_.world); }
void MpiDeviceComm::allgather(const void* d_send, void* d_recv, int64_t bytes_each) {
  if (bytes_each >= kMpiChunk) throw Error("MpiDeviceComm::allgather: pieces must stay below 1 GiB");
  MPI_Request r;
  mpi_check(MPI_Iallgather(d_send, static_cast<int>(bytes_each), MPI_BYTE, d_recv, static_cast<int>(bytes_each), MPI_BYTE,
                           ctx_.world, &r),
            "MPI_Iallgather");
  mpi_wait(r, "MPI_Iallgather", "all-gather of " + watchdog::human_bytes(bytes_each) + " per rank");
}
void MpiDeviceComm::allreduce_max_u64(uint64_t* d, int64_t n) { moc::allreduce_max_u64(d, n, ctx_.world); }

// ---- CPU search over decoded wire batches
void CpuDeviceSearch::solve(const WireBatch& b, void* out, ResultFormat fmt) {
  if (fmt != ResultFormat::R12) throw Error("CpuDeviceSearch returns R12 results");
  RecordBatch rb;
  rb.offsets.resize(static_cast<size_t>(b.n) + 1);
  if (b.off_shift) {
    expand_offsets(b.offsets, b.off_shift, b.lengths, b.len_bits, b.len_base, b.n, rb.offsets.data());
  } else {
    std::memcpy(rb.offsets.data(), b.offsets, 8 * (static_cast<size_t>(b.n) + 1));
  }
  const int64_t c0 = rb.offsets[0], letters = rb.offsets[b.n] - c0;
  for (auto& o : rb.offsets) o -= c0;
  rb.codes.resize(static_cast<size_t>(letters));
  if (b.packed33)
    unpack33(b.letters, c0, letters, rb.codes.data());
  else if (b.packed5)
    unpack5(b.letters, c0, letters, rb.codes.data());
  else
    std::memcpy(rb.codes.data(), b.letters + c0, static_cast<size_t>(letters));
  solve_batch_cpu(table_, seq1_.data(), static_cast<int64_t>(seq1_.size()), rb, static_cast<Result*>(out), sem_,
                  threads_);
}

void CpuDeviceSearch::search_keys(const uint8_t* codes, const int64_t* offsets, const int64_t*, int64_t n, int part,
                                  int parts, uint64_t* keys) {
  RecordBatch rb;
  rb.offsets.assign(offsets, offsets + n + 1);
  const int64_t c0 = rb.offsets[0];
  for (auto& o : rb.offsets) o -= c0;
  rb.codes.assign(codes + c0, codes + c0 + rb.offsets[n]);
  solve_keys_cpu(table_, seq1_.data(), static_cast<int64_t>(seq1_.size()), rb, part, parts, keys, sem_, threads_);
}

void CpuDeviceSearch::finalize_keys(const uint8_t* codes, const int64_t* offsets, const int64_t*, int64_t n,
                                    const uint64_t* keys, Result* out) {
  const int64_t L1 = static_cast<int64_t>(seq1_.size());
#pragma omp parallel for schedule(dynamic, 64) if (n > 4096)
  for (int64_t i = 0; i < n; ++i)
    out[i] = resolve_key(table_, seq1_.data(), L1, codes + offsets[i], offsets[i + 1] - offsets[i], keys[i]);
}

}  // namespace moc
