// CPU stand-ins for the rccl transport's device layer (moc/device_comm.hpp): "device" memory is host
// memory, the comm lane is MPI (point-to-point groups, broadcast, MAX all-reduce), and the search is the
// OpenMP CPU engine after decoding the wire formats. `final --transport=rccl-emul` runs the rccl
// transport's batch driver through them on any ranks, which is how its multi-rank logic (plan, packing,
// chunked pipeline, narrow-result gather, context-parallel reduce) is tested without GPUs.
#pragma once

#include <mpi.h>

#include <vector>

#include "moc/comm.hpp"
#include "moc/device_comm.hpp"
#include "moc/score_table.hpp"

namespace moc {

class MpiDeviceComm final : public DeviceComm {
 public:
  explicit MpiDeviceComm(const MpiContext& ctx) : ctx_(ctx) {}
  ~MpiDeviceComm() override;
  int rank() const override { return ctx_.rank; }
  int size() const override { return ctx_.size; }
  const char* name() const override { return "mpi-emulated"; }
  void* dev_alloc(int64_t bytes) override;
  void dev_free(void* p) override;
  void* host_alloc(int64_t bytes) override { return dev_alloc(bytes); }
  void host_free(void* p) override { dev_free(p); }
  int upload(void* d, const void* h, int64_t bytes) override;
  void wait_upload(int) override {}
  int upload_after(void* d, const void* h, int64_t bytes, int) override { return upload(d, h, bytes); }
  void wait_upload_host(int) override {}
  void download(void* h, const void* d, int64_t bytes) override;
  void group_start() override;
  void group_end() override;
  void send(const void* d, int64_t bytes, int peer) override;
  void recv(void* d, int64_t bytes, int peer) override;
  void bcast(void* d, int64_t bytes, int root) override;
  void allgather(const void* d_send, void* d_recv, int64_t bytes_each) override;
  void allreduce_max_u64(uint64_t* d, int64_t n) override;
  void sync() override {}
  int mark() override { return 0; }
  void wait_mark(int) override {}

 private:
  const MpiContext& ctx_;
  int depth_ = 0;
  std::vector<MPI_Request> reqs_;
  std::vector<ReqInfo> infos_;  // peer and size of each request (named by a comm timeout)
};

class CpuDeviceSearch final : public DeviceSearch {
 public:
  CpuDeviceSearch(const ScoreTable& t, const std::vector<uint8_t>& seq1, Semantics sem, int threads)
      : table_(t), seq1_(seq1), sem_(sem), threads_(threads) {}
  // the narrow form whenever the lengths fit 8 bits, so the emulation exercises that wire path too
  bool streams_packed(int64_t, int64_t max_l2) const override { return max_l2 <= 255; }
  ResultFormat result_format(int64_t, int64_t, bool) const override { return ResultFormat::R12; }
  void solve(const WireBatch& b, void* out, ResultFormat fmt) override;
  void search_keys(const uint8_t* codes, const int64_t* offsets, const int64_t* h_offsets, int64_t n, int part,
                   int parts, uint64_t* keys) override;
  void finalize_keys(const uint8_t* codes, const int64_t* offsets, const int64_t* h_offsets, int64_t n,
                     const uint64_t* keys, Result* out) override;
  double last_kernel_ms() const override { return 0.0; }
  R2Params last_r2() const override { return R2Params{}; }

 private:
  ScoreTable table_;
  std::vector<uint8_t> seq1_;
  Semantics sem_;
  int threads_;
};

}  // namespace moc
