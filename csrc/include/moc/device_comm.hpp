// The rccl transport's device layer, ROCm-free so `final` (and its CPU-only builds and tests) can drive it.
//
// Reference: MPI_Bcast x4, MPI_Scatter of fixed 2000-byte records and MPI_Gather x3 of three int arrays, on
// host memory, blocking, rooted at 0 (main.c:149-152, 174, 195-197), then a cudaMemcpy of the chunk
// (cudaFunctions.cu:201) — every byte crosses the host twice.
//
// Here the distribution of a batch is written once (device_batch.cpp) against two narrow interfaces:
//   DeviceComm   — one rank's device memory and its communicator, stream-ordered: RCCL over xGMI on GPU
//                  ranks (the GPU plugin), or MpiDeviceComm, which emulates it over host memory and MPI
//                  point-to-point, so the very same driver runs on CPU-only ranks (--transport=rccl-emul)
//                  and the multi-rank logic is tested without GPUs;
//   DeviceSearch — the rank's engine over device-resident wire-format batches (moc/wire.hpp).
#pragma once

#include <cstdint>
#include <functional>
#include <string>
#include <vector>

#include "moc/common.hpp"
#include "moc/problem.hpp"
#include "moc/wire.hpp"

namespace moc {

// Phase hooks of the caller's timer / fault injection (the device batch runs its own phases).
struct PhaseHooks {
  std::function<void(const char*)> begin;  // starts a phase (and fires the fault hook for it)
  std::function<void()> end;
};

class DeviceComm {
 public:
  virtual ~DeviceComm() = default;
  virtual int rank() const = 0;
  virtual int size() const = 0;
  virtual const char* name() const = 0;
  // device memory of this rank, and page-locked host staging for asynchronous uploads
  virtual void* dev_alloc(int64_t bytes) = 0;
  virtual void dev_free(void* p) = 0;
  virtual void* host_alloc(int64_t bytes) = 0;
  virtual void host_free(void* p) = 0;
  // host -> device on the copy lane (returns at once); the ticket orders later comm-lane work after it
  virtual int upload(void* d, const void* h, int64_t bytes) = 0;
  virtual void wait_upload(int ticket) = 0;
  // the same, queued behind the comm-lane point `after` (a mark; -1: nothing): a device staging buffer the
  // comm lane still sends from is overwritten only once that send is done
  virtual int upload_after(void* d, const void* h, int64_t bytes, int after) = 0;
  // the host waits until an upload has read its host buffer (before reusing the staging)
  virtual void wait_upload_host(int ticket) = 0;
  // device -> host on the comm lane; the host waits for it (and for everything queued before)
  virtual void download(void* h, const void* d, int64_t bytes) = 0;
  // comm-lane collectives on device buffers (send/recv between group_start and group_end are one group)
  virtual void group_start() = 0;
  virtual void group_end() = 0;
  virtual void send(const void* d, int64_t bytes, int peer) = 0;
  virtual void recv(void* d, int64_t bytes, int peer) = 0;
  virtual void bcast(void* d, int64_t bytes, int root) = 0;
  virtual void allgather(const void* d_send, void* d_recv, int64_t bytes_each) = 0;
  virtual void allreduce_max_u64(uint64_t* d, int64_t n) = 0;
  // host waits for the comm lane; throws on asynchronous communicator errors
  virtual void sync() = 0;
  // a point of the comm lane, and a host wait for just that point (pipelines reuse staging buffers)
  virtual int mark() = 0;
  virtual void wait_mark(int mark) = 0;
  // Every host wait above (sync, download, wait_mark, wait_upload_host, group_end) polls against the job's
  // comm deadline (moc/runtime/watchdog.hpp) and throws CommTimeout naming what is outstanding.
  // Test hook (--inject-fault=stall-device:PHASE): the comm lane is held busy for `seconds` (a bounded device
  // spin on GPUs; the calling thread sleeps on the MPI emulation).
  virtual void inject_stall(double seconds);
  // Completion events the layer holds right now (pooled: bounded by the pipeline depth, not the job).
  virtual int64_t events_live() const { return 0; }
};

class DeviceSearch {
 public:
  virtual ~DeviceSearch() = default;
  // Whether batches of this length range travel as packed letters + narrow lengths + sparse offsets
  // (else packed letters + dense offsets), and the result format the rank returns for that form.
  virtual bool streams_packed(int64_t min_l2, int64_t max_l2) const = 0;
  virtual ResultFormat result_format(int64_t min_l2, int64_t max_l2, bool packed_form) const = 0;
  // A device-resident wire batch (offsets rebased to 0) -> results in `fmt` at d_out (comm lane order).
  virtual void solve(const WireBatch& d_batch, void* d_out, ResultFormat fmt) = 0;
  // Context-parallel share of every record (byte codes, dense offsets from 0; h_offsets: host copy) ->
  // packed pass-1 keys; and the root's resolve of the MAX-reduced keys into results (R12; needs the batch).
  virtual void search_keys(const uint8_t* d_codes, const int64_t* d_offsets, const int64_t* h_offsets, int64_t n,
                           int part, int parts, uint64_t* d_keys) = 0;
  virtual void finalize_keys(const uint8_t* d_codes, const int64_t* d_offsets, const int64_t* h_offsets, int64_t n,
                             const uint64_t* d_keys, Result* d_out) = 0;
  virtual double last_kernel_ms() const = 0;
  virtual R2Params last_r2() const = 0;
};

// Device and page-locked host buffers of the batch driver, kept across batches (a streaming job allocates
// and page-locks them once): numbered slots that only grow. Every batch ends with the comm lane drained,
// so a slot is free again when the next batch asks for it.
class DeviceScratch {
 public:
  explicit DeviceScratch(DeviceComm& dc) : dc_(dc) {}
  ~DeviceScratch();
  DeviceScratch(const DeviceScratch&) = delete;
  DeviceScratch& operator=(const DeviceScratch&) = delete;
  char* dev(int slot, int64_t bytes) { return get(dev_, slot, bytes, false); }
  char* host(int slot, int64_t bytes) { return get(host_, slot, bytes, true); }

 private:
  struct Buf {
    void* p = nullptr;
    int64_t cap = 0;
  };
  char* get(std::vector<Buf>& v, int slot, int64_t bytes, bool host);
  DeviceComm& dc_;
  std::vector<Buf> dev_, host_;
};

// What one device batch produced: on the root, every rank's results in its own format (host memory of the
// scratch, valid until the next batch).
struct DeviceBatchOut {
  std::vector<ResultRun> runs;
  std::vector<std::vector<char>> storage;  // backing memory of runs (the context-parallel path)
  double compute_ms = 0, kernel_ms = 0;    // this rank
  int64_t scattered_bytes = 0;             // root: device bytes sent to the other ranks
  // what crossed the comm: bytes this rank sent (root: its slices' pieces; a peer: its results), the root's
  // bytes to each rank (index = rank, its own 0), and the root's distribution time from its first piece on
  // the wire to the last one delivered (the per-peer rate of a multi-GPU run: peer_bytes / distribute_ms)
  int64_t sent_bytes = 0;
  std::vector<int64_t> peer_bytes;
  double distribute_ms = 0;
  std::vector<int64_t> rank_records;       // every rank's records (root)
  // device_batch_text: the batch's search cells and letters (root); an input error (every rank; the
  // message on the root), in which case nothing was searched
  int64_t cells = 0, letters = 0;
  std::vector<int> fill_order;  // device_batch_text (root): the ranks in the order their slices were encoded
  bool input_error = false;
  std::string error;
};

// One batch over the device layer. Record slices (cp = false): the root packs each rank's slice into the
// wire form that rank's engine streams, piece by piece (<= 64 MiB: letter blocks, offsets, lengths), the
// ranks' pieces interleaved round-robin with the root's own; a three-slot pipeline packs piece i+1 (host
// threads) while piece i uploads (copy lane) and piece i-1 goes out over xGMI (comm lane, ordered after its
// upload on the device, no host wait); every rank searches its slice in device memory and the narrow
// results are gathered to the root.
// Context parallel (cp = true): the batch is broadcast, each rank searches its share of every record's
// offsets, the packed keys are MAX-all-reduced, the root decodes them.
// `rb` (bytes + offsets from 0) and `bounds` (p+1 record bounds) are read on the root only.
// `scratch` (optional): buffers kept across the caller's batches.
DeviceBatchOut device_batch(DeviceComm& dc, DeviceSearch& ds, const RecordBatch* rb, int64_t n, int64_t total_chars,
                            const std::vector<int64_t>& bounds, bool cp, const PhaseHooks& hooks,
                            DeviceScratch* scratch = nullptr);

class BulkParser;
// The same record-slice batch straight from the input text: the root encodes each rank's slice
// (BulkParser::fill_slice after pass 1; `parser` and the p+1 record `bounds` are read on the root only)
// into that rank's wire block in page-locked memory, its own first (uploaded while the peers' are encoded),
// then the peers', and sends a block's pieces while it
// encodes the next rank's slice (no intermediate byte-code batch). Phases: "fill" (root), "distribute",
// "compute", "gather". An input error found in any slice comes back on every rank (nothing searched).
// `record_base`: the global index of the parser's record 0 (a streamed batch's area parser), for the
// error messages; `results_slot` 0/1: which of two page-locked result buffers the root's runs point into
// (a streaming caller prints batch b from one while batch b+1 is gathered into the other).
DeviceBatchOut device_batch_text(DeviceComm& dc, DeviceSearch& ds, const BulkParser* parser,
                                 const std::vector<int64_t>& bounds, const PhaseHooks& hooks,
                                 DeviceScratch* scratch = nullptr, int64_t record_base = 0, int results_slot = 0);

}  // namespace moc
