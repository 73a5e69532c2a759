// Distributed layer of the native CLI: MPI bootstrap + host collectives, RCCL device collectives,
// and the node-shared input window.
//
// Reference collectives: MPI_Bcast x4 (main.c:149-152, incl. the 16-int weights
// over-read, bug B3), MPI_Scatter of fixed 2000-byte records (main.c:174) and MPI_Gather x3
// (main.c:195-197), all blocking, host-memory, rooted at 0, and with no device binding (B14).
//
// Here:
//   * MpiContext   — MPI_Init_thread, world + node-local communicators, local rank -> device.
//   * host helpers — exact-count broadcasts, 64-bit-safe Scatterv/Gatherv of bytes.
//   * SharedWindow — MPI_Win_allocate_shared over the node communicator: the root parses the input
//                    into it once and every rank DMAs its own slice over its own PCIe link.
// RcclComm (moc/rccl_comm.hpp) adds the RCCL device collectives on top of an MpiContext.
#pragma once

#include <mpi.h>

#include <cstdint>
#include <string>
#include <vector>

#include "moc/common.hpp"
#include "moc/runtime/host_region.hpp"
#include "moc/runtime/releaser.hpp"

namespace moc {

// MPI start-up without the hardware discovery nothing here uses. MPICH's MPI_Init loads a full hwloc
// topology of the host: on the MI355X box (256 PUs, 367 PCI devices) that is 170-220 ms of a tiny job's
// ~210 ms at one rank and 350 ms at eight — the `x86` component binds to every PU to run cpuid, `linuxio`
// scans every PCI device, `linux` reads every PU's sysfs topology (and eight ranks do it at once). With
// hwloc's `no_os` component alone (a flat topology from the CPU count) MPI_Init takes 2-4 ms at 1-8 ranks
// (profiles/mpi_init_variants_box.log, profiles/mpi_init_floor_box.log). Nothing in this framework reads
// MPI's topology: ranks find their node through MPI_COMM_TYPE_SHARED, their device from the node-local
// rank and their NUMA node from the device's own sysfs entry. `full` keeps MPI's discovery; a
// HWLOC_COMPONENTS the user set is always kept. Call before any other thread starts (setenv).
void mpi_prepare_env(bool lean_topology);

class MpiContext {
 public:
  MpiContext(int* argc, char*** argv);
  ~MpiContext();
  MpiContext(const MpiContext&) = delete;
  MpiContext& operator=(const MpiContext&) = delete;

  int rank = 0, size = 1;
  int local_rank = 0, local_size = 1;
  int node_count = 1;
  MPI_Comm world = MPI_COMM_WORLD;
  MPI_Comm node = MPI_COMM_NULL;  // ranks sharing this node's memory
  bool single_node() const { return node_count == 1; }
  std::string hostname;

  [[noreturn]] void abort(int code, const std::string& msg) const;
};

void mpi_check(int rc, const char* what);

// A pending point-to-point request's peer and size, named when a wait on it times out.
struct ReqInfo {
  int peer = -1;
  int64_t bytes = 0;
  bool send = false;
};
// MPI_Waitall under the job's comm deadline (moc/runtime/watchdog.hpp: CommTimeout when it passes).
// `infos` (optional, parallel to reqs) describes the requests still pending then. Leaves reqs empty.
void mpi_wait_all(std::vector<MPI_Request>& reqs, const char* what, const std::vector<ReqInfo>* infos = nullptr);
// One request (a non-blocking collective) under the deadline; `detail` describes it in the message.
void mpi_wait(MPI_Request& req, const char* what, const std::string& detail = {});
// MPI_Barrier under the deadline.
void barrier(MPI_Comm comm, const char* what);

// Broadcast of arbitrary byte counts (>2 GiB safe) from root.
void bcast_bytes(void* buf, int64_t bytes, int root, MPI_Comm comm);
// Root sends counts[r] bytes at displs[r] of sendbuf to rank r (64-bit safe, any sizes).
void scatterv_bytes(const void* sendbuf, const std::vector<int64_t>& counts, const std::vector<int64_t>& displs,
                    void* recvbuf, int root, MPI_Comm comm);
// Inverse of scatterv_bytes.
void gatherv_bytes(const void* sendbuf, int64_t count, void* recvbuf, const std::vector<int64_t>& counts,
                   const std::vector<int64_t>& displs, int root, MPI_Comm comm);

// In-place element-wise MAX over all ranks of n uint64 values (context-parallel key combine, §5.7).
void allreduce_max_u64(uint64_t* buf, int64_t n, MPI_Comm comm);

class SharedWindow {
 public:
  // Collective over ctx.node; only the node's local rank 0 allocates `bytes` (others pass 0). A node with a
  // single rank shares nothing: it maps private memory advised for 2 MiB pages instead of an MPI segment
  // (the node's tmpfs has no huge pages), which cuts the page faults of the fill, the pages to pin and
  // the cost of the unmap by 512x.
  SharedWindow(const MpiContext& ctx, int64_t bytes);
  ~SharedWindow();
  char* base() const { return base_; }
  int64_t bytes() const { return bytes_; }
  void fence() const;  // MPI_Win_sync + node barrier: makes the owner's writes visible
  // Collective over the node: every rank allocates (faults in) its 1/local_size share of the window's
  // pages with its threads, so the owner's later fill runs into present pages (a shared mapping has no
  // huge pages here: 4 KiB faults, ~1 us each, are what a single-threaded fill would pay one by one).
  void prefault_shares(const MpiContext& ctx);
  // Not collective: ranks other than the node's local rank 0 return the window's pages to the OS in
  // shares (MADV_REMOVE), in parallel, while local rank 0 goes on (e.g. the root printing). The contents
  // are gone afterwards; the later collective free then has nothing left to release.
  void release_shares(const MpiContext& ctx);
  // Single-rank nodes (private mapping) only, no-op otherwise: every later release of this window's pages
  // goes through `rel` (FIFO, background thread) instead of the caller's thread. `rel` must outlive the
  // queued tasks (drain it before the process ends).
  void set_releaser(BackgroundReleaser* rel) { releaser_ = map_ ? rel : nullptr; }
  // Returns the whole 2 MiB pages inside [off, off+len) to the OS (asynchronously with a releaser). The
  // caller must not touch that range again. No-op for an MPI window (its pages are shared with peers).
  void discard(int64_t off, int64_t len);

 private:
  MPI_Win win_ = MPI_WIN_NULL;
  MPI_Comm comm_ = MPI_COMM_NULL;
  char* base_ = nullptr;
  int64_t bytes_ = 0;
  void* map_ = nullptr;  // a node with one rank: private anonymous mapping (transparent huge pages)
  size_t map_bytes_ = 0;
  BackgroundReleaser* releaser_ = nullptr;
};

// Per-rank segments of one node-shared window: every rank of the node allocates its own segment (its
// result slice), placed on the owner's NUMA node (MPI's noncontiguous allocation + a memory-policy
// binding by the owner before its first touch), and every rank can address every segment — the root
// prints straight from them, so no gather copy exists. A node with one rank maps private memory.
class SegmentWindow {
 public:
  // Collective over ctx.node. numa_node >= 0 binds this rank's segment there.
  SegmentWindow(const MpiContext& ctx, int64_t my_bytes, int numa_node = -1);
  ~SegmentWindow();
  SegmentWindow(const SegmentWindow&) = delete;
  SegmentWindow& operator=(const SegmentWindow&) = delete;
  char* mine() const { return segment(local_rank_); }
  char* segment(int local_rank) const { return seg_[static_cast<size_t>(local_rank)]; }
  void fence() const;  // MPI_Win_sync + node barrier: makes every owner's writes visible
  void set_releaser(BackgroundReleaser* rel) { region_.set_releaser(rel); }

 private:
  MPI_Win win_ = MPI_WIN_NULL;
  MPI_Comm comm_ = MPI_COMM_NULL;
  int local_rank_ = 0;
  std::vector<char*> seg_;
  HostRegion region_;  // one rank on the node
};

}  // namespace moc
