// Large private host buffers for one rank's slice of a job: an anonymous mapping, 2 MiB aligned and
// advised for transparent huge pages (512x fewer page faults on first touch, pages to page-lock and
// pages to unmap than 4 KiB pages), optionally bound to a NUMA node before anything touches it — so
// the pages of a GPU rank's letters land next to its GPU's PCIe root complex whichever thread of the
// process writes them first. The unmap can be handed to a BackgroundReleaser.
//
// Reference: malloc'ed fixed-stride buffers that are never freed (main.c:93, 168; bug B7), all on
// whatever node the root's first touch picked.
#pragma once

#include <cstddef>
#include <cstdint>

#include "moc/runtime/releaser.hpp"

namespace moc {

class HostRegion {
 public:
  HostRegion() = default;
  // bytes rounded up to whole 2 MiB pages; numa_node < 0: no binding (first touch decides)
  explicit HostRegion(size_t bytes, int numa_node = -1);
  ~HostRegion();
  HostRegion(HostRegion&& o) noexcept { *this = static_cast<HostRegion&&>(o); }
  HostRegion& operator=(HostRegion&& o) noexcept;
  HostRegion(const HostRegion&) = delete;
  HostRegion& operator=(const HostRegion&) = delete;

  char* data() const { return base_; }
  size_t size() const { return bytes_; }
  template <typename T>
  T* as() const {
    return reinterpret_cast<T*>(base_);
  }
  // Faults every page in now, OpenMP threads over the region (a registration that finds the pages absent
  // faults them in on one thread).
  void prefault();
  // Later release (destruction) goes through `rel` (FIFO, background thread); rel must outlive it.
  void set_releaser(BackgroundReleaser* rel) { releaser_ = rel; }

 private:
  void release();
  void* map_ = nullptr;
  size_t map_bytes_ = 0;
  char* base_ = nullptr;
  size_t bytes_ = 0;
  BackgroundReleaser* releaser_ = nullptr;
};

// A regular file mapped read-only and private (its page-cache pages, shared with every other process that
// maps or reads the file: nothing is copied), followed by at least 64 zero bytes of anonymous memory so
// vector loads may run past the end. Several ranks of one node map the same --input file this way
// instead of one rank reading it into a node-shared segment that every rank then faults in page by page
// (a 1.3 GB input: 0.64 s of segment set-up at 2 ranks on the MI355X box). Unmaps on destruction
// (or on `rel`, when set).
class MappedFile {
 public:
  MappedFile() = default;
  // the first `bytes` bytes of `path`; throws moc::Error when it cannot be opened or mapped
  MappedFile(const char* path, size_t bytes);
  ~MappedFile();
  MappedFile(const MappedFile&) = delete;
  MappedFile& operator=(const MappedFile&) = delete;
  const char* data() const { return base_; }
  size_t size() const { return bytes_; }
  void set_releaser(BackgroundReleaser* rel) { releaser_ = rel; }

 private:
  char* base_ = nullptr;
  size_t bytes_ = 0, map_bytes_ = 0;
  BackgroundReleaser* releaser_ = nullptr;
};

// Writes one byte of every 4 KiB page of [p, p + bytes) (zero), OpenMP-parallel: allocates the pages of
// a fresh shared mapping up front, several threads (and ranks) faulting at once instead of one copy loop
// faulting them in one by one. The contents become zero.
void prefault_pages(char* p, size_t bytes);

// Binds [p, p + bytes) to NUMA node `node` (MPOL_PREFERRED: falls back elsewhere when the node is
// full); best effort, returns false when the kernel refuses. Pages already present are not moved.
bool bind_range_to_node(void* p, size_t bytes, int node);

}  // namespace moc
