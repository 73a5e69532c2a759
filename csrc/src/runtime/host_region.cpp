// HostRegion (moc/runtime/host_region.hpp): huge-page-advised, optionally NUMA-bound private buffers.
#include "moc/runtime/host_region.hpp"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <string>

#include "moc/common.hpp"

namespace moc {

namespace {
constexpr size_t kHuge = size_t{2} << 20;
}

bool bind_range_to_node(void* p, size_t bytes, int node) {
  if (node < 0 || bytes == 0 || node >= 1024) return false;
  unsigned long mask[1024 / (8 * sizeof(unsigned long))] = {0};
  mask[node / (8 * sizeof(unsigned long))] |= 1ul << (node % (8 * sizeof(unsigned long)));
  constexpr int kMpolPreferred = 1;
  const uintptr_t lo = reinterpret_cast<uintptr_t>(p) & ~uintptr_t{4095};
  const uintptr_t hi = reinterpret_cast<uintptr_t>(p) + bytes;
  return syscall(SYS_mbind, reinterpret_cast<void*>(lo), hi - lo, kMpolPreferred, mask, sizeof(mask) * 8, 0) == 0;
}

void prefault_pages(char* p, size_t bytes) {
  constexpr size_t kPage = 4096;
  const int64_t pages = static_cast<int64_t>((bytes + kPage - 1) / kPage);
#pragma omp parallel for schedule(static) if (pages > 1024)
  for (int64_t q = 0; q < pages; ++q) p[static_cast<size_t>(q) * kPage] = 0;
}

HostRegion::HostRegion(size_t bytes, int numa_node) {
  // below 1 MiB: plain 4 KiB pages (a huge page's first touch zeroes 2 MiB — 0.2-2 ms for a buffer of a
  // few bytes, the whole search time of a reference-sized input)
  const bool huge = bytes >= (size_t{1} << 20);
  const size_t align = huge ? kHuge : size_t{4096};
  const size_t want = (std::max<size_t>(bytes, 1) + align - 1) & ~(align - 1);
  map_bytes_ = huge ? want + kHuge : want;  // slack to start on a 2 MiB boundary
  map_ = mmap(nullptr, map_bytes_, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (map_ == MAP_FAILED) {
    map_ = nullptr;
    throw Error("HostRegion: cannot map " + std::to_string(map_bytes_) + " bytes");
  }
  base_ = reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(map_) + align - 1) & ~(align - 1));
  bytes_ = bytes;
  if (huge) (void)madvise(base_, want, MADV_HUGEPAGE);  // advisory: 4 KiB pages if THP is off
  if (numa_node >= 0) (void)bind_range_to_node(base_, want, numa_node);
}

void HostRegion::prefault() {
  if (base_) prefault_pages(base_, bytes_);
}

HostRegion& HostRegion::operator=(HostRegion&& o) noexcept {
  if (this != &o) {
    release();
    map_ = o.map_;
    map_bytes_ = o.map_bytes_;
    base_ = o.base_;
    bytes_ = o.bytes_;
    releaser_ = o.releaser_;
    o.map_ = nullptr;
    o.base_ = nullptr;
    o.bytes_ = o.map_bytes_ = 0;
  }
  return *this;
}

HostRegion::~HostRegion() { release(); }

void HostRegion::release() {
  if (!map_) return;
  void* m = map_;
  const size_t len = map_bytes_;
  map_ = nullptr;
  base_ = nullptr;
  bytes_ = map_bytes_ = 0;
  if (releaser_)
    releaser_->defer([m, len] { munmap(m, len); });
  else
    munmap(m, len);
}

MappedFile::MappedFile(const char* path, size_t bytes) {
  const size_t page = static_cast<size_t>(sysconf(_SC_PAGESIZE));
  map_bytes_ = (bytes + 64 + page - 1) / page * page;
  // zero pages first, then the file over their front: the tail past the file's last page stays anonymous
  void* m = mmap(nullptr, map_bytes_, PROT_READ, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
  if (m == MAP_FAILED) throw Error("cannot reserve " + std::to_string(map_bytes_) + " bytes for " + path);
  base_ = static_cast<char*>(m);
  bytes_ = bytes;
  if (bytes == 0) return;
  const int fd = ::open(path, O_RDONLY | O_CLOEXEC);
  void* f = fd < 0 ? MAP_FAILED : mmap(base_, bytes, PROT_READ, MAP_PRIVATE | MAP_FIXED, fd, 0);
  if (fd >= 0) ::close(fd);
  if (f == MAP_FAILED) {
    munmap(base_, map_bytes_);
    base_ = nullptr;
    throw Error(std::string("cannot map ") + path);
  }
}

MappedFile::~MappedFile() {
  if (!base_) return;
  void* b = base_;
  const size_t n = map_bytes_;
  if (releaser_) {
    releaser_->defer([b, n] { munmap(b, n); });
  } else {
    munmap(b, n);
  }
}

}  // namespace moc
