// Process-wide registry of page-locked host memory (hipHostRegister) made through this library.
//
// The zero-copy streaming path hands host addresses straight to a kernel, so it must know that EVERY
// page a kernel touches is mapped for the GPU — asking the runtime about the first and last byte of a
// range is not enough (two neighbouring registrations can cover both ends with an unmapped gap between
// them; a kernel that walks into the gap faults). HIP offers no query for a registration's extent
// (hipMemGetAddressRange reports the size but no base for registered host memory on ROCm 7.2), so the
// library records every registration it makes and answers coverage questions from that record.
#pragma once

#include <cstddef>
#include <cstdint>
#include <utility>
#include <vector>

namespace moc {
namespace pinned {

// Page-locks (hipHostRegisterMapped) the pages of [p, p+bytes) that are not yet registered, as one
// registration per maximal uncovered run. Returns the bases of the registrations made (to release).
std::vector<void*> register_range(const void* p, size_t bytes);
// Releases registrations made by register_range.
void unregister(const std::vector<void*>& bases);
// Page-locked allocation (hipHostMalloc, NUMA placement by the caller's memory policy), recorded in the
// registry like a registration so the streaming paths accept it; release with free_host.
void* alloc_host(size_t bytes);
void free_host(void* p);
// True when every byte of [p, p+bytes) lies in registrations made through this registry.
bool covers(const void* p, size_t bytes);
// Device address of host pointer p inside a covered range (nullptr if not covered). On ROCm's unified
// address space this is p itself; a runtime that maps registrations elsewhere gets single-registration
// ranges only.
const void* device_address(const void* p, size_t bytes);
// Splits [p, p+bytes) at the boundaries of the registrations it touches: each piece (offset, length)
// lies inside ONE registration or outside all of them. The runtime resolves a host pointer of an async
// copy to the single registration containing it and rejects copies that run past its end
// (hipErrorInvalidValue), which neighbouring arrays pinned as separate runs (sharing a page) produce.
std::vector<std::pair<size_t, size_t>> segments(const void* p, size_t bytes);

}  // namespace pinned
}  // namespace moc
