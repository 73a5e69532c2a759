#include "moc/runtime/pinned.hpp"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <map>
#include <mutex>

#include "moc/runtime/hip_check.hpp"
#include "moc/runtime/log.hpp"

namespace moc {
namespace pinned {

namespace {
constexpr uintptr_t kPage = 4096;

std::mutex& mu() {
  static std::mutex m;
  return m;
}
// base -> end of every live registration (non-overlapping by construction)
std::map<uintptr_t, uintptr_t>& regs() {
  static std::map<uintptr_t, uintptr_t> r;
  return r;
}

// First registration whose end is beyond x (the one containing x, or the next one).
std::map<uintptr_t, uintptr_t>::iterator at_or_after(uintptr_t x) {
  auto& r = regs();
  auto it = r.upper_bound(x);
  if (it != r.begin()) {
    auto prev = std::prev(it);
    if (prev->second > x) return prev;
  }
  return it;
}

bool covers_locked(uintptr_t b, uintptr_t e, bool single) {
  auto& r = regs();
  auto it = at_or_after(b);
  uintptr_t x = b;
  while (x < e) {
    if (it == r.end() || it->first > x) return false;  // gap at x
    x = it->second;
    if (single && x < e) return false;
    ++it;
  }
  return true;
}
}  // namespace

std::vector<void*> register_range(const void* p, size_t bytes) {
  std::vector<void*> made;
  if (!p || bytes == 0) return made;
  const uintptr_t b = reinterpret_cast<uintptr_t>(p) & ~(kPage - 1);
  const uintptr_t e = (reinterpret_cast<uintptr_t>(p) + bytes + kPage - 1) & ~(kPage - 1);
  std::lock_guard<std::mutex> lock(mu());
  auto& r = regs();
  uintptr_t x = b;
  auto it = at_or_after(b);
  while (x < e) {
    if (it != r.end() && it->first <= x) {  // already covered up to it->second
      x = it->second;
      ++it;
      continue;
    }
    const uintptr_t run_end = std::min(e, it == r.end() ? e : it->first);
    const hipError_t rc = hipHostRegister(reinterpret_cast<void*>(x), run_end - x, hipHostRegisterMapped);
    if (rc != hipSuccess) {
      // all or nothing: the runs registered by this call are dropped again (a caller that catches the
      // error never receives them, so nobody else could unregister them; a later mapping at the same
      // addresses would then count as page-locked)
      (void)hipGetLastError();
      for (void* q : made) {
        (void)hipHostUnregister(q);
        r.erase(reinterpret_cast<uintptr_t>(q));
      }
      (void)hipGetLastError();
      MOC_HIP_CHECK(rc);
    }
    r.emplace(x, run_end);
    made.push_back(reinterpret_cast<void*>(x));
    x = run_end;
    it = at_or_after(x);
  }
  return made;
}

void unregister(const std::vector<void*>& bases) {
  std::lock_guard<std::mutex> lock(mu());
  for (void* p : bases) {
    const hipError_t e = hipHostUnregister(p);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      MOC_LOG_WARN("hipHostUnregister(%p): %s", p, hipGetErrorString(e));
    }
    regs().erase(reinterpret_cast<uintptr_t>(p));
  }
}

void* alloc_host(size_t bytes) {
  void* p = nullptr;
  MOC_HIP_CHECK(hipHostMalloc(&p, std::max<size_t>(bytes, 1), hipHostMallocMapped | hipHostMallocNumaUser));
  const uintptr_t b = reinterpret_cast<uintptr_t>(p) & ~(kPage - 1);
  const uintptr_t e = (reinterpret_cast<uintptr_t>(p) + std::max<size_t>(bytes, 1) + kPage - 1) & ~(kPage - 1);
  std::lock_guard<std::mutex> lock(mu());
  regs().emplace(b, e);
  return p;
}

void free_host(void* p) {
  if (!p) return;
  {
    std::lock_guard<std::mutex> lock(mu());
    regs().erase(reinterpret_cast<uintptr_t>(p) & ~(kPage - 1));
  }
  (void)hipHostFree(p);
}

bool covers(const void* p, size_t bytes) {
  if (!p) return false;
  const uintptr_t b = reinterpret_cast<uintptr_t>(p);
  std::lock_guard<std::mutex> lock(mu());
  return covers_locked(b, b + std::max<size_t>(bytes, 1), false);
}

const void* device_address(const void* p, size_t bytes) {
  if (!p) return nullptr;
  const uintptr_t b = reinterpret_cast<uintptr_t>(p);
  bool multi = false;
  {
    std::lock_guard<std::mutex> lock(mu());
    if (!covers_locked(b, b + std::max<size_t>(bytes, 1), false)) return nullptr;
    multi = !covers_locked(b, b + std::max<size_t>(bytes, 1), true);
  }
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, const_cast<void*>(p), 0) != hipSuccess || !d) {
    (void)hipGetLastError();
    return nullptr;
  }
  // several registrations are contiguous for the device only in a unified address space (d == p)
  if (multi && d != p) return nullptr;
  return d;
}

std::vector<std::pair<size_t, size_t>> segments(const void* p, size_t bytes) {
  std::vector<std::pair<size_t, size_t>> out;
  if (!p || bytes == 0) return out;
  const uintptr_t b = reinterpret_cast<uintptr_t>(p), e = b + bytes;
  std::lock_guard<std::mutex> lock(mu());
  auto& r = regs();
  auto it = at_or_after(b);
  uintptr_t x = b;
  while (x < e) {
    uintptr_t y;
    if (it != r.end() && it->first <= x) {  // inside a registration: up to its end
      y = std::min(e, it->second);
      ++it;
    } else {  // unregistered: up to the next registration
      y = std::min(e, it == r.end() ? e : it->first);
    }
    out.emplace_back(static_cast<size_t>(x - b), static_cast<size_t>(y - x));
    x = y;
  }
  return out;
}

}  // namespace pinned
}  // namespace moc
