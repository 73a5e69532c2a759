// Deadline polling of the distributed layer's waits (moc/runtime/watchdog.hpp).
#include "moc/runtime/watchdog.hpp"

#include <atomic>
#include <chrono>
#include <cstdio>
#include <mutex>
#include <thread>

namespace moc {
namespace watchdog {

namespace {
std::atomic<double> g_timeout_s{kDefaultTimeoutS};
std::atomic<int> g_rank{-1};
std::mutex g_mu;
std::string g_phase;  // under g_mu
}  // namespace

void set_timeout_s(double s) { g_timeout_s.store(s); }
double timeout_s() { return g_timeout_s.load(); }
void set_phase(const char* phase) {
  std::lock_guard<std::mutex> lock(g_mu);
  g_phase = phase ? phase : "";
}
std::string phase() {
  std::lock_guard<std::mutex> lock(g_mu);
  return g_phase;
}
void set_rank(int rank) { g_rank.store(rank); }
int rank() { return g_rank.load(); }

std::string human_bytes(int64_t bytes) {
  char buf[32];
  if (bytes < 1024)
    std::snprintf(buf, sizeof buf, "%lld B", static_cast<long long>(bytes));
  else if (bytes < (int64_t{1} << 20))
    std::snprintf(buf, sizeof buf, "%.1f KiB", bytes / 1024.0);
  else if (bytes < (int64_t{1} << 30))
    std::snprintf(buf, sizeof buf, "%.1f MiB", bytes / 1048576.0);
  else
    std::snprintf(buf, sizeof buf, "%.2f GiB", bytes / 1073741824.0);
  return buf;
}

void wait(const std::function<bool()>& done, const WaitSpec& spec) {
  using clock = std::chrono::steady_clock;
  if (done()) return;
  const double limit = timeout_s();
  const clock::time_point t0 = clock::now();
  clock::time_point next_check = t0;
  // spin (with a yield) for the first 2 ms: the latency of a small collective is MPI's / the stream's own
  constexpr auto kSpin = std::chrono::milliseconds(2);
  auto sleep = std::chrono::microseconds(20);
  const bool busy = spec.poll == Poll::Busy;
  unsigned polls = 0;
  while (!done()) {
    if (busy) {
      // a yield between polls past the first few: ranks oversubscribing their cores (more ranks and OpenMP
      // threads than CPUs) hand the core to the peer they wait for, as MPICH's own blocking waits do
      if (++polls > 64) std::this_thread::yield();
      if ((polls & 63u) != 0) continue;  // the clock every 64 polls
    }
    const clock::time_point now = clock::now();
    if (spec.check && now >= next_check) {
      spec.check();
      next_check = now + std::chrono::milliseconds(1);
    }
    const double waited = std::chrono::duration<double>(now - t0).count();
    if (limit > 0 && waited > limit) {
      if (spec.expire) spec.expire();
      char head[160];
      std::snprintf(head, sizeof head, "comm timeout: rank %d waited %.1f s (--comm-timeout %g)", rank(), waited, limit);
      const std::string ph = phase();  // unset in a plugin's copy: the caller's fatal message adds it
      std::string msg = head + (ph.empty() ? std::string() : " in phase '" + ph + "'") + " for " + spec.what;
      if (spec.outstanding) {
        const std::string o = spec.outstanding();
        if (!o.empty()) msg += "; outstanding: " + o;
      }
      throw CommTimeout(msg);
    }
    if (busy) continue;
    if (now - t0 < kSpin) {
      std::this_thread::yield();
    } else {
      std::this_thread::sleep_for(sleep);
      if (sleep < std::chrono::microseconds(1000)) sleep *= 2;
    }
  }
}

}  // namespace watchdog
}  // namespace moc
