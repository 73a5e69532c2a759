// Host timers — the native replacement for the vendored CUDA-Samples StopWatchLinux
// (inc/helper_timer.h:215-343: start/stop/reset/getTime/getAverageTime over sessions), which the
// reference ships but never uses. Device-side timing uses hipEvents (runtime/device.hpp).
#pragma once

#include <chrono>
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace moc {

class Stopwatch {
 public:
  using clock = std::chrono::steady_clock;
  void start() {
    t0_ = clock::now();
    running_ = true;
  }
  void stop() {
    if (!running_) return;
    total_ += std::chrono::duration<double, std::milli>(clock::now() - t0_).count();
    ++sessions_;
    running_ = false;
  }
  void reset() {
    total_ = 0;
    sessions_ = 0;
    running_ = false;
  }
  // Total milliseconds over all completed sessions (+ the running one).
  double total_ms() const {
    double t = total_;
    if (running_) t += std::chrono::duration<double, std::milli>(clock::now() - t0_).count();
    return t;
  }
  double average_ms() const { return sessions_ ? total_ / sessions_ : 0.0; }
  int sessions() const { return sessions_; }

 private:
  clock::time_point t0_{};
  double total_ = 0;
  int sessions_ = 0;
  bool running_ = false;
};

// Ordered named phases, emitted as one JSON object (the --timing output). Each phase is also a roctx
// range (runtime/trace.hpp), so profiler timelines carry the same phase names.
class PhaseTimer {
 public:
  void begin(const std::string& name);  // closes the open phase, if any
  void end();
  void add(const std::string& name, double ms) {
    for (auto& p : phases_)
      if (p.first == name) {
        p.second += ms;
        return;
      }
    phases_.emplace_back(name, ms);
  }
  double get(const std::string& name) const {
    for (auto& p : phases_)
      if (p.first == name) return p.second;
    return 0.0;
  }
  const std::vector<std::pair<std::string, double>>& phases() const { return phases_; }
  std::string json(const std::vector<std::pair<std::string, double>>& extra = {}) const;

 private:
  std::string cur_;
  bool open_ = false;
  Stopwatch sw_;
  std::vector<std::pair<std::string, double>> phases_;
};

inline double now_seconds() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace moc
