// Deferred release of large host memory on a background thread (and, as a plain FIFO worker, the ordered
// background writes of the result writer's pipe path, io.cpp write_results).
//
// Returning gigabytes of pages to the OS (munmap of the node window, freeing the input buffer) costs
// ~40 ms per GB of 4 KiB pages and sits on the job's critical path when done inline (reference: there is
// no counterpart — its buffers are never freed, main.c:213-240). The root's tail after the search is
// printing, which needs only the results, so the pages nobody reads any more are returned while it runs.
//
// Tasks run in FIFO order on one worker thread, so several operations on the same mapping (discard an
// interior range, then unmap the whole) can never reorder: an address range is only unmapped once, after
// everything queued before it, and no later mmap can receive it while a queued task still names it.
#pragma once

#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>

namespace moc {

class BackgroundReleaser {
 public:
  BackgroundReleaser() = default;
  BackgroundReleaser(const BackgroundReleaser&) = delete;
  BackgroundReleaser& operator=(const BackgroundReleaser&) = delete;
  ~BackgroundReleaser() { stop(); }

  // Queues fn; the worker thread starts with the first task.
  void defer(std::function<void()> fn) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      q_.push_back(std::move(fn));
      ++pending_;
    }
    if (!worker_.joinable()) worker_ = std::thread([this] { loop(); });
    cv_.notify_one();
  }

  // Blocks until every queued task has run.
  void drain() {
    std::unique_lock<std::mutex> lk(mu_);
    idle_.wait(lk, [this] { return pending_ == 0; });
  }

  // Drains and joins the worker.
  void stop() {
    if (!worker_.joinable()) return;
    {
      std::lock_guard<std::mutex> lk(mu_);
      quit_ = true;
    }
    cv_.notify_one();
    worker_.join();
  }

 private:
  void loop() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [this] { return quit_ || !q_.empty(); });
      if (q_.empty()) return;  // quit_ and nothing left
      std::function<void()> fn = std::move(q_.front());
      q_.pop_front();
      lk.unlock();
      fn();
      fn = nullptr;  // captured owners are released on this thread too
      lk.lock();
      if (--pending_ == 0) idle_.notify_all();
    }
  }

  std::mutex mu_;
  std::condition_variable cv_, idle_;
  std::deque<std::function<void()>> q_;
  int64_t pending_ = 0;
  bool quit_ = false;
  std::thread worker_;
};

}  // namespace moc
