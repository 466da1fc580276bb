// Host worker pool for the route build: buildRouteDb's per-prefix work is
// independent once the SPF rows it reads are memoized, so it is split over
// host threads (ORH_HOST_THREADS, default min(16, hardware threads)). The
// reference Decision runs it on one thread; results do not depend on the
// split (each prefix's entry is computed by exactly one worker and merged in
// a fixed order).
#pragma once

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <cstdlib>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace openr_amd {

class WorkerPool {
 public:
  static WorkerPool& instance() {
    static WorkerPool pool;
    return pool;
  }
  size_t size() const { return workers_.size() + 1; }  // the caller works too

  // fn(worker, begin, end) over [0, n) in size() contiguous chunks; the first
  // exception (if any) is rethrown on the caller
  void parallelFor(size_t n, const std::function<void(size_t, size_t, size_t)>& fn) {
    const size_t parts = std::min(size(), std::max<size_t>(n, 1));
    if (parts <= 1) {
      fn(0, 0, n);
      return;
    }
    std::unique_lock<std::mutex> lock(mu_);
    job_ = &fn;
    n_ = n;
    parts_ = parts;
    next_ = 1;  // chunk 0 is the caller's
    pending_ = parts - 1;
    err_ = nullptr;
    ++gen_;
    cv_.notify_all();
    lock.unlock();
    runChunk(0);
    lock.lock();
    // the caller keeps claiming chunks too: a worker that wakes late then
    // finds nothing left instead of holding the phase up
    while (next_ < parts_) {
      const size_t c = next_++;
      lock.unlock();
      runChunk(c);
      lock.lock();
      --pending_;
    }
    done_.wait(lock, [&] { return pending_ == 0; });
    job_ = nullptr;
    if (err_) std::rethrow_exception(err_);
  }

 private:
  WorkerPool() {
    size_t t = std::min<size_t>(16, std::max(1u, std::thread::hardware_concurrency()));
    if (const char* e = std::getenv("ORH_HOST_THREADS")) t = std::max(1, std::atoi(e));
    for (size_t i = 1; i < t; ++i) workers_.emplace_back([this] { loop(); });
  }
  ~WorkerPool() {
    {
      std::lock_guard<std::mutex> lock(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& w : workers_) w.join();
  }

  void runChunk(size_t c) {
    const size_t b = n_ * c / parts_, e = n_ * (c + 1) / parts_;
    try {
      (*job_)(c, b, e);
    } catch (...) {
      std::lock_guard<std::mutex> lock(mu_);
      if (!err_) err_ = std::current_exception();
    }
  }

  void loop() {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> lock(mu_);
    for (;;) {
      cv_.wait(lock, [&] { return stop_ || (gen_ != seen && job_ && next_ < parts_); });
      if (stop_) return;
      seen = gen_;
      while (job_ && next_ < parts_) {
        const size_t c = next_++;
        lock.unlock();
        runChunk(c);
        lock.lock();
        if (--pending_ == 0) done_.notify_one();
      }
    }
  }

  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  const std::function<void(size_t, size_t, size_t)>* job_{nullptr};
  size_t n_{0}, parts_{0}, next_{0}, pending_{0};
  uint64_t gen_{0};
  bool stop_{false};
  std::exception_ptr err_;
};

// Frees large containers off the caller's thread: a 1M-route DecisionRouteDb
// is ~5M heap nodes, ~0.7 s of free() (C5), which a Decision thread holding
// routeDb_ would otherwise pay on every full rebuild. One background thread
// destroys what is posted, in order; at exit it drains the queue.
class Reclaimer {
 public:
  static Reclaimer& instance() {
    static Reclaimer r;
    return r;
  }
  // false when the reclaimer is already shut down (the caller frees inline)
  bool post(std::function<void()> fn) {
    std::lock_guard<std::mutex> lock(mu_);
    if (stop_) return false;
    q_.push_back(std::move(fn));
    cv_.notify_one();
    return true;
  }
  // waits until everything posted so far is freed (tests, memory accounting)
  void drain() {
    std::unique_lock<std::mutex> lock(mu_);
    idle_.wait(lock, [&] { return q_.empty() && !busy_; });
  }
  // false once the reclaimer was destroyed (static destruction at exit)
  static bool usable() { return state_.load() != 2; }

 private:
  Reclaimer() : th_([this] { loop(); }) { state_ = 1; }
  ~Reclaimer() {
    state_ = 2;
    {
      std::lock_guard<std::mutex> lock(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  void loop() {
    std::unique_lock<std::mutex> lock(mu_);
    for (;;) {
      cv_.wait(lock, [&] { return stop_ || !q_.empty(); });
      if (q_.empty()) return;  // stopping, nothing left
      auto fn = std::move(q_.front());
      q_.pop_front();
      busy_ = true;
      lock.unlock();
      fn();
      fn = nullptr;
      lock.lock();
      busy_ = false;
      if (q_.empty()) idle_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_, idle_;
  std::deque<std::function<void()>> q_;
  bool stop_{false}, busy_{false};
  static inline std::atomic<int> state_{0};  // 0 never built, 1 running, 2 destroyed
  std::thread th_;
};

}  // namespace openr_amd
