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
#include <cstdlib>
#include <exception>
#include <climits>
#include <functional>
#include <cstdio>
#include <cstring>
#include <malloc.h>
#include <mutex>
#include <pthread.h>
#include <sched.h>
#include <string>
#include <stdexcept>
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
  // true on a pool worker, and on the caller while it runs a parallelFor
  // (a nested parallelFor would deadlock: callers check and run inline)
  static bool busyHere() { return inJob_; }

  // fn(worker, begin, end) over [0, n) in size() contiguous chunks; the first
  // exception (if any) is rethrown on the caller
  // chunks > 0: that many chunks (claimed dynamically by the threads; for
  // uneven per-item cost), fn's first argument then ranges over them
  void parallelFor(size_t n, const std::function<void(size_t, size_t, size_t)>& fn, size_t chunks = 0) {
    const size_t parts = std::min(chunks ? chunks : size(), std::max<size_t>(n, 1));
    if (parts <= 1 || inJob_) {
      fn(0, 0, n);
      return;
    }
    // one job at a time: callers on other threads (multi-device builds drive
    // each device from its own thread) queue here and then get the whole pool
    std::lock_guard<std::mutex> turn(callerMu_);
    struct Mark {
      Mark() { inJob_ = true; }
      ~Mark() { inJob_ = false; }
    } mark;
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
    tuneAllocator();
    // the caller plus workers: at most 16, and one CPU of the process's share
    // left to the HIP runtime's threads (a cgroup quota below the affinity
    // mask throttles a pool that fills it: profiles/r05/ cpu.stat A/B)
    size_t t = std::min<size_t>(16, usableCpus() > 2 ? usableCpus() - 1 : usableCpus());
    if (const char* e = std::getenv("ORH_HOST_THREADS")) t = std::max(1, std::atoi(e));
    // each worker pinned to its own physical core of the caller's socket,
    // nearest core ids first, instead of left to the scheduler, which spreads
    // them over sockets and away from the memory the caller filled: C3 build
    // 4.0 -> 2.9 ms, C5 53-58 -> 44-48 ms on one box
    // (profiles/r06/ac_pool_pin_ab.txt). Only the pool's own threads are
    // pinned. Default: on in a single-process run, off when WORLD_SIZE > 1
    // (ranks on one node would pick overlapping cores); ORH_POOL_PIN=0 / 1
    // forces it
    const char* pe = std::getenv("ORH_POOL_PIN");
    const char* ws = std::getenv("WORLD_SIZE");
    const bool pin = pe ? pe[0] == '1' : !(ws && std::atoi(ws) > 1);
    const std::vector<int> pins = pin ? nearCores(t - 1) : std::vector<int>{};
    for (size_t i = 1; i < t; ++i) {
      workers_.emplace_back([this] { loop(); });
      if (i - 1 < pins.size()) {
        cpu_set_t one;
        CPU_ZERO(&one);
        CPU_SET(pins[i - 1], &one);
        pthread_setaffinity_np(workers_.back().native_handle(), sizeof one, &one);
      }
    }
  }
  static int readInt(const std::string& path) {
    FILE* f = std::fopen(path.c_str(), "r");
    if (!f) return -1;
    int v = -1;
    if (std::fscanf(f, "%d", &v) != 1) v = -1;
    std::fclose(f);
    return v;
  }
  // up to n CPUs of the affinity mask: one hardware thread per physical core
  // of the calling thread's package, by distance of cpu id from the caller's
  static std::vector<int> nearCores(size_t n) {
    std::vector<int> out;
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof set, &set) != 0) return out;
    const int me = sched_getcpu();
    if (me < 0) return out;
    auto topo = [](int c, const char* f) {
      return readInt("/sys/devices/system/cpu/cpu" + std::to_string(c) + "/topology/" + f);
    };
    const int pkg = topo(me, "physical_package_id");
    std::vector<std::pair<int, int>> cand;  // (distance, cpu)
    std::vector<std::pair<int, int>> seen;  // (package, core)
    for (int c = 0; c < CPU_SETSIZE; ++c) {
      if (!CPU_ISSET(c, &set) || c == me) continue;
      const int p = topo(c, "physical_package_id"), core = topo(c, "core_id");
      if (p != pkg || core < 0) continue;
      if (std::find(seen.begin(), seen.end(), std::make_pair(p, core)) != seen.end()) continue;
      seen.emplace_back(p, core);
      cand.emplace_back(std::abs(c - me), c);
    }
    std::sort(cand.begin(), cand.end());
    for (size_t i = 0; i < cand.size() && out.size() < n; ++i) out.push_back(cand[i].second);
    return out;
  }
  // CPUs this process may use: the affinity mask, capped by the cgroup v2
  // quota (cpu.max "quota period")
  static size_t usableCpus() {
    size_t n = std::max(1u, std::thread::hardware_concurrency());
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof set, &set) == 0) n = std::max(1, CPU_COUNT(&set));
    if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
      char q[32] = {};
      long period = 0;
      if (std::fscanf(f, "%31s %ld", q, &period) == 2 && std::strcmp(q, "max") != 0 && period > 0)
        n = std::min<size_t>(n, static_cast<size_t>(std::max(1L, std::atol(q) / period)));
      std::fclose(f);
    }
    return n;
  }
  // Route databases are millions of small heap objects built and freed on
  // every rebuild. glibc by default returns freed arena tops to the kernel
  // and maps mid-sized blocks one by one, so each build faults its pages in
  // again: keep freed memory in the arenas (no trim, 256 MB top pad, mmap
  // only past 32 MB). C3 build 29.7 -> 16.6 ms, C5 first rebuild 467 -> 193
  // ms, delta 39.5 -> 24.6 ms (profiles/r03/p_malloc_ab.txt). The process
  // then keeps its peak heap, and the settings are process-global, so a
  // library must not impose them: opt-in with ORH_MALLOC_TUNE=1 (the host
  // application owns its allocator policy; bench.py opts in).
  static void tuneAllocator() {
    const char* e = std::getenv("ORH_MALLOC_TUNE");
    if (!e || std::atoi(e) != 1) return;
    mallopt(M_TRIM_THRESHOLD, INT_MAX);
    mallopt(M_TOP_PAD, 256 << 20);
    mallopt(M_MMAP_THRESHOLD, 32 << 20);  // glibc's largest accepted value
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
    inJob_ = true;
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
  std::mutex callerMu_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  const std::function<void(size_t, size_t, size_t)>* job_{nullptr};
  size_t n_{0}, parts_{0}, next_{0}, pending_{0};
  uint64_t gen_{0};
  bool stop_{false};
  std::exception_ptr err_;
  static inline thread_local bool inJob_ = false;
};

// parts[w] -> into, shard by shard on the pool (ShardedMap parts: nodes are
// spliced, no entry is copied); a key in two parts is a duplicate route
// (RouteUpdate.h:39 CHECK)
template <class Map>
void mergeParts(Map& into, std::vector<Map>& parts, WorkerPool& pool) {
  std::atomic<bool> dup{false};
  pool.parallelFor(Map::kShards, [&](size_t, size_t b, size_t e) {
    for (size_t s = b; s < e; ++s) {
      auto& dst = into.shard(s);
      size_t n = dst.size();
      for (auto& p : parts) n += p.shard(s).size();
      dst.reserve(n);
      for (auto& p : parts) {
        dst.merge(p.shard(s));
        if (!p.shard(s).empty()) dup = true;
      }
    }
  });
  if (dup) throw std::logic_error("duplicate unicast route");
}

}  // namespace openr_amd
