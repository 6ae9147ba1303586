// A small persistent worker pool for the host side of a batch: the chain
// walk, the descriptor/staging writes.  Packets are independent, so a batch
// splits into chunks of consecutive packets that any thread may take.
//
// One batch uses the pool at a time; a batch that finds it busy (another RX/TX
// thread mid-batch) runs its chunks on its own thread instead of waiting.
// The pool is never destroyed: its workers sleep on a condition variable and
// simply end with the process.
#pragma once

#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <time.h>

#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace uinet {

// CPU time of the calling thread (CLOCK_THREAD_CPUTIME_ID), nanoseconds.
inline uint64_t thread_cpu_ns() {
  timespec ts;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

// CPU time that pool helpers spent on this thread's pool runs (and, nested,
// on the runs those helpers made): uinet_cksum_host_cpu adds it to the
// calling thread's own CPU time.
inline thread_local uint64_t t_pool_helper_ns = 0;

class HostPool {
 public:
  // fn(j) for every j in [0, jobs), on at most `threads` threads (the caller
  // is one of them).  Returns when every job has finished.  Helpers float over
  // the process's CPUs (pinning them, the knob host_pin until round 6, never
  // won: profiles/r06/pruned/).
  void run(int jobs, int threads, const std::function<void(int)>& fn) {
    if (threads <= 1 || jobs <= 1 || !busy_.try_lock()) {
      for (int j = 0; j < jobs; j++) fn(j);
      return;
    }
    std::lock_guard<std::mutex> own(busy_, std::adopt_lock);
    grow(threads - 1);
    {
      std::lock_guard<std::mutex> g(mu_);
      fn_ = &fn;
      jobs_ = jobs;
      next_.store(0, std::memory_order_relaxed);
      helpers_ = threads - 1;
      pending_ = threads - 1;
      gen_++;
    }
    cv_.notify_all();
    drain();
    std::unique_lock<std::mutex> g(mu_);
    done_.wait(g, [&] { return pending_ == 0; });
    fn_ = nullptr;
    t_pool_helper_ns += helper_ns_;
    helper_ns_ = 0;
  }

 private:
  void drain() {
    for (int j; (j = next_.fetch_add(1, std::memory_order_relaxed)) < jobs_;) (*fn_)(j);
  }
  void grow(int n) {
    while ((int)workers_.size() < n) {
      const int id = (int)workers_.size();
      workers_.emplace_back([this, id] { loop(id); });
      workers_.back().detach();
    }
  }
  void loop(int id) {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return gen_ != seen; });
        seen = gen_;
        if (id >= helpers_) continue;  // not part of this run
      }
      // this helper's CPU time for the run, including what helpers of runs
      // it made itself spent (a multi-device shard's own walk pool)
      const uint64_t c0 = thread_cpu_ns() + t_pool_helper_ns;
      drain();
      const uint64_t c1 = thread_cpu_ns() + t_pool_helper_ns;
      std::lock_guard<std::mutex> g(mu_);
      helper_ns_ += c1 - c0;
      if (--pending_ == 0) done_.notify_one();
    }
  }

  std::mutex busy_;  // held by the batch using the pool
  std::mutex mu_;
  std::condition_variable cv_, done_;
  std::vector<std::thread> workers_;
  const std::function<void(int)>* fn_ = nullptr;
  std::atomic<int> next_{0};
  int jobs_ = 0, helpers_ = 0, pending_ = 0;
  uint64_t helper_ns_ = 0;  // helpers' CPU time in the current run (under mu_)
  uint64_t gen_ = 0;
};

inline HostPool& host_pool() {
  static HostPool* p = new HostPool;  // intentionally leaked, see above
  return *p;
}

}  // namespace uinet
