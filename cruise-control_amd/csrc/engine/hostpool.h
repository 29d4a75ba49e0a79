// A process-wide pool of host threads for the engine's data-parallel host loops (the snapshot directory's syncs:
// every broker's sorted view and its rows' upload). The calling thread takes part in its own loop and returns as soon
// as every index is done; helpers wake on a condition variable and share the remaining indices, so a short loop runs
// on the caller alone without waiting for a wake-up. Jobs are reference-counted: a helper that wakes after the loop
// finished finds nothing left and drops its reference. One loop at a time per process; a caller that finds the pool
// busy (another session's loop) runs its loop alone. CCMI_SYNC_THREADS (default 8) counts the caller. A helper runs
// each job on the CPU mask of the job's caller (CpuMask::follow): the pool belongs to no session's NUMA node.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include <immintrin.h>
#include <pthread.h>

#include "threadpin.h"

namespace ccmi {

class HostPool {
 public:
  static HostPool& get() {
    static HostPool* p = new HostPool();  // never destroyed: helpers stay parked on the condition variable
    return *p;
  }
  int threads() const { return threads_; }
  // f(i) for every i in [0, n), on the caller and the helpers; returns when all are done
  void parallelFor(int n, const std::function<void(int)>& f) {
    if (n <= 0) return;
    std::unique_lock<std::mutex> busy(runMu_, std::try_to_lock);
    if (threads_ <= 1 || n == 1 || !busy.owns_lock()) {
      for (int i = 0; i < n; ++i) f(i);
      return;
    }
    auto job = std::make_shared<Job>(n, f);
    job->mask = CpuMask::current();  // the helpers run this job on the caller's CPUs
    {
      std::lock_guard<std::mutex> l(mu_);
      job_ = job;
      ++gen_;
    }
    cv_.notify_all();
    run(*job);
    while (job->done.load(std::memory_order_acquire) < n) _mm_pause();
    std::lock_guard<std::mutex> l(mu_);
    if (job_ == job) job_.reset();
  }

 private:
  struct Job {
    Job(int n_, const std::function<void(int)>& f_) : n(n_), f(f_) {}
    const int n;
    std::function<void(int)> f;
    CpuMask mask;
    std::atomic<int> next{0}, done{0};
  };
  static void run(Job& j) {
    for (int i; (i = j.next.fetch_add(1, std::memory_order_relaxed)) < j.n;) {
      j.f(i);
      j.done.fetch_add(1, std::memory_order_release);
    }
  }
  HostPool() {
    const char* e = std::getenv("CCMI_SYNC_THREADS");
    threads_ = e ? std::max(1, std::atoi(e)) : 8;
    for (int t = 1; t < threads_; ++t) std::thread([this] { loop(); }).detach();
  }
  void loop() {
    pthread_setname_np(pthread_self(), "ccmi-sync");
    uint64_t seen = 0;
    CpuMask mine = CpuMask::current();
    for (;;) {
      std::shared_ptr<Job> j;
      {
        std::unique_lock<std::mutex> l(mu_);
        cv_.wait(l, [&] { return gen_ != seen; });
        seen = gen_;
        j = job_;
      }
      if (j) {
        mine.follow(j->mask);
        run(*j);
      }
    }
  }
  int threads_ = 1;
  std::mutex runMu_, mu_;
  std::condition_variable cv_;
  std::shared_ptr<Job> job_;
  uint64_t gen_ = 0;
};

}  // namespace ccmi
