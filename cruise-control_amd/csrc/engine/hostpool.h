// A process-wide pool of host threads for the engine's data-parallel host loops (the snapshot directory's syncs:
// every broker's sorted view and its rows' upload). The calling thread takes part in its own loop and returns as soon
// as every index is done; helpers wake on a condition variable and share the remaining indices, so a short loop runs
// on the caller alone without waiting for a wake-up. Jobs are reference-counted: a helper that wakes after the loop
// finished finds nothing left and drops its reference. The helpers form crews of CCMI_SYNC_THREADS - 1 (the count
// includes the caller; default 8); a crew runs one loop at a time, and concurrent sessions (one per GPU of a node, or
// several what-if sessions) each take a free crew — a new one is started on demand up to CCMI_SYNC_CREWS (default 8);
// a caller that finds every crew busy runs its loop alone. A helper runs each job on the CPU mask of the job's caller
// (CpuMask::follow): the crews belong to no session's NUMA node.
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
    static HostPool* p = new HostPool();  // never destroyed: helpers stay parked on their crews' condition variables
    return *p;
  }
  int threads() const { return threads_; }
  // f(i) for every i in [0, n), on the caller and a crew's helpers; returns when all are done
  void parallelFor(int n, const std::function<void(int)>& f) {
    if (n <= 0) return;
    Crew* c = threads_ > 1 && n > 1 ? acquire() : nullptr;
    if (!c) {
      for (int i = 0; i < n; ++i) f(i);
      return;
    }
    auto job = std::make_shared<Job>(n, f);
    job->mask = CpuMask::current();  // the helpers run this job on the caller's CPUs
    {
      std::lock_guard<std::mutex> l(c->mu);
      c->job = job;
      ++c->gen;
    }
    c->cv.notify_all();
    run(*job);
    while (job->done.load(std::memory_order_acquire) < n) _mm_pause();
    {
      std::lock_guard<std::mutex> l(c->mu);
      if (c->job == job) c->job.reset();
    }
    release(c);
  }

 private:
  struct Job {
    Job(int n_, const std::function<void(int)>& f_) : n(n_), f(f_) {}
    const int n;
    std::function<void(int)> f;
    CpuMask mask;
    std::atomic<int> next{0}, done{0};
  };
  struct Crew {  // threads_ - 1 helpers sharing one job slot
    std::mutex mu;
    std::condition_variable cv;
    std::shared_ptr<Job> job;
    uint64_t gen = 0;
    bool busy = false;  // guarded by HostPool::crewMu_
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
    const char* c = std::getenv("CCMI_SYNC_CREWS");
    maxCrews_ = c ? std::max(1, std::atoi(c)) : 8;
  }
  Crew* acquire() {
    std::lock_guard<std::mutex> l(crewMu_);
    for (auto& c : crews_)
      if (!c->busy) {
        c->busy = true;
        return c.get();
      }
    if ((int)crews_.size() >= maxCrews_) return nullptr;
    crews_.push_back(std::unique_ptr<Crew>(new Crew()));  // never destroyed: its helpers hold its address
    Crew* c = crews_.back().get();
    c->busy = true;
    for (int t = 1; t < threads_; ++t) std::thread([this, c] { loop(c); }).detach();
    return c;
  }
  void release(Crew* c) {
    std::lock_guard<std::mutex> l(crewMu_);
    c->busy = false;
  }
  void loop(Crew* c) {
    pthread_setname_np(pthread_self(), "ccmi-sync");
    uint64_t seen = 0;
    CpuMask mine = CpuMask::current();
    for (;;) {
      std::shared_ptr<Job> j;
      {
        std::unique_lock<std::mutex> l(c->mu);
        c->cv.wait(l, [&] { return c->gen != seen; });
        seen = c->gen;
        j = c->job;
      }
      if (j) {
        mine.follow(j->mask);
        run(*j);
      }
    }
  }
  int threads_ = 1, maxCrews_ = 8;
  std::mutex crewMu_;
  std::vector<std::unique_ptr<Crew>> crews_;  // guarded by crewMu_
};

}  // namespace ccmi
