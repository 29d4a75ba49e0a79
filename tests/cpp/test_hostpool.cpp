// Unit checks of engine/hostpool.h (built and run by tests/test_hostpool_cpp.py, CPU only): concurrent callers each
// run their loop to completion on a crew of their own (or alone when every crew is busy), every index exactly once,
// and a crew is reused by later loops.
#include <atomic>
#include <cstdio>
#include <thread>
#include <vector>

#include "hostpool.h"

using namespace ccmi;

static std::atomic<int> fails{0};
#define CHECK(c, ...)                    \
  do {                                   \
    if (!(c)) {                          \
      std::fprintf(stderr, __VA_ARGS__); \
      std::fprintf(stderr, "\n");        \
      ++fails;                           \
    }                                    \
  } while (0)

static void loops(int caller, int rounds) {
  HostPool& pool = HostPool::get();
  for (int k = 0; k < rounds; ++k) {
    const int n = 1 + (caller * 7919 + k * 104729) % 5000;
    std::vector<std::atomic<int>> hits(n);
    for (auto& h : hits) h.store(0);
    pool.parallelFor(n, [&](int i) { hits[i].fetch_add(1, std::memory_order_relaxed); });
    for (int i = 0; i < n; ++i) CHECK(hits[i].load() == 1, "caller %d round %d: index %d ran %d times", caller, k, i, hits[i].load());
  }
}

int main() {
  // one caller, then 12 concurrent callers (more than the default 8 crews: some loops run alone)
  loops(0, 50);
  std::vector<std::thread> ts;
  for (int c = 1; c <= 12; ++c) ts.emplace_back(loops, c, 40);
  for (auto& t : ts) t.join();
  if (fails.load()) return 1;
  std::printf("hostpool ok\n");
  return 0;
}
