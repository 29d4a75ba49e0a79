// Host-side phase profile of the goal drivers (CCMI_PROFILE=1 in the environment prints it per session to
// stderr). Thread-local, so concurrent sessions on different threads do not mix.
#pragma once
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

namespace ccmi {

enum Phase {
  PH_RDG_OUT, PH_RDG_IN, PH_RES_OUT, PH_RES_IN, PH_SWAP, PH_DEV_SCAN, PH_DEV_STATS, PH_RELOCATE, PH_CAND_BUILD,
  PH_SORTED_INIT, PH_UPDATE, PH_PQ_INIT, PH_FLATTEN, PH_TREE_BUILD, PH_ORDER, PH_OTHER_GOALS, PH_SCAN_STAGE, PH_SCAN_WAIT, PH_COUNT
};

struct PhaseProf {
  double ms[PH_COUNT] = {};
  int64_t n[PH_COUNT] = {};
  bool on = std::getenv("CCMI_PROFILE") != nullptr;
  void print(const char* tag) const {
    static const char* names[PH_COUNT] = {"rdg.moveOut", "rdg.moveIn", "res.moveOut", "res.moveIn", "res.swap",
                                          "device.scan", "device.stats", "relocate", "cand.build", "sorted.init",
                                          "goal.update", "pq.init", "flatten", "tree.build", "order.repair",
                                          "other.goals", "scan.stage", "scan.wait"};
    if (!on) return;
    std::fprintf(stderr, "[ccmi profile %s]\n", tag);
    for (int i = 0; i < PH_COUNT; ++i)
      if (n[i]) std::fprintf(stderr, "  %-14s %10.1f ms %10lld calls %8.2f us/call\n", names[i], ms[i], (long long)n[i],
                             1e3 * ms[i] / n[i]);
  }
};

inline PhaseProf& prof() {
  static thread_local PhaseProf p;
  return p;
}

struct PhaseScope {
  int ph;
  bool on;
  std::chrono::steady_clock::time_point t0;
  explicit PhaseScope(int p) : ph(p), on(prof().on) {
    if (on) t0 = std::chrono::steady_clock::now();
  }
  ~PhaseScope() {
    if (!on) return;
    prof().ms[ph] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    prof().n[ph]++;
  }
};

}  // namespace ccmi
