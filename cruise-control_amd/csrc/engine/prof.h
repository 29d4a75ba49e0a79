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
  PH_SORTED_INIT, PH_UPDATE, PH_PQ_INIT, PH_FLATTEN, PH_TREE_BUILD, PH_ORDER, PH_OTHER_GOALS, PH_SCAN_STAGE, PH_SCAN_WAIT,
  PH_LEAD_OUT, PH_LEAD_IN, PH_REP_OUT, PH_REP_IN, PH_COUNT
};

struct PhaseProf {
  double ms[PH_COUNT] = {};
  int64_t n[PH_COUNT] = {};
  // device scans attributed to the innermost enclosing driver phase (rdg/res/swap/other goals)
  int driver = -1;
  double scanMs[PH_COUNT] = {};
  int64_t scans[PH_COUNT] = {};
  const int64_t* candCounter = nullptr;  // the engine's reference-equivalent candidate count
  int64_t cands[PH_COUNT] = {};
  int64_t payload[PH_COUNT] = {};  // scan-server command bytes (rows, requests, snapshot uploads) per driver
  void addPayload(int64_t b) {
    if (on && driver >= 0) payload[driver] += b;
  }
  bool on = std::getenv("CCMI_PROFILE") != nullptr;
  // named event counters (diagnostics of the drivers' control flow)
  static constexpr int kCounters = 64;
  const char* counterName[kCounters] = {};
  int64_t counter[kCounters] = {};
  void count(int i, const char* name, int64_t d = 1) {
    if (!on) return;
    counterName[i] = name;
    counter[i] += d;
  }
  void print(const char* tag) const {
    static const char* names[PH_COUNT] = {"rdg.moveOut", "rdg.moveIn", "res.moveOut", "res.moveIn", "res.swap",
                                          "device.scan", "device.stats", "relocate", "cand.build", "sorted.init",
                                          "goal.update", "pq.init", "flatten", "tree.build", "order.repair",
                                          "other.goals", "scan.stage", "scan.wait",
                                          "lrd.leadOut", "lrd.leadIn", "lrd.repOut", "lrd.repIn"};
    if (!on) return;
    std::fprintf(stderr, "[ccmi profile %s]\n", tag);
    for (int i = 0; i < PH_COUNT; ++i)
      if (n[i]) {
        std::fprintf(stderr, "  %-14s %10.1f ms %10lld calls %8.2f us/call", names[i], ms[i], (long long)n[i],
                     1e3 * ms[i] / n[i]);
        if (scans[i])
          std::fprintf(stderr, "   [%lld scans, %.1f ms in scans, %lld candidates, %.1f MB payload]",
                       (long long)scans[i], scanMs[i], (long long)cands[i], payload[i] * 1e-6);
        std::fprintf(stderr, "\n");
      }
    for (int i = 0; i < kCounters; ++i)
      if (counterName[i]) std::fprintf(stderr, "  #%-28s %12lld\n", counterName[i], (long long)counter[i]);
  }
};

inline PhaseProf& prof() {
  static thread_local PhaseProf p;
  return p;
}

// Adds the scope's nanoseconds to named counter i (CCMI_PROFILE only)
struct NsScope {
  int i;
  const char* name;
  bool on;
  std::chrono::steady_clock::time_point t0;
  NsScope(int idx, const char* n) : i(idx), name(n), on(prof().on) {
    if (on) t0 = std::chrono::steady_clock::now();
  }
  ~NsScope() {
    if (on)
      prof().count(i, name,
                   (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0)
                       .count());
  }
};

inline bool isDriverPhase(int p) {
  return p == PH_RDG_OUT || p == PH_RDG_IN || p == PH_RES_OUT || p == PH_RES_IN || p == PH_SWAP || p == PH_OTHER_GOALS ||
         p == PH_LEAD_OUT || p == PH_LEAD_IN || p == PH_REP_OUT || p == PH_REP_IN;
}

struct PhaseScope {
  int ph;
  bool on;
  int prevDriver = -1;
  int64_t c0 = 0;
  std::chrono::steady_clock::time_point t0;
  explicit PhaseScope(int p) : ph(p), on(prof().on) {
    if (!on) return;
    t0 = std::chrono::steady_clock::now();
    if (isDriverPhase(p)) {
      prevDriver = prof().driver;
      prof().driver = p;
      if (prof().candCounter) c0 = *prof().candCounter;
    }
  }
  ~PhaseScope() {
    if (!on) return;
    PhaseProf& P = prof();
    const double dt = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    P.ms[ph] += dt;
    P.n[ph]++;
    if (isDriverPhase(ph)) {
      P.driver = prevDriver;
      if (P.candCounter) P.cands[ph] += *P.candCounter - c0;
    }
    if (ph == PH_DEV_SCAN && P.driver >= 0) {
      P.scans[P.driver]++;
      P.scanMs[P.driver] += dt;
    }
  }
};

}  // namespace ccmi
