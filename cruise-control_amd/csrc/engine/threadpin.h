// The NUMA pin of the thread that drives a session, scoped to ONE API call: the caller's CPU mask is narrowed to the
// CPUs of the GPU's NUMA node on entry and restored on exit, so the library leaves no lasting side effect on a caller's
// thread (a JVM pool thread that later runs unrelated work). Every scan is a round trip through host memory (the command
// through the BAR, the result into a host-mapped mailbox the thread spins on): 20 us from the GPU's socket, 30 us from
// the other one (profiles/r04/numa_ab.txt). Threads the library owns (the sync and tree helpers) take the mask of the
// caller whose job they run (CpuMask::follow), so they never keep another session's pin.
//
//   CCMI_NUMA_PIN=0       never pin
//   CCMI_NUMA_CPULIST=L   use the cpulist L ("0-3,8") instead of the device's PCI local_cpulist (tests)
#pragma once
#include <pthread.h>
#include <sched.h>

#include <cstdlib>
#include <string>

namespace ccmi {

// The device's PCI sysfs local_cpulist (device.cpp; the CPU emulation has none): false when unknown
bool deviceLocalCpuList(int ordinal, std::string& out);

inline bool parseCpuList(const std::string& list, cpu_set_t* set) {
  CPU_ZERO(set);
  size_t i = 0;
  while (i < list.size()) {  // "a-b,c,..."
    char* end = nullptr;
    const long a = std::strtol(list.c_str() + i, &end, 10);
    if (end == list.c_str() + i) return false;
    long b = a;
    i = (size_t)(end - list.c_str());
    if (i < list.size() && list[i] == '-') {
      b = std::strtol(list.c_str() + i + 1, &end, 10);
      i = (size_t)(end - list.c_str());
    }
    for (long c = a; c <= b && c < CPU_SETSIZE; ++c) CPU_SET((int)c, set);
    if (i < list.size() && list[i] == ',') ++i;
    else break;
  }
  return CPU_COUNT(set) > 0;
}

// A thread's CPU mask, for helper threads that follow the thread they work for: a pool helper takes the mask of the
// caller whose job it runs (so a session's helpers run on its GPU's node while the call is pinned, and on the caller's
// own mask otherwise), instead of keeping the mask of whichever call created it.
struct CpuMask {
  cpu_set_t set;
  bool valid = false;
  static CpuMask current() {
    CpuMask m;
    m.valid = pthread_getaffinity_np(pthread_self(), sizeof(m.set), &m.set) == 0;
    return m;
  }
  // make this thread's mask `want` (no syscall when it already is)
  void follow(const CpuMask& want) {
    if (!want.valid || (valid && CPU_EQUAL(&set, &want.set))) return;
    if (pthread_setaffinity_np(pthread_self(), sizeof(want.set), &want.set) == 0) *this = want;
  }
};

class ThreadPin {
 public:
  explicit ThreadPin(int ordinal) {
    const char* e = std::getenv("CCMI_NUMA_PIN");
    if (e && e[0] == '0') return;
    std::string list;
    const char* forced = std::getenv("CCMI_NUMA_CPULIST");
    if (forced) list = forced;
    else if (!deviceLocalCpuList(ordinal, list)) return;
    cpu_set_t local, both;
    if (!parseCpuList(list, &local)) return;
    if (pthread_getaffinity_np(pthread_self(), sizeof(prev_), &prev_) != 0) return;
    CPU_AND(&both, &prev_, &local);
    // the caller pinned the thread elsewhere on purpose (empty intersection), or it is local already
    if (CPU_COUNT(&both) == 0 || CPU_EQUAL(&both, &prev_)) return;
    set_ = pthread_setaffinity_np(pthread_self(), sizeof(both), &both) == 0;
  }
  ~ThreadPin() {
    if (set_) (void)pthread_setaffinity_np(pthread_self(), sizeof(prev_), &prev_);
  }
  ThreadPin(const ThreadPin&) = delete;
  ThreadPin& operator=(const ThreadPin&) = delete;

 private:
  bool set_ = false;
  cpu_set_t prev_;
};

}  // namespace ccmi
