// Device side of a session: HBM tables, a pinned staging ring for row updates and scan requests, and
// the launch/readback protocol of one scan:
//   H2D  one hipMemcpyAsync of [row updates | request arrays | result word = ~0]
//   K4   apply_rows     (only if rows are dirty)
//   K1/5 scan_cross or scan_swap
//   D2H  8-byte result, hipStreamSynchronize
// Everything runs on one HIP stream per session, so HIP events on that stream time the kernels.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "devtypes.h"

namespace ccmi {


// Algorithmic bytes per evaluated candidate: destination-broker record 4x f64 util, 4x f64 capacity,
// f64 potential NW_OUT, f64 leader NW_IN, i32 replica/leader/rack/topic-replica counts = 96 B.
constexpr int64_t kBytesPerCandidate = 96;

struct DevicePerf {
  int64_t scanLaunches = 0;
  int64_t scanPairs = 0;   // device-evaluated candidates (speculation included), pair-space size per launch
  double scanKernelMs = 0;
  int64_t scanBytes = 0;   // algorithmic bytes (96 B per evaluated candidate)
  int64_t statsLaunches = 0;
  double statsKernelMs = 0;
  int64_t statsBytes = 0;
  int64_t syncs = 0;
};

class Device {
 public:
  Device(int ordinal, int B, int R, int P, int T, int maxGoalSlots);
  ~Device();
  Device(const Device&) = delete;
  Device& operator=(const Device&) = delete;

  // initial upload (host arrays in device layout)
  void uploadStatic(const double* bCapRM, const int32_t* rPart, const int32_t* rOrig, const int32_t* pOff,
                    const int32_t* topicNrep);
  void uploadDynamic(const double* bUtilRM, const int32_t* bNrep, const int32_t* bNlead, const double* bPot,
                     const uint8_t* bAlive, const double* rUtilRM, const int32_t* rBroker, const uint8_t* rFlags,
                     const int32_t* pBrokers, const int32_t* topicCountDense /* [T][ldB] */);
  void setAllowed(int slot, const uint8_t* allowedB);

  // pending row updates (flushed with the next launch)
  std::vector<BrokerRow> brows;
  std::vector<ReplicaRow> rrows;
  std::vector<PartitionRow> prows;
  std::vector<TopicCountDelta> tdeltas;

  // returns the winning key or -1
  int64_t scanCross(const DevProgram& prog, const int32_t* reps, int K, const int32_t* cands, int N);
  int64_t scanSwap(const DevProgram& prog, const int32_t* srcs, int S, const int32_t* cbOff, int M,
                   const int32_t* cbRep, int nCand, int64_t* visited);
  int64_t scanPairs(const DevProgram& prog, const int32_t* pr, const int32_t* pb, int n);
  void stats(const StatsParams& P, const uint8_t* allowedAliveHost, StatsOut* out);
  void flushOnly();

  DevicePerf perf;
  bool timing = false;  // record HIP events around kernels (bench/profiling)
  int ldB() const { return ldB_; }

 private:
  int ordinal_, B_, R_, P_, T_, ldB_, G_;
  void* st_ = nullptr;  // hipStream_t
  // tables
  double *bUtil_ = nullptr, *bCap_ = nullptr, *bPot_ = nullptr, *rUtil_ = nullptr;
  int32_t *bNrep_ = nullptr, *bNlead_ = nullptr, *rPart_ = nullptr, *rBroker_ = nullptr, *rOrig_ = nullptr;
  int32_t *pOff_ = nullptr, *pBrokers_ = nullptr, *topicCount_ = nullptr, *topicNrep_ = nullptr;
  uint8_t *bAlive_ = nullptr, *allowed_ = nullptr, *rFlags_ = nullptr, *allowedAlive_ = nullptr;
  void *topicScratch_ = nullptr, *statsOut_ = nullptr;
  // staging
  char* hStage_ = nullptr;
  char* dStage_ = nullptr;
  size_t stageCap_ = 0;
  unsigned long long* hResult_ = nullptr;
  void *ev0_ = nullptr, *ev1_ = nullptr;  // hipEvent_t
  DevTables tables() const;
  size_t updatesBytes() const;
  size_t packUpdates(size_t off, int& nb, int& nr, int& np, int& nt, size_t& obr, size_t& orr, size_t& opr, size_t& otd);
  void ensureStage(size_t bytes);
  void launchApply(int nb, int nr, int np, int nt, size_t obr, size_t orr, size_t opr, size_t otd);
  int64_t finishScan(size_t resultOff, size_t bytes);
  int32_t* rowVisited_ = nullptr;
  size_t rowVisitedCap_ = 0;
};


}  // namespace ccmi
