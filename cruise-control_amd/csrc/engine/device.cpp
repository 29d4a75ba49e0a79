// Device tables, staging and launch protocol (see device.h).
#include "device.h"

#include <hip/hip_runtime.h>

#include <cstring>
#include <stdexcept>

namespace ccmi {

#define ST ((hipStream_t)st_)
#define EV0 ((hipEvent_t)ev0_)
#define EV1 ((hipEvent_t)ev1_)

hipError_t launchScanCross(const DevTables& T, const DevProgram& prog, const int32_t* reps, const int32_t* cands, int K,
                           int N, unsigned long long* result, hipStream_t st);
hipError_t launchScanSwap(const DevTables& T, const DevProgram& prog, const int32_t* srcs, int S, const int32_t* cbOff,
                          const int32_t* cbRep, int M, unsigned long long* result, int32_t* rowVisited, hipStream_t st,
                          hipEvent_t ev0, hipEvent_t ev1);
hipError_t launchScanPairs(const DevTables& T, const DevProgram& prog, const int32_t* pr, const int32_t* pb, int n,
                           unsigned long long* result, hipStream_t st);
hipError_t launchApplyRows(double* bUtil, int32_t* bNrep, int32_t* bNlead, double* bPot, uint8_t* bAlive, int B,
                           const BrokerRow* brows, int nb, double* rUtil, int32_t* rBroker, uint8_t* rFlags, int R,
                           const ReplicaRow* rrows, int nr, const int32_t* pOff, int32_t* pBrokers,
                           const PartitionRow* prows, int np, int32_t* topicCount, int ldB, const TopicCountDelta* tdel,
                           int nt, hipStream_t st);
hipError_t launchStats(const StatsParams& P, const int32_t* tc, const int32_t* topicNrep, const double* bUtil,
                       const double* bCap, const int32_t* bNrep, const int32_t* bNlead, const double* bPot,
                       const uint8_t* bAlive, const uint8_t* allowedAlive, TopicPartial* scratch, StatsOut* out,
                       int ldB, hipStream_t st, hipEvent_t evTopic0, hipEvent_t evTopic1);

static void hipCheck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error in ") + what + ": " + hipGetErrorString(e));
}

template <class T>
static void dalloc(T** p, size_t n) {
  hipCheck(hipMalloc((void**)p, (n ? n : 1) * sizeof(T)), "hipMalloc");
}

static size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

Device::Device(int ordinal, int B, int R, int P, int T, int maxGoalSlots)
    : ordinal_(ordinal), B_(B), R_(R), P_(P), T_(T), ldB_((B + 3) & ~3), G_(maxGoalSlots) {
  int n = 0;
  hipCheck(hipGetDeviceCount(&n), "hipGetDeviceCount");
  if (ordinal < 0 || ordinal >= n) throw std::runtime_error("no HIP device with ordinal " + std::to_string(ordinal));
  hipCheck(hipSetDevice(ordinal), "hipSetDevice");
  hipDeviceProp_t prop;
  hipCheck(hipGetDeviceProperties(&prop, ordinal), "hipGetDeviceProperties");
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    throw std::runtime_error(std::string("libccmi is built for gfx950, device is ") + prop.gcnArchName);
  hipCheck(hipStreamCreateWithFlags((hipStream_t*)&st_, hipStreamNonBlocking), "hipStreamCreate");
  dalloc(&bUtil_, (size_t)4 * B);
  dalloc(&bCap_, (size_t)4 * B);
  dalloc(&bPot_, B);
  dalloc(&bNrep_, B);
  dalloc(&bNlead_, B);
  dalloc(&bAlive_, B);
  dalloc(&allowed_, (size_t)G_ * B);
  dalloc(&allowedAlive_, ldB_);
  dalloc(&rUtil_, (size_t)4 * R);
  dalloc(&rPart_, R);
  dalloc(&rBroker_, R);
  dalloc(&rOrig_, R);
  dalloc(&rFlags_, R);
  dalloc(&pOff_, (size_t)P + 1);
  dalloc(&pBrokers_, R);
  dalloc(&topicCount_, (size_t)T * ldB_);
  dalloc(&topicNrep_, T);
  hipCheck(hipMalloc(&topicScratch_, (size_t)(T ? T : 1) * sizeof(TopicPartial)), "hipMalloc");
  hipCheck(hipMalloc(&statsOut_, 1024), "hipMalloc");
  hipCheck(hipMemset(allowed_, 0, (size_t)G_ * B), "hipMemset");
  hipCheck(hipHostMalloc((void**)&hResult_, 1024, hipHostMallocDefault), "hipHostMalloc");
  ensureStage(1 << 20);
  hipCheck(hipEventCreate((hipEvent_t*)&ev0_), "hipEventCreate");
  hipCheck(hipEventCreate((hipEvent_t*)&ev1_), "hipEventCreate");
}

Device::~Device() {
  (void)hipSetDevice(ordinal_);
  if (ST) (void)hipStreamSynchronize(ST);
  void* ps[] = {bUtil_, bCap_, bPot_, bNrep_, bNlead_, bAlive_, allowed_, allowedAlive_, rUtil_, rPart_, rBroker_,
                rOrig_, rFlags_, pOff_, pBrokers_, topicCount_, topicNrep_, topicScratch_, statsOut_, dStage_,
                rowVisited_};
  for (void* p : ps)
    if (p) (void)hipFree(p);
  if (hStage_) (void)hipHostFree(hStage_);
  if (hResult_) (void)hipHostFree(hResult_);
  if (ev0_) (void)hipEventDestroy(EV0);
  if (ev1_) (void)hipEventDestroy(EV1);
  if (ST) (void)hipStreamDestroy(ST);
}

void Device::ensureStage(size_t bytes) {
  if (bytes <= stageCap_) return;
  size_t cap = stageCap_ ? stageCap_ : (1 << 20);
  while (cap < bytes) cap <<= 1;
  if (hStage_) (void)hipHostFree(hStage_);
  if (dStage_) (void)hipFree(dStage_);
  hipCheck(hipHostMalloc((void**)&hStage_, cap, hipHostMallocDefault), "hipHostMalloc stage");
  hipCheck(hipMalloc((void**)&dStage_, cap), "hipMalloc stage");
  stageCap_ = cap;
}

DevTables Device::tables() const {
  DevTables t;
  t.bUtil = bUtil_;
  t.bCap = bCap_;
  t.bNrep = bNrep_;
  t.bAlive = bAlive_;
  t.allowed = allowed_;
  t.rUtil = rUtil_;
  t.rPart = rPart_;
  t.rBroker = rBroker_;
  t.rOrig = rOrig_;
  t.rFlags = rFlags_;
  t.pOff = pOff_;
  t.pBrokers = pBrokers_;
  t.B = B_;
  t.R = R_;
  t.P = P_;
  return t;
}

void Device::uploadStatic(const double* bCapRM, const int32_t* rPart, const int32_t* rOrig, const int32_t* pOff,
                          const int32_t* topicNrep) {
  hipCheck(hipSetDevice(ordinal_), "hipSetDevice");
  hipCheck(hipMemcpy(bCap_, bCapRM, sizeof(double) * 4 * B_, hipMemcpyHostToDevice), "upload bCap");
  hipCheck(hipMemcpy(rPart_, rPart, sizeof(int32_t) * R_, hipMemcpyHostToDevice), "upload rPart");
  hipCheck(hipMemcpy(rOrig_, rOrig, sizeof(int32_t) * R_, hipMemcpyHostToDevice), "upload rOrig");
  hipCheck(hipMemcpy(pOff_, pOff, sizeof(int32_t) * (P_ + 1), hipMemcpyHostToDevice), "upload pOff");
  hipCheck(hipMemcpy(topicNrep_, topicNrep, sizeof(int32_t) * T_, hipMemcpyHostToDevice), "upload topicNrep");
}

void Device::uploadDynamic(const double* bUtilRM, const int32_t* bNrep, const int32_t* bNlead, const double* bPot,
                           const uint8_t* bAlive, const double* rUtilRM, const int32_t* rBroker, const uint8_t* rFlags,
                           const int32_t* pBrokers, const int32_t* topicCountDense) {
  hipCheck(hipSetDevice(ordinal_), "hipSetDevice");
  hipCheck(hipMemcpy(bUtil_, bUtilRM, sizeof(double) * 4 * B_, hipMemcpyHostToDevice), "upload bUtil");
  hipCheck(hipMemcpy(bNrep_, bNrep, sizeof(int32_t) * B_, hipMemcpyHostToDevice), "upload bNrep");
  hipCheck(hipMemcpy(bNlead_, bNlead, sizeof(int32_t) * B_, hipMemcpyHostToDevice), "upload bNlead");
  hipCheck(hipMemcpy(bPot_, bPot, sizeof(double) * B_, hipMemcpyHostToDevice), "upload bPot");
  hipCheck(hipMemcpy(bAlive_, bAlive, B_, hipMemcpyHostToDevice), "upload bAlive");
  hipCheck(hipMemcpy(rUtil_, rUtilRM, sizeof(double) * 4 * R_, hipMemcpyHostToDevice), "upload rUtil");
  hipCheck(hipMemcpy(rBroker_, rBroker, sizeof(int32_t) * R_, hipMemcpyHostToDevice), "upload rBroker");
  hipCheck(hipMemcpy(rFlags_, rFlags, R_, hipMemcpyHostToDevice), "upload rFlags");
  hipCheck(hipMemcpy(pBrokers_, pBrokers, sizeof(int32_t) * R_, hipMemcpyHostToDevice), "upload pBrokers");
  hipCheck(hipMemcpy(topicCount_, topicCountDense, sizeof(int32_t) * (size_t)T_ * ldB_, hipMemcpyHostToDevice),
           "upload topicCount");
}

void Device::setAllowed(int slot, const uint8_t* allowedB) {
  if (slot < 0 || slot >= G_) throw std::runtime_error("goal slot out of range");
  hipCheck(hipMemcpyAsync(allowed_ + (size_t)slot * B_, allowedB, B_, hipMemcpyHostToDevice, ST), "upload allowed");
  hipCheck(hipStreamSynchronize(ST), "sync");
}

size_t Device::updatesBytes() const {
  return align16(brows.size() * sizeof(BrokerRow)) + align16(rrows.size() * sizeof(ReplicaRow)) +
         align16(prows.size() * sizeof(PartitionRow)) + align16(tdeltas.size() * sizeof(TopicCountDelta));
}

size_t Device::packUpdates(size_t off, int& nb, int& nr, int& np, int& nt, size_t& obr, size_t& orr, size_t& opr,
                           size_t& otd) {
  nb = (int)brows.size();
  nr = (int)rrows.size();
  np = (int)prows.size();
  nt = (int)tdeltas.size();
  size_t need = off + align16(nb * sizeof(BrokerRow)) + align16(nr * sizeof(ReplicaRow)) +
                align16(np * sizeof(PartitionRow)) + align16(nt * sizeof(TopicCountDelta));
  ensureStage(need + (1 << 16));
  obr = off;
  std::memcpy(hStage_ + obr, brows.data(), nb * sizeof(BrokerRow));
  orr = obr + align16(nb * sizeof(BrokerRow));
  std::memcpy(hStage_ + orr, rrows.data(), nr * sizeof(ReplicaRow));
  opr = orr + align16(nr * sizeof(ReplicaRow));
  std::memcpy(hStage_ + opr, prows.data(), np * sizeof(PartitionRow));
  otd = opr + align16(np * sizeof(PartitionRow));
  std::memcpy(hStage_ + otd, tdeltas.data(), nt * sizeof(TopicCountDelta));
  brows.clear();
  rrows.clear();
  prows.clear();
  tdeltas.clear();
  return otd + align16(nt * sizeof(TopicCountDelta));
}

void Device::launchApply(int nb, int nr, int np, int nt, size_t obr, size_t orr, size_t opr, size_t otd) {
  if (nb + nr + np + nt == 0) return;
  hipCheck(launchApplyRows(bUtil_, bNrep_, bNlead_, bPot_, bAlive_, B_, (const BrokerRow*)(dStage_ + obr), nb, rUtil_,
                           rBroker_, rFlags_, R_, (const ReplicaRow*)(dStage_ + orr), nr, pOff_, pBrokers_,
                           (const PartitionRow*)(dStage_ + opr), np, topicCount_, ldB_,
                           (const TopicCountDelta*)(dStage_ + otd), nt, ST),
           "apply_rows");
}

void Device::flushOnly() {
  int nb, nr, np, nt;
  size_t obr, orr, opr, otd;
  size_t used = packUpdates(0, nb, nr, np, nt, obr, orr, opr, otd);
  if (nb + nr + np + nt == 0) return;
  hipCheck(hipMemcpyAsync(dStage_, hStage_, used, hipMemcpyHostToDevice, ST), "H2D stage");
  launchApply(nb, nr, np, nt, obr, orr, opr, otd);
  hipCheck(hipStreamSynchronize(ST), "sync");
  perf.syncs++;
}

int64_t Device::finishScan(size_t resultOff, size_t bytes) {
  hipCheck(hipMemcpyAsync(hResult_, dStage_ + resultOff, bytes, hipMemcpyDeviceToHost, ST), "D2H result");
  hipCheck(hipStreamSynchronize(ST), "sync");
  perf.syncs++;
  if (timing) {
    float ms = 0.f;
    hipCheck(hipEventElapsedTime(&ms, EV0, EV1), "hipEventElapsedTime");
    perf.scanKernelMs += ms;
  }
  const unsigned long long v = *hResult_;
  return v == ~0ull ? -1 : (int64_t)v;
}

int64_t Device::scanCross(const DevProgram& prog, const int32_t* reps, int K, const int32_t* cands, int N) {
  if (K <= 0 || N <= 0) return -1;
  if ((uint64_t)K * (uint64_t)N >= (1ull << 31)) throw std::runtime_error("scan too large");
  ensureStage(updatesBytes() + align16((size_t)K * 4) + align16((size_t)N * 4) + 64);
  int nb, nr, np, nt;
  size_t obr, orr, opr, otd;
  size_t off = packUpdates(0, nb, nr, np, nt, obr, orr, opr, otd);
  const size_t oRep = off;
  const size_t oCand = oRep + align16((size_t)K * 4);
  const size_t oRes = oCand + align16((size_t)N * 4);
  const size_t used = oRes + 16;
  std::memcpy(hStage_ + oRep, reps, (size_t)K * 4);
  std::memcpy(hStage_ + oCand, cands, (size_t)N * 4);
  *(unsigned long long*)(hStage_ + oRes) = ~0ull;
  hipCheck(hipMemcpyAsync(dStage_, hStage_, used, hipMemcpyHostToDevice, ST), "H2D stage");
  launchApply(nb, nr, np, nt, obr, orr, opr, otd);
  if (timing) (void)hipEventRecord(EV0, ST);
  hipCheck(launchScanCross(tables(), prog, (const int32_t*)(dStage_ + oRep), (const int32_t*)(dStage_ + oCand), K, N,
                           (unsigned long long*)(dStage_ + oRes), ST),
           "scan_cross");
  if (timing) (void)hipEventRecord(EV1, ST);
  perf.scanLaunches++;
  perf.scanPairs += (int64_t)K * N;
  perf.scanBytes += (int64_t)K * N * kBytesPerCandidate;
  return finishScan(oRes, 8);
}

int64_t Device::scanSwap(const DevProgram& prog, const int32_t* srcs, int S, const int32_t* cbOff, int M,
                         const int32_t* cbRep, int nCand, int64_t* visited) {
  *visited = 0;
  if (S <= 0 || M <= 0 || nCand <= 0) return -1;
  const size_t rows = (size_t)S * M;
  if (rows > rowVisitedCap_) {
    if (rowVisited_) (void)hipFree(rowVisited_);
    rowVisitedCap_ = rows * 2;
    hipCheck(hipMalloc((void**)&rowVisited_, rowVisitedCap_ * sizeof(int32_t)), "hipMalloc rowVisited");
  }
  ensureStage(updatesBytes() + align16((size_t)S * 4) + align16((size_t)(M + 1) * 4) + align16((size_t)nCand * 4) + 64);
  int nb, nr, np, nt;
  size_t obr, orr, opr, otd;
  size_t off = packUpdates(0, nb, nr, np, nt, obr, orr, opr, otd);
  const size_t oSrc = off;
  const size_t oOff = oSrc + align16((size_t)S * 4);
  const size_t oRep = oOff + align16((size_t)(M + 1) * 4);
  const size_t oRes = oRep + align16((size_t)nCand * 4);
  const size_t used = oRes + 16;
  std::memcpy(hStage_ + oSrc, srcs, (size_t)S * 4);
  std::memcpy(hStage_ + oOff, cbOff, (size_t)(M + 1) * 4);
  std::memcpy(hStage_ + oRep, cbRep, (size_t)nCand * 4);
  *(unsigned long long*)(hStage_ + oRes) = ~0ull;
  *(unsigned long long*)(hStage_ + oRes + 8) = 0ull;
  hipCheck(hipMemcpyAsync(dStage_, hStage_, used, hipMemcpyHostToDevice, ST), "H2D stage");
  launchApply(nb, nr, np, nt, obr, orr, opr, otd);
  hipCheck(launchScanSwap(tables(), prog, (const int32_t*)(dStage_ + oSrc), S, (const int32_t*)(dStage_ + oOff),
                          (const int32_t*)(dStage_ + oRep), M, (unsigned long long*)(dStage_ + oRes), rowVisited_, ST,
                          timing ? EV0 : nullptr, timing ? EV1 : nullptr),
           "scan_swap");
  perf.scanLaunches++;
  perf.scanPairs += (int64_t)S * nCand;
  perf.scanBytes += (int64_t)S * nCand * kBytesPerCandidate;
  const int64_t key = finishScan(oRes, 16);
  *visited = (int64_t)hResult_[1];
  return key;
}

int64_t Device::scanPairs(const DevProgram& prog, const int32_t* pr, const int32_t* pb, int n) {
  if (n <= 0) return -1;
  ensureStage(updatesBytes() + 2 * align16((size_t)n * 4) + 64);
  int nb, nr, np, nt;
  size_t obr, orr, opr, otd;
  size_t off = packUpdates(0, nb, nr, np, nt, obr, orr, opr, otd);
  const size_t oR = off;
  const size_t oB = oR + align16((size_t)n * 4);
  const size_t oRes = oB + align16((size_t)n * 4);
  const size_t used = oRes + 16;
  std::memcpy(hStage_ + oR, pr, (size_t)n * 4);
  std::memcpy(hStage_ + oB, pb, (size_t)n * 4);
  *(unsigned long long*)(hStage_ + oRes) = ~0ull;
  hipCheck(hipMemcpyAsync(dStage_, hStage_, used, hipMemcpyHostToDevice, ST), "H2D stage");
  launchApply(nb, nr, np, nt, obr, orr, opr, otd);
  if (timing) (void)hipEventRecord(EV0, ST);
  hipCheck(launchScanPairs(tables(), prog, (const int32_t*)(dStage_ + oR), (const int32_t*)(dStage_ + oB), n,
                           (unsigned long long*)(dStage_ + oRes), ST),
           "scan_pairs");
  if (timing) (void)hipEventRecord(EV1, ST);
  perf.scanLaunches++;
  perf.scanPairs += n;
  perf.scanBytes += (int64_t)n * kBytesPerCandidate;
  return finishScan(oRes, 8);
}

void Device::stats(const StatsParams& P, const uint8_t* allowedAliveHost, StatsOut* out) {
  int nb, nr, np, nt;
  size_t obr, orr, opr, otd;
  size_t used = packUpdates(0, nb, nr, np, nt, obr, orr, opr, otd);
  if (used) hipCheck(hipMemcpyAsync(dStage_, hStage_, used, hipMemcpyHostToDevice, ST), "H2D stage");
  launchApply(nb, nr, np, nt, obr, orr, opr, otd);
  hipCheck(hipMemcpyAsync(allowedAlive_, allowedAliveHost, ldB_, hipMemcpyHostToDevice, ST), "H2D allowedAlive");
  hipCheck(launchStats(P, topicCount_, topicNrep_, bUtil_, bCap_, bNrep_, bNlead_, bPot_, bAlive_, allowedAlive_,
                       (TopicPartial*)topicScratch_, (StatsOut*)statsOut_, ldB_, ST, timing ? EV0 : nullptr,
                       timing ? EV1 : nullptr),
           "stats");
  hipCheck(hipMemcpyAsync(hResult_, statsOut_, sizeof(StatsOut), hipMemcpyDeviceToHost, ST), "D2H stats");
  hipCheck(hipStreamSynchronize(ST), "sync");
  perf.syncs++;
  perf.statsLaunches++;
  perf.statsBytes += (int64_t)T_ * ldB_ * 4 + (int64_t)ldB_ + (int64_t)T_ * 4;
  if (timing) {
    float ms = 0.f;
    hipCheck(hipEventElapsedTime(&ms, EV0, EV1), "hipEventElapsedTime");
    perf.statsKernelMs += ms;
  }
  std::memcpy((void*)out, hResult_, sizeof(StatsOut));
}

}  // namespace ccmi
