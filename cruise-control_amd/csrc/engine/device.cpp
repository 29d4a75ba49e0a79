// Device tables, staging and launch protocol (see device.h).
#include "device.h"
#include "prof.h"

#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

#include <sched.h>

namespace ccmi {

#define ST ((hipStream_t)st_)
#define EV0 ((hipEvent_t)ev0_)
#define EV1 ((hipEvent_t)ev1_)

hipError_t launchScanCross(const DevTables& T, const MutTables& M, const UpdateList& U, const DevProgram& prog,
                           const int32_t* reps, const int32_t* cands, int K, int Nr, int N, int c0,
                           unsigned long long* result, unsigned int* done, unsigned long long* mail,
                           unsigned long long seq, hipStream_t st);
hipError_t launchScanSwap(const DevTables& T, const DevProgram& prog, const int32_t* srcs, int S, const int32_t* cbOff,
                          const int32_t* cbRep, int M, unsigned long long* result, int32_t* rowVisited,
                          unsigned long long* mail, unsigned long long seq, hipStream_t st, hipEvent_t ev0,
                          hipEvent_t ev1);
hipError_t launchScanPairs(const DevTables& T, const MutTables& M, const UpdateList& U, const DevProgram& prog,
                           const int32_t* pr, const int32_t* pb, int n, int keyBase, unsigned long long* result,
                           unsigned int* done, unsigned long long* mail, unsigned long long seq, hipStream_t st);
hipError_t launchPrep(const MutTables& M, const UpdateList& U, const int4* req, int4* dReq, int nReq4,
                      unsigned long long* result, unsigned int* done, hipStream_t st);
hipError_t launchChainPairs(const DevTables& T, const ChainTables& C, const DevProgram& prog, const int32_t* pr,
                            const int32_t* pb, const int32_t* next, int n, int maxAccepts, int32_t* log,
                            ChainResultDev* out, hipStream_t st);
hipError_t launchChainRackRows(const DevTables& T, const ChainTables& C, const DevProgram& prog, const int32_t* rows,
                               int n, const int32_t* cands, int N, int32_t* log, ChainResultDev* out, hipStream_t st);
hipError_t launchSyncLoads(const ChainTables& C, const LoadRow* lrows, int nl, const SlotRow* srows, int ns,
                           hipStream_t st);
hipError_t launchStats(const StatsParams& P, const int32_t* tc, const int32_t* topicNrep, const BrokerRec* brokers,
                       const uint8_t* allowedAlive, TopicPartial* scratch, StatsOut* out, int ldB, hipStream_t st,
                       hipEvent_t evTopic0, hipEvent_t evTopic1);

static void hipCheck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error in ") + what + ": " + hipGetErrorString(e));
}

template <class T>
static void dalloc(T** p, size_t n) {
  hipCheck(hipMalloc((void**)p, (n ? n : 1) * sizeof(T)), "hipMalloc");
}

static size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

// HIP's current device is per host thread and starts at 0; a session may run on a thread other than the one that
// created it (the reference's precompute pool, bench.py --requests-per-gpu). Every public entry point that touches
// the device makes the session's ordinal current for its duration and restores the caller's device afterwards.
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int ordinal) {
    hipCheck(hipGetDevice(&prev), "hipGetDevice");
    if (prev != ordinal) hipCheck(hipSetDevice(ordinal), "hipSetDevice");
    else prev = -1;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

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
  dalloc(&brokers_, (size_t)B);
  dalloc(&replicas_, (size_t)R);
  dalloc(&parts_, (size_t)P);
  hBrokers_.assign(B, BrokerRec{});
  hParts_.assign(P, PartitionRec{});
  allowedHost_.assign(B, 0u);
  dalloc(&allowedAlive_, ldB_);
  dalloc(&topicCount_, (size_t)T * ldB_);
  dalloc(&topicNrep_, T);
  dalloc(&tUpper_, T);
  dalloc(&tLower_, T);
  dalloc(&dResult_, 4);
  dalloc(&dDone_, 4);
  hipCheck(hipMalloc(&topicScratch_, (size_t)(T ? T : 1) * sizeof(TopicPartial)), "hipMalloc");
  hipCheck(hipMalloc(&statsOut_, 1024), "hipMalloc");
  hipCheck(hipMemset(dDone_, 0, 4 * sizeof(unsigned int)), "hipMemset");
  hipCheck(hipMemset(dResult_, 0xff, 2 * sizeof(unsigned long long)), "hipMemset");
  // host-coherent (fine-grained) mapped memory: kernels read the staging area and write the mailbox directly
  hipCheck(hipHostMalloc((void**)&hResult_, 1024, hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc");
  hipCheck(hipHostGetDevicePointer((void**)&hResultDev_, hResult_, 0), "hipHostGetDevicePointer");
  std::memset(hResult_, 0, 1024);
  ensureStage(1 << 20);
  ensureReq(1 << 20);
  if (std::getenv("CCMI_STAMPS")) {
    dalloc(&stamps_, 1024 * 8);
    hipCheck(hipMemset(stamps_, 0, 1024 * 8 * sizeof(unsigned long long)), "hipMemset");
  }
  hipCheck(hipEventCreate((hipEvent_t*)&ev0_), "hipEventCreate");
  hipCheck(hipEventCreate((hipEvent_t*)&ev1_), "hipEventCreate");
}

Device::~Device() {
  (void)hipSetDevice(ordinal_);
  if (ST) (void)hipStreamSynchronize(ST);
  if (stamps_) {  // average in-launch phase times of the last 1024 cross/pair scans (workgroup 0)
    std::vector<unsigned long long> h(1024 * 8);
    if (hipMemcpy(h.data(), stamps_, h.size() * 8, hipMemcpyDeviceToHost) == hipSuccess) {
      double acc[5] = {0, 0, 0, 0, 0};
      int n = 0;
      for (int i = 0; i < 1024; ++i) {
        const unsigned long long* t = &h[i * 8];
        if (!t[0] || !t[1] || !t[2] || !t[3] || !t[4] || !t[5] || t[5] < t[0]) continue;
        for (int k = 0; k < 5; ++k) acc[k] += (double)(t[k + 1] - t[k]) * 0.01;  // 100 MHz -> us
        n++;
      }
      if (n)
        std::fprintf(stderr, "[ccmi stamps] %d launches: stage %.2f us, loads+predicate %.2f us, blockMin %.2f us, "
                             "tail %.2f us, publish %.2f us\n",
                     n, acc[0] / n, acc[1] / n, acc[2] / n, acc[3] / n, acc[4] / n);
    }
    (void)hipFree(stamps_);
  }
  void* ps[] = {brokers_, replicas_, parts_, allowedAlive_, topicCount_, topicNrep_, topicScratch_, statsOut_, dReq_,
                rowVisited_, dResult_, dDone_, tUpper_, tLower_, dRLoad_, dBLoad_, dBLnw_, dBPot_, dPOff_, dPSlots_,
                dPLeader_, dChainLog_, dChainOut_};
  for (void* p : ps)
    if (p) (void)hipFree(p);
  if (hStage_) (void)hipHostFree(hStage_);
  if (hResult_) (void)hipHostFree(hResult_);
  if (ev0_) (void)hipEventDestroy(EV0);
  if (ev1_) (void)hipEventDestroy(EV1);
  if (ST) (void)hipStreamDestroy(ST);
}

// Staging is only rewritten after the previous request completed (every request waits for its mailbox), so
// growing it in place is safe.
void Device::ensureStage(size_t bytes) {
  if (bytes <= stageCap_) return;
  size_t cap = stageCap_ ? stageCap_ : (1 << 20);
  while (cap < bytes) cap <<= 1;
  char* fresh = nullptr;
  hipCheck(hipHostMalloc((void**)&fresh, cap, hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc stage");
  if (hStage_) {
    std::memcpy(fresh, hStage_, stageUsed_);
    (void)hipHostFree(hStage_);
  }
  hStage_ = fresh;
  hipCheck(hipHostGetDevicePointer((void**)&hStageDev_, hStage_, 0), "hipHostGetDevicePointer");
  stageCap_ = cap;
}

void Device::ensureReq(size_t bytes) {
  if (bytes <= reqCap_) return;
  size_t cap = reqCap_ ? reqCap_ : (1 << 20);
  while (cap < bytes) cap <<= 1;
  if (dReq_) (void)hipFree(dReq_);
  hipCheck(hipMalloc((void**)&dReq_, cap), "hipMalloc request");
  reqCap_ = cap;
}

DevTables Device::tables() const {
  DevTables t;
  t.brokers = brokers_;
  t.replicas = replicas_;
  t.parts = parts_;
  t.topicCount = topicCount_;
  t.tUpper = tUpper_;
  t.tLower = tLower_;
  t.stamps = stamps_;
  t.B = B_;
  t.R = R_;
  t.P = P_;
  t.ldB = ldB_;
  return t;
}

// Static columns are kept in host copies of the broker / partition records until uploadDynamic packs and
// uploads the whole records (the caller uploads static columns first).
void Device::uploadStatic(const double* bCapRM, const int32_t* rPart, const int32_t* rOrig, const int32_t* pOff,
                          const int32_t* topicNrep, const int32_t* bRack, const int32_t* pTopic) {
  DeviceGuard dg(ordinal_);
  for (int b = 0; b < B_; ++b) {
    BrokerRec& x = hBrokers_[b];
    for (int k = 0; k < 4; ++k) x.cap[k] = bCapRM[(size_t)k * B_ + b];
    x.rack = bRack[b];
  }
  hRPart_.assign(rPart, rPart + R_);
  hROrig_.assign(rOrig, rOrig + R_);
  hPOff_.assign(pOff, pOff + P_ + 1);
  for (int p = 0; p < P_; ++p) {
    hParts_[p].topic = pTopic[p];
    hParts_[p].n = pOff[p + 1] - pOff[p];
  }
  bRackHost_.assign(bRack, bRack + B_);
  hipCheck(hipMemcpy(topicNrep_, topicNrep, sizeof(int32_t) * T_, hipMemcpyHostToDevice), "upload topicNrep");
}

void Device::uploadDynamic(const double* bUtilRM, const int32_t* bNrep, const int32_t* bNlead, const double* bPot,
                           const double* bLeadNwIn, const uint8_t* bAlive, const double* rUtilRM,
                           const int32_t* rBroker, const uint8_t* rFlags, const int32_t* pBrokers,
                           const double* pLeadNwOut, const int32_t* topicCountDense) {
  DeviceGuard dg(ordinal_);
  for (int b = 0; b < B_; ++b) {
    BrokerRec& x = hBrokers_[b];
    for (int k = 0; k < 4; ++k) x.util[k] = bUtilRM[(size_t)k * B_ + b];
    x.nrep = bNrep[b];
    x.nlead = bNlead[b];
    x.pot = bPot[b];
    x.lbi = bLeadNwIn[b];
    x.alive = bAlive[b];
    x.allowedBits = allowedHost_[b];
  }
  std::vector<ReplicaRec> reps(R_);
  for (int r = 0; r < R_; ++r) {
    ReplicaRec& x = reps[r];
    std::memset(&x, 0, sizeof(x));
    for (int k = 0; k < 4; ++k) x.util[k] = rUtilRM[(size_t)k * R_ + r];
    x.broker = rBroker[r];
    x.part = hRPart_[r];
    x.orig = hROrig_[r];
    x.flags = rFlags[r] | (bAlive[hROrig_[r]] ? 0 : RF_ORIG_DEAD);
  }
  for (int p = 0; p < P_; ++p) {
    PartitionRec& x = hParts_[p];
    for (int k = 0; k < kMaxRf; ++k) {
      const bool in = k < x.n;
      x.brokers[k] = in ? pBrokers[hPOff_[p] + k] : -1;
      x.racks[k] = (int16_t)(in ? bRackHost_[x.brokers[k]] : -1);
    }
    x.leadNwOut = pLeadNwOut[p];
  }
  hipCheck(hipMemcpy(brokers_, hBrokers_.data(), sizeof(BrokerRec) * B_, hipMemcpyHostToDevice), "upload brokers");
  hipCheck(hipMemcpy(replicas_, reps.data(), sizeof(ReplicaRec) * R_, hipMemcpyHostToDevice), "upload replicas");
  hipCheck(hipMemcpy(parts_, hParts_.data(), sizeof(PartitionRec) * P_, hipMemcpyHostToDevice), "upload partitions");
  hipCheck(hipMemcpy(topicCount_, topicCountDense, sizeof(int32_t) * (size_t)T_ * ldB_, hipMemcpyHostToDevice),
           "upload topicCount");
  hRPart_.clear();
  hROrig_.clear();
}

void Device::setAllowed(int slot, const uint8_t* allowedB) {
  DeviceGuard dg(ordinal_);
  if (slot < 0 || slot >= G_) throw std::runtime_error("goal slot out of range");
  for (int b = 0; b < B_; ++b)
    allowedHost_[b] = (allowedHost_[b] & ~(1u << slot)) | (allowedB[b] ? (1u << slot) : 0u);
  // strided write of BrokerRec::allowedBits (the rest of every record is left alone)
  hipCheck(hipMemcpy2DAsync(&brokers_[0].allowedBits, sizeof(BrokerRec), allowedHost_.data(), sizeof(uint32_t),
                            sizeof(uint32_t), B_, hipMemcpyHostToDevice, ST),
           "upload allowed");
  hipCheck(hipStreamSynchronize(ST), "sync");
}

void Device::setExclusions(const uint8_t* exclLead, const uint8_t* exclMove) {
  DeviceGuard dg(ordinal_);
  const uint32_t mask = (1u << kExclLeadBit) | (1u << kExclMoveBit);
  for (int b = 0; b < B_; ++b)
    allowedHost_[b] = (allowedHost_[b] & ~mask) | (exclLead[b] ? (1u << kExclLeadBit) : 0u) |
                      (exclMove[b] ? (1u << kExclMoveBit) : 0u);
  hipCheck(hipMemcpy2DAsync(&brokers_[0].allowedBits, sizeof(BrokerRec), allowedHost_.data(), sizeof(uint32_t),
                            sizeof(uint32_t), B_, hipMemcpyHostToDevice, ST),
           "upload exclusions");
  hipCheck(hipStreamSynchronize(ST), "sync");
}

void Device::setTopicLimits(const int32_t* upper, const int32_t* lower) {
  DeviceGuard dg(ordinal_);
  hipCheck(hipMemcpyAsync(tUpper_, upper, sizeof(int32_t) * T_, hipMemcpyHostToDevice, ST), "upload tUpper");
  hipCheck(hipMemcpyAsync(tLower_, lower, sizeof(int32_t) * T_, hipMemcpyHostToDevice, ST), "upload tLower");
  hipCheck(hipStreamSynchronize(ST), "sync");
}

size_t Device::updatesBytes() const {
  return align16(brows.size() * sizeof(BrokerRow)) + align16(rrows.size() * sizeof(ReplicaRow)) +
         align16(prows.size() * sizeof(PartitionRow)) + align16(tdeltas.size() * sizeof(TopicCountDelta));
}

// [broker rows | replica rows | partition rows | topic deltas] at the start of the staging area
Device::Staged Device::packUpdates(size_t extra) {
  Staged g;
  g.nb = (int)brows.size();
  g.nr = (int)rrows.size();
  g.np = (int)prows.size();
  g.nt = (int)tdeltas.size();
  stageUsed_ = 0;
  ensureStage(updatesBytes() + extra + 64);
  g.obr = 0;
  std::memcpy(hStage_ + g.obr, brows.data(), g.nb * sizeof(BrokerRow));
  g.orr = g.obr + align16(g.nb * sizeof(BrokerRow));
  std::memcpy(hStage_ + g.orr, rrows.data(), g.nr * sizeof(ReplicaRow));
  g.opr = g.orr + align16(g.nr * sizeof(ReplicaRow));
  std::memcpy(hStage_ + g.opr, prows.data(), g.np * sizeof(PartitionRow));
  g.otd = g.opr + align16(g.np * sizeof(PartitionRow));
  std::memcpy(hStage_ + g.otd, tdeltas.data(), g.nt * sizeof(TopicCountDelta));
  g.end = g.otd + align16(g.nt * sizeof(TopicCountDelta));
  brows.clear();
  rrows.clear();
  prows.clear();
  tdeltas.clear();
  stageUsed_ = g.end;
  return g;
}

// One `prep` launch: apply the staged rows, copy `reqBytes` of request (staged at g.end) into HBM, and (for a
// scan) reset the result words and the arrival counter.
void Device::launchPrepFor(const Staged& g, size_t reqBytes, bool scan) {
  const int nReq4 = (int)(align16(reqBytes) / 16);
  if (nReq4) ensureReq((size_t)nReq4 * 16);
  hipCheck(launchPrep(mutTables(), stagedList(g), (const int4*)(hStageDev_ + g.end), (int4*)dReq_, nReq4,
                      scan ? dResult_ : nullptr, scan ? dDone_ : nullptr, ST),
           "prep");
}

// Spin on the host-mapped mailbox for `seq`; a stream error (or a stream that drained without publishing)
// is reported instead of spinning forever.
void Device::waitMail(unsigned long long seq) {
  PhaseScope ps(PH_SCAN_WAIT);
  volatile unsigned long long* mail = hResult_;
  const unsigned long long want = seq & 0xffffffffull;
  uint64_t spins = 0;
  while ((__atomic_load_n(&mail[0], __ATOMIC_ACQUIRE) >> 32) != want) {
    if ((++spins & 1023) == 0) {
      const hipError_t q = hipStreamQuery(ST);
      if (q == hipSuccess) {
        if ((__atomic_load_n(&mail[0], __ATOMIC_ACQUIRE) >> 32) == want) break;
        throw std::runtime_error("scan finished without publishing its result");
      }
      if (q != hipErrorNotReady) hipCheck(q, "scan");
    }
    // a scan is ~10-30 us; past ~1 ms of spinning the host core is yielded between polls so concurrent sessions
    // (and the JVM's own threads) get it back
    if (spins > (1u << 16)) sched_yield();
    else __builtin_ia32_pause();
  }
  perf.syncs++;
}

// A shard with nothing to scan still applies its pending row updates so every shard's tables stay identical.
void Device::flushPending() {
  DeviceGuard dg(ordinal_);
  if (!brows.empty() || !rrows.empty() || !prows.empty() || !tdeltas.empty()) flushOnly();
}

void Device::flushOnly() {
  DeviceGuard dg(ordinal_);
  if (brows.empty() && rrows.empty() && prows.empty() && tdeltas.empty()) return;
  const Staged g = packUpdates(0);
  launchPrepFor(g, 0, false);
  hipCheck(hipStreamSynchronize(ST), "sync");
  perf.syncs++;
}

int64_t Device::finishScan() {
  waitMail(seq_);
  if (timing) {
    hipCheck(hipEventSynchronize(EV1), "hipEventSynchronize");
    float ms = 0.f;
    hipCheck(hipEventElapsedTime(&ms, EV0, EV1), "hipEventElapsedTime");
    perf.scanKernelMs += ms;
  }
  const unsigned long long lo = hResult_[0] & 0xffffffffull;  // key + 1, 0 = no winner
  return lo == 0 ? -1 : (int64_t)(lo - 1);
}

// A cross/pair scan is one launch when its update list fits the kernel's LDS overlay and its request is
// small enough to read straight from host memory; otherwise `prep` applies the rows and copies the request
// into HBM first.
// Requests are read by the scan straight from the host-mapped staging area (rows that lose to an earlier winner
// are never read, so copying the request into HBM first would only add a launch and a full PCIe read).
constexpr size_t kDirectRequestBytes = 8 << 20;

UpdateList Device::stagedList(const Staged& g) const { return overlayFor(g); }

UpdateList Device::overlayFor(const Staged& g) const {
  UpdateList u;
  u.brows = (const BrokerRow*)(hStageDev_ + g.obr);
  u.rrows = (const ReplicaRow*)(hStageDev_ + g.orr);
  u.prows = (const PartitionRow*)(hStageDev_ + g.opr);
  u.tdel = (const TopicCountDelta*)(hStageDev_ + g.otd);
  u.nb = g.nb;
  u.nr = g.nr;
  u.np = g.np;
  u.nt = g.nt;
  return u;
}

MutTables Device::mutTables() const {
  return MutTables{brokers_, replicas_, parts_, topicCount_, ldB_};
}

// Returns the request base the scan reads (host-mapped staging or the HBM copy) and the update list it
// applies itself (empty when prep ran).
// Topic-count deltas are atomics applied by workgroup 0 during the launch, so a program that reads topic counts
// always has them applied by `prep` first.
const char* Device::stageScan(const Staged& g, size_t req, bool readsTopicCounts, UpdateList& u) {
  const bool fits = g.nb <= kOverlayRows && g.nr <= kOverlayRows && g.np <= kOverlayRows &&
                    !(readsTopicCounts && g.nt > 0);
  if (fits && req <= kDirectRequestBytes) {
    u = overlayFor(g);
    perf.singleLaunch++;
    return hStageDev_ + g.end;
  }
  launchPrepFor(g, req, false);
  u = UpdateList{nullptr, nullptr, nullptr, nullptr, 0, 0, 0, 0};
  return dReq_;
}

int64_t Device::scanCross(const DevProgram& prog, const int32_t* reps, int K, const int32_t* cands, int N, int c0,
                          int c1) {
  DeviceGuard dg(ordinal_);
  const int Nr = c1 - c0;
  if (K <= 0 || Nr <= 0) {
    flushPending();
    return -1;
  }
  if ((uint64_t)K * (uint64_t)N >= (1ull << 31)) throw std::runtime_error("scan too large");
  const size_t oCand = align16((size_t)K * 4);
  const size_t req = oCand + align16((size_t)Nr * 4);
  UpdateList u;
  const char* base;
  {
    PhaseScope ps(PH_SCAN_STAGE);
    const Staged g = packUpdates(req);
    std::memcpy(hStage_ + g.end, reps, (size_t)K * 4);
    std::memcpy(hStage_ + g.end + oCand, cands + c0, (size_t)Nr * 4);
    base = stageScan(g, req, (prog.needs & NEED_TOPIC) != 0, u);
  }
  ++seq_;
  if (timing) (void)hipEventRecord(EV0, ST);
  hipCheck(launchScanCross(tables(), mutTables(), u, prog, (const int32_t*)base, (const int32_t*)(base + oCand), K, Nr,
                           N, c0, dResult_, dDone_, hResultDev_, seq_, ST),
           "scan_cross");
  if (timing) (void)hipEventRecord(EV1, ST);
  perf.scanLaunches++;
  perf.scanPairs += (int64_t)K * Nr;
  perf.scanBytes += (int64_t)K * Nr * kBytesPerCandidate;
  const int64_t key = finishScan();
  // candidates this launch had to evaluate: every row before the winner's and the winner's row up to the winner
  perf.scanRequired += key < 0 ? (int64_t)K * Nr : (key / N) * Nr + (key % N - c0) + 1;
  return key;
}

int64_t Device::scanSwap(const DevProgram& prog, const int32_t* srcs, int S, const int32_t* cbOff, int M,
                         const int32_t* cbRep, int nCand, int64_t* visited) {
  DeviceGuard dg(ordinal_);
  *visited = 0;
  if (S <= 0 || M <= 0 || nCand <= 0) return -1;
  const size_t rows = (size_t)S * M;
  if (rows > rowVisitedCap_) {
    if (rowVisited_) (void)hipFree(rowVisited_);
    rowVisitedCap_ = rows * 2;
    hipCheck(hipMalloc((void**)&rowVisited_, rowVisitedCap_ * sizeof(int32_t)), "hipMalloc rowVisited");
  }
  const size_t oOff = align16((size_t)S * 4);
  const size_t oRep = oOff + align16((size_t)(M + 1) * 4);
  const size_t req = oRep + align16((size_t)nCand * 4);
  const Staged g = packUpdates(req);
  std::memcpy(hStage_ + g.end, srcs, (size_t)S * 4);
  std::memcpy(hStage_ + g.end + oOff, cbOff, (size_t)(M + 1) * 4);
  std::memcpy(hStage_ + g.end + oRep, cbRep, (size_t)nCand * 4);
  launchPrepFor(g, req, true);
  ++seq_;
  hipCheck(launchScanSwap(tables(), prog, (const int32_t*)dReq_, S, (const int32_t*)(dReq_ + oOff),
                          (const int32_t*)(dReq_ + oRep), M, dResult_, rowVisited_, hResultDev_, seq_, ST,
                          timing ? EV0 : nullptr, timing ? EV1 : nullptr),
           "scan_swap");
  perf.scanLaunches++;
  perf.scanPairs += (int64_t)S * nCand;
  perf.scanBytes += (int64_t)S * nCand * kBytesPerCandidate;
  (void)finishScan();
  const unsigned long long best = hResult_[1];
  *visited = (int64_t)hResult_[2];
  perf.scanRequired += *visited;
  return best == ~0ull ? -1 : (int64_t)best;
}

int64_t Device::scanPairs(const DevProgram& prog, const int32_t* pr, const int32_t* pb, int p0, int p1) {
  DeviceGuard dg(ordinal_);
  const int n = p1 - p0;
  if (n <= 0) {
    flushPending();
    return -1;
  }
  const size_t oB = align16((size_t)n * 4);
  const size_t req = oB + align16((size_t)n * 4);
  const Staged g = packUpdates(req);
  std::memcpy(hStage_ + g.end, pr + p0, (size_t)n * 4);
  std::memcpy(hStage_ + g.end + oB, pb + p0, (size_t)n * 4);
  UpdateList u;
  const char* base = stageScan(g, req, (prog.needs & NEED_TOPIC) != 0, u);
  ++seq_;
  if (timing) (void)hipEventRecord(EV0, ST);
  hipCheck(launchScanPairs(tables(), mutTables(), u, prog, (const int32_t*)base, (const int32_t*)(base + oB), n, p0,
                           dResult_, dDone_, hResultDev_, seq_, ST),
           "scan_pairs");
  if (timing) (void)hipEventRecord(EV1, ST);
  perf.scanLaunches++;
  perf.scanPairs += n;
  perf.scanBytes += (int64_t)n * kBytesPerCandidate;
  const int64_t key = finishScan();
  perf.scanRequired += key < 0 ? (int64_t)n : key - p0 + 1;
  return key;
}

void Device::stats(const StatsParams& P, const uint8_t* allowedAliveHost, StatsOut* out) {
  DeviceGuard dg(ordinal_);
  const size_t req = align16((size_t)ldB_);
  const Staged g = packUpdates(req);
  std::memcpy(hStage_ + g.end, allowedAliveHost, (size_t)ldB_);
  launchPrepFor(g, req, false);
  hipCheck(hipMemcpyAsync(allowedAlive_, dReq_, (size_t)ldB_, hipMemcpyDeviceToDevice, ST), "allowedAlive");
  hipCheck(launchStats(P, topicCount_, topicNrep_, brokers_, allowedAlive_, (TopicPartial*)topicScratch_,
                       (StatsOut*)statsOut_, ldB_, ST, timing ? EV0 : nullptr, timing ? EV1 : nullptr),
           "stats");
  hipCheck(hipMemcpyAsync(statsHost_, statsOut_, sizeof(StatsOut), hipMemcpyDeviceToHost, ST), "D2H stats");
  hipCheck(hipStreamSynchronize(ST), "sync");
  perf.syncs++;
  perf.statsLaunches++;
  perf.statsBytes += (int64_t)T_ * ldB_ * 4 + (int64_t)ldB_ + (int64_t)T_ * 4;
  if (timing) {
    float ms = 0.f;
    hipCheck(hipEventElapsedTime(&ms, EV0, EV1), "hipEventElapsedTime");
    perf.statsKernelMs += ms;
  }
  std::memcpy((void*)out, statsHost_, sizeof(StatsOut));
}

}  // namespace ccmi

namespace ccmi {

// ------------------------------------------------------------------------------------------------ chains
void Device::uploadLoads(int W, const LoadVec* rLoad, const LoadVec* bLoad, const LoadVec* bLnw, const LoadVec* bPot,
                         const int32_t* pSlots, const int32_t* pLeader) {
  DeviceGuard dg(ordinal_);
  W_ = W;
  dalloc(&dRLoad_, (size_t)R_);
  dalloc(&dBLoad_, (size_t)B_);
  dalloc(&dBLnw_, (size_t)B_);
  dalloc(&dBPot_, (size_t)B_);
  dalloc(&dPOff_, (size_t)P_ + 1);
  dalloc(&dPSlots_, (size_t)R_);
  dalloc(&dPLeader_, (size_t)P_);
  dalloc(&dChainOut_, 1);
  hipCheck(hipMemcpy(dRLoad_, rLoad, sizeof(LoadVec) * R_, hipMemcpyHostToDevice), "upload replica loads");
  hipCheck(hipMemcpy(dBLoad_, bLoad, sizeof(LoadVec) * B_, hipMemcpyHostToDevice), "upload broker loads");
  hipCheck(hipMemcpy(dBLnw_, bLnw, sizeof(LoadVec) * B_, hipMemcpyHostToDevice), "upload leadership loads");
  hipCheck(hipMemcpy(dBPot_, bPot, sizeof(LoadVec) * B_, hipMemcpyHostToDevice), "upload potential loads");
  hipCheck(hipMemcpy(dPOff_, hPOff_.data(), sizeof(int32_t) * (P_ + 1), hipMemcpyHostToDevice), "upload pOff");
  hipCheck(hipMemcpy(dPSlots_, pSlots, sizeof(int32_t) * R_, hipMemcpyHostToDevice), "upload pSlots");
  hipCheck(hipMemcpy(dPLeader_, pLeader, sizeof(int32_t) * P_, hipMemcpyHostToDevice), "upload pLeader");
}

ChainTables Device::chainTables() const {
  ChainTables c;
  c.brokers = brokers_;
  c.replicas = replicas_;
  c.parts = parts_;
  c.topicCount = topicCount_;
  c.ldB = ldB_;
  c.W = W_;
  c.rLoad = dRLoad_;
  c.bLoad = dBLoad_;
  c.bLnw = dBLnw_;
  c.bPot = dBPot_;
  c.pOff = dPOff_;
  c.pSlots = dPSlots_;
  c.pLeader = dPLeader_;
  return c;
}

// [row updates | load rows | slot rows | request]; launches sync_loads and prep (rows applied, request copied into
// HBM at dReq_). `fill` writes the request into the staging area.
template <class F>
size_t Device::stageChainCopy(size_t reqBytes, Staged& g, size_t& oReq, F fill) {
  if (!dRLoad_) throw std::runtime_error("device chain state not uploaded");
  const size_t nl = lrows.size(), ns = srows.size();
  const size_t oL = 0, oS = align16(nl * sizeof(LoadRow)), oR = oS + align16(ns * sizeof(SlotRow));
  g = packUpdates(oR + reqBytes);
  std::memcpy(hStage_ + g.end + oL, lrows.data(), nl * sizeof(LoadRow));
  std::memcpy(hStage_ + g.end + oS, srows.data(), ns * sizeof(SlotRow));
  fill(hStage_ + g.end + oR);
  hipCheck(launchSyncLoads(chainTables(), (const LoadRow*)(hStageDev_ + g.end + oL), (int)nl,
                           (const SlotRow*)(hStageDev_ + g.end + oS), (int)ns, ST),
           "sync_loads");
  lrows.clear();
  srows.clear();
  // prep copies [g.end + oR, + reqBytes) into dReq_ when given the request at that offset
  Staged h = g;
  h.end = g.end + oR;
  launchPrepFor(h, reqBytes, false);
  oReq = 0;
  return g.end + oR;
}

Device::ChainResult Device::chainPairs(const DevProgram& prog, const int32_t* pr, const int32_t* pb,
                                       const int32_t* next, int n, int maxAccepts, std::vector<int32_t>& log) {
  DeviceGuard dg(ordinal_);
  ChainResult res;
  log.clear();
  if (n <= 0) {
    flushPending();
    return res;
  }
  const size_t oB = align16((size_t)n * 4), oN = oB + align16((size_t)n * 4), req = oN + align16((size_t)n * 4);
  Staged g;
  size_t oReq = 0;
  const size_t at = stageChainCopy(req, g, oReq, [&](char* base) {
    std::memcpy(base, pr, (size_t)n * 4);
    std::memcpy(base + oB, pb, (size_t)n * 4);
    std::memcpy(base + oN, next, (size_t)n * 4);
  });
  (void)at;
  if ((size_t)n > chainLogCap_) {
    if (dChainLog_) (void)hipFree(dChainLog_);
    chainLogCap_ = (size_t)n * 2;
    dalloc(&dChainLog_, chainLogCap_);
  }
  if (timing) (void)hipEventRecord(EV0, ST);
  hipCheck(launchChainPairs(tables(), chainTables(), prog, (const int32_t*)dReq_, (const int32_t*)(dReq_ + oB),
                            (const int32_t*)(dReq_ + oN), n, maxAccepts, dChainLog_, dChainOut_, ST),
           "chain_pairs");
  if (timing) (void)hipEventRecord(EV1, ST);
  ChainResultDev out;
  hipCheck(hipMemcpyAsync(&out, dChainOut_, sizeof(out), hipMemcpyDeviceToHost, ST), "chain result");
  hipCheck(hipStreamSynchronize(ST), "chain");
  perf.syncs++;
  perf.scanLaunches++;
  perf.chainLaunches++;
  perf.scanPairs += (int64_t)out.visited;
  perf.scanRequired += (int64_t)out.visited;
  if (timing) {
    float ms = 0.f;
    hipCheck(hipEventElapsedTime(&ms, EV0, EV1), "hipEventElapsedTime");
    perf.scanKernelMs += ms;
  }
  res.accepts = (int64_t)out.accepts;
  res.visited = (int64_t)out.visited;
  log.resize((size_t)res.accepts);
  if (res.accepts)
    hipCheck(hipMemcpy(log.data(), dChainLog_, sizeof(int32_t) * res.accepts, hipMemcpyDeviceToHost), "chain log");
  return res;
}

Device::ChainResult Device::chainRackRows(const DevProgram& prog, const int32_t* rows, int n, const int32_t* cands,
                                          int N, std::vector<int32_t>& log) {
  DeviceGuard dg(ordinal_);
  ChainResult res;
  log.clear();
  if (n <= 0) {
    flushPending();
    return res;
  }
  const size_t oC = align16((size_t)n * 4), req = oC + align16((size_t)N * 4);
  Staged g;
  size_t oReq = 0;
  (void)stageChainCopy(req, g, oReq, [&](char* base) {
    std::memcpy(base, rows, (size_t)n * 4);
    std::memcpy(base + oC, cands, (size_t)N * 4);
  });
  if ((size_t)2 * n > chainLogCap_) {
    if (dChainLog_) (void)hipFree(dChainLog_);
    chainLogCap_ = (size_t)4 * n;
    dalloc(&dChainLog_, chainLogCap_);
  }
  if (timing) (void)hipEventRecord(EV0, ST);
  hipCheck(launchChainRackRows(tables(), chainTables(), prog, (const int32_t*)dReq_, n, (const int32_t*)(dReq_ + oC), N,
                               dChainLog_, dChainOut_, ST),
           "chain_rack_rows");
  if (timing) (void)hipEventRecord(EV1, ST);
  ChainResultDev out;
  hipCheck(hipMemcpyAsync(&out, dChainOut_, sizeof(out), hipMemcpyDeviceToHost, ST), "chain result");
  hipCheck(hipStreamSynchronize(ST), "chain");
  perf.syncs++;
  perf.scanLaunches++;
  perf.chainLaunches++;
  if (timing) {
    float ms = 0.f;
    hipCheck(hipEventElapsedTime(&ms, EV0, EV1), "hipEventElapsedTime");
    perf.scanKernelMs += ms;
  }
  res.accepts = (int64_t)out.accepts;
  res.failRow = (int64_t)out.failRow;
  log.resize((size_t)res.accepts * 2);
  if (res.accepts)
    hipCheck(hipMemcpy(log.data(), dChainLog_, sizeof(int32_t) * 2 * res.accepts, hipMemcpyDeviceToHost), "chain log");
  int64_t evaluated = res.failRow ? N : 0;
  for (size_t i = 1; i < log.size(); i += 2) evaluated += log[i] + 1;
  perf.scanPairs += evaluated;
  perf.scanRequired += evaluated;
  return res;
}

}  // namespace ccmi
