// TEST INFRASTRUCTURE ONLY — never linked into libccmi.so.
//
// A sequential host implementation of ccmi::Device (cruise-control_amd/csrc/engine/device.h) used to build
// tests/emu/libccmi_emu.so, so the engine's host driver logic (batching, speculation/un-polling, winner
// decoding, resumption) can be parity-checked against the CPU oracle on machines without a GPU. It
// evaluates the same predicates.h conjunctions as the gfx950 kernels, pair by pair in reference order.
// The product library always uses the HIP implementation (device.cpp) and fails loudly without a gfx950.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <vector>

#include "apply.h"
#include "device.h"
#include "intra.h"
#include "predicates.h"
#include "rackrows.h"
#include "threadpin.h"
#include "shard_rccl.h"

namespace ccmi {

// No RCCL in the emulation: sharded emulation sessions use ccmi_session_set_shard with a test combiner.
struct RcclShard {};
bool rcclUniqueId(uint8_t*) { return false; }
RcclShard* rcclCreate(int, int, int, const uint8_t*) { throw std::runtime_error("RCCL device error: emulation build"); }
void rcclDestroy(RcclShard*) {}
int rcclMin(void*, int64_t*) { return 1; }

namespace {
struct Emu {
  int B, R, P, T, ldB, G;
  std::vector<double> bUtil, bCap, bPot, rUtil, bLeadNwIn, pLeadNwOut;
  std::vector<double> hUtil, hCap;  // [B][3] host values of each broker (empty: every host holds one broker)
  std::vector<int32_t> bNrep, bNlead, rPart, rBroker, rOrig, pOff, pBrokers, topicCount, topicNrep;
  std::vector<int32_t> bRack, pTopic, tUpper, tLower, bSet, rSet;
  std::vector<int32_t> pIneligOff, pIneligB;  // Partition._ineligibleBrokers (empty: none)
  std::vector<int32_t> topicLead, tMinLead;   // Broker.numLeadersFor counts (empty: not kept), MinTopicLeaders minima
  std::vector<int32_t> tLeadLim;              // TopicLeaderReplicaDistributionGoal (upper, lower) per topic
  std::vector<uint8_t> bAlive, rFlags;
  std::vector<uint32_t> allowed;
  // chain state (device.h uploadLoads)
  int W = 1;
  std::vector<LoadVec> lRep, lBrk, lLnw, lPot;
  std::vector<LoadVec> lHost;  // Host._load (brokers sharing hosts; empty otherwise)
  std::vector<int32_t> bHostOf, hOffE, hBrkE;
  std::vector<int32_t> pSlots, pLeader;
  // disk state (device.h uploadDisks)
  int D = 0;
  std::vector<int32_t> bDiskOff, bDisks, rOrigDisk, rTie;
  std::vector<double> dCap, dUtilIn, dUtil, rDu, upper, lower;
  std::vector<uint8_t> dAlive, dbAlive;
  std::vector<float> rScore;
  std::vector<int32_t> hist;
};
struct View {
  const Emu& e;
  double bu(int b, int res) const { return e.bUtil[(size_t)res * e.B + b]; }
  double bcap(int b, int res) const { return e.bCap[(size_t)res * e.B + b]; }
  bool hostMode() const { return !e.hCap.empty(); }
  double hu(int b, int res) const { return e.hCap.empty() ? bu(b, res) : e.hUtil[3 * (size_t)b + res]; }
  double hcap(int b, int res) const { return e.hCap.empty() ? bcap(b, res) : e.hCap[3 * (size_t)b + res]; }
  int nrep(int b) const { return e.bNrep[b]; }
  bool alive(int b) const { return e.bAlive[b] != 0; }
  bool allowed(int slot, int b) const { return (e.allowed[b] >> slot) & 1u; }
  double ru(int r, int res) const { return e.rUtil[(size_t)res * e.R + r]; }
  int flags(int r) const { return e.rFlags[r]; }
  int rbroker(int r) const { return e.rBroker[r]; }
  int rorig(int r) const { return e.rOrig[r]; }
  bool origOff(int r) const { return (e.rFlags[r] & RF_ORIG_OFFLINE) || !alive(e.rOrig[r]); }
  int rpart(int r) const { return e.rPart[r]; }
  int pbegin(int p) const { return e.pOff[p]; }
  int pend(int p) const { return e.pOff[p + 1]; }
  int pbroker(int i) const { return e.pBrokers[i]; }
  bool hosts(int p, int b) const {
    bool has = false;
    for (int i = pbegin(p); i < pend(p); ++i) has |= (pbroker(i) == b);
    return has;
  }
  int rack(int b) const { return e.bRack[b]; }
  bool ineligible(int p, int b) const {
    if (e.pIneligOff.empty()) return false;
    for (int k = e.pIneligOff[p]; k < e.pIneligOff[p + 1]; ++k)
      if (e.pIneligB[k] == b) return true;
    return false;
  }
  bool otherOnRack(int p, int self, int rk) const {
    for (int i = pbegin(p); i < pend(p); ++i)
      if (pbroker(i) != self && e.bRack[pbroker(i)] == rk) return true;
    return false;
  }
  int slotRack(int, int b) const { return e.bRack[b]; }
  int rackCount(int p, int rk) const {
    int c = 0;
    for (int i = pbegin(p); i < pend(p); ++i) c += e.bRack[pbroker(i)] == rk ? 1 : 0;
    return c;
  }
  int nlead(int b) const { return e.bNlead[b]; }
  double pot(int b) const { return e.bPot[b]; }
  double lnwin(int b) const { return e.bLeadNwIn[b]; }
  double pLeadNwOut(int p) const { return e.pLeadNwOut[p]; }
  int ptopic(int p) const { return e.pTopic[p]; }
  int tcount(int t, int b) const { return e.topicCount[(size_t)t * e.ldB + b]; }
  int tUpper(int t) const { return e.tUpper[t]; }
  int tLower(int t) const { return e.tLower[t]; }
  int bset(int b) const { return e.bSet.empty() ? -1 : e.bSet[b]; }
  int rbset(int r) const { return e.rSet.empty() ? -1 : e.rSet[r]; }
  int tlead(int t, int b) const { return e.topicLead.at((size_t)t * e.ldB + b); }
  int tMinLead(int t) const { return e.tMinLead.empty() ? -1 : e.tMinLead[t]; }
  int tLeadUpper(int t) const { return e.tLeadLim.at(2 * (size_t)t); }
  int tLeadLower(int t) const { return e.tLeadLim.at(2 * (size_t)t + 1); }
  // RackAwareGoal.rackAwareEligibleBrokers membership for (replica r, destination d)
  bool rackEligible(int r, int d) const {
    std::vector<int> racks;
    for (int i = pbegin(rpart(r)); i < pend(rpart(r)); ++i) racks.push_back(e.bRack[pbroker(i)]);
    for (size_t i = 0; i < racks.size(); ++i)
      if (racks[i] == e.bRack[rbroker(r)]) {
        racks.erase(racks.begin() + i);
        break;
      }
    for (int x : racks)
      if (x == e.bRack[d]) return false;
    return true;
  }
};
Emu& E(void* st) { return *static_cast<Emu*>(st); }
}  // namespace

int Device::countGfx950() {  // one emulated device, or CCMI_EMU_DEVICES (tests of the multi-device host paths)
  const char* e = std::getenv("CCMI_EMU_DEVICES");
  return e ? std::max(1, std::atoi(e)) : 1;
}
bool deviceLocalCpuList(int, std::string&) { return false; }  // no PCI device

Device::Device(int ordinal, int B, int R, int P, int T, int maxGoalSlots)
    : ordinal_(ordinal), B_(B), R_(R), P_(P), T_(T), ldB_((B + 3) & ~3), G_(maxGoalSlots) {
  auto* e = new Emu();
  e->B = B;
  e->R = R;
  e->P = P;
  e->T = T;
  e->ldB = ldB_;
  e->G = maxGoalSlots;
  e->allowed.assign(B, 0u);
  st_ = e;
}
Device::~Device() { delete static_cast<Emu*>(st_); }

void Device::collectServerBusy() {}  // no scan server in the emulator

void Device::uploadIneligible(const int32_t* off, const int32_t* brokers, int n) {
  if (n <= 0) return;
  Emu& e = E(st_);
  e.pIneligOff.assign(off, off + P_ + 1);
  e.pIneligB.assign(brokers, brokers + n);
}
void Device::uploadStatic(const double* bCapRM, const int32_t* rPart, const int32_t* rOrig, const int32_t* pOff,
                          const int32_t* topicNrep, const int32_t* bRack, const int32_t* pTopic) {
  Emu& e = E(st_);
  e.bRack.assign(bRack, bRack + B_);
  e.pTopic.assign(pTopic, pTopic + P_);
  e.tUpper.assign(T_, 0);
  e.tLower.assign(T_, 0);
  e.bCap.assign(bCapRM, bCapRM + 4 * (size_t)B_);
  e.rPart.assign(rPart, rPart + R_);
  e.rOrig.assign(rOrig, rOrig + R_);
  e.pOff.assign(pOff, pOff + P_ + 1);
  e.topicNrep.assign(topicNrep, topicNrep + T_);
}
void Device::uploadDynamic(const double* bUtilRM, const int32_t* bNrep, const int32_t* bNlead, const double* bPot,
                           const double* bLeadNwIn, const uint8_t* bAlive, const double* rUtilRM,
                           const int32_t* rBroker, const uint8_t* rFlags, const int32_t* pBrokers,
                           const double* pLeadNwOut, const int32_t* tc) {
  Emu& e = E(st_);
  e.bLeadNwIn.assign(bLeadNwIn, bLeadNwIn + B_);
  e.pLeadNwOut.assign(pLeadNwOut, pLeadNwOut + P_);
  e.bUtil.assign(bUtilRM, bUtilRM + 4 * (size_t)B_);
  e.bNrep.assign(bNrep, bNrep + B_);
  e.bNlead.assign(bNlead, bNlead + B_);
  e.bPot.assign(bPot, bPot + B_);
  e.bAlive.assign(bAlive, bAlive + B_);
  e.rUtil.assign(rUtilRM, rUtilRM + 4 * (size_t)R_);
  e.rBroker.assign(rBroker, rBroker + R_);
  e.rFlags.assign(rFlags, rFlags + R_);
  e.pBrokers.assign(pBrokers, pBrokers + R_);
  e.topicCount.assign(tc, tc + (size_t)T_ * ldB_);
}
void Device::setAllowed(int slot, const uint8_t* a) {
  auto& al = E(st_).allowed;
  for (int b = 0; b < B_; ++b) al[b] = (al[b] & ~(1u << slot)) | (a[b] ? (1u << slot) : 0u);
}
void Device::setExclusions(const uint8_t* lead, const uint8_t* move, const uint8_t* isNew) {
  Emu& e = E(st_);
  const uint32_t mask = (1u << kExclLeadBit) | (1u << kExclMoveBit) | (1u << kNewBit);
  for (int b = 0; b < e.B; ++b)
    e.allowed[b] = (e.allowed[b] & ~mask) | (lead[b] ? (1u << kExclLeadBit) : 0u) |
                   (move[b] ? (1u << kExclMoveBit) : 0u) | (isNew[b] ? (1u << kNewBit) : 0u);
}
void Device::setTopicLimits(const int32_t* upper, const int32_t* lower) {
  E(st_).tUpper.assign(upper, upper + T_);
  E(st_).tLower.assign(lower, lower + T_);
}

void Device::enableTopicLeaders(const int32_t* dense) {
  E(st_).topicLead.assign(dense, dense + (size_t)T_ * ldB_);
}
void Device::setMinLeaders(const int32_t* tMin) { E(st_).tMinLead.assign(tMin, tMin + T_); }
void Device::setTopicLeadLimits(const int32_t* lim) { E(st_).tLeadLim.assign(lim, lim + 2 * (size_t)T_); }

void Device::setBrokerSets(const int32_t* brokerSet, const int32_t* replicaSet) {
  E(st_).bSet.assign(brokerSet, brokerSet + B_);
  E(st_).rSet.assign(replicaSet, replicaSet + R_);
}

void Device::uploadHosts(const double* hutil, const double* hcap) {
  Emu& e = E(st_);
  e.hUtil.assign(hutil, hutil + 3 * (size_t)B_);
  e.hCap.assign(hcap, hcap + 3 * (size_t)B_);
}

void Device::flushPending() { flushOnly(); }

void Device::flushOnly() {
  Emu& e = E(st_);
  for (const BrokerRow& x : brows) {
    for (int k = 0; k < 4; ++k) e.bUtil[(size_t)k * B_ + x.b] = x.util[k];
    e.bNrep[x.b] = x.nrep;
    e.bNlead[x.b] = x.nlead;
    e.bPot[x.b] = x.potNwOut;
    e.bLeadNwIn[x.b] = x.leadNwIn;
    e.bAlive[x.b] = (uint8_t)x.alive;
    if (!e.hCap.empty())
      for (int k = 0; k < 3; ++k) e.hUtil[3 * (size_t)x.b + k] = x.hutil[k];
  }
  for (const ReplicaRow& x : rrows) {
    for (int k = 0; k < 4; ++k) e.rUtil[(size_t)k * R_ + x.r] = x.util[k];
    e.rBroker[x.r] = x.broker;
    e.rFlags[x.r] = (uint8_t)x.flags;
  }
  for (const PartitionRow& x : prows) {
    for (int k = 0; k < x.n; ++k) e.pBrokers[e.pOff[x.p] + k] = x.brokers[k];
    e.pLeadNwOut[x.p] = x.leadNwOut;
  }
  for (const TopicCountDelta& d : tdeltas) (d.kind ? e.topicLead : e.topicCount).at((size_t)d.topic * ldB_ + d.broker) += d.delta;
  brows.clear();
  rrows.clear();
  prows.clear();
  tdeltas.clear();
}

// The engine's speculative host work, run where a real scan would be in flight: to completion, or for at most
// CCMI_EMU_IDLE_CALLS calls (tests: a partly done speculation the engine must finish itself)
static void runIdleWork(const std::function<bool()>& w) {
  if (!w) return;
  const char* e = std::getenv("CCMI_EMU_IDLE_CALLS");
  const long cap = e ? std::atol(e) : -1;
  for (long n = 0; (cap < 0 || n < cap) && w(); ++n) {
  }
}

int64_t Device::scanCross(const DevProgram& prog, const int32_t* reps, int K, const int32_t* cands, int N, int c0,
                          int c1) {
  runIdleWork(idleWork);
  flushOnly();
  View v{E(st_)};
  perf.scanLaunches++;
  perf.scanPairs += (int64_t)K * (c1 - c0);
  for (int k = 0; k < K; ++k)
    for (int j = c0; j < c1; ++j) {
      if (prog.filter == FILTER_RACK_AWARE && !v.rackEligible(reps[k], cands[j])) continue;
      if (candidateBlocked(prog, v, reps[k], cands[j])) continue;
      if (moveCandidateAccepted(prog, v, reps[k], cands[j])) return (int64_t)k * N + j;
    }
  return -1;
}

int64_t Device::scanPairs(const DevProgram& prog, const int32_t* pr, const int32_t* pb, int p0, int p1) {
  runIdleWork(idleWork);
  flushOnly();
  View v{E(st_)};
  perf.scanLaunches++;
  perf.scanPairs += p1 - p0;
  for (int q = p0; q < p1; ++q) {
    if (candidateBlocked(prog, v, pr[q], pb[q])) continue;
    if (moveCandidateAccepted(prog, v, pr[q], pb[q])) return q;
  }
  return -1;
}

int64_t Device::scanSwap(const DevProgram& prog, const int32_t* srcs, int S, const int32_t* cbOff, int M,
                         const int32_t* cbRep, int nCand, const SwapLimit& lim, int64_t* visited) {
  flushOnly();
  View v{E(st_)};
  perf.scanLaunches++;
  perf.scanPairs += (int64_t)S * nCand;
  *visited = 0;
  for (int m = 0; m < M; ++m)
    for (int s = 0; s < S; ++s) {
      const int c0 = cbOff[m], c1 = cbOff[m + 1];
      if (c0 == c1) continue;
      const int db = E(st_).rBroker[cbRep[c0]];
      if (swapRowExcluded(prog, v, srcs[s], db)) continue;
      for (int j = c0; j < c1; ++j) {
        if (lim.res >= 0) {  // the scan_swap limit filter: rows failing it are no candidates
          const double u = v.ru(cbRep[j], lim.res);
          if (!(lim.above ? u > lim.limit : u < lim.limit)) continue;
        }
        const int o = swapCandidateOutcome(prog, v, srcs[s], cbRep[j], db);
        (*visited)++;
        if (o == 1) return ((int64_t)((int64_t)m * S + s) << 24) | (j - c0);
        if (o == 2) break;
      }
    }
  return -1;
}

// ------------------------------------------------------------------------------------------------ chains
// The chain kernels' decisions, one candidate at a time, with apply.h on record mirrors of the emulated tables.
namespace {
struct EmuApply {
  Emu& e;
  int W;
  std::vector<BrokerRec> brokers;
  std::vector<ReplicaRec> replicas;
  std::vector<PartitionRec> parts;
  explicit EmuApply(Emu& em) : e(em), W(em.W) {
    brokers.assign(e.B, BrokerRec{});
    for (int b = 0; b < e.B; ++b) {
      BrokerRec& x = brokers[b];
      for (int k = 0; k < 4; ++k) {
        x.util[k] = e.bUtil[(size_t)k * e.B + b];
        x.cap[k] = e.bCap[(size_t)k * e.B + b];
      }
      x.pot = e.bPot[b];
      x.lbi = e.bLeadNwIn[b];
      x.nrep = e.bNrep[b];
      x.nlead = e.bNlead[b];
      x.rack = e.bRack[b];
      x.allowedBits = e.allowed[b];
      x.alive = e.bAlive[b];
      for (int k = 0; k < 3; ++k) x.hutil[k] = e.hUtil.empty() ? x.util[k] : e.hUtil[3 * (size_t)b + k];
    }
    replicas.assign(e.R, ReplicaRec{});
    for (int r = 0; r < e.R; ++r) {
      ReplicaRec& x = replicas[r];
      for (int k = 0; k < 4; ++k) x.util[k] = e.rUtil[(size_t)k * e.R + r];
      x.broker = e.rBroker[r];
      x.part = e.rPart[r];
      x.orig = e.rOrig[r];
      x.flags = e.rFlags[r];
    }
    parts.assign(e.P, PartitionRec{});
    for (int p = 0; p < e.P; ++p) {
      PartitionRec& x = parts[p];
      x.n = e.pOff[p + 1] - e.pOff[p];
      x.topic = e.pTopic[p];
      for (int k = 0; k < kMaxRf; ++k) {
        x.brokers[k] = k < x.n ? e.pBrokers[e.pOff[p] + k] : -1;
        x.racks[k] = (int16_t)(k < x.n ? e.bRack[x.brokers[k]] : -1);
      }
      x.leadNwOut = e.pLeadNwOut[p];
    }
  }
  LoadVec sc[2];
  LoadVec& scratch(int i) { return sc[i]; }
  LoadVec& rLoad(int r) { return e.lRep[r]; }
  LoadVec& bLoad(int b) { return e.lBrk[b]; }
  LoadVec& bLnw(int b) { return e.lLnw[b]; }
  LoadVec& bPot(int b) { return e.lPot[b]; }
  bool hostsOn() const { return !e.lHost.empty(); }
  int host(int b) const { return e.bHostOf[b]; }
  LoadVec& hLoad(int h) { return e.lHost[h]; }
  int hostBegin(int h) const { return e.hOffE[h]; }
  int hostEnd(int h) const { return e.hOffE[h + 1]; }
  int hostBroker(int i) const { return e.hBrkE[i]; }
  ReplicaRec& rep(int r) { return replicas[r]; }
  BrokerRec& brk(int b) { return brokers[b]; }
  PartitionRec& part(int p) { return parts[p]; }
  int& slot(int p, int i) { return e.pSlots[e.pOff[p] + i]; }
  int& leader(int p) { return e.pLeader[p]; }
  void topicAdd(int t, int b, int d) { e.topicCount[(size_t)t * e.ldB + b] += d; }
  void topicLeadAdd(int t, int b, int d) {
    if (!e.topicLead.empty()) e.topicLead[(size_t)t * e.ldB + b] += d;
  }
  // the records a move touched, back into the emulated columns the predicates read
  void writeBroker(int b) {
    const BrokerRec& x = brokers[b];
    for (int k = 0; k < 4; ++k) e.bUtil[(size_t)k * e.B + b] = x.util[k];
    e.bPot[b] = x.pot;
    e.bLeadNwIn[b] = x.lbi;
    e.bNrep[b] = x.nrep;
    e.bNlead[b] = x.nlead;
    if (hostsOn())  // the host utilization of every broker of b's host (applyHostUtil wrote them all)
      for (int i = hostBegin(host(b)); i < hostEnd(host(b)); ++i) {
        const int y = hostBroker(i);
        for (int k = 0; k < 3; ++k) e.hUtil[3 * (size_t)y + k] = brokers[y].hutil[k];
      }
  }
  void writeReplica(int r) {
    const ReplicaRec& x = replicas[r];
    for (int k = 0; k < 4; ++k) e.rUtil[(size_t)k * e.R + r] = x.util[k];
    e.rBroker[r] = x.broker;
    e.rFlags[r] = (uint8_t)x.flags;
  }
  void writePartition(int p) {
    const PartitionRec& x = parts[p];
    for (int k = 0; k < x.n; ++k) e.pBrokers[e.pOff[p] + k] = x.brokers[k];
    e.pLeadNwOut[p] = x.leadNwOut;
  }
  void moveReplica(int r, int dst) {
    const int src = replicas[r].broker, p = replicas[r].part;
    applyRelocateReplica(*this, r, dst);
    writeBroker(src);
    writeBroker(dst);
    writeReplica(r);
    writePartition(p);
  }
  void moveLeadership(int p, int src, int dst) {
    std::vector<int> reps;
    for (int i = 0; i < parts[p].n; ++i) reps.push_back(slot(p, i));
    applyRelocateLeadership(*this, p, src, dst);
    writeBroker(src);
    writeBroker(dst);
    for (int r : reps) writeReplica(r);
    writePartition(p);
  }
};
}  // namespace

void Device::uploadHostLoads(int H, const LoadVec* hLoad, const int32_t* bHost, const int32_t* hOff,
                             const int32_t* hBrk) {
  Emu& e = E(st_);
  e.lHost.assign(hLoad, hLoad + H);
  e.bHostOf.assign(bHost, bHost + B_);
  e.hOffE.assign(hOff, hOff + H + 1);
  e.hBrkE.assign(hBrk, hBrk + hOff[H]);
}

void Device::uploadLoads(int W, const LoadVec* rLoad, const LoadVec* bLoad, const LoadVec* bLnw, const LoadVec* bPot,
                         const int32_t* pSlots, const int32_t* pLeader) {
  Emu& e = E(st_);
  e.W = W;
  e.lRep.assign(rLoad, rLoad + R_);
  e.lBrk.assign(bLoad, bLoad + B_);
  e.lLnw.assign(bLnw, bLnw + B_);
  e.lPot.assign(bPot, bPot + B_);
  e.pSlots.assign(pSlots, pSlots + R_);
  e.pLeader.assign(pLeader, pLeader + P_);
}

static void emuSyncLoads(Emu& e, std::vector<LoadRow>& lrows, std::vector<SlotRow>& srows) {
  for (const LoadRow& x : lrows) {
    std::vector<LoadVec>& v = x.kind == LR_REPLICA ? e.lRep
                              : (x.kind == LR_BROKER       ? e.lBrk
                                 : (x.kind == LR_LEADERSHIP_NW ? e.lLnw : (x.kind == LR_HOST ? e.lHost : e.lPot)));
    v[x.id] = x.v;
  }
  for (const SlotRow& x : srows) {
    for (int k = 0; k < e.pOff[x.p + 1] - e.pOff[x.p]; ++k) e.pSlots[e.pOff[x.p] + k] = x.slots[k];
    e.pLeader[x.p] = x.leader;
  }
  lrows.clear();
  srows.clear();
}

Device::ChainResult Device::chainPairs(const DevProgram& prog, const int32_t* pr, const int32_t* pb, const int32_t* next,
                                       int n, int maxAccepts, std::vector<int32_t>& log) {
  flushOnly();
  Emu& e = E(st_);
  emuSyncLoads(e, lrows, srows);
  ChainResult res;
  log.clear();
  if (n <= 0) return res;
  perf.scanLaunches++;
  perf.chainLaunches++;
  EmuApply A(e);
  View v{e};
  int start = 0;
  while (start < n && res.accepts < maxAccepts) {
    int best = -1;
    for (int q = start; q < n && best < 0; ++q) {
      if (candidateBlocked(prog, v, pr[q], pb[q])) continue;
      if (moveCandidateAccepted(prog, v, pr[q], pb[q])) best = q;
    }
    if (best < 0) {
      res.visited += n - start;
      break;
    }
    res.visited += best - start + 1;
    log.push_back(best);
    res.accepts++;
    if (prog.action == DA_LEADERSHIP) A.moveLeadership(e.rPart[pr[best]], e.rBroker[pr[best]], pb[best]);
    else A.moveReplica(pr[best], pb[best]);
    start = next[best];
  }
  perf.scanPairs += res.visited;
  return res;
}

namespace {
struct EmuRackView {  // rackrows.h view over the emulated tables
  const Emu& e;
  int rack(int b) const { return e.bRack[b]; }
  bool alive(int b) const { return e.bAlive[b] != 0; }
  uint32_t bits(int b) const { return e.allowed[b]; }
  int flags(int r) const { return e.rFlags[r] | (e.bAlive[e.rOrig[r]] ? 0 : RF_ORIG_DEAD); }
  int rorig(int r) const { return e.rOrig[r]; }
  int rbroker(int r) const { return e.rBroker[r]; }
  int rpart(int r) const { return e.rPart[r]; }
  int pn(int p) const { return e.pOff[p + 1] - e.pOff[p]; }
  int pbroker(int p, int i) const { return e.pBrokers[e.pOff[p] + i]; }
  bool ineligible(int p, int b) const { return View{e}.ineligible(p, b); }
};
}  // namespace

int64_t Device::rackRowsGroups(const DevProgram& prog, const int32_t* rows, int n, const int32_t* order,
                               const int32_t* gOff, int G, const int32_t* cands, int N, int32_t* res) {
  flushOnly();
  if (n <= 0 || G <= 0) return 0;
  Emu& e = E(st_);
  perf.scanLaunches++;
  int64_t evaluated = 0;
  for (int g = 0; g < G; ++g)
    evaluated += rackRowsGroup(EmuRackView{e}, prog, rows, order, gOff[g], gOff[g + 1], cands, N, res);
  perf.scanPairs += evaluated;
  return evaluated;
}

Device::ChainResult Device::chainRackRows(const DevProgram& prog, const int32_t* rows, int n, const int32_t* cands,
                                          int N, std::vector<int32_t>& log) {
  flushOnly();
  Emu& e = E(st_);
  emuSyncLoads(e, lrows, srows);
  ChainResult res;
  log.clear();
  if (n <= 0) return res;
  perf.scanLaunches++;
  perf.chainLaunches++;
  EmuApply A(e);
  View v{e};
  for (int k = 0; k < n; ++k) {
    const int r = rows[k], src = e.rBroker[r];
    const bool keep = !v.otherOnRack(e.rPart[r], src, e.bRack[src]);
    if (v.alive(src) && !currentOffline(v, r) && keep) continue;
    int best = -1;
    for (int j = 0; j < N && best < 0; ++j) {
      if (!v.rackEligible(r, cands[j])) continue;
      if (candidateBlocked(prog, v, r, cands[j])) continue;
      if (moveCandidateAccepted(prog, v, r, cands[j])) best = j;
    }
    if (best < 0) {
      res.failRow = k + 1;
      break;
    }
    log.push_back(k);
    log.push_back(best);
    res.accepts++;
    A.moveReplica(r, cands[best]);
  }
  return res;
}

void Device::stats(const StatsParams& P, const uint8_t* aa, StatsOut* out) {
  flushOnly();
  Emu& e = E(st_);
  perf.statsLaunches++;
  const int B = P.B, na = P.numAllowed;
  std::memset(out, 0, sizeof(*out));
  for (int res = 0; res < 4; ++res) {
    double hot = 0, cold = 1.7976931348623157e308, var = 0;
    int bal = 0;
    const bool host = res < 3 && !e.hCap.empty();  // ClusterModelStats.java:297-303
    for (int b = 0; b < B; ++b) {
      if (!e.bAlive[b]) continue;
      const double u = host ? e.hUtil[3 * (size_t)b + res] : e.bUtil[(size_t)res * B + b];
      hot = u > hot ? u : hot;
      cold = u < cold ? u : cold;
      if (aa[b]) {
        const double cap = host ? e.hCap[3 * (size_t)b + res] : e.bCap[(size_t)res * B + b];
        const double pct = u / cap;
        if (pct >= P.lowerThr[res] && pct <= P.upperThr[res]) bal++;
        const double d = u - P.avgPct[res] * cap;
        var += d * d;
      }
    }
    out->numBalanced[res] = bal;
    out->resAvg[res] = P.clusterUtil[res] / na;
    out->resMax[res] = hot;
    out->resMin[res] = cold;
    out->resStd[res] = std::sqrt(var / na);
  }
  {
    const double s = P.potSum;
    const double avgPct = s / P.potCapacity;
    double hot = 0, cold = 1.7976931348623157e308, var = 0;
    int under = 0;
    for (int b = 0; b < B; ++b) {
      if (!e.bAlive[b]) continue;
      const double u = e.bPot[b], cap = e.bCap[(size_t)2 * B + b];
      hot = u > hot ? u : hot;
      cold = u < cold ? u : cold;
      if (aa[b]) {
        if (u / cap <= P.nwOutCapThreshold) under++;
        const double d = u - avgPct * cap;
        var += d * d;
      }
    }
    out->pnwAvg = s / na;
    out->pnwMax = hot;
    out->pnwMin = cold;
    out->pnwStd = std::sqrt(var / na);
    out->numUnderPot = under;
  }
  for (int which = 0; which < 2; ++which) {
    const std::vector<int32_t>& cnt = which == 0 ? e.bNrep : e.bNlead;
    const int64_t total = which == 0 ? P.repTotal : P.leadTotal;
    int mx = 0, mn = 0x7fffffff;
    for (int b = 0; b < B; ++b) {
      mx = cnt[b] > mx ? cnt[b] : mx;
      mn = cnt[b] < mn ? cnt[b] : mn;
    }
    const double avg = (double)total / na;
    double var = 0;
    for (int b = 0; b < B; ++b)
      if (e.bAlive[b] && aa[b]) {
        const double d = (double)cnt[b] - avg;
        var += (d * d) / na;
      }
    if (which == 0) {
      out->repAvg = avg;
      out->repStd = std::sqrt(var);
      out->repMax = mx;
      out->repMin = mn;
    } else {
      out->leadAvg = avg;
      out->leadStd = std::sqrt(var);
      out->leadMax = mx;
      out->leadMin = mn;
    }
  }
  double avgSum = 0, sdSum = 0;
  int tmx = 0, tmn = 0x7fffffff;
  for (int t = 0; t < P.T; ++t) {
    const double avg = (double)e.topicNrep[t] / na;
    double var = 0;
    int mx = 0, mn = 0x7fffffff;
    for (int b = 0; b < B; ++b) {
      const int n = e.topicCount[(size_t)t * ldB_ + b];
      mx = n > mx ? n : mx;
      mn = n < mn ? n : mn;
      if (aa[b]) {
        const double d = n - avg;
        var += (d * d) / na;
      }
    }
    avgSum += avg;
    sdSum += std::sqrt(var);
    tmx = mx > tmx ? mx : tmx;
    tmn = mn < tmn ? mn : tmn;
  }
  out->topicAvg = avgSum / P.T;
  out->topicStd = sdSum / P.T;
  out->topicMax = tmx;
  out->topicMin = tmn;
}

// ------------------------------------------------------------------------------------------------ K6 (sequential)
void Device::uploadDisks(int D, const int32_t* bDiskOff, const int32_t* bDisks, const double* dCap,
                         const uint8_t* dAlive, const uint8_t* bAlive, const int32_t* rOrigDisk, const double* rDu,
                         const float* rScore, const int32_t* rTie) {
  Emu& e = E(st_);
  e.D = D;
  e.bDiskOff.assign(bDiskOff, bDiskOff + B_ + 1);
  e.bDisks.assign(bDisks, bDisks + D);
  e.dCap.assign(dCap, dCap + D);
  e.dAlive.assign(dAlive, dAlive + D);
  e.dbAlive.assign(bAlive, bAlive + B_);
  e.rOrigDisk.assign(rOrigDisk, rOrigDisk + R_);
  e.rDu.assign(rDu, rDu + R_);
  e.rScore.assign(rScore, rScore + R_);
  e.rTie.assign(rTie, rTie + R_);
  e.dUtilIn.assign(D, 0.0);
  e.dUtil.assign(D, 0.0);
  e.upper.assign((size_t)G_ * B_, 0.0);
  e.lower.assign((size_t)G_ * B_, 0.0);
  e.hist.assign((size_t)B_ * kIntraHist * (kIntraMaxDisks + 1), 0);
}

void Device::setDiskUtil(const double* dUtil) {
  Emu& e = E(st_);
  e.dUtilIn.assign(dUtil, dUtil + e.D);
}

void Device::intraRun(const IntraRequest& q, IntraResult& out) {
  Emu& e = E(st_);
  const int E_ = q.eOff[B_];
  std::vector<int32_t> eDisk(q.eDisk, q.eDisk + E_), snapA(E_ + 1), snapB(E_ + 1), ordRev(E_ + 1), ordFwd(E_ + 1);
  std::vector<int64_t> logOff(B_, 0);
  std::vector<int32_t> cap(B_, 0);
  int64_t total = 0;
  for (int i = 0; i < q.nBrokers; ++i) {  // the bound of a broker's program (device.cpp re-runs with it)
    const int b = q.brokers[i];
    logOff[b] = total;
    cap[b] = (int32_t)(6 * (e.bDiskOff[b + 1] - e.bDiskOff[b] + 1) * (q.eOff[b + 1] - q.eOff[b]) + 64);
    total += cap[b];
  }
  std::vector<int32_t> rep(total + 1), src(total + 1), dst(total + 1);
  out.count.assign(B_, 0);
  out.status.assign(B_, 0);
  out.cand.assign(B_, 0);
  IntraArgs A{};
  A.goal = q.goal;
  A.capThr = q.capThr;
  A.margin = q.margin;
  A.nPrior = q.nPrior;
  for (int k = 0; k < q.nPrior; ++k) {
    A.prior[k].kind = q.priorKind[k];
    A.prior[k].upper = e.upper.data() + (size_t)q.priorSlot[k] * B_;
    A.prior[k].lower = e.lower.data() + (size_t)q.priorSlot[k] * B_;
  }
  A.brokers = q.brokers;
  A.nBrokers = q.nBrokers;
  A.bDiskOff = e.bDiskOff.data();
  A.bDisks = e.bDisks.data();
  A.dCap = e.dCap.data();
  A.dAlive = e.dAlive.data();
  A.dUtilIn = e.dUtilIn.data();
  A.dUtil = e.dUtil.data();
  A.eOff = q.eOff;
  A.eRep = q.eRep;
  A.eDiskIn = q.eDisk;
  A.eDisk = eDisk.data();
  A.rDu = e.rDu.data();
  A.rScore = e.rScore.data();
  A.rTie = e.rTie.data();
  A.rOrigDisk = e.rOrigDisk.data();
  A.rSel = q.rSel;
  A.snapA = snapA.data();
  A.snapB = snapB.data();
  A.ordRev = ordRev.data();
  A.ordFwd = ordFwd.data();
  std::vector<int32_t> nSel(B_, 0);
  A.nSel = nSel.data();
  std::vector<double> eDu(E_ + 1);  // intra_sort's entry-indexed gathers
  std::vector<int32_t> eOrig(E_ + 1);
  for (int k = 0; k < E_; ++k) {
    eDu[k] = e.rDu[q.eRep[k]];
    eOrig[k] = e.rOrigDisk[q.eRep[k]];
  }
  A.eDu = eDu.data();
  A.eOrig = eOrig.data();
  for (int i = 0; i < q.nBrokers; ++i) {  // kernels/intra.hip intra_sort: selected entries by their unique keys
    const int b = q.brokers[i];
    for (int pass = 0; pass < 2; ++pass) {
      std::vector<std::pair<uint64_t, int32_t>> keyed;
      for (int k = q.eOff[b]; k < q.eOff[b + 1]; ++k) {
        const int r = q.eRep[k];
        if (q.rSel[r]) keyed.push_back({intraSortKey(e.rScore[r], e.rTie[r], pass == 0), k});
      }
      std::sort(keyed.begin(), keyed.end());
      int32_t* ord = (pass == 0 ? ordRev.data() : ordFwd.data()) + q.eOff[b];
      for (size_t k = 0; k < keyed.size(); ++k) ord[k] = keyed[k].second;
      nSel[b] = (int)keyed.size();
    }
  }
  A.hist = e.hist.data();
  A.upperOut = e.upper.data() + (size_t)q.slot * B_;
  A.lowerOut = e.lower.data() + (size_t)q.slot * B_;
  A.logOff = logOff.data();
  A.logCap = cap.data();
  A.logRep = rep.data();
  A.logSrc = src.data();
  A.logDst = dst.data();
  A.logCount = out.count.data();
  A.status = out.status.data();
  A.cand = out.cand.data();
  for (int i = 0; i < q.nBrokers; ++i) {
    IntraBroker ib(A, q.brokers[i]);
    ib.run();
  }
  perf.intraLaunches++;
  out.off.assign(B_ + 1, 0);
  for (int b = 0; b < B_; ++b) out.off[b + 1] = out.off[b] + out.count[b];
  out.rep.resize(out.off[B_]);
  out.src.resize(out.off[B_]);
  out.dst.resize(out.off[B_]);
  for (int b = 0; b < B_; ++b)
    for (int k = 0; k < out.count[b]; ++k) {
      out.rep[out.off[b] + k] = rep[logOff[b] + k];
      out.src[out.off[b] + k] = src[logOff[b] + k];
      out.dst[out.off[b] + k] = dst[logOff[b] + k];
    }
  if (q.goal == IG_USAGE) {
    out.upper.assign(e.upper.begin() + (size_t)q.slot * B_, e.upper.begin() + (size_t)(q.slot + 1) * B_);
    out.lower.assign(e.lower.begin() + (size_t)q.slot * B_, e.lower.begin() + (size_t)(q.slot + 1) * B_);
  }
}

void Device::statsDisks(double balance, DiskStatsOut* out) {
  Emu& e = E(st_);
  double var = 0;
  int unb = 0, na = 0;
  for (int b = 0; b < B_; ++b) {
    if (!e.dbAlive[b]) continue;
    double cap = 0, util = 0;
    for (int k = e.bDiskOff[b]; k < e.bDiskOff[b + 1]; ++k) {
      const int d = e.bDisks[k];
      if (e.dAlive[d]) {
        cap += e.dCap[d];
        util += e.dUtilIn[d];
      }
    }
    const double avg = cap > 0 ? util / cap : 1.0;
    const double upper = avg * balance, lm = 2 - balance, lower = avg * (lm > 0 ? lm : 0.0);
    for (int k = e.bDiskOff[b]; k < e.bDiskOff[b + 1]; ++k) {
      const int d = e.bDisks[k];
      if (!e.dAlive[d]) continue;
      const double pct = e.dCap[d] > 0 ? e.dUtilIn[d] / e.dCap[d] : 1.0;
      if (pct > upper || pct < lower) unb++;
      var += (pct - avg) * (pct - avg);
      na++;
    }
  }
  out->varSum = var;
  out->unbalanced = unb;
  out->numAlive = na;
}

}  // namespace ccmi

namespace ccmi {
void Device::stopServer() {}  // the emulation has no scan server: every scan is evaluated in place

// Queue scans: the directory is host bookkeeping here (no pool); the rows are evaluated in key order, which is the
// order the server's first fit reports.
bool Device::queueUsable() const { return serverAllowed_; }
void Device::qdirBind(uint64_t key) {
  if (key == qdirKey_ && !qdirSnap_.empty()) return;
  qdirKey_ = key;
  qdirSpan_ = 1;
  qdirSnap_.assign(B_, nullptr);
}
void Device::limitServerBlocks(int) {}
void Device::callBegin() {}
void Device::callEnd() {}

// Shard groups: the emulation has no scan server, so every combine is the host side of the protocol (shard_group.h).
CombineBlock* Device::allocCombineBlock() {
  auto* b = new CombineBlock();
  initCombineBlock(b);
  return b;
}
void Device::freeCombineBlock(CombineBlock* b) { delete b; }
void Device::attachGroup(CombineBlock* blk, int count, int rank) {
  grpHost_ = blk;
  grpDev_ = 0;
  grpCount_ = count;
  grpRank_ = rank;
  grpCalls_ = 0;
  grpHostSeq_ = 0;
  devCombined_ = false;
  groupMail_.assign(8, 0ull);
  __atomic_store_n(&blk->mail[rank], (unsigned long long)(uintptr_t)groupMail_.data(), __ATOMIC_RELEASE);
}
int64_t Device::groupCombineHost(int64_t key) {
  const int slot = (int)(grpCalls_ & 1);
  ++grpCalls_;
  return groupHostMin(grpHost_, slot, grpRank_, grpCount_, key, ++grpHostSeq_, 120.0);
}

bool Device::qdirSetMany(const std::vector<int32_t>& bs,
                         const std::vector<std::shared_ptr<const std::vector<int32_t>>>& snaps) {
  // CCMI_SNAPSHOT_POOL_ROWS: the pool the real directory lives in, in rows of whole 128-byte lines: a directory whose
  // snapshots do not fit it together is refused, as Device::qdirSetMany refuses it
  if (const char* pr = std::getenv("CCMI_SNAPSHOT_POOL_ROWS")) {
    const size_t cap = (size_t)std::max(1024ll, std::atoll(pr)) & ~(size_t)7;
    std::vector<size_t> len(B_, 0);
    for (int b = 0; b < B_; ++b) len[b] = qdirSnap_[b] ? qdirSnap_[b]->size() : 0;
    for (size_t i = 0; i < bs.size(); ++i) len[bs[i]] = snaps[i]->size();
    size_t need = 0;
    for (size_t n : len) need += (n + 7) & ~(size_t)7;
    if (need > cap) return false;
  }
  for (size_t i = 0; i < bs.size(); ++i)
    if (!qdirSet(bs[i], snaps[i])) return false;
  return true;
}

bool Device::qdirSet(int b, std::shared_ptr<const std::vector<int32_t>> v) {
  if (qdirSnap_.empty() || b < 0 || b >= B_) throw std::logic_error("qdirSet before qdirBind");
  for (int r : *v)
    if (rowBroker_ && rowBroker_[r] != b) throw std::logic_error("snapshot segment is not current for its broker");
  qdirSpan_ = std::max(qdirSpan_, (int)v->size());
  qdirSnap_[b] = std::move(v);
  return true;
}
int64_t Device::scanQueue(const DevProgram& prog, int head, int skip0, const int32_t* tail, int nTail,
                          const int32_t* cands, int N) {
  runIdleWork(idleWork);
  flushOnly();
  View v{E(st_)};
  perf.scanLaunches++;
  const int span = qdirSpan_, hasHead = head >= 0 ? 1 : 0;
  for (int i = 0; i < hasHead + nTail; ++i) {
    const auto& rows = *qdirSnap_.at(i < hasHead ? head : tail[i - hasHead]);
    for (size_t r = i == 0 ? (size_t)skip0 : 0; r < rows.size(); ++r)
      for (int j = 0; j < N; ++j) {
        perf.scanPairs++;
        if (candidateBlocked(prog, v, rows[r], cands[j])) continue;
        if (moveCandidateAccepted(prog, v, rows[r], cands[j])) return ((int64_t)i * span + (int64_t)r) * N + j;
      }
  }
  return -1;
}

// no snapshot pool either (segsUsable() is false, so the engine flattens first; kept for the link)
int64_t Device::scanSegs(const DevProgram& prog, const std::vector<SegIn>& segs, const int32_t* cands, int N, int c0,
                         int c1) {
  runIdleWork(idleWork);
  segFlat_.clear();
  for (const SegIn& sg : segs)
    if (sg.v->size() > sg.skip) segFlat_.insert(segFlat_.end(), sg.v->begin() + sg.skip, sg.v->end());
  return scanCross(prog, segFlat_.data(), (int)segFlat_.size(), cands, N, c0, c1);
}
}  // namespace ccmi
