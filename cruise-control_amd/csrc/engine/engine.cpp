// Engine: goal drivers with device-batched candidate scans (see engine.h for the reference map).
#include "engine.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <thread>

#include "device.h"
#include "predicates.h"
#include "rackrows.h"
#include "prof.h"
#include "threadpin.h"

namespace ccmi {

namespace {

constexpr double kBalanceMargin = 0.9;  // ResourceDistributionGoal.BALANCE_MARGIN / ReplicaDistributionAbstractGoal

// Speculative move-in batches: a scan launch costs about as much as evaluating ~10^4 more rows (the rows of one
// batch are evaluated in one sweep of the resident workgroups and the launch is latency bound), so batches
// start at a few thousand rows and grow fast while nothing is accepted.
// CCMI_FIRST_BATCH / CCMI_BATCH_GROWTH override the first two (tuning diagnostics; results do not depend on them).
size_t envSize(const char* name, size_t dflt) {
  const char* v = std::getenv(name);
  const size_t x = v ? (size_t)std::strtoull(v, nullptr, 10) : 0;
  return x ? x : dflt;
}
size_t envCount(const char* name, size_t dflt) {  // unset: dflt; "0" turns the feature off
  const char* v = std::getenv(name);
  return v ? (size_t)std::strtoull(v, nullptr, 10) : dflt;
}
const size_t kFirstBatchRows = envSize("CCMI_FIRST_BATCH", 2048), kBatchGrowth = envSize("CCMI_BATCH_GROWTH", 8);
// snapshots of upcoming queue polls computed while a move-in scan is in flight (Device::idleWork); 0 = off
const size_t kIdleSnapshots = envCount("CCMI_IDLE_SNAPSHOTS", 8);
// puts of the speculative entry tree per poll of an in-flight move-out scan; 0 = off (read per call: tests vary it)
size_t idleTreePuts() { return envCount("CCMI_IDLE_TREE_PUTS", 64); }
constexpr size_t kMaxBatchRows = (size_t)1 << 18;

// Host view of the model for predicates.h (same expressions the kernels evaluate).
struct HostView {
  const Model& m;
  const std::vector<const std::vector<uint8_t>*>& allowedBySlot;
  const std::vector<int32_t>& tUp;
  const std::vector<int32_t>& tLo;
  const std::vector<int32_t>& bSet;  // BrokerSetAwareGoal: broker set of every broker / replica (empty: none)
  const std::vector<int32_t>& rSet;
  const std::vector<int32_t>& tMin;  // MinTopicLeadersPerBrokerGoal minima (empty: none)
  const std::vector<int32_t>& tLim;  // TopicLeaderReplicaDistributionGoal limits [T][2] (empty: none)
  double bu(int b, int res) const { return m.bu(b, res); }
  double bcap(int b, int res) const { return m.cap(b, res); }
  bool hostMode() const { return m.hostMode(); }
  double hu(int b, int res) const { return m.hu(b, res); }
  double hcap(int b, int res) const { return m.hcap(b, res); }
  int nrep(int b) const { return m.nrep(b); }
  bool alive(int b) const { return m.alive(b); }
  bool allowed(int slot, int b) const { return (*allowedBySlot[slot])[b] != 0; }
  double ru(int r, int res) const { return m.ru(r, res); }
  int flags(int r) const { return (m.rLeader[r] ? RF_LEADER : 0) | (m.rOrigOff[r] ? RF_ORIG_OFFLINE : 0); }
  int rbroker(int r) const { return m.rBroker[r]; }
  int rorig(int r) const { return m.rOrig[r]; }
  bool origOff(int r) const { return m.origOffline(r); }
  int rpart(int r) const { return m.rPart[r]; }
  int pbegin(int p) const { return m.pOff[p]; }
  int pend(int p) const { return m.pOff[p + 1]; }
  int pbroker(int i) const { return m.rBroker[m.pSlots[i]]; }
  bool hosts(int p, int b) const {
    bool has = false;
    for (int i = pbegin(p); i < pend(p); ++i) has |= (pbroker(i) == b);
    return has;
  }
  int rack(int b) const { return m.bRack[b]; }
  bool ineligible(int p, int b) const { return m.ineligible(p, b); }
  bool otherOnRack(int p, int self, int rk) const {
    for (int i = pbegin(p); i < pend(p); ++i)
      if (pbroker(i) != self && m.bRack[pbroker(i)] == rk) return true;
    return false;
  }
  int slotRack(int, int b) const { return m.bRack[b]; }
  int rackCount(int p, int rk) const {
    int c = 0;
    for (int i = pbegin(p); i < pend(p); ++i) c += m.bRack[pbroker(i)] == rk ? 1 : 0;
    return c;
  }
  int nlead(int b) const { return m.bNlead[b]; }
  double pot(int b) const { return m.potNwOut(b); }
  double lnwin(int b) const { return m.leadNwIn(b); }
  double pLeadNwOut(int p) const { return m.pLeadNwOut(p); }
  int ptopic(int p) const { return m.pTopic[p]; }
  int tcount(int t, int b) const { return m.tcount(t, b); }
  int tUpper(int t) const { return tUp[t]; }
  int tLower(int t) const { return tLo[t]; }
  int bset(int b) const { return bSet.empty() ? -1 : bSet[b]; }
  int rbset(int r) const { return rSet.empty() ? -1 : rSet[r]; }
  int tlead(int t, int b) const { return m.tlead(t, b); }
  int tMinLead(int t) const { return tMin.empty() ? -1 : tMin[t]; }
  int tLeadUpper(int t) const { return tLim[2 * t]; }
  int tLeadLower(int t) const { return tLim[2 * t + 1]; }
};

uint32_t needsOf(const DevGoal& g) {
  switch (g.kind) {
    case DG_RACK_AWARE:
    case DG_RACK_AWARE_DISTRIBUTION: return NEED_RACK;
    case DG_POTENTIAL_NW_OUT: return NEED_POT;
    case DG_TOPIC_REPLICA_DISTRIBUTION: return NEED_TOPIC;
    case DG_LEADER_REPLICA_DISTRIBUTION: return NEED_LEAD;
    case DG_LEADER_BYTES_IN: return NEED_LBI;
    case DG_MIN_TOPIC_LEADERS: return NEED_TLEAD;
    case DG_TOPIC_LEADER_DISTRIBUTION: return NEED_TLEAD | NEED_TLLIM;
    default: return 0;
  }
}

}  // namespace

size_t idleTreePutsPerPoll() { return idleTreePuts(); }

std::vector<int> GoalImpl::brokersToBalance(Engine& e) {
  std::vector<int> v(e.m.B);
  for (int b = 0; b < e.m.B; ++b) v[b] = b;
  return v;
}

// GoalUtils.computeResourceUtilizationBalanceThreshold (GoalUtils.java:550-602)
double Engine::threshold(double avgPct, int res, bool lower) const {
  const bool low = avgPct <= bc.lowUtil[res];
  double bp = bc.resBalance[res];
  if (opt.triggered) bp *= bc.goalViolationMultiplier;
  const double margin = (bp - 1) * kBalanceMargin;
  if (lower) return low ? 0.0 : avgPct * jmax(0, (1 - margin));
  const double t = avgPct * (1 + margin);
  return low ? jmax(t, bc.lowUtil[res] * kBalanceMargin) : t;
}

DevProgram Engine::program(const GoalImpl& self, int action) const {
  DevProgram p;
  std::memset(&p, 0, sizeof(p));
  p.action = action;
  // the conjunction of AnalyzerUtils.isProposalAcceptableForOptimizedGoals ends at a terminal goal (it throws)
  size_t nOpt = 0;
  while (nOpt < priors.size() && !(nOpt > 0 && priors[nOpt - 1]->terminal)) ++nOpt;
  p.nGoals = 1 + (int)nOpt;
  if (p.nGoals > kMaxGoals) throw Unsupported("too many goals in one chain");
  p.goals[0] = self.dg;
  for (size_t i = 0; i < nOpt; ++i) p.goals[i + 1] = priors[i]->dg;
  p.needs = 0;
  for (int i = 0; i < p.nGoals; ++i) p.needs |= needsOf(p.goals[i]);
  p.filter = FILTER_NONE;
  // GoalUtils.eligibleBrokers (GoalUtils.java:122-160): without requested destinations a LEADER replica's move
  // skips brokers excluded for leadership — replica-dependent, so it is checked per candidate on the device
  p.exclLeadMove = (opt.anyExclLead && !opt.anyRequested && action == DA_MOVE) ? 1 : 0;
  p.swapExcl = (action == DA_SWAP && (opt.anyExclLead || opt.anyExclMove)) ? 1 : 0;
  // GoalUtils.eligibleBrokers returns before the new-broker filter when destinations are requested (:189-191);
  // eligibleReplicasForSwap has no such return
  p.newOnly = (m.numNew > 0 && (action == DA_SWAP || !opt.anyRequested)) ? 1 : 0;
  return p;
}

// The replica-dependent candidate filters of GoalUtils.eligibleBrokers, as the device applies them
// (predicates.h candidateBlocked): a (replica, destination) candidate the reference never visits.
bool Engine::blocked(const DevProgram& prog, int r, int b) const {
  if (prog.exclLeadMove && m.rLeader[r] && opt.exclLead[b]) return true;
  return prog.newOnly && !m.isNew(b) && b != m.rOrig[r];
}

// GoalUtils.eligibleBrokers (GoalUtils.java:122-160), the replica-independent part: requested destinations,
// brokers excluded for replica moves, and (leadership moves) brokers excluded for leadership. The leader-replica
// move case is the device's exclLeadMove check.
void Engine::eligible(const std::vector<int32_t>& in, int action, std::vector<int32_t>& out) const {
  out.clear();
  for (int b : in) {
    if (action == DA_LEADERSHIP && opt.anyExclLead && opt.exclLead[b]) continue;
    if (opt.anyRequested) {
      if (action != DA_LEADERSHIP && !opt.requested[b]) continue;
    } else if (opt.anyExclMove && action == DA_MOVE && opt.exclMove[b]) {
      continue;
    }
    out.push_back(b);
  }
}

int64_t Engine::visitCount(int action, int r, const int32_t* cands, size_t n, bool skipHosts) const {
  DevProgram prog;
  std::memset(&prog, 0, sizeof(prog));
  prog.exclLeadMove = (opt.anyExclLead && !opt.anyRequested && action == DA_MOVE) ? 1 : 0;
  prog.newOnly = (m.numNew > 0 && !opt.anyRequested) ? 1 : 0;
  if (!skipHosts && !prog.exclLeadMove && !prog.newOnly) return (int64_t)n;
  const int p = m.rPart[r];
  int64_t c = 0;
  for (size_t q = 0; q < n; ++q) {
    if (skipHosts && m.replicaOn(p, cands[q]) >= 0) continue;
    c += blocked(prog, r, cands[q]) ? 0 : 1;
  }
  return c;
}

// Reference-equivalent candidates of a cross scan whose rows skip replica-dependent ineligible brokers (blocked):
// every row before the hit visits its eligible list, the hit row up to and including the winner.
int64_t Engine::exclLeadCount(const DevProgram& prog, const int32_t* reps, int K, const std::vector<int32_t>& cands,
                              int64_t key) const {
  const int N = (int)cands.size();
  if (prog.newOnly) {
    const int rows = key >= 0 ? (int)(key / N) : K;
    int64_t c = 0;
    for (int k = 0; k <= rows && k < K; ++k) {
      const int upto = k < rows ? N : (int)(key % N) + 1;
      for (int j = 0; j < upto; ++j) c += blocked(prog, reps[k], cands[j]) ? 0 : 1;
    }
    return c;
  }
  int nEx = 0;
  for (int b : cands) nEx += opt.exclLead[b] ? 1 : 0;
  const int rows = key >= 0 ? (int)(key / N) : K;
  int64_t c = 0;
  for (int k = 0; k < rows; ++k) c += N - (m.rLeader[reps[k]] ? nEx : 0);
  if (key >= 0) {
    const int j = (int)(key % N);
    int exBefore = 0;
    if (m.rLeader[reps[rows]])
      for (int q = 0; q < j; ++q) exBefore += opt.exclLead[cands[q]] ? 1 : 0;
    c += j + 1 - exBefore;
  }
  return c;
}

int64_t Engine::crossScan(GoalImpl& self, int action, const std::vector<int32_t>& reps, size_t r0,
                          const std::vector<int32_t>& cands, int filter, bool count, size_t r1) {
  const size_t end = r1 == (size_t)-1 ? reps.size() : std::min(r1, reps.size());
  const int K = (int)(end - r0), N = (int)cands.size();
  if (K <= 0) return -1;
  if (N == 0) return -1;  // every replica visits an empty eligible list
  PhaseScope ps(PH_DEV_SCAN);
  m.flushToDevice();
  DevProgram prog = program(self, action);
  prog.filter = filter;
  // Rows are scanned in windows: a first-fit winner in the first rows is the same winner whatever follows them,
  // so a scan that is usually won early does not send (nor evaluate) every row. The first window can also be a
  // probe of the first row's first kProbeCols columns, used while this goal's scans mostly end there.
  constexpr int kRowWindow = 32, kProbeCols = 1024;
  auto scanRows = [&](int k0, int nk, int cEnd) -> int64_t {  // rows [k0, k0 + nk) x columns [0, cEnd) of N
    const int s0 = (int)((int64_t)cEnd * shard.rank / shard.count), s1 = (int)((int64_t)cEnd * (shard.rank + 1) / shard.count);
    dev->armGroupCombine();
    const int64_t k = combine(dev->scanCross(prog, reps.data() + r0 + k0, nk, cands.data(), N, s0, s1));
    return k < 0 ? -1 : k + (int64_t)k0 * N;
  };
  static const bool windows = !std::getenv("CCMI_SCAN_NO_WINDOWS");  // A/B diagnostics: one scan over every row
  int64_t key = -1;
  int done = 0;  // rows fully scanned without a winner
  bool found = !windows;
  if (!windows) key = scanRows(0, K, N);
  if (!found && N > 2 * kProbeCols && self.probeHitRate > 0.9) {
    key = scanRows(0, 1, kProbeCols);
    found = key >= 0;
    self.probeHitRate = 0.95 * self.probeHitRate + (found ? 0.05 : 0.0);
  }
  if (!found && K > 2 * kRowWindow) {
    key = scanRows(0, kRowWindow, N);
    found = key >= 0;
    done = kRowWindow;
  }
  if (!found) key = scanRows(done, K - done, N);
  if (windows && key >= 0 && N > 2 * kProbeCols && !(self.probeHitRate > 0.9))  // learn whether the probe would win
    self.probeHitRate = 0.95 * self.probeHitRate + (key < kProbeCols ? 0.05 : 0.0);
  checkTerminal(key);
  if (count) {
    if (prog.exclLeadMove || prog.newOnly) candidates += exclLeadCount(prog, reps.data() + r0, K, cands, key);
    else candidates += key >= 0 ? key + 1 : (int64_t)K * N;
  }
  return key;
}

int64_t Engine::crossScanSegs(GoalImpl& self, int action, const std::vector<SnapSeg>& segs,
                              const std::vector<int32_t>& cands) {
  DevProgram prog = program(self, action);
  if (!dev->segsUsable() || shard.count > 1 || prog.exclLeadMove || prog.newOnly) {
    std::vector<int32_t> flat;
    {
      PhaseScope pf(PH_FLATTEN);
      for (const SnapSeg& sg : segs)
        if (sg.v->size() > sg.skip) flat.insert(flat.end(), sg.v->begin() + sg.skip, sg.v->end());
    }
    return crossScan(self, action, flat, 0, cands);
  }
  int64_t K = 0;
  for (const SnapSeg& sg : segs) K += sg.v->size() > sg.skip ? (int64_t)(sg.v->size() - sg.skip) : 0;
  const int N = (int)cands.size();
  if (K <= 0 || N == 0) return -1;
  PhaseScope ps(PH_DEV_SCAN);
  m.flushToDevice();
  prog.filter = FILTER_NONE;
  dev->armGroupCombine();
  const int64_t key = combine(dev->scanSegs(prog, segs, cands.data(), N, 0, N));
  checkTerminal(key);
  candidates += key >= 0 ? key + 1 : K * N;
  return key;
}

bool Engine::queueOn(const GoalImpl& self, int action) const {
  static const bool off = std::getenv("CCMI_QUEUE_SCAN") && std::getenv("CCMI_QUEUE_SCAN")[0] == '0';
  // (a destination-sharded session scans the whole queue on every rank: identical models, identical first fit)
  if (off || !dev->queueUsable() || !shardQueueAllowed) return false;
  const DevProgram prog = program(self, action);
  return !prog.exclLeadMove && !prog.newOnly;
}

namespace {
uint64_t specKey(const Model::Spec& s, uint32_t selEpoch) {  // identity of the directory's contents
  uint64_t h = 1469598103934665603ull;
  auto mix = [&h](uint64_t v) { h = (h ^ v) * 1099511628211ull; };
  mix(s.selLeaders);
  mix(s.selFollowers);
  mix(s.selImmigrants);
  mix(s.selImmOrOffline);
  mix(s.selOffline);
  mix(s.selExclTopics);
  mix(s.selExclMust);
  mix(s.selMustTopics);
  mix((uint64_t)(int64_t)s.selAboveRes);
  mix((uint64_t)(int64_t)s.selBelowRes);
  uint64_t u;
  std::memcpy(&u, &s.aboveLimit, 8);
  mix(u);
  std::memcpy(&u, &s.belowLimit, 8);
  mix(u);
  mix(s.prioOffline);
  mix(s.prioImmigrants);
  mix((uint64_t)(int64_t)s.scoreRes);
  mix(s.scoreReverse);
  mix(selEpoch);
  return h | 1ull;  // never 0 (an unbound directory)
}
}  // namespace

bool Engine::queueReady(const GoalImpl& self, int action, const Model::Spec& spec) {
  if (!queueOn(self, action)) return false;
  PhaseScope ps(PH_DEV_SCAN);
  return queueSyncTry(spec);
}

void Engine::queueSync(const Model::Spec& spec) {
  if (!queueSyncTry(spec))
    throw Unsupported("the snapshot directory outgrew the snapshot pool (CCMI_SNAPSHOT_POOL_ROWS) during a move-in loop");
}

// Every broker's directory entry current for `spec`: all of them when the directory was filled for another Spec (or
// the pool wrapped under it), otherwise only the brokers relocations touched since the last sync (Model::verLog).
// False when the directory's snapshots do not fit the pool together; the directory is then left unbound.
bool Engine::queueSyncTry(const Model::Spec& spec) {
  PhaseScope ps(PH_FLATTEN);
  const uint64_t key = specKey(spec, m.selEpoch);
  QueueSync& q = qsync_;
  if (q.stamp.size() != (size_t)m.B) q.stamp.assign(m.B, 0);
  bool full = !q.bound || q.key != key || dev->qdirKey() != key || q.epoch != dev->poolEpoch();
  // the listed brokers' snapshots and their rows' upload, on the host pool (hostpool.h) when there are many
  auto setMany = [&](const std::vector<int32_t>& bs) {
    {
      NsScope ns(52, "queue.ns.snapshots");
      m.snapshotMany(spec, bs, q.snaps);
    }
    NsScope ns(53, "queue.ns.uploads");
    const bool ok = dev->qdirSetMany(bs, q.snaps);
    q.snaps.clear();
    return ok;
  };
  auto unbind = [&]() {
    q.bound = false;
    return false;
  };
  for (int attempt = 0; attempt < 3; ++attempt) {
    const auto t0 = prof().on ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point();
    auto ns = [&] {
      return (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    };
    q.todo.clear();
    if (full) {
      dev->qdirBind(key);
      q.bound = true;
      q.key = key;
      q.epoch = dev->poolEpoch();
      q.logPos = m.verLog.size();
      for (int b = 0; b < m.B; ++b) q.todo.push_back(b);
      if (!setMany(q.todo)) return unbind();
      prof().count(20, "queue.dir.full", 1);
      if (prof().on) prof().count(28, "queue.full.ns", ns());
    } else {
      ++q.round;
      const size_t end = m.verLog.size();
      for (size_t k = q.logPos; k < end; ++k) {
        const int b = m.verLog[k];
        if (q.stamp[b] == q.round) continue;
        q.stamp[b] = q.round;
        q.todo.push_back(b);
      }
      if (!setMany(q.todo)) return unbind();
      q.logPos = end;
      prof().count(29, "queue.sync.brokers", (int64_t)q.todo.size());
      if (prof().on) prof().count(30, "queue.inc.ns", ns());
    }
    if (q.epoch == dev->poolEpoch()) return true;  // no pool wrap while setting: every entry points at live rows
    full = true;
  }
  return unbind();  // the pool keeps wrapping: the directory does not fit it
}

int64_t Engine::queueScan(GoalImpl& self, int action, const Model::Spec& spec, int head, int skip0,
                          const int32_t* tail, int nTail, const std::vector<int32_t>& cands) {
  const int hasHead = head >= 0 ? 1 : 0;
  const int n = hasHead + nTail, N = (int)cands.size();
  if (n == 0 || N == 0) return -1;
  PhaseScope ps(PH_DEV_SCAN);
  queueSync(spec);
  m.flushToDevice();
  const DevProgram prog = program(self, action);
  const int64_t key = dev->scanQueue(prog, head, skip0, tail, nTail, cands.data(), N);
  checkTerminal(key);
  // reference-equivalent candidates: every row of the entries before the winner's, then its rows up to the winner
  const int span = dev->queueSpan();
  const int wi = key < 0 ? n : (int)(key / N / span);
  int64_t rows = 0;
  for (int i = 0; i < wi; ++i) {
    const int len = dev->qdirLen(i < hasHead ? head : tail[i - hasHead]), s0 = i == 0 ? skip0 : 0;
    rows += len > s0 ? len - s0 : 0;
  }
  if (key < 0) candidates += rows * N;
  else candidates += (rows + (key / N) % span - (wi == 0 ? skip0 : 0)) * N + key % N + 1;
  return key;
}

// CCMI_FORCE_COMBINE=1 sends single-shard keys through the combiner too (diagnostics: exercises the RCCL path of a
// one-rank communicator on a one-GPU box)
static bool forceCombine() {
  const char* e = std::getenv("CCMI_FORCE_COMBINE");  // read per call: only one-shard sessions with a combiner ask
  return e && e[0] == '1';
}

int64_t Engine::combine(int64_t localKey) const {
  const bool onDevice = dev->takeDeviceCombined();  // (also disarms the group combine)
  if (shard.count <= 1 && !(shard.fn && forceCombine())) return localKey;
  dev->perf.combines++;
  if (onDevice) return localKey;  // a shard group's scan server published the group minimum
  int64_t k = localKey < 0 ? INT64_MAX : localKey;
  if (!shard.fn || shard.fn(shard.ctx, &k) != 0) throw std::runtime_error("shard combine (MIN allreduce) failed");
  return k == INT64_MAX ? -1 : k;
}

int64_t Engine::pairScan(GoalImpl& self, const std::vector<int32_t>& pr, const std::vector<int32_t>& pb, int action,
                         bool count) {
  if (pr.empty()) return -1;
  PhaseScope ps(PH_DEV_SCAN);
  m.flushToDevice();
  const int n = (int)pr.size();
  const int p0 = (int)((int64_t)n * shard.rank / shard.count), p1 = (int)((int64_t)n * (shard.rank + 1) / shard.count);
  const DevProgram prog = program(self, action);
  dev->armGroupCombine();
  const int64_t key = combine(dev->scanPairs(prog, pr.data(), pb.data(), p0, p1));
  checkTerminal(key);
  if (!count) return key;
  if (prog.exclLeadMove || prog.newOnly) {
    const size_t end = key >= 0 ? (size_t)key + 1 : pr.size();
    for (size_t q = 0; q < end; ++q) candidates += blocked(prog, pr[q], pb[q]) ? 0 : 1;
  } else {
    candidates += key >= 0 ? key + 1 : (int64_t)pr.size();
  }
  return key;
}

int64_t Engine::swapScan(GoalImpl& self, const std::vector<int32_t>& srcs, const std::vector<int32_t>& cbOff,
                         const std::vector<int32_t>& cbRep, const SwapLimit& lim) {
  if (srcs.empty() || cbRep.empty()) return -1;
  PhaseScope ps(PH_DEV_SCAN);
  m.flushToDevice();
  int64_t visited = 0;
  const DevProgram prog = program(self, DA_SWAP);
  // eligibleReplicasForSwap CASE#2 (GoalUtils.java:289-294): an old source broker and a NEW destination make the
  // reference call removeIf on an unmodifiable SortedSet view; the first such row (rows are candidate-broker major)
  // throws unless an earlier row accepts a swap
  int64_t throwRow = -1;
  if (prog.newOnly) {
    if (lim.res >= 0) throw std::logic_error("swapScan: a limit-free candidate list with new brokers");
    const int S = (int)srcs.size();
    for (int g = 0; g + 1 < (int)cbOff.size() && throwRow < 0; ++g) {
      if (cbOff[g] == cbOff[g + 1]) continue;
      const int db = m.rBroker[cbRep[cbOff[g]]];
      if (!m.isNew(db)) continue;
      for (int s = 0; s < S; ++s) {
        const int sr = srcs[s];
        const bool excl = prog.swapExcl && !m.origOffline(sr) &&
                          ((opt.anyExclMove && opt.exclMove[db]) || (m.rLeader[sr] && opt.anyExclLead && opt.exclLead[db]));
        if (!excl && !m.isNew(m.rBroker[sr])) {
          throwRow = (int64_t)g * S + s;
          break;
        }
      }
    }
  }
  const int64_t key = dev->scanSwap(prog, srcs.data(), (int)srcs.size(), cbOff.data(), (int)cbOff.size() - 1,
                                    cbRep.data(), (int)cbRep.size(), lim, &visited);
  if (throwRow >= 0 && (key < 0 || (key >> 24) > throwRow))
    throw Unsupported("UnsupportedOperationException: removeIf on an unmodifiable sorted replica view");
  checkTerminal(key);
  candidates += visited;
  return key;
}

bool Engine::chainsOn() const {
  static const bool off = std::getenv("CCMI_NO_CHAINS") != nullptr;
  // a chain would apply the move a terminal goal refuses; chains keep the host loads of brokers sharing hosts too
  // (apply.h host lanes). A destination-sharded session runs every chain whole on each rank: the ranks hold identical
  // models, so they make the same decisions without a combine.
  return !off && !terminalOptimized();
}

bool Engine::terminalOptimized() const {
  for (const GoalImpl* g : priors)
    if (g->terminal) return true;
  return false;
}
void Engine::checkTerminal(int64_t key) const {
  if (key < 0) return;
  for (const GoalImpl* g : priors)
    if (g->terminal) throw StateError("No goal should be executed after " + g->name);
}

GoalImpl* Engine::optimizedOfKind(int kind) const {
  for (const auto& g : optimized)
    if (g->kind == kind) return g.get();
  return nullptr;
}

int64_t Engine::chainPairs(GoalImpl& self, int action, const std::vector<int32_t>& pr, const std::vector<int32_t>& pb,
                           const std::vector<int32_t>& next, int maxAccepts, std::vector<int32_t>& log) {
  PhaseScope ps(PH_DEV_SCAN);
  const bool tp = prof().on;  // CCMI_PROFILE: ns in the row flushes, the program, the device round trip
  auto tnow = [] { return std::chrono::steady_clock::now(); };
  auto ns = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
    return (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count();
  };
  const auto c0 = tp ? tnow() : std::chrono::steady_clock::time_point();
  m.flushToDevice();
  m.flushChainLoads();
  const auto c1 = tp ? tnow() : c0;
  const DevProgram prog = program(self, action);
  const auto c2 = tp ? tnow() : c0;
  const Device::ChainResult r =
      dev->chainPairs(prog, pr.data(), pb.data(), next.data(), (int)pr.size(), maxAccepts, log);
  if (tp) {
    const auto c3 = tnow();
    prof().count(32, "chain.ns.flush", ns(c0, c1));
    prof().count(33, "chain.ns.program", ns(c1, c2));
    prof().count(34, "chain.ns.device", ns(c2, c3));
    prof().count(35, "chain.calls", 1);
  }
  if (prog.exclLeadMove || prog.newOnly) {
    // the device counts every pair it passes; the reference never visits the blocked ones (the filters are static
    // over a leadership chain: original brokers, NEW states and exclusions do not change)
    int64_t visited = 0;
    int start = 0;
    auto add = [&](int a, int b) {
      for (int q = a; q < b; ++q) visited += blocked(prog, pr[q], pb[q]) ? 0 : 1;
    };
    for (size_t i = 0; i < (size_t)r.accepts; ++i) {
      add(start, log[i] + 1);
      start = next[log[i]];
    }
    if (r.accepts < maxAccepts) add(start, (int)pr.size());
    candidates += visited;
  } else {
    candidates += r.visited;
  }
  return r.accepts;
}

int64_t Engine::chainRackRows(GoalImpl& self, const std::vector<int32_t>& rows, const std::vector<int32_t>& cands,
                              std::vector<int32_t>& log) {
  PhaseScope ps(PH_DEV_SCAN);
  m.flushToDevice();
  m.flushChainLoads();
  DevProgram prog = program(self, DA_MOVE);
  prog.filter = FILTER_RACK_AWARE;
  const Device::ChainResult r = dev->chainRackRows(prog, rows.data(), (int)rows.size(), cands.data(),
                                                   (int)cands.size(), log);
  return r.failRow;
}

void Engine::rackRowsGroups(GoalImpl& self, const std::vector<int32_t>& rows, const std::vector<int32_t>& cands,
                            std::vector<int32_t>& res) {
  PhaseScope ps(PH_DEV_SCAN);
  m.flushToDevice();
  DevProgram prog = program(self, DA_MOVE);
  prog.filter = FILTER_RACK_AWARE;
  if (prog.nGoals != 1) throw std::logic_error("rackRowsGroups needs a program without optimized goals");
  // the rows of each partition, in row order (a counting sort by partition)
  const int n = (int)rows.size();
  std::vector<int32_t> cnt((size_t)m.P + 1, 0), order(n), gOff;
  for (int r : rows) cnt[(size_t)m.rPart[r] + 1]++;
  for (int p = 0; p < m.P; ++p) cnt[(size_t)p + 1] += cnt[p];
  std::vector<int32_t> at(cnt.begin(), cnt.end() - 1);
  for (int k = 0; k < n; ++k) order[at[m.rPart[rows[k]]]++] = k;
  gOff.push_back(0);
  for (int p = 0; p < m.P; ++p)
    if (cnt[(size_t)p + 1] > cnt[p]) gOff.push_back(cnt[(size_t)p + 1]);
  res.assign(n, kRackKeep);
  dev->rackRowsGroups(prog, rows.data(), n, order.data(), gOff.data(), (int)gOff.size() - 1, cands.data(),
                      (int)cands.size(), res.data());
}

int Engine::acceptance(int gi, const ccmi_action& a) {
  {
    const int ia = intraAcceptance(*optimized.at(gi), *this, a);
    if (ia >= 0) return ia;
    if (a.type == CCMI_INTRA_BROKER_REPLICA_MOVEMENT || a.type == CCMI_INTRA_BROKER_REPLICA_SWAP)
      throw std::invalid_argument("Unsupported balancing action " + std::to_string(a.type) + " is provided.");
  }
  if (optimized.at(gi)->terminal) throw StateError("No goal should be executed after " + optimized.at(gi)->name);
  std::vector<const std::vector<uint8_t>*> allowedBySlot(kMaxSlots, nullptr);
  for (auto& g : optimized) allowedBySlot[g->dg.allowedSlot] = &g->allowed;
  HostView v{m, allowedBySlot, topicUpper, topicLower, brokerSetOf, replicaSetOf, minLeadOf, topicLeadLim};
  const GoalImpl& g = *optimized.at(gi);
  const int sr = m.replicaOn(a.partition, a.source_broker);
  if (sr < 0) throw std::invalid_argument("no replica of the partition on the source broker");
  if (a.type == CCMI_INTER_BROKER_REPLICA_SWAP) {
    const int dr = m.replicaOn(a.destination_partition, a.destination_broker);
    if (dr < 0) throw std::invalid_argument("no replica of the destination partition on the destination broker");
    return goalAcceptSwap(g.dg, v, sr, a.source_broker, dr, a.destination_broker);
  }
  const int action = a.type == CCMI_LEADERSHIP_MOVEMENT ? DA_LEADERSHIP : DA_MOVE;
  if (a.type != CCMI_INTER_BROKER_REPLICA_MOVEMENT && a.type != CCMI_LEADERSHIP_MOVEMENT)
    throw std::invalid_argument("Unsupported balancing action");
  if (goalAcceptMove(g.dg, v, action, sr, a.source_broker, a.destination_broker)) return CCMI_ACCEPT;
  // AbstractRackAwareGoal.actionAcceptance rejects a replica move with BROKER_REJECT (AbstractRackAwareGoal.java:
  // 100-106); every other goal's rejected move or leadership move is a REPLICA_REJECT
  // BrokerSetAwareGoal.actionAcceptance: BROKER_REJECT too (BrokerSetAwareGoal.java:240-246)
  const bool rack = g.dg.kind == DG_RACK_AWARE || g.dg.kind == DG_RACK_AWARE_DISTRIBUTION ||
                    g.dg.kind == DG_BROKER_SET_AWARE;
  return rack && action == DA_MOVE ? CCMI_BROKER_REJECT : CCMI_REPLICA_REJECT;
}

ccmi_cluster_stats Engine::stats() {
  PhaseScope ps(PH_DEV_STATS);
  m.flushToDevice();
  const int ldB = dev->ldB();
  std::vector<uint8_t> aa(ldB, 0);
  int na = 0;
  for (int b = 0; b < m.B; ++b)
    if (m.alive(b) && !(opt.anyExclMove && opt.exclMove[b])) {
      aa[b] = 1;
      na++;
    }
  StatsParams P;
  std::memset(&P, 0, sizeof(P));
  P.B = m.B;
  P.T = m.T;
  P.numAllowed = na;
  for (int res = 0; res < 4; ++res) {
    P.clusterUtil[res] = m.clusterUtil(res);
    P.avgPct[res] = P.clusterUtil[res] / m.capacityWithAllowedReplicaMoves(res, opt.exclMove);
    P.upperThr[res] = threshold(P.avgPct[res], res, false);
    P.lowerThr[res] = threshold(P.avgPct[res], res, true);
  }
  P.potCapacity = m.capacityWithAllowedReplicaMoves(R_NW_OUT, opt.exclMove);
  P.nwOutCapThreshold = bc.capThreshold[R_NW_OUT];
  for (int b = 0; b < m.B; ++b) {
    if (aa[b]) P.potSum += m.potNwOut(b);
    P.repTotal += m.nrep(b);
    P.leadTotal += m.bNlead[b];
  }
  StatsOut o;
  dev->stats(P, aa.data(), &o);
  ccmi_cluster_stats s;
  std::memset(&s, 0, sizeof(s));
  for (int r = 0; r < 4; ++r) {
    s.resource_avg[r] = o.resAvg[r];
    s.resource_max[r] = o.resMax[r];
    s.resource_min[r] = o.resMin[r];
    s.resource_std[r] = o.resStd[r];
    s.num_balanced_brokers_by_resource[r] = o.numBalanced[r];
  }
  s.potential_nw_out_avg = o.pnwAvg;
  s.potential_nw_out_max = o.pnwMax;
  s.potential_nw_out_min = o.pnwMin;
  s.potential_nw_out_std = o.pnwStd;
  s.num_brokers_under_potential_nw_out = o.numUnderPot;
  s.replica_avg = o.repAvg;
  s.replica_std = o.repStd;
  s.replica_max = o.repMax;
  s.replica_min = o.repMin;
  s.leader_avg = o.leadAvg;
  s.leader_std = o.leadStd;
  s.leader_max = o.leadMax;
  s.leader_min = o.leadMin;
  s.topic_replica_avg = o.topicAvg;
  s.topic_replica_std = o.topicStd;
  s.topic_replica_max = o.topicMax;
  s.topic_replica_min = o.topicMin;
  s.num_brokers = m.B;
  s.num_replicas_in_cluster = m.R;
  s.num_topics = m.T;
  if (m.D > 0) {  // ClusterModelStats.populateStatsForDisks (ClusterModelStats.java:489-511)
    if (m.diskDirty) {
      dev->setDiskUtil(m.dUtil.data());
      m.diskDirty = false;
    }
    DiskStatsOut ds{};
    dev->statsDisks(bc.resBalance[R_DISK], &ds);
    s.num_unbalanced_disks = ds.unbalanced;
    s.disk_utilization_std = ds.numAlive > 0 ? std::sqrt(ds.varSum / ds.numAlive) : 0.0;
  }
  {
    std::vector<uint8_t> seen(m.P, 0);
    int n = 0;
    for (int r = 0; r < m.R; ++r)
      if (m.selfHealing[r] && !seen[m.rPart[r]]) {
        seen[m.rPart[r]] = 1;
        n++;
      }
    s.num_partitions_with_offline_replicas = n;
  }
  return s;
}

// AbstractGoal.optimize (AbstractGoal.java:81-135) + the per-goal bookkeeping of GoalOptimizer.optimizations
bool Engine::optimizeGoal(std::unique_ptr<GoalImpl> g, const std::vector<GoalImpl*>& priorSet, ccmi_goal_result* res) {
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  const int64_t c0 = candidates;
  const size_t a0 = m.log.size();
  const int64_t l0 = dev->perf.scanLaunches + dev->perf.intraLaunches, p0 = dev->perf.scanPairs;
  struct Clear {
    Model& m;
    ~Clear() {
      m.clearTracked();
      prof().candCounter = nullptr;
    }
  } guard{m};
  prof().candCounter = &candidates;
  // optimizedGoals in the session's order; a goal's slot is free unless an entry of `optimized` holds it
  priors.clear();
  for (const auto& h : optimized)
    if (std::find(priorSet.begin(), priorSet.end(), h.get()) != priorSet.end()) priors.push_back(h.get());
  if (priors.size() != priorSet.size()) throw std::invalid_argument("optimized goal not held by the session");
  uint32_t used = 0;
  for (const auto& h : optimized) used |= 1u << h->dg.allowedSlot;
  newSlot = 0;
  while (newSlot < kMaxSlots && (used >> newSlot) & 1u) ++newSlot;
  if (newSlot >= kMaxSlots) throw Unsupported("no free goal slot");
  struct ClearPriors {
    std::vector<GoalImpl*>& p;
    ~ClearPriors() { p.clear(); }
  } clearPriors{priors};
  g->succeeded = true;
  g->prov = provisionResponse(CCMI_PROVISION_UNDECIDED);  // AbstractGoal.java:87
  try {
    return optimizeGoalImpl(g, res, t0, c0, a0, l0, p0);
  } catch (OptimizationFailure& f) {  // AbstractGoal.java:125-126 (a Goal outside that template keeps its own response)
    lastFailure = !g->abstractGoal ? g->prov
                  : f.hasRec      ? provisionResponse(CCMI_PROVISION_UNDER_PROVISIONED, f.rec)
                                  : provisionResponse(CCMI_PROVISION_UNDER_PROVISIONED);
    throw;
  }
}

// GoalUtils.validateProvisionResponse (GoalUtils.java:619-650)
ccmi_provision_response validateProvision(const ccmi_provision_response& p, const Model& m, int minBrokers) {
  if (p.status != CCMI_PROVISION_OVER_PROVISIONED) return p;
  int alive = 0;
  for (int b = 0; b < m.B; ++b) alive += m.alive(b) ? 1 : 0;
  if (alive < minBrokers) return provisionResponse(CCMI_PROVISION_RIGHT_SIZED);
  if (!p.has_recommendation) throw std::invalid_argument("Expected to have exactly 1 provision recommendation, but got: 0");
  const int maxAllowedToDrop = alive - m.maxRf;
  if (p.recommendation.num_brokers <= maxAllowedToDrop) return p;
  if (maxAllowedToDrop > 0) {
    ccmi_provision_recommendation r = provisionRec(CCMI_PROVISION_OVER_PROVISIONED);
    r.num_brokers = maxAllowedToDrop;
    return provisionResponse(CCMI_PROVISION_OVER_PROVISIONED, r);
  }
  return provisionResponse(CCMI_PROVISION_RIGHT_SIZED);
}

bool Engine::optimizeGoalImpl(std::unique_ptr<GoalImpl>& g, ccmi_goal_result* res, std::chrono::steady_clock::time_point t0,
                              int64_t c0, size_t a0, int64_t l0, int64_t p0) {
  using clk = std::chrono::steady_clock;
  {  // the leadership loops' K7 chains are opt-in (CCMI_PAIR_CHAINS=1, read per goal): one pair scan per decision with
     // the move applied on the host is faster (profiles/r06/README.md, chain A/B)
    const char* pc = std::getenv("CCMI_PAIR_CHAINS");
    pairChains = pc && pc[0] == '1' && !std::getenv("CCMI_NO_PAIR_CHAINS");
  }
  const ccmi_cluster_stats before = stats();
  g->finished = false;
  g->dg.allowedSlot = newSlot;
  g->init(*this);
  g->dg.allowedSlot = newSlot;
  dev->setAllowed(g->dg.allowedSlot, g->allowed.data());
  if (opt.anyExclLead || opt.anyExclMove || m.numNew > 0 || exclOnDevice) {
    const std::vector<uint8_t> none(m.B, 0);
    std::vector<uint8_t> isNew(m.B, 0);
    for (int b = 0; b < m.B; ++b) isNew[b] = m.isNew(b) ? 1 : 0;
    dev->setExclusions(opt.anyExclLead ? opt.exclLead.data() : none.data(),
                       opt.anyExclMove ? opt.exclMove.data() : none.data(), isNew.data());
    exclOnDevice = opt.anyExclLead || opt.anyExclMove || m.numNew > 0;
  }
  const bool brokenEmpty = m.numDead == 0 && m.numBadDisk == 0;
  bool exclWithReplicas = false;
  for (int b = 0; b < m.B; ++b)
    if (m.alive(b) && opt.anyExclMove && opt.exclMove[b] && m.nrep(b) > 0) exclWithReplicas = true;
  while (!g->finished) {
    if (!g->rebalanceAll(*this))
      for (int b : g->brokersToBalance(*this)) g->rebalance(*this, b);
    PhaseScope ps(PH_UPDATE);
    g->update(*this);
  }
  const ccmi_cluster_stats after = stats();
  if (brokenEmpty && !exclWithReplicas && g->compareStats(after, before) < 0)
    throw StateError("Optimization for goal " + g->name + " failed because the optimized result is worse than before.");
  const bool ok = g->succeeded;
  g->prov = validateProvision(g->prov, m, bc.overMinBrokers);
  if (res) {
    res->provision = g->prov;
    res->goal_kind = g->kind;
    res->succeeded = ok ? 1 : 0;
    res->candidates = candidates - c0;
    res->actions = (int64_t)(m.log.size() - a0);
    res->device_launches = dev->perf.scanLaunches + dev->perf.intraLaunches - l0;
    res->device_candidates = dev->perf.scanPairs - p0;
  }
  m.clearTracked();
  static const bool perGoalProfile = std::getenv("CCMI_PROFILE") && std::string(std::getenv("CCMI_PROFILE")) == "goal";
  if (perGoalProfile) {  // CCMI_PROFILE=goal: one phase profile per goal
    prof().print(g->name.c_str());
    PhaseProf fresh;
    fresh.candCounter = prof().candCounter;
    prof() = fresh;
  }
  // GoalOptimizer keeps one instance per goal class: a re-optimized kind replaces its older entry
  for (size_t i = 0; i < optimized.size(); ++i)
    if (optimized[i]->kind == g->kind) {
      optimized.erase(optimized.begin() + (long)i);
      break;
    }
  optimized.push_back(std::move(g));
  if (res) {
    res->stats = stats();  // GoalOptimizer.statsByGoalPriority
    res->seconds = std::chrono::duration<double>(clk::now() - t0).count();
  }
  return ok;
}

// ======================================================================================= ReplicaDistributionGoal
namespace {

// The drivers' broker PriorityQueues: an OrderedQueue (O(n) build from a maintained order) when no queued
// broker can change key while queued, otherwise the exact java.util.PriorityQueue emulation.
template <class Cmp>
class LiveQueue {
 public:
  explicit LiveQueue(Cmp c) : oq_(c), pq_(c) {}
  void init(int /*capacity*/, bool ordered) { ordered_ = ordered; }
  bool ordered() const { return ordered_; }
  void push_sorted(int x) { oq_.sorted().push_back(x); }
  std::vector<int>& sortedRun() { return oq_.sorted(); }
  bool empty() const { return ordered_ ? oq_.empty() : pq_.empty(); }
  int peek() const { return ordered_ ? oq_.peek() : pq_.peek(); }
  int poll() { return ordered_ ? oq_.poll() : pq_.poll(); }
  void add(int x) {
    if (ordered_) oq_.add(x);
    else pq_.add(x);
  }
  // a likely future poll (-1: none known)
  int upcoming(size_t k) const { return ordered_ ? oq_.upcoming(k) : -1; }
  // ordered form with nothing re-added: the remaining poll order is a contiguous run (OrderedQueue::runData)
  bool runOnly() const { return ordered_ && oq_.heapEmpty(); }
  // ordered form: the re-added heap's next element, its poll, and the run's elements that poll before x
  bool heapEmpty() const { return oq_.heapEmpty(); }
  int heapPeek() const { return oq_.heapPeek(); }
  int heapPoll() { return oq_.heapPoll(); }
  size_t runBefore(int x) const { return oq_.runBefore(x); }
  const int* runData() const { return oq_.runData(); }
  size_t runLeft() const { return oq_.runLeft(); }
  void skipRun(size_t k) { oq_.skipRun(k); }
  // speculatively polled entries whose keys did not change, in reverse poll order
  void unpoll(int x) {
    if (ordered_) oq_.unpoll(x);
    else pq_.add(x);
  }

 private:
  bool ordered_ = false;
  OrderedQueue<Cmp> oq_;
  JavaPQ<Cmp> pq_;
};

class ReplicaDistribution : public GoalImpl {
 public:
  ReplicaDistribution() {
    kind = CCMI_GOAL_REPLICA_DISTRIBUTION;
    name = "ReplicaDistributionGoal";
  }
  static constexpr int kName = 4 * CCMI_GOAL_REPLICA_DISTRIBUTION;
  int upper = 0, lower = 0;
  bool anyAbove = false, anyUnder = false;

  bool excluded(int b) const { return !allowed[b]; }

  // ReplicaDistributionAbstractGoal.initGoalState + ReplicaDistributionGoal.initGoalState
  void init(Engine& e) override {
    Model& m = e.m;
    allowed.assign(m.B, 0);
    int n = 0;
    for (int b = 0; b < m.B; ++b)
      if (m.alive(b) && !(e.opt.anyExclMove && e.opt.exclMove[b])) {
        allowed[b] = 1;
        n++;
      }
    if (n == 0)
      throw OptimizationFailure("[" + name + "] All alive brokers are excluded from replica moves.", underBrokers(m.maxRf));
    const double avg = m.R / (double)n;
    const double adj = (e.bc.replicaBalance - 1) * kBalanceMargin;
    upper = (int)std::ceil(avg * (1 + adj));
    lower = (int)std::floor(avg * jmax(0, (1 - adj)));
    dg = DevGoal{};
    dg.kind = DG_REPLICA_DISTRIBUTION;
    dg.upper = upper;
    dg.lower = lower;
    dg.fixOffline = 0;
    dg.allowedSlot = e.newSlot;
    const bool selfHealing = m.numSelfHealing > 0;
    for (int b = 0; b < m.B; ++b) {
      Model::Spec s;
      s.selImmigrants = e.opt.onlyImmigrants;
      s.selImmOrOffline = selfHealing && m.alive(b);
      s.selExclTopics = e.opt.anyExclTopic;
      s.prioOffline = selfHealing;
      s.prioImmigrants = !e.opt.onlyImmigrants;
      s.scoreRes = R_DISK;
      s.scoreReverse = false;
      m.track(b, kName, s);
    }
  }

  // ReplicaDistributionAbstractGoal.updateGoalState (:187-229), then ReplicaDistributionGoal's provisioning
  // (ReplicaDistributionGoal.java:85-107), every round
  void update(Engine& e) override {
    if (anyAbove) succeeded = false;
    if (anyUnder) succeeded = false;
    anyAbove = anyUnder = false;
    Model& m = e.m;
    [&] {
      for (int r = 0; r < m.R; ++r)
        if (m.selfHealing[r] && m.curOffline(r)) {
          if (dg.fixOffline)  // GoalUtils.ensureNoOfflineReplicas rethrown
            throw OptimizationFailure("[" + name + "] Cannot remove replica from broker " +
                                          std::to_string(m.bId[m.rBroker[r]]),
                                      underBrokers(1));
          dg.fixOffline = 1;
          return;
        }
      finished = true;
    }();
    int numAllowed = 0;
    bool anyAboveMax = false;
    for (int b = 0; b < m.B; ++b) {
      numAllowed += allowed[b] ? 1 : 0;
      if (m.alive(b) && (int64_t)m.nrep(b) > e.bc.overMaxReplicasPerBroker) anyAboveMax = true;
    }
    const int numBrokersToDrop = numAllowed - (int)(m.R / e.bc.overMaxReplicasPerBroker);
    if (numBrokersToDrop > 0 && !anyAboveMax) {
      ccmi_provision_recommendation rec = provisionRec(CCMI_PROVISION_OVER_PROVISIONED);
      rec.num_brokers = numBrokersToDrop;
      prov = provisionResponse(CCMI_PROVISION_OVER_PROVISIONED, rec);
    } else {
      prov = provisionResponse(CCMI_PROVISION_RIGHT_SIZED);
    }
  }

  int compareStats(const ccmi_cluster_stats& after, const ccmi_cluster_stats& before) const override {
    const double d1 = after.replica_std, d2 = before.replica_std;
    if (d1 - d2 > 1e-5) return -1;
    if (d2 - d1 > 1e-5) return 1;
    return 0;
  }

  // ReplicaDistributionGoal.rebalanceForBroker (:181-224)
  void rebalance(Engine& e, int b) override {
    Model& m = e.m;
    const int n = m.nrep(b), off = m.bNoff[b];
    const bool excl = excluded(b);
    const bool less = off > 0 || n > upper || excl;
    const bool more = !excl && m.alive(b) && n - off < lower;
    if (m.alive(b) && !more && !less) return;
    if (m.numNew > 0 && !m.isNew(b) && !less) return;
    if (((m.numSelfHealing > 0 && m.bNoff[b] == 0) || e.opt.onlyImmigrants) && less && m.bNimm[b] == 0) return;
    if (less && moveOut(e, b)) anyAbove = true;
    if (more && moveIn(e, b)) anyUnder = true;
  }

  // rebalanceByMovingReplicasOut (:226-276): batches = runs of equal offline status
  bool moveOut(Engine& e, int b) {
    PhaseScope ps(PH_RDG_OUT);
    Model& m = e.m;
    const bool fix = dg.fixOffline != 0;
    auto cmp = [&m](int x, int y) {
      const int c = jcmpInt(m.nrep(x), m.nrep(y));
      return c ? c : jcmpInt(m.bId[x], m.bId[y]);
    };
    RbTreeSet<decltype(cmp)> cand(cmp);
    {
      std::vector<int> ins, order;
      for (int x = 0; x < m.B; ++x)
        if (m.alive(x) && (fix || m.nrep(x) < upper)) ins.push_back(x);
      if (fix) order = ins;
      else javaHashSetOrder(ins, order);  // Collectors.toSet()
      for (int x : order) cand.add(x);
    }
    cand.trackSequence();  // inorder() per accepted move is a copy
    const int upperSrc = excluded(b) ? 0 : upper;
    bool wasUnable = false;
    const std::vector<int32_t> list = m.sorted(b, kName);  // sortedReplicas(true): a clone
    std::vector<int32_t> inorder, cands, batch;
    size_t i = 0;
    while (i < list.size()) {
      if (!m.curOffline(list[i]) && wasUnable && m.nrep(b) <= upperSrc) return false;
      const bool runOffline = m.curOffline(list[i]);
      size_t e2 = i;
      while (e2 < list.size() && m.curOffline(list[e2]) == runOffline) ++e2;
      batch.assign(list.begin() + i, list.begin() + e2);
      // the tree's maintained sequence itself (no copy) when no eligibility filter applies
      const std::vector<int32_t>* seq = cand.sequence();
      if (!seq) {
        cand.inorder(inorder);
        seq = &inorder;
      }
      const std::vector<int32_t>& cl = e.eligibleView(*seq, DA_MOVE, cands);
      const int64_t key = e.crossScan(*this, DA_MOVE, batch, 0, cl);
      if (key < 0) {
        if (runOffline) wasUnable = true;
        i = e2;
        continue;
      }
      const int N = (int)cl.size();
      const int k = (int)(key / N), j = (int)(key % N);
      if (runOffline && k > 0) wasUnable = true;
      const int r = batch[k], dst = cl[j];  // (read before the tree changes below)
      m.relocateReplica(m.rPart[r], b, dst);
      if (m.nrep(b) <= (m.bNoff[b] == 0 ? upperSrc : 0)) return false;
      cand.remove(dst);
      if (m.nrep(dst) < upper || fix) cand.add(dst);
      i = i + k + 1;
    }
    return m.nrep(b) != 0;
  }

  // rebalanceByMovingReplicasIn (:278-340): speculative multi-source batches over the source queue
  bool moveIn(Engine& e, int dest) {
    PhaseScope ps(PH_RDG_IN);
    Model& m = e.m;
    auto cmp = [&m](int b1, int b2) {
      const int r = jcmpInt(m.bNoff[b2], m.bNoff[b1]);
      if (r == 0) {
        const int r2 = jcmpInt(m.nrep(b2), m.nrep(b1));
        return r2 == 0 ? jcmpInt(m.bId[b1], m.bId[b2]) : r2;
      }
      return r;
    };
    JavaPQ<decltype(cmp)> pq(cmp);
    if (dg.fixOffline) {
      for (int s = 0; s < m.B; ++s)
        if (s != dest) pq.add(s);
    } else {
      for (int s = 0; s < m.B; ++s)
        if (m.nrep(s) > lower || m.bNoff[s] > 0 || excluded(s)) pq.add(s);
    }
    std::vector<int32_t> single{dest}, cands;
    e.eligible(single, DA_MOVE, cands);
    if (cands.empty()) return true;  // every replica visits an empty candidate list
    struct Seg {
      int src;
      std::vector<int32_t> list;  // clone of the source's sorted replicas
      size_t start;
    };
    std::vector<Seg> segs;
    std::vector<int32_t> flat;
    size_t target = kFirstBatchRows;
    bool haveCur = false;
    Seg cur;
    while (haveCur || !pq.empty()) {
      segs.clear();
      flat.clear();
      if (haveCur) {  // the source being iterated continues first (its clone, after the winner)
        segs.push_back(std::move(cur));
        haveCur = false;
        flat.insert(flat.end(), segs.back().list.begin() + segs.back().start, segs.back().list.end());
      }
      while (!pq.empty() && (segs.empty() || flat.size() < target)) {
        const int s = pq.poll();
        segs.push_back({s, m.sorted(s, kName), 0});
        flat.insert(flat.end(), segs.back().list.begin(), segs.back().list.end());
      }
      const int64_t key = e.crossScan(*this, DA_MOVE, flat, 0, cands);
      if (key < 0) {
        target = std::min<size_t>(target * kBatchGrowth, kMaxBatchRows);
        continue;  // all segments exhausted; sources are not re-enqueued
      }
      target = kFirstBatchRows;
      size_t q = (size_t)key, mIdx = 0;
      while (q >= segs[mIdx].list.size() - segs[mIdx].start) {
        q -= segs[mIdx].list.size() - segs[mIdx].start;
        ++mIdx;
      }
      Seg& hit = segs[mIdx];
      const size_t idx = hit.start + q;
      const int r = hit.list[idx];
      m.relocateReplica(m.rPart[r], hit.src, dest);
      if (m.nrep(dest) >= lower) return false;
      for (size_t t = mIdx + 1; t < segs.size(); ++t) pq.add(segs[t].src);  // un-poll speculative sources
      bool requeued = false;
      if (!pq.empty()) {
        const int top = pq.peek();
        const int res = jcmpInt(m.bNoff[hit.src], m.bNoff[top]);
        if (res == -1 || (res == 0 && m.nrep(hit.src) < m.nrep(top))) {
          pq.add(hit.src);
          requeued = true;
        }
      }
      if (!requeued && idx + 1 < hit.list.size()) {
        cur = std::move(hit);
        cur.start = idx + 1;
        haveCur = true;
      }
    }
    return true;
  }
};

// ======================================================================================= ResourceDistributionGoal
// Builds ResourceDistributionGoal.moveOut's entry-state candidate TreeSet on a helper thread while the driver scans:
// the same put sequence (members in ascending id, placed by their entry (key, id) rank) the driver would otherwise run
// when its lazy candidate order stops being exact. Most calls never need the tree: a newer submission cancels the
// build in flight, and the driver waits (on a condition variable) only in take(). On by default for clusters of at
// least CCMI_TREE_WORKER_MIN brokers (2048; smaller trees are cheaper to build on the driver thread), CCMI_TREE_WORKER=0
// turns it off. profiles/r04/tree_worker_ab_*.txt: tree.build 1.12 -> 0.79 s and whole C2 proposals 7.36-7.43 ->
// 6.15-6.71 s on one box (round 3's version, which spun on the driver side, had cost 1.3-2.5 s on some boxes).
// Workers are leased per move-out call from one process-wide pool (TreeWorkerPool) of at most CCMI_TREE_WORKERS
// threads (default 8, one per session of an 8-GPU node's plain multi-GPU bench): concurrent sessions share them, and a
// call that finds none free builds on its own thread.
class TreeWorker {
 public:
  struct RankOnly {  // buildByRank never compares
    int operator()(int, int) const { return 0; }
  };
  using Tree = RbTreeSet<RankOnly>;
  TreeWorker() : tree_(RankOnly{}), th_([this] { loop(); }) {}
  ~TreeWorker() {
    {
      std::lock_guard<std::mutex> l(mu_);
      stop_ = true;
      cancel_.store(true);
    }
    cv_.notify_one();
    th_.join();
  }
  // members in entry (key, id) order, over B brokers
  void submit(const std::vector<int32_t>& order, int B, bool withSequence) {
    {
      std::lock_guard<std::mutex> l(mu_);
      next_.assign(order.begin(), order.end());
      nextB_ = B;
      nextSeq_ = withSequence;
      nextMask_ = CpuMask::current();  // built on the submitting thread's CPUs (its session's pin, if any)
      tSubmit_ = std::chrono::steady_clock::now();
      ++gen_;
      cancel_.store(true, std::memory_order_relaxed);  // the build in flight (if any) is stale
    }
    cv_.notify_one();
  }
  // the build in flight (if any) is no longer wanted (the lease ends)
  void cancel() { cancel_.store(true, std::memory_order_relaxed); }
  // the latest submission's tree (waits for it); its structure is handed over with RbTreeSet::adopt
  Tree& take() {
    const auto tTake = std::chrono::steady_clock::now();
    std::unique_lock<std::mutex> l(mu_);
    const uint64_t want = gen_;
    cvDone_.wait(l, [&] { return done_ == want; });
    if (prof().on) {  // CCMI_PROFILE: submit -> worker start, the build, submit -> take (ns)
      auto ns = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
        return (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count();
      };
      prof().count(48, "tree.ns.wake", ns(tSubmit_, tStart_));
      prof().count(49, "tree.ns.work", ns(tStart_, tDone_));
      prof().count(50, "tree.ns.needed", ns(tSubmit_, tTake));
    }
    return tree_;
  }

 private:
  void loop() {
    pthread_setname_np(pthread_self(), "ccmi-tree");
    uint64_t started = 0;
    CpuMask mine = CpuMask::current(), want;
    for (;;) {
      uint64_t gen;
      {
        std::unique_lock<std::mutex> l(mu_);
        cv_.wait(l, [&] { return stop_ || gen_ != started; });
        if (stop_) return;
        gen = started = gen_;
        tStart_ = std::chrono::steady_clock::now();
        order_.swap(next_);
        B_ = nextB_;
        seq_ = nextSeq_;
        want = nextMask_;
        cancel_.store(false, std::memory_order_relaxed);
      }
      mine.follow(want);
      tree_.clear();
      rank_.assign(B_, -1);  // -1: not a member
      for (size_t i = 0; i < order_.size(); ++i) rank_[order_[i]] = (int32_t)i;
      ids_.clear();
      for (int x = 0; x < B_; ++x)
        if (rank_[x] >= 0) ids_.push_back(x);
      tree_.buildByRank(std::move(ids_), std::move(rank_), &cancel_, seq_);
      if (!cancel_.load(std::memory_order_relaxed)) {
        {
          std::lock_guard<std::mutex> l(mu_);
          tDone_ = std::chrono::steady_clock::now();
          done_ = gen;
        }
        cvDone_.notify_one();
      }
    }
  }
  Tree tree_;
  std::vector<int32_t> next_, order_, rank_;
  std::vector<int> ids_;
  int nextB_ = 0, B_ = 0;
  bool nextSeq_ = true, seq_ = true;  // the tree's in-order sequence is wanted (RbTreeSet::buildByRank)
  CpuMask nextMask_;                  // the submitter's CPU mask (guarded by mu_)
  uint64_t gen_ = 0;   // submissions (guarded by mu_)
  uint64_t done_ = 0;  // the submission whose tree is complete in tree_ (guarded by mu_)
  std::atomic<bool> cancel_{false};
  std::chrono::steady_clock::time_point tSubmit_, tStart_, tDone_;  // (guarded by mu_)
  std::mutex mu_;
  std::condition_variable cv_, cvDone_;
  bool stop_ = false;
  std::thread th_;
};

// The process-wide helper pool: threads are created on demand up to the cap and kept for reuse.
class TreeWorkerPool {
 public:
  static TreeWorkerPool& get() {
    static TreeWorkerPool* p = new TreeWorkerPool();  // never destroyed: idle workers are parked on a condition variable
    return *p;
  }
  std::unique_ptr<TreeWorker> lease() {
    std::lock_guard<std::mutex> l(mu_);
    if (!free_.empty()) {
      auto w = std::move(free_.back());
      free_.pop_back();
      return w;
    }
    if (live_ >= cap_) return nullptr;
    ++live_;
    return std::make_unique<TreeWorker>();
  }
  void give(std::unique_ptr<TreeWorker> w) {
    if (!w) return;
    w->cancel();
    std::lock_guard<std::mutex> l(mu_);
    free_.push_back(std::move(w));
  }

 private:
  TreeWorkerPool() {
    const char* e = std::getenv("CCMI_TREE_WORKERS");
    cap_ = e ? std::max(0, std::atoi(e)) : 8;
  }
  std::mutex mu_;
  std::vector<std::unique_ptr<TreeWorker>> free_;
  int live_ = 0, cap_ = 8;
};
struct TreeLease {  // one move-out call's worker (or none)
  std::unique_ptr<TreeWorker> w;
  ~TreeLease() { TreeWorkerPool::get().give(std::move(w)); }
};

class ResourceDistribution : public GoalImpl {
 public:
  explicit ResourceDistribution(int kindIn) {
    kind = kindIn;
    switch (kindIn) {
      case CCMI_GOAL_CPU_USAGE_DISTRIBUTION: res = R_CPU; name = "CpuUsageDistributionGoal"; break;
      case CCMI_GOAL_NW_IN_USAGE_DISTRIBUTION: res = R_NW_IN; name = "NetworkInboundUsageDistributionGoal"; break;
      case CCMI_GOAL_NW_OUT_USAGE_DISTRIBUTION: res = R_NW_OUT; name = "NetworkOutboundUsageDistributionGoal"; break;
      default: res = R_DISK; name = "DiskUsageDistributionGoal"; break;
    }
  }
  int res = 0;
  double upperThr = 0, lowerThr = 0;
  bool fix = false;
  bool exclAlive = false;                 // an alive broker is excluded for replica moves
  bool posCap = true;                     // every broker has a positive capacity of `res`
  bool lowUtil = false;                   // _isLowUtilization
  ccmi_provision_recommendation overRec{};  // _overProvisionedRecommendation
  Model::SnapTable snapTab;  // moveIn's candidate-broker snapshots (one Spec per phase)
  Model::SnapTable swapTab;  // the swap phase's polled brokers' limit-free snapshots
  std::vector<uint8_t> queued;  // moveInLeadership: a group's broker is in the candidate queue (other entries: stale)
  // leadership move-out on a materialised tree: contains() per broker memoised for one scan's rows
  std::vector<uint32_t> containsStamp_;
  std::vector<uint8_t> containsVal_;
  uint32_t containsGen_ = 0;
  int nameBase() const { return 4 * kind; }
  int nameId(bool reverse, bool leader) const { return nameBase() + (reverse ? 1 : 0) + (leader ? 2 : 0); }
  bool excluded(int b) const { return !allowed[b]; }

  // isLoadAboveBalanceLowerLimit / isLoadUnderBalanceUpperLimit with a null load (:880-927): for a host resource the
  // host or the broker within the limit
  bool aboveLower(const Model& m, int b) const {
    const bool broker = m.bu(b, res) + 0 >= m.cap(b, res) * lowerThr;
    return isHostRes(res) && m.sharedHosts ? (m.hu(b, res) + 0 >= m.hcap(b, res) * lowerThr) || broker : broker;
  }
  bool underUpper(const Model& m, int b, double thr) const {
    const bool broker = m.bu(b, res) - 0 <= m.cap(b, res) * thr;
    return isHostRes(res) && m.sharedHosts ? (m.hu(b, res) - 0 <= m.hcap(b, res) * thr) || broker : broker;
  }
  // ClusterModel.aliveBrokersUnderThreshold / aliveBrokersOverThreshold membership (ClusterModel.java:1080-1126) of
  // an alive broker: the broker check for a broker resource, the host check for a host resource
  bool underThreshold(const Model& m, int x, double thr) const {
    if (isBrokerRes(res) && m.bu(x, res) >= m.cap(x, res) * thr) return false;
    return !(isHostRes(res) && m.hu(x, res) >= m.hcap(x, res) * thr);
  }
  bool overThreshold(const Model& m, int x, double thr) const {
    if (isBrokerRes(res) && m.bu(x, res) <= m.cap(x, res) * thr) return false;
    return !(isHostRes(res) && m.hu(x, res) <= m.hcap(x, res) * thr);
  }
  // host and broker decide membership differently (brokers sharing a host): no (pct, id)-prefix shortcuts
  bool hostMembership(const Model& m) const { return m.sharedHosts && isHostRes(res); }
  int cmpBroker(const Model& m, int x, int y) const {
    const int c = jcmpDouble(m.pct(x, res), m.pct(y, res));
    return c ? c : jcmpInt(m.bId[x], m.bId[y]);
  }

  std::vector<int> brokersToBalance(Engine& e) override {
    if (e.m.numNew == 0) return GoalImpl::brokersToBalance(e);
    std::vector<int> v;
    for (int b = 0; b < e.m.B; ++b)
      if (e.m.isNew(b)) v.push_back(b);
    return v;
  }

  // initGoalState (:234-278)
  void init(Engine& e) override {
    Model& m = e.m;
    allowed.assign(m.B, 0);
    int n = 0;
    for (int b = 0; b < m.B; ++b)
      if (m.alive(b) && !(e.opt.anyExclMove && e.opt.exclMove[b])) {
        allowed[b] = 1;
        n++;
      }
    if (n == 0)
      throw OptimizationFailure("[" + name + "] All alive brokers are excluded from replica moves.", underBrokers(m.maxRf));
    exclAlive = false;
    posCap = true;
    for (int b = 0; b < m.B; ++b) {
      exclAlive |= m.alive(b) && !allowed[b];
      posCap &= m.cap(b, res) > 0;
    }
    fix = false;
    const double util = m.clusterUtil(res);
    const double capacity = m.capacityWithAllowedReplicaMoves(res, e.opt.exclMove);
    const double avgPct = util / capacity;
    upperThr = e.threshold(avgPct, res, false);
    lowerThr = e.threshold(avgPct, res, true);
    lowUtil = avgPct <= e.bc.lowUtil[res];
    if (lowUtil) {
      // the over-provisioned recommendation with a typical broker of maximal capacity, first in the
      // _brokersAllowedReplicaMove HashSet<Integer> order (ResourceDistributionGoal.java:262-296)
      std::vector<int> ids, ord;
      for (int b = 0; b < m.B; ++b)
        if (allowed[b]) ids.push_back(b);
      javaHashSetOrder(ids, ord);
      int typical = -1;
      double maxCapacity = 0.0;
      for (int b : ord)
        if (m.cap(b, res) > maxCapacity) {
          typical = b;
          maxCapacity = m.cap(b, res);
        }
      const double typicalCapacity = m.cap(typical, res);
      const int allowedNumBrokers = (int)(util / e.bc.lowUtil[res] / typicalCapacity);
      overRec = provisionRec(CCMI_PROVISION_OVER_PROVISIONED);
      overRec.num_brokers = std::max(n - allowedNumBrokers, 1);
      overRec.typical_broker_capacity = typicalCapacity;
      overRec.typical_broker_id = m.bId[typical];
      overRec.resource = res;
    }
    dg = DevGoal{};
    dg.kind = DG_RESOURCE_DISTRIBUTION;
    dg.resource = res;
    dg.upperThr = upperThr;
    dg.lowerThr = lowerThr;
    dg.fixOffline = 0;
    dg.allowedSlot = e.newSlot;
  }

  // updateGoalState (:301-349)
  void update(Engine& e) override {
    Model& m = e.m;
    bool anyAboveUpper = false, anyUnderLower = false;
    for (int b = 0; b < m.B; ++b) {
      if (!m.alive(b)) continue;
      if (!underUpper(m, b, upperThr)) anyAboveUpper = true;
      if (!excluded(b) && !aboveLower(m, b)) anyUnderLower = true;
    }
    if (anyAboveUpper) succeeded = false;
    else if (lowUtil) prov = provisionResponse(CCMI_PROVISION_OVER_PROVISIONED, overRec);
    if (anyUnderLower) succeeded = false;
    else if (!anyAboveUpper && !lowUtil) prov = provisionResponse(CCMI_PROVISION_RIGHT_SIZED);
    for (int r = 0; r < m.R; ++r)
      if (m.selfHealing[r] && m.curOffline(r)) {
        if (fix)  // GoalUtils.ensureNoOfflineReplicas rethrown
          throw OptimizationFailure("[" + name + "] Cannot remove replica from broker " + std::to_string(m.bId[m.rBroker[r]]),
                                    underBrokers(1));
        fix = true;
        dg.fixOffline = 1;
        return;
      }
    finished = true;
  }

  int compareStats(const ccmi_cluster_stats& after, const ccmi_cluster_stats& before) const override {
    const int n1 = after.num_balanced_brokers_by_resource[res], n2 = before.num_balanced_brokers_by_resource[res];
    if (n2 > n1 && jcmpDouble(before.resource_std[res], after.resource_std[res]) < 0) return -1;
    return 1;
  }

  // rebalanceForBroker (:379-435)
  void rebalance(Engine& e, int b) override {
    Model& m = e.m;
    const int off = m.bNoff[b];
    const bool excl = excluded(b);
    bool less = off > 0 || excl || !underUpper(m, b, upperThr);
    bool more = !excl && !aboveLower(m, b);
    bool immOnly = false;
    if (m.bNoff[b] == 0) {
      if (!more && !less) return;
      immOnly = m.numSelfHealing > 0 || e.opt.onlyImmigrants;
      if (immOnly && less && m.bNimm[b] == 0) return;
    }
    if ((res == R_NW_OUT || res == R_CPU) && !(fix && m.bNoff[b] > 0)) {
      if (less && !moveOut(e, b, DA_LEADERSHIP)) less = false;
      if (more && !moveIn(e, b, DA_LEADERSHIP, false)) more = false;
    }
    bool unbalanced = false;
    if (less && moveOut(e, b, DA_MOVE)) unbalanced = swapOut(e, b, immOnly);
    if (more && moveIn(e, b, DA_MOVE, immOnly)) unbalanced = unbalanced || swapIn(e, b, immOnly);
  }

  // sortedCandidateReplicas (:543-569)
  int trackCandidates(Engine& e, int b, double limit, bool asc, bool followersOnly, bool leadersOnly, bool immOnly) {
    const int id = nameId(!asc, leadersOnly);
    e.m.track(b, id, candidateSpec(e, limit, asc, followersOnly, leadersOnly, immOnly));
    return id;
  }
  Model::Spec candidateSpec(Engine& e, double limit, bool asc, bool followersOnly, bool leadersOnly, bool immOnly) {
    Model& m = e.m;
    Model::Spec s;
    s.selFollowers = followersOnly;
    s.selLeaders = leadersOnly;
    s.selImmigrants = immOnly;
    s.selExclTopics = e.opt.anyExclTopic;
    s.prioOffline = m.numSelfHealing > 0;
    if (asc) {
      if (limit < 1.7976931348623157e308) {
        s.selBelowRes = res;
        s.belowLimit = limit;
      }
      s.scoreReverse = false;
    } else {
      s.selAboveRes = res;
      s.aboveLimit = limit;
      s.scoreReverse = true;
    }
    s.scoreRes = res;
    return s;
  }

  double firstOnlineLoad(const Model& m, const std::vector<int32_t>& v, bool wantMax) const {
    double x = m.ru(v.front(), res);
    for (int r : v) {
      if (m.curOffline(r)) continue;
      if (wantMax ? m.ru(r, res) > x : m.ru(r, res) < x) x = m.ru(r, res);
      break;
    }
    return x;
  }

  // rebalanceByMovingLoadOut (:779-863)
  //
  // The candidate TreeSet (sortedAliveBrokersUnderThreshold, keyed on LIVE utilization) is emulated without
  // materialising it while that is provably exact: its in-order walk is the maintained (pct, id) order
  // filtered by membership, and TreeMap.remove(dst) after dst's key moved from k to k' finds dst's node
  // whenever no other member's key lies strictly between k and k' (every ancestor then sends the search for
  // k' the same way it sent k). When that does not hold, the exact tree is built by replaying the entry
  // state and every remove/add so far with the keys each broker had at that time, and the reference's
  // stale-key behaviour follows from the real structure.
  bool moveOut(Engine& e, int b, int action) {
    PhaseScope ps(PH_RES_OUT);
    Model& m = e.m;
    std::vector<std::pair<int, double>> ovr;  // brokers whose key differs from the live one during a replay
    auto key = [&](int x) {
      for (const auto& o : ovr)
        if (o.first == x) return o.second;
      return m.pct(x, res);
    };
    auto cmp = [&](int x, int y) {
      const int c = jcmpDouble(key(x), key(y));
      return c ? c : jcmpInt(m.bId[x], m.bId[y]);
    };
    RbTreeSet<decltype(cmp)> cand(cmp);
    bool built = false;
    std::vector<uint8_t>& inSet = e.scratchB;
    inSet.assign(m.B, 0);
    std::vector<int32_t> inorder;
    {
      PhaseScope pi(PH_PQ_INIT);
      const auto& ord = m.brokersByPct(res);
      auto under = [&](int x) { return fix || underThreshold(m, x, upperThr); };  // aliveBrokersUnderThreshold
      if (m.numDead == 0 && posCap && !ord.empty() && upperThr > 0 && !hostMembership(m)) {
        // every broker alive with a positive capacity: membership is a prefix of the (pct, id) order except within a
        // relative 1e-9 band around the threshold, where the exact product test decides each broker
        size_t lo = (size_t)(std::partition_point(ord.begin(), ord.end(),
                                                  [&](int x) { return m.pct(x, res) < upperThr * (1 - 1e-9); }) -
                             ord.begin());
        size_t hi = (size_t)(std::partition_point(ord.begin() + lo, ord.end(),
                                                        [&](int x) { return m.pct(x, res) <= upperThr * (1 + 1e-9); }) -
                                   ord.begin());
        if (fix) lo = hi = ord.size();
        inorder.assign(ord.begin(), ord.begin() + lo);
        for (size_t k = lo; k < hi; ++k)
          if (under(ord[k])) inorder.push_back(ord[k]);
        for (int x : inorder) inSet[x] = 1;
      } else {
        for (int x : ord) {
          if (!m.alive(x) || !under(x)) continue;
          inSet[x] = 1;
          inorder.push_back(x);
        }
      }
    }
    // The entry tree is built on a helper thread from the call's entry on (it runs beside this call's host work and
    // scans; materialise() adopts it), for clusters of at least CCMI_TREE_WORKER_MIN brokers (2048); CCMI_TREE_WORKER=0
    // builds on this thread instead, a few puts per poll of the in-flight scans (Device::idleWork). Read per call.
    const char* wEnv = std::getenv("CCMI_TREE_WORKER");
    const char* minEnv = std::getenv("CCMI_TREE_WORKER_MIN");
    TreeLease lease;
    if (!(wEnv && wEnv[0] == '0') && m.B >= (minEnv ? std::atoi(minEnv) : 2048)) lease.w = TreeWorkerPool::get().lease();
    const bool useWorker = lease.w != nullptr;
    // `inorder` is the members' entry (key, id) order; the leadership form only searches the tree
    if (useWorker) lease.w->submit(inorder, m.B, action != DA_LEADERSHIP);
    const int64_t relocBeforeEntry = m.lastRelocNs;  // CCMI_PROFILE: how long the entry state had been final
    struct Step {
      int dst;
      double keyAfter;
      bool add;
      double bKeyAfter;  // b's key after the move (b may be a member whose node keeps its entry position)
    };
    std::vector<Step> hist;
    std::vector<std::pair<int, double>> entryKey;  // pct at entry of every broker a move changed
    std::vector<uint8_t> entryIn;
    auto noteEntry = [&](int x) {
      for (const auto& o : entryKey)
        if (o.first == x) return;
      entryKey.push_back({x, m.pct(x, res)});
    };
    std::vector<int32_t> rank;
    int specState = 0;  // the speculative entry-tree build: 0 not started, 1 puts in progress, 2 complete
    std::vector<int32_t> entryOrder;
    auto materialise = [&]() {
      PhaseScope pi(PH_TREE_BUILD);
      // CCMI_PROFILE: nanoseconds in the order construction (16), the put sequence (17) and the replay (18)
      const bool tp = prof().on;
      auto tnow = [] { return std::chrono::steady_clock::now(); };
      auto ns = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
        return (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count();
      };
      auto t0 = tp ? tnow() : std::chrono::steady_clock::time_point();
      auto t1 = t0;
      ovr = entryKey;
      if (useWorker) {
        if (tp && relocBeforeEntry > 0) {  // the entry state was final this long before the tree was wanted
          const int64_t lead =
              (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t0.time_since_epoch()).count() -
              relocBeforeEntry;
          prof().count(51, "out.tree.lead.ns", std::min<int64_t>(lead, 1000000));
          if (lead >= 150000) prof().count(63, "out.tree.lead.ge150us", 1);
        }
        cand.adopt(lease.w->take());
      } else if (specState > 0) {  // the entry tree was started while scans were in flight: finish its puts
        if (tp) t1 = tnow();
        cand.buildStep((size_t)-1);
        prof().count(19, "tree.spec.finished", 1);
      } else {
        // Entry-time (key, id) order of the members: the maintained live order with the few brokers whose key
        // moved since entry put back at their entry keys; the tree is then built by the same put sequence (ids in
        // aliveBrokers order) with integer rank compares.
        std::vector<int32_t> order;
        order.reserve(m.B);
        std::vector<uint8_t>& changed = e.scratchB2;
        changed.assign(m.B, 0);
        for (const auto& o : entryKey) changed[o.first] = 1;
        for (int x : m.brokersByPct(res))
          if (entryIn[x] && !changed[x]) order.push_back(x);
        // the changed members sorted by their entry keys, merged into the unchanged ones (whose live key is the
        // entry key)
        std::vector<std::pair<int, double>> moved;
        for (const auto& o : entryKey)
          if (entryIn[o.first]) moved.push_back(o);
        auto lessKey = [&](double ka, int a, double kb, int bb) {
          const int c = jcmpDouble(ka, kb);
          return c ? c < 0 : m.bId[a] < m.bId[bb];
        };
        std::sort(moved.begin(), moved.end(), [&](const std::pair<int, double>& x, const std::pair<int, double>& y) {
          return lessKey(x.second, x.first, y.second, y.first);
        });
        std::vector<int32_t> merged;
        merged.reserve(order.size() + moved.size());
        size_t u = 0;
        for (const auto& o : moved) {
          while (u < order.size() && lessKey(m.pct(order[u], res), order[u], o.second, o.first)) merged.push_back(order[u++]);
          merged.push_back(o.first);
        }
        while (u < order.size()) merged.push_back(order[u++]);
        order.swap(merged);
        rank.assign(m.B, 0);
        for (size_t i = 0; i < order.size(); ++i) rank[order[i]] = (int32_t)i;
        std::vector<int> ids;
        ids.reserve(order.size());
        for (int x = 0; x < m.B; ++x)
          if (entryIn[x]) ids.push_back(x);
        if (tp) t1 = tnow();
        cand.buildByRank(ids, rank);
      }
      auto t2 = tp ? tnow() : t0;
      // The leadership form only searches the set: no in-order sequence. The replica-move form walks the set in order
      // for every candidate list: the build's sequence is kept through a short replay (each step shifts it once),
      // a long replay runs without it and the sequence is taken once afterwards (a walk over every node).
      if (action == DA_LEADERSHIP || hist.size() > 4) cand.untrackSequence();
      prof().count(15, "tree.replay.steps", (int64_t)hist.size());
      for (const Step& h : hist) {
        for (auto& o : ovr) {
          if (o.first == h.dst) o.second = h.keyAfter;
          if (o.first == b) o.second = h.bKeyAfter;
        }
        cand.remove(h.dst);
        if (h.add) cand.add(h.dst);
      }
      if (action != DA_LEADERSHIP) cand.trackSequence();
      if (tp) {
        prof().count(16, "tree.ns.order", ns(t0, t1));
        prof().count(17, "tree.ns.build", ns(t1, t2));
        prof().count(18, "tree.ns.replay", ns(t2, tnow()));
      }
      ovr.clear();
      built = true;
    };
    // b's own key changes with every move while its node stays where it was put. The replica-move form keeps
    // the lazy order with b at that position as long as every member's live key still fits its place in the order
    // (checked after each move); the leadership form, which keeps no order, builds the tree.
    entryIn = inSet;
    if (inSet[b] && action == DA_LEADERSHIP) materialise();
    // While this call's scans are in flight (Device::idleWork) the entry tree's put sequence is started from the entry
    // order, a bounded number of puts per poll, so a later materialise() has fewer puts left (or none).
    const Device::IdleScope idleScope{e.dev};
    const size_t treePuts = idleTreePuts();
    if (!built && !useWorker && treePuts > 0) {
      entryOrder.assign(inorder.begin(), inorder.end());
      e.dev->idleWork = [&]() {
        if (built || specState == 2) return false;
        if (specState == 0) {
          std::vector<int32_t> rk(m.B, 0);
          for (size_t i = 0; i < entryOrder.size(); ++i) rk[entryOrder[i]] = (int32_t)i;
          std::vector<int> ids;
          ids.reserve(entryOrder.size());
          for (int x = 0; x < m.B; ++x)
            if (entryIn[x]) ids.push_back(x);
          cand.buildStart(std::move(ids), std::move(rk));
          specState = 1;
          return true;
        }
        if (cand.buildStep(treePuts)) specState = 2;
        return specState == 1;
      };
    }
    auto memberBetween = [&](int dst, double k0, double k1) {
      // is a member other than dst strictly between (k0, id(dst)) and (k1, id(dst)) in (pct, id) order?
      const double lo = jcmpDouble(k0, k1) <= 0 ? k0 : k1, hi = jcmpDouble(k0, k1) <= 0 ? k1 : k0;
      const int id = m.bId[dst];
      auto cmpKey = [&](int x, double k) {
        const int c = jcmpDouble(m.pct(x, res), k);
        return c ? c : jcmpInt(m.bId[x], id);
      };
      const auto& ord = m.brokersByPct(res);
      auto it = std::partition_point(ord.begin(), ord.end(), [&](int x) { return cmpKey(x, lo) <= 0; });
      for (; it != ord.end() && cmpKey(*it, hi) < 0; ++it)
        if (*it != dst && inSet[*it]) return true;
      return false;
    };
    const bool lead = action == DA_LEADERSHIP;
    const bool selfHealing = m.numSelfHealing > 0;
    Model::Spec s;
    s.selLeaders = lead;
    s.selImmigrants = e.opt.onlyImmigrants;
    s.selImmOrOffline = selfHealing && m.alive(b);
    s.selExclTopics = e.opt.anyExclTopic;
    s.prioOffline = selfHealing;
    s.prioImmigrants = !e.opt.onlyImmigrants;
    s.scoreRes = res;
    s.scoreReverse = true;
    const int id = nameId(true, lead);
    m.track(b, id, s);
    std::vector<int32_t> list = m.sorted(b, id);  // clone
    // the loop breaks at the first online replica with zero utilization (static during the loop)
    size_t z = 0;
    while (z < list.size() && (m.curOffline(list[z]) || m.ru(list[z], res) != 0.0)) ++z;
    list.resize(z);
    const double upperSrc = excluded(b) ? 0 : upperThr;
    std::vector<int32_t> cands, pr, pb, fol;
    std::vector<int32_t> pairOwner;
    // Leadership form: each row's candidate brokers (its online followers that are members, eligible, in live (key, id)
    // order) are kept between scans. Before the set is materialised only dst's membership and key change per accept
    // (b leads every row), so only rows with dst among their followers are rebuilt; after it, every row is (a search in
    // the stale-key tree may change for any broker).
    std::vector<std::vector<int32_t>> rowCands, rowFol;
    std::vector<uint8_t> rowValid, rowFolSet;
    if (lead) {
      rowCands.resize(list.size());
      rowValid.assign(list.size(), 0);
      rowFol.resize(list.size());
      rowFolSet.assign(list.size(), 0);
    }
    size_t i = 0;
    while (i < list.size()) {
      int dst = -1;
      size_t hitIdx = 0;
      if (!lead) {
        const std::vector<int32_t>* cl;
        {
          PhaseScope pc(PH_CAND_BUILD);
          // built: the tree's maintained sequence itself (no copy); else the lazy order, kept up to date below
          const std::vector<int32_t>* seq = built ? cand.sequence() : &inorder;
          if (!seq) {
            cand.inorder(inorder);
            seq = &inorder;
          }
          cl = &e.eligibleView(*seq, DA_MOVE, cands);
        }
        const int64_t key = e.crossScan(*this, DA_MOVE, list, i, *cl);
        if (key < 0) break;
        const int N = (int)cl->size();
        hitIdx = i + (size_t)(key / N);
        dst = (*cl)[key % N];
      } else {
        {
          PhaseScope pc(PH_CAND_BUILD);
          pr.clear();
          pb.clear();
          pairOwner.clear();
          // the tree does not change within one scan's rows: each broker's search runs once per scan (generation-
          // stamped memo, never cleared); a row's online followers do not change while b moves its leaders (a
          // leadership move touches only its own partition), so they are taken once per row
          if (built && ++containsGen_ == 0) {
            containsStamp_.assign(m.B, 0);
            containsGen_ = 1;
          }
          if (built && containsStamp_.size() != (size_t)m.B) containsStamp_.assign(m.B, 0);
          if (built && containsVal_.size() != (size_t)m.B) containsVal_.assign(m.B, 0);
          auto inCand = [&](int fb) {
            if (!built) return inSet[fb] != 0;
            if (containsStamp_[fb] != containsGen_) {
              containsStamp_[fb] = containsGen_;
              containsVal_[fb] = cand.contains(fb) ? 1 : 0;
            }
            return containsVal_[fb] != 0;
          };
          for (size_t q = i; q < list.size(); ++q) {
            const int r = list[q];
            std::vector<int32_t>& rc = rowCands[q];
            if (built || !rowValid[q]) {
              std::vector<int32_t>& rf = rowFol[q];
              if (!rowFolSet[q]) {
                m.onlineFollowerBrokers(m.rPart[r], rf);
                rowFolSet[q] = 1;
              }
              inorder.clear();
              for (int fb : rf)
                if (inCand(fb)) inorder.push_back(fb);
              std::sort(inorder.begin(), inorder.end(), [&](int x, int y) { return cmpBroker(m, x, y) < 0; });
              inorder.erase(std::unique(inorder.begin(), inorder.end()), inorder.end());
              e.eligible(inorder, DA_LEADERSHIP, rc);
              rowValid[q] = 1;
            }
            for (int fb : rc) {
              pr.push_back(r);
              pb.push_back(fb);
              pairOwner.push_back((int)q);
            }
          }
        }
        const int64_t key = e.pairScan(*this, pr, pb);
        if (key < 0) break;
        hitIdx = (size_t)pairOwner[key];
        dst = pb[key];
      }
      const double dstBefore = m.pct(dst, res);
      if (!built) {
        noteEntry(b);
        noteEntry(dst);
      }
      if (!lead) m.relocateReplica(m.rPart[list[hitIdx]], b, dst);
      else m.relocateLeadership(m.rPart[list[hitIdx]], b, dst);
      if (underUpper(m, b, upperSrc) && !(fix && m.bNoff[b] > 0)) {
        prof().count(10, "out.done");
        m.clearTracked(b);
        return false;
      }
      const bool add = m.pct(dst, res) < upperThr;
      prof().count(lead ? 6 : 7, lead ? "out.lead.accept" : "out.move.accept");
      if (built) prof().count(8, "out.built.accept");
      if (!built) {
        // The set is a consistent search tree iff its in-order sequence is sorted by the LIVE (key, id): then
        // TreeMap.remove(dst) finds dst's node and add(dst) puts it at its sorted place. Only b's and dst's keys
        // moved since the sequence was last sorted, so it is sorted iff each of them still fits between its
        // neighbours (leadership form: no member strictly between dst's old and new key, b being no member).
        bool clean;
        size_t at = 0;
        auto less = [&](int x, int y) { return m.cmpBrokerPct(res, x, y) < 0; };
        if (lead) {
          clean = !memberBetween(dst, dstBefore, m.pct(dst, res));
        } else {
          PhaseScope pc(PH_CAND_BUILD);
          const size_t n = inorder.size();
          at = (size_t)(std::find(inorder.begin(), inorder.end(), dst) - inorder.begin());
          if (at == n) throw std::logic_error("moveOut: the lazy candidate order lost its destination");
          auto fits = [&](size_t k) {
            return (k == 0 || less(inorder[k - 1], inorder[k])) && (k + 1 == n || less(inorder[k], inorder[k + 1]));
          };
          clean = fits(at);
          if (clean && inSet[b]) {
            const size_t bj = (size_t)(std::find(inorder.begin(), inorder.end(), b) - inorder.begin());
            clean = bj == n || fits(bj);
          }
        }
        if (!clean) {
          prof().count(9, "out.materialise");
          materialise();
        } else {
          hist.push_back({dst, m.pct(dst, res), add, m.pct(b, res)});
          inSet[dst] = add ? 1 : 0;
          if (!lead) {
            PhaseScope pc(PH_CAND_BUILD);
            inorder.erase(inorder.begin() + (ptrdiff_t)at);
            if (add) inorder.insert(std::lower_bound(inorder.begin(), inorder.end(), dst, less), dst);
          } else {
            for (size_t q = hitIdx + 1; q < list.size(); ++q)
              if (rowValid[q] && m.replicaOn(m.rPart[list[q]], dst) >= 0) rowValid[q] = 0;
          }
          i = hitIdx + 1;
          continue;
        }
      }
      cand.remove(dst);
      if (add) cand.add(dst);
      i = hitIdx + 1;
    }
    m.clearTracked(b);
    return m.nrep(b) != 0;
  }

  // a candidate broker of rebalanceByMovingLoadIn's queue (:450-462): alive, utilization above the lower threshold
  // (above 0 for a broker excluded for replica moves)
  bool moveInMember(const Model& m, int c) const {
    return m.alive(c) && m.pct(c, res) > (excluded(c) ? 0.0 : lowerThr);
  }

  // rebalanceByMovingLoadIn (:437-526): speculative multi-candidate-broker batches over the live views
  bool moveIn(Engine& e, int b, int action, bool immOnly) {
    PhaseScope ps(PH_RES_IN);
    Model& m = e.m;
    if (m.numNew > 0 && !m.isNew(b)) return true;
    const bool followersOnly = e.opt.anyExclLead && e.opt.exclLead[b];
    auto rcmp = [this, &m](int x, int y) { return cmpBroker(m, y, x); };
    // SortedReplicas are lazily initialised (SortedReplicas.java:47-193) and every key change re-inserts the
    // replica, so a polled candidate broker's live view is the snapshot of a fresh initialisation: nothing needs
    // to be tracked (the reference restarts its live iteration with indicesToSkip after an accept, :484-522).
    const Model::Spec spec = candidateSpec(e, 0.0, false, followersOnly, res == R_NW_OUT, immOnly);
    LiveQueue<decltype(rcmp)> pq(rcmp);
    {
      PhaseScope pi(PH_PQ_INIT);
      const auto& ord = m.brokersByPct(res);
      auto member = [&](int c) { return moveInMember(m, c); };
      // only b's key changes while brokers are queued (moves go cb -> b, cb polled): exact unless b is queued
      pq.init(m.B, !member(b));
      if (pq.ordered() && m.numDead == 0 && !exclAlive && !ord.empty() && m.pct(ord.back(), res) == m.pct(ord.back(), res)) {
        // every broker is alive and allowed, and no key is NaN: the members are exactly the suffix of the (pct, id)
        // order above the lower threshold, queued in reverse
        const auto first = std::partition_point(ord.begin(), ord.end(), [&](int c) { return !(m.pct(c, res) > lowerThr); });
        pq.sortedRun().assign(ord.rbegin(), std::make_reverse_iterator(first));
      } else {
        for (auto it = ord.rbegin(); it != ord.rend(); ++it)
          if (member(*it)) pq.push_sorted(*it);
      }
      if (!pq.ordered())
        for (int c = 0; c < m.B; ++c)
          if (member(c)) pq.add(c);
    }
    std::vector<int32_t> single{b}, cands;
    e.eligible(single, action, cands);
    // b outside the eligible set (e.g. not a requested destination): every polled replica visits an empty
    // candidate list, nothing moves and nothing is counted — the loop's outcome without walking every broker
    if (cands.empty()) return true;
    if (action == DA_LEADERSHIP && pq.ordered()) return moveInLeadership(e, b, pq, spec);
    if (action == DA_MOVE && pq.ordered() && e.queueReady(*this, action, spec)) return moveInQueue(e, b, pq, spec, cands);
    // rows: the current broker's remaining view, then the polled brokers' snapshots (device-resident segments)
    using Seg = SnapSeg;
    auto segLen = [](const Seg& x) { return x.v->size() > x.skip ? x.v->size() - x.skip : 0; };
    std::vector<Seg> segs;
    size_t target = kFirstBatchRows;
    bool haveCur = false;
    Seg cur{nullptr, 0, 0};
    auto cond = [&]() { return action == DA_MOVE || m.bNlead[b] != m.nrep(b); };
    while (haveCur || (!pq.empty() && cond())) {
      size_t rows = 0;
      {
        PhaseScope pf(PH_FLATTEN);
        segs.clear();
        if (haveCur) {
          cur.v = m.snapshotInShared(snapTab, cur.cb, spec);
          segs.push_back(cur);
          rows += segLen(cur);
          haveCur = false;
        }
        while (!pq.empty() && (segs.empty() || rows < target) && segs.size() < (size_t)kMaxSegs && cond()) {
          const int cb = pq.poll();
          segs.push_back({m.snapshotInShared(snapTab, cb, spec), cb, 0});
          rows += segLen(segs.back());
        }
      }
      if (segs.empty()) break;
      // while the scan is in flight, the snapshots of the next brokers the queue will poll (cached per broker version,
      // so an unused one costs only host time that would otherwise be spent waiting)
      size_t ahead = 0;
      const Device::IdleScope idleScope{e.dev};
      e.dev->idleWork = [&]() {
        const int cb = pq.upcoming(ahead);
        if (cb < 0 || ahead >= kIdleSnapshots) return false;
        ++ahead;
        (void)m.snapshotInShared(snapTab, cb, spec);
        return true;
      };
      const int64_t key = cands.empty() ? -1 : e.crossScanSegs(*this, action, segs, cands);
      e.dev->idleWork = nullptr;  // (idleScope also clears it on a throw)
      if (key < 0) {
        target = std::min<size_t>(target * kBatchGrowth, kMaxBatchRows);
        continue;
      }
      target = kFirstBatchRows;
      size_t q = (size_t)key, mi = 0;
      while (q >= segLen(segs[mi])) {
        q -= segLen(segs[mi]);
        ++mi;
      }
      const Seg hit = segs[mi];
      const size_t idx = hit.skip + q;  // index in cb's live view == iteratedIndices at the hit
      const int r = (*hit.v)[idx];
      if (action == DA_MOVE) m.relocateReplica(m.rPart[r], hit.cb, b);
      else m.relocateLeadership(m.rPart[r], hit.cb, b);
      if (aboveLower(m, b)) {
        prof().count(action == DA_MOVE ? 0 : 3, action == DA_MOVE ? "in.move.done" : "in.lead.done");
        return false;
      }
      for (size_t t = segs.size(); t-- > mi + 1;) pq.unpoll(segs[t].cb);  // un-poll speculative brokers
      if (!pq.empty() && m.pct(hit.cb, res) < m.pct(pq.peek(), res)) {
        prof().count(action == DA_MOVE ? 1 : 4, action == DA_MOVE ? "in.move.readd" : "in.lead.readd");
        pq.add(hit.cb);
      } else {
        prof().count(action == DA_MOVE ? 2 : 5, action == DA_MOVE ? "in.move.continue" : "in.lead.continue");
        cur = {nullptr, hit.cb, idx};
        haveCur = true;
      }
    }
    return true;
  }

  // rebalanceByMovingLoadIn for INTER_BROKER_REPLICA_MOVEMENT (:437-526) with an ordered candidate queue, one device
  // command per accepted move: the reference polls candidate brokers in (utilization %, id) descending order and walks
  // each one's live sorted-replica view (restarting it after an accept, :484-522) until a replica is accepted into b.
  // The rows of EVERY queued broker go to the device in one queue scan (Engine::queueScan), in poll order, so the
  // scan's first fit is the reference's next accept however deep in the queue it lies; brokers before the winner's
  // are consumed (polled, as the reference polled them), the ones after it are un-polled.
  template <class Q>
  bool moveInQueue(Engine& e, int b, Q& pq, const Model::Spec& spec, const std::vector<int32_t>& cands) {
    Model& m = e.m;
    std::vector<int32_t> merged;
    int curCb = -1, curSkip = 0;
    const int N = (int)cands.size();
    while (curCb >= 0 || !pq.empty()) {
      // the queue's poll order: its remaining sorted run as it is, or (after a re-add) every element polled in order
      const bool run = pq.runOnly();
      if (!run) {
        PhaseScope pf(PH_FLATTEN);
        merged.clear();
        while (!pq.empty()) merged.push_back(pq.poll());
      }
      const int32_t* tail = run ? pq.runData() : merged.data();
      const int nTail = (int)(run ? pq.runLeft() : merged.size());
      const int head = curCb, hasHead = head >= 0 ? 1 : 0;
      const int64_t key = e.queueScan(*this, DA_MOVE, spec, head, hasHead ? curSkip : 0, tail, nTail, cands);
      if (key < 0) return true;  // every queued broker polled, nothing accepted
      const int span = e.dev->queueSpan();
      const int64_t row = key / N;
      const int i = (int)(row / span), idx = (int)(row % span);
      const int cb = i < hasHead ? head : tail[i - hasHead];
      const int r = e.dev->qdirRows(cb)[idx];  // cb's live view == the snapshot the scan read
      // the brokers up to the winner's are polled (the reference polled them); the ones after it stay queued
      const int polled = i < hasHead ? 0 : i - hasHead + 1;
      if (run) pq.skipRun((size_t)polled);
      else
        for (int t = nTail; t-- > polled;) pq.unpoll(merged[t]);
      m.relocateReplica(m.rPart[r], cb, b);
      if (aboveLower(m, b)) {
        prof().count(0, "in.move.done");
        return false;
      }
      if (!pq.empty() && m.pct(cb, res) < m.pct(pq.peek(), res)) {
        prof().count(1, "in.move.readd");
        pq.add(cb);
        curCb = -1;
      } else {
        prof().count(2, "in.move.continue");
        curCb = cb;
        curSkip = idx;  // the reference's iteration resumes at the same index of the view without r
      }
    }
    return true;
  }

  // rebalanceByMovingLoadIn for LEADERSHIP_MOVEMENT (:437-526) with an ordered candidate queue. A row (replica r on
  // candidate broker cb) can only be accepted when GoalUtils.legitMove holds (GoalUtils.java:213-226): r is a leader
  // and b hosts a replica of r's partition — so the only acceptable rows are the leaders of b's own follower
  // partitions. Each scan sends exactly those rows to the device, in the reference's row order (the current broker's
  // remaining view first, then the queued brokers in poll order = comparator order, each in its sorted-replica
  // order); the rows between them are walked by the reference without a possible accept, so they are counted as
  // reference-equivalent candidates from the snapshot sizes but not evaluated.
  template <class Q>
  bool moveInLeadership(Engine& e, int b, Q& pq, const Model::Spec& spec) {
    Model& m = e.m;
    struct Row {
      int cb;
      size_t idx;
      int r;
    };
    std::vector<Row> rows;
    std::vector<int32_t> pr, pb;
    int curCb = -1;
    size_t curSkip = 0;
    auto cond = [&]() { return m.bNlead[b] != m.nrep(b); };
    // The candidate brokers' live views: the goal's snapshot table (host only; a view is re-derived when its broker's
    // version changes), or with CCMI_LEAD_DIR=1 the queue scans' snapshot directory, kept current for `spec` after
    // every accept — which uploads the changed brokers' rows each time instead of once before the next queue scan.
    static const bool leadDir = std::getenv("CCMI_LEAD_DIR") && std::getenv("CCMI_LEAD_DIR")[0] == '1';
    const bool dir = leadDir && e.queueOn(*this, DA_LEADERSHIP);
    if (dir) e.queueSyncSpec(spec);
    auto snap = [&](int c) -> const std::vector<int32_t>& {
      return dir ? e.dev->qdirRows(c) : m.snapshotIn(snapTab, c, spec);
    };
    auto size = [&](int c) { return dir ? e.dev->qdirRows(c).size() : m.viewSize(snapTab, c, spec); };
    auto indexOf = [&](int c, int r) {
      const auto& v = snap(c);
      const uint64_t k = m.replicaKey(spec, r);
      return (size_t)(std::lower_bound(v.begin(), v.end(), k, [&](int x, uint64_t kk) { return m.replicaKey(spec, x) < kk; }) -
                      v.begin());
    };
    // b's follower replicas grouped by the broker leading their partition (leaders move only by this loop's accepts,
    // which make b the leader): a group's rows change only when its broker's view changes (version) or b leads one of
    // its partitions, so the rows' view order is cached per group and recomputed only then
    struct Group {
      int c;
      std::vector<int32_t> rbs;
      // (sort key, leader replica) of each rbs[k]'s partition leader on c, sorted — c's view order, the view being
      // sorted by the unique Model::replicaKey — recomputed whenever c's version changes (which every accept from c
      // does: the moved partition's leader is then b, excluded at the refresh; leaders move only by this loop's
      // accepts), so between refreshes the rows need no model lookups. A row's view index itself is looked up only
      // for the current broker's rows and the winner's.
      std::vector<std::pair<uint64_t, int32_t>> byKey;
      uint32_t ver = ~0u;
    };
    constexpr size_t kNoIdx = ~(size_t)0;
    std::vector<Group> groups;
    // The groups in poll order (the queue's reversed broker comparator). Only cb's key changes between scans (leadership
    // moves cb -> b; b leads none of these partitions' leaders), so after an accept cb's group alone is re-placed and
    // the rows are the groups' sorted rows walked in this order: the order a sort of all rows by (poll order, view
    // index) gives, without the sort.
    std::vector<int> order;
    auto before = [&](int gx, int gy) { return cmpBroker(m, groups[gy].c, groups[gx].c) < 0; };
    {
      PhaseScope pf(PH_FLATTEN);
      NsScope ns(42, "lead.in.ns.setup");
      std::vector<std::pair<int, int>> lb;
      for (int rb : m.bRepl[b])
        if (!m.rLeader[rb]) lb.push_back({m.rBroker[m.pLeader[m.rPart[rb]]], rb});
      std::sort(lb.begin(), lb.end());
      for (const auto& x : lb) {
        if (groups.empty() || groups.back().c != x.first) groups.push_back(Group{x.first, {}, {}, ~0u});
        groups.back().rbs.push_back(x.second);
      }
      order.resize(groups.size());
      for (size_t i = 0; i < groups.size(); ++i) order[i] = (int)i;
      std::sort(order.begin(), order.end(), before);
      // `queued` is read for the groups' brokers only: they start queued when they are members (the ordered queue
      // holds exactly the members); polls and re-adds keep them current below
      if (queued.size() != (size_t)m.B) queued.assign(m.B, 0);
      for (const Group& g : groups) queued[g.c] = moveInMember(m, g.c) ? 1 : 0;
    }
    auto emit = [&](Group& g) {  // the group's rows in view order (recomputed on a new version)
      if (g.ver != m.bVer[g.c]) {
        NsScope ns(43, "lead.in.ns.refresh");
        prof().count(44, "lead.in.refreshes");
        g.byKey.clear();
        for (size_t k = 0; k < g.rbs.size(); ++k) {
          const int rb = g.rbs[k];
          if (m.rLeader[rb]) continue;  // b leads that partition now: no leader row elsewhere
          const int lr = m.pLeader[m.rPart[rb]];
          if (m.rBroker[lr] != g.c || !m.selects(spec, lr)) continue;
          g.byKey.push_back({m.replicaKey(spec, lr), (int32_t)lr});
        }
        std::sort(g.byKey.begin(), g.byKey.end());
        g.ver = m.bVer[g.c];
      }
      if (g.c == curCb) {  // the current broker's view resumes at index curSkip (reference iteratedIndices)
        for (const auto& e : g.byKey) {
          const size_t idx = indexOf(g.c, e.second);
          if (idx >= curSkip) rows.push_back({g.c, idx, e.second});
        }
        return;
      }
      for (const auto& e : g.byKey) rows.push_back({g.c, kNoIdx, e.second});
    };
    while (curCb >= 0 || (!pq.empty() && cond())) {
      {
        PhaseScope pf(PH_FLATTEN);
        NsScope ns(47, "lead.in.ns.rows");
        rows.clear();
        if (curCb >= 0)  // the current broker's remaining view first
          for (Group& g : groups)
            if (g.c == curCb) emit(g);
        for (int gi : order) {
          Group& g = groups[gi];
          if (g.c != curCb && queued[g.c]) emit(g);
        }
        pr.clear();
        pb.clear();
        for (const Row& x : rows) {
          pr.push_back(x.r);
          pb.push_back(b);
        }
      }
      const int64_t key = rows.empty() ? -1 : e.pairScan(*this, pr, pb, DA_LEADERSHIP, false);
      // reference-equivalent rows visited up to the accepted row (or everything left when nothing is accepted)
      int64_t visited = 0;
      Row hitRow{-1, 0, -1};
      const Row* hit = nullptr;
      if (key >= 0) {
        hitRow = rows[(size_t)key];
        if (hitRow.idx == kNoIdx) hitRow.idx = indexOf(hitRow.cb, hitRow.r);  // (the model is as the scan saw it)
        hit = &hitRow;
      }
      {
      NsScope ns(45, "lead.in.ns.polls");
      if (curCb >= 0) {
        if (hit && hit->cb == curCb) {
          visited += (int64_t)(hit->idx - curSkip + 1);
        } else {
          const size_t n = size(curCb);
          visited += n > curSkip ? (int64_t)(n - curSkip) : 0;
          curCb = -1;
        }
      }
      if (!(hit && hit->cb == curCb) && pq.ordered() && !dir && (hit || cond())) {
        // The polls up to the hit's broker (or all of them; cond() does not change while polling) in runs: the sorted
        // run's brokers before the re-added heap's next one in one pass, then that one.
        m.bindSnapTable(snapTab, spec);
        int64_t sum = 0, polls = 0;
        bool found = false;
        auto takeRun = [&](size_t k) {
          const int* run = pq.runData();
          for (size_t q = 0; q < k; ++q) {
            queued[run[q]] = 0;
            sum += (int64_t)m.viewSizeBound(snapTab, run[q]);
          }
          pq.skipRun(k);
          polls += (int64_t)k;
        };
        auto hitIn = [&](size_t k) {  // the hit's broker among the run's next k: its position, else k
          const int* run = pq.runData();
          size_t j = 0;
          while (j < k && run[j] != hit->cb) ++j;
          return j;
        };
        while (!pq.empty()) {
          const bool heapEmpty = pq.heapEmpty();
          const size_t k = heapEmpty ? pq.runLeft() : pq.runBefore(pq.heapPeek());
          if (hit) {
            const size_t j = hitIn(k);
            if (j < k) {
              takeRun(j);
              pq.skipRun(1);
              ++polls;
              found = true;
              break;
            }
          }
          takeRun(k);
          if (heapEmpty) break;
          const int c = pq.heapPoll();
          queued[c] = 0;
          ++polls;
          if (hit && c == hit->cb) {
            found = true;
            break;
          }
          sum += (int64_t)m.viewSizeBound(snapTab, c);
        }
        if (hit && !found) throw std::logic_error("moveInLeadership: the winner's broker is not queued");
        prof().count(46, "lead.in.polls", polls);
        visited += sum + (hit ? (int64_t)hit->idx + 1 : 0);
        if (hit) queued[hit->cb] = 0;
      } else if (!(hit && hit->cb == curCb)) {
        while (!pq.empty() && (hit || cond())) {
          const int c = pq.poll();
          prof().count(46, "lead.in.polls");
          queued[c] = 0;
          if (hit && c == hit->cb) {
            visited += (int64_t)hit->idx + 1;
            break;
          }
          visited += (int64_t)size(c);
        }
      }
      }
      e.candidates += visited;
      if (!hit) break;
      const int cb = hit->cb;
      const size_t idx = hit->idx;
      m.relocateLeadership(m.rPart[hit->r], cb, b);
      if (dir) e.queueSyncSpec(spec);  // cb's and b's views changed
      for (size_t i = 0; i < order.size(); ++i)  // cb's key moved: re-place its group in the poll order
        if (groups[order[i]].c == cb) {
          const int gi = order[i];
          order.erase(order.begin() + (ptrdiff_t)i);
          size_t j = 0;
          while (j < order.size() && !before(gi, order[j])) ++j;
          order.insert(order.begin() + (ptrdiff_t)j, gi);
          break;
        }
      if (aboveLower(m, b)) {
        prof().count(3, "in.lead.done");
        return false;
      }
      if (!pq.empty() && m.pct(cb, res) < m.pct(pq.peek(), res)) {
        prof().count(4, "in.lead.readd");
        pq.add(cb);
        queued[cb] = 1;
        curCb = -1;
      } else {
        prof().count(5, "in.lead.continue");
        curCb = cb;
        curSkip = idx;
      }
    }
    return true;
  }

  bool swapCommon(Engine& e, int b, bool out, bool immOnly) {
    PhaseScope ps(PH_SWAP);
    Model& m = e.m;
    if (!m.alive(b) || (e.opt.anyExclMove && e.opt.exclMove[b])) return true;
    // The source's and the polled candidates' SortedReplicas are read as fresh snapshots (see moveIn): their
    // names are distinct and untracked when the swap phase ends.
    const Model::Spec srcSpec = out ? candidateSpec(e, 0.0, false, false, res == R_NW_OUT, immOnly)
                                    : candidateSpec(e, 1.7976931348623157e308, true, false, false, immOnly);
    if (m.snapshot(b, srcSpec)->empty()) return true;
    const double limit = firstOnlineLoad(m, *m.snapshot(b, srcSpec), out);
    const bool followersOnly = e.opt.anyExclLead && e.opt.exclLead[b];
    auto cmpUp = [this, &m](int x, int y) { return cmpBroker(m, x, y); };
    auto cmpDown = [this, &m](int x, int y) { return cmpBroker(m, y, x); };
    LiveQueue<decltype(cmpUp)> pqUp(cmpUp);
    LiveQueue<decltype(cmpDown)> pqDown(cmpDown);
    auto pqEmpty = [&]() { return out ? pqUp.empty() : pqDown.empty(); };
    auto pqPoll = [&]() { return out ? pqUp.poll() : pqDown.poll(); };
    auto pqAdd = [&](int x) {
      if (out) pqUp.add(x);
      else pqDown.add(x);
    };
    auto pqUnpoll = [&](int x) {
      if (out) pqUp.unpoll(x);
      else pqDown.unpoll(x);
    };
    {
      PhaseScope pi(PH_PQ_INIT);
      NsScope ns(54, "swap.ns.pqinit");
      // candidates: out = alive brokers under the upper limit hosting replicas (a Collectors.toSet() whose
      // insertion order does not matter to a PriorityQueue); in = alive brokers above the lower limit
      auto member = [&](int x) {
        if (!m.alive(x)) return false;
        if (out) return underThreshold(m, x, upperThr) && m.nrep(x) > 0;
        return overThreshold(m, x, lowerThr);
      };
      // swaps change only b and the polled broker; the ordered form is exact unless b itself is queued
      const bool ordered = !member(b);
      const auto& ord = m.brokersByPct(res);
      if (out) {
        pqUp.init(m.B, ordered);
        if (ordered) {
          for (int x : ord)
            if (member(x)) pqUp.push_sorted(x);
        } else {
          std::vector<int> under, order;
          for (int x = 0; x < m.B; ++x)
            if (member(x)) under.push_back(x);
          javaHashSetOrder(under, order);
          for (int c : order) pqUp.add(c);
        }
      } else {
        pqDown.init(m.B, ordered);
        if (ordered) {
          for (auto it = ord.rbegin(); it != ord.rend(); ++it)
            if (member(*it)) pqDown.push_sorted(*it);
        } else {
          for (int x = 0; x < m.B; ++x)
            if (member(x)) pqDown.add(x);
        }
      }
    }
    const Model::Spec candSpec = out ? candidateSpec(e, limit, true, followersOnly, false, immOnly)
                                     : candidateSpec(e, limit, false, followersOnly, res == R_NW_OUT, immOnly);
    // The limit filter does not enter the sort key, so a candidate's list is its limit-free sorted snapshot (cached
    // per broker version across swap calls with different limits) filtered by the limit: the same list, no re-sort.
    Model::Spec baseSpec = candSpec;
    const Model::Spec noLimit;
    baseSpec.selAboveRes = noLimit.selAboveRes;
    baseSpec.aboveLimit = noLimit.aboveLimit;
    baseSpec.selBelowRes = noLimit.selBelowRes;
    baseSpec.belowLimit = noLimit.belowLimit;
    std::vector<int32_t> srcs, cbOff, cbRep, polled;
    std::vector<std::shared_ptr<const std::vector<int32_t>>> polledSnaps;
    // Without new brokers the limit test runs on the device (SwapLimit) over the limit-free lists; with new brokers
    // the host filters (eligibleReplicasForSwap's CASE#2 depends on which filtered lists are empty).
    SwapLimit lim;
    const bool devLimit = m.numNew == 0;
    if (devLimit) {
      lim.res = candSpec.selBelowRes >= 0 ? candSpec.selBelowRes : candSpec.selAboveRes;
      lim.above = candSpec.selBelowRes >= 0 ? 0 : 1;
      lim.limit = candSpec.selBelowRes >= 0 ? candSpec.belowLimit : candSpec.aboveLimit;
    }
    size_t target = 4;
    while (!pqEmpty()) {
      {  // the polled brokers' candidate rows (limit filter) and the source rows
        PhaseScope pc(PH_CAND_BUILD);
        polled.clear();
        cbOff.assign(1, 0);
        cbRep.clear();
        while (!pqEmpty() && (polled.empty() || polled.size() < target)) polled.push_back(pqPoll());
        prof().count(57, "swap.polled", (int64_t)polled.size());
        {
          NsScope ns(55, "swap.ns.snapshots");
          m.snapshotManyIn(swapTab, baseSpec, polled, polledSnaps);  // (many misses: their sorts on the host pool)
        }
        NsScope ns(56, "swap.ns.rows");
        for (size_t pi = 0; pi < polled.size(); ++pi) {
          const auto& v = polledSnaps[pi];
          if (devLimit)
            cbRep.insert(cbRep.end(), v->begin(), v->end());
          else
            for (int r : *v)  // baseSpec's other selections already hold: only the limit test remains
              if ((candSpec.selAboveRes < 0 || m.ru(r, candSpec.selAboveRes) > candSpec.aboveLimit) &&
                  (candSpec.selBelowRes < 0 || m.ru(r, candSpec.selBelowRes) < candSpec.belowLimit))
                cbRep.push_back(r);
          cbOff.push_back((int32_t)cbRep.size());
        }
        srcs = *m.snapshot(b, srcSpec);
      }
      const int64_t key = e.swapScan(*this, srcs, cbOff, cbRep, lim);
      if (key < 0) {
        target = std::min<size_t>(target * 2, 1024);
        continue;  // every polled broker exhausted without a swap
      }
      target = 4;
      const int64_t row = key >> 24;
      const int j = (int)(key & 0xFFFFFF);
      const int mi = (int)(row / (int64_t)srcs.size());
      const int si = (int)(row % (int64_t)srcs.size());
      const int cb = polled[mi];
      const int sr = srcs[si];
      const int dr = cbRep[cbOff[mi] + j];
      const int dp = m.rPart[dr];
      m.relocateReplica(m.rPart[sr], b, cb);
      m.relocateReplica(dp, cb, b);
      const bool done = out ? underUpper(m, b, upperThr) : aboveLower(m, b);
      if (done) return false;
      for (size_t t = polled.size(); t-- > (size_t)mi + 1;) pqUnpoll(polled[t]);  // un-poll speculative brokers
      pqAdd(cb);
    }
    return true;
  }
  bool swapOut(Engine& e, int b, bool immOnly) { return swapCommon(e, b, true, immOnly); }
  bool swapIn(Engine& e, int b, bool immOnly) { return swapCommon(e, b, false, immOnly); }
};

}  // namespace

std::unique_ptr<GoalImpl> makeGoal(int kind) {
  if (isIntraGoalKind(kind)) return makeIntraGoal(kind);
  switch (kind) {
    case CCMI_GOAL_REPLICA_DISTRIBUTION: return std::make_unique<ReplicaDistribution>();
    case CCMI_GOAL_DISK_USAGE_DISTRIBUTION:
    case CCMI_GOAL_NW_IN_USAGE_DISTRIBUTION:
    case CCMI_GOAL_NW_OUT_USAGE_DISTRIBUTION:
    case CCMI_GOAL_CPU_USAGE_DISTRIBUTION: return std::make_unique<ResourceDistribution>(kind);
    default: return makeMoreGoal(kind);
  }
}

}  // namespace ccmi
