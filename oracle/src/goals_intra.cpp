// ORACLE — test infrastructure only (see jsem.h header).
// Intra-broker (JBOD) goals, restated line by line:
//   AbstractGoal.maybeMoveReplicaBetweenDisks      analyzer/goals/AbstractGoal.java:351-378
//   AbstractGoal.maybeSwapReplicaBetweenDisks      analyzer/goals/AbstractGoal.java:389-430
//   GoalUtils.legitMoveBetweenDisks                analyzer/goals/GoalUtils.java:237-244
//   IntraBrokerDiskCapacityGoal                    analyzer/goals/IntraBrokerDiskCapacityGoal.java:81-291
//   IntraBrokerDiskUsageDistributionGoal           analyzer/goals/IntraBrokerDiskUsageDistributionGoal.java:78-543
//   java.util.TimSort (arrays < MIN_MERGE = 32)    countRunAndMakeAscending + binarySort (JDK 11)
// Reference behaviours kept on purpose:
//   * maybeSwapReplicaBetweenDisks relocates the destination replica to sourceReplica.disk() AFTER the source replica
//     has moved, i.e. onto its own disk: the "swap" moves only the source replica (plus a remove/add of the destination
//     replica on its disk, which can change the last bits of that disk's utilization).
//   * the capacity goal sorts candidate disks with ((Double) (allowance2 - allowance1)).intValue(), which is not a
//     total order; the JDK's binary insertion sort is restated so the resulting order is the reference's.
//   * the swap phases re-enqueue a candidate disk after a pass without a swap; with no state change the loop only
//     ends at PER_DISK_SWAP_TIMEOUT_MS (500 ms). Here the loop ends as soon as the queue returns to a state it had
//     since the last applied swap (the state can no longer change, so the reference spins until its timeout).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <set>

#include "goals.h"

namespace oracle {

namespace {

bool legitMoveBetweenDisks(const ClusterModel& cm, int r, int d) {
  return d >= 0 && cm.disks[d].broker == cm.replicas[r].broker && cm.disks[d].alive;
}

SortSpec intraSpec(const OptimizationOptions& o, bool reverse) {
  SortSpec sp;
  sp.selection.push_back({SelFn::ONLINE});
  if (!o.excludedTopics.empty()) sp.selection.push_back({SelFn::EXCLUDED_TOPICS});
  sp.priority.push_back(PrioFn::DISK_IMMIGRANTS);
  sp.score = reverse ? ScoreFn::REVERSE_BY_GROUP : ScoreFn::BY_GROUP;
  sp.scoreResource = DISK;
  return sp;
}

// TimSort.sort for nRemaining < MIN_MERGE: countRunAndMakeAscending then binarySort (TimSort.java)
template <class Cmp>
void javaSmallSort(std::vector<int>& a, Cmp c) {
  const int lo = 0, hi = (int)a.size();
  if (hi - lo < 2) return;
  if (hi - lo >= 32) throw std::invalid_argument("more than 31 logdirs on a broker: TimSort merge path not restated");
  int runHi = lo + 1;
  if (c(a[runHi++], a[lo]) < 0) {
    while (runHi < hi && c(a[runHi], a[runHi - 1]) < 0) runHi++;
    std::reverse(a.begin() + lo, a.begin() + runHi);
  } else {
    while (runHi < hi && c(a[runHi], a[runHi - 1]) >= 0) runHi++;
  }
  int start = runHi;
  if (start == lo) start++;
  for (; start < hi; start++) {
    const int pivot = a[start];
    int left = lo, right = start;
    while (left < right) {
      const int mid = (left + right) >> 1;
      if (c(pivot, a[mid]) < 0) right = mid;
      else left = mid + 1;
    }
    for (int k = start; k > left; --k) a[k] = a[k - 1];
    a[left] = pivot;
  }
}

std::string diskString(const ClusterModel& cm, int d) {  // Disk.toString
  char buf[512];
  std::snprintf(buf, sizeof(buf), "Disk[logdir=%s,state=%s,capacity=%f,replicaCount=%d]", cm.disks[d].logdir.c_str(),
                cm.disks[d].alive ? "ALIVE" : "DEAD", cm.disks[d].capacity, (int)cm.disks[d].replicas.size());
  return buf;
}

void checkIntraAction(const BalancingAction& a, const std::string& goal) {
  if (a.sourceDisk < 0 || a.destinationDisk < 0)
    throw std::invalid_argument(goal + " does not support balancing action not specifying logdir.");
}

}  // namespace

// ===================================================================== AbstractGoal helpers
int AbstractGoal::maybeMoveReplicaBetweenDisks(ClusterModel& cm, int r, const std::vector<int>& candidateDisks,
                                               const GoalList& g) {
  for (int d : candidateDisks) {
    cm.countCandidate();
    const Replica& rep = cm.replicas[r];
    BalancingAction a{rep.partition, rep.broker, cm.disks[d].broker, ActionType::INTRA_BROKER_REPLICA_MOVEMENT, -1,
                      rep.disk, d};
    if (!legitMoveBetweenDisks(cm, r, d)) continue;
    if (!selfSatisfied(cm, a)) continue;
    if (isProposalAcceptableForOptimizedGoals(g, a, cm) == Acceptance::ACCEPT) {
      cm.relocateReplicaToDisk(rep.partition, rep.broker, d);
      return d;
    }
  }
  return -1;
}

int AbstractGoal::maybeSwapReplicaBetweenDisks(ClusterModel& cm, int src, const std::vector<int>& candidates,
                                               const GoalList& g) {
  for (int dr : candidates) {
    cm.countCandidate();
    const Replica& s = cm.replicas[src];
    const Replica& t = cm.replicas[dr];
    BalancingAction swap{s.partition, cm.disks[s.disk].broker, cm.disks[t.disk].broker,
                         ActionType::INTRA_BROKER_REPLICA_SWAP, t.partition, s.disk, t.disk};
    if (!legitMoveBetweenDisks(cm, src, t.disk)) return -1;
    if (!legitMoveBetweenDisks(cm, dr, s.disk)) continue;
    if (!selfSatisfied(cm, swap)) return -1;
    if (isProposalAcceptableForOptimizedGoals(g, swap, cm) == Acceptance::ACCEPT) {
      cm.relocateReplicaToDisk(s.partition, s.broker, t.disk);
      // sourceReplica.disk() is read after the first relocation (AbstractGoal.java:421-422)
      cm.relocateReplicaToDisk(t.partition, t.broker, cm.replicas[src].disk);
      return dr;
    }
  }
  return -1;
}

// ===================================================================== IntraBrokerDiskCapacityGoal
bool IntraBrokerDiskCapacityGoal::overLimit(const ClusterModel& cm, int d) const {
  return cm.disks[d].utilization > cm.disks[d].capacity * bc_.capacityThreshold[DISK];
}
bool IntraBrokerDiskCapacityGoal::underLimitAfterAdding(const ClusterModel& cm, int d, double util) const {
  const double limit = cm.disks[d].capacity * bc_.capacityThreshold[DISK];
  return cm.disks[d].utilization + util < limit;
}

void IntraBrokerDiskCapacityGoal::initGoalState(ClusterModel& cm, const OptimizationOptions& o) {
  const double thr = bc_.capacityThreshold[DISK];
  for (int b : cm.aliveBrokers()) {
    const double existing = cm.brokerUtil(b, DISK);
    const double allowed = cm.brokers[b].capacity[DISK] * thr;
    if (allowed < existing) {
      char buf[256];
      std::snprintf(buf, sizeof(buf),
                    "[%s] Insufficient disk capacity at broker %d (Utilization %.2f, Allowed Capacity %.2f).",
                    name().c_str(), cm.brokers[b].id, existing, allowed);
      ProvisionRec rec = underBrokers(1);  // IntraBrokerDiskCapacityGoal.java:92-95
      rec.totalCapacity = existing / thr;
      throw OptimizationFailure(buf, rec);
    }
  }
  cm.excludedTopicsSel = o.excludedTopics;
  const SortSpec sp = intraSpec(o, true);
  for (int b = 0; b < (int)cm.brokers.size(); ++b) cm.trackSortedReplicas(b, replicaSortName(true, false), sp);
}

void IntraBrokerDiskCapacityGoal::rebalanceForBroker(int b, ClusterModel& cm, const GoalList& g,
                                                     const OptimizationOptions&) {
  std::vector<int> over;
  for (int d : cm.brokers[b].disks)
    if (cm.disks[d].alive && overLimit(cm, d)) over.push_back(d);
  if (over.empty()) return;
  std::vector<int> cands;
  for (int d : cm.brokers[b].disks)
    if (std::find(over.begin(), over.end(), d) == over.end()) cands.push_back(d);
  const double thr = bc_.capacityThreshold[DISK];
  javaSmallSort(cands, [&](int d1, int d2) {
    const double a1 = cm.disks[d1].capacity * thr - cm.disks[d1].utilization;
    const double a2 = cm.disks[d2].capacity * thr - cm.disks[d2].utilization;
    return jDoubleToInt(a2 - a1);
  });
  const std::string nm = replicaSortName(true, false);
  for (int d : over) {
    for (int r : cm.diskSortedReplicasClone(d, nm)) {
      maybeMoveReplicaBetweenDisks(cm, r, cands, g);
      if (!overLimit(cm, d)) break;
    }
  }
}

void IntraBrokerDiskCapacityGoal::updateGoalState(ClusterModel& cm, const OptimizationOptions&) {
  for (int b : brokersToBalance(cm))
    for (int d : cm.brokers[b].disks)
      if (cm.disks[d].alive && overLimit(cm, d)) {
        char buf[768];
        std::snprintf(buf, sizeof(buf), "[%s] Utilization (%.2f) for disk %s on broker %d is above capacity limit.",
                      name().c_str(), cm.disks[d].utilization, diskString(cm, d).c_str(), cm.brokers[b].id);
        ProvisionRec rec;  // IntraBrokerDiskCapacityGoal.java:236-239
        rec.numDisks = 1;
        rec.totalCapacity = cm.disks[d].utilization / bc_.capacityThreshold[DISK];
        throw OptimizationFailure(buf, rec);
      }
  finished_ = true;
}

bool IntraBrokerDiskCapacityGoal::selfSatisfied(ClusterModel& cm, const BalancingAction& a) {
  const int r = cm.replicaOnBroker(a.partition, a.sourceBroker);
  const double du = cm.replicaUtil(r, DISK);
  return du > 0 && underLimitAfterAdding(cm, a.destinationDisk, du);
}

Acceptance IntraBrokerDiskCapacityGoal::actionAcceptance(const BalancingAction& a, ClusterModel& cm) {
  checkIntraAction(a, name());
  const int sr = cm.replicaOnBroker(a.partition, a.sourceBroker);
  const int dd = cm.diskOf(a.destinationBroker, cm.disks[a.destinationDisk].logdir);
  switch (a.type) {
    case ActionType::INTRA_BROKER_REPLICA_SWAP: {
      const int dr = cm.replicaOnBroker(a.destPartition, a.destinationBroker);
      const double su = cm.replicaUtil(sr, DISK), du = cm.replicaUtil(dr, DISK);
      const double delta = du - su;
      const bool ok = delta > 0 ? underLimitAfterAdding(cm, cm.replicas[sr].disk, delta)
                                : underLimitAfterAdding(cm, cm.replicas[dr].disk, -delta);
      return ok ? Acceptance::ACCEPT : Acceptance::REPLICA_REJECT;
    }
    case ActionType::INTRA_BROKER_REPLICA_MOVEMENT:
      return underLimitAfterAdding(cm, dd, cm.replicaUtil(sr, DISK)) ? Acceptance::ACCEPT : Acceptance::REPLICA_REJECT;
    case ActionType::LEADERSHIP_MOVEMENT: return Acceptance::ACCEPT;
    default: throw std::invalid_argument("Unsupported balancing action");
  }
}

// ===================================================================== IntraBrokerDiskUsageDistributionGoal
void IntraBrokerDiskUsageDistributionGoal::initGoalState(ClusterModel& cm, const OptimizationOptions& o) {
  const double margin = (bc_.resourceBalancePercentage[DISK] - 1) * 0.9;  // BALANCE_MARGIN
  upper_.assign(cm.brokers.size(), 0.0);
  lower_.assign(cm.brokers.size(), 0.0);
  for (int b : brokersToBalance(cm)) {
    const double avg = cm.averageDiskUtilizationPct(b);
    upper_[b] = avg * (1 + margin);
    lower_[b] = avg * jmax(0, (1 - margin));
  }
  cm.excludedTopicsSel = o.excludedTopics;
  const SortSpec rev = intraSpec(o, true), fwd = intraSpec(o, false);
  for (int b = 0; b < (int)cm.brokers.size(); ++b) cm.trackSortedReplicas(b, replicaSortName(true, false), rev);
  for (int b = 0; b < (int)cm.brokers.size(); ++b) cm.trackSortedReplicas(b, replicaSortName(false, false), fwd);
}

void IntraBrokerDiskUsageDistributionGoal::updateGoalState(ClusterModel& cm, const OptimizationOptions&) {
  bool above = false, below = false;
  for (int b : brokersToBalance(cm))
    for (int d : cm.brokers[b].disks)
      if (cm.disks[d].alive) {
        if (cm.diskUtilizationPct(d) > upper_[b]) above = true;
        if (cm.diskUtilizationPct(d) < lower_[b]) below = true;
      }
  if (above || below) succeeded_ = false;
  finished_ = true;
}

double IntraBrokerDiskUsageDistributionGoal::sourceUtilizationDelta(const BalancingAction& a, ClusterModel& cm) const {
  checkIntraAction(a, name());
  const int sr = cm.replicaOnBroker(a.partition, a.sourceBroker);
  switch (a.type) {
    case ActionType::INTRA_BROKER_REPLICA_SWAP: {
      const int dr = cm.replicaOnBroker(a.destPartition, a.sourceBroker);
      return cm.replicaUtil(dr, DISK) - cm.replicaUtil(sr, DISK);
    }
    case ActionType::LEADERSHIP_MOVEMENT: return 0;
    case ActionType::INTRA_BROKER_REPLICA_MOVEMENT: return -cm.replicaUtil(sr, DISK);
    default: throw std::invalid_argument("Unsupported balancing action");
  }
}

bool IntraBrokerDiskUsageDistributionGoal::isChangeViolatingLimit(const ClusterModel& cm, double delta, int s,
                                                                  int t) const {
  const int b = cm.disks[s].broker;
  const double up = upper_[b], lo = lower_[b];
  const Disk& sd = cm.disks[s];
  const Disk& td = cm.disks[t];
  const double srcAllow = delta > 0 ? sd.capacity * up - sd.utilization : sd.utilization - sd.capacity * lo;
  const double dstAllow = delta > 0 ? td.utilization - td.capacity * lo : td.capacity * up - td.utilization;
  return (srcAllow >= 0 && srcAllow < std::fabs(delta)) || (dstAllow >= 0 && dstAllow < std::fabs(delta));
}

bool IntraBrokerDiskUsageDistributionGoal::isGettingMoreBalanced(const ClusterModel& cm, int s, int t,
                                                                 double delta) const {
  const double prev = cm.diskUtilizationPct(s) - cm.diskUtilizationPct(t);
  const double next = prev + delta / cm.disks[s].capacity + delta / cm.disks[t].capacity;
  return std::fabs(next) < std::fabs(prev);
}

Acceptance IntraBrokerDiskUsageDistributionGoal::actionAcceptance(const BalancingAction& a, ClusterModel& cm) {
  const double delta = sourceUtilizationDelta(a, cm);
  const int s = cm.diskOf(a.sourceBroker, cm.disks[a.sourceDisk].logdir);
  const int t = cm.diskOf(a.sourceBroker, cm.disks[a.destinationDisk].logdir);  // broker(sourceBrokerId).disk(...)
  if (delta == 0) return Acceptance::ACCEPT;
  if (isChangeViolatingLimit(cm, delta, s, t)) return Acceptance::REPLICA_REJECT;
  return isGettingMoreBalanced(cm, s, t, delta) ? Acceptance::ACCEPT : Acceptance::REPLICA_REJECT;
}

bool IntraBrokerDiskUsageDistributionGoal::selfSatisfied(ClusterModel& cm, const BalancingAction& a) {
  const double delta = sourceUtilizationDelta(a, cm);
  return delta != 0 && actionAcceptance(a, cm) == Acceptance::ACCEPT;
}

int IntraBrokerDiskUsageDistributionGoal::compareStats(const ClusterModelStats& s1, const ClusterModelStats& s2) const {
  if (s1.numUnbalancedDisks > s2.numUnbalancedDisks || s1.diskUtilizationStDev > s2.diskUtilizationStDev) return -1;
  return 1;
}

void IntraBrokerDiskUsageDistributionGoal::rebalanceForBroker(int b, ClusterModel& cm, const GoalList& g,
                                                              const OptimizationOptions&) {
  const double up = upper_[b], lo = lower_[b];
  for (int d : cm.brokers[b].disks) {
    if (!cm.disks[d].alive) continue;
    if (cm.diskUtilizationPct(d) > up) {
      if (moveLoadOut(d, cm, g)) swapLoadOut(d, cm, g);
    }
    if (cm.diskUtilizationPct(d) < lo) {
      if (moveLoadIn(d, cm, g)) swapLoadIn(d, cm, g);
    }
  }
}

bool IntraBrokerDiskUsageDistributionGoal::moveLoadIn(int disk, ClusterModel& cm, const GoalList& g) {
  const int b = cm.disks[disk].broker;
  const double brokerUtil = cm.averageDiskUtilizationPct(b);
  JPriorityQueue pq([&](int d1, int d2) { return dcompare(cm.diskUtilizationPct(d2), cm.diskUtilizationPct(d1)); });
  for (int cd : cm.brokers[b].disks)
    if (cm.disks[cd].alive && cm.diskUtilizationPct(cd) > brokerUtil) pq.add(cd);
  const std::string nm = replicaSortName(true, false);
  while (!pq.empty()) {
    const int cd = pq.poll();
    for (int r : cm.diskSortedReplicasClone(cd, nm)) {
      if (maybeMoveReplicaBetweenDisks(cm, r, {disk}, g) >= 0) {
        if (cm.diskUtilizationPct(disk) > lower_[b]) return false;
        if (!pq.empty() && cm.diskUtilizationPct(cd) < cm.diskUtilizationPct(pq.peek())) {
          pq.add(cd);
          break;
        }
      }
    }
  }
  return true;
}

bool IntraBrokerDiskUsageDistributionGoal::moveLoadOut(int disk, ClusterModel& cm, const GoalList& g) {
  const int b = cm.disks[disk].broker;
  const double brokerUtil = cm.averageDiskUtilizationPct(b);
  JPriorityQueue pq([&](int d1, int d2) { return dcompare(cm.diskUtilizationPct(d1), cm.diskUtilizationPct(d2)); });
  for (int cd : cm.brokers[b].disks)
    if (cm.disks[cd].alive && cm.diskUtilizationPct(cd) < brokerUtil) pq.add(cd);
  const std::string nm = replicaSortName(true, false);
  while (!pq.empty()) {
    const int cd = pq.poll();
    for (int r : cm.diskSortedReplicasClone(disk, nm)) {
      if (maybeMoveReplicaBetweenDisks(cm, r, {cd}, g) >= 0) {
        if (cm.diskUtilizationPct(disk) < upper_[b]) return false;
        if (!pq.empty() && cm.diskUtilizationPct(cd) > cm.diskUtilizationPct(pq.peek())) {
          pq.add(cd);
          break;
        }
      }
    }
  }
  return true;
}

void IntraBrokerDiskUsageDistributionGoal::swapLoadOut(int disk, ClusterModel& cm, const GoalList& g) {
  const int b = cm.disks[disk].broker;
  JPriorityQueue pq([&](int d1, int d2) { return dcompare(cm.diskUtilizationPct(d1), cm.diskUtilizationPct(d2)); });
  for (int cd : cm.brokers[b].disks)
    if (cm.disks[cd].alive && cm.diskUtilizationPct(cd) < upper_[b]) pq.add(cd);
  const std::string rev = replicaSortName(true, false), fwd = replicaSortName(false, false);
  std::set<std::vector<int>> seen;  // queue states since the last applied swap
  while (!pq.empty()) {
    const int cd = pq.poll();
    bool swapped = false;
    for (int src : cm.diskSortedReplicasClone(disk, rev)) {
      if (maybeSwapReplicaBetweenDisks(cm, src, cm.diskSortedReplicasClone(cd, fwd), g) >= 0) {
        if (cm.diskUtilizationPct(disk) < upper_[b]) return;
        swapped = true;
        break;
      }
    }
    if (cm.diskUtilizationPct(cd) < upper_[b]) pq.add(cd);
    if (swapped) seen.clear();
    else if (!seen.insert(pq.heap()).second) return;  // no state change can follow: the reference spins to its timeout
    if (seen.size() > 16) throw std::invalid_argument("swap phase queue cycle longer than 16 states");
  }
}

void IntraBrokerDiskUsageDistributionGoal::swapLoadIn(int disk, ClusterModel& cm, const GoalList& g) {
  const int b = cm.disks[disk].broker;
  JPriorityQueue pq([&](int d1, int d2) { return dcompare(cm.diskUtilizationPct(d2), cm.diskUtilizationPct(d1)); });
  for (int cd : cm.brokers[b].disks)
    if (cm.disks[cd].alive && cm.diskUtilizationPct(cd) > lower_[b]) pq.add(cd);
  const std::string rev = replicaSortName(true, false), fwd = replicaSortName(false, false);
  std::set<std::vector<int>> seen;
  while (!pq.empty()) {
    const int cd = pq.poll();
    bool swapped = false;
    for (int src : cm.diskSortedReplicasClone(disk, fwd)) {
      if (maybeSwapReplicaBetweenDisks(cm, src, cm.diskSortedReplicasClone(cd, rev), g) >= 0) {
        if (cm.diskUtilizationPct(disk) > lower_[b]) return;
        swapped = true;
        break;
      }
    }
    if (cm.diskUtilizationPct(cd) > lower_[b]) pq.add(cd);
    if (swapped) seen.clear();
    else if (!seen.insert(pq.heap()).second) return;
    if (seen.size() > 16) throw std::invalid_argument("swap phase queue cycle longer than 16 states");
  }
}

}  // namespace oracle
