// ORACLE — test infrastructure only (see jsem.h header). Line-by-line restatement of the goal
// drivers; every function names the reference lines it follows.
#include "goals.h"

#include <algorithm>
#include <cmath>

namespace oracle {

// ===================================================================== GoalUtils / AnalyzerUtils
// GoalUtils.eligibleBrokers + filterOutBrokersExcludedFor{Leadership,ReplicaMove} (GoalUtils.java:122-199)
std::vector<int> eligibleBrokers(ClusterModel& cm, int replica, const std::vector<int>& candidates, ActionType a,
                                 const OptimizationOptions& o) {
  std::vector<int> out(candidates);
  auto removeIf = [&](auto pred) { out.erase(std::remove_if(out.begin(), out.end(), pred), out.end()); };
  const bool reqEmpty = o.requestedDestinationBrokerIds.empty();
  if (reqEmpty || a == ActionType::LEADERSHIP_MOVEMENT) {
    if (!o.excludedBrokersForLeadership.empty() && (a == ActionType::LEADERSHIP_MOVEMENT || cm.replicas[replica].isLeader))
      removeIf([&](int b) { return o.excludedBrokersForLeadership.count(cm.brokers[b].id) > 0; });
  } else {
    removeIf([&](int b) { return o.requestedDestinationBrokerIds.count(cm.brokers[b].id) == 0; });
  }
  if (reqEmpty) {
    if (!o.excludedBrokersForReplicaMove.empty() && a == ActionType::INTER_BROKER_REPLICA_MOVEMENT)
      removeIf([&](int b) { return o.excludedBrokersForReplicaMove.count(cm.brokers[b].id) > 0; });
  } else if (a != ActionType::LEADERSHIP_MOVEMENT) {
    removeIf([&](int b) { return o.requestedDestinationBrokerIds.count(cm.brokers[b].id) == 0; });
  }
  if (!reqEmpty) return out;
  if (cm.newBrokers.empty()) return out;
  int orig = cm.replicas[replica].origBroker;
  removeIf([&](int b) { return !(cm.brokers[b].isNew() || b == orig); });
  return out;
}

// GoalUtils.legitMove (GoalUtils.java:213-226)
bool legitMove(ClusterModel& cm, int replica, int dest, ActionType a) {
  const Replica& r = cm.replicas[replica];
  switch (a) {
    case ActionType::INTER_BROKER_REPLICA_MOVEMENT:
      return cm.partitions[r.partition].ineligibleBrokers.count(dest) == 0 && cm.replicaOnBroker(r.partition, dest) < 0;
    case ActionType::LEADERSHIP_MOVEMENT:
      return r.isLeader && cm.replicaOnBroker(r.partition, dest) >= 0;
    default:
      return false;
  }
}

// AnalyzerUtils.isProposalAcceptableForOptimizedGoals (AnalyzerUtils.java:169-179)
Acceptance isProposalAcceptableForOptimizedGoals(const GoalList& g, const BalancingAction& a, ClusterModel& cm) {
  for (Goal* goal : g) {
    Acceptance acc = goal->actionAcceptance(a, cm);
    if (acc != Acceptance::ACCEPT) return acc;
  }
  return Acceptance::ACCEPT;
}

// GoalUtils.ensureNoOfflineReplicas (GoalUtils.java:307-318)
void ensureNoOfflineReplicas(ClusterModel& cm, const std::string& goal) {
  for (int r : cm.selfHealingEligibleReplicas)
    if (cm.isCurrentOffline(r))
      throw OptimizationFailure("[" + goal + "] Cannot remove replica from broker " +
                                    std::to_string(cm.brokers[cm.replicas[r].broker].id),
                                underBrokers(1));
}
void ensureReplicasMoveOffBrokersWithBadDisks(ClusterModel& cm, const std::string& goal) {
  for (int b : cm.brokersWithBadDisks)
    for (int r : cm.brokers[b].replicas)
      if (cm.partitions[cm.replicas[r].partition].ineligibleBrokers.count(b))
        throw OptimizationFailure("[" + goal + "] A replica was moved back to broker with broken disk.", underBrokers(1));
}

// Iteration order of a java.util.HashSet<Broker> built by add() in the given order (Collectors.toSet()):
// Broker.hashCode() == id, HashMap.hash() spreads h ^ (h >>> 16), table doubles at size > 0.75*cap,
// list bins keep insertion order (resize split preserves it); a 9th node in a bin resizes when the
// table is < 64 and treeifies otherwise (not emulated: reported as an error).
std::vector<int> javaHashSetOrderIntKeys(const std::vector<int>& ins) {
  int cap = 16;
  auto spread = [](int h) { return h ^ (int)((unsigned)h >> 16); };
  std::vector<std::vector<int>> tab(cap);
  int size = 0;
  auto resize = [&]() {
    int ncap = cap * 2;
    std::vector<std::vector<int>> nt(ncap);
    for (int i = 0; i < cap; ++i)
      for (int k : tab[i]) nt[spread(k) & (ncap - 1)].push_back(k);
    tab.swap(nt);
    cap = ncap;
  };
  for (int k : ins) {
    auto& bin = tab[spread(k) & (cap - 1)];
    if (std::find(bin.begin(), bin.end(), k) != bin.end()) continue;
    bin.push_back(k);
    if ((int)bin.size() >= 9) {
      if (cap < 64) resize();
      else throw std::runtime_error("java HashMap tree bin not emulated");
    }
    if (++size > (int)(cap * 0.75)) resize();
  }
  std::vector<int> out;
  out.reserve(size);
  for (int i = 0; i < cap; ++i)
    for (int k : tab[i]) out.push_back(k);
  return out;
}

// ===================================================================== AbstractGoal
std::vector<int> AbstractGoal::brokersToBalance(ClusterModel& cm) {
  std::vector<int> out(cm.brokers.size());
  for (size_t i = 0; i < out.size(); ++i) out[i] = (int)i;
  return out;
}

// AbstractGoal.optimize (AbstractGoal.java:81-135)
bool AbstractGoal::optimize(ClusterModel& cm, const GoalList& optimizedGoals, const OptimizationOptions& o) {
  struct Clear {
    ClusterModel& cm;
    ~Clear() { cm.clearSortedReplicas(); }
  } clearGuard{cm};
  succeeded_ = true;
  provision_ = ProvisionResp{};  // UNDECIDED for every optimize call
  try {
    return optimizeImpl(cm, optimizedGoals, o);
  } catch (OptimizationFailure& e) {
    provision_ = ProvisionResp{PROV_UNDER, e.hasRec, e.rec};  // AbstractGoal.java:125-126
    throw;
  }
}
bool AbstractGoal::optimizeImpl(ClusterModel& cm, const GoalList& optimizedGoals, const OptimizationOptions& o) {
  ClusterModelStats before = computeStats(cm, bc_, o);
  finished_ = false;
  initGoalState(cm, o);
  bool brokenEmpty = cm.deadBrokers.empty() && cm.brokersWithBadDisks.empty();
  bool excludedWithReplicas = false;
  for (int b : cm.aliveBrokers())
    if (o.excludedBrokersForReplicaMove.count(cm.brokers[b].id) && !cm.brokers[b].replicas.empty())
      excludedWithReplicas = true;
  while (!finished_) {
    for (int b : brokersToBalance(cm)) rebalanceForBroker(b, cm, optimizedGoals, o);
    updateGoalState(cm, o);
  }
  ClusterModelStats after = computeStats(cm, bc_, o);
  if (brokenEmpty && !excludedWithReplicas) {
    if (compareStats(after, before) < 0)
      throw std::logic_error("Optimization for goal " + name() + " failed because the optimized result is worse than before.");
  }
  provision_ = validateProvisionResponse(provision_, cm, bc_.overprovisionedMinBrokers);
  return succeeded_;
}

// GoalUtils.validateProvisionResponse (GoalUtils.java:619-650)
ProvisionResp validateProvisionResponse(const ProvisionResp& p, ClusterModel& cm, int overprovisionedMinBrokers) {
  if (p.status != PROV_OVER) return p;
  const int alive = (int)cm.aliveBrokers().size();
  if (alive < overprovisionedMinBrokers) return ProvisionResp{PROV_RIGHT_SIZED};
  if (!p.hasRec) throw std::invalid_argument("Expected to have exactly 1 provision recommendation, but got: 0");
  const int maxAllowedToDrop = alive - cm.maxReplicationFactor;
  if (p.rec.numBrokers <= maxAllowedToDrop) return p;
  if (maxAllowedToDrop > 0) {
    ProvisionRec r;
    r.status = PROV_OVER;
    r.numBrokers = maxAllowedToDrop;
    return ProvisionResp{PROV_OVER, true, r};
  }
  return ProvisionResp{PROV_RIGHT_SIZED};
}

// AbstractGoal.maybeApplyBalancingAction (AbstractGoal.java:230-272)
int AbstractGoal::maybeApplyBalancingAction(ClusterModel& cm, int replica, const std::vector<int>& candidates,
                                            ActionType action, const GoalList& g, const OptimizationOptions& o) {
  std::vector<int> eligible = eligibleBrokers(cm, replica, candidates, action, o);
  for (int b : eligible) {
    cm.countCandidate();
    BalancingAction proposal{cm.replicas[replica].partition, cm.replicas[replica].broker, b, action, -1};
    if (!legitMove(cm, replica, b, action)) continue;
    if (!selfSatisfied(cm, proposal)) continue;
    Acceptance acc = isProposalAcceptableForOptimizedGoals(g, proposal, cm);
    if (acc == Acceptance::ACCEPT) {
      if (action == ActionType::LEADERSHIP_MOVEMENT)
        cm.relocateLeadership(proposal.partition, proposal.sourceBroker, b);
      else if (action == ActionType::INTER_BROKER_REPLICA_MOVEMENT)
        cm.relocateReplica(proposal.partition, proposal.sourceBroker, b);
      return b;
    }
  }
  return -1;
}

// AbstractGoal.maybeApplySwapAction (AbstractGoal.java:287-338) with
// GoalUtils.eligibleReplicasForSwap (GoalUtils.java:258-298)
int AbstractGoal::maybeApplySwapAction(ClusterModel& cm, int src, const std::vector<int>& candidates, const GoalList& g,
                                       const OptimizationOptions& o) {
  if (candidates.empty()) return -1;
  int destBroker = cm.replicas[candidates.front()].broker;
  const Replica& sr = cm.replicas[src];
  if (o.excludedBrokersForLeadership.count(cm.brokers[destBroker].id) && !cm.isOriginalOffline(src) && sr.isLeader)
    return -1;
  if (o.excludedBrokersForReplicaMove.count(cm.brokers[destBroker].id) && !cm.isOriginalOffline(src)) return -1;
  int srcBroker = sr.broker;
  if (!(cm.newBrokers.empty() ||
        (cm.brokers[srcBroker].isNew() && (cm.brokers[destBroker].isNew() || sr.origBroker == destBroker)))) {
    if (cm.brokers[destBroker].isNew())
      throw UnsupportedOperation("UnsupportedOperationException: removeIf on an unmodifiable sorted replica view");
    return -1;
  }
  for (int dr : candidates) {
    cm.countCandidate();
    BalancingAction swap{sr.partition, srcBroker, destBroker, ActionType::INTER_BROKER_REPLICA_SWAP,
                         cm.replicas[dr].partition};
    if (!legitMove(cm, src, destBroker, ActionType::INTER_BROKER_REPLICA_MOVEMENT)) return -1;
    if (!legitMove(cm, dr, srcBroker, ActionType::INTER_BROKER_REPLICA_MOVEMENT)) continue;
    if (!selfSatisfied(cm, swap)) return -1;
    Acceptance acc = isProposalAcceptableForOptimizedGoals(g, swap, cm);
    if (acc == Acceptance::ACCEPT) {
      int dp = cm.replicas[dr].partition;
      cm.relocateReplica(sr.partition, srcBroker, destBroker);
      cm.relocateReplica(dp, destBroker, srcBroker);
      return dr;
    } else if (acc == Acceptance::BROKER_REJECT) {
      return -1;
    }
  }
  return -1;
}

// ===================================================================== ReplicaDistributionGoal
bool ReplicaDistributionGoal::underUpperAfter(const ClusterModel& cm, int b, int count, bool add) const {
  int lim = cm.brokers[b].isAlive() ? upper_ : 0;
  return add ? count + 1 <= lim : count - 1 <= lim;
}
bool ReplicaDistributionGoal::aboveLowerAfter(const ClusterModel& cm, int b, int count, bool add) const {
  int lim = cm.brokers[b].isAlive() ? lower_ : 0;
  return add ? count + 1 >= lim : count - 1 >= lim;
}

// ReplicaDistributionGoal.actionAcceptance (ReplicaDistributionGoal.java:119-138)
Acceptance ReplicaDistributionGoal::actionAcceptance(const BalancingAction& a, ClusterModel& cm) {
  switch (a.type) {
    case ActionType::INTER_BROKER_REPLICA_SWAP:
    case ActionType::LEADERSHIP_MOVEMENT:
      return Acceptance::ACCEPT;
    case ActionType::INTER_BROKER_REPLICA_MOVEMENT: {
      int s = a.sourceBroker, d = a.destinationBroker;
      bool ok = underUpperAfter(cm, d, (int)cm.brokers[d].replicas.size(), true) &&
                (isExcludedForReplicaMove(cm, s) || aboveLowerAfter(cm, s, (int)cm.brokers[s].replicas.size(), false));
      return ok ? Acceptance::ACCEPT : Acceptance::REPLICA_REJECT;
    }
    default:
      throw std::invalid_argument("Unsupported balancing action");
  }
}

// ReplicaDistributionGoalStatsComparator (ReplicaDistributionGoal.java:342-362)
int ReplicaDistributionGoal::compareStats(const ClusterModelStats& s1, const ClusterModelStats& s2) const {
  double d1 = s1.repStd, d2 = s2.repStd;
  const double eps = 1e-5;
  if (d1 - d2 > eps) return -1;  // AnalyzerUtils.compare(stDev2, stDev1, EPSILON)
  if (d2 - d1 > eps) return 1;
  return 0;
}

// ReplicaDistributionAbstractGoal.initGoalState + ReplicaDistributionGoal.initGoalState
void ReplicaDistributionGoal::initGoalState(ClusterModel& cm, const OptimizationOptions& o) {
  allowed_.assign(cm.brokers.size(), 0);
  numAllowed_ = 0;
  for (int b : cm.aliveBrokers())
    if (!o.excludedBrokersForReplicaMove.count(cm.brokers[b].id)) {
      allowed_[b] = 1;
      numAllowed_++;
    }
  if (numAllowed_ == 0)
    throw OptimizationFailure("[" + name() + "] All alive brokers are excluded from replica moves.",
                              underBrokers(cm.maxReplicationFactor));
  avgReplicasOnAliveBroker_ = cm.numReplicas() / (double)numAllowed_;
  fixOfflineReplicasOnly_ = false;
  double adj = (bc_.replicaBalancePercentage - 1) * 0.9;
  upper_ = (int)std::ceil(avgReplicasOnAliveBroker_ * (1 + adj));
  lower_ = (int)std::floor(avgReplicasOnAliveBroker_ * jmax(0, (1 - adj)));
  bool selfHealing = !cm.selfHealingEligibleReplicas.empty();
  for (size_t b = 0; b < cm.brokers.size(); ++b) {
    SortSpec spec;
    if (o.onlyMoveImmigrantReplicas) spec.selection.push_back({SelFn::IMMIGRANTS});
    if (selfHealing && cm.brokers[b].isAlive()) spec.selection.push_back({SelFn::IMMIGRANT_OR_OFFLINE});
    if (!o.excludedTopics.empty()) spec.selection.push_back({SelFn::EXCLUDED_TOPICS});
    if (selfHealing) spec.priority.push_back(PrioFn::OFFLINE);
    if (!o.onlyMoveImmigrantReplicas) spec.priority.push_back(PrioFn::IMMIGRANTS);
    spec.score = ScoreFn::BY_GROUP;
    spec.scoreResource = DISK;
    cm.trackSortedReplicas((int)b, replicaSortName(false, false), spec);
  }
}

// ReplicaDistributionAbstractGoal.updateGoalState (:187-229), then ReplicaDistributionGoal's provisioning
// (ReplicaDistributionGoal.java:85-107), every round
void ReplicaDistributionGoal::updateGoalState(ClusterModel& cm, const OptimizationOptions&) {
  [&] {
    if (!aboveUpper_.empty()) {
      aboveUpper_.clear();
      succeeded_ = false;
    }
    if (!underLower_.empty()) {
      underLower_.clear();
      succeeded_ = false;
    }
    try {
      ensureNoOfflineReplicas(cm, name());
    } catch (OptimizationFailure&) {
      if (fixOfflineReplicasOnly_) throw;
      fixOfflineReplicasOnly_ = true;
      return;
    }
    ensureReplicasMoveOffBrokersWithBadDisks(cm, name());
    finished_ = true;
  }();
  const int allowedNumBrokers = (int)(cm.numReplicas() / bc_.overprovisionedMaxReplicasPerBroker);
  const int numBrokersToDrop = numAllowed_ - allowedNumBrokers;
  bool anyAboveMax = false;
  for (int b : cm.aliveBrokers())
    if ((int64_t)cm.brokers[b].replicas.size() > bc_.overprovisionedMaxReplicasPerBroker) anyAboveMax = true;
  if (numBrokersToDrop > 0 && !anyAboveMax) {
    ProvisionRec rec;
    rec.status = PROV_OVER;
    rec.numBrokers = numBrokersToDrop;
    provision_ = ProvisionResp{PROV_OVER, true, rec};
  } else {
    provision_ = ProvisionResp{PROV_RIGHT_SIZED};
  }
}

bool ReplicaDistributionGoal::selfSatisfied(ClusterModel& cm, const BalancingAction& a) {
  int sr = cm.replicaOnBroker(a.partition, a.sourceBroker);
  if (fixOfflineReplicasOnly_ && cm.isCurrentOffline(sr)) return true;
  return actionAcceptance(a, cm) == Acceptance::ACCEPT;
}

// ReplicaDistributionGoal.rebalanceForBroker (ReplicaDistributionGoal.java:181-224)
void ReplicaDistributionGoal::rebalanceForBroker(int b, ClusterModel& cm, const GoalList& g,
                                                 const OptimizationOptions& o) {
  const Broker& br = cm.brokers[b];
  int numReplicas = (int)br.replicas.size();
  int numOffline = br.numOffline;
  bool excluded = isExcludedForReplicaMove(cm, b);
  bool requireLess = numOffline > 0 || numReplicas > upper_ || excluded;
  bool requireMore = !excluded && br.isAlive() && numReplicas - numOffline < lower_;
  if (br.isAlive() && !requireMore && !requireLess) return;
  if (!cm.newBrokers.empty() && !br.isNew() && !requireLess) return;
  if (((!cm.selfHealingEligibleReplicas.empty() && br.numOffline == 0) || o.onlyMoveImmigrantReplicas) && requireLess &&
      br.numImmigrants == 0)
    return;
  if (requireLess && rebalanceByMovingReplicasOut(b, cm, g, o)) aboveUpper_.insert(b);
  if (requireMore && rebalanceByMovingReplicasIn(b, cm, g, o)) underLower_.insert(b);
}

// ReplicaDistributionGoal.rebalanceByMovingReplicasOut (ReplicaDistributionGoal.java:226-276)
bool ReplicaDistributionGoal::rebalanceByMovingReplicasOut(int b, ClusterModel& cm, const GoalList& g,
                                                           const OptimizationOptions& o) {
  JTreeSet candidates([&cm](int x, int y) {
    int c = icompare((int)cm.brokers[x].replicas.size(), (int)cm.brokers[y].replicas.size());
    return c != 0 ? c : icompare(cm.brokers[x].id, cm.brokers[y].id);
  });
  std::vector<int> toAdd;
  if (fixOfflineReplicasOnly_) {
    toAdd = cm.aliveBrokers();
  } else {
    std::vector<int> filtered;
    for (int x : cm.aliveBrokers())
      if ((int)cm.brokers[x].replicas.size() < upper_) filtered.push_back(x);
    toAdd = javaHashSetOrderIntKeys(filtered);  // Collectors.toSet()
  }
  for (int x : toAdd) candidates.add(x);
  int upperForSource = isExcludedForReplicaMove(cm, b) ? 0 : upper_;
  bool wasUnableToMoveOffline = false;
  std::vector<int> list;
  for (int r : cm.sortedReplicasClone(b, replicaSortName(false, false))) {
    if (!cm.isCurrentOffline(r)) {
      if (wasUnableToMoveOffline && (int)cm.brokers[b].replicas.size() <= upperForSource) return false;
    }
    candidates.toVector(list);
    int dest = maybeApplyBalancingAction(cm, r, list, ActionType::INTER_BROKER_REPLICA_MOVEMENT, g, o);
    if (dest >= 0) {
      if ((int)cm.brokers[b].replicas.size() <= (cm.brokers[b].numOffline == 0 ? upperForSource : 0)) return false;
      candidates.remove(dest);
      if ((int)cm.brokers[dest].replicas.size() < upper_ || fixOfflineReplicasOnly_) candidates.add(dest);
    } else if (cm.isCurrentOffline(r)) {
      wasUnableToMoveOffline = true;
    }
  }
  return !cm.brokers[b].replicas.empty();
}

// ReplicaDistributionGoal.rebalanceByMovingReplicasIn (ReplicaDistributionGoal.java:278-340)
bool ReplicaDistributionGoal::rebalanceByMovingReplicasIn(int dest, ClusterModel& cm, const GoalList& g,
                                                          const OptimizationOptions& o) {
  JPriorityQueue pq([&cm](int b1, int b2) {
    int r = icompare(cm.brokers[b2].numOffline, cm.brokers[b1].numOffline);
    if (r == 0) {
      int r2 = icompare((int)cm.brokers[b2].replicas.size(), (int)cm.brokers[b1].replicas.size());
      return r2 == 0 ? icompare(cm.brokers[b1].id, cm.brokers[b2].id) : r2;
    }
    return r;
  });
  const int B = (int)cm.brokers.size();
  if (fixOfflineReplicasOnly_) {
    for (int s = 0; s < B; ++s)
      if (s != dest) pq.add(s);
  } else {
    for (int s = 0; s < B; ++s)
      if ((int)cm.brokers[s].replicas.size() > lower_ || cm.brokers[s].numOffline > 0 || isExcludedForReplicaMove(cm, s))
        pq.add(s);
  }
  std::vector<int> cand{dest};
  while (!pq.empty()) {
    int src = pq.poll();
    for (int r : cm.sortedReplicasClone(src, replicaSortName(false, false))) {
      int moved = maybeApplyBalancingAction(cm, r, cand, ActionType::INTER_BROKER_REPLICA_MOVEMENT, g, o);
      if (moved >= 0) {
        if ((int)cm.brokers[dest].replicas.size() >= lower_) return false;
        if (!pq.empty()) {
          int top = pq.peek();
          int res = icompare(cm.brokers[src].numOffline, cm.brokers[top].numOffline);
          if (res == -1 || (res == 0 && cm.brokers[src].replicas.size() < cm.brokers[top].replicas.size())) {
            pq.add(src);
            break;
          }
        }
      }
    }
  }
  return true;
}

// ===================================================================== ResourceDistributionGoal
std::string ResourceDistributionGoal::name() const {
  switch (resource_) {
    case CPU: return "CpuUsageDistributionGoal";
    case NW_IN: return "NetworkInboundUsageDistributionGoal";
    case NW_OUT: return "NetworkOutboundUsageDistributionGoal";
    default: return "DiskUsageDistributionGoal";
  }
}

std::vector<int> ResourceDistributionGoal::brokersToBalance(ClusterModel& cm) {
  if (cm.newBrokers.empty()) return AbstractGoal::brokersToBalance(cm);
  return std::vector<int>(cm.newBrokers.begin(), cm.newBrokers.end());
}

// ResourceDistributionGoal.isLoadAboveBalanceLowerLimitAfterChange (:880-902); replicaLoadOf < 0 => null load
bool ResourceDistributionGoal::aboveLowerAfterChange(ClusterModel& cm, int r, int b, bool add) {
  double delta = r < 0 ? 0 : cm.replicaUtil(r, resource_);
  double lim = cm.brokers[b].capacity[resource_] * lowerThr_;
  double u = cm.brokerUtil(b, resource_);
  bool brokerAbove = add ? u + delta >= lim : u - delta >= lim;
  if (isHostResource(resource_)) {
    double hlim = cm.hostCapacity(b, resource_) * lowerThr_;
    double hu = cm.hostUtil(b, resource_);
    bool hostAbove = add ? hu + delta >= hlim : hu - delta >= hlim;
    return hostAbove || brokerAbove;
  }
  return brokerAbove;
}
// ResourceDistributionGoal.isLoadUnderBalanceUpperLimitAfterChange (:904-927)
bool ResourceDistributionGoal::underUpperAfterChange(ClusterModel& cm, int r, int b, bool add, double thr) {
  double delta = r < 0 ? 0 : cm.replicaUtil(r, resource_);
  double lim = cm.brokers[b].capacity[resource_] * thr;
  double u = cm.brokerUtil(b, resource_);
  bool brokerUnder = add ? u + delta <= lim : u - delta <= lim;
  if (isHostResource(resource_)) {
    double hlim = cm.hostCapacity(b, resource_) * thr;
    double hu = cm.hostUtil(b, resource_);
    bool hostUnder = add ? hu + delta <= hlim : hu - delta <= hlim;
    return hostUnder || brokerUnder;
  }
  return brokerUnder;
}
// :943-980
bool ResourceDistributionGoal::isAcceptableAfterReplicaMove(ClusterModel& cm, int sr, int dest) {
  double delta = -cm.replicaUtil(sr, resource_);
  return isGettingMoreBalanced(cm, cm.replicas[sr].broker, delta, dest);
}
bool ResourceDistributionGoal::isSelfSatisfiedAfterSwap(ClusterModel& cm, int sr, int dr) {
  double delta = cm.replicaUtil(dr, resource_) - cm.replicaUtil(sr, resource_);
  return isGettingMoreBalanced(cm, cm.replicas[sr].broker, delta, cm.replicas[dr].broker);
}
bool ResourceDistributionGoal::isGettingMoreBalanced(ClusterModel& cm, int sb, double delta, int db) {
  double su = cm.brokerUtil(sb, resource_), du = cm.brokerUtil(db, resource_);
  double sc = cm.brokers[sb].capacity[resource_], dc = cm.brokers[db].capacity[resource_];
  double prevDiff = (su / sc) - (du / dc);
  double nextDiff = prevDiff + (delta / sc) + (delta / dc);
  return std::fabs(nextDiff) < std::fabs(prevDiff);
}
// :982-1037
bool ResourceDistributionGoal::isSwapViolatingLimit(ClusterModel& cm, int sr, int dr) {
  double delta = cm.replicaUtil(dr, resource_) - cm.replicaUtil(sr, resource_);
  bool v = isSwapViolatingContainerLimit(cm, delta, sr, dr, false);
  if (!v || !isHostResource(resource_)) return v;
  return isSwapViolatingContainerLimit(cm, delta, sr, dr, true);
}
// the container is the broker, or with `host` the broker's host (r -> r.broker().host().load() / capacityFor)
bool ResourceDistributionGoal::isSwapViolatingContainerLimit(ClusterModel& cm, double delta, int sr, int dr, bool host) {
  int sb = cm.replicas[sr].broker, db = cm.replicas[dr].broker;
  auto util = [&](int b) { return host ? cm.hostUtil(b, resource_) : cm.brokerUtil(b, resource_); };
  auto cap = [&](int b) { return host ? cm.hostCapacity(b, resource_) : cm.brokers[b].capacity[resource_]; };
  double su = util(sb), du = util(db);
  bool underUpper;
  if (delta > 0) underUpper = su + delta <= cap(sb) * upperThr_;
  else underUpper = du - delta <= cap(db) * upperThr_;
  if (!underUpper) return true;
  bool aboveLower;
  if (delta < 0) aboveLower = su + delta >= cap(sb) * lowerThr_;
  else aboveLower = du - delta >= cap(db) * lowerThr_;
  return !aboveLower;
}

// ResourceDistributionGoal.actionAcceptance (:101-156) + subclass overrides (Disk/NwIn accept leadership moves)
Acceptance ResourceDistributionGoal::actionAcceptance(const BalancingAction& a, ClusterModel& cm) {
  if ((resource_ == DISK || resource_ == NW_IN) && a.type == ActionType::LEADERSHIP_MOVEMENT) return Acceptance::ACCEPT;
  return baseAcceptance(a, cm);
}
Acceptance ResourceDistributionGoal::baseAcceptance(const BalancingAction& a, ClusterModel& cm) {
  int sb = a.sourceBroker, db = a.destinationBroker;
  int sr = cm.replicaOnBroker(a.partition, sb);
  switch (a.type) {
    case ActionType::INTER_BROKER_REPLICA_SWAP: {
      int dr = cm.replicaOnBroker(a.destPartition, db);
      double delta = cm.replicaUtil(dr, resource_) - cm.replicaUtil(sr, resource_);
      if (delta == 0) return Acceptance::ACCEPT;
      bool both = delta > 0 ? (aboveLowerLimit(cm, db) && underUpperLimit(cm, sb))
                            : (aboveLowerLimit(cm, sb) && underUpperLimit(cm, db));
      if (both) return isSwapViolatingLimit(cm, sr, dr) ? Acceptance::REPLICA_REJECT : Acceptance::ACCEPT;
      return isSelfSatisfiedAfterSwap(cm, sr, dr) ? Acceptance::ACCEPT : Acceptance::REPLICA_REJECT;
    }
    case ActionType::INTER_BROKER_REPLICA_MOVEMENT:
    case ActionType::LEADERSHIP_MOVEMENT: {
      bool srcExcluded = isExcludedForReplicaMove(sb);
      if ((srcExcluded || aboveLowerLimit(cm, sb)) && underUpperLimit(cm, db)) {
        return (underUpperAfterChange(cm, sr, db, true) && (srcExcluded || aboveLowerAfterChange(cm, sr, sb, false)))
                   ? Acceptance::ACCEPT
                   : Acceptance::REPLICA_REJECT;
      } else if (srcExcluded) {
        return cm.replicaUtil(sr, resource_) == 0.0 ? Acceptance::ACCEPT : Acceptance::REPLICA_REJECT;
      }
      return isAcceptableAfterReplicaMove(cm, sr, db) ? Acceptance::ACCEPT : Acceptance::REPLICA_REJECT;
    }
    default:
      throw std::invalid_argument("Unsupported balancing action");
  }
}

// ResourceDistributionGoalStatsComparator (:1039-1070)
int ResourceDistributionGoal::compareStats(const ClusterModelStats& s1, const ClusterModelStats& s2) const {
  int n1 = s1.numBalancedBrokersByResource[resource_], n2 = s2.numBalancedBrokersByResource[resource_];
  if (n2 > n1) {
    double after = s1.resStd[resource_], before = s2.resStd[resource_];
    if (dcompare(before, after) < 0) return -1;
  }
  return 1;
}

// ResourceDistributionGoal.selfSatisfied (:199-224)
bool ResourceDistributionGoal::selfSatisfied(ClusterModel& cm, const BalancingAction& a) {
  int db = a.destinationBroker;
  int sr = cm.replicaOnBroker(a.partition, a.sourceBroker);
  if (fixOfflineReplicasOnly_ && cm.isCurrentOffline(sr)) return a.type == ActionType::INTER_BROKER_REPLICA_MOVEMENT;
  switch (a.type) {
    case ActionType::INTER_BROKER_REPLICA_SWAP: {
      int dr = cm.replicaOnBroker(a.destPartition, db);
      double delta = cm.replicaUtil(dr, resource_) - cm.replicaUtil(sr, resource_);
      return delta != 0 && !isSwapViolatingLimit(cm, sr, dr);
    }
    case ActionType::INTER_BROKER_REPLICA_MOVEMENT:
    case ActionType::LEADERSHIP_MOVEMENT:
      return underUpperAfterChange(cm, sr, db, true) && aboveLowerAfterChange(cm, sr, cm.replicas[sr].broker, false);
    default:
      throw std::invalid_argument("Unsupported balancing action");
  }
}

// ResourceDistributionGoal.initGoalState (:234-278)
void ResourceDistributionGoal::initGoalState(ClusterModel& cm, const OptimizationOptions& o) {
  allowed_.assign(cm.brokers.size(), 0);
  int n = 0;
  for (int b : cm.aliveBrokers())
    if (!o.excludedBrokersForReplicaMove.count(cm.brokers[b].id)) {
      allowed_[b] = 1;
      n++;
    }
  if (n == 0)
    throw OptimizationFailure("[" + name() + "] All alive brokers are excluded from replica moves.",
                              underBrokers(cm.maxReplicationFactor));
  fixOfflineReplicasOnly_ = false;
  double resourceUtilization = expectedUtil(cm.load, resource_, cm.W);
  double capacity = cm.capacityWithAllowedReplicaMovesFor(resource_, o);
  double avgPct = resourceUtilization / capacity;
  upperThr_ = computeResourceUtilizationBalanceThreshold(avgPct, resource_, bc_, o.triggeredByGoalViolation, 0.9, false);
  lowerThr_ = computeResourceUtilizationBalanceThreshold(avgPct, resource_, bc_, o.triggeredByGoalViolation, 0.9, true);
  isLowUtilization_ = avgPct <= bc_.lowUtilizationThreshold[resource_];
  if (isLowUtilization_) {
    // brokerIdWithMaxCapacity over _brokersAllowedReplicaMove (a HashSet<Integer>, strict >) (:268-296)
    std::vector<int> ids;
    for (int b : cm.aliveBrokers())
      if (allowed_[b]) ids.push_back(b);
    int typical = -1;
    double maxCapacity = 0.0;
    for (int b : javaHashSetOrderIntKeys(ids))
      if (cm.brokers[b].capacity[resource_] > maxCapacity) {
        typical = b;
        maxCapacity = cm.brokers[b].capacity[resource_];
      }
    const double typicalCapacity = cm.brokers[typical].capacity[resource_];
    const double allowedCapacity = resourceUtilization / bc_.lowUtilizationThreshold[resource_];
    const int allowedNumBrokers = (int)(allowedCapacity / typicalCapacity);
    overRec_ = ProvisionRec{};
    overRec_.status = PROV_OVER;
    overRec_.numBrokers = std::max(n - allowedNumBrokers, 1);
    overRec_.typicalBrokerCapacity = typicalCapacity;
    overRec_.typicalBrokerId = cm.brokers[typical].id;
    overRec_.resource = resource_;
  }
}

// ResourceDistributionGoal.updateGoalState (:301-349)
void ResourceDistributionGoal::updateGoalState(ClusterModel& cm, const OptimizationOptions&) {
  bool anyAbove = false, anyUnder = false;
  for (int b : cm.aliveBrokers()) {
    if (!underUpperLimit(cm, b)) anyAbove = true;
    if (!isExcludedForReplicaMove(b) && !aboveLowerLimit(cm, b)) anyUnder = true;
  }
  if (anyAbove) succeeded_ = false;
  else if (isLowUtilization_) provision_ = ProvisionResp{PROV_OVER, true, overRec_};
  if (anyUnder) succeeded_ = false;
  else if (!anyAbove && !isLowUtilization_) provision_ = ProvisionResp{PROV_RIGHT_SIZED};
  try {
    ensureNoOfflineReplicas(cm, name());
  } catch (OptimizationFailure&) {
    if (fixOfflineReplicasOnly_) throw;
    fixOfflineReplicasOnly_ = true;
    return;
  }
  ensureReplicasMoveOffBrokersWithBadDisks(cm, name());
  finished_ = true;
}

// ResourceDistributionGoal.rebalanceForBroker (:379-435)
void ResourceDistributionGoal::rebalanceForBroker(int b, ClusterModel& cm, const GoalList& g,
                                                  const OptimizationOptions& o) {
  int numOffline = cm.brokers[b].numOffline;
  bool excluded = isExcludedForReplicaMove(b);
  bool requireLess = numOffline > 0 || excluded || !underUpperLimit(cm, b);
  bool requireMore = !excluded && !aboveLowerLimit(cm, b);
  bool moveImmigrantsOnly = false;
  if (cm.brokers[b].numOffline == 0) {
    if (!requireMore && !requireLess) return;
    moveImmigrantsOnly = !cm.selfHealingEligibleReplicas.empty() || o.onlyMoveImmigrantReplicas;
    if (moveImmigrantsOnly && requireLess && cm.brokers[b].numImmigrants == 0) return;
  }
  if ((resource_ == NW_OUT || resource_ == CPU) && !(fixOfflineReplicasOnly_ && cm.brokers[b].numOffline > 0)) {
    if (requireLess && !rebalanceByMovingLoadOut(b, cm, g, ActionType::LEADERSHIP_MOVEMENT, o)) requireLess = false;
    if (requireMore && !rebalanceByMovingLoadIn(b, cm, g, ActionType::LEADERSHIP_MOVEMENT, o, false)) requireMore = false;
  }
  bool unbalanced = false;
  if (requireLess) {
    if (rebalanceByMovingLoadOut(b, cm, g, ActionType::INTER_BROKER_REPLICA_MOVEMENT, o))
      unbalanced = rebalanceBySwappingLoadOut(b, cm, g, o, moveImmigrantsOnly);
  }
  if (requireMore) {
    if (rebalanceByMovingLoadIn(b, cm, g, ActionType::INTER_BROKER_REPLICA_MOVEMENT, o, moveImmigrantsOnly))
      unbalanced = unbalanced || rebalanceBySwappingLoadIn(b, cm, g, o, moveImmigrantsOnly);
  }
  (void)unbalanced;
}

// ResourceDistributionGoal.sortedCandidateReplicas (:543-569)
std::string ResourceDistributionGoal::sortedCandidateReplicas(int b, ClusterModel& cm, const OptimizationOptions& o,
                                                              double loadLimit, bool isAscending, bool followersOnly,
                                                              bool leadersOnly, bool immigrantsOnly) {
  SortSpec spec;
  if (followersOnly) spec.selection.push_back({SelFn::FOLLOWERS});
  if (leadersOnly) spec.selection.push_back({SelFn::LEADERS});
  if (immigrantsOnly) spec.selection.push_back({SelFn::IMMIGRANTS});
  if (!o.excludedTopics.empty()) spec.selection.push_back({SelFn::EXCLUDED_TOPICS});
  if (!cm.selfHealingEligibleReplicas.empty()) spec.priority.push_back(PrioFn::OFFLINE);
  if (isAscending) {
    if (loadLimit < 1.7976931348623157e308) spec.selection.push_back({SelFn::BELOW_LIMIT, resource_, loadLimit});
    spec.score = ScoreFn::BY_GROUP;
  } else {
    spec.selection.push_back({SelFn::ABOVE_LIMIT, resource_, loadLimit});
    spec.score = ScoreFn::REVERSE_BY_GROUP;
  }
  spec.scoreResource = resource_;
  std::string nm = replicaSortName(!isAscending, leadersOnly);
  cm.trackSortedReplicas(b, nm, spec);
  return nm;
}

// getMaxReplicaLoad / getMinReplicaLoad (:571-597)
double ResourceDistributionGoal::getMaxReplicaLoad(ClusterModel& cm, const std::vector<int>& s) const {
  double m = cm.replicaUtil(s.front(), resource_);
  for (int r : s) {
    if (cm.isCurrentOffline(r)) continue;
    if (cm.replicaUtil(r, resource_) > m) m = cm.replicaUtil(r, resource_);
    break;
  }
  return m;
}
double ResourceDistributionGoal::getMinReplicaLoad(ClusterModel& cm, const std::vector<int>& s) const {
  double m = cm.replicaUtil(s.front(), resource_);
  for (int r : s) {
    if (cm.isCurrentOffline(r)) continue;
    if (cm.replicaUtil(r, resource_) < m) m = cm.replicaUtil(r, resource_);
    break;
  }
  return m;
}

// ResourceDistributionGoal.rebalanceByMovingLoadIn (:437-526)
bool ResourceDistributionGoal::rebalanceByMovingLoadIn(int b, ClusterModel& cm, const GoalList& g, ActionType at,
                                                       const OptimizationOptions& o, bool moveImmigrantsOnly) {
  if (!cm.newBrokers.empty() && !cm.brokers[b].isNew()) return true;
  bool moveFollowersOnly = o.excludedBrokersForLeadership.count(cm.brokers[b].id) > 0;
  JPriorityQueue pq([this, &cm](int x, int y) { return cmpBroker(cm, y, x); });  // _brokerComparator.reversed()
  std::string sortName;
  bool haveName = false;
  for (int c : cm.aliveBrokers()) {
    if (cm.utilizationPct(c, resource_) > (isExcludedForReplicaMove(c) ? 0.0 : lowerThr_)) {
      sortName = sortedCandidateReplicas(c, cm, o, 0.0, false, moveFollowersOnly, resource_ == NW_OUT, moveImmigrantsOnly);
      haveName = true;
      pq.add(c);
    }
  }
  std::vector<int> single{b};
  while (!pq.empty() && (at == ActionType::INTER_BROKER_REPLICA_MOVEMENT ||
                         (at == ActionType::LEADERSHIP_MOVEMENT &&
                          cm.brokers[b].numLeaders != (int)cm.brokers[b].replicas.size()))) {
    int cb = pq.poll();
    const auto& view = cm.sortedReplicasView(cb, sortName);  // live unmodifiable view
    bool ready = false;
    int indicesToSkip = 0;
    while (!ready) {
      int iterated = indicesToSkip;
      int maxIdx = (int)view.size();
      bool moved = false;
      for (auto it = view.begin(); it != view.end(); ++it) {
        if (indicesToSkip > 0) {
          indicesToSkip--;
          continue;
        }
        int r = *it;
        int dst = maybeApplyBalancingAction(cm, r, single, at, g, o);
        if (dst >= 0) {
          if (aboveLowerLimit(cm, b)) {
            cm.untrackSortedReplicas(sortName);
            return false;
          }
          indicesToSkip = iterated;
          if (!pq.empty() && cm.utilizationPct(cb, resource_) < cm.utilizationPct(pq.peek(), resource_)) {
            pq.add(cb);
            ready = true;
          }
          moved = true;
          break;
        }
        iterated++;
      }
      (void)moved;
      if (iterated == maxIdx) ready = true;
    }
  }
  if (haveName) cm.untrackSortedReplicas(sortName);
  return true;
}

// ResourceDistributionGoal.rebalanceBySwappingLoadOut (:599-687)
bool ResourceDistributionGoal::rebalanceBySwappingLoadOut(int b, ClusterModel& cm, const GoalList& g,
                                                          const OptimizationOptions& o, bool moveImmigrantsOnly) {
  if (!cm.brokers[b].isAlive() || o.excludedBrokersForReplicaMove.count(cm.brokers[b].id)) return true;
  std::string srcName = sortedCandidateReplicas(b, cm, o, 0.0, false, false, resource_ == NW_OUT, moveImmigrantsOnly);
  if (cm.sortedReplicasView(b, srcName).empty()) {
    cm.brokerUntrackSortedReplicas(b, srcName);
    return true;
  }
  std::vector<int> srcSnapshot = cm.sortedReplicasClone(b, srcName);
  double maxSrcLoad = getMaxReplicaLoad(cm, srcSnapshot);
  bool followersOnly = o.excludedBrokersForLeadership.count(cm.brokers[b].id) > 0;
  JPriorityQueue pq([this, &cm](int x, int y) { return cmpBroker(cm, x, y); });
  std::string candName;
  std::vector<int> under;
  for (int c : cm.aliveBrokersUnderThreshold(resource_, upperThr_))
    if (!cm.brokers[c].replicas.empty()) under.push_back(c);
  for (int c : javaHashSetOrderIntKeys(under)) {
    candName = sortedCandidateReplicas(c, cm, o, maxSrcLoad, true, followersOnly, false, moveImmigrantsOnly);
    pq.add(c);
  }
  std::vector<int> candSnapshot;
  while (!pq.empty()) {
    int cb = pq.poll();
    int swappedIn = -1;
    const auto& srcView = cm.sortedReplicasView(b, srcName);
    for (auto it = srcView.begin(); it != srcView.end(); ++it) {
      int sr = *it;
      const auto& cview = cm.sortedReplicasView(cb, candName);
      candSnapshot.assign(cview.begin(), cview.end());
      int s = maybeApplySwapAction(cm, sr, candSnapshot, g, o);
      if (s >= 0) {
        if (underUpperLimit(cm, b)) {
          cm.clearSortedReplicas();
          return false;
        }
        swappedIn = s;
        break;
      }
    }
    if (swappedIn >= 0) pq.add(cb);
  }
  cm.clearSortedReplicas();
  return true;
}

// ResourceDistributionGoal.rebalanceBySwappingLoadIn (:689-777)
bool ResourceDistributionGoal::rebalanceBySwappingLoadIn(int b, ClusterModel& cm, const GoalList& g,
                                                         const OptimizationOptions& o, bool moveImmigrantsOnly) {
  if (!cm.brokers[b].isAlive() || o.excludedBrokersForReplicaMove.count(cm.brokers[b].id)) return true;
  std::string srcName =
      sortedCandidateReplicas(b, cm, o, 1.7976931348623157e308, true, false, false, moveImmigrantsOnly);
  if (cm.sortedReplicasView(b, srcName).empty()) {
    cm.brokerUntrackSortedReplicas(b, srcName);
    return true;
  }
  std::vector<int> srcSnapshot = cm.sortedReplicasClone(b, srcName);
  double minSrcLoad = getMinReplicaLoad(cm, srcSnapshot);
  bool followersOnly = o.excludedBrokersForLeadership.count(cm.brokers[b].id) > 0;
  JPriorityQueue pq([this, &cm](int x, int y) { return cmpBroker(cm, y, x); });
  std::string candName;
  for (int c : cm.aliveBrokersOverThreshold(resource_, lowerThr_)) {
    candName = sortedCandidateReplicas(c, cm, o, minSrcLoad, false, followersOnly, resource_ == NW_OUT, moveImmigrantsOnly);
    pq.add(c);
  }
  std::vector<int> candSnapshot;
  while (!pq.empty()) {
    int cb = pq.poll();
    int swappedIn = -1;
    const auto& srcView = cm.sortedReplicasView(b, srcName);
    for (auto it = srcView.begin(); it != srcView.end(); ++it) {
      int sr = *it;
      const auto& cview = cm.sortedReplicasView(cb, candName);
      candSnapshot.assign(cview.begin(), cview.end());
      int s = maybeApplySwapAction(cm, sr, candSnapshot, g, o);
      if (s >= 0) {
        if (aboveLowerLimit(cm, b)) {
          cm.clearSortedReplicas();
          return false;
        }
        swappedIn = s;
        break;
      }
    }
    if (swappedIn >= 0) pq.add(cb);
  }
  cm.clearSortedReplicas();
  return true;
}

// ResourceDistributionGoal.rebalanceByMovingLoadOut (:779-863)
bool ResourceDistributionGoal::rebalanceByMovingLoadOut(int b, ClusterModel& cm, const GoalList& g, ActionType at,
                                                        const OptimizationOptions& o) {
  JTreeSet candidates([this, &cm](int x, int y) { return cmpBroker(cm, x, y); });
  if (fixOfflineReplicasOnly_) {
    for (int x : cm.aliveBrokers()) candidates.add(x);
  } else {
    for (int x : cm.aliveBrokersUnderThreshold(resource_, upperThr_)) candidates.add(x);
  }
  bool selfHealing = !cm.selfHealingEligibleReplicas.empty();
  SortSpec spec;
  if (at == ActionType::LEADERSHIP_MOVEMENT) spec.selection.push_back({SelFn::LEADERS});
  if (o.onlyMoveImmigrantReplicas) spec.selection.push_back({SelFn::IMMIGRANTS});
  if (selfHealing && cm.brokers[b].isAlive()) spec.selection.push_back({SelFn::IMMIGRANT_OR_OFFLINE});
  if (!o.excludedTopics.empty()) spec.selection.push_back({SelFn::EXCLUDED_TOPICS});
  if (selfHealing) spec.priority.push_back(PrioFn::OFFLINE);
  if (!o.onlyMoveImmigrantReplicas) spec.priority.push_back(PrioFn::IMMIGRANTS);
  spec.score = ScoreFn::REVERSE_BY_GROUP;
  spec.scoreResource = resource_;
  std::string nm = replicaSortName(true, at == ActionType::LEADERSHIP_MOVEMENT);
  cm.trackSortedReplicas(b, nm, spec);
  std::vector<int> toMove = cm.sortedReplicasClone(b, nm);
  double upperForSource = isExcludedForReplicaMove(b) ? 0 : upperThr_;
  std::vector<int> list;
  for (int r : toMove) {
    if (!cm.isCurrentOffline(r)) {
      if (cm.replicaUtil(r, resource_) == 0.0) break;
    }
    if (at == ActionType::LEADERSHIP_MOVEMENT) {
      list.clear();
      for (int fb : cm.onlineFollowerBrokers(cm.replicas[r].partition))
        if (candidates.contains(fb)) list.push_back(fb);
      std::sort(list.begin(), list.end(), [&](int x, int y) { return cmpBroker(cm, x, y) < 0; });
      list.erase(std::unique(list.begin(), list.end()), list.end());
    } else {
      candidates.toVector(list);
    }
    int dst = maybeApplyBalancingAction(cm, r, list, at, g, o);
    if (dst >= 0) {
      if (underUpperAfterChange(cm, -1, b, false, upperForSource) &&
          !(fixOfflineReplicasOnly_ && cm.brokers[b].numOffline > 0)) {
        cm.brokerClearSortedReplicas(b);
        return false;
      }
      candidates.remove(dst);
      if (cm.utilizationPct(dst, resource_) < upperThr_) candidates.add(dst);
    }
  }
  cm.brokerClearSortedReplicas(b);
  return !cm.brokers[b].replicas.empty();
}

}  // namespace oracle
