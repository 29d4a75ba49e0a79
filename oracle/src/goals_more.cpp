// ORACLE — test infrastructure only (see jsem.h header). Line-by-line restatement of the remaining
// default goals (RackAware, MinTopicLeadersPerBroker, ReplicaCapacity, Capacity x4, PotentialNwOut,
// TopicReplicaDistribution, LeaderReplicaDistribution, LeaderBytesInDistribution). Every method names the
// reference method it follows; file paths are relative to
// cruise-control/src/main/java/com/linkedin/kafka/cruisecontrol/analyzer/goals/.
#include <algorithm>
#include <cmath>

#include "brokersets.h"
#include "goals.h"

namespace oracle {

namespace {

std::vector<int> sortedBy(std::vector<int> v, const std::function<int(int, int)>& cmp) {
  std::stable_sort(v.begin(), v.end(), [&](int a, int b) { return cmp(a, b) < 0; });
  return v;
}

// GoalUtils.aliveBrokersNotExcludedForReplicaMove (GoalUtils.java:476-484) as a membership vector
std::vector<char> allowedForReplicaMove(const ClusterModel& cm, const OptimizationOptions& o, int* count) {
  std::vector<char> allowed(cm.brokers.size(), 0);
  int n = 0;
  for (int b : cm.aliveBrokers())
    if (!o.excludedBrokersForReplicaMove.count(cm.brokers[b].id)) {
      allowed[b] = 1;
      n++;
    }
  if (count) *count = n;
  return allowed;
}

bool hasOfflineReplicas(const ClusterModel& cm, int b) { return cm.brokers[b].offlineSet.size() > 0; }

}  // namespace

// ===================================================================== RackAwareGoal
// RackAwareGoal.doesReplicaMoveViolateActionAcceptance (RackAwareGoal.java:57-66): any OTHER broker of the
// partition on the destination's rack
bool RackAwareGoal::violates(ClusterModel& cm, int r, int dst) const {
  const int self = cm.replicas[r].broker, dstRack = cm.brokers[dst].rack;
  for (int x : cm.partitions[cm.replicas[r].partition].replicas) {
    const int b = cm.replicas[x].broker;
    if (b != self && cm.brokers[b].rack == dstRack) return true;
  }
  return false;
}

// AbstractRackAwareGoal.actionAcceptance (AbstractRackAwareGoal.java:90-117)
Acceptance RackAwareGoal::actionAcceptance(const BalancingAction& a, ClusterModel& cm) {
  switch (a.type) {
    case ActionType::LEADERSHIP_MOVEMENT:
      return Acceptance::ACCEPT;
    case ActionType::INTER_BROKER_REPLICA_MOVEMENT:
    case ActionType::INTER_BROKER_REPLICA_SWAP: {
      if (violates(cm, cm.replicaOnBroker(a.partition, a.sourceBroker), a.destinationBroker))
        return Acceptance::BROKER_REJECT;
      if (a.type == ActionType::INTER_BROKER_REPLICA_SWAP &&
          violates(cm, cm.replicaOnBroker(a.destPartition, a.destinationBroker), a.sourceBroker))
        return Acceptance::REPLICA_REJECT;
      return Acceptance::ACCEPT;
    }
    default:
      throw std::invalid_argument("Unsupported balancing action");
  }
}

// RackAwareGoal.initGoalState (RackAwareGoal.java:82-124)
void RackAwareGoal::initGoalState(ClusterModel& cm, const OptimizationOptions& o) {
  std::set<int> aliveRacks;
  for (int b : cm.aliveBrokers()) aliveRacks.insert(cm.brokers[b].rack);
  const int numAliveRacks = (int)aliveRacks.size();
  if (!o.excludedTopics.empty()) {
    // replicationFactorByTopic entries in HashMap<String, Integer> order: the first included topic whose
    // replication factor exceeds the alive racks names the shortfall (RackAwareGoal.java:77-94)
    JHashSet byTopic([&cm](int x, int y) { return cm.topicNames[x].compare(cm.topicNames[y]); });
    for (int t = 0; t < cm.numTopics(); ++t) byTopic.add(t, cm.topicHash[t]);
    int maxIncluded = 1;
    for (int t : byTopic.order()) {
      if (o.excludedTopics.count(t)) continue;
      maxIncluded = std::max(maxIncluded, cm.replicationFactorByTopic[t]);
      if (maxIncluded > numAliveRacks) {
        ProvisionRec rec;
        rec.numRacks = maxIncluded - numAliveRacks;
        throw OptimizationFailure("[RackAwareGoal] Insufficient number of racks to distribute included replicas (Current: " +
                                      std::to_string(numAliveRacks) + ", Needed: " + std::to_string(maxIncluded) + ").",
                                  rec);
      }
    }
  } else if (cm.maxReplicationFactor > numAliveRacks) {
    ProvisionRec rec;
    rec.numRacks = cm.maxReplicationFactor - numAliveRacks;
    throw OptimizationFailure("[RackAwareGoal] Insufficient number of racks to distribute each replica (Current: " +
                                  std::to_string(numAliveRacks) + ", Needed: " + std::to_string(cm.maxReplicationFactor) +
                                  ").",
                              rec);
  }
  // over-provisioned in racks (:103-109)
  const int numExtraRacks = numAliveRacks - cm.maxReplicationFactor;
  if (numExtraRacks >= bc_.overprovisionedMinExtraRacks) {
    ProvisionRec rec;
    rec.status = PROV_OVER;
    rec.numRacks = numExtraRacks - bc_.overprovisionedMinExtraRacks + 1;
    provision_ = ProvisionResp{PROV_OVER, true, rec};
  }
  SortSpec spec;
  if (o.onlyMoveImmigrantReplicas) spec.selection.push_back({SelFn::IMMIGRANTS});
  if (!o.excludedTopics.empty()) spec.selection.push_back({SelFn::EXCLUDED_TOPICS});
  for (size_t b = 0; b < cm.brokers.size(); ++b) cm.trackSortedReplicas((int)b, replicaSortName(false, false), spec);
}

// RackAwareGoal.updateGoalState (RackAwareGoal.java:131-143) + ensureRackAware (:159-185): partitions of excluded
// topics are not checked
void RackAwareGoal::updateGoalState(ClusterModel& cm, const OptimizationOptions& o) {
  for (size_t p = 0; p < cm.partitions.size(); ++p) {
    if (o.excludedTopics.count(cm.partitions[p].topic)) continue;
    std::set<int> racks;
    for (int r : cm.partitions[p].replicas) racks.insert(cm.brokers[cm.replicas[r].broker].rack);
    if (racks.size() != cm.partitions[p].replicas.size()) {
      ProvisionRec rec;
      rec.numRacks = (int)(cm.partitions[p].replicas.size() - racks.size());
      throw OptimizationFailure("[RackAwareGoal] Partition " + std::to_string(p) + " is not rack-aware.", rec);
    }
  }
  ensureNoOfflineReplicas(cm, name());
  ensureReplicasMoveOffBrokersWithBadDisks(cm, name());
  if (provision_.status != PROV_OVER) provision_ = ProvisionResp{PROV_RIGHT_SIZED};
  finished_ = true;
}

// RackAwareGoal.shouldKeepInTheCurrentBroker (RackAwareGoal.java:214-225)
bool RackAwareGoal::shouldKeepInTheCurrentBroker(ClusterModel& cm, int r) const {
  const int self = cm.replicas[r].broker, myRack = cm.brokers[self].rack;
  for (int x : cm.partitions[cm.replicas[r].partition].replicas) {
    const int b = cm.replicas[x].broker;
    if (cm.brokers[b].rack == myRack && b != self) return false;
  }
  return true;
}

// RackAwareGoal.rackAwareEligibleBrokers (RackAwareGoal.java:193-211): alive brokers (by id) whose rack is not
// in the partition's rack list with ONE occurrence of the replica's own rack removed
std::vector<int> RackAwareGoal::rackAwareEligibleBrokers(ClusterModel& cm, int r) const {
  std::vector<int> racks;
  for (int b : cm.partitionBrokersSet(cm.replicas[r].partition)) racks.push_back(cm.brokers[b].rack);
  auto it = std::find(racks.begin(), racks.end(), cm.brokers[cm.replicas[r].broker].rack);
  if (it != racks.end()) racks.erase(it);
  std::vector<int> out;
  for (int b : cm.aliveBrokers())
    if (std::find(racks.begin(), racks.end(), cm.brokers[b].rack) == racks.end()) out.push_back(b);
  return out;
}

// AbstractRackAwareGoal.rebalanceForBroker (AbstractRackAwareGoal.java:144-170), throwExceptionIfCannotMove = true
void RackAwareGoal::rebalanceForBroker(int b, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o) {
  for (int r : cm.sortedReplicasClone(b, replicaSortName(false, false))) {
    if (cm.brokers[b].isAlive() && !cm.isCurrentOffline(r) && shouldKeepInTheCurrentBroker(cm, r)) continue;
    std::vector<int> eligible = rackAwareEligibleBrokers(cm, r);
    if (maybeApplyBalancingAction(cm, r, eligible, ActionType::INTER_BROKER_REPLICA_MOVEMENT, g, o) < 0)
      throw OptimizationFailure("[RackAwareGoal] Cannot move replica of partition " +
                                    std::to_string(cm.replicas[r].partition) + " to a rack-aware broker.",
                                underBrokers(1));  // AbstractRackAwareGoal.java:162-163 (excludedRackIds not carried)
  }
}

// ===================================================================== RackAwareDistributionGoal
// numPartitionReplicasByRackId (RackAwareDistributionGoal.java:113-119): Partition.partitionBrokers() by rack
std::map<int, int> RackAwareDistributionGoal::numReplicasByRack(const ClusterModel& cm, int p) const {
  std::map<int, int> out;
  for (int b : cm.partitionBrokersSet(p)) out[cm.brokers[b].rack] += 1;
  return out;
}

static int getOrZero(const std::map<int, int>& m, int k) {
  auto it = m.find(k);
  return it == m.end() ? 0 : it->second;
}

// doesReplicaMoveViolateActionAcceptance (:88-104)
bool RackAwareDistributionGoal::violates(ClusterModel& cm, int r, int dst) const {
  const int dstRack = cm.brokers[dst].rack, srcRack = cm.brokers[cm.replicas[r].broker].rack;
  if (srcRack == dstRack) return false;
  const std::map<int, int> n = numReplicasByRack(cm, cm.replicas[r].partition);
  return getOrZero(n, dstRack) >= getOrZero(n, srcRack);
}

// AbstractRackAwareGoal.actionAcceptance (AbstractRackAwareGoal.java:96-118)
Acceptance RackAwareDistributionGoal::actionAcceptance(const BalancingAction& a, ClusterModel& cm) {
  switch (a.type) {
    case ActionType::LEADERSHIP_MOVEMENT:
      return Acceptance::ACCEPT;
    case ActionType::INTER_BROKER_REPLICA_MOVEMENT:
    case ActionType::INTER_BROKER_REPLICA_SWAP:
      if (violates(cm, cm.replicaOnBroker(a.partition, a.sourceBroker), a.destinationBroker))
        return Acceptance::BROKER_REJECT;
      if (a.type == ActionType::INTER_BROKER_REPLICA_SWAP &&
          violates(cm, cm.replicaOnBroker(a.destPartition, a.destinationBroker), a.sourceBroker))
        return Acceptance::REPLICA_REJECT;
      return Acceptance::ACCEPT;
    default:
      throw std::invalid_argument("Unsupported balancing action");
  }
}

// initGoalState (:139-164) with BalanceLimit (:407-427)
void RackAwareDistributionGoal::initGoalState(ClusterModel& cm, const OptimizationOptions& o) {
  int n = 0;
  allowed_ = allowedForReplicaMove(cm, o, &n);
  if (n == 0) {
    ProvisionRec rec;
    rec.numBrokers = cm.maxReplicationFactor;
    throw OptimizationFailure("[" + name() + "] All alive brokers are excluded from replica moves.", rec);
  }
  std::set<int> racks;  // ClusterModel.aliveRacksAllowedReplicaMoves (ClusterModel.java:658-662, Rack.java:146-153)
  for (size_t b = 0; b < cm.brokers.size(); ++b)
    if (allowed_[b]) racks.insert(cm.brokers[b].rack);
  numRacks_ = (int)racks.size();
  if (numRacks_ == 0) {
    ProvisionRec rec;
    rec.numRacks = cm.maxReplicationFactor;
    throw OptimizationFailure("All alive racks are excluded from replica moves.", rec);
  }
  const int numExtraRacks = numRacks_ - cm.maxReplicationFactor;
  if (numExtraRacks >= bc_.overprovisionedMinExtraRacks) {
    ProvisionRec rec;
    rec.status = PROV_OVER;
    rec.numRacks = numExtraRacks - bc_.overprovisionedMinExtraRacks + 1;
    provision_ = ProvisionResp{PROV_OVER, true, rec};
  }
  SortSpec spec;
  if (o.onlyMoveImmigrantReplicas) spec.selection.push_back({SelFn::IMMIGRANTS});
  if (!o.excludedTopics.empty()) spec.selection.push_back({SelFn::EXCLUDED_TOPICS});
  for (size_t b = 0; b < cm.brokers.size(); ++b) cm.trackSortedReplicas((int)b, replicaSortName(false, false), spec);
}

// shouldKeepInTheCurrentBroker (:305-334)
bool RackAwareDistributionGoal::shouldKeepInTheCurrentBroker(ClusterModel& cm, int r) const {
  const int b = cm.replicas[r].broker;
  if (!allowed_[b]) return false;
  const int p = cm.replicas[r].partition;
  const int rf = (int)cm.partitionBrokersSet(p).size();
  const std::map<int, int> n = numReplicasByRack(cm, p);
  const int base = baseLimit(rf), limit = numRacksWithOneMoreReplica(rf);
  const int upper = base + (limit == 0 ? 0 : 1);
  const int here = n.at(cm.brokers[b].rack);
  if (here <= base) return true;
  if (here > upper) return false;
  int over = 0;
  for (const auto& kv : n) over += kv.second > base ? 1 : 0;
  return over <= limit;
}

// rackAwareEligibleBrokers (:246-302): TreeSet by (replicas of the partition on the broker's rack, broker id)
std::vector<int> RackAwareDistributionGoal::rackAwareEligibleBrokers(ClusterModel& cm, int r) const {
  const int p = cm.replicas[r].partition;
  const std::vector<int> partitionBrokers = cm.partitionBrokersSet(p);
  std::map<int, int> n = numReplicasByRack(cm, p);
  n[cm.brokers[cm.replicas[r].broker].rack] -= 1;  // merge(rack, -1, Integer::sum): a 0 entry stays
  const int rf = (int)partitionBrokers.size();
  const int base = baseLimit(rf);
  int over = 0;
  for (const auto& kv : n) over += kv.second > base ? 1 : 0;
  const bool canMoveToRacksAtBaseLimit = over < numRacksWithOneMoreReplica(rf);
  std::vector<int> out;
  for (int b : cm.aliveBrokers()) {
    const int here = getOrZero(n, cm.brokers[b].rack);
    if (here < base || (canMoveToRacksAtBaseLimit && here == base))
      if (std::find(partitionBrokers.begin(), partitionBrokers.end(), b) == partitionBrokers.end()) out.push_back(b);
  }
  std::sort(out.begin(), out.end(), [&](int a, int b) {
    const int ca = getOrZero(n, cm.brokers[a].rack), cb = getOrZero(n, cm.brokers[b].rack);
    return ca != cb ? ca < cb : cm.brokers[a].id < cm.brokers[b].id;
  });
  return out;
}

// AbstractRackAwareGoal.rebalanceForBroker (AbstractRackAwareGoal.java:144-170), throwExceptionIfCannotMove = false
void RackAwareDistributionGoal::rebalanceForBroker(int b, ClusterModel& cm, const GoalList& g,
                                                   const OptimizationOptions& o) {
  for (int r : cm.sortedReplicasClone(b, replicaSortName(false, false))) {
    if (cm.brokers[b].isAlive() && !cm.isCurrentOffline(r) && shouldKeepInTheCurrentBroker(cm, r)) continue;
    maybeApplyBalancingAction(cm, r, rackAwareEligibleBrokers(cm, r), ActionType::INTER_BROKER_REPLICA_MOVEMENT, g, o);
  }
}

// updateGoalState (:175-188) and ensureRackAwareDistribution (:342-383) over clusterModel.leaderReplicas(): a
// HashSet<Replica> filled from the model's partition map
void RackAwareDistributionGoal::updateGoalState(ClusterModel& cm, const OptimizationOptions& o) {
  ensureNoOfflineReplicas(cm, name());
  JHashSet parts([&cm](int x, int y) {
    const int c = cm.topicNames[cm.partitions[x].topic].compare(cm.topicNames[cm.partitions[y].topic]);
    return c != 0 ? c : icompare(cm.partitions[x].number, cm.partitions[y].number);
  });
  for (size_t p = 0; p < cm.partitions.size(); ++p) parts.add((int)p, cm.tpHash((int)p));
  JHashSet leaders([&cm](int x, int y) { return cm.replicaCompareTo(x, y); });
  for (int p : parts.order()) leaders.add(cm.partitions[p].leader, cm.replicaHash(cm.partitions[p].leader));
  for (int l : leaders.order()) {
    const int p = cm.replicas[l].partition;
    if (o.excludedTopics.count(cm.partitions[p].topic)) continue;
    const std::map<int, int> n = numReplicasByRack(cm, p);
    int mx = 0, mn = 1 << 30;
    for (const auto& kv : n) {
      mx = std::max(mx, kv.second);
      mn = std::min(mn, kv.second);
    }
    if (mx > 1 && ((int)n.size() < numRacks_ || mx - mn > 1))
      throw OptimizationFailure("[" + name() + "] Partition " + std::to_string(p) + " is not rack-aware.",
                                underBrokers(1));  // .excludedRackIds(...) not carried
  }
  ensureReplicasMoveOffBrokersWithBadDisks(cm, name());
  if (provision_.status != PROV_OVER) provision_ = ProvisionResp{PROV_RIGHT_SIZED};
  finished_ = true;
}

// ===================================================================== MinTopicLeadersPerBrokerGoal
// MinTopicLeadersPerBrokerGoal.java. With the default topics.with.min.leaders.per.broker ("", matches no topic) the
// map of topics is empty: the goal accepts every action (actionAffectsRelevantTopics is false, :265-271) and only
// moves offline replicas away (moveAwayOfflineReplicas, :444-464).

// the topic HashSet<String> a stream over clusterModel.topics() collects into (Utils.getTopicNamesMatchedWithPattern,
// Collectors.toSet()), iterated as _mustHaveTopicMinLeadersPerBroker.keySet() (a HashMap filled in that order)
std::vector<int> topicHashSetOrder(const ClusterModel& cm, const std::vector<int>& insertion) {
  JHashSet s([&cm](int a, int b) { return icompare(cm.topicRank[a], cm.topicRank[b]); });
  for (int t : insertion) s.add(t, cm.topicHash[t]);
  return s.order();
}

// isEligibleToHaveLeaders (:439-442)
bool MinTopicLeadersPerBrokerGoal::eligibleToHaveLeaders(const ClusterModel& cm, int b, const OptimizationOptions& o) {
  const int id = cm.brokers[b].id;
  return !o.excludedBrokersForLeadership.count(id) && !o.excludedBrokersForReplicaMove.count(id);
}

// doesLeaderRemoveViolateOptimizedGoal (:141-153)
bool MinTopicLeadersPerBrokerGoal::leaderRemoveViolates(ClusterModel& cm, int r) const {
  if (!cm.replicas[r].isLeader) return false;
  const int t = cm.partitions[cm.replicas[r].partition].topic;
  auto it = minLeaders_.find(t);
  if (it == minLeaders_.end()) return false;
  return cm.numLeadersFor(cm.replicas[r].broker, t) <= it->second;
}

// actionAcceptance (:97-131) with actionAffectsRelevantTopics (:265-271)
Acceptance MinTopicLeadersPerBrokerGoal::actionAcceptance(const BalancingAction& a, ClusterModel& cm) {
  const bool relevant = minLeaders_.count(cm.partitions[a.partition].topic) ||
                        (a.type == ActionType::INTER_BROKER_REPLICA_SWAP &&
                         minLeaders_.count(cm.partitions[a.destPartition].topic));
  if (!relevant) return Acceptance::ACCEPT;
  switch (a.type) {
    case ActionType::LEADERSHIP_MOVEMENT:
    case ActionType::INTER_BROKER_REPLICA_MOVEMENT:
      return leaderRemoveViolates(cm, cm.replicaOnBroker(a.partition, a.sourceBroker)) ? Acceptance::REPLICA_REJECT
                                                                                       : Acceptance::ACCEPT;
    case ActionType::INTER_BROKER_REPLICA_SWAP: {  // acceptReplicaSwap (:116-131)
      const int sr = cm.replicaOnBroker(a.partition, a.sourceBroker);
      const int dr = cm.replicaOnBroker(a.destPartition, a.destinationBroker);
      const bool sl = cm.replicas[sr].isLeader, dl = cm.replicas[dr].isLeader;
      if (!sl && !dl) return Acceptance::ACCEPT;
      if (sl && dl && cm.partitions[a.partition].topic == cm.partitions[a.destPartition].topic) return Acceptance::ACCEPT;
      if (leaderRemoveViolates(cm, sr) || leaderRemoveViolates(cm, dr)) return Acceptance::REPLICA_REJECT;
      return Acceptance::ACCEPT;
    }
    default:
      throw std::invalid_argument("Unsupported balancing action");
  }
}

// initGoalState (:163-192) with its sanity checks (:198-241)
void MinTopicLeadersPerBrokerGoal::initGoalState(ClusterModel& cm, const OptimizationOptions& o) {
  minLeaders_.clear();
  mustOrder_.clear();
  if (bc_.minLeaderTopics.empty()) return;
  {
    std::vector<int> all(cm.topicNames.size());
    for (size_t t = 0; t < all.size(); ++t) all[t] = (int)t;
    std::vector<char> match(cm.topicNames.size(), 0);
    for (int t : bc_.minLeaderTopics) match.at(t) = 1;
    std::vector<int> matched;
    for (int t : topicHashSetOrder(cm, all))  // clusterModel.topics(): a HashSet<String>
      if (match[t]) matched.push_back(t);
    mustOrder_ = topicHashSetOrder(cm, matched);
  }
  // clusterModel.numLeadersPerTopic: one leader per partition
  std::map<int, int> numLeaders;
  for (const Partition& p : cm.partitions)
    if (std::find(mustOrder_.begin(), mustOrder_.end(), p.topic) != mustOrder_.end()) numLeaders[p.topic]++;
  int eligible = 0;
  for (int b : cm.aliveBrokers()) eligible += eligibleToHaveLeaders(cm, b, o) ? 1 : 0;
  for (int t : mustOrder_)
    minLeaders_[t] = bc_.minTopicLeadersPerBroker == 0 ? (eligible == 0 ? 0 : numLeaders[t] / eligible)
                                                        : bc_.minTopicLeadersPerBroker;
  // validateTopicsWithMinLeaderIsNotExcluded (:198-215): the excluded ones joined in HashSet<String> order
  if (!o.excludedTopics.empty()) {
    std::vector<int> bad;
    for (int t : mustOrder_)
      if (o.excludedTopics.count(t)) bad.push_back(t);
    if (!bad.empty()) {
      std::string s;
      for (int t : topicHashSetOrder(cm, bad)) s += (s.empty() ? "" : ", ") + cm.topicNames[t];
      throw OptimizationFailure("[" + name() + "] Topics that must have a minimum number of leaders per broker cannot be "
                                "excluded. This error implies a config error. Topics should not be excluded=[" + s +
                                "] (see topics.with.min.leaders.per.broker).");
    }
  }
  // validateEnoughLeaderToDistribute (:217-230) over numLeadersByTopicNames (a HashMap<String, Integer>)
  for (int t : mustOrder_) {
    const int total = eligible * minLeaders_[t];
    if (numLeaders[t] < total) {
      ProvisionRec rec;
      rec.numPartitions = total;
      throw OptimizationFailure("[" + name() + "] Cannot distribute " + std::to_string(numLeaders[t]) + " leaders over " +
                                    std::to_string(eligible) + " broker(s) with minimum required per broker leader count " +
                                    std::to_string(minLeaders_[t]) + " for topic " + cm.topicNames[t] + ".",
                                rec);
    }
  }
  // validateBrokersAllowedReplicaMoveExist (:232-241)
  int allowed = 0;
  allowedForReplicaMove(cm, o, &allowed);
  if (allowed == 0) {
    ProvisionRec rec;
    rec.numBrokers = cm.maxReplicationFactor;
    throw OptimizationFailure("[" + name() + "] All alive brokers are excluded from replica moves.", rec);
  }
  SortSpec spec;
  if (o.onlyMoveImmigrantReplicas) spec.selection.push_back({SelFn::IMMIGRANTS});
  Selection incl{SelFn::INCLUDED_TOPICS};
  incl.topics = std::make_shared<std::unordered_set<int>>(mustOrder_.begin(), mustOrder_.end());
  spec.selection.push_back(incl);
  if (!o.onlyMoveImmigrantReplicas) spec.priority.push_back(PrioFn::IMMIGRANTS);
  for (size_t b = 0; b < cm.brokers.size(); ++b) cm.trackSortedReplicas((int)b, replicaSortName(false, false), spec);
}

// selfSatisfied (:252-263)
bool MinTopicLeadersPerBrokerGoal::selfSatisfied(ClusterModel& cm, const BalancingAction& a) {
  const int r = cm.replicaOnBroker(a.partition, a.sourceBroker);
  if (cm.isCurrentOffline(r)) return a.type == ActionType::INTER_BROKER_REPLICA_MOVEMENT;
  const int t = cm.partitions[a.partition].topic;
  return cm.numLeadersFor(a.sourceBroker, t) > minLeaders_.at(t);
}

// updateGoalState (:279-288); ensureBrokersAllHaveEnoughLeaderOfTopics only logs
void MinTopicLeadersPerBrokerGoal::updateGoalState(ClusterModel& cm, const OptimizationOptions&) {
  ensureNoOfflineReplicas(cm, name());
  ensureReplicasMoveOffBrokersWithBadDisks(cm, name());
  finished_ = true;
}

// rebalanceForBroker (:317-334)
void MinTopicLeadersPerBrokerGoal::rebalanceForBroker(int b, ClusterModel& cm, const GoalList& g,
                                                      const OptimizationOptions& o) {
  moveAwayOfflineReplicas(b, cm, g, o);
  if (minLeaders_.empty()) return;
  if (!(cm.brokers[b].isAlive() && eligibleToHaveLeaders(cm, b, o))) return;
  for (int t : mustOrder_) moveLeaderOfTopicToBroker(t, b, cm, g, o);
}

// maybeMoveLeaderOfTopicToBroker (:336-409) with getBrokersWithExcessiveLeaderToMove (:418-430). The priority
// queue's keys (live leader counts) only change for the broker just polled (a move goes from it to `b`, which is
// never queued: its count is below the minimum), so polling the smallest (count desc, id) is the queue's order.
void MinTopicLeadersPerBrokerGoal::moveLeaderOfTopicToBroker(int t, int b, ClusterModel& cm, const GoalList& g,
                                                             const OptimizationOptions& o) {
  const int mn = minLeaders_.at(t);
  int recv = cm.numLeadersFor(b, t);
  if (recv >= mn) return;
  const std::string sortName = replicaSortName(false, false);
  std::vector<int> followers;
  for (int r : cm.sortedReplicasClone(b, sortName))
    if (!cm.replicas[r].isLeader && cm.partitions[cm.replicas[r].partition].topic == t) followers.push_back(r);
  for (int f : followers) {
    const int leader = cm.partitions[cm.replicas[f].partition].leader;
    if (cm.numLeadersFor(cm.replicas[leader].broker, t) > mn &&
        maybeApplyBalancingAction(cm, leader, {b}, ActionType::LEADERSHIP_MOVEMENT, g, o) >= 0) {
      if (++recv >= mn) return;
    }
  }
  std::vector<int> pq;
  for (int x : cm.aliveBrokers())
    if (cm.numLeadersFor(x, t) > mn) pq.push_back(x);
  while (!pq.empty()) {
    size_t best = 0;
    for (size_t i = 1; i < pq.size(); ++i) {
      const int ci = cm.numLeadersFor(pq[i], t), cb = cm.numLeadersFor(pq[best], t);
      if (ci > cb || (ci == cb && cm.brokers[pq[i]].id < cm.brokers[pq[best]].id)) best = i;
    }
    const int giver = pq[best];
    pq.erase(pq.begin() + (long)best);
    std::vector<int> leaders;
    for (int r : cm.sortedReplicasClone(giver, sortName))
      if (cm.replicas[r].isLeader && cm.partitions[cm.replicas[r].partition].topic == t) leaders.push_back(r);
    bool moved = false;
    int giverCount = (int)leaders.size();
    for (int l : leaders)
      if (maybeApplyBalancingAction(cm, l, {b}, ActionType::INTER_BROKER_REPLICA_MOVEMENT, g, o) >= 0) {
        moved = true;
        break;
      }
    if (moved) {
      if (++recv >= mn) return;
      if (--giverCount > mn) pq.push_back(giver);
    }
  }
}

// moveAwayOfflineReplicas (:444-464)
void MinTopicLeadersPerBrokerGoal::moveAwayOfflineReplicas(int b, ClusterModel& cm, const GoalList& g,
                                                           const OptimizationOptions& o) {
  if (!hasOfflineReplicas(cm, b)) return;
  // TreeSet by (replica count, id) over alive brokers: iterated in its construction order afterwards
  std::vector<int> eligible = sortedBy(cm.aliveBrokers(), [&](int x, int y) {
    int c = icompare((int)cm.brokers[x].replicas.size(), (int)cm.brokers[y].replicas.size());
    return c != 0 ? c : icompare(cm.brokers[x].id, cm.brokers[y].id);
  });
  // new HashSet<>(srcBroker.currentOfflineReplicas())
  std::vector<int> offline = JHashSet::copyOf(cm.brokers[b].offlineSet).order();
  for (int r : offline)
    if (maybeApplyBalancingAction(cm, r, eligible, ActionType::INTER_BROKER_REPLICA_MOVEMENT, g, o) < 0)
      throw OptimizationFailure("[MinTopicLeadersPerBrokerGoal] Cannot remove offline replica from broker " +
                                    std::to_string(cm.brokers[b].id),
                                underBrokers(1));
}

// ===================================================================== PreferredLeaderElectionGoal
// PreferredLeaderElectionGoal.optimize (PreferredLeaderElectionGoal.java:117-190)
bool PreferredLeaderElectionGoal::optimize(ClusterModel& cm, const GoalList&, const OptimizationOptions& o) {
  provision_ = ProvisionResp{};
  if (o.triggeredByGoalViolation)  // sanityCheckOptimizationOptions (:79-83)
    throw std::invalid_argument(name() + " goal does not support use by goal violation detector.");
  // demoted brokers: their replicas go to the end of the partitions' replica lists (Partition.moveReplicaToEnd),
  // their leaders' partitions are the ones to re-elect (clusterModel.aliveBrokers(): a HashSet<Broker>)
  bool hasDemoted = false;
  std::set<int> partitionsToMove;
  for (int b : javaHashSetOrderIntKeys(cm.aliveBrokers())) {
    const Broker& br = cm.brokers[b];
    if (br.state != BrokerState::DEMOTED) {
      for (int d : br.disks) {  // Broker.disks(): logdir order (:114-124)
        if (!cm.disks[d].demoted) continue;
        hasDemoted = true;
        const std::vector<int> reps = cm.disks[d].replicaSet.order();  // Disk.replicas()
        for (int r : reps) cm.moveReplicaToEnd(r);
        for (int r : reps)  // Disk.leaderReplicas()
          if (cm.replicas[r].isLeader) partitionsToMove.insert(cm.replicas[r].partition);
      }
      continue;
    }
    hasDemoted = true;
    for (int r : br.replicaSet.order()) cm.moveReplicaToEnd(r);  // Broker.replicas(): HashSet order
    for (int r : br.leaderSet.order()) partitionsToMove.insert(cm.replicas[r].partition);
  }
  // clusterModel.getPartitionsByTopic(): topics by name, each topic's partitions in the
  // HashMap<TopicPartition, Partition> iteration order of the model's partitions
  JHashSet all([&cm](int x, int y) {
    const int c = cm.topicNames[cm.partitions[x].topic].compare(cm.topicNames[cm.partitions[y].topic]);
    return c != 0 ? c : icompare(cm.partitions[x].number, cm.partitions[y].number);
  });
  for (size_t p = 0; p < cm.partitions.size(); ++p) all.add((int)p, cm.tpHash((int)p));
  std::vector<std::vector<int>> byTopic(cm.numTopics());
  for (int p : all.order()) byTopic[cm.partitions[p].topic].push_back(p);
  std::vector<int> topics(cm.numTopics());
  for (int t = 0; t < cm.numTopics(); ++t) topics[t] = t;
  std::sort(topics.begin(), topics.end(), [&cm](int a, int b) { return cm.topicNames[a] < cm.topicNames[b]; });
  bool relocated = false;
  for (int t : topics)
    for (int p : byTopic[t]) {
      if (hasDemoted && !partitionsToMove.count(p)) continue;
      const std::vector<int> reps = cm.partitions[p].replicas;
      for (size_t i = 0; i < reps.size(); ++i) {
        if (!hasDemoted && i > 0) break;  // only the first (preferred) replica
        const int r = reps[i], cand = cm.replicas[r].broker;
        if (!cm.brokers[cand].isAlive()) continue;
        if (cm.isCurrentOffline(r)) continue;
        if (!cm.replicas[r].isLeader) {
          if (o.excludedBrokersForLeadership.count(cm.brokers[cand].id)) continue;
          cm.relocateLeadership(p, cm.replicas[cm.partitions[p].leader].broker, cand);
          relocated = true;
        }
        break;
      }
    }
  return relocated;
}

// ===================================================================== ReplicaCapacityGoal
// ReplicaCapacityGoal.actionAcceptance (ReplicaCapacityGoal.java:69-82)
Acceptance ReplicaCapacityGoal::actionAcceptance(const BalancingAction& a, ClusterModel& cm) {
  switch (a.type) {
    case ActionType::INTER_BROKER_REPLICA_MOVEMENT:
      return (int64_t)cm.brokers[a.destinationBroker].replicas.size() < bc_.maxReplicasPerBroker
                 ? Acceptance::ACCEPT
                 : Acceptance::REPLICA_REJECT;
    case ActionType::INTER_BROKER_REPLICA_SWAP:
    case ActionType::LEADERSHIP_MOVEMENT:
      return Acceptance::ACCEPT;
    default:
      throw std::invalid_argument("Unsupported balancing action");
  }
}
// ReplicaCapacityGoal.initGoalState (:100-150)
void ReplicaCapacityGoal::initGoalState(ClusterModel& cm, const OptimizationOptions& o) {
  int64_t total = 0;
  for (size_t b = 0; b < cm.brokers.size(); ++b) {
    const Broker& br = cm.brokers[b];
    total += (int64_t)br.replicas.size();
    if (!br.isAlive()) {
      selfHealingMode_ = true;
      continue;
    }
    // replicas of excluded topics stay where they are (:125-138); on a BAD_DISKS broker the offline ones leave
    if (br.hasBadDisks()) selfHealingMode_ = true;
    if (o.excludedTopics.empty()) continue;
    int64_t excluded = 0;
    for (int r : br.replicas)
      if (o.excludedTopics.count(cm.partitions[cm.replicas[r].partition].topic) &&
          !(br.hasBadDisks() && cm.isCurrentOffline(r)))
        excluded++;
    if (excluded > bc_.maxReplicasPerBroker)
      throw OptimizationFailure("[ReplicaCapacityGoal] Replicas of excluded topics in broker: " + std::to_string(excluded) +
                                " exceeds the maximum allowed number of replicas per broker: " +
                                std::to_string(bc_.maxReplicasPerBroker) + ".");
  }
  int allowed = 0;
  allowedForReplicaMove(cm, o, &allowed);
  const int64_t maxInCluster = bc_.maxReplicasPerBroker * allowed;
  if (total > maxInCluster) {
    const int minRequired = (int)std::ceil(total / (double)bc_.maxReplicasPerBroker);  // :145-148
    throw OptimizationFailure("[ReplicaCapacityGoal] Total replicas in cluster: " + std::to_string(total) +
                                  " exceeds the maximum allowed replicas in cluster: " + std::to_string(maxInCluster),
                              underBrokers(minRequired - allowed));
  }
  SortSpec spec;
  if (o.onlyMoveImmigrantReplicas) spec.selection.push_back({SelFn::IMMIGRANTS});
  if (!o.excludedTopics.empty()) spec.selection.push_back({SelFn::EXCLUDED_TOPICS});
  for (size_t b = 0; b < cm.brokers.size(); ++b) cm.trackSortedReplicas((int)b, replicaSortName(false, false), spec);
}
bool ReplicaCapacityGoal::selfSatisfied(ClusterModel& cm, const BalancingAction& a) {
  return (int64_t)cm.brokers[a.destinationBroker].replicas.size() < bc_.maxReplicasPerBroker;
}
// ReplicaCapacityGoal.updateGoalState (:165-181) + ensureReplicaCapacitySatisfied (:183-196)
void ReplicaCapacityGoal::updateGoalState(ClusterModel& cm, const OptimizationOptions&) {
  ensureNoOfflineReplicas(cm, name());
  ensureReplicasMoveOffBrokersWithBadDisks(cm, name());
  if (!selfHealingMode_) {
    for (size_t b = 0; b < cm.brokers.size(); ++b)
      if ((int64_t)cm.brokers[b].replicas.size() > bc_.maxReplicasPerBroker)
        throw OptimizationFailure("[ReplicaCapacityGoal] Replica count in broker " + std::to_string(b) +
                                      " exceeds the maximum allowed number of replicas per broker.",
                                  underBrokers(1));
    finished_ = true;
  } else {
    selfHealingMode_ = false;
  }
}
// ReplicaCapacityGoal.rebalanceForBroker (:221-263) with eligibleBrokers (:265-278, BrokerReplicaCount order)
void ReplicaCapacityGoal::rebalanceForBroker(int b, ClusterModel& cm, const GoalList& g,
                                             const OptimizationOptions& o) {
  for (int r : cm.sortedReplicasClone(b, replicaSortName(false, false))) {
    const bool offline = cm.isCurrentOffline(r);
    if ((int64_t)cm.brokers[b].replicas.size() <= bc_.maxReplicasPerBroker && !offline) break;
    std::vector<int> eligible;
    for (int x : cm.aliveBrokers())
      if ((selfHealingMode_ || (int64_t)cm.brokers[x].replicas.size() < bc_.maxReplicasPerBroker) &&
          cm.brokers[x].id != cm.brokers[b].id)
        eligible.push_back(x);
    eligible = sortedBy(eligible, [&](int x, int y) {
      int c = icompare((int)cm.brokers[x].replicas.size(), (int)cm.brokers[y].replicas.size());
      return c != 0 ? c : icompare(cm.brokers[x].id, cm.brokers[y].id);
    });
    if (maybeApplyBalancingAction(cm, r, eligible, ActionType::INTER_BROKER_REPLICA_MOVEMENT, g, o) < 0) {
      if (!cm.brokers[b].isAlive())
        throw OptimizationFailure("[ReplicaCapacityGoal] Failed to move dead broker replica.", underBrokers(1));
      if (offline) throw OptimizationFailure("[ReplicaCapacityGoal] Failed to move offline replica.", underBrokers(1));
    }
  }
}

// ===================================================================== CapacityGoal
std::string CapacityGoal::name() const {
  switch (resource_) {
    case CPU: return "CpuCapacityGoal";
    case NW_IN: return "NetworkInboundCapacityGoal";
    case NW_OUT: return "NetworkOutboundCapacityGoal";
    default: return "DiskCapacityGoal";
  }
}
// CapacityGoal.isUtilizationUnderLimitAfterAddingLoad (CapacityGoal.java:455-475)
bool CapacityGoal::underLimitAfterAdding(ClusterModel& cm, int b, double u) const {
  const double thr = bc_.capacityThreshold[resource_];
  if (isHostResource(resource_)) {
    if (cm.hostUtil(b, resource_) + u >= cm.hostCapacity(b, resource_) * thr) return false;
  }
  if (isBrokerResource(resource_)) return cm.brokerUtil(b, resource_) + u < cm.brokers[b].capacity[resource_] * thr;
  return true;
}
// CapacityGoal.isMovementAcceptableForCapacity (:431-436) / isSwapAcceptableForCapacity (:438-447)
bool CapacityGoal::movementAcceptable(ClusterModel& cm, int sr, int dst) const {
  return underLimitAfterAdding(cm, dst, cm.replicaUtil(sr, resource_));
}
bool CapacityGoal::swapAcceptable(ClusterModel& cm, int sr, int dr) const {
  const double su = cm.replicaUtil(sr, resource_), du = cm.replicaUtil(dr, resource_);
  const double delta = du - su;
  return delta > 0 ? underLimitAfterAdding(cm, cm.replicas[sr].broker, delta)
                   : underLimitAfterAdding(cm, cm.replicas[dr].broker, -delta);
}
// CapacityGoal.actionAcceptance (:75-90); DiskCapacityGoal / NetworkInboundCapacityGoal accept every leadership
// movement (DiskCapacityGoal.java:40-43, NetworkInboundCapacityGoal.java:40-43)
Acceptance CapacityGoal::actionAcceptance(const BalancingAction& a, ClusterModel& cm) {
  if (a.type == ActionType::LEADERSHIP_MOVEMENT && (resource_ == DISK || resource_ == NW_IN)) return Acceptance::ACCEPT;
  const int sr = cm.replicaOnBroker(a.partition, a.sourceBroker);
  switch (a.type) {
    case ActionType::INTER_BROKER_REPLICA_SWAP:
      return swapAcceptable(cm, sr, cm.replicaOnBroker(a.destPartition, a.destinationBroker))
                 ? Acceptance::ACCEPT
                 : Acceptance::REPLICA_REJECT;
    case ActionType::INTER_BROKER_REPLICA_MOVEMENT:
    case ActionType::LEADERSHIP_MOVEMENT:
      return movementAcceptable(cm, sr, a.destinationBroker) ? Acceptance::ACCEPT : Acceptance::REPLICA_REJECT;
    default:
      throw std::invalid_argument("Unsupported balancing action");
  }
}
bool CapacityGoal::selfSatisfied(ClusterModel& cm, const BalancingAction& a) {
  return movementAcceptable(cm, cm.replicaOnBroker(a.partition, a.sourceBroker), a.destinationBroker);
}
// CapacityGoal.initGoalState (:120-170)
void CapacityGoal::initGoalState(ClusterModel& cm, const OptimizationOptions& o) {
  const double existing = expectedUtil(cm.load, resource_, cm.W);
  const double capacity = cm.capacityWithAllowedReplicaMovesFor(resource_, o);
  const double allowedCapacity = capacity * bc_.capacityThreshold[resource_];
  if (allowedCapacity < existing) {
    int allowed = 0;
    const std::vector<char> allowedB = allowedForReplicaMove(cm, o, &allowed);
    if (allowed == 0)
      throw OptimizationFailure("[" + name() + "] All alive brokers are excluded from replica moves.",
                                underBrokers(cm.maxReplicationFactor));
    // a typical broker: the first of aliveBrokersNotExcludedForReplicaMove (a HashSet<Integer>) (:160-166)
    std::vector<int> ids;
    for (int b : cm.aliveBrokers())
      if (allowedB[b]) ids.push_back(b);
    const int typical = javaHashSetOrderIntKeys(ids).front();
    const double typicalCapacity = cm.brokers[typical].capacity[resource_];
    const double missing = existing - allowedCapacity;
    ProvisionRec rec = underBrokers((int)std::ceil(missing / (typicalCapacity * bc_.capacityThreshold[resource_])),
                                    resource_);
    rec.typicalBrokerCapacity = typicalCapacity;
    rec.typicalBrokerId = cm.brokers[typical].id;
    throw OptimizationFailure("[" + name() + "] Insufficient capacity for " + resourceName(resource_) + ".", rec);
  }
  const bool selfHealing = !cm.selfHealingEligibleReplicas.empty();
  SortSpec all;
  if (o.onlyMoveImmigrantReplicas) all.selection.push_back({SelFn::IMMIGRANTS});
  if (!o.excludedTopics.empty()) all.selection.push_back({SelFn::EXCLUDED_TOPICS});
  if (selfHealing) all.priority.push_back(PrioFn::OFFLINE);
  if (!o.onlyMoveImmigrantReplicas) all.priority.push_back(PrioFn::IMMIGRANTS);
  all.score = ScoreFn::REVERSE_BY_GROUP;
  all.scoreResource = resource_;
  SortSpec leaders;
  leaders.selection.push_back({SelFn::LEADERS});
  if (o.onlyMoveImmigrantReplicas) leaders.selection.push_back({SelFn::IMMIGRANTS});
  if (!o.excludedTopics.empty()) leaders.selection.push_back({SelFn::EXCLUDED_TOPICS});
  if (!o.onlyMoveImmigrantReplicas) leaders.priority.push_back(PrioFn::IMMIGRANTS);
  leaders.score = ScoreFn::REVERSE_BY_GROUP;
  leaders.scoreResource = resource_;
  for (size_t b = 0; b < cm.brokers.size(); ++b) {
    cm.trackSortedReplicas((int)b, replicaSortName(true, false), all);
    cm.trackSortedReplicas((int)b, replicaSortName(true, true), leaders);
  }
}
// CapacityGoal.updateGoalState (:180-190) + ensureUtilizationUnderCapacity (:192-225)
void CapacityGoal::updateGoalState(ClusterModel& cm, const OptimizationOptions&) {
  const double thr = bc_.capacityThreshold[resource_];
  for (size_t b = 0; b < cm.brokers.size(); ++b) {
    const bool hasReplicas = !cm.brokers[b].replicas.empty();
    if (isHostResource(resource_) && !cm.hostReplicasEmpty((int)b) &&
        cm.hostUtil((int)b, resource_) > cm.hostCapacity((int)b, resource_) * thr)
      throw OptimizationFailure("[" + name() + "] utilization for host is above capacity limit.", underBrokers(1, resource_));
    if (isBrokerResource(resource_) && hasReplicas &&
        cm.brokerUtil((int)b, resource_) > cm.brokers[b].capacity[resource_] * thr)
      throw OptimizationFailure("[" + name() + "] utilization for broker is above capacity limit.",
                                underBrokers(1, resource_));
  }
  ensureNoOfflineReplicas(cm, name());
  ensureReplicasMoveOffBrokersWithBadDisks(cm, name());
  finished_ = true;
}
// CapacityGoal.isUtilizationOverLimit (:410-428)
bool CapacityGoal::utilizationOverLimit(ClusterModel& cm, int b, double brokerLimit, double hostLimit) const {
  const bool hasReplicas = !cm.brokers[b].replicas.empty();
  if (!cm.hostReplicasEmpty(b) && isHostResource(resource_) && cm.hostUtil(b, resource_) > hostLimit) return true;
  if (hasReplicas && isBrokerResource(resource_)) return cm.brokerUtil(b, resource_) > brokerLimit;
  return false;
}
// CapacityGoal.rebalanceForBroker (:235-330) + postSanityCheck (:332-355)
void CapacityGoal::rebalanceForBroker(int b, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o) {
  const double thr = bc_.capacityThreshold[resource_];
  const double brokerLimit = cm.brokers[b].capacity[resource_] * thr;
  const double hostLimit = cm.hostCapacity(b, resource_) * thr;
  bool over = utilizationOverLimit(cm, b, brokerLimit, hostLimit);
  if (!over && !hasOfflineReplicas(cm, b)) return;
  if (resource_ == NW_OUT || resource_ == CPU) {
    for (int leader : cm.sortedReplicasClone(b, replicaSortName(true, true))) {
      // Partition.onlineFollowers() sorted by GoalUtils.sortReplicasInAscendingOrderByBrokerResourceUtilization
      std::vector<int> followers;
      for (int x : cm.partitions[cm.replicas[leader].partition].replicas)
        if (!cm.replicas[x].isLeader && !cm.isCurrentOffline(x)) followers.push_back(x);
      followers = sortedBy(followers, [&](int x, int y) {
        int c = dcompare(cm.brokerUtil(cm.replicas[x].broker, resource_), cm.brokerUtil(cm.replicas[y].broker, resource_));
        return c != 0 ? c : icompare(cm.brokers[cm.replicas[x].broker].id, cm.brokers[cm.replicas[y].broker].id);
      });
      std::vector<int> eligible;
      for (int x : followers) eligible.push_back(cm.replicas[x].broker);
      maybeApplyBalancingAction(cm, leader, eligible, ActionType::LEADERSHIP_MOVEMENT, g, o);
      over = utilizationOverLimit(cm, b, brokerLimit, hostLimit);
      if (!over) break;
    }
  }
  if (over || hasOfflineReplicas(cm, b)) {
    // ClusterModel.sortedAliveBrokersUnderThreshold (ClusterModel.java:1049-1066): a snapshot list
    std::vector<int> under = sortedBy(cm.aliveBrokersUnderThreshold(resource_, thr), [&](int x, int y) {
      int hc = 0;
      if (isHostResource(resource_)) hc = dcompare(cm.hostUtil(x, resource_), cm.hostUtil(y, resource_));
      return hc == 0 ? dcompare(cm.brokerUtil(x, resource_), cm.brokerUtil(y, resource_)) : hc;
    });
    for (int r : cm.sortedReplicasClone(b, replicaSortName(true, false))) {
      maybeApplyBalancingAction(cm, r, under, ActionType::INTER_BROKER_REPLICA_MOVEMENT, g, o);
      over = utilizationOverLimit(cm, b, brokerLimit, hostLimit);
      if (!over && !hasOfflineReplicas(cm, b)) break;
    }
  }
  if (over)
    throw OptimizationFailure("[" + name() + "] Utilization of broker " + std::to_string(b) +
                                  " violated capacity limit for resource " + resourceName(resource_) + ".",
                              underBrokers(1, resource_));
  if (hasOfflineReplicas(cm, b))
    throw OptimizationFailure("[" + name() + "] Cannot remove offline replicas from broker " + std::to_string(b) + ".",
                              underBrokers(1, resource_));
}

// ===================================================================== PotentialNwOutGoal
// PotentialNwOutGoal.actionAcceptance (PotentialNwOutGoal.java:73-84) + isReplicaRelocationAcceptable (:86-113)
Acceptance PotentialNwOutGoal::actionAcceptance(const BalancingAction& a, ClusterModel& cm) {
  switch (a.type) {
    case ActionType::LEADERSHIP_MOVEMENT:
      return Acceptance::ACCEPT;
    case ActionType::INTER_BROKER_REPLICA_SWAP:
    case ActionType::INTER_BROKER_REPLICA_MOVEMENT: {
      if (selfSatisfied(cm, a)) return Acceptance::ACCEPT;
      const int sr = cm.replicaOnBroker(a.partition, a.sourceBroker);
      const double destU = cm.potentialNwOut(a.destinationBroker);
      const double srcU = cm.potentialNwOut(cm.replicas[sr].broker);
      const double srU = leaderNwOutOf(cm, cm.replicas[sr].partition);
      const double maxU = jmax(destU, srcU);
      if (a.type == ActionType::INTER_BROKER_REPLICA_SWAP) {
        const double drU = leaderNwOutOf(cm, a.destPartition);
        if (srcU + drU - srU > maxU) return Acceptance::REPLICA_REJECT;
        return destU + srU - drU <= maxU ? Acceptance::ACCEPT : Acceptance::REPLICA_REJECT;
      }
      return destU + srU <= maxU ? Acceptance::ACCEPT : Acceptance::REPLICA_REJECT;
    }
    default:
      throw std::invalid_argument("Unsupported balancing action");
  }
}
// PotentialNwOutGoal.brokersToBalance (:140-150)
std::vector<int> PotentialNwOutGoal::brokersToBalance(ClusterModel& cm) {
  std::set<int> broken(cm.deadBrokers.begin(), cm.deadBrokers.end());
  for (int b : cm.brokersWithBadDisks) broken.insert(b);
  if (broken.empty()) return AbstractGoal::brokersToBalance(cm);
  return std::vector<int>(broken.begin(), broken.end());
}
// PotentialNwOutGoal.selfSatisfied (:152-183)
bool PotentialNwOutGoal::selfSatisfied(ClusterModel& cm, const BalancingAction& a) {
  const int sr = cm.replicaOnBroker(a.partition, a.sourceBroker);
  if (fixOfflineReplicasOnly_ && cm.isCurrentOffline(sr)) return a.type == ActionType::INTER_BROKER_REPLICA_MOVEMENT;
  const int db = a.destinationBroker, sb = cm.replicas[sr].broker;
  const double destU = cm.potentialNwOut(db);
  const double destCap = cm.brokers[db].capacity[NW_OUT] * bc_.capacityThreshold[NW_OUT];
  const double srU = leaderNwOutOf(cm, cm.replicas[sr].partition);
  if (a.type != ActionType::INTER_BROKER_REPLICA_SWAP) return destCap >= destU + srU;
  const double drU = leaderNwOutOf(cm, a.destPartition);
  if (destCap < destU + srU - drU) return false;
  const double srcU = cm.potentialNwOut(sb);
  const double srcCap = cm.brokers[sb].capacity[NW_OUT] * bc_.capacityThreshold[NW_OUT];
  return srcCap >= srcU + drU - srU;
}
// PotentialNwOutGoal.initGoalState (:185-195)
void PotentialNwOutGoal::initGoalState(ClusterModel& cm, const OptimizationOptions& o) {
  fixOfflineReplicasOnly_ = false;
  SortSpec spec;
  if (o.onlyMoveImmigrantReplicas) spec.selection.push_back({SelFn::IMMIGRANTS});
  if (!o.excludedTopics.empty()) spec.selection.push_back({SelFn::EXCLUDED_TOPICS});
  for (size_t b = 0; b < cm.brokers.size(); ++b) cm.trackSortedReplicas((int)b, replicaSortName(false, false), spec);
}
// PotentialNwOutGoal.updateGoalState (:197-213)
void PotentialNwOutGoal::updateGoalState(ClusterModel& cm, const OptimizationOptions&) {
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
// PotentialNwOutGoal.rebalanceForBroker (:225-290) with brokersUnderEstimatedMaxPossibleNwOut (:292-304)
void PotentialNwOutGoal::rebalanceForBroker(int b, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o) {
  const double thr = bc_.capacityThreshold[NW_OUT];
  const double limit = cm.brokers[b].capacity[NW_OUT] * thr;
  bool over = !cm.brokers[b].replicas.empty() && cm.potentialNwOut(b) > limit;
  if (!over && !(fixOfflineReplicasOnly_ && hasOfflineReplicas(cm, b))) return;
  // candidate set: HashSet<Broker> (iteration order by id hash buckets)
  std::vector<int> candidates;
  if (fixOfflineReplicasOnly_) {
    candidates = cm.aliveBrokers();
  } else {
    std::vector<int> under;
    for (int x : cm.aliveBrokers())
      if (cm.potentialNwOut(x) < cm.brokers[x].capacity[NW_OUT] * thr) under.push_back(x);
    candidates = javaHashSetOrderIntKeys(under);
  }
  for (int r : cm.sortedReplicasClone(b, replicaSortName(false, false))) {
    // new ArrayList<>(candidateBrokers), removeAll(partition brokers), stable sort descending by leadership NW_OUT
    std::vector<int> eligible;
    for (int x : candidates) {
      bool inPartition = false;
      for (int y : cm.partitions[cm.replicas[r].partition].replicas) inPartition |= (cm.replicas[y].broker == x);
      if (!inPartition) eligible.push_back(x);
    }
    eligible = sortedBy(eligible, [&](int x, int y) {
      return dcompare(expectedUtil(cm.brokers[y].leadershipLoadForNwResources, NW_OUT, cm.W),
                      expectedUtil(cm.brokers[x].leadershipLoadForNwResources, NW_OUT, cm.W));
    });
    const int dst = maybeApplyBalancingAction(cm, r, eligible, ActionType::INTER_BROKER_REPLICA_MOVEMENT, g, o);
    if (dst >= 0) {
      over = !cm.brokers[b].replicas.empty() && cm.potentialNwOut(b) > limit;
      if (!over && !(fixOfflineReplicasOnly_ && hasOfflineReplicas(cm, b))) break;
      if (!fixOfflineReplicasOnly_) {
        if (cm.potentialNwOut(dst) > cm.brokers[dst].capacity[NW_OUT] * thr)
          candidates.erase(std::find(candidates.begin(), candidates.end(), dst));
      }
    }
  }
  if (over) succeeded_ = false;
}

// ===================================================================== TopicReplicaDistributionGoal
bool TopicReplicaDistributionGoal::underUpperAfter(const ClusterModel& cm, int topic, int b, bool add) const {
  const int n = count(cm, b, topic);
  const int lim = cm.brokers[b].isAlive() ? upper_[topic] : 0;
  return add ? n + 1 <= lim : n - 1 <= lim;
}
bool TopicReplicaDistributionGoal::aboveLowerAfter(const ClusterModel& cm, int topic, int b, bool add) const {
  const int n = count(cm, b, topic);
  const int lim = cm.brokers[b].isAlive() ? lower_[topic] : 0;
  return add ? n + 1 >= lim : n - 1 >= lim;
}
// TopicReplicaDistributionGoal.actionAcceptance (TopicReplicaDistributionGoal.java:153-182)
Acceptance TopicReplicaDistributionGoal::actionAcceptance(const BalancingAction& a, ClusterModel& cm) {
  const int sb = a.sourceBroker, db = a.destinationBroker;
  const int st = cm.partitions[a.partition].topic;
  switch (a.type) {
    case ActionType::INTER_BROKER_REPLICA_SWAP: {
      const int dt = cm.partitions[a.destPartition].topic;
      if (st == dt) return Acceptance::ACCEPT;
      const bool s2d = underUpperAfter(cm, st, db, true) && aboveLowerAfter(cm, st, sb, false);
      return (s2d && underUpperAfter(cm, dt, sb, true) && aboveLowerAfter(cm, dt, db, false))
                 ? Acceptance::ACCEPT
                 : Acceptance::REPLICA_REJECT;
    }
    case ActionType::LEADERSHIP_MOVEMENT:
      return Acceptance::ACCEPT;
    case ActionType::INTER_BROKER_REPLICA_MOVEMENT:
      return (underUpperAfter(cm, st, db, true) && (isExcluded(sb) || aboveLowerAfter(cm, st, sb, false)))
                 ? Acceptance::ACCEPT
                 : Acceptance::REPLICA_REJECT;
    default:
      throw std::invalid_argument("Unsupported balancing action");
  }
}
int TopicReplicaDistributionGoal::compareStats(const ClusterModelStats& s1, const ClusterModelStats& s2) const {
  const double d1 = s1.topicStd, d2 = s2.topicStd;
  const double eps = 1e-5;
  if (d1 - d2 > eps) return -1;  // AnalyzerUtils.compare(stdDev2, stdDev1, EPSILON)
  if (d2 - d1 > eps) return 1;
  return 0;
}
// TopicReplicaDistributionGoal.initGoalState (:225-270) with balance limits (:103-145)
void TopicReplicaDistributionGoal::initGoalState(ClusterModel& cm, const OptimizationOptions& o) {
  int numAllowed = 0;
  allowed_ = allowedForReplicaMove(cm, o, &numAllowed);
  if (numAllowed == 0)
    throw OptimizationFailure("[" + name() + "] All alive brokers are excluded from replica moves.",
                              underBrokers(cm.maxReplicationFactor));
  // GoalUtils.topicsToRebalance (GoalUtils.java:439-452): the self-healing replicas' topics, or all topics but the
  // excluded ones
  rebalanceTopic_.assign(cm.numTopics(), cm.selfHealingEligibleReplicas.empty() ? 1 : 0);
  for (int r : cm.selfHealingEligibleReplicas) rebalanceTopic_[cm.partitions[cm.replicas[r].partition].topic] = 1;
  if (cm.selfHealingEligibleReplicas.empty())
    for (int t : o.excludedTopics) rebalanceTopic_[t] = 0;
  const double margin = (bc_.topicReplicaBalancePercentage - 1) * 0.9;
  upper_.assign(cm.numTopics(), 0);
  lower_.assign(cm.numTopics(), 0);
  for (int t = 0; t < cm.numTopics(); ++t) {
    const double avg = cm.numReplicasByTopic[t] / (double)numAllowed;
    const int cu = (int)std::ceil(avg * (1 + margin));
    const int umin = (int)(std::ceil(avg) + bc_.topicReplicaBalanceMinGap);
    const int umax = (int)(std::ceil(avg) + bc_.topicReplicaBalanceMaxGap);
    upper_[t] = std::max(umin, std::min(cu, umax));
    const int cl = (int)std::floor(avg * jmax(0, (1 - margin)));
    const int lmax = std::max(0, (int)(std::floor(avg) - bc_.topicReplicaBalanceMinGap));
    const int lmin = std::max(0, (int)(std::floor(avg) - bc_.topicReplicaBalanceMaxGap));
    lower_[t] = std::max(lmin, std::min(cl, lmax));
  }
  const bool selfHealing = !cm.selfHealingEligibleReplicas.empty();
  for (size_t b = 0; b < cm.brokers.size(); ++b) {
    SortSpec spec;
    if (o.onlyMoveImmigrantReplicas) spec.selection.push_back({SelFn::IMMIGRANTS});
    if (selfHealing && cm.brokers[b].isAlive()) spec.selection.push_back({SelFn::IMMIGRANT_OR_OFFLINE});
    if (!o.excludedTopics.empty()) spec.selection.push_back({SelFn::EXCLUDED_TOPICS});
    cm.trackSortedReplicas((int)b, replicaSortName(false, false), spec);
  }
  fixOfflineReplicasOnly_ = false;
}
bool TopicReplicaDistributionGoal::selfSatisfied(ClusterModel& cm, const BalancingAction& a) {
  const int sr = cm.replicaOnBroker(a.partition, a.sourceBroker);
  if (fixOfflineReplicasOnly_ && cm.isCurrentOffline(sr)) return a.type == ActionType::INTER_BROKER_REPLICA_MOVEMENT;
  const int st = cm.partitions[a.partition].topic;
  return underUpperAfter(cm, st, a.destinationBroker, true) &&
         (isExcluded(a.sourceBroker) || aboveLowerAfter(cm, st, a.sourceBroker, false));
}
// TopicReplicaDistributionGoal.updateGoalState (:318-345)
void TopicReplicaDistributionGoal::updateGoalState(ClusterModel& cm, const OptimizationOptions&) {
  if (anyAbove_) {
    anyAbove_ = false;
    succeeded_ = false;
  }
  if (anyUnder_) {
    anyUnder_ = false;
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
}
// TopicReplicaDistributionGoal.rebalanceForBroker (:395-443) + skipBrokerRebalance (:348-377)
void TopicReplicaDistributionGoal::rebalanceForBroker(int b, ClusterModel& cm, const GoalList& g,
                                                      const OptimizationOptions& o) {
  const Broker& br = cm.brokers[b];
  for (int topic : br.topicKeys.order()) {  // Broker.topics(): HashMap key order
    if (!rebalanceTopic_[topic]) continue;
    int n = 0, nOff = 0;
    bool hasImm = false;
    for (int r : br.replicas)
      if (cm.partitions[cm.replicas[r].partition].topic == topic) {
        n++;
        if (br.offlineSet.contains(r, cm.replicaHash(r))) nOff++;
        if (cm.isImmigrant(r)) hasImm = true;
      }
    const bool excluded = isExcluded(b);
    const bool requireLess = nOff > 0 || n > upper_[topic] || excluded;
    const bool requireMore = !excluded && br.isAlive() && n - nOff < lower_[topic];
    if (br.isAlive() && !requireMore && !requireLess) continue;
    if (!cm.newBrokers.empty() && !br.isNew() && !requireLess) continue;
    if (!cm.selfHealingEligibleReplicas.empty() && requireLess && nOff == 0 && !hasImm) continue;
    if (o.onlyMoveImmigrantReplicas && requireLess && !hasImm) continue;
    if (requireLess && moveOut(b, topic, cm, g, o)) anyAbove_ = true;
    if (requireMore && moveIn(b, topic, cm, g, o)) anyUnder_ = true;
  }
}
// TopicReplicaDistributionGoal.replicasToMoveOut (:445-451): TreeSet(broker.replicaComparator()) of the topic's
// replicas retained to the tracked sorted set's members
std::vector<int> TopicReplicaDistributionGoal::replicasToMoveOut(ClusterModel& cm, int b, int topic) {
  const Broker& br = cm.brokers[b];
  const auto& tracked = cm.sortedReplicasView(b, replicaSortName(false, false));
  std::vector<int> out;
  for (int r : br.replicas)
    if (cm.partitions[cm.replicas[r].partition].topic == topic && tracked.count(r)) out.push_back(r);
  std::sort(out.begin(), out.end(), [&](int x, int y) {
    const bool ox = br.offlineSet.contains(x, cm.replicaHash(x)), oy = br.offlineSet.contains(y, cm.replicaHash(y));
    if (ox != oy) return ox;
    const bool ix = cm.isImmigrant(x), iy = cm.isImmigrant(y);
    if (ix != iy) return ix;
    return cm.partitions[cm.replicas[x].partition].number < cm.partitions[cm.replicas[y].partition].number;
  });
  return out;
}
// TopicReplicaDistributionGoal.rebalanceByMovingReplicasOut (:453-505)
bool TopicReplicaDistributionGoal::moveOut(int b, int topic, ClusterModel& cm, const GoalList& g,
                                           const OptimizationOptions& o) {
  JTreeSet candidates([&cm, this, topic](int x, int y) {
    int c = icompare(count(cm, x, topic), count(cm, y, topic));
    return c != 0 ? c : icompare(cm.brokers[x].id, cm.brokers[y].id);
  });
  std::vector<int> toAdd;
  if (fixOfflineReplicasOnly_) {
    toAdd = cm.aliveBrokers();
  } else {
    std::vector<int> filtered;
    for (int x : cm.aliveBrokers())
      if (count(cm, x, topic) < upper_[topic]) filtered.push_back(x);
    toAdd = javaHashSetOrderIntKeys(filtered);  // Collectors.toSet()
  }
  for (int x : toAdd) candidates.add(x);
  int n = 0, nOff = 0;
  for (int r : cm.brokers[b].replicas)
    if (cm.partitions[cm.replicas[r].partition].topic == topic) {
      n++;
      if (cm.brokers[b].offlineSet.contains(r, cm.replicaHash(r))) nOff++;
    }
  const int upperForSource = isExcluded(b) ? 0 : upper_[topic];
  bool wasUnableToMoveOffline = false;
  for (int r : replicasToMoveOut(cm, b, topic)) {
    if (wasUnableToMoveOffline && !cm.isCurrentOffline(r) && n <= upperForSource) return false;
    const bool wasOffline = cm.isCurrentOffline(r);
    const int dst = maybeApplyBalancingAction(cm, r, candidates.toVector(), ActionType::INTER_BROKER_REPLICA_MOVEMENT,
                                              g, o);
    if (dst >= 0) {
      if (wasOffline) nOff--;
      if (--n <= (nOff == 0 ? upperForSource : 0)) return false;
      candidates.remove(dst);
      if (count(cm, dst, topic) < upper_[topic] || fixOfflineReplicasOnly_) candidates.add(dst);
    } else if (wasOffline) {
      wasUnableToMoveOffline = true;
    }
  }
  return count(cm, b, topic) != 0;
}
// TopicReplicaDistributionGoal.rebalanceByMovingReplicasIn (:507-570)
bool TopicReplicaDistributionGoal::moveIn(int dest, int topic, ClusterModel& cm, const GoalList& g,
                                          const OptimizationOptions& o) {
  auto offlineCount = [&](int x) {
    int k = 0;
    for (int r : cm.brokers[x].replicas)
      if (cm.partitions[cm.replicas[r].partition].topic == topic && cm.brokers[x].offlineSet.contains(r, cm.replicaHash(r)))
        k++;
    return k;
  };
  JPriorityQueue pq([&](int b1, int b2) {
    const int r = icompare(offlineCount(b2), offlineCount(b1));
    if (r == 0) {
      const int r2 = icompare(count(cm, b2, topic), count(cm, b1, topic));
      return r2 == 0 ? icompare(cm.brokers[b1].id, cm.brokers[b2].id) : r2;
    }
    return r;
  });
  if (fixOfflineReplicasOnly_) {
    for (size_t s = 0; s < cm.brokers.size(); ++s)
      if ((int)s != dest) pq.add((int)s);
  } else {
    for (size_t s = 0; s < cm.brokers.size(); ++s)
      if (count(cm, (int)s, topic) > lower_[topic] || hasOfflineReplicas(cm, (int)s) || isExcluded((int)s))
        pq.add((int)s);
  }
  int n = count(cm, dest, topic);
  const std::vector<int> candidates{dest};
  while (!pq.empty()) {
    const int src = pq.poll();
    std::vector<int> toMove = replicasToMoveOut(cm, src, topic);
    int nOff = 0;
    for (int r : toMove)
      if (cm.brokers[src].offlineSet.contains(r, cm.replicaHash(r))) nOff++;
    for (int r : toMove) {
      const bool wasOffline = cm.isCurrentOffline(r);
      if (maybeApplyBalancingAction(cm, r, candidates, ActionType::INTER_BROKER_REPLICA_MOVEMENT, g, o) >= 0) {
        if (wasOffline) nOff--;
        if (++n >= lower_[topic]) return false;
        if (!pq.empty() && nOff == 0 && count(cm, src, topic) < count(cm, pq.peek(), topic)) {
          pq.add(src);
          break;
        }
      }
    }
  }
  return true;
}

// ===================================================================== TopicLeaderReplicaDistributionGoal
// (TopicLeaderReplicaDistributionGoal.java). Java int arithmetic wraps; the limits of a cluster whose alive brokers
// are all excluded from replica moves come from an infinite or NaN average (x / 0.0).
namespace {
int32_t jAddInt(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
int32_t jSubInt(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }
}  // namespace

// isLeadershipGoalSatisfiable + isTopicLeaderCount{Under,Above}…AfterChange (:231-256)
bool TopicLeaderReplicaDistributionGoal::satisfiable(const ClusterModel& cm, int topic, int src, int dst) const {
  const int up = cm.brokers[dst].isAlive() ? upper_[topic] : 0;
  if (!(cm.numLeadersFor(dst, topic) + 1 <= up)) return false;
  if (isExcluded(src)) return true;
  const int lo = cm.brokers[src].isAlive() ? lower_[topic] : 0;
  return cm.numLeadersFor(src, topic) - 1 >= lo;
}
// actionAcceptance (:181-229)
Acceptance TopicLeaderReplicaDistributionGoal::actionAcceptance(const BalancingAction& a, ClusterModel& cm) {
  const int sb = a.sourceBroker, db = a.destinationBroker;
  const int st = cm.partitions[a.partition].topic;
  const int sr = cm.replicaOnBroker(a.partition, sb);
  const bool sl = cm.replicas[sr].isLeader;
  auto verdict = [](bool ok) { return ok ? Acceptance::ACCEPT : Acceptance::REPLICA_REJECT; };
  switch (a.type) {
    case ActionType::INTER_BROKER_REPLICA_SWAP: {
      const int dt = cm.partitions[a.destPartition].topic;
      const bool dl = cm.replicas[cm.replicaOnBroker(a.destPartition, db)].isLeader;
      if (st == dt && sl && dl) return Acceptance::ACCEPT;
      if (!sl && !dl) return Acceptance::ACCEPT;
      if (sl && !dl) return verdict(satisfiable(cm, st, sb, db));
      if (!sl && dl) return verdict(satisfiable(cm, dt, db, sb));
      return verdict(satisfiable(cm, st, sb, db) && satisfiable(cm, dt, db, sb));
    }
    case ActionType::LEADERSHIP_MOVEMENT:
      return verdict(satisfiable(cm, st, sb, db));
    case ActionType::INTER_BROKER_REPLICA_MOVEMENT:
      if (!sl) return Acceptance::ACCEPT;
      return verdict(satisfiable(cm, st, sb, db));
    default:
      throw std::invalid_argument("Unsupported balancing action");
  }
}
// initGoalState (:298-347) with balancePercentageWithMargin / clampLower / clampUpper / balance{Upper,Lower}Limit
// (:101-168)
void TopicLeaderReplicaDistributionGoal::initGoalState(ClusterModel& cm, const OptimizationOptions& o) {
  int numAllowed = 0;
  allowed_ = allowedForReplicaMove(cm, o, &numAllowed);  // an empty set is allowed: leadership-only balancing
  // GoalUtils.topicsToRebalance (GoalUtils.java:439-452)
  rebalanceTopic_.assign(cm.numTopics(), cm.selfHealingEligibleReplicas.empty() ? 1 : 0);
  for (int r : cm.selfHealingEligibleReplicas) rebalanceTopic_[cm.partitions[cm.replicas[r].partition].topic] = 1;
  if (cm.selfHealingEligibleReplicas.empty())
    for (int t : o.excludedTopics) rebalanceTopic_[t] = 0;
  double pct = bc_.topicLeaderReplicaBalancePercentage;
  if (o.triggeredByGoalViolation) pct *= bc_.goalViolationDistributionThresholdMultiplier;
  const double margin = (pct - 1) * bc_.topicLeaderReplicaDistributionGoalBalanceMargin;
  // ClusterModel.numLeadersPerTopic (ClusterModel.java:276-285): one leader per partition
  std::vector<int> numLeaders(cm.numTopics(), 0);
  for (const Partition& p : cm.partitions) numLeaders[p.topic]++;
  const int minGap = bc_.topicLeaderReplicaBalanceMinGap, maxGap = bc_.topicLeaderReplicaBalanceMaxGap;
  upper_.assign(cm.numTopics(), 0);
  lower_.assign(cm.numTopics(), 0);
  for (int t = 0; t < cm.numTopics(); ++t) {
    const double avg = numLeaders[t] / (double)numAllowed;
    const int32_t ceilAvg = jDoubleToInt(std::ceil(avg)), floorAvg = jDoubleToInt(std::floor(avg));
    const int32_t cu = jDoubleToInt(std::ceil(avg * (1 + margin)));
    upper_[t] = std::max(jAddInt(ceilAvg, minGap), std::min(cu, jAddInt(ceilAvg, maxGap)));
    const int32_t cl = jDoubleToInt(std::floor(avg * jmax(0, (1 - margin))));
    const int32_t lmin = std::max(0, jSubInt(floorAvg, maxGap)), lmax = std::max(0, jSubInt(floorAvg, minGap));
    lower_[t] = std::max(lmin, std::min(cl, lmax));
  }
  const bool selfHealing = !cm.selfHealingEligibleReplicas.empty();
  for (size_t b = 0; b < cm.brokers.size(); ++b) {
    SortSpec spec;
    if (o.onlyMoveImmigrantReplicas) spec.selection.push_back({SelFn::IMMIGRANTS});
    if (selfHealing && cm.brokers[b].isAlive()) spec.selection.push_back({SelFn::IMMIGRANT_OR_OFFLINE});
    if (!o.excludedTopics.empty()) spec.selection.push_back({SelFn::EXCLUDED_TOPICS});
    spec.selection.push_back({SelFn::LEADERS});
    cm.trackSortedReplicas((int)b, replicaSortName(false, true), spec);
  }
  fixOfflineReplicasOnly_ = false;
}
// selfSatisfied (:359-374)
bool TopicLeaderReplicaDistributionGoal::selfSatisfied(ClusterModel& cm, const BalancingAction& a) {
  const int sr = cm.replicaOnBroker(a.partition, a.sourceBroker);
  if (fixOfflineReplicasOnly_ && cm.isCurrentOffline(sr)) return a.type == ActionType::INTER_BROKER_REPLICA_MOVEMENT;
  return satisfiable(cm, cm.partitions[a.partition].topic, a.sourceBroker, a.destinationBroker);
}
// updateGoalState (:382-424)
void TopicLeaderReplicaDistributionGoal::updateGoalState(ClusterModel& cm, const OptimizationOptions&) {
  if (anyAbove_ || anyUnder_) {
    anyAbove_ = anyUnder_ = false;
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
}
// rebalanceForBroker (:518-583) + skipBrokerRebalance and its helpers (:426-504)
void TopicLeaderReplicaDistributionGoal::rebalanceForBroker(int b, ClusterModel& cm, const GoalList& g,
                                                            const OptimizationOptions& o) {
  const Broker& br = cm.brokers[b];
  for (int topic : br.topicKeys.order()) {  // Broker.topics(): HashMap key order
    if (!rebalanceTopic_[topic]) continue;
    // the tracked leaders-only view's leaders of the topic
    int n = 0, nOff = 0;
    bool hasImm = false;
    for (int r : cm.sortedReplicasView(b, replicaSortName(false, true))) {
      if (!cm.replicas[r].isLeader || cm.partitions[cm.replicas[r].partition].topic != topic) continue;
      n++;
      if (br.offlineSet.contains(r, cm.replicaHash(r))) nOff++;
      if (cm.isImmigrant(r)) hasImm = true;
    }
    const bool excluded = isExcluded(b);
    const bool requireLess = nOff > 0 || n > upper_[topic] || excluded;
    const bool requireMore = !excluded && br.isAlive() && n - nOff < lower_[topic];
    if (br.isAlive() && !requireMore && !requireLess) continue;
    if (!cm.newBrokers.empty() && !br.isNew() && !requireLess) continue;
    if (!cm.selfHealingEligibleReplicas.empty() && requireLess && nOff == 0 && !hasImm) continue;
    if (o.onlyMoveImmigrantReplicas && requireLess && !hasImm) continue;
    if (requireLess && moveOut(b, topic, cm, g, o)) anyAbove_ = true;
    if (requireMore && moveIn(b, topic, cm, g, o)) anyUnder_ = true;
  }
}
// leadersOfTopicInBroker (:585-589)
std::vector<int> TopicLeaderReplicaDistributionGoal::leadersOf(const ClusterModel& cm, int b, int topic) const {
  std::vector<int> out;
  for (int r : cm.brokers[b].replicas)
    if (cm.replicas[r].isLeader && cm.partitions[cm.replicas[r].partition].topic == topic) out.push_back(r);
  return out;
}
// replicasToMoveOut (:591-596): TreeSet(broker.replicaComparator()) of the topic's leaders retained to the tracked
// leaders-only view
std::vector<int> TopicLeaderReplicaDistributionGoal::replicasToMoveOut(ClusterModel& cm, int b, int topic) {
  const Broker& br = cm.brokers[b];
  const auto& tracked = cm.sortedReplicasView(b, replicaSortName(false, true));
  std::vector<int> out;
  for (int r : leadersOf(cm, b, topic))
    if (tracked.count(r)) out.push_back(r);
  std::sort(out.begin(), out.end(), [&](int x, int y) {
    const bool ox = br.offlineSet.contains(x, cm.replicaHash(x)), oy = br.offlineSet.contains(y, cm.replicaHash(y));
    if (ox != oy) return ox;
    const bool ix = cm.isImmigrant(x), iy = cm.isImmigrant(y);
    if (ix != iy) return ix;
    return cm.partitions[cm.replicas[x].partition].number < cm.partitions[cm.replicas[y].partition].number;
  });
  return out;
}
// rebalanceByMovingLeadersOut (:598-678)
bool TopicLeaderReplicaDistributionGoal::moveOut(int b, int topic, ClusterModel& cm, const GoalList& g,
                                                 const OptimizationOptions& o) {
  JTreeSet candidates([&cm, topic](int x, int y) {
    int c = icompare(cm.numLeadersFor(x, topic), cm.numLeadersFor(y, topic));
    if (c == 0) c = icompare(cm.brokers[x].numLeaders, cm.brokers[y].numLeaders);
    return c != 0 ? c : icompare(cm.brokers[x].id, cm.brokers[y].id);
  });
  std::vector<int> toAdd;
  if (fixOfflineReplicasOnly_) {
    toAdd = cm.aliveBrokers();
  } else {
    std::vector<int> filtered;
    for (int x : cm.aliveBrokers())
      if (cm.numLeadersFor(x, topic) < upper_[topic]) filtered.push_back(x);
    toAdd = javaHashSetOrderIntKeys(filtered);  // Collectors.toSet()
  }
  for (int x : toAdd) candidates.add(x);
  const std::vector<int> leaders = leadersOf(cm, b, topic);
  int n = (int)leaders.size(), nOff = 0;
  for (int r : leaders)
    if (cm.brokers[b].offlineSet.contains(r, cm.replicaHash(r))) nOff++;
  const int upperForSource = upper_[topic];
  bool wasUnableToMoveOffline = false;
  for (int r : replicasToMoveOut(cm, b, topic)) {
    if (wasUnableToMoveOffline && !cm.isCurrentOffline(r) && n <= upperForSource) return false;
    const bool wasOffline = cm.isCurrentOffline(r);
    const int p = cm.replicas[r].partition;
    // destination candidates per action type, each a HashSet built from the TreeSet's stream
    std::vector<int> lead, move;
    for (int x : candidates.toVector()) {
      const int xr = cm.replicaOnBroker(p, x);
      if (xr >= 0 && !cm.replicas[xr].isLeader) lead.push_back(x);  // Partition.followerBrokers()
      if (xr < 0) move.push_back(x);
    }
    int dst = maybeApplyBalancingAction(cm, r, javaHashSetOrderIntKeys(lead), ActionType::LEADERSHIP_MOVEMENT, g, o);
    if (dst < 0)
      dst = maybeApplyBalancingAction(cm, r, javaHashSetOrderIntKeys(move), ActionType::INTER_BROKER_REPLICA_MOVEMENT,
                                      g, o);
    if (dst >= 0) {
      if (wasOffline) nOff--;
      if (--n <= (nOff == 0 ? upperForSource : 0)) return false;
      candidates.removeIf([dst](int x) { return x == dst; });
      if (cm.numLeadersFor(dst, topic) < upper_[topic] || fixOfflineReplicasOnly_) candidates.add(dst);
    } else if (wasOffline) {
      wasUnableToMoveOffline = true;
    }
  }
  return !leadersOf(cm, b, topic).empty();
}
// rebalanceByMovingLeadersIn (:680-778)
bool TopicLeaderReplicaDistributionGoal::moveIn(int dest, int topic, ClusterModel& cm, const GoalList& g,
                                                const OptimizationOptions& o) {
  const int B = (int)cm.brokers.size();
  std::vector<int> offlineBy(B), leadersBy(B);  // offlineByBroker / topicLeadersByBroker
  for (int x = 0; x < B; ++x) {
    leadersBy[x] = cm.numLeadersFor(x, topic);
    int k = 0;
    for (int r : leadersOf(cm, x, topic))
      if (cm.brokers[x].offlineSet.contains(r, cm.replicaHash(r))) k++;
    offlineBy[x] = k;
  }
  JPriorityQueue pq([&](int b1, int b2) {
    const int r = icompare(offlineBy[b2], offlineBy[b1]);
    if (r != 0) return r;
    const int r2 = icompare(leadersBy[b2], leadersBy[b1]);
    if (r2 != 0) return r2;
    const int r3 = icompare(cm.brokers[b2].numLeaders, cm.brokers[b1].numLeaders);
    return r3 == 0 ? icompare(cm.brokers[b2].id, cm.brokers[b1].id) : r3;
  });
  for (int s = 0; s < B; ++s) {  // ClusterModel.brokers(): ascending id
    if (fixOfflineReplicasOnly_) {
      if (s != dest) pq.add(s);
    } else if (cm.numLeadersFor(s, topic) > lower_[topic] || hasOfflineReplicas(cm, s) || isExcluded(s)) {
      pq.add(s);
    }
  }
  int n = cm.numLeadersFor(dest, topic);
  const std::vector<int> candidates{dest};
  while (!pq.empty()) {
    const int src = pq.poll();
    const std::vector<int> toMove = replicasToMoveOut(cm, src, topic);
    int nOff = 0;
    for (int r : toMove)
      if (cm.brokers[src].offlineSet.contains(r, cm.replicaHash(r))) nOff++;
    for (int r : toMove) {
      const bool wasOffline = cm.isCurrentOffline(r);
      const bool destHas = cm.replicaOnBroker(cm.replicas[r].partition, dest) >= 0;
      ActionType action;
      if (isExcluded(dest)) {
        if (!destHas) continue;  // leadership transfer impossible
        action = ActionType::LEADERSHIP_MOVEMENT;
      } else {
        action = destHas ? ActionType::LEADERSHIP_MOVEMENT : ActionType::INTER_BROKER_REPLICA_MOVEMENT;
      }
      if (maybeApplyBalancingAction(cm, r, candidates, action, g, o) >= 0) {
        if (wasOffline) {
          nOff--;
          offlineBy[src] = std::max(0, offlineBy[src] - 1);
        }
        leadersBy[src] = std::max(0, leadersBy[src] - 1);
        leadersBy[dest] += 1;
        if (++n >= lower_[topic]) return false;
        if (!pq.empty() && nOff == 0 && cm.numLeadersFor(src, topic) < cm.numLeadersFor(pq.peek(), topic)) {
          pq.add(src);
          break;
        }
      }
    }
  }
  return true;
}

// ===================================================================== LeaderReplicaDistributionGoal
// ReplicaDistributionAbstractGoal.initGoalState (ReplicaDistributionAbstractGoal.java:124-152) with
// numInterestedReplicas = number of leaders and leader.replica.count.balance.threshold
void LeaderReplicaDistributionGoal::initGoalState(ClusterModel& cm, const OptimizationOptions& o) {
  int numAllowed = 0;
  allowed_ = allowedForReplicaMove(cm, o, &numAllowed);
  if (numAllowed == 0)
    throw OptimizationFailure("[" + name() + "] All alive brokers are excluded from replica moves.",
                              underBrokers(cm.maxReplicationFactor));
  const double avg = cm.partitions.size() / (double)numAllowed;  // ClusterModel.numLeaderReplicas()
  fixOfflineReplicasOnly_ = false;
  const double adj = (bc_.leaderReplicaBalancePercentage - 1) * 0.9;
  upper_ = (int)std::ceil(avg * (1 + adj));
  lower_ = (int)std::floor(avg * jmax(0, (1 - adj)));
}
// LeaderReplicaDistributionGoal.isLeaderMovementSatisfiable (LeaderReplicaDistributionGoal.java:117-123)
Acceptance LeaderReplicaDistributionGoal::leaderMovementSatisfiable(ClusterModel& cm, int src, int dst) const {
  const int nd = cm.brokers[dst].numLeaders, ns = cm.brokers[src].numLeaders;
  const int ud = cm.brokers[dst].isAlive() ? upper_ : 0;
  const int ls = cm.brokers[src].isAlive() ? lower_ : 0;
  return (nd + 1 <= ud && (isExcluded(src) || ns - 1 >= ls)) ? Acceptance::ACCEPT : Acceptance::REPLICA_REJECT;
}
// LeaderReplicaDistributionGoal.actionAcceptance (:91-115)
Acceptance LeaderReplicaDistributionGoal::actionAcceptance(const BalancingAction& a, ClusterModel& cm) {
  const int sr = cm.replicaOnBroker(a.partition, a.sourceBroker);
  switch (a.type) {
    case ActionType::INTER_BROKER_REPLICA_SWAP: {
      const int dr = cm.replicaOnBroker(a.destPartition, a.destinationBroker);
      if (cm.replicas[sr].isLeader && !cm.replicas[dr].isLeader)
        return leaderMovementSatisfiable(cm, a.sourceBroker, a.destinationBroker);
      if (!cm.replicas[sr].isLeader && cm.replicas[dr].isLeader)
        return leaderMovementSatisfiable(cm, a.destinationBroker, a.sourceBroker);
      return Acceptance::ACCEPT;
    }
    case ActionType::INTER_BROKER_REPLICA_MOVEMENT:
      if (cm.replicas[sr].isLeader) return leaderMovementSatisfiable(cm, a.sourceBroker, a.destinationBroker);
      return Acceptance::ACCEPT;
    case ActionType::LEADERSHIP_MOVEMENT:
      return leaderMovementSatisfiable(cm, a.sourceBroker, a.destinationBroker);
    default:
      throw std::invalid_argument("Unsupported balancing action");
  }
}
int LeaderReplicaDistributionGoal::compareStats(const ClusterModelStats& s1, const ClusterModelStats& s2) const {
  const double d1 = s1.leadStd, d2 = s2.leadStd;
  const double eps = 1e-5;
  if (d1 - d2 > eps) return -1;
  if (d2 - d1 > eps) return 1;
  return 0;
}
// ReplicaDistributionAbstractGoal.selfSatisfied (:170-181)
bool LeaderReplicaDistributionGoal::selfSatisfied(ClusterModel& cm, const BalancingAction& a) {
  const int sr = cm.replicaOnBroker(a.partition, a.sourceBroker);
  if (fixOfflineReplicasOnly_ && cm.isCurrentOffline(sr)) return true;
  return actionAcceptance(a, cm) == Acceptance::ACCEPT;
}
// ReplicaDistributionAbstractGoal.updateGoalState (:183-223)
void LeaderReplicaDistributionGoal::updateGoalState(ClusterModel& cm, const OptimizationOptions&) {
  if (anyAbove_) {
    anyAbove_ = false;
    succeeded_ = false;
  }
  if (anyUnder_) {
    anyUnder_ = false;
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
}
// LeaderReplicaDistributionGoal.rebalanceForBroker (:137-166)
void LeaderReplicaDistributionGoal::rebalanceForBroker(int b, ClusterModel& cm, const GoalList& g,
                                                       const OptimizationOptions& o) {
  const Broker& br = cm.brokers[b];
  const int nl = br.numLeaders;
  const bool excluded = isExcluded(b);
  const bool lessLeaders = br.isAlive() && nl > (excluded ? 0 : upper_);
  const bool moreLeaders = !excluded && br.isAlive() && nl < lower_;
  const bool lessReplicas = fixOfflineReplicasOnly_ && hasOfflineReplicas(cm, b);
  if (((lessLeaders && moveLeadershipOut(b, cm, g, o)) || lessReplicas) && moveReplicasOut(b, cm, g, o)) {
    if (!lessReplicas) anyAbove_ = true;
  } else if (moreLeaders && moveLeadershipIn(b, cm, g, o) && moveLeaderReplicasIn(b, cm, g, o)) {
    anyUnder_ = true;
  }
}
// LeaderReplicaDistributionGoal.rebalanceByMovingLeadershipOut (:168-203)
bool LeaderReplicaDistributionGoal::moveLeadershipOut(int b, ClusterModel& cm, const GoalList& g,
                                                      const OptimizationOptions& o) {
  if (!cm.deadBrokers.empty()) return true;
  const int upperForSource = isExcluded(b) ? 0 : upper_;
  int nl = cm.brokers[b].numLeaders;
  // new HashSet<>(broker.leaderReplicas())
  const std::vector<int> leaders = JHashSet::copyOf(cm.brokers[b].leaderSet).order();
  for (int leader : leaders) {
    if (o.excludedTopics.count(cm.partitions[cm.replicas[leader].partition].topic)) continue;
    // partition brokers (a HashSet) minus b and brokers hosting an offline replica, collected into a HashSet
    std::vector<int> cands;
    for (int x : cm.partitionBrokersSet(cm.replicas[leader].partition)) {
      if (x == b) continue;
      if (cm.isCurrentOffline(cm.replicaOnBroker(cm.replicas[leader].partition, x))) continue;
      cands.push_back(x);
    }
    cands = javaHashSetOrderIntKeys(cands);
    if (maybeApplyBalancingAction(cm, leader, cands, ActionType::LEADERSHIP_MOVEMENT, g, o) >= 0) {
      if (--nl <= upperForSource) return false;
    }
  }
  return true;
}
// LeaderReplicaDistributionGoal.rebalanceByMovingLeadershipIn (:205-240)
bool LeaderReplicaDistributionGoal::moveLeadershipIn(int b, ClusterModel& cm, const GoalList& g,
                                                     const OptimizationOptions& o) {
  if (!cm.deadBrokers.empty() || o.excludedBrokersForLeadership.count(cm.brokers[b].id)) return true;
  int nl = cm.brokers[b].numLeaders;
  const std::vector<int> candidates{b};
  for (int r : cm.brokers[b].replicaSet.order()) {  // Broker.replicas(): HashSet order
    if (cm.replicas[r].isLeader || cm.isCurrentOffline(r) || o.excludedTopics.count(cm.partitions[cm.replicas[r].partition].topic))
      continue;
    const int leader = cm.partitions[cm.replicas[r].partition].leader;
    if (maybeApplyBalancingAction(cm, leader, candidates, ActionType::LEADERSHIP_MOVEMENT, g, o) >= 0) {
      if (++nl >= lower_) return false;
    }
  }
  return true;
}
// LeaderReplicaDistributionGoal.rebalanceByMovingReplicasOut (:242-300)
bool LeaderReplicaDistributionGoal::moveReplicasOut(int b, ClusterModel& cm, const GoalList& g,
                                                    const OptimizationOptions& o) {
  JTreeSet candidates = fixOfflineReplicasOnly_
                            ? JTreeSet([&cm](int x, int y) {
                                int c = icompare((int)cm.brokers[x].replicas.size(), (int)cm.brokers[y].replicas.size());
                                return c != 0 ? c : icompare(cm.brokers[x].id, cm.brokers[y].id);
                              })
                            : JTreeSet([&cm](int x, int y) {
                                int c = icompare(cm.brokers[x].numLeaders, cm.brokers[y].numLeaders);
                                return c != 0 ? c : icompare(cm.brokers[x].id, cm.brokers[y].id);
                              });
  if (fixOfflineReplicasOnly_) {
    for (int x : cm.aliveBrokers()) candidates.add(x);
  } else {
    std::vector<int> filtered;
    for (int x : cm.aliveBrokers())
      if (cm.brokers[x].numLeaders < upper_) filtered.push_back(x);
    for (int x : javaHashSetOrderIntKeys(filtered)) candidates.add(x);
  }
  const int upperLimit = fixOfflineReplicasOnly_ ? 0 : upper_;
  const std::string sortName = replicaSortName(false, !fixOfflineReplicasOnly_);
  SortSpec spec;
  if (!fixOfflineReplicasOnly_) spec.selection.push_back({SelFn::LEADERS});
  if (fixOfflineReplicasOnly_) spec.selection.push_back({SelFn::OFFLINE});
  if ((!fixOfflineReplicasOnly_ && !cm.selfHealingEligibleReplicas.empty()) || o.onlyMoveImmigrantReplicas)
    spec.selection.push_back({SelFn::IMMIGRANTS});
  if (!o.excludedTopics.empty()) spec.selection.push_back({SelFn::EXCLUDED_TOPICS});
  cm.trackSortedReplicas(b, sortName, spec);
  std::vector<int> list = cm.sortedReplicasClone(b, sortName);
  int n = (int)list.size();
  for (int r : list) {
    const int dst = maybeApplyBalancingAction(cm, r, candidates.toVector(), ActionType::INTER_BROKER_REPLICA_MOVEMENT,
                                              g, o);
    if (dst >= 0) {
      if (--n <= upperLimit) {
        cm.brokerUntrackSortedReplicas(b, sortName);
        return false;
      }
      candidates.remove(dst);
      if (cm.brokers[dst].numLeaders < upper_ || fixOfflineReplicasOnly_) candidates.add(dst);
    }
  }
  cm.brokerUntrackSortedReplicas(b, sortName);
  return true;
}
// LeaderReplicaDistributionGoal.rebalanceByMovingLeaderReplicasIn (:302-352)
bool LeaderReplicaDistributionGoal::moveLeaderReplicasIn(int b, ClusterModel& cm, const GoalList& g,
                                                         const OptimizationOptions& o) {
  if (o.excludedBrokersForLeadership.count(cm.brokers[b].id)) return true;
  JPriorityQueue pq([&cm](int b1, int b2) {
    const int r = icompare(cm.brokers[b2].numLeaders, cm.brokers[b1].numLeaders);
    return r == 0 ? icompare(cm.brokers[b1].id, cm.brokers[b2].id) : r;
  });
  for (int x : cm.aliveBrokers())
    if (cm.brokers[x].numLeaders > lower_) pq.add(x);
  const std::vector<int> candidates{b};
  const std::string sortName = replicaSortName(false, true);
  SortSpec spec;
  spec.selection.push_back({SelFn::LEADERS});
  if (!cm.deadBrokers.empty() || !cm.brokersWithBadDisks.empty() || o.onlyMoveImmigrantReplicas)
    spec.selection.push_back({SelFn::IMMIGRANTS});
  if (!o.excludedTopics.empty()) spec.selection.push_back({SelFn::EXCLUDED_TOPICS});
  for (size_t x = 0; x < cm.brokers.size(); ++x) cm.trackSortedReplicas((int)x, sortName, spec);
  int nl = cm.brokers[b].numLeaders;
  while (!pq.empty()) {
    const int src = pq.poll();
    for (int r : cm.sortedReplicasClone(src, sortName)) {
      if (maybeApplyBalancingAction(cm, r, candidates, ActionType::INTER_BROKER_REPLICA_MOVEMENT, g, o) >= 0) {
        if (++nl >= lower_) {
          cm.untrackSortedReplicas(sortName);
          return false;
        }
        if (!pq.empty() && cm.brokers[src].numLeaders < cm.brokers[pq.peek()].numLeaders) {
          pq.add(src);
          break;
        }
      }
    }
  }
  cm.untrackSortedReplicas(sortName);
  return true;
}

// ===================================================================== LeaderBytesInDistributionGoal
// LeaderBytesInDistributionGoal.initMeanLeaderBytesIn (LeaderBytesInDistributionGoal.java:250-257)
void LeaderBytesInDistributionGoal::initMean(ClusterModel& cm) {
  if (mean_ == 0.0) {
    JDoubleSum s;
    for (int b : cm.aliveBrokers()) s.add(cm.leadershipNwIn(b));
    mean_ = s.result() / numAllowed_;
  }
}
// LeaderBytesInDistributionGoal.balanceThreshold (:264-271)
double LeaderBytesInDistributionGoal::threshold(ClusterModel& cm, int b) {
  initMean(cm);
  const double low = bc_.lowUtilizationThreshold[NW_IN] * cm.brokers[b].capacity[NW_IN];
  return jmax(mean_ * bc_.resourceBalancePercentage[NW_IN], low);
}
// LeaderBytesInDistributionGoal.actionAcceptance (:69-120)
Acceptance LeaderBytesInDistributionGoal::actionAcceptance(const BalancingAction& a, ClusterModel& cm) {
  const int sr = cm.replicaOnBroker(a.partition, a.sourceBroker);
  const int db = a.destinationBroker;
  initMean(cm);
  if (!cm.replicas[sr].isLeader) {
    switch (a.type) {
      case ActionType::INTER_BROKER_REPLICA_SWAP:
        if (!cm.replicas[cm.replicaOnBroker(a.destPartition, db)].isLeader) return Acceptance::ACCEPT;
        break;
      case ActionType::INTER_BROKER_REPLICA_MOVEMENT:
        return Acceptance::ACCEPT;
      case ActionType::LEADERSHIP_MOVEMENT:
        throw std::logic_error("Attempt to move leadership from the follower.");
      default:
        throw std::invalid_argument("Unsupported balancing action");
    }
  }
  const double srU = cm.replicaUtil(sr, NW_IN);
  double newDest;
  switch (a.type) {
    case ActionType::INTER_BROKER_REPLICA_SWAP: {
      const double drU = cm.replicaUtil(cm.replicaOnBroker(a.destPartition, db), NW_IN);
      newDest = cm.leadershipNwIn(db) + srU - drU;
      const double newSrc = cm.leadershipNwIn(a.sourceBroker) + drU - srU;
      if (newSrc > threshold(cm, a.sourceBroker)) return Acceptance::REPLICA_REJECT;
      break;
    }
    case ActionType::INTER_BROKER_REPLICA_MOVEMENT:
    case ActionType::LEADERSHIP_MOVEMENT:
      newDest = cm.leadershipNwIn(db) + srU;
      break;
    default:
      throw std::invalid_argument("Unsupported balancing action");
  }
  return !(newDest > threshold(cm, db)) ? Acceptance::ACCEPT : Acceptance::REPLICA_REJECT;
}
// LeaderBytesInDistributionGoalStatsComparator (:273-300)
int LeaderBytesInDistributionGoal::compareStats(const ClusterModelStats& s1, const ClusterModelStats& s2) const {
  const double meanPre = s1.resAvg[NW_IN];
  const double thr = meanPre * bc_.resourceBalancePercentage[NW_IN];
  if (s1.resMax[NW_IN] <= thr) return 1;
  const double d1 = std::sqrt(s2.resStd[NW_IN]), d2 = std::sqrt(s1.resStd[NW_IN]);
  const double eps = resourceEpsilon(NW_IN, d1, d2);  // AnalyzerUtils.compare(d1, d2, Resource.NW_IN)
  if (d2 - d1 > eps) return -1;
  if (d1 - d2 > eps) return 1;
  return 0;
}
// LeaderBytesInDistributionGoal.brokersToBalance (:142-152)
std::vector<int> LeaderBytesInDistributionGoal::brokersToBalance(ClusterModel& cm) {
  std::vector<int> out;
  for (size_t b = 0; b < cm.brokers.size(); ++b)
    if (cm.leadershipNwIn((int)b) > threshold(cm, (int)b)) out.push_back((int)b);
  return out;
}
bool LeaderBytesInDistributionGoal::selfSatisfied(ClusterModel& cm, const BalancingAction& a) {
  if (a.type != ActionType::LEADERSHIP_MOVEMENT) throw std::logic_error("expected leadership movement");
  return actionAcceptance(a, cm) == Acceptance::ACCEPT;
}
// LeaderBytesInDistributionGoal.initGoalState (:162-185)
void LeaderBytesInDistributionGoal::initGoalState(ClusterModel& cm, const OptimizationOptions& o) {
  allowedForReplicaMove(cm, o, &numAllowed_);
  if (numAllowed_ == 0)
    throw OptimizationFailure("[" + name() + "] All alive brokers are excluded from replica moves.",
                              underBrokers(cm.maxReplicationFactor));
  mean_ = 0.0;
  overLimit_ = false;
  SortSpec spec;
  spec.selection.push_back({SelFn::LEADERS});
  if (!o.excludedTopics.empty()) spec.selection.push_back({SelFn::EXCLUDED_TOPICS});
  spec.score = ScoreFn::REVERSE_BY_GROUP;
  spec.scoreResource = NW_IN;
  for (size_t b = 0; b < cm.brokers.size(); ++b) cm.trackSortedReplicas((int)b, replicaSortName(true, true), spec);
}
// LeaderBytesInDistributionGoal.updateGoalState (:194-201)
void LeaderBytesInDistributionGoal::updateGoalState(ClusterModel&, const OptimizationOptions&) {
  if (overLimit_) succeeded_ = false;
  overLimit_ = false;
  finished_ = true;
}
// LeaderBytesInDistributionGoal.rebalanceForBroker (:203-233)
void LeaderBytesInDistributionGoal::rebalanceForBroker(int b, ClusterModel& cm, const GoalList& g,
                                                       const OptimizationOptions& o) {
  const double thr = threshold(cm, b);
  if (cm.leadershipNwIn(b) < thr) return;
  bool over = true;
  std::vector<int> leaders = cm.sortedReplicasClone(b, replicaSortName(true, true));
  for (size_t i = 0; over && i < leaders.size(); ++i) {
    const int leader = leaders[i];
    std::vector<int> followers;
    for (int x : cm.partitions[cm.replicas[leader].partition].replicas)
      if (!cm.replicas[x].isLeader && !cm.isCurrentOffline(x)) followers.push_back(cm.replicas[x].broker);
    followers = sortedBy(followers, [&](int x, int y) {
      return dcompare(cm.leadershipNwIn(x), cm.leadershipNwIn(y));
    });
    maybeApplyBalancingAction(cm, leader, followers, ActionType::LEADERSHIP_MOVEMENT, g, o);
    over = cm.leadershipNwIn(b) > thr;
  }
  if (over) overLimit_ = true;
}

}  // namespace oracle

namespace oracle {

// ===================================================================== BrokerSetAwareGoal (BrokerSetAwareGoal.java)

// initGoalState (:80-129): BrokerSetResolutionHelper over the resolver data with NoOpBrokerSetAssignmentPolicy's
// rackIdByBrokerId form (NoOpBrokerSetAssignmentPolicy.java:70-86: every broker in no set joins "unmapped")
void BrokerSetAwareGoal::initGoalState(ClusterModel& cm, const OptimizationOptions& o) {
  int n = 0;
  allowedForReplicaMove(cm, o, &n);
  if (n == 0) {
    ProvisionRec rec;
    rec.numBrokers = cm.maxReplicationFactor;
    throw OptimizationFailure("[" + name() + "] All alive brokers are excluded from replica moves.", rec);
  }
  // _mustHaveTopicLeadersPerBroker (MinTopicLeadersPerBrokerGoal's topics) and _excludedTopics = those + the
  // options' excluded topics (:136-139)
  mustHaveTopics_.clear();
  mustHaveTopics_.insert(bc_.minLeaderTopics.begin(), bc_.minLeaderTopics.end());
  excludedTopics_.clear();
  excludedTopics_.insert(o.excludedTopics.begin(), o.excludedTopics.end());
  excludedTopics_.insert(mustHaveTopics_.begin(), mustHaveTopics_.end());
  SortSpec spec;
  if (o.onlyMoveImmigrantReplicas) spec.selection.push_back({SelFn::IMMIGRANTS});
  if (!excludedTopics_.empty()) {
    Selection ex{SelFn::EXCLUDED_TOPICS};
    ex.topics = std::make_shared<std::unordered_set<int>>(excludedTopics_.begin(), excludedTopics_.end());
    spec.selection.push_back(ex);
  }
  for (size_t b = 0; b < cm.brokers.size(); ++b) cm.trackSortedReplicas((int)b, replicaSortName(false, false), spec);
  if (bc_.brokerSets.empty()) throw std::invalid_argument("[" + name() + "] no broker sets (BrokerSetResolutionException)");
  brokersByBrokerSet_.clear();
  brokerSetIdByBrokerId_.clear();
  brokerSetIdByTopic_.clear();
  std::set<int> mapped;
  for (const auto& kv : bc_.brokerSets)
    for (int id : kv.second) {
      brokersByBrokerSet_[kv.first].insert(id);
      mapped.insert(id);
    }
  for (const auto& br : cm.brokers)
    if (!mapped.count(br.id)) brokersByBrokerSet_["unmapped"].insert(br.id);
  for (const auto& kv : brokersByBrokerSet_)
    for (int id : kv.second) brokerSetIdByBrokerId_[id] = kv.first;
}

std::string BrokerSetAwareGoal::brokerSetId(int brokerId) const {
  auto it = brokerSetIdByBrokerId_.find(brokerId);
  if (it == brokerSetIdByBrokerId_.end())
    throw std::invalid_argument("Failed to resolve BrokerSet for Broker " + std::to_string(brokerId));
  return it->second;
}

std::string BrokerSetAwareGoal::brokerSetIdForReplica(ClusterModel& cm, int r) {
  if (bc_.brokerSetPolicy == 1)  // ReplicaToOriginalBrokerSetMappingPolicy.java:20-26
    return brokerSetId(cm.brokers[cm.replicas[r].origBroker].id);
  // TopicNameHashBrokerSetMappingPolicy.java:30-70: consistent hash of the topic over the sorted set ids
  const std::string& topic = cm.topicNames[cm.partitions[cm.replicas[r].partition].topic];
  auto it = brokerSetIdByTopic_.find(topic);
  if (it != brokerSetIdByTopic_.end()) return it->second;
  std::vector<std::string> sorted;
  for (const auto& kv : brokersByBrokerSet_) sorted.push_back(kv.first);
  std::sort(sorted.begin(), sorted.end());
  const std::string id = sorted[topicNameHashBucket(topic, (int)sorted.size())];
  brokerSetIdByTopic_[topic] = id;
  return id;
}

// doesReplicaMoveViolateActionAcceptance (:262-275)
bool BrokerSetAwareGoal::violates(ClusterModel& cm, int r, int dst) {
  try {
    return brokerSetIdForReplica(cm, r) != brokerSetId(cm.brokers[dst].id);
  } catch (std::invalid_argument&) {
    return true;
  }
}

// actionAcceptance (:229-257)
Acceptance BrokerSetAwareGoal::actionAcceptance(const BalancingAction& a, ClusterModel& cm) {
  // offline replicas MinTopicLeadersPerBrokerGoal moves: its topics are accepted whatever the action (:258-264)
  if (mustHaveTopics_.count(cm.partitions[a.partition].topic)) return Acceptance::ACCEPT;
  switch (a.type) {
    case ActionType::LEADERSHIP_MOVEMENT:
      return Acceptance::ACCEPT;
    case ActionType::INTER_BROKER_REPLICA_MOVEMENT:
    case ActionType::INTER_BROKER_REPLICA_SWAP:
      if (violates(cm, cm.replicaOnBroker(a.partition, a.sourceBroker), a.destinationBroker))
        return Acceptance::BROKER_REJECT;
      if (a.type == ActionType::INTER_BROKER_REPLICA_SWAP &&
          violates(cm, cm.replicaOnBroker(a.destPartition, a.destinationBroker), a.sourceBroker))
        return Acceptance::REPLICA_REJECT;
      return Acceptance::ACCEPT;
    default:
      throw std::invalid_argument("Unsupported balancing action");
  }
}

// rebalanceForBroker (:159-188)
void BrokerSetAwareGoal::rebalanceForBroker(int b, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o) {
  const std::string current = brokerSetId(cm.brokers[b].id);
  for (int r : cm.sortedReplicasClone(b, replicaSortName(false, false))) {
    const std::string want = brokerSetIdForReplica(cm, r);
    if (cm.brokers[b].isAlive() && want == current) continue;
    std::vector<int> in;  // aliveBrokers() filtered by the set, Collectors.toSet()
    for (int x : cm.aliveBrokers())
      if (brokersByBrokerSet_.at(want).count(cm.brokers[x].id)) in.push_back(x);
    const std::vector<int> eligible = javaHashSetOrderIntKeys(in);
    if (maybeApplyBalancingAction(cm, r, eligible, ActionType::INTER_BROKER_REPLICA_MOVEMENT, g, o) < 0) {
      std::string ids = "[";
      for (size_t i = 0; i < eligible.size(); ++i) ids += (i ? ", " : "") + std::to_string(cm.brokers[eligible[i]].id);
      ProvisionRec rec;
      rec.numBrokers = cm.maxReplicationFactor;
      const int p = cm.replicas[r].partition;
      throw OptimizationFailure("[" + name() + "] Cannot move replica " + cm.topicNames[cm.partitions[p].topic] + "-" +
                                    std::to_string(cm.partitions[p].number) + " on broker " +
                                    std::to_string(cm.brokers[b].id) + " to " + ids + "] on brokerSet " + want,
                                rec);
    }
  }
}

// updateGoalState (:139-147) + ensureBrokerSetAware (:149-167) over getPartitionsByTopic (a TreeMap by name)
void BrokerSetAwareGoal::updateGoalState(ClusterModel& cm, const OptimizationOptions& o) {
  ensureNoOfflineReplicas(cm, name());
  ensureReplicasMoveOffBrokersWithBadDisks(cm, name());
  std::map<std::string, std::vector<int>> byTopic;
  for (size_t p = 0; p < cm.partitions.size(); ++p) byTopic[cm.topicNames[cm.partitions[p].topic]].push_back((int)p);
  for (const auto& kv : byTopic) {
    const int t = cm.partitions[kv.second.front()].topic;
    if (excludedTopics_.count(t)) continue;
    std::set<int> ids;
    std::vector<int> insertion;
    for (int p : kv.second)
      for (int r : cm.partitions[p].replicas) {
        const int id = cm.brokers[cm.replicas[r].broker].id;
        if (ids.insert(id).second) insertion.push_back(id);
      }
    bool contained = false;
    for (const auto& bs : brokersByBrokerSet_) {
      bool all = true;
      for (int id : ids) all = all && bs.second.count(id);
      contained = contained || all;
    }
    if (contained) continue;
    std::string s = "[";
    const std::vector<int> order = javaHashSetOrderIntKeys(insertion);
    for (size_t i = 0; i < order.size(); ++i) s += (i ? ", " : "") + std::to_string(order[i]);
    throw OptimizationFailure("[" + name() + "] Topic " + kv.first + " is not brokerSet-aware. brokers (" + s + "]).");
  }
  finished_ = true;
}

}  // namespace oracle
