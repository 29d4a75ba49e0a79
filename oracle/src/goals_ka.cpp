// ORACLE — test infrastructure only (see jsem.h header). Line-by-line restatement of the Kafka-assigner mode goals
// (paths relative to cruise-control/src/main/java/com/linkedin/kafka/cruisecontrol/analyzer/):
//   kafkaassigner/KafkaAssignerEvenRackAwareGoal.java, kafkaassigner/KafkaAssignerDiskUsageDistributionGoal.java,
//   kafkaassigner/KafkaAssignerUtils.java, goals/internals/BrokerAndSortedReplicas.java.
// ClusterModel.getPartitionsByTopic (model/ClusterModel.java:253-262) is a TreeMap by topic name whose lists follow
// the HashMap<TopicPartition, Partition> iteration order; TopicPartition is not Comparable, so two partitions with
// equal hashCode in one treeified bin would be ordered by System.identityHashCode in the reference (unpinnable): the
// restatement orders them by (topic name, partition number), as PreferredLeaderElectionGoal's restatement does.
#include <algorithm>
#include <cmath>
#include <limits>

#include "goals.h"

namespace oracle {

namespace {

const char* kSizeErr = "fromKey > toKey";

// getPartitionsByTopic: partitions by topic name, each list in HashMap<TopicPartition, Partition> order
std::vector<std::vector<int>> partitionsByTopic(const ClusterModel& cm) {
  JHashSet tps([&cm](int x, int y) {
    const int c = cm.topicNames[cm.partitions[x].topic].compare(cm.topicNames[cm.partitions[y].topic]);
    return c != 0 ? c : icompare(cm.partitions[x].number, cm.partitions[y].number);
  });
  for (size_t p = 0; p < cm.partitions.size(); ++p) tps.add((int)p, cm.tpHash((int)p));
  std::vector<int> topics(cm.numTopics());
  for (int t = 0; t < cm.numTopics(); ++t) topics[t] = t;
  std::sort(topics.begin(), topics.end(), [&](int a, int b) { return cm.topicRank[a] < cm.topicRank[b]; });
  std::vector<std::vector<int>> byTopic(cm.numTopics());
  for (int p : tps.order()) byTopic[cm.partitions[p].topic].push_back(p);
  std::vector<std::vector<int>> out;
  for (int t : topics)
    if (!byTopic[t].empty()) out.push_back(byTopic[t]);
  return out;
}

// Replica.toString (model/Replica.java:338-343)
std::string replicaString(const ClusterModel& cm, int r) {
  const Replica& x = cm.replicas[r];
  const Partition& p = cm.partitions[x.partition];
  auto b = [](bool v) { return v ? std::string("true") : std::string("false"); };
  return "Replica[isLeader=" + b(x.isLeader) + ",rack=" + cm.racks[cm.brokers[x.broker].rack].id +
         ",broker=" + std::to_string(cm.brokers[x.broker].id) + ",TopicPartition=" + cm.topicNames[p.topic] + "-" +
         std::to_string(p.number) + ",origBroker=" + std::to_string(cm.brokers[x.origBroker].id) +
         ",isOriginalOffline=" + b(cm.isOriginalOffline(r)) + ",isCurrentOffline=" + b(cm.isCurrentOffline(r)) + "]";
}

int numAliveRacks(const ClusterModel& cm) {
  std::vector<char> alive(cm.racks.size(), 0);
  for (const Broker& b : cm.brokers)
    if (b.isAlive()) alive[b.rack] = 1;
  int n = 0;
  for (char a : alive) n += a;
  return n;
}

}  // namespace

void kafkaAssignerSanityCheck(const OptimizationOptions& o) {
  if (o.triggeredByGoalViolation)
    throw std::invalid_argument("Kafka Assigner goals do not support usage by goal violation detector.");
  if (o.onlyMoveImmigrantReplicas)
    throw std::invalid_argument("Kafka Assigner goals do not support usage of modifying topic replication factor.");
}

// ===================================================================== KafkaAssignerEvenRackAwareGoal
// optimize (:119-165) with initGoalState (:80-117), ensureRackAwareSatisfiable (:318-343), ensureRackAware (:351-373)
bool KafkaAssignerEvenRackAwareGoal::optimize(ClusterModel& cm, const GoalList& optimizedGoals,
                                              const OptimizationOptions& o) {
  kafkaAssignerSanityCheck(o);
  if (!optimizedGoals.empty())
    throw std::invalid_argument("Goals " + std::to_string(optimizedGoals.size()) + " cannot be optimized before " + name() + ".");
  const std::unordered_set<int>& excluded = o.excludedTopics;
  // ensureRackAwareSatisfiable
  const int racks = numAliveRacks(cm);
  if (!excluded.empty()) {
    std::vector<int> insertion(cm.numTopics());
    for (int t = 0; t < cm.numTopics(); ++t) insertion[t] = t;
    int maxRf = 1;
    for (int t : topicHashSetOrder(cm, insertion)) {  // _replicationFactorByTopic: HashMap<String, Integer> order
      if (excluded.count(t)) continue;
      maxRf = std::max(maxRf, cm.replicationFactorByTopic[t]);
      if (maxRf > racks)
        throw OptimizationFailure("[" + name() + "] Insufficient number of racks to distribute included replicas (Current: " +
                                  std::to_string(racks) + ", Needed: " + std::to_string(maxRf) + ").");
    }
  } else if (cm.maxReplicationFactor > racks) {
    throw OptimizationFailure("[" + name() + "] Insufficient number of racks to distribute each replica (Current: " +
                              std::to_string(racks) + ", Needed: " + std::to_string(cm.maxReplicationFactor) + ").");
  }
  const std::vector<std::vector<int>> byTopic = partitionsByTopic(cm);
  // the number of excluded replicas by position for each broker: leader at 0, followers in replica-list order
  std::vector<std::map<int, int>> excludedByPos(cm.brokers.size());
  for (const auto& parts : byTopic)
    for (int p : parts) {
      const Partition& part = cm.partitions[p];
      if (!excluded.count(part.topic)) continue;
      int pos = 0;
      excludedByPos[cm.replicas[part.leader].broker][pos]++;
      for (int r : part.replicas) {
        if (r == part.leader) continue;
        excludedByPos[cm.replicas[r].broker][++pos]++;
      }
    }
  byPosition_.assign(cm.maxReplicationFactor, {});
  for (int i = 0; i < cm.maxReplicationFactor; ++i)
    for (int b : cm.aliveBrokers()) {
      auto it = excludedByPos[b].find(i);
      byPosition_[i].insert({it == excludedByPos[b].end() ? 0 : it->second, cm.brokers[b].id});
    }
  // STEP1: the leader first in every partition's replica list
  for (const auto& parts : byTopic)
    for (int p : parts) {
      Partition& part = cm.partitions[p];
      if (part.replicas[0] != part.leader) {
        const size_t at = (size_t)(std::find(part.replicas.begin(), part.replicas.end(), part.leader) - part.replicas.begin());
        std::swap(part.replicas[0], part.replicas[at]);
      }
    }
  // STEP2
  for (int position = 0; position < cm.maxReplicationFactor; ++position)
    for (const auto& parts : byTopic)
      for (int p : parts) {
        const Partition& part = cm.partitions[p];
        if ((int)part.replicas.size() <= position) continue;
        const int r = part.replicas[position];
        if (excluded.count(part.topic) && !cm.isOriginalOffline(r)) continue;  // shouldExclude (:307-310)
        if (!maybeApplyMove(cm, p, position))
          throw OptimizationFailure("[" + name() + "] Unable to apply move for replica " +
                                    replicaString(cm, cm.partitions[p].replicas[position]) + ".");
      }
  ensureNoOfflineReplicas(cm, name());
  // ensureRackAware: every included partition has its replicas on distinct racks
  for (size_t p = 0; p < cm.partitions.size(); ++p) {
    const Partition& part = cm.partitions[p];
    if (excluded.count(part.topic)) continue;
    std::set<int> brokers, racksSeen;
    for (int r : part.replicas)
      if (r != part.leader) brokers.insert(cm.replicas[r].broker);
    for (int b : brokers) racksSeen.insert(cm.brokers[b].rack);
    racksSeen.insert(cm.brokers[cm.replicas[part.leader].broker].rack);
    if (racksSeen.size() != brokers.size() + 1)
      throw OptimizationFailure("Optimization for goal " + name() + " failed for rack-awareness of partition " +
                                cm.topicNames[part.topic] + "-" + std::to_string(part.number));
  }
  return true;
}

// maybeApplyMove (:185-247)
bool KafkaAssignerEvenRackAwareGoal::maybeApplyMove(ClusterModel& cm, int p, int position) {
  std::set<int> ineligibleRacks;
  for (int pos = 0; pos < position; ++pos) ineligibleRacks.insert(cm.brokers[cm.replicas[cm.partitions[p].replicas[pos]].broker].rack);
  auto& set = byPosition_[position];
  for (auto it = set.begin(); it != set.end(); ++it) {
    const int dest = it->second;  // broker id == index
    if (ineligibleRacks.count(cm.brokers[dest].rack)) continue;
    const int destReplica = cm.replicaOnBroker(p, dest);
    const int r = cm.partitions[p].replicas[position];
    const int src = cm.replicas[r].broker;
    if (destReplica < 0) {
      cm.relocateReplica(p, src, dest);
    } else if (cm.brokers[dest].id != cm.brokers[src].id && cm.brokers[src].isAlive()) {
      if (position == 0) {
        cm.relocateLeadership(p, src, dest);
      } else {
        // followerPosition (:256-265) then Partition.swapFollowerPositions (Partition.java:162-172)
        std::vector<int>& reps = cm.partitions[p].replicas;
        size_t destPos = 0;
        while (destPos < reps.size() && cm.replicas[reps[destPos]].broker != dest) ++destPos;
        if (destPos == reps.size()) throw std::invalid_argument("Partition has no follower on " + std::to_string(dest) + ".");
        if (cm.replicas[reps[position]].isLeader || cm.replicas[reps[destPos]].isLeader)
          throw std::invalid_argument("not a follower");
        std::swap(reps[position], reps[destPos]);
      }
    } else if (!cm.brokers[src].isAlive()) {
      continue;
    }
    const std::pair<int, int> e{it->first + 1, it->second};
    set.erase(it);
    set.insert(e);
    return true;
  }
  return false;
}

// isReplicaMoveViolateRackAwareness (:410-423): another broker of the partition on the destination's rack
bool KafkaAssignerEvenRackAwareGoal::violates(const ClusterModel& cm, int replica, int dest) const {
  const int p = cm.replicas[replica].partition, self = cm.replicas[replica].broker;
  for (int r : cm.partitions[p].replicas) {
    const int b = cm.replicas[r].broker;
    if (b != self && cm.brokers[b].rack == cm.brokers[dest].rack) return true;
  }
  return false;
}

// actionAcceptance (:385-408)
Acceptance KafkaAssignerEvenRackAwareGoal::actionAcceptance(const BalancingAction& a, ClusterModel& cm) {
  switch (a.type) {
    case ActionType::LEADERSHIP_MOVEMENT: return Acceptance::ACCEPT;
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

// ===================================================================== KafkaAssignerDiskUsageDistributionGoal
Acceptance KafkaAssignerDiskUsageDistributionGoal::actionAcceptance(const BalancingAction&, ClusterModel&) {
  throw std::logic_error("No goal should be executed after " + name());  // IllegalStateException (:540-543)
}

namespace {

struct Kadud {
  ClusterModel& cm;
  const std::unordered_set<int>& excluded;
  // BrokerAndSortedReplicas: per alive broker a TreeSet ordered by (replica size, Replica.compareTo)
  std::vector<std::unique_ptr<JTreeSet>> sorted;

  double replicaSize(int r) const { return cm.replicaUtil(r, DISK); }
  double diskUsage(int b) const {  // diskUsage(Broker) (:577-581)
    const double cap = cm.brokers[b].capacity[DISK];
    return dcompare(cap, 0.0) < 1 ? 0.0 : cm.brokerUtil(b, DISK) / cap;
  }
  double brokerSize(int b) const { return diskUsage(b) * cm.brokers[b].capacity[DISK]; }
  int rackOf(int b) const { return cm.brokers[b].rack; }
  bool partitionOnRack(int p, int rack) const {  // partition(tp).partitionRacks() contains rack
    for (int r : cm.partitions[p].replicas)
      if (rackOf(cm.replicas[r].broker) == rack) return true;
    return false;
  }
  // possibleToMove (:481-491)
  bool possibleToMove(int r, int dest) const {
    const int p = cm.replicas[r].partition;
    const bool case1 = !partitionOnRack(p, rackOf(dest));
    const bool case2 = rackOf(cm.replicas[r].broker) == rackOf(dest) && cm.replicaOnBroker(p, dest) < 0;
    return case1 || case2;
  }
  // canSwap (:504-518)
  bool canSwap(int r1, int r2) const {
    const int b1 = cm.replicas[r1].broker, b2 = cm.replicas[r2].broker;
    const bool sameRack = b1 != b2 && rackOf(b1) == rackOf(b2);
    const bool rackAware = !partitionOnRack(cm.replicas[r1].partition, rackOf(b2)) &&
                           !partitionOnRack(cm.replicas[r2].partition, rackOf(b1));
    return (sameRack || rackAware) && cm.replicas[r1].isLeader == cm.replicas[r2].isLeader;
  }
  // ReplicaWrapper order over a broker's sorted replicas (a fresh TreeSet<ReplicaWrapper>: sorted, deduplicated)
  std::vector<int> wrappers(int b, bool followersOnly) const {
    std::vector<int> v;
    for (int r : sorted[b]->toVector()) {
      const bool ex = excluded.count(cm.partitions[cm.replicas[r].partition].topic) > 0;
      if (followersOnly ? (!cm.replicas[r].isLeader || ex) : !ex) v.push_back(r);
    }
    auto cmpW = [&](int x, int y) {
      const int c = dcompare(replicaSize(x), replicaSize(y));
      return c != 0 ? c : cm.replicaCompareTo(x, y);
    };
    std::sort(v.begin(), v.end(), [&](int x, int y) { return cmpW(x, y) < 0; });
    v.erase(std::unique(v.begin(), v.end(), [&](int x, int y) { return cmpW(x, y) == 0; }), v.end());
    return v;
  }

  // findReplicaToSwapWith (:398-466) over the ascending wrapper list `w`
  int findReplicaToSwapWith(int replica, const std::vector<int>& w, double target, double minS, double maxS) const {
    if (minS > maxS) return -1;
    if (dcompare(minS, maxS) > 0) throw std::invalid_argument(kSizeErr);  // TreeMap.subMap with NaN bounds
    // subSet((MAX_REPLICA, minS) exclusive, (MIN_REPLICA, maxS) exclusive): sizes strictly inside (minS, maxS)
    size_t lo = 0, hi = w.size();
    while (lo < w.size() && dcompare(replicaSize(w[lo]), minS) <= 0) ++lo;
    while (hi > lo && dcompare(replicaSize(w[hi - 1]), maxS) >= 0) --hi;
    if (lo >= hi) return -1;
    // ascending iterator over [ia, hi) and descending over [lo, id] (indices into w); -1 = no iterator
    long ia = -1, idd = -1;
    bool asc = false, desc = false;
    if (target <= minS) {
      asc = true;
      ia = (long)lo;
    } else if (target >= maxS) {
      desc = true;
      idd = (long)hi - 1;
    } else {
      asc = desc = true;
      ia = (long)lo;
      while (ia < (long)hi && dcompare(replicaSize(w[ia]), target) < 0) ++ia;  // tailSet((MIN_REPLICA, target), true)
      idd = (long)hi - 1;
      while (idd >= (long)lo && dcompare(replicaSize(w[idd]), target) > 0) --idd;  // headSet((MAX_REPLICA, target), true)
    }
    long low = -1, high = -1, cand = -1;  // wrapper indices, -1 = null (the reference compares references)
    for (;;) {
      if (cand == high) high = asc && ia < (long)hi ? ia++ : -1;
      if (cand == low) low = desc && idd >= (long)lo ? idd-- : -1;
      if (high < 0 && low < 0) return -1;
      if (high < 0) {
        cand = low;
      } else if (low < 0) {
        cand = high;
      } else {
        const double lowDiff = target - replicaSize(w[low]);
        const double highDiff = replicaSize(w[high]) - target;
        cand = lowDiff <= highDiff ? low : high;
      }
      if (canSwap(replica, w[cand])) return w[cand];
    }
  }

  // swapReplicas (:268-383)
  bool swapReplicas(int toSwap, int toSwapWith, double mean) {
    const double capS = cm.brokers[toSwap].capacity[DISK], capW = cm.brokers[toSwapWith].capacity[DISK];
    const double sizeToChange = capS * mean - brokerSize(toSwap);
    const std::vector<int> mine = wrappers(toSwap, false);
    const std::vector<int> leadersW = wrappers(toSwapWith, false), followersW = wrappers(toSwapWith, true);
    const size_t n = mine.size();
    for (size_t k = 0; k < n; ++k) {
      const int replicaToSwap = sizeToChange > 0 ? mine[k] : mine[n - 1 - k];
      if (excluded.count(cm.partitions[cm.replicas[replicaToSwap].partition].topic)) continue;
      if (!possibleToMove(replicaToSwap, toSwapWith)) continue;
      const std::vector<int>& candidates = cm.replicas[replicaToSwap].isLeader ? leadersW : followersW;
      const double sizeToSwap = replicaSize(replicaToSwap);
      if (sizeToChange < 0 && sizeToSwap == 0) break;
      double maxSize = std::numeric_limits<double>::max();
      double minSize = std::numeric_limits<double>::denorm_min();  // Double.MIN_VALUE
      if (sizeToChange > 0) {
        minSize = sizeToSwap;
        const double maxSizeOfBrokerToSwap = diskUsage(toSwapWith) * capS;
        const double currentSizeOfBrokerToSwap = brokerSize(toSwap);
        maxSize = jmin(maxSize, maxSizeOfBrokerToSwap - (currentSizeOfBrokerToSwap - sizeToSwap));
        const double minSizeOfBrokerToSwapWith = diskUsage(toSwap) * capW;
        const double currentSizeOfBrokerToSwapWith = brokerSize(toSwapWith);
        maxSize = jmin(maxSize, (currentSizeOfBrokerToSwapWith + sizeToSwap) - minSizeOfBrokerToSwapWith);
      } else {
        maxSize = sizeToSwap;
        const double minSizeOfBrokerToSwap = diskUsage(toSwapWith) * capS;
        const double currentSizeOfBrokerToSwap = brokerSize(toSwap);
        minSize = jmax(minSize, minSizeOfBrokerToSwap - (currentSizeOfBrokerToSwap - sizeToSwap));
        const double maxSizeOfBrokerToSwapWith = diskUsage(toSwap) * capW;
        const double currentSizeOfBrokerToSwapWith = brokerSize(toSwapWith);
        minSize = jmax(minSize, (currentSizeOfBrokerToSwapWith + sizeToSwap) - maxSizeOfBrokerToSwapWith);
      }
      minSize += 0.4;  // REPLICA_CONVERGENCE_DELTA
      maxSize -= 0.4;
      const double targetSize = sizeToSwap + sizeToChange;
      const int with = candidates.empty() ? -1 : findReplicaToSwapWith(replicaToSwap, candidates, targetSize, minSize, maxSize);
      if (with >= 0) {
        const int pWith = cm.replicas[with].partition, pMine = cm.replicas[replicaToSwap].partition;
        cm.relocateReplica(pWith, toSwapWith, toSwap);
        cm.relocateReplica(pMine, toSwap, toSwapWith);
        sorted[toSwap]->remove(replicaToSwap);
        sorted[toSwap]->add(with);
        sorted[toSwapWith]->remove(with);
        sorted[toSwapWith]->add(replicaToSwap);
        return true;
      }
    }
    return false;
  }
};

}  // namespace

// optimize (:107-144) with checkAndOptimize (:197-252) and isOptimized (:156-181)
bool KafkaAssignerDiskUsageDistributionGoal::optimize(ClusterModel& cm, const GoalList&, const OptimizationOptions& o) {
  kafkaAssignerSanityCheck(o);
  Kadud k{cm, o.excludedTopics, {}};
  const double mean = expectedUtil(cm.load, DISK, cm.W) / cm.clusterCapacity[DISK];
  const double margin = (bc_.resourceBalancePercentage[DISK] - 1) * 0.9;
  const double upper = mean * (1 + margin), lower = mean * jmax(0, (1 - margin));
  k.sorted.resize(cm.brokers.size());
  std::vector<int> alive = cm.aliveBrokers();
  for (int b : alive) {
    k.sorted[b] = std::make_unique<JTreeSet>([&cm, &k](int x, int y) {
      int c = dcompare(k.replicaSize(x), k.replicaSize(y));
      if (c == 0) c = cm.replicaCompareTo(x, y);
      return c == 0 ? cm.replicaCompareTo(x, y) : c;
    });
    for (int r : cm.brokers[b].replicaSet.order()) k.sorted[b]->add(r);  // addAll(broker.replicas())
  }
  auto brokerLess = [&](int x, int y) {
    const int c = dcompare(k.diskUsage(x), k.diskUsage(y));
    return c != 0 ? c < 0 : cm.brokers[x].id < cm.brokers[y].id;
  };
  std::vector<int> all = alive;  // allBrokers: a TreeSet kept consistent (members leave before a swap, re-enter after)
  std::sort(all.begin(), all.end(), brokerLess);
  bool improved;
  do {
    improved = false;
    const std::vector<int> snapshot = all;
    for (int toOptimize : snapshot) {
      // checkAndOptimize
      const double usage = k.diskUsage(toOptimize);
      std::vector<int> cands;
      const size_t at = (size_t)(std::find(all.begin(), all.end(), toOptimize) - all.begin());
      if (usage > upper) {
        cands.assign(all.begin(), all.begin() + (ptrdiff_t)at);  // headSet(toOptimize), ascending
      } else if (usage < lower) {
        cands.assign(all.rbegin(), all.rend() - (ptrdiff_t)at);  // tailSet(toOptimize) reversed
      } else {
        continue;
      }
      bool done = false;
      for (int toSwapWith : cands) {
        if (toSwapWith == toOptimize || std::fabs(k.diskUsage(toSwapWith) - k.diskUsage(toOptimize)) < 0.0001) continue;
        const bool swapped = k.swapReplicas(toOptimize, toSwapWith, mean);
        std::sort(all.begin(), all.end(), brokerLess);  // removeAll + addAll with the new keys
        if (swapped) {
          done = true;
          break;
        }
      }
      if (done) improved = true;
    }
  } while (improved);
  for (int b : alive) {
    const double u = k.diskUsage(b);
    if (u < lower || u > upper) return false;
  }
  return true;
}

}  // namespace oracle
