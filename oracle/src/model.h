// ORACLE — test infrastructure only (see jsem.h header). CPU restatement of the reference's
// in-memory cluster model, following these reference files line by line:
//   MetricValues        cruise-control-core/.../aggregator/MetricValues.java:17-221
//   AggregatedMetricValues  cruise-control-core/.../aggregator/AggregatedMetricValues.java:26-233
//   Load                cruise-control/src/main/java/.../model/Load.java:29-327
//   ModelUtils          .../model/ModelUtils.java:64-80 (follower CPU), :162-176 (expectedUtilizationFor)
//   Replica             .../model/Replica.java:25-395
//   Partition           .../model/Partition.java
//   Broker              .../model/Broker.java:336-510
//   ClusterModel        .../model/ClusterModel.java:362-441,546-564,1049-1126
//   SortedReplicas(+Helper, ReplicaSortFunctionFactory)  .../model/SortedReplicas.java,
//                       SortedReplicasHelper.java, ReplicaSortFunctionFactory.java
//   Disk                .../model/Disk.java (JBOD: Broker._diskByLogdir TreeMap, Broker.java:56,80-83,336-366,519-543)
//   Host                .../model/Host.java (load, capacity of the alive brokers, replica set; Rack._hosts keyed by
//                       name within a rack, Rack.java:256-262)
// RandomCluster names every host after its broker (RandomCluster.java:80,87); a desc's broker_host shares hosts.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "jsem.h"

namespace oracle {

enum Resource { CPU = 0, NW_IN = 1, NW_OUT = 2, DISK = 3, NUM_RESOURCES = 4 };
// Metric slots: KafkaMetricDef COMMON metrics that carry a resource group (KafkaMetricDef.java:43-53).
enum Metric { M_CPU = 0, M_DISK = 1, M_LBI = 2, M_LBO = 3, M_RBI = 4, M_RBO = 5, NUM_METRICS = 6 };
constexpr int MAXW = 5;

inline bool isHostResource(int r) { return r != DISK; }         // Resource.java:18-25
inline bool isBrokerResource(int r) { return r == CPU || r == DISK; }
inline double resourceEpsilonAbs(int r) { return r == CPU ? 0.001 : (r == DISK ? 100.0 : 10.0); }
inline double resourceEpsilon(int r, double v1, double v2) {     // Resource.epsilon
  return jmax(resourceEpsilonAbs(r), 0.0008 * (v1 + v2));
}
// Metric ids of a resource group, in MetricDef.metricInfoForGroup order.
inline int groupSize(int r) { return (r == NW_IN || r == NW_OUT) ? 2 : 1; }
inline int groupMetric(int r, int k) {
  switch (r) {
    case CPU: return M_CPU;
    case DISK: return M_DISK;
    case NW_IN: return k == 0 ? M_LBI : M_RBI;
    default: return k == 0 ? M_LBO : M_RBO;
  }
}
const char* resourceName(int r);

enum class BrokerState { ALIVE = 0, DEAD = 1, NEW = 2, DEMOTED = 3, BAD_DISKS = 4 };
enum class ActionType { INTER_BROKER_REPLICA_MOVEMENT = 0, LEADERSHIP_MOVEMENT = 1, INTER_BROKER_REPLICA_SWAP = 2,
                        INTRA_BROKER_REPLICA_MOVEMENT = 3, INTRA_BROKER_REPLICA_SWAP = 4 };
enum class Acceptance { ACCEPT = 0, REPLICA_REJECT = 1, BROKER_REJECT = 2 };

// ------------------------------------------------------------------ MetricValues
struct MV {
  float v[MAXW];
  double sum;
};
inline void mvZero(MV& m, int W) {
  for (int i = 0; i < W; ++i) m.v[i] = 0.0f;
  m.sum = 0.0;
}
inline void mvAdd(MV& a, const MV& b, int W) {          // MetricValues.add(MetricValues)
  for (int i = 0; i < W; ++i) {
    double toAdd = (double)b.v[i];
    a.v[i] = (float)((double)a.v[i] + toAdd);
    a.sum += toAdd;
  }
}
inline void mvSub(MV& a, const MV& b, int W) {          // MetricValues.subtract(MetricValues)
  for (int i = 0; i < W; ++i) {
    double toDeduct = (double)b.v[i];
    a.v[i] = (float)((double)a.v[i] - toDeduct);
    a.sum -= toDeduct;
  }
}
inline void mvSet(MV& a, int i, double value) {         // MetricValues.set
  a.sum += value - (double)a.v[i];
  a.v[i] = (float)value;
}
inline float mvAvg(const MV& a, int W) { return (float)(a.sum / W); }

// ------------------------------------------------------------------ Load / AggregatedMetricValues
struct Load {
  uint8_t mask = 0;  // bit m set <=> metric m present in the HashMap<Short, MetricValues>
  MV m[NUM_METRICS];
  bool empty() const { return mask == 0; }
};
// AggregatedMetricValues.add(other): computeIfAbsent + MetricValues.add for each metric of other.
inline void amvAdd(Load& dst, const Load& src, int W) {
  for (int k = 0; k < NUM_METRICS; ++k) {
    if (!(src.mask & (1u << k))) continue;
    if (!(dst.mask & (1u << k))) {
      mvZero(dst.m[k], W);
      dst.mask |= (uint8_t)(1u << k);
    }
    mvAdd(dst.m[k], src.m[k], W);
  }
}
inline void amvSub(Load& dst, const Load& src, int W) {
  for (int k = 0; k < NUM_METRICS; ++k) {
    if (!(src.mask & (1u << k))) continue;
    if (!(dst.mask & (1u << k))) throw std::runtime_error("Cannot subtract a values from a non-existing MetricValues");
    mvSub(dst.m[k], src.m[k], W);
  }
}
// Load.addLoad(Load) / subtractLoad(Load): no emptiness guard.
inline void loadAddLoad(Load& dst, const Load& src, int W) { amvAdd(dst, src, W); }
inline void loadSubLoad(Load& dst, const Load& src, int W) { amvSub(dst, src, W); }
// Load.addLoad(AggregatedMetricValues) / subtractLoad(AggregatedMetricValues): guarded by !isEmpty().
inline void loadAddDelta(Load& dst, const Load& delta, int W) {
  if (!dst.empty()) amvAdd(dst, delta, W);
}
inline void loadSubDelta(Load& dst, const Load& delta, int W) {
  if (!dst.empty()) amvSub(dst, delta, W);
}
// ModelUtils.expectedUtilizationFor(resource, aggregatedMetricValues).
inline double expectedUtil(const Load& l, int res, int W) {
  if (l.empty()) return 0.0;
  double result = 0;
  for (int k = 0; k < groupSize(res); ++k) {
    const MV& mv = l.m[groupMetric(res, k)];
    result += (res == DISK) ? (double)mv.v[0] : (double)mvAvg(mv, W);
  }
  return jmax(result, 0.0);
}
// AggregatedMetricValues.valuesForGroup(group, def, shareValueArray=true).avg()
inline float groupAvg(const Load& l, int res, int W) {
  if (groupSize(res) == 1) return mvAvg(l.m[groupMetric(res, 0)], W);
  MV acc;
  mvZero(acc, W);
  for (int k = 0; k < groupSize(res); ++k) mvAdd(acc, l.m[groupMetric(res, k)], W);
  return mvAvg(acc, W);
}

// ------------------------------------------------------------------ entities
struct Replica {
  int partition = -1;
  int broker = -1;
  int origBroker = -1;
  bool isLeader = false;
  bool origOfflineFlag = false;
  Load load;
  // membership flags in the current broker's HashSets
  bool inBrokerLeaders = false, inBrokerImmigrants = false, inBrokerOffline = false;
  int posInBroker = -1;
  int disk = -1, origDisk = -1;  // Replica._disk / _originalDisk (-1 = null)
};

struct Partition {
  int topic = -1;
  int number = -1;
  std::vector<int> replicas;  // Partition._replicas order (leader moved to 0 on leadership relocation)
  int leader = -1;
  std::unordered_set<int> ineligibleBrokers;
};

struct DeadlineReached : std::exception {
  const char* what() const noexcept override { return "deadline reached"; }
};

class ClusterModel;

// SortedReplicas selection / priority / score functions (ReplicaSortFunctionFactory.java)
enum class SelFn { LEADERS, FOLLOWERS, ONLINE, OFFLINE, IMMIGRANTS, IMMIGRANT_OR_OFFLINE, EXCLUDED_TOPICS,
                   ABOVE_LIMIT, BELOW_LIMIT, INCLUDED_TOPICS };
struct Selection {
  SelFn fn;
  int resource = 0;
  double limit = 0.0;
  // EXCLUDED_TOPICS: the set (null = ClusterModel.excludedTopicsSel); INCLUDED_TOPICS: selectReplicasBasedOnIncludedTopics
  std::shared_ptr<const std::unordered_set<int>> topics;
};
enum class PrioFn { IMMIGRANTS, OFFLINE, DISK_IMMIGRANTS };
enum class ScoreFn { NONE, BY_GROUP, REVERSE_BY_GROUP };
struct SortSpec {
  std::vector<Selection> selection;
  std::vector<PrioFn> priority;
  ScoreFn score = ScoreFn::NONE;
  int scoreResource = 0;
};

struct ReplicaCmp {
  const ClusterModel* cm;
  const SortSpec* spec;
  bool operator()(int a, int b) const;  // strict-weak less
  int compare(int a, int b) const;
};

struct SortedReplicas {
  SortSpec spec;
  bool initialized = false;
  std::set<int, ReplicaCmp> set;
  int owner;       // broker index
  int disk = -1;   // disk index for a disk's SortedReplicas (initialised from Disk.replicas())
  SortedReplicas(const ClusterModel* cm, SortSpec s, int broker);
};

struct Disk {  // model/Disk.java
  int broker = -1;
  std::string logdir;
  double capacity = 0;  // -1 when dead (DEAD_DISK_CAPACITY)
  bool alive = true;
  double utilization = 0;
  std::set<int> replicas;  // Disk._replicas contents
  JHashSet replicaSet;     // Disk._replicas as the HashSet PreferredLeaderElectionGoal iterates (demoted disks)
  bool demoted = false;    // Disk.State.DEMOTED (ccmi.h disk_demoted)
  std::map<std::string, std::unique_ptr<SortedReplicas>> sorted;
};

struct Broker {
  int id = -1;
  int rack = -1;
  BrokerState state = BrokerState::ALIVE;
  double capacity[NUM_RESOURCES] = {0, 0, 0, 0};
  std::vector<int> replicas;  // HashSet<Replica> contents (order not semantically used)
  int numLeaders = 0, numImmigrants = 0, numOffline = 0;
  std::unordered_map<int, int> topicReplicaCount;  // _topicReplicas keyset -> count (keys never removed)
  std::unordered_map<int, int> topicLeaderCount;   // Broker.numLeadersFor(topic), kept with every leader change
  Load load;
  Load leadershipLoadForNwResources;
  std::map<std::string, std::unique_ptr<SortedReplicas>> sorted;
  // Java iteration order of Broker._replicas / _leaderReplicas (HashSet<Replica>) and of the
  // Broker._topicReplicas key set (HashMap<String, ...>, keys never removed)
  JHashSet replicaSet, leaderSet, topicKeys;
  JHashSet offlineSet;  // Broker._currentOfflineReplicas
  std::vector<int> disks;  // Broker._diskByLogdir values (TreeMap: logdir order)
  bool isAlive() const { return state != BrokerState::DEAD; }
  bool isNew() const { return state == BrokerState::NEW; }
  bool hasBadDisks() const { return state == BrokerState::BAD_DISKS; }
};

struct Rack {
  std::string id;
  std::vector<int> brokers;
};

struct Host {  // model/Host.java
  std::vector<int> brokers;
  Load load;                               // Host._load: every add/subtract of its brokers' replica loads
  double capacity[NUM_RESOURCES] = {0, 0, 0, 0};  // Host._hostCapacity
  int aliveBrokers = 0;
  int numReplicas = 0;                     // Host._replicas.size()
};

struct BalancingAction {
  int partition;         // tp
  int sourceBroker;      // broker index
  int destinationBroker;
  ActionType type;
  int destPartition = -1;  // swap
  int sourceDisk = -1, destinationDisk = -1;  // intra-broker actions (sourceBrokerLogdir / destinationBrokerLogdir)
};

struct ActionRecord {
  int type;   // ActionType
  int partition;
  int src;
  int dst;
  int destPartition;
  int srcDisk = -1, dstDisk = -1;
};

struct OptimizationOptions {
  std::unordered_set<int> excludedTopics;
  std::unordered_set<int> excludedBrokersForLeadership;
  std::unordered_set<int> excludedBrokersForReplicaMove;
  bool triggeredByGoalViolation = false;
  std::unordered_set<int> requestedDestinationBrokerIds;
  bool onlyMoveImmigrantReplicas = false;
  bool fastMode = true;  // timeouts are disabled in parity mode regardless
};

class ClusterModel {
 public:
  int W = 1;
  std::vector<Broker> brokers;  // index == broker id
  std::vector<Rack> racks;
  std::vector<Host> hosts;
  std::vector<int> brokerHost;  // Broker.host()
  std::vector<std::string> topicNames;
  std::vector<int32_t> topicHash;  // String.hashCode of each topic name
  std::vector<int> topicRank;  // rank of topic name in String.compareTo order
  std::vector<Partition> partitions;
  std::vector<Replica> replicas;
  std::vector<int> numReplicasByTopic;
  std::vector<int> replicationFactorByTopic;
  int maxReplicationFactor = 1;
  Load load;  // cluster load
  std::vector<Load> potentialLeadershipLoad;
  std::set<int> selfHealingEligibleReplicas;
  std::set<int> newBrokers, deadBrokers, brokersWithBadDisks;
  double clusterCapacity[NUM_RESOURCES] = {0, 0, 0, 0};
  std::vector<ActionRecord> actionLog;
  bool recordActions = true;
  std::vector<Disk> disks;
  std::vector<std::pair<int, int>> diskAssignLog;  // (replica, disk) of fixture Disk.addReplica calls (desc replay)
  std::unordered_set<int> excludedTopicsSel;  // ReplicaSortFunctionFactory.selectReplicasBasedOnExcludedTopics set
  // instrumentation: reference-equivalent candidate evaluations
  int64_t candidatesEvaluated = 0;
  // CPU-baseline sampling (bench.py): stop the optimization at a wall-clock deadline (steady clock, seconds) and
  // account the time spent in ClusterModelStats separately. 0 = no deadline.
  double deadline = 0;
  mutable double statsSeconds = 0;
  void countCandidate() {
    if ((++candidatesEvaluated & 4095) == 0 && deadline > 0) checkDeadline();
  }
  void checkDeadline() const;

  // --- construction (ClusterModel.createRack/createBroker/createReplica/setReplicaLoad)
  int createRack(const std::string& id);
  // host < 0: a host of its own (RandomCluster: host named after the broker)
  int createBroker(int rackIdx, int brokerId, const double cap[NUM_RESOURCES], int host = -1);
  int ensureTopic(const std::string& name);
  int createPartition(int topic, int number);
  int createReplica(int brokerIdx, int partition, int index, bool isLeader, bool isOffline, int disk = -1);
  void setReplicaLoad(int replica, const Load& amv);  // amv carries the MetricValues as created by the caller
  void finalizeTopics();
  void setBrokerState(int brokerIdx, BrokerState s);
  void refreshCapacity();
  // --- disks (JBOD)
  int createDisk(int brokerIdx, const std::string& logdir, double capacity);  // BrokerCapacityInfo logdir entry
  int diskOf(int brokerIdx, const std::string& logdir) const;                  // Broker.disk(logdir), -1 = null
  void diskAddReplica(int d, int r);     // Disk.addReplica (Disk.java:113-121)
  void diskRemoveReplica(int d, int r);  // Disk.removeReplica (:139-146)
  void markReplicaOriginalOffline(int r);
  void markDiskDead(int brokerIdx, int d);  // ClusterModel.markDiskDead -> Broker.markDiskDead (Broker.java:537-543)
  double diskUtilizationPct(int d) const {  // GoalUtils.diskUtilizationPercentage (GoalUtils.java:397-400)
    return disks[d].capacity > 0 ? disks[d].utilization / disks[d].capacity : 1.0;
  }
  double averageDiskUtilizationPct(int b) const;  // GoalUtils.averageDiskUtilizationPercentage (:379-389)
  std::vector<int> replicaDiskFlat() const;       // [P][RF] disk of each replica slot (-1 = null)
  // ClusterModel.relocateReplica(tp, brokerId, destinationLogdir) (ClusterModel.java:362-366)
  void relocateReplicaToDisk(int partition, int brokerIdx, int dstDisk);
  SortedReplicas& trackedDiskSortedReplicas(int d, const std::string& name);
  std::vector<int> diskSortedReplicasClone(int d, const std::string& name);

  // --- queries
  Broker& broker(int idx) { return brokers[idx]; }
  const Broker& broker(int idx) const { return brokers[idx]; }
  int replicaOnBroker(int partition, int brokerIdx) const;  // Broker.replica(tp): -1 if none
  int numLeadersFor(int brokerIdx, int topic) const;         // Broker.numLeadersFor (Broker.java:202-204)
  bool isOriginalOffline(int r) const {
    const Replica& rep = replicas[r];
    return rep.origOfflineFlag || !brokers[rep.origBroker].isAlive();
  }
  bool isCurrentOffline(int r) const {
    const Replica& rep = replicas[r];
    return (isOriginalOffline(r) && rep.broker == rep.origBroker) || !brokers[rep.broker].isAlive();
  }
  bool isImmigrant(int r) const { return replicas[r].origBroker != replicas[r].broker; }
  double replicaUtil(int r, int res) const { return expectedUtil(replicas[r].load, res, W); }
  double brokerUtil(int b, int res) const { return expectedUtil(brokers[b].load, res, W); }
  // Broker.host().load().expectedUtilizationFor / Host.capacityFor (Host.java: -1 without alive brokers) /
  // Host.replicas().isEmpty()
  double hostUtil(int b, int res) const { return expectedUtil(hosts[brokerHost[b]].load, res, W); }
  double hostCapacity(int b, int res) const {
    const Host& h = hosts[brokerHost[b]];
    return h.aliveBrokers > 0 ? h.capacity[res] : -1.0;
  }
  bool hostReplicasEmpty(int b) const { return hosts[brokerHost[b]].numReplicas == 0; }
  // GoalUtils.utilization
  double utilizationPct(int b, int res) const {
    double c = brokers[b].capacity[res];
    return c > 0 ? brokerUtil(b, res) / c : 1.0;
  }
  int numReplicas() const { return (int)replicas.size(); }
  // TopicPartition.hashCode (kafka-clients: 31 * (31 + partition) + topic.hashCode()) and
  // Replica.hashCode (Replica.java:392-394: Objects.hash(tp, originalBroker.id()))
  int32_t tpHash(int p) const { return jHashMix(jHashMix(1, partitions[p].number), topicHash[partitions[p].topic]); }
  int32_t replicaHash(int r) const {
    return jHashMix(jHashMix(1, tpHash(replicas[r].partition)), brokers[replicas[r].origBroker].id);
  }
  // Replica.compareTo (Replica.java:349-377): offline first, partition number, original broker id, topic name
  int replicaCompareTo(int a, int b) const;
  // Partition.partitionBrokers(): HashSet<Broker> filled in partition replica order (Broker.hashCode == id)
  std::vector<int> partitionBrokersSet(int p) const;
  double leadershipNwIn(int b) const { return expectedUtil(brokers[b].leadershipLoadForNwResources, NW_IN, W); }
  double potentialNwOut(int b) const { return expectedUtil(potentialLeadershipLoad[b], NW_OUT, W); }
  int numTopics() const { return (int)topicNames.size(); }
  std::vector<int> aliveBrokers() const;  // HashSet<Broker> iteration order == ascending id here
  std::vector<int> aliveBrokersUnderThreshold(int res, double thr) const;
  std::vector<int> aliveBrokersOverThreshold(int res, double thr) const;
  double capacityWithAllowedReplicaMovesFor(int res, const OptimizationOptions& o) const;
  std::vector<int> onlineFollowerBrokers(int partition) const;

  // --- mutation (ClusterModel.relocateReplica / relocateLeadership)
  void relocateReplica(int partition, int srcBroker, int dstBroker);
  bool relocateLeadership(int partition, int srcBroker, int dstBroker);
  void moveReplicaToEnd(int replica);  // Partition.moveReplicaToEnd (Partition.java:192-197)

  // --- sorted replicas (Broker.trackSortedReplicas / SortedReplicas)
  void trackSortedReplicas(int brokerIdx, const std::string& name, const SortSpec& spec);
  void untrackSortedReplicas(const std::string& name);  // ClusterModel.untrackSortedReplicas
  void brokerUntrackSortedReplicas(int brokerIdx, const std::string& name);
  void clearSortedReplicas();
  void brokerClearSortedReplicas(int brokerIdx);
  SortedReplicas& trackedSortedReplicas(int brokerIdx, const std::string& name);
  const std::set<int, ReplicaCmp>& sortedReplicasView(int brokerIdx, const std::string& name);
  std::vector<int> sortedReplicasClone(int brokerIdx, const std::string& name);
  bool passesSelection(const SortSpec& spec, int r) const;

  // --- distribution snapshots (ClusterModel.getReplicaDistribution / getLeaderDistribution)
  std::vector<int> replicaDistributionFlat() const;  // [P][RF] broker ids in partition order
  std::vector<int> leaderDistribution() const;

 private:
  void brokerAddReplica(int b, int r);
  int brokerRemoveReplica(int b, int partition);
  Load brokerMakeFollower(int b, int partition);
  void brokerMakeLeader(int b, int partition, const Load& delta);
  Load replicaMakeFollower(int r);
  void sortedAdd(int b, int r);
  void sortedRemove(int b, int r);
};

// ((Double) x).intValue(): NaN -> 0, saturating, truncation toward zero (JLS 5.1.3)
inline int32_t jDoubleToInt(double x) {
  if (x != x) return 0;
  if (x >= 2147483647.0) return 2147483647;
  if (x <= -2147483648.0) return (int32_t)0x80000000;
  return (int32_t)x;
}

}  // namespace oracle
