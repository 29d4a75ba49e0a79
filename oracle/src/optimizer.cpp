// ORACLE — test infrastructure only (see jsem.h header).
#include "optimizer.h"

#include <chrono>

#include "../../include/ccmi.h"

namespace oracle {

std::unique_ptr<Goal> makeGoal(int kind, const BalancingConstraint& bc) {
  switch (kind) {
    case CCMI_GOAL_RACK_AWARE: return std::make_unique<RackAwareGoal>(bc);
    case CCMI_GOAL_MIN_TOPIC_LEADERS_PER_BROKER: return std::make_unique<MinTopicLeadersPerBrokerGoal>(bc);
    case CCMI_GOAL_REPLICA_CAPACITY: return std::make_unique<ReplicaCapacityGoal>(bc);
    case CCMI_GOAL_DISK_CAPACITY: return std::make_unique<CapacityGoal>(bc, DISK);
    case CCMI_GOAL_NW_IN_CAPACITY: return std::make_unique<CapacityGoal>(bc, NW_IN);
    case CCMI_GOAL_NW_OUT_CAPACITY: return std::make_unique<CapacityGoal>(bc, NW_OUT);
    case CCMI_GOAL_CPU_CAPACITY: return std::make_unique<CapacityGoal>(bc, CPU);
    case CCMI_GOAL_POTENTIAL_NW_OUT: return std::make_unique<PotentialNwOutGoal>(bc);
    case CCMI_GOAL_TOPIC_REPLICA_DISTRIBUTION: return std::make_unique<TopicReplicaDistributionGoal>(bc);
    case CCMI_GOAL_TOPIC_LEADER_REPLICA_DISTRIBUTION: return std::make_unique<TopicLeaderReplicaDistributionGoal>(bc);
    case CCMI_GOAL_LEADER_REPLICA_DISTRIBUTION: return std::make_unique<LeaderReplicaDistributionGoal>(bc);
    case CCMI_GOAL_LEADER_BYTES_IN_DISTRIBUTION: return std::make_unique<LeaderBytesInDistributionGoal>(bc);
    case CCMI_GOAL_REPLICA_DISTRIBUTION: return std::make_unique<ReplicaDistributionGoal>(bc);
    case CCMI_GOAL_DISK_USAGE_DISTRIBUTION: return std::make_unique<ResourceDistributionGoal>(bc, DISK);
    case CCMI_GOAL_NW_IN_USAGE_DISTRIBUTION: return std::make_unique<ResourceDistributionGoal>(bc, NW_IN);
    case CCMI_GOAL_NW_OUT_USAGE_DISTRIBUTION: return std::make_unique<ResourceDistributionGoal>(bc, NW_OUT);
    case CCMI_GOAL_CPU_USAGE_DISTRIBUTION: return std::make_unique<ResourceDistributionGoal>(bc, CPU);
    case CCMI_GOAL_INTRA_BROKER_DISK_CAPACITY: return std::make_unique<IntraBrokerDiskCapacityGoal>(bc);
    case CCMI_GOAL_INTRA_BROKER_DISK_USAGE_DISTRIBUTION:
      return std::make_unique<IntraBrokerDiskUsageDistributionGoal>(bc);
    case CCMI_GOAL_PREFERRED_LEADER_ELECTION: return std::make_unique<PreferredLeaderElectionGoal>(bc);
    case CCMI_GOAL_RACK_AWARE_DISTRIBUTION: return std::make_unique<RackAwareDistributionGoal>(bc);
    case CCMI_GOAL_BROKER_SET_AWARE: return std::make_unique<BrokerSetAwareGoal>(bc);
    case CCMI_GOAL_KAFKA_ASSIGNER_EVEN_RACK_AWARE: return std::make_unique<KafkaAssignerEvenRackAwareGoal>(bc);
    case CCMI_GOAL_KAFKA_ASSIGNER_DISK_USAGE_DISTRIBUTION:
      return std::make_unique<KafkaAssignerDiskUsageDistributionGoal>(bc);
    default: throw std::invalid_argument("goal kind not in oracle scope: " + std::to_string(kind));
  }
}

namespace {
thread_local ProvisionResp g_lastFailure;
}
const ProvisionResp& lastFailureProvision() { return g_lastFailure; }

bool isIntraBrokerGoal(int kind) {
  return kind == CCMI_GOAL_INTRA_BROKER_DISK_CAPACITY || kind == CCMI_GOAL_INTRA_BROKER_DISK_USAGE_DISTRIBUTION;
}

// GoalOptimizer.optimizations (GoalOptimizer.java:435-524). Distributions are ReplicaPlacementInfo lists: the broker
// and (with JBOD placement) the disk of every replica slot (ClusterModel.getReplicaDistribution :167-182).
OptimizerResult optimizations(ClusterModel& cm, const std::vector<int>& goalKinds, const BalancingConstraint& bc,
                              const OptimizationOptions& o) {
  using clk = std::chrono::steady_clock;
  auto t0 = clk::now();
  OptimizerResult res;
  // Broker- and disk-granularity goals reject each other's actions with IllegalArgumentException (e.g.
  // ResourceDistributionGoal.actionAcceptance default branch, IntraBrokerDiskCapacityGoal.actionAcceptance :120-124);
  // a chain mixing them is refused up front.
  int intra = 0;
  for (int k : goalKinds) intra += isIntraBrokerGoal(k) ? 1 : 0;
  if (intra != 0 && intra != (int)goalKinds.size())
    throw std::invalid_argument("intra-broker goals cannot be optimized together with inter-broker goals");
  if (intra != 0 && cm.disks.empty()) throw std::invalid_argument("intra-broker goals need replica placement over disks");
  cm.excludedTopicsSel = o.excludedTopics;  // ReplicaSortFunctionFactory.selectReplicasBasedOnExcludedTopics's set
  std::vector<std::shared_ptr<Goal>> owned;
  for (int k : goalKinds) owned.push_back(makeGoal(k, bc));
  const std::vector<int> initDist = cm.replicaDistributionFlat(), initDisks = cm.replicaDiskFlat();
  const std::vector<int> initLeaders = cm.leaderDistribution();
  auto leaderDisks = [&]() {
    std::vector<int> out;
    for (const Partition& p : cm.partitions) out.push_back(cm.replicas[p.leader].disk);
    return out;
  };
  const std::vector<int> initLeaderDisks = leaderDisks();
  res.initStats = computeStats(cm, bc, o);
  GoalList optimized;
  std::vector<int> preDist = initDist, preDisks = initDisks, preLeaders = initLeaders, preLeaderDisks = initLeaderDisks;
  bool first = true;
  for (auto& g : owned) {
    if (!first) {
      preDist = cm.replicaDistributionFlat();
      preDisks = cm.replicaDiskFlat();
      preLeaders = cm.leaderDistribution();
      preLeaderDisks = leaderDisks();
    }
    first = false;
    auto gs = clk::now();
    int64_t c0 = cm.candidatesEvaluated;
    size_t a0 = cm.actionLog.size();
    bool succeeded;
    try {
      succeeded = g->optimize(cm, optimized, o);
    } catch (OptimizationFailure&) {
      g_lastFailure = g->provision();
      throw;
    }
    optimized.push_back(g.get());
    GoalResult gr;
    gr.name = g->name();
    gr.succeeded = succeeded;
    gr.stats = computeStats(cm, bc, o);
    gr.seconds = std::chrono::duration<double>(clk::now() - gs).count();
    gr.candidates = cm.candidatesEvaluated - c0;
    gr.actions = (int64_t)(cm.actionLog.size() - a0);
    gr.provision = g->provision();
    gr.hasDiff = cm.replicaDistributionFlat() != preDist || cm.replicaDiskFlat() != preDisks ||
                 cm.leaderDistribution() != preLeaders || leaderDisks() != preLeaderDisks;
    res.goals.push_back(gr);
  }
  // AnalyzerUtils.getDiff (AnalyzerUtils.java:63-93)
  const std::vector<int> finalDist = cm.replicaDistributionFlat(), finalDisks = cm.replicaDiskFlat();
  size_t off = 0;
  for (size_t p = 0; p < cm.partitions.size(); ++p) {
    const Partition& part = cm.partitions[p];
    const size_t n = part.replicas.size();
    std::vector<int> oldR(initDist.begin() + off, initDist.begin() + off + n);
    std::vector<int> newR(finalDist.begin() + off, finalDist.begin() + off + n);
    std::vector<int> oldD(initDisks.begin() + off, initDisks.begin() + off + n);
    std::vector<int> newD(finalDisks.begin() + off, finalDisks.begin() + off + n);
    off += n;
    const int finalLeader = cm.replicas[part.leader].broker, finalLeaderDisk = cm.replicas[part.leader].disk;
    if (oldR == newR && oldD == newD && initLeaders[p] == finalLeader && initLeaderDisks[p] == finalLeaderDisk) continue;
    int pos = 0;  // finalReplicas.indexOf(finalLeaderPlacementInfo), then swap with slot 0
    for (size_t k = 0; k < n; ++k)
      if (newR[k] == finalLeader && newD[k] == finalLeaderDisk) {
        pos = (int)k;
        break;
      }
    std::swap(newR[pos], newR[0]);
    std::swap(newD[pos], newD[0]);
    Proposal pr;
    pr.partition = (int)p;
    pr.partitionSize = (int)cm.replicaUtil(part.leader, DISK);
    pr.oldLeader = initLeaders[p];
    pr.oldReplicas = oldR;
    pr.newReplicas = newR;
    pr.oldDisks = oldD;
    pr.newDisks = newD;
    res.proposals.push_back(std::move(pr));
  }
  res.seconds = std::chrono::duration<double>(clk::now() - t0).count();
  res.candidates = cm.candidatesEvaluated;
  res.optimizedGoals = owned;
  return res;
}

GoalResult goalOptimize(ClusterModel& cm, Goal& g, const GoalList& optimizedGoals, const BalancingConstraint& bc,
                        const OptimizationOptions& o) {
  using clk = std::chrono::steady_clock;
  cm.excludedTopicsSel = o.excludedTopics;
  const std::vector<int> preDist = cm.replicaDistributionFlat(), preDisks = cm.replicaDiskFlat();
  const std::vector<int> preLeaders = cm.leaderDistribution();
  auto leaderDisks = [&]() {
    std::vector<int> out;
    for (const Partition& p : cm.partitions) out.push_back(cm.replicas[p.leader].disk);
    return out;
  };
  const std::vector<int> preLeaderDisks = leaderDisks();
  const auto gs = clk::now();
  const int64_t c0 = cm.candidatesEvaluated;
  const size_t a0 = cm.actionLog.size();
  GoalResult gr;
  try {
    gr.succeeded = g.optimize(cm, optimizedGoals, o);
  } catch (OptimizationFailure&) {
    g_lastFailure = g.provision();
    throw;
  }
  gr.name = g.name();
  gr.stats = computeStats(cm, bc, o);
  gr.seconds = std::chrono::duration<double>(clk::now() - gs).count();
  gr.candidates = cm.candidatesEvaluated - c0;
  gr.actions = (int64_t)(cm.actionLog.size() - a0);
  gr.provision = g.provision();
  gr.hasDiff = cm.replicaDistributionFlat() != preDist || cm.replicaDiskFlat() != preDisks ||
               cm.leaderDistribution() != preLeaders || leaderDisks() != preLeaderDisks;
  return gr;
}

}  // namespace oracle
