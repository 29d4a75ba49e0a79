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
    case CCMI_GOAL_LEADER_REPLICA_DISTRIBUTION: return std::make_unique<LeaderReplicaDistributionGoal>(bc);
    case CCMI_GOAL_LEADER_BYTES_IN_DISTRIBUTION: return std::make_unique<LeaderBytesInDistributionGoal>(bc);
    case CCMI_GOAL_REPLICA_DISTRIBUTION: return std::make_unique<ReplicaDistributionGoal>(bc);
    case CCMI_GOAL_DISK_USAGE_DISTRIBUTION: return std::make_unique<ResourceDistributionGoal>(bc, DISK);
    case CCMI_GOAL_NW_IN_USAGE_DISTRIBUTION: return std::make_unique<ResourceDistributionGoal>(bc, NW_IN);
    case CCMI_GOAL_NW_OUT_USAGE_DISTRIBUTION: return std::make_unique<ResourceDistributionGoal>(bc, NW_OUT);
    case CCMI_GOAL_CPU_USAGE_DISTRIBUTION: return std::make_unique<ResourceDistributionGoal>(bc, CPU);
    default: throw std::invalid_argument("goal kind not in oracle scope: " + std::to_string(kind));
  }
}

// GoalOptimizer.optimizations (GoalOptimizer.java:435-524)
OptimizerResult optimizations(ClusterModel& cm, const std::vector<int>& goalKinds, const BalancingConstraint& bc,
                              const OptimizationOptions& o) {
  using clk = std::chrono::steady_clock;
  auto t0 = clk::now();
  OptimizerResult res;
  std::vector<std::unique_ptr<Goal>> owned;
  for (int k : goalKinds) owned.push_back(makeGoal(k, bc));
  std::vector<int> initDist = cm.replicaDistributionFlat();
  std::vector<int> initLeaders = cm.leaderDistribution();
  res.initStats = computeStats(cm, bc, o);
  GoalList optimized;
  std::vector<int> preDist, preLeaders;
  bool first = true;
  for (auto& g : owned) {
    if (first) {
      preDist = initDist;
      preLeaders = initLeaders;
      first = false;
    } else {
      preDist = cm.replicaDistributionFlat();
      preLeaders = cm.leaderDistribution();
    }
    auto gs = clk::now();
    int64_t c0 = cm.candidatesEvaluated;
    size_t a0 = cm.actionLog.size();
    bool succeeded = g->optimize(cm, optimized, o);
    optimized.push_back(g.get());
    GoalResult gr;
    gr.name = g->name();
    gr.succeeded = succeeded;
    gr.stats = computeStats(cm, bc, o);
    gr.seconds = std::chrono::duration<double>(clk::now() - gs).count();
    gr.candidates = cm.candidatesEvaluated - c0;
    gr.actions = (int64_t)(cm.actionLog.size() - a0);
    gr.hasDiff = (cm.replicaDistributionFlat() != preDist) || (cm.leaderDistribution() != preLeaders);
    res.goals.push_back(gr);
  }
  // AnalyzerUtils.getDiff
  std::vector<int> finalDist = cm.replicaDistributionFlat();
  size_t off = 0;
  for (size_t p = 0; p < cm.partitions.size(); ++p) {
    const Partition& part = cm.partitions[p];
    size_t n = part.replicas.size();
    std::vector<int> oldR(initDist.begin() + off, initDist.begin() + off + n);
    std::vector<int> newR(finalDist.begin() + off, finalDist.begin() + off + n);
    off += n;
    int finalLeader = cm.replicas[part.leader].broker;
    if (oldR == newR && initLeaders[p] == finalLeader) continue;
    if (newR[0] != finalLeader) {
      int pos = 0;
      for (size_t k = 0; k < n; ++k)
        if (newR[k] == finalLeader) pos = (int)k;
      newR[pos] = newR[0];
      newR[0] = finalLeader;
    }
    Proposal pr;
    pr.partition = (int)p;
    pr.partitionSize = (int)cm.replicaUtil(part.leader, DISK);
    pr.oldLeader = initLeaders[p];
    pr.oldReplicas = oldR;
    pr.newReplicas = newR;
    res.proposals.push_back(std::move(pr));
  }
  res.seconds = std::chrono::duration<double>(clk::now() - t0).count();
  res.candidates = cm.candidatesEvaluated;
  return res;
}

}  // namespace oracle
