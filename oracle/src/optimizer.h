// ORACLE — test infrastructure only (see jsem.h header).
// GoalOptimizer.optimizations restatement (analyzer/GoalOptimizer.java:435-524) and
// AnalyzerUtils.getDiff/hasDiff (analyzer/AnalyzerUtils.java:55-158).
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "goals.h"

namespace oracle {

struct GoalResult {
  std::string name;
  bool succeeded;
  bool hasDiff;
  double seconds;
  ClusterModelStats stats;  // GoalOptimizer.statsByGoalPriority entry
  int64_t candidates;
  int64_t actions;
  ProvisionResp provision;  // Goal.provisionResponse after the goal
};
// provisionResponse of the goal whose OptimizationFailure ended the last optimizations() call on this thread
const ProvisionResp& lastFailureProvision();

struct Proposal {  // ExecutionProposal (executor/ExecutionProposal.java:58-)
  int partition;
  int partitionSize;  // (int) leader DISK util
  int oldLeader;
  std::vector<int> oldReplicas, newReplicas;  // broker ids, new list has the leader first
  std::vector<int> oldDisks, newDisks;        // the logdir half of ReplicaPlacementInfo (disk index, -1 = null)
};

struct OptimizerResult {
  ClusterModelStats initStats;
  std::vector<GoalResult> goals;
  std::vector<Proposal> proposals;
  double seconds = 0;
  int64_t candidates = 0;
  std::vector<std::shared_ptr<Goal>> optimizedGoals;  // kept for Goal.actionAcceptance queries after the run
};

std::unique_ptr<Goal> makeGoal(int kind, const BalancingConstraint& bc);  // kinds: include/ccmi.h ccmi_goal_kind
bool isIntraBrokerGoal(int kind);

OptimizerResult optimizations(ClusterModel& cm, const std::vector<int>& goalKinds, const BalancingConstraint& bc,
                              const OptimizationOptions& o);

// One Goal.optimize(clusterModel, optimizedGoals, optimizationOptions) (Goal.java:60-68) with the caller's
// optimizedGoals set, as GoalViolationDetector.optimizeForGoal calls it (GoalViolationDetector.java:314) and as a
// goal-by-goal caller would; the result carries the goal's stats afterwards and AnalyzerUtils.hasDiff.
GoalResult goalOptimize(ClusterModel& cm, Goal& g, const GoalList& optimizedGoals, const BalancingConstraint& bc,
                        const OptimizationOptions& o);

}  // namespace oracle
