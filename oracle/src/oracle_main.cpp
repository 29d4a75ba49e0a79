// ORACLE — test infrastructure only (see jsem.h header). CLI used to time the CPU restatement and
// to print a summary: oracle_cc <config C0|C1|C2|C3|custom args> [goal kinds...]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/ccmi.h"
#include "optimizer.h"
#include "random_cluster.h"

using namespace oracle;

int main(int argc, char** argv) {
  ClusterProperties p;
  std::string cfg = argc > 1 ? argv[1] : "C0";
  std::vector<int> goals;
  BalancingConstraint bc;
  if (cfg == "C0") {
    goals = {CCMI_GOAL_REPLICA_DISTRIBUTION, CCMI_GOAL_DISK_USAGE_DISTRIBUTION, CCMI_GOAL_NW_IN_USAGE_DISTRIBUTION,
             CCMI_GOAL_NW_OUT_USAGE_DISTRIBUTION, CCMI_GOAL_CPU_USAGE_DISTRIBUTION};
    for (int r = 0; r < 4; ++r) {
      bc.resourceBalancePercentage[r] = 1.05;
      bc.capacityThreshold[r] = 0.8;
    }
    bc.maxReplicasPerBroker = 1500;
  } else if (cfg == "C1") {
    p.numRacks = 20;
    p.numBrokers = 1000;
    p.numReplicas = 99999;
    goals = {CCMI_GOAL_REPLICA_DISTRIBUTION, CCMI_GOAL_DISK_USAGE_DISTRIBUTION, CCMI_GOAL_NW_IN_USAGE_DISTRIBUTION,
             CCMI_GOAL_NW_OUT_USAGE_DISTRIBUTION, CCMI_GOAL_CPU_USAGE_DISTRIBUTION};
  } else if (cfg == "C2") {
    p.numRacks = 100;
    p.numBrokers = 10000;
    p.numReplicas = 999999;
    p.numTopics = 10000;
    goals = {CCMI_GOAL_REPLICA_DISTRIBUTION, CCMI_GOAL_DISK_USAGE_DISTRIBUTION, CCMI_GOAL_NW_IN_USAGE_DISTRIBUTION,
             CCMI_GOAL_NW_OUT_USAGE_DISTRIBUTION, CCMI_GOAL_CPU_USAGE_DISTRIBUTION};
  } else {
    std::fprintf(stderr, "usage: oracle_cc C0|C1|C2 [goal kinds]\n");
    return 2;
  }
  if (argc > 2) {
    goals.clear();
    for (int i = 2; i < argc; ++i) goals.push_back(std::atoi(argv[i]));
  }
  ClusterModel cm;
  auto t0 = std::chrono::steady_clock::now();
  randomCluster(cm, p);
  double gen = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  std::printf("generated %s: B=%zu T=%zu P=%zu R=%zu in %.2fs\n", cfg.c_str(), cm.brokers.size(), cm.topicNames.size(),
              cm.partitions.size(), cm.replicas.size(), gen);
  OptimizationOptions o;
  OptimizerResult res = optimizations(cm, goals, bc, o);
  for (auto& g : res.goals)
    std::printf("  %-40s succeeded=%d diff=%d %8.3fs candidates=%lld actions=%lld repStd=%.6f\n", g.name.c_str(),
                g.succeeded, g.hasDiff, g.seconds, (long long)g.candidates, (long long)g.actions, g.stats.repStd);
  std::printf("total %.3fs candidates=%lld actions=%zu proposals=%zu\n", res.seconds, (long long)res.candidates,
              cm.actionLog.size(), res.proposals.size());
  return 0;
}
