// ORACLE — test infrastructure only (see jsem.h header).
// ClusterModelStats.populate restatement: cruise-control/src/main/java/.../model/ClusterModelStats.java:84-511
// plus the BalancingConstraint analyzer knobs it reads (analyzer/BalancingConstraint.java:54-105,
// defaults config/constants/AnalyzerConfig.java:58-464).
#pragma once
#include <map>
#include <string>
#include <vector>
#include "model.h"

namespace oracle {

struct BalancingConstraint {
  double resourceBalancePercentage[NUM_RESOURCES] = {1.10, 1.10, 1.10, 1.10};
  double capacityThreshold[NUM_RESOURCES] = {0.7, 0.8, 0.8, 0.8};  // CPU, NW_IN, NW_OUT, DISK
  double lowUtilizationThreshold[NUM_RESOURCES] = {0.0, 0.0, 0.0, 0.0};
  double replicaBalancePercentage = 1.10;
  double leaderReplicaBalancePercentage = 1.10;
  double topicReplicaBalancePercentage = 3.00;
  int topicReplicaBalanceMinGap = 2;
  int topicReplicaBalanceMaxGap = 40;
  double goalViolationDistributionThresholdMultiplier = 1.0;
  int64_t maxReplicasPerBroker = 10000;
  int64_t overprovisionedMaxReplicasPerBroker = 1500;
  int overprovisionedMinBrokers = 3;
  int overprovisionedMinExtraRacks = 2;  // AnalyzerConfig.DEFAULT_OVERPROVISIONED_MIN_EXTRA_RACKS
  // BrokerSetAwareGoal: brokerSetResolver() data (BrokerSetFileResolver: broker set id -> broker ids) and
  // replicaToBrokerSetMappingPolicy() (0 TopicNameHash, 1 ReplicaToOriginal)
  std::map<std::string, std::vector<int>> brokerSets;
  int brokerSetPolicy = 0;
  // topics.with.min.leaders.per.broker as the topics it matches (topic indices), min.topic.leaders.per.broker
  // (BalancingConstraint.java:92-93, AnalyzerConfig.java:401-414)
  std::vector<int> minLeaderTopics;
  int minTopicLeadersPerBroker = 1;
  // TopicLeaderReplicaDistributionGoal (BalancingConstraint.java:85-88, AnalyzerConfig.java:112-146)
  double topicLeaderReplicaBalancePercentage = 1.10;
  int topicLeaderReplicaBalanceMinGap = 2;
  int topicLeaderReplicaBalanceMaxGap = 10;
  double topicLeaderReplicaDistributionGoalBalanceMargin = 0.9;
};

struct ClusterModelStats {
  double resAvg[NUM_RESOURCES], resMax[NUM_RESOURCES], resMin[NUM_RESOURCES], resStd[NUM_RESOURCES];
  int numBalancedBrokersByResource[NUM_RESOURCES];
  double pnwAvg, pnwMax, pnwMin, pnwStd;
  int numBrokersUnderPotentialNwOut;
  double repAvg, repStd;
  int repMax, repMin;
  double leadAvg, leadStd;
  int leadMax, leadMin;
  double topicAvg, topicStd;
  int topicMax, topicMin;
  int numBrokers, numReplicasInCluster, numPartitionsWithOfflineReplicas, numTopics;
  int numUnbalancedDisks;
  double diskUtilizationStDev;
};

// GoalUtils.computeResourceUtilizationBalanceThreshold (GoalUtils.java:550-602)
double computeResourceUtilizationBalanceThreshold(double avgUtilizationPercentage, int resource,
                                                  const BalancingConstraint& bc, bool triggeredByGoalViolation,
                                                  double balanceMargin, bool isLowerThreshold);

ClusterModelStats computeStats(const ClusterModel& cm, const BalancingConstraint& bc, const OptimizationOptions& o);

}  // namespace oracle
