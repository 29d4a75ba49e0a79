// ORACLE — test infrastructure only (see jsem.h header).
// Restatement of the reference fixture generator RandomCluster.generate/populate/markBrokenBrokers
// (cruise-control/src/test/java/.../model/RandomCluster.java:53-455), seeds from
// TestConstants.java:19-26, capacities from src/test/resources/DefaultCapacityConfig.json.
#pragma once
#include "model.h"

namespace oracle {

struct ClusterProperties {
  int numRacks = 10;
  int numBrokers = 40;
  int numDeadBrokers = 0;
  int numBrokersWithBadDisk = 0;
  int numReplicas = 50001;
  int numTopics = 3000;
  int minReplication = 3;
  int maxReplication = 3;
  double meanCpu = 0.01;
  double meanDisk = 100.0;
  double meanNwIn = 100.0;
  double meanNwOut = 100.0;
  int distribution = 0;  // 0 UNIFORM, 1 LINEAR, 2 EXPONENTIAL
  bool rackAware = false;
  bool leaderInFirstPosition = true;
  // POPULATE_REPLICA_PLACEMENT_INFO (ccmi_random_cluster_props.jbod): 1 = testCapacityConfigJBOD.json,
  // 2 = numLogdirs logdirs "/mnt/data-<i>" with logdirCapacity[] on every broker
  int jbod = 0;
  int numLogdirs = 0;
  double logdirCapacity[8] = {0, 0, 0, 0, 0, 0, 0, 0};
};

// generate() + populate(); returns a fully loaded model (W = 1).
void randomCluster(ClusterModel& cm, const ClusterProperties& p);

}  // namespace oracle
