// Owner of the arrays behind a generated ccmi_cluster_desc (ccmi_random_cluster / ccmi_cluster_buffers_free).
#pragma once
#include <string>
#include <vector>

#include "ccmi.h"

struct ccmi_cluster_buffers {
  ccmi_cluster_desc desc;
  std::vector<int32_t> brokerId, brokerRack, brokerState;
  std::vector<double> brokerCap;
  std::vector<std::string> topicStr;
  std::vector<const char*> topicPtr;
  std::vector<int32_t> partTopic, partNumber, partOff, partReplicas;
  std::vector<int32_t> repPart, repBroker;
  std::vector<uint8_t> repLeader, repOffline;
  std::vector<float> repLoad;
  // JBOD placement
  std::vector<int32_t> diskBroker, diskAssignReplica, diskAssignDisk;
  std::vector<std::string> diskStr;
  std::vector<const char*> diskPtr;
  std::vector<double> diskCap;
};
