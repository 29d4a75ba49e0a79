// ORACLE — test infrastructure only (see jsem.h header).
// Goal plugin restatement:
//   Goal interface          analyzer/goals/Goal.java:39-164
//   AbstractGoal            analyzer/goals/AbstractGoal.java:81-430
//   GoalUtils               analyzer/goals/GoalUtils.java:122-602
//   AnalyzerUtils.isProposalAcceptableForOptimizedGoals  analyzer/AnalyzerUtils.java:169-179
//   ReplicaDistributionAbstractGoal / ReplicaDistributionGoal
//                           analyzer/goals/ReplicaDistributionAbstractGoal.java, ReplicaDistributionGoal.java
//   ResourceDistributionGoal (+ Cpu/Disk/NetworkInbound/NetworkOutbound UsageDistributionGoal)
//                           analyzer/goals/ResourceDistributionGoal.java:55-1078
// Wall-clock fast-mode timeouts are treated as infinite (parity mode).
#pragma once
#include <functional>
#include <map>
#include <set>
#include <stdexcept>
#include <string>
#include <vector>

#include "model.h"
#include "stats.h"

namespace oracle {

// analyzer/ProvisionStatus.java, ProvisionRecommendation.java (-1 = unset, DEFAULT_OPTIONAL_INT / _DOUBLE),
// ProvisionResponse.java (one goal's response: its status and, for UNDER/OVER, its own recommendation or none)
enum ProvisionStatus { PROV_UNDECIDED = 0, PROV_RIGHT_SIZED = 1, PROV_UNDER = 2, PROV_OVER = 3 };
struct ProvisionRec {
  int status = PROV_UNDER;
  int numBrokers = -1, numRacks = -1, numDisks = -1, numPartitions = -1, typicalBrokerId = -1, resource = -1;
  double typicalBrokerCapacity = -1.0, totalCapacity = -1.0;
};
inline ProvisionRec underBrokers(int n, int resource = -1) {
  ProvisionRec r;
  r.numBrokers = n;
  r.resource = resource;
  return r;
}
struct ProvisionResp {
  int status = PROV_UNDECIDED;
  bool hasRec = false;
  ProvisionRec rec;
};

// OptimizationFailureException with its (optional) ProvisionRecommendation
struct OptimizationFailure : std::runtime_error {
  explicit OptimizationFailure(const std::string& m) : std::runtime_error(m) {}
  OptimizationFailure(const std::string& m, const ProvisionRec& r) : std::runtime_error(m), hasRec(true), rec(r) {}
  bool hasRec = false;
  ProvisionRec rec;
};
// java.lang.UnsupportedOperationException thrown inside the reference's goal code
struct UnsupportedOperation : std::runtime_error {
  using std::runtime_error::runtime_error;
};

class Goal;
using GoalList = std::vector<Goal*>;

class Goal {
 public:
  virtual ~Goal() = default;
  virtual std::string name() const = 0;
  virtual bool isHardGoal() const = 0;
  virtual bool optimize(ClusterModel& cm, const GoalList& optimizedGoals, const OptimizationOptions& o) = 0;
  virtual Acceptance actionAcceptance(const BalancingAction& a, ClusterModel& cm) = 0;
  // ClusterModelStatsComparator.compare(after, before): < 0 means "before" is preferred.
  virtual int compareStats(const ClusterModelStats& s1, const ClusterModelStats& s2) const = 0;
  // Goal.provisionResponse (Goal.java:155-164)
  const ProvisionResp& provision() const { return provision_; }

 protected:
  ProvisionResp provision_;
};

class AbstractGoal : public Goal {
 public:
  explicit AbstractGoal(const BalancingConstraint& bc) : bc_(bc) {}
  bool optimize(ClusterModel& cm, const GoalList& optimizedGoals, const OptimizationOptions& o) override;
  bool optimizeImpl(ClusterModel& cm, const GoalList& optimizedGoals, const OptimizationOptions& o);

 protected:
  virtual void initGoalState(ClusterModel& cm, const OptimizationOptions& o) = 0;
  virtual void updateGoalState(ClusterModel& cm, const OptimizationOptions& o) = 0;
  virtual void rebalanceForBroker(int broker, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o) = 0;
  virtual bool selfSatisfied(ClusterModel& cm, const BalancingAction& a) = 0;
  virtual std::vector<int> brokersToBalance(ClusterModel& cm);

  int maybeApplyBalancingAction(ClusterModel& cm, int replica, const std::vector<int>& candidates, ActionType action,
                                const GoalList& g, const OptimizationOptions& o);
  // candidates: in-order snapshot of the candidate broker's tracked sorted set (live view at call time)
  int maybeApplySwapAction(ClusterModel& cm, int srcReplica, const std::vector<int>& candidateReplicas,
                           const GoalList& g, const OptimizationOptions& o);
  // AbstractGoal.maybeMoveReplicaBetweenDisks / maybeSwapReplicaBetweenDisks (AbstractGoal.java:351-430)
  int maybeMoveReplicaBetweenDisks(ClusterModel& cm, int replica, const std::vector<int>& candidateDisks,
                                   const GoalList& g);
  int maybeSwapReplicaBetweenDisks(ClusterModel& cm, int srcReplica, const std::vector<int>& candidateReplicas,
                                   const GoalList& g);
  std::string replicaSortName(bool reverse, bool leaderOnly) const {
    return name() + (reverse ? "-REVERSE" : "") + (leaderOnly ? "-LEADER" : "");
  }

  BalancingConstraint bc_;
  bool finished_ = false;
  bool succeeded_ = true;
};

// GoalUtils helpers
ProvisionResp validateProvisionResponse(const ProvisionResp& p, ClusterModel& cm, int overprovisionedMinBrokers);
std::vector<int> eligibleBrokers(ClusterModel& cm, int replica, const std::vector<int>& candidates, ActionType a,
                                 const OptimizationOptions& o);
bool legitMove(ClusterModel& cm, int replica, int destBroker, ActionType a);
Acceptance isProposalAcceptableForOptimizedGoals(const GoalList& g, const BalancingAction& a, ClusterModel& cm);
void ensureNoOfflineReplicas(ClusterModel& cm, const std::string& goal);
void ensureReplicasMoveOffBrokersWithBadDisks(ClusterModel& cm, const std::string& goal);
std::vector<int> javaHashSetOrderIntKeys(const std::vector<int>& insertionOrder);

class ReplicaDistributionGoal : public AbstractGoal {
 public:
  using AbstractGoal::AbstractGoal;
  std::string name() const override { return "ReplicaDistributionGoal"; }
  bool isHardGoal() const override { return false; }
  Acceptance actionAcceptance(const BalancingAction& a, ClusterModel& cm) override;
  int compareStats(const ClusterModelStats& s1, const ClusterModelStats& s2) const override;

  int balanceUpperLimit() const { return upper_; }
  int balanceLowerLimit() const { return lower_; }

 protected:
  void initGoalState(ClusterModel& cm, const OptimizationOptions& o) override;
  void updateGoalState(ClusterModel& cm, const OptimizationOptions& o) override;
  void rebalanceForBroker(int broker, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o) override;
  bool selfSatisfied(ClusterModel& cm, const BalancingAction& a) override;

 private:
  bool rebalanceByMovingReplicasOut(int broker, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o);
  bool rebalanceByMovingReplicasIn(int broker, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o);
  bool isExcludedForReplicaMove(const ClusterModel& cm, int b) const { return !allowed_[b]; }
  bool underUpperAfter(const ClusterModel& cm, int b, int count, bool add) const;
  bool aboveLowerAfter(const ClusterModel& cm, int b, int count, bool add) const;

  bool fixOfflineReplicasOnly_ = false;
  std::set<int> aboveUpper_, underLower_;
  double avgReplicasOnAliveBroker_ = 0;
  int upper_ = 0, lower_ = 0;
  std::vector<char> allowed_;
  int numAllowed_ = 0;
};

class ResourceDistributionGoal : public AbstractGoal {
 public:
  ResourceDistributionGoal(const BalancingConstraint& bc, int resource) : AbstractGoal(bc), resource_(resource) {}
  std::string name() const override;
  bool isHardGoal() const override { return false; }
  Acceptance actionAcceptance(const BalancingAction& a, ClusterModel& cm) override;
  int compareStats(const ClusterModelStats& s1, const ClusterModelStats& s2) const override;
  double balanceUpperThreshold() const { return upperThr_; }
  double balanceLowerThreshold() const { return lowerThr_; }

 protected:
  void initGoalState(ClusterModel& cm, const OptimizationOptions& o) override;
  void updateGoalState(ClusterModel& cm, const OptimizationOptions& o) override;
  void rebalanceForBroker(int broker, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o) override;
  bool selfSatisfied(ClusterModel& cm, const BalancingAction& a) override;
  std::vector<int> brokersToBalance(ClusterModel& cm) override;

 private:
  Acceptance baseAcceptance(const BalancingAction& a, ClusterModel& cm);
  bool rebalanceByMovingLoadOut(int broker, ClusterModel& cm, const GoalList& g, ActionType at,
                                const OptimizationOptions& o);
  bool rebalanceByMovingLoadIn(int broker, ClusterModel& cm, const GoalList& g, ActionType at,
                               const OptimizationOptions& o, bool moveImmigrantsOnly);
  bool rebalanceBySwappingLoadOut(int broker, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o,
                                  bool moveImmigrantsOnly);
  bool rebalanceBySwappingLoadIn(int broker, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o,
                                 bool moveImmigrantsOnly);
  std::string sortedCandidateReplicas(int broker, ClusterModel& cm, const OptimizationOptions& o, double loadLimit,
                                      bool isAscending, bool followersOnly, bool leadersOnly, bool immigrantsOnly);
  double getMaxReplicaLoad(ClusterModel& cm, const std::vector<int>& sorted) const;
  double getMinReplicaLoad(ClusterModel& cm, const std::vector<int>& sorted) const;

  bool isExcludedForReplicaMove(int b) const { return !allowed_[b]; }
  bool aboveLowerLimit(ClusterModel& cm, int b) { return aboveLowerAfterChange(cm, -1, b, true); }
  bool underUpperLimit(ClusterModel& cm, int b) { return underUpperAfterChange(cm, -1, b, false, upperThr_); }
  bool aboveLowerAfterChange(ClusterModel& cm, int replicaLoadOf, int b, bool add);
  bool underUpperAfterChange(ClusterModel& cm, int replicaLoadOf, int b, bool add, double thr);
  bool underUpperAfterChange(ClusterModel& cm, int replicaLoadOf, int b, bool add) {
    return underUpperAfterChange(cm, replicaLoadOf, b, add, upperThr_);
  }
  bool isAcceptableAfterReplicaMove(ClusterModel& cm, int srcReplica, int destBroker);
  bool isSelfSatisfiedAfterSwap(ClusterModel& cm, int srcReplica, int destReplica);
  bool isGettingMoreBalanced(ClusterModel& cm, int srcBroker, double delta, int destBroker);
  bool isSwapViolatingLimit(ClusterModel& cm, int srcReplica, int destReplica);
  bool isSwapViolatingContainerLimit(ClusterModel& cm, double delta, int srcReplica, int destReplica, bool host);
  int cmpBroker(ClusterModel& cm, int a, int b) const {
    int c = dcompare(cm.utilizationPct(a, resource_), cm.utilizationPct(b, resource_));
    return c != 0 ? c : icompare(cm.brokers[a].id, cm.brokers[b].id);
  }

  int resource_;
  bool fixOfflineReplicasOnly_ = false;
  double upperThr_ = 0, lowerThr_ = 0;
  std::vector<char> allowed_;
  bool isLowUtilization_ = false;
  ProvisionRec overRec_;  // _overProvisionedRecommendation
};

// ===================================================================== remaining default goals
//   RackAwareGoal / AbstractRackAwareGoal  analyzer/goals/RackAwareGoal.java, AbstractRackAwareGoal.java
//   MinTopicLeadersPerBrokerGoal           analyzer/goals/MinTopicLeadersPerBrokerGoal.java (default config:
//                                          no topic matches, so only moveAwayOfflineReplicas acts)
//   ReplicaCapacityGoal                    analyzer/goals/ReplicaCapacityGoal.java
//   CapacityGoal (Disk/NwIn/NwOut/Cpu)     analyzer/goals/CapacityGoal.java
//   PotentialNwOutGoal                     analyzer/goals/PotentialNwOutGoal.java
//   TopicReplicaDistributionGoal           analyzer/goals/TopicReplicaDistributionGoal.java
//   LeaderReplicaDistributionGoal          analyzer/goals/LeaderReplicaDistributionGoal.java (+ ReplicaDistributionAbstractGoal)
//   LeaderBytesInDistributionGoal          analyzer/goals/LeaderBytesInDistributionGoal.java

class RackAwareGoal : public AbstractGoal {
 public:
  using AbstractGoal::AbstractGoal;
  std::string name() const override { return "RackAwareGoal"; }
  bool isHardGoal() const override { return true; }
  Acceptance actionAcceptance(const BalancingAction& a, ClusterModel& cm) override;
  int compareStats(const ClusterModelStats&, const ClusterModelStats&) const override { return 0; }

 protected:
  void initGoalState(ClusterModel& cm, const OptimizationOptions& o) override;
  void updateGoalState(ClusterModel& cm, const OptimizationOptions& o) override;
  void rebalanceForBroker(int broker, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o) override;
  bool selfSatisfied(ClusterModel&, const BalancingAction&) override { return true; }

 private:
  bool violates(ClusterModel& cm, int replica, int destBroker) const;
  bool shouldKeepInTheCurrentBroker(ClusterModel& cm, int replica) const;
  std::vector<int> rackAwareEligibleBrokers(ClusterModel& cm, int replica) const;
};

//   RackAwareDistributionGoal              analyzer/goals/RackAwareDistributionGoal.java (not in default.goals)
class RackAwareDistributionGoal : public AbstractGoal {
 public:
  using AbstractGoal::AbstractGoal;
  std::string name() const override { return "RackAwareDistributionGoal"; }
  bool isHardGoal() const override { return true; }
  Acceptance actionAcceptance(const BalancingAction& a, ClusterModel& cm) override;
  int compareStats(const ClusterModelStats&, const ClusterModelStats&) const override { return 0; }

 protected:
  void initGoalState(ClusterModel& cm, const OptimizationOptions& o) override;
  void updateGoalState(ClusterModel& cm, const OptimizationOptions& o) override;
  void rebalanceForBroker(int broker, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o) override;
  bool selfSatisfied(ClusterModel&, const BalancingAction&) override { return true; }

 private:
  std::map<int, int> numReplicasByRack(const ClusterModel& cm, int p) const;
  bool violates(ClusterModel& cm, int replica, int destBroker) const;
  bool shouldKeepInTheCurrentBroker(ClusterModel& cm, int replica) const;
  std::vector<int> rackAwareEligibleBrokers(ClusterModel& cm, int replica) const;
  int baseLimit(int rf) const { return rf / numRacks_; }
  int numRacksWithOneMoreReplica(int rf) const { return rf % numRacks_; }
  std::vector<char> allowed_;
  int numRacks_ = 0;  // BalanceLimit._numAliveRacksAllowedReplicaMoves
};

//   BrokerSetAwareGoal                     analyzer/goals/BrokerSetAwareGoal.java (not in default.goals), with
//                                          BrokerSetResolutionHelper + NoOpBrokerSetAssignmentPolicy (config/)
class BrokerSetAwareGoal : public AbstractGoal {
 public:
  using AbstractGoal::AbstractGoal;
  std::string name() const override { return "BrokerSetAwareGoal"; }
  bool isHardGoal() const override { return true; }
  Acceptance actionAcceptance(const BalancingAction& a, ClusterModel& cm) override;
  int compareStats(const ClusterModelStats&, const ClusterModelStats&) const override { return 0; }

 protected:
  void initGoalState(ClusterModel& cm, const OptimizationOptions& o) override;
  void updateGoalState(ClusterModel& cm, const OptimizationOptions& o) override;
  void rebalanceForBroker(int broker, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o) override;
  bool selfSatisfied(ClusterModel&, const BalancingAction&) override { return true; }

 private:
  std::string brokerSetId(int brokerId) const;                      // BrokerSetResolutionHelper.brokerSetId
  std::string brokerSetIdForReplica(ClusterModel& cm, int replica);  // ReplicaToBrokerSetMappingPolicy
  bool violates(ClusterModel& cm, int replica, int destBroker);
  std::map<std::string, std::set<int>> brokersByBrokerSet_;  // broker ids
  std::map<int, std::string> brokerSetIdByBrokerId_;
  std::map<std::string, std::string> brokerSetIdByTopic_;    // TopicNameHashBrokerSetMappingPolicy cache
  std::set<int> excludedTopics_, mustHaveTopics_;
};

class MinTopicLeadersPerBrokerGoal : public AbstractGoal {
 public:
  using AbstractGoal::AbstractGoal;
  std::string name() const override { return "MinTopicLeadersPerBrokerGoal"; }
  bool isHardGoal() const override { return false; }
  Acceptance actionAcceptance(const BalancingAction& a, ClusterModel& cm) override;
  int compareStats(const ClusterModelStats&, const ClusterModelStats&) const override { return 0; }

 protected:
  void initGoalState(ClusterModel& cm, const OptimizationOptions& o) override;
  void updateGoalState(ClusterModel& cm, const OptimizationOptions& o) override;
  void rebalanceForBroker(int broker, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o) override;
  bool selfSatisfied(ClusterModel& cm, const BalancingAction& a) override;

 private:
  static bool eligibleToHaveLeaders(const ClusterModel& cm, int b, const OptimizationOptions& o);
  bool leaderRemoveViolates(ClusterModel& cm, int r) const;
  void moveAwayOfflineReplicas(int b, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o);
  void moveLeaderOfTopicToBroker(int t, int b, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o);
  std::vector<int> mustOrder_;   // _mustHaveTopicMinLeadersPerBroker.keySet() in HashMap iteration order
  std::map<int, int> minLeaders_;  // topic -> minimum leaders per eligible broker
};
// iteration order of a HashSet<String> of topic names filled in `insertion` order
std::vector<int> topicHashSetOrder(const ClusterModel& cm, const std::vector<int>& insertion);

// Kafka-assigner mode goals (analyzer/kafkaassigner/; in `goals`, not in default.goals). They implement Goal directly
// (no AbstractGoal template, no acceptance conjunction over optimized goals).
class KafkaAssignerEvenRackAwareGoal : public Goal {
 public:
  explicit KafkaAssignerEvenRackAwareGoal(const BalancingConstraint&) {}
  std::string name() const override { return "KafkaAssignerEvenRackAwareGoal"; }
  bool isHardGoal() const override { return true; }
  bool optimize(ClusterModel& cm, const GoalList& optimizedGoals, const OptimizationOptions& o) override;
  Acceptance actionAcceptance(const BalancingAction& a, ClusterModel& cm) override;
  int compareStats(const ClusterModelStats&, const ClusterModelStats&) const override { return 0; }

 private:
  bool maybeApplyMove(ClusterModel& cm, int p, int position);
  bool violates(const ClusterModel& cm, int replica, int destBroker) const;
  // _aliveBrokerReplicaCountByPosition: per position a TreeSet<BrokerReplicaCount> ordered by (count, id); an entry
  // leaves through its iterator and comes back with the incremented count, so the set stays sorted
  std::vector<std::set<std::pair<int, int>>> byPosition_;  // (replica count, broker id)
};
class KafkaAssignerDiskUsageDistributionGoal : public Goal {
 public:
  explicit KafkaAssignerDiskUsageDistributionGoal(const BalancingConstraint& bc) : bc_(bc) {}
  std::string name() const override { return "KafkaAssignerDiskUsageDistributionGoal"; }
  bool isHardGoal() const override { return true; }
  bool optimize(ClusterModel& cm, const GoalList& optimizedGoals, const OptimizationOptions& o) override;
  Acceptance actionAcceptance(const BalancingAction& a, ClusterModel& cm) override;
  // DiskDistributionGoalStatsComparator (:608-632)
  int compareStats(const ClusterModelStats& s1, const ClusterModelStats& s2) const override {
    return s2.numBalancedBrokersByResource[DISK] > s1.numBalancedBrokersByResource[DISK] ? -1 : 1;
  }

 private:
  BalancingConstraint bc_;
};
// KafkaAssignerUtils.sanityCheckOptimizationOptions (KafkaAssignerUtils.java:20-26)
void kafkaAssignerSanityCheck(const OptimizationOptions& o);

// PreferredLeaderElectionGoal (analyzer/goals/PreferredLeaderElectionGoal.java) with skipUrpDemotion = false,
// excludeFollowerDemotion = false (the no-argument constructor GoalOptimizer uses): demoted brokers, then demoted disks
// (ccmi.h disk_demoted) of the other alive brokers.
class PreferredLeaderElectionGoal : public Goal {
 public:
  explicit PreferredLeaderElectionGoal(const BalancingConstraint&) {}
  std::string name() const override { return "PreferredLeaderElectionGoal"; }
  bool isHardGoal() const override { return false; }
  bool optimize(ClusterModel& cm, const GoalList& optimizedGoals, const OptimizationOptions& o) override;
  Acceptance actionAcceptance(const BalancingAction&, ClusterModel&) override { return Acceptance::ACCEPT; }
  int compareStats(const ClusterModelStats&, const ClusterModelStats&) const override { return 0; }
};

class ReplicaCapacityGoal : public AbstractGoal {
 public:
  using AbstractGoal::AbstractGoal;
  std::string name() const override { return "ReplicaCapacityGoal"; }
  bool isHardGoal() const override { return true; }
  Acceptance actionAcceptance(const BalancingAction& a, ClusterModel& cm) override;
  int compareStats(const ClusterModelStats&, const ClusterModelStats&) const override { return 0; }

 protected:
  void initGoalState(ClusterModel& cm, const OptimizationOptions& o) override;
  void updateGoalState(ClusterModel& cm, const OptimizationOptions& o) override;
  void rebalanceForBroker(int broker, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o) override;
  bool selfSatisfied(ClusterModel& cm, const BalancingAction& a) override;

 private:
  bool selfHealingMode_ = false;
};

class CapacityGoal : public AbstractGoal {
 public:
  CapacityGoal(const BalancingConstraint& bc, int resource) : AbstractGoal(bc), resource_(resource) {}
  std::string name() const override;
  bool isHardGoal() const override { return true; }
  Acceptance actionAcceptance(const BalancingAction& a, ClusterModel& cm) override;
  int compareStats(const ClusterModelStats&, const ClusterModelStats&) const override { return 0; }

 protected:
  void initGoalState(ClusterModel& cm, const OptimizationOptions& o) override;
  void updateGoalState(ClusterModel& cm, const OptimizationOptions& o) override;
  void rebalanceForBroker(int broker, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o) override;
  bool selfSatisfied(ClusterModel& cm, const BalancingAction& a) override;

 private:
  bool utilizationOverLimit(ClusterModel& cm, int b, double brokerLimit, double hostLimit) const;
  bool underLimitAfterAdding(ClusterModel& cm, int b, double util) const;
  bool movementAcceptable(ClusterModel& cm, int srcReplica, int destBroker) const;
  bool swapAcceptable(ClusterModel& cm, int srcReplica, int destReplica) const;
  int resource_;
};

class PotentialNwOutGoal : public AbstractGoal {
 public:
  using AbstractGoal::AbstractGoal;
  std::string name() const override { return "PotentialNwOutGoal"; }
  bool isHardGoal() const override { return false; }
  Acceptance actionAcceptance(const BalancingAction& a, ClusterModel& cm) override;
  int compareStats(const ClusterModelStats& s1, const ClusterModelStats& s2) const override {
    return icompare(s1.numBrokersUnderPotentialNwOut, s2.numBrokersUnderPotentialNwOut);
  }

 protected:
  void initGoalState(ClusterModel& cm, const OptimizationOptions& o) override;
  void updateGoalState(ClusterModel& cm, const OptimizationOptions& o) override;
  void rebalanceForBroker(int broker, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o) override;
  bool selfSatisfied(ClusterModel& cm, const BalancingAction& a) override;
  std::vector<int> brokersToBalance(ClusterModel& cm) override;

 private:
  double leaderNwOutOf(ClusterModel& cm, int partition) const {
    return cm.replicaUtil(cm.partitions[partition].leader, NW_OUT);
  }
  bool fixOfflineReplicasOnly_ = false;
};

class TopicReplicaDistributionGoal : public AbstractGoal {
 public:
  using AbstractGoal::AbstractGoal;
  std::string name() const override { return "TopicReplicaDistributionGoal"; }
  bool isHardGoal() const override { return false; }
  Acceptance actionAcceptance(const BalancingAction& a, ClusterModel& cm) override;
  int compareStats(const ClusterModelStats& s1, const ClusterModelStats& s2) const override;
  int upperLimit(int topic) const { return upper_[topic]; }
  int lowerLimit(int topic) const { return lower_[topic]; }

 protected:
  void initGoalState(ClusterModel& cm, const OptimizationOptions& o) override;
  void updateGoalState(ClusterModel& cm, const OptimizationOptions& o) override;
  void rebalanceForBroker(int broker, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o) override;
  bool selfSatisfied(ClusterModel& cm, const BalancingAction& a) override;

 private:
  int count(const ClusterModel& cm, int b, int topic) const {
    auto it = cm.brokers[b].topicReplicaCount.find(topic);
    return it == cm.brokers[b].topicReplicaCount.end() ? 0 : it->second;
  }
  bool underUpperAfter(const ClusterModel& cm, int topic, int b, bool add) const;
  bool aboveLowerAfter(const ClusterModel& cm, int topic, int b, bool add) const;
  std::vector<int> replicasToMoveOut(ClusterModel& cm, int b, int topic);
  bool moveOut(int b, int topic, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o);
  bool moveIn(int b, int topic, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o);
  bool isExcluded(int b) const { return !allowed_[b]; }
  bool fixOfflineReplicasOnly_ = false;
  std::vector<int> upper_, lower_;
  std::vector<char> rebalanceTopic_;
  std::vector<char> allowed_;
  bool anyAbove_ = false, anyUnder_ = false;
};

//   TopicLeaderReplicaDistributionGoal     analyzer/goals/TopicLeaderReplicaDistributionGoal.java (in `goals`, not in
//                                          default.goals)
class TopicLeaderReplicaDistributionGoal : public AbstractGoal {
 public:
  using AbstractGoal::AbstractGoal;
  std::string name() const override { return "TopicLeaderReplicaDistributionGoal"; }
  bool isHardGoal() const override { return false; }
  Acceptance actionAcceptance(const BalancingAction& a, ClusterModel& cm) override;
  // GoalUtils.HardGoalStatsComparator (TopicLeaderReplicaDistributionGoal.java:269-272)
  int compareStats(const ClusterModelStats&, const ClusterModelStats&) const override { return 0; }
  int upperLimit(int topic) const { return upper_[topic]; }
  int lowerLimit(int topic) const { return lower_[topic]; }

 protected:
  void initGoalState(ClusterModel& cm, const OptimizationOptions& o) override;
  void updateGoalState(ClusterModel& cm, const OptimizationOptions& o) override;
  void rebalanceForBroker(int broker, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o) override;
  bool selfSatisfied(ClusterModel& cm, const BalancingAction& a) override;

 private:
  bool satisfiable(const ClusterModel& cm, int topic, int src, int dst) const;
  std::vector<int> leadersOf(const ClusterModel& cm, int b, int topic) const;
  std::vector<int> replicasToMoveOut(ClusterModel& cm, int b, int topic);
  bool moveOut(int b, int topic, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o);
  bool moveIn(int b, int topic, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o);
  bool isExcluded(int b) const { return !allowed_[b]; }
  bool fixOfflineReplicasOnly_ = false;
  std::vector<int> upper_, lower_;
  std::vector<char> rebalanceTopic_;
  std::vector<char> allowed_;
  bool anyAbove_ = false, anyUnder_ = false;
};

class LeaderReplicaDistributionGoal : public AbstractGoal {
 public:
  using AbstractGoal::AbstractGoal;
  std::string name() const override { return "LeaderReplicaDistributionGoal"; }
  bool isHardGoal() const override { return false; }
  Acceptance actionAcceptance(const BalancingAction& a, ClusterModel& cm) override;
  int compareStats(const ClusterModelStats& s1, const ClusterModelStats& s2) const override;
  int balanceUpperLimit() const { return upper_; }
  int balanceLowerLimit() const { return lower_; }

 protected:
  void initGoalState(ClusterModel& cm, const OptimizationOptions& o) override;
  void updateGoalState(ClusterModel& cm, const OptimizationOptions& o) override;
  void rebalanceForBroker(int broker, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o) override;
  bool selfSatisfied(ClusterModel& cm, const BalancingAction& a) override;

 private:
  Acceptance leaderMovementSatisfiable(ClusterModel& cm, int src, int dst) const;
  bool moveLeadershipOut(int b, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o);
  bool moveLeadershipIn(int b, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o);
  bool moveReplicasOut(int b, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o);
  bool moveLeaderReplicasIn(int b, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o);
  bool isExcluded(int b) const { return !allowed_[b]; }
  bool fixOfflineReplicasOnly_ = false;
  int upper_ = 0, lower_ = 0;
  std::vector<char> allowed_;
  bool anyAbove_ = false, anyUnder_ = false;
};

class LeaderBytesInDistributionGoal : public AbstractGoal {
 public:
  using AbstractGoal::AbstractGoal;
  std::string name() const override { return "LeaderBytesInDistributionGoal"; }
  bool isHardGoal() const override { return false; }
  Acceptance actionAcceptance(const BalancingAction& a, ClusterModel& cm) override;
  int compareStats(const ClusterModelStats& s1, const ClusterModelStats& s2) const override;
  double meanLeaderBytesIn() const { return mean_; }

 protected:
  void initGoalState(ClusterModel& cm, const OptimizationOptions& o) override;
  void updateGoalState(ClusterModel& cm, const OptimizationOptions& o) override;
  void rebalanceForBroker(int broker, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o) override;
  bool selfSatisfied(ClusterModel& cm, const BalancingAction& a) override;
  std::vector<int> brokersToBalance(ClusterModel& cm) override;

 private:
  void initMean(ClusterModel& cm);
  double threshold(ClusterModel& cm, int b);
  double mean_ = 0.0;
  int numAllowed_ = 0;
  bool overLimit_ = false;
};

// ===================================================================== intra-broker (JBOD) goals
//   IntraBrokerDiskCapacityGoal             analyzer/goals/IntraBrokerDiskCapacityGoal.java:40-291
//   IntraBrokerDiskUsageDistributionGoal    analyzer/goals/IntraBrokerDiskUsageDistributionGoal.java:50-543
//   GoalUtils.legitMoveBetweenDisks         analyzer/goals/GoalUtils.java:237-244
// The per-disk swap timeout (PER_DISK_SWAP_TIMEOUT_MS, 500 ms) is treated as infinite like the fast-mode timeouts.

class IntraBrokerDiskCapacityGoal : public AbstractGoal {
 public:
  using AbstractGoal::AbstractGoal;
  std::string name() const override { return "IntraBrokerDiskCapacityGoal"; }
  bool isHardGoal() const override { return true; }
  Acceptance actionAcceptance(const BalancingAction& a, ClusterModel& cm) override;
  int compareStats(const ClusterModelStats&, const ClusterModelStats&) const override { return 0; }

 protected:
  void initGoalState(ClusterModel& cm, const OptimizationOptions& o) override;
  void updateGoalState(ClusterModel& cm, const OptimizationOptions& o) override;
  void rebalanceForBroker(int broker, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o) override;
  bool selfSatisfied(ClusterModel& cm, const BalancingAction& a) override;
  std::vector<int> brokersToBalance(ClusterModel& cm) override { return cm.aliveBrokers(); }

 private:
  bool overLimit(const ClusterModel& cm, int d) const;
  bool underLimitAfterAdding(const ClusterModel& cm, int d, double util) const;
};

class IntraBrokerDiskUsageDistributionGoal : public AbstractGoal {
 public:
  using AbstractGoal::AbstractGoal;
  std::string name() const override { return "IntraBrokerDiskUsageDistributionGoal"; }
  bool isHardGoal() const override { return false; }
  Acceptance actionAcceptance(const BalancingAction& a, ClusterModel& cm) override;
  int compareStats(const ClusterModelStats& s1, const ClusterModelStats& s2) const override;
  double upperThreshold(int b) const { return upper_[b]; }
  double lowerThreshold(int b) const { return lower_[b]; }

 protected:
  void initGoalState(ClusterModel& cm, const OptimizationOptions& o) override;
  void updateGoalState(ClusterModel& cm, const OptimizationOptions& o) override;
  void rebalanceForBroker(int broker, ClusterModel& cm, const GoalList& g, const OptimizationOptions& o) override;
  bool selfSatisfied(ClusterModel& cm, const BalancingAction& a) override;
  std::vector<int> brokersToBalance(ClusterModel& cm) override { return cm.aliveBrokers(); }

 private:
  double sourceUtilizationDelta(const BalancingAction& a, ClusterModel& cm) const;
  bool isChangeViolatingLimit(const ClusterModel& cm, double delta, int srcDisk, int dstDisk) const;
  bool isGettingMoreBalanced(const ClusterModel& cm, int srcDisk, int dstDisk, double delta) const;
  bool moveLoadIn(int disk, ClusterModel& cm, const GoalList& g);
  bool moveLoadOut(int disk, ClusterModel& cm, const GoalList& g);
  void swapLoadOut(int disk, ClusterModel& cm, const GoalList& g);
  void swapLoadIn(int disk, ClusterModel& cm, const GoalList& g);
  std::vector<double> upper_, lower_;  // _balanceUpperThresholdByBroker / _balanceLowerThresholdByBroker
};

}  // namespace oracle
