// Engine: the session-level goal optimizer. Goal drivers keep the reference's sequential control flow
// on the host (they decide WHICH candidate lists are scanned and in what order, with the JDK collection
// semantics the decisions depend on); every candidate-predicate evaluation runs on the device as a
// batched first-fit scan, speculating over whole replica lists, popped candidate brokers and source-
// replica x candidate-replica swap grids. After a winning (replica, destination) the host applies the
// move to its model, marks the touched rows dirty, and resumes the reference loop right after the winner.
//
// Reference control flow restated here:
//   GoalOptimizer.optimizations               analyzer/GoalOptimizer.java:435-524
//   AbstractGoal.optimize                     analyzer/goals/AbstractGoal.java:81-135
//   ReplicaDistributionGoal                   analyzer/goals/ReplicaDistributionGoal.java:151-340
//   ReplicaDistributionAbstractGoal           analyzer/goals/ReplicaDistributionAbstractGoal.java:79-229
//   ResourceDistributionGoal                  analyzer/goals/ResourceDistributionGoal.java:234-863
#pragma once
#include <chrono>
#include <memory>
#include <string>
#include <vector>

#include "snapseg.h"
#include "brokersets.h"
#include "ccmi.h"
#include "devtypes.h"
#include "errors.h"
#include "model.h"

namespace ccmi {

class Device;

struct Options {  // OptimizationOptions
  std::vector<uint8_t> exclMove, exclLead, requested;  // [B] flags
  std::vector<uint8_t> exclTopic;                      // [T] excludedTopics (intra-broker goals)
  bool anyExclMove = false, anyExclLead = false, anyRequested = false, anyExclTopic = false;
  bool triggered = false, onlyImmigrants = false;
};

struct Constraint {  // BalancingConstraint
  double resBalance[4], capThreshold[4], lowUtil[4];
  double replicaBalance, goalViolationMultiplier;
  double leaderReplicaBalance, topicReplicaBalance;
  int32_t topicMinGap, topicMaxGap;
  // TopicLeaderReplicaDistributionGoal: topic.leader.replica.count.balance.{threshold,min.gap,max.gap} and
  // topic.leader.replica.distribution.goal.balance.margin
  double topicLeaderBalance = 1.10, topicLeaderMargin = 0.9;
  int32_t topicLeaderMinGap = 2, topicLeaderMaxGap = 10;
  int64_t maxReplicasPerBroker;
  int64_t overMaxReplicasPerBroker;   // overprovisioned.max.replicas.per.broker
  int32_t overMinBrokers;             // overprovisioned.min.brokers
  int32_t overprovisionedMinExtraRacks;
  // topics.with.min.leaders.per.broker as the matched topic indices (ascending) and min.topic.leaders.per.broker
  std::vector<int32_t> minLeaderTopics;
  int32_t minTopicLeadersPerBroker = 1;
};

class Engine;

// Puts of a speculative candidate-tree build per poll of an in-flight scan (Device::idleWork; CCMI_IDLE_TREE_PUTS,
// 0 = off). Read per call.
size_t idleTreePutsPerPoll();

// Destination-sharded scans: every shard runs the same host drivers on an identical replica of
// the model and scans only its slice of each candidate list; `combine` MIN-reduces the shards' first-fit keys
// (keys are global list positions, so the minimum is the reference's first accepted candidate).
struct Shard {
  int rank = 0, count = 1;
  ccmi_allreduce_min_fn fn = nullptr;
  void* ctx = nullptr;
};

class GoalImpl {
 public:
  virtual ~GoalImpl() = default;
  int kind = 0;
  std::string name;
  DevGoal dg{};  // frozen acceptance state
  std::vector<uint8_t> allowed;
  bool succeeded = true;
  bool finished = false;
  ccmi_provision_response prov{};  // Goal.provisionResponse
  // crossScan's first-row probe (Engine::crossScan): recent share of scans won within the probe's columns
  double probeHitRate = 0.0;
  // Goal.actionAcceptance throws IllegalStateException (KafkaAssignerDiskUsageDistributionGoal): as an optimized goal
  // it ends the optimization at the first candidate that reaches it (Engine::program stops the conjunction there)
  bool terminal = false;
  bool abstractGoal = true;  // extends AbstractGoal (its optimize turns an OptimizationFailureException into UNDER)
  virtual void init(Engine& e) = 0;
  virtual void rebalance(Engine& e, int b) = 0;
  virtual void update(Engine& e) = 0;
  virtual std::vector<int> brokersToBalance(Engine& e);
  // One device chain for the whole broker loop of a round (returns false when the goal has none, or chains are off)
  virtual bool rebalanceAll(Engine&) { return false; }
  virtual int compareStats(const ccmi_cluster_stats& after, const ccmi_cluster_stats& before) const = 0;
};

class Engine {
 public:
  Engine(Model& m, Device* dev) : m(m), dev(dev) {}
  Model& m;
  Device* dev;
  Options opt;
  Constraint bc{};
  Shard shard;
  // The goals this session has optimized, one per goal kind (GoalOptimizer holds one instance per goal class, so a
  // re-optimized kind replaces its older entry), in the order each was last optimized. A goal's frozen acceptance
  // state (DevGoal, allowed-broker slot) lives here for as long as it may appear in a later optimizedGoals set.
  std::vector<std::unique_ptr<GoalImpl>> optimized;
  // Goal.optimize's optimizedGoals (Goal.java:60-68) for the running optimization: entries of `optimized`, in its
  // order (AnalyzerUtils.isProposalAcceptableForOptimizedGoals, AnalyzerUtils.java:169-179). Only these goals'
  // actionAcceptance joins the candidate conjunction.
  std::vector<GoalImpl*> priors;
  int64_t candidates = 0;
  ccmi_provision_response lastFailure{};  // provisionResponse of the goal whose OptimizationFailure ended the last call
  std::vector<uint8_t> scratchB, scratchB2;  // per-broker scratch flags for the goal drivers
  std::vector<int32_t> topicUpper, topicLower;  // TopicReplicaDistributionGoal limits (device copy: setTopicLimits)
  BrokerSets brokerSets;                        // BalancingConstraint broker sets of the current call
  std::vector<int32_t> brokerSetOf, replicaSetOf;  // BrokerSetAwareGoal state (device copy: setBrokerSets)
  std::vector<int32_t> minLeadOf;  // MinTopicLeadersPerBrokerGoal's minimum per topic, -1 = not its topic (setMinLeaders)
  std::vector<int32_t> topicLeadLim;  // TopicLeaderReplicaDistributionGoal (upper, lower) per topic (setTopicLeadLimits)

  // one Goal.optimize(clusterModel, optimizedGoals = priorSet, options); throws OptimizationFailure / StateError.
  // priorSet: entries of `optimized`. On success the goal joins `optimized` (replacing an entry of its kind).
  bool optimizeGoal(std::unique_ptr<GoalImpl> g, const std::vector<GoalImpl*>& priorSet, ccmi_goal_result* res);
  // The entry of `optimized` of a goal kind, or null
  GoalImpl* optimizedOfKind(int kind) const;
  // allowedBits slot of the goal being optimized (set before GoalImpl::init; DevGoal.allowedSlot)
  int newSlot = 0;
  bool optimizeGoalImpl(std::unique_ptr<GoalImpl>& g, ccmi_goal_result* res, std::chrono::steady_clock::time_point t0,
                        int64_t c0, size_t a0, int64_t l0, int64_t p0);
  ccmi_cluster_stats stats();
  int acceptance(int goalIndex, const ccmi_action& a);

  // device scans: return winning index or -1; add reference-equivalent candidate counts
  //   crossScan: rows reps[r0, r1) x cands, key = k * N + j; `count` adds the reference-equivalent candidates
  //   (callers with candidate filters or early exits count themselves)
  int64_t crossScan(GoalImpl& self, int action, const std::vector<int32_t>& reps, size_t r0,
                    const std::vector<int32_t>& cands, int filter = FILTER_NONE, bool count = true,
                    size_t r1 = (size_t)-1);
  // crossScan over the concatenation of snapshot segments (Device::scanSegs: the rows stay device-resident)
  int64_t crossScanSegs(GoalImpl& self, int action, const std::vector<SnapSeg>& segs,
                        const std::vector<int32_t>& cands);
  // Queue scans (Device::scanQueue): the rows of every broker of [head (if >= 0)] ++ tail[0, nTail) (poll order; entry 0
  // from row skip0) x cands in
  // ONE device command, each broker's rows its snapshot under `spec` from the device-resident snapshot directory.
  // Returns the key (Device::scanQueue) or -1 and adds the reference-equivalent candidates. queueOn: the path applies
  // (one shard, a usable server, no replica-dependent candidate filters; CCMI_QUEUE_SCAN=0 turns it off).
  bool queueOn(const GoalImpl& self, int action) const;
  // queueOn, and the snapshot directory set for `spec`: false when the directory does not fit the snapshot pool (the
  // caller then takes the segment path, which uploads only the polled brokers' snapshots). Called before a move-in
  // loop changes any state, so the fallback starts from the same state.
  bool queueReady(const GoalImpl& self, int action, const Model::Spec& spec);
  // Shard groups: the queue path is allowed only when every rank can take it (set at attach, ccmi_api.cpp)
  bool shardQueueAllowed = true;
  // the snapshot directory current for `spec` (Device::qdirRows / qdirLen then give every broker's live view)
  void queueSyncSpec(const Model::Spec& spec) { queueSync(spec); }
  int64_t queueScan(GoalImpl& self, int action, const Model::Spec& spec, int head, int skip0, const int32_t* tail,
                    int nTail, const std::vector<int32_t>& cands);
  int64_t exclLeadCount(const DevProgram& prog, const int32_t* reps, int K, const std::vector<int32_t>& cands,
                        int64_t key) const;
  bool blocked(const DevProgram& prog, int r, int b) const;
  bool exclOnDevice = false;  // the device's broker exclusion bits are set
  bool terminalOptimized() const;  // an optimized goal is `terminal`
  void checkTerminal(int64_t key) const;  // a candidate reached a terminal optimized goal: IllegalStateException
  int64_t pairScan(GoalImpl& self, const std::vector<int32_t>& pr, const std::vector<int32_t>& pb,
                   int action = DA_LEADERSHIP, bool count = true);
  int64_t swapScan(GoalImpl& self, const std::vector<int32_t>& srcs, const std::vector<int32_t>& cbOff,
                   const std::vector<int32_t>& cbRep, const SwapLimit& lim = SwapLimit());
  void eligible(const std::vector<int32_t>& in, int action, std::vector<int32_t>& out) const;
  // eligible() without the copy when no exclusion applies to the action (the result is `in` itself, else `scratch`)
  const std::vector<int32_t>& eligibleView(const std::vector<int32_t>& in, int action,
                                           std::vector<int32_t>& scratch) const {
    const bool keepsAll = action == DA_LEADERSHIP ? !opt.anyExclLead : (!opt.anyRequested && !opt.anyExclMove);
    if (keepsAll) return in;
    eligible(in, action, scratch);
    return scratch;
  }
  // Reference-visited candidates of replica r over cands[0, n) (eligible lists): the entries the replica-dependent
  // filters of GoalUtils.eligibleBrokers keep (blocked), skipping brokers that host r's partition when
  // `skipHosts` (candidate lists the device scans whole while the reference's list leaves the hosts out).
  int64_t visitCount(int action, int r, const int32_t* cands, size_t n, bool skipHosts = false) const;

  double threshold(double avgPct, int res, bool lower) const;  // GoalUtils.computeResourceUtilizationBalanceThreshold

  // Chains (Device::chainPairs / chainRackRows, kernel K7): the device makes a sequence of the reference loop's
  // decisions in one launch, applying each move before the next; the engine replays the logged moves into the host
  // model (Model::replaying). Not used for destination-sharded sessions. CCMI_NO_CHAINS=1 turns them off.
  bool chainsOn() const;
  bool pairChains = false;  // the leadership loops run as K7 chains (CCMI_PAIR_CHAINS=1, set per goal; chainsOn too)
  int64_t chainPairs(GoalImpl& self, int action, const std::vector<int32_t>& pr, const std::vector<int32_t>& pb,
                     const std::vector<int32_t>& next, int maxAccepts, std::vector<int32_t>& log);
  int64_t chainRackRows(GoalImpl& self, const std::vector<int32_t>& rows, const std::vector<int32_t>& cands,
                        std::vector<int32_t>& log);
  // RackAwareGoal's rows with no optimized goals, decided per partition on the device (Device::rackRowsGroups, nothing
  // applied there): res[k] = accepted candidate index, kRackKeep or kRackFail
  void rackRowsGroups(GoalImpl& self, const std::vector<int32_t>& rows, const std::vector<int32_t>& cands,
                      std::vector<int32_t>& res);

 private:
  // the snapshot directory's catch-up state: the Spec + selection it was filled for, the pool epoch it refers to and
  // the position in Model::verLog up to which every changed broker's entry was set again
  struct QueueSync {
    bool bound = false;
    uint64_t key = 0;
    uint32_t epoch = 0;
    size_t logPos = 0;
    std::vector<uint32_t> stamp;  // [B] the round a broker was last set in (dedupes the log)
    uint32_t round = 0;
    std::vector<std::shared_ptr<const std::vector<int32_t>>> snaps;  // a sync's snapshots (scratch)
    std::vector<int32_t> todo;                                       // a sync's brokers (scratch)
  };
  QueueSync qsync_;
  void queueSync(const Model::Spec& spec);
  bool queueSyncTry(const Model::Spec& spec);  // queueSync, false (directory unbound) when it does not fit the pool
  DevProgram program(const GoalImpl& self, int action) const;
  int64_t combine(int64_t localKey) const;
  void refreshAllowed(GoalImpl& g);
};

std::unique_ptr<GoalImpl> makeGoal(int kind);
std::unique_ptr<GoalImpl> makeMoreGoal(int kind);  // engine_goals.cpp: the remaining default goals
std::unique_ptr<GoalImpl> makeIntraGoal(int kind);  // engine_intra.cpp: the intra-broker (JBOD) goals
bool isIntraGoalKind(int kind);
// Goal.actionAcceptance of an intra-broker goal (host model), or -1 when `g` is not one
int intraAcceptance(const GoalImpl& g, const Engine& e, const ccmi_action& a);


}  // namespace ccmi
