"""OptimizationVerifier restatement (TEST INFRASTRUCTURE): the reference's oracle-independent invariants over one
optimization result, applied to the CPU oracle AND to the product library.

cruise-control/src/test/java/com/linkedin/kafka/cruisecontrol/analyzer/OptimizationVerifier.java
  executeGoalsFor            :112-219 (one pass: separateHardGoalsAndSoftGoals = false)
  verifyGoalViolations       :221-230
  verifyBrokenBrokers        :232-250
  verifySoftGoalReplicaMovements :252-292
  verifyNewBrokers           :294-317
  verifyRegression           :319-336
with every goal's ClusterModelStatsComparator (goals/*.java clusterModelStatsComparator()).
"""
from __future__ import annotations

import json
import math
import os
from typing import Dict, List, Optional, Sequence

import ccmi

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
RES = {"CPU": 0, "NW_IN": 1, "NW_OUT": 2, "DISK": 3}
EPSILON = 1e-5                                        # AnalyzerUtils.EPSILON (AnalyzerUtils.java:33)
RESOURCE_EPSILON = (0.001, 10.0, 10.0, 100.0)         # Resource.java:17-25 (CPU, NW_IN, NW_OUT, DISK)
EPSILON_PERCENT = 0.0008                              # Resource.java:31


def _compare(d1: float, d2: float, eps: float) -> int:  # AnalyzerUtils.compare (AnalyzerUtils.java:202-213)
    if d2 - d1 > eps:
        return -1
    if d1 - d2 > eps:
        return 1
    return 0


def _compare_res(d1: float, d2: float, res: int) -> int:  # AnalyzerUtils.compare(d1, d2, Resource) :189-192
    return _compare(d1, d2, max(RESOURCE_EPSILON[res], EPSILON_PERCENT * (d1 + d2)))


def _std_cmp(key):
    # ReplicaDistributionGoal.java:345-356, LeaderReplicaDistributionGoal.java:373-383,
    # TopicReplicaDistributionGoal.java:576-587: compare(stDev2 (before), stDev1 (after), EPSILON)
    return lambda after, before, bc: _compare(before[key], after[key], EPSILON)


def _resource_distribution_cmp(res):  # ResourceDistributionGoal.java:1043-1064
    def cmp(after, before, bc):
        if before["num_balanced_brokers_by_resource"][res] > after["num_balanced_brokers_by_resource"][res]:
            if before["resource_std"][res] < after["resource_std"][res]:  # Double.compare(before, after) < 0
                return -1
        return 1
    return cmp


def _leader_bytes_in_cmp(after, before, bc):  # LeaderBytesInDistributionGoal.java:264-281
    threshold = after["resource_avg"][1] * bc.resource_balance_percentage[1]
    if after["resource_max"][1] <= threshold:
        return 1
    return _compare_res(math.sqrt(before["resource_std"][1]), math.sqrt(after["resource_std"][1]), 1)


def _intra_usage_cmp(after, before, bc):  # IntraBrokerDiskUsageDistributionGoal.java:501-517
    if (after["num_unbalanced_disks"] > before["num_unbalanced_disks"]
            or after["disk_utilization_std"] > before["disk_utilization_std"]):
        return -1
    return 1


def _potential_nw_out_cmp(after, before, bc):  # PotentialNwOutGoal.java:350-360
    a, b = after["num_brokers_under_potential_nw_out"], before["num_brokers_under_potential_nw_out"]
    return (a > b) - (a < b)


COMPARATORS = {
    "ReplicaDistributionGoal": _std_cmp("replica_std"),
    "LeaderReplicaDistributionGoal": _std_cmp("leader_std"),
    "TopicReplicaDistributionGoal": _std_cmp("topic_replica_std"),
    "PotentialNwOutGoal": _potential_nw_out_cmp,
    "CpuUsageDistributionGoal": _resource_distribution_cmp(0),
    "NetworkInboundUsageDistributionGoal": _resource_distribution_cmp(1),
    "NetworkOutboundUsageDistributionGoal": _resource_distribution_cmp(2),
    "DiskUsageDistributionGoal": _resource_distribution_cmp(3),
    "LeaderBytesInDistributionGoal": _leader_bytes_in_cmp,
    "IntraBrokerDiskUsageDistributionGoal": _intra_usage_cmp,
    # DiskDistributionGoalStatsComparator (KafkaAssignerDiskUsageDistributionGoal.java:608-632)
    "KafkaAssignerDiskUsageDistributionGoal": lambda after, before, bc: (
        -1 if before["num_balanced_brokers_by_resource"][3] > after["num_balanced_brokers_by_resource"][3] else 1),
}  # hard goals, MinTopicLeaders, PreferredLeaderElection: comparisons are irrelevant (return 0)


def verify_regression(goal_results, pre_stats: dict, bc: ccmi.BalancingConstraint) -> Optional[str]:
    """verifyRegression (:319-336): every goal's stats do not compare worse than the previous goal's."""
    prev = pre_stats
    for g in goal_results:
        cmp = COMPARATORS.get(g.name)
        if cmp is not None and cmp(g.stats, prev, bc) < 0:
            return f"Failed goal comparison {g.name}"
        prev = g.stats
    return None


def verify_goal_violations(goal_results) -> Optional[str]:
    """verifyGoalViolations (:221-230): no goal is left violated after the optimization (GoalOptimizer.java:479-481:
    violatedGoalNamesAfterOptimization holds the goals whose optimize() returned false)."""
    violated = [g.name for g in goal_results if not g.succeeded]
    return f"Failed to optimize goal {violated}" if violated else None


def verify_broken_brokers(dead: Sequence[int], final_replica_brokers: Sequence[int]) -> Optional[str]:
    """verifyBrokenBrokers (:232-250): no replica remains on a dead broker."""
    left = set(final_replica_brokers) & set(dead)
    return f"replicas left on dead brokers {sorted(left)}" if left else None


def verify_soft_goal_replica_movements(proposals, offline_by_partition: Dict[int, set], goals: Sequence[str]) \
        -> Optional[str]:
    """verifySoftGoalReplicaMovements (:252-292), one pass: with no hard goal in the list, every replica a proposal
    removes from a broker must be an originally offline replica (immigrants cannot exist in one pass)."""
    if any(ccmi.Goal(n).is_hard_goal() for n in goals):
        return None
    for p in proposals:
        removed = set(p.old_replicas) - set(p.new_replicas)
        for b in removed:
            if b not in offline_by_partition.get(p.partition, set()):
                return f"soft goal moved online replica of partition {p.partition} from broker {b}"
    return None


def deterministic_models() -> dict:
    with open(os.path.join(GOLDEN, "deterministic_clusters.json")) as f:
        return json.load(f)


def build_model(m: dict) -> ccmi.FlatCluster:
    """Replay one transcribed DeterministicCluster model through ClusterModelBuilder."""
    b = ccmi.ClusterModelBuilder()
    for bid in sorted(m["racks"], key=int):
        b.create_broker(m["racks"][bid], int(bid), m["capacity"], m.get("logdirs"))
    for broker, topic, part, index, leader, *logdir in m["replicas"]:
        b.create_replica(m["racks"][str(broker)], broker, topic, part, index, leader, logdir=logdir[0] if logdir else None)
    for broker, topic, part, cpu, nw_in, nw_out, disk in m["loads"]:
        b.set_replica_load(m["racks"][str(broker)], broker, topic, part, cpu, nw_in, nw_out, disk)
    for d in m["dead"]:
        b.set_broker_state(d, "DEAD")
    return b.build()


def offline_replicas(flat: ccmi.FlatCluster, m: dict) -> Dict[int, set]:
    """selfHealingEligibleReplicas by partition index -> original broker ids (replicas on dead brokers)."""
    out: Dict[int, set] = {}
    d = flat.desc
    for r in range(d.num_replicas):
        if d.replica_broker[r] in m["dead"]:
            out.setdefault(d.replica_partition[r], set()).add(d.replica_broker[r])
    return out


def final_replica_brokers(replica_distribution: List[int]) -> List[int]:
    return list(replica_distribution)


def model_facts(broker_state: Sequence[int], replica_broker: Sequence[int], replica_partition: Sequence[int],
                replica_offline: Sequence[int]):
    """(dead broker ids, selfHealingEligibleReplicas by partition -> original brokers) of a flattened model before
    optimization: replicas on DEAD brokers or flagged original-offline (ClusterModel.selfHealingEligibleReplicas,
    ClusterModel.java:203-205, filled by setBrokerState DEAD and offline replicas; broker ids equal indices in the flattened ABI)."""
    dead = [b for b, s in enumerate(broker_state) if s == ccmi.BROKER_STATES["DEAD"]]
    dead_set = set(dead)
    offline: Dict[int, set] = {}
    for r, b in enumerate(replica_broker):
        if b in dead_set or replica_offline[r]:
            offline.setdefault(replica_partition[r], set()).add(b)
    return dead, offline


def desc_facts(desc):
    n = desc.num_replicas
    return model_facts([desc.broker_state[b] for b in range(desc.num_brokers)], desc.replica_broker[:n],
                       desc.replica_partition[:n], desc.replica_offline[:n])


def reference_verifications(dead, offline, goals, goal_results, pre_stats, bc, final_brokers=None, proposals=None) \
        -> Dict[str, Optional[str]]:
    """executeGoalsFor's verification switch (OptimizationVerifier.java:177-216) for one pass: the outcome of
    GOAL_VIOLATION, BROKEN_BROKERS and REGRESSION (None = passes; "n/a" = the reference skips it for this model).
    BROKEN_BROKERS runs only with dead brokers (:185-201) and needs the final assignment and the proposals;
    REGRESSION only without self-healing eligible replicas (:203-209). NEW_BROKERS is test_new_brokers.py's."""
    out: Dict[str, Optional[str]] = {"GOAL_VIOLATION": verify_goal_violations(goal_results)}
    if not dead:
        out["BROKEN_BROKERS"] = "n/a"
    elif final_brokers is None:
        out["BROKEN_BROKERS"] = "not evaluated"
    else:
        out["BROKEN_BROKERS"] = (verify_broken_brokers(dead, final_brokers)
                                 or verify_soft_goal_replica_movements(proposals, offline, goals))
    out["REGRESSION"] = "n/a" if offline else verify_regression(goal_results, pre_stats, bc)
    return out


class GoalRecord:
    """A golden's goals_result entry in the shape verify_regression / verify_goal_violations read."""

    def __init__(self, d: dict):
        self.name, self.succeeded, self.stats = d["name"], d["succeeded"], d.get("stats")
