"""The callers either side of the optimizer path:

* GoalViolationDetector batches (detector/GoalViolationDetector.java:176-332): every detection goal optimized alone
  with isTriggeredByGoalViolation on the initial model (run as concurrent device sessions); fixable / unfixable
  violations, the aggregated provision response and the balancedness score (KafkaCruiseControlUtils.java:844-870,
  GoalViolationDetector.refreshBalancednessScore :276-282) against the oracle doing the same goal by goal.
* Proposal output: OptimizerResult.getProposalSummaryForJson (OptimizerResult.java:300-320) with the movement stats
  (:259-279) and on-demand balancedness scores (:123-131), ExecutionProposal.getJsonStructure
  (ExecutionProposal.java:266-270).
"""
import json

import pytest

import ccmi
from oracle_binding import OracleCluster
from parity import constraint

DEFAULT_GOALS = list(ccmi.DEFAULT_GOALS)
PROPS = dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300)


def test_balancedness_costs_kat():
    """balancednessCostByGoal: weights grow by the priority weight towards higher priority, hard goals carry the
    strictness weight, and the costs sum to MAX_BALANCEDNESS_SCORE."""
    goals = ccmi.goals_from_names(DEFAULT_GOALS)
    cost = ccmi.balancedness_cost_by_goal(goals, 1.1, 1.5)
    assert abs(sum(cost.values()) - 100.0) < 1e-9
    w = {}
    prev = 1 / 1.1
    for g in reversed(goals):
        cur = 1.1 * prev
        w[g.name()] = cur * (1.5 if g.is_hard_goal() else 1)
        prev = cur
    total = sum(w.values())
    for n in w:
        assert cost[n] == 100.0 * w[n] / total
    assert cost["RackAwareGoal"] > cost["ReplicaCapacityGoal"] > cost["ReplicaDistributionGoal"]
    with pytest.raises(ccmi.IllegalArgumentException):
        ccmi.balancedness_cost_by_goal(goals, 0.0, 1.5)


def _oracle_detect(desc, goals, bc, opts):
    fixable, unfixable, prov = [], [], ccmi.ProvisionResponse("UNDECIDED")
    for g in goals:
        oc = OracleCluster.from_desc(desc)
        try:
            r = oc.optimize([g], bc, opts)[0]
        except ccmi.OptimizationFailureException as e:
            unfixable.append(g)
            prov.aggregate(e.provision)
            continue
        if oc.proposals():
            fixable.append(g)
        prov.aggregate(r.provision)
    return fixable, unfixable, prov


@pytest.mark.parametrize("props,max_replicas", [(PROPS, 3000), (PROPS, 250), (dict(num_brokers=40), 3000)],
                         ids=["b20", "b20-replica-capacity-violated", "b40"])
def test_emu_goal_violation_detector_matches_oracle(emu_lib, oracle_lib, props, max_replicas):
    bc = constraint(1.05, max_replicas)
    buf = ccmi.RandomCluster.generate(emu_lib, **props)
    det = ccmi.GoalViolationDetector(DEFAULT_GOALS, bc, lib=emu_lib, max_concurrency=4)
    v = det.detect(buf.desc, buf, excluded_topics=[1])
    opts = ccmi.OptimizationOptions(excluded_topics=[1], is_triggered_by_goal_violation=True)
    fixable, unfixable, prov = _oracle_detect(buf.desc, DEFAULT_GOALS, bc, opts)
    assert (v.fixable, v.unfixable) == (fixable, unfixable)
    assert v.provision_response == prov
    assert v.balancedness_score == 100.0 - sum(det.cost[g] for g in fixable + unfixable)
    assert fixable, "the random cluster violates some goal"


def test_emu_goal_violation_detector_skips_offline_replicas(emu_lib):
    buf = ccmi.RandomCluster.generate(emu_lib, num_racks=6, num_brokers=24, num_replicas=4800, num_topics=30,
                                      num_dead_brokers=2)
    v = ccmi.GoalViolationDetector(DEFAULT_GOALS, lib=emu_lib).detect(buf.desc, buf)
    assert v.skipped_due_to_offline_replicas and v.balancedness_score == -1.0 and not v.fixable


def _check_proposal_summary_json(lib):
    """OptimizerResult.getProposalSummaryForJson (OptimizerResult.java:301-319) over the product's proposals."""
    bc = constraint(1.05, 3000)
    buf = ccmi.RandomCluster.generate(lib, **PROPS)
    cm = ccmi.ClusterModel.from_buffers(buf)
    res = ccmi.GoalOptimizer(bc).optimizations(cm, ccmi.goals_from_names(DEFAULT_GOALS),
                                               ccmi.OptimizationOptions(excluded_topics=[1, 2],
                                                                        excluded_brokers_for_leadership=[3]))
    summary = res.proposal_summary_json()
    json.dumps(summary)  # serialisable
    assert set(summary) == {"numReplicaMovements", "dataToMoveMB", "numIntraBrokerReplicaMovements",
                            "intraBrokerDataToMoveMB", "numLeaderMovements", "recentWindows",
                            "monitoredPartitionsPercentage", "excludedTopics", "excludedBrokersForLeadership",
                            "excludedBrokersForReplicaMove", "onDemandBalancednessScoreBefore",
                            "onDemandBalancednessScoreAfter", "provisionStatus", "provisionRecommendation"}
    props = res.proposals
    replica_moves = [p for p in props if sorted(p.old_replicas) != sorted(p.new_replicas)]
    assert summary["numReplicaMovements"] == len(replica_moves)
    assert summary["numLeaderMovements"] == len(props) - len(replica_moves)
    assert summary["dataToMoveMB"] == sum(len(set(p.new_replicas) - set(p.old_replicas)) * p.partition_size
                                          for p in replica_moves)
    assert summary["excludedTopics"] == ["T1", "T2"] and summary["excludedBrokersForLeadership"] == [3]
    assert summary["onDemandBalancednessScoreAfter"] >= summary["onDemandBalancednessScoreBefore"]
    assert summary["provisionStatus"] == res.provision_response.status
    rows = res.proposals_json()
    assert len(rows) == len(props) and set(rows[0]) == {"topicPartition", "oldLeader", "oldReplicas", "newReplicas"}
    # the oracle's proposal set gives the same summary
    oc = OracleCluster.from_desc(buf.desc)
    oc.optimize(DEFAULT_GOALS, bc, ccmi.OptimizationOptions(excluded_topics=[1, 2], excluded_brokers_for_leadership=[3]))
    key = lambda p: (p.partition, tuple(p.old_replicas), tuple(p.new_replicas), p.old_leader)  # noqa: E731
    assert sorted(map(key, oc.proposals())) == sorted(map(key, props))


def test_emu_proposal_summary_json(emu_lib, oracle_lib):
    _check_proposal_summary_json(emu_lib)


@pytest.mark.gpu
def test_gpu_proposal_summary_json(gpu_lib, oracle_lib):
    _check_proposal_summary_json(gpu_lib)


def test_emu_intra_broker_summary(emu_lib):
    """Intra-broker (JBOD) proposals count as intra-broker replica movements."""
    buf = ccmi.RandomCluster.generate(emu_lib, num_racks=5, num_brokers=20, num_replicas=6000, num_topics=200,
                                      rack_aware=1, jbod=2, num_logdirs=4, logdir_capacity=[75000.0] * 4)
    cm = ccmi.ClusterModel.from_buffers(buf)
    bc = constraint(1.05, 3000)
    res = ccmi.GoalOptimizer(bc).optimizations(cm, ccmi.goals_from_names(list(ccmi.INTRA_BROKER_GOALS)))
    s = res.proposal_summary_json()
    assert s["numIntraBrokerReplicaMovements"] > 0 and s["numReplicaMovements"] == 0
    assert s["intraBrokerDataToMoveMB"] > 0


@pytest.mark.gpu
def test_gpu_goal_violation_detector_matches_oracle(gpu_lib, oracle_lib):
    bc = constraint(1.05, 250)
    buf = ccmi.RandomCluster.generate(gpu_lib, **PROPS)
    v = ccmi.GoalViolationDetector(DEFAULT_GOALS, bc, lib=gpu_lib, max_concurrency=8).detect(buf.desc, buf)
    opts = ccmi.OptimizationOptions(is_triggered_by_goal_violation=True)
    fixable, unfixable, prov = _oracle_detect(buf.desc, DEFAULT_GOALS, bc, opts)
    assert (v.fixable, v.unfixable) == (fixable, unfixable)
    assert v.provision_response == prov
