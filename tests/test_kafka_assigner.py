"""Kafka-assigner mode goals (analyzer/kafkaassigner/KafkaAssignerEvenRackAwareGoal.java,
KafkaAssignerDiskUsageDistributionGoal.java; in `goals`, not in default.goals).

Pinned by the reference's own tests elsewhere in this suite: the DeterministicClusterTest kafka-assigner decks
(DeterministicClusterTest.java:200-215, tests/test_deterministic.py) and the ExcludedTopicsTest rows
(ExcludedTopicsTest.java:278-302, tests/test_excluded_topics.py). Here the product matches the oracle bit for bit on
RandomCluster inputs (replica moves, leadership moves, follower-position swaps and disk-usage swaps), on chains where a
later goal's candidates go through KafkaAssignerEvenRackAwareGoal.actionAcceptance (the rack-awareness predicate), and
where a goal after KafkaAssignerDiskUsageDistributionGoal hits its IllegalStateException at the first candidate.
"""
import random

import pytest

import ccmi
from oracle_binding import OracleCluster
from parity import check_desc_against_oracle

KA_EVEN, KA_DISK = "KafkaAssignerEvenRackAwareGoal", "KafkaAssignerDiskUsageDistributionGoal"


def _constraint():
    bc = ccmi.BalancingConstraint()
    bc.set_resource_balance_percentage(1.05)
    bc.set_capacity_threshold(0.8)
    return bc


CASES = {
    "pair": (dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=60), [KA_EVEN, KA_DISK], None),
    "pair-dead": (dict(num_racks=6, num_brokers=24, num_replicas=4800, num_topics=30, num_dead_brokers=2),
                  [KA_EVEN, KA_DISK], None),
    "pair-excluded": (dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=60), [KA_EVEN, KA_DISK],
                      dict(excluded_topics=[1, 4, 9])),
    "even-then-distribution": (dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=60),
                               [KA_EVEN, "ReplicaDistributionGoal", "LeaderReplicaDistributionGoal"], None),
    "disk-then-goal": (dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=60),
                       [KA_DISK, "NetworkOutboundUsageDistributionGoal"], None),
    "too-few-racks": (dict(num_racks=2, num_brokers=12, num_replicas=3000, num_topics=20), [KA_EVEN, KA_DISK], None),
    "goal-violation": (dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=60), [KA_EVEN],
                       dict(is_triggered_by_goal_violation=True)),
}


def _case(lib, name):
    props, goals, opts = CASES[name]
    buf = ccmi.RandomCluster.generate(lib, **props)
    options = ccmi.OptimizationOptions(**opts) if opts else None
    return check_desc_against_oracle(lib, buf.desc, buf, goals, _constraint(), options)


@pytest.mark.parametrize("name", list(CASES))
def test_emu_kafka_assigner_matches_oracle(emu_lib, oracle_lib, name):
    cm, res, oc = _case(emu_lib, name)
    if name in ("pair", "pair-dead", "pair-excluded", "even-then-distribution"):
        assert res is not None and res.goal_results[0].actions > 0
    if name in ("disk-then-goal", "too-few-racks", "goal-violation"):
        assert res is None  # both raised the same exception (IllegalStateException / OptimizationFailure / IllegalArgument)


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CASES))
def test_gpu_kafka_assigner_matches_oracle(gpu_lib, oracle_lib, name):
    _case(gpu_lib, name)


def _acceptance_pairs(lib):
    """KafkaAssignerEvenRackAwareGoal.actionAcceptance (:385-408) on random moves, leadership moves and swaps."""
    buf = ccmi.RandomCluster.generate(lib, num_racks=5, num_brokers=20, num_replicas=6000, num_topics=60)
    bc = _constraint()
    cm = ccmi.ClusterModel(buf.desc, device=0, lib=lib, keepalive=buf)
    ccmi.GoalOptimizer(bc).optimizations(cm, ccmi.goals_from_names([KA_EVEN]))
    oc = OracleCluster.from_desc(buf.desc)
    oc.optimize([KA_EVEN], bc)
    assert cm.actions() == oc.actions() and cm.replica_distribution() == oc.replica_distribution()
    dist, d = cm.replica_distribution(), buf.desc
    rng = random.Random(5)
    out = []
    for i in range(600):
        slot = rng.randrange(d.num_replicas)
        p = d.replica_partition[d.partition_replicas[slot]]
        src = dist[slot]
        kind = i % 3
        dp = -1
        if kind == 0:
            typ, dst = ccmi.ACTION_TYPES.index("INTER_BROKER_REPLICA_MOVEMENT"), rng.randrange(d.num_brokers)
        elif kind == 1:
            typ, dst = ccmi.ACTION_TYPES.index("LEADERSHIP_MOVEMENT"), rng.randrange(d.num_brokers)
        else:
            s2 = rng.randrange(d.num_replicas)
            typ, dst, dp = ccmi.ACTION_TYPES.index("INTER_BROKER_REPLICA_SWAP"), dist[s2], \
                d.replica_partition[d.partition_replicas[s2]]
        if dst == src:
            continue
        out.append((cm.action_acceptance_by_goal(KA_EVEN, typ, p, src, dst, dp),
                    oc.action_acceptance(0, typ, p, src, dst, dp)))
    return out


def test_emu_kafka_assigner_acceptance_matches_oracle(emu_lib, oracle_lib):
    pairs = _acceptance_pairs(emu_lib)
    assert all(g == w for g, w in pairs)
    assert {w for _, w in pairs} >= {"ACCEPT", "BROKER_REJECT", "REPLICA_REJECT"}


@pytest.mark.gpu
def test_gpu_kafka_assigner_acceptance_matches_oracle(gpu_lib, oracle_lib):
    assert all(g == w for g, w in _acceptance_pairs(gpu_lib))


def test_emu_kafka_assigner_disk_goal_acceptance_throws(emu_lib, oracle_lib):
    """KafkaAssignerDiskUsageDistributionGoal.actionAcceptance: IllegalStateException (:540-543)."""
    buf = ccmi.RandomCluster.generate(emu_lib, num_racks=5, num_brokers=20, num_replicas=6000, num_topics=60)
    cm = ccmi.ClusterModel(buf.desc, device=0, lib=emu_lib, keepalive=buf)
    ccmi.GoalOptimizer(_constraint()).optimizations(cm, ccmi.goals_from_names([KA_DISK]))
    with pytest.raises(ccmi.IllegalStateException):
        cm.action_acceptance_by_goal(KA_DISK, 1, 0, cm.leader_distribution()[0], (cm.leader_distribution()[0] + 1) % 20)
