"""RackAwareDistributionGoal (analyzer/goals/RackAwareDistributionGoal.java) and Goal.actionAcceptance parity.

* Live parity against the oracle on RandomCluster models that are not rack-aware (replication factor above, at and
  below the rack count, dead brokers, brokers excluded for replica moves): the goal alone, the goal as a prior goal of
  the distribution goals (its acceptance runs inside every scan), and RandomClusterTest's goal list
  (RandomClusterTest.java:103-121) restricted to the goals of this build.
* The reference-held pins are elsewhere: ExcludedTopicsTest rows (test_excluded_topics.py), ExcludedBrokersFor*
  rows (test_excluded_brokers.py), DeterministicClusterTest decks and RackAwareGoalTest for both rack goals
  (test_deterministic.py).
* ccmi_action_acceptance against the oracle's Goal.actionAcceptance for every goal of a chain, on random moves,
  leadership moves and swaps after the optimization (ACCEPT / REPLICA_REJECT / BROKER_REJECT exactly).
"""
import random

import pytest

import ccmi
from parity import check_product_against_oracle

# RandomClusterTest.java:103-121 without BrokerSetAwareGoal (not in this build)
RANDOM_CLUSTER_GOALS = ["RackAwareGoal", "RackAwareDistributionGoal", "MinTopicLeadersPerBrokerGoal",
                        "ReplicaCapacityGoal", "DiskCapacityGoal", "NetworkInboundCapacityGoal",
                        "NetworkOutboundCapacityGoal", "CpuCapacityGoal", "ReplicaDistributionGoal",
                        "PotentialNwOutGoal", "DiskUsageDistributionGoal", "NetworkInboundUsageDistributionGoal",
                        "NetworkOutboundUsageDistributionGoal", "CpuUsageDistributionGoal",
                        "LeaderReplicaDistributionGoal", "LeaderBytesInDistributionGoal",
                        "TopicReplicaDistributionGoal", "PreferredLeaderElectionGoal"]
RAD = ["RackAwareDistributionGoal"]

CASES = [
    # replication factor 4 over 3 racks: one rack holds two replicas of every partition
    (dict(num_racks=3, num_brokers=12, num_replicas=2400, num_topics=60, min_replication=4, max_replication=4),
     RAD, None),
    (dict(num_racks=5, num_brokers=20, num_replicas=3000, num_topics=100), RAD, None),
    (dict(num_racks=2, num_brokers=10, num_replicas=1500, num_topics=50, min_replication=3, max_replication=3),
     RAD, None),
    (dict(num_racks=4, num_brokers=16, num_replicas=2400, num_topics=60, num_dead_brokers=2), RAD, None),
    (dict(num_racks=4, num_brokers=16, num_replicas=2400, num_topics=60), RAD,
     dict(excluded_brokers_for_replica_move=[1, 6])),
    (dict(num_racks=3, num_brokers=12, num_replicas=2400, num_topics=60, min_replication=4, max_replication=4),
     RAD + list(ccmi.C1_GOALS), None),
    (dict(num_racks=4, num_brokers=16, num_replicas=2400, num_topics=60, num_dead_brokers=1),
     RANDOM_CLUSTER_GOALS, None),
    (dict(num_racks=3, num_brokers=12, num_replicas=1800, num_topics=40),
     ["RackAwareDistributionGoal", "ReplicaCapacityGoal", "ReplicaDistributionGoal",
      "TopicReplicaDistributionGoal", "LeaderReplicaDistributionGoal"], None),
]
IDS = [f"{i}-{len(g)}goals" for i, (_, g, _) in enumerate(CASES)]


def _opts(o):
    return ccmi.OptimizationOptions(**o) if o else None


@pytest.mark.parametrize("props,goals,opts", CASES, ids=IDS)
def test_emu_rack_aware_distribution_matches_oracle(emu_lib, oracle_lib, props, goals, opts):
    check_product_against_oracle(emu_lib, props, goals, 1.05, max_replicas=3000, options=_opts(opts))


def random_actions(desc, dist, leaders, n, seed):
    """Inter-broker moves / leadership moves / swaps in the action-log layout, all referring to replicas that
    exist: (type, partition, source, destination, destination partition)."""
    rng = random.Random(seed)
    off = [desc.partition_offset[i] for i in range(desc.num_partitions + 1)]
    P, B = desc.num_partitions, desc.num_brokers
    brokers_of = [dist[off[p]:off[p + 1]] for p in range(P)]
    out = []
    while len(out) < n:
        p = rng.randrange(P)
        kind = rng.randrange(3)
        if kind == 0:
            src = rng.choice(brokers_of[p])
            dst = rng.randrange(B)
            if dst not in brokers_of[p]:
                out.append((0, p, src, dst, -1))
        elif kind == 1:
            followers = [b for b in brokers_of[p] if b != leaders[p]]
            if followers:
                out.append((1, p, leaders[p], rng.choice(followers), -1))
        else:
            q = rng.randrange(P)
            src, dst = rng.choice(brokers_of[p]), rng.choice(brokers_of[q])
            if p != q and src != dst and dst not in brokers_of[p] and src not in brokers_of[q]:
                out.append((2, p, src, dst, q))
    return out


def check_acceptance_against_oracle(lib, props, goals, n=400):
    cm, res, oc = check_product_against_oracle(lib, props, goals, 1.05, max_replicas=3000)
    assert res is not None
    buf = ccmi.RandomCluster.generate(lib, **props)
    desc = buf.desc
    acts = random_actions(desc, oc.replica_distribution(), oc.leader_distribution(), n, 7)
    seen = set()
    for gi, g in enumerate(goals):
        for a in acts:
            got = cm.action_acceptance(gi, *a)
            want = oc.action_acceptance(gi, *a)
            assert got == want, (g, a, got, want)
            seen.add((g, want))
    return seen


ACC_CASES = [
    (dict(num_racks=3, num_brokers=12, num_replicas=1800, num_topics=40),
     ["RackAwareDistributionGoal", "MinTopicLeadersPerBrokerGoal", "ReplicaCapacityGoal", "DiskCapacityGoal",
      "NetworkInboundCapacityGoal", "NetworkOutboundCapacityGoal", "CpuCapacityGoal", "ReplicaDistributionGoal",
      "PotentialNwOutGoal", "DiskUsageDistributionGoal", "NetworkInboundUsageDistributionGoal",
      "NetworkOutboundUsageDistributionGoal", "CpuUsageDistributionGoal", "TopicReplicaDistributionGoal",
      "LeaderReplicaDistributionGoal", "LeaderBytesInDistributionGoal"]),
    (dict(num_racks=5, num_brokers=15, num_replicas=1500, num_topics=30, rack_aware=1), ["RackAwareGoal"] +
     list(ccmi.C1_GOALS)),
]


@pytest.mark.parametrize("props,goals", ACC_CASES, ids=["all-goals", "rack-aware-c1"])
def test_emu_action_acceptance_matches_oracle(emu_lib, oracle_lib, props, goals):
    seen = check_acceptance_against_oracle(emu_lib, props, goals)
    kinds = {w for _, w in seen}
    assert "ACCEPT" in kinds and "REPLICA_REJECT" in kinds  # the sample reaches both outcomes


@pytest.mark.gpu
@pytest.mark.parametrize("props,goals,opts", CASES, ids=IDS)
def test_gpu_rack_aware_distribution_matches_oracle(gpu_lib, oracle_lib, props, goals, opts):
    check_product_against_oracle(gpu_lib, props, goals, 1.05, max_replicas=3000, options=_opts(opts))


@pytest.mark.gpu
@pytest.mark.parametrize("props,goals", ACC_CASES, ids=["all-goals", "rack-aware-c1"])
def test_gpu_action_acceptance_matches_oracle(gpu_lib, oracle_lib, props, goals):
    check_acceptance_against_oracle(gpu_lib, props, goals)
