"""TopicLeaderReplicaDistributionGoal (analyzer/goals/TopicLeaderReplicaDistributionGoal.java; in `goals`, not in
default.goals: AnalyzerConfig.java:297-319).

Pinning: TopicLeaderReplicaDistributionGoalTest (analyzer/TopicLeaderReplicaDistributionGoalTest.java:43-145) on its
own cluster (makeSimpleClusterModel :43-72: 6 brokers on racks "rack" + (id % 3), topics T0/T1; broker b leads
assigner(b, t) partitions of topic t, each with one follower on broker (b + 1) % 6; every replica's load is
(cpu 1, nw_in 10, nw_out 13, disk 5) over one window) with topic.leader.replica.count.balance.min.gap = max.gap = 0
(getOptimizerResult :130-144):
  * testGoalNoopOnSatisfiable: 2 leaders of each topic per broker -> no violation before or after, every broker keeps
    avg = 2 leaders of each topic;
  * testGoalLinearLeaderGrowth: 2 * id leaders -> violated before, not after, every broker ends with exactly the
    (integer) average of each topic;
  * testGoalPreferBrokerWithHigherTotalLeaderOnEquality: T0 [6, 6, 4, 5, 5, 5], T1 [4, 5, 5, 5, 5, 5] -> violated
    before, not after, every broker within avg +- 1 of each topic.
The oracle restatement passes the three; the product (emulation and gfx950) matches the oracle bit for bit on them and
on RandomCluster cases (the goal alone, with tight gaps, with dead brokers, leadership-only balancing when every alive
broker is excluded from replica moves, and inside a chain of default goals), plus Goal.actionAcceptance sweeps.
"""
import random

import pytest

import ccmi
from oracle_binding import OracleCluster
from parity import check_desc_against_oracle, check_product_against_oracle

TLRD = "TopicLeaderReplicaDistributionGoal"
CAPACITY = {"CPU": 100.0, "DISK": 300000.0, "NW_IN": 300000.0, "NW_OUT": 200000.0}  # TestConstants.BROKER_CAPACITY


def build(assigner, num_brokers=6):
    """makeSimpleClusterModel (:43-72)."""
    b = ccmi.ClusterModelBuilder()
    rack = lambda x: f"rack{x % 3}"  # noqa: E731
    for x in range(num_brokers):
        b.create_rack(rack(x))
        b.create_broker(rack(x), x, CAPACITY, host=f"broker{x}")
    count = {}
    for x in range(num_brokers):
        for t in range(2):
            topic = f"T{t}"
            for _ in range(assigner(x, t)):
                p = count.get(topic, 0)
                count[topic] = p + 1
                b.create_replica(rack(x), x, topic, p, 0, True)
                b.set_replica_load(rack(x), x, topic, p, 1.0, 10.0, 13.0, 5.0)
                f = (x + 1) % num_brokers
                b.create_replica(rack(f), f, topic, p, 1, False)
                b.set_replica_load(rack(f), f, topic, p, 1.0, 10.0, 13.0, 5.0)
    return b.build()


def kat_constraint():
    bc = ccmi.BalancingConstraint()
    bc.topic_leader_replica_balance_min_gap = 0
    bc.topic_leader_replica_balance_max_gap = 0
    return bc


PREFER = [[6, 6, 4], [4, 5, 5]]
KATS = {
    "noop": (lambda b, t: 2, False, 0),
    "linear": (lambda b, t: 2 * b, True, 0),
    "prefer-higher-total": (lambda b, t: PREFER[t][b] if b < len(PREFER[t]) else 5, True, 1),
}


def _leaders_by_topic(flat, leaders):
    """{topic: [leaders per broker]} from the session's per-partition leader brokers."""
    out = {"T0": [0] * 6, "T1": [0] * 6}
    for p, (topic, _) in flat.partitions.items():
        out[topic][leaders[p]] += 1
    return out


def _check_kat(case, flat, violated_before, violated_after, leaders):
    _, before, slack = KATS[case]
    assert bool(violated_before) == before, violated_before
    assert violated_after == []
    for topic, counts in _leaders_by_topic(flat, leaders).items():
        avg = sum(counts) // len(counts)
        for c in counts:
            assert avg - slack <= c <= avg + slack, (topic, counts)


@pytest.mark.parametrize("case", list(KATS))
def test_oracle_topic_leader_distribution_kat(oracle_lib, case):
    flat = build(KATS[case][0])
    oc = OracleCluster.from_desc(flat.desc)
    res = oc.optimize([TLRD], kat_constraint())
    before = [r.name for r in res if r.has_diff or not r.succeeded]
    after = [r.name for r in res if not r.succeeded]
    _check_kat(case, flat, before, after, oc.leader_distribution())


def _product_kat(lib, case):
    flat = build(KATS[case][0])
    cm, res, _ = check_desc_against_oracle(lib, flat.desc, flat, [TLRD], kat_constraint())
    _check_kat(case, flat, res.violated_goals_before, res.violated_goals_after, cm.leader_distribution())


@pytest.mark.parametrize("case", list(KATS))
def test_emu_topic_leader_distribution_kat(emu_lib, oracle_lib, case):
    _product_kat(emu_lib, case)


@pytest.mark.gpu
@pytest.mark.parametrize("case", list(KATS))
def test_gpu_topic_leader_distribution_kat(gpu_lib, oracle_lib, case):
    _product_kat(gpu_lib, case)


# ----------------------------------------------------------------------------------------------- RandomCluster parity
def _constraint(min_gap=None, max_gap=None, pct=None, multiplier=None):
    bc = ccmi.BalancingConstraint()
    if multiplier is not None:
        bc.goal_violation_distribution_threshold_multiplier = multiplier
    bc.set_resource_balance_percentage(1.05)
    bc.set_capacity_threshold(0.8)
    if min_gap is not None:
        bc.topic_leader_replica_balance_min_gap = min_gap
    if max_gap is not None:
        bc.topic_leader_replica_balance_max_gap = max_gap
    if pct is not None:
        bc.topic_leader_replica_balance_percentage = pct
    return bc


# a chain in AnalyzerConfig `goals` order (TopicLeaderReplicaDistributionGoal right after ReplicaCapacityGoal)
CHAIN = ["RackAwareGoal", "ReplicaCapacityGoal", TLRD, "DiskCapacityGoal", "ReplicaDistributionGoal",
         "LeaderReplicaDistributionGoal", "TopicReplicaDistributionGoal"]
RANDOM = {
    "alone": (dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=60), [TLRD], {}, None),
    "tight-gaps": (dict(num_racks=4, num_brokers=16, num_replicas=4200, num_topics=40), [TLRD],
                   dict(min_gap=0, max_gap=0), None),
    "skewed-leaders": (dict(num_racks=4, num_brokers=12, num_replicas=3000, num_topics=20, leader_in_first_position=1),
                       [TLRD], dict(min_gap=0, max_gap=1, pct=1.02), None),
    # offline replicas leave the dead brokers first (RackAwareGoal), then the goal runs in self-healing mode
    "self-healing": (dict(num_racks=6, num_brokers=24, num_replicas=4800, num_topics=30, num_dead_brokers=3),
                     ["RackAwareGoal", TLRD], {}, None),
    # a broker needing more leaders can be its own source (rebalanceByMovingLeadersIn queues every broker with more
    # leaders than the lower limit, counted over all its leaders, while requireMoreLeaders counts the tracked view's);
    # its leadership "move" to itself makes ClusterModel.relocateLeadership throw IllegalArgumentException
    # (ClusterModel.java:415-421) in the reference, in the oracle and in the product alike
    "dead-brokers": (dict(num_racks=6, num_brokers=24, num_replicas=4800, num_topics=30, num_dead_brokers=3,
                          leader_in_first_position=1), ["RackAwareGoal", TLRD], dict(min_gap=0, max_gap=2), None),
    # the goal's offline leaders stay: its own fixOfflineReplicasOnly round, then OptimizationFailureException
    "dead-brokers-alone": (dict(num_racks=6, num_brokers=24, num_replicas=4800, num_topics=30, num_dead_brokers=3,
                                leader_in_first_position=1), [TLRD], dict(min_gap=0, max_gap=2), None),
    "chain": (dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=60), CHAIN, dict(min_gap=1, max_gap=3),
              None),
    # moves the replica and leader distribution goals already optimized reject
    "after-distribution": (dict(num_racks=4, num_brokers=16, num_replicas=4200, num_topics=40),
                           ["ReplicaDistributionGoal", "LeaderReplicaDistributionGoal", TLRD],
                           dict(min_gap=0, max_gap=0), None),
    "triggered": (dict(num_racks=4, num_brokers=16, num_replicas=4200, num_topics=40), [TLRD],
                  dict(min_gap=0, max_gap=3, pct=1.02, multiplier=1.5), dict(is_triggered_by_goal_violation=True)),
    "immigrants-only": (dict(num_racks=4, num_brokers=16, num_replicas=4200, num_topics=40),
                        ["ReplicaDistributionGoal", TLRD], dict(min_gap=0, max_gap=0),
                        dict(only_move_immigrant_replicas=True)),
    "larger": (dict(num_racks=8, num_brokers=48, num_replicas=24000, num_topics=120), [TLRD],
               dict(min_gap=0, max_gap=1), None),
}


def _random_case(lib, case):
    props, goals, gaps, opts = RANDOM[case]
    buf = ccmi.RandomCluster.generate(lib, **props)
    options = ccmi.OptimizationOptions(**opts) if opts else None
    cm, res, oc = check_desc_against_oracle(lib, buf.desc, buf, goals, _constraint(**gaps), options)
    return cm, res


@pytest.mark.parametrize("case", list(RANDOM))
def test_emu_topic_leader_distribution_random_matches_oracle(emu_lib, oracle_lib, case):
    cm, res = _random_case(emu_lib, case)
    if case in ("tight-gaps", "skewed-leaders", "after-distribution", "larger"):
        assert res is not None and any(r.actions > 0 for r in res.goal_results if r.name == TLRD)
    if case in ("dead-brokers", "dead-brokers-alone"):
        assert res is None  # both sides raised the same exception after the same actions
    if case == "self-healing":
        assert res is not None and res.goal_results[1].candidates > res.goal_results[1].actions


@pytest.mark.gpu
@pytest.mark.parametrize("case", list(RANDOM))
def test_gpu_topic_leader_distribution_random_matches_oracle(gpu_lib, oracle_lib, case):
    _random_case(gpu_lib, case)


def _leadership_only(lib):
    """Every alive broker excluded for replica moves: the goal proceeds with leadership movements only
    (initGoalState :311-318; the limits then come from x / 0.0 averages)."""
    props = dict(num_racks=4, num_brokers=10, num_replicas=2100, num_topics=12)
    buf = ccmi.RandomCluster.generate(lib, **props)
    options = ccmi.OptimizationOptions(excluded_brokers_for_replica_move=list(range(10)))
    return check_desc_against_oracle(lib, buf.desc, buf, [TLRD], _constraint(min_gap=0, max_gap=0), options)


def test_emu_topic_leader_distribution_leadership_only(emu_lib, oracle_lib):
    _leadership_only(emu_lib)


@pytest.mark.gpu
def test_gpu_topic_leader_distribution_leadership_only(gpu_lib, oracle_lib):
    _leadership_only(gpu_lib)


# ----------------------------------------------------------------------------------------------- actionAcceptance
def _acceptance_pairs(lib):
    """actionAcceptance (:181-229) of random moves, leadership moves and swaps after a chain ending in the goal."""
    props = dict(num_racks=4, num_brokers=16, num_replicas=4200, num_topics=40)
    buf = ccmi.RandomCluster.generate(lib, **props)
    bc = _constraint(min_gap=0, max_gap=1)
    goals = ["ReplicaDistributionGoal", TLRD]
    cm = ccmi.ClusterModel(buf.desc, device=0, lib=lib, keepalive=buf)
    ccmi.GoalOptimizer(bc).optimizations(cm, ccmi.goals_from_names(goals))
    oc = OracleCluster.from_desc(buf.desc)
    oc.optimize(goals, bc)
    assert cm.actions() == oc.actions()
    dist = cm.replica_distribution()
    leaders = cm.leader_distribution()
    d = buf.desc
    rng = random.Random(7)
    slots_of = {}
    for slot in range(d.num_replicas):
        slots_of.setdefault(d.replica_partition[d.partition_replicas[slot]], []).append(slot)
    out = []
    for i in range(600):
        slot = rng.randrange(d.num_replicas)
        p = d.replica_partition[d.partition_replicas[slot]]
        src = dist[slot]
        kind = i % 3
        if kind == 0:  # replica movement to a broker without the partition
            dst = rng.randrange(d.num_brokers)
            if any(dist[s] == dst for s in slots_of[p]):
                continue
            typ, dp = ccmi.ACTION_TYPES.index("INTER_BROKER_REPLICA_MOVEMENT"), -1
        elif kind == 1:  # leadership movement from the leader to a follower
            src = leaders[p]
            dst = dist[rng.choice(slots_of[p])]
            if dst == src:
                continue
            typ, dp = ccmi.ACTION_TYPES.index("LEADERSHIP_MOVEMENT"), -1
        else:  # swap with a replica of another partition on another broker
            s2 = rng.randrange(d.num_replicas)
            dp = d.replica_partition[d.partition_replicas[s2]]
            dst = dist[s2]
            if dst == src or dp == p:
                continue
            typ = ccmi.ACTION_TYPES.index("INTER_BROKER_REPLICA_SWAP")
        got = cm.action_acceptance_by_goal(TLRD, typ, p, src, dst, dp)
        want = oc.action_acceptance(1, typ, p, src, dst, dp)
        out.append((got, want))
    return out


def test_emu_topic_leader_distribution_acceptance_matches_oracle(emu_lib, oracle_lib):
    pairs = _acceptance_pairs(emu_lib)
    assert all(g == w for g, w in pairs)
    assert {w for _, w in pairs} >= {"ACCEPT", "REPLICA_REJECT"}


@pytest.mark.gpu
def test_gpu_topic_leader_distribution_acceptance_matches_oracle(gpu_lib, oracle_lib):
    pairs = _acceptance_pairs(gpu_lib)
    assert all(g == w for g, w in pairs)


def test_default_constraint_fields():
    """ccmi_default_constraint carries AnalyzerConfig's defaults (:112-146)."""
    bc = ccmi.BalancingConstraint()
    s = bc.to_struct()
    assert (s.topic_leader_replica_balance_percentage, s.topic_leader_replica_balance_min_gap,
            s.topic_leader_replica_balance_max_gap, s.topic_leader_replica_balance_margin) == (1.10, 2, 10, 0.9)
