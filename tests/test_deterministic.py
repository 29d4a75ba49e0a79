"""The reference's own hand-built clusters and invariants pin the oracle and the product.

* DeterministicClusterTest decks (analyzer/DeterministicClusterTest.java:93-352) on the transcribed
  DeterministicCluster models (tests/golden/deterministic_clusters.json, tests/golden/make_deterministic.py): the
  reference test passes when OptimizationVerifier.executeGoalsFor returns true (NEW_BROKERS, BROKEN_BROKERS,
  REGRESSION) or the chain fails with "Insufficient capacity for" (:355-365). Both the oracle and the product must
  pass that test, and the product must match the oracle bit for bit.
* RackAwareGoalTest (analyzer/RackAwareGoalTest.java:74-178): with the rack-id mapper exactly one proposal moving a
  replica of the partition to broker 2; without it no proposal.
* deadBroker (DeterministicCluster.java:1763-1826) with the default goals: BROKEN_BROKERS and the soft-goal rule.
"""
import pytest

import ccmi
from oracle_binding import OracleCluster
from parity import check_desc_against_oracle
from verifier import (build_model, deterministic_models, offline_replicas, verify_broken_brokers,
                      verify_regression, verify_soft_goal_replica_movements)

# DeterministicClusterTest.java:97-115 in priority order (every goal of the deck is in this build).
DECK_GOALS_ALL = ["RackAwareGoal", "RackAwareDistributionGoal", "MinTopicLeadersPerBrokerGoal", "ReplicaCapacityGoal",
                  "DiskCapacityGoal", "NetworkInboundCapacityGoal", "NetworkOutboundCapacityGoal", "CpuCapacityGoal",
                  "ReplicaDistributionGoal", "PotentialNwOutGoal", "DiskUsageDistributionGoal",
                  "NetworkInboundUsageDistributionGoal", "NetworkOutboundUsageDistributionGoal",
                  "CpuUsageDistributionGoal", "LeaderReplicaDistributionGoal", "LeaderBytesInDistributionGoal",
                  "TopicReplicaDistributionGoal", "PreferredLeaderElectionGoal"]
DECK_GOALS = [g for g in DECK_GOALS_ALL if g in ccmi.GOAL_KINDS]

HIGH_BALANCE, MEDIUM_BALANCE, LOW_BALANCE = 1.65, 1.25, 1.05     # TestConstants.java:29-32
HIGH_CAP, MEDIUM_CAP, LOW_CAP = 0.9, 0.8, 0.7                     # TestConstants.java:33-35


def deck_constraint(balance=None, capacity=None, min_leader_topics="", min_leaders=1):
    """getDefaultCruiseControlProperties (DeterministicClusterTest.java:338-345): max.replicas.per.broker 6; the deck's
    topics.with.min.leaders.per.broker / min.topic.leaders.per.broker overrides."""
    bc = ccmi.BalancingConstraint()
    bc.max_replicas_per_broker = 6
    if balance is not None:
        bc.set_resource_balance_percentage(balance)
    if capacity is not None:
        bc.set_capacity_threshold(capacity)
    bc.topics_with_min_leaders_per_broker = min_leader_topics
    bc.min_topic_leaders_per_broker = min_leaders
    return bc


TOPIC_MUST = "must_have_leader_replica_on_broker_topic"  # TestConstants.TOPIC_MUST_HAVE_LEADER_REPLICAS_ON_BROKERS
MIN_LEADER = ["MinTopicLeadersPerBrokerGoal"]


def decks():
    out = []
    # TEST DECK #3 / #4: capacity thresholds on the small and medium clusters (:152-170)
    for model in ("smallClusterModel", "mediumClusterModel"):
        for cap in (HIGH_CAP, MEDIUM_CAP, LOW_CAP):
            out.append((f"deck34-{model}-cap{cap}", model, DECK_GOALS, deck_constraint(MEDIUM_BALANCE, cap)))
    # TEST DECK #5: broker capacities; the constraint is the last one of deck #4 (:172-197)
    for size in ("LARGE", "MEDIUM", "SMALL"):
        for model in ("smallClusterModel", "mediumClusterModel"):
            out.append((f"deck5-{model}-{size}", f"{model}_{size}", DECK_GOALS, deck_constraint(MEDIUM_BALANCE, LOW_CAP)))
    # TEST DECK #1 / #2: balance percentages with topics.with.min.leaders.per.broker = T2 (small) / A (medium)
    # (:133-150)
    for model, topic in (("smallClusterModel", "T2"), ("mediumClusterModel", "A")):
        for bal in (HIGH_BALANCE, MEDIUM_BALANCE, LOW_BALANCE):
            out.append((f"deck12-{model}-bal{bal}", model, DECK_GOALS, deck_constraint(bal, MEDIUM_CAP, topic)))
    # MinTopicLeadersPerBrokerGoal decks (:217-253); leaderReplicaPerBrokerUnsatisfiable expects the failure
    must = deck_constraint(min_leader_topics=TOPIC_MUST)
    out.append(("minLeader-satisfiable", "minLeaderReplicaPerBrokerSatisfiable", MIN_LEADER, must))
    out.append(("minLeader-satisfiable2", "minLeaderReplicaPerBrokerSatisfiable2", MIN_LEADER, must))
    out.append(("minLeader-unsatisfiable", "leaderReplicaPerBrokerUnsatisfiable", MIN_LEADER, must, None, True))
    # satisfiable3 sets only min.topic.leaders.per.broker = 4 (the topic pattern stays empty) (:232-235)
    out.append(("minLeader-satisfiable3", "minLeaderReplicaPerBrokerSatisfiable3", MIN_LEADER,
                deck_constraint(min_leaders=4)))
    out.append(("minLeader-satisfiable4", "minLeaderReplicaPerBrokerSatisfiable4", MIN_LEADER,
                deck_constraint(min_leader_topics=r"topic\d", min_leaders=1)))
    out.append(("minLeader-satisfiable5", "minLeaderReplicaPerBrokerSatisfiable5", MIN_LEADER,
                deck_constraint(min_leader_topics=r"topic\d", min_leaders=0)))
    # the remaining DeterministicCluster models with the whole deck list
    for model in ("unbalanced", "unbalanced2", "unbalancedWithAFollower", "rackAwareSatisfiable",
                  "rackAwareSatisfiable2", "deadBroker"):
        out.append((f"model-{model}", model, DECK_GOALS, deck_constraint(MEDIUM_BALANCE, MEDIUM_CAP)))
    # three replicas of one partition on two racks: RackAwareGoal must fail (RackAwareGoal.java:112-121)
    out.append(("model-rackAwareUnsatisfiable", "rackAwareUnsatisfiable", DECK_GOALS,
                deck_constraint(MEDIUM_BALANCE, MEDIUM_CAP), "Insufficient number of racks"))
    # Kafka-assigner decks (:200-215): verifications BROKEN_BROKERS and REGRESSION, the constraint of deck #5;
    # rackAwareUnsatisfiable expects the OptimizationFailureException
    ka = ["KafkaAssignerEvenRackAwareGoal", "KafkaAssignerDiskUsageDistributionGoal"]
    for model in ("smallClusterModel", "mediumClusterModel", "rackAwareSatisfiable"):
        out.append((f"kafkaAssigner-{model}", model, ka, deck_constraint(MEDIUM_BALANCE, LOW_CAP)))
    out.append(("kafkaAssigner-rackAwareUnsatisfiable", "rackAwareUnsatisfiable", ka,
                deck_constraint(MEDIUM_BALANCE, LOW_CAP), None, True))
    out.append(("deadBroker-default-goals", "deadBroker", list(ccmi.DEFAULT_GOALS), ccmi.BalancingConstraint()))
    out.append(("deadBroker-soft-goals", "deadBroker", list(ccmi.C1_GOALS), ccmi.BalancingConstraint()))
    return out


def _deck(d):
    """(id, model, goals, constraint, allowed failure message, OptimizationFailureException expected)"""
    d = tuple(d) + (None, False)[len(d) - 4:]
    return d[:4] + (d[4] or "Insufficient capacity for", d[5])


DECKS = [_deck(d) for d in decks()]
DECK_IDS = [d[0] for d in DECKS]


def run_verified(runner, model_name, goals, bc, allowed_failure="Insufficient capacity for", expect_failure=False):
    """executeGoalsFor + the DeterministicClusterTest.test() acceptance rule (an OptimizationFailureException is a
    pass only with the allowed message, or whenever the deck expects it), on `runner` (oracle or product)."""
    m = deterministic_models()[model_name]
    flat = build_model(m)
    pre, res, err = runner(flat, goals, bc)
    if expect_failure:
        assert isinstance(err, ccmi.OptimizationFailureException), err
        return flat, None
    if err is not None:
        assert isinstance(err, ccmi.OptimizationFailureException) and allowed_failure in str(err), err
        return flat, None
    final, proposals, goal_results = res
    problems = []
    if m["dead"]:  # BROKEN_BROKERS (OptimizationVerifier.java:185-201): with dead brokers, and the soft-goal rule
        problems += [verify_broken_brokers(m["dead"], final),
                     verify_soft_goal_replica_movements(proposals, offline_replicas(flat, m), goals)]
    else:  # REGRESSION applies when no replica is self-healing eligible
        problems.append(verify_regression(goal_results, pre, bc))
    problems = [p for p in problems if p]
    assert not problems, problems
    return flat, res


def oracle_runner(flat, goals, bc):
    oc = OracleCluster.from_desc(flat.desc)
    pre = oc.stats(bc)
    try:
        res = oc.optimize(goals, bc)
    except ccmi.CruiseControlError as e:
        return pre, None, e
    return pre, (oc.replica_distribution(), oc.proposals(), res), None


def product_runner(lib):
    def run(flat, goals, bc):
        cm = ccmi.ClusterModel(flat.desc, device=0, lib=lib, keepalive=flat)
        pre = cm.cluster_stats(bc)
        try:
            res = ccmi.GoalOptimizer(bc).optimizations(cm, ccmi.goals_from_names(goals))
        except ccmi.CruiseControlError as e:
            return pre, None, e
        return pre, (cm.replica_distribution(), res.proposals, res.goal_results), None
    return run


@pytest.mark.parametrize("deck", DECKS, ids=DECK_IDS)
def test_oracle_passes_deterministic_deck(oracle_lib, deck):
    _, model, goals, bc, allowed, expect = deck
    run_verified(oracle_runner, model, goals, bc, allowed, expect)


# RackAwareGoalTest.goalNames (:57-61): the test runs for both rack goals
RACK_GOALS = ["RackAwareDistributionGoal", "RackAwareGoal"]


def _rack_mapper_proposals(runner_lib, mapped, goal):
    m = deterministic_models()["rackIdMapper" if mapped else "withoutRackIdMapper"]
    flat = build_model(m)
    if runner_lib is None:
        oc = OracleCluster.from_desc(flat.desc)
        oc.optimize([goal], ccmi.BalancingConstraint())
        return oc.proposals()
    cm = ccmi.ClusterModel(flat.desc, device=0, lib=runner_lib, keepalive=flat)
    return ccmi.GoalOptimizer().optimizations(cm, [getattr(ccmi, goal)()]).proposals


def check_rack_mapper_kat(runner_lib, goal):
    """RackAwareGoalTest.testRackIdMapper (:74-130) / testWithoutRackIdMapper (:137-178)."""
    assert _rack_mapper_proposals(runner_lib, False, goal) == []
    props = _rack_mapper_proposals(runner_lib, True, goal)
    assert len(props) == 1
    p = props[0]
    assert p.partition == 0
    assert set(p.old_replicas) - set(p.new_replicas) & {0, 1}
    assert set(p.new_replicas) - set(p.old_replicas) == {2}


@pytest.mark.parametrize("goal", RACK_GOALS)
def test_oracle_rack_id_mapper_kat(oracle_lib, goal):
    check_rack_mapper_kat(None, goal)


@pytest.mark.parametrize("deck", DECKS, ids=DECK_IDS)
def test_emu_deterministic_deck_matches_oracle(emu_lib, oracle_lib, deck):
    """The engine's host logic (test-only sequential Device emulation): the same deck passes and matches the oracle
    bit for bit."""
    _, model, goals, bc, allowed, expect = deck
    run_verified(product_runner(emu_lib), model, goals, bc, allowed, expect)
    flat = build_model(deterministic_models()[model])
    check_desc_against_oracle(emu_lib, flat.desc, flat, goals, bc)


@pytest.mark.parametrize("goal", RACK_GOALS)
def test_emu_rack_id_mapper_kat(emu_lib, goal):
    check_rack_mapper_kat(emu_lib, goal)


@pytest.mark.gpu
@pytest.mark.parametrize("deck", DECKS, ids=DECK_IDS)
def test_gpu_deterministic_deck_matches_oracle(gpu_lib, oracle_lib, deck):
    _, model, goals, bc, allowed, expect = deck
    run_verified(product_runner(gpu_lib), model, goals, bc, allowed, expect)
    flat = build_model(deterministic_models()[model])
    check_desc_against_oracle(gpu_lib, flat.desc, flat, goals, bc)


@pytest.mark.gpu
@pytest.mark.parametrize("goal", RACK_GOALS)
def test_gpu_rack_id_mapper_kat(gpu_lib, goal):
    check_rack_mapper_kat(gpu_lib, goal)
