"""Known-answer tests transcribed from the reference's single-goal exclusion suites, run on the transcribed
DeterministicCluster models (tests/golden/deterministic_clusters.json):

* analyzer/ExcludedBrokersForLeadershipTest.java:96-262 (data) and :265-300 (test)
* analyzer/ExcludedBrokersForReplicaMoveTest.java:112-250 (data) and :253-292 (test)

Each row: goal, excluded brokers, expected exception (OptimizationFailureException or none), model, dead brokers,
expected Goal.optimize() return value, and (replica-move suite) whether proposals are expected. The goal is built
by AnalyzerUnitTestUtils.goal (AnalyzerUnitTestUtils.java:28-46): max.replicas.per.broker 5, topic replica balance
1.2, resource balance 1.05, capacity threshold 0.8; options = OptimizationOptions(∅, excluded..., ∅) (fast mode on;
the engine never cuts a loop short, see include/ccmi.h). Rows whose goal this build does not implement, or whose
model needs JBOD disks (unbalanced4/5), are reported as skipped with the reason.
"""
import pytest

import ccmi
from oracle_binding import OracleCluster
from parity import check_desc_against_oracle
from verifier import build_model, deterministic_models

ALL3 = [0, 1, 2]  # RACK_BY_BROKER.keySet()
MIN_LEADER = "MinTopicLeadersPerBrokerGoal"
# topics.with.min.leaders.per.broker = TestConstants.TOPIC_MUST_HAVE_LEADER_REPLICAS_ON_BROKERS (configOverrides)
MUST = {"topics_with_min_leaders_per_broker": "must_have_leader_replica_on_broker_topic"}
SAT, SAT2 = "minLeaderReplicaPerBrokerSatisfiable", "minLeaderReplicaPerBrokerSatisfiable2"
UNSAT, LUNSAT = "minLeaderReplicaPerBrokerUnsatisfiable", "leaderReplicaPerBrokerUnsatisfiable"
OFE = "OptimizationFailureException"

# (suite, tid, goal, excluded, exception, model, dead, expected_optimized, expected_proposals)
LEADERSHIP = [
    ("RackAwareGoal", [1], None, "rackAwareSatisfiable", [], True),
    ("RackAwareGoal", [1], None, "rackAwareSatisfiable", [0], True),
    ("RackAwareGoal", [], None, "rackAwareSatisfiable", [], True),
    ("RackAwareGoal", [], None, "rackAwareSatisfiable", [0], True),
    ("RackAwareGoal", [1], "OptimizationFailureException", "rackAwareUnsatisfiable", [], None),
    ("RackAwareGoal", [1], "OptimizationFailureException", "rackAwareUnsatisfiable", [0], None),
    ("RackAwareDistributionGoal", [1], None, "rackAwareSatisfiable", [], True),
    ("RackAwareDistributionGoal", [1], None, "rackAwareSatisfiable", [0], True),
    ("RackAwareDistributionGoal", [], None, "rackAwareSatisfiable", [], True),
    ("RackAwareDistributionGoal", [], None, "rackAwareSatisfiable", [0], True),
    ("RackAwareDistributionGoal", [1], None, "rackAwareUnsatisfiable", [], True),
    ("RackAwareDistributionGoal", [1], "OptimizationFailureException", "rackAwareUnsatisfiable", [0], None),
    ("ReplicaCapacityGoal", [1], None, "unbalanced", [], True),
    ("ReplicaCapacityGoal", [1], None, "unbalanced", [0], True),
    ("ReplicaCapacityGoal", ALL3, None, "unbalanced", [], True),
    ("ReplicaCapacityGoal", ALL3, "OptimizationFailureException", "unbalanced", [0], None),
] + [row for g in ("CpuCapacityGoal", "DiskCapacityGoal", "NetworkInboundCapacityGoal", "NetworkOutboundCapacityGoal")
     for row in [(g, [1], None, "unbalanced", [], True),
                 (g, [1], "OptimizationFailureException", "unbalanced", [0], None),
                 (g, ALL3, "OptimizationFailureException", "unbalanced", [], None),
                 (g, ALL3, "OptimizationFailureException", "unbalanced", [0], None)]] + \
    [row for g in ("DiskUsageDistributionGoal", "NetworkInboundUsageDistributionGoal",
                   "NetworkOutboundUsageDistributionGoal", "CpuUsageDistributionGoal")
     for row in [(g, [1], None, "unbalanced", [], False),
                 (g, [1], None, "unbalanced", [0], False),
                 (g, ALL3, None, "unbalanced", [], False),
                 (g, ALL3, "OptimizationFailureException", "unbalanced", [0], None)]] + [
    ("LeaderBytesInDistributionGoal", [1], None, "unbalanced", [], False),
    ("LeaderBytesInDistributionGoal", [1], None, "unbalanced", [0], False),
    ("LeaderBytesInDistributionGoal", ALL3, None, "unbalanced", [], False),
    ("LeaderBytesInDistributionGoal", ALL3, None, "unbalanced", [0], False),
    ("PotentialNwOutGoal", [1], None, "unbalanced", [], True),
    ("PotentialNwOutGoal", [1], None, "unbalanced", [0], False),
    ("PotentialNwOutGoal", ALL3, None, "unbalanced", [], False),
    ("PotentialNwOutGoal", ALL3, "OptimizationFailureException", "unbalanced", [0], None),
    ("TopicReplicaDistributionGoal", [1], None, "unbalanced", [], True),
    ("TopicReplicaDistributionGoal", [1], None, "unbalanced", [0], True),
    ("TopicReplicaDistributionGoal", ALL3, None, "unbalanced", [], True),
    ("TopicReplicaDistributionGoal", ALL3, "OptimizationFailureException", "unbalanced", [0], None),
    ("ReplicaDistributionGoal", [1], None, "unbalanced2", [], True),
    ("ReplicaDistributionGoal", [1], None, "unbalanced2", [0], False),
    ("ReplicaDistributionGoal", ALL3, None, "unbalanced2", [], False),
    ("ReplicaDistributionGoal", ALL3, "OptimizationFailureException", "unbalanced2", [0], None),
    ("LeaderReplicaDistributionGoal", [1], None, "unbalanced3", [], True),
    ("LeaderReplicaDistributionGoal", [0], None, "unbalanced3", [], True),
    ("LeaderReplicaDistributionGoal", ALL3, None, "unbalanced3", [], False),
    ("LeaderReplicaDistributionGoal", [], None, "unbalanced3", [0], True),
    ("PreferredLeaderElectionGoal", [], None, "unbalanced3", [], True),
    ("PreferredLeaderElectionGoal", [1], None, "unbalanced3", [], False),
    ("PreferredLeaderElectionGoal", ALL3, None, "unbalanced3", [], False),
] + [
    # ExcludedBrokersForLeadershipTest.java:151-192 (MinTopicLeadersPerBrokerGoal with the must-have topic)
    (MIN_LEADER, [1], None, SAT, [], True, MUST), (MIN_LEADER, [1], None, SAT2, [], True, MUST),
    (MIN_LEADER, [], OFE, UNSAT, [], None, MUST), (MIN_LEADER, [0], OFE, UNSAT, [], None, MUST),
    (MIN_LEADER, [0, 1], None, UNSAT, [], True, MUST),
    (MIN_LEADER, [1], OFE, SAT, [0], False, MUST), (MIN_LEADER, [1], OFE, SAT2, [0], False, MUST),
    (MIN_LEADER, [1], OFE, LUNSAT, [0], True, MUST),
    (MIN_LEADER, [], None, SAT, [], True, MUST), (MIN_LEADER, [], None, SAT2, [], True, MUST),
    (MIN_LEADER, [], None, SAT, [0], True, MUST), (MIN_LEADER, [], None, SAT2, [0], True, MUST),
    (MIN_LEADER, [], None, LUNSAT, [0], True, MUST),
]
# ExcludedBrokersForLeadershipTest.java:148-174 (the PotentialNwOutGoal rows) are the "PotentialNwOutGoal" rows above;
# its BrokerSetAwareGoal rows (:247-261) are in test_broker_set.py.

REPLICA_MOVE = [
    ("RackAwareGoal", [1], None, "rackAwareSatisfiable", [], True, True),
    ("RackAwareGoal", [2], "OptimizationFailureException", "rackAwareSatisfiable", [], None, None),
    ("RackAwareGoal", [2], "OptimizationFailureException", "rackAwareSatisfiable", [0], None, None),
    ("RackAwareGoal", [], None, "rackAwareSatisfiable", [], True, True),
    ("RackAwareGoal", [], None, "rackAwareSatisfiable", [0], True, True),
    ("RackAwareGoal", [1], "OptimizationFailureException", "rackAwareUnsatisfiable", [], None, None),
    ("RackAwareGoal", [1], "OptimizationFailureException", "rackAwareUnsatisfiable", [0], None, None),
    ("RackAwareDistributionGoal", [1], None, "rackAwareSatisfiable", [], True, True),
    ("RackAwareDistributionGoal", [2], None, "rackAwareSatisfiable", [], True, False),
    ("RackAwareDistributionGoal", [2], "OptimizationFailureException", "rackAwareSatisfiable", [0], None, None),
    ("RackAwareDistributionGoal", [], None, "rackAwareSatisfiable", [], True, True),
    ("RackAwareDistributionGoal", [], None, "rackAwareSatisfiable", [0], True, True),
    ("RackAwareDistributionGoal", [1], None, "rackAwareUnsatisfiable", [], True, False),
    ("RackAwareDistributionGoal", [1], "OptimizationFailureException", "rackAwareUnsatisfiable", [0], None, None),
    ("RackAwareDistributionGoal", [0], None, "rackAwareSatisfiable2", [], True, True),
    ("ReplicaCapacityGoal", [1], None, "unbalanced", [], True, False),
    ("ReplicaCapacityGoal", [1], None, "unbalanced", [0], True, True),
    ("ReplicaCapacityGoal", ALL3, "OptimizationFailureException", "unbalanced", [], None, None),
    ("ReplicaCapacityGoal", ALL3, "OptimizationFailureException", "unbalanced", [0], None, None),
] + [row for g in ("CpuCapacityGoal", "DiskCapacityGoal", "NetworkInboundCapacityGoal", "NetworkOutboundCapacityGoal")
     for row in [(g, [1], None, "unbalanced", [], True, True),
                 (g, [1], "OptimizationFailureException", "unbalanced", [0], None, None),
                 (g, ALL3, "OptimizationFailureException", "unbalanced", [], None, None),
                 (g, ALL3, "OptimizationFailureException", "unbalanced", [0], None, None),
                 (g, [1], "OptimizationFailureException", "unbalanced2", [], None, None)]] + \
    [row for g in ("DiskUsageDistributionGoal", "NetworkInboundUsageDistributionGoal",
                   "NetworkOutboundUsageDistributionGoal", "CpuUsageDistributionGoal")
     for row in [(g, [1], None, "unbalanced", [], True, True),
                 (g, [1], None, "unbalanced", [0], True, True),
                 (g, ALL3, "OptimizationFailureException", "unbalanced", [], None, None),
                 (g, ALL3, "OptimizationFailureException", "unbalanced", [0], None, None)]] + [
    ("LeaderBytesInDistributionGoal", [1], None, "unbalanced", [], False, False),
    ("LeaderBytesInDistributionGoal", [1], None, "unbalanced", [0], False, False),
    ("LeaderBytesInDistributionGoal", ALL3, "OptimizationFailureException", "unbalanced", [], None, None),
    ("LeaderBytesInDistributionGoal", ALL3, "OptimizationFailureException", "unbalanced", [0], None, None),
    ("LeaderBytesInDistributionGoal", [1], None, "unbalancedWithAFollower", [], True, True),
    ("PotentialNwOutGoal", [1], None, "unbalanced", [], True, True),
    ("PotentialNwOutGoal", [1], None, "unbalanced", [0], False, True),
    ("PotentialNwOutGoal", ALL3, None, "unbalanced", [], False, False),
    ("PotentialNwOutGoal", ALL3, "OptimizationFailureException", "unbalanced", [0], None, None),
    ("TopicReplicaDistributionGoal", [1], None, "unbalanced5", [], True, True),
    ("TopicReplicaDistributionGoal", [1], None, "unbalanced", [0], True, True),
    ("TopicReplicaDistributionGoal", ALL3, "OptimizationFailureException", "unbalanced4", [], None, None),
    ("TopicReplicaDistributionGoal", ALL3, "OptimizationFailureException", "unbalanced4", [0], None, None),
    ("ReplicaDistributionGoal", [1], None, "unbalanced2", [], True, True),
    ("ReplicaDistributionGoal", [1], None, "unbalanced2", [0], True, True),
    ("ReplicaDistributionGoal", ALL3, "OptimizationFailureException", "unbalanced2", [], None, None),
    ("ReplicaDistributionGoal", ALL3, "OptimizationFailureException", "unbalanced2", [0], None, None),
    ("ReplicaDistributionGoal", [1, 2], None, "unbalanced2", [], True, True),
    ("LeaderReplicaDistributionGoal", [1], None, "unbalanced3", [], True, False),
    ("LeaderReplicaDistributionGoal", [1], None, "unbalanced3", [0], False, True),
    ("LeaderReplicaDistributionGoal", ALL3, "OptimizationFailureException", "unbalanced3", [], None, None),
    ("LeaderReplicaDistributionGoal", [2], "OptimizationFailureException", "unbalanced3", [0], None, None),
    ("LeaderReplicaDistributionGoal", [0], None, "unbalanced3", [1], False, True),
] + [
    # ExcludedBrokersForReplicaMoveTest.java:226-271 (MinTopicLeadersPerBrokerGoal with the must-have topic)
    (MIN_LEADER, [], None, SAT, [], True, True, MUST), (MIN_LEADER, [], None, SAT2, [], True, True, MUST),
    (MIN_LEADER, [1], None, SAT, [], True, True, MUST), (MIN_LEADER, [1], None, SAT2, [], True, True, MUST),
    (MIN_LEADER, [2], None, SAT, [], True, False, MUST), (MIN_LEADER, [2], None, SAT2, [], True, True, MUST),
    (MIN_LEADER, [], None, SAT, [0], True, True, MUST), (MIN_LEADER, [], None, SAT2, [0], True, True, MUST),
    (MIN_LEADER, [], None, SAT, [2], True, True, MUST), (MIN_LEADER, [], None, SAT2, [2], True, True, MUST),
    (MIN_LEADER, [1], OFE, SAT, [2], None, None, MUST), (MIN_LEADER, [1], OFE, SAT2, [2], None, None, MUST),
    (MIN_LEADER, [0], OFE, SAT, [2], None, None, MUST), (MIN_LEADER, [0], None, SAT2, [2], True, True, MUST),
]


def goal_constraint(overrides=None):
    """AnalyzerUnitTestUtils.goal (AnalyzerUnitTestUtils.java:28-37) with the row's config overrides."""
    bc = ccmi.BalancingConstraint()
    for k, v in (overrides or {}).items():
        setattr(bc, k, v)
    bc.max_replicas_per_broker = 5
    bc.topic_replica_balance_percentage = 1.2
    bc.set_resource_balance_percentage(1.05)
    bc.set_capacity_threshold(0.8)
    return bc


def _rows(suite):
    out = []
    for i, row in enumerate(LEADERSHIP if suite == "leadership" else REPLICA_MOVE):
        over = row[-1] if isinstance(row[-1], dict) else None
        if over is not None:
            row = row[:-1]
        goal, excl, exc, model, dead, opt = row[:6]
        props = row[6] if len(row) > 6 else None
        marks = []
        if goal not in ccmi.GOAL_KINDS:
            marks.append(pytest.mark.skip(reason=f"{goal} is not in this build"))
        elif model not in deterministic_models():
            marks.append(pytest.mark.skip(reason=f"{model} is a JBOD model (logdirs)"))
        out.append(pytest.param(suite, goal, excl, exc, model, dead, opt, props, over, marks=marks,
                                id=f"{suite}-{i}-{goal}-{model}-x{''.join(map(str, excl))}-d{''.join(map(str, dead))}"))
    return out


CASES = _rows("leadership") + _rows("replica_move")


def _model(model, dead):
    m = dict(deterministic_models()[model])
    m["dead"] = sorted(set(m["dead"]) | set(dead))
    return build_model(m)


def _options(suite, excl):
    if suite == "leadership":
        return ccmi.OptimizationOptions(excluded_brokers_for_leadership=excl)
    return ccmi.OptimizationOptions(excluded_brokers_for_replica_move=excl)


def run_case(runner, suite, goal, excl, exc, model, dead, opt, props, over=None):
    """ExcludedBrokersFor{Leadership,ReplicaMove}Test.test(): returns (succeeded, proposals) or raises."""
    flat = _model(model, dead)
    opts = _options(suite, excl)
    bc = goal_constraint(over)
    if exc is not None:
        with pytest.raises(getattr(ccmi, exc)) as ei:
            runner(flat, goal, opts, bc)
        assert ei.value.provision.status == "UNDER_PROVISIONED"  # (:375 / :422)
        return
    succeeded, proposals, provision = runner(flat, goal, opts, bc)
    assert succeeded == opt
    assert provision.status != "UNDER_PROVISIONED"  # the cluster cannot be under-provisioned (:357 / :404)
    if excl and suite == "leadership":
        # no leadership move from an online replica to a broker excluded for leadership
        for p in proposals:
            if p.new_replicas[0] != p.old_leader and p.new_replicas[0] in excl:
                assert p.old_leader in dead, p
    if excl and suite == "replica_move":
        assert bool(proposals) == props
        for p in proposals:
            assert not (set(p.new_replicas) - set(p.old_replicas)) & set(excl), p


def oracle_runner(flat, goal, opts, bc):
    oc = OracleCluster.from_desc(flat.desc)
    res = oc.optimize([goal], bc, opts)
    return res[0].succeeded, oc.proposals(), res[0].provision


def product_runner(lib):
    def run(flat, goal, opts, bc):
        cm = ccmi.ClusterModel(flat.desc, device=0, lib=lib, keepalive=flat)
        g = getattr(ccmi, goal)(constraint=bc)
        ok = g.optimize(cm, set(), opts)
        return ok, cm.proposals(), g.provision
    return run


@pytest.mark.parametrize("suite,goal,excl,exc,model,dead,opt,props,over", CASES)
def test_oracle_excluded_brokers_kat(oracle_lib, suite, goal, excl, exc, model, dead, opt, props, over):
    run_case(oracle_runner, suite, goal, excl, exc, model, dead, opt, props, over)


@pytest.mark.parametrize("suite,goal,excl,exc,model,dead,opt,props,over", CASES)
def test_emu_excluded_brokers_kat(emu_lib, suite, goal, excl, exc, model, dead, opt, props, over):
    run_case(product_runner(emu_lib), suite, goal, excl, exc, model, dead, opt, props, over)


@pytest.mark.gpu
@pytest.mark.parametrize("suite,goal,excl,exc,model,dead,opt,props,over", CASES)
def test_gpu_excluded_brokers_kat(gpu_lib, suite, goal, excl, exc, model, dead, opt, props, over):
    run_case(product_runner(gpu_lib), suite, goal, excl, exc, model, dead, opt, props, over)


@pytest.mark.parametrize("suite,goal,excl,exc,model,dead,opt,props,over", CASES)
def test_emu_excluded_brokers_matches_oracle(emu_lib, oracle_lib, suite, goal, excl, exc, model, dead, opt, props,
                                             over):
    """Move for move (or the same exception, message, action log and recommendation) against the oracle."""
    flat = _model(model, dead)
    check_desc_against_oracle(emu_lib, flat.desc, flat, [goal], goal_constraint(over), _options(suite, excl))


@pytest.mark.gpu
@pytest.mark.parametrize("suite,goal,excl,exc,model,dead,opt,props,over", CASES)
def test_gpu_excluded_brokers_matches_oracle(gpu_lib, oracle_lib, suite, goal, excl, exc, model, dead, opt, props,
                                             over):
    flat = _model(model, dead)
    check_desc_against_oracle(gpu_lib, flat.desc, flat, [goal], goal_constraint(over), _options(suite, excl))
