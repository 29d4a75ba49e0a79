"""Known-answer tests transcribed from the reference's excluded-topics suite, run on the transcribed DeterministicCluster
models (tests/golden/deterministic_clusters.json):

* analyzer/ExcludedTopicsTest.java:117-323 (data) and :325-365 (test)

Each row: goal, excluded topics, expected exception (OptimizationFailureException or none), model, dead brokers,
expected Goal.optimize() return value, and whether proposals are expected (checked when topics are excluded, as the
reference does). A proposal of an excluded topic may only take replicas off dead brokers. Goals are built by
AnalyzerUnitTestUtils.goal (max.replicas.per.broker 5, topic replica balance 1.2, resource balance 1.05, capacity
threshold 0.8), with the row's config overrides. Rows whose goal this build does not implement are reported as skipped.

The product (CPU emulation, and gfx950 under -m gpu) must also equal the oracle move for move on every row.
"""
import pytest

import ccmi
from oracle_binding import OracleCluster
from parity import check_desc_against_oracle
from test_excluded_brokers import goal_constraint
from verifier import build_model, deterministic_models

T1, T2 = "T1", "T2"
TOPIC0, TOPIC1 = "topic0", "topic1"  # TestConstants.TOPIC0 / TOPIC1
MIN_GAP_40 = {"topic_replica_balance_min_gap": 40}
TOPIC_MUST = "must_have_leader_replica_on_broker_topic"  # TestConstants.TOPIC_MUST_HAVE_LEADER_REPLICAS_ON_BROKERS
MIN_LEADERS = {"topics_with_min_leaders_per_broker": TOPIC_MUST}

# (goal, excluded, exception, model, dead, expected_optimized, expected_proposals, constraint overrides)
ROWS = [
    ("RackAwareGoal", [T1], None, "rackAwareSatisfiable", [], True, False),
    ("RackAwareGoal", [T1], None, "rackAwareSatisfiable", [0], True, True),
    ("RackAwareGoal", [], None, "rackAwareSatisfiable", [], True, True),
    ("RackAwareGoal", [], None, "rackAwareSatisfiable", [0], True, True),
    ("RackAwareGoal", [T1], None, "rackAwareUnsatisfiable", [], True, False),
    ("RackAwareGoal", [T1], "OptimizationFailureException", "rackAwareUnsatisfiable", [0], None, None),
    ("RackAwareGoal", [], "OptimizationFailureException", "rackAwareUnsatisfiable", [], None, None),
    ("RackAwareGoal", [], "OptimizationFailureException", "rackAwareUnsatisfiable", [0], None, None),
    ("RackAwareDistributionGoal", [T1], None, "rackAwareSatisfiable", [], True, False),
    ("RackAwareDistributionGoal", [T1], None, "rackAwareSatisfiable", [0], True, True),
    ("RackAwareDistributionGoal", [], None, "rackAwareSatisfiable", [], True, True),
    ("RackAwareDistributionGoal", [], None, "rackAwareSatisfiable", [0], True, True),
    ("RackAwareDistributionGoal", [T1], None, "rackAwareUnsatisfiable", [], True, False),
    ("RackAwareDistributionGoal", [T1], "OptimizationFailureException", "rackAwareUnsatisfiable", [0], None, None),
    ("RackAwareDistributionGoal", [], None, "rackAwareUnsatisfiable", [], True, True),
    ("RackAwareDistributionGoal", [], "OptimizationFailureException", "rackAwareUnsatisfiable", [0], None, None),
    ("ReplicaCapacityGoal", [T1], None, "unbalanced", [], True, False),
    ("ReplicaCapacityGoal", [T1], None, "unbalanced", [0], True, True),
    ("ReplicaCapacityGoal", [T1, T2], None, "unbalanced", [], True, False),
    ("ReplicaCapacityGoal", [T1, T2], None, "unbalanced", [0], True, True),
] + [row for g in ("CpuCapacityGoal", "DiskCapacityGoal", "NetworkInboundCapacityGoal", "NetworkOutboundCapacityGoal")
     for row in [(g, [T1], None, "unbalanced", [], True, True),
                 (g, [T1], None, "unbalanced", [0], True, True),
                 (g, [T1, T2], "OptimizationFailureException", "unbalanced", [], None, None),
                 (g, [T1, T2], None, "unbalanced", [0], True, True)]] + \
    [row for g in ("DiskUsageDistributionGoal", "NetworkInboundUsageDistributionGoal",
                   "NetworkOutboundUsageDistributionGoal", "CpuUsageDistributionGoal")
     for row in [(g, [T1], None, "unbalanced", [], False, False),
                 (g, [T1], None, "unbalanced", [0], True, True),
                 (g, [T1, T2], None, "unbalanced", [], False, False),
                 (g, [T1, T2], None, "unbalanced", [0], True, True)]] + [
    ("LeaderBytesInDistributionGoal", [T1], None, "unbalanced", [], False, False),
    ("LeaderBytesInDistributionGoal", [T1], None, "unbalanced", [0], False, False),
    ("LeaderBytesInDistributionGoal", [T1, T2], None, "unbalanced", [], False, False),
    ("LeaderBytesInDistributionGoal", [T1, T2], None, "unbalanced", [0], False, False),
    ("PotentialNwOutGoal", [T1], None, "unbalanced", [], True, True),
    ("PotentialNwOutGoal", [T1], None, "unbalanced", [0], True, True),
    ("PotentialNwOutGoal", [T1, T2], None, "unbalanced", [], False, False),
    ("PotentialNwOutGoal", [T1, T2], None, "unbalanced", [0], True, True),
    ("TopicReplicaDistributionGoal", [T1], None, "unbalanced5", [], True, False, MIN_GAP_40),
    ("TopicReplicaDistributionGoal", [T1], None, "unbalanced", [0], True, True),
    ("TopicReplicaDistributionGoal", [T1, T2], None, "unbalanced", [], True, False),
    ("TopicReplicaDistributionGoal", [T1, T2], None, "unbalanced", [0], True, True),
    ("TopicReplicaDistributionGoal", [T1], None, "unbalanced5", [], True, True),
    ("ReplicaDistributionGoal", [T1], None, "unbalanced2", [], True, True),
    ("ReplicaDistributionGoal", [T1], None, "unbalanced2", [0], True, True),
    ("ReplicaDistributionGoal", [T1, T2], None, "unbalanced2", [], False, False),
    ("ReplicaDistributionGoal", [T1, T2], None, "unbalanced2", [0], True, True),
    ("LeaderReplicaDistributionGoal", [], None, "unbalanced3", [], True, True),
    ("LeaderReplicaDistributionGoal", [T1], None, "unbalanced3", [], True, True),
    ("LeaderReplicaDistributionGoal", [T1, T2], None, "unbalanced3", [], False, False),
    ("LeaderReplicaDistributionGoal", [], None, "unbalanced3", [0], True, True),
    # ExcludedTopicsTest.java:171-182: topics.with.min.leaders.per.broker = the must-have topic; excluding an unrelated
    # topic optimizes, excluding the must-have topic is a config error
    ("MinTopicLeadersPerBrokerGoal", [T1], None, "minLeaderReplicaPerBrokerSatisfiable", [], True, True, MIN_LEADERS),
    ("MinTopicLeadersPerBrokerGoal", [TOPIC_MUST], "OptimizationFailureException",
     "minLeaderReplicaPerBrokerSatisfiable", [], None, None, MIN_LEADERS),
    # ExcludedTopicsTest.java:278-302
    ("KafkaAssignerEvenRackAwareGoal", [T1], None, "rackAwareSatisfiable", [], True, False),
    ("KafkaAssignerEvenRackAwareGoal", [T1], None, "rackAwareSatisfiable", [0], True, True),
    ("KafkaAssignerEvenRackAwareGoal", [], None, "rackAwareSatisfiable", [], True, True),
    ("KafkaAssignerEvenRackAwareGoal", [], None, "rackAwareSatisfiable", [0], True, True),
    ("KafkaAssignerEvenRackAwareGoal", [T1], None, "rackAwareUnsatisfiable", [], True, False),
    ("KafkaAssignerEvenRackAwareGoal", [T1], "OptimizationFailureException", "rackAwareUnsatisfiable", [0], None, None),
    ("KafkaAssignerEvenRackAwareGoal", [], "OptimizationFailureException", "rackAwareUnsatisfiable", [], None, None),
    ("KafkaAssignerEvenRackAwareGoal", [], "OptimizationFailureException", "rackAwareUnsatisfiable", [0], None, None),
]
# The BrokerSetAwareGoal rows (:304-320) are in test_broker_set.py.


def _cases():
    out = []
    for i, row in enumerate(ROWS):
        goal, excl, exc, model, dead, opt, props = row[:7]
        over = row[7] if len(row) > 7 else {}
        marks = []
        if goal not in ccmi.GOAL_KINDS:
            marks.append(pytest.mark.skip(reason=f"{goal} is not in this build"))
        out.append(pytest.param(goal, excl, exc, model, dead, opt, props, over, marks=marks,
                                id=f"{i}-{goal}-{model}-x{'+'.join(excl) or 'none'}-d{''.join(map(str, dead))}"))
    return out


CASES = _cases()


def _model(model, dead):
    m = dict(deterministic_models()[model])
    m["dead"] = sorted(set(m["dead"]) | set(dead))
    return build_model(m)


def _constraint(over):
    bc = goal_constraint()
    for k, v in over.items():
        setattr(bc, k, v)
    return bc


def _options(flat, excl):
    # a name the cluster does not have matches nothing (Set<String>.contains)
    idx = [flat.topics.index(t) for t in excl if t in flat.topics]
    return ccmi.OptimizationOptions(excluded_topics=idx)


def run_case(runner, goal, excl, exc, model, dead, opt, props, over):
    """ExcludedTopicsTest.test(): the goal's optimize() result, and no proposal that moves an excluded topic's
    replica off an alive broker."""
    flat = _model(model, dead)
    opts = _options(flat, excl)
    if exc is not None:
        with pytest.raises(getattr(ccmi, exc)) as ei:
            runner(flat, goal, opts, _constraint(over))
        # ExcludedTopicsTest.java:363 sits after the throwing call (JUnit ExpectedException), so the reference never
        # checks it; AbstractGoal.optimize does set UNDER_PROVISIONED (AbstractGoal.java:125-126), the kafka-assigner
        # goals (no AbstractGoal) keep UNDECIDED
        want = "UNDECIDED" if goal.startswith("KafkaAssigner") else "UNDER_PROVISIONED"
        assert ei.value.provision.status == want
        return
    succeeded, proposals, provision = runner(flat, goal, opts, _constraint(over))
    assert succeeded == opt
    assert provision.status != "UNDER_PROVISIONED"  # ExcludedTopicsTest.java:342
    if excl:
        assert bool(proposals) == props
        excluded_idx = {flat.topics.index(t) for t in excl if t in flat.topics}
        for p in proposals:
            if flat.desc.partition_topic[p.partition] in excluded_idx:
                removed = set(p.old_replicas) - set(p.new_replicas)
                assert removed <= set(dead) | set(deterministic_models()[model]["dead"]), p


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


@pytest.mark.parametrize("goal,excl,exc,model,dead,opt,props,over", CASES)
def test_oracle_excluded_topics_kat(oracle_lib, goal, excl, exc, model, dead, opt, props, over):
    run_case(oracle_runner, goal, excl, exc, model, dead, opt, props, over)


@pytest.mark.parametrize("goal,excl,exc,model,dead,opt,props,over", CASES)
def test_emu_excluded_topics_kat(emu_lib, goal, excl, exc, model, dead, opt, props, over):
    run_case(product_runner(emu_lib), goal, excl, exc, model, dead, opt, props, over)


@pytest.mark.parametrize("goal,excl,exc,model,dead,opt,props,over", CASES)
def test_emu_excluded_topics_matches_oracle(emu_lib, oracle_lib, goal, excl, exc, model, dead, opt, props, over):
    # rows that expect an OptimizationFailureException compare the exception class, message, action log and
    # recommendation (check_desc_against_oracle)
    flat = _model(model, dead)
    check_desc_against_oracle(emu_lib, flat.desc, flat, [goal], _constraint(over), _options(flat, excl))


@pytest.mark.gpu
@pytest.mark.parametrize("goal,excl,exc,model,dead,opt,props,over", CASES)
def test_gpu_excluded_topics_kat(gpu_lib, goal, excl, exc, model, dead, opt, props, over):
    run_case(product_runner(gpu_lib), goal, excl, exc, model, dead, opt, props, over)


@pytest.mark.gpu
@pytest.mark.parametrize("goal,excl,exc,model,dead,opt,props,over", CASES)
def test_gpu_excluded_topics_matches_oracle(gpu_lib, oracle_lib, goal, excl, exc, model, dead, opt, props, over):
    flat = _model(model, dead)
    check_desc_against_oracle(gpu_lib, flat.desc, flat, [goal], _constraint(over), _options(flat, excl))
