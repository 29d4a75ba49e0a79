"""The caller's optimizedGoals set at the boundary (ABI v8).

Goal.optimize(clusterModel, optimizedGoals, options) (Goal.java:60-68) constrains a goal's moves by the
actionAcceptance of exactly the goals in `optimizedGoals` (AbstractGoal.maybeApplyBalancingAction ->
AnalyzerUtils.isProposalAcceptableForOptimizedGoals, AnalyzerUtils.java:169-179), whatever else ran on the model:
* GoalViolationDetector.optimizeForGoal calls optimize(clusterModel, Collections.emptySet(), options)
  (GoalViolationDetector.java:314) and reuses the model for the next goal whenever a goal changed nothing
  (:193-211, newModelNeeded);
* GoalOptimizer.optimizations starts every call with an empty set (GoalOptimizer.java:449) and adds each goal after it
  ran (:471), so a second call on the same model does not inherit the first call's goals;
* a caller may pass any subset of the goals that optimized the model (a non-prefix set).
Every case runs on one product session (CPU emulation; gfx950 under -m gpu) and one oracle model and must match
bit for bit: action log, placement, goal results and stats.
"""
import pytest

import ccmi
from oracle_binding import OracleCluster
from parity import compare_stats, constraint

PROPS = dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300)
RACK_AWARE_PROPS = dict(PROPS, rack_aware=1)


def _same(cm, oc):
    assert cm.actions() == oc.actions()
    assert cm.replica_distribution() == oc.replica_distribution()
    assert cm.leader_distribution() == oc.leader_distribution()


def _same_result(name, ok, r, o):
    """ok: the product's Goal.optimize return; r: its ccmi_goal_result; o: the oracle's GoalResult."""
    assert (name, ok, r.candidates, r.actions, bool(r.has_diff)) == \
        (o.name, o.succeeded, o.candidates, o.actions, o.has_diff)
    compare_stats(ccmi.stats_to_dict(r.stats), o.stats)


def _goal_optimize(cm, name, prior, bc, options=None):
    """Goal.optimize through the boundary, returning (succeeded, ccmi_goal_result)."""
    g = ccmi.goals_from_names([name], bc)[0]
    r = cm._goal_optimize(g, prior, options)
    return bool(r.succeeded), r


def _detector_sequence(lib, props, goals, bc):
    """GoalViolationDetector.run's loop (GoalViolationDetector.java:189-216): one model while goals change nothing,
    every goal with an empty optimizedGoals set and OptimizationOptions triggered by goal violation."""
    opts = ccmi.OptimizationOptions(is_triggered_by_goal_violation=True)
    buf = ccmi.RandomCluster.generate(lib, **props)
    cm = oc = None
    new_model = True
    outcome = []
    reused = 0
    for name in goals:
        if new_model:
            cm = ccmi.ClusterModel.from_buffers(buf)
            oc = OracleCluster.from_desc(buf.desc)
        else:
            reused += 1
        try:
            o = oc.goal_optimize(name, (), bc, opts)
        except ccmi.OptimizationFailureException:
            with pytest.raises(ccmi.OptimizationFailureException):
                _goal_optimize(cm, name, (), bc, opts)
            outcome.append((name, "unfixable"))
            new_model = True
            continue
        ok, r = _goal_optimize(cm, name, (), bc, opts)
        _same_result(name, ok, r, o)
        _same(cm, oc)
        outcome.append((name, "fixable" if o.has_diff else None))
        new_model = o.has_diff
    return outcome, reused


# RackAwareGoal and the capacity goals change nothing on a rack-aware placement, so the goals after them run on the
# same model with an empty set: their moves are free to break rack awareness (the oracle shows they do).
DETECTOR_GOALS = ["RackAwareGoal", "DiskCapacityGoal", "ReplicaDistributionGoal", "NetworkInboundCapacityGoal",
                  "CpuUsageDistributionGoal", "LeaderReplicaDistributionGoal"]


def test_oracle_empty_set_differs_from_prior_set(oracle_lib):
    """The set matters: ReplicaDistributionGoal after RackAwareGoal on the same model moves differently with
    optimizedGoals = {} than with {RackAwareGoal} (the empty set lets it break rack awareness)."""
    bc = constraint(1.05)
    runs = []
    for prior in ((), ("RackAwareGoal",)):
        oc = OracleCluster.random(**RACK_AWARE_PROPS)
        assert not oc.goal_optimize("RackAwareGoal", (), bc).has_diff
        oc.goal_optimize("ReplicaDistributionGoal", prior, bc)
        runs.append(oc.actions())
    assert runs[0] != runs[1]


def _check_detector(lib):
    outcome, reused = _detector_sequence(lib, RACK_AWARE_PROPS, DETECTOR_GOALS, constraint(1.05))
    assert reused >= 2, outcome  # goals ran on a model a previous goal left unchanged


def _non_prefix_set(lib):
    """Goals optimized one by one with growing sets, then one with a non-prefix set {first, third}."""
    bc = constraint(1.05)
    buf = ccmi.RandomCluster.generate(lib, **PROPS)
    cm = ccmi.ClusterModel.from_buffers(buf)
    oc = OracleCluster.from_desc(buf.desc)
    chain = [("ReplicaCapacityGoal", ()), ("ReplicaDistributionGoal", ("ReplicaCapacityGoal",)),
             ("DiskUsageDistributionGoal", ("ReplicaCapacityGoal", "ReplicaDistributionGoal")),
             ("NetworkInboundUsageDistributionGoal", ("DiskUsageDistributionGoal", "ReplicaCapacityGoal")),
             ("LeaderReplicaDistributionGoal", ("NetworkInboundUsageDistributionGoal",)),
             ("ReplicaDistributionGoal", ("LeaderReplicaDistributionGoal", "DiskUsageDistributionGoal")),
             ("CpuUsageDistributionGoal", ("ReplicaDistributionGoal", "ReplicaCapacityGoal", "ReplicaCapacityGoal"))]
    for name, prior in chain:
        o = oc.goal_optimize(name, prior, bc)
        ok, r = _goal_optimize(cm, name, [ccmi.GOAL_KINDS[p] for p in prior], bc)
        _same_result(name, ok, r, o)
        _same(cm, oc)
    # acceptance by kind: the session's latest ReplicaDistributionGoal instance, as the oracle's
    for a in cm.actions()[-30:]:
        for g in ("ReplicaDistributionGoal", "NetworkInboundUsageDistributionGoal", "ReplicaCapacityGoal"):
            assert cm.action_acceptance_by_goal(g, a[0], a[1], a[3], a[2]) == \
                oc.action_acceptance_by_goal(g, a[0], a[1], a[3], a[2])


def _two_optimizations_calls(lib):
    """A second GoalOptimizer.optimizations on the same model starts from an empty optimizedGoals set."""
    bc = constraint(1.05)
    buf = ccmi.RandomCluster.generate(lib, **RACK_AWARE_PROPS)
    cm = ccmi.ClusterModel.from_buffers(buf)
    oc = OracleCluster.from_desc(buf.desc)
    for goals in (["RackAwareGoal", "ReplicaCapacityGoal"], ["ReplicaDistributionGoal", "DiskUsageDistributionGoal"]):
        res = ccmi.GoalOptimizer(bc).optimizations(cm, ccmi.goals_from_names(goals))
        ores = oc.optimize(goals, bc)
        for r, o in zip(res.goal_results, ores):
            assert (r.name, r.succeeded, r.candidates, r.actions) == (o.name, o.succeeded, o.candidates, o.actions)
            compare_stats(r.stats, o.stats)
        _same(cm, oc)


def _unsupported_sets(lib):
    """A goal the session does not hold (run in the JVM, or a JVM-only class) cannot join the device conjunction:
    UnsupportedOperationException before anything changes, so the caller runs the goal in the JVM."""
    buf = ccmi.RandomCluster.generate(lib, **PROPS)
    cm = ccmi.ClusterModel.from_buffers(buf)
    bc = constraint(1.05)
    for prior in ([ccmi.GOAL_KINDS["RackAwareGoal"]], [-1]):
        with pytest.raises(ccmi.UnsupportedOperationException):
            _goal_optimize(cm, "ReplicaDistributionGoal", prior, bc)
        assert cm.actions() == []
    with pytest.raises(ccmi.IllegalArgumentException):
        ccmi.ReplicaDistributionGoal().optimize(cm, ccmi.OptimizationOptions())
    ok, _ = _goal_optimize(cm, "DiskUsageDistributionGoal", [], bc)
    assert ok and cm.actions()


def test_emu_detector_sequence_one_session(emu_lib, oracle_lib):
    _check_detector(emu_lib)


def test_emu_non_prefix_optimized_set(emu_lib, oracle_lib):
    _non_prefix_set(emu_lib)


def test_emu_second_optimizations_call_starts_empty(emu_lib, oracle_lib):
    _two_optimizations_calls(emu_lib)


def test_emu_unheld_goal_is_unsupported(emu_lib):
    _unsupported_sets(emu_lib)


@pytest.mark.gpu
def test_gpu_detector_sequence_one_session(gpu_lib, oracle_lib):
    _check_detector(gpu_lib)


@pytest.mark.gpu
def test_gpu_non_prefix_optimized_set(gpu_lib, oracle_lib):
    _non_prefix_set(gpu_lib)


@pytest.mark.gpu
def test_gpu_second_optimizations_call_starts_empty(gpu_lib, oracle_lib):
    _two_optimizations_calls(gpu_lib)


@pytest.mark.gpu
def test_gpu_unheld_goal_is_unsupported(gpu_lib):
    _unsupported_sets(gpu_lib)
