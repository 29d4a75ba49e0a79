"""Shared parity helpers: run the product library (HIP build, or the test-only emulation) on a golden case and
compare with the committed fixture and/or a live oracle run on the identical flattened input."""
import json
import os

import pytest

import ccmi
from oracle_binding import OracleCluster
from test_oracle_kat import check_against_golden
from verifier import desc_facts, reference_verifications

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden(name):
    with open(os.path.join(GOLDEN, f"{name}.json")) as f:
        return json.load(f)


def constraint(balance, max_replicas=None, capacity=None):
    bc = ccmi.BalancingConstraint()
    if balance is not None:
        bc.set_resource_balance_percentage(balance)
        bc.set_capacity_threshold(0.8)
    if capacity is not None:
        bc.set_capacity_threshold(capacity)
    if max_replicas is not None:
        bc.max_replicas_per_broker = max_replicas
    return bc


def run_product(lib, props, goals, balance, device=0, max_replicas=None, options=None, capacity=None):
    buf = ccmi.RandomCluster.generate(lib, **props)
    cm = ccmi.ClusterModel.from_buffers(buf, device=device)
    res = ccmi.GoalOptimizer(constraint(balance, max_replicas, capacity)).optimizations(
        cm, ccmi.goals_from_names(goals), options)
    return buf, cm, res


def golden_options(g):
    return ccmi.OptimizationOptions(**g["options"]) if g.get("options") else None


def assign_shared_hosts(buf, per_host):
    """Brokers of a RandomCluster sharing hosts: within every rack (ascending rack index), consecutive brokers by id fill
    hosts of `per_host` brokers (Rack._hosts keys a host by name within its rack, model/Rack.java:256-262). Sets
    desc.broker_host and returns the host array (keep it alive with the buffers). No reference fixture shares a host
    (RandomCluster names every host after its broker, RandomCluster.java:80,87): parity on these models is pinned by
    the oracle's Host restatement and ClusterModel.sanityCheck's host sums (tests/test_hosts.py)."""
    import ctypes as C
    d = buf.desc
    by_rack = {}
    for b in range(d.num_brokers):
        by_rack.setdefault(d.broker_rack[b], []).append(b)
    host = [0] * d.num_brokers
    nxt = 0
    for rack in sorted(by_rack):
        for i, b in enumerate(by_rack[rack]):
            if i % per_host == 0:
                nxt += 1
            host[b] = nxt - 1
    arr = (C.c_int32 * d.num_brokers)(*host)
    d.broker_host = C.cast(arr, C.POINTER(C.c_int32))
    return arr


def check_product_against_golden(lib, name, per_goal_stats=False):
    """The product on a golden case: action log, assignment, leaders, per-goal (name, succeeded, candidates,
    actions) and final stats; with per_goal_stats every goal's ClusterModelStats (goldens that store them)."""
    g = golden(name)
    bc = constraint(g["resource_balance_percentage"], g.get("max_replicas_per_broker"), g.get("capacity_threshold"))
    buf = ccmi.RandomCluster.generate(lib, **g["props"])
    hosts = assign_shared_hosts(buf, g["brokers_per_host"]) if g.get("brokers_per_host") else None
    cm = ccmi.ClusterModel(buf.desc, device=0, lib=lib, keepalive=(buf, hosts)) if hosts is not None \
        else ccmi.ClusterModel.from_buffers(buf)
    pre = cm.cluster_stats(bc)
    res = ccmi.GoalOptimizer(bc).optimizations(cm, ccmi.goals_from_names(g["goals"]), golden_options(g))
    check_against_golden(g, cm.actions(), cm.replica_distribution(), cm.leader_distribution(), res.goal_results,
                         res.goal_results[-1].stats, replica_disks=cm.replica_disks())
    if per_goal_stats:
        for r, e in zip(res.goal_results, g["goals_result"]):
            if "stats" in e:
                compare_stats(r.stats, e["stats"])
    if "verifications" in g:  # the oracle's outcome, recorded when the golden was made
        assert verify_like_reference(buf.desc, g["goals"], res, pre, bc, cm) == g["verifications"]
    return cm, res


def verify_like_reference(desc, goals, res, pre, bc, cm):
    """OptimizationVerifier on the product's result (tests/verifier.py). RandomClusterTest.java:126-128 and
    RandomSelfHealingTest.java:132-134 require BROKEN_BROKERS and REGRESSION to pass for the default goals;
    GOAL_VIOLATION is asserted by the reference only for the KafkaAssigner goals, so it is returned (and compared
    with the oracle's / the golden's) rather than required. violatedGoalsAfterOptimization is the product's own
    OptimizerResult field (GoalOptimizer.java:479-481); it must name the goals reported as not succeeded."""
    assert res.violated_goals_after == [r.name for r in res.goal_results if not r.succeeded]
    dead, offline = desc_facts(desc)
    v = reference_verifications(dead, offline, goals, res.goal_results, pre, bc, cm.replica_distribution(),
                                res.proposals)
    assert v["BROKEN_BROKERS"] in (None, "n/a") and v["REGRESSION"] in (None, "n/a"), v
    return v


def compare_stats(a, b, rel=1e-9):
    for k, v in b.items():
        got = a[k]
        for x, y in zip(got if isinstance(got, list) else [got], v if isinstance(v, list) else [v]):
            if x != x and y != y:  # NaN on both sides (e.g. topic stats of a cluster without topics: 0 / 0)
                continue
            assert x == pytest.approx(y, rel=rel, abs=1e-12), k


def _key(p):
    return (p.partition, p.partition_size, p.old_leader, tuple(p.old_replicas), tuple(p.new_replicas),
            tuple(p.old_disks or ()), tuple(p.new_disks or ()))


def check_product_against_oracle(lib, props, goals, balance=None, device=0, max_replicas=None, options=None,
                                 verify=False):
    """Live parity: same flattened input into both; action log, final assignment/leaders, per-goal results and
    every goal's post-optimization ClusterModelStats. A chain that fails (OptimizationFailureException for a hard
    goal) must fail in both with the same exception and message after the same action log."""
    buf = ccmi.RandomCluster.generate(lib, **props)
    return check_desc_against_oracle(lib, buf.desc, buf, goals, constraint(balance, max_replicas), options, device,
                                     verify)


def check_desc_against_oracle(lib, desc, keepalive, goals, bc, options=None, device=0, verify=False):
    """check_product_against_oracle on any flattened model (RandomCluster buffers or a ClusterModelBuilder's
    FlatCluster). Returns (session, OptimizerResult or None when both raised, oracle cluster)."""
    cm = ccmi.ClusterModel(desc, device=device, lib=lib, keepalive=keepalive)
    oc = OracleCluster.from_desc(desc)
    if verify:  # pre-optimization ClusterModelStats for REGRESSION, themselves compared with the oracle's
        pre = cm.cluster_stats(bc, options)
        compare_stats(pre, oc.stats(bc, options))
    perr = oerr = None
    try:
        res = ccmi.GoalOptimizer(bc).optimizations(cm, ccmi.goals_from_names(goals), options)
    except ccmi.CruiseControlError as e:
        perr = e
    try:
        ores = oc.optimize(goals, bc, options)
    except Exception as e:  # noqa: BLE001 - the oracle binding raises the same exception classes
        oerr = e
    if perr is not None or oerr is not None:
        assert (type(perr).__name__, str(perr)) == (type(oerr).__name__, str(oerr))
        assert cm.actions() == oc.actions()
        # the failed goal's provision response (UNDER_PROVISIONED with the exception's recommendation)
        assert getattr(perr, "provision", None) == getattr(oerr, "provision", None)
        return cm, None, oc
    pa, oa = cm.actions(), oc.actions()
    for i, (x, y) in enumerate(zip(pa, oa)):
        assert x == y, f"first action mismatch at {i}: {x} vs {y}"
    assert len(pa) == len(oa)
    assert cm.replica_distribution() == oc.replica_distribution()
    assert cm.leader_distribution() == oc.leader_distribution()
    assert cm.replica_disks() == oc.replica_disks()
    for r, o in zip(res.goal_results, ores):
        assert (r.name, r.succeeded, r.candidates, r.actions) == (o.name, o.succeeded, o.candidates, o.actions), \
            ((r.name, r.succeeded, r.candidates, r.actions), (o.name, o.succeeded, o.candidates, o.actions))
        assert r.provision == o.provision, (r.name, r.provision, o.provision)
        compare_stats(r.stats, o.stats)
    # Set<ExecutionProposal>: order-free
    assert sorted(map(_key, res.proposals)) == sorted(map(_key, oc.proposals()))
    if verify:
        verify_like_reference(desc, goals, res, pre, bc, cm)
    return cm, res, oc
