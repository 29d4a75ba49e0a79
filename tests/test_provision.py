"""Provision responses (Goal.provisionResponse, ProvisionResponse.aggregate).

Pinning (the reference's own tests):
* ProvisionResponseTest.testNullRecommendation (analyzer/ProvisionResponseTest.java:124-220): aggregation cases 1-4.
* LowResourceUtilizationTest (analyzer/LowResourceUtilizationTest.java:58-175): smallClusterModel with
  BROKER_CAPACITY (CPU 200, DISK 1000, NW_IN 2000, NW_OUT 2000), each usage-distribution goal with its low
  utilization threshold 1% under the max broker utilization (rebalances) or 1% over max / balance margin (does not):
  the goal succeeds, reports OVER_PROVISIONED, and hasDiff is as expected.
* Excluded{Topics,BrokersForLeadership,BrokersForReplicaMove}Test: UNDER_PROVISIONED after an
  OptimizationFailureException, never UNDER_PROVISIONED after a successful optimize (test_excluded_*.py run that
  assertion on every row).
Beyond those, every parity check (tests/parity.py) compares each goal's provision response and the failing goal's
with the oracle's.
"""
import pytest

import ccmi
from ccmi import ProvisionRecommendation as Rec
from ccmi import ProvisionResponse as Resp
from oracle_binding import OracleCluster
from parity import check_desc_against_oracle
from test_excluded_brokers import goal_constraint
from verifier import build_model, deterministic_models

UNDER_REC = Rec("UNDER_PROVISIONED", num_brokers=3, typical_broker_id=0, resource="CPU", typical_broker_capacity=1000)
OVER_REC = Rec("OVER_PROVISIONED", num_brokers=4, typical_broker_id=1, resource="CPU", typical_broker_capacity=1600)
STATUSES = ccmi.PROVISION_STATUSES


def generated(status):
    """ProvisionResponseTest.generateProvisionResponse (:44-57)."""
    if status == "UNDER_PROVISIONED":
        return Resp(status, UNDER_REC, "UnderRecommender")
    if status == "OVER_PROVISIONED":
        return Resp(status, OVER_REC, "OverRecommender")
    return Resp(status)


def test_provision_response_aggregation_kat():
    with pytest.raises(ccmi.IllegalArgumentException):
        Resp("OVER_PROVISIONED", OVER_REC, None)
    with pytest.raises(ccmi.IllegalArgumentException):
        Resp("RIGHT_SIZED", OVER_REC, "x")
    # Case-1: anything aggregated into UNDER_PROVISIONED stays UNDER_PROVISIONED; UNDER recommendations accumulate
    for s in STATUSES:
        u = Resp("UNDER_PROVISIONED", UNDER_REC, "Case1").aggregate(generated(s))
        assert u.status == "UNDER_PROVISIONED"
        assert len(u.recommendation_by_recommender) == (2 if s == "UNDER_PROVISIONED" else 1)
        assert u.recommendation_by_recommender["Case1"].num_brokers == 3
    # Case-2: UNDECIDED aggregated with P is P (recommendations included)
    for s in STATUSES:
        other = generated(s)
        u = Resp("UNDECIDED").aggregate(other)
        assert u.status == s and u.recommendation_by_recommender == other.recommendation_by_recommender
    # Case-3.1: RIGHT_SIZED with RIGHT_SIZED or OVER_PROVISIONED is RIGHT_SIZED without recommendations
    r = Resp("RIGHT_SIZED").aggregate(generated("RIGHT_SIZED"))
    assert r.status == "RIGHT_SIZED" and not r.recommendation_by_recommender
    r.aggregate(generated("OVER_PROVISIONED"))
    assert r.status == "RIGHT_SIZED" and not r.recommendation_by_recommender
    # Case-3.2: OVER_PROVISIONED with RIGHT_SIZED clears the recommendation
    o = Resp("OVER_PROVISIONED", OVER_REC, "Case3.2").aggregate(generated("RIGHT_SIZED"))
    assert o.status == "RIGHT_SIZED" and not o.recommendation_by_recommender
    # Case-4: OVER_PROVISIONED with OVER_PROVISIONED accumulates
    o = Resp("OVER_PROVISIONED", OVER_REC, "Case4").aggregate(generated("OVER_PROVISIONED"))
    assert o.status == "OVER_PROVISIONED" and set(o.recommendation_by_recommender) == {"Case4", "OverRecommender"}


# LowResourceUtilizationTest.data (:58-110): (goal, low-utilization threshold of its resource, expect rebalance)
MAX_UTIL = {"CPU": 0.3475, "DISK": 0.28, "NW_IN": 0.13, "NW_OUT": 0.1475}
GOAL_RES = [("CpuUsageDistributionGoal", "CPU"), ("DiskUsageDistributionGoal", "DISK"),
            ("NetworkInboundUsageDistributionGoal", "NW_IN"), ("NetworkOutboundUsageDistributionGoal", "NW_OUT")]
LOW_UTIL_CASES = [(g, r, thr, expect) for g, r in GOAL_RES
                  for thr, expect in ((float(repr(MAX_UTIL[r] * 0.99)), True),
                                      (float(repr(MAX_UTIL[r] / 0.9 * 1.01)), False))]
LOW_UTIL_IDS = [f"{g}-{'rebalance' if e else 'none'}" for g, _, _, e in LOW_UTIL_CASES]


def _small_cluster():
    m = dict(deterministic_models()["smallClusterModel"])
    m["capacity"] = {"CPU": 200.0, "DISK": 1000.0, "NW_IN": 2000.0, "NW_OUT": 2000.0}  # LowResourceUtilizationTest:40-43
    return build_model(m)


def _low_util_constraint(res, thr):
    bc = goal_constraint()
    lows = list(bc.low_utilization_threshold)
    lows[ccmi.RESOURCES.index(res)] = thr
    bc.low_utilization_threshold = tuple(lows)
    return bc


def _run_low_util(runner, goal, res, thr, expect):
    flat = _small_cluster()
    ok, provision, proposals = runner(flat, goal, _low_util_constraint(res, thr))
    assert ok
    assert provision.status == "OVER_PROVISIONED"
    rec = provision.recommendation_by_recommender[goal]
    # GoalUtils.validateProvisionResponse caps the brokers to drop at alive brokers - max replication factor (3 - 2
    # here) and then keeps only numBrokers
    assert rec.num_brokers == 1 and rec.resource in (res, None)
    assert bool(proposals) == expect


def _oracle(flat, goal, bc):
    oc = OracleCluster.from_desc(flat.desc)
    r = oc.optimize([goal], bc)[0]
    return r.succeeded, r.provision, oc.proposals()


def _product(lib):
    def run(flat, goal, bc):
        cm = ccmi.ClusterModel(flat.desc, device=0, lib=lib, keepalive=flat)
        g = getattr(ccmi, goal)(constraint=bc)
        ok = g.optimize(cm)
        return ok, g.provision, cm.proposals()
    return run


@pytest.mark.parametrize("goal,res,thr,expect", LOW_UTIL_CASES, ids=LOW_UTIL_IDS)
def test_oracle_low_resource_utilization_kat(oracle_lib, goal, res, thr, expect):
    _run_low_util(_oracle, goal, res, thr, expect)


@pytest.mark.parametrize("goal,res,thr,expect", LOW_UTIL_CASES, ids=LOW_UTIL_IDS)
def test_emu_low_resource_utilization_kat(emu_lib, oracle_lib, goal, res, thr, expect):
    _run_low_util(_product(emu_lib), goal, res, thr, expect)
    flat = _small_cluster()
    check_desc_against_oracle(emu_lib, flat.desc, flat, [goal], _low_util_constraint(res, thr))


def test_emu_failure_provision_and_chain_aggregate(emu_lib, oracle_lib):
    """An OptimizationFailureException carries the failed goal's UNDER_PROVISIONED response (RackAwareGoal with too
    few racks: numRacks = replication factor - alive racks); a successful chain aggregates its goals' responses."""
    flat = build_model(deterministic_models()["rackAwareUnsatisfiable"])
    cm = ccmi.ClusterModel(flat.desc, device=0, lib=emu_lib, keepalive=flat)
    with pytest.raises(ccmi.OptimizationFailureException) as ei:
        ccmi.GoalOptimizer(goal_constraint()).optimizations(cm, ccmi.goals_from_names(["RackAwareGoal"]))
    p = ei.value.provision
    assert p.status == "UNDER_PROVISIONED" and p.recommendation_by_recommender["RackAwareGoal"].num_racks >= 1
    buf = ccmi.RandomCluster.generate(emu_lib, num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300)
    cm = ccmi.ClusterModel.from_buffers(buf)
    bc = goal_constraint()
    bc.max_replicas_per_broker = 3000
    res = ccmi.GoalOptimizer(bc).optimizations(cm, ccmi.goals_from_names(list(ccmi.DEFAULT_GOALS)))
    agg = ccmi.ProvisionResponse("UNDECIDED")
    for g in res.goal_results:
        agg.aggregate(g.provision)
    assert res.provision_response == agg and agg.status in STATUSES
    assert {g.name: g.provision.status for g in res.goal_results}["RackAwareGoal"] in ("RIGHT_SIZED", "OVER_PROVISIONED")


@pytest.mark.gpu
@pytest.mark.parametrize("goal,res,thr,expect", LOW_UTIL_CASES, ids=LOW_UTIL_IDS)
def test_gpu_low_resource_utilization_kat(gpu_lib, oracle_lib, goal, res, thr, expect):
    _run_low_util(_product(gpu_lib), goal, res, thr, expect)
