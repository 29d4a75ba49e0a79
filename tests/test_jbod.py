"""JBOD: replica placement over disks and the intra-broker goals (BASELINE configs[4]).

Pinning, as for the other goals (the reference is Java and cannot run here):
* IntraBrokerRebalanceTest (analyzer/IntraBrokerRebalanceTest.java:96-148): RandomCluster BASE_PROPERTIES with
  POPULATE_REPLICA_PLACEMENT_INFO (testCapacityConfigJBOD.json), rack-aware populate, LOW_BALANCE 1.05 /
  MEDIUM_CAPACITY 0.8 / max.replicas.per.broker 2000, each intra-broker goal alone and both; deck #1 healthy, deck #2
  excluded topics T1/T2, deck #3 five dead brokers and five brokers with a dead disk. The reference passes when
  OptimizationVerifier finds no violated goal (GOAL_VIOLATION) and no regression (REGRESSION).
* DeterministicClusterTest's swap decks on unbalanced4 (DeterministicClusterTest.java:123-129, ZERO_BALANCE 1.0):
  DiskUsageDistributionGoal (an inter-broker goal on a JBOD model) and IntraBrokerDiskUsageDistributionGoal.
* the product generator's JBOD desc equals the oracle RandomCluster's, and the product (emulation on CPU, gfx950 on
  the GPU) matches the oracle bit for bit on every case (actions with disks, brokers, disks, leaders, per-goal
  results, stats within 1e-9, proposals with logdirs).
"""
import pytest

import ccmi
from oracle_binding import OracleCluster, desc_arrays
from parity import check_desc_against_oracle, check_product_against_golden
from verifier import build_model, deterministic_models, verify_regression

INTRA = list(ccmi.INTRA_BROKER_GOALS)
JBOD_BASE = dict(jbod=1, rack_aware=1)
JBOD_BROKEN = dict(jbod=1, rack_aware=1, num_dead_brokers=5, num_brokers_with_bad_disk=5)
T1_T2 = [1, 2]  # topic indices of "T1", "T2" in RandomCluster's topic list


def rebalance_constraint(capacity=0.8):
    """IntraBrokerRebalanceTest.java:103-111."""
    bc = ccmi.BalancingConstraint()
    bc.max_replicas_per_broker = 2000
    bc.set_resource_balance_percentage(1.05)
    bc.set_capacity_threshold(capacity)
    return bc


def decks():
    out = []
    for deck, props, excluded in (("healthy", JBOD_BASE, None), ("excluded", JBOD_BASE, T1_T2),
                                  ("broken", JBOD_BROKEN, None)):
        for goals in ([INTRA[0]], [INTRA[1]], INTRA):
            out.append((f"{deck}-{'+'.join(g[len('IntraBroker'):] for g in goals)}", props, goals, excluded, 0.8))
    # the capacity goal with work to do (disks over 0.15 / 0.2 of their capacity)
    for cap in (0.15, 0.2):
        out.append((f"healthy-cap{cap}", JBOD_BASE, INTRA, None, cap))
    # half of the topics excluded: the selection function changes the decisions
    out.append(("excluded-half", JBOD_BASE, [INTRA[1]], list(range(0, 3000, 2)), 0.8))
    # C4's layout at a small scale (4 logdirs: java.util.Random's first draws put a broker's replicas on one disk)
    out.append(("four-logdirs", dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=200, rack_aware=1,
                                     jbod=2, num_logdirs=4, logdir_capacity=[75000.0] * 4), INTRA, None, 0.8))
    return out


DECKS = decks()
IDS = [d[0] for d in DECKS]


def _options(excluded):
    return ccmi.OptimizationOptions(excluded_topics=excluded) if excluded else None


@pytest.mark.parametrize("deck", DECKS, ids=IDS)
def test_oracle_passes_intra_broker_rebalance_deck(oracle_lib, deck):
    _, props, goals, excluded, cap = deck
    oc = OracleCluster.random(**props)
    bc = rebalance_constraint(cap)
    pre = oc.stats(bc)
    res = oc.optimize(goals, bc, _options(excluded))
    if deck in DECKS[:9]:  # IntraBrokerRebalanceTest's own decks: every goal succeeds
        assert all(r.succeeded for r in res), [(r.name, r.succeeded) for r in res]  # GOAL_VIOLATION
    assert verify_regression(res, pre, bc) is None  # REGRESSION


@pytest.mark.parametrize("props", [JBOD_BASE, JBOD_BROKEN, DECKS[-1][1]], ids=["base", "broken", "four-logdirs"])
def test_generator_jbod_desc_matches_oracle(emu_lib, oracle_lib, props):
    buf = ccmi.RandomCluster.generate(emu_lib, **props)
    ex = OracleCluster.random(**props).export()
    da = desc_arrays(buf.desc)
    for k, v in da.items():
        if k in ex:
            assert (list(v) if isinstance(v, (list, tuple)) else v) == ex[k], k
    assert buf.desc.num_disks > 0 and buf.desc.num_disk_assignments == buf.desc.num_replicas


@pytest.mark.parametrize("deck", DECKS, ids=IDS)
def test_emu_intra_broker_deck_matches_oracle(emu_lib, oracle_lib, deck):
    _, props, goals, excluded, cap = deck
    buf = ccmi.RandomCluster.generate(emu_lib, **props)
    cm, res, oc = check_desc_against_oracle(emu_lib, buf.desc, buf, goals, rebalance_constraint(cap),
                                            _options(excluded))
    assert res is not None
    assert cm.perf().intra_launches == len(goals)


SWAP_DECKS = [("unbalanced4", ["IntraBrokerDiskUsageDistributionGoal"]),
              ("unbalanced4", ["DiskUsageDistributionGoal"]),
              ("unbalanced4", INTRA),
              ("unbalanced5", ["IntraBrokerDiskUsageDistributionGoal"]),
              ("unbalanced5", ["DiskUsageDistributionGoal"])]


def _zero_balance():
    """DeterministicClusterTest.java:122-124 (getDefaultCruiseControlProperties: max.replicas.per.broker 6)."""
    bc = ccmi.BalancingConstraint()
    bc.max_replicas_per_broker = 6
    bc.set_resource_balance_percentage(1.0)
    return bc


def test_oracle_unbalanced4_swap_decks(oracle_lib):
    """The two reference decks pass REGRESSION; the intra-broker one moves replicas between the two disks of each
    broker, with swaps (a swap is logged as the source move and a remove/add of the destination replica)."""
    for goals in (["DiskUsageDistributionGoal"], ["IntraBrokerDiskUsageDistributionGoal"]):
        flat = build_model(deterministic_models()["unbalanced4"])
        oc = OracleCluster.from_desc(flat.desc)
        pre = oc.stats(_zero_balance())
        res = oc.optimize(goals, _zero_balance())
        assert verify_regression(res, pre, _zero_balance()) is None
    acts = oc.actions()
    assert acts and all(a[0] == 3 and a[2] == a[3] for a in acts)
    assert any(a[5] == a[6] for a in acts)


@pytest.mark.parametrize("model,goals", SWAP_DECKS, ids=[f"{m}-{'+'.join(g)}" for m, g in SWAP_DECKS])
def test_emu_swap_deck_matches_oracle(emu_lib, oracle_lib, model, goals):
    flat = build_model(deterministic_models()[model])
    check_desc_against_oracle(emu_lib, flat.desc, flat, goals, _zero_balance())


def test_emu_intra_action_acceptance(emu_lib, oracle_lib):
    """ccmi_action_acceptance for the intra-broker goals (IntraBrokerDiskCapacityGoal.java:115-136,
    IntraBrokerDiskUsageDistributionGoal.java:146-243) against the model after the chain."""
    flat = build_model(deterministic_models()["unbalanced4"])
    cm = ccmi.ClusterModel(flat.desc, device=0, lib=emu_lib, keepalive=flat)
    ccmi.GoalOptimizer(_zero_balance()).optimizations(cm, ccmi.goals_from_names(["IntraBrokerDiskUsageDistributionGoal"]))
    disks = cm.replica_disks()  # partition p has one replica (slot p)
    # move partition 0's replica to the other disk of broker 0 (disks 0/1 are broker 0's /mnt/i00 and /mnt/i01)
    src = disks[0]
    got = cm.action_acceptance(0, 3, 0, 0, 0, -1, src, 1 - src)
    assert got in ("ACCEPT", "REPLICA_REJECT")
    with pytest.raises(ccmi.IllegalArgumentException):
        cm.action_acceptance(0, 0, 0, 0, 1)  # an inter-broker action has no logdirs
    with pytest.raises(ccmi.IllegalArgumentException):  # a chain may not mix the two granularities
        ccmi.GoalOptimizer(_zero_balance()).optimizations(
            cm, ccmi.goals_from_names(["IntraBrokerDiskCapacityGoal", "DiskUsageDistributionGoal"]))
    with pytest.raises(ccmi.IllegalArgumentException):  # nor may a goal's optimizedGoals set
        ccmi.DiskUsageDistributionGoal(constraint=_zero_balance()).optimize(
            cm, [ccmi.IntraBrokerDiskUsageDistributionGoal()], ccmi.OptimizationOptions())


@pytest.mark.gpu
@pytest.mark.parametrize("deck", DECKS, ids=IDS)
def test_gpu_intra_broker_deck_matches_oracle(gpu_lib, oracle_lib, deck):
    _, props, goals, excluded, cap = deck
    buf = ccmi.RandomCluster.generate(gpu_lib, **props)
    cm, res, oc = check_desc_against_oracle(gpu_lib, buf.desc, buf, goals, rebalance_constraint(cap),
                                            _options(excluded))
    assert res is not None
    assert cm.perf().intra_launches >= len(goals)


@pytest.mark.gpu
@pytest.mark.parametrize("model,goals", SWAP_DECKS, ids=[f"{m}-{'+'.join(g)}" for m, g in SWAP_DECKS])
def test_gpu_swap_deck_matches_oracle(gpu_lib, oracle_lib, model, goals):
    flat = build_model(deterministic_models()[model])
    check_desc_against_oracle(gpu_lib, flat.desc, flat, goals, _zero_balance())


@pytest.mark.gpu
def test_gpu_matches_c4_golden(gpu_lib):
    """C4 (BASELINE configs[4]) against the committed oracle golden (tests/golden/make_golden.py c4)."""
    cm, res = check_product_against_golden(gpu_lib, "c4", per_goal_stats=True)
    assert cm.perf().intra_launches >= 2
