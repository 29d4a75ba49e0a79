"""CPU tests that pin the oracle (oracle/, the C++ restatement) before anything is checked against it.

* GoalUtilsTest.java:31-71 — the only exact KAT for the resource balance-threshold formula.
* java.util.Random — published JDK values plus an independent restatement of the documented LCG
  (third-party arithmetic absent from /root/reference: RandomCluster's placement depends on it).
* the committed golden fixtures (tests/golden/*.json, written by tests/golden/make_golden.py).
"""
import ctypes as C
import hashlib
import json
import os
import struct

import pytest

import ccmi
from oracle_binding import Oracle, OracleCluster
from verifier import model_facts, reference_verifications

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
BALANCE_MARGIN = 0.9  # ResourceDistributionGoal.BALANCE_MARGIN


def _threshold(low_util, is_lower, avg=0.3, balance=1.3, multiplier=1.2, triggered=True):
    return Oracle.lib().oc_balance_threshold(avg, 0, balance, low_util, multiplier, int(triggered), BALANCE_MARGIN,
                                            int(is_lower))


def test_balance_threshold_kat(oracle_lib):
    """GoalUtilsTest.testComputeResourceUtilizationBalanceThreshold, all five cases, delta 0.0."""
    assert _threshold(0.4, True) == 0.0
    assert _threshold(0.4, False) == 0.3 * (1 + ((1.3 * 1.2) - 1) * BALANCE_MARGIN)
    assert _threshold(0.6, False) == 0.6 * BALANCE_MARGIN
    assert _threshold(0.2, True) == 0.3 * (1 - ((1.3 * 1.2) - 1) * BALANCE_MARGIN)
    assert _threshold(0.2, False) == 0.3 * (1 + ((1.3 * 1.2) - 1) * BALANCE_MARGIN)


def test_balance_threshold_not_triggered(oracle_lib):
    # GoalUtils.java:579-602: without goal-violation triggering the multiplier is not applied
    assert _threshold(0.2, False, triggered=False) == 0.3 * (1 + (1.3 - 1) * BALANCE_MARGIN)


class _JRandom:
    """Independent restatement of java.util.Random (JDK docs: 48-bit LCG, multiplier 0x5DEECE66D, addend 0xB)."""
    M = (1 << 48) - 1

    def __init__(self, seed):
        self.s = (seed ^ 0x5DEECE66D) & self.M

    def next(self, bits):
        self.s = (self.s * 0x5DEECE66D + 0xB) & self.M
        v = self.s >> (48 - bits)
        return v - (1 << bits) if v >= 1 << (bits - 1) else v

    def next_int(self, bound):
        if bound & -bound == bound:
            return (bound * (self.next(31) & 0x7FFFFFFF)) >> 31
        while True:
            bits = self.next(31) & 0x7FFFFFFF
            val = bits % bound
            if bits - val + (bound - 1) < (1 << 31):
                return val

    def next_double(self):
        a = self.next(26) & ((1 << 26) - 1)
        b = self.next(27) & ((1 << 27) - 1)
        return ((a << 27) + b) * (1.0 / (1 << 53))


def _probe(seed, bound, n):
    ints, dbls = (C.c_int32 * n)(), (C.c_double * n)()
    Oracle.lib().oc_java_random_probe(seed, bound, n, ints, dbls)
    return list(ints), list(dbls)


def test_java_random_published_values(oracle_lib):
    # Widely published JDK outputs: new Random(0).nextDouble(), new Random(42).nextDouble()
    assert _probe(0, 10, 1)[1][0] == 0.730967787376657
    assert _probe(42, 10, 1)[1][0] == 0.7275636800328681
    assert _probe(42, 10, 1)[0][0] == 0  # new Random(42).nextInt(10)


@pytest.mark.parametrize("seed,bound", [(0, 10), (42, 3), (1234567, 1000), (-5, 1 << 10), (3140, 99999),
                                        (987654321012, 7)])
def test_java_random_matches_restatement(oracle_lib, seed, bound):
    ints, dbls = _probe(seed, bound, 200)
    r1, r2 = _JRandom(seed), _JRandom(seed)
    assert ints == [r1.next_int(bound) for _ in range(200)]
    assert dbls == [r2.next_double() for _ in range(200)]


def _golden(name):
    with open(os.path.join(GOLDEN, f"{name}.json")) as f:
        return json.load(f)


def _sha(ints):
    return hashlib.sha256(struct.pack(f"<{len(ints)}q", *ints)).hexdigest()


def _constraint(g):
    bc = ccmi.BalancingConstraint()
    if g["resource_balance_percentage"] is not None:
        bc.set_resource_balance_percentage(g["resource_balance_percentage"])
        bc.set_capacity_threshold(0.8)
    if g.get("capacity_threshold") is not None:
        bc.set_capacity_threshold(g["capacity_threshold"])
    if g.get("max_replicas_per_broker") is not None:
        bc.max_replicas_per_broker = g["max_replicas_per_broker"]
    return bc


def golden_action(a):
    """Action tuples of models without disks keep their 5-field golden form (the disk fields are -1)."""
    a = tuple(a)
    return a[:5] if len(a) == 7 and a[5] == -1 and a[6] == -1 else a


def check_against_golden(g, actions, replica_dist, leader_dist, goal_results, final_stats, rel=1e-9,
                         replica_disks=None):
    """Shared by the oracle, emulation and GPU tests."""
    actions = [golden_action(a) for a in actions]
    if "replica_disks_sha256" in g:  # JBOD goldens: the logdir half of every ReplicaPlacementInfo
        assert replica_disks is not None and _sha(replica_disks) == g["replica_disks_sha256"]
    if "actions" in g:
        for i, (x, y) in enumerate(zip(actions, g["actions"])):
            assert tuple(x) == tuple(y), f"first action mismatch at {i}"
    assert len(actions) == g["num_actions"]
    assert _sha([x for a in actions for x in a]) == g["actions_sha256"]
    assert _sha(replica_dist) == g["replica_distribution_sha256"]
    assert _sha(leader_dist) == g["leader_distribution_sha256"]
    for r, e in zip(goal_results, g["goals_result"]):
        assert (r.name, r.succeeded, r.candidates, r.actions) == (e["name"], e["succeeded"], e["candidates"],
                                                                  e["actions"])
    for k, v in g["final_stats"].items():
        got = final_stats[k]
        for x, y in zip(got if isinstance(got, list) else [got], v if isinstance(v, list) else [v]):
            assert x == pytest.approx(y, rel=rel, abs=1e-12), k


GOLDEN_CASES = ["small_20b", "dead_2of10", "rack_aware_dead", "c0", "c1", "small_20b_default", "dead_3of24_default",
                "rack_aware_dead_default", "c0_default", "jbod_base", "jbod_base_cap15"]


@pytest.mark.parametrize("name", GOLDEN_CASES)
def test_oracle_matches_golden(oracle_lib, name):
    g = _golden(name)
    oc = OracleCluster.random(**g["props"])
    assert (oc.B, oc.T, oc.P, oc.R) == tuple(g["sizes"][k] for k in ("brokers", "topics", "partitions", "replicas"))
    bc = _constraint(g)
    a0 = oc.export()
    facts = model_facts(a0["broker_state"], a0["replica_broker"], a0["replica_partition"], a0["offline"])
    pre = oc.stats(bc)
    res = oc.optimize(g["goals"], bc)
    check_against_golden(g, oc.actions(), oc.replica_distribution(), oc.leader_distribution(), res, res[-1].stats,
                         rel=0.0, replica_disks=oc.replica_disks())
    # OptimizationVerifier on the oracle (RandomClusterTest.java:126-128): BROKEN_BROKERS and REGRESSION pass, and
    # the recorded outcome of all three is reproduced
    v = reference_verifications(*facts, g["goals"], res, pre, bc, oc.replica_distribution(), oc.proposals())
    assert v == g["verifications"]
    assert v["BROKEN_BROKERS"] in (None, "n/a") and v["REGRESSION"] in (None, "n/a"), v
