"""BrokerSetAwareGoal (analyzer/goals/BrokerSetAwareGoal.java) pinned by the reference's own tests:

* TopicNameHashBrokerSetMappingPolicyTest.java:62-85 / :92-125 — topics "A".."D" of mediumClusterModel map to
  BS2, BS1, BS1, BS1 over {BS1, BS2} and to BS2, BS1, BS3, BS3 over {BS1, BS2, BS3} (Guava murmur3_128 +
  consistentHash, restated in the oracle and in the product, include/ccmi.h ccmi_topic_broker_set);
* DeterministicClusterTest.java:255-334 — the broker-set decks on DeterministicCluster.brokerSet* models
  (tests/golden/broker_set_clusters.json, make_broker_set_models.py) with resources/testBrokerSets.json
  (Blue {0,1,2}, Green {3,4,5}; broker 6 of RACK_BY_BROKER5 joins "unmapped") and ReplicaToOriginalBrokerSetMappingPolicy
  (getDefaultCruiseControlProperties, :337-344): the verifier invariants must hold, and the Unsatisfiable decks must
  fail with OptimizationFailureException;
* ExcludedTopicsTest.java:303-321 — the BrokerSetAwareGoal rows.

The product (CPU emulation; gfx950 under -m gpu) must equal the oracle move for move on every deck, on RandomCluster
cases under the TopicNameHash policy, and in Goal.actionAcceptance.
"""
import json
import os
import random

import pytest

import ccmi
from oracle_binding import Oracle, OracleCluster
from parity import check_desc_against_oracle
from test_deterministic import oracle_runner, product_runner
from verifier import build_model, offline_replicas, verify_broken_brokers, verify_regression, \
    verify_soft_goal_replica_movements

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "broker_set_clusters.json")) as _f:
    FIX = json.load(_f)
MODELS = FIX["models"]
TEST_BROKER_SETS = FIX["broker_sets"]["sets"]

BSA = "BrokerSetAwareGoal"
DECK_GOALS = [BSA, "RackAwareGoal", "RackAwareDistributionGoal", "ReplicaCapacityGoal", "DiskCapacityGoal",
              "NetworkInboundCapacityGoal", "NetworkOutboundCapacityGoal", "CpuCapacityGoal"]
OFE = "OptimizationFailureException"


def deck_constraint(policy="ReplicaToOriginalBrokerSetMappingPolicy"):
    bc = ccmi.BalancingConstraint()
    bc.max_replicas_per_broker = 6
    bc.goal_violation_distribution_threshold_multiplier = 2.0
    bc.broker_sets = TEST_BROKER_SETS
    bc.broker_set_policy = policy
    return bc


# DeterministicClusterTest.java:264-334: (model, goals, expected exception)
DECKS = []
for _m in ("brokerSetSatisfiable1", "brokerSetSatisfiable2", "brokerSetSatisfiable3", "brokerSetSatisfiable4"):
    DECKS += [(_m, [BSA], None), (_m, DECK_GOALS, None)]
DECKS += [("brokerSetSatisfiable5", [BSA], None), ("brokerSetSatisfiable5", [BSA, "DiskCapacityGoal"], None),
          ("brokerSetSatisfiable5", ["DiskCapacityGoal", BSA], None)]
for _m in ("brokerSetSatisfiable6", "brokerSetSatisfiable8"):
    DECKS += [(_m, [BSA], None), (_m, DECK_GOALS, None)]
DECKS += [("brokerSetUnSatisfiable1", [BSA], OFE), ("brokerSetUnSatisfiable1", DECK_GOALS, OFE),
          ("brokerSetUnSatisfiable1", ["DiskCapacityGoal", BSA], OFE),
          ("brokerSetUnSatisfiable3", [BSA], OFE), ("brokerSetUnSatisfiable3", DECK_GOALS, OFE),
          ("brokerSetUnSatisfiable4", ["DiskUsageDistributionGoal", BSA], OFE),
          ("brokerSetUnSatisfiable4", [BSA, "DiskUsageDistributionGoal"], None)]
DECK_IDS = [f"{m}-{'+'.join(g.replace('Goal', '') for g in goals)}" for m, goals, _ in DECKS]


def run_deck(runner, model, goals, expected):
    m = MODELS[model]
    flat = build_model(m)
    pre, res, err = runner(flat, goals, deck_constraint())
    if expected == OFE:
        assert isinstance(err, ccmi.OptimizationFailureException), (err, res)
        return flat
    if err is not None:  # DeterministicClusterTest.test(): only "Insufficient capacity for" may fail
        assert isinstance(err, ccmi.OptimizationFailureException) and "Insufficient capacity for" in str(err), err
        return flat
    final, proposals, goal_results = res
    problems = [verify_broken_brokers(m["dead"], final),
                verify_soft_goal_replica_movements(proposals, offline_replicas(flat, m), goals),
                verify_regression(goal_results, pre, deck_constraint())]
    problems = [p for p in problems if p]
    assert not problems, problems
    # the reference's sanity check passed: every topic now lives inside one broker set
    d = flat.desc
    sets = {b: n for n, ids in TEST_BROKER_SETS.items() for b in ids}
    by_topic = {}
    for slot in range(d.num_replicas):
        p = d.replica_partition[d.partition_replicas[slot]]
        by_topic.setdefault(d.partition_topic[p], set()).add(sets.get(final[slot], "unmapped"))
    assert all(len(v) == 1 for v in by_topic.values()), by_topic
    return flat


# ----------------------------------------------------------------------------------------------- KAT: topic hash
KAT = [(["BS1", "BS2"], {"A": "BS2", "B": "BS1", "C": "BS1", "D": "BS1"}),
       (["BS1", "BS2", "BS3"], {"A": "BS2", "B": "BS1", "C": "BS3", "D": "BS3"})]


def test_oracle_topic_name_hash_kat(oracle_lib):
    for sets, expected in KAT:
        for topic, bs in expected.items():
            assert sets[Oracle.lib().oc_topic_broker_set(topic.encode(), len(sets))] == bs


def test_abi_topic_name_hash_kat():
    L = ccmi.Library.get().lib
    for sets, expected in KAT:
        for topic, bs in expected.items():
            assert sets[L.ccmi_topic_broker_set(topic.encode(), len(sets))] == bs


def test_abi_topic_name_hash_matches_oracle_on_many_names(oracle_lib):
    L = ccmi.Library.get().lib
    rng = random.Random(7)
    for i in range(3000):
        name = "".join(rng.choice("abcdefghijklmnopqrstuvwxyz_-.0123456789") for _ in range(rng.randint(0, 40)))
        n = rng.randint(1, 50)
        assert L.ccmi_topic_broker_set(name.encode(), n) == Oracle.lib().oc_topic_broker_set(name.encode(), n), name


# ----------------------------------------------------------------------------------------------- decks
@pytest.mark.parametrize("deck", DECKS, ids=DECK_IDS)
def test_oracle_broker_set_deck(oracle_lib, deck):
    run_deck(oracle_runner, *deck)


@pytest.mark.parametrize("deck", DECKS, ids=DECK_IDS)
def test_emu_broker_set_deck_matches_oracle(emu_lib, oracle_lib, deck):
    model, goals, expected = deck
    flat = run_deck(product_runner(emu_lib), model, goals, expected)
    check_desc_against_oracle(emu_lib, flat.desc, flat, goals, deck_constraint())


@pytest.mark.gpu
@pytest.mark.parametrize("deck", DECKS, ids=DECK_IDS)
def test_gpu_broker_set_deck_matches_oracle(gpu_lib, oracle_lib, deck):
    model, goals, expected = deck
    flat = run_deck(product_runner(gpu_lib), model, goals, expected)
    check_desc_against_oracle(gpu_lib, flat.desc, flat, goals, deck_constraint())


# ----------------------------------------------------------------------------------------------- ExcludedTopicsTest
TOPIC0, TOPIC1 = "topic0", "topic1"
# ExcludedTopicsTest.java:303-321: (model, excluded, exception, optimized, proposals)
EXCL_ROWS = [("brokerSetSatisfiable1", [TOPIC0], None, True, False),
             ("brokerSetSatisfiable2", [TOPIC0], None, True, False),
             ("brokerSetUnSatisfiable1", [], OFE, None, None),
             ("brokerSetSatisfiableAfterTopicExclusion", [TOPIC1], None, True, False)]


def _excl_run(lib, model, excluded):
    flat = build_model(MODELS[model])
    names = [flat.desc.topic_names[t].decode() for t in range(flat.desc.num_topics)]
    opts = ccmi.OptimizationOptions(excluded_topics=[names.index(t) for t in excluded if t in names])
    bc = deck_constraint()
    if lib is None:
        oc = OracleCluster.from_desc(flat.desc)
        res = oc.optimize([BSA], bc, opts)
        return res[0].succeeded, oc.proposals()
    cm = ccmi.ClusterModel(flat.desc, device=0, lib=lib, keepalive=flat)
    res = ccmi.GoalOptimizer(bc).optimizations(cm, [ccmi.BrokerSetAwareGoal()], opts)
    return res.goal_results[0].succeeded, res.proposals


def check_excl_row(lib, row):
    model, excluded, exc, optimized, proposals = row
    if exc == OFE:
        with pytest.raises(ccmi.OptimizationFailureException):
            _excl_run(lib, model, excluded)
        return
    ok, props = _excl_run(lib, model, excluded)
    assert bool(ok) == optimized
    assert bool(props) == proposals


@pytest.mark.parametrize("row", EXCL_ROWS, ids=[f"{r[0]}-{r[1]}" for r in EXCL_ROWS])
def test_oracle_excluded_topics_rows(oracle_lib, row):
    check_excl_row(None, row)


@pytest.mark.parametrize("row", EXCL_ROWS, ids=[f"{r[0]}-{r[1]}" for r in EXCL_ROWS])
def test_emu_excluded_topics_rows(emu_lib, row):
    check_excl_row(emu_lib, row)


@pytest.mark.gpu
@pytest.mark.parametrize("row", EXCL_ROWS, ids=[f"{r[0]}-{r[1]}" for r in EXCL_ROWS])
def test_gpu_excluded_topics_rows(gpu_lib, row):
    check_excl_row(gpu_lib, row)


# ----------------------------------------------------------------------------------------------- RandomCluster
def random_case(num_topics, unmapped=False):
    """A RandomCluster with broker sets "east" 0..11 and "west" 12..23 under the default TopicNameHash policy: most
    topics start spread over both sets, so the goal moves many replicas. unmapped=True leaves broker 23 out of the data
    (NoOpBrokerSetAssignmentPolicy puts it into "unmapped"): a topic hashed to that one-broker set cannot be placed and
    the goal fails, as in the reference."""
    buf = ccmi.RandomCluster.generate(num_racks=4, num_brokers=24, num_replicas=1200, num_topics=num_topics)
    bc = ccmi.BalancingConstraint()
    bc.broker_sets = {"east": list(range(0, 12)), "west": list(range(12, 23 if unmapped else 24))}
    return buf, bc


@pytest.mark.parametrize("goals", [[BSA], [BSA, "ReplicaCapacityGoal", "DiskCapacityGoal", "ReplicaDistributionGoal",
                                          "CpuUsageDistributionGoal", "LeaderReplicaDistributionGoal"]],
                         ids=["alone", "chain"])
def test_emu_random_topic_hash_matches_oracle(emu_lib, oracle_lib, goals):
    buf, bc = random_case(40)
    _, res, _ = check_desc_against_oracle(emu_lib, buf.desc, buf, goals, bc)
    assert res is not None and res.goal_results[0].actions > 100  # the goal succeeded after many moves


def test_emu_random_unmapped_broker_fails_like_oracle(emu_lib, oracle_lib):
    buf, bc = random_case(40, unmapped=True)
    _, res, _ = check_desc_against_oracle(emu_lib, buf.desc, buf, [BSA], bc)
    assert res is None  # both raised the same OptimizationFailureException


def test_emu_broker_set_member_outside_session_ignored(emu_lib, oracle_lib):
    """Members are the session's dense broker indices (ccmi_builder_broker_ids order); -1 or an id outside [0, B) (a
    Kafka id the model does not hold) resolves to no broker, as an absent broker does in the reference: "west" naming
    1001 and -1 instead of broker 23 leaves 23 unmapped, exactly the unmapped case, with the same failure."""
    buf, bc = random_case(40, unmapped=True)
    bc.broker_sets["west"] = bc.broker_sets["west"] + [1001, -1]
    _, res, _ = check_desc_against_oracle(emu_lib, buf.desc, buf, [BSA], bc)
    assert res is None


@pytest.mark.gpu
@pytest.mark.parametrize("goals", [[BSA], [BSA, "ReplicaCapacityGoal", "DiskCapacityGoal", "ReplicaDistributionGoal",
                                          "CpuUsageDistributionGoal", "LeaderReplicaDistributionGoal"]],
                         ids=["alone", "chain"])
def test_gpu_random_topic_hash_matches_oracle(gpu_lib, oracle_lib, goals):
    buf, bc = random_case(40)
    check_desc_against_oracle(gpu_lib, buf.desc, buf, goals, bc)


# ----------------------------------------------------------------------------------------------- actionAcceptance
def _acceptance_pairs(lib):
    """BrokerSetAwareGoal.actionAcceptance on random moves after a broker-set chain: product vs oracle."""
    buf, bc = random_case(60)
    goals = [BSA, "ReplicaDistributionGoal"]
    cm = ccmi.ClusterModel(buf.desc, device=0, lib=lib, keepalive=buf)
    ccmi.GoalOptimizer(bc).optimizations(cm, ccmi.goals_from_names(goals))
    oc = OracleCluster.from_desc(buf.desc)
    oc.optimize(goals, bc)
    assert cm.actions() == oc.actions()
    dist = cm.replica_distribution()
    d = buf.desc
    rng = random.Random(11)
    out = []
    for _ in range(300):
        slot = rng.randrange(d.num_replicas)
        p = d.replica_partition[d.partition_replicas[slot]]
        src = dist[slot]
        dst = rng.randrange(d.num_brokers)
        typ = ccmi.ACTION_TYPES.index("INTER_BROKER_REPLICA_MOVEMENT")
        got = cm.action_acceptance_by_goal(BSA, typ, p, src, dst)
        want = oc.action_acceptance(0, typ, p, src, dst)
        out.append((got, want))
    return out


def test_emu_broker_set_acceptance_matches_oracle(emu_lib, oracle_lib):
    pairs = _acceptance_pairs(emu_lib)
    assert all(g == w for g, w in pairs)
    assert {w for _, w in pairs} >= {"ACCEPT", "BROKER_REJECT"}


@pytest.mark.gpu
def test_gpu_broker_set_acceptance_matches_oracle(gpu_lib, oracle_lib):
    pairs = _acceptance_pairs(gpu_lib)
    assert all(g == w for g, w in pairs)


# ------------------------------------------------------------------------------------------ non-dense Kafka ids
def _builder_model_with_kafka_ids(lib):
    """A LoadMonitor-built model whose Kafka broker ids are 1000 + 7 i (not the dense session indices)."""
    import ctypes as C
    rng = random.Random(5)
    m = ccmi.LoadMonitorModel(num_windows=1, lib=lib)
    kafka = [1000 + 7 * i for i in range(24)]
    cap = {"CPU": 100.0, "NW_IN": 100000.0, "NW_OUT": 100000.0, "DISK": 500000.0}
    for i, k in enumerate(kafka):
        m.create_broker(f"rack{i % 4}", f"h{k}", k, cap)
    for t in range(40):
        for p in range(10):
            reps = rng.sample(kafka, 3)
            met = {mm: [C.c_float(rng.uniform(1, 50)).value] for mm in ccmi.LoadMonitorModel.METRICS}
            met["CPU_USAGE"] = [C.c_float(rng.uniform(0, 0.02)).value]
            m.populate_partition(f"topic{t}", p, reps, reps[0], met)
    return m, kafka


def _kafka_id_sets(lib):
    """broker_sets name Kafka ids; BalancingConstraint.to_struct maps them through the session's broker_ids() to the
    dense indices of ccmi_balancing_constraint (an id the model does not hold, 99, maps to -1 = no broker). The oracle
    gets the same sets written as indices: both must agree bit for bit."""
    m, kafka = _builder_model_with_kafka_ids(lib)
    cm = ccmi.ClusterModel(m.desc(), device=0, lib=lib, keepalive=m)
    assert cm.broker_ids() == sorted(kafka)
    by_kafka = ccmi.BalancingConstraint()
    by_kafka.broker_sets = {"east": kafka[:12] + [99], "west": kafka[12:]}
    by_index = ccmi.BalancingConstraint()
    by_index.broker_sets = {"east": list(range(12)) + [-1], "west": list(range(12, 24))}
    res = ccmi.GoalOptimizer(by_kafka).optimizations(cm, ccmi.goals_from_names([BSA]))
    oc = OracleCluster.from_desc(m.desc())
    ores = oc.optimize([BSA], by_index)
    assert cm.actions() == oc.actions() and res.goal_results[0].actions == ores[0].actions > 0
    assert cm.replica_distribution() == oc.replica_distribution()


def test_emu_broker_sets_by_kafka_id(emu_lib, oracle_lib):
    _kafka_id_sets(emu_lib)


@pytest.mark.gpu
def test_gpu_broker_sets_by_kafka_id(gpu_lib, oracle_lib):
    _kafka_id_sets(gpu_lib)
