"""New brokers: RandomClusterTest.testNewBrokers (analyzer/RandomClusterTest.java:198-244), the parameterized
suites RandomCluster{Uniform,Linear,Exp}DistNewBrokerTest run it over.

The cluster is balanced once, rebuilt from its balanced state with every replica created where it now lives (so its
original broker is its current one), and two NEW brokers are added (ids B and B+1, racks "1" and "2",
TestConstants.BROKER_CAPACITY: RandomClusterTest.java:231-239). The goals then run again. Paths this exercises:
GoalUtils.eligibleBrokers' new-broker filter (GoalUtils.java:193-198), eligibleReplicasForSwap CASE#1/#3 (:276-297),
ResourceDistributionGoal / ReplicaDistributionGoal / TopicReplicaDistributionGoal brokersToBalance and skip rules.

Pinning: OptimizationVerifier NEW_BROKERS (OptimizationVerifier.java:293-317: no old broker receives a replica, every
new broker's DISK utilization reaches the balance lower limit) and REGRESSION on the oracle; product (CPU emulation,
gfx950 under -m gpu) equals the oracle bit for bit. The rebuilt model keeps the oracle's replica and slot order
(the reference iterates getPartitionsByTopic(), a HashMap: the order only changes tie-breaking, not the pinning).
"""
import pytest

import ccmi
from oracle_binding import ArrayDesc, OracleCluster
from parity import check_desc_against_oracle
from verifier import verify_regression

DEFAULT_GOALS = list(ccmi.DEFAULT_GOALS)
BROKER_CAPACITY = [100.0, 300000.0, 200000.0, 300000.0]  # TestConstants.java:105-107 (CPU, NW_IN, NW_OUT, DISK)
DISK_METRIC = ccmi.METRIC_OF_RESOURCE["DISK"]


def constraint(max_replicas=1500):
    """RandomClusterTest.java:130-139: LOW_BALANCE_PERCENTAGE 1.05, MEDIUM_CAPACITY_THRESHOLD 0.8."""
    bc = ccmi.BalancingConstraint()
    bc.max_replicas_per_broker = max_replicas
    bc.set_resource_balance_percentage(1.05)
    bc.set_capacity_threshold(0.8)
    return bc


CASES = [
    (dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300), DEFAULT_GOALS, 1500),
    (dict(num_racks=5, num_brokers=40, num_replicas=12000, num_topics=500), DEFAULT_GOALS, 3000),
    (dict(num_brokers=40, num_replicas=12000, num_topics=500, min_replication=4, max_replication=4),
     DEFAULT_GOALS, 1500),
    (dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300), list(ccmi.C1_GOALS), 1500),
    # RandomClusterTest.data's own rows (RandomClusterTest.java:143-176) over BASE_PROPERTIES (TestConstants.java:89-95)
    (dict(num_brokers=80), DEFAULT_GOALS, 1500),
    (dict(num_replicas=50000, min_replication=5, max_replication=5), DEFAULT_GOALS, 3000),
]
IDS = ["b20", "b40", "rf4", "c1goals", "ref-brokers80", "ref-rf5"]


def new_broker_model(props, goals, bc, n_new=2):
    """RandomClusterTest.testNewBrokers: rebalance, rebuild from the balanced state, add NEW brokers."""
    oc = OracleCluster.random(**props)
    oc.optimize(goals, bc)
    a = oc.export()
    B, R = len(a["broker_rack"]), len(a["replica_partition"])
    a["broker_state"] = [0] * B + [ccmi.BROKER_STATES["NEW"]] * n_new
    a["broker_rack"] = a["broker_rack"] + [1 + i for i in range(n_new)]
    a["cap"] = a["cap"] + BROKER_CAPACITY * n_new
    a["offline"] = [0] * R
    return ArrayDesc(a, oc.W)


def verify_new_brokers(desc, oc, bc):
    """OptimizationVerifier.verifyNewBrokers (:293-317) on the oracle's final state."""
    a = oc.export()
    B = desc.num_brokers
    new = {b for b in range(B) if desc.broker_state[b] == ccmi.BROKER_STATES["NEW"]}
    # no old broker holds a replica it did not start with (Replica.originalBroker() == broker)
    for p in range(desc.num_partitions):
        o0, o1 = desc.partition_offset[p], desc.partition_offset[p + 1]
        before = {desc.replica_broker[desc.partition_replicas[i]] for i in range(o0, o1)}
        after = {a["replica_broker"][r] for r in a["partition_replicas"][o0:o1]}
        assert (after - before) <= new, (p, before, after)
    # each new broker's DISK utilization is at least the cluster's average times (2 - balance percentage)
    W = oc.W
    disk = [0.0] * B
    for r in range(desc.num_replicas):
        disk[a["replica_broker"][r]] += a["load"][(r * 6 + DISK_METRIC) * W + W - 1]
    cap = [a["cap"][4 * b + 3] for b in range(B)]
    lower = sum(disk) / sum(cap) * (2 - 1.05)
    for b in new:
        assert disk[b] / cap[b] >= lower, (b, disk[b] / cap[b], lower)


@pytest.mark.parametrize("props,goals,max_replicas", CASES, ids=IDS)
def test_oracle_new_brokers_verifications(oracle_lib, props, goals, max_replicas):
    bc = constraint(max_replicas)
    m = new_broker_model(props, goals, bc)
    oc = OracleCluster.from_desc(m.desc)
    pre = oc.stats(bc)
    res = oc.optimize(goals, bc)
    verify_new_brokers(m.desc, oc, bc)               # NEW_BROKERS
    assert verify_regression(res, pre, bc) is None   # REGRESSION (no self-healing replicas)
    assert oc.actions(), "the new brokers received nothing"


@pytest.mark.parametrize("props,goals,max_replicas", CASES, ids=IDS)
def test_emu_new_brokers_match_oracle(emu_lib, oracle_lib, props, goals, max_replicas):
    bc = constraint(max_replicas)
    m = new_broker_model(props, goals, bc)
    check_desc_against_oracle(emu_lib, m.desc, m, goals, bc)


def test_emu_new_brokers_with_requested_destinations(emu_lib, oracle_lib):
    """Requested destinations switch the new-broker filter of eligibleBrokers off (GoalUtils.java:189-191) but not
    the one of eligibleReplicasForSwap."""
    bc = constraint(1500)
    m = new_broker_model(CASES[0][0], DEFAULT_GOALS, bc)
    opts = ccmi.OptimizationOptions(requested_destination_broker_ids=[3, 7, 20, 21], fast_mode=False)
    check_desc_against_oracle(emu_lib, m.desc, m, DEFAULT_GOALS, bc, opts)


@pytest.mark.gpu
@pytest.mark.parametrize("props,goals,max_replicas", CASES, ids=IDS)
def test_gpu_new_brokers_match_oracle(gpu_lib, oracle_lib, props, goals, max_replicas):
    bc = constraint(max_replicas)
    m = new_broker_model(props, goals, bc)
    check_desc_against_oracle(gpu_lib, m.desc, m, goals, bc)
