"""Model ingestion: LoadMonitor.clusterModel through the native builder (ccmi_builder_*).

Pinned by LoadMonitorTest (monitor/LoadMonitorTest.java), whose clusters are two nodes (rack0, rack1) with every
partition on [0, 1] led by node 0 (MonitorUnitTestUtils.java:36-39,105-112), and whose aggregated windows follow from
CruiseControlUnitTestUtils.populateSampleAggregator (cruise-control-core, :37-58): window i, sample j records
i * 10 + j for every metric (CPU / 100), so a window's AVG is i * 10 + 1.5 and its LATEST i * 10 + 3
(KafkaMetricDef.java:43-53 aggregation functions). The expected utilizations of the partition leader are the test's
own assertions (delta 0.0).

Follower loads and the order-dependent shared-value mutation are checked against the oracle's restatement
(oracle/src/ingest.cpp), and a builder-made cluster runs the default goals bit-exactly against the oracle.
"""
import ctypes as C
import random

import pytest

import ccmi
from parity import check_desc_against_oracle, constraint

CAP = {"CPU": 100.0, "NW_IN": 100000.0, "NW_OUT": 100000.0, "DISK": 1000000.0}
M = ccmi.LoadMonitorModel.METRICS


def _windows(window_ids, samples=4):
    """Aggregated leader metrics for populateSampleAggregator windows (newest first)."""
    avg = [i * 10 + (samples - 1) / 2.0 for i in reversed(window_ids)]
    latest = [i * 10 + samples - 1 for i in reversed(window_ids)]
    met = {m: list(avg) for m in M}
    met["DISK_USAGE"] = latest
    met["CPU_USAGE"] = [C.c_float(v / 100.0).value for v in avg]
    return met


def _expected_util(load, W):
    """Load.expectedUtilizationFor (ModelUtils): CPU / NW resources average their group over the windows, DISK
    takes the newest window. load[metric][window]."""
    def avg(*ms):
        return sum(sum(load[m][w] for m in ms) for w in range(W)) / W
    return {"CPU": avg(0), "NW_IN": avg(2, 4), "NW_OUT": avg(3, 5), "DISK": load[1][0]}


def _two_node_model(lib, W):
    m = ccmi.LoadMonitorModel(num_windows=W, lib=lib)
    m.create_broker("rack0", "localhost", 0, CAP)
    m.create_broker("rack1", "localhost", 1, CAP)
    return m


def _leader_util(m, part_index=0):
    d = m.desc()
    loads = m.replica_loads()
    for r in range(d.partition_offset[part_index], d.partition_offset[part_index + 1]):
        if d.replica_is_leader[r]:
            return _expected_util(loads[r], d.num_windows)
    raise AssertionError("no leader")


def test_load_monitor_basic_cluster_model_kat(emu_lib):
    """LoadMonitorTest.testBasicClusterModel (:264-283): windows 0 and 1 -> CPU 6.5, NW_IN / NW_OUT / DISK 13."""
    m = _two_node_model(emu_lib, 2)
    for t, p in (("topic0", 0), ("topic0", 1), ("topic1", 0), ("topic1", 1)):
        m.populate_partition(t, p, [0, 1], 0, _windows([0, 1]))
    assert _leader_util(m) == {"CPU": 6.5, "NW_IN": 13.0, "NW_OUT": 13.0, "DISK": 13.0}


def test_load_monitor_one_window_kats(emu_lib):
    """LoadMonitorTest :338-345 (window 0 only: DISK 3, CPU 1.5, NW 3) and :433-443 (window 1: DISK 13, CPU 11.5,
    NW 23; T1P1 with one sample in window 1: all 10, NW 20)."""
    m = _two_node_model(emu_lib, 1)
    m.populate_partition("topic0", 0, [0, 1], 0, _windows([0]))
    assert _leader_util(m) == {"CPU": 1.5, "NW_IN": 3.0, "NW_OUT": 3.0, "DISK": 3.0}
    m = _two_node_model(emu_lib, 1)
    m.populate_partition("topic0", 0, [0, 1], 0, _windows([1]))
    m.populate_partition("topic1", 1, [0, 1], 0, _windows([1], samples=1))
    assert _leader_util(m, 0) == {"CPU": 11.5, "NW_IN": 23.0, "NW_OUT": 23.0, "DISK": 13.0}
    assert _leader_util(m, 1) == {"CPU": 10.0, "NW_IN": 20.0, "NW_OUT": 20.0, "DISK": 10.0}


def test_engine_sees_ingested_loads(emu_lib):
    """The session built from the ingested desc: ClusterModelStats over the two brokers of the basic model."""
    m = _two_node_model(emu_lib, 2)
    m.populate_partition("topic0", 0, [0, 1], 0, _windows([0, 1]))
    cm = ccmi.ClusterModel(m.desc(), device=0, lib=emu_lib, keepalive=m)
    s = cm.cluster_stats(ccmi.BalancingConstraint())
    assert s["resource_max"] == [6.5, 13.0, 13.0, 13.0]  # the leader's broker (CPU, NW_IN, NW_OUT, DISK)
    assert s["resource_min"][2] == 0.0                     # a follower has no NW_OUT


def _oracle_partition(oracle_lib, W, leader_flags, met):
    n = len(leader_flags)
    vals = [float(x) for mm in M for x in met[mm]]
    out = (C.c_float * (n * 6 * W))()
    oracle_lib.oc_ingest_partition.restype = C.c_int32
    oracle_lib.oc_ingest_partition(W, n, (C.c_uint8 * n)(*leader_flags), (C.c_float * len(vals))(*vals), out)
    return [[[out[(i * 6 + mm) * W + w] for w in range(W)] for mm in range(6)] for i in range(n)]


def _random_cluster_via_builder(lib, seed, W=3, B=12, racks=3, topics=20, parts=8, dead=(), bad=(), offline_p=0.0):
    rng = random.Random(seed)
    m = ccmi.LoadMonitorModel(num_windows=W, lib=lib)
    ids = list(range(B))
    rng.shuffle(ids)  # populateClusterCapacity may shuffle the nodes
    for b in ids:
        if b in dead:
            continue
        m.create_broker(f"rack{b % racks}", f"h{b}", b, CAP)
    expected = []
    for t in range(topics):
        for p in range(parts):
            rf = rng.choice([2, 3, 3, 4])
            reps = rng.sample(range(B), rf)
            for b in reps:
                if b in dead:
                    m.create_broker(f"rack{b % racks}", f"UNKNOWN-{b}", b, CAP, alive=False)
            leader = reps[rng.randrange(rf)]
            met = {mm: [C.c_float(rng.uniform(0, 50)).value for _ in range(W)] for mm in M}
            met["CPU_USAGE"] = [C.c_float(rng.uniform(0, 0.02)).value for _ in range(W)]
            if rng.random() < 0.2:
                met["REPLICATION_BYTES_OUT_RATE"] = [0.0] * W  # not reported (Kafka), filled for the leader
            if rng.random() < 0.1:
                for mm in ("LEADER_BYTES_IN", "REPLICATION_BYTES_IN_RATE", "LEADER_BYTES_OUT",
                           "REPLICATION_BYTES_OUT_RATE"):
                    met[mm] = [0.0] * W  # idle partition: follower CPU 0
            off = [b for b in reps if b in bad and rng.random() < offline_p]
            m.populate_partition(f"topic{t}", p, reps, leader, met, offline=off)
            expected.append(([1 if b == leader else 0 for b in reps], met))
    for b in dead:
        m.set_broker_state(b, "DEAD")
    for b in bad:
        m.set_broker_state(b, "BAD_DISKS")
    return m, expected


def test_follower_loads_match_oracle(emu_lib, oracle_lib):
    """Every replica load the builder derives equals the oracle's restatement of populatePartitionLoad (leader first
    or not, unreported replication bytes out, idle partitions)."""
    W = 3
    m, expected = _random_cluster_via_builder(emu_lib, 11, W=W)
    loads = m.replica_loads()
    d = m.desc()
    for p, (flags, met) in enumerate(expected):
        want = _oracle_partition(oracle_lib, W, flags, met)
        got = loads[d.partition_offset[p]:d.partition_offset[p + 1]]
        assert got == want, p


def test_builder_errors(emu_lib):
    m = ccmi.LoadMonitorModel(num_windows=2, lib=emu_lib)
    m.create_broker("r", "h", 3, CAP)
    with pytest.raises(ccmi.IllegalArgumentException, match="unknown broker"):
        m.populate_partition("t", 0, [3, 4], 3, _windows([0, 1]))
    with pytest.raises(ccmi.IllegalArgumentException, match="windows"):
        m.populate_partition("t", 0, [3], 3, _windows([0]))
    with pytest.raises(ccmi.IllegalArgumentException, match="created twice"):
        m.create_broker("r", "h", 3, CAP)
    m.create_broker("r2", "h", 7, CAP, alive=False)
    m.create_broker("r", "h", 7, CAP, alive=False)  # handleDeadBroker on a known broker: no-op
    m.populate_partition("t", 0, [3, 7], None, _windows([0, 1]))  # offline partition: skipped
    assert m.desc().num_replicas == 0
    m.populate_partition("t", 1, [7, 3], 3, _windows([0, 1]))
    assert m.broker_ids() == [3, 7]
    d = m.desc()
    assert [d.replica_broker[r] for r in range(2)] == [1, 0] and d.broker_state[1] == 1  # dense ids, 7 is DEAD


INGEST_CASES = [
    dict(seed=1),
    dict(seed=2, dead=(4, 9)),
    dict(seed=3, bad=(2, 5), offline_p=0.5),
]


@pytest.mark.parametrize("case", INGEST_CASES, ids=["alive", "dead", "bad-disks"])
def test_emu_ingested_model_matches_oracle(emu_lib, oracle_lib, case):
    m, _ = _random_cluster_via_builder(emu_lib, **case)
    check_desc_against_oracle(emu_lib, m.desc(), m, list(ccmi.DEFAULT_GOALS), constraint(1.05, 3000))


@pytest.mark.gpu
@pytest.mark.parametrize("case", INGEST_CASES, ids=["alive", "dead", "bad-disks"])
def test_gpu_ingested_model_matches_oracle(gpu_lib, oracle_lib, case):
    m, _ = _random_cluster_via_builder(gpu_lib, **case)
    check_desc_against_oracle(gpu_lib, m.desc(), m, list(ccmi.DEFAULT_GOALS), constraint(1.05, 3000))
