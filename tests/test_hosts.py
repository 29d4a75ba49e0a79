"""Hosts (include/ccmi.h broker_host; ABI v8 host aggregates).

The reference keeps a Host per (rack, host name) (Rack._hosts.computeIfAbsent, model/Rack.java:256-262; LoadMonitor
passes node.host(), LoadMonitor.java:602; handleDeadBroker names a dead broker's host UNKNOWN_HOST-<n>,
ClusterModel.java:776-777) with its own load, capacity and replica set (model/Host.java). CapacityGoal and
ResourceDistributionGoal test the host resources CPU, NW_IN and NW_OUT (Resource.java:19-25) against the host
(CapacityGoal.java:230-239,284-366,389-408,455-475; ResourceDistributionGoal.java:880-927,982-1037;
ClusterModel.aliveBrokers{Under,Over}Threshold / sortedAliveBrokersUnderThreshold :1049-1126), and ClusterModelStats
reports host utilization for them (ClusterModelStats.java:297-303).

No reference fixture shares a host (RandomCluster names every host after its broker, RandomCluster.java:80,87), so the
shared-host decisions are pinned by the restatement (oracle/src/model.cpp Host bookkeeping) and by the reference's own
ClusterModel.sanityCheck invariant: a host's utilization is the sum of its brokers' (ClusterModel.java:1224-1235,
checked here within Resource.epsilon). Product (CPU emulation; gfx950 under -m gpu) and oracle agree bit for bit.
"""
import ctypes as C

import pytest

import ccmi
from oracle_binding import OracleCluster
from parity import assign_shared_hosts, check_desc_against_oracle, constraint

CAP = {"CPU": 100.0, "DISK": 300000.0, "NW_IN": 300000.0, "NW_OUT": 200000.0}
HOST_GOALS = ["CpuCapacityGoal", "NetworkInboundCapacityGoal", "NetworkOutboundCapacityGoal",
              "CpuUsageDistributionGoal", "NetworkInboundUsageDistributionGoal",
              "NetworkOutboundUsageDistributionGoal"]
DEFAULT_GOALS = list(ccmi.DEFAULT_GOALS)


def _model(hosts, nw_in=None):
    """6 brokers on 2 racks; hosts[b] names broker b's host (None: a host of its own). nw_in[b] overrides the NW_IN
    load of broker b's leader replicas."""
    b = ccmi.ClusterModelBuilder()
    for bid in range(6):
        b.create_broker(f"r{bid % 2}", bid, CAP, host=hosts[bid])
    for t in range(4):
        for p in range(6):
            brokers = [(p + t) % 6, (p + t + 1) % 6]
            for i, br in enumerate(brokers):
                b.create_replica(f"r{br % 2}", br, f"T{t}", p, i, i == 0)
                nwi = 10.0 * (t + 1) if nw_in is None else nw_in[br]
                b.set_replica_load(f"r{br % 2}", br, f"T{t}", p, 1.0 + p, nwi, 5.0 * (p + 1), 100.0 + t)
    return b.build()


SHARED = ["hA", "hB", "hA", None, "hC", "hC"]  # 0 and 2 share hA in r0; "hC" names one host in r0 and one in r1
SHARED_SAME_RACK = ["hA", "hB", "hA", "hB", None, None]  # 0 and 2 share hA in r0, 1 and 3 share hB in r1
SAME_NAME_OTHER_RACKS = ["h", "h", None, None, None, None]  # one name in two racks: two hosts
OWN = [f"h{b}" for b in range(6)]


def _shared_random(lib, per_host=2, **props):
    """A RandomCluster whose brokers share hosts (parity.assign_shared_hosts). Returns (buffers, host array kept alive
    with them)."""
    buf = ccmi.RandomCluster.generate(lib, **props)
    return buf, assign_shared_hosts(buf, per_host)


RANDOM = dict(num_racks=5, num_brokers=24, num_replicas=6000, num_topics=300)


# ------------------------------------------------------------------------------------------------ oracle
def test_oracle_host_is_sum_of_its_brokers(oracle_lib, emu_lib):
    """ClusterModel.sanityCheck (ClusterModel.java:1224-1235): after a chain that moves replicas and leaders, each
    host's utilization equals its brokers' summed utilization within Resource.epsilon."""
    buf, arr = _shared_random(emu_lib, per_host=3, **RANDOM)
    oc = OracleCluster.from_desc(buf.desc)
    oc.optimize(DEFAULT_GOALS, constraint(1.05))
    assert oc.actions()
    d = buf.desc
    members = {}
    for b in range(d.num_brokers):
        members.setdefault(arr[b], []).append(b)
    for h, bs in members.items():
        for res in range(3):
            total = sum(oc.broker_util(b, res) for b in bs)
            host = oc.host_util(bs[0], res)
            eps = max({0: 0.001, 1: 10.0, 2: 10.0}[res], 0.0008 * (host + total))
            assert abs(host - total) <= eps, (h, res, host, total)


def test_oracle_host_capacity_changes_the_decision(oracle_lib):
    """NW_IN is a host-only resource: broker 0 alone is over its NW_IN capacity limit, but on a host with broker 2
    the host is under the host limit (twice the capacity), so NetworkInboundCapacityGoal has nothing to do."""
    nw = [260000.0 / 8, 10.0, 1000.0, 10.0, 10.0, 10.0]
    own = OracleCluster.from_desc(_model(OWN, nw).desc)
    shared = OracleCluster.from_desc(_model(SHARED_SAME_RACK, nw).desc)
    bc = ccmi.BalancingConstraint()
    assert own.optimize(["NetworkInboundCapacityGoal"], bc)[0].actions > 0
    assert shared.optimize(["NetworkInboundCapacityGoal"], bc)[0].actions == 0


# ------------------------------------------------------------------------------------------------ product vs oracle
@pytest.mark.parametrize("hosts", [SHARED, SHARED_SAME_RACK], ids=["shared", "shared-same-rack"])
@pytest.mark.parametrize("goals", [["ReplicaDistributionGoal"] + HOST_GOALS, DEFAULT_GOALS], ids=["host-goals", "default"])
def test_emu_shared_host_builder_matches_oracle(emu_lib, oracle_lib, hosts, goals):
    flat = _model(hosts)
    check_desc_against_oracle(emu_lib, flat.desc, flat, goals, ccmi.BalancingConstraint())


@pytest.mark.parametrize("per_host", [2, 3])
def test_emu_shared_host_random_cluster_matches_oracle(emu_lib, oracle_lib, per_host):
    buf, arr = _shared_random(emu_lib, per_host=per_host, **RANDOM)
    _, res, _ = check_desc_against_oracle(emu_lib, buf.desc, (buf, arr), DEFAULT_GOALS, constraint(1.05))
    assert res is not None and res.goal_results


def test_emu_shared_host_dead_brokers_match_oracle(emu_lib, oracle_lib):
    """Host.setBrokerState: a dead broker's capacity leaves its host (the host stays alive with its other broker)."""
    buf, arr = _shared_random(emu_lib, per_host=2, **dict(RANDOM, num_dead_brokers=3, rack_aware=1))
    check_desc_against_oracle(emu_lib, buf.desc, (buf, arr), DEFAULT_GOALS, constraint(1.05))


@pytest.mark.parametrize("hosts", [OWN, SAME_NAME_OTHER_RACKS, [None] * 6], ids=["named", "same-name", "unnamed"])
def test_emu_distinct_hosts_run_every_goal(emu_lib, oracle_lib, hosts):
    flat = _model(hosts)
    check_desc_against_oracle(emu_lib, flat.desc, flat, ["ReplicaDistributionGoal"] + HOST_GOALS,
                              ccmi.BalancingConstraint())


def test_emu_host_index_across_racks_is_invalid(emu_lib):
    flat = _model(OWN)
    bad = (ccmi.C.c_int32 * 6)(0, 0, 1, 2, 3, 4)  # brokers 0 (r0) and 1 (r1) on one host index
    flat.desc.broker_host = ccmi.C.cast(bad, ccmi.C.POINTER(ccmi.C.c_int32))
    with pytest.raises(ccmi.IllegalArgumentException, match="different racks"):
        ccmi.ClusterModel(flat.desc, device=0, lib=emu_lib, keepalive=(flat, bad))


def _load_monitor_shared(lib):
    """The native builder keys hosts by (rack, name); a broker only partitions name (handleDeadBroker) is alone on an
    UNKNOWN_HOST; two live brokers named on one host share it."""
    m = ccmi.LoadMonitorModel(num_windows=1, lib=lib)
    m.create_broker("rack0", "node-a", 0, CAP)
    m.create_broker("rack1", "node-a", 1, CAP)  # same name, other rack: another host
    m.create_broker("rack0", "node-b", 2, CAP)
    m.create_broker("rack0", "node-b", 3, CAP)  # shares node-b with broker 2
    m.create_broker("rack1", "node-c", 4, CAP)
    for p in range(12):
        reps = [p % 5, (p + 2) % 5]
        if 3 in reps and p % 4 == 0:
            reps = [x if x != 3 else 5 for x in reps]
            m.create_broker("rack1", "node-d", 5, CAP, alive=False)  # dead: UNKNOWN_HOST-0
        m.populate_partition("t", p, reps, reps[0], {"CPU_USAGE": [0.02 + 0.01 * p], "DISK_USAGE": [10.0 + p],
                                                    "LEADER_BYTES_IN": [1000.0 * (p + 1)],
                                                    "LEADER_BYTES_OUT": [800.0 * (p + 1)]})
    return m


def test_emu_load_monitor_shared_host_matches_oracle(emu_lib, oracle_lib):
    m = _load_monitor_shared(emu_lib)
    d = m.desc()
    hosts = [d.broker_host[b] for b in range(d.num_brokers)]
    assert hosts[2] == hosts[3] and len(set(hosts)) == d.num_brokers - 1
    check_desc_against_oracle(emu_lib, d, m, ["ReplicaDistributionGoal"] + HOST_GOALS, ccmi.BalancingConstraint())


# ------------------------------------------------------------------------------------------------ gfx950
@pytest.mark.gpu
@pytest.mark.parametrize("hosts", [SHARED, SHARED_SAME_RACK], ids=["shared", "shared-same-rack"])
@pytest.mark.parametrize("goals", [["ReplicaDistributionGoal"] + HOST_GOALS, DEFAULT_GOALS], ids=["host-goals", "default"])
def test_gpu_shared_host_builder_matches_oracle(gpu_lib, oracle_lib, hosts, goals):
    flat = _model(hosts)
    check_desc_against_oracle(gpu_lib, flat.desc, flat, goals, ccmi.BalancingConstraint())


@pytest.mark.gpu
@pytest.mark.parametrize("per_host", [2, 3])
def test_gpu_shared_host_random_cluster_matches_oracle(gpu_lib, oracle_lib, per_host):
    buf, arr = _shared_random(gpu_lib, per_host=per_host, **RANDOM)
    check_desc_against_oracle(gpu_lib, buf.desc, (buf, arr), DEFAULT_GOALS, constraint(1.05))


@pytest.mark.gpu
def test_gpu_shared_host_dead_brokers_match_oracle(gpu_lib, oracle_lib):
    buf, arr = _shared_random(gpu_lib, per_host=2, **dict(RANDOM, num_dead_brokers=3, rack_aware=1))
    check_desc_against_oracle(gpu_lib, buf.desc, (buf, arr), DEFAULT_GOALS, constraint(1.05))


@pytest.mark.gpu
def test_gpu_load_monitor_shared_host_matches_oracle(gpu_lib, oracle_lib):
    m = _load_monitor_shared(gpu_lib)
    check_desc_against_oracle(gpu_lib, m.desc(), m, ["ReplicaDistributionGoal"] + HOST_GOALS,
                              ccmi.BalancingConstraint())


# ------------------------------------------------------------------------------------------------ C1 with shared hosts
# tests/golden/c1_shared_hosts_default.json: C1's cluster, two brokers of a rack per host, the 16 default goals — the
# K7 chains (LeaderReplicaDistribution, RackAware with optimized goals) apply moves with the host loads on the device
# (apply.h host lanes). Pinned by the oracle's Host restatement only (no reference fixture shares a host).
@pytest.mark.parametrize("pair_chains", ["0", "1"])
def test_emu_c1_shared_hosts_matches_golden(emu_lib, oracle_lib, monkeypatch, pair_chains):
    from parity import check_product_against_golden
    monkeypatch.setenv("CCMI_PAIR_CHAINS", pair_chains)
    cm, _ = check_product_against_golden(emu_lib, "c1_shared_hosts_default")
    if pair_chains == "1":
        assert cm.perf().chain_launches > 0  # the chains ran with shared hosts


@pytest.mark.gpu
@pytest.mark.parametrize("pair_chains", ["0", "1"])
def test_gpu_c1_shared_hosts_matches_golden(gpu_lib, oracle_lib, monkeypatch, pair_chains):
    from parity import check_product_against_golden
    monkeypatch.setenv("CCMI_PAIR_CHAINS", pair_chains)
    cm, res = check_product_against_golden(gpu_lib, "c1_shared_hosts_default", per_goal_stats=True)
    if pair_chains == "1":
        assert cm.perf().chain_launches + cm.perf().server_chains > 0
