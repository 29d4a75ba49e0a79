"""Hosts at the boundary (include/ccmi.h broker_host, ABI v6).

The reference keeps a Host per (rack, host name) (Rack._hosts.computeIfAbsent, model/Rack.java:256-262; LoadMonitor
passes node.host(), LoadMonitor.java:602; handleDeadBroker names a dead broker's host UNKNOWN_HOST-<n>,
ClusterModel.java:776-777). CapacityGoal and ResourceDistributionGoal test host load against host capacity for the
host resources CPU, NW_IN and NW_OUT (CapacityGoal.java:230-239,395-399,457-466; ResourceDistributionGoal.java:890-923;
Resource.java:19-25). With one broker per host that is the broker's own load and capacity, which is what this build
evaluates; a chain with one of those goals on a model where brokers share a host fails with
UnsupportedOperationException (CCMI_E_UNSUPPORTED) rather than produce decisions the reference would not make.
Goals that never read hosts run normally on such models and match the oracle.
"""
import pytest

import ccmi
from parity import check_desc_against_oracle

CAP = {"CPU": 100.0, "DISK": 300000.0, "NW_IN": 300000.0, "NW_OUT": 200000.0}
HOST_GOALS = ["CpuCapacityGoal", "NetworkInboundCapacityGoal", "NetworkOutboundCapacityGoal",
              "CpuUsageDistributionGoal", "NetworkInboundUsageDistributionGoal",
              "NetworkOutboundUsageDistributionGoal"]


def _model(hosts):
    """6 brokers on 2 racks; hosts[b] names broker b's host (None: a host of its own)."""
    b = ccmi.ClusterModelBuilder()
    for bid in range(6):
        b.create_broker(f"r{bid % 2}", bid, CAP, host=hosts[bid])
    for t in range(4):
        for p in range(6):
            brokers = [(p + t) % 6, (p + t + 1) % 6]
            for i, br in enumerate(brokers):
                b.create_replica(f"r{br % 2}", br, f"T{t}", p, i, i == 0)
                b.set_replica_load(f"r{br % 2}", br, f"T{t}", p, 1.0 + p, 10.0 * (t + 1), 5.0 * (p + 1), 100.0 + t)
    return b.build()


SHARED = ["hA", "hB", "hA", None, "hC", "hC"]       # brokers 0 and 2 share hA in rack r0
SAME_NAME_OTHER_RACKS = ["h", "h", None, None, None, None]  # one name in two racks: two hosts
OWN = [f"h{b}" for b in range(6)]


@pytest.mark.parametrize("goal", HOST_GOALS)
def test_emu_shared_host_rejects_host_resource_goals(emu_lib, goal):
    flat = _model(SHARED)
    cm = ccmi.ClusterModel(flat.desc, device=0, lib=emu_lib, keepalive=flat)
    with pytest.raises(ccmi.UnsupportedOperationException, match="sharing a host"):
        ccmi.GoalOptimizer().optimizations(cm, ccmi.goals_from_names(["ReplicaDistributionGoal", goal]))
    assert cm.actions() == []  # rejected before any goal ran


@pytest.mark.parametrize("goals", [["ReplicaDistributionGoal", "DiskCapacityGoal", "LeaderReplicaDistributionGoal"],
                                   ["RackAwareGoal", "TopicReplicaDistributionGoal", "DiskUsageDistributionGoal"]])
def test_emu_shared_host_other_goals_match_oracle(emu_lib, oracle_lib, goals):
    flat = _model(SHARED)
    check_desc_against_oracle(emu_lib, flat.desc, flat, goals, ccmi.BalancingConstraint())


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


def test_emu_load_monitor_hosts(emu_lib):
    """The native builder keys hosts by (rack, name); a broker only partitions name (handleDeadBroker) is alone on an
    UNKNOWN_HOST."""
    m = ccmi.LoadMonitorModel(num_windows=1, lib=emu_lib)
    m.create_broker("rack0", "node-a", 0, CAP)
    m.create_broker("rack1", "node-a", 1, CAP)  # same name, other rack: another host
    m.create_broker("rack0", "node-b", 2, CAP)
    m.create_broker("rack0", "node-b", 3, CAP, alive=False)  # dead: UNKNOWN_HOST-0
    for p in range(4):
        m.populate_partition("t", p, [p % 4, (p + 1) % 4], p % 4, {"CPU_USAGE": [0.05], "DISK_USAGE": [10.0]})
    d = m.desc()
    hosts = [d.broker_host[b] for b in range(4)]
    assert len(set(hosts)) == 4
    cm = ccmi.ClusterModel(d, device=0, lib=emu_lib, keepalive=m)
    ccmi.GoalOptimizer().optimizations(cm, ccmi.goals_from_names(["CpuCapacityGoal"]))
    m2 = ccmi.LoadMonitorModel(num_windows=1, lib=emu_lib)
    m2.create_broker("rack0", "node-a", 0, CAP)
    m2.create_broker("rack0", "node-a", 1, CAP)  # two brokers on one host
    m2.populate_partition("t", 0, [0, 1], 0, {"CPU_USAGE": [0.5]})
    d2 = m2.desc()
    assert d2.broker_host[0] == d2.broker_host[1]
    cm2 = ccmi.ClusterModel(d2, device=0, lib=emu_lib, keepalive=m2)
    with pytest.raises(ccmi.UnsupportedOperationException):
        ccmi.GoalOptimizer().optimizations(cm2, ccmi.goals_from_names(["CpuCapacityGoal"]))


@pytest.mark.gpu
def test_gpu_shared_host_rejects_and_other_goals_match_oracle(gpu_lib, oracle_lib):
    flat = _model(SHARED)
    cm = ccmi.ClusterModel(flat.desc, device=0, lib=gpu_lib, keepalive=flat)
    with pytest.raises(ccmi.UnsupportedOperationException):
        ccmi.GoalOptimizer().optimizations(cm, ccmi.goals_from_names(["CpuCapacityGoal"]))
    check_desc_against_oracle(gpu_lib, flat.desc, flat, ["ReplicaDistributionGoal", "DiskCapacityGoal",
                                                         "LeaderReplicaDistributionGoal"], ccmi.BalancingConstraint())
