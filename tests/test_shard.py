"""Destination-sharded scans with world_size 2 and 3 over torch.distributed gloo on CPU: every rank
scans its slice of each candidate list, ranks MIN-combine their first-fit keys, and the result must be the
unsharded result — identical action log, assignment, leaders and reference-equivalent candidate counts on every
rank — and must match the CPU oracle."""
import json
import os
import socket

import pytest
import torch.multiprocessing as mp

import ccmi
from oracle_binding import OracleCluster
from parity import constraint

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,props,goals,balance", [
    (2, dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300), list(ccmi.DEFAULT_GOALS), 1.05),
    (3, dict(num_racks=3, num_brokers=10, num_replicas=3000, num_topics=100, num_dead_brokers=2), list(ccmi.C1_GOALS),
     None),
])
def test_sharded_scans_match_unsharded_and_oracle(emu_lib, oracle_lib, tmp_path, world, props, goals, balance):
    import shard_worker

    mp.start_processes(shard_worker.run, args=(world, _free_port(), props, goals, balance, str(tmp_path),
                                               emu_lib.path), nprocs=world, join=True, start_method="spawn")
    outs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(world)]
    for o in outs:
        assert o["error"] is None
        assert o["combines"] > 0
        for k in ("actions", "replica_distribution", "leader_distribution", "goals"):
            assert o[k] == outs[0][k], k
    # every rank scanned only its slice: together they evaluated the candidate space once
    buf = ccmi.RandomCluster.generate(emu_lib, **props)
    oc = OracleCluster.from_desc(buf.desc)
    ores = oc.optimize(goals, constraint(balance))
    assert [tuple(a) for a in outs[0]["actions"]] == oc.actions()
    assert outs[0]["replica_distribution"] == oc.replica_distribution()
    assert [tuple(g) for g in outs[0]["goals"]] == [(r.name, r.succeeded, r.candidates, r.actions) for r in ores]


@pytest.mark.parametrize("world", [2, 3])
def test_shm_combiner_matches_oracle(emu_lib, oracle_lib, tmp_path, world):
    """The built-in host shared-memory combiner (ccmi_session_attach_shm, shard_shm.cpp): every rank makes the
    oracle's decisions with the same reference-equivalent candidate counts."""
    import shard_worker

    props = dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300)
    goals = list(ccmi.DEFAULT_GOALS)
    mp.start_processes(shard_worker.run, args=(world, _free_port(), props, goals, 1.05, str(tmp_path), emu_lib.path,
                                               "shm"), nprocs=world, join=True, start_method="spawn")
    outs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(world)]
    buf = ccmi.RandomCluster.generate(emu_lib, **props)
    oc = OracleCluster.from_desc(buf.desc)
    ores = oc.optimize(goals, constraint(1.05))
    for o in outs:
        assert o["error"] is None and o["combines"] > 0
        assert [tuple(a) for a in o["actions"]] == oc.actions()
        assert [tuple(g) for g in o["goals"]] == [(r.name, r.succeeded, r.candidates, r.actions) for r in ores]


def test_shm_combiner_rejects_bad_arguments(emu_lib):
    buf = ccmi.RandomCluster.generate(emu_lib, num_racks=3, num_brokers=6, num_replicas=60, num_topics=5)
    cm = ccmi.ClusterModel.from_buffers(buf, device=0)
    with pytest.raises(ccmi.IllegalArgumentException):
        cm.attach_shm(2, 2, "/ccmi_bad_rank")
    with pytest.raises(ccmi.IllegalArgumentException):
        cm.attach_shm(0, 1, "no_leading_slash")


@pytest.mark.gpu
def test_gpu_shm_combiner_keeps_scan_server(gpu_lib, oracle_lib, tmp_path):
    """Two shard processes on the gfx950 device over the shared-memory combiner: both keep their scan server (64
    workgroups each, so both are resident on one card) and make the oracle's decisions."""
    import shard_worker

    props = dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300)
    goals = list(ccmi.DEFAULT_GOALS)
    mp.start_processes(shard_worker.run, args=(2, _free_port(), props, goals, 1.05, str(tmp_path), gpu_lib.path,
                                               "shm", {"CCMI_SERVER_BLOCKS": "64"}),
                       nprocs=2, join=True, start_method="spawn")
    outs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(2)]
    buf = ccmi.RandomCluster.generate(gpu_lib, **props)
    oc = OracleCluster.from_desc(buf.desc)
    ores = oc.optimize(goals, constraint(1.05))
    for o in outs:
        assert o["error"] is None and o["combines"] > 0 and o["server_launches"] > 0
        assert [tuple(a) for a in o["actions"]] == oc.actions()
        assert [tuple(g) for g in o["goals"]] == [(r.name, r.succeeded, r.candidates, r.actions) for r in ores]


@pytest.mark.gpu
def test_gpu_sharded_scans_match_oracle(gpu_lib, oracle_lib, tmp_path):
    """Two shard processes on the gfx950 device (gloo combiner): the kernels' column / pair slices with global
    keys reproduce the oracle's decisions."""
    import shard_worker

    props = dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300)
    goals = list(ccmi.DEFAULT_GOALS)
    mp.start_processes(shard_worker.run, args=(2, _free_port(), props, goals, 1.05, str(tmp_path), gpu_lib.path),
                       nprocs=2, join=True, start_method="spawn")
    outs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(2)]
    buf = ccmi.RandomCluster.generate(gpu_lib, **props)
    oc = OracleCluster.from_desc(buf.desc)
    ores = oc.optimize(goals, constraint(1.05))
    for o in outs:
        assert o["error"] is None and o["combines"] > 0
        assert [tuple(a) for a in o["actions"]] == oc.actions()
        assert [tuple(g) for g in o["goals"]] == [(r.name, r.succeeded, r.candidates, r.actions) for r in ores]


@pytest.mark.gpu
def test_gpu_rccl_combiner_one_rank(gpu_lib, oracle_lib, monkeypatch):
    """The built-in RCCL combiner (shard_rccl.cpp: host -> HBM, ncclAllReduce MIN, HBM -> host per scan) on a
    one-rank communicator, forced onto every scan with CCMI_FORCE_COMBINE=1: the same decisions as the oracle. (Two
    RCCL ranks cannot share the one GPU of a test box; the multi-rank path runs in the driver's 8-GPU bench.)"""
    monkeypatch.setenv("CCMI_FORCE_COMBINE", "1")
    props = dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300)
    goals = list(ccmi.C1_GOALS)
    buf = ccmi.RandomCluster.generate(gpu_lib, **props)
    cm = ccmi.ClusterModel.from_buffers(buf, device=0)
    cm.attach_rccl(0, 1, ccmi.rccl_unique_id(gpu_lib))
    cm.reset_perf()
    res = ccmi.GoalOptimizer(constraint(1.05)).optimizations(cm, ccmi.goals_from_names(goals))
    assert cm.perf().combines > 0
    oc = OracleCluster.from_desc(buf.desc)
    ores = oc.optimize(goals, constraint(1.05))
    assert cm.actions() == oc.actions()
    assert [(r.name, r.succeeded, r.candidates, r.actions) for r in res.goal_results] == \
        [(r.name, r.succeeded, r.candidates, r.actions) for r in ores]
