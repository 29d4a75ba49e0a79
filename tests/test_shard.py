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


def _group_run(lib, props, goals, world, device_of=lambda r: 0):
    """One process, `world` sessions of one sharded proposal in a shard group (ccmi_shard_group_*), each optimized on
    its own thread; returns the sessions and their results."""
    from concurrent.futures import ThreadPoolExecutor
    buf = ccmi.RandomCluster.generate(lib, **props)
    group = ccmi.ShardGroup(world, lib)
    sessions = []
    for r in range(world):
        cm = ccmi.ClusterModel(buf.desc, device=device_of(r), lib=lib, keepalive=buf)
        cm.attach_group(group, r)
        cm.reset_perf()
        sessions.append(cm)
    opt = ccmi.GoalOptimizer(constraint(1.05))
    with ThreadPoolExecutor(world) as pool:
        results = list(pool.map(lambda cm: opt.optimizations(cm, ccmi.goals_from_names(goals)), sessions))
    return buf, sessions, results


def _check_group_against_oracle(buf, sessions, results, goals):
    oc = OracleCluster.from_desc(buf.desc)
    ores = oc.optimize(goals, constraint(1.05))
    for cm, res in zip(sessions, results):
        assert cm.perf().combines > 0
        assert cm.actions() == oc.actions()
        assert [(r.name, r.succeeded, r.candidates, r.actions) for r in res.goal_results] == \
            [(r.name, r.succeeded, r.candidates, r.actions) for r in ores]


@pytest.mark.parametrize("world", [2, 3])
def test_shard_group_one_process_matches_oracle(emu_lib, oracle_lib, world):
    """A shard group in one process (the emulation combines on the host side of the group protocol): every rank makes
    the oracle's decisions with the reference-equivalent candidate counts."""
    props = dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300)
    goals = list(ccmi.DEFAULT_GOALS)
    _check_group_against_oracle(*_group_run(emu_lib, props, goals, world), goals)


def test_shard_group_rejects_bad_rank(emu_lib):
    buf = ccmi.RandomCluster.generate(emu_lib, num_racks=3, num_brokers=6, num_replicas=60, num_topics=5)
    cm = ccmi.ClusterModel.from_buffers(buf, device=0)
    group = ccmi.ShardGroup(2, emu_lib)
    with pytest.raises(ccmi.IllegalArgumentException):
        cm.attach_group(group, 2)
    with pytest.raises(ccmi.IllegalArgumentException):
        ccmi.ShardGroup(0, emu_lib)


@pytest.mark.gpu
@pytest.mark.parametrize("shared_servers", ["1", "0"])
def test_gpu_shard_group_same_gpu_twice(gpu_lib, oracle_lib, monkeypatch, shared_servers):
    """One process, two sessions on device ordinal 0 as the two ranks of a shard group. With
    CCMI_GROUP_SHARED_SERVERS=1 each rank gets a scan server with half the device's workgroup budget and every served
    scan is combined ON THE DEVICE (the server's last workgroup folds the rank's key into the group's pinned-host slot,
    and the group's last rank publishes the minimum into both mailboxes); by default ranks sharing a GPU launch per scan
    and combine on their host threads (a launch could wait behind the other rank's persistent server). Both decide
    exactly as the oracle."""
    monkeypatch.setenv("CCMI_GROUP_SHARED_SERVERS", shared_servers)
    props = dict(num_racks=5, num_brokers=40, num_replicas=12000, num_topics=400)
    goals = list(ccmi.DEFAULT_GOALS)
    buf, sessions, results = _group_run(gpu_lib, props, goals, 2)
    _check_group_against_oracle(buf, sessions, results, goals)
    served = [cm.perf().server_scans for cm in sessions]
    if shared_servers == "1":
        assert min(served) > 0
    else:
        assert max(served) == 0


def test_shard_group_mixed_device_layout(emu_lib, oracle_lib):
    """Three ranks, two of them sharing a device (those launch per scan: their queue scans are off) and one on a device
    of its own: the queue-scan path is decided group-wide, so every rank runs the same scans, pairs its combines with
    the others' and makes the oracle's decisions (a per-rank decision mismatched the slot pairing)."""
    props = dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300)
    goals = list(ccmi.DEFAULT_GOALS)
    buf, sessions, results = _group_run(emu_lib, props, goals, 3, device_of=lambda r: [0, 0, 1][r])
    _check_group_against_oracle(buf, sessions, results, goals)
    assert len({cm.perf().combines for cm in sessions}) == 1


def test_shard_group_survives_destroyed_session(emu_lib, oracle_lib):
    """A session destroyed while attached leaves its rank's slot empty: attaching another session to that rank later
    reads no freed memory, and the group then optimizes as usual."""
    import gc
    props = dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300)
    buf = ccmi.RandomCluster.generate(emu_lib, **props)
    group = ccmi.ShardGroup(2, emu_lib)
    gone = ccmi.ClusterModel(buf.desc, device=0, lib=emu_lib, keepalive=buf)
    gone.attach_group(group, 1)
    del gone
    gc.collect()
    sessions = []
    for r in range(2):
        cm = ccmi.ClusterModel(buf.desc, device=r, lib=emu_lib, keepalive=buf)
        cm.attach_group(group, r)
        cm.reset_perf()
        sessions.append(cm)
    from concurrent.futures import ThreadPoolExecutor
    goals = list(ccmi.C1_GOALS)
    opt = ccmi.GoalOptimizer(constraint(1.05))
    with ThreadPoolExecutor(2) as pool:
        results = list(pool.map(lambda cm: opt.optimizations(cm, ccmi.goals_from_names(goals)), sessions))
    _check_group_against_oracle(buf, sessions, results, goals)


def test_shm_combiner_refuses_stale_block(emu_lib):
    """A block a crashed run left under the job's name seconds ago (rank 0 created it, then gave up waiting) is refused
    by a rank of a new job whose nonce differs — the v9 age window alone would have accepted it — and accepted by a
    rank carrying the nonce rank 0 stamped (ccmi_session_attach_shm_job, ABI v12)."""
    name = f"/ccmi_stale_{os.getpid()}"
    buf = ccmi.RandomCluster.generate(emu_lib, num_racks=3, num_brokers=6, num_replicas=60, num_topics=5)
    crashed = ccmi.ClusterModel.from_buffers(buf, device=0)
    try:
        with pytest.raises(ccmi.CruiseControlError):  # rank 0 of the crashed job: rank 1 never came
            crashed.attach_shm(0, 2, name, job_nonce=1111, timeout_s=0.5)
        assert os.path.exists(f"/dev/shm{name}")  # the stale block stays behind, well inside 120 s
        late = ccmi.ClusterModel.from_buffers(buf, device=0)
        with pytest.raises(ccmi.CruiseControlError):  # a new job's rank 1 waits for its own rank 0, never attaching the stale one
            late.attach_shm(1, 2, name, job_nonce=2222, timeout_s=1.0)
        same = ccmi.ClusterModel.from_buffers(buf, device=0)
        same.attach_shm(1, 2, name, job_nonce=1111, timeout_s=1.0)  # the nonce matches: it is that job's block
    finally:
        if os.path.exists(f"/dev/shm{name}"):
            os.unlink(f"/dev/shm{name}")
