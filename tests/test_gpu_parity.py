"""GPU parity: the HIP build of libccmi.so on a gfx950 device against the committed golden fixtures and a live
oracle run on the identical flattened input (bit-exact actions / assignment / leaders, stats within 1e-9)."""
import pytest

import ccmi
from oracle_binding import OracleCluster
from parity import check_product_against_golden, check_product_against_oracle, compare_stats, constraint
from test_oracle_kat import GOLDEN_CASES

pytestmark = pytest.mark.gpu

C1_GOALS = list(ccmi.C1_GOALS)
DEFAULT_GOALS = list(ccmi.DEFAULT_GOALS)


@pytest.mark.parametrize("name", GOLDEN_CASES)
def test_gpu_matches_golden(gpu_lib, oracle_lib, name):
    cm, res = check_product_against_golden(gpu_lib, name)
    # the device path ran (no host fallback exists; this guards the counters the bench relies on)
    assert sum(g.device_launches for g in res.goal_results) > 0
    assert cm.perf().scan_launches + cm.perf().intra_launches > 0


# The headline configurations (BASELINE configs[2] and [3]) and C2 with the C1 goal chain, against committed oracle
# goldens (tests/golden/make_golden.py: c2_c1goals, c2_default, c3_default; the oracle needs about an hour for each).
@pytest.mark.parametrize("name", ["c2_c1goals", "c2_default", "c3_default"])
def test_gpu_matches_headline_golden(gpu_lib, name):
    cm, res = check_product_against_golden(gpu_lib, name, per_goal_stats=True)
    assert cm.perf().scan_launches > 0


@pytest.mark.parametrize("props,balance", [
    (dict(num_racks=2, num_brokers=4, num_replicas=300, num_topics=10), None),
    (dict(num_racks=3, num_brokers=7, num_replicas=1400, num_topics=40, min_replication=2, max_replication=2), 1.02),
    (dict(num_racks=4, num_brokers=16, num_replicas=4800, num_topics=200, distribution=1), 1.05),
    (dict(num_racks=4, num_brokers=16, num_replicas=4800, num_topics=200, distribution=2), 1.2),
    (dict(num_racks=3, num_brokers=9, num_replicas=2700, num_topics=60, num_dead_brokers=3, rack_aware=1), 1.05),
    (dict(num_racks=8, num_brokers=300, num_replicas=30000, num_topics=1000), 1.05),
])
def test_gpu_matches_oracle(gpu_lib, oracle_lib, props, balance):
    check_product_against_oracle(gpu_lib, props, C1_GOALS, balance)


# RandomClusterTest (src/test/java/.../analyzer/RandomClusterTest.java:139-183) rows on TestConstants.BASE_PROPERTIES
# with the default goal list: broker count 80/140, replica count 65004..75006 (max replicas 3000), topic count
# 7000/8000, replication factor 4/5.
@pytest.mark.parametrize("props,max_replicas", [
    (dict(num_brokers=80), 1500),
    (dict(num_brokers=140), 1500),
    (dict(num_replicas=65004), 3000),
    (dict(num_replicas=75006), 3000),
    (dict(num_topics=7000), 3000),
    (dict(num_replicas=50000, min_replication=4, max_replication=4), 3000),
    (dict(num_replicas=50000 - (50000 % 5), min_replication=5, max_replication=5), 3000),
    (dict(num_dead_brokers=5, rack_aware=1, leader_in_first_position=1), 3000),
])
def test_gpu_random_cluster_default_goals(gpu_lib, oracle_lib, props, max_replicas):
    # with OptimizationVerifier's BROKEN_BROKERS / REGRESSION (RandomClusterTest.java:126-128) on the product
    check_product_against_oracle(gpu_lib, props, DEFAULT_GOALS, 1.05, max_replicas=max_replicas, verify=True)


@pytest.mark.parametrize("goals", [DEFAULT_GOALS[::-1], DEFAULT_GOALS[7:] + DEFAULT_GOALS[:7],
                                   ["LeaderBytesInDistributionGoal", "TopicReplicaDistributionGoal",
                                    "LeaderReplicaDistributionGoal", "NetworkOutboundCapacityGoal", "RackAwareGoal"]])
def test_gpu_goal_orders(gpu_lib, oracle_lib, goals):
    check_product_against_oracle(gpu_lib, dict(num_racks=4, num_brokers=16, num_replicas=2400, num_topics=60),
                                 goals, 1.05)


@pytest.mark.parametrize("goals", [["CpuUsageDistributionGoal"],
                                   ["NetworkOutboundUsageDistributionGoal", "ReplicaDistributionGoal"],
                                   ["DiskUsageDistributionGoal", "DiskUsageDistributionGoal"]])
def test_gpu_goal_subsets(gpu_lib, oracle_lib, goals):
    check_product_against_oracle(gpu_lib, dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300),
                                 goals, 1.05)


@pytest.mark.parametrize("split,wgs", [("1", "256"), ("2", "256"), ("4", "256"), ("4", "24")])
def test_gpu_goal_parallel_tiles_match_oracle(gpu_lib, oracle_lib, monkeypatch, split, wgs):
    """Scan-server commands with 1, 2 or 4 wavefronts per candidate (ServerCmd.goalParts, each wave a share of the
    goals) decide exactly as the oracle; with a 24-workgroup split budget larger scans fall back to fewer parts."""
    monkeypatch.setenv("CCMI_GOAL_SPLIT", split)
    monkeypatch.setenv("CCMI_GOAL_SPLIT_WGS", wgs)
    check_product_against_oracle(gpu_lib, dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300),
                                 DEFAULT_GOALS, 1.05)
    check_product_against_oracle(gpu_lib, dict(num_racks=8, num_brokers=300, num_replicas=30000, num_topics=1000),
                                 C1_GOALS, 1.05)


@pytest.mark.parametrize("width", ["full", "adaptive"])
def test_gpu_scan_width_matches_oracle(gpu_lib, oracle_lib, monkeypatch, width):
    """Server scans with every tile of the first sweep on its own workgroup (CCMI_SCAN_WIDTH=full) and with the first
    sweep sized from the site's last winner (the default): the strided later sweeps find any winner past a short first
    sweep, so both decide exactly as the oracle."""
    monkeypatch.setenv("CCMI_SCAN_WIDTH", width)
    check_product_against_oracle(gpu_lib, dict(num_racks=8, num_brokers=300, num_replicas=30000, num_topics=1000),
                                 C1_GOALS, 1.05)
    check_product_against_oracle(gpu_lib, dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300),
                                 DEFAULT_GOALS, 1.05)


@pytest.mark.parametrize("split", ["0", "1"])
def test_gpu_shared_goal_pair_scans_match_oracle(gpu_lib, oracle_lib, monkeypatch, split):
    """Pair scans of at most four tiles with each tile's goals shared by several scan-server workgroups that AND their
    accept masks (CCMI_WG_GOAL_SPLIT=1, the default) and with every goal on one workgroup (0): the same conjunction, so
    both decide exactly as the oracle — the leadership loops of LeaderReplicaDistribution / LeaderBytesIn and the
    resource goals' leadership move-in are pair scans."""
    monkeypatch.setenv("CCMI_WG_GOAL_SPLIT", split)
    check_product_against_oracle(gpu_lib, dict(num_racks=8, num_brokers=300, num_replicas=30000, num_topics=1000),
                                 ["LeaderReplicaDistributionGoal", "CpuUsageDistributionGoal",
                                  "NetworkOutboundUsageDistributionGoal", "LeaderBytesInDistributionGoal"], 1.05)
    check_product_against_oracle(gpu_lib, dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300),
                                 DEFAULT_GOALS, 1.05)


def test_gpu_snapshot_pool_wraps_match_oracle(gpu_lib, oracle_lib, monkeypatch):
    """A snapshot pool of 64K rows wraps many times per proposal (each wrap restarts the scan server and re-sets the
    whole queue directory): the queue scans still read only current snapshots and decide exactly as the oracle."""
    monkeypatch.setenv("CCMI_SNAPSHOT_POOL_ROWS", "65536")
    check_product_against_oracle(gpu_lib, dict(num_racks=8, num_brokers=300, num_replicas=30000, num_topics=1000),
                                 C1_GOALS, 1.05)


@pytest.mark.parametrize("pool_rows", ["4096", "12288", "16384", "20480", "24576"])
def test_gpu_snapshot_directory_larger_than_pool_matches_oracle(gpu_lib, oracle_lib, monkeypatch, pool_rows):
    """Snapshot pools around the size of a queue directory (≈10 000 leader rows, ≈30 000 replica rows on this cluster):
    a directory that does not fit — before a wrap, or only after one when the segment path had cached part of it — is
    refused and the move-in loop takes the segment path (the wrap branch once wrote past the pool); the
    segment path's own wraps rebuild its table. Same decisions as the oracle."""
    monkeypatch.setenv("CCMI_SNAPSHOT_POOL_ROWS", pool_rows)
    check_product_against_oracle(gpu_lib, dict(num_racks=8, num_brokers=300, num_replicas=30000, num_topics=1000),
                                 C1_GOALS, 1.05)
    check_product_against_oracle(gpu_lib, dict(num_racks=8, num_brokers=300, num_replicas=30000, num_topics=1000),
                                 DEFAULT_GOALS, 1.05)


@pytest.mark.parametrize("props", [dict(), dict(num_racks=20, num_brokers=1000, num_replicas=99999, num_topics=3000),
                                   dict(num_racks=3, num_brokers=10, num_replicas=3000, num_topics=100,
                                        num_dead_brokers=2)])
def test_gpu_cluster_stats_before_optimization(gpu_lib, oracle_lib, props):
    """Fused ClusterModelStats reduction on the untouched model vs ClusterModelStats.populate restatement."""
    buf = ccmi.RandomCluster.generate(gpu_lib, **props)
    cm = ccmi.ClusterModel.from_buffers(buf, device=0)
    oc = OracleCluster.from_desc(buf.desc)
    for bal in (None, 1.05):
        compare_stats(cm.cluster_stats(constraint(bal)), oc.stats(constraint(bal)))
    assert cm.perf().stats_launches > 0


def test_gpu_sessions_are_independent(gpu_lib, oracle_lib):
    """Two sessions on one device (the what-if mode bench.py uses) do not interfere."""
    props = dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300)
    buf = ccmi.RandomCluster.generate(gpu_lib, **props)
    a = ccmi.ClusterModel.from_buffers(buf, device=0)
    b = ccmi.ClusterModel.from_buffers(buf, device=0)
    opt = ccmi.GoalOptimizer(constraint(1.05))
    ra = opt.optimizations(a, ccmi.goals_from_names(C1_GOALS))
    rb = opt.optimizations(b, ccmi.goals_from_names(C1_GOALS))
    assert a.actions() == b.actions() and len(a.actions()) > 0
    assert ra.candidates == rb.candidates


def test_gpu_concurrent_sessions_match_sequential(gpu_lib, oracle_lib):
    """Concurrent what-if requests on one device (one host thread and one HIP stream per session, the
    precompute pool of GoalOptimizer.java:117-119; bench.py --requests-per-gpu) make the same decisions as a
    sequential run and as the oracle."""
    from concurrent.futures import ThreadPoolExecutor
    props = dict(num_racks=5, num_brokers=40, num_replicas=12000, num_topics=400)
    buf = ccmi.RandomCluster.generate(gpu_lib, **props)
    opt = ccmi.GoalOptimizer(constraint(1.05))
    seq = ccmi.ClusterModel.from_buffers(buf, device=0)
    rs = opt.optimizations(seq, ccmi.goals_from_names(C1_GOALS))
    sessions = [ccmi.ClusterModel.from_buffers(buf, device=0) for _ in range(6)]
    with ThreadPoolExecutor(len(sessions)) as pool:
        results = list(pool.map(lambda s: opt.optimizations(s, ccmi.goals_from_names(C1_GOALS)), sessions))
    assert len(seq.actions()) > 0
    for s, r in zip(sessions, results):
        assert s.actions() == seq.actions()
        assert r.candidates == rs.candidates
        assert s.proposals() == seq.proposals()
    check_product_against_oracle(gpu_lib, props, C1_GOALS, 1.05)


def test_gpu_acceptance_after_optimization(gpu_lib):
    """Goal.actionAcceptance through the C ABI on the optimized goals of a session; an out-of-range goal index
    is an IllegalArgumentException."""
    buf = ccmi.RandomCluster.generate(gpu_lib, num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300)
    cm = ccmi.ClusterModel.from_buffers(buf, device=0)
    ccmi.GoalOptimizer(constraint(1.05)).optimizations(cm, ccmi.goals_from_names(C1_GOALS))
    with pytest.raises(ccmi.IllegalArgumentException):
        cm.action_acceptance(len(C1_GOALS), 0, 0, 0, 1)
    acts = cm.actions()
    assert acts
    a = acts[-1]
    for gi in range(len(C1_GOALS)):
        # the reverse of the last applied action is a legal question to ask every optimized goal
        assert cm.action_acceptance(gi, a[0], a[1], a[3], a[2]) in ccmi.ACCEPTANCE


# C3 shape (BASELINE configs[3]): dead brokers + requestedDestinationBrokerIds (RemoveBrokersRunnable.java:107-126),
# at the RandomSelfHealingTest size (BASE_PROPERTIES, rack-aware leader-first placement) and a small cluster.
@pytest.mark.parametrize("props,requested", [
    (dict(num_dead_brokers=5, rack_aware=1, leader_in_first_position=1), range(5, 25)),
    (dict(num_racks=6, num_brokers=24, num_replicas=4800, num_topics=30, num_dead_brokers=3, rack_aware=1,
          leader_in_first_position=1), range(3, 12)),
])
def test_gpu_requested_destinations_match_oracle(gpu_lib, oracle_lib, props, requested):
    opts = ccmi.OptimizationOptions(requested_destination_broker_ids=list(requested), fast_mode=False)
    check_product_against_oracle(gpu_lib, props, DEFAULT_GOALS, 1.05, max_replicas=3000, options=opts)


@pytest.mark.parametrize("props,opts,goals", [
    (dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300),
     dict(excluded_brokers_for_leadership=[0, 3, 7]), DEFAULT_GOALS),
    (dict(num_racks=6, num_brokers=24, num_replicas=4800, num_topics=30, num_dead_brokers=3),
     dict(excluded_brokers_for_replica_move=[4, 9], excluded_brokers_for_leadership=[5, 13]), DEFAULT_GOALS),
    (dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300),
     dict(excluded_brokers_for_leadership=[1, 2], excluded_brokers_for_replica_move=[3]), list(ccmi.C1_GOALS)),
    (dict(num_brokers=40), dict(excluded_brokers_for_leadership=[0, 1, 2, 3], excluded_brokers_for_replica_move=[4]),
     DEFAULT_GOALS),
    # excludedTopics (selectReplicasBasedOnExcludedTopics in every goal; tests/test_excluded_topics.py for the KATs)
    (dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300),
     dict(excluded_topics=list(range(0, 300, 3))), DEFAULT_GOALS),
    (dict(num_racks=6, num_brokers=24, num_replicas=4800, num_topics=30, num_dead_brokers=3),
     dict(excluded_topics=[1, 2, 5, 8, 13, 21]), DEFAULT_GOALS),
    (dict(num_brokers=40), dict(excluded_topics=list(range(0, 3000, 7))), list(ccmi.C1_GOALS)),
])
def test_gpu_broker_exclusions_match_oracle(gpu_lib, oracle_lib, props, opts, goals):
    """Leader-replica exclusion and swap-row exclusion run as device checks (allowedBits bits 30/31)."""
    check_product_against_oracle(gpu_lib, props, goals, 1.05, max_replicas=3000,
                                 options=ccmi.OptimizationOptions(fast_mode=False, **opts))


@pytest.mark.parametrize("world", [1, 2])
def test_gpu_xcd_sliced_scans_match_oracle(gpu_lib, oracle_lib, tmp_path, monkeypatch, world):
    """The XCD-sliced scan_cross tiling (normally only for scans with >= 2048 destination columns) forced on for every
    scan of a 301-broker cluster: uneven last slices (N not a multiple of 8), a grid cap that is not a multiple of 8,
    and (world 2) the global keys of a destination-sharded session. Fresh processes read the overrides."""
    import json

    import torch.multiprocessing as mp

    import shard_worker
    from test_shard import _free_port

    monkeypatch.setenv("CCMI_XCD_SLICE_MIN_COLS", "7")
    monkeypatch.setenv("CCMI_GRID_CAP", "13")
    props = dict(num_racks=7, num_brokers=301, num_replicas=30000, num_topics=900)
    mp.start_processes(shard_worker.run, args=(world, _free_port(), props, DEFAULT_GOALS, 1.05, str(tmp_path),
                                               gpu_lib.path), nprocs=world, join=True, start_method="spawn")
    buf = ccmi.RandomCluster.generate(gpu_lib, **props)
    oc = OracleCluster.from_desc(buf.desc)
    ores = oc.optimize(DEFAULT_GOALS, constraint(1.05))
    for r in range(world):
        o = json.load(open(tmp_path / f"rank{r}.json"))
        assert o["error"] is None
        assert [tuple(a) for a in o["actions"]] == oc.actions()
        assert [tuple(g) for g in o["goals"]] == [(x.name, x.succeeded, x.candidates, x.actions) for x in ores]


@pytest.mark.parametrize("props,goals", [
    (dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300, num_brokers_with_bad_disk=3), DEFAULT_GOALS),
    (dict(num_brokers_with_bad_disk=1), DEFAULT_GOALS),
    (dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300, num_brokers_with_bad_disk=5),
     list(ccmi.C1_GOALS)),
])
def test_gpu_bad_disk_brokers_match_oracle(gpu_lib, oracle_lib, props, goals):
    """Partition._ineligibleBrokers on the device (DevTables.pIneligOff/pIneligB in legitMove)."""
    check_product_against_oracle(gpu_lib, props, goals, 1.05, max_replicas=3000)


@pytest.mark.parametrize("pair_chains", ["0", "1"])
def test_gpu_leadership_pair_chains_match_oracle(gpu_lib, oracle_lib, monkeypatch, pair_chains):
    """LeaderReplicaDistributionGoal's leadership loops as one pair scan per decision (the default) and as K7 chains
    (CCMI_PAIR_CHAINS=1, moves applied on the device): both decide exactly as the oracle."""
    monkeypatch.setenv("CCMI_PAIR_CHAINS", pair_chains)
    check_product_against_oracle(gpu_lib, dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300),
                                 DEFAULT_GOALS, 1.05)
    check_product_against_oracle(gpu_lib, dict(num_racks=8, num_brokers=300, num_replicas=30000, num_topics=1000),
                                 ["LeaderReplicaDistributionGoal", "CpuUsageDistributionGoal",
                                  "LeaderReplicaDistributionGoal"], 1.05)


def test_gpu_chain_outlasting_stuck_bound(gpu_lib, oracle_lib, monkeypatch):
    """A K7 chain runs on workgroup 0 of the scan server alone; the other workgroups must wait for it however long it
    takes instead of applying the stuck-command bound to a command they are not part of. With the bound at 2 ms and
    every chain padded to 5 ms (test-only CCMI_CHAIN_DELAY_US), a proposal with chains still completes on the server
    and decides exactly as the oracle."""
    monkeypatch.setenv("CCMI_SERVER_STUCK_MS", "2")
    monkeypatch.setenv("CCMI_CHAIN_DELAY_US", "5000")
    monkeypatch.setenv("CCMI_PAIR_CHAINS", "1")
    props = dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300)
    buf = ccmi.RandomCluster.generate(gpu_lib, **props)
    cm = ccmi.ClusterModel.from_buffers(buf, device=0)
    cm.reset_perf()
    res = ccmi.GoalOptimizer(constraint(1.05)).optimizations(cm, ccmi.goals_from_names(DEFAULT_GOALS))
    p = cm.perf()
    assert p.server_chains > 0 and p.server_scans > 0
    oc = OracleCluster.from_desc(buf.desc)
    ores = oc.optimize(DEFAULT_GOALS, constraint(1.05))
    assert cm.actions() == oc.actions()
    assert [(r.name, r.succeeded, r.candidates, r.actions) for r in res.goal_results] == \
        [(r.name, r.succeeded, r.candidates, r.actions) for r in ores]
