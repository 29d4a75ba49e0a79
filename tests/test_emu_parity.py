"""CPU parity of the engine's host logic (batching, speculation, un-polling, winner decoding) through the
test-only sequential Device emulation (tests/emu) — same C ABI, same predicates as the gfx950 kernels."""
import pytest

import ccmi
from parity import check_product_against_golden, check_product_against_oracle
from test_oracle_kat import GOLDEN_CASES

C1_GOALS = list(ccmi.C1_GOALS)
DEFAULT_GOALS = list(ccmi.DEFAULT_GOALS)


@pytest.mark.parametrize("name", GOLDEN_CASES)
def test_emu_matches_golden(emu_lib, oracle_lib, name):
    check_product_against_golden(emu_lib, name)


@pytest.mark.parametrize("props,balance", [
    (dict(num_racks=2, num_brokers=4, num_replicas=300, num_topics=10), None),
    (dict(num_racks=3, num_brokers=7, num_replicas=1400, num_topics=40, min_replication=2, max_replication=2), 1.02),
    (dict(num_racks=4, num_brokers=16, num_replicas=4800, num_topics=200, distribution=1), 1.05),
    (dict(num_racks=4, num_brokers=16, num_replicas=4800, num_topics=200, distribution=2), 1.2),
    (dict(num_racks=3, num_brokers=9, num_replicas=2700, num_topics=60, num_dead_brokers=3, rack_aware=1), 1.05),
])
def test_emu_matches_oracle(emu_lib, oracle_lib, props, balance):
    check_product_against_oracle(emu_lib, props, C1_GOALS, balance)


@pytest.mark.parametrize("goals", [["CpuUsageDistributionGoal"], ["NetworkOutboundUsageDistributionGoal",
                                                                  "ReplicaDistributionGoal"],
                                   ["DiskUsageDistributionGoal", "DiskUsageDistributionGoal"]])
def test_emu_goal_subsets(emu_lib, oracle_lib, goals):
    check_product_against_oracle(emu_lib, dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300),
                                 goals, 1.05)


# RandomClusterTest (src/test/java/.../analyzer/RandomClusterTest.java:98-183) parameter rows, default goals,
# balance 1.05 / capacity 0.8 / max.replicas.per.broker 1500 (3000 from the replica-count rows on), scaled down
# in broker/replica counts so the CPU suite stays fast; the GPU suite runs the full-size rows.
@pytest.mark.parametrize("props,max_replicas", [
    (dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300), 1500),
    (dict(num_racks=4, num_brokers=16, num_replicas=2400, num_topics=60, min_replication=4, max_replication=4), 3000),
    (dict(num_racks=6, num_brokers=24, num_replicas=4800, num_topics=30, num_dead_brokers=3), 1500),
    (dict(num_racks=3, num_brokers=9, num_replicas=2700, num_topics=60, num_dead_brokers=3, rack_aware=1), 1500),
    (dict(num_racks=4, num_brokers=16, num_replicas=2400, num_topics=60), 140),  # ReplicaCapacityGoal must move
    # full-size RandomClusterTest rows (BASE_PROPERTIES): many moves per broker exercise the candidate-tree
    # materialisation with several moved brokers
    (dict(num_topics=7000), 3000),
    (dict(num_brokers=80), 1500),
])
def test_emu_default_goals_match_oracle(emu_lib, oracle_lib, props, max_replicas):
    check_product_against_oracle(emu_lib, props, DEFAULT_GOALS, 1.05, max_replicas=max_replicas, verify=True)


@pytest.mark.parametrize("goals", [DEFAULT_GOALS[::-1], DEFAULT_GOALS[7:] + DEFAULT_GOALS[:7],
                                   ["LeaderBytesInDistributionGoal", "TopicReplicaDistributionGoal",
                                    "LeaderReplicaDistributionGoal", "NetworkOutboundCapacityGoal", "RackAwareGoal"]])
def test_emu_goal_orders(emu_lib, oracle_lib, goals):
    """Other priority orders: every goal's actionAcceptance runs as a prior-goal predicate of the others (a hard goal
    that cannot be satisfied must fail identically in both)."""
    check_product_against_oracle(emu_lib, dict(num_racks=4, num_brokers=16, num_replicas=2400, num_topics=60),
                                 goals, 1.05)


# C3 shape (BASELINE configs[3]): dead brokers (self-healing) with a requested destination broker set, as
# RemoveBrokersRunnable builds OptimizationOptions (RemoveBrokersRunnable.java:107-126) — the 7-arg
# OptimizationOptions with requestedDestinationBrokerIds, filtered by GoalUtils.eligibleBrokers
# (GoalUtils.java:122-160); leadership moves ignore the requested set.
@pytest.mark.parametrize("props,requested,goals", [
    (dict(num_racks=6, num_brokers=24, num_replicas=4800, num_topics=30, num_dead_brokers=3, rack_aware=1,
          leader_in_first_position=1), range(3, 12), DEFAULT_GOALS),
    (dict(num_racks=4, num_brokers=16, num_replicas=2400, num_topics=60, num_dead_brokers=2, rack_aware=1,
          leader_in_first_position=1), range(2, 10), DEFAULT_GOALS),
    (dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300), [1, 4, 7, 9, 12, 15, 18], C1_GOALS),
])
def test_emu_requested_destinations_match_oracle(emu_lib, oracle_lib, props, requested, goals):
    opts = ccmi.OptimizationOptions(requested_destination_broker_ids=list(requested), fast_mode=False)
    check_product_against_oracle(emu_lib, props, goals, 1.05, max_replicas=3000, options=opts)


# OptimizationOptions broker exclusions (GoalUtils.eligibleBrokers / filterOutBrokersExcludedFor{Leadership,
# ReplicaMove}, GoalUtils.java:122-199; eligibleReplicasForSwap :258-274; ResourceDistributionGoal followers-only
# phases :451,629,719) and onlyMoveImmigrantReplicas.
EXCLUSION_CASES = [
    (dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300),
     dict(excluded_brokers_for_replica_move=[2, 5, 11]), DEFAULT_GOALS),
    (dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300),
     dict(excluded_brokers_for_leadership=[0, 3, 7]), DEFAULT_GOALS),
    (dict(num_racks=6, num_brokers=24, num_replicas=4800, num_topics=30, num_dead_brokers=3),
     dict(excluded_brokers_for_replica_move=[4, 9], excluded_brokers_for_leadership=[5, 13]), DEFAULT_GOALS),
    (dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300),
     dict(excluded_brokers_for_leadership=[1, 2], excluded_brokers_for_replica_move=[3]), C1_GOALS),
    (dict(num_racks=6, num_brokers=24, num_replicas=4800, num_topics=30, num_dead_brokers=3),
     dict(only_move_immigrant_replicas=True), DEFAULT_GOALS),
    # excludedTopics: ReplicaSortFunctionFactory.selectReplicasBasedOnExcludedTopics in every goal's sorted replicas,
    # RackAwareGoal's included-topic rack check, ReplicaCapacityGoal's excluded-replica check,
    # TopicReplicaDistributionGoal's topicsToRebalance, LeaderReplicaDistributionGoal's leadership loops
    (dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300),
     dict(excluded_topics=list(range(0, 300, 3))), DEFAULT_GOALS),
    (dict(num_racks=6, num_brokers=24, num_replicas=4800, num_topics=30, num_dead_brokers=3),
     dict(excluded_topics=[1, 2, 5, 8, 13, 21]), DEFAULT_GOALS),
    (dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300, leader_in_first_position=1),
     dict(excluded_topics=list(range(150))), C1_GOALS),
]


@pytest.mark.parametrize("props,opts,goals", EXCLUSION_CASES)
def test_emu_broker_exclusions_match_oracle(emu_lib, oracle_lib, props, opts, goals):
    check_product_against_oracle(emu_lib, props, goals, 1.05, max_replicas=3000,
                                 options=ccmi.OptimizationOptions(fast_mode=False, **opts))


# Brokers with bad disks (Broker.State.BAD_DISKS) without disk information: RandomCluster marks one replica of each
# broken broker original-offline (RandomCluster.java:409-449). Exercises Partition._ineligibleBrokers
# (canAssignReplicaToBroker in GoalUtils.legitMove), the self-healing branches for BAD_DISKS brokers and
# ensureReplicasMoveOffBrokersWithBadDisks.
BAD_DISK_CASES = [
    (dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300, num_brokers_with_bad_disk=3), DEFAULT_GOALS),
    (dict(num_brokers_with_bad_disk=1), DEFAULT_GOALS),
    (dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300, num_brokers_with_bad_disk=5), C1_GOALS),
    (dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300, num_brokers_with_bad_disk=2),
     DEFAULT_GOALS[::-1]),
]


@pytest.mark.parametrize("props,goals", BAD_DISK_CASES)
def test_emu_bad_disk_brokers_match_oracle(emu_lib, oracle_lib, props, goals):
    check_product_against_oracle(emu_lib, props, goals, 1.05, max_replicas=3000)


@pytest.mark.parametrize("calls,puts", [("0", "512"), ("2", "7"), ("-1", "1")])
def test_emu_speculative_host_work_matches_oracle(emu_lib, oracle_lib, monkeypatch, calls, puts):
    """Device::idleWork (host work while a scan is in flight): the move-out entry tree started a few puts at a time
    and finished by materialise(), and the move-in snapshots of upcoming polls, left undone, partly done or done —
    the decisions are the oracle's either way."""
    monkeypatch.setenv("CCMI_EMU_IDLE_CALLS", calls)
    monkeypatch.setenv("CCMI_IDLE_TREE_PUTS", puts)
    check_product_against_oracle(emu_lib, dict(num_brokers=80), DEFAULT_GOALS, 1.05, max_replicas=1500)


@pytest.mark.parametrize("props", [dict(num_brokers=80), dict(num_racks=5, num_brokers=20, num_replicas=6000,
                                                               num_topics=300)])
def test_emu_tree_worker_matches_oracle(emu_lib, oracle_lib, monkeypatch, props):
    """The move-out entry tree built on the helper thread (TreeWorker, on by default from 2048 brokers; forced here for
    small clusters): adopted by materialise(), or superseded by the next call's submission when no step needs it."""
    monkeypatch.setenv("CCMI_TREE_WORKER", "1")
    monkeypatch.setenv("CCMI_TREE_WORKER_MIN", "1")
    check_product_against_oracle(emu_lib, props, DEFAULT_GOALS, 1.05, max_replicas=1500)


@pytest.mark.parametrize("pool_rows", ["1024", "4096", "12000"])
def test_emu_queue_directory_larger_than_pool_falls_back(emu_lib, oracle_lib, monkeypatch, pool_rows):
    """A snapshot directory that does not fit the snapshot pool (CCMI_SNAPSHOT_POOL_ROWS) is refused before the move-in
    loop changes any state, and the loop takes the segment path instead of failing: same decisions as the
    oracle."""
    monkeypatch.setenv("CCMI_SNAPSHOT_POOL_ROWS", pool_rows)
    check_product_against_oracle(emu_lib, dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300),
                                 DEFAULT_GOALS, 1.05)
