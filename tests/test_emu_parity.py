"""CPU parity of the engine's host logic (batching, speculation, un-polling, winner decoding) through the
test-only sequential Device emulation (tests/emu) — same C ABI, same predicates as the gfx950 kernels."""
import pytest

from parity import check_product_against_golden, check_product_against_oracle

C1_GOALS = ["ReplicaDistributionGoal", "DiskUsageDistributionGoal", "NetworkInboundUsageDistributionGoal",
            "NetworkOutboundUsageDistributionGoal", "CpuUsageDistributionGoal"]


@pytest.mark.parametrize("name", ["small_20b", "dead_2of10", "rack_aware_dead", "c0", "c1"])
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
