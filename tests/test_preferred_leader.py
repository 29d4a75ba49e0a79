"""PreferredLeaderElectionGoal (analyzer/goals/PreferredLeaderElectionGoal.java:117-190), not in default.goals but
part of DeterministicClusterTest's deck list (tests/test_deterministic.py runs it there).

Pinning: PreferredLeaderElectionGoalTest (analyzer/PreferredLeaderElectionGoalTest.java:60-219) on its own cluster
(createClusterModel :331-392: 5 brokers on 4 racks, topics topic0..topic3 with 3 partitions of 3 replicas, zero
loads): without demoted brokers every partition's first replica leads afterwards; with broker 0 DEMOTED the
partitions it did not lead keep their leader, and for the ones it led the first replica leads and broker 0's replica
is last. testOptimizeWithDemotedDisks / testOptimizeWithDemotedBrokersAndDisks (:128-219) build the same cluster with
replica placement over two logdirs (populateDiskInfo: logdir(index, broker) alternates /mnt/i00 and /mnt/i01,
:434-436) and demote disks (ccmi.h disk_demoted): the partitions led from a demoted disk re-elect the first replica and
the demoted replicas go last. The provision status stays UNDECIDED. The skipUrpDemotion / excludeFollowerDemotion
variants (:222-310) need the Kafka Cluster metadata and constructor flags GoalOptimizer never sets; they are not
transcribed. The product matches the oracle bit for bit (slot order included: Partition.moveReplicaToEnd changes
the replica lists, and so the proposals).
"""
import pytest

import ccmi
from oracle_binding import OracleCluster
from parity import check_desc_against_oracle

RACKS = {0: "r0", 1: "r0", 2: "r1", 3: "r2", 4: "r3"}
# (broker, topic, partition, index, leader) in createReplicaAndSetLoad order (:350-392)
REPLICAS = [
    (0, "topic0", 0, 0, True), (1, "topic0", 1, 0, True), (2, "topic0", 2, 0, True),
    (3, "topic1", 0, 0, False), (4, "topic1", 1, 0, False), (0, "topic1", 2, 0, False),
    (1, "topic2", 0, 0, False), (2, "topic2", 1, 0, False), (3, "topic2", 2, 0, False),
    (4, "topic0", 0, 1, False), (2, "topic0", 1, 1, False), (0, "topic0", 2, 1, False),
    (1, "topic1", 0, 1, True), (3, "topic1", 1, 1, True), (4, "topic1", 2, 1, True),
    (2, "topic2", 0, 1, False), (0, "topic2", 1, 1, False), (1, "topic2", 2, 1, False),
    (3, "topic0", 0, 2, False), (4, "topic0", 1, 2, False), (3, "topic0", 2, 2, False),
    (2, "topic1", 0, 2, False), (0, "topic1", 1, 2, False), (2, "topic1", 2, 2, False),
    (4, "topic2", 0, 2, True), (3, "topic2", 1, 2, True), (4, "topic2", 2, 2, True),
    (3, "topic3", 0, 0, True), (4, "topic3", 1, 0, True), (4, "topic3", 2, 0, True),
    (0, "topic3", 0, 1, False), (2, "topic3", 1, 1, False), (3, "topic3", 2, 1, False),
    (4, "topic3", 0, 2, False), (3, "topic3", 1, 2, False), (2, "topic3", 2, 2, False),
]
CAPACITY = {"CPU": 100.0, "DISK": 300000.0, "NW_IN": 300000.0, "NW_OUT": 200000.0}  # TestConstants.BROKER_CAPACITY
LOGDIRS = ["/mnt/i00", "/mnt/i01"]  # TestConstants.LOGDIR0 / LOGDIR1, DISK_CAPACITY 150000 each (:100-110)
# logdir(populateDiskInfo, index, brokerId) arguments of each createReplicaAndSetLoad call above (:350-392)
LOGDIR_ARGS = [(0, 0), (0, 1), (0, 2), (0, 3), (0, 4), (0, 0), (0, 1), (0, 2), (0, 3),
               (1, 4), (1, 2), (1, 0), (1, 1), (1, 3), (1, 4), (1, 2), (1, 0), (1, 1),
               (2, 3), (2, 4), (2, 3), (2, 2), (2, 0), (2, 2), (2, 4), (2, 3), (2, 4),
               (0, 4), (0, 3), (0, 4), (1, 4), (1, 3), (1, 4), (2, 4), (2, 3), (2, 4)]


def build(demoted=(), demoted_disks=None):
    """createClusterModel(_, populateDiskInfo = demoted_disks is not None); demoted_disks: (broker, logdir) pairs."""
    jbod = demoted_disks is not None
    b = ccmi.ClusterModelBuilder()
    for r in range(4):
        b.create_rack(f"r{r}")
    for bid in range(5):
        b.create_broker(RACKS[bid], bid, CAPACITY, {d: 150000.0 for d in LOGDIRS} if jbod else None, host=f"h{bid}")
    for (broker, topic, part, index, leader), (i, bid) in zip(REPLICAS, LOGDIR_ARGS):
        b.create_replica(RACKS[broker], broker, topic, part, index, leader,
                         logdir=LOGDIRS[(i + bid) % 2] if jbod else None)
        b.set_replica_load(RACKS[broker], broker, topic, part, 0.0, 0.0, 0.0, 0.0)
    for d in demoted:
        b.set_broker_state(d, "DEMOTED")
    for broker, logdir in demoted_disks or ():
        b.set_disk_state(broker, logdir, "DEMOTED")
    return b.build()


def _disk_index(broker, logdir):  # the builder creates each broker's two disks in LOGDIRS order
    return 2 * broker + LOGDIRS.index(logdir)


def _partition_lists(flat, dist, leaders):
    """(topic, partition) -> (replica brokers in Partition._replicas order, leader broker)."""
    d = flat.desc
    out = {}
    for p, (topic, num) in flat.partitions.items():
        out[(topic, num)] = (dist[d.partition_offset[p]:d.partition_offset[p + 1]], leaders[p])
    return out


def _leaders_before(flat):
    d = flat.desc
    return {flat.partitions[d.replica_partition[r]]: d.replica_broker[r]
            for r in range(d.num_replicas) if d.replica_is_leader[r]}


def _check_without_demoted(flat, dist, leaders):
    for (topic, num), (brokers, leader) in _partition_lists(flat, dist, leaders).items():
        if topic != "topic3":
            assert leader == brokers[0], (topic, num)  # only the first replica leads (:72-79)


def _check_with_demoted(flat, dist, leaders, demoted=0):
    before = _leaders_before(flat)
    for (topic, num), (brokers, leader) in _partition_lists(flat, dist, leaders).items():
        if topic == "topic3":
            continue
        if before[(topic, num)] != demoted:
            assert leader == before[(topic, num)], (topic, num)  # (:112-114)
        else:
            assert leader == brokers[0], (topic, num)
            if demoted in brokers:
                assert brokers[-1] == demoted, (topic, num)  # the demoted replica is last (:117-122)


def _check_demoted_disks(flat, dist, leaders, disks, demoted_brokers, demoted_disks):
    """testOptimizeWithDemotedDisks / ...BrokersAndDisks (:152-172, :198-218): partitions (topic0..2) not led from a
    demoted broker or disk keep their leader; the others are led by their first replica, and every replica on a
    demoted broker or disk is last."""
    d = flat.desc
    dd = {_disk_index(b, ld) for b, ld in demoted_disks}
    before = _leaders_before(flat)
    to_demote = {flat.partitions[d.replica_partition[r]] for r in range(d.num_replicas)
                 if d.replica_is_leader[r] and (d.replica_broker[r] in demoted_brokers or d.replica_disk[r] in dd)}
    for p, (topic, num) in flat.partitions.items():
        if topic == "topic3":
            continue
        o0, o1 = d.partition_offset[p], d.partition_offset[p + 1]
        brokers, slot_disks = dist[o0:o1], disks[o0:o1]
        if (topic, num) not in to_demote:
            assert leaders[p] == before[(topic, num)], (topic, num)
            continue
        assert leaders[p] == brokers[0], (topic, num)
        for i, (b, k) in enumerate(zip(brokers, slot_disks)):
            if b in demoted_brokers or k in dd:
                assert i == len(brokers) - 1, (topic, num, b)


def _oracle(flat):
    oc = OracleCluster.from_desc(flat.desc)
    res = oc.optimize(["PreferredLeaderElectionGoal"])
    return res[0], oc.replica_distribution(), oc.leader_distribution(), oc.replica_disks()


def _product(lib, flat):
    cm = ccmi.ClusterModel(flat.desc, device=0, lib=lib, keepalive=flat)
    res = ccmi.GoalOptimizer().optimizations(cm, ccmi.goals_from_names(["PreferredLeaderElectionGoal"]))
    return res.goal_results[0], cm.replica_distribution(), cm.leader_distribution(), cm.replica_disks()


# testOptimizeWithDemotedDisks (:128-132) and testOptimizeWithDemotedBrokersAndDisks (:175-179)
DISK_CASES = {"disks": ((), [(0, LOGDIRS[0]), (1, LOGDIRS[1])]), "broker-and-disk": ((0,), [(1, LOGDIRS[0])])}


@pytest.mark.parametrize("demoted", [(), (0,)], ids=["no-demotion", "broker0-demoted"])
def test_oracle_preferred_leader_election_kat(oracle_lib, demoted):
    flat = build(demoted)
    g, dist, leaders, _ = _oracle(flat)
    assert g.provision.status == "UNDECIDED"
    (_check_with_demoted if demoted else _check_without_demoted)(flat, dist, leaders)


@pytest.mark.parametrize("demoted", [(), (0,)], ids=["no-demotion", "broker0-demoted"])
def test_emu_preferred_leader_election_kat(emu_lib, oracle_lib, demoted):
    flat = build(demoted)
    g, dist, leaders, _ = _product(emu_lib, flat)
    assert g.provision.status == "UNDECIDED"
    (_check_with_demoted if demoted else _check_without_demoted)(flat, dist, leaders)
    check_desc_against_oracle(emu_lib, flat.desc, flat, ["PreferredLeaderElectionGoal"], ccmi.BalancingConstraint())


@pytest.mark.parametrize("case", list(DISK_CASES))
def test_oracle_preferred_leader_election_demoted_disks_kat(oracle_lib, case):
    brokers, disks = DISK_CASES[case]
    flat = build(brokers, disks)
    g, dist, leaders, rdisks = _oracle(flat)
    assert g.provision.status == "UNDECIDED"
    _check_demoted_disks(flat, dist, leaders, rdisks, brokers, disks)


@pytest.mark.parametrize("case", list(DISK_CASES))
def test_emu_preferred_leader_election_demoted_disks_kat(emu_lib, oracle_lib, case):
    brokers, disks = DISK_CASES[case]
    flat = build(brokers, disks)
    g, dist, leaders, rdisks = _product(emu_lib, flat)
    assert g.provision.status == "UNDECIDED"
    _check_demoted_disks(flat, dist, leaders, rdisks, brokers, disks)
    check_desc_against_oracle(emu_lib, flat.desc, flat, ["PreferredLeaderElectionGoal"], ccmi.BalancingConstraint())


def test_emu_preferred_leader_election_rejects_goal_violation_use(emu_lib, oracle_lib):
    flat = build()
    cm = ccmi.ClusterModel(flat.desc, device=0, lib=emu_lib, keepalive=flat)
    with pytest.raises(ccmi.IllegalArgumentException):
        ccmi.GoalOptimizer().optimizations(cm, ccmi.goals_from_names(["PreferredLeaderElectionGoal"]),
                                           ccmi.OptimizationOptions(is_triggered_by_goal_violation=True))


@pytest.mark.parametrize("props", [dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300),
                                   dict(num_racks=6, num_brokers=24, num_replicas=4800, num_topics=30,
                                        num_dead_brokers=3, leader_in_first_position=1)], ids=["healthy", "dead"])
def test_emu_default_goals_then_election_match_oracle(emu_lib, oracle_lib, props):
    from parity import check_product_against_oracle
    check_product_against_oracle(emu_lib, props, list(ccmi.DEFAULT_GOALS) + ["PreferredLeaderElectionGoal"], 1.05,
                                 max_replicas=3000)


@pytest.mark.gpu
@pytest.mark.parametrize("demoted", [(), (0,)], ids=["no-demotion", "broker0-demoted"])
def test_gpu_preferred_leader_election_kat(gpu_lib, oracle_lib, demoted):
    flat = build(demoted)
    g, dist, leaders, _ = _product(gpu_lib, flat)
    (_check_with_demoted if demoted else _check_without_demoted)(flat, dist, leaders)
    check_desc_against_oracle(gpu_lib, flat.desc, flat, ["PreferredLeaderElectionGoal"], ccmi.BalancingConstraint())


@pytest.mark.gpu
@pytest.mark.parametrize("case", list(DISK_CASES))
def test_gpu_preferred_leader_election_demoted_disks_kat(gpu_lib, oracle_lib, case):
    brokers, disks = DISK_CASES[case]
    flat = build(brokers, disks)
    g, dist, leaders, rdisks = _product(gpu_lib, flat)
    _check_demoted_disks(flat, dist, leaders, rdisks, brokers, disks)
    check_desc_against_oracle(gpu_lib, flat.desc, flat, ["PreferredLeaderElectionGoal"], ccmi.BalancingConstraint())
