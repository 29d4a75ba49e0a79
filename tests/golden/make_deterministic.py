"""Transcribe the reference's hand-built test clusters into data fixtures (tests/golden/deterministic_clusters.json).

Every model below restates one DeterministicCluster / RackAwareGoalTest factory method call by call (file:line
given per model, paths relative to cruise-control/src/test/java/com/linkedin/kafka/cruisecontrol/):
  brokers   getHomogeneousCluster(rackByBroker, capacity)       common/DeterministicCluster.java:1893-1921
  replicas  ClusterModel.createReplica(rack, broker, tp, index, isLeader) in call order
  loads     ClusterModel.setReplicaLoad(rack, broker, tp, getAggregatedMetricValues(cpu, nwIn, nwOut, disk))
            in call order (KafkaCruiseControlUnitTestUtils.java:90-100)
  dead      ClusterModel.setBrokerState(id, DEAD)
  logdirs   JBOD models: every broker's disk capacity by logdir (getHomogeneousCluster diskCapacityByLogDir) and the
            logdir given to createReplica (6th replica field)
The tests replay the calls through ccmi.ClusterModelBuilder (every createReplica first, then the loads in their
call order; for the models here that yields the same aggregates as the Java call interleaving, because every
follower created after its leader's load would receive exactly the leader's load either way).

    python tests/golden/make_deterministic.py      # writes tests/golden/deterministic_clusters.json
"""
import json
import os
import struct

HERE = os.path.dirname(os.path.abspath(__file__))

# common/TestConstants.java:29-39,99-107
TYPICAL_CPU_CAPACITY = 100.0
LARGE_BROKER_CAPACITY = 300000.0
MEDIUM_BROKER_CAPACITY = 200000.0
SMALL_BROKER_CAPACITY = 10.0
BROKER_CAPACITY = dict(CPU=TYPICAL_CPU_CAPACITY, DISK=LARGE_BROKER_CAPACITY, NW_IN=LARGE_BROKER_CAPACITY,
                       NW_OUT=MEDIUM_BROKER_CAPACITY)
# common/DeterministicCluster.java:47-53
RACK_BY_BROKER = {0: 0, 1: 0, 2: 1}
RACK_BY_BROKER2 = {0: 0, 1: 1, 2: 1}
T1, T2 = "T1", "T2"
TOPIC_A, TOPIC_B, TOPIC_C, TOPIC_D = "A", "B", "C", "D"


class Model:
    def __init__(self, source, rack_by_broker, capacity=None):
        self.d = dict(source=source, racks={str(b): str(r) for b, r in rack_by_broker.items()},
                      capacity=dict(capacity or BROKER_CAPACITY), replicas=[], loads=[], dead=[])

    def create(self, broker, topic, partition, index, leader, logdir=None):
        self.d["replicas"].append([broker, topic, partition, index, bool(leader)] + ([logdir] if logdir else []))
        return self

    def load(self, broker, topic, partition, cpu, nw_in, nw_out, disk):
        for v in (cpu, nw_in, nw_out, disk):
            assert struct.unpack("<f", struct.pack("<f", v))[0] == v  # exact in float32: the window value is the sum
        self.d["loads"].append([broker, topic, partition, cpu, nw_in, nw_out, disk])
        return self


def unbalanced():  # DeterministicCluster.java:200-220
    m = Model("DeterministicCluster.java:200-220 unbalanced()", RACK_BY_BROKER)
    m.create(0, T1, 0, 0, True).create(0, T2, 0, 0, True)
    v = (TYPICAL_CPU_CAPACITY / 2, LARGE_BROKER_CAPACITY / 2, MEDIUM_BROKER_CAPACITY / 2, LARGE_BROKER_CAPACITY / 2)
    m.load(0, T1, 0, *v).load(0, T2, 0, *v)
    return m


def unbalanced2():  # DeterministicCluster.java:154-178
    m = unbalanced()
    m.d["source"] = "DeterministicCluster.java:154-178 unbalanced2()"
    m.create(1, T1, 1, 0, True).create(0, T2, 1, 0, True).create(0, T1, 2, 0, True).create(0, T2, 2, 0, True)
    v = (TYPICAL_CPU_CAPACITY / 2, LARGE_BROKER_CAPACITY / 2, MEDIUM_BROKER_CAPACITY / 2, LARGE_BROKER_CAPACITY / 2)
    m.load(1, T1, 1, *v).load(0, T2, 1, *v).load(0, T1, 2, *v).load(0, T2, 2, *v)
    return m


def unbalanced3():  # DeterministicCluster.java:123-147 (leaders in index 1)
    m = Model("DeterministicCluster.java:123-147 unbalanced3()", RACK_BY_BROKER)
    m.create(1, T1, 0, 0, False).create(1, T2, 0, 0, False).create(0, T1, 0, 1, True).create(0, T2, 0, 1, True)
    v = (TYPICAL_CPU_CAPACITY / 2, LARGE_BROKER_CAPACITY / 2, MEDIUM_BROKER_CAPACITY / 2, LARGE_BROKER_CAPACITY / 2)
    m.load(0, T1, 0, *v).load(0, T2, 0, *v).load(1, T1, 0, *v).load(1, T2, 0, *v)
    return m


def unbalanced_with_a_follower():  # DeterministicCluster.java:183-195
    m = unbalanced()
    m.d["source"] = "DeterministicCluster.java:183-195 unbalancedWithAFollower()"
    m.create(2, T1, 0, 1, False)
    m.load(2, T1, 0, TYPICAL_CPU_CAPACITY / 8, LARGE_BROKER_CAPACITY / 2, 0.0, LARGE_BROKER_CAPACITY / 2)
    return m


def rack_aware_satisfiable():  # DeterministicCluster.java:227-244
    m = Model("DeterministicCluster.java:227-244 rackAwareSatisfiable()", RACK_BY_BROKER)
    m.create(0, T1, 0, 0, True).create(1, T1, 0, 1, False)
    m.load(0, T1, 0, 40.0, 100.0, 130.0, 75.0).load(1, T1, 0, 5.0, 100.0, 0.0, 75.0)
    return m


def rack_aware_satisfiable2():  # DeterministicCluster.java:251-267
    m = Model("DeterministicCluster.java:251-267 rackAwareSatisfiable2()", RACK_BY_BROKER2)
    m.create(0, T1, 0, 0, True).create(2, T1, 0, 1, False)
    m.load(0, T1, 0, 40.0, 100.0, 130.0, 75.0).load(2, T1, 0, 5.0, 100.0, 0.0, 75.0)
    return m


def rack_aware_unsatisfiable():  # DeterministicCluster.java:274-284
    m = rack_aware_satisfiable()
    m.d["source"] = "DeterministicCluster.java:274-284 rackAwareUnsatisfiable()"
    m.create(2, T1, 0, 2, False)
    m.load(2, T1, 0, 60.0, 100.0, 130.0, 75.0)
    return m


def small_cluster_model(capacity=None, tag=""):  # DeterministicCluster.java:1713-1746
    m = Model(f"DeterministicCluster.java:1713-1746 smallClusterModel({tag or 'BROKER_CAPACITY'})", RACK_BY_BROKER,
              capacity)
    m.create(0, T1, 0, 0, True).create(2, T1, 0, 1, False).create(1, T1, 1, 0, True).create(0, T1, 1, 1, False)
    m.create(1, T2, 0, 0, True).create(2, T2, 0, 1, False).create(0, T2, 1, 0, True).create(2, T2, 1, 1, False)
    m.create(0, T2, 2, 0, True).create(1, T2, 2, 1, False)
    m.load(0, T1, 0, 20.0, 100.0, 130.0, 75.0).load(2, T1, 0, 5.0, 100.0, 0.0, 75.0)
    m.load(1, T1, 1, 15.0, 90.0, 110.0, 55.0).load(0, T1, 1, 4.5, 90.0, 0.0, 55.0)
    m.load(1, T2, 0, 5.0, 5.0, 6.0, 5.0).load(2, T2, 0, 4.0, 5.0, 0.0, 5.0)
    m.load(0, T2, 1, 25.0, 25.0, 45.0, 55.0).load(2, T2, 1, 10.5, 25.0, 0.0, 55.0)
    m.load(0, T2, 2, 20.0, 45.0, 120.0, 95.0).load(1, T2, 2, 8.0, 45.0, 0.0, 95.0)
    return m


def dead_broker(capacity=None):  # DeterministicCluster.java:1763-1826
    m = Model("DeterministicCluster.java:1763-1826 deadBroker(BROKER_CAPACITY)", {0: 0, 1: 1, 2: 2, 3: 3, 4: 4},
              capacity)
    creates = [(1, T1, 0, 0, True), (2, T1, 0, 1, False), (1, T1, 1, 0, True), (3, T1, 1, 1, False),
               (1, T1, 2, 0, True), (4, T1, 2, 1, False), (2, T1, 3, 0, True), (0, T1, 3, 1, False),
               (1, T2, 0, 0, True), (2, T2, 0, 1, False), (1, T2, 1, 0, True), (3, T2, 1, 1, False),
               (1, T2, 2, 0, True), (4, T2, 2, 1, False), (3, T2, 3, 0, True), (0, T2, 3, 1, False)]
    for c in creates:
        m.create(*c)
    loads = [(1, T1, 0, 20.0, 100.0, 200.0, 100.0), (2, T1, 0, 15.0, 100.0, 0.0, 100.0),
             (1, T1, 1, 20.0, 90.0, 180.0, 100.0), (3, T1, 1, 15.0, 90.0, 0.0, 100.0),
             (1, T1, 2, 15.0, 75.0, 150.0, 100.0), (4, T1, 2, 12.0, 75.0, 0.0, 100.0),
             (2, T1, 3, 15.0, 60.0, 120.0, 100.0), (0, T1, 3, 12.5, 60.0, 0.0, 100.0),
             (1, T2, 0, 18.0, 100.0, 200.0, 100.0), (2, T2, 0, 14.0, 100.0, 0.0, 100.0),
             (1, T2, 1, 18.0, 90.0, 180.0, 100.0), (3, T2, 1, 14.0, 90.0, 0.0, 100.0),
             (1, T2, 2, 12.0, 75.0, 150.0, 100.0), (4, T2, 2, 10.0, 75.0, 0.0, 100.0),
             (3, T2, 3, 12.0, 60.0, 120.0, 100.0), (0, T2, 3, 10.5, 60.0, 0.0, 100.0)]
    for x in loads:
        m.load(*x)
    m.d["dead"] = [0]
    return m


def medium_cluster_model(capacity=None, tag=""):  # DeterministicCluster.java:1836-1879
    m = Model(f"DeterministicCluster.java:1836-1879 mediumClusterModel({tag or 'BROKER_CAPACITY'})", RACK_BY_BROKER,
              capacity)
    creates = [(1, TOPIC_A, 0, 0, True), (0, TOPIC_A, 0, 1, False), (0, TOPIC_A, 1, 0, True),
               (2, TOPIC_A, 1, 1, False), (0, TOPIC_A, 2, 0, True), (2, TOPIC_A, 2, 1, False),
               (1, TOPIC_B, 0, 0, True), (2, TOPIC_B, 0, 1, False), (2, TOPIC_C, 0, 0, True),
               (1, TOPIC_C, 0, 1, False), (1, TOPIC_D, 0, 0, True), (2, TOPIC_D, 0, 1, False)]
    for c in creates:
        m.create(*c)
    # setReplicaLoad in a different order from the creates (the aggregates depend on it)
    loads = [(0, TOPIC_A, 0, 5.0, 5.0, 0.0, 4.0), (0, TOPIC_A, 1, 5.0, 3.0, 10.0, 8.0),
             (0, TOPIC_A, 2, 5.0, 2.0, 10.0, 6.0), (1, TOPIC_B, 0, 5.0, 4.0, 10.0, 7.0),
             (1, TOPIC_C, 0, 5.0, 6.0, 0.0, 4.0), (1, TOPIC_D, 0, 5.0, 5.0, 10.0, 6.0),
             (1, TOPIC_A, 0, 5.0, 4.0, 10.0, 10.0), (2, TOPIC_B, 0, 2.0, 2.0, 0.0, 5.0),
             (2, TOPIC_C, 0, 1.0, 8.0, 10.0, 4.0), (2, TOPIC_D, 0, 2.0, 8.0, 0.0, 7.0),
             (2, TOPIC_A, 1, 3.0, 4.0, 0.0, 6.0), (2, TOPIC_A, 2, 4.0, 5.0, 0.0, 3.0)]
    for x in loads:
        m.load(*x)
    return m


# common/TestConstants.java:100-110
LOGDIR0, LOGDIR1 = "/mnt/i00", "/mnt/i01"
DISK_CAPACITY = {LOGDIR0: LARGE_BROKER_CAPACITY / 2, LOGDIR1: LARGE_BROKER_CAPACITY / 2}


def create_unbalanced(topics, num_partitions, source):  # DeterministicCluster.java:81-108 createUnbalanced
    m = Model(source, {0: 0, 1: 1})
    m.d["logdirs"] = dict(DISK_CAPACITY)
    for topic in topics:
        for i in range(num_partitions):
            broker = 1 if i > 3 else 0
            logdir = LOGDIR0 if i % 4 < 2 else LOGDIR1
            m.create(broker, topic, i, 0, True, logdir)
            f = i / 2.0 - 1.5
            m.load(broker, topic, i, TYPICAL_CPU_CAPACITY / 5 + TYPICAL_CPU_CAPACITY / 50 * f,
                   LARGE_BROKER_CAPACITY / 5 + LARGE_BROKER_CAPACITY / 50 * f,
                   MEDIUM_BROKER_CAPACITY / 5 + MEDIUM_BROKER_CAPACITY / 50 * f,
                   LARGE_BROKER_CAPACITY / 5 + LARGE_BROKER_CAPACITY / 50 * f)
    return m


def rack_id_mapper_cluster(mapped):  # analyzer/RackAwareGoalTest.java:74-100 and :137-161
    # brokerToRack = {0: "A::0", 1: "B::0", 2: "C::1"}; IgnorePrefixRackIdMapper strips the "X::" prefix
    racks = {0: "A::0", 1: "B::0", 2: "C::1"}
    if mapped:
        racks = {b: r.split("::", 1)[1] for b, r in racks.items()}
    src = ("RackAwareGoalTest.java:74-100 testRackIdMapper (IgnorePrefixRackIdMapper)" if mapped
           else "RackAwareGoalTest.java:137-161 testWithoutRackIdMapper")
    m = Model(src, racks)
    m.create(0, "topic", 0, 0, True).create(1, "topic", 0, 1, False)
    m.load(0, "topic", 0, 40.0, 100.0, 130.0, 75.0).load(1, "topic", 0, 5.0, 100.0, 0.0, 75.0)
    return m


# MinTopicLeadersPerBrokerGoal models: common/TestConstants.java:14-18, DeterministicCluster.java:55-61
TOPIC_MUST = "must_have_leader_replica_on_broker_topic"  # TestConstants.TOPIC_MUST_HAVE_LEADER_REPLICAS_ON_BROKERS
TOPIC0, TOPIC1 = "topic0", "topic1"
RACK_BY_BROKER3 = {0: 0, 1: 1, 2: 1, 3: 1}
HALF = (TYPICAL_CPU_CAPACITY / 2, LARGE_BROKER_CAPACITY / 2, MEDIUM_BROKER_CAPACITY / 2, LARGE_BROKER_CAPACITY / 2)


def min_leader_unsatisfiable():  # DeterministicCluster.java:296-316 minLeaderReplicaPerBrokerUnsatisfiable()
    m = Model("DeterministicCluster.java:296-316 minLeaderReplicaPerBrokerUnsatisfiable()", RACK_BY_BROKER2)
    m.create(0, TOPIC_MUST, 0, 0, True).create(1, TOPIC_MUST, 0, 1, False)
    m.load(0, TOPIC_MUST, 0, *HALF).load(1, TOPIC_MUST, 0, *HALF)
    return m


def min_leader_satisfiable():  # DeterministicCluster.java:329-365 minLeaderReplicaPerBrokerSatisfiable()
    m = Model("DeterministicCluster.java:329-365 minLeaderReplicaPerBrokerSatisfiable()", RACK_BY_BROKER2)
    m.create(0, TOPIC_MUST, 0, 0, True).create(0, TOPIC_MUST, 1, 0, True)
    m.create(1, TOPIC_MUST, 2, 0, True).create(1, TOPIC_MUST, 0, 1, False)
    m.create(2, TOPIC_MUST, 2, 1, False).create(2, TOPIC_MUST, 1, 1, False)
    # five setReplicaLoad calls: the T_P1 follower on broker 2 keeps an empty Load
    for b, p in ((0, 0), (0, 1), (1, 0), (1, 2), (2, 2)):
        m.load(b, TOPIC_MUST, p, *HALF)
    return m


def min_leader_satisfiable2():  # DeterministicCluster.java:378-416 minLeaderReplicaPerBrokerSatisfiable2()
    m = Model("DeterministicCluster.java:378-416 minLeaderReplicaPerBrokerSatisfiable2()", RACK_BY_BROKER2)
    m.create(0, TOPIC_MUST, 0, 0, True).create(0, TOPIC_MUST, 1, 0, True).create(0, TOPIC_MUST, 2, 0, True)
    m.create(1, TOPIC_MUST, 1, 1, False)
    m.create(2, TOPIC_MUST, 0, 1, False).create(2, TOPIC_MUST, 2, 1, False)
    for b, p in ((0, 0), (2, 0), (0, 1), (1, 1), (2, 2), (0, 2)):
        m.load(b, TOPIC_MUST, p, *HALF)
    return m


def min_leader_two_topics(partitions, source):  # DeterministicCluster.java:429-488 / :501-574 (Satisfiable4 / 5)
    m = Model(source, RACK_BY_BROKER2)
    tps = [(t, p) for t in (TOPIC0, TOPIC1) for p in range(partitions)]
    for t, p in tps:
        m.create(0, t, p, 0, True)
    for t, p in tps:
        m.create(1, t, p, 1, False)
    for b in (0, 1):
        for t, p in tps:
            m.load(b, t, p, *HALF)
    return m


def min_leader_satisfiable3():  # DeterministicCluster.java:588-645 minLeaderReplicaPerBrokerSatisfiable3()
    m = Model("DeterministicCluster.java:588-645 minLeaderReplicaPerBrokerSatisfiable3()", RACK_BY_BROKER3)
    # create + setReplicaLoad interleaved; every load is the same, so the aggregates do not depend on the order.
    # Every replica is created at index 0: a later one goes in front of the partition's earlier one.
    for broker, parts, leader in ((1, range(0, 4), True), (1, range(4, 10), False), (2, range(4, 10), True),
                                  (2, range(10, 16), False), (3, range(10, 16), True), (3, range(0, 4), False)):
        for i in parts:
            m.create(broker, TOPIC_MUST, i, 0, leader)
            m.load(broker, TOPIC_MUST, i, *HALF)
    return m


def leader_replica_unsatisfiable():  # DeterministicCluster.java:1591-1620 leaderReplicaPerBrokerUnsatisfiable()
    m = Model("DeterministicCluster.java:1591-1620 leaderReplicaPerBrokerUnsatisfiable()", RACK_BY_BROKER2)
    m.create(0, TOPIC_MUST, 0, 0, True).create(0, TOPIC_MUST, 1, 0, True)
    m.create(1, TOPIC_MUST, 1, 1, False).create(2, TOPIC_MUST, 0, 1, False)
    for b, p in ((0, 0), (2, 0), (0, 1), (1, 1)):
        m.load(b, TOPIC_MUST, p, *HALF)
    return m


def uniform(c):
    return dict(CPU=c, DISK=c, NW_IN=c, NW_OUT=c)


def models():
    out = {
        "unbalanced": unbalanced(), "unbalanced2": unbalanced2(), "unbalanced3": unbalanced3(),
        "unbalancedWithAFollower": unbalanced_with_a_follower(), "rackAwareSatisfiable": rack_aware_satisfiable(),
        "rackAwareSatisfiable2": rack_aware_satisfiable2(), "rackAwareUnsatisfiable": rack_aware_unsatisfiable(),
        "smallClusterModel": small_cluster_model(), "mediumClusterModel": medium_cluster_model(),
        "deadBroker": dead_broker(),
        "rackIdMapper": rack_id_mapper_cluster(True), "withoutRackIdMapper": rack_id_mapper_cluster(False),
        "unbalanced4": create_unbalanced([T1], 8, "DeterministicCluster.java:77-108 unbalanced4()"),
        # Set.of(T1, T2) iterates in a per-JVM salted order; transcribed as T1 then T2
        "unbalanced5": create_unbalanced([T1, T2], 14, "DeterministicCluster.java:113-116 unbalanced5() (T1, T2)"),
        "minLeaderReplicaPerBrokerUnsatisfiable": min_leader_unsatisfiable(),
        "minLeaderReplicaPerBrokerSatisfiable": min_leader_satisfiable(),
        "minLeaderReplicaPerBrokerSatisfiable2": min_leader_satisfiable2(),
        "minLeaderReplicaPerBrokerSatisfiable3": min_leader_satisfiable3(),
        "minLeaderReplicaPerBrokerSatisfiable4": min_leader_two_topics(
            3, "DeterministicCluster.java:429-488 minLeaderReplicaPerBrokerSatisfiable4()"),
        "minLeaderReplicaPerBrokerSatisfiable5": min_leader_two_topics(
            4, "DeterministicCluster.java:501-574 minLeaderReplicaPerBrokerSatisfiable5()"),
        "leaderReplicaPerBrokerUnsatisfiable": leader_replica_unsatisfiable(),
    }
    # DeterministicClusterTest deck #5 (DeterministicClusterTest.java:181-197): uniform capacities
    for name, c in (("LARGE", LARGE_BROKER_CAPACITY), ("MEDIUM", MEDIUM_BROKER_CAPACITY),
                    ("SMALL", SMALL_BROKER_CAPACITY)):
        out[f"smallClusterModel_{name}"] = small_cluster_model(uniform(c), f"{name}_BROKER_CAPACITY x4")
        out[f"mediumClusterModel_{name}"] = medium_cluster_model(uniform(c), f"{name}_BROKER_CAPACITY x4")
    return {k: v.d for k, v in out.items()}


def main():
    path = os.path.join(HERE, "deterministic_clusters.json")
    with open(path, "w") as f:
        json.dump(models(), f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
