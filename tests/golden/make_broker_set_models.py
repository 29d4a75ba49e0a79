"""Transcribe the reference's broker-set test clusters into data fixtures (tests/golden/broker_set_clusters.json).

Source (paths relative to cruise-control/src/test/): java/com/linkedin/kafka/cruisecontrol/common/DeterministicCluster.java
brokerSetSatisfiable1..8 and brokerSetUnSatisfiable1/3 (:663-1420), whose bodies are regular sequences of
  getHomogeneousCluster(RACK_BY_BROKERn, TestConstants.BROKER_CAPACITY, null)           brokers (:56-61 rack maps)
  cluster.createReplica(rack, broker, topicXPartitionY, index, isLeader)                 in call order
  cluster.setReplicaLoad(rack, broker, topicXPartitionY, aggregatedMetricValues | createLoad(cpu, nwIn, nwOut, disk), ..)
with topicXPartitionY = new TopicPartition(TOPICX, Y) (TOPIC0 "topic0", TOPIC1 "topic1", TestConstants.java:14-15) and
aggregatedMetricValues = getAggregatedMetricValues(TestConstants.X / k, ...). This script reads those calls from the
reference text (generation time only, in the build container) and writes the resulting data: the same format as
make_deterministic.py (brokers / replicas / loads), plus the broker sets of resources/testBrokerSets.json (the
BrokerSetFileResolver data of KafkaCruiseControlUnitTestUtils.java:52-78, a data file of the reference's tests).

    python tests/golden/make_broker_set_models.py
"""
import json
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/cruise-control/src/test"
SRC = os.path.join(REF, "java/com/linkedin/kafka/cruisecontrol/common/DeterministicCluster.java")
BROKER_SETS = os.path.join(REF, "resources/testBrokerSets.json")

CONST = {"TYPICAL_CPU_CAPACITY": 100.0, "LARGE_BROKER_CAPACITY": 300000.0, "MEDIUM_BROKER_CAPACITY": 200000.0}
BROKER_CAPACITY = dict(CPU=100.0, DISK=300000.0, NW_IN=300000.0, NW_OUT=200000.0)
TOPICS = {"TOPIC0": "topic0", "TOPIC1": "topic1"}
NAMES = ["brokerSetSatisfiable1", "brokerSetSatisfiable2", "brokerSetSatisfiable3", "brokerSetSatisfiable4",
         "brokerSetSatisfiable5", "brokerSetSatisfiable6", "brokerSetSatisfiable7", "brokerSetSatisfiable8",
         "brokerSetUnSatisfiable1", "brokerSetUnSatisfiable3", "brokerSetUnSatisfiable4",
         "brokerSetSatisfiableAfterTopicExclusion"]


def rack_maps(text):
    out = {}
    for name, body in re.findall(r"(RACK_BY_BROKER\d*) = Map\.of\(([^)]*)\)", text):
        xs = [int(x) for x in body.split(",")]
        out[name] = {xs[i]: xs[i + 1] for i in range(0, len(xs), 2)}
    return out


def value(expr):
    expr = expr.strip()
    m = re.fullmatch(r"TestConstants\.(\w+)\s*/\s*(\d+)", expr)
    if m:
        return CONST[m.group(1)] / int(m.group(2))
    return float(expr)


def method_body(text, name):
    i = text.index(f"public static ClusterModel {name}()")
    j = text.index("return cluster;", i)
    return text[i:j], text[: i].count("\n") + 1, text[: j].count("\n") + 1


def transcribe(text, name, racks):
    body, l0, l1 = method_body(text, name)
    stmts = [re.sub(r"\s+", " ", s).strip() for s in re.sub(r"//[^\n]*", "", body).split(";")]
    rack_name = re.search(r"getHomogeneousCluster\((RACK_BY_BROKER\d*), TestConstants\.BROKER_CAPACITY", body).group(1)
    d = dict(source=f"DeterministicCluster.java:{l0}-{l1} {name}()",
             racks={str(b): str(r) for b, r in sorted(racks[rack_name].items())},
             capacity=dict(BROKER_CAPACITY), replicas=[], loads=[], dead=[])
    tps, default = {}, None
    for s in stmts:
        m = re.search(r"TopicPartition (\w+) = new TopicPartition\((\w+), (\d+)\)", s)
        if m:
            tps[m.group(1)] = (TOPICS[m.group(2)], int(m.group(3)))
            continue
        m = re.search(r"aggregatedMetricValues = getAggregatedMetricValues\((.*)\)$", s)
        if m:
            default = [value(x) for x in m.group(1).split(",")]
            continue
        m = re.search(r"cluster\.createReplica\([^,]+, (\d+), (\w+), (\d+), (true|false)\)", s)
        if m:
            topic, part = tps[m.group(2)]
            d["replicas"].append([int(m.group(1)), topic, part, int(m.group(3)), m.group(4) == "true"])
            continue
        m = re.search(r"cluster\.setReplicaLoad\([^,]+, (\d+), (\w+), (aggregatedMetricValues|createLoad\(([^)]*)\))", s)
        if m:
            topic, part = tps[m.group(2)]
            vals = default if m.group(3) == "aggregatedMetricValues" else [value(x) for x in m.group(4).split(",")]
            d["loads"].append([int(m.group(1)), topic, part] + vals)
            continue
        assert "cluster." not in s, f"{name}: unparsed statement {s}"
    return d


def main():
    with open(SRC) as f:
        text = f.read()
    racks = rack_maps(text)
    models = {n: transcribe(text, n, racks) for n in NAMES}
    with open(BROKER_SETS) as f:
        sets = {bs["brokerSetId"]: bs["brokerIds"] for bs in json.load(f)["brokerSets"]}
    out = dict(broker_sets=dict(source="resources/testBrokerSets.json", sets=sets), models=models)
    path = os.path.join(HERE, "broker_set_clusters.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path, {n: len(m["replicas"]) for n, m in models.items()})


if __name__ == "__main__":
    main()
