"""Regenerate the golden fixtures in this directory from the CPU oracle (oracle/, a C++ restatement of the
reference GoalOptimizer path — see oracle/README and DESIGN.md §Oracle).

The reference is Java and cannot be built here (no JDK, no network), and no reference test pins
exact replica->broker assignments for RandomCluster, so these fixtures are the regression pin for the action
log. The oracle itself is pinned by the reference's known-answer tests in tests/test_oracle_kat.py.

    python tests/golden/make_golden.py            # writes tests/golden/*.json
"""
import hashlib
import json
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from oracle_binding import OracleCluster  # noqa: E402
import ccmi  # noqa: E402

C1_GOALS = ["ReplicaDistributionGoal", "DiskUsageDistributionGoal", "NetworkInboundUsageDistributionGoal",
            "NetworkOutboundUsageDistributionGoal", "CpuUsageDistributionGoal"]

# name -> (RandomCluster overrides, resource balance percentage or None, store the full action list)
CASES = {
    "small_20b": (dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300), 1.05, True),
    "dead_2of10": (dict(num_racks=3, num_brokers=10, num_replicas=3000, num_topics=100, num_dead_brokers=2), None,
                   True),
    "rack_aware_dead": (dict(num_racks=3, num_brokers=10, num_replicas=3000, num_topics=100, num_dead_brokers=2,
                             rack_aware=1), 1.05, True),
    "c0": (dict(), 1.05, False),
    "c1": (dict(num_racks=20, num_brokers=1000, num_replicas=99999, num_topics=3000), None, False),
}


def constraint(balance):
    bc = ccmi.BalancingConstraint()
    if balance is not None:
        bc.set_resource_balance_percentage(balance)
        bc.set_capacity_threshold(0.8)
    return bc


def sha(ints):
    return hashlib.sha256(struct.pack(f"<{len(ints)}q", *ints)).hexdigest()


def flat_actions(actions):
    return [x for a in actions for x in a]


def desc_digest(arrays):
    h = hashlib.sha256()
    for k in sorted(arrays):
        v = arrays[k]
        if k == "topics":
            h.update("\n".join(v).encode())
        elif k in ("cap", "load"):
            h.update(struct.pack(f"<{len(v)}d", *v))
        else:
            h.update(struct.pack(f"<{len(v)}q", *v))
    return h.hexdigest()


def make(name):
    props, balance, full = CASES[name]
    oc = OracleCluster.random(**props)
    results = oc.optimize(C1_GOALS, constraint(balance))
    acts = oc.actions()
    out = dict(name=name, props=props, resource_balance_percentage=balance, goals=C1_GOALS,
               sizes=dict(brokers=oc.B, topics=oc.T, partitions=oc.P, replicas=oc.R),
               desc_sha256=desc_digest(oc.export()),
               num_actions=len(acts), actions_sha256=sha(flat_actions(acts)),
               replica_distribution_sha256=sha(oc.replica_distribution()),
               leader_distribution_sha256=sha(oc.leader_distribution()),
               goals_result=[dict(name=r.name, succeeded=r.succeeded, candidates=r.candidates, actions=r.actions)
                             for r in results],
               final_stats=results[-1].stats)
    if full:
        out["actions"] = acts
    return out


def main():
    for name in (sys.argv[1:] or CASES):
        d = make(name)
        with open(os.path.join(HERE, f"{name}.json"), "w") as f:
            json.dump(d, f, indent=1)
        print(name, d["num_actions"], "actions")


if __name__ == "__main__":
    main()
