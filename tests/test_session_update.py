"""The boundary's session-update and acceptance-by-kind entry points.

* ccmi_session_apply: actions decided outside the session (a JVM goal earlier in a mixed chain, an executed proposal
  batch) are applied to the resident model as ClusterModel.relocateReplica / relocateLeadership do
  (ClusterModel.java:362-425), and later goals see exactly that model: the product (CPU emulation; gfx950 under
  -m gpu) and the oracle apply the same actions and then optimize the same chain, bit for bit.
* ccmi_action_acceptance_by_kind: Goal.actionAcceptance keyed by goal class, equal to the index-keyed call.
"""
import pytest

import ccmi
from oracle_binding import OracleCluster
from parity import compare_stats, constraint

C1_GOALS = list(ccmi.C1_GOALS)
DEFAULT_GOALS = list(ccmi.DEFAULT_GOALS)
PROPS = dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300)


def _external_actions(props, goals, bc):
    """Actions a JVM-side prefix of the chain would have made (the oracle optimizing `goals`)."""
    oc = OracleCluster.random(**props)
    oc.optimize(goals, bc)
    return oc.actions()


def _apply_then_optimize(lib, props, prefix, rest, bc):
    acts = _external_actions(props, prefix, bc)
    assert acts
    buf = ccmi.RandomCluster.generate(lib, **props)
    cm = ccmi.ClusterModel.from_buffers(buf)
    oc = OracleCluster.from_desc(buf.desc)
    assert cm.apply(acts) == len(acts)
    oc.apply(acts)
    assert cm.replica_distribution() == oc.replica_distribution()
    assert cm.leader_distribution() == oc.leader_distribution()
    compare_stats(cm.cluster_stats(bc), oc.stats(bc))
    res = ccmi.GoalOptimizer(bc).optimizations(cm, ccmi.goals_from_names(rest))
    ores = oc.optimize(rest, bc)
    assert cm.actions() == oc.actions()
    assert cm.replica_distribution() == oc.replica_distribution()
    assert cm.leader_distribution() == oc.leader_distribution()
    for r, o in zip(res.goal_results, ores):
        assert (r.name, r.succeeded, r.candidates, r.actions) == (o.name, o.succeeded, o.candidates, o.actions)
        compare_stats(r.stats, o.stats)
    # the proposals are the diff against the session's initial placement, external moves included
    final = cm.replica_distribution()
    init = [buf.desc.replica_broker[buf.desc.partition_replicas[i]] for i in range(buf.desc.num_replicas)]
    changed = {p for p in range(buf.desc.num_partitions)
               if sorted(init[buf.desc.partition_offset[p]:buf.desc.partition_offset[p + 1]]) !=
               sorted(final[buf.desc.partition_offset[p]:buf.desc.partition_offset[p + 1]])}
    assert changed <= {p.partition for p in cm.proposals()}
    return cm


CASES = [(C1_GOALS[:2], C1_GOALS[2:]), (DEFAULT_GOALS[:8], DEFAULT_GOALS[8:]),
         (["LeaderReplicaDistributionGoal"], ["CpuUsageDistributionGoal", "LeaderBytesInDistributionGoal"])]
IDS = ["c1-after-diskusage", "default-second-half", "after-leader-moves"]


@pytest.mark.parametrize("prefix,rest", CASES, ids=IDS)
def test_emu_apply_then_optimize_matches_oracle(emu_lib, oracle_lib, prefix, rest):
    _apply_then_optimize(emu_lib, PROPS, prefix, rest, constraint(1.05))


def test_emu_apply_swaps_and_validation(emu_lib, oracle_lib):
    """Swaps apply as their two relocations; invalid actions are refused with the count applied so far."""
    buf = ccmi.RandomCluster.generate(emu_lib, **PROPS)
    cm = ccmi.ClusterModel.from_buffers(buf)
    d = buf.desc
    # partitions 0 and 1 with their first replicas on different brokers that do not host the other partition
    part_brokers = lambda p: [d.replica_broker[d.partition_replicas[i]]  # noqa: E731
                              for i in range(d.partition_offset[p], d.partition_offset[p + 1])]
    p0 = 0
    for p1 in range(1, d.num_partitions):
        b0, b1 = part_brokers(p0)[0], part_brokers(p1)[0]
        if b0 != b1 and b1 not in part_brokers(p0) and b0 not in part_brokers(p1):
            break
    swap = (2, p0, b0, b1, p1, -1, -1)
    assert cm.apply([swap]) == 1
    oc = OracleCluster.from_desc(d)
    oc.apply([swap])
    assert cm.replica_distribution() == oc.replica_distribution()
    assert cm.actions() == oc.actions()
    bad = (0, p0, b0, b1, -1, -1, -1)  # partition 0 is no longer on b0
    with pytest.raises(ccmi.IllegalArgumentException):
        cm.apply([bad])
    leader_on_follower = (1, p0, b1, part_brokers(p0)[1], -1, -1, -1)
    with pytest.raises(ccmi.IllegalArgumentException):
        cm.apply([leader_on_follower] * 2)  # the second one fails: b1 no longer leads


def test_emu_acceptance_by_kind_equals_by_index(emu_lib):
    buf = ccmi.RandomCluster.generate(emu_lib, **PROPS)
    cm = ccmi.ClusterModel.from_buffers(buf)
    ccmi.GoalOptimizer(constraint(1.05)).optimizations(cm, ccmi.goals_from_names(C1_GOALS))
    acts = cm.actions()
    for a in acts[-20:]:
        for gi, g in enumerate(C1_GOALS):
            assert cm.action_acceptance_by_goal(g, a[0], a[1], a[3], a[2]) == \
                cm.action_acceptance(gi, a[0], a[1], a[3], a[2])
    with pytest.raises(ccmi.IllegalArgumentException):
        cm.action_acceptance_by_goal("RackAwareGoal", 0, 0, 0, 1)


@pytest.mark.gpu
@pytest.mark.parametrize("prefix,rest", CASES, ids=IDS)
def test_gpu_apply_then_optimize_matches_oracle(gpu_lib, oracle_lib, prefix, rest):
    _apply_then_optimize(gpu_lib, PROPS, prefix, rest, constraint(1.05))
