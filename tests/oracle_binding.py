"""ctypes binding of the CPU oracle (oracle/build/liboracle_cc.so) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module, and only as the
checker / CPU baseline. The product path (cruise-control_amd/) never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys
from typing import List, Optional

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cruise-control_amd"))
import ccmi  # noqa: E402

ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "build", "liboracle_cc.so")


def build_oracle() -> str:
    if not os.path.exists(ORACLE_LIB) or any(
            os.path.getmtime(os.path.join(ORACLE_DIR, "src", f)) > os.path.getmtime(ORACLE_LIB)
            for f in os.listdir(os.path.join(ORACLE_DIR, "src"))):
        subprocess.run(["make", "-C", ORACLE_DIR, "-j8"], check=True, capture_output=True)
    return ORACLE_LIB


class Oracle:
    _lib = None

    @classmethod
    def lib(cls):
        if cls._lib is None:
            L = C.CDLL(build_oracle())
            L.oc_random_cluster.restype = C.c_void_p
            L.oc_random_cluster.argtypes = [C.POINTER(ccmi.RandomClusterProps)]
            L.oc_from_desc.restype = C.c_void_p
            L.oc_from_desc.argtypes = [C.POINTER(ccmi.ClusterDesc)]
            L.oc_free.argtypes = [C.c_void_p]
            L.oc_sizes.argtypes = [C.c_void_p, C.POINTER(C.c_int32)]
            L.oc_topic_name.restype = C.c_char_p
            L.oc_topic_name.argtypes = [C.c_void_p, C.c_int]
            L.oc_export.argtypes = [C.c_void_p] + [C.POINTER(C.c_int32)] * 2 + [C.POINTER(C.c_double)] + \
                [C.POINTER(C.c_int32)] * 6 + [C.POINTER(C.c_uint8)] * 2 + [C.POINTER(C.c_float)]
            L.oc_optimize.restype = C.c_int
            L.oc_optimize.argtypes = [C.c_void_p, C.POINTER(C.c_int32), C.c_int, C.POINTER(ccmi.ConstraintStruct),
                                      C.POINTER(ccmi.OptionsStruct), C.POINTER(ccmi.GoalResultStruct)]
            L.oc_goal_optimize.restype = C.c_int
            L.oc_goal_optimize.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_int32), C.c_int32,
                                           C.POINTER(ccmi.ConstraintStruct), C.POINTER(ccmi.OptionsStruct),
                                           C.POINTER(ccmi.GoalResultStruct)]
            L.oc_action_acceptance_by_kind.restype = C.c_int32
            L.oc_action_acceptance_by_kind.argtypes = [C.c_void_p, C.c_int32, C.POINTER(ccmi.ActionStruct)]
            L.oc_broker_util.restype = C.c_double
            L.oc_broker_util.argtypes = [C.c_void_p, C.c_int, C.c_int]
            L.oc_host_util.restype = C.c_double
            L.oc_host_util.argtypes = [C.c_void_p, C.c_int, C.c_int]
            L.oc_error.restype = C.c_char_p
            L.oc_error.argtypes = [C.c_void_p]
            L.oc_last_seconds.restype = C.c_double
            L.oc_last_seconds.argtypes = [C.c_void_p]
            L.oc_candidates.restype = C.c_int64
            L.oc_candidates.argtypes = [C.c_void_p]
            L.oc_action_count.restype = C.c_int64
            L.oc_action_count.argtypes = [C.c_void_p]
            L.oc_actions.argtypes = [C.c_void_p, C.POINTER(ccmi.ActionStruct)]
            L.oc_last_failure_provision.argtypes = [C.c_void_p, C.POINTER(ccmi.ProvisionRespStruct)]
            L.oc_topic_broker_set.restype = C.c_int32
            L.oc_topic_broker_set.argtypes = [C.c_char_p, C.c_int32]
            L.oc_action_acceptance.restype = C.c_int32
            L.oc_action_acceptance.argtypes = [C.c_void_p, C.c_int32, C.POINTER(ccmi.ActionStruct)]
            L.oc_apply.restype = C.c_int32
            L.oc_apply.argtypes = [C.c_void_p, C.POINTER(ccmi.ActionStruct), C.c_int64]
            L.oc_replica_distribution.argtypes = [C.c_void_p, C.POINTER(C.c_int32)]
            L.oc_leader_distribution.argtypes = [C.c_void_p, C.POINTER(C.c_int32)]
            L.oc_stats.argtypes = [C.c_void_p, C.POINTER(ccmi.ConstraintStruct), C.POINTER(ccmi.OptionsStruct),
                                   C.POINTER(ccmi.StatsStruct)]
            L.oc_proposal_count.restype = C.c_int64
            L.oc_proposal_count.argtypes = [C.c_void_p]
            L.oc_proposals.argtypes = [C.c_void_p, C.c_int] + [C.POINTER(C.c_int32)] * 5
            L.oc_java_random_probe.restype = C.c_int64
            L.oc_java_random_probe.argtypes = [C.c_int64, C.c_int, C.c_int, C.POINTER(C.c_int32),
                                               C.POINTER(C.c_double)]
            L.oc_set_deadline.argtypes = [C.c_void_p, C.c_double]
            L.oc_stats_seconds.restype = C.c_double
            L.oc_stats_seconds.argtypes = [C.c_void_p]
            L.oc_num_disks.restype = C.c_int32
            L.oc_num_disks.argtypes = [C.c_void_p]
            L.oc_disk_logdir.restype = C.c_char_p
            L.oc_disk_logdir.argtypes = [C.c_void_p, C.c_int]
            L.oc_export_disks.argtypes = [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_double),
                                          C.POINTER(C.c_int32)]
            L.oc_num_disk_assignments.restype = C.c_int64
            L.oc_num_disk_assignments.argtypes = [C.c_void_p]
            L.oc_disk_assignments.argtypes = [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
            L.oc_replica_disks.argtypes = [C.c_void_p, C.POINTER(C.c_int32)]
            L.oc_disk_utilization.restype = C.c_double
            L.oc_disk_utilization.argtypes = [C.c_void_p, C.c_int]
            L.oc_proposal_disks.argtypes = [C.c_void_p, C.c_int] + [C.POINTER(C.c_int32)] * 2
            L.oc_balance_threshold.restype = C.c_double
            L.oc_balance_threshold.argtypes = [C.c_double, C.c_int, C.c_double, C.c_double, C.c_double, C.c_int,
                                               C.c_double, C.c_int]
            cls._lib = L
        return cls._lib


class OracleCluster:
    """A CPU-oracle ClusterModel."""

    def __init__(self, handle: int):
        if not handle:
            raise RuntimeError("oracle failed to build the cluster")
        self.h = C.c_void_p(handle)
        self.L = Oracle.lib()
        sz = (C.c_int32 * 6)()
        self.L.oc_sizes(self.h, sz)
        self.B, self.T, self.P, self.R, self.racks, self.W = list(sz)
        self.last_results = None

    @staticmethod
    def random(**overrides) -> "OracleCluster":
        return OracleCluster(Oracle.lib().oc_random_cluster(C.byref(ccmi.RandomCluster.props(**overrides))))

    @staticmethod
    def from_desc(desc: ccmi.ClusterDesc) -> "OracleCluster":
        return OracleCluster(Oracle.lib().oc_from_desc(C.byref(desc)))

    def topic_names(self) -> List[str]:
        if getattr(self, "_topics", None) is None:
            self._topics = [self.L.oc_topic_name(self.h, t).decode() for t in range(self.T)]
        return self._topics

    def __del__(self):
        try:
            self.L.oc_free(self.h)
        except Exception:
            pass

    def export(self) -> dict:
        B, T, P, R, W = self.B, self.T, self.P, self.R, self.W
        a = dict(broker_rack=(C.c_int32 * B)(), broker_state=(C.c_int32 * B)(), cap=(C.c_double * (4 * B))(),
                 partition_topic=(C.c_int32 * P)(), partition_number=(C.c_int32 * P)(),
                 partition_offset=(C.c_int32 * (P + 1))(), partition_replicas=(C.c_int32 * R)(),
                 replica_partition=(C.c_int32 * R)(), replica_broker=(C.c_int32 * R)(),
                 is_leader=(C.c_uint8 * R)(), offline=(C.c_uint8 * R)(), load=(C.c_float * (R * 6 * W))())
        self.L.oc_export(self.h, a["broker_rack"], a["broker_state"], a["cap"], a["partition_topic"],
                         a["partition_number"], a["partition_offset"], a["partition_replicas"], a["replica_partition"],
                         a["replica_broker"], a["is_leader"], a["offline"], a["load"])
        out = {k: list(v) for k, v in a.items()}
        out["topics"] = [self.L.oc_topic_name(self.h, t).decode() for t in range(T)]
        D = self.L.oc_num_disks(self.h)
        out["num_disks"] = D
        if D:
            db, dc, rd = (C.c_int32 * D)(), (C.c_double * D)(), (C.c_int32 * R)()
            self.L.oc_export_disks(self.h, db, dc, rd)
            n = self.L.oc_num_disk_assignments(self.h)
            ar, ad = (C.c_int32 * max(1, n))(), (C.c_int32 * max(1, n))()
            self.L.oc_disk_assignments(self.h, ar, ad)
            out.update(disk_broker=list(db), disk_capacity=list(dc), replica_disk=list(rd),
                       disk_logdir=[self.L.oc_disk_logdir(self.h, d).decode() for d in range(D)],
                       disk_assign_replica=list(ar[:n]), disk_assign_disk=list(ad[:n]))
        return out

    def optimize(self, goal_names: List[str], constraint: Optional[ccmi.BalancingConstraint] = None,
                 options: Optional[ccmi.OptimizationOptions] = None):
        kinds = (C.c_int32 * len(goal_names))(*[ccmi.GOAL_KINDS[n] for n in goal_names])
        res = (ccmi.GoalResultStruct * len(goal_names))()
        o, keep = (options or ccmi.OptimizationOptions()).to_struct()
        c = (constraint or ccmi.BalancingConstraint()).to_struct(self.topic_names())
        st = self.L.oc_optimize(self.h, kinds, len(goal_names), C.byref(c), C.byref(o), res)
        if st != 0:
            err = ccmi._STATUS.get(st, RuntimeError)(self.L.oc_error(self.h).decode())
            if isinstance(err, ccmi.OptimizationFailureException):
                p = ccmi.ProvisionRespStruct()
                self.L.oc_last_failure_provision(self.h, C.byref(p))
                err.provision = ccmi.ProvisionResponse.from_struct(p, ccmi._goal_of_message(str(err)))
            raise err
        self.last_results = [ccmi.GoalResult(ccmi.GOAL_NAMES[r.goal_kind], bool(r.succeeded), bool(r.has_diff),
                                             r.seconds, r.candidates, 0, 0, r.actions, ccmi.stats_to_dict(r.stats),
                                             ccmi.ProvisionResponse.from_struct(r.provision,
                                                                                ccmi.GOAL_NAMES[r.goal_kind]))
                             for r in res]
        return self.last_results

    def _raise(self, st: int):
        err = ccmi._STATUS.get(st, RuntimeError)(self.L.oc_error(self.h).decode())
        if isinstance(err, ccmi.OptimizationFailureException):
            p = ccmi.ProvisionRespStruct()
            self.L.oc_last_failure_provision(self.h, C.byref(p))
            err.provision = ccmi.ProvisionResponse.from_struct(p, ccmi._goal_of_message(str(err)))
        raise err

    def goal_optimize(self, goal_name: str, optimized_goals=(), constraint: Optional[ccmi.BalancingConstraint] = None,
                      options: Optional[ccmi.OptimizationOptions] = None) -> ccmi.GoalResult:
        """Goal.optimize(clusterModel, optimizedGoals, options) for one goal: optimized_goals are names of goals this
        model has optimized (the instance of their latest optimization)."""
        prior = [ccmi.GOAL_KINDS[n] if isinstance(n, str) else int(n) for n in optimized_goals]
        kinds = (C.c_int32 * max(1, len(prior)))(*prior)
        r = ccmi.GoalResultStruct()
        o, keep = (options or ccmi.OptimizationOptions()).to_struct()
        c = (constraint or ccmi.BalancingConstraint()).to_struct(self.topic_names())
        st = self.L.oc_goal_optimize(self.h, ccmi.GOAL_KINDS[goal_name], kinds, len(prior), C.byref(c), C.byref(o),
                                     C.byref(r))
        if st != 0:
            self._raise(st)
        return ccmi.GoalResult(goal_name, bool(r.succeeded), bool(r.has_diff), r.seconds, r.candidates, 0, 0,
                               r.actions, ccmi.stats_to_dict(r.stats),
                               ccmi.ProvisionResponse.from_struct(r.provision, goal_name))

    def action_acceptance_by_goal(self, goal_name: str, action_type: int, partition: int, source: int,
                                  destination: int, destination_partition: int = -1) -> str:
        a = ccmi.ActionStruct(action_type, partition, source, destination, destination_partition, -1, -1)
        v = self.L.oc_action_acceptance_by_kind(self.h, ccmi.GOAL_KINDS[goal_name], C.byref(a))
        if v < 0:
            raise ValueError(self.L.oc_error(self.h).decode())
        return ccmi.ACCEPTANCE[v]

    def seconds(self) -> float:
        return self.L.oc_last_seconds(self.h)

    def broker_util(self, b: int, res: int) -> float:
        return self.L.oc_broker_util(self.h, b, res)

    def host_util(self, b: int, res: int) -> float:
        """Utilization of broker b's host (Broker.host().load().expectedUtilizationFor)."""
        return self.L.oc_host_util(self.h, b, res)

    def optimize_until(self, goal_names: List[str], seconds: float, constraint=None, options=None):
        """CPU-baseline sample: run the chain until `seconds` of wall time have passed (or it completes).
        Returns (completed, candidates evaluated, seconds spent in ClusterModelStats)."""
        kinds = (C.c_int32 * len(goal_names))(*[ccmi.GOAL_KINDS[n] for n in goal_names])
        res = (ccmi.GoalResultStruct * len(goal_names))()
        o, keep = (options or ccmi.OptimizationOptions()).to_struct()
        c = (constraint or ccmi.BalancingConstraint()).to_struct(self.topic_names())
        self.L.oc_set_deadline(self.h, seconds)
        st = self.L.oc_optimize(self.h, kinds, len(goal_names), C.byref(c), C.byref(o), res)
        self.L.oc_set_deadline(self.h, 0.0)
        if st not in (0, 99):
            raise ccmi._STATUS.get(st, RuntimeError)(self.L.oc_error(self.h).decode())
        return st == 0, self.L.oc_candidates(self.h), self.L.oc_stats_seconds(self.h)

    def apply(self, actions) -> None:
        acts = list(actions)
        arr = (ccmi.ActionStruct * max(1, len(acts)))(*[ccmi.ActionStruct(*a) for a in acts])
        st = self.L.oc_apply(self.h, arr, len(acts))
        if st != 0:
            raise ccmi._STATUS.get(st, RuntimeError)(self.L.oc_error(self.h).decode())

    def action_acceptance(self, goal_index: int, action_type: int, partition: int, source: int, destination: int,
                          destination_partition: int = -1) -> str:
        """Goal.actionAcceptance of the goal_index-th goal of the last optimize() on the current model."""
        a = ccmi.ActionStruct(action_type, partition, source, destination, destination_partition, -1, -1)
        v = self.L.oc_action_acceptance(self.h, goal_index, C.byref(a))
        if v < 0:
            raise ValueError(self.L.oc_error(self.h).decode())
        return ccmi.ACCEPTANCE[v]

    def actions(self) -> List[tuple]:
        n = self.L.oc_action_count(self.h)
        buf = (ccmi.ActionStruct * max(1, n))()
        self.L.oc_actions(self.h, buf)
        return [(a.type, a.partition, a.source_broker, a.destination_broker, a.destination_partition,
                 a.source_disk, a.destination_disk) for a in buf[:n]]

    def replica_disks(self) -> List[int]:
        out = (C.c_int32 * self.R)()
        self.L.oc_replica_disks(self.h, out)
        return list(out)

    def disk_utilization(self, d: int) -> float:
        return self.L.oc_disk_utilization(self.h, d)

    def replica_distribution(self) -> List[int]:
        out = (C.c_int32 * self.R)()
        self.L.oc_replica_distribution(self.h, out)
        return list(out)

    def leader_distribution(self) -> List[int]:
        out = (C.c_int32 * self.P)()
        self.L.oc_leader_distribution(self.h, out)
        return list(out)

    def stats(self, constraint=None, options=None) -> dict:
        s = ccmi.StatsStruct()
        o, keep = (options or ccmi.OptimizationOptions()).to_struct()
        c = (constraint or ccmi.BalancingConstraint()).to_struct(self.topic_names())
        self.L.oc_stats(self.h, C.byref(c), C.byref(o), C.byref(s))
        return ccmi.stats_to_dict(s)

    def proposals(self, max_rf: int = 8) -> List[ccmi.ExecutionProposal]:
        n = self.L.oc_proposal_count(self.h)
        if n == 0:
            return []
        part, size, old_leader = (C.c_int32 * n)(), (C.c_int32 * n)(), (C.c_int32 * n)()
        old_r, new_r = (C.c_int32 * (n * max_rf))(), (C.c_int32 * (n * max_rf))()
        self.L.oc_proposals(self.h, max_rf, part, size, old_leader, old_r, new_r)
        old_d, new_d = (C.c_int32 * (n * max_rf))(), (C.c_int32 * (n * max_rf))()
        self.L.oc_proposal_disks(self.h, max_rf, old_d, new_d)
        out = []
        for i in range(n):
            rf = sum(1 for x in old_r[i * max_rf:(i + 1) * max_rf] if x >= 0)
            out.append(ccmi.ExecutionProposal(part[i], size[i], old_leader[i], list(old_r[i * max_rf:i * max_rf + rf]),
                                              list(new_r[i * max_rf:i * max_rf + rf]),
                                              list(old_d[i * max_rf:i * max_rf + rf]),
                                              list(new_d[i * max_rf:i * max_rf + rf])))
        return out


def desc_arrays(desc: ccmi.ClusterDesc) -> dict:
    """Flattened desc as python lists (same keys as OracleCluster.export)."""
    B, P, R, W, T = desc.num_brokers, desc.num_partitions, desc.num_replicas, desc.num_windows, desc.num_topics
    out = dict(broker_rack=desc.broker_rack[:B], broker_state=desc.broker_state[:B],
                cap=desc.broker_capacity[:4 * B], partition_topic=desc.partition_topic[:P],
                partition_number=desc.partition_number[:P], partition_offset=desc.partition_offset[:P + 1],
                partition_replicas=desc.partition_replicas[:R], replica_partition=desc.replica_partition[:R],
                replica_broker=desc.replica_broker[:R], is_leader=desc.replica_is_leader[:R],
                offline=desc.replica_offline[:R], load=desc.replica_load[:R * 6 * W],
                topics=[desc.topic_names[t].decode() for t in range(T)], num_disks=desc.num_disks)
    D, n = desc.num_disks, desc.num_disk_assignments
    if D:
        out.update(disk_broker=desc.disk_broker[:D], disk_capacity=desc.disk_capacity[:D],
                   replica_disk=desc.replica_disk[:R] if desc.replica_disk else [-1] * R,
                   disk_logdir=[desc.disk_logdir[d].decode() for d in range(D)],
                   disk_assign_replica=desc.disk_assign_replica[:n], disk_assign_disk=desc.disk_assign_disk[:n])
    return out


class ArrayDesc:
    """A ccmi_cluster_desc over python lists with the keys of OracleCluster.export (no disks): the inverse of
    desc_arrays, for test models derived from another model's state (e.g. RandomClusterTest.testNewBrokers)."""

    def __init__(self, a: dict, num_windows: int = 1):
        B, P, R = len(a["broker_rack"]), len(a["partition_topic"]), len(a["replica_partition"])
        T = len(a["topics"])
        arr = lambda ct, xs: (ct * max(1, len(xs)))(*xs)  # noqa: E731
        self.keep = dict(
            broker_id=arr(C.c_int32, list(range(B))), broker_rack=arr(C.c_int32, a["broker_rack"]),
            broker_state=arr(C.c_int32, a["broker_state"]), broker_capacity=arr(C.c_double, a["cap"]),
            topic_names=arr(C.c_char_p, [t.encode() for t in a["topics"]]),
            partition_topic=arr(C.c_int32, a["partition_topic"]), partition_number=arr(C.c_int32, a["partition_number"]),
            partition_offset=arr(C.c_int32, a["partition_offset"]),
            partition_replicas=arr(C.c_int32, a["partition_replicas"]),
            replica_partition=arr(C.c_int32, a["replica_partition"]), replica_broker=arr(C.c_int32, a["replica_broker"]),
            replica_is_leader=arr(C.c_uint8, a["is_leader"]), replica_offline=arr(C.c_uint8, a["offline"]),
            replica_load=arr(C.c_float, a["load"]),
            replica_load_order=arr(C.c_int32, a.get("load_order", list(range(R)))))
        d = ccmi.ClusterDesc()
        d.num_windows, d.num_racks, d.num_brokers = num_windows, max(a["broker_rack"]) + 1, B
        d.num_topics, d.num_partitions, d.num_replicas = T, P, R
        for k, v in self.keep.items():
            setattr(d, k, C.cast(v, type(getattr(d, k))) if k != "topic_names" else v)
        self.desc = d
