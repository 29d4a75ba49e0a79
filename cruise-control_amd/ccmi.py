"""Python binding of libccmi.so (include/ccmi.h) mirroring the reference's optimizer interface.

Names follow the reference so parity tests read like the reference's own tests:

  ClusterModel            <- com.linkedin.kafka.cruisecontrol.model.ClusterModel (a device session)
  GoalOptimizer           <- analyzer/GoalOptimizer.java  (optimizations(), GoalOptimizer.java:435-524)
  <Goal>                  <- analyzer/goals/*Goal.java     (name(), optimize(), actionAcceptance())
  OptimizationOptions     <- analyzer/OptimizationOptions.java
  BalancingConstraint     <- analyzer/BalancingConstraint.java (AnalyzerConfig.java defaults)
  OptimizerResult         <- analyzer/OptimizerResult.java  (proposals, per-goal stats)
  ExecutionProposal       <- executor/ExecutionProposal.java
  RandomCluster           <- src/test/.../model/RandomCluster.java (fixture generator)

Errors map to the reference's exceptions: OptimizationFailureException, IllegalStateException,
IllegalArgumentException; a missing/unsupported device raises DeviceError (no CPU fallback exists).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence

_HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_LIB = os.path.join(_HERE, "libccmi.so")

RESOURCES = ("CPU", "NW_IN", "NW_OUT", "DISK")
CPU, NW_IN, NW_OUT, DISK = range(4)

GOAL_KINDS: Dict[str, int] = {
    "RackAwareGoal": 0,
    "MinTopicLeadersPerBrokerGoal": 1,
    "ReplicaCapacityGoal": 2,
    "DiskCapacityGoal": 3,
    "NetworkInboundCapacityGoal": 4,
    "NetworkOutboundCapacityGoal": 5,
    "CpuCapacityGoal": 6,
    "ReplicaDistributionGoal": 7,
    "PotentialNwOutGoal": 8,
    "DiskUsageDistributionGoal": 9,
    "NetworkInboundUsageDistributionGoal": 10,
    "NetworkOutboundUsageDistributionGoal": 11,
    "CpuUsageDistributionGoal": 12,
    "TopicReplicaDistributionGoal": 13,
    "LeaderReplicaDistributionGoal": 14,
    "LeaderBytesInDistributionGoal": 15,
    "IntraBrokerDiskCapacityGoal": 16,
    "IntraBrokerDiskUsageDistributionGoal": 17,
    "PreferredLeaderElectionGoal": 18,
    "RackAwareDistributionGoal": 19,
    "BrokerSetAwareGoal": 20,
    "TopicLeaderReplicaDistributionGoal": 21,
    "KafkaAssignerEvenRackAwareGoal": 22,
    "KafkaAssignerDiskUsageDistributionGoal": 23,
}
GOAL_NAMES = {v: k for k, v in GOAL_KINDS.items()}
# default.goals in priority order (config/constants/AnalyzerConfig.java:352-367, TestConstants.DEFAULT_GOALS_VALUES)
DEFAULT_GOALS = ("RackAwareGoal", "MinTopicLeadersPerBrokerGoal", "ReplicaCapacityGoal", "DiskCapacityGoal",
                 "NetworkInboundCapacityGoal", "NetworkOutboundCapacityGoal", "CpuCapacityGoal",
                 "ReplicaDistributionGoal", "PotentialNwOutGoal", "DiskUsageDistributionGoal",
                 "NetworkInboundUsageDistributionGoal", "NetworkOutboundUsageDistributionGoal",
                 "CpuUsageDistributionGoal", "TopicReplicaDistributionGoal", "LeaderReplicaDistributionGoal",
                 "LeaderBytesInDistributionGoal")
# config C1's chain
C1_GOALS = ("ReplicaDistributionGoal", "DiskUsageDistributionGoal", "NetworkInboundUsageDistributionGoal",
            "NetworkOutboundUsageDistributionGoal", "CpuUsageDistributionGoal")
# intra.broker.goals (AnalyzerConfig INTRA_BROKER_GOALS default, IntraBrokerRebalanceTest.java:105-106)
INTRA_BROKER_GOALS = ("IntraBrokerDiskCapacityGoal", "IntraBrokerDiskUsageDistributionGoal")
# Goals whose drivers are implemented in this build.
IMPLEMENTED = DEFAULT_GOALS + INTRA_BROKER_GOALS + ("PreferredLeaderElectionGoal", "RackAwareDistributionGoal",
                                                   "BrokerSetAwareGoal", "TopicLeaderReplicaDistributionGoal",
                                                   "KafkaAssignerEvenRackAwareGoal",
                                                   "KafkaAssignerDiskUsageDistributionGoal")
# replica.to.broker.set.mapping.policy.class values (include/ccmi.h ccmi_broker_set_policy)
BROKER_SET_POLICIES = {"TopicNameHashBrokerSetMappingPolicy": 0, "ReplicaToOriginalBrokerSetMappingPolicy": 1}

ACTION_TYPES = ("INTER_BROKER_REPLICA_MOVEMENT", "LEADERSHIP_MOVEMENT", "INTER_BROKER_REPLICA_SWAP",
                "INTRA_BROKER_REPLICA_MOVEMENT", "INTRA_BROKER_REPLICA_SWAP")
ACCEPTANCE = ("ACCEPT", "REPLICA_REJECT", "BROKER_REJECT")


# ----------------------------------------------------------------------------------------------- ctypes layouts
class ClusterDesc(C.Structure):
    _fields_ = [("num_windows", C.c_int32), ("num_racks", C.c_int32), ("num_brokers", C.c_int32),
                ("broker_id", C.POINTER(C.c_int32)), ("broker_rack", C.POINTER(C.c_int32)),
                ("broker_state", C.POINTER(C.c_int32)), ("broker_capacity", C.POINTER(C.c_double)),
                ("num_topics", C.c_int32), ("topic_names", C.POINTER(C.c_char_p)),
                ("num_partitions", C.c_int32), ("partition_topic", C.POINTER(C.c_int32)),
                ("partition_number", C.POINTER(C.c_int32)), ("partition_offset", C.POINTER(C.c_int32)),
                ("partition_replicas", C.POINTER(C.c_int32)), ("num_replicas", C.c_int32),
                ("replica_partition", C.POINTER(C.c_int32)), ("replica_broker", C.POINTER(C.c_int32)),
                ("replica_is_leader", C.POINTER(C.c_uint8)), ("replica_offline", C.POINTER(C.c_uint8)),
                ("replica_load", C.POINTER(C.c_float)), ("replica_load_order", C.POINTER(C.c_int32)),
                ("num_disks", C.c_int32), ("disk_broker", C.POINTER(C.c_int32)),
                ("disk_logdir", C.POINTER(C.c_char_p)), ("disk_capacity", C.POINTER(C.c_double)),
                ("replica_disk", C.POINTER(C.c_int32)), ("num_disk_assignments", C.c_int32),
                ("disk_assign_replica", C.POINTER(C.c_int32)), ("disk_assign_disk", C.POINTER(C.c_int32)),
                ("num_replica_loads", C.c_int32), ("broker_host", C.POINTER(C.c_int32)),
                ("disk_demoted", C.POINTER(C.c_uint8))]


class ConstraintStruct(C.Structure):
    _fields_ = [("resource_balance_percentage", C.c_double * 4), ("capacity_threshold", C.c_double * 4),
                ("low_utilization_threshold", C.c_double * 4), ("replica_balance_percentage", C.c_double),
                ("leader_replica_balance_percentage", C.c_double), ("topic_replica_balance_percentage", C.c_double),
                ("topic_replica_balance_min_gap", C.c_int32), ("topic_replica_balance_max_gap", C.c_int32),
                ("goal_violation_distribution_threshold_multiplier", C.c_double),
                ("max_replicas_per_broker", C.c_int64), ("overprovisioned_max_replicas_per_broker", C.c_int64),
                ("overprovisioned_min_brokers", C.c_int32), ("overprovisioned_min_extra_racks", C.c_int32),
                ("num_broker_sets", C.c_int32), ("broker_set_policy", C.c_int32),
                ("broker_set_names", C.POINTER(C.c_char_p)), ("broker_set_offset", C.POINTER(C.c_int32)),
                ("broker_set_members", C.POINTER(C.c_int32)), ("min_leader_topics", C.POINTER(C.c_int32)),
                ("num_min_leader_topics", C.c_int32), ("min_topic_leaders_per_broker", C.c_int32),
                ("topic_leader_replica_balance_percentage", C.c_double),
                ("topic_leader_replica_balance_min_gap", C.c_int32), ("topic_leader_replica_balance_max_gap", C.c_int32),
                ("topic_leader_replica_balance_margin", C.c_double)]


class OptionsStruct(C.Structure):
    _fields_ = [("excluded_topics", C.POINTER(C.c_int32)), ("num_excluded_topics", C.c_int32),
                ("excluded_brokers_for_leadership", C.POINTER(C.c_int32)),
                ("num_excluded_brokers_for_leadership", C.c_int32),
                ("excluded_brokers_for_replica_move", C.POINTER(C.c_int32)),
                ("num_excluded_brokers_for_replica_move", C.c_int32), ("triggered_by_goal_violation", C.c_int32),
                ("requested_destination_broker_ids", C.POINTER(C.c_int32)),
                ("num_requested_destination_broker_ids", C.c_int32), ("only_move_immigrant_replicas", C.c_int32),
                ("fast_mode", C.c_int32)]


class ActionStruct(C.Structure):
    _fields_ = [("type", C.c_int32), ("partition", C.c_int32), ("source_broker", C.c_int32),
                ("destination_broker", C.c_int32), ("destination_partition", C.c_int32),
                ("source_disk", C.c_int32), ("destination_disk", C.c_int32)]


class StatsStruct(C.Structure):
    _fields_ = [("resource_avg", C.c_double * 4), ("resource_max", C.c_double * 4),
                ("resource_min", C.c_double * 4), ("resource_std", C.c_double * 4),
                ("num_balanced_brokers_by_resource", C.c_int32 * 4), ("potential_nw_out_avg", C.c_double),
                ("potential_nw_out_max", C.c_double), ("potential_nw_out_min", C.c_double),
                ("potential_nw_out_std", C.c_double), ("num_brokers_under_potential_nw_out", C.c_int32),
                ("replica_avg", C.c_double), ("replica_std", C.c_double), ("replica_max", C.c_int32),
                ("replica_min", C.c_int32), ("leader_avg", C.c_double), ("leader_std", C.c_double),
                ("leader_max", C.c_int32), ("leader_min", C.c_int32), ("topic_replica_avg", C.c_double),
                ("topic_replica_std", C.c_double), ("topic_replica_max", C.c_int32), ("topic_replica_min", C.c_int32),
                ("num_brokers", C.c_int32), ("num_replicas_in_cluster", C.c_int32),
                ("num_partitions_with_offline_replicas", C.c_int32), ("num_topics", C.c_int32),
                ("num_unbalanced_disks", C.c_int32), ("disk_utilization_std", C.c_double)]


class ProvisionRecStruct(C.Structure):
    _fields_ = [("status", C.c_int32), ("num_brokers", C.c_int32), ("num_racks", C.c_int32), ("num_disks", C.c_int32),
                ("num_partitions", C.c_int32), ("typical_broker_id", C.c_int32), ("resource", C.c_int32),
                ("pad", C.c_int32), ("typical_broker_capacity", C.c_double), ("total_capacity", C.c_double)]


class ProvisionRespStruct(C.Structure):
    _fields_ = [("status", C.c_int32), ("has_recommendation", C.c_int32), ("recommendation", ProvisionRecStruct)]


class GoalResultStruct(C.Structure):
    _fields_ = [("goal_kind", C.c_int32), ("succeeded", C.c_int32), ("has_diff", C.c_int32), ("seconds", C.c_double),
                ("candidates", C.c_int64), ("device_candidates", C.c_int64), ("device_launches", C.c_int64),
                ("actions", C.c_int64), ("stats", StatsStruct), ("provision", ProvisionRespStruct)]


class RandomClusterProps(C.Structure):
    _fields_ = [("num_racks", C.c_int32), ("num_brokers", C.c_int32), ("num_dead_brokers", C.c_int32),
                ("num_brokers_with_bad_disk", C.c_int32), ("num_replicas", C.c_int32), ("num_topics", C.c_int32),
                ("min_replication", C.c_int32), ("max_replication", C.c_int32), ("mean_cpu", C.c_double),
                ("mean_disk", C.c_double), ("mean_nw_in", C.c_double), ("mean_nw_out", C.c_double),
                ("distribution", C.c_int32), ("rack_aware", C.c_int32), ("leader_in_first_position", C.c_int32),
                ("jbod", C.c_int32), ("num_logdirs", C.c_int32), ("logdir_capacity", C.c_double * 8)]


class PerfStruct(C.Structure):
    _fields_ = [("scan_launches", C.c_int64), ("scan_kernel_ms", C.c_double), ("scan_bytes", C.c_int64),
                ("stats_launches", C.c_int64), ("stats_kernel_ms", C.c_double), ("stats_bytes", C.c_int64),
                ("host_syncs", C.c_int64), ("scan_required", C.c_int64), ("chain_launches", C.c_int64),
                ("intra_launches", C.c_int64), ("intra_kernel_ms", C.c_double), ("intra_bytes", C.c_int64),
                ("cross_launches", C.c_int64), ("cross_required", C.c_int64), ("cross_kernel_ms", C.c_double),
                ("combines", C.c_int64), ("server_launches", C.c_int64), ("server_scans", C.c_int64),
                ("server_required", C.c_int64), ("server_busy_ms", C.c_double),
                ("server_payload_bytes", C.c_int64), ("server_chains", C.c_int64),
                ("server_idle_exits", C.c_int64), ("server_resident_ms", C.c_double),
                ("intra_sort_launches", C.c_int64), ("intra_sort_ms", C.c_double)]


# ----------------------------------------------------------------------------------------------- errors
class CruiseControlError(RuntimeError):
    pass


class OptimizationFailureException(CruiseControlError):
    pass


class IllegalStateException(CruiseControlError):
    pass


class IllegalArgumentException(CruiseControlError):
    pass


class UnsupportedOperationException(CruiseControlError):
    pass


class DeviceError(CruiseControlError):
    pass


_STATUS = {1: IllegalArgumentException, 2: DeviceError, 3: OptimizationFailureException, 4: IllegalStateException,
           5: UnsupportedOperationException}

ABI_VERSION = 12  # CCMI_ABI_VERSION of include/ccmi.h
EXPORTED_SYMBOLS = (
    "ccmi_last_error", "ccmi_abi_version", "ccmi_device_count", "ccmi_default_constraint", "ccmi_default_random_cluster_props",
    "ccmi_random_cluster", "ccmi_cluster_buffers_desc", "ccmi_cluster_buffers_free", "ccmi_session_create",
    "ccmi_session_destroy", "ccmi_optimizations", "ccmi_goal_optimize", "ccmi_action_acceptance",
    "ccmi_action_acceptance_by_kind", "ccmi_session_apply", "ccmi_last_failure_provision",
    "ccmi_compute_cluster_stats", "ccmi_action_log_count", "ccmi_action_log_copy", "ccmi_replica_distribution",
    "ccmi_leader_distribution", "ccmi_replica_disks", "ccmi_proposal_count", "ccmi_proposals",
    "ccmi_proposal_disks", "ccmi_perf", "ccmi_perf_reset",
    "ccmi_set_kernel_timing", "ccmi_session_set_shard", "ccmi_rccl_unique_id", "ccmi_session_attach_rccl",
    "ccmi_session_attach_shm", "ccmi_session_attach_shm_job", "ccmi_shard_group_create", "ccmi_shard_group_destroy", "ccmi_session_attach_group",
    "ccmi_topic_broker_set",
    "ccmi_builder_create", "ccmi_builder_destroy", "ccmi_builder_create_broker", "ccmi_builder_add_disk",
    "ccmi_builder_populate_partition", "ccmi_builder_set_broker_state", "ccmi_builder_set_disk_state",
    "ccmi_builder_desc", "ccmi_builder_broker_ids")

# int (*)(void* ctx, int64_t* key): replace *key by the MIN over all shards, return 0 (include/ccmi.h)
AllreduceMinFn = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_int64))


class Library:
    """Loaded libccmi.so (or, in CPU tests only, the emulation build from tests/emu)."""

    _cache: Dict[str, "Library"] = {}

    def __init__(self, path: str = DEFAULT_LIB):
        if not os.path.exists(path):
            raise DeviceError(f"{path} not found: build it with __graft_entry__.build() (no CPU fallback exists)")
        self.path = path
        self.lib = C.CDLL(path)
        L = self.lib
        if L.ccmi_abi_version() != ABI_VERSION:  # the struct layouts below are ABI_VERSION's (include/ccmi.h)
            raise DeviceError(f"{path} has ABI {L.ccmi_abi_version()}, this binding needs {ABI_VERSION}: rebuild it")
        L.ccmi_last_error.restype = C.c_char_p
        L.ccmi_random_cluster.argtypes = [C.POINTER(RandomClusterProps), C.POINTER(C.c_void_p)]
        L.ccmi_cluster_buffers_desc.restype = C.POINTER(ClusterDesc)
        L.ccmi_cluster_buffers_desc.argtypes = [C.c_void_p]
        L.ccmi_cluster_buffers_free.argtypes = [C.c_void_p]
        L.ccmi_session_create.argtypes = [C.c_int32, C.POINTER(ClusterDesc), C.POINTER(C.c_void_p)]
        L.ccmi_session_destroy.argtypes = [C.c_void_p]
        L.ccmi_optimizations.argtypes = [C.c_void_p, C.POINTER(C.c_int32), C.c_int32, C.POINTER(ConstraintStruct),
                                         C.POINTER(OptionsStruct), C.POINTER(GoalResultStruct)]
        L.ccmi_goal_optimize.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_int32), C.c_int32,
                                         C.POINTER(ConstraintStruct), C.POINTER(OptionsStruct),
                                         C.POINTER(GoalResultStruct)]
        L.ccmi_action_acceptance.argtypes = [C.c_void_p, C.c_int32, C.POINTER(ActionStruct), C.POINTER(C.c_int32)]
        L.ccmi_action_acceptance_by_kind.argtypes = [C.c_void_p, C.c_int32, C.POINTER(ActionStruct),
                                                     C.POINTER(C.c_int32)]
        L.ccmi_session_apply.argtypes = [C.c_void_p, C.POINTER(ActionStruct), C.c_int64, C.POINTER(C.c_int64)]
        L.ccmi_last_failure_provision.argtypes = [C.c_void_p, C.POINTER(ProvisionRespStruct)]
        L.ccmi_compute_cluster_stats.argtypes = [C.c_void_p, C.POINTER(ConstraintStruct), C.POINTER(OptionsStruct),
                                                 C.POINTER(StatsStruct)]
        L.ccmi_action_log_count.restype = C.c_int64
        L.ccmi_action_log_count.argtypes = [C.c_void_p]
        L.ccmi_action_log_copy.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.POINTER(ActionStruct)]
        L.ccmi_replica_distribution.argtypes = [C.c_void_p, C.POINTER(C.c_int32)]
        L.ccmi_leader_distribution.argtypes = [C.c_void_p, C.POINTER(C.c_int32)]
        L.ccmi_proposal_count.restype = C.c_int64
        L.ccmi_proposal_count.argtypes = [C.c_void_p]
        L.ccmi_proposals.argtypes = [C.c_void_p, C.c_int32] + [C.POINTER(C.c_int32)] * 5
        L.ccmi_proposal_disks.argtypes = [C.c_void_p, C.c_int32] + [C.POINTER(C.c_int32)] * 2
        L.ccmi_replica_disks.argtypes = [C.c_void_p, C.POINTER(C.c_int32)]
        L.ccmi_builder_create.argtypes = [C.c_int32, C.POINTER(C.c_void_p)]
        L.ccmi_builder_destroy.argtypes = [C.c_void_p]
        L.ccmi_builder_destroy.restype = None
        L.ccmi_builder_create_broker.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.c_int32,
                                                 C.POINTER(C.c_double), C.c_int32]
        L.ccmi_builder_add_disk.argtypes = [C.c_void_p, C.c_int32, C.c_char_p, C.c_double]
        L.ccmi_builder_populate_partition.argtypes = [C.c_void_p, C.c_char_p, C.c_int32, C.POINTER(C.c_int32),
                                                      C.c_int32, C.c_int32, C.POINTER(C.c_uint8),
                                                      C.POINTER(C.c_char_p), C.POINTER(C.c_float)]
        L.ccmi_builder_set_broker_state.argtypes = [C.c_void_p, C.c_int32, C.c_int32]
        L.ccmi_builder_set_disk_state.argtypes = [C.c_void_p, C.c_int32, C.c_char_p, C.c_int32]
        L.ccmi_builder_desc.argtypes = [C.c_void_p, C.POINTER(ClusterDesc)]
        L.ccmi_builder_broker_ids.argtypes = [C.c_void_p, C.POINTER(C.c_int32)]
        L.ccmi_perf.argtypes = [C.c_void_p, C.POINTER(PerfStruct)]
        L.ccmi_perf_reset.argtypes = [C.c_void_p]
        L.ccmi_set_kernel_timing.argtypes = [C.c_void_p, C.c_int32]
        L.ccmi_session_set_shard.argtypes = [C.c_void_p, C.c_int32, C.c_int32, AllreduceMinFn, C.c_void_p]
        L.ccmi_rccl_unique_id.argtypes = [C.POINTER(C.c_uint8)]
        L.ccmi_session_attach_rccl.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.POINTER(C.c_uint8)]
        L.ccmi_session_attach_shm.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_char_p]
        L.ccmi_session_attach_shm_job.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_char_p, C.c_uint64, C.c_double]
        L.ccmi_shard_group_create.argtypes = [C.c_int32, C.POINTER(C.c_void_p)]
        L.ccmi_shard_group_destroy.argtypes = [C.c_void_p]
        L.ccmi_session_attach_group.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
        L.ccmi_default_constraint.argtypes = [C.POINTER(ConstraintStruct)]
        L.ccmi_topic_broker_set.restype = C.c_int32
        L.ccmi_topic_broker_set.argtypes = [C.c_char_p, C.c_int32]
        L.ccmi_default_random_cluster_props.argtypes = [C.POINTER(RandomClusterProps)]
        L.ccmi_device_count.restype = C.c_int32
        L.ccmi_device_count.argtypes = []

    def device_count(self) -> int:
        """Visible gfx950 devices (ccmi_device_count)."""
        return int(self.lib.ccmi_device_count())

    @classmethod
    def get(cls, path: str = DEFAULT_LIB) -> "Library":
        if path not in cls._cache:
            cls._cache[path] = Library(path)
        return cls._cache[path]

    def check(self, status: int) -> None:
        if status != 0:
            msg = self.lib.ccmi_last_error().decode(errors="replace")
            raise _STATUS.get(status, CruiseControlError)(msg)


# ----------------------------------------------------------------------------------------------- options / constraint
@dataclass
class BalancingConstraint:
    resource_balance_percentage: Sequence[float] = (1.10, 1.10, 1.10, 1.10)
    capacity_threshold: Sequence[float] = (0.7, 0.8, 0.8, 0.8)
    low_utilization_threshold: Sequence[float] = (0.0, 0.0, 0.0, 0.0)
    replica_balance_percentage: float = 1.10
    goal_violation_distribution_threshold_multiplier: float = 1.0
    max_replicas_per_broker: int = 10000
    leader_replica_balance_percentage: float = 1.10
    topic_replica_balance_percentage: float = 3.00
    topic_replica_balance_min_gap: int = 2
    topic_replica_balance_max_gap: int = 40
    overprovisioned_min_extra_racks: int = 2  # AnalyzerConfig.DEFAULT_OVERPROVISIONED_MIN_EXTRA_RACKS
    # BrokerSetAwareGoal: BalancingConstraint.brokerSetResolver() data (broker set id -> broker ids, the content of
    # broker.set.config.file for BrokerSetFileResolver) and replica.to.broker.set.mapping.policy.class. Brokers in no
    # set join "unmapped" (NoOpBrokerSetAssignmentPolicy, the default broker.set.assignment.policy.class).
    broker_sets: Optional[Dict[str, Sequence[int]]] = None
    broker_set_policy: str = "TopicNameHashBrokerSetMappingPolicy"
    # topics.with.min.leaders.per.broker (a regex; "" matches no topic) and min.topic.leaders.per.broker
    # (AnalyzerConfig.java:401-414). The pattern is matched against the session's topic names as
    # Utils.getTopicNamesMatchedWithPattern does (Pattern.matcher(topic).matches() = re.fullmatch; common/Utils.java:26-36).
    topics_with_min_leaders_per_broker: str = ""
    min_topic_leaders_per_broker: int = 1
    # TopicLeaderReplicaDistributionGoal: topic.leader.replica.count.balance.{threshold,min.gap,max.gap} and
    # topic.leader.replica.distribution.goal.balance.margin (AnalyzerConfig.java:112-146)
    topic_leader_replica_balance_percentage: float = 1.10
    topic_leader_replica_balance_min_gap: int = 2
    topic_leader_replica_balance_max_gap: int = 10
    topic_leader_replica_balance_margin: float = 0.9

    def set_resource_balance_percentage(self, p: float) -> None:  # BalancingConstraint.setResourceBalancePercentage
        self.resource_balance_percentage = (p, p, p, p)

    def set_capacity_threshold(self, t: float) -> None:
        self.capacity_threshold = (t, t, t, t)

    def min_leader_topics(self, topic_names: Optional[Sequence[str]]) -> List[int]:
        """Topic indices topics.with.min.leaders.per.broker matches (Utils.getTopicNamesMatchedWithPattern)."""
        if not self.topics_with_min_leaders_per_broker:
            return []
        import re
        pat = re.compile(self.topics_with_min_leaders_per_broker)
        if topic_names is None:
            raise IllegalArgumentException("topics.with.min.leaders.per.broker needs the cluster's topic names")
        return [t for t, n in enumerate(topic_names) if pat.fullmatch(n)]

    def to_struct(self, topic_names: Optional[Sequence[str]] = None,
                  broker_ids: Optional[Sequence[int]] = None) -> ConstraintStruct:
        """broker_ids: the session's Kafka broker id of every broker index (ClusterModel.broker_ids); the broker ids
        of `broker_sets` are mapped through it to the session's dense indices (ccmi_balancing_constraint
        broker_set_members), an id the model does not hold to -1. None: ids are the indices."""
        s = ConstraintStruct()
        s.resource_balance_percentage[:] = list(self.resource_balance_percentage)
        s.capacity_threshold[:] = list(self.capacity_threshold)
        s.low_utilization_threshold[:] = list(self.low_utilization_threshold)
        s.replica_balance_percentage = self.replica_balance_percentage
        s.leader_replica_balance_percentage = self.leader_replica_balance_percentage
        s.topic_replica_balance_percentage = self.topic_replica_balance_percentage
        s.topic_replica_balance_min_gap = self.topic_replica_balance_min_gap
        s.topic_replica_balance_max_gap = self.topic_replica_balance_max_gap
        s.goal_violation_distribution_threshold_multiplier = self.goal_violation_distribution_threshold_multiplier
        s.max_replicas_per_broker = self.max_replicas_per_broker
        s.overprovisioned_max_replicas_per_broker = 1500
        s.overprovisioned_min_brokers = 3
        s.overprovisioned_min_extra_racks = self.overprovisioned_min_extra_racks
        s.topic_leader_replica_balance_percentage = self.topic_leader_replica_balance_percentage
        s.topic_leader_replica_balance_min_gap = self.topic_leader_replica_balance_min_gap
        s.topic_leader_replica_balance_max_gap = self.topic_leader_replica_balance_max_gap
        s.topic_leader_replica_balance_margin = self.topic_leader_replica_balance_margin
        if self.broker_sets:
            names = list(self.broker_sets)
            index_of = None if broker_ids is None else {int(k): i for i, k in enumerate(broker_ids)}
            members = [int(b) if index_of is None else index_of.get(int(b), -1)
                       for n in names for b in self.broker_sets[n]]
            offs = [0]
            for n in names:
                offs.append(offs[-1] + len(self.broker_sets[n]))
            keep = [(C.c_char_p * len(names))(*[n.encode() for n in names]), (C.c_int32 * len(offs))(*offs),
                    (C.c_int32 * max(1, len(members)))(*members)]
            s._keep = keep  # the arrays live as long as the struct
            s.num_broker_sets = len(names)
            s.broker_set_names = C.cast(keep[0], C.POINTER(C.c_char_p))
            s.broker_set_offset = C.cast(keep[1], C.POINTER(C.c_int32))
            s.broker_set_members = C.cast(keep[2], C.POINTER(C.c_int32))
        if self.broker_set_policy not in BROKER_SET_POLICIES:
            raise IllegalArgumentException(f"unknown broker set mapping policy {self.broker_set_policy}")
        s.broker_set_policy = BROKER_SET_POLICIES[self.broker_set_policy]
        if self.min_topic_leaders_per_broker < 0:  # ConfigDef atLeast(0)
            raise IllegalArgumentException("min.topic.leaders.per.broker must be at least 0")
        s.min_topic_leaders_per_broker = self.min_topic_leaders_per_broker
        mlt = self.min_leader_topics(topic_names)
        if mlt:
            a = (C.c_int32 * len(mlt))(*mlt)
            s._keep_mlt = a
            s.min_leader_topics = C.cast(a, C.POINTER(C.c_int32))
            s.num_min_leader_topics = len(mlt)
        return s


@dataclass
class OptimizationOptions:
    excluded_topics: Sequence[int] = ()
    excluded_brokers_for_leadership: Sequence[int] = ()
    excluded_brokers_for_replica_move: Sequence[int] = ()
    is_triggered_by_goal_violation: bool = False
    requested_destination_broker_ids: Sequence[int] = ()
    only_move_immigrant_replicas: bool = False
    # The reference defaults fastMode to true (OptimizationOptions 6-arg ctor), which caps every per-broker loop by a
    # wall-clock timeout (fast.mode.per.broker.move.timeout.ms) and makes the result depend on host speed. The
    # engine never cuts a loop short — the result fast mode reaches when no timeout fires — so the binding defaults
    # to False to say so explicitly; fast_mode=True is accepted and behaves identically.
    fast_mode: bool = False

    def to_struct(self):
        keep = []

        def arr(xs):
            a = (C.c_int32 * max(1, len(xs)))(*xs)
            keep.append(a)
            return C.cast(a, C.POINTER(C.c_int32)), len(xs)

        s = OptionsStruct()
        s.excluded_topics, s.num_excluded_topics = arr(list(self.excluded_topics))
        s.excluded_brokers_for_leadership, s.num_excluded_brokers_for_leadership = arr(
            list(self.excluded_brokers_for_leadership))
        s.excluded_brokers_for_replica_move, s.num_excluded_brokers_for_replica_move = arr(
            list(self.excluded_brokers_for_replica_move))
        s.triggered_by_goal_violation = int(self.is_triggered_by_goal_violation)
        s.requested_destination_broker_ids, s.num_requested_destination_broker_ids = arr(
            list(self.requested_destination_broker_ids))
        s.only_move_immigrant_replicas = int(self.only_move_immigrant_replicas)
        s.fast_mode = int(self.fast_mode)
        return s, keep


# ----------------------------------------------------------------------------------------------- goals
class Goal:
    """A goal plugin by reference simple class name (Goal.name(), AbstractGoal.java:141-144)."""

    def __init__(self, name: Optional[str] = None, constraint: Optional[BalancingConstraint] = None):
        self._name = name or type(self).__name__
        if self._name not in GOAL_KINDS:
            raise IllegalArgumentException(f"unknown goal {self._name}")
        self.constraint = constraint

    def name(self) -> str:
        return self._name

    @property
    def kind(self) -> int:
        return GOAL_KINDS[self._name]

    # Goal.isHardGoal(): AbstractRackAwareGoal (both rack goals), BrokerSetAwareGoal, CapacityGoal, ReplicaCapacityGoal,
    # IntraBrokerDiskCapacityGoal return true (analyzer/goals/*.java)
    HARD_GOALS = ("RackAwareGoal", "RackAwareDistributionGoal", "BrokerSetAwareGoal", "ReplicaCapacityGoal",
                  "DiskCapacityGoal", "NetworkInboundCapacityGoal", "NetworkOutboundCapacityGoal", "CpuCapacityGoal",
                  "IntraBrokerDiskCapacityGoal", "KafkaAssignerEvenRackAwareGoal",
                  "KafkaAssignerDiskUsageDistributionGoal")

    def is_hard_goal(self) -> bool:
        return self._name in self.HARD_GOALS

    def optimize(self, cluster: "ClusterModel", optimized_goals: Iterable["Goal"] = (),
                 options: Optional[OptimizationOptions] = None) -> bool:
        """Goal.optimize(clusterModel, optimizedGoals, optimizationOptions) (Goal.java:60-68). Only the goals in
        `optimized_goals` constrain this goal's moves through their actionAcceptance; each must have been optimized
        on this session (else UnsupportedOperationException: the JVM would run the goal). The session
        keeps this goal, with its frozen state, for later optimized_goals sets."""
        if isinstance(optimized_goals, OptimizationOptions):
            raise IllegalArgumentException("Goal.optimize(cluster, optimized_goals, options): optimized_goals first")
        res = cluster._goal_optimize(self, optimized_goals, options)
        return bool(res.succeeded)

    def __repr__(self) -> str:
        return self._name


for _n in GOAL_KINDS:
    globals()[_n] = type(_n, (Goal,), {})


# ----------------------------------------------------------------------------------------------- results
PROVISION_STATUSES = ("UNDECIDED", "RIGHT_SIZED", "UNDER_PROVISIONED", "OVER_PROVISIONED")  # ProvisionStatus.java


@dataclass
class ProvisionRecommendation:
    """analyzer/ProvisionRecommendation.java (-1 = unset; topic pattern and excluded rack ids not carried)."""
    status: str
    num_brokers: int = -1
    num_racks: int = -1
    num_disks: int = -1
    num_partitions: int = -1
    typical_broker_id: int = -1
    resource: Optional[str] = None
    typical_broker_capacity: float = -1.0
    total_capacity: float = -1.0


RESOURCE_NAMES = {"CPU": "cpu", "NW_IN": "networkInbound", "NW_OUT": "networkOutbound", "DISK": "disk"}  # Resource.java


def _recommendation_text(r: "ProvisionRecommendation") -> str:
    s = f"{'Add' if r.status == 'UNDER_PROVISIONED' else 'Remove'} at least "
    if r.num_brokers != -1:
        s += f"{r.num_brokers} broker{'s' if r.num_brokers > 1 else ''}"
    elif r.num_racks != -1:
        s += f"{r.num_racks} rack{'s' if r.num_racks > 1 else ''} with brokers"
    elif r.num_disks != -1:
        s += f"{r.num_disks} disk{'s' if r.num_disks > 1 else ''}"
    if r.typical_broker_id != -1:
        s += f" with the same {RESOURCE_NAMES[r.resource]} capacity ({r.typical_broker_capacity:.2f}) as broker-" \
             f"{r.typical_broker_id}"
    elif r.resource is not None:
        s += f" for {RESOURCE_NAMES[r.resource]}"
    if r.total_capacity != -1.0:
        s += f" with a total capacity of {r.total_capacity:.2f}"
    return s + "."


def _goal_of_message(msg: str) -> str:
    """The goal name an OptimizationFailureException message starts with ("[GoalName] ...")."""
    return msg[1:msg.index("]")] if msg.startswith("[") and "]" in msg else ""


class ProvisionResponse:
    """analyzer/ProvisionResponse.java: a status and the recommendations by recommender (goal name);
    aggregate() follows ProvisionResponse.aggregate (:97-129)."""

    def __init__(self, status: str = "UNDECIDED", recommendation: Optional[ProvisionRecommendation] = None,
                 recommender: Optional[str] = None):
        if recommendation is not None and status not in ("UNDER_PROVISIONED", "OVER_PROVISIONED"):
            raise IllegalArgumentException(f"Recommendation is irrelevant for provision status {status}.")
        self.status = status
        self.recommendation_by_recommender: Dict[str, ProvisionRecommendation] = {}
        if recommendation is not None:
            if recommender is None:
                raise IllegalArgumentException("The recommender cannot be null.")
            self.recommendation_by_recommender[recommender] = recommendation

    @staticmethod
    def from_struct(p: "ProvisionRespStruct", recommender: str) -> "ProvisionResponse":
        status = PROVISION_STATUSES[p.status]
        if not p.has_recommendation:
            return ProvisionResponse(status)
        r = p.recommendation
        rec = ProvisionRecommendation(PROVISION_STATUSES[r.status], r.num_brokers, r.num_racks, r.num_disks,
                                      r.num_partitions, r.typical_broker_id,
                                      RESOURCES[r.resource] if r.resource >= 0 else None, r.typical_broker_capacity,
                                      r.total_capacity)
        return ProvisionResponse(status, rec, recommender)

    def aggregate(self, other: "ProvisionResponse") -> "ProvisionResponse":
        if self.status == "UNDER_PROVISIONED":
            if other.status == "UNDER_PROVISIONED":
                self.recommendation_by_recommender.update(other.recommendation_by_recommender)
        elif other.status == "UNDER_PROVISIONED":
            self.status = "UNDER_PROVISIONED"
            self.recommendation_by_recommender = dict(other.recommendation_by_recommender)
        elif other.status == "RIGHT_SIZED":
            self.status = "RIGHT_SIZED"
            self.recommendation_by_recommender = {}
        elif other.status == "OVER_PROVISIONED":
            if self.status in ("OVER_PROVISIONED", "UNDECIDED"):
                self.status = "OVER_PROVISIONED"
                self.recommendation_by_recommender.update(other.recommendation_by_recommender)
        return self

    def recommendation(self) -> str:
        """ProvisionResponse.recommendation(): "[recommender] text" per recommendation (ProvisionRecommendation.toString,
        ProvisionRecommendation.java:364-398)."""
        return " ".join(f"[{k}] {_recommendation_text(v)}" for k, v in self.recommendation_by_recommender.items())

    def __eq__(self, other) -> bool:
        return isinstance(other, ProvisionResponse) and (self.status, self.recommendation_by_recommender) == \
            (other.status, other.recommendation_by_recommender)

    def __repr__(self) -> str:
        return f"ProvisionResponse({self.status}, {self.recommendation_by_recommender})"


@dataclass
class ExecutionProposal:
    partition: int
    partition_size: int
    old_leader: int
    old_replicas: List[int]
    new_replicas: List[int]
    old_disks: Optional[List[int]] = None  # logdir half of ReplicaPlacementInfo (disk indices; JBOD models)
    new_disks: Optional[List[int]] = None


@dataclass
class GoalResult:
    name: str
    succeeded: bool
    has_diff: bool
    seconds: float
    candidates: int
    device_candidates: int
    device_launches: int
    actions: int
    stats: Dict[str, object]
    provision: Optional[ProvisionResponse] = None  # Goal.provisionResponse after the goal


class OptimizerResult:
    """analyzer/OptimizerResult.java: per-goal results, the ExecutionProposals and the ordered action log. The
    proposals and the action log are read from the session on first access (the session keeps them until its next
    optimization), so a caller that only needs the statistics does not pay for converting them."""

    def __init__(self, goal_results: List[GoalResult], cluster: "ClusterModel", seconds: float,
                 violated_goals_after: List[str]):
        self.goal_results = goal_results
        self.seconds = seconds
        self.violated_goals_after = violated_goals_after
        self._cluster = cluster
        self._num_actions = cluster.lib.lib.ccmi_action_log_count(cluster.handle)
        self._proposals: Optional[List[ExecutionProposal]] = None
        self._actions: Optional[List[tuple]] = None

    @property
    def proposals(self) -> List[ExecutionProposal]:
        if self._proposals is None:
            self._proposals = self._cluster.proposals()
        return self._proposals

    @property
    def actions(self) -> List[tuple]:
        if self._actions is None:
            self._actions = self._cluster.actions()[:self._num_actions]
        return self._actions

    @property
    def candidates(self) -> int:
        return sum(g.candidates for g in self.goal_results)

    # GoalOptimizer.optimizations (:480-485): a goal is violated before the optimization when it moved something or
    # did not succeed, and after it when it did not succeed
    @property
    def violated_goals_before(self) -> List[str]:
        return [g.name for g in self.goal_results if g.has_diff or not g.succeeded]

    @property
    def violated_goals_after_optimization(self) -> List[str]:
        return list(self.violated_goals_after)

    def _balancedness(self, violated: Sequence[str]) -> float:
        """OptimizerResult.onDemandBalancednessScore (OptimizerResult.java:123-131)."""
        score = MAX_BALANCEDNESS_SCORE
        cost = getattr(self, "balancedness_cost_by_goal", {})
        for g in self.goal_results:
            if g.name in violated:
                score -= cost.get(g.name, 0.0)
        return score

    @property
    def on_demand_balancedness_score_before(self) -> float:
        return self._balancedness(self.violated_goals_before)

    @property
    def on_demand_balancedness_score_after(self) -> float:
        return self._balancedness(self.violated_goals_after)

    def goal_result_description(self, goal_name: str) -> str:
        """OptimizerResult.goalResultDescription (:243-246)."""
        if goal_name not in self.violated_goals_before:
            return "NO-ACTION"
        return "VIOLATED" if goal_name in self.violated_goals_after else "FIXED"

    def movement_stats(self) -> List[int]:
        """OptimizerResult.getMovementStats (:259-279): inter-broker replica moves and MB, intra-broker replica moves
        and MB, leadership moves, over the ExecutionProposals (replicasToAdd / replicasToRemove /
        replicasToMoveBetweenDisksByBroker of ExecutionProposal.java:169-245)."""
        n_inter = mb_inter = n_intra = mb_intra = n_lead = 0
        for p in self.proposals:
            # ExecutionProposal.java:74-78: additions / removals by broker id; a replica whose (broker, logdir) is new
            # on a broker that keeps the partition moves between disks
            old_b, new_b = set(p.old_replicas), set(p.new_replicas)
            to_add, to_remove = new_b - old_b, old_b - new_b
            old_pl = set(zip(p.old_replicas, p.old_disks or [-1] * len(p.old_replicas)))
            between_disks = [b for b, d in zip(p.new_replicas, p.new_disks or [-1] * len(p.new_replicas))
                             if b not in to_add and (b, d) not in old_pl]
            if to_add or to_remove:
                n_inter += 1
                mb_inter += len(to_add) * p.partition_size
            elif between_disks:
                n_intra += len(between_disks)
                mb_intra += p.partition_size * len(between_disks)
            else:
                n_lead += 1
        return [n_inter, mb_inter, n_intra, mb_intra, n_lead]

    def proposal_summary_json(self) -> Dict[str, object]:
        """OptimizerResult.getProposalSummaryForJson (OptimizerResult.java:300-320)."""
        m = self.movement_stats()
        opts = getattr(self, "options", None) or OptimizationOptions()
        names = self._cluster.topic_names()
        prov = self.provision_response
        return {
            "numReplicaMovements": m[0], "dataToMoveMB": m[1], "numIntraBrokerReplicaMovements": m[2],
            "intraBrokerDataToMoveMB": m[3], "numLeaderMovements": m[4],
            "recentWindows": self._cluster.desc.num_windows, "monitoredPartitionsPercentage": 100.0,
            "excludedTopics": sorted(names[t] for t in opts.excluded_topics),
            "excludedBrokersForLeadership": sorted(opts.excluded_brokers_for_leadership),
            "excludedBrokersForReplicaMove": sorted(opts.excluded_brokers_for_replica_move),
            "onDemandBalancednessScoreBefore": self.on_demand_balancedness_score_before,
            "onDemandBalancednessScoreAfter": self.on_demand_balancedness_score_after,
            "provisionStatus": prov.status, "provisionRecommendation": prov.recommendation(),
        }

    def proposals_json(self) -> List[Dict[str, object]]:
        """ExecutionProposal.getJsonStructure (ExecutionProposal.java:266-270) of every proposal."""
        names = self._cluster.topic_names()
        d = self._cluster.desc
        return [{"topicPartition": f"{names[d.partition_topic[p.partition]]}-{d.partition_number[p.partition]}",
                 "oldLeader": p.old_leader, "oldReplicas": list(p.old_replicas), "newReplicas": list(p.new_replicas)}
                for p in self.proposals]

    @property
    def provision_response(self) -> ProvisionResponse:
        """The aggregated provision response GoalOptimizer.optimizations reports (GoalOptimizer.java:456-496)."""
        agg = ProvisionResponse("UNDECIDED")
        for g in self.goal_results:
            if g.provision is not None:
                agg.aggregate(g.provision)
        return agg


def stats_to_dict(s: StatsStruct) -> Dict[str, object]:
    out = {}
    for name, typ in StatsStruct._fields_:
        v = getattr(s, name)
        out[name] = list(v) if hasattr(v, "__len__") else v
    return out


# ----------------------------------------------------------------------------------------------- cluster / session
class ClusterBuffers:
    """Owns a generated flattened cluster (RandomCluster fixture)."""

    def __init__(self, lib: Library, handle: int):
        self.lib = lib
        self.handle = C.c_void_p(handle)
        self.desc = lib.lib.ccmi_cluster_buffers_desc(self.handle).contents

    def __del__(self):
        try:
            self.lib.lib.ccmi_cluster_buffers_free(self.handle)
        except Exception:
            pass


class RandomCluster:
    """RandomCluster.generate + populate (RandomCluster.java:53-336) with TestConstants.BASE_PROPERTIES defaults."""

    BASE = dict(num_racks=10, num_brokers=40, num_dead_brokers=0, num_brokers_with_bad_disk=0, num_replicas=50001,
                num_topics=3000, min_replication=3, max_replication=3, mean_cpu=0.01, mean_disk=100.0,
                mean_nw_in=100.0, mean_nw_out=100.0, distribution=0, rack_aware=0, leader_in_first_position=1)

    @staticmethod
    def props(**overrides) -> RandomClusterProps:
        d = dict(RandomCluster.BASE)
        d.update(overrides)
        p = RandomClusterProps()
        for k, v in d.items():
            if k == "logdir_capacity":
                v = (C.c_double * 8)(*(list(v) + [0.0] * (8 - len(v))))
            setattr(p, k, v)
        return p

    @staticmethod
    def generate(lib: Optional[Library] = None, **overrides) -> ClusterBuffers:
        lib = lib or Library.get()
        h = C.c_void_p()
        lib.check(lib.lib.ccmi_random_cluster(C.byref(RandomCluster.props(**overrides)), C.byref(h)))
        return ClusterBuffers(lib, h.value)


METRIC_OF_RESOURCE = {"CPU": 0, "NW_IN": 2, "NW_OUT": 3, "DISK": 1}  # first metric id of each resource group
BROKER_STATES = {"ALIVE": 0, "DEAD": 1, "NEW": 2, "DEMOTED": 3, "BAD_DISKS": 4}
DISK_STATES = {"ALIVE": 0, "DEAD": 1, "DEMOTED": 2}


class ClusterModelBuilder:
    """Builds the flattened model (ccmi_cluster_desc) with the reference's ClusterModel construction API
    (model/ClusterModel.java: createRack :948, createBroker :923, createReplica :800-880, setReplicaLoad :738-760,
    setBrokerState :297-336) — the calls LoadMonitor.clusterModel and the test fixtures make. Construction order is
    kept: replicas are indexed in createReplica order, every Partition._replicas list is built by list insertion at
    the given index (Partition.addLeader/addFollower), and setReplicaLoad order becomes replica_load_order.

    Loads follow KafkaCruiseControlUnitTestUtils.getAggregatedMetricValues: the whole resource value goes to the
    first metric id of the resource group (KafkaCruiseControlUnitTestUtils.java:90-145). Broker ids must be 0..B-1.
    An optional rack-id mapper (AnalyzerConfig rack.aware.goal.rack.id.mapper.class) is applied here: racks that map
    to the same id become one rack index."""

    def __init__(self, num_windows: int = 1, rack_id_mapper=None):
        self.W = num_windows
        self.mapper = rack_id_mapper or (lambda r: r)
        self.rack_index: Dict[str, int] = {}
        self.brokers: Dict[int, tuple] = {}   # id -> (rack index, capacity[4])
        self.state: Dict[int, int] = {}
        self.topics: List[str] = []
        self.topic_index: Dict[str, int] = {}
        self.parts: Dict[tuple, int] = {}     # (topic, partition) -> partition index
        self.part_list: List[List[int]] = []  # Partition._replicas (replica indices)
        self.rep_part: List[int] = []
        self.rep_broker: List[int] = []
        self.rep_leader: List[int] = []
        self.rep_offline: List[int] = []
        self.rep_load: List[Optional[List[float]]] = []
        self.load_order: List[int] = []
        self.disks: List[tuple] = []          # (broker, logdir, capacity) in creation order
        self.disk_index: Dict[tuple, int] = {}
        self.disk_demoted: Dict[int, int] = {}
        self.rep_disk: List[int] = []
        self.host: Dict[int, str] = {}        # broker id -> host name (Rack._hosts key); absent = its own host

    def create_rack(self, rack_id: str) -> None:
        self.rack_index.setdefault(str(self.mapper(str(rack_id))), len(self.rack_index))

    def create_broker(self, rack_id: str, broker_id: int, capacity: Dict[str, float],
                      disk_capacity_by_logdir: Optional[Dict[str, float]] = None, host: Optional[str] = None) -> None:
        """createBroker with a BrokerCapacityInfo; disk_capacity_by_logdir populates the replica placement over
        disks (Broker.java:80-83; negative capacity = dead disk). `host` names the broker's host within its rack
        (Rack._hosts); brokers without one get a host of their own."""
        self.create_rack(rack_id)
        if host is not None:
            self.host[broker_id] = str(host)
        self.brokers[broker_id] = (self.rack_index[str(self.mapper(str(rack_id)))],
                                   [float(capacity[r]) for r in RESOURCES])
        for logdir, cap in (disk_capacity_by_logdir or {}).items():
            self.disk_index[(broker_id, logdir)] = len(self.disks)
            self.disks.append((broker_id, logdir, float(cap)))

    def _replica(self, broker_id: int, topic: str, partition: int) -> int:
        for r in self.part_list[self.parts[(topic, partition)]]:
            if self.rep_broker[r] == broker_id:
                return r
        raise IllegalArgumentException(f"no replica of {topic}-{partition} on broker {broker_id}")

    def create_replica(self, rack_id: str, broker_id: int, topic: str, partition: int, index: int, is_leader: bool,
                       is_offline: bool = False, logdir: Optional[str] = None) -> int:
        if topic not in self.topic_index:
            self.topic_index[topic] = len(self.topics)
            self.topics.append(topic)
        key = (topic, partition)
        if key not in self.parts:
            self.parts[key] = len(self.part_list)
            self.part_list.append([])
        r = len(self.rep_part)
        self.rep_part.append(self.parts[key])
        self.rep_broker.append(broker_id)
        self.rep_leader.append(1 if is_leader else 0)
        self.rep_offline.append(1 if is_offline else 0)
        self.rep_load.append(None)
        if logdir is not None and (broker_id, logdir) not in self.disk_index:
            raise IllegalStateException(f"Missing disk information for disk {logdir} on broker {broker_id}")
        self.rep_disk.append(self.disk_index[(broker_id, logdir)] if logdir is not None else -1)
        self.part_list[self.parts[key]].insert(index, r)
        return r

    def set_replica_load(self, rack_id: str, broker_id: int, topic: str, partition: int, cpu: float, nw_in: float,
                         nw_out: float, disk: float) -> None:
        r = self._replica(broker_id, topic, partition)
        if self.rep_load[r] is not None:
            raise IllegalStateException(f"The load for {topic}-{partition} on broker {broker_id} already has metric values.")
        load = [0.0] * 6
        for res, v in (("CPU", cpu), ("NW_IN", nw_in), ("NW_OUT", nw_out), ("DISK", disk)):
            load[METRIC_OF_RESOURCE[res]] = float(v)
        self.rep_load[r] = load
        self.load_order.append(r)

    def set_broker_state(self, broker_id: int, state: str) -> None:
        self.state[broker_id] = BROKER_STATES[state]

    def set_disk_state(self, broker_id: int, logdir: str, state: str) -> None:
        """Disk.setState: "DEMOTED" or "ALIVE" (DemoteBrokerRunnable.java:144-148)."""
        if (broker_id, logdir) not in self.disk_index:
            raise IllegalStateException(f"Broker {broker_id} does not have logdir {logdir}.")
        if state not in ("ALIVE", "DEMOTED"):
            raise IllegalArgumentException(f"unsupported disk state {state}")
        self.disk_demoted[self.disk_index[(broker_id, logdir)]] = 1 if state == "DEMOTED" else 0

    def build(self) -> "FlatCluster":
        return FlatCluster(self)


class FlatCluster:
    """Owner of the arrays behind a ClusterModelBuilder's desc (keep it alive while sessions use the desc)."""

    def __init__(self, bld: ClusterModelBuilder):
        B = len(bld.brokers)
        if sorted(bld.brokers) != list(range(B)):
            raise IllegalArgumentException("broker ids must be 0..B-1")
        R, P, T, W = len(bld.rep_part), len(bld.part_list), len(bld.topics), bld.W
        # a replica without setReplicaLoad keeps an empty Load (it is left out of replica_load_order)
        arr = lambda ct, xs: (ct * max(1, len(xs)))(*xs)  # noqa: E731
        self.keep = dict(
            broker_id=arr(C.c_int32, list(range(B))),
            broker_rack=arr(C.c_int32, [bld.brokers[b][0] for b in range(B)]),
            broker_state=arr(C.c_int32, [bld.state.get(b, 0) for b in range(B)]),
            broker_capacity=arr(C.c_double, [c for b in range(B) for c in bld.brokers[b][1]]),
            topic_names=arr(C.c_char_p, [t.encode() for t in bld.topics]),
            partition_topic=arr(C.c_int32, [0] * P), partition_number=arr(C.c_int32, [0] * P),
            partition_offset=arr(C.c_int32, [0] * (P + 1)),
            partition_replicas=arr(C.c_int32, [r for lst in bld.part_list for r in lst]),
            replica_partition=arr(C.c_int32, bld.rep_part), replica_broker=arr(C.c_int32, bld.rep_broker),
            replica_is_leader=arr(C.c_uint8, bld.rep_leader), replica_offline=arr(C.c_uint8, bld.rep_offline),
            replica_load=arr(C.c_float, [x for r in range(R) for x in (bld.rep_load[r] or [0.0] * 6) for _ in range(W)]),
            replica_load_order=arr(C.c_int32, bld.load_order))
        D = len(bld.disks)
        if D:
            self.keep.update(disk_broker=arr(C.c_int32, [x[0] for x in bld.disks]),
                             disk_logdir=arr(C.c_char_p, [x[1].encode() for x in bld.disks]),
                             disk_capacity=arr(C.c_double, [x[2] for x in bld.disks]),
                             replica_disk=arr(C.c_int32, bld.rep_disk),
                             disk_demoted=arr(C.c_uint8, [bld.disk_demoted.get(k, 0) for k in range(D)]))
        if bld.host:  # one host per (rack, name); a broker without a name is alone on its host
            index: Dict[tuple, int] = {}
            hosts = []
            for b in range(B):
                key = (bld.brokers[b][0], bld.host[b]) if b in bld.host else ("own", b)
                hosts.append(index.setdefault(key, len(index)))
            self.keep["broker_host"] = arr(C.c_int32, hosts)
        for (topic, num), p in bld.parts.items():
            self.keep["partition_topic"][p] = bld.topic_index[topic]
            self.keep["partition_number"][p] = num
        off = 0
        for p, lst in enumerate(bld.part_list):
            self.keep["partition_offset"][p] = off
            off += len(lst)
        self.keep["partition_offset"][P] = off
        d = ClusterDesc()
        d.num_windows, d.num_racks, d.num_brokers = W, len(bld.rack_index), B
        d.num_topics, d.num_partitions, d.num_replicas = T, P, R
        d.num_disks = D
        d.num_replica_loads = len(bld.load_order)
        for k, v in self.keep.items():
            setattr(d, k, C.cast(v, type(getattr(d, k))) if k not in ("topic_names", "disk_logdir") else v)
        self.desc = d
        self.topics = list(bld.topics)
        self.partitions = {p: key for key, p in bld.parts.items()}


class LoadMonitorModel:
    """Model ingestion through the native builder (ccmi_builder_*): the calls LoadMonitor.clusterModel makes
    (monitor/LoadMonitor.java:491-543) — createRack/createBroker for every live node, handleDeadBroker for the brokers
    only partitions name, MonitorUtils.populatePartitionLoad per partition with its aggregated leader metrics, and
    setBadBrokerState — produce the flattened model directly. Replica loads are derived natively
    (getAggregatedMetricValues: CPU to percentage, replication bytes out, follower NW_OUT / CPU).

        m = LoadMonitorModel(num_windows=2)
        m.create_broker("r0", "h0", 0, {"CPU": 100, "NW_IN": 1e5, "NW_OUT": 1e5, "DISK": 1e6})
        m.populate_partition("T0", 0, replicas=[0, 1], leader=0, metrics={"CPU_USAGE": [0.115, 0.015], ...})
        cm = ClusterModel(m.desc(), keepalive=m)
    """

    METRICS = ("CPU_USAGE", "DISK_USAGE", "LEADER_BYTES_IN", "LEADER_BYTES_OUT", "REPLICATION_BYTES_IN_RATE",
               "REPLICATION_BYTES_OUT_RATE")

    def __init__(self, num_windows: int = 1, lib: Optional[Library] = None):
        self.lib = lib or Library.get()
        self.W = num_windows
        h = C.c_void_p()
        self.lib.check(self.lib.lib.ccmi_builder_create(num_windows, C.byref(h)))
        self.handle = h
        self._desc = None

    def __del__(self):
        try:
            self.lib.lib.ccmi_builder_destroy(self.handle)
        except Exception:
            pass

    def create_broker(self, rack: str, host: str, broker_id: int, capacity: Dict[str, float],
                      alive: bool = True, disk_capacity_by_logdir: Optional[Dict[str, float]] = None) -> None:
        cap = (C.c_double * 4)(*[float(capacity[r]) for r in RESOURCES])
        self.lib.check(self.lib.lib.ccmi_builder_create_broker(self.handle, rack.encode(), host.encode(), broker_id,
                                                               cap, 1 if alive else 0))
        for logdir, c in (disk_capacity_by_logdir or {}).items():
            self.lib.check(self.lib.lib.ccmi_builder_add_disk(self.handle, broker_id, logdir.encode(), float(c)))

    def populate_partition(self, topic: str, partition: int, replicas: Sequence[int], leader: Optional[int],
                           metrics: Dict[str, Sequence[float]], offline: Sequence[int] = (),
                           logdirs: Optional[Sequence[Optional[str]]] = None) -> None:
        """metrics: aggregated leader values per metric name, newest window first (missing metrics are 0)."""
        n = len(replicas)
        vals = []
        for m in self.METRICS:
            w = list(metrics.get(m, [0.0] * self.W))
            if len(w) != self.W:
                raise IllegalArgumentException(f"{m}: {len(w)} windows, expected {self.W}")
            vals += [float(x) for x in w]
        off = (C.c_uint8 * n)(*[1 if b in set(offline) else 0 for b in replicas])
        ld = (C.c_char_p * n)(*[(x.encode() if x else None) for x in logdirs]) if logdirs else None
        self.lib.check(self.lib.lib.ccmi_builder_populate_partition(
            self.handle, topic.encode(), partition, (C.c_int32 * n)(*replicas), n,
            -1 if leader is None else leader, off, ld, (C.c_float * len(vals))(*vals)))
        self._desc = None

    def set_broker_state(self, broker_id: int, state: str) -> None:
        self.lib.check(self.lib.lib.ccmi_builder_set_broker_state(self.handle, broker_id, BROKER_STATES[state]))
        self._desc = None

    def set_disk_state(self, broker_id: int, logdir: str, state: str) -> None:
        """Disk.setState (DemoteBrokerRunnable.java:144-148): "ALIVE" or "DEMOTED"."""
        self.lib.check(self.lib.lib.ccmi_builder_set_disk_state(self.handle, broker_id, logdir.encode(),
                                                                DISK_STATES[state]))
        self._desc = None

    def desc(self) -> ClusterDesc:
        if self._desc is None:
            d = ClusterDesc()
            self.lib.check(self.lib.lib.ccmi_builder_desc(self.handle, C.byref(d)))
            self._desc = d
        return self._desc

    def broker_ids(self) -> List[int]:
        """Kafka broker id of every dense broker index of desc()."""
        d = self.desc()
        out = (C.c_int32 * d.num_brokers)()
        self.lib.check(self.lib.lib.ccmi_builder_broker_ids(self.handle, out))
        return list(out)

    def replica_loads(self) -> List[List[List[float]]]:
        """[replica][metric][window] of the flattened model (the values setReplicaLoad received)."""
        d = self.desc()
        W = d.num_windows
        return [[[d.replica_load[(r * 6 + m) * W + w] for w in range(W)] for m in range(6)]
                for r in range(d.num_replicas)]


class ClusterModel:
    """A device-resident model session (ccmi_session)."""

    def __init__(self, desc: ClusterDesc, device: int = 0, lib: Optional[Library] = None, keepalive=None):
        self.lib = lib or Library.get()
        self._keep = keepalive
        self.desc = desc
        h = C.c_void_p()
        self.lib.check(self.lib.lib.ccmi_session_create(device, C.byref(desc), C.byref(h)))
        self.handle = h
        self.num_partitions = desc.num_partitions
        self.num_replicas = desc.num_replicas

    def topic_names(self) -> List[str]:
        return [self.desc.topic_names[t].decode() for t in range(self.desc.num_topics)]

    def broker_ids(self) -> List[int]:
        """Kafka broker id of every broker index: the LoadMonitorModel's id table when the desc came from one
        (ccmi_builder_broker_ids), else the desc's broker_id."""
        if hasattr(self._keep, "broker_ids"):
            return list(self._keep.broker_ids())
        return [self.desc.broker_id[b] for b in range(self.desc.num_brokers)]

    @staticmethod
    def from_buffers(buf: ClusterBuffers, device: int = 0) -> "ClusterModel":
        return ClusterModel(buf.desc, device=device, lib=buf.lib, keepalive=buf)

    def close(self) -> None:
        if self.handle:
            self.lib.lib.ccmi_session_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _goal_optimize(self, goal: Goal, optimized_goals: Iterable[Goal],
                       options: Optional[OptimizationOptions]) -> GoalResultStruct:
        res = GoalResultStruct()
        o, keep = (options or OptimizationOptions()).to_struct()
        c = (goal.constraint or BalancingConstraint()).to_struct(self.topic_names(), self.broker_ids())
        prior = [g.kind if isinstance(g, Goal) else int(g) for g in optimized_goals]
        kinds = (C.c_int32 * max(1, len(prior)))(*prior)
        self._checked(self.lib.lib.ccmi_goal_optimize(self.handle, goal.kind, kinds, len(prior), C.byref(c),
                                                      C.byref(o), C.byref(res)))
        goal.provision = ProvisionResponse.from_struct(res.provision, goal.name())
        return res

    def _checked(self, status: int) -> None:
        """lib.check, attaching the failed goal's provision response to an OptimizationFailureException."""
        try:
            self.lib.check(status)
        except OptimizationFailureException as e:
            e.provision = self.last_failure_provision(_goal_of_message(str(e)))
            raise

    def last_failure_provision(self, recommender: str = "") -> ProvisionResponse:
        out = ProvisionRespStruct()
        self.lib.check(self.lib.lib.ccmi_last_failure_provision(self.handle, C.byref(out)))
        return ProvisionResponse.from_struct(out, recommender)

    def action_acceptance(self, optimized_goal_index: int, action_type: int, partition: int, source: int,
                          destination: int, destination_partition: int = -1, source_disk: int = -1,
                          destination_disk: int = -1) -> str:
        a = ActionStruct(action_type, partition, source, destination, destination_partition, source_disk,
                         destination_disk)
        out = C.c_int32()
        self.lib.check(self.lib.lib.ccmi_action_acceptance(self.handle, optimized_goal_index, C.byref(a),
                                                           C.byref(out)))
        return ACCEPTANCE[out.value]

    def action_acceptance_by_goal(self, goal_name: str, action_type: int, partition: int, source: int,
                                  destination: int, destination_partition: int = -1, source_disk: int = -1,
                                  destination_disk: int = -1) -> str:
        """Goal.actionAcceptance of the optimized goal with this name (ccmi_action_acceptance_by_kind)."""
        a = ActionStruct(action_type, partition, source, destination, destination_partition, source_disk,
                         destination_disk)
        out = C.c_int32()
        self.lib.check(self.lib.lib.ccmi_action_acceptance_by_kind(self.handle, GOAL_KINDS[goal_name], C.byref(a),
                                                                   C.byref(out)))
        return ACCEPTANCE[out.value]

    def apply(self, actions) -> int:
        """Apply actions decided elsewhere (tuples in the action-log layout: type, partition, source,
        destination, destination partition, source disk, destination disk) to the resident model
        (ccmi_session_apply). Returns the number applied; raises on the first invalid one."""
        acts = list(actions)
        arr = (ActionStruct * max(1, len(acts)))(*[ActionStruct(*a) for a in acts])
        done = C.c_int64()
        self.lib.check(self.lib.lib.ccmi_session_apply(self.handle, arr, len(acts), C.byref(done)))
        return done.value

    def cluster_stats(self, constraint: Optional[BalancingConstraint] = None,
                      options: Optional[OptimizationOptions] = None) -> Dict[str, object]:
        s = StatsStruct()
        o, keep = (options or OptimizationOptions()).to_struct()
        c = (constraint or BalancingConstraint()).to_struct(self.topic_names(), self.broker_ids())
        self.lib.check(self.lib.lib.ccmi_compute_cluster_stats(self.handle, C.byref(c), C.byref(o), C.byref(s)))
        return stats_to_dict(s)

    def actions(self) -> List[tuple]:
        n = self.lib.lib.ccmi_action_log_count(self.handle)
        buf = (ActionStruct * max(1, n))()
        if n:
            self.lib.check(self.lib.lib.ccmi_action_log_copy(self.handle, 0, n, buf))
        return [(a.type, a.partition, a.source_broker, a.destination_broker, a.destination_partition,
                 a.source_disk, a.destination_disk) for a in buf[:n]]

    def replica_distribution(self) -> List[int]:
        out = (C.c_int32 * self.num_replicas)()
        self.lib.check(self.lib.lib.ccmi_replica_distribution(self.handle, out))
        return list(out)

    def replica_disks(self) -> List[int]:
        """Disk index of every replica slot in partition order (the logdir of getReplicaDistribution)."""
        out = (C.c_int32 * self.num_replicas)()
        self.lib.check(self.lib.lib.ccmi_replica_disks(self.handle, out))
        return list(out)

    def leader_distribution(self) -> List[int]:
        out = (C.c_int32 * self.num_partitions)()
        self.lib.check(self.lib.lib.ccmi_leader_distribution(self.handle, out))
        return list(out)

    def proposals(self, max_rf: int = 8) -> List[ExecutionProposal]:
        n = self.lib.lib.ccmi_proposal_count(self.handle)
        if n == 0:
            return []
        part = (C.c_int32 * n)()
        size = (C.c_int32 * n)()
        old_leader = (C.c_int32 * n)()
        old_r = (C.c_int32 * (n * max_rf))()
        new_r = (C.c_int32 * (n * max_rf))()
        self.lib.check(self.lib.lib.ccmi_proposals(self.handle, max_rf, part, size, old_leader, old_r, new_r))
        old_d = (C.c_int32 * (n * max_rf))()
        new_d = (C.c_int32 * (n * max_rf))()
        self.lib.check(self.lib.lib.ccmi_proposal_disks(self.handle, max_rf, old_d, new_d))
        out = []
        for i in range(n):
            rf = sum(1 for x in old_r[i * max_rf:(i + 1) * max_rf] if x >= 0)
            sl = slice(i * max_rf, i * max_rf + rf)
            out.append(ExecutionProposal(part[i], size[i], old_leader[i], list(old_r[sl]), list(new_r[sl]),
                                         list(old_d[sl]), list(new_d[sl])))
        return out

    def perf(self) -> PerfStruct:
        p = PerfStruct()
        self.lib.check(self.lib.lib.ccmi_perf(self.handle, C.byref(p)))
        return p

    def reset_perf(self) -> None:
        self.lib.lib.ccmi_perf_reset(self.handle)

    def set_kernel_timing(self, enabled: bool) -> None:
        self.lib.lib.ccmi_set_kernel_timing(self.handle, int(enabled))

    def set_shard(self, rank: int, count: int, combine_min) -> None:
        """Destination-sharded mode with a caller-supplied combiner: combine_min(local_key:int) -> global min key
        (None / -1 for no candidate on this shard). Used with torch.distributed gloo in the CPU tests."""
        none = (1 << 63) - 1

        def _fn(_ctx, key_ptr):
            try:
                k = key_ptr[0]
                key_ptr[0] = int(combine_min(k if k != none else none))
                return 0
            except Exception:  # noqa: BLE001 - reported as a failed combine by the engine
                return 1

        self._combine_cb = AllreduceMinFn(_fn)  # keep the trampoline alive with the session
        self.lib.check(self.lib.lib.ccmi_session_set_shard(self.handle, rank, count, self._combine_cb, None))

    def attach_rccl(self, rank: int, count: int, unique_id: bytes) -> None:
        """Destination-sharded mode over the built-in RCCL combiner (one int64 MIN allreduce per scan)."""
        buf = (C.c_uint8 * 128).from_buffer_copy(unique_id)
        self.lib.check(self.lib.lib.ccmi_session_attach_rccl(self.handle, rank, count, buf))

    def attach_shm(self, rank: int, count: int, name: str, job_nonce: int = 0, timeout_s: float = 0.0) -> None:
        """Destination-sharded mode over the built-in host shared-memory combiner (ranks on one node): one int64 MIN
        per scan in a POSIX shared-memory block; the scan server stays on. `job_nonce` (the same nonzero value on
        every rank, ccmi_session_attach_shm_job, ABI v12): the other ranks refuse a block rank 0 of this job did not
        stamp with it, however recent; `timeout_s` bounds the waits (0 = 120 s)."""
        if job_nonce or timeout_s:
            self.lib.check(self.lib.lib.ccmi_session_attach_shm_job(self.handle, rank, count, name.encode(),
                                                                    job_nonce & (2 ** 64 - 1), float(timeout_s)))
        else:
            self.lib.check(self.lib.lib.ccmi_session_attach_shm(self.handle, rank, count, name.encode()))

    def attach_group(self, group: "ShardGroup", rank: int) -> None:
        """Rank `rank` of a one-process shard group (ShardGroup): the scan server combines the ranks' keys on the
        device; this session's optimizations must run on a thread of its own, concurrently with the other ranks'."""
        self.lib.check(self.lib.lib.ccmi_session_attach_group(self.handle, group.handle, rank))
        self._group = group  # the group outlives the session


class ShardGroup:
    """The ranks of one destination-sharded proposal driven from ONE process (ccmi_shard_group_*, ABI v11): one
    session per rank (typically one per GPU), each optimized on its own host thread; a scan the session's scan server
    ran is MIN-combined with the other ranks' on the device, through pinned host memory every GPU maps. Keep the group
    alive while its sessions are."""

    def __init__(self, count: int, lib: Optional["Library"] = None):
        self.lib = lib or Library.get()
        h = C.c_void_p()
        self.lib.check(self.lib.lib.ccmi_shard_group_create(count, C.byref(h)))
        self.handle = h
        self.count = count

    def __del__(self):
        if getattr(self, "handle", None):
            self.lib.lib.ccmi_shard_group_destroy(self.handle)
            self.handle = None


def rccl_unique_id(lib: Optional["Library"] = None) -> bytes:
    """ncclGetUniqueId through libccmi (rank 0 broadcasts it to the other ranks)."""
    lib = lib or Library.get()
    buf = (C.c_uint8 * 128)()
    lib.check(lib.lib.ccmi_rccl_unique_id(buf))
    return bytes(buf)


class GoalOptimizer:
    """GoalOptimizer.optimizations (GoalOptimizer.java:435-524) on a device session. priority_weight /
    strictness_weight: goal.balancedness.priority.weight / goal.balancedness.strictness.weight (AnalyzerConfig.java:
    374-385) for the on-demand balancedness score."""

    def __init__(self, constraint: Optional[BalancingConstraint] = None, priority_weight: float = 1.1,
                 strictness_weight: float = 1.5):
        self.constraint = constraint or BalancingConstraint()
        self.priority_weight = priority_weight
        self.strictness_weight = strictness_weight

    def optimizations(self, cluster: ClusterModel, goals_by_priority: Sequence[Goal],
                      options: Optional[OptimizationOptions] = None) -> OptimizerResult:
        if not goals_by_priority:
            raise IllegalArgumentException("At least one goal must be provided to get an optimization result.")
        kinds = (C.c_int32 * len(goals_by_priority))(*[g.kind for g in goals_by_priority])
        results = (GoalResultStruct * len(goals_by_priority))()
        o, keep = (options or OptimizationOptions()).to_struct()
        c = self.constraint.to_struct(cluster.topic_names(), cluster.broker_ids())
        import time
        t0 = time.perf_counter()
        cluster._checked(cluster.lib.lib.ccmi_optimizations(cluster.handle, kinds, len(goals_by_priority),
                                                            C.byref(c), C.byref(o), results))
        dt = time.perf_counter() - t0
        grs = [GoalResult(GOAL_NAMES[r.goal_kind], bool(r.succeeded), bool(r.has_diff), r.seconds, r.candidates,
                          r.device_candidates, r.device_launches, r.actions, stats_to_dict(r.stats),
                          ProvisionResponse.from_struct(r.provision, GOAL_NAMES[r.goal_kind])) for r in results]
        res = OptimizerResult(grs, cluster, dt, [g.name for g in grs if not g.succeeded])
        res.options = options or OptimizationOptions()
        res.balancedness_cost_by_goal = balancedness_cost_by_goal(goals_by_priority, self.priority_weight,
                                                                  self.strictness_weight)
        return res


MAX_BALANCEDNESS_SCORE = 100.0  # KafkaCruiseControlUtils.MAX_BALANCEDNESS_SCORE
BALANCEDNESS_SCORE_WITH_OFFLINE_REPLICAS = -1.0  # GoalViolationDetector.java:69


@dataclass
class GoalViolations:
    """detector/GoalViolations: the violated detection goals by fixability, the aggregated provision response and
    the balancedness score GoalViolationDetector.run() leaves behind."""
    fixable: List[str]
    unfixable: List[str]
    provision_response: "ProvisionResponse"
    balancedness_score: float
    skipped_due_to_offline_replicas: bool = False
    seconds: float = 0.0


class GoalViolationDetector:
    """GoalViolationDetector.run (detector/GoalViolationDetector.java:176-332) as a what-if batch.

    Each detection goal is optimized on its own, without optimized goals, with OptimizationOptions
    (excluded topics / brokers, isTriggeredByGoalViolation = true; DefaultOptimizationOptionsGenerator.java:17-25):
    an OptimizationFailureException makes it an unfixable violation, a diff a fixable one. The reference reuses the
    model only after a goal that changed nothing, so every goal sees the initial model: the goals are independent and
    run as concurrent device sessions (one host thread and HIP stream each, `max_concurrency` at a time) instead of
    one after the other. A model with dead brokers or broken disks is skipped (skipDueToOfflineReplicas :259-273)."""

    def __init__(self, detection_goals: Sequence[str], constraint: Optional[BalancingConstraint] = None,
                 priority_weight: float = 1.1, strictness_weight: float = 1.5, lib: Optional[Library] = None,
                 device: Optional[int] = None, max_concurrency: int = 8, devices: Optional[Sequence[int]] = None):
        self.goals = list(detection_goals)
        self.constraint = constraint or BalancingConstraint()
        self.cost = balancedness_cost_by_goal(goals_from_names(self.goals), priority_weight, strictness_weight)
        self.lib = lib or Library.get()
        # the sessions go round-robin over `devices` (default: every visible gfx950; `device` pins them to one)
        if devices is None:
            devices = [device] if device is not None else list(range(max(1, self.lib.device_count())))
        self.devices = list(devices)
        self.max_concurrency = max_concurrency

    def detect(self, desc: ClusterDesc, keepalive=None, excluded_topics: Sequence[int] = (),
               excluded_brokers_for_leadership: Sequence[int] = (),
               excluded_brokers_for_replica_move: Sequence[int] = ()) -> GoalViolations:
        import time
        from concurrent.futures import ThreadPoolExecutor
        t0 = time.perf_counter()
        states = [desc.broker_state[b] for b in range(desc.num_brokers)]
        if BROKER_STATES["DEAD"] in states or BROKER_STATES["BAD_DISKS"] in states:
            return GoalViolations([], [], ProvisionResponse("UNDECIDED"), BALANCEDNESS_SCORE_WITH_OFFLINE_REPLICAS, True,
                                  time.perf_counter() - t0)
        opts = OptimizationOptions(excluded_topics=list(excluded_topics),
                                   excluded_brokers_for_leadership=list(excluded_brokers_for_leadership),
                                   excluded_brokers_for_replica_move=list(excluded_brokers_for_replica_move),
                                   is_triggered_by_goal_violation=True)

        def one(i_name):  # GoalViolationDetector.optimizeForGoal (:296-331)
            i, name = i_name
            cm = ClusterModel(desc, device=self.devices[i % len(self.devices)], lib=self.lib, keepalive=keepalive)
            goal = goals_from_names([name], self.constraint)[0]
            try:
                goal.optimize(cm, set(), opts)
            except OptimizationFailureException as e:
                return name, "unfixable", e.provision
            diff = cm.proposals()
            return name, ("fixable" if diff else None), goal.provision

        with ThreadPoolExecutor(max(1, min(self.max_concurrency, len(self.goals)))) as pool:
            outcomes = list(pool.map(one, enumerate(self.goals)))
        fixable = [n for n, v, _ in outcomes if v == "fixable"]
        unfixable = [n for n, v, _ in outcomes if v == "unfixable"]
        prov = ProvisionResponse("UNDECIDED")
        for _, _, p in outcomes:
            if p is not None:
                prov.aggregate(p)
        score = MAX_BALANCEDNESS_SCORE - sum(self.cost[n] for n in fixable + unfixable)  # refreshBalancednessScore
        return GoalViolations(fixable, unfixable, prov, score, False, time.perf_counter() - t0)


def balancedness_cost_by_goal(goals: Sequence[Goal], priority_weight: float = 1.1,
                              strictness_weight: float = 1.5) -> Dict[str, float]:
    """KafkaCruiseControlUtils.balancednessCostByGoal (KafkaCruiseControlUtils.java:844-870)."""
    if not goals:
        raise IllegalArgumentException("At least one goal must be provided to get the balancedness cost.")
    if priority_weight <= 0 or strictness_weight <= 0:
        raise IllegalArgumentException(f"Balancedness weights must be positive (priority:{priority_weight:f}, "
                                       f"strictness:{strictness_weight:f}).")
    cost: Dict[str, float] = {}
    weight_sum = 0.0
    previous = 1 / priority_weight
    for g in reversed(list(goals)):
        current = priority_weight * previous
        c = current * (strictness_weight if g.is_hard_goal() else 1)
        weight_sum += c
        cost[g.name()] = c
        previous = current
    return {k: MAX_BALANCEDNESS_SCORE * v / weight_sum for k, v in cost.items()}


def goals_from_names(names: Sequence[str], constraint: Optional[BalancingConstraint] = None) -> List[Goal]:
    return [globals()[n](constraint=constraint) for n in names]
