/*
 * ccmi.h — C ABI of the MI355X proposal engine (libccmi.so).
 *
 * Drop-in boundary for Cruise Control's goal-optimizer hot path. Every entry point replaces a
 * reference interface (paths relative to cruise-control/src/main/java/com/linkedin/kafka/cruisecontrol/):
 *
 *   ccmi_session_create        <- the ClusterModel a caller hands to GoalOptimizer.optimizations
 *                                 (model/ClusterModel.java:135-139 createRack/createBroker/createReplica/
 *                                 setReplicaLoad, :395-446); the desc is the flattened model.
 *   ccmi_optimizations         <- GoalOptimizer.optimizations(ClusterModel, List<Goal>, OperationProgress,
 *                                 Map, OptimizationOptions)  analyzer/GoalOptimizer.java:435-524
 *   ccmi_goal_optimize         <- Goal.optimize(ClusterModel, Set<Goal>, OptimizationOptions)
 *                                 analyzer/goals/Goal.java:60-66, AbstractGoal.java:81-135
 *   ccmi_action_acceptance     <- Goal.actionAcceptance(BalancingAction, ClusterModel)
 *                                 analyzer/goals/Goal.java:68-80
 *   ccmi_compute_cluster_stats <- ClusterModel.getClusterStats(BalancingConstraint, OptimizationOptions)
 *                                 model/ClusterModel.java:137-139 -> ClusterModelStats.populate :84-102
 *   ccmi_action_log_*          <- the ordered relocateReplica/relocateLeadership calls a goal makes
 *                                 (model/ClusterModel.java:380-441); a Java shim replays them so the
 *                                 caller's ClusterModel ends in the identical state.
 *   ccmi_replica_distribution / ccmi_leader_distribution
 *                              <- ClusterModel.getReplicaDistribution / getLeaderDistribution :167-198
 *   ccmi_proposals             <- AnalyzerUtils.getDiff -> Set<ExecutionProposal>  analyzer/AnalyzerUtils.java:55-93
 *   ccmi_random_cluster        <- test fixture RandomCluster.generate+populate
 *                                 (src/test/java/.../model/RandomCluster.java:53-455)
 *
 * Plain C: pointers + sizes only. All arrays are caller-owned for inputs and copied in.
 * Errors: every call returns ccmi_status; the last error text is available from ccmi_last_error().
 * Threading: a session is single-threaded; the library is thread-safe across sessions.
 */
#ifndef CCMI_H_
#define CCMI_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CCMI_ABI_VERSION 12

typedef enum ccmi_status {
  CCMI_OK = 0,
  CCMI_E_INVALID = 1,     /* IllegalArgumentException */
  CCMI_E_DEVICE = 2,      /* HIP runtime / device failure, or no gfx950 device */
  CCMI_E_OPT_FAILURE = 3, /* OptimizationFailureException */
  CCMI_E_STATE = 4,       /* IllegalStateException (e.g. stats regression check, AbstractGoal.java:114-117) */
  CCMI_E_UNSUPPORTED = 5  /* goal kind / option outside the implemented scope */
} ccmi_status;

/* common/Resource.java:17-25 ids */
typedef enum ccmi_resource { CCMI_CPU = 0, CCMI_NW_IN = 1, CCMI_NW_OUT = 2, CCMI_DISK = 3, CCMI_NUM_RESOURCES = 4 } ccmi_resource;

/* KafkaMetricDef COMMON metrics that carry a resource group (monitor/metricdefinition/KafkaMetricDef.java:43-53) */
typedef enum ccmi_metric {
  CCMI_M_CPU_USAGE = 0,
  CCMI_M_DISK_USAGE = 1,
  CCMI_M_LEADER_BYTES_IN = 2,
  CCMI_M_LEADER_BYTES_OUT = 3,
  CCMI_M_REPLICATION_BYTES_IN = 4,
  CCMI_M_REPLICATION_BYTES_OUT = 5,
  CCMI_NUM_METRICS = 6
} ccmi_metric;

/* model/Broker.java State */
typedef enum ccmi_broker_state {
  CCMI_BROKER_ALIVE = 0,
  CCMI_BROKER_DEAD = 1,
  CCMI_BROKER_NEW = 2,
  CCMI_BROKER_DEMOTED = 3,
  CCMI_BROKER_BAD_DISKS = 4
} ccmi_broker_state;

/* model/Disk.java State (ALIVE, DEAD, DEMOTED) */
typedef enum ccmi_disk_state { CCMI_DISK_ALIVE = 0, CCMI_DISK_DEAD = 1, CCMI_DISK_DEMOTED = 2 } ccmi_disk_state;

/* analyzer/ActionType.java */
typedef enum ccmi_action_type {
  CCMI_INTER_BROKER_REPLICA_MOVEMENT = 0,
  CCMI_LEADERSHIP_MOVEMENT = 1,
  CCMI_INTER_BROKER_REPLICA_SWAP = 2,
  CCMI_INTRA_BROKER_REPLICA_MOVEMENT = 3,
  CCMI_INTRA_BROKER_REPLICA_SWAP = 4
} ccmi_action_type;

/* analyzer/ActionAcceptance.java */
typedef enum ccmi_acceptance { CCMI_ACCEPT = 0, CCMI_REPLICA_REJECT = 1, CCMI_BROKER_REJECT = 2 } ccmi_acceptance;

/* Goal plugins by reference simple class name (Goal.name(), AbstractGoal.java:141-144); numbering follows
 * the default.goals priority order (config/constants/AnalyzerConfig.java:352-367). */
typedef enum ccmi_goal_kind {
  CCMI_GOAL_RACK_AWARE = 0,                        /* RackAwareGoal */
  CCMI_GOAL_MIN_TOPIC_LEADERS_PER_BROKER = 1,      /* MinTopicLeadersPerBrokerGoal */
  CCMI_GOAL_REPLICA_CAPACITY = 2,                  /* ReplicaCapacityGoal */
  CCMI_GOAL_DISK_CAPACITY = 3,                     /* DiskCapacityGoal */
  CCMI_GOAL_NW_IN_CAPACITY = 4,                    /* NetworkInboundCapacityGoal */
  CCMI_GOAL_NW_OUT_CAPACITY = 5,                   /* NetworkOutboundCapacityGoal */
  CCMI_GOAL_CPU_CAPACITY = 6,                      /* CpuCapacityGoal */
  CCMI_GOAL_REPLICA_DISTRIBUTION = 7,              /* ReplicaDistributionGoal */
  CCMI_GOAL_POTENTIAL_NW_OUT = 8,                  /* PotentialNwOutGoal */
  CCMI_GOAL_DISK_USAGE_DISTRIBUTION = 9,           /* DiskUsageDistributionGoal */
  CCMI_GOAL_NW_IN_USAGE_DISTRIBUTION = 10,         /* NetworkInboundUsageDistributionGoal */
  CCMI_GOAL_NW_OUT_USAGE_DISTRIBUTION = 11,        /* NetworkOutboundUsageDistributionGoal */
  CCMI_GOAL_CPU_USAGE_DISTRIBUTION = 12,           /* CpuUsageDistributionGoal */
  CCMI_GOAL_TOPIC_REPLICA_DISTRIBUTION = 13,       /* TopicReplicaDistributionGoal */
  CCMI_GOAL_LEADER_REPLICA_DISTRIBUTION = 14,      /* LeaderReplicaDistributionGoal */
  CCMI_GOAL_LEADER_BYTES_IN_DISTRIBUTION = 15,     /* LeaderBytesInDistributionGoal */
  CCMI_GOAL_INTRA_BROKER_DISK_CAPACITY = 16,       /* IntraBrokerDiskCapacityGoal */
  CCMI_GOAL_INTRA_BROKER_DISK_USAGE_DISTRIBUTION = 17, /* IntraBrokerDiskUsageDistributionGoal */
  CCMI_GOAL_PREFERRED_LEADER_ELECTION = 18,         /* PreferredLeaderElectionGoal (not in default.goals) */
  CCMI_GOAL_RACK_AWARE_DISTRIBUTION = 19,           /* RackAwareDistributionGoal (not in default.goals) */
  CCMI_GOAL_BROKER_SET_AWARE = 20,                  /* BrokerSetAwareGoal (not in default.goals) */
  CCMI_GOAL_TOPIC_LEADER_REPLICA_DISTRIBUTION = 21, /* TopicLeaderReplicaDistributionGoal (ABI v7; in goals, not in
                                                       default.goals: AnalyzerConfig.java:297-319) */
  CCMI_GOAL_KAFKA_ASSIGNER_EVEN_RACK_AWARE = 22,     /* KafkaAssignerEvenRackAwareGoal (ABI v7; in goals) */
  CCMI_GOAL_KAFKA_ASSIGNER_DISK_USAGE_DISTRIBUTION = 23 /* KafkaAssignerDiskUsageDistributionGoal (ABI v7; in goals) */
} ccmi_goal_kind;

/* AnalyzerConfig replica.to.broker.set.mapping.policy.class (config/ReplicaToBrokerSetMappingPolicy.java) */
typedef enum ccmi_broker_set_policy {
  CCMI_BROKER_SET_TOPIC_NAME_HASH = 0,  /* TopicNameHashBrokerSetMappingPolicy (the default) */
  CCMI_BROKER_SET_ORIGINAL_BROKER = 1   /* ReplicaToOriginalBrokerSetMappingPolicy */
} ccmi_broker_set_policy;

/*
 * Flattened ClusterModel. Semantics of construction (mirrors the reference's model building):
 *   brokers are created in index order (broker_id[b] == b in ABI v1), then for r = 0..R-1 in index order
 *   replica r is created on replica_broker[r] (ClusterModel.createReplica) and its load is set
 *   (ClusterModel.setReplicaLoad) — so broker/host/cluster/potential-leadership aggregates accumulate in
 *   replica index order exactly as the Java model does (or, with replica_load_order, all replicas are created
 *   first and the loads are set in that order); finally each partition's replica list is put in
 *   partition_offset CSR order and broker states other than ALIVE are applied in broker index order
 *   (ClusterModel.setBrokerState).
 */
typedef struct ccmi_cluster_desc {
  int32_t num_windows;               /* W, 1..5 (num.partition.metrics.windows) */
  int32_t num_racks;
  int32_t num_brokers;               /* B */
  const int32_t* broker_id;          /* [B] */
  const int32_t* broker_rack;        /* [B] rack index */
  const int32_t* broker_state;       /* [B] ccmi_broker_state */
  const double* broker_capacity;     /* [B*4] ccmi_resource order */
  int32_t num_topics;                /* T */
  const char* const* topic_names;    /* [T] ASCII topic names (Replica.compareTo tie-break) */
  int32_t num_partitions;            /* P */
  const int32_t* partition_topic;    /* [P] */
  const int32_t* partition_number;   /* [P] */
  const int32_t* partition_offset;   /* [P+1] CSR into a permutation of replicas (Partition._replicas order) */
  const int32_t* partition_replicas; /* [R] replica indices, grouped by partition via partition_offset */
  int32_t num_replicas;              /* R */
  const int32_t* replica_partition;  /* [R] */
  const int32_t* replica_broker;     /* [R] */
  const uint8_t* replica_is_leader;  /* [R] */
  const uint8_t* replica_offline;    /* [R] isOriginalOffline flag (replica on a broken disk) */
  const float* replica_load;         /* [R * 6 * W] float window values, ccmi_metric order, newest first */
  /* Optional [R] permutation (NULL = interleaved). When set, every replica is created first (index order) and
   * ClusterModel.setReplicaLoad is then called in this order — the construction order of hand-built models such as
   * DeterministicCluster.mediumClusterModel (DeterministicCluster.java:1836-1879), where it changes the float
   * rounding of the broker / potential-leadership aggregates. */
  const int32_t* replica_load_order;
  /* Replica placement over disks (JBOD; Broker._diskByLogdir, model/Broker.java:56,80-83, model/Disk.java).
   * num_disks = 0: no placement information (Replica.disk() == null everywhere). Otherwise disk d belongs to
   * broker disk_broker[d], is named disk_logdir[d] (a broker's disks iterate in logdir String order, the TreeMap)
   * and has disk_capacity[d] (negative = dead disk, Disk.java:58-66; a dead broker's disks are dead).
   * replica_disk[r] is the disk given to ClusterModel.createReplica (the replica's original disk, -1 = none); its
   * utilization accumulates when the replica's load is set (Disk.addReplicaLoad). After the model is built, the
   * disk_assign pairs replay Disk.addReplica(replica) in order — the test fixture's placement step
   * (RandomCluster.java:315-331) for replicas created without a disk (their original disk stays null). */
  int32_t num_disks;
  const int32_t* disk_broker;        /* [D] */
  const char* const* disk_logdir;    /* [D] */
  const double* disk_capacity;       /* [D] */
  const int32_t* replica_disk;       /* [R] or NULL (all -1) */
  int32_t num_disk_assignments;
  const int32_t* disk_assign_replica; /* [num_disk_assignments] */
  const int32_t* disk_assign_disk;    /* [num_disk_assignments] */
  /* ABI v5: entries of replica_load_order (0 = num_replicas). A replica the order omits never gets
   * ClusterModel.setReplicaLoad: its Load stays empty (model/Load.java isEmpty), as in hand-built fixtures such as
   * DeterministicCluster.minLeaderReplicaPerBrokerSatisfiable (DeterministicCluster.java:321-361). */
  int32_t num_replica_loads;
  /* ABI v6: the host of every broker ([B] host index in [0, B), or NULL = each broker on a host of its own). Hosts
   * belong to a rack and are keyed by name within it (Rack._hosts.computeIfAbsent, model/Rack.java:256-262;
   * LoadMonitor passes node.host(), LoadMonitor.java:602), so brokers sharing an index must share a rack. ABI v8: a
   * host keeps the reference's aggregates (model/Host.java): the load of its brokers' replicas, updated with every
   * replica and leadership move in the reference's order; its capacity, the sum of its brokers' capacities in broker
   * index order minus those of dead brokers (Host.capacityFor: -1 without an alive broker); its replica count. The
   * host resources (Resource.isHostResource: CPU, NW_IN, NW_OUT) are checked against them where the reference does:
   * CapacityGoal.java:230-239,284-366,389-408,455-475, ResourceDistributionGoal.java:880-927,982-1037,
   * ClusterModel.aliveBrokers{Under,Over}Threshold / sortedAliveBrokersUnderThreshold (:1049-1126) and
   * ClusterModelStats.java:297-303. */
  const int32_t* broker_host;
  /* ABI v6: [D] 1 = the disk is Disk.State.DEMOTED (DemoteBrokerRunnable.java:144-148), or NULL. Only
   * PreferredLeaderElectionGoal reads it (PreferredLeaderElectionGoal.java:114-124). */
  const uint8_t* disk_demoted;
} ccmi_cluster_desc;

/* analyzer/BalancingConstraint.java; defaults AnalyzerConfig.java:58-464 via ccmi_default_constraint */
typedef struct ccmi_balancing_constraint {
  double resource_balance_percentage[4];
  double capacity_threshold[4];
  double low_utilization_threshold[4];
  double replica_balance_percentage;
  double leader_replica_balance_percentage;
  double topic_replica_balance_percentage;
  int32_t topic_replica_balance_min_gap;
  int32_t topic_replica_balance_max_gap;
  double goal_violation_distribution_threshold_multiplier;
  int64_t max_replicas_per_broker;
  int64_t overprovisioned_max_replicas_per_broker;
  int32_t overprovisioned_min_brokers;
  int32_t overprovisioned_min_extra_racks;
  /* BrokerSetAwareGoal (ABI v4): BalancingConstraint.brokerSetResolver() — the broker set id -> broker ids data of
   * BrokerSetFileResolver (config/BrokerSetFileResolver.java:42-82), whose brokers missing from every set the engine
   * assigns as NoOpBrokerSetAssignmentPolicy does (to "unmapped", NoOpBrokerSetAssignmentPolicy.java:70-86) — and
   * BalancingConstraint.replicaToBrokerSetMappingPolicy(). num_broker_sets = 0: no broker set data (BrokerSetAwareGoal
   * then fails as a BrokerSetResolutionException would, CCMI_E_INVALID). Other goals ignore these fields. */
  int32_t num_broker_sets;
  int32_t broker_set_policy;              /* ccmi_broker_set_policy */
  const char* const* broker_set_names;    /* [num_broker_sets] brokerSetId */
  const int32_t* broker_set_offset;       /* [num_broker_sets + 1] CSR into broker_set_members */
  const int32_t* broker_set_members;      /* broker indices of the session, in [0, B): a Kafka id's position in
                                           * ccmi_builder_broker_ids (ascending Kafka ids); -1 (any id outside
                                           * [0, B)) = a broker the model does not hold, ignored */
  /* MinTopicLeadersPerBrokerGoal (ABI v5): the topics topics.with.min.leaders.per.broker matches — the caller's
   * Utils.getTopicNamesMatchedWithPattern(BalancingConstraint.topicsWithMinLeadersPerBrokerPattern(), topics)
   * (common/Utils.java:26-36, BalancingConstraint.java:92,275-277), as topic indices of the session's desc (0 topics =
   * the default empty pattern) — and min.topic.leaders.per.broker (BalancingConstraint.java:93,285-287; 0 = the
   * dynamic leaders / eligible brokers). BrokerSetAwareGoal reads the same topic set (BrokerSetAwareGoal.java:
   * 136-139,262). */
  const int32_t* min_leader_topics;
  int32_t num_min_leader_topics;
  int32_t min_topic_leaders_per_broker;
  /* TopicLeaderReplicaDistributionGoal (ABI v7): topic.leader.replica.count.balance.threshold (default 1.10),
   * topic.leader.replica.count.balance.min.gap (2) / .max.gap (10) and
   * topic.leader.replica.distribution.goal.balance.margin (0.9) (AnalyzerConfig.java:112-146,
   * BalancingConstraint.java:85-88,145-167). */
  double topic_leader_replica_balance_percentage;
  int32_t topic_leader_replica_balance_min_gap;
  int32_t topic_leader_replica_balance_max_gap;
  double topic_leader_replica_balance_margin;
} ccmi_balancing_constraint;

/* analyzer/OptimizationOptions.java (7-field form) */
typedef struct ccmi_opt_options {
  const int32_t* excluded_topics; /* topic indices (OptimizationOptions.excludedTopics; every goal's
                                     selectReplicasBasedOnExcludedTopics and excluded-topic checks) */
  int32_t num_excluded_topics;
  const int32_t* excluded_brokers_for_leadership;
  int32_t num_excluded_brokers_for_leadership;
  const int32_t* excluded_brokers_for_replica_move;
  int32_t num_excluded_brokers_for_replica_move;
  int32_t triggered_by_goal_violation;
  const int32_t* requested_destination_broker_ids;
  int32_t num_requested_destination_broker_ids;
  int32_t only_move_immigrant_replicas;
  int32_t fast_mode; /* accepted for API parity. The reference's fast mode (default true) cuts per-broker loops at a
                        wall-clock timeout (AnalyzerConfig fast.mode.per.broker.move.timeout.ms, 500 ms), so its
                        result depends on host speed; the engine never cuts a loop short, i.e. it always returns
                        the result fast mode reaches when no timeout fires (= fast_mode 0). */
} ccmi_opt_options;

typedef struct ccmi_action {
  int32_t type;                  /* ccmi_action_type */
  int32_t partition;             /* partition index (desc order) */
  int32_t source_broker;
  int32_t destination_broker;
  int32_t destination_partition; /* swaps only, else -1 */
  int32_t source_disk;           /* intra-broker actions: disk indices (desc order), else -1. The action log records */
  int32_t destination_disk;      /* an intra-broker swap as its two relocateReplica(tp, broker, logdir) calls. */
} ccmi_action;

/* model/ClusterModelStats.java fields */
typedef struct ccmi_cluster_stats {
  double resource_avg[4], resource_max[4], resource_min[4], resource_std[4];
  int32_t num_balanced_brokers_by_resource[4];
  double potential_nw_out_avg, potential_nw_out_max, potential_nw_out_min, potential_nw_out_std;
  int32_t num_brokers_under_potential_nw_out;
  double replica_avg, replica_std;
  int32_t replica_max, replica_min;
  double leader_avg, leader_std;
  int32_t leader_max, leader_min;
  double topic_replica_avg, topic_replica_std;
  int32_t topic_replica_max, topic_replica_min;
  int32_t num_brokers, num_replicas_in_cluster, num_partitions_with_offline_replicas, num_topics;
  int32_t num_unbalanced_disks;
  double disk_utilization_std;
} ccmi_cluster_stats;

/* analyzer/ProvisionStatus.java */
typedef enum ccmi_provision_status {
  CCMI_PROVISION_UNDECIDED = 0,
  CCMI_PROVISION_RIGHT_SIZED = 1,
  CCMI_PROVISION_UNDER_PROVISIONED = 2,
  CCMI_PROVISION_OVER_PROVISIONED = 3
} ccmi_provision_status;

/* analyzer/ProvisionRecommendation.java: -1 = unset (DEFAULT_OPTIONAL_INT / DEFAULT_OPTIONAL_DOUBLE). The
 * recommendation's topic pattern and excluded rack ids are not carried. */
typedef struct ccmi_provision_recommendation {
  int32_t status;                 /* a ccmi_provision_status: UNDER or OVER */
  int32_t num_brokers, num_racks, num_disks, num_partitions;
  int32_t typical_broker_id;      /* broker id */
  int32_t resource;               /* ccmi resource index (CPU, NW_IN, NW_OUT, DISK) */
  int32_t pad;
  double typical_broker_capacity;
  double total_capacity;
} ccmi_provision_recommendation;

/* One goal's Goal.provisionResponse() (analyzer/ProvisionResponse.java): its status and, when the goal recorded one,
 * its own recommendation (recommendationByRecommender.get(goal name)). After an OptimizationFailureException the
 * status is UNDER_PROVISIONED with the exception's recommendation (AbstractGoal.java:125-126); on success it has been
 * through GoalUtils.validateProvisionResponse (:619-650). Aggregating goals' responses (ProvisionResponse.aggregate,
 * OptimizerResult's provision status) is the caller's, over the per-goal results. */
typedef struct ccmi_provision_response {
  int32_t status;                 /* ccmi_provision_status */
  int32_t has_recommendation;
  ccmi_provision_recommendation recommendation;
} ccmi_provision_response;

typedef struct ccmi_goal_result {
  int32_t goal_kind;
  int32_t succeeded;            /* Goal.optimize return value */
  int32_t has_diff;             /* AnalyzerUtils.hasDiff after this goal */
  double seconds;               /* wall time of the goal */
  int64_t candidates;           /* reference-equivalent candidate evaluations (BASELINE.md unit) */
  int64_t device_candidates;    /* candidates evaluated on the device, speculation included */
  int64_t device_launches;      /* scan-kernel launches */
  int64_t actions;              /* relocate* calls recorded in the action log */
  ccmi_cluster_stats stats;     /* ClusterModelStats after the goal (GoalOptimizer.statsByGoalPriority) */
  ccmi_provision_response provision;
} ccmi_goal_result;

/* Test fixture generator: RandomCluster properties (common/ClusterProperty.java + populate() flags) */
typedef struct ccmi_random_cluster_props {
  int32_t num_racks, num_brokers, num_dead_brokers, num_brokers_with_bad_disk;
  int32_t num_replicas, num_topics, min_replication, max_replication;
  double mean_cpu, mean_disk, mean_nw_in, mean_nw_out;
  int32_t distribution;          /* 0 UNIFORM, 1 LINEAR, 2 EXPONENTIAL */
  int32_t rack_aware;
  int32_t leader_in_first_position;
  /* POPULATE_REPLICA_PLACEMENT_INFO: 0 none; 1 the reference's JBOD capacity file (testCapacityConfigJBOD.json:
   * brokers 0/1/2 overridden, default broker 10 logdirs); 2 every broker num_logdirs logdirs "/mnt/d<i>" with
   * capacities logdir_capacity[i] (the C4 layout; non-disk capacities from DefaultCapacityConfig.json). */
  int32_t jbod;
  int32_t num_logdirs;
  double logdir_capacity[8];
} ccmi_random_cluster_props;

typedef struct ccmi_session ccmi_session;
typedef struct ccmi_cluster_buffers ccmi_cluster_buffers; /* owns the arrays behind a generated desc */

const char* ccmi_last_error(void);
int32_t ccmi_abi_version(void);
/* Number of visible gfx950 devices (on an MI355X node: HIP ordinals 0..n-1, the `device` of ccmi_session_create);
 * 0 when none. What-if batches (GoalViolationDetector) spread their sessions over them. */
int32_t ccmi_device_count(void);
void ccmi_default_constraint(ccmi_balancing_constraint* out);
void ccmi_default_random_cluster_props(ccmi_random_cluster_props* out); /* TestConstants.BASE_PROPERTIES */

ccmi_status ccmi_random_cluster(const ccmi_random_cluster_props* props, ccmi_cluster_buffers** out);
/* TopicNameHashBrokerSetMappingPolicy.brokerSetIdForTopic (config/TopicNameHashBrokerSetMappingPolicy.java:60-70): the
 * index, in String order of the broker set ids, of the set a topic maps to among num_broker_sets sets —
 * Guava Hashing.consistentHash(|murmur3_128(topic, UTF-8).asInt()|, num_broker_sets). -1 if num_broker_sets < 1. */
int32_t ccmi_topic_broker_set(const char* topic, int32_t num_broker_sets);
const ccmi_cluster_desc* ccmi_cluster_buffers_desc(const ccmi_cluster_buffers* buf);
void ccmi_cluster_buffers_free(ccmi_cluster_buffers* buf);

/*
 * Model ingestion: LoadMonitor.clusterModel (monitor/LoadMonitor.java:491-543) builds the ClusterModel from the Kafka
 * metadata, the broker capacities and each partition's aggregated leader metrics; this builder takes the same calls
 * and produces the flattened ccmi_cluster_desc directly (no Java ClusterModel needed for the engine's side):
 *   ccmi_builder_create_broker  ClusterModel.createRack + createBroker for a live node (populateClusterCapacity
 *                               :563-600), or handleDeadBroker for a dead one (alive = 0; a no-op if it exists)
 *   ccmi_builder_add_disk       a logdir of a JBOD broker (BrokerCapacityInfo.diskCapacityByLogDir)
 *   ccmi_builder_populate_partition
 *                               MonitorUtils.populatePartitionLoad (MonitorUtils.java:415-479): one createReplica +
 *                               setReplicaLoad per replica of PartitionInfo.replicas() in order, the loads derived
 *                               from the partition's aggregated leader metrics by getAggregatedMetricValues (:215-265):
 *                               CPU unit interval -> percentage once per partition, the leader's replication bytes
 *                               out = leader bytes in x followers, a follower's NW_OUT = 0 and CPU from
 *                               ModelUtils.getFollowerCpuUtilFromLeaderLoad (0.7 / 0.15 / 0.15 weights), all in the
 *                               reference's float MetricValues arithmetic. leader_broker_id < 0 = offline partition
 *                               (no replicas created, LoadMonitor logs and skips it).
 *   ccmi_builder_set_broker_state  setBadBrokerState (MonitorUtils.java:349-356) and NEW / DEMOTED marking
 *   ccmi_builder_desc           the flattened model (valid until ccmi_builder_destroy). Brokers are indexed in
 *                               ascending id order; broker_id[b] = b in the desc, and ccmi_builder_broker_ids maps an
 *                               index back to the Kafka broker id (HashSet<Broker> iteration ties follow the dense
 *                               index, which equals the reference's order when the ids are 0..B-1).
 * leader_metrics: [6 * W] floats, ccmi_metric order, newest window first (ValuesAndExtrapolations.metricValues()).
 */
typedef struct ccmi_model_builder ccmi_model_builder;
ccmi_status ccmi_builder_create(int32_t num_windows, ccmi_model_builder** out);
void ccmi_builder_destroy(ccmi_model_builder* b);
ccmi_status ccmi_builder_create_broker(ccmi_model_builder* b, const char* rack, const char* host, int32_t broker_id,
                                       const double capacity[4], int32_t alive);
ccmi_status ccmi_builder_add_disk(ccmi_model_builder* b, int32_t broker_id, const char* logdir, double capacity);
ccmi_status ccmi_builder_populate_partition(ccmi_model_builder* b, const char* topic, int32_t partition,
                                            const int32_t* replica_broker_ids, int32_t num_replicas,
                                            int32_t leader_broker_id, const uint8_t* offline,
                                            const char* const* logdirs, const float* leader_metrics);
ccmi_status ccmi_builder_set_broker_state(ccmi_model_builder* b, int32_t broker_id, int32_t state);
/* Disk.setState for a disk added with ccmi_builder_add_disk: CCMI_DISK_ALIVE or CCMI_DISK_DEMOTED (a dead disk is
 * given by a negative capacity). */
ccmi_status ccmi_builder_set_disk_state(ccmi_model_builder* b, int32_t broker_id, const char* logdir, int32_t state);
ccmi_status ccmi_builder_desc(ccmi_model_builder* b, ccmi_cluster_desc* out);
ccmi_status ccmi_builder_broker_ids(const ccmi_model_builder* b, int32_t* out);

/* device_ordinal: the HIP device the session's tables live on (one session = one device). Destination-sharded
 * sessions are one per process and GPU, joined by ccmi_session_set_shard / ccmi_session_attach_rccl below. */
ccmi_status ccmi_session_create(int32_t device_ordinal, const ccmi_cluster_desc* desc, ccmi_session** out);
ccmi_status ccmi_session_destroy(ccmi_session* s);

/* Run a whole goal chain (GoalOptimizer.optimizations). results: caller array of n_goals entries. Every goal's
 * optimizedGoals are the goals before it in this call (GoalOptimizer.java:449,467-471), not earlier calls' goals. */
ccmi_status ccmi_optimizations(ccmi_session* s, const int32_t* goal_kinds, int32_t n_goals,
                               const ccmi_balancing_constraint* constraint, const ccmi_opt_options* options,
                               ccmi_goal_result* results);
/*
 * Goal.optimize(ClusterModel, Set<Goal> optimizedGoals, OptimizationOptions) (analyzer/goals/Goal.java:60-68,
 * AbstractGoal.java:81-135). The session keeps every goal it has optimized — one per goal kind, as GoalOptimizer keeps
 * one instance per goal class, a re-optimized kind replacing its older entry — with the frozen state its
 * actionAcceptance reads. optimized_goal_kinds[0, num_optimized_goals) is the caller's optimizedGoals set (ABI v8): only
 * those goals' actionAcceptance joins the candidate conjunction (AnalyzerUtils.isProposalAcceptableForOptimizedGoals,
 * AnalyzerUtils.java:169-179), whatever else the session has run. GoalOptimizer passes the goals optimized earlier in the
 * same optimizations() call; GoalViolationDetector passes the empty set on a model it reuses across goals
 * (GoalViolationDetector.java:193-211,314). Duplicate kinds count once; order does not matter.
 * A kind the session has not optimized — a goal whose optimize ran in the JVM, or a goal class that exists only in the
 * JVM (pass any kind outside ccmi_goal_kind, e.g. -1) — returns CCMI_E_UNSUPPORTED before anything changes: its
 * actionAcceptance is not available to the device, so the caller runs this goal in the JVM instead.
 */
ccmi_status ccmi_goal_optimize(ccmi_session* s, int32_t goal_kind, const int32_t* optimized_goal_kinds,
                               int32_t num_optimized_goals, const ccmi_balancing_constraint* constraint,
                               const ccmi_opt_options* options, ccmi_goal_result* result);
/* Acceptance of an action by the i-th goal the session holds (the goals it has optimized, one per kind, in the order
 * each was last optimized: after one ccmi_optimizations call on a fresh session, the chain position). */
ccmi_status ccmi_action_acceptance(ccmi_session* s, int32_t optimized_goal_index, const ccmi_action* action,
                                   int32_t* acceptance);
/* Goal.actionAcceptance keyed by the goal plugin (ccmi_goal_kind) instead of the chain position: the most recently
 * optimized goal of that kind (GoalOptimizer holds one instance per goal class). CCMI_E_INVALID when the session
 * has not optimized that kind. */
ccmi_status ccmi_action_acceptance_by_kind(ccmi_session* s, int32_t goal_kind, const ccmi_action* action,
                                           int32_t* acceptance);
/* Session update by deltas: apply actions decided outside this session (a JVM goal earlier in a mixed chain, an
 * executed proposal batch) to the resident model, in order, as ClusterModel.relocateReplica /
 * relocateLeadership / relocateReplica(tp, broker, logdir) do (a swap is its two relocateReplica calls,
 * AbstractGoal.maybeApplySwapAction :316-317). Only the touched rows are re-sent to the device, so a mixed-chain hop
 * costs O(actions), not an O(R) re-flatten. Actions are validated first (the replica exists on the source, the
 * destination does not host the partition / hosts a follower, disks belong to the broker); the first invalid one
 * fails the call with CCMI_E_INVALID and `*applied` (optional) = actions applied before it. Applied actions join
 * the action log and the proposals (the diff against the session's initial placement). */
ccmi_status ccmi_session_apply(ccmi_session* s, const ccmi_action* actions, int64_t n, int64_t* applied);
/* Goal.provisionResponse of the goal whose OptimizationFailureException (CCMI_E_OPT_FAILURE) ended the session's last
 * optimization call: UNDER_PROVISIONED with the exception's ProvisionRecommendation (AbstractGoal.java:125-130). */
ccmi_status ccmi_last_failure_provision(const ccmi_session* s, ccmi_provision_response* out);
ccmi_status ccmi_compute_cluster_stats(ccmi_session* s, const ccmi_balancing_constraint* constraint,
                               const ccmi_opt_options* options, ccmi_cluster_stats* out);

int64_t ccmi_action_log_count(const ccmi_session* s);
ccmi_status ccmi_action_log_copy(const ccmi_session* s, int64_t first, int64_t count, ccmi_action* out);
/* [R] current broker of each replica slot in partition CSR order / [P] leader broker per partition */
ccmi_status ccmi_replica_distribution(const ccmi_session* s, int32_t* out);
ccmi_status ccmi_leader_distribution(const ccmi_session* s, int32_t* out);
/* [R] current disk of each replica slot in partition CSR order (-1 = no disk) */
ccmi_status ccmi_replica_disks(const ccmi_session* s, int32_t* out);
/* ExecutionProposals: count, then per proposal: partition, size, old leader, RF; old and new broker lists
 * (new list leader-first) packed into old_out/new_out with stride max_rf. */
int64_t ccmi_proposal_count(const ccmi_session* s);
ccmi_status ccmi_proposals(const ccmi_session* s, int32_t max_rf, int32_t* partition, int32_t* size,
                           int32_t* old_leader, int32_t* old_out, int32_t* new_out);
/* The logdir half of the proposals' ReplicaPlacementInfo lists (disk indices, -1 = none), same packing. */
ccmi_status ccmi_proposal_disks(const ccmi_session* s, int32_t max_rf, int32_t* old_disk_out, int32_t* new_disk_out);

/*
 * Destination-sharded mode (one process per GPU): every rank creates a session on its own device from the same
 * desc, runs the same goal chain, and scans only its slice [N*rank/count, N*(rank+1)/count) of every candidate
 * list. After each scan the engine calls `fn(ctx, key)`, which must replace *key by the MIN over all ranks
 * (INT64_MAX = no accepted candidate) and return 0; the result is the reference's first accepted candidate, so
 * every rank applies the same move. Swap scans and statistics run unsharded on every rank.
 * ccmi_session_attach_rccl installs the built-in RCCL combiner (one int64 MIN allreduce over xGMI per scan);
 * ccmi_rccl_unique_id produces the 128-byte id rank 0 broadcasts to the others.
 */
typedef int (*ccmi_allreduce_min_fn)(void* ctx, int64_t* key);
ccmi_status ccmi_session_set_shard(ccmi_session* s, int32_t rank, int32_t count, ccmi_allreduce_min_fn fn, void* ctx);
ccmi_status ccmi_rccl_unique_id(uint8_t out[128]);
ccmi_status ccmi_session_attach_rccl(ccmi_session* s, int32_t rank, int32_t count, const uint8_t unique_id[128]);
/* ABI v9. ccmi_session_attach_shm: the built-in combiner for ranks on one node — a MIN over one int64 per rank in a
 * POSIX shared-memory block `name` ("/name"; rank 0 creates it, the others open it, and every rank waits until all
 * `count` ranks are attached, at most 120 s). No GPU work per combine, so the session keeps its scan server. */
ccmi_status ccmi_session_attach_shm(ccmi_session* s, int32_t rank, int32_t count, const char* name);
/* ABI v12. ccmi_session_attach_shm with a job nonce: every rank passes the same nonzero `job_nonce` (e.g. rank 0's
 * start time broadcast over the job's process group); rank 0 stamps it into the block and the other ranks attach only
 * to a block carrying it, so a block a crashed run left under the same name is refused however recent (nonce 0: the
 * v9 rule, a block older than the timeout is stale). `timeout_s` bounds every wait (0 = 120 s). */
ccmi_status ccmi_session_attach_shm_job(ccmi_session* s, int32_t rank, int32_t count, const char* name,
                                        uint64_t job_nonce, double timeout_s);
/* ABI v11. Shard groups: the ranks of one sharded proposal driven from ONE process, one host thread per session
 * (typically one session per GPU of the node, each thread calling ccmi_optimizations on its own session). The ranks'
 * first-fit keys are MIN-combined in a block of pinned host memory every device maps: a scan the session's resident
 * scan server ran is combined by the server itself (its last workgroup folds the key in with system-scope atomics and
 * counts the rank in; no kernel waits for another rank), any other scan by the host thread on the same slots; whichever
 * rank arrives last (a server's workgroup or a host thread) publishes the group minimum into every rank's mailbox. A
 * destroyed session leaves its rank's slot empty and a destroyed group detaches its sessions. The queue-scan path is
 * taken only when every rank can take it (decided at each attach), so all ranks run the same scans and combines. Replaces the per-scan host MIN of GoalOptimizer's single-threaded loop with nothing on the
 * host between the ranks' scans. */
typedef struct ccmi_shard_group ccmi_shard_group;
ccmi_status ccmi_shard_group_create(int32_t count, ccmi_shard_group** out);
ccmi_status ccmi_shard_group_destroy(ccmi_shard_group* g);
ccmi_status ccmi_session_attach_group(ccmi_session* s, ccmi_shard_group* g, int32_t rank);

/* Measurement hooks used by bench.py: device time of the last optimization's scan kernels (HIP events
 * on the engine stream) and their algorithmic bytes. */
typedef struct ccmi_perf_counters {
  int64_t scan_launches;
  double scan_kernel_ms;       /* sum of HIP-event durations of the scan kernel */
  int64_t scan_bytes;          /* algorithmic bytes (DESIGN.md per-candidate figure x candidates) */
  int64_t stats_launches;
  double stats_kernel_ms;
  int64_t stats_bytes;
  int64_t host_syncs;
  int64_t scan_required;       /* candidates the scans had to evaluate: every device list up to its winner (the
                                  algorithmic work; smaller than `candidates` where the engine never sends rows that
                                  cannot be accepted, e.g. non-legit leadership rows) */
  int64_t chain_launches;      /* K7 chain launches (several decisions applied on the device per launch) */
  int64_t intra_launches;      /* K6 intra-broker launches (one per intra-broker goal, plus overflow re-runs) */
  double intra_kernel_ms;      /* HIP-event duration of the K6 intra_brokers launches */
  int64_t intra_bytes;         /* algorithmic bytes of K6 */
  int64_t cross_launches;      /* the scan_cross share of scan_launches / scan_required / scan_kernel_ms (the kernel */
  int64_t cross_required;      /* tools/pmc_summary.py prices against its own FETCH_SIZE / WRITE_SIZE counters) */
  double cross_kernel_ms;
  int64_t combines;            /* shard-combiner calls (RCCL / host MIN-allreduce of a scan's first-fit key) */
  /* ABI v6: the persistent scan server (K8): its launches (each also counts in scan_launches), the cross / pair scans
   * it served (no launch each), their candidates up to the winner, and its busy time (first workgroup seeing a
   * command to the result published, summed over commands) */
  int64_t server_launches;
  int64_t server_scans;
  int64_t server_required;
  double server_busy_ms;
  int64_t server_payload_bytes; /* command payload the host wrote into device memory for the server */
  /* ABI v8: K7 chains the running server took as commands (SOP_CHAIN: no launch, no server stop and relaunch; the
   * chain_launches above count only chains that ran as their own launch), and commands the server's idle watchdog
   * ended before it saw them (each then ran as a launch) */
  int64_t server_chains;
  int64_t server_idle_exits;
  /* ABI v9: HIP-event time from each scan-server launch to its exit, summed (with ccmi_set_kernel_timing on): the
   * residency a rocprofv3 kernel trace reports for scan_server, idle polling included */
  double server_resident_ms;
  /* ABI v10: K6's per-call sort (intra_sort, one launch per intra-broker call) timed apart from intra_brokers, whose
   * HIP-event time intra_kernel_ms now holds alone */
  int64_t intra_sort_launches;
  double intra_sort_ms;
} ccmi_perf_counters;
ccmi_status ccmi_perf(const ccmi_session* s, ccmi_perf_counters* out);
void ccmi_perf_reset(ccmi_session* s);
/* Record HIP events around every scan/stats kernel (adds a little host overhead; off by default). */
void ccmi_set_kernel_timing(ccmi_session* s, int32_t enabled);

#ifdef __cplusplus
}
#endif
#endif /* CCMI_H_ */
