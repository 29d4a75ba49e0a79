// ORACLE — test infrastructure only (see jsem.h header). C entry points (liboracle_cc.so) used by
// tests/ (ctypes) and bench.py's cpu_baseline leg. Shares only the data layout of include/ccmi.h.
#include <algorithm>
#include <chrono>
#include <cstring>
#include <memory>
#include <string>

#include "../../include/ccmi.h"
#include "brokersets.h"
#include "optimizer.h"
#include "random_cluster.h"

using namespace oracle;

namespace {
struct Handle {
  ClusterModel cm;
  OptimizerResult last;
  std::string err;
  // Goal instances that have optimized this model, one per goal kind (GoalOptimizer's one instance per goal class),
  // for the optimizedGoals sets of oc_goal_optimize
  std::vector<std::pair<int, std::shared_ptr<Goal>>> held;
  void hold(int kind, std::shared_ptr<Goal> g) {
    for (auto& e : held)
      if (e.first == kind) {
        e.second = std::move(g);
        return;
      }
    held.emplace_back(kind, std::move(g));
  }
  Goal* heldOf(int kind) const {
    for (auto& e : held)
      if (e.first == kind) return e.second.get();
    return nullptr;
  }
};

BalancingConstraint toBc(const ccmi_balancing_constraint* c) {
  BalancingConstraint bc;
  if (!c) return bc;
  for (int r = 0; r < 4; ++r) {
    bc.resourceBalancePercentage[r] = c->resource_balance_percentage[r];
    bc.capacityThreshold[r] = c->capacity_threshold[r];
    bc.lowUtilizationThreshold[r] = c->low_utilization_threshold[r];
  }
  bc.replicaBalancePercentage = c->replica_balance_percentage;
  bc.leaderReplicaBalancePercentage = c->leader_replica_balance_percentage;
  bc.topicReplicaBalancePercentage = c->topic_replica_balance_percentage;
  bc.topicReplicaBalanceMinGap = c->topic_replica_balance_min_gap;
  bc.topicReplicaBalanceMaxGap = c->topic_replica_balance_max_gap;
  bc.goalViolationDistributionThresholdMultiplier = c->goal_violation_distribution_threshold_multiplier;
  bc.maxReplicasPerBroker = c->max_replicas_per_broker;
  bc.overprovisionedMaxReplicasPerBroker = c->overprovisioned_max_replicas_per_broker;
  bc.overprovisionedMinBrokers = c->overprovisioned_min_brokers;
  bc.overprovisionedMinExtraRacks = c->overprovisioned_min_extra_racks;
  for (int i = 0; i < c->num_broker_sets; ++i) {
    auto& v = bc.brokerSets[c->broker_set_names[i]];
    for (int k = c->broker_set_offset[i]; k < c->broker_set_offset[i + 1]; ++k) v.push_back(c->broker_set_members[k]);
  }
  bc.brokerSetPolicy = c->broker_set_policy;
  for (int i = 0; i < c->num_min_leader_topics; ++i) bc.minLeaderTopics.push_back(c->min_leader_topics[i]);
  bc.minTopicLeadersPerBroker = c->min_topic_leaders_per_broker;
  bc.topicLeaderReplicaBalancePercentage = c->topic_leader_replica_balance_percentage;
  bc.topicLeaderReplicaBalanceMinGap = c->topic_leader_replica_balance_min_gap;
  bc.topicLeaderReplicaBalanceMaxGap = c->topic_leader_replica_balance_max_gap;
  bc.topicLeaderReplicaDistributionGoalBalanceMargin = c->topic_leader_replica_balance_margin;
  return bc;
}

OptimizationOptions toOpts(const ccmi_opt_options* o) {
  OptimizationOptions oo;
  if (!o) return oo;
  for (int i = 0; i < o->num_excluded_topics; ++i) oo.excludedTopics.insert(o->excluded_topics[i]);
  for (int i = 0; i < o->num_excluded_brokers_for_leadership; ++i)
    oo.excludedBrokersForLeadership.insert(o->excluded_brokers_for_leadership[i]);
  for (int i = 0; i < o->num_excluded_brokers_for_replica_move; ++i)
    oo.excludedBrokersForReplicaMove.insert(o->excluded_brokers_for_replica_move[i]);
  oo.triggeredByGoalViolation = o->triggered_by_goal_violation != 0;
  for (int i = 0; i < o->num_requested_destination_broker_ids; ++i)
    oo.requestedDestinationBrokerIds.insert(o->requested_destination_broker_ids[i]);
  oo.onlyMoveImmigrantReplicas = o->only_move_immigrant_replicas != 0;
  oo.fastMode = o->fast_mode != 0;
  return oo;
}

void toCProvision(const ProvisionResp& p, ccmi_provision_response* o) {
  std::memset(o, 0, sizeof(*o));
  o->status = p.status;
  o->has_recommendation = p.hasRec ? 1 : 0;
  ccmi_provision_recommendation& r = o->recommendation;
  r.status = p.hasRec ? p.rec.status : 0;
  r.num_brokers = p.hasRec ? p.rec.numBrokers : -1;
  r.num_racks = p.hasRec ? p.rec.numRacks : -1;
  r.num_disks = p.hasRec ? p.rec.numDisks : -1;
  r.num_partitions = p.hasRec ? p.rec.numPartitions : -1;
  r.typical_broker_id = p.hasRec ? p.rec.typicalBrokerId : -1;
  r.resource = p.hasRec ? p.rec.resource : -1;
  r.typical_broker_capacity = p.hasRec ? p.rec.typicalBrokerCapacity : -1.0;
  r.total_capacity = p.hasRec ? p.rec.totalCapacity : -1.0;
}

void toCStats(const ClusterModelStats& s, ccmi_cluster_stats* o) {
  for (int r = 0; r < 4; ++r) {
    o->resource_avg[r] = s.resAvg[r];
    o->resource_max[r] = s.resMax[r];
    o->resource_min[r] = s.resMin[r];
    o->resource_std[r] = s.resStd[r];
    o->num_balanced_brokers_by_resource[r] = s.numBalancedBrokersByResource[r];
  }
  o->potential_nw_out_avg = s.pnwAvg;
  o->potential_nw_out_max = s.pnwMax;
  o->potential_nw_out_min = s.pnwMin;
  o->potential_nw_out_std = s.pnwStd;
  o->num_brokers_under_potential_nw_out = s.numBrokersUnderPotentialNwOut;
  o->replica_avg = s.repAvg;
  o->replica_std = s.repStd;
  o->replica_max = s.repMax;
  o->replica_min = s.repMin;
  o->leader_avg = s.leadAvg;
  o->leader_std = s.leadStd;
  o->leader_max = s.leadMax;
  o->leader_min = s.leadMin;
  o->topic_replica_avg = s.topicAvg;
  o->topic_replica_std = s.topicStd;
  o->topic_replica_max = s.topicMax;
  o->topic_replica_min = s.topicMin;
  o->num_brokers = s.numBrokers;
  o->num_replicas_in_cluster = s.numReplicasInCluster;
  o->num_partitions_with_offline_replicas = s.numPartitionsWithOfflineReplicas;
  o->num_topics = s.numTopics;
  o->num_unbalanced_disks = s.numUnbalancedDisks;
  o->disk_utilization_std = s.diskUtilizationStDev;
}
}  // namespace

extern "C" {

void* oc_random_cluster(const ccmi_random_cluster_props* p) {
  auto* h = new Handle();
  ClusterProperties cp;
  cp.numRacks = p->num_racks;
  cp.numBrokers = p->num_brokers;
  cp.numDeadBrokers = p->num_dead_brokers;
  cp.numBrokersWithBadDisk = p->num_brokers_with_bad_disk;
  cp.numReplicas = p->num_replicas;
  cp.numTopics = p->num_topics;
  cp.minReplication = p->min_replication;
  cp.maxReplication = p->max_replication;
  cp.meanCpu = p->mean_cpu;
  cp.meanDisk = p->mean_disk;
  cp.meanNwIn = p->mean_nw_in;
  cp.meanNwOut = p->mean_nw_out;
  cp.distribution = p->distribution;
  cp.rackAware = p->rack_aware != 0;
  cp.leaderInFirstPosition = p->leader_in_first_position != 0;
  cp.jbod = p->jbod;
  cp.numLogdirs = p->num_logdirs;
  for (int i = 0; i < 8; ++i) cp.logdirCapacity[i] = p->logdir_capacity[i];
  try {
    randomCluster(h->cm, cp);
  } catch (std::exception& e) {
    delete h;
    return nullptr;
  }
  return h;
}

// Build the model from a flattened desc exactly as ccmi.h documents (replica index order replay).
void* oc_from_desc(const ccmi_cluster_desc* d) {
  auto* h = new Handle();
  ClusterModel& cm = h->cm;
  try {
    cm.W = d->num_windows;
    for (int i = 0; i < d->num_racks; ++i) cm.createRack(std::to_string(i));
    // broker_host: dense host indices (Rack._hosts by name); NULL = a host per broker
    for (int b = 0; b < d->num_brokers; ++b)
      cm.createBroker(d->broker_rack[b], d->broker_id[b], &d->broker_capacity[4 * b],
                      d->broker_host ? d->broker_host[b] : -1);
    for (int t = 0; t < d->num_topics; ++t) {
      cm.topicNames.push_back(d->topic_names[t]);
      cm.topicHash.push_back(jStringHash(cm.topicNames.back()));
      cm.numReplicasByTopic.push_back(0);
      cm.replicationFactorByTopic.push_back(0);
    }
    for (int k = 0; k < d->num_disks; ++k) {
      if (cm.createDisk(d->disk_broker[k], d->disk_logdir[k], d->disk_capacity[k]) != k)
        throw std::runtime_error("disk index mismatch");
      cm.disks[k].demoted = d->disk_demoted && d->disk_demoted[k];
    }
    std::vector<char> created(d->num_partitions, 0);
    const int W = d->num_windows;
    // ClusterModel.setReplicaLoad with getAggregatedMetricValues-style windows (KafkaCruiseControlUnitTestUtils)
    auto setLoad = [&](int r) {
      Load amv;
      amv.mask = 0x3F;
      for (int k = 0; k < NUM_METRICS; ++k) {
        amv.m[k].sum = 0.0;
        for (int w = 0; w < W; ++w) {
          amv.m[k].v[w] = d->replica_load[((size_t)r * NUM_METRICS + k) * W + w];
          amv.m[k].sum += (double)amv.m[k].v[w];
        }
      }
      cm.setReplicaLoad(r, amv);
    };
    for (int r = 0; r < d->num_replicas; ++r) {
      int p = d->replica_partition[r];
      if (!created[p]) {
        while ((int)cm.partitions.size() <= p) cm.createPartition(d->partition_topic[cm.partitions.size()],
                                                                   d->partition_number[cm.partitions.size()]);
        created[p] = 1;
      }
      int b = d->replica_broker[r];
      int idx = (int)cm.partitions[p].replicas.size();
      const int disk = (d->num_disks > 0 && d->replica_disk) ? d->replica_disk[r] : -1;
      int rr = cm.createReplica(b, p, idx, d->replica_is_leader[r] != 0, d->replica_offline[r] != 0, disk);
      if (rr != r) throw std::runtime_error("replica index mismatch");
      if (!d->replica_load_order) setLoad(rr);
    }
    // hand-built models: every createReplica first, then setReplicaLoad in the caller's order
    if (d->replica_load_order) {
      const int n = d->num_replica_loads > 0 ? d->num_replica_loads : d->num_replicas;
      for (int i = 0; i < n; ++i) setLoad(d->replica_load_order[i]);
    }
    for (int p = 0; p < d->num_partitions; ++p) {
      auto& lst = cm.partitions[p].replicas;
      lst.assign(d->partition_replicas + d->partition_offset[p], d->partition_replicas + d->partition_offset[p + 1]);
    }
    cm.finalizeTopics();
    for (int i = 0; i < d->num_disk_assignments; ++i) cm.diskAddReplica(d->disk_assign_disk[i], d->disk_assign_replica[i]);
    for (int b = 0; b < d->num_brokers; ++b)
      if (d->broker_state[b] != CCMI_BROKER_ALIVE) cm.setBrokerState(b, (BrokerState)d->broker_state[b]);
  } catch (std::exception& e) {
    delete h;
    return nullptr;
  }
  return h;
}

void oc_free(void* h) { delete (Handle*)h; }

void oc_sizes(void* hv, int32_t* out) {
  auto* h = (Handle*)hv;
  out[0] = (int32_t)h->cm.brokers.size();
  out[1] = (int32_t)h->cm.topicNames.size();
  out[2] = (int32_t)h->cm.partitions.size();
  out[3] = (int32_t)h->cm.replicas.size();
  out[4] = (int32_t)h->cm.racks.size();
  out[5] = h->cm.W;
}
const char* oc_topic_name(void* hv, int t) { return ((Handle*)hv)->cm.topicNames[t].c_str(); }

// Export the *initial* model in desc layout (valid before any optimization).
void oc_export(void* hv, int32_t* broker_rack, int32_t* broker_state, double* cap, int32_t* partition_topic,
               int32_t* partition_number, int32_t* partition_offset, int32_t* partition_replicas,
               int32_t* replica_partition, int32_t* replica_broker, uint8_t* is_leader, uint8_t* offline, float* load) {
  auto* h = (Handle*)hv;
  ClusterModel& cm = h->cm;
  for (size_t b = 0; b < cm.brokers.size(); ++b) {
    broker_rack[b] = cm.brokers[b].rack;
    broker_state[b] = (int32_t)cm.brokers[b].state;
    for (int r = 0; r < 4; ++r) cap[4 * b + r] = cm.brokers[b].capacity[r];  // as given at creation (the desc form)
  }
  int off = 0;
  for (size_t p = 0; p < cm.partitions.size(); ++p) {
    partition_topic[p] = cm.partitions[p].topic;
    partition_number[p] = cm.partitions[p].number;
    partition_offset[p] = off;
    for (int r : cm.partitions[p].replicas) partition_replicas[off++] = r;
  }
  partition_offset[cm.partitions.size()] = off;
  const int W = cm.W;
  for (size_t r = 0; r < cm.replicas.size(); ++r) {
    const Replica& rep = cm.replicas[r];
    replica_partition[r] = rep.partition;
    replica_broker[r] = rep.broker;
    is_leader[r] = rep.isLeader;
    offline[r] = rep.origOfflineFlag;
    for (int k = 0; k < NUM_METRICS; ++k)
      for (int w = 0; w < W; ++w) load[((size_t)r * NUM_METRICS + k) * W + w] = rep.load.m[k].v[w];
  }
}

// Disks of the initial model (valid before any optimization): count, then per disk broker / capacity / logdir, and
// the Disk.addReplica replay (replicas created without a disk that were placed afterwards) in placement order.
int32_t oc_num_disks(void* hv) { return (int32_t)((Handle*)hv)->cm.disks.size(); }
const char* oc_disk_logdir(void* hv, int d) { return ((Handle*)hv)->cm.disks[d].logdir.c_str(); }
void oc_export_disks(void* hv, int32_t* disk_broker, double* disk_capacity, int32_t* replica_disk) {
  auto* h = (Handle*)hv;
  for (size_t d = 0; d < h->cm.disks.size(); ++d) {
    disk_broker[d] = h->cm.disks[d].broker;
    disk_capacity[d] = h->cm.disks[d].capacity;
  }
  for (size_t r = 0; r < h->cm.replicas.size(); ++r) replica_disk[r] = h->cm.replicas[r].origDisk;
}
int64_t oc_num_disk_assignments(void* hv) { return (int64_t)((Handle*)hv)->cm.diskAssignLog.size(); }
void oc_disk_assignments(void* hv, int32_t* replica, int32_t* disk) {
  auto* h = (Handle*)hv;
  for (size_t i = 0; i < h->cm.diskAssignLog.size(); ++i) {
    replica[i] = h->cm.diskAssignLog[i].first;
    disk[i] = h->cm.diskAssignLog[i].second;
  }
}
void oc_replica_disks(void* hv, int32_t* out) {
  auto v = ((Handle*)hv)->cm.replicaDiskFlat();
  std::memcpy(out, v.data(), v.size() * sizeof(int32_t));
}
double oc_disk_utilization(void* hv, int d) { return ((Handle*)hv)->cm.disks[d].utilization; }

int oc_optimize(void* hv, const int32_t* goals, int n, const ccmi_balancing_constraint* c, const ccmi_opt_options* o,
                ccmi_goal_result* results) {
  auto* h = (Handle*)hv;
  try {
    std::vector<int> kinds(goals, goals + n);
    h->last = optimizations(h->cm, kinds, toBc(c), toOpts(o));
    for (int i = 0; i < n; ++i) h->hold(goals[i], h->last.optimizedGoals[i]);
    for (int i = 0; i < n; ++i) {
      const GoalResult& g = h->last.goals[i];
      ccmi_goal_result& r = results[i];
      std::memset(&r, 0, sizeof(r));
      r.goal_kind = goals[i];
      r.succeeded = g.succeeded;
      r.has_diff = g.hasDiff;
      r.seconds = g.seconds;
      r.candidates = g.candidates;
      r.actions = g.actions;
      toCStats(g.stats, &r.stats);
      toCProvision(g.provision, &r.provision);
    }
    return 0;
  } catch (DeadlineReached&) {
    h->err = "deadline reached";
    return 99;
  } catch (OptimizationFailure& e) {
    h->err = e.what();
    return CCMI_E_OPT_FAILURE;
  } catch (UnsupportedOperation& e) {
    h->err = e.what();
    return CCMI_E_UNSUPPORTED;
  } catch (std::invalid_argument& e) {  // IllegalArgumentException
    h->err = e.what();
    return CCMI_E_INVALID;
  } catch (std::logic_error& e) {
    h->err = e.what();
    return CCMI_E_STATE;
  } catch (std::exception& e) {
    h->err = e.what();
    return CCMI_E_INVALID;
  }
}
// Goal.optimize(cm, optimizedGoals, options) for one goal kind; optimizedGoals = the held goals of set_kinds
// (CCMI_E_UNSUPPORTED when one is not held). The goal is held afterwards.
int oc_goal_optimize(void* hv, int32_t kind, const int32_t* set_kinds, int32_t n_set, const ccmi_balancing_constraint* c,
                     const ccmi_opt_options* o, ccmi_goal_result* result) {
  auto* h = (Handle*)hv;
  try {
    GoalList set;
    for (int i = 0; i < n_set; ++i) {
      Goal* g = h->heldOf(set_kinds[i]);
      if (!g) throw UnsupportedOperation("optimized goal kind " + std::to_string(set_kinds[i]) + " is not held");
      if (std::find(set.begin(), set.end(), g) == set.end()) set.push_back(g);
    }
    if (isIntraBrokerGoal(kind) && h->cm.disks.empty())
      throw std::invalid_argument("intra-broker goals need replica placement over disks");
    for (Goal* g : set)
      for (auto& e : h->held)
        if (e.second.get() == g && isIntraBrokerGoal(e.first) != isIntraBrokerGoal(kind))
          throw std::invalid_argument("intra-broker goals cannot be optimized together with inter-broker goals");
    const BalancingConstraint bc = toBc(c);
    std::shared_ptr<Goal> g = makeGoal(kind, bc);
    const GoalResult gr = goalOptimize(h->cm, *g, set, bc, toOpts(o));
    h->hold(kind, g);
    ccmi_goal_result& r = *result;
    std::memset(&r, 0, sizeof(r));
    r.goal_kind = kind;
    r.succeeded = gr.succeeded;
    r.has_diff = gr.hasDiff;
    r.seconds = gr.seconds;
    r.candidates = gr.candidates;
    r.actions = gr.actions;
    toCStats(gr.stats, &r.stats);
    toCProvision(gr.provision, &r.provision);
    return 0;
  } catch (OptimizationFailure& e) {
    h->err = e.what();
    return CCMI_E_OPT_FAILURE;
  } catch (UnsupportedOperation& e) {
    h->err = e.what();
    return CCMI_E_UNSUPPORTED;
  } catch (std::invalid_argument& e) {
    h->err = e.what();
    return CCMI_E_INVALID;
  } catch (std::logic_error& e) {
    h->err = e.what();
    return CCMI_E_STATE;
  } catch (std::exception& e) {
    h->err = e.what();
    return CCMI_E_INVALID;
  }
}
// Goal.actionAcceptance of the held goal of a kind: 0/1/2, or -1 with the message in oc_error
int32_t oc_action_acceptance_by_kind(void* hv, int32_t kind, const ccmi_action* a) {
  auto* h = (Handle*)hv;
  try {
    Goal* g = h->heldOf(kind);
    if (!g) throw std::invalid_argument("goal kind not held");
    BalancingAction ba;
    ba.type = (ActionType)a->type;
    ba.partition = a->partition;
    ba.sourceBroker = a->source_broker;
    ba.destinationBroker = a->destination_broker;
    ba.destPartition = a->destination_partition;
    ba.sourceDisk = a->source_disk;
    ba.destinationDisk = a->destination_disk;
    return (int32_t)g->actionAcceptance(ba, h->cm);
  } catch (std::exception& e) {
    h->err = e.what();
    return -1;
  }
}
const char* oc_error(void* hv) { return ((Handle*)hv)->err.c_str(); }
// CPU-baseline sampling: the next oc_optimize stops (status 99) once `seconds` of wall time have passed
void oc_set_deadline(void* hv, double seconds) {
  auto* h = (Handle*)hv;
  const double now = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  h->cm.deadline = seconds > 0 ? now + seconds : 0;
}
double oc_stats_seconds(void* hv) { return ((Handle*)hv)->cm.statsSeconds; }
double oc_last_seconds(void* hv) { return ((Handle*)hv)->last.seconds; }
int64_t oc_candidates(void* hv) { return ((Handle*)hv)->cm.candidatesEvaluated; }

// Apply externally decided actions (ClusterModel.relocateReplica / relocateLeadership / relocateReplica to a logdir)
// in order; returns 0 or CCMI_E_INVALID (message in oc_error).
void oc_last_failure_provision(void*, ccmi_provision_response* out) { toCProvision(lastFailureProvision(), out); }

int32_t oc_apply(void* hv, const ccmi_action* a, int64_t n) {
  auto* h = (Handle*)hv;
  ClusterModel& cm = h->cm;
  try {
    for (int64_t i = 0; i < n; ++i) {
      const ccmi_action& x = a[i];
      switch (x.type) {
        case CCMI_INTER_BROKER_REPLICA_MOVEMENT:
          cm.relocateReplica(x.partition, x.source_broker, x.destination_broker);
          break;
        case CCMI_LEADERSHIP_MOVEMENT:
          if (!cm.relocateLeadership(x.partition, x.source_broker, x.destination_broker))
            throw std::invalid_argument("source replica is not the leader");
          break;
        case CCMI_INTER_BROKER_REPLICA_SWAP:
          cm.relocateReplica(x.partition, x.source_broker, x.destination_broker);
          cm.relocateReplica(x.destination_partition, x.destination_broker, x.source_broker);
          break;
        case CCMI_INTRA_BROKER_REPLICA_MOVEMENT:
          cm.relocateReplicaToDisk(x.partition, x.source_broker, x.destination_disk);
          break;
        case CCMI_INTRA_BROKER_REPLICA_SWAP:
          cm.relocateReplicaToDisk(x.partition, x.source_broker, x.destination_disk);
          cm.relocateReplicaToDisk(x.destination_partition, x.source_broker, x.source_disk);
          break;
        default:
          throw std::invalid_argument("unknown action type");
      }
    }
    return 0;
  } catch (std::exception& e) {
    h->err = e.what();
    return CCMI_E_INVALID;
  }
}

// Goal.actionAcceptance of the gi-th goal of the last oc_optimize on the current model: 0/1/2 (ccmi_acceptance),
// or -1 with the message in oc_error (an action the goal does not support, an unknown replica)
int32_t oc_action_acceptance(void* hv, int32_t gi, const ccmi_action* a) {
  auto* h = (Handle*)hv;
  try {
    if (gi < 0 || gi >= (int32_t)h->last.optimizedGoals.size()) throw std::invalid_argument("goal index out of range");
    BalancingAction ba;
    ba.type = (ActionType)a->type;
    ba.partition = a->partition;
    ba.sourceBroker = a->source_broker;
    ba.destinationBroker = a->destination_broker;
    ba.destPartition = a->destination_partition;
    ba.sourceDisk = a->source_disk;
    ba.destinationDisk = a->destination_disk;
    return (int32_t)h->last.optimizedGoals[gi]->actionAcceptance(ba, h->cm);
  } catch (std::exception& e) {
    h->err = e.what();
    return -1;
  }
}

// TopicNameHashBrokerSetMappingPolicy's bucket for a topic among num_sets sorted broker set ids
int32_t oc_topic_broker_set(const char* topic, int32_t num_sets) {
  return num_sets < 1 ? -1 : topicNameHashBucket(topic, num_sets);
}

int64_t oc_action_count(void* hv) { return (int64_t)((Handle*)hv)->cm.actionLog.size(); }
void oc_actions(void* hv, ccmi_action* out) {
  auto* h = (Handle*)hv;
  for (size_t i = 0; i < h->cm.actionLog.size(); ++i) {
    const ActionRecord& a = h->cm.actionLog[i];
    out[i] = {a.type, a.partition, a.src, a.dst, a.destPartition, a.srcDisk, a.dstDisk};
  }
}
void oc_replica_distribution(void* hv, int32_t* out) {
  auto v = ((Handle*)hv)->cm.replicaDistributionFlat();
  std::memcpy(out, v.data(), v.size() * sizeof(int32_t));
}
void oc_leader_distribution(void* hv, int32_t* out) {
  auto v = ((Handle*)hv)->cm.leaderDistribution();
  std::memcpy(out, v.data(), v.size() * sizeof(int32_t));
}
void oc_stats(void* hv, const ccmi_balancing_constraint* c, const ccmi_opt_options* o, ccmi_cluster_stats* out) {
  auto* h = (Handle*)hv;
  toCStats(computeStats(h->cm, toBc(c), toOpts(o)), out);
}
int64_t oc_proposal_count(void* hv) { return (int64_t)((Handle*)hv)->last.proposals.size(); }
void oc_proposals(void* hv, int max_rf, int32_t* partition, int32_t* size, int32_t* old_leader, int32_t* old_out,
                  int32_t* new_out) {
  auto* h = (Handle*)hv;
  for (size_t i = 0; i < h->last.proposals.size(); ++i) {
    const Proposal& p = h->last.proposals[i];
    partition[i] = p.partition;
    size[i] = p.partitionSize;
    old_leader[i] = p.oldLeader;
    for (int k = 0; k < max_rf; ++k) {
      old_out[i * max_rf + k] = k < (int)p.oldReplicas.size() ? p.oldReplicas[k] : -1;
      new_out[i * max_rf + k] = k < (int)p.newReplicas.size() ? p.newReplicas[k] : -1;
    }
  }
}
void oc_proposal_disks(void* hv, int max_rf, int32_t* old_out, int32_t* new_out) {
  auto* h = (Handle*)hv;
  for (size_t i = 0; i < h->last.proposals.size(); ++i) {
    const Proposal& p = h->last.proposals[i];
    for (int k = 0; k < max_rf; ++k) {
      old_out[i * max_rf + k] = k < (int)p.oldDisks.size() ? p.oldDisks[k] : -1;
      new_out[i * max_rf + k] = k < (int)p.newDisks.size() ? p.newDisks[k] : -1;
    }
  }
}
// Replica utilization of broker b / resource (for host-side checks in tests).
double oc_broker_util(void* hv, int b, int res) { return ((Handle*)hv)->cm.brokerUtil(b, res); }
// Utilization of broker b's host (Broker.host().load().expectedUtilizationFor)
double oc_host_util(void* hv, int b, int res) { return ((Handle*)hv)->cm.hostUtil(b, res); }
// Exact RB-tree / PQ / Random probes for the known-answer tests.
int64_t oc_java_random_probe(int64_t seed, int bound, int n, int32_t* ints, double* doubles) {
  JRandom r(seed), r2(seed);
  for (int i = 0; i < n; ++i) ints[i] = r.nextInt(bound);
  for (int i = 0; i < n; ++i) doubles[i] = r2.nextDouble();
  return r.seed;
}
double oc_balance_threshold(double avg, int res, double balancePct, double lowUtil, double multiplier, int triggered,
                            double margin, int isLower) {
  BalancingConstraint bc;
  bc.resourceBalancePercentage[res] = balancePct;
  bc.lowUtilizationThreshold[res] = lowUtil;
  bc.goalViolationDistributionThresholdMultiplier = multiplier;
  return computeResourceUtilizationBalanceThreshold(avg, res, bc, triggered != 0, margin, isLower != 0);
}
}
