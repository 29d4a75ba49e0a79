// C ABI of libccmi.so (include/ccmi.h). Exceptions never cross the boundary: every entry point maps them to a
// ccmi_status and keeps the message for ccmi_last_error() (thread-local).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "ccmi.h"
#include "engine/buffers.h"
#include "engine/device.h"
#include "engine/engine.h"
#include "engine/model.h"
#include "engine/prof.h"
#include "engine/shard_rccl.h"
#include "engine/shard_shm.h"
#include "engine/threadpin.h"

namespace ccmi {
ccmi_cluster_buffers* generateRandomCluster(const ccmi_random_cluster_props& p);
}

struct ccmi_session;
struct ccmi_shard_group {
  ccmi::CombineBlock* blk = nullptr;
  int32_t count = 0;
  // attached sessions by rank; a destroyed session clears its slot and a destroyed group its sessions' back pointers,
  // so neither side is ever read after it is freed
  std::vector<ccmi_session*> ranks;
};
static void groupDetach(ccmi_session* s);

struct ccmi_session {
  ~ccmi_session() {
    groupDetach(this);
    ccmi::rcclDestroy(rccl);
    ccmi::shmDestroy(shm);
  }
  ccmi::Model model;
  std::unique_ptr<ccmi::Device> device;
  std::unique_ptr<ccmi::Engine> engine;
  ccmi::RcclShard* rccl = nullptr;
  ccmi::ShmShard* shm = nullptr;
  ccmi_shard_group* group = nullptr;  // the shard group this session is a rank of (ccmi_session_attach_group)
  int32_t groupRank = -1;
  int deviceOrdinal = 0;
  std::vector<int32_t> initDist, initLeaders;  // for ExecutionProposal diffs
  std::vector<int32_t> initDisks, initLeaderDisks;  // the logdir half of ReplicaPlacementInfo (JBOD)
  struct Prop {
    int32_t partition, size, oldLeader;
    std::vector<int32_t> oldR, newR, oldD, newD;
  };
  std::vector<Prop> proposals;
};

static void groupDetach(ccmi_session* s) {
  if (!s->group) return;
  auto& ranks = s->group->ranks;
  if ((size_t)s->groupRank < ranks.size() && ranks[(size_t)s->groupRank] == s) ranks[(size_t)s->groupRank] = nullptr;
  s->group = nullptr;
  s->groupRank = -1;
}

namespace {
thread_local std::string g_err;

ccmi_status fail(ccmi_status s, const std::string& msg) {
  g_err = msg;
  return s;
}

}  // namespace

namespace ccmi {
void setLastError(const std::string& msg) { g_err = msg; }
}  // namespace ccmi

namespace {

template <class F>
ccmi_status guarded(F&& f) {
  try {
    return f();
  } catch (ccmi::OptimizationFailure& e) {
    return fail(CCMI_E_OPT_FAILURE, e.what());
  } catch (ccmi::StateError& e) {
    return fail(CCMI_E_STATE, e.what());
  } catch (ccmi::Unsupported& e) {
    return fail(CCMI_E_UNSUPPORTED, e.what());
  } catch (std::invalid_argument& e) {
    return fail(CCMI_E_INVALID, e.what());
  } catch (std::exception& e) {
    const std::string w = e.what();
    return fail(w.rfind("HIP", 0) == 0 || w.find("gfx950") != std::string::npos || w.find("device") != std::string::npos
                    ? CCMI_E_DEVICE
                    : CCMI_E_INVALID,
                w);
  }
}

void setOptions(ccmi_session* s, const ccmi_balancing_constraint* c, const ccmi_opt_options* o) {
  ccmi::Engine& e = *s->engine;
  ccmi_balancing_constraint def;
  ccmi_default_constraint(&def);
  if (!c) c = &def;
  for (int r = 0; r < 4; ++r) {
    e.bc.resBalance[r] = c->resource_balance_percentage[r];
    e.bc.capThreshold[r] = c->capacity_threshold[r];
    e.bc.lowUtil[r] = c->low_utilization_threshold[r];
  }
  e.bc.replicaBalance = c->replica_balance_percentage;
  e.bc.goalViolationMultiplier = c->goal_violation_distribution_threshold_multiplier;
  e.bc.leaderReplicaBalance = c->leader_replica_balance_percentage;
  e.bc.topicReplicaBalance = c->topic_replica_balance_percentage;
  e.bc.topicMinGap = c->topic_replica_balance_min_gap;
  e.bc.topicMaxGap = c->topic_replica_balance_max_gap;
  e.bc.topicLeaderBalance = c->topic_leader_replica_balance_percentage;
  e.bc.topicLeaderMinGap = c->topic_leader_replica_balance_min_gap;
  e.bc.topicLeaderMaxGap = c->topic_leader_replica_balance_max_gap;
  e.bc.topicLeaderMargin = c->topic_leader_replica_balance_margin;
  e.bc.maxReplicasPerBroker = c->max_replicas_per_broker;
  e.bc.overMaxReplicasPerBroker = c->overprovisioned_max_replicas_per_broker;
  e.bc.overMinBrokers = c->overprovisioned_min_brokers;
  e.bc.overprovisionedMinExtraRacks = c->overprovisioned_min_extra_racks;
  e.brokerSets.resolve(c, s->model.bId);
  e.bc.minLeaderTopics.clear();
  if (c->num_min_leader_topics > 0 && !c->min_leader_topics) throw std::invalid_argument("null min_leader_topics");
  for (int i = 0; i < c->num_min_leader_topics; ++i) {
    const int t = c->min_leader_topics[i];
    if (t < 0 || t >= s->model.T) throw std::invalid_argument("min-leader topic out of range");
    e.bc.minLeaderTopics.push_back(t);
  }
  std::sort(e.bc.minLeaderTopics.begin(), e.bc.minLeaderTopics.end());
  e.bc.minLeaderTopics.erase(std::unique(e.bc.minLeaderTopics.begin(), e.bc.minLeaderTopics.end()),
                             e.bc.minLeaderTopics.end());
  if (c->min_topic_leaders_per_broker < 0) throw std::invalid_argument("min.topic.leaders.per.broker must be >= 0");
  e.bc.minTopicLeadersPerBroker = c->min_topic_leaders_per_broker;
  const int B = s->model.B;
  ccmi::Options opt;
  opt.exclMove.assign(B, 0);
  opt.exclLead.assign(B, 0);
  opt.requested.assign(B, 0);
  opt.exclTopic.assign(s->model.T, 0);
  if (o) {
    for (int i = 0; i < o->num_excluded_topics; ++i) {
      const int t = o->excluded_topics[i];
      if (t < 0 || t >= s->model.T) throw std::invalid_argument("excluded topic out of range");
      opt.exclTopic[t] = 1;
      opt.anyExclTopic = true;
    }
    // broker-id sets of OptimizationOptions: ids of brokers that are not in the cluster match nothing (Set.contains)
    for (int i = 0; i < o->num_excluded_brokers_for_leadership; ++i) {
      const int b = o->excluded_brokers_for_leadership[i];
      if (b < 0 || b >= B) continue;
      opt.exclLead[b] = 1;
      opt.anyExclLead = true;
    }
    for (int i = 0; i < o->num_excluded_brokers_for_replica_move; ++i) {
      const int b = o->excluded_brokers_for_replica_move[i];
      if (b < 0 || b >= B) continue;
      opt.exclMove[b] = 1;
      opt.anyExclMove = true;
    }
    opt.onlyImmigrants = o->only_move_immigrant_replicas != 0;
    for (int i = 0; i < o->num_requested_destination_broker_ids; ++i) {
      opt.anyRequested = true;  // a non-empty set filters candidates even when none of its ids is a broker
      const int b = o->requested_destination_broker_ids[i];
      if (b < 0 || b >= B) continue;
      opt.requested[b] = 1;
    }
    opt.triggered = o->triggered_by_goal_violation != 0;
  }
  e.opt = std::move(opt);
  s->model.setExcludedTopicSelection(e.opt.exclTopic);
  std::vector<uint8_t> must(s->model.T, 0);
  for (int t : e.bc.minLeaderTopics) must[t] = 1;
  s->model.setMustTopicSelection(must);
}

// The scan server (device.h) never outlives the API call that started it.
struct StopServerOnExit {
  ccmi_session* s;
  ~StopServerOnExit() {
    try {
      if (s && s->device) s->device->stopServer();
    } catch (std::exception&) {
    }
  }
};
// An optimization call in progress on the session's device: concurrent calls share the device's scan-server budget
// (Device::ensureServer). Declared before StopServerOnExit, so the server is stopped before the call stops counting.
struct ActiveCall {
  ccmi_session* s;
  explicit ActiveCall(ccmi_session* x) : s(x) { s->device->callBegin(); }
  ~ActiveCall() { s->device->callEnd(); }
  ActiveCall(const ActiveCall&) = delete;
  ActiveCall& operator=(const ActiveCall&) = delete;
};

std::vector<int32_t> replicaDist(const ccmi::Model& m) {
  std::vector<int32_t> v(m.R);
  for (int i = 0; i < m.R; ++i) v[i] = m.rBroker[m.pSlots[i]];
  return v;
}
std::vector<int32_t> leaderDist(const ccmi::Model& m) {
  std::vector<int32_t> v(m.P);
  for (int p = 0; p < m.P; ++p) v[p] = m.rBroker[m.pLeader[p]];
  return v;
}
std::vector<int32_t> leaderDiskDist(const ccmi::Model& m) {
  std::vector<int32_t> v(m.P);
  for (int p = 0; p < m.P; ++p) v[p] = m.rDisk[m.pLeader[p]];
  return v;
}
// ClusterModel.getReplicaDistribution / getLeaderDistribution with ReplicaPlacementInfo(broker, logdir)
struct Placement {
  std::vector<int32_t> dist, leaders, disks, leaderDisks;
  explicit Placement(const ccmi::Model& m)
      : dist(replicaDist(m)), leaders(leaderDist(m)), disks(m.replicaDisks()), leaderDisks(leaderDiskDist(m)) {}
  bool operator!=(const Placement& o) const {
    return dist != o.dist || leaders != o.leaders || disks != o.disks || leaderDisks != o.leaderDisks;
  }
};

// A chain is either broker-granularity or disk-granularity: each kind's actionAcceptance rejects the other's actions
// with IllegalArgumentException (e.g. ResourceDistributionGoal.actionAcceptance default branch,
// IntraBrokerDiskCapacityGoal.actionAcceptance :120-124), so a mixed chain is refused up front.
void validateChain(const ccmi_session* s, const int32_t* kinds, int n, const std::vector<ccmi::GoalImpl*>& priors = {}) {
  int intra = 0;
  for (int i = 0; i < n; ++i) intra += ccmi::isIntraGoalKind(kinds[i]) ? 1 : 0;
  for (const ccmi::GoalImpl* g : priors) intra += ccmi::isIntraGoalKind(g->kind) ? 1 : 0;
  const int total = n + (int)priors.size();
  if (intra != 0 && intra != total)
    throw std::invalid_argument("intra-broker goals cannot be optimized together with inter-broker goals");
}

// AnalyzerUtils.getDiff (AnalyzerUtils.java:63-93) against the session's initial placement
void buildProposals(ccmi_session* s) {
  const ccmi::Model& m = s->model;
  s->proposals.clear();
  const std::vector<int32_t> fin = replicaDist(m), finD = m.replicaDisks();
  for (int p = 0; p < m.P; ++p) {
    const int a = m.pOff[p], n = m.pOff[p + 1] - a;
    std::vector<int32_t> oldR(s->initDist.begin() + a, s->initDist.begin() + a + n);
    std::vector<int32_t> newR(fin.begin() + a, fin.begin() + a + n);
    std::vector<int32_t> oldD(s->initDisks.begin() + a, s->initDisks.begin() + a + n);
    std::vector<int32_t> newD(finD.begin() + a, finD.begin() + a + n);
    const int finalLeader = m.rBroker[m.pLeader[p]], finalLeaderDisk = m.rDisk[m.pLeader[p]];
    if (oldR == newR && oldD == newD && s->initLeaders[p] == finalLeader && s->initLeaderDisks[p] == finalLeaderDisk)
      continue;
    int pos = 0;  // finalReplicas.indexOf(finalLeaderPlacementInfo), then swapped with slot 0
    for (int k = 0; k < n; ++k)
      if (newR[k] == finalLeader && newD[k] == finalLeaderDisk) {
        pos = k;
        break;
      }
    std::swap(newR[pos], newR[0]);
    std::swap(newD[pos], newD[0]);
    s->proposals.push_back({p, (int32_t)m.ru(m.pLeader[p], ccmi::R_DISK), s->initLeaders[p], oldR, newR, oldD, newD});
  }
}
}  // namespace

extern "C" {

const char* ccmi_last_error(void) { return g_err.c_str(); }
int32_t ccmi_abi_version(void) { return CCMI_ABI_VERSION; }
int32_t ccmi_device_count(void) {
  try {
    return ccmi::Device::countGfx950();
  } catch (std::exception&) {
    return 0;
  }
}

int32_t ccmi_topic_broker_set(const char* topic, int32_t num_broker_sets) {
  if (!topic) return -1;
  return ccmi::bsets::topicBrokerSet(topic, num_broker_sets);
}

void ccmi_default_constraint(ccmi_balancing_constraint* c) {
  std::memset(c, 0, sizeof(*c));
  for (int r = 0; r < 4; ++r) {
    c->resource_balance_percentage[r] = 1.10;
    c->capacity_threshold[r] = r == CCMI_CPU ? 0.7 : 0.8;
    c->low_utilization_threshold[r] = 0.0;
  }
  c->replica_balance_percentage = 1.10;
  c->leader_replica_balance_percentage = 1.10;
  c->topic_replica_balance_percentage = 3.00;
  c->topic_replica_balance_min_gap = 2;
  c->topic_replica_balance_max_gap = 40;
  c->goal_violation_distribution_threshold_multiplier = 1.0;
  c->max_replicas_per_broker = 10000;
  c->overprovisioned_max_replicas_per_broker = 1500;
  c->overprovisioned_min_brokers = 3;
  c->overprovisioned_min_extra_racks = 2;
  c->min_topic_leaders_per_broker = 1;  // AnalyzerConfig.DEFAULT_MIN_TOPIC_LEADERS_PER_BROKER
  c->topic_leader_replica_balance_percentage = 1.10;  // AnalyzerConfig.java:112-146
  c->topic_leader_replica_balance_min_gap = 2;
  c->topic_leader_replica_balance_max_gap = 10;
  c->topic_leader_replica_balance_margin = 0.9;
}

void ccmi_default_random_cluster_props(ccmi_random_cluster_props* p) {
  std::memset(p, 0, sizeof(*p));
  p->num_racks = 10;
  p->num_brokers = 40;
  p->num_replicas = 50001;
  p->num_topics = 3000;
  p->min_replication = 3;
  p->max_replication = 3;
  p->mean_cpu = 0.01;
  p->mean_disk = 100.0;
  p->mean_nw_in = 100.0;
  p->mean_nw_out = 100.0;
  p->distribution = 0;
  p->rack_aware = 0;
  p->leader_in_first_position = 1;
}

ccmi_status ccmi_random_cluster(const ccmi_random_cluster_props* props, ccmi_cluster_buffers** out) {
  return guarded([&] {
    if (!props || !out) throw std::invalid_argument("null argument");
    *out = ccmi::generateRandomCluster(*props);
    return CCMI_OK;
  });
}
const ccmi_cluster_desc* ccmi_cluster_buffers_desc(const ccmi_cluster_buffers* buf) { return buf ? &buf->desc : nullptr; }
void ccmi_cluster_buffers_free(ccmi_cluster_buffers* buf) { delete buf; }

ccmi_status ccmi_session_create(int32_t device_ordinal, const ccmi_cluster_desc* desc, ccmi_session** out) {
  return guarded([&] {
    if (!desc || !out) throw std::invalid_argument("null argument");
    const ccmi::ThreadPin pin(device_ordinal);  // the session's host memory is first touched on the GPU's node
    auto s = std::make_unique<ccmi_session>();
    s->model.build(*desc);
    ccmi::Model& m = s->model;
    s->device = std::make_unique<ccmi::Device>(device_ordinal, m.B, m.R, m.P, m.T, ccmi::kMaxSlots);
    s->device->setRowSource(m.rBroker.data(), m.rPart.data(), m.pTopic.data());
    s->deviceOrdinal = device_ordinal;
    // device layout: resource-major broker/replica columns
    std::vector<double> capRM((size_t)4 * m.B), utilRM((size_t)4 * m.B), rutilRM((size_t)4 * m.R), pot(m.B);
    std::vector<double> lbi(m.B), plno(m.P);
    std::vector<int32_t> nrep(m.B), pBrokers(m.R);
    std::vector<uint8_t> alive(m.B), flags(m.R);
    for (int b = 0; b < m.B; ++b) {
      for (int k = 0; k < 4; ++k) {
        capRM[(size_t)k * m.B + b] = m.cap(b, k);
        utilRM[(size_t)k * m.B + b] = m.bu(b, k);
      }
      nrep[b] = m.nrep(b);
      alive[b] = m.alive(b);
      pot[b] = m.potNwOut(b);
      lbi[b] = m.leadNwIn(b);
    }
    for (int p = 0; p < m.P; ++p) plno[p] = m.pLeadNwOut(p);
    for (int r = 0; r < m.R; ++r) {
      for (int k = 0; k < 4; ++k) rutilRM[(size_t)k * m.R + r] = m.ru(r, k);
      flags[r] = (m.rLeader[r] ? ccmi::RF_LEADER : 0) | (m.rOrigOff[r] ? ccmi::RF_ORIG_OFFLINE : 0);
    }
    for (int i = 0; i < m.R; ++i) pBrokers[i] = m.rBroker[m.pSlots[i]];
    s->device->uploadStatic(capRM.data(), m.rPart.data(), m.rOrig.data(), m.pOff.data(), m.topicNrep.data(),
                            m.bRack.data(), m.pTopic.data());
    s->device->uploadIneligible(m.pIneligOff.data(), m.pIneligB.data(), (int)m.pIneligB.size());
    s->device->uploadDynamic(utilRM.data(), nrep.data(), m.bNlead.data(), pot.data(), lbi.data(), alive.data(),
                             rutilRM.data(), m.rBroker.data(), flags.data(), pBrokers.data(), plno.data(),
                             m.topicCountDense.data());
    s->device->uploadLoads(m.W, m.rLoad.data(), m.bLoad.data(), m.bLnw.data(), m.bPot.data(), m.pSlots.data(),
                           m.pLeader.data());
    if (m.D > 0) {
      std::vector<uint8_t> bAlive(m.B), dAlive(m.dAlive);
      std::vector<double> rDu(m.R);
      std::vector<float> rScore(m.R);
      for (int b = 0; b < m.B; ++b) bAlive[b] = m.alive(b) ? 1 : 0;
      for (int r = 0; r < m.R; ++r) {
        rDu[r] = m.ru(r, ccmi::R_DISK);
        rScore[r] = m.rScoreC[4 * (size_t)r + ccmi::R_DISK];
      }
      s->device->uploadDisks(m.D, m.bDiskOff.data(), m.bDisks.data(), m.dCap.data(), dAlive.data(), bAlive.data(),
                             m.rOrigDisk.data(), rDu.data(), rScore.data(), m.rStatic.data());
      s->device->setDiskUtil(m.dUtil.data());
      m.diskDirty = false;
    }
    if (m.sharedHosts) {  // Host._load for the chain kernels' moves, with each host's brokers (CSR)
      std::vector<int32_t> hOff(1, 0), hBrk;
      for (int h = 0; h < m.H; ++h) {
        hBrk.insert(hBrk.end(), m.hBrokers[h].begin(), m.hBrokers[h].end());
        hOff.push_back((int32_t)hBrk.size());
      }
      s->device->uploadHostLoads(m.H, m.hLoad.data(), m.bHost.data(), hOff.data(), hBrk.data());
    }
    if (m.sharedHosts) {  // every broker's host utilization and capacity of the host resources
      std::vector<double> hu((size_t)3 * m.B), hc((size_t)3 * m.B);
      for (int b = 0; b < m.B; ++b)
        for (int k = 0; k < 3; ++k) {
          hu[3 * (size_t)b + k] = m.hu(b, k);
          hc[3 * (size_t)b + k] = m.hcap(b, k);
        }
      s->device->uploadHosts(hu.data(), hc.data());
    }
    m.dev = s->device.get();
    s->engine = std::make_unique<ccmi::Engine>(m, s->device.get());
    s->initDist = replicaDist(m);
    s->initLeaders = leaderDist(m);
    s->initDisks = m.replicaDisks();
    s->initLeaderDisks = leaderDiskDist(m);
    *out = s.release();
    return CCMI_OK;
  });
}

ccmi_status ccmi_session_set_shard(ccmi_session* s, int32_t rank, int32_t count, ccmi_allreduce_min_fn fn, void* ctx) {
  return guarded([&] {
    if (!s) throw std::invalid_argument("null session");
    if (count < 1 || rank < 0 || rank >= count) throw std::invalid_argument("shard rank out of range");
    if (count > 1 && !fn) throw std::invalid_argument("a sharded session needs a combiner");
    s->engine->shard = ccmi::Shard{rank, count, fn, ctx};
    // a combiner makes every scan wait for other ranks (or a collective kernel): a resident server could hold the
    // hardware queue those need, so a combined session launches per scan
    s->device->setServerAllowed(fn == nullptr);
    return CCMI_OK;
  });
}

ccmi_status ccmi_rccl_unique_id(uint8_t out[128]) {
  return guarded([&] {
    if (!out) throw std::invalid_argument("null argument");
    if (!ccmi::rcclUniqueId(out)) throw std::runtime_error("RCCL device error: ncclGetUniqueId failed");
    return CCMI_OK;
  });
}

ccmi_status ccmi_session_attach_rccl(ccmi_session* s, int32_t rank, int32_t count, const uint8_t unique_id[128]) {
  return guarded([&] {
    if (!s || !unique_id) throw std::invalid_argument("null argument");
    if (count < 1 || rank < 0 || rank >= count) throw std::invalid_argument("shard rank out of range");
    ccmi::rcclDestroy(s->rccl);
    s->rccl = nullptr;
    s->rccl = ccmi::rcclCreate(s->deviceOrdinal, rank, count, unique_id);
    s->engine->shard = ccmi::Shard{rank, count, &ccmi::rcclMin, s->rccl};
    s->device->setServerAllowed(false);  // the collective kernels must not queue behind a resident server
    return CCMI_OK;
  });
}

ccmi_status ccmi_session_attach_shm(ccmi_session* s, int32_t rank, int32_t count, const char* name) {
  return ccmi_session_attach_shm_job(s, rank, count, name, 0, 0.0);
}

ccmi_status ccmi_session_attach_shm_job(ccmi_session* s, int32_t rank, int32_t count, const char* name,
                                        uint64_t job_nonce, double timeout_s) {
  return guarded([&] {
    if (!s || !name) throw std::invalid_argument("null argument");
    if (count < 1 || rank < 0 || rank >= count) throw std::invalid_argument("shard rank out of range");
    if (!(timeout_s >= 0.0)) throw std::invalid_argument("negative timeout");
    ccmi::shmDestroy(s->shm);
    s->shm = nullptr;
    s->shm = ccmi::shmCreate(name, rank, count, timeout_s > 0.0 ? timeout_s : 120.0, job_nonce);
    s->engine->shard = ccmi::Shard{rank, count, &ccmi::shmMin, s->shm};
    s->device->setServerAllowed(true);  // the combine is host memory only: the scan server stays resident
    return CCMI_OK;
  });
}

namespace {

// The queue-scan path is decided group-wide: every rank must run the same scans so that the combines (made by the
// queue path's fallbacks, never by a queue scan itself) pair up. It is allowed only when every rank is attached and
// every rank's device can serve queue scans; recomputed for all attached ranks at each attach.
void groupQueueDecision(ccmi_shard_group* g) {
  bool all = true;
  for (ccmi_session* x : g->ranks) all = all && x && x->device->queueUsable();
  for (ccmi_session* x : g->ranks)
    if (x) x->engine->shardQueueAllowed = all;
}

// the shard-group combiner for scans the scan server did not combine (shard_group.h): the host side of the protocol
int groupMin(void* ctx, int64_t* key) {
  try {
    auto* dev = static_cast<ccmi::Device*>(ctx);
    const int64_t g = dev->groupCombineHost(*key == INT64_MAX ? -1 : *key);
    *key = g < 0 ? INT64_MAX : g;
    return 0;
  } catch (std::exception&) {
    return 1;
  }
}
}  // namespace

ccmi_status ccmi_shard_group_create(int32_t count, ccmi_shard_group** out) {
  return guarded([&] {
    if (!out) throw std::invalid_argument("null argument");
    if (count < 1 || count > ccmi::kGroupMaxRanks) throw std::invalid_argument("shard count out of range");
    auto g = std::make_unique<ccmi_shard_group>();
    g->blk = ccmi::Device::allocCombineBlock();
    g->count = count;
    *out = g.release();
    return CCMI_OK;
  });
}

ccmi_status ccmi_shard_group_destroy(ccmi_shard_group* g) {
  return guarded([&] {
    if (g) {
      for (ccmi_session* x : g->ranks)
        if (x) {
          x->group = nullptr;
          x->groupRank = -1;
        }
      ccmi::Device::freeCombineBlock(g->blk);
    }
    delete g;
    return CCMI_OK;
  });
}

ccmi_status ccmi_session_attach_group(ccmi_session* s, ccmi_shard_group* g, int32_t rank) {
  return guarded([&] {
    if (!s || !g) throw std::invalid_argument("null argument");
    if (rank < 0 || rank >= g->count) throw std::invalid_argument("shard rank out of range");
    s->device->attachGroup(g->blk, g->count, rank);
    s->engine->shard = ccmi::Shard{rank, g->count, &groupMin, s->device.get()};
    s->device->setServerAllowed(true);  // the server combines on the device: it stays resident
    // Ranks sharing a GPU: a kernel one rank launches can wait behind another rank's persistent server (hardware queues
    // and CU slots are per device), while that server's command waits for the launching rank's arrival. Such ranks
    // launch per scan and combine on their host threads; CCMI_GROUP_SHARED_SERVERS=1 instead gives each of them a
    // server with an equal share of the device's workgroup budget (tests of the device-side combine on one GPU).
    if (g->ranks.size() != (size_t)g->count) g->ranks.resize((size_t)g->count, nullptr);
    if (g->ranks[(size_t)rank] && g->ranks[(size_t)rank] != s) throw std::invalid_argument("shard rank already attached");
    groupDetach(s);
    g->ranks[(size_t)rank] = s;
    s->group = g;
    s->groupRank = rank;
    std::vector<ccmi_session*> same;
    for (ccmi_session* x : g->ranks)
      if (x && x->deviceOrdinal == s->deviceOrdinal) same.push_back(x);
    if (same.size() > 1) {
      const bool shared = std::getenv("CCMI_GROUP_SHARED_SERVERS") && std::getenv("CCMI_GROUP_SHARED_SERVERS")[0] == '1';
      for (ccmi_session* x : same) {
        if (shared) x->device->limitServerBlocks((int)(256 / same.size()) / 8 * 8);
        else x->device->setServerAllowed(false);
      }
    }
    groupQueueDecision(g);
    return CCMI_OK;
  });
}

ccmi_status ccmi_session_destroy(ccmi_session* s) {
  return guarded([&] {
    ccmi::prof().print("session");
    ccmi::prof() = ccmi::PhaseProf();
    delete s;
    return CCMI_OK;
  });
}

ccmi_status ccmi_goal_optimize(ccmi_session* s, int32_t goal_kind, const int32_t* optimized_goal_kinds,
                               int32_t num_optimized_goals, const ccmi_balancing_constraint* c,
                               const ccmi_opt_options* o, ccmi_goal_result* result) {
  return guarded([&] {
    if (!s) throw std::invalid_argument("null session");
    if (num_optimized_goals < 0 || (num_optimized_goals > 0 && !optimized_goal_kinds))
      throw std::invalid_argument("null optimized_goal_kinds");
    // Set<Goal> optimizedGoals: each kind resolves to the session's own optimization of it (its frozen state); a goal
    // the session does not hold (run in the JVM, or a JVM-only goal class) cannot join the device conjunction
    std::vector<ccmi::GoalImpl*> priors;
    for (int i = 0; i < num_optimized_goals; ++i) {
      ccmi::GoalImpl* g = s->engine->optimizedOfKind(optimized_goal_kinds[i]);
      if (!g)
        throw ccmi::Unsupported("optimized goal kind " + std::to_string(optimized_goal_kinds[i]) +
                                " has not been optimized by this session: its actionAcceptance is not available here");
      if (std::find(priors.begin(), priors.end(), g) == priors.end()) priors.push_back(g);
    }
    auto g = ccmi::makeGoal(goal_kind);
    const ccmi::ThreadPin pin(s->deviceOrdinal);  // restored when the call returns
    const ActiveCall active(s);
    StopServerOnExit stop{s};
    setOptions(s, c, o);
    validateChain(s, &goal_kind, 1, priors);
    ccmi_goal_result tmp;
    std::memset(&tmp, 0, sizeof(tmp));
    const Placement pre(s->model);
    s->engine->optimizeGoal(std::move(g), priors, &tmp);
    tmp.has_diff = Placement(s->model) != pre ? 1 : 0;
    if (result) *result = tmp;
    buildProposals(s);
    return CCMI_OK;
  });
}

ccmi_status ccmi_optimizations(ccmi_session* s, const int32_t* goal_kinds, int32_t n_goals,
                               const ccmi_balancing_constraint* c, const ccmi_opt_options* o, ccmi_goal_result* results) {
  return guarded([&] {
    if (!s || (!goal_kinds && n_goals > 0)) throw std::invalid_argument("null argument");
    if (n_goals <= 0) throw std::invalid_argument("At least one goal must be provided to get an optimization result.");
    const ccmi::ThreadPin pin(s->deviceOrdinal);  // restored when the call returns
    const ActiveCall active(s);
    StopServerOnExit stop{s};
    setOptions(s, c, o);
    validateChain(s, goal_kinds, n_goals);
    for (int i = 0; i < n_goals; ++i) (void)ccmi::makeGoal(goal_kinds[i]);  // fail fast on unsupported kinds
    // optimizedGoals starts empty for every call (GoalOptimizer.java:449) and collects this call's goals (:471)
    std::vector<int32_t> done;
    for (int i = 0; i < n_goals; ++i) {
      ccmi_goal_result tmp;
      std::memset(&tmp, 0, sizeof(tmp));
      const Placement pre(s->model);
      std::vector<ccmi::GoalImpl*> priors;
      for (int32_t k : done) priors.push_back(s->engine->optimizedOfKind(k));
      s->engine->optimizeGoal(ccmi::makeGoal(goal_kinds[i]), priors, &tmp);
      if (std::find(done.begin(), done.end(), goal_kinds[i]) == done.end()) done.push_back(goal_kinds[i]);
      tmp.has_diff = Placement(s->model) != pre ? 1 : 0;
      if (results) results[i] = tmp;
    }
    buildProposals(s);
    return CCMI_OK;
  });
}

ccmi_status ccmi_action_acceptance(ccmi_session* s, int32_t idx, const ccmi_action* a, int32_t* acceptance) {
  return guarded([&] {
    if (!s || !a || !acceptance) throw std::invalid_argument("null argument");
    if (idx < 0 || idx >= (int)s->engine->optimized.size()) throw std::invalid_argument("optimized goal index out of range");
    *acceptance = s->engine->acceptance(idx, *a);
    return CCMI_OK;
  });
}

ccmi_status ccmi_last_failure_provision(const ccmi_session* s, ccmi_provision_response* out) {
  return guarded([&] {
    if (!s || !out) throw std::invalid_argument("null argument");
    *out = s->engine->lastFailure;
    return CCMI_OK;
  });
}

ccmi_status ccmi_action_acceptance_by_kind(ccmi_session* s, int32_t kind, const ccmi_action* a, int32_t* acceptance) {
  return guarded([&] {
    if (!s || !a || !acceptance) throw std::invalid_argument("null argument");
    const auto& opt = s->engine->optimized;
    for (int i = (int)opt.size() - 1; i >= 0; --i)
      if (opt[i]->kind == kind) {
        *acceptance = s->engine->acceptance(i, *a);
        return CCMI_OK;
      }
    throw std::invalid_argument("the session has not optimized goal kind " + std::to_string(kind));
  });
}

ccmi_status ccmi_session_apply(ccmi_session* s, const ccmi_action* actions, int64_t n, int64_t* applied) {
  if (applied) *applied = 0;
  // the proposals are the diff against the initial placement after every action applied, also when a later one fails
  const ccmi_status st = [&] {
    return guarded([&] {
      if (!s || (n > 0 && !actions) || n < 0) throw std::invalid_argument("null argument");
      ccmi::Model& m = s->model;
      auto partition = [&](int p) {
        if (p < 0 || p >= m.P) throw std::invalid_argument("partition out of range");
      };
      auto broker = [&](int b) {
        if (b < 0 || b >= m.B) throw std::invalid_argument("broker out of range");
      };
      auto movable = [&](int p, int src, int dst) {  // ClusterModel.relocateReplica preconditions
        partition(p);
        broker(src);
        broker(dst);
        if (m.replicaOn(p, src) < 0) throw std::invalid_argument("source broker does not host the partition");
        if (m.replicaOn(p, dst) >= 0) throw std::invalid_argument("destination broker already hosts the partition");
      };
      auto diskMove = [&](int p, int b, int sd, int dd) {
        partition(p);
        broker(b);
        const int r = m.replicaOn(p, b);
        if (r < 0) throw std::invalid_argument("broker does not host the partition");
        if (sd < 0 || sd >= m.D || dd < 0 || dd >= m.D || m.dBroker[sd] != b || m.dBroker[dd] != b)
          throw std::invalid_argument("disk out of range or not on the broker");
        if (m.rDisk[r] != sd) throw std::invalid_argument("replica is not on the source disk");
        m.relocateReplicaToDisk(p, b, dd);
      };
      for (int64_t i = 0; i < n; ++i) {
        const ccmi_action& a = actions[i];
        switch (a.type) {
          case CCMI_INTER_BROKER_REPLICA_MOVEMENT:
            movable(a.partition, a.source_broker, a.destination_broker);
            m.relocateReplica(a.partition, a.source_broker, a.destination_broker);
            break;
          case CCMI_LEADERSHIP_MOVEMENT: {
            partition(a.partition);
            broker(a.source_broker);
            broker(a.destination_broker);
            const int sr = m.replicaOn(a.partition, a.source_broker), dr = m.replicaOn(a.partition, a.destination_broker);
            if (sr < 0 || !m.rLeader[sr]) throw std::invalid_argument("source replica is not the leader");
            if (dr < 0 || m.rLeader[dr]) throw std::invalid_argument("destination broker hosts no follower of the partition");
            m.relocateLeadership(a.partition, a.source_broker, a.destination_broker);
            break;
          }
          case CCMI_INTER_BROKER_REPLICA_SWAP:
            movable(a.partition, a.source_broker, a.destination_broker);
            partition(a.destination_partition);
            if (m.replicaOn(a.destination_partition, a.destination_broker) < 0 ||
                m.replicaOn(a.destination_partition, a.source_broker) >= 0)
              throw std::invalid_argument("swap destination replica cannot move to the source broker");
            m.relocateReplica(a.partition, a.source_broker, a.destination_broker);
            m.relocateReplica(a.destination_partition, a.destination_broker, a.source_broker);
            break;
          case CCMI_INTRA_BROKER_REPLICA_MOVEMENT:
            diskMove(a.partition, a.source_broker, a.source_disk, a.destination_disk);
            break;
          case CCMI_INTRA_BROKER_REPLICA_SWAP: {
            partition(a.destination_partition);
            const int r2 = m.replicaOn(a.destination_partition, a.source_broker);
            if (r2 < 0 || m.rDisk[r2] != a.destination_disk)
              throw std::invalid_argument("swap destination replica is not on the destination disk");
            diskMove(a.partition, a.source_broker, a.source_disk, a.destination_disk);
            diskMove(a.destination_partition, a.source_broker, a.destination_disk, a.source_disk);
            break;
          }
          default:
            throw std::invalid_argument("unknown action type");
        }
        if (applied) *applied = i + 1;
      }
      return CCMI_OK;
    });
  }();
  try {
    if (s) buildProposals(s);
  } catch (std::exception& e) {
    // a rejected action's message (the last error when st != OK) stays first
    const std::string msg = std::string("rebuilding the proposals failed: ") + e.what();
    return fail(st == CCMI_OK ? CCMI_E_INVALID : st, st == CCMI_OK ? msg : g_err + "; " + msg);
  }
  return st;
}

ccmi_status ccmi_compute_cluster_stats(ccmi_session* s, const ccmi_balancing_constraint* c, const ccmi_opt_options* o,
                                       ccmi_cluster_stats* out) {
  return guarded([&] {
    if (!s || !out) throw std::invalid_argument("null argument");
    setOptions(s, c, o);
    *out = s->engine->stats();
    return CCMI_OK;
  });
}

int64_t ccmi_action_log_count(const ccmi_session* s) { return s ? (int64_t)s->model.log.size() : 0; }

ccmi_status ccmi_action_log_copy(const ccmi_session* s, int64_t first, int64_t count, ccmi_action* out) {
  return guarded([&] {
    if (!s || !out) throw std::invalid_argument("null argument");
    if (first < 0 || count < 0 || first + count > (int64_t)s->model.log.size()) throw std::invalid_argument("range");
    for (int64_t i = 0; i < count; ++i) {
      const ccmi::ActionRec& a = s->model.log[first + i];
      out[i] = {a.type, a.partition, a.src, a.dst, a.destPartition, a.srcDisk, a.dstDisk};
    }
    return CCMI_OK;
  });
}

ccmi_status ccmi_replica_distribution(const ccmi_session* s, int32_t* out) {
  return guarded([&] {
    if (!s || !out) throw std::invalid_argument("null argument");
    const auto v = replicaDist(s->model);
    std::memcpy(out, v.data(), v.size() * sizeof(int32_t));
    return CCMI_OK;
  });
}

ccmi_status ccmi_leader_distribution(const ccmi_session* s, int32_t* out) {
  return guarded([&] {
    if (!s || !out) throw std::invalid_argument("null argument");
    const auto v = leaderDist(s->model);
    std::memcpy(out, v.data(), v.size() * sizeof(int32_t));
    return CCMI_OK;
  });
}

ccmi_status ccmi_replica_disks(const ccmi_session* s, int32_t* out) {
  return guarded([&] {
    if (!s || !out) throw std::invalid_argument("null argument");
    const auto v = s->model.replicaDisks();
    std::memcpy(out, v.data(), v.size() * sizeof(int32_t));
    return CCMI_OK;
  });
}

int64_t ccmi_proposal_count(const ccmi_session* s) { return s ? (int64_t)s->proposals.size() : 0; }

ccmi_status ccmi_proposal_disks(const ccmi_session* s, int32_t max_rf, int32_t* old_disk_out, int32_t* new_disk_out) {
  return guarded([&] {
    if (!s || !old_disk_out || !new_disk_out) throw std::invalid_argument("null argument");
    for (size_t i = 0; i < s->proposals.size(); ++i) {
      const auto& p = s->proposals[i];
      for (int k = 0; k < max_rf; ++k) {
        old_disk_out[i * max_rf + k] = k < (int)p.oldD.size() ? p.oldD[k] : -1;
        new_disk_out[i * max_rf + k] = k < (int)p.newD.size() ? p.newD[k] : -1;
      }
    }
    return CCMI_OK;
  });
}

ccmi_status ccmi_proposals(const ccmi_session* s, int32_t max_rf, int32_t* partition, int32_t* size,
                           int32_t* old_leader, int32_t* old_out, int32_t* new_out) {
  return guarded([&] {
    if (!s) throw std::invalid_argument("null session");
    for (size_t i = 0; i < s->proposals.size(); ++i) {
      const auto& p = s->proposals[i];
      partition[i] = p.partition;
      size[i] = p.size;
      old_leader[i] = p.oldLeader;
      for (int k = 0; k < max_rf; ++k) {
        old_out[i * max_rf + k] = k < (int)p.oldR.size() ? p.oldR[k] : -1;
        new_out[i * max_rf + k] = k < (int)p.newR.size() ? p.newR[k] : -1;
      }
    }
    return CCMI_OK;
  });
}

ccmi_status ccmi_perf(const ccmi_session* s, ccmi_perf_counters* out) {
  return guarded([&] {
    if (!s || !out) throw std::invalid_argument("null argument");
    s->device->collectServerBusy();
    const auto& p = s->device->perf;
    out->scan_launches = p.scanLaunches;
    out->scan_kernel_ms = p.scanKernelMs;
    out->scan_bytes = p.scanBytes;
    out->stats_launches = p.statsLaunches;
    out->stats_kernel_ms = p.statsKernelMs;
    out->stats_bytes = p.statsBytes;
    out->host_syncs = p.syncs;
    out->scan_required = p.scanRequired;
    out->chain_launches = p.chainLaunches;
    out->intra_launches = p.intraLaunches;
    out->intra_kernel_ms = p.intraKernelMs;
    out->intra_sort_launches = p.intraSorts;
    out->intra_sort_ms = p.intraSortMs;
    out->intra_bytes = p.intraBytes;
    out->cross_launches = p.crossLaunches;
    out->cross_required = p.crossRequired;
    out->cross_kernel_ms = p.crossKernelMs;
    out->combines = p.combines;
    out->server_launches = p.serverLaunches;
    out->server_scans = p.serverScans;
    out->server_required = p.serverRequired;
    out->server_busy_ms = p.serverBusyMs;
    out->server_payload_bytes = p.serverPayloadBytes;
    out->server_chains = p.serverChains;
    out->server_idle_exits = p.serverIdleExits;
    out->server_resident_ms = p.serverResidentMs;
    return CCMI_OK;
  });
}

void ccmi_perf_reset(ccmi_session* s) {
  if (s) {
    s->device->collectServerBusy();
    s->device->perf = ccmi::DevicePerf();
  }
}

void ccmi_set_kernel_timing(ccmi_session* s, int32_t enabled) {
  if (s) s->device->timing = enabled != 0;
}

}  // extern "C"
