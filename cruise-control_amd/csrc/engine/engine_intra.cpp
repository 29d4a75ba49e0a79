// Intra-broker (JBOD) goals: IntraBrokerDiskCapacityGoal and IntraBrokerDiskUsageDistributionGoal.
// The host keeps AbstractGoal.optimize's frame (initGoalState, updateGoalState, the regression check in
// Engine::optimizeGoal); the broker loop is one K6 launch (intra.h, kernels/intra.hip) whose per-broker action records
// the host replays, in broker-id order, into its model (ClusterModel.relocateReplica(tp, broker, logdir)).
//   IntraBrokerDiskCapacityGoal.initGoalState / updateGoalState   IntraBrokerDiskCapacityGoal.java:81-108,223-245
//   IntraBrokerDiskUsageDistributionGoal.updateGoalState           IntraBrokerDiskUsageDistributionGoal.java:106-137
//   actionAcceptance (ccmi_action_acceptance)                      IntraBrokerDiskCapacityGoal.java:115-136,
//                                                                  IntraBrokerDiskUsageDistributionGoal.java:146-243
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>

#include "device.h"
#include "engine.h"
#include "intra.h"
#include "prof.h"

namespace ccmi {

namespace {

std::string fmt2(const char* f, ...) __attribute__((format(printf, 1, 2)));
std::string fmt2(const char* f, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, f);
  std::vsnprintf(buf, sizeof(buf), f, ap);
  va_end(ap);
  return buf;
}

class IntraGoalImpl : public GoalImpl {
 public:
  explicit IntraGoalImpl(int k) {
    kind = k;
    ig = k == CCMI_GOAL_INTRA_BROKER_DISK_CAPACITY ? IG_CAPACITY : IG_USAGE;
    name = ig == IG_CAPACITY ? "IntraBrokerDiskCapacityGoal" : "IntraBrokerDiskUsageDistributionGoal";
  }
  int ig;
  std::vector<double> upper, lower;  // _balanceUpperThresholdByBroker / _balanceLowerThresholdByBroker

  void init(Engine& e) override {
    Model& m = e.m;
    allowed.assign(m.B, 1);
    std::memset(&dg, 0, sizeof(dg));
    dg.kind = kind;
    dg.resource = R_DISK;
    if (m.D == 0) throw std::invalid_argument(name + " needs the replica placement over disks (JBOD)");
    if (m.diskGhosts)
      throw Unsupported(name + " after inter-broker moves of a JBOD session (replicas left on their source disks)");
    for (const GoalImpl* g : e.priors)
      if (!isIntraGoalKind(g->kind))
        throw std::invalid_argument("intra-broker goals cannot be optimized together with inter-broker goals");
    if (ig == IG_CAPACITY) {  // IntraBrokerDiskCapacityGoal.initGoalState
      const double thr = e.bc.capThreshold[R_DISK];
      for (int b = 0; b < m.B; ++b) {
        if (!m.alive(b)) continue;
        const double existing = m.bu(b, R_DISK), allowedCap = m.cap(b, R_DISK) * thr;
        if (allowedCap < existing) {
          ccmi_provision_recommendation rec = underBrokers(1);  // IntraBrokerDiskCapacityGoal.java:92-95
          rec.total_capacity = existing / thr;
          throw OptimizationFailure(fmt2("[%s] Insufficient disk capacity at broker %d (Utilization %.2f, Allowed "
                                         "Capacity %.2f).",
                                         name.c_str(), m.bId[b], existing, allowedCap),
                                    rec);
        }
      }
    }
  }

  bool rebalanceAll(Engine& e) override;
  void rebalance(Engine&, int) override {}

  void update(Engine& e) override {
    const Model& m = e.m;
    if (ig == IG_CAPACITY) {
      const double thr = e.bc.capThreshold[R_DISK];
      for (int b = 0; b < m.B; ++b) {
        if (!m.alive(b)) continue;
        for (int k = m.bDiskOff[b]; k < m.bDiskOff[b + 1]; ++k) {
          const int d = m.bDisks[k];
          if (m.dAlive[d] && m.dUtil[d] > m.dCap[d] * thr) {
            ccmi_provision_recommendation rec = provisionRec();  // IntraBrokerDiskCapacityGoal.java:236-239
            rec.num_disks = 1;
            rec.total_capacity = m.dUtil[d] / thr;
            throw OptimizationFailure(fmt2("[%s] Utilization (%.2f) for disk Disk[logdir=%s,state=%s,capacity=%f,"
                                           "replicaCount=%d] on broker %d is above capacity limit.",
                                           name.c_str(), m.dUtil[d], m.dLogdir[d].c_str(), "ALIVE", m.dCap[d],
                                           (int)m.dMembers[d].size(), m.bId[b]),
                                      rec);
          }
        }
      }
    } else {
      bool out = false;
      for (int b = 0; b < m.B; ++b) {
        if (!m.alive(b)) continue;
        for (int k = m.bDiskOff[b]; k < m.bDiskOff[b + 1]; ++k) {
          const int d = m.bDisks[k];
          if (!m.dAlive[d]) continue;
          if (m.diskPct(d) > upper[b] || m.diskPct(d) < lower[b]) out = true;
        }
      }
      if (out) succeeded = false;
    }
    finished = true;
  }

  int compareStats(const ccmi_cluster_stats& a, const ccmi_cluster_stats& b) const override {
    if (ig == IG_CAPACITY) return 0;  // GoalUtils.HardGoalStatsComparator
    if (a.num_unbalanced_disks > b.num_unbalanced_disks || a.disk_utilization_std > b.disk_utilization_std) return -1;
    return 1;
  }

  // Goal.actionAcceptance on the host model
  int accept(const Engine& e, const ccmi_action& a) const {
    const Model& m = e.m;
    if (a.source_disk < 0 || a.destination_disk < 0 || a.source_disk >= m.D || a.destination_disk >= m.D)
      throw std::invalid_argument(name + " does not support balancing action not specifying logdir.");
    const int sr = m.replicaOn(a.partition, a.source_broker);
    if (sr < 0) throw std::invalid_argument("no replica of the partition on the source broker");
    const double thr = e.bc.capThreshold[R_DISK];
    auto under = [&](int d, double add) { return m.dUtil[d] + add < m.dCap[d] * thr; };
    if (ig == IG_CAPACITY) {
      switch (a.type) {
        case CCMI_INTRA_BROKER_REPLICA_SWAP: {
          const int dr = m.replicaOn(a.destination_partition, a.destination_broker);
          if (dr < 0) throw std::invalid_argument("no replica of the destination partition on the destination broker");
          const double delta = m.ru(dr, R_DISK) - m.ru(sr, R_DISK);
          return (delta > 0 ? under(m.rDisk[sr], delta) : under(m.rDisk[dr], -delta)) ? CCMI_ACCEPT
                                                                                       : CCMI_REPLICA_REJECT;
        }
        case CCMI_INTRA_BROKER_REPLICA_MOVEMENT: {
          const int dd = m.diskOf(a.destination_broker, m.dLogdir[a.destination_disk]);
          return under(dd, m.ru(sr, R_DISK)) ? CCMI_ACCEPT : CCMI_REPLICA_REJECT;
        }
        case CCMI_LEADERSHIP_MOVEMENT: return CCMI_ACCEPT;
        default: throw std::invalid_argument("Unsupported balancing action " + std::to_string(a.type) + " is provided.");
      }
    }
    double delta;
    switch (a.type) {
      case CCMI_INTRA_BROKER_REPLICA_SWAP: {
        const int dr = m.replicaOn(a.destination_partition, a.source_broker);
        if (dr < 0) throw std::invalid_argument("no replica of the destination partition on the broker");
        delta = m.ru(dr, R_DISK) - m.ru(sr, R_DISK);
        break;
      }
      case CCMI_LEADERSHIP_MOVEMENT: delta = 0; break;
      case CCMI_INTRA_BROKER_REPLICA_MOVEMENT: delta = -m.ru(sr, R_DISK); break;
      default: throw std::invalid_argument("Unsupported balancing action " + std::to_string(a.type) + " is provided.");
    }
    const int s = m.diskOf(a.source_broker, m.dLogdir[a.source_disk]);
    const int t = m.diskOf(a.source_broker, m.dLogdir[a.destination_disk]);
    if (delta == 0) return CCMI_ACCEPT;
    const int bb = m.dBroker[s];
    const double u = upper[bb], l = lower[bb];
    const double srcAllow = delta > 0 ? m.dCap[s] * u - m.dUtil[s] : m.dUtil[s] - m.dCap[s] * l;
    const double dstAllow = delta > 0 ? m.dUtil[t] - m.dCap[t] * l : m.dCap[t] * u - m.dUtil[t];
    const double ad = std::fabs(delta);
    if ((srcAllow >= 0 && srcAllow < ad) || (dstAllow >= 0 && dstAllow < ad)) return CCMI_REPLICA_REJECT;
    const double prev = m.diskPct(s) - m.diskPct(t);
    const double next = prev + delta / m.dCap[s] + delta / m.dCap[t];
    return std::fabs(next) < std::fabs(prev) ? CCMI_ACCEPT : CCMI_REPLICA_REJECT;
  }
};

// The broker loop of AbstractGoal.optimize as one K6 launch, then the replay of its records.
bool IntraGoalImpl::rebalanceAll(Engine& e) {
  PhaseScope ps(PH_DEV_SCAN);
  Model& m = e.m;
  IntraRequest q;
  q.goal = ig;
  q.capThr = e.bc.capThreshold[R_DISK];
  q.margin = (e.bc.resBalance[R_DISK] - 1) * 0.9;  // BALANCE_MARGIN
  q.slot = dg.allowedSlot;
  for (const GoalImpl* g : e.priors) {
    const auto* p = static_cast<const IntraGoalImpl*>(g);
    if (q.nPrior >= kIntraMaxPrior) throw std::invalid_argument("too many optimized intra-broker goals");
    q.priorKind[q.nPrior] = p->ig;
    q.priorSlot[q.nPrior] = p->dg.allowedSlot;
    q.nPrior++;
  }
  std::vector<int32_t> brokers, eOff(m.B + 1, 0), eRep, eDisk;
  std::vector<uint8_t> rSel(m.R, 0);
  for (int r = 0; r < m.R; ++r) {
    // selectOnlineReplicas && selectReplicasBasedOnExcludedTopics (ReplicaSortFunctionFactory.java:135-146)
    bool sel = !m.curOffline(r);
    if (sel && e.opt.anyExclTopic && !m.origOffline(r) && e.opt.exclTopic[m.pTopic[m.rPart[r]]]) sel = false;
    rSel[r] = sel ? 1 : 0;
  }
  eRep.reserve(m.R);
  eDisk.reserve(m.R);
  for (int b = 0; b < m.B; ++b) {
    eOff[b] = (int32_t)eRep.size();
    if (m.alive(b)) brokers.push_back(b);
    for (int r : m.bRepl[b])
      if (m.rDisk[r] >= 0) {
        eRep.push_back(r);
        eDisk.push_back(m.rDisk[r]);
      }
  }
  eOff[m.B] = (int32_t)eRep.size();
  q.brokers = brokers.data();
  q.nBrokers = (int32_t)brokers.size();
  q.eOff = eOff.data();
  q.eRep = eRep.data();
  q.eDisk = eDisk.data();
  q.rSel = rSel.data();
  if (m.diskDirty) {
    e.dev->setDiskUtil(m.dUtil.data());
    m.diskDirty = false;
  }
  IntraResult res;
  e.dev->intraRun(q, res);
  for (int b : brokers)
    if (res.status[b] == IS_CYCLE) throw std::invalid_argument("swap phase queue cycle longer than 16 states");
  if (ig == IG_USAGE) {
    upper = res.upper;
    lower = res.lower;
  }
  m.log.reserve(m.log.size() + res.rep.size());
  for (int b : brokers) {
    e.candidates += res.cand[b];
    for (int64_t i = res.off[b]; i < res.off[b + 1]; ++i) {
      const int r = res.rep[i], dst = res.dst[i];
      if (r < 0 || r >= m.R || m.rBroker[r] != b || m.rDisk[r] != res.src[i] || dst < 0 || dst >= m.D ||
          m.dBroker[dst] != b)
        throw std::runtime_error("device intra-broker record does not match the host model");
      m.replayDiskMove(r, res.src[i], dst);  // ClusterModel.relocateReplica(tp, broker, logdir)
    }
  }
  return true;
}

}  // namespace

bool isIntraGoalKind(int kind) {
  return kind == CCMI_GOAL_INTRA_BROKER_DISK_CAPACITY || kind == CCMI_GOAL_INTRA_BROKER_DISK_USAGE_DISTRIBUTION;
}

std::unique_ptr<GoalImpl> makeIntraGoal(int kind) { return std::make_unique<IntraGoalImpl>(kind); }

int intraAcceptance(const GoalImpl& g, const Engine& e, const ccmi_action& a) {
  if (!isIntraGoalKind(g.kind)) return -1;
  return static_cast<const IntraGoalImpl&>(g).accept(e, a);
}

}  // namespace ccmi
