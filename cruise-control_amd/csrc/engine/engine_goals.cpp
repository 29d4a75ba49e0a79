// Goal drivers for the rest of the default goal list (engine.h has the engine; engine.cpp the distribution goals).
//
// Each driver restates the reference goal's control flow on the host — which brokers it visits, which
// replicas it tries in which order, which candidate list each replica gets, when it stops — and hands every
// candidate-predicate evaluation to a device scan. Where consecutive replicas share one candidate list the
// driver scans them as one batch (rows = replicas, columns = candidates, winner = smallest (row, column)),
// replays the host-side bookkeeping of the rows before the winner, and resumes right after it.
//
// Reference code restated here (paths under cruise-control/src/main/java/com/linkedin/kafka/cruisecontrol/):
//   RackAwareGoal / AbstractRackAwareGoal   analyzer/goals/RackAwareGoal.java:82-225, AbstractRackAwareGoal.java:144-170
//   MinTopicLeadersPerBrokerGoal            analyzer/goals/MinTopicLeadersPerBrokerGoal.java:276-330,444-466
//   ReplicaCapacityGoal                     analyzer/goals/ReplicaCapacityGoal.java:100-290
//   CapacityGoal (+ Disk/NwIn/NwOut/Cpu)    analyzer/goals/CapacityGoal.java:120-355
//   PotentialNwOutGoal                      analyzer/goals/PotentialNwOutGoal.java:140-331
//   TopicReplicaDistributionGoal            analyzer/goals/TopicReplicaDistributionGoal.java:225-570
//   LeaderReplicaDistributionGoal           analyzer/goals/LeaderReplicaDistributionGoal.java:137-364,
//                                           ReplicaDistributionAbstractGoal.java:60-160
//   LeaderBytesInDistributionGoal           analyzer/goals/LeaderBytesInDistributionGoal.java:142-271
//   BrokerSetAwareGoal                      analyzer/goals/BrokerSetAwareGoal.java:80-275 (not in default.goals)
//   TopicLeaderReplicaDistributionGoal      analyzer/goals/TopicLeaderReplicaDistributionGoal.java:298-778 (in goals,
//                                           not in default.goals)
//   GoalUtils.ensureNoOfflineReplicas       analyzer/goals/GoalUtils.java:307-318
#include <algorithm>
#include <cmath>
#include <limits>
#include <set>
#include <unordered_map>

#include "device.h"
#include "engine.h"
#include "predicates.h"
#include "rackrows.h"
#include "prof.h"

namespace ccmi {

namespace {

constexpr double kBalanceMargin = 0.9;

// sort-name ids of the tracked SortedReplicas: replicaSortName(goal, reverse, leaderOnly)
int sortId(int kind, bool reverse, bool leaderOnly) { return 100 + 8 * kind + (reverse ? 1 : 0) + (leaderOnly ? 2 : 0); }

std::vector<int32_t> aliveById(const Model& m) {  // ClusterModel.aliveBrokers() iteration (HashSet<Broker>, ids < table)
  std::vector<int32_t> v;
  for (int b = 0; b < m.B; ++b)
    if (m.alive(b)) v.push_back(b);
  return v;
}

bool hasOffline(const Model& m, int b) { return m.bOfflineSet[b].size() > 0; }  // !currentOfflineReplicas().isEmpty()

// GoalUtils.ensureNoOfflineReplicas
void ensureNoOfflineReplicas(const Model& m, const std::string& name) {
  for (int r = 0; r < m.R; ++r)
    if (m.selfHealing[r] && m.curOffline(r))
      throw OptimizationFailure("[" + name + "] Cannot remove replica from broker " + std::to_string(m.bId[m.rBroker[r]]),
                                underBrokers(1));
}

// GoalUtils.ensureReplicasMoveOffBrokersWithBadDisks (GoalUtils.java:327-338)
void ensureReplicasMoveOffBadDisks(const Model& m, const std::string& name) {
  for (int b = 0; b < m.B; ++b)
    if (m.bState[b] == BState::BAD_DISKS)
      for (int r : m.bRepl[b])
        if (m.ineligible(m.rPart[r], b))
          throw OptimizationFailure("[" + name + "] A replica was moved back to broker with broken disk.", underBrokers(1));
}

// GoalUtils.aliveBrokersNotExcludedForReplicaMove
int allowedForReplicaMove(const Engine& e, std::vector<uint8_t>& allowed) {
  allowed.assign(e.m.B, 0);
  int n = 0;
  for (int b = 0; b < e.m.B; ++b)
    if (e.m.alive(b) && !(e.opt.anyExclMove && e.opt.exclMove[b])) {
      allowed[b] = 1;
      n++;
    }
  return n;
}

template <class C>
void stableSortBy(std::vector<int32_t>& v, C cmp) {
  std::stable_sort(v.begin(), v.end(), [&](int a, int b) { return cmp(a, b) < 0; });
}

int cmpStd(double after, double before) {  // stats comparator on a standard deviation (AnalyzerUtils.compare, 1e-5)
  if (after - before > 1e-5) return -1;
  if (before - after > 1e-5) return 1;
  return 0;
}

// ======================================================================================= RackAwareGoal
class RackAware : public GoalImpl {
 public:
  RackAware() {
    kind = CCMI_GOAL_RACK_AWARE;
    name = "RackAwareGoal";
  }
  std::vector<int32_t> alive;

  // initGoalState (RackAwareGoal.java:82-124)
  void init(Engine& e) override {
    Model& m = e.m;
    allowedForReplicaMove(e, allowed);
    std::set<int> racks;
    for (int b = 0; b < m.B; ++b)
      if (m.alive(b)) racks.insert(m.bRack[b]);
    const int numRacks = (int)racks.size();
    if (e.opt.anyExclTopic) {
      // replicationFactorByTopic entries in HashMap<String, Integer> order: the first included topic whose
      // replication factor exceeds the alive racks names the shortfall (:77-94)
      std::vector<int> rf(m.T, 1);
      for (int p = 0; p < m.P; ++p) rf[m.pTopic[p]] = std::max(rf[m.pTopic[p]], m.pOff[p + 1] - m.pOff[p]);
      TopicSet byTopic(&m.topicOrder);
      for (int t = 0; t < m.T; ++t) byTopic.add(t, m.topicHash[t]);
      std::vector<int32_t> order;
      byTopic.order(order);
      int maxIncluded = 1;
      for (int t : order) {
        if (e.opt.exclTopic[t]) continue;
        maxIncluded = std::max(maxIncluded, rf[t]);
        if (maxIncluded > numRacks) {
          ccmi_provision_recommendation rec = provisionRec();
          rec.num_racks = maxIncluded - numRacks;
          throw OptimizationFailure("[" + name + "] Insufficient number of racks to distribute included replicas (Current: " +
                                        std::to_string(numRacks) + ", Needed: " + std::to_string(maxIncluded) + ").",
                                    rec);
        }
      }
    } else if (m.maxRf > numRacks) {
      ccmi_provision_recommendation rec = provisionRec();
      rec.num_racks = m.maxRf - numRacks;
      throw OptimizationFailure("[" + name + "] Insufficient number of racks to distribute each replica (Current: " +
                                    std::to_string(numRacks) + ", Needed: " + std::to_string(m.maxRf) + ").",
                                rec);
    }
    // over-provisioned in racks (RackAwareGoal.java:103-109)
    const int numExtraRacks = numRacks - m.maxRf;
    if (numExtraRacks >= e.bc.overprovisionedMinExtraRacks) {
      ccmi_provision_recommendation rec = provisionRec(CCMI_PROVISION_OVER_PROVISIONED);
      rec.num_racks = numExtraRacks - e.bc.overprovisionedMinExtraRacks + 1;
      prov = provisionResponse(CCMI_PROVISION_OVER_PROVISIONED, rec);
    }
    Model::Spec s;
    s.selImmigrants = e.opt.onlyImmigrants;
    s.selExclTopics = e.opt.anyExclTopic;
    for (int b = 0; b < m.B; ++b) m.track(b, sortId(kind, false, false), s);
    alive = aliveById(m);
    dg = DevGoal{};
    dg.kind = DG_RACK_AWARE;
    dg.allowedSlot = e.newSlot;
  }

  // shouldKeepInTheCurrentBroker (:214-225)
  static bool keep(const Model& m, int r) {
    const int self = m.rBroker[r], rk = m.bRack[self], p = m.rPart[r];
    for (int i = m.pOff[p]; i < m.pOff[p + 1]; ++i) {
      const int x = m.rBroker[m.pSlots[i]];
      if (x != self && m.bRack[x] == rk) return false;
    }
    return true;
  }
  // candidates of `cands[0, upto)` that rackAwareEligibleBrokers keeps (:193-211) and, for a leader replica,
  // filterOutBrokersExcludedForLeadership leaves (GoalUtils.java:122-135)
  static int64_t eligibleCount(const Engine& e, int r, const std::vector<int32_t>& cands, size_t upto) {
    const Model& m = e.m;
    const bool exclLead = e.opt.anyExclLead && !e.opt.anyRequested && m.rLeader[r];
    const bool newOnly = m.numNew > 0 && !e.opt.anyRequested;  // GoalUtils.eligibleBrokers :193-198
    int racks[kMaxRf];
    int n = 0;
    const int p = m.rPart[r];
    for (int i = m.pOff[p]; i < m.pOff[p + 1]; ++i) racks[n++] = m.bRack[m.rBroker[m.pSlots[i]]];
    for (int i = 0; i < n; ++i)
      if (racks[i] == m.bRack[m.rBroker[r]]) {
        racks[i] = racks[--n];
        break;
      }
    int64_t c = 0;
    for (size_t j = 0; j < upto; ++j) {
      bool in = true;
      for (int i = 0; i < n; ++i) in &= racks[i] != m.bRack[cands[j]];
      if (exclLead && e.opt.exclLead[cands[j]]) in = false;
      if (newOnly && !m.isNew(cands[j]) && cands[j] != m.rOrig[r]) in = false;
      c += in;
    }
    return c;
  }

  // The whole broker loop as ONE device chain: the rows are, broker by broker (brokersToBalance order) and in each
  // broker's sorted-replica order, the replicas that violate rack awareness or are offline when the goal starts. A
  // replica can only stop violating during the loop (every move goes to a rack the partition does not use yet), and
  // replicas moved onto later brokers are rack-aware there, so the device re-checks each row's
  // shouldKeepInTheCurrentBroker when it reaches it and skips it if it now holds; everything else it decides and
  // applies in order. The host replays the logged moves and counts the reference-equivalent candidates.
  //
  // With no optimized goals a row's decision reads only its own partition, so the rows are decided per partition on
  // the device in one launch (rackrows.h, Engine::rackRowsGroups) and the host applies the accepted moves in row order:
  // no device-side apply, no sequential decision chain.
  bool rebalanceAll(Engine& e) override {
    const bool groups = e.priors.empty() && !std::getenv("CCMI_RACK_CHAIN");
    if (!groups && !e.chainsOn()) return false;
    PhaseScope ps(PH_OTHER_GOALS);
    Model& m = e.m;
    const std::vector<int> order = brokersToBalance(e);
    std::vector<std::vector<int32_t>> byBroker(m.B);
    for (int r = 0; r < m.R; ++r) {
      const int b = m.rBroker[r];
      if (m.alive(b) && !m.curOffline(r) && keep(m, r)) continue;
      if (e.opt.onlyImmigrants && !m.immigrant(r)) continue;  // the tracked selection (immigrants only,
      if (e.opt.anyExclTopic && !m.origOffline(r) && e.opt.exclTopic[m.pTopic[m.rPart[r]]]) continue;  // topics)
      byBroker[b].push_back(r);
    }
    Model::Spec spec;
    spec.selImmigrants = e.opt.onlyImmigrants;
    spec.selExclTopics = e.opt.anyExclTopic;
    std::vector<int32_t> rows, cands, log;
    for (int b : order) {
      auto& v = byBroker[b];
      std::sort(v.begin(), v.end(), [&](int x, int y) { return m.replicaKey(spec, x) < m.replicaKey(spec, y); });
      rows.insert(rows.end(), v.begin(), v.end());
    }
    e.eligible(alive, DA_MOVE, cands);
    int64_t failRow = 0;
    if (groups) {
      std::vector<int32_t> res;
      e.rackRowsGroups(*this, rows, cands, res);
      for (size_t k = 0; k < rows.size(); ++k) {
        if (res[k] == kRackFail) {
          failRow = (int64_t)k + 1;
          break;
        }
        if (res[k] == kRackKeep) continue;
        const int r = rows[k], j = res[k];
        e.candidates += eligibleCount(e, r, cands, (size_t)j + 1);
        m.relocateReplica(m.rPart[r], m.rBroker[r], cands[j]);
      }
    } else {
      failRow = e.chainRackRows(*this, rows, cands, log);
      Model::Replay rp(m);
      for (size_t i = 0; i + 1 < log.size(); i += 2) {
        const int r = rows[log[i]], j = log[i + 1];
        e.candidates += eligibleCount(e, r, cands, (size_t)j + 1);
        m.relocateReplica(m.rPart[r], m.rBroker[r], cands[j]);
      }
    }
    if (failRow > 0) {
      const int r = rows[failRow - 1];
      e.candidates += eligibleCount(e, r, cands, cands.size());
      throw OptimizationFailure("[" + name + "] Cannot move replica of partition " + std::to_string(m.rPart[r]) +
                                    " to a rack-aware broker.",
                                underBrokers(1));
    }
    return true;
  }

  // AbstractRackAwareGoal.rebalanceForBroker (:144-170), throwExceptionIfCannotMove = true
  void rebalance(Engine& e, int b) override {
    PhaseScope ps(PH_OTHER_GOALS);
    Model& m = e.m;
    const std::vector<int32_t> list = m.sorted(b, sortId(kind, false, false));
    std::vector<int32_t> one(1), cands;
    e.eligible(alive, DA_MOVE, cands);
    for (int r : list) {
      if (m.alive(b) && !m.curOffline(r) && keep(m, r)) continue;
      one[0] = r;
      const int64_t key = e.crossScan(*this, DA_MOVE, one, 0, cands, FILTER_RACK_AWARE, false);
      e.candidates += eligibleCount(e, r, cands, key >= 0 ? (size_t)key + 1 : cands.size());
      if (key < 0)
        throw OptimizationFailure("[" + name + "] Cannot move replica of partition " + std::to_string(m.rPart[r]) +
                                      " to a rack-aware broker.",
                                  underBrokers(1));
      m.relocateReplica(m.rPart[r], b, cands[key]);
    }
  }

  // updateGoalState (:131-143) + ensureRackAware (:159-185)
  void update(Engine& e) override {
    Model& m = e.m;
    for (int p = 0; p < m.P; ++p) {
      if (e.opt.anyExclTopic && e.opt.exclTopic[m.pTopic[p]]) continue;  // excluded topics are not checked
      int racks[kMaxRf];
      const int n = m.pOff[p + 1] - m.pOff[p];
      for (int i = 0; i < n; ++i) {
        racks[i] = m.bRack[m.rBroker[m.pSlots[m.pOff[p] + i]]];
        for (int j = 0; j < i; ++j)
          if (racks[j] == racks[i]) {
            int distinct = 0;  // ProvisionRecommendation.numRacks = replicas - distinct racks (:177-180)
            for (int a = 0; a < n; ++a) {
              const int rk = m.bRack[m.rBroker[m.pSlots[m.pOff[p] + a]]];
              bool seen = false;
              for (int c = 0; c < a; ++c) seen |= m.bRack[m.rBroker[m.pSlots[m.pOff[p] + c]]] == rk;
              distinct += seen ? 0 : 1;
            }
            ccmi_provision_recommendation rec = provisionRec();
            rec.num_racks = n - distinct;
            throw OptimizationFailure("[" + name + "] Partition " + std::to_string(p) + " is not rack-aware.", rec);
          }
      }
    }
    ensureNoOfflineReplicas(m, name);
    if (prov.status != CCMI_PROVISION_OVER_PROVISIONED) prov = provisionResponse(CCMI_PROVISION_RIGHT_SIZED);
    finished = true;
  }
  int compareStats(const ccmi_cluster_stats&, const ccmi_cluster_stats&) const override { return 0; }
};

struct PartitionOrder {  // TopicPartition in a HashMap bin: (topic, partition)
  const Model* m;
  int cmp(int a, int b) const {
    const int c = m->topicNames[m->pTopic[a]].compare(m->topicNames[m->pTopic[b]]);
    return c ? c : jcmpInt(m->pNumber[a], m->pNumber[b]);
  }
};

// ======================================================================================= RackAwareDistributionGoal
// RackAwareDistributionGoal.java:139-383 + AbstractRackAwareGoal.rebalanceForBroker (:144-170) with
// throwExceptionIfCannotMove = false: replicas of a partition spread as evenly as possible over the alive racks
// allowed replica moves (BalanceLimit :403-448: base = rf / racks, rf % racks racks hold one more). Each replica that
// must move gets its own candidate list — the TreeSet of eligible brokers by (partition replicas on the broker's rack
// after removing this one, broker id) — and one device scan over it.
class RackAwareDist : public GoalImpl {
 public:
  RackAwareDist() {
    kind = CCMI_GOAL_RACK_AWARE_DISTRIBUTION;
    name = "RackAwareDistributionGoal";
  }
  std::vector<int32_t> alive;
  int numRacks = 0;  // BalanceLimit._numAliveRacksAllowedReplicaMoves

  // initGoalState (:139-164)
  void init(Engine& e) override {
    Model& m = e.m;
    if (allowedForReplicaMove(e, allowed) == 0) {
      ccmi_provision_recommendation rec = provisionRec();
      rec.num_brokers = m.maxRf;
      throw OptimizationFailure("[" + name + "] All alive brokers are excluded from replica moves.", rec);
    }
    std::set<int> racks;  // ClusterModel.aliveRacksAllowedReplicaMoves (ClusterModel.java:658-662)
    for (int b = 0; b < m.B; ++b)
      if (allowed[b]) racks.insert(m.bRack[b]);
    numRacks = (int)racks.size();
    const int numExtraRacks = numRacks - m.maxRf;
    if (numExtraRacks >= e.bc.overprovisionedMinExtraRacks) {
      ccmi_provision_recommendation rec = provisionRec(CCMI_PROVISION_OVER_PROVISIONED);
      rec.num_racks = numExtraRacks - e.bc.overprovisionedMinExtraRacks + 1;
      prov = provisionResponse(CCMI_PROVISION_OVER_PROVISIONED, rec);
    }
    Model::Spec s;
    s.selImmigrants = e.opt.onlyImmigrants;
    s.selExclTopics = e.opt.anyExclTopic;
    for (int b = 0; b < m.B; ++b) m.track(b, sortId(kind, false, false), s);
    alive = aliveById(m);
    dg = DevGoal{};
    dg.kind = DG_RACK_AWARE_DISTRIBUTION;
    dg.allowedSlot = e.newSlot;
  }

  // numPartitionReplicasByRackId (:113-119) as (rack, count) pairs
  static int rackCounts(const Model& m, int p, int* rk, int* cnt) {
    int n = 0;
    for (int i = m.pOff[p]; i < m.pOff[p + 1]; ++i) {
      const int x = m.bRack[m.rBroker[m.pSlots[i]]];
      int k = 0;
      while (k < n && rk[k] != x) ++k;
      if (k == n) {
        rk[n] = x;
        cnt[n++] = 0;
      }
      cnt[k]++;
    }
    return n;
  }

  // shouldKeepInTheCurrentBroker (:305-334)
  bool keep(const Model& m, int r) const {
    const int b = m.rBroker[r], p = m.rPart[r];
    if (!allowed[b]) return false;
    const int rf = m.pOff[p + 1] - m.pOff[p];
    int rk[kMaxRf], cnt[kMaxRf];
    const int n = rackCounts(m, p, rk, cnt);
    const int base = rf / numRacks, extra = rf % numRacks, upper = base + (extra == 0 ? 0 : 1);
    int mine = 0;
    for (int k = 0; k < n; ++k)
      if (rk[k] == m.bRack[b]) mine = cnt[k];
    if (mine <= base) return true;
    if (mine > upper) return false;
    int over = 0;
    for (int k = 0; k < n; ++k) over += cnt[k] > base ? 1 : 0;
    return over <= extra;
  }

  // rackAwareEligibleBrokers (:246-302): the TreeSet order (count of the broker's rack, id)
  void eligibleFor(const Model& m, int r, std::vector<int32_t>& out) const {
    const int p = m.rPart[r];
    const int rf = m.pOff[p + 1] - m.pOff[p];
    int rk[kMaxRf], cnt[kMaxRf];
    const int n = rackCounts(m, p, rk, cnt);
    for (int k = 0; k < n; ++k)
      if (rk[k] == m.bRack[m.rBroker[r]]) cnt[k]--;
    const int base = rf / numRacks;
    int over = 0;
    for (int k = 0; k < n; ++k) over += cnt[k] > base ? 1 : 0;
    const bool canMoveToBase = over < rf % numRacks;
    auto countOf = [&](int b) {
      for (int k = 0; k < n; ++k)
        if (rk[k] == m.bRack[b]) return cnt[k];
      return 0;
    };
    out.clear();
    for (int b : alive) {
      const int c = countOf(b);
      if (!(c < base || (canMoveToBase && c == base))) continue;
      bool hosts = false;
      for (int i = m.pOff[p]; i < m.pOff[p + 1]; ++i) hosts |= m.rBroker[m.pSlots[i]] == b;
      if (!hosts) out.push_back(b);
    }
    std::sort(out.begin(), out.end(), [&](int a, int b) {
      const int ca = countOf(a), cb = countOf(b);
      return ca != cb ? ca < cb : m.bId[a] < m.bId[b];
    });
  }

  void rebalance(Engine& e, int b) override {
    PhaseScope ps(PH_OTHER_GOALS);
    Model& m = e.m;
    const std::vector<int32_t> list = m.sorted(b, sortId(kind, false, false));
    std::vector<int32_t> one(1), tree, cands;
    for (int r : list) {
      if (m.alive(b) && !m.curOffline(r) && keep(m, r)) continue;
      eligibleFor(m, r, tree);
      e.eligible(tree, DA_MOVE, cands);
      one[0] = r;
      const int64_t key = e.crossScan(*this, DA_MOVE, one, 0, cands);
      if (key >= 0) m.relocateReplica(m.rPart[r], b, cands[key]);  // else: logged and skipped (:166)
    }
  }

  // updateGoalState (:175-188) + ensureRackAwareDistribution (:342-383) over clusterModel.leaderReplicas() (a
  // HashSet<Replica> of the partitions' leaders, filled in the model's partition-map order)
  void update(Engine& e) override {
    Model& m = e.m;
    ensureNoOfflineReplicas(m, name);
    PartitionOrder po{&m};
    JHashSet<PartitionOrder> parts(&po);
    for (int p = 0; p < m.P; ++p) parts.add(p, jMix(jMix(1, m.pNumber[p]), m.topicHash[m.pTopic[p]]));
    std::vector<int32_t> order, leaders;
    parts.order(order);
    ReplicaSet ls(&m.replicaOrder);
    for (int p : order) ls.add(m.pLeader[p], m.replicaHash(m.pLeader[p]));
    ls.order(leaders);
    for (int l : leaders) {
      const int p = m.rPart[l];
      if (e.opt.anyExclTopic && e.opt.exclTopic[m.pTopic[p]]) continue;
      int rk[kMaxRf], cnt[kMaxRf];
      const int n = rackCounts(m, p, rk, cnt);
      int mx = 0, mn = 1 << 30;
      for (int k = 0; k < n; ++k) {
        mx = std::max(mx, cnt[k]);
        mn = std::min(mn, cnt[k]);
      }
      if (mx > 1 && (n < numRacks || mx - mn > 1))
        throw OptimizationFailure("[" + name + "] Partition " + std::to_string(p) + " is not rack-aware.",
                                  underBrokers(1));  // .excludedRackIds(...) is not carried by the ABI
    }
    if (prov.status != CCMI_PROVISION_OVER_PROVISIONED) prov = provisionResponse(CCMI_PROVISION_RIGHT_SIZED);
    finished = true;
  }
  int compareStats(const ccmi_cluster_stats&, const ccmi_cluster_stats&) const override { return 0; }
};

// ======================================================================================= MinTopicLeadersPerBrokerGoal
// With the default topics.with.min.leaders.per.broker (no topic matches) the goal accepts every action and only
// moves offline replicas away (moveAwayOfflineReplicas). With topics, every eligible broker gets at least the minimum
// number of leaders of each: first by leadership moves from the partitions' leaders (single-candidate pair scans), then
// by moving a leader replica in from the broker with the most leaders of the topic (one cross scan over its leaders).
// The per-(topic, broker) leader counts live in the model and on the device (Model::enableTopicLeaders).
class MinTopicLeaders : public GoalImpl {
 public:
  MinTopicLeaders() {
    kind = CCMI_GOAL_MIN_TOPIC_LEADERS_PER_BROKER;
    name = "MinTopicLeadersPerBrokerGoal";
  }
  std::vector<int32_t> mustOrder;  // _mustHaveTopicMinLeadersPerBroker.keySet() iteration order
  std::vector<int32_t> minOf;      // [T] minimum, -1 = not a topic of the goal

  bool eligibleToHaveLeaders(const Engine& e, int b) const {  // isEligibleToHaveLeaders (:439-442)
    return !(e.opt.anyExclLead && e.opt.exclLead[b]) && !(e.opt.anyExclMove && e.opt.exclMove[b]);
  }

  // HashSet<String> iteration order of topics added in `ins` order
  static std::vector<int32_t> topicSetOrder(const Model& m, const std::vector<int32_t>& ins) {
    TopicSet s(&m.topicOrder);
    for (int t : ins) s.add(t, m.topicHash[t]);
    std::vector<int32_t> out;
    s.order(out);
    return out;
  }

  // initGoalState (:163-192) with validateTopicsWithMinLeaderIsNotExcluded / validateEnoughLeaderToDistribute /
  // validateBrokersAllowedReplicaMoveExist (:198-241)
  void init(Engine& e) override {
    Model& m = e.m;
    const int nAllowed = allowedForReplicaMove(e, allowed);
    dg = DevGoal{};
    dg.kind = DG_ACCEPT_ALL;
    dg.allowedSlot = e.newSlot;
    mustOrder.clear();
    minOf.assign(m.T, -1);
    if (e.bc.minLeaderTopics.empty()) return;
    {  // Utils.getTopicNamesMatchedWithPattern: clusterModel.topics() (a HashSet) streamed into Collectors.toSet()
      std::vector<int32_t> all(m.T), matched;
      for (int t = 0; t < m.T; ++t) all[t] = t;
      std::vector<uint8_t> match(m.T, 0);
      for (int t : e.bc.minLeaderTopics) match[t] = 1;
      for (int t : topicSetOrder(m, all))
        if (match[t]) matched.push_back(t);
      mustOrder = topicSetOrder(m, matched);
    }
    std::vector<int32_t> numLeaders(m.T, 0);  // clusterModel.numLeadersPerTopic: one leader per partition
    for (int p = 0; p < m.P; ++p) numLeaders[m.pTopic[p]]++;
    int eligible = 0;
    for (int b = 0; b < m.B; ++b) eligible += m.alive(b) && eligibleToHaveLeaders(e, b) ? 1 : 0;
    const int cfg = e.bc.minTopicLeadersPerBroker;
    for (int t : mustOrder) minOf[t] = cfg == 0 ? (eligible == 0 ? 0 : numLeaders[t] / eligible) : cfg;
    if (e.opt.anyExclTopic) {
      std::vector<int32_t> bad;
      for (int t : mustOrder)
        if (e.opt.exclTopic[t]) bad.push_back(t);
      if (!bad.empty()) {
        std::string s;
        for (int t : topicSetOrder(m, bad)) s += (s.empty() ? "" : ", ") + m.topicNames[t];
        throw OptimizationFailure("[" + name + "] Topics that must have a minimum number of leaders per broker cannot be "
                                  "excluded. This error implies a config error. Topics should not be excluded=[" + s +
                                  "] (see topics.with.min.leaders.per.broker).");
      }
    }
    for (int t : mustOrder) {
      const int total = eligible * minOf[t];
      if (numLeaders[t] < total) {
        ccmi_provision_recommendation rec = provisionRec();
        rec.num_partitions = total;
        throw OptimizationFailure("[" + name + "] Cannot distribute " + std::to_string(numLeaders[t]) + " leaders over " +
                                      std::to_string(eligible) +
                                      " broker(s) with minimum required per broker leader count " +
                                      std::to_string(minOf[t]) + " for topic " + m.topicNames[t] + ".",
                                  rec);
      }
    }
    if (nAllowed == 0)
      throw OptimizationFailure("[" + name + "] All alive brokers are excluded from replica moves.", underBrokers(m.maxRf));
    Model::Spec s;
    s.selImmigrants = e.opt.onlyImmigrants;
    s.selMustTopics = true;
    s.prioImmigrants = !e.opt.onlyImmigrants;
    for (int b = 0; b < m.B; ++b) m.track(b, sortId(kind, false, false), s);
    m.enableTopicLeaders();
    e.minLeadOf = minOf;
    e.dev->setMinLeaders(minOf.data());
    dg.kind = DG_MIN_TOPIC_LEADERS;
  }

  // maybeMoveLeaderOfTopicToBroker (:336-409) with getBrokersWithExcessiveLeaderToMove (:418-430). The queue's keys (live
  // leader counts) change only for the broker just polled: a move goes from it to `b`, which is never queued (its count
  // is below the minimum). So polling the largest (count, then smallest id) is the PriorityQueue's order.
  void moveLeaderOfTopic(Engine& e, int t, int b) {
    Model& m = e.m;
    const int mn = minOf[t];
    int recv = m.tlead(t, b);
    if (recv >= mn) return;
    const int id = sortId(kind, false, false);
    std::vector<int32_t> followers, pr(1), pb(1, b), one(1, b), cands;
    for (int r : m.sorted(b, id))
      if (!m.rLeader[r] && m.pTopic[m.rPart[r]] == t) followers.push_back(r);
    e.eligible(one, DA_LEADERSHIP, cands);
    for (int f : followers) {
      const int leader = m.pLeader[m.rPart[f]];
      if (m.tlead(t, m.rBroker[leader]) <= mn) continue;
      if (cands.empty()) continue;  // maybeApplyBalancingAction over an empty eligible list
      pr[0] = leader;
      if (e.pairScan(*this, pr, pb, DA_LEADERSHIP) < 0) continue;
      m.relocateLeadership(m.rPart[leader], m.rBroker[leader], b);
      if (++recv >= mn) return;
    }
    std::vector<int32_t> queue;
    for (int x : aliveById(m))
      if (m.tlead(t, x) > mn) queue.push_back(x);
    e.eligible(one, DA_MOVE, cands);
    std::vector<int32_t> leaders;
    while (!queue.empty()) {
      size_t best = 0;
      for (size_t i = 1; i < queue.size(); ++i) {
        const int ci = m.tlead(t, queue[i]), cb = m.tlead(t, queue[best]);
        if (ci > cb || (ci == cb && m.bId[queue[i]] < m.bId[queue[best]])) best = i;
      }
      const int giver = queue[best];
      queue.erase(queue.begin() + (long)best);
      leaders.clear();
      for (int r : m.sorted(giver, id))
        if (m.rLeader[r] && m.pTopic[m.rPart[r]] == t) leaders.push_back(r);
      int giverCount = (int)leaders.size();
      const int64_t key = e.crossScan(*this, DA_MOVE, leaders, 0, cands);
      if (key < 0) continue;
      const int r = leaders[key / (int64_t)cands.size()];
      m.relocateReplica(m.rPart[r], giver, b);
      if (++recv >= mn) return;
      if (--giverCount > mn) queue.push_back(giver);
    }
  }

  // rebalanceForBroker (:317-334)
  void rebalance(Engine& e, int b) override {
    moveAwayOffline(e, b);
    if (mustOrder.empty()) return;
    PhaseScope ps(PH_OTHER_GOALS);
    if (!(e.m.alive(b) && eligibleToHaveLeaders(e, b))) return;
    for (int t : mustOrder) moveLeaderOfTopic(e, t, b);
  }

  // moveAwayOfflineReplicas (:444-464)
  void moveAwayOffline(Engine& e, int b) {
    PhaseScope ps(PH_OTHER_GOALS);
    Model& m = e.m;
    if (!hasOffline(m, b)) return;
    std::vector<int32_t> order = aliveById(m), cands, offline, one(1);
    std::sort(order.begin(), order.end(), [&](int x, int y) {  // TreeSet by (replica count, id), built once
      return m.nrep(x) != m.nrep(y) ? m.nrep(x) < m.nrep(y) : x < y;
    });
    e.eligible(order, DA_MOVE, cands);
    ReplicaSet copy;  // new HashSet<>(srcBroker.currentOfflineReplicas())
    copy.assignCopy(m.bOfflineSet[b]);
    copy.order(offline);
    for (int r : offline) {
      one[0] = r;
      const int64_t key = e.crossScan(*this, DA_MOVE, one, 0, cands);
      if (key < 0)
        throw OptimizationFailure("[" + name + "] Cannot remove offline replica from broker " + std::to_string(m.bId[b]),
                                  underBrokers(1));
      m.relocateReplica(m.rPart[r], b, cands[key]);
    }
  }
  // updateGoalState (:279-288): the leader-count check only logs
  void update(Engine& e) override {
    ensureNoOfflineReplicas(e.m, name);
    ensureReplicasMoveOffBadDisks(e.m, name);
    finished = true;
  }
  int compareStats(const ccmi_cluster_stats&, const ccmi_cluster_stats&) const override { return 0; }
};

// ======================================================================================= ReplicaCapacityGoal
class ReplicaCapacity : public GoalImpl {
 public:
  ReplicaCapacity() {
    kind = CCMI_GOAL_REPLICA_CAPACITY;
    name = "ReplicaCapacityGoal";
  }
  bool selfHealingMode = false;
  int64_t maxR = 0;

  // initGoalState (:100-150)
  void init(Engine& e) override {
    Model& m = e.m;
    maxR = e.bc.maxReplicasPerBroker;
    selfHealingMode = m.numDead > 0 || m.numBadDisk > 0;
    if (e.opt.anyExclTopic) {
      // replicas of excluded topics stay where they are (:116-139); on a BAD_DISKS broker the offline ones leave
      for (int b = 0; b < m.B; ++b) {
        if (!m.alive(b)) continue;
        const bool badDisks = m.bState[b] == BState::BAD_DISKS;
        int64_t excluded = 0;
        for (int r : m.bRepl[b])
          if (e.opt.exclTopic[m.pTopic[m.rPart[r]]] && !(badDisks && m.curOffline(r))) excluded++;
        if (excluded > maxR)
          throw OptimizationFailure("[" + name + "] Replicas of excluded topics in broker: " + std::to_string(excluded) +
                                    " exceeds the maximum allowed number of replicas per broker: " +
                                    std::to_string(maxR) + ".");
      }
    }
    const int n = allowedForReplicaMove(e, allowed);
    const int64_t maxInCluster = maxR * n;
    if ((int64_t)m.R > maxInCluster) {
      const int minRequired = (int)std::ceil(m.R / (double)maxR);  // ReplicaCapacityGoal.java:145-148
      throw OptimizationFailure("[" + name + "] Total replicas in cluster: " + std::to_string(m.R) +
                                    " exceeds the maximum allowed replicas in cluster: " + std::to_string(maxInCluster),
                                underBrokers(minRequired - n));
    }
    Model::Spec s;
    s.selImmigrants = e.opt.onlyImmigrants;
    s.selExclTopics = e.opt.anyExclTopic;
    for (int b = 0; b < m.B; ++b) m.track(b, sortId(kind, false, false), s);
    dg = DevGoal{};
    dg.kind = DG_REPLICA_CAPACITY;
    dg.maxReplicas = maxR;
    dg.allowedSlot = e.newSlot;
  }

  // rebalanceForBroker (:221-263): rows that share one eligibleBrokers list (it only changes after a move) are
  // scanned together; failed rows before the winner are checked for the dead-broker / offline-replica failures.
  void rebalance(Engine& e, int b) override {
    PhaseScope ps(PH_OTHER_GOALS);
    Model& m = e.m;
    // the loop's break on its first replica (within the limit, and the first replica — offline ones sort first — not
    // offline) without sorting the broker's replicas: bNoff counts b's current offline replicas
    if ((int64_t)m.nrep(b) <= maxR && m.bNoff[b] == 0) return;
    const std::vector<int32_t> list = m.sorted(b, sortId(kind, false, false));
    std::vector<int32_t> order, cands;
    auto fail = [&](int r) {
      if (!m.alive(b)) throw OptimizationFailure("[" + name + "] Failed to move dead broker replica.", underBrokers(1));
      if (m.curOffline(r)) throw OptimizationFailure("[" + name + "] Failed to move offline replica.", underBrokers(1));
    };
    auto less = [&](int x, int y) { return m.nrep(x) != m.nrep(y) ? m.nrep(x) < m.nrep(y) : x < y; };
    bool built = false;
    size_t i = 0;
    while (i < list.size()) {
      size_t end = i;
      while (end < list.size() && !((int64_t)m.nrep(b) <= maxR && !m.curOffline(list[end]))) ++end;
      if (end == i) return;  // the break of the reference loop
      if (!built) {  // eligibleBrokers: a TreeSet by (replica count, id), rebuilt per replica in the reference;
                     // between replicas only the last destination's count changes, so it is repositioned below
        for (int x = 0; x < m.B; ++x)
          if (m.alive(x) && (selfHealingMode || (int64_t)m.nrep(x) < maxR) && x != b) order.push_back(x);
        std::sort(order.begin(), order.end(), less);
        built = true;
      }
      e.eligible(order, DA_MOVE, cands);
      const int64_t key = e.crossScan(*this, DA_MOVE, list, i, cands, FILTER_NONE, true, end);
      if (key < 0) {
        for (size_t q = i; q < end; ++q) fail(list[q]);
        i = end;
        continue;
      }
      const size_t k = i + (size_t)(key / (int64_t)cands.size());
      for (size_t q = i; q < k; ++q) fail(list[q]);
      const int dst = cands[key % (int64_t)cands.size()];
      order.erase(std::find(order.begin(), order.end(), dst));  // key (count) of dst changes with the move
      m.relocateReplica(m.rPart[list[k]], b, dst);
      if (selfHealingMode || (int64_t)m.nrep(dst) < maxR)
        order.insert(std::lower_bound(order.begin(), order.end(), dst, less), dst);
      i = k + 1;
    }
  }

  // updateGoalState (:165-181) + ensureReplicaCapacitySatisfied (:183-196)
  void update(Engine& e) override {
    Model& m = e.m;
    ensureNoOfflineReplicas(m, name);
    if (!selfHealingMode) {
      for (int b = 0; b < m.B; ++b)
        if ((int64_t)m.nrep(b) > maxR)
          throw OptimizationFailure("[" + name + "] Replica count in broker " + std::to_string(b) +
                                        " exceeds the maximum allowed number of replicas per broker.",
                                    underBrokers(1));
      finished = true;
    } else {
      selfHealingMode = false;
    }
  }
  int compareStats(const ccmi_cluster_stats&, const ccmi_cluster_stats&) const override { return 0; }
};

// ======================================================================================= CapacityGoal
class Capacity : public GoalImpl {
 public:
  explicit Capacity(int kindIn) {
    kind = kindIn;
    switch (kindIn) {
      case CCMI_GOAL_CPU_CAPACITY: res = R_CPU; name = "CpuCapacityGoal"; break;
      case CCMI_GOAL_NW_IN_CAPACITY: res = R_NW_IN; name = "NetworkInboundCapacityGoal"; break;
      case CCMI_GOAL_NW_OUT_CAPACITY: res = R_NW_OUT; name = "NetworkOutboundCapacityGoal"; break;
      default: res = R_DISK; name = "DiskCapacityGoal"; break;
    }
  }
  int res = 0;
  double thr = 0;
  static const char* resName(int r) {
    switch (r) {
      case R_CPU: return "CPU";
      case R_NW_IN: return "NW_IN";
      case R_NW_OUT: return "NW_OUT";
      default: return "DISK";
    }
  }

  // initGoalState (:120-170)
  void init(Engine& e) override {
    Model& m = e.m;
    thr = e.bc.capThreshold[res];
    const int n = allowedForReplicaMove(e, allowed);
    const double existing = m.clusterUtil(res);
    const double capacity = m.capacityWithAllowedReplicaMoves(res, e.opt.exclMove);
    if (capacity * thr < existing) {
      if (n == 0)
        throw OptimizationFailure("[" + name + "] All alive brokers are excluded from replica moves.", underBrokers(m.maxRf));
      // a typical broker: the first of aliveBrokersNotExcludedForReplicaMove (a HashSet<Integer>) (:160-166)
      std::vector<int> ids, ord;
      for (int b = 0; b < m.B; ++b)
        if (allowed[b]) ids.push_back(b);
      javaHashSetOrder(ids, ord);
      const int typical = ord.front();
      const double typicalCapacity = m.cap(typical, res);
      ccmi_provision_recommendation rec =
          underBrokers((int)std::ceil((existing - capacity * thr) / (typicalCapacity * thr)), res);
      rec.typical_broker_capacity = typicalCapacity;
      rec.typical_broker_id = m.bId[typical];
      throw OptimizationFailure("[" + name + "] Insufficient capacity for " + resName(res) + ".", rec);
    }
    const bool selfHealing = m.numSelfHealing > 0;
    Model::Spec all;
    all.selImmigrants = e.opt.onlyImmigrants;
    all.selExclTopics = e.opt.anyExclTopic;
    all.prioOffline = selfHealing;
    all.prioImmigrants = !e.opt.onlyImmigrants;
    all.scoreRes = res;
    all.scoreReverse = true;
    Model::Spec leaders;
    leaders.selLeaders = true;
    leaders.selImmigrants = e.opt.onlyImmigrants;
    leaders.selExclTopics = e.opt.anyExclTopic;
    leaders.prioImmigrants = !e.opt.onlyImmigrants;
    leaders.scoreRes = res;
    leaders.scoreReverse = true;
    for (int b = 0; b < m.B; ++b) {
      m.track(b, sortId(kind, true, false), all);
      m.track(b, sortId(kind, true, true), leaders);
    }
    dg = DevGoal{};
    dg.kind = DG_CAPACITY;
    dg.resource = res;
    dg.capThr = thr;
    dg.allowedSlot = e.newSlot;
  }

  // isUtilizationOverLimit (:389-408) with rebalanceForBroker's limits, computed once per broker (:282-284)
  struct Limits {
    double broker, host;
  };
  Limits limits(const Model& m, int b) const { return {m.cap(b, res) * thr, m.hcap(b, res) * thr}; }
  bool over(const Model& m, int b, const Limits& L) const {
    if (!m.hostEmpty(b) && isHostRes(res) && m.hu(b, res) > L.host) return true;
    if (m.nrep(b) > 0 && isBrokerRes(res)) return m.bu(b, res) > L.broker;
    return false;
  }

  // rebalanceForBroker (:274-349)
  void rebalance(Engine& e, int b) override {
    PhaseScope ps(PH_OTHER_GOALS);
    Model& m = e.m;
    const Limits L = limits(m, b);
    auto over = [&](const Model& mm, int x) { return this->over(mm, x, L); };
    bool isOver = over(m, b);
    if (!isOver && !hasOffline(m, b)) return;
    if (res == R_NW_OUT || res == R_CPU) {
      const std::vector<int32_t> leaders = m.sorted(b, sortId(kind, true, true));
      std::vector<int32_t> pr, pb, owner, fol;
      // each row's sorted eligible followers, kept between scans: a move changes the utilization of b (the leader of
      // every row) and dst only, so only rows with dst among their followers are re-sorted
      std::vector<std::vector<int32_t>> rowCands(leaders.size());
      std::vector<uint8_t> rowValid(leaders.size(), 0);
      size_t i = 0;
      while (i < leaders.size()) {
        // every remaining leader with its online followers' brokers by (utilization, id)
        pr.clear();
        pb.clear();
        owner.clear();
        for (size_t q = i; q < leaders.size(); ++q) {
          const int r = leaders[q];
          std::vector<int32_t>& elig = rowCands[q];
          if (!rowValid[q]) {
            m.onlineFollowerBrokers(m.rPart[r], fol);
            std::sort(fol.begin(), fol.end(), [&](int x, int y) {
              const int c = jcmpDouble(m.bu(x, res), m.bu(y, res));
              return c ? c < 0 : x < y;
            });
            e.eligible(fol, DA_LEADERSHIP, elig);
            rowValid[q] = 1;
          }
          for (int x : elig) {
            pr.push_back(r);
            pb.push_back(x);
            owner.push_back((int)q);
          }
        }
        const int64_t key = e.pairScan(*this, pr, pb);
        if (key < 0) break;
        const size_t k = (size_t)owner[key];
        const int dst = pb[key];
        m.relocateLeadership(m.rPart[leaders[k]], b, dst);
        isOver = over(m, b);
        if (!isOver) break;
        i = k + 1;
        for (size_t q = i; q < leaders.size(); ++q)
          if (rowValid[q] && m.replicaOn(m.rPart[leaders[q]], dst) >= 0) rowValid[q] = 0;
      }
    }
    if (isOver || hasOffline(m, b)) {
      // sortedAliveBrokersUnderThreshold (ClusterModel.java:1049-1095): a snapshot list; aliveBrokersUnderThreshold
      // checks the broker for a broker resource and the host for a host resource, and the sort compares host
      // utilization first for a host resource
      std::vector<int32_t> under, cands;
      for (int x = 0; x < m.B; ++x) {
        if (!m.alive(x)) continue;
        if (isBrokerRes(res) && m.bu(x, res) >= m.cap(x, res) * thr) continue;
        if (isHostRes(res) && m.hu(x, res) >= m.hcap(x, res) * thr) continue;
        under.push_back(x);
      }
      stableSortBy(under, [&](int x, int y) {
        const int hc = isHostRes(res) ? jcmpDouble(m.hu(x, res), m.hu(y, res)) : 0;
        return hc == 0 ? jcmpDouble(m.bu(x, res), m.bu(y, res)) : hc;
      });
      e.eligible(under, DA_MOVE, cands);
      const std::vector<int32_t> list = m.sorted(b, sortId(kind, true, false));
      size_t i = 0;
      while (i < list.size()) {
        const int64_t key = e.crossScan(*this, DA_MOVE, list, i, cands);
        if (key < 0) break;
        const size_t k = i + (size_t)(key / (int64_t)cands.size());
        m.relocateReplica(m.rPart[list[k]], b, cands[key % (int64_t)cands.size()]);
        isOver = over(m, b);
        if (!isOver && !hasOffline(m, b)) break;
        i = k + 1;
      }
    }
    // postSanityCheck (:332-355)
    if (isOver)
      throw OptimizationFailure("[" + name + "] Utilization of broker " + std::to_string(b) +
                                    " violated capacity limit for resource " + resName(res) + ".",
                                underBrokers(1, res));
    if (hasOffline(m, b))
      throw OptimizationFailure("[" + name + "] Cannot remove offline replicas from broker " + std::to_string(b) + ".",
                                underBrokers(1, res));
  }

  // updateGoalState (:180-190) + ensureUtilizationUnderCapacity (:192-225)
  void update(Engine& e) override {
    Model& m = e.m;
    for (int b = 0; b < m.B; ++b) {  // the host check first (a host resource), then the broker check (a broker resource)
      if (isHostRes(res) && !m.hostEmpty(b) && m.hu(b, res) > m.hcap(b, res) * thr)
        throw OptimizationFailure("[" + name + "] utilization for host is above capacity limit.", underBrokers(1, res));
      if (isBrokerRes(res) && m.nrep(b) > 0 && m.bu(b, res) > m.cap(b, res) * thr)
        throw OptimizationFailure("[" + name + "] utilization for broker is above capacity limit.",
                                  underBrokers(1, res));
    }
    ensureNoOfflineReplicas(m, name);
    finished = true;
  }
  int compareStats(const ccmi_cluster_stats&, const ccmi_cluster_stats&) const override { return 0; }
};

// ======================================================================================= PotentialNwOutGoal
class PotentialNwOut : public GoalImpl {
 public:
  PotentialNwOut() {
    kind = CCMI_GOAL_POTENTIAL_NW_OUT;
    name = "PotentialNwOutGoal";
  }
  bool fix = false;
  double thr = 0;

  void init(Engine& e) override {  // initGoalState (:185-195)
    Model& m = e.m;
    allowedForReplicaMove(e, allowed);
    thr = e.bc.capThreshold[R_NW_OUT];
    fix = false;
    Model::Spec s;
    s.selImmigrants = e.opt.onlyImmigrants;
    s.selExclTopics = e.opt.anyExclTopic;
    for (int b = 0; b < m.B; ++b) m.track(b, sortId(kind, false, false), s);
    dg = DevGoal{};
    dg.kind = DG_POTENTIAL_NW_OUT;
    dg.capThr = thr;
    dg.allowedSlot = e.newSlot;
  }
  // brokersToBalance (:140-150): the broken brokers if any, else all
  std::vector<int> brokersToBalance(Engine& e) override {
    if (e.m.numDead == 0) return GoalImpl::brokersToBalance(e);
    std::vector<int> v;
    for (int b = 0; b < e.m.B; ++b)
      if (!e.m.alive(b)) v.push_back(b);
    return v;
  }
  bool over(const Model& m, int b) const { return m.nrep(b) > 0 && m.potNwOut(b) > m.cap(b, R_NW_OUT) * thr; }

  // rebalanceForBroker (:270-331). The reference re-sorts the candidate list per replica; the sorted order only
  // changes after a move, so the remaining replicas are scanned against the whole sorted list at once: a
  // partition broker fails legitMove exactly where the reference had removed it, and is left out of the count.
  void rebalance(Engine& e, int b) override {
    PhaseScope ps(PH_OTHER_GOALS);
    Model& m = e.m;
    bool isOver = over(m, b);
    if (!isOver && !(fix && hasOffline(m, b))) return;
    std::vector<int32_t> candidates;
    if (fix) {
      candidates = aliveById(m);
    } else {
      std::vector<int> under;
      for (int x = 0; x < m.B; ++x)
        if (m.alive(x) && m.potNwOut(x) < m.cap(x, R_NW_OUT) * thr) under.push_back(x);
      std::vector<int> ord;
      javaHashSetOrder(under, ord);  // brokersUnderEstimatedMaxPossibleNwOut: a HashSet
      candidates.assign(ord.begin(), ord.end());
    }
    const std::vector<int32_t> list = m.sorted(b, sortId(kind, false, false));
    std::vector<int32_t> sortedC, cands, pos(m.B, -1);
    size_t i = 0;
    while (i < list.size()) {
      sortedC = candidates;
      stableSortBy(sortedC, [&](int x, int y) {
        return jcmpDouble(m.ops.util(m.bLnw[y], R_NW_OUT), m.ops.util(m.bLnw[x], R_NW_OUT));
      });
      e.eligible(sortedC, DA_MOVE, cands);
      for (size_t j = 0; j < cands.size(); ++j) pos[cands[j]] = (int)j;
      const int64_t key = e.crossScan(*this, DA_MOVE, list, i, cands, FILTER_NONE, false);
      const size_t N = cands.size();
      const size_t kEnd = key < 0 ? list.size() : i + (size_t)(key / (int64_t)std::max<size_t>(N, 1));
      const bool newOnly = m.numNew > 0 && !e.opt.anyRequested;
      auto rowCount = [&](int r, size_t upto) {  // visited eligible brokers of one row: partition brokers removed
        int64_t c = (int64_t)upto;
        const int p = m.rPart[r];
        // a leader replica skips brokers excluded for leadership (GoalUtils.java:170-180); with NEW brokers only NEW
        // brokers or the replica's original broker are eligible (:193-198)
        const bool exclLead = e.opt.anyExclLead && !e.opt.anyRequested && m.rLeader[r];
        if (newOnly || exclLead) {
          c = 0;
          for (size_t j = 0; j < upto; ++j) {
            const int x = cands[j];
            if (m.replicaOn(p, x) >= 0) continue;
            if (newOnly && !(m.isNew(x) || x == m.rOrig[r])) continue;
            if (exclLead && e.opt.exclLead[x]) continue;
            c++;
          }
          return c;
        }
        for (int s = m.pOff[p]; s < m.pOff[p + 1]; ++s) {
          const int x = pos[m.rBroker[m.pSlots[s]]];
          if (x >= 0 && (size_t)x < upto) c--;
        }
        return c;
      };
      for (size_t q = i; q < kEnd && q < list.size(); ++q) e.candidates += rowCount(list[q], N);
      if (key >= 0) e.candidates += rowCount(list[kEnd], (size_t)(key % (int64_t)N) + 1);
      for (int x : cands) pos[x] = -1;
      if (key < 0) break;
      const int dst = cands[key % (int64_t)N];
      m.relocateReplica(m.rPart[list[kEnd]], b, dst);
      isOver = over(m, b);
      if (!isOver && !(fix && hasOffline(m, b))) break;
      if (!fix && m.potNwOut(dst) > m.cap(dst, R_NW_OUT) * thr)
        candidates.erase(std::find(candidates.begin(), candidates.end(), dst));
      i = kEnd + 1;
    }
    if (isOver) succeeded = false;
  }
  // updateGoalState (:197-213)
  void update(Engine& e) override {
    Model& m = e.m;
    for (int r = 0; r < m.R; ++r)
      if (m.selfHealing[r] && m.curOffline(r)) {
        if (fix)
          throw OptimizationFailure("[" + name + "] Cannot remove replica from broker " + std::to_string(m.bId[m.rBroker[r]]),
                                    underBrokers(1));
        fix = true;
        dg.fixOffline = 1;
        return;
      }
    finished = true;
  }
  int compareStats(const ccmi_cluster_stats& after, const ccmi_cluster_stats& before) const override {
    return jcmpInt(after.num_brokers_under_potential_nw_out, before.num_brokers_under_potential_nw_out);
  }
};

// ======================================================================================= TopicReplicaDistributionGoal
class TopicReplicaDistribution : public GoalImpl {
 public:
  TopicReplicaDistribution() {
    kind = CCMI_GOAL_TOPIC_REPLICA_DISTRIBUTION;
    name = "TopicReplicaDistributionGoal";
  }
  bool fix = false, anyAbove = false, anyUnder = false;
  std::vector<uint8_t> rebalanceTopic;
  std::vector<int32_t> upper, lower;
  std::vector<int32_t> topicsScratch, perOff, perN;
  std::vector<uint32_t> perStamp;
  std::vector<uint8_t> perImm;
  uint32_t stamp = 0;
  int sid() const { return sortId(kind, false, false); }
  bool excluded(int b) const { return !allowed[b]; }

  // initGoalState (:225-270) with the gap-based limits (:95-150)
  void init(Engine& e) override {
    Model& m = e.m;
    const int n = allowedForReplicaMove(e, allowed);
    if (n == 0)
      throw OptimizationFailure("[" + name + "] All alive brokers are excluded from replica moves.", underBrokers(m.maxRf));
    const bool selfHealing = m.numSelfHealing > 0;
    rebalanceTopic.assign(m.T, selfHealing ? 0 : 1);
    if (selfHealing)
      for (int r = 0; r < m.R; ++r)
        if (m.selfHealing[r]) rebalanceTopic[m.pTopic[m.rPart[r]]] = 1;
    if (!selfHealing && e.opt.anyExclTopic)  // GoalUtils.topicsToRebalance (GoalUtils.java:439-452)
      for (int t = 0; t < m.T; ++t)
        if (e.opt.exclTopic[t]) rebalanceTopic[t] = 0;
    const double margin = (e.bc.topicReplicaBalance - 1) * kBalanceMargin;
    upper.assign(m.T, 0);
    lower.assign(m.T, 0);
    for (int t = 0; t < m.T; ++t) {
      const double avg = m.topicNrep[t] / (double)n;
      const int cu = (int)std::ceil(avg * (1 + margin));
      const int umin = (int)(std::ceil(avg) + e.bc.topicMinGap), umax = (int)(std::ceil(avg) + e.bc.topicMaxGap);
      upper[t] = std::max(umin, std::min(cu, umax));
      const int cl = (int)std::floor(avg * jmax(0, (1 - margin)));
      const int lmax = std::max(0, (int)(std::floor(avg) - e.bc.topicMinGap));
      const int lmin = std::max(0, (int)(std::floor(avg) - e.bc.topicMaxGap));
      lower[t] = std::max(lmin, std::min(cl, lmax));
    }
    for (int b = 0; b < m.B; ++b) {
      Model::Spec s;
      s.selImmigrants = e.opt.onlyImmigrants;
      s.selImmOrOffline = selfHealing && m.alive(b);
      s.selExclTopics = e.opt.anyExclTopic;
      m.track(b, sid(), s);
    }
    fix = false;
    e.topicUpper = upper;
    e.topicLower = lower;
    e.dev->setTopicLimits(upper.data(), lower.data());
    dg = DevGoal{};
    dg.kind = DG_TOPIC_REPLICA_DISTRIBUTION;
    dg.allowedSlot = e.newSlot;
  }

  // updateGoalState (:318-345)
  void update(Engine& e) override {
    if (anyAbove) succeeded = false;
    if (anyUnder) succeeded = false;
    anyAbove = anyUnder = false;
    Model& m = e.m;
    for (int r = 0; r < m.R; ++r)
      if (m.selfHealing[r] && m.curOffline(r)) {
        if (fix)
          throw OptimizationFailure("[" + name + "] Cannot remove replica from broker " + std::to_string(m.bId[m.rBroker[r]]),
                                    underBrokers(1));
        fix = true;
        dg.fixOffline = 1;
        return;
      }
    finished = true;
  }
  int compareStats(const ccmi_cluster_stats& after, const ccmi_cluster_stats& before) const override {
    return cmpStd(after.topic_replica_std, before.topic_replica_std);
  }

  // rebalanceForBroker (:386-443) + skipBrokerRebalance (:348-377)
  void rebalance(Engine& e, int b) override {
    PhaseScope ps(PH_OTHER_GOALS);
    Model& m = e.m;
    std::vector<int32_t>& topics = topicsScratch;
    // per-topic (offline count, has immigrant) of this broker's replicas, one pass (recounted after moves); the
    // per-topic slots are valid for the current stamp only
    if (perStamp.size() != (size_t)m.T) {
      perStamp.assign(m.T, 0);
      perOff.assign(m.T, 0);
      perN.assign(m.T, 0);
      perImm.assign(m.T, 0);
    }
    auto recount = [&]() {
      ++stamp;
      for (int r : m.bRepl[b]) {
        const int t = m.pTopic[m.rPart[r]];
        if (perStamp[t] != stamp) {
          perStamp[t] = stamp;
          perOff[t] = 0;
          perN[t] = 0;
          perImm[t] = 0;
        }
        perOff[t] += m.rInOff[r];
        perN[t] += 1;
        perImm[t] |= m.rInImm[r];
      }
    };
    recount();
    m.bTopicKeys[b].order(topics);  // Broker.topics(): HashMap key order (keys stay after a topic's last replica left)
    for (int t : topics) {
      if (!rebalanceTopic[t]) continue;
      const bool seen = perStamp[t] == stamp;
      // b's replica count of t from the same pass (Broker.numReplicasOfTopicInBroker) instead of the [T][B] count
      // table, whose row-per-topic layout makes every lookup here a cache miss
      const int nOff = seen ? perOff[t] : 0, hasImm = seen ? perImm[t] : 0, n = seen ? perN[t] : 0;
      const bool excl = excluded(b);
      const bool requireLess = nOff > 0 || n > upper[t] || excl;
      const bool requireMore = !excl && m.alive(b) && n - nOff < lower[t];
      if (m.alive(b) && !requireMore && !requireLess) continue;
      if (m.numNew > 0 && !m.isNew(b) && !requireLess) continue;
      if (m.numSelfHealing > 0 && requireLess && nOff == 0 && !hasImm) continue;
      if (e.opt.onlyImmigrants && requireLess && !hasImm) continue;
      if (requireLess && moveOut(e, b, t)) anyAbove = true;
      if (requireMore && moveIn(e, b, t)) anyUnder = true;
      if (requireLess || requireMore) recount();  // the moves changed this broker's replicas
    }
  }

  // replicasToMoveOut (:445-451): the topic's replicas of b that the tracked set selects, ordered by
  // Broker.replicaComparator (offline first, immigrants first, partition number)
  void replicasToMoveOut(Model& m, int b, int t, std::vector<int32_t>& out) {
    out.clear();
    for (int r : m.bRepl[b])
      if (m.pTopic[m.rPart[r]] == t && selected(m, b, r)) out.push_back(r);
    std::sort(out.begin(), out.end(), [&](int x, int y) {
      const bool ox = m.rInOff[x] != 0, oy = m.rInOff[y] != 0;
      if (ox != oy) return ox;
      const bool ix = m.rInImm[x] != 0, iy = m.rInImm[y] != 0;
      if (ix != iy) return ix;
      return m.pNumber[m.rPart[x]] < m.pNumber[m.rPart[y]];
    });
  }
  // membership in the tracked SortedReplicas of b (its selection functions, evaluated on live state)
  bool selected(const Model& m, int b, int r) const {
    for (const auto& t : m.tracked[b])
      if (t.nameId == sid()) return m.selects(t.spec, r);
    return true;
  }

  // rebalanceByMovingReplicasOut (:453-505): consecutive rows share the live TreeSet's in-order list until a move
  bool moveOut(Engine& e, int b, int t) {
    Model& m = e.m;
    auto cmp = [&m, t](int x, int y) {
      const int c = jcmpInt(m.tcount(t, x), m.tcount(t, y));
      return c ? c : jcmpInt(m.bId[x], m.bId[y]);
    };
    RbTreeSet<decltype(cmp)> cand(cmp);
    {
      std::vector<int> ins, order;
      for (int x = 0; x < m.B; ++x)
        if (m.alive(x) && (fix || m.tcount(t, x) < upper[t])) ins.push_back(x);
      if (fix) order = ins;
      else javaHashSetOrder(ins, order);  // Collectors.toSet()
      for (int x : order) cand.add(x);
    }
    cand.trackSequence();
    int n = m.tcount(t, b), nOff = 0;
    for (int r : m.bRepl[b])
      if (m.pTopic[m.rPart[r]] == t && m.rInOff[r]) nOff++;
    const int upperSrc = excluded(b) ? 0 : upper[t];
    bool wasUnable = false;
    std::vector<int32_t> list, inorder, cands;
    replicasToMoveOut(m, b, t, list);
    size_t i = 0;
    while (i < list.size()) {
      // a run of rows with equal offline status: the early return is decided at the run's first row
      if (wasUnable && !m.curOffline(list[i]) && n <= upperSrc) return false;
      const bool runOffline = m.curOffline(list[i]);
      size_t end = i;
      while (end < list.size() && m.curOffline(list[end]) == runOffline) ++end;
      const std::vector<int32_t>* seq = cand.sequence();  // the maintained sequence itself (no copy)
      if (!seq) {
        cand.inorder(inorder);
        seq = &inorder;
      }
      const std::vector<int32_t>& cl = e.eligibleView(*seq, DA_MOVE, cands);
      const int64_t key = e.crossScan(*this, DA_MOVE, list, i, cl, FILTER_NONE, true, end);
      if (key < 0) {
        if (runOffline) wasUnable = true;
        i = end;
        continue;
      }
      const size_t N = cl.size();
      const size_t k = i + (size_t)(key / (int64_t)N);
      if (runOffline && k > i) wasUnable = true;
      const int r = list[k], dst = cl[key % (int64_t)N];  // (read before the tree changes below)
      const bool wasOffline = m.curOffline(r);
      m.relocateReplica(m.rPart[r], b, dst);
      if (wasOffline) nOff--;
      if (--n <= (nOff == 0 ? upperSrc : 0)) return false;
      cand.remove(dst);
      if (m.tcount(t, dst) < upper[t] || fix) cand.add(dst);
      i = k + 1;
    }
    return m.tcount(t, b) != 0;
  }

  // rebalanceByMovingReplicasIn (:507-570)
  bool moveIn(Engine& e, int dest, int t) {
    Model& m = e.m;
    auto offCount = [&](int x) {
      int k = 0;
      for (int r : m.bRepl[x])
        if (m.pTopic[m.rPart[r]] == t && m.rInOff[r]) k++;
      return k;
    };
    auto cmp = [&](int b1, int b2) {
      const int r = jcmpInt(offCount(b2), offCount(b1));
      if (r == 0) {
        const int r2 = jcmpInt(m.tcount(t, b2), m.tcount(t, b1));
        return r2 == 0 ? jcmpInt(m.bId[b1], m.bId[b2]) : r2;
      }
      return r;
    };
    JavaPQ<decltype(cmp)> pq(cmp);
    for (int s = 0; s < m.B; ++s) {
      if (fix) {
        if (s != dest) pq.add(s);
      } else if (m.tcount(t, s) > lower[t] || hasOffline(m, s) || excluded(s)) {
        pq.add(s);
      }
    }
    int n = m.tcount(t, dest);
    std::vector<int32_t> single{dest}, cands, toMove;
    e.eligible(single, DA_MOVE, cands);
    while (!pq.empty()) {
      const int src = pq.poll();
      replicasToMoveOut(m, src, t, toMove);
      int nOff = 0;
      for (int r : toMove)
        if (m.rInOff[r]) nOff++;
      size_t i = 0;
      while (i < toMove.size()) {
        const int64_t key = cands.empty() ? -1 : e.crossScan(*this, DA_MOVE, toMove, i, cands);
        if (key < 0) break;
        const size_t k = i + (size_t)key;
        const bool wasOffline = m.curOffline(toMove[k]);
        m.relocateReplica(m.rPart[toMove[k]], src, dest);
        if (wasOffline) nOff--;
        if (++n >= lower[t]) return false;
        if (!pq.empty() && nOff == 0 && m.tcount(t, src) < m.tcount(t, pq.peek())) {
          pq.add(src);
          break;
        }
        i = k + 1;
      }
    }
    return true;
  }
};

// ======================================================================================= TopicLeaderReplicaDistributionGoal
// Per-topic leader counts (Broker.numLeadersFor) live in the model and on the device (Model::enableTopicLeaders);
// the goal's per-topic limits go to the device as (upper, lower) pairs.
class TopicLeaderReplicaDistribution : public GoalImpl {
 public:
  TopicLeaderReplicaDistribution() {
    kind = CCMI_GOAL_TOPIC_LEADER_REPLICA_DISTRIBUTION;
    name = "TopicLeaderReplicaDistributionGoal";
  }
  bool fix = false, anyAbove = false, anyUnder = false;
  std::vector<uint8_t> rebalanceTopic;  // the keys of _avgTopicLeaderReplicasOnAliveBroker (topicsToRebalance)
  std::vector<int32_t> upper, lower;
  Model::Spec specAlive, specDead;  // selection functions of the tracked leaders-only view (alive / dead broker)
  bool excluded(int b) const { return !allowed[b]; }
  const Model::Spec& spec(const Model& m, int b) const { return m.alive(b) ? specAlive : specDead; }

  // initGoalState (:298-347) with the limits of balancePercentageWithMargin / clampLower / clampUpper (:101-168); an
  // empty _brokersAllowedReplicaMove is allowed (leadership-only balancing): the average is then x / 0.0
  void init(Engine& e) override {
    Model& m = e.m;
    const int n = allowedForReplicaMove(e, allowed);
    const bool selfHealing = m.numSelfHealing > 0;
    rebalanceTopic.assign(m.T, selfHealing ? 0 : 1);
    if (selfHealing)
      for (int r = 0; r < m.R; ++r)
        if (m.selfHealing[r]) rebalanceTopic[m.pTopic[m.rPart[r]]] = 1;
    if (!selfHealing && e.opt.anyExclTopic)  // GoalUtils.topicsToRebalance (GoalUtils.java:439-452)
      for (int t = 0; t < m.T; ++t)
        if (e.opt.exclTopic[t]) rebalanceTopic[t] = 0;
    double pct = e.bc.topicLeaderBalance;
    if (e.opt.triggered) pct *= e.bc.goalViolationMultiplier;
    const double margin = (pct - 1) * e.bc.topicLeaderMargin;
    std::vector<int32_t> leaders(m.T, 0);  // ClusterModel.numLeadersPerTopic: one leader per partition
    for (int p = 0; p < m.P; ++p) leaders[m.pTopic[p]]++;
    const int32_t minGap = e.bc.topicLeaderMinGap, maxGap = e.bc.topicLeaderMaxGap;
    upper.assign(m.T, 0);
    lower.assign(m.T, 0);
    e.topicLeadLim.assign(2 * (size_t)m.T, 0);
    for (int t = 0; t < m.T; ++t) {
      const double avg = leaders[t] / (double)n;
      const int32_t ceilAvg = jD2I(std::ceil(avg)), floorAvg = jD2I(std::floor(avg));
      const int32_t cu = jD2I(std::ceil(avg * (1 + margin)));
      upper[t] = std::max(jAddI(ceilAvg, minGap), std::min(cu, jAddI(ceilAvg, maxGap)));
      const int32_t cl = jD2I(std::floor(avg * jmax(0, (1 - margin))));
      lower[t] = std::max(std::max(0, jSubI(floorAvg, maxGap)), std::min(cl, std::max(0, jSubI(floorAvg, minGap))));
      e.topicLeadLim[2 * (size_t)t] = upper[t];
      e.topicLeadLim[2 * (size_t)t + 1] = lower[t];
    }
    specAlive = Model::Spec{};
    specAlive.selLeaders = true;
    specAlive.selImmigrants = e.opt.onlyImmigrants;
    specAlive.selExclTopics = e.opt.anyExclTopic;
    specDead = specAlive;
    specAlive.selImmOrOffline = selfHealing;
    fix = false;
    m.enableTopicLeaders();
    e.dev->setTopicLeadLimits(e.topicLeadLim.data());
    dg = DevGoal{};
    dg.kind = DG_TOPIC_LEADER_DISTRIBUTION;
    dg.allowedSlot = e.newSlot;
  }

  // updateGoalState (:382-424)
  void update(Engine& e) override {
    if (anyAbove || anyUnder) succeeded = false;
    anyAbove = anyUnder = false;
    Model& m = e.m;
    for (int r = 0; r < m.R; ++r)
      if (m.selfHealing[r] && m.curOffline(r)) {
        if (fix)
          throw OptimizationFailure("[" + name + "] Cannot remove replica from broker " + std::to_string(m.bId[m.rBroker[r]]),
                                    underBrokers(1));
        fix = true;
        dg.fixOffline = 1;
        return;
      }
    ensureReplicasMoveOffBadDisks(m, name);
    finished = true;
  }
  // GoalUtils.HardGoalStatsComparator (:269-272)
  int compareStats(const ccmi_cluster_stats&, const ccmi_cluster_stats&) const override { return 0; }

  // rebalanceForBroker (:518-583) + skipBrokerRebalance and its helpers (:426-504)
  void rebalance(Engine& e, int b) override {
    PhaseScope ps(PH_OTHER_GOALS);
    Model& m = e.m;
    std::vector<int32_t> topics;
    m.bTopicKeys[b].order(topics);  // Broker.topics(): HashMap key order
    // per topic: the tracked view's leaders, their offline count, whether one is an immigrant (recounted after moves)
    struct Count {
      int n = 0, off = 0;
      bool imm = false;
    };
    std::unordered_map<int, Count> per;
    auto recount = [&]() {
      per.clear();
      const Model::Spec& s = spec(m, b);
      for (int r : m.bRepl[b]) {
        if (!m.rLeader[r] || !m.selects(s, r)) continue;
        Count& c = per[m.pTopic[m.rPart[r]]];
        c.n++;
        c.off += m.rInOff[r] ? 1 : 0;
        c.imm |= m.rInImm[r] != 0;
      }
    };
    recount();
    for (int t : topics) {
      if (!rebalanceTopic[t]) continue;
      const auto it = per.find(t);
      const Count c = it == per.end() ? Count{} : it->second;
      const bool excl = excluded(b);
      const bool requireLess = c.off > 0 || c.n > upper[t] || excl;
      const bool requireMore = !excl && m.alive(b) && c.n - c.off < lower[t];
      if (m.alive(b) && !requireMore && !requireLess) continue;
      if (m.numNew > 0 && !m.isNew(b) && !requireLess) continue;
      if (m.numSelfHealing > 0 && requireLess && c.off == 0 && !c.imm) continue;
      if (e.opt.onlyImmigrants && requireLess && !c.imm) continue;
      if (requireLess && moveOut(e, b, t)) anyAbove = true;
      if (requireMore && moveIn(e, b, t)) anyUnder = true;
      recount();
    }
  }

  // replicasToMoveOut (:591-596): the topic's leaders of b that the tracked view selects, ordered by
  // Broker.replicaComparator (offline first, immigrants first, partition number)
  void replicasToMoveOut(const Model& m, int b, int t, std::vector<int32_t>& out) const {
    out.clear();
    const Model::Spec& s = spec(m, b);
    for (int r : m.bRepl[b])
      if (m.rLeader[r] && m.pTopic[m.rPart[r]] == t && m.selects(s, r)) out.push_back(r);
    std::sort(out.begin(), out.end(), [&](int x, int y) {
      const bool ox = m.rInOff[x] != 0, oy = m.rInOff[y] != 0;
      if (ox != oy) return ox;
      const bool ix = m.rInImm[x] != 0, iy = m.rInImm[y] != 0;
      if (ix != iy) return ix;
      return m.pNumber[m.rPart[x]] < m.pNumber[m.rPart[y]];
    });
  }

  // rebalanceByMovingLeadersOut (:598-678). Every leader first tries a leadership transfer to the candidates
  // hosting a follower, then a replica move to the candidates not hosting the partition, each over a HashSet built
  // from the candidate TreeSet. Rows of one offline-status run are scanned together: one pair scan over all rows'
  // leadership candidates, then cross scans of the rows before the first leadership winner; a replica-move list is
  // the ascending-id list of all candidates (the device rejects the hosts) whenever the row's HashSet has no bucket
  // collisions, else the row's own HashSet order.
  bool moveOut(Engine& e, int b, int t) {
    Model& m = e.m;
    auto cmp = [&m, t](int x, int y) {
      int c = jcmpInt(m.tlead(t, x), m.tlead(t, y));
      if (c == 0) c = jcmpInt(m.bNlead[x], m.bNlead[y]);
      return c ? c : jcmpInt(m.bId[x], m.bId[y]);
    };
    RbTreeSet<decltype(cmp)> cand(cmp);
    {
      PhaseScope pi(PH_PQ_INIT);
      std::vector<int> ins, order;
      for (int x = 0; x < m.B; ++x)
        if (m.alive(x) && (fix || m.tlead(t, x) < upper[t])) ins.push_back(x);
      if (fix) order = ins;  // ClusterModel.aliveBrokers(): ascending id
      else javaHashSetOrder(ins, order);  // Collectors.toSet()
      // the same TreeSet.add sequence, placed by rank (the comparator is a total order on these brokers)
      std::vector<int32_t> byKey(ins.begin(), ins.end()), rank(m.B, 0);
      std::sort(byKey.begin(), byKey.end(), [&](int x, int y) { return cmp(x, y) < 0; });
      for (size_t i = 0; i < byKey.size(); ++i) rank[byKey[i]] = (int32_t)i;
      cand.buildByRank(order, rank);
    }
    int n = 0, nOff = 0;
    for (int r : m.bRepl[b])
      if (m.rLeader[r] && m.pTopic[m.rPart[r]] == t) {
        n++;
        nOff += m.rInOff[r] ? 1 : 0;
      }
    const int upperSrc = upper[t];
    std::vector<int32_t> list;
    replicasToMoveOut(m, b, t, list);
    bool wasUnable = false;
    std::vector<int> inorder, ins, hs;
    std::vector<int32_t> pos(m.B, -1), pr, pb, leadOff, ids, idElig, own, hs32;
    size_t i = 0;
    while (i < list.size()) {
      if (wasUnable && !m.curOffline(list[i]) && n <= upperSrc) return false;
      const bool runOffline = m.curOffline(list[i]);
      size_t end = i;
      while (end < list.size() && m.curOffline(list[end]) == runOffline) ++end;
      for (int x : inorder) pos[x] = -1;
      cand.inorder(inorder);
      for (size_t q = 0; q < inorder.size(); ++q) pos[inorder[q]] = (int32_t)q;
      // the candidates hosting one of the row's partition's replicas, in TreeSet order
      auto hostsInOrder = [&](int r, bool followersOnly, std::vector<int>& out) {
        out.clear();
        const int p = m.rPart[r];
        for (int s = m.pOff[p]; s < m.pOff[p + 1]; ++s) {
          const int rr = m.pSlots[s], x = m.rBroker[rr];
          if (pos[x] >= 0 && !(followersOnly && m.rLeader[rr])) out.push_back(x);
        }
        std::sort(out.begin(), out.end(), [&](int x, int y) { return pos[x] < pos[y]; });
      };
      // leadership candidates of every row: HashSet of the candidates in Partition.followerBrokers()
      pr.clear();
      pb.clear();
      leadOff.assign(1, 0);
      {
        PhaseScope pc(PH_CAND_BUILD);
        for (size_t k = i; k < end; ++k) {
          hostsInOrder(list[k], true, ins);
          javaHashSetOrder(ins, hs);
          hs32.assign(hs.begin(), hs.end());
          e.eligible(hs32, DA_LEADERSHIP, own);
          for (int x : own) {
            pr.push_back(list[k]);
            pb.push_back(x);
          }
          leadOff.push_back((int32_t)pr.size());
        }
      }
      const int64_t keyL = e.pairScan(*this, pr, pb, DA_LEADERSHIP, false);
      size_t kL = end;  // the row owning pair keyL: the last row whose pairs start at or before it
      if (keyL >= 0) kL = i + (size_t)(std::upper_bound(leadOff.begin(), leadOff.end(), (int32_t)keyL) - leadOff.begin()) - 1;
      // replica-move candidates: ascending ids (the HashSet order when the row's set has no bucket collisions)
      ids.assign(inorder.begin(), inorder.end());
      std::sort(ids.begin(), ids.end());
      e.eligible(ids, DA_MOVE, idElig);
      auto idOrdered = [&](int r) {
        hostsInOrder(r, false, ins);
        const size_t size = inorder.size() - ins.size();
        int32_t maxId = -1;
        for (size_t q = ids.size(); q-- > 0;)
          if (std::find(ins.begin(), ins.end(), ids[q]) == ins.end()) {
            maxId = ids[q];
            break;
          }
        return maxId < (int32_t)javaHashSetCapacity(size);
      };
      auto ownMoves = [&](int r, std::vector<int32_t>& out) {
        hostsInOrder(r, false, ins);
        std::vector<int> f;
        for (int x : inorder)
          if (std::find(ins.begin(), ins.end(), x) == ins.end()) f.push_back(x);
        javaHashSetOrder(f, hs);
        hs32.assign(hs.begin(), hs.end());
        e.eligible(hs32, DA_MOVE, out);
      };
      size_t winRow = (size_t)-1;
      int winDst = -1, winAction = DA_MOVE;
      int64_t visited = 0;
      for (size_t j = i; j < kL;) {
        if (idOrdered(list[j])) {
          size_t j2 = j + 1;
          while (j2 < kL && idOrdered(list[j2])) ++j2;
          const int64_t key = e.crossScan(*this, DA_MOVE, list, j, idElig, FILTER_NONE, false, j2);
          const size_t N = idElig.size(), last = key >= 0 ? j + (size_t)(key / (int64_t)N) : j2;
          for (size_t k = j; k < last; ++k)
            visited += e.visitCount(DA_MOVE, list[k], idElig.data(), N, true);
          if (key >= 0) {
            winRow = last;
            winDst = idElig[key % (int64_t)N];
            visited += e.visitCount(DA_MOVE, list[last], idElig.data(), (size_t)(key % (int64_t)N) + 1, true);
            break;
          }
          j = j2;
        } else {
          ownMoves(list[j], own);
          const int64_t key = e.crossScan(*this, DA_MOVE, list, j, own, FILTER_NONE, false, j + 1);
          visited += e.visitCount(DA_MOVE, list[j], own.data(), key >= 0 ? (size_t)key + 1 : own.size());
          if (key >= 0) {
            winRow = j;
            winDst = own[key];
            break;
          }
          ++j;
        }
      }
      if (winRow == (size_t)-1 && kL < end) {
        winRow = kL;
        winDst = pb[keyL];
        winAction = DA_LEADERSHIP;
      }
      // leadership candidates visited: every row before the winner's, the winner's up to a leadership winner
      const size_t rowsDone = winRow == (size_t)-1 ? end : winRow;
      for (size_t k = i; k < rowsDone; ++k)
        visited += e.visitCount(DA_LEADERSHIP, list[k], pb.data() + leadOff[k - i], leadOff[k - i + 1] - leadOff[k - i]);
      if (winRow != (size_t)-1) {
        const int32_t a = leadOff[winRow - i], z = winAction == DA_LEADERSHIP ? (int32_t)keyL + 1 : leadOff[winRow - i + 1];
        visited += e.visitCount(DA_LEADERSHIP, list[winRow], pb.data() + a, z - a);
      }
      e.candidates += visited;
      if (winRow == (size_t)-1) {
        if (runOffline) wasUnable = true;
        i = end;
        continue;
      }
      if (runOffline && winRow > i) wasUnable = true;
      const int r = list[winRow];
      const bool wasOffline = m.curOffline(r);
      if (winAction == DA_LEADERSHIP) m.relocateLeadership(m.rPart[r], b, winDst);
      else m.relocateReplica(m.rPart[r], b, winDst);
      if (wasOffline) nOff--;
      if (--n <= (nOff == 0 ? upperSrc : 0)) return false;
      cand.removeIf([winDst](int x) { return x == winDst; });
      if (m.tlead(t, winDst) < upper[t] || fix) cand.add(winDst);
      i = winRow + 1;
    }
    return m.tlead(t, b) != 0;
  }

  // rebalanceByMovingLeadersIn (:680-778). The queue keys on the precomputed offline / topic-leader maps (updated
  // for the source and b only) and the live leader counts, with JDK heap semantics for stale keys. A source's rows
  // go to the device in runs of one action (b hosting the partition: leadership movement, else replica movement).
  bool moveIn(Engine& e, int dest, int t) {
    Model& m = e.m;
    std::vector<int32_t> offBy(m.B, 0), tlBy(m.B, 0), offl;
    for (int x = 0; x < m.B; ++x) {
      tlBy[x] = m.tlead(t, x);
      if (m.bOfflineSet[x].size() == 0) continue;
      m.bOfflineSet[x].order(offl);
      for (int r : offl) offBy[x] += (m.rLeader[r] && m.pTopic[m.rPart[r]] == t) ? 1 : 0;
    }
    auto cmp = [&](int b1, int b2) {
      int c = jcmpInt(offBy[b2], offBy[b1]);
      if (c == 0) c = jcmpInt(tlBy[b2], tlBy[b1]);
      if (c == 0) c = jcmpInt(m.bNlead[b2], m.bNlead[b1]);
      return c == 0 ? jcmpInt(m.bId[b2], m.bId[b1]) : c;
    };
    JavaPQ<decltype(cmp)> pq(cmp);
    {
      PhaseScope pi(PH_PQ_INIT);
      for (int s = 0; s < m.B; ++s) {  // ClusterModel.brokers(): ascending id
        if (fix) {
          if (s != dest) pq.add(s);
        } else if (m.tlead(t, s) > lower[t] || hasOffline(m, s) || excluded(s)) {
          pq.add(s);
        }
      }
    }
    int n = m.tlead(t, dest);
    const bool destExcl = excluded(dest);
    std::vector<int32_t> single{dest}, candMove, candLead, toMove, rows, rowIdx, pbs;
    e.eligible(single, DA_MOVE, candMove);
    e.eligible(single, DA_LEADERSHIP, candLead);
    auto actionOf = [&](int r) {  // -1: skipped (an excluded b cannot take a replica)
      const bool has = m.replicaOn(m.rPart[r], dest) >= 0;
      if (destExcl && !has) return -1;
      return has ? (int)DA_LEADERSHIP : (int)DA_MOVE;
    };
    while (!pq.empty()) {
      const int src = pq.poll();
      replicasToMoveOut(m, src, t, toMove);
      int nOff = 0;
      for (int r : toMove) nOff += m.rInOff[r] ? 1 : 0;
      size_t i = 0;
      while (i < toMove.size()) {
        const int act = actionOf(toMove[i]);
        if (act < 0) {
          ++i;
          continue;
        }
        rows.clear();
        rowIdx.clear();
        size_t j = i;
        for (; j < toMove.size(); ++j) {
          const int a = actionOf(toMove[j]);
          if (a < 0) continue;
          if (a != act) break;
          rows.push_back(toMove[j]);
          rowIdx.push_back((int32_t)j);
        }
        int64_t key = -1;
        if (act == DA_MOVE) {
          if (!candMove.empty()) key = e.crossScan(*this, DA_MOVE, rows, 0, candMove);
        } else if (!candLead.empty()) {
          pbs.assign(rows.size(), dest);
          key = e.pairScan(*this, rows, pbs, DA_LEADERSHIP, true);
        }
        if (key < 0) {
          i = j;
          continue;
        }
        const size_t k = (size_t)rowIdx[key];
        const int r = toMove[k];
        const bool wasOffline = m.curOffline(r);
        if (act == DA_MOVE) m.relocateReplica(m.rPart[r], src, dest);
        else m.relocateLeadership(m.rPart[r], src, dest);
        if (wasOffline) {
          nOff--;
          offBy[src] = std::max(0, offBy[src] - 1);
        }
        tlBy[src] = std::max(0, tlBy[src] - 1);
        tlBy[dest] += 1;
        if (++n >= lower[t]) return false;
        if (!pq.empty() && nOff == 0 && m.tlead(t, src) < m.tlead(t, pq.peek())) {
          pq.add(src);
          break;
        }
        i = k + 1;
      }
    }
    return true;
  }
};

// ======================================================================================= LeaderReplicaDistributionGoal
// The leadership loops use one pair scan per decision, the move applied on the host; CCMI_PAIR_CHAINS=1 runs each
// call as one K7 chain instead (device-side applies: slower at C2, profiles/r06/README.md)
inline bool pairChainsOn(const Engine& e) { return e.pairChains && e.chainsOn(); }
template <class Q>
bool LeaderReplicaDistribution_moveInQueue(Engine& e, GoalImpl& self, int b, Q& pq, const Model::Spec& spec,
                                           const std::vector<int32_t>& cands, int nl, int lower);

class LeaderReplicaDistribution : public GoalImpl {
 public:
  LeaderReplicaDistribution() {
    kind = CCMI_GOAL_LEADER_REPLICA_DISTRIBUTION;
    name = "LeaderReplicaDistributionGoal";
  }
  bool fix = false, anyAbove = false, anyUnder = false;
  int upper = 0, lower = 0;
  bool excluded(int b) const { return !allowed[b]; }

  // ReplicaDistributionAbstractGoal.initGoalState (:124-152), numInterestedReplicas = number of leaders
  void init(Engine& e) override {
    Model& m = e.m;
    const int n = allowedForReplicaMove(e, allowed);
    if (n == 0)
      throw OptimizationFailure("[" + name + "] All alive brokers are excluded from replica moves.", underBrokers(m.maxRf));
    const double avg = m.numLeaderReplicas() / (double)n;
    fix = false;
    const double adj = (e.bc.leaderReplicaBalance - 1) * kBalanceMargin;
    upper = (int)std::ceil(avg * (1 + adj));
    lower = (int)std::floor(avg * jmax(0, (1 - adj)));
    dg = DevGoal{};
    dg.kind = DG_LEADER_REPLICA_DISTRIBUTION;
    dg.upper = upper;
    dg.lower = lower;
    dg.allowedSlot = e.newSlot;
  }
  // updateGoalState (ReplicaDistributionAbstractGoal.java:183-223)
  void update(Engine& e) override {
    if (anyAbove) succeeded = false;
    if (anyUnder) succeeded = false;
    anyAbove = anyUnder = false;
    Model& m = e.m;
    for (int r = 0; r < m.R; ++r)
      if (m.selfHealing[r] && m.curOffline(r)) {
        if (fix)
          throw OptimizationFailure("[" + name + "] Cannot remove replica from broker " + std::to_string(m.bId[m.rBroker[r]]),
                                    underBrokers(1));
        fix = true;
        dg.fixOffline = 1;
        return;
      }
    finished = true;
  }
  int compareStats(const ccmi_cluster_stats& after, const ccmi_cluster_stats& before) const override {
    return cmpStd(after.leader_std, before.leader_std);
  }

  // rebalanceForBroker (:137-166)
  void rebalance(Engine& e, int b) override {
    PhaseScope ps(PH_OTHER_GOALS);
    Model& m = e.m;
    const int nl = m.bNlead[b];
    const bool excl = excluded(b);
    const bool lessLeaders = m.alive(b) && nl > (excl ? 0 : upper);
    const bool moreLeaders = !excl && m.alive(b) && nl < lower;
    const bool lessReplicas = fix && hasOffline(m, b);
    if (((lessLeaders && moveLeadershipOut(e, b)) || lessReplicas) && moveReplicasOut(e, b)) {
      if (!lessReplicas) anyAbove = true;
    } else if (moreLeaders && moveLeadershipIn(e, b) && moveLeaderReplicasIn(e, b)) {
      anyUnder = true;
    }
  }

  // rebalanceByMovingLeadershipOut (:168-203): every leader's candidate set is fixed, so all remaining leaders
  // are scanned as one pair list and the scan resumes after each winner
  bool moveLeadershipOut(Engine& e, int b) {
    Model& m = e.m;
    PhaseScope lp(PH_LEAD_OUT);
    if (m.numDead > 0) return true;
    const int upperSrc = excluded(b) ? 0 : upper;
    int nl = m.bNlead[b];
    ReplicaSet copy;  // new HashSet<>(broker.leaderReplicas())
    copy.assignCopy(m.bLeaderSet[b]);
    std::vector<int32_t> leaders;
    copy.order(leaders);
    std::vector<int32_t> pr, pb, owner;
    std::vector<int> ins, hs, hs2, elig;
    {
      PhaseScope pc(PH_CAND_BUILD);
      for (size_t q = 0; q < leaders.size(); ++q) {
        const int r = leaders[q], p = m.rPart[r];
        if (e.opt.anyExclTopic && e.opt.exclTopic[m.pTopic[p]]) continue;  // leaders of excluded topics stay
        ins.clear();
        for (int s = m.pOff[p]; s < m.pOff[p + 1]; ++s) ins.push_back(m.rBroker[m.pSlots[s]]);
        javaHashSetOrder(ins, hs);  // Partition.partitionBrokers()
        ins.clear();
        for (int x : hs)
          if (x != b && !m.curOffline(m.replicaOn(p, x))) ins.push_back(x);
        javaHashSetOrder(ins, hs2);  // Collectors.toSet()
        std::vector<int32_t> c32(hs2.begin(), hs2.end()), el;
        e.eligible(c32, DA_LEADERSHIP, el);
        for (int x : el) {
          pr.push_back(r);
          pb.push_back(x);
          owner.push_back((int)q);
        }
      }
    }
    if (pairChainsOn(e)) {  // one device chain: after an accept the scan resumes at the next leader's pairs
      std::vector<int32_t> next(pr.size()), log;
      int ng = (int)pr.size();
      for (int q = (int)pr.size() - 1; q >= 0; --q) {
        if (q + 1 < (int)pr.size() && owner[q + 1] != owner[q]) ng = q + 1;
        next[q] = ng;
      }
      const int want = nl - upperSrc;
      const int64_t acc = e.chainPairs(*this, DA_LEADERSHIP, pr, pb, next, want, log);
      Model::Replay rp(m);
      for (int q : log) m.relocateLeadership(m.rPart[pr[q]], b, pb[q]);
      return acc < want;
    }
    size_t start = 0;
    std::vector<int32_t> spr, spb;
    while (start < pr.size()) {
      spr.assign(pr.begin() + start, pr.end());
      spb.assign(pb.begin() + start, pb.end());
      const int64_t key = e.pairScan(*this, spr, spb);
      if (key < 0) break;
      const size_t at = start + (size_t)key;
      const int r = pr[at];
      m.relocateLeadership(m.rPart[r], b, pb[at]);
      if (--nl <= upperSrc) return false;
      start = at + 1;
      while (start < pr.size() && owner[start] == owner[at]) ++start;  // next leader
    }
    return true;
  }

  // rebalanceByMovingLeadershipIn (:205-240)
  bool moveLeadershipIn(Engine& e, int b) {
    Model& m = e.m;
    PhaseScope lp(PH_LEAD_IN);
    if (m.numDead > 0 || (e.opt.anyExclLead && e.opt.exclLead[b])) return true;
    int nl = m.bNlead[b];
    std::vector<int32_t> reps, pr, pb;
    m.bReplicaSet[b].order(reps);  // Broker.replicas(): HashSet order
    std::vector<int32_t> single{b}, cands;
    e.eligible(single, DA_LEADERSHIP, cands);
    if (cands.empty()) return true;
    for (int r : reps) {
      if (m.rLeader[r] || m.curOffline(r) || (e.opt.anyExclTopic && e.opt.exclTopic[m.pTopic[m.rPart[r]]])) continue;
      pr.push_back(m.pLeader[m.rPart[r]]);
      pb.push_back(b);
    }
    if (pairChainsOn(e)) {  // one device chain over the fixed pair list
      if (pr.empty()) return true;
      std::vector<int32_t> next(pr.size()), log;
      for (size_t q = 0; q < pr.size(); ++q) next[q] = (int32_t)q + 1;
      const int want = lower - nl;
      const int64_t acc = e.chainPairs(*this, DA_LEADERSHIP, pr, pb, next, want, log);
      Model::Replay rp(m);
      for (int q : log) m.relocateLeadership(m.rPart[pr[q]], m.rBroker[pr[q]], b);
      return acc < want;
    }
    size_t start = 0;
    std::vector<int32_t> spr, spb;
    while (start < pr.size()) {
      spr.assign(pr.begin() + start, pr.end());
      spb.assign(pb.begin() + start, pb.end());
      const int64_t key = e.pairScan(*this, spr, spb);
      if (key < 0) break;
      const size_t at = start + (size_t)key;
      m.relocateLeadership(m.rPart[pr[at]], m.rBroker[pr[at]], b);
      if (++nl >= lower) return false;
      start = at + 1;
    }
    return true;
  }

  // rebalanceByMovingReplicasOut (:242-300)
  bool moveReplicasOut(Engine& e, int b) {
    Model& m = e.m;
    PhaseScope lp(PH_REP_OUT);
    const bool f = fix;
    auto cmp = [&m, f](int x, int y) {
      const int c = f ? jcmpInt(m.nrep(x), m.nrep(y)) : jcmpInt(m.bNlead[x], m.bNlead[y]);
      return c ? c : jcmpInt(m.bId[x], m.bId[y]);
    };
    RbTreeSet<decltype(cmp)> cand(cmp);
    // Non-fix form: the set's in-order sequence at entry is the members' (leader count, id) order, which is all the
    // first scan needs; the tree itself (its put sequence decides where stale keys send later searches) is needed only
    // from the first accepted move on. Its puts start now and run while the first scan is in flight; a call whose
    // first scan accepts nothing never completes them.
    std::vector<int32_t> entryOrder;
    bool treeReady = true;
    {
      PhaseScope pi(PH_PQ_INIT);
      if (fix) {
        for (int x : aliveById(m)) cand.add(x);
      } else {
        std::vector<int> ins, order;
        for (int x = 0; x < m.B; ++x)
          if (m.alive(x) && m.bNlead[x] < upper) ins.push_back(x);
        javaHashSetOrder(ins, order);  // Collectors.toSet()
        // the same TreeSet.add sequence, placed by rank (the comparator is a total order on these brokers)
        std::vector<int32_t> byKey, rank(m.B, 0);
        bool idsAsc = true;
        for (int x = 1; x < m.B && idsAsc; ++x) idsAsc = m.bId[x - 1] < m.bId[x];
        if (idsAsc && std::is_sorted(ins.begin(), ins.end()) && !ins.empty()) {
          // counting sort by leader count (0 <= count < upper); `ins` is in ascending index = id order
          std::vector<int32_t> start(upper + 1, 0);
          for (int x : ins) start[m.bNlead[x] + 1]++;
          for (int c = 0; c < upper; ++c) start[c + 1] += start[c];
          byKey.resize(ins.size());
          for (int x : ins) byKey[start[m.bNlead[x]]++] = x;
        } else {
          byKey.assign(ins.begin(), ins.end());
          std::sort(byKey.begin(), byKey.end(), [&](int x, int y) { return cmp(x, y) < 0; });
        }
        for (size_t i = 0; i < byKey.size(); ++i) rank[byKey[i]] = (int32_t)i;
        entryOrder = std::move(byKey);
        cand.buildStart(std::move(order), std::move(rank));
        treeReady = false;
      }
    }
    auto finishTree = [&]() {
      if (treeReady) return;
      PhaseScope pi(PH_PQ_INIT);
      cand.buildStep((size_t)-1);
      cand.trackSequence();
      treeReady = true;
    };
    if (treeReady) cand.trackSequence();
    const Device::IdleScope idleScope{e.dev};
    const size_t treePuts = idleTreePutsPerPoll();
    if (!treeReady && treePuts > 0) e.dev->idleWork = [&]() { return !cand.buildStep(treePuts); };
    const int upperLimit = fix ? 0 : upper;
    const int id = sortId(kind, false, !fix);
    Model::Spec s;
    s.selLeaders = !fix;
    s.selOffline = fix;
    s.selImmigrants = (!fix && m.numSelfHealing > 0) || e.opt.onlyImmigrants;
    s.selExclTopics = e.opt.anyExclTopic;
    m.track(b, id, s);
    const std::vector<int32_t> list = m.sorted(b, id);
    int n = (int)list.size();
    std::vector<int32_t> inorder, cands;
    size_t i = 0;
    while (i < list.size()) {
      // the tree's maintained sequence (or, before the tree is needed, the entry order) itself: no copy
      const std::vector<int32_t>* seq = treeReady ? cand.sequence() : &entryOrder;
      if (!seq) {
        cand.inorder(inorder);
        seq = &inorder;
      }
      const std::vector<int32_t>& cl = e.eligibleView(*seq, DA_MOVE, cands);
      const int64_t key = e.crossScan(*this, DA_MOVE, list, i, cl);
      e.dev->idleWork = nullptr;  // the remaining puts, if the tree is needed, are finished below
      if (key < 0) break;
      const size_t N = cl.size();
      const size_t k = i + (size_t)(key / (int64_t)N);
      const int dst = cl[key % (int64_t)N];  // (read before the tree changes below)
      m.relocateReplica(m.rPart[list[k]], b, dst);
      if (--n <= upperLimit) {
        m.untrack(b, id);
        return false;
      }
      finishTree();
      cand.remove(dst);
      if (m.bNlead[dst] < upper || fix) cand.add(dst);
      i = k + 1;
    }
    m.untrack(b, id);
    return true;
  }

  // rebalanceByMovingLeaderReplicasIn (:302-352). Queued brokers never change key while queued (moves go from
  // the polled source to b, and b is not queued), so the queue polls in comparator order and speculatively
  // polled sources can be put back: the next sources' sorted leaders are scanned together with the current
  // one's (growing the batch while nothing is accepted), exactly as RDG moveIn does.
  Model::SnapTable snapTab;
  bool moveLeaderReplicasIn(Engine& e, int b) {
    Model& m = e.m;
    PhaseScope lp(PH_REP_IN);
    if (e.opt.anyExclLead && e.opt.exclLead[b]) return true;
    auto cmp = [&m](int b1, int b2) {
      const int r = jcmpInt(m.bNlead[b2], m.bNlead[b1]);
      return r == 0 ? jcmpInt(m.bId[b1], m.bId[b2]) : r;
    };
    // No queued broker changes key while queued, so the PriorityQueue polls in comparator order: an OrderedQueue over
    // the members sorted by (leader count descending, id) — a counting sort when indices are in id order
    OrderedQueue<decltype(cmp)> pq(cmp);
    {
      PhaseScope pi(PH_PQ_INIT);
      std::vector<int>& run = pq.sorted();
      bool idsAsc = true;
      for (int x = 1; x < m.B && idsAsc; ++x) idsAsc = m.bId[x - 1] < m.bId[x];
      int maxLead = 0;
      for (int x = 0; x < m.B; ++x) maxLead = std::max(maxLead, m.bNlead[x]);
      if (idsAsc && maxLead < (1 << 20)) {
        std::vector<int32_t> start(maxLead + 2, 0);
        size_t n = 0;
        for (int x = 0; x < m.B; ++x)
          if (m.alive(x) && m.bNlead[x] > lower) {
            start[maxLead - m.bNlead[x] + 1]++;
            ++n;
          }
        for (int c = 0; c <= maxLead; ++c) start[c + 1] += start[c];
        run.resize(n);
        for (int x = 0; x < m.B; ++x)
          if (m.alive(x) && m.bNlead[x] > lower) run[start[maxLead - m.bNlead[x]]++] = x;
      } else {
        for (int x = 0; x < m.B; ++x)
          if (m.alive(x) && m.bNlead[x] > lower) run.push_back(x);
        std::sort(run.begin(), run.end(), [&](int x, int y) { return cmp(x, y) < 0; });
      }
    }
    const int id = sortId(kind, false, true);
    Model::Spec s;
    s.selLeaders = true;
    s.selImmigrants = m.numDead > 0 || m.numBadDisk > 0 || e.opt.onlyImmigrants;
    s.selExclTopics = e.opt.anyExclTopic;
    // The sources' SortedReplicas are tracked only for this call (the reference tracks them on entry and untracks
    // on exit) and initialised lazily on first poll; a source only loses replicas afterwards (moves go to b, whose
    // view is never read), so its live view equals a fresh snapshot of its current replicas: snapshots (cached per
    // broker version) replace the tracked views and their per-poll clones.
    (void)id;
    int nl = m.bNlead[b];
    std::vector<int32_t> single{b}, cands;
    e.eligible(single, DA_MOVE, cands);
    if (cands.empty()) return true;  // every source replica visits an empty candidate list: nothing moves
    if (e.queueReady(*this, DA_MOVE, s)) return LeaderReplicaDistribution_moveInQueue(e, *this, b, pq, s, cands, nl, lower);
    // rows: the sources' sorted leaders (snapshots held by snapTab until the next model change; device-resident
    // segments of the snapshot pool)
    auto segLen = [](const SnapSeg& x) { return x.v->size() > x.skip ? x.v->size() - x.skip : 0; };
    std::vector<SnapSeg> segs;
    size_t target = 2048;
    bool haveCur = false;
    SnapSeg cur{nullptr, 0, 0};
    while (haveCur || !pq.empty()) {
      segs.clear();
      size_t rows = 0;
      if (haveCur) {  // the source being iterated continues first, after its winner
        cur.v = m.snapshotInShared(snapTab, cur.cb, s);
        segs.push_back(cur);
        rows += segLen(cur);
        haveCur = false;
      }
      while (!pq.empty() && (segs.empty() || rows < target) && segs.size() < (size_t)kMaxSegs) {
        const int src = pq.poll();
        segs.push_back({m.snapshotInShared(snapTab, src, s), src, 0});
        rows += segLen(segs.back());
      }
      size_t ahead = 0;  // snapshots of the next sources, computed while the scan is in flight (Device::idleWork)
      const Device::IdleScope idleScope{e.dev};
      e.dev->idleWork = [&]() {
        const int src = pq.upcoming(ahead);
        if (src < 0 || ahead >= 8) return false;
        ++ahead;
        (void)m.snapshotInShared(snapTab, src, s);
        return true;
      };
      const int64_t key = cands.empty() ? -1 : e.crossScanSegs(*this, DA_MOVE, segs, cands);
      e.dev->idleWork = nullptr;
      if (key < 0) {
        target = std::min<size_t>(target * 8, (size_t)1 << 18);
        continue;  // every polled source exhausted; none is re-enqueued
      }
      target = 2048;
      size_t q = (size_t)key, mi = 0;
      while (q >= segLen(segs[mi])) {
        q -= segLen(segs[mi]);
        ++mi;
      }
      const SnapSeg hit = segs[mi];
      const size_t idx = hit.skip + q;
      const size_t hitSize = hit.v->size();
      m.relocateReplica(m.rPart[(*hit.v)[idx]], hit.cb, b);
      if (++nl >= lower) return false;
      for (size_t t = segs.size(); t-- > mi + 1;) pq.unpoll(segs[t].cb);  // un-poll speculative sources
      if (!pq.empty() && m.bNlead[hit.cb] < m.bNlead[pq.peek()]) {
        pq.add(hit.cb);
      } else if (idx + 1 < hitSize) {
        // the live view lost exactly the moved replica: the entries after it keep their order, so the iteration
        // continues at the same index of the source's fresh snapshot
        cur = {nullptr, hit.cb, idx};
        haveCur = true;
      }
    }
    return true;
  }
};

// rebalanceByMovingLeaderReplicasIn over the whole source queue in one command per accepted move (Engine::queueScan,
// SOP_QUEUE; ResourceDistribution::moveInQueue is the same loop for the resource goals): the rows of every queued
// source — its sorted leaders, the snapshot directory's view for `spec` — in poll order, so the scan's first fit is the
// reference's next accept however deep in the queue it lies; sources polled before the winner's are consumed, the ones
// after it stay queued. After an accept the source is re-added (fewer leaders than the queue's head), or iterated on at
// the same index of its view without the moved replica, or dropped when that was its last row (:302-352).
template <class Q>
bool LeaderReplicaDistribution_moveInQueue(Engine& e, GoalImpl& self, int b, Q& pq, const Model::Spec& spec,
                                           const std::vector<int32_t>& cands, int nl, int lower) {
  Model& m = e.m;
  std::vector<int32_t> merged;
  int curCb = -1, curSkip = 0;
  const int N = (int)cands.size();
  while (curCb >= 0 || !pq.empty()) {
    const bool run = pq.heapEmpty();
    if (!run) {
      merged.clear();
      while (!pq.empty()) merged.push_back(pq.poll());
    }
    const int32_t* tail = run ? pq.runData() : merged.data();
    const int nTail = (int)(run ? pq.runLeft() : merged.size());
    const int head = curCb, hasHead = head >= 0 ? 1 : 0;
    const int64_t key = e.queueScan(self, DA_MOVE, spec, head, hasHead ? curSkip : 0, tail, nTail, cands);
    if (key < 0) return true;  // every queued source exhausted; none is re-enqueued
    const int span = e.dev->queueSpan();
    const int64_t row = key / N;
    const int i = (int)(row / span), idx = (int)(row % span);
    const int cb = i < hasHead ? head : tail[i - hasHead];
    const int r = e.dev->qdirRows(cb)[idx];
    const int hitSize = e.dev->qdirLen(cb);
    const int polled = i < hasHead ? 0 : i - hasHead + 1;
    if (run) pq.skipRun((size_t)polled);
    else
      for (int t = nTail; t-- > polled;) pq.unpoll(merged[t]);
    m.relocateReplica(m.rPart[r], cb, b);
    if (++nl >= lower) return false;
    if (!pq.empty() && m.bNlead[cb] < m.bNlead[pq.peek()]) {
      pq.add(cb);
      curCb = -1;
    } else if (idx + 1 < hitSize) {
      curCb = cb;  // the view without the moved replica, from the same index
      curSkip = idx;
    } else {
      curCb = -1;
    }
  }
  return true;
}

// ======================================================================================= LeaderBytesInDistributionGoal
class LeaderBytesIn : public GoalImpl {
 public:
  LeaderBytesIn() {
    kind = CCMI_GOAL_LEADER_BYTES_IN_DISTRIBUTION;
    name = "LeaderBytesInDistributionGoal";
  }
  double mean = 0.0;
  int numAllowed = 0;
  bool overLimit = false;
  double balance = 0, lowUtil = 0;

  // initMeanLeaderBytesIn (:250-257): cached on first use (recomputed while it is 0.0)
  void initMean(Engine& e) {
    if (mean == 0.0) {
      JDoubleSum s;
      for (int b = 0; b < e.m.B; ++b)
        if (e.m.alive(b)) s.add(e.m.leadNwIn(b));
      mean = s.result() / numAllowed;
      dg.lbiMean = mean;
    }
  }
  // balanceThreshold (:264-271)
  double threshold(Engine& e, int b) {
    initMean(e);
    return jmax(mean * balance, lowUtil * e.m.cap(b, R_NW_IN));
  }
  void init(Engine& e) override {  // initGoalState (:162-185)
    Model& m = e.m;
    numAllowed = allowedForReplicaMove(e, allowed);
    if (numAllowed == 0)
      throw OptimizationFailure("[" + name + "] All alive brokers are excluded from replica moves.", underBrokers(m.maxRf));
    mean = 0.0;
    overLimit = false;
    balance = e.bc.resBalance[R_NW_IN];
    lowUtil = e.bc.lowUtil[R_NW_IN];
    Model::Spec s;
    s.selLeaders = true;
    s.selExclTopics = e.opt.anyExclTopic;
    s.scoreRes = R_NW_IN;
    s.scoreReverse = true;
    for (int b = 0; b < m.B; ++b) m.track(b, sortId(kind, true, true), s);
    dg = DevGoal{};
    dg.kind = DG_LEADER_BYTES_IN;
    dg.lbiBalance = balance;
    dg.lbiLowUtil = lowUtil;
    dg.allowedSlot = e.newSlot;
  }
  // brokersToBalance (:142-152)
  std::vector<int> brokersToBalance(Engine& e) override {
    std::vector<int> v;
    for (int b = 0; b < e.m.B; ++b)
      if (e.m.leadNwIn(b) > threshold(e, b)) v.push_back(b);
    return v;
  }
  // rebalanceForBroker (:203-233): all remaining leaders' follower lists in one pair scan; lists are rebuilt
  // after each move because they are sorted by live leader bytes-in
  void rebalance(Engine& e, int b) override {
    PhaseScope ps(PH_OTHER_GOALS);
    Model& m = e.m;
    const double thr = threshold(e, b);
    if (m.leadNwIn(b) < thr) return;
    bool over = true;
    const std::vector<int32_t> leaders = m.sorted(b, sortId(kind, true, true));
    std::vector<int32_t> pr, pb, owner, fol;
    // each row's sorted eligible followers, kept between scans: a move changes the bytes-in of b (the leader of every
    // row) and dst, so only rows with dst among their followers are re-sorted
    std::vector<std::vector<int32_t>> rowCands(leaders.size());
    std::vector<uint8_t> rowValid(leaders.size(), 0);
    size_t i = 0;
    while (over && i < leaders.size()) {
      pr.clear();
      pb.clear();
      owner.clear();
      for (size_t q = i; q < leaders.size(); ++q) {
        const int r = leaders[q];
        std::vector<int32_t>& elig = rowCands[q];
        if (!rowValid[q]) {
          m.onlineFollowerBrokers(m.rPart[r], fol);
          stableSortBy(fol, [&](int x, int y) { return jcmpDouble(m.leadNwIn(x), m.leadNwIn(y)); });
          e.eligible(fol, DA_LEADERSHIP, elig);
          rowValid[q] = 1;
        }
        for (int x : elig) {
          pr.push_back(r);
          pb.push_back(x);
          owner.push_back((int)q);
        }
      }
      const int64_t key = e.pairScan(*this, pr, pb);
      if (key < 0) break;
      const size_t k = (size_t)owner[key];
      const int dst = pb[key];
      m.relocateLeadership(m.rPart[leaders[k]], b, dst);
      over = m.leadNwIn(b) > thr;
      i = k + 1;
      for (size_t q = i; q < leaders.size(); ++q)
        if (rowValid[q] && m.replicaOn(m.rPart[leaders[q]], dst) >= 0) rowValid[q] = 0;
    }
    if (over) overLimit = true;
  }
  void update(Engine&) override {  // updateGoalState (:194-201)
    if (overLimit) succeeded = false;
    overLimit = false;
    finished = true;
  }
  // LeaderBytesInDistributionGoalStatsComparator (:273-300)
  int compareStats(const ccmi_cluster_stats& after, const ccmi_cluster_stats& before) const override {
    const double meanPre = after.resource_avg[R_NW_IN];
    const double thr = meanPre * balance;
    if (after.resource_max[R_NW_IN] <= thr) return 1;
    const double d1 = std::sqrt(before.resource_std[R_NW_IN]), d2 = std::sqrt(after.resource_std[R_NW_IN]);
    // AnalyzerUtils.compare(d1, d2, Resource.NW_IN): Resource.epsilon = max(10, 0.0008 * (d1 + d2))
    const double eps = jmax(10.0, 0.0008 * (d1 + d2));
    if (d2 - d1 > eps) return -1;
    if (d1 - d2 > eps) return 1;
    return 0;
  }
};

}  // namespace

// ======================================================================================= PreferredLeaderElectionGoal
// PreferredLeaderElectionGoal.optimize (PreferredLeaderElectionGoal.java:117-190), the no-argument constructor
// (skipUrpDemotion = excludeFollowerDemotion = false). A one-pass leadership election with no candidate search: every
// partition's leadership goes to its first alive, online replica (with demoted brokers: only the partitions they led,
// after their replicas moved to the end of the replica lists; the same for demoted disks of other alive brokers,
// :114-124), so it runs on the host model and the device only sees the touched rows.

class PreferredLeaderElection : public GoalImpl {
 public:
  PreferredLeaderElection() {
    kind = CCMI_GOAL_PREFERRED_LEADER_ELECTION;
    name = "PreferredLeaderElectionGoal";
  }
  void init(Engine& e) override {
    if (e.opt.triggered)  // sanityCheckOptimizationOptions (:79-83)
      throw std::invalid_argument(name + " goal does not support use by goal violation detector.");
    allowedForReplicaMove(e, allowed);
    dg = DevGoal{};
    dg.kind = DG_ACCEPT_ALL;  // actionAcceptance: ACCEPT
    dg.allowedSlot = e.newSlot;
  }
  bool rebalanceAll(Engine& e) override {
    PhaseScope ps(PH_OTHER_GOALS);
    Model& m = e.m;
    bool hasDemoted = false;
    std::vector<uint8_t> toMove(m.P, 0);
    std::vector<int> alive, ord;
    for (int b = 0; b < m.B; ++b)
      if (m.alive(b)) alive.push_back(b);
    javaHashSetOrder(alive, ord);  // clusterModel.aliveBrokers(): a HashSet<Broker>
    std::vector<int32_t> reps;
    for (int b : ord) {
      if (m.bState[b] != BState::DEMOTED) {
        // demoted disks of a broker that is not demoted, in logdir order (Broker.disks(): the TreeMap's values)
        for (int k = m.bDiskOff[b]; m.anyDemotedDisk && k < m.bDiskOff[b + 1]; ++k) {
          const int d = m.bDisks[k];
          if (!m.dDemoted[d]) continue;
          hasDemoted = true;
          // Disk.replicas(): the HashSet, which keeps replicas inter-broker moves took elsewhere
          m.dReplicaSet[d].order(reps);
          for (int r : reps) m.moveReplicaToEnd(r);
          for (int r : reps)  // Disk.leaderReplicas(): the same set filtered by isLeader
            if (m.rLeader[r]) toMove[m.rPart[r]] = 1;
        }
        continue;
      }
      hasDemoted = true;
      m.bReplicaSet[b].order(reps);  // Broker.replicas(): HashSet order
      for (int r : reps) m.moveReplicaToEnd(r);
      m.bLeaderSet[b].order(reps);
      for (int r : reps) toMove[m.rPart[r]] = 1;
    }
    // clusterModel.getPartitionsByTopic(): topics by name, each topic's partitions in the model's
    // HashMap<TopicPartition, Partition> iteration order
    PartitionOrder po{&m};
    JHashSet<PartitionOrder> all(&po);
    for (int p = 0; p < m.P; ++p) all.add(p, jMix(jMix(1, m.pNumber[p]), m.topicHash[m.pTopic[p]]));
    std::vector<int32_t> order;
    all.order(order);
    std::vector<std::vector<int32_t>> byTopic(m.T);
    for (int p : order) byTopic[m.pTopic[p]].push_back(p);
    std::vector<int> topics(m.T);
    for (int t = 0; t < m.T; ++t) topics[t] = t;
    std::sort(topics.begin(), topics.end(), [&m](int a, int b) { return m.topicNames[a] < m.topicNames[b]; });
    bool relocated = false;
    for (int t : topics)
      for (int p : byTopic[t]) {
        if (hasDemoted && !toMove[p]) continue;
        for (int i = m.pOff[p]; i < m.pOff[p + 1]; ++i) {
          if (!hasDemoted && i > m.pOff[p]) break;  // only the first (preferred) replica
          const int r = m.pSlots[i], cand = m.rBroker[r];
          if (!m.alive(cand)) continue;
          if (m.curOffline(r)) continue;
          if (!m.rLeader[r]) {
            if (e.opt.anyExclLead && e.opt.exclLead[cand]) continue;
            m.relocateLeadership(p, m.rBroker[m.pLeader[p]], cand);
            relocated = true;
          }
          break;
        }
      }
    succeeded = relocated;  // Goal.optimize returns whether a leadership moved
    return true;
  }
  void rebalance(Engine&, int) override {}
  void update(Engine&) override { finished = true; }
  int compareStats(const ccmi_cluster_stats&, const ccmi_cluster_stats&) const override { return 0; }
};

// ======================================================================================= Kafka-assigner mode goals
// analyzer/kafkaassigner/KafkaAssignerEvenRackAwareGoal.java and KafkaAssignerDiskUsageDistributionGoal.java (in
// `goals`, not in default.goals). Both implement Goal directly: no candidate conjunction over optimized goals, so
// their decisions are made on the host (rack membership tests and replica-size searches over one broker pair);
// as optimized goals they act through the device predicates (EvenRackAware: the rack-awareness predicate, identical
// to RackAwareGoal's acceptance; DiskUsageDistribution: terminal, any later candidate ends the optimization).

// getPartitionsByTopic: topics by name, each topic's partitions in HashMap<TopicPartition, Partition> order
std::vector<std::vector<int32_t>> kaPartitionsByTopic(const Model& m) {
  PartitionOrder po{&m};
  JHashSet<PartitionOrder> all(&po);
  for (int p = 0; p < m.P; ++p) all.add(p, jMix(jMix(1, m.pNumber[p]), m.topicHash[m.pTopic[p]]));
  std::vector<int32_t> order;
  all.order(order);
  std::vector<std::vector<int32_t>> byTopic(m.T);
  for (int p : order) byTopic[m.pTopic[p]].push_back(p);
  std::vector<int> topics(m.T);
  for (int t = 0; t < m.T; ++t) topics[t] = t;
  std::sort(topics.begin(), topics.end(), [&m](int a, int b) { return m.topicNames[a] < m.topicNames[b]; });
  std::vector<std::vector<int32_t>> out;
  for (int t : topics)
    if (!byTopic[t].empty()) out.push_back(std::move(byTopic[t]));
  return out;
}

// KafkaAssignerUtils.sanityCheckOptimizationOptions (KafkaAssignerUtils.java:20-26)
void kaSanityCheck(const Engine& e) {
  if (e.opt.triggered) throw std::invalid_argument("Kafka Assigner goals do not support usage by goal violation detector.");
  if (e.opt.onlyImmigrants)
    throw std::invalid_argument("Kafka Assigner goals do not support usage of modifying topic replication factor.");
}

class KafkaAssignerEvenRackAware : public GoalImpl {
 public:
  KafkaAssignerEvenRackAware() {
    kind = CCMI_GOAL_KAFKA_ASSIGNER_EVEN_RACK_AWARE;
    name = "KafkaAssignerEvenRackAwareGoal";
    abstractGoal = false;
  }
  void init(Engine& e) override {
    kaSanityCheck(e);
    if (!e.priors.empty())  // optimizedGoals non-empty (KafkaAssignerEvenRackAwareGoal.java:125-128)
      throw std::invalid_argument("Goals " + std::to_string(e.priors.size()) + " cannot be optimized before " + name + ".");
    allowed.assign(e.m.B, 1);
    dg = DevGoal{};
    dg.kind = DG_RACK_AWARE;  // actionAcceptance (:385-408): the rack-awareness test of RackAwareGoal
    dg.allowedSlot = e.newSlot;
  }
  // Replica.toString (Replica.java:338-343); racks are named by their index
  static std::string replicaString(const Model& m, int r) {
    auto tf = [](bool v) { return std::string(v ? "true" : "false"); };
    const int p = m.rPart[r], b = m.rBroker[r];
    return "Replica[isLeader=" + tf(m.rLeader[r] != 0) + ",rack=" + std::to_string(m.bRack[b]) + ",broker=" +
           std::to_string(m.bId[b]) + ",TopicPartition=" + m.topicNames[m.pTopic[p]] + "-" + std::to_string(m.pNumber[p]) +
           ",origBroker=" + std::to_string(m.bId[m.rOrig[r]]) + ",isOriginalOffline=" + tf(m.origOffline(r)) +
           ",isCurrentOffline=" + tf(m.curOffline(r)) + "]";
  }
  // optimize (:119-165)
  bool rebalanceAll(Engine& e) override {
    PhaseScope ps(PH_OTHER_GOALS);
    Model& m = e.m;
    auto excl = [&](int t) { return e.opt.anyExclTopic && e.opt.exclTopic[t] != 0; };
    // ensureRackAwareSatisfiable (:318-343): distinct racks with an alive broker
    std::vector<uint8_t> rackAlive(m.B + 1, 0);
    int racks = 0;
    for (int b = 0; b < m.B; ++b)
      if (m.alive(b) && !rackAlive[m.bRack[b]]) {
        rackAlive[m.bRack[b]] = 1;
        ++racks;
      }
    std::vector<int32_t> rf(m.T, 0);
    for (int p = 0; p < m.P; ++p) rf[m.pTopic[p]] = std::max<int32_t>(rf[m.pTopic[p]], m.pOff[p + 1] - m.pOff[p]);
    if (e.opt.anyExclTopic) {
      std::vector<int32_t> seen, order;
      for (int t = 0; t < m.T; ++t) seen.push_back(t);
      TopicOrder to{&m};
      TopicSet ts(&to);
      for (int t : seen) ts.add(t, m.topicHash[t]);
      ts.order(order);  // _replicationFactorByTopic: a HashMap<String, Integer>
      int maxRf = 1;
      for (int t : order) {
        if (excl(t)) continue;
        maxRf = std::max(maxRf, (int)rf[t]);
        if (maxRf > racks)
          throw OptimizationFailure("[" + name + "] Insufficient number of racks to distribute included replicas (Current: " +
                                    std::to_string(racks) + ", Needed: " + std::to_string(maxRf) + ").");
      }
    } else if (m.maxRf > racks) {
      throw OptimizationFailure("[" + name + "] Insufficient number of racks to distribute each replica (Current: " +
                                std::to_string(racks) + ", Needed: " + std::to_string(m.maxRf) + ").");
    }
    const auto byTopic = kaPartitionsByTopic(m);
    // brokers by (replica count at the position, id); the count starts at the excluded topics' replicas there
    std::vector<std::vector<int32_t>> excludedAt(m.maxRf, std::vector<int32_t>(m.B, 0));
    for (const auto& parts : byTopic)
      for (int p : parts) {
        if (!excl(m.pTopic[p])) continue;
        excludedAt[0][m.rBroker[m.pLeader[p]]]++;
        int pos = 0;
        for (int s = m.pOff[p]; s < m.pOff[p + 1]; ++s)
          if (m.pSlots[s] != m.pLeader[p] && ++pos < m.maxRf) excludedAt[pos][m.rBroker[m.pSlots[s]]]++;
      }
    std::vector<std::set<std::pair<int, int>>> counts(m.maxRf);
    for (int i = 0; i < m.maxRf; ++i)
      for (int b = 0; b < m.B; ++b)
        if (m.alive(b)) counts[i].insert({excludedAt[i][b], m.bId[b]});
    // STEP1: the leader first
    for (const auto& parts : byTopic)
      for (int p : parts) {
        int at = m.pOff[p];
        while (m.pSlots[at] != m.pLeader[p]) ++at;
        if (at != m.pOff[p]) m.swapSlots(p, 0, at - m.pOff[p]);
      }
    // STEP2: every position over every partition, the first (count, id) broker off the racks of the earlier positions
    std::vector<int32_t> rackOfId(m.B);
    for (int b = 0; b < m.B; ++b) rackOfId[m.bId[b]] = m.bRack[b];
    for (int pos = 0; pos < m.maxRf; ++pos)
      for (const auto& parts : byTopic)
        for (int p : parts) {
          const int n = m.pOff[p + 1] - m.pOff[p];
          if (n <= pos) continue;
          const int r = m.pSlots[m.pOff[p] + pos];
          if (excl(m.pTopic[p]) && !m.origOffline(r)) continue;  // shouldExclude (:307-310)
          int usedRacks[kMaxRf], nr = 0;
          for (int q = 0; q < pos; ++q) usedRacks[nr++] = m.bRack[m.rBroker[m.pSlots[m.pOff[p] + q]]];
          auto& set = counts[pos];
          bool placed = false;
          for (auto it = set.begin(); it != set.end(); ++it) {
            const int dest = it->second;  // broker id == index (model.cpp)
            bool rackUsed = false;
            for (int q = 0; q < nr; ++q) rackUsed |= usedRacks[q] == rackOfId[dest];
            if (rackUsed) continue;
            const int src = m.rBroker[r];
            const int there = m.replicaOn(p, dest);
            if (there < 0) {
              m.relocateReplica(p, src, dest);
            } else if (dest != src && m.alive(src)) {
              if (pos == 0) {
                m.relocateLeadership(p, src, dest);
              } else {
                int at = 0;
                while (m.rBroker[m.pSlots[m.pOff[p] + at]] != dest) ++at;
                if (m.rLeader[m.pSlots[m.pOff[p] + pos]] || m.rLeader[m.pSlots[m.pOff[p] + at]])
                  throw std::invalid_argument("not a follower");  // Partition.swapFollowerPositions (:162-172)
                m.swapSlots(p, pos, at);
              }
            } else if (!m.alive(src)) {
              continue;
            }
            const std::pair<int, int> up{it->first + 1, it->second};
            set.erase(it);
            set.insert(up);
            placed = true;
            break;
          }
          if (!placed)
            throw OptimizationFailure("[" + name + "] Unable to apply move for replica " +
                                      replicaString(m, m.pSlots[m.pOff[p] + pos]) + ".");
        }
    ensureNoOfflineReplicas(m, name);
    // ensureRackAware (:351-373): every included partition on distinct racks
    for (int p = 0; p < m.P; ++p) {
      if (excl(m.pTopic[p])) continue;
      for (int s = m.pOff[p]; s < m.pOff[p + 1]; ++s)
        for (int u = s + 1; u < m.pOff[p + 1]; ++u)
          if (m.bRack[m.rBroker[m.pSlots[s]]] == m.bRack[m.rBroker[m.pSlots[u]]])
            throw OptimizationFailure("Optimization for goal " + name + " failed for rack-awareness of partition " +
                                      m.topicNames[m.pTopic[p]] + "-" + std::to_string(m.pNumber[p]));
    }
    succeeded = true;
    return true;
  }
  void rebalance(Engine&, int) override {}
  void update(Engine&) override { finished = true; }
  int compareStats(const ccmi_cluster_stats&, const ccmi_cluster_stats&) const override { return 0; }
};

class KafkaAssignerDiskUsageDistribution : public GoalImpl {
 public:
  KafkaAssignerDiskUsageDistribution() {
    kind = CCMI_GOAL_KAFKA_ASSIGNER_DISK_USAGE_DISTRIBUTION;
    name = "KafkaAssignerDiskUsageDistributionGoal";
    terminal = true;  // actionAcceptance throws IllegalStateException (:540-543)
    abstractGoal = false;
  }
  void init(Engine& e) override {
    kaSanityCheck(e);
    allowed.assign(e.m.B, 1);
    dg = DevGoal{};
    dg.kind = DG_ACCEPT_ALL;
    dg.allowedSlot = e.newSlot;
  }

  // optimize (:107-144) with checkAndOptimize (:197-252), swapReplicas (:268-383), isOptimized (:156-181)
  bool rebalanceAll(Engine& e) override {
    PhaseScope ps(PH_OTHER_GOALS);
    Model& m = e.m;
    const ReplicaOrder ro{&m};
    auto size = [&m](int r) { return m.ru(r, R_DISK); };
    auto usage = [&m](int b) {  // diskUsage(Broker) (:577-581)
      const double cap = m.cap(b, R_DISK);
      return jcmpDouble(cap, 0.0) < 1 ? 0.0 : m.bu(b, R_DISK) / cap;
    };
    auto bsize = [&](int b) { return usage(b) * m.cap(b, R_DISK); };
    auto excl = [&](int r) { return e.opt.anyExclTopic && e.opt.exclTopic[m.pTopic[m.rPart[r]]] != 0; };
    const double mean = m.clusterUtil(R_DISK) / m.clusterCap[R_DISK];
    const double margin = (e.bc.resBalance[R_DISK] - 1) * kBalanceMargin;
    const double upper = mean * (1 + margin), lower = mean * jmax(0, (1 - margin));
    // BrokerAndSortedReplicas: per alive broker a TreeSet by (replica size, Replica.compareTo) on live keys
    auto rcmp = [&](int x, int y) {
      const int c = jcmpDouble(size(x), size(y));
      return c ? c : ro.cmp(x, y);
    };
    using Sorted = RbTreeSet<decltype(rcmp)>;
    std::vector<std::unique_ptr<Sorted>> sorted(m.B);
    std::vector<int32_t> reps, all;
    for (int b = 0; b < m.B; ++b) {
      if (!m.alive(b)) continue;
      all.push_back(b);
      sorted[b] = std::make_unique<Sorted>(rcmp);
      m.bReplicaSet[b].order(reps);
      for (int r : reps) sorted[b]->add(r);
    }
    auto brokerLess = [&](int x, int y) {
      const int c = jcmpDouble(usage(x), usage(y));
      return c ? c < 0 : m.bId[x] < m.bId[y];
    };
    std::sort(all.begin(), all.end(), brokerLess);
    // a fresh TreeSet<ReplicaWrapper> of a broker's sorted replicas (followersOnly: !isLeader or excluded topic)
    std::vector<int> tmp;
    auto wrappers = [&](int b, bool followersOnly, std::vector<int32_t>& out) {
      sorted[b]->inorder(tmp);
      out.clear();
      for (int r : tmp)
        if (followersOnly ? (!m.rLeader[r] || excl(r)) : !excl(r)) out.push_back(r);
      std::sort(out.begin(), out.end(), [&](int x, int y) { return rcmp(x, y) < 0; });
      out.erase(std::unique(out.begin(), out.end(), [&](int x, int y) { return rcmp(x, y) == 0; }), out.end());
    };
    auto onRack = [&m](int p, int rack) {  // partition(tp).partitionRacks() contains rack
      for (int s = m.pOff[p]; s < m.pOff[p + 1]; ++s)
        if (m.bRack[m.rBroker[m.pSlots[s]]] == rack) return true;
      return false;
    };
    auto canSwap = [&](int r1, int r2) {  // (:504-518)
      const int b1 = m.rBroker[r1], b2 = m.rBroker[r2];
      const bool sameRack = b1 != b2 && m.bRack[b1] == m.bRack[b2];
      const bool aware = !onRack(m.rPart[r1], m.bRack[b2]) && !onRack(m.rPart[r2], m.bRack[b1]);
      return (sameRack || aware) && m.rLeader[r1] == m.rLeader[r2];
    };
    // findReplicaToSwapWith (:398-466): nearest to the target size first, from both sides of it
    auto findWith = [&](int r1, const std::vector<int32_t>& w, double target, double minS, double maxS) -> int {
      if (minS > maxS) return -1;
      if (jcmpDouble(minS, maxS) > 0) throw std::invalid_argument("fromKey > toKey");
      const auto lo = std::partition_point(w.begin(), w.end(), [&](int r) { return jcmpDouble(size(r), minS) <= 0; });
      const auto hi = std::partition_point(lo, w.end(), [&](int r) { return jcmpDouble(size(r), maxS) < 0; });
      if (lo == hi) return -1;
      const long upEnd = hi - w.begin(), downEnd = lo - w.begin();
      bool asc = false, desc = false;
      long up = 0, down = -1;
      if (target <= minS) {
        asc = true;
        up = lo - w.begin();
      } else if (target >= maxS) {
        desc = true;
        down = upEnd - 1;
      } else {  // tailSet((MIN_REPLICA, target), true) ascending, headSet((MAX_REPLICA, target), true) descending
        asc = desc = true;
        up = std::partition_point(lo, hi, [&](int r) { return jcmpDouble(size(r), target) < 0; }) - w.begin();
        down = (std::partition_point(lo, hi, [&](int r) { return jcmpDouble(size(r), target) <= 0; }) - w.begin()) - 1;
      }
      long low = -1, high = -1, cand = -1;
      for (;;) {
        if (cand == high) high = asc && up < upEnd ? up++ : -1;
        if (cand == low) low = desc && down >= downEnd ? down-- : -1;
        if (high < 0 && low < 0) return -1;
        if (high < 0) cand = low;
        else if (low < 0) cand = high;
        else cand = (target - size(w[low])) <= (size(w[high]) - target) ? low : high;
        if (canSwap(r1, w[cand])) return w[cand];
      }
    };
    std::vector<int32_t> mine, leadW, follW;
    auto swapReplicas = [&](int a, int bw) {
      const double capA = m.cap(a, R_DISK), capW = m.cap(bw, R_DISK);
      const double sizeToChange = capA * mean - bsize(a);
      wrappers(a, false, mine);
      wrappers(bw, false, leadW);
      wrappers(bw, true, follW);
      const size_t n = mine.size();
      for (size_t k = 0; k < n; ++k) {
        const int r = sizeToChange > 0 ? mine[k] : mine[n - 1 - k];
        if (excl(r)) continue;
        // possibleToMove (:481-491)
        const int p = m.rPart[r];
        if (!(!onRack(p, m.bRack[bw]) || (m.bRack[m.rBroker[r]] == m.bRack[bw] && m.replicaOn(p, bw) < 0))) continue;
        const std::vector<int32_t>& w = m.rLeader[r] ? leadW : follW;
        const double s = size(r);
        if (sizeToChange < 0 && s == 0) break;
        double maxSize = std::numeric_limits<double>::max(), minSize = std::numeric_limits<double>::denorm_min();
        if (sizeToChange > 0) {
          minSize = s;
          maxSize = jmin(maxSize, usage(bw) * capA - (bsize(a) - s));
          maxSize = jmin(maxSize, (bsize(bw) + s) - usage(a) * capW);
        } else {
          maxSize = s;
          minSize = jmax(minSize, usage(bw) * capA - (bsize(a) - s));
          minSize = jmax(minSize, (bsize(bw) + s) - usage(a) * capW);
        }
        minSize += 0.4;  // REPLICA_CONVERGENCE_DELTA
        maxSize -= 0.4;
        const int with = w.empty() ? -1 : findWith(r, w, s + sizeToChange, minSize, maxSize);
        if (with < 0) continue;
        m.relocateReplica(m.rPart[with], bw, a);
        m.relocateReplica(p, a, bw);
        sorted[a]->remove(r);
        sorted[a]->add(with);
        sorted[bw]->remove(with);
        sorted[bw]->add(r);
        return true;
      }
      return false;
    };
    bool improved;
    do {
      improved = false;
      const std::vector<int32_t> snapshot = all;
      for (int b : snapshot) {
        const double u = usage(b);
        const size_t at = (size_t)(std::find(all.begin(), all.end(), b) - all.begin());
        std::vector<int32_t> cands;
        if (u > upper) cands.assign(all.begin(), all.begin() + (ptrdiff_t)at);
        else if (u < lower) cands.assign(all.rbegin(), all.rend() - (ptrdiff_t)at);
        else continue;
        for (int w : cands) {
          if (w == b || std::fabs(usage(w) - usage(b)) < 0.0001) continue;  // USAGE_EQUALITY_DELTA
          const bool swapped = swapReplicas(b, w);
          if (swapped) {
            std::sort(all.begin(), all.end(), brokerLess);
            improved = true;
            break;
          }
        }
      }
    } while (improved);
    succeeded = true;
    for (int b = 0; b < m.B; ++b)
      if (m.alive(b) && (usage(b) < lower || usage(b) > upper)) succeeded = false;
    return true;
  }
  void rebalance(Engine&, int) override {}
  void update(Engine&) override { finished = true; }
  int compareStats(const ccmi_cluster_stats&, const ccmi_cluster_stats&) const override { return 0; }
};

// ======================================================================================= BrokerSetAwareGoal
// A hard goal: every replica must sit in the broker set its mapping policy names (TopicNameHash: the topic's set;
// ReplicaToOriginal: its original broker's set). Broker sets come with the call's BalancingConstraint (brokersets.h);
// the device reads BrokerRec.bset / ReplicaRec.bset when this goal is the optimized one or a prior one.
class BrokerSetAware : public GoalImpl {
 public:
  BrokerSetAware() {
    kind = CCMI_GOAL_BROKER_SET_AWARE;
    name = "BrokerSetAwareGoal";
  }
  std::vector<int32_t> alive;

  static std::string idList(const Model& m, const std::vector<int32_t>& v) {
    std::string out = "[";
    for (size_t i = 0; i < v.size(); ++i) out += (i ? ", " : "") + std::to_string(m.bId[v[i]]);
    return out + "]";
  }

  // initGoalState (BrokerSetAwareGoal.java:80-129)
  void init(Engine& e) override {
    Model& m = e.m;
    if (allowedForReplicaMove(e, allowed) == 0)
      throw OptimizationFailure("[" + name + "] All alive brokers are excluded from replica moves.", underBrokers(m.maxRf));
    // _excludedTopics = MinTopicLeadersPerBrokerGoal's topics + the options' excluded topics (:136-139)
    Model::Spec s;
    s.selImmigrants = e.opt.onlyImmigrants;
    s.selExclMust = e.opt.anyExclTopic || !e.bc.minLeaderTopics.empty();
    for (int b = 0; b < m.B; ++b) m.track(b, sortId(kind, false, false), s);
    // BrokerSetResolutionHelper + the mapping policy, frozen for the goal (the policy caches per topic)
    const BrokerSets& bs = e.brokerSets;
    if (bs.numSets == 0) throw std::invalid_argument("[" + name + "] no broker sets (BrokerSetResolutionException)");
    e.brokerSetOf = bs.ofBroker;
    e.replicaSetOf.assign(m.R, -1);
    std::vector<int32_t> topicSet;
    if (bs.policy == CCMI_BROKER_SET_TOPIC_NAME_HASH) {
      topicSet.resize(m.T);
      for (int t = 0; t < m.T; ++t) topicSet[t] = bsets::topicBrokerSet(m.topicNames[t], bs.numSets);
    }
    for (int r = 0; r < m.R; ++r)
      e.replicaSetOf[r] = (bs.policy == CCMI_BROKER_SET_TOPIC_NAME_HASH ? topicSet[m.pTopic[m.rPart[r]]]
                                                                        : e.brokerSetOf[m.rOrig[r]]) |
                          (m.mustTopicSel[m.pTopic[m.rPart[r]]] ? kBsetMust : 0);
    e.dev->setBrokerSets(e.brokerSetOf.data(), e.replicaSetOf.data());
    alive = aliveById(m);
    dg = DevGoal{};
    dg.kind = DG_BROKER_SET_AWARE;
    dg.allowedSlot = e.newSlot;
  }

  // rebalanceForBroker (:159-188): each misplaced replica goes to the first acceptable alive broker of its set in
  // HashSet<Broker> order, or the goal fails
  void rebalance(Engine& e, int b) override {
    PhaseScope ps(PH_OTHER_GOALS);
    Model& m = e.m;
    const std::vector<int32_t> list = m.sorted(b, sortId(kind, false, false));
    const int cur = e.brokerSetOf[b];
    std::vector<int32_t> one(1), ins, order, cands;
    for (int r : list) {
      const int want = bsetIndex(e.replicaSetOf[r]);
      if (m.alive(b) && want == cur) continue;
      ins.clear();
      for (int x : alive)
        if (e.brokerSetOf[x] == want) ins.push_back(x);
      javaHashSetOrder(ins, order);  // Collectors.toSet()
      e.eligible(order, DA_MOVE, cands);
      one[0] = r;
      const int64_t key = cands.empty() ? -1 : e.crossScan(*this, DA_MOVE, one, 0, cands);
      if (key < 0)
        throw OptimizationFailure("[" + name + "] Cannot move replica " + m.topicNames[m.pTopic[m.rPart[r]]] + "-" +
                                      std::to_string(m.pNumber[m.rPart[r]]) + " on broker " + std::to_string(m.bId[b]) +
                                      " to " + idList(m, order) + " on brokerSet " + e.brokerSets.names[want],
                                  underBrokers(m.maxRf));
      m.relocateReplica(m.rPart[r], b, cands[key]);
    }
  }

  // updateGoalState (:139-147) + ensureBrokerSetAware (:149-167)
  void update(Engine& e) override {
    Model& m = e.m;
    ensureNoOfflineReplicas(m, name);
    for (int b = 0; b < m.B; ++b)  // GoalUtils.ensureReplicasMoveOffBrokersWithBadDisks
      if (m.bState[b] == BState::BAD_DISKS)
        for (int r : m.bRepl[b])
          if (m.ineligible(m.rPart[r], b))
            throw OptimizationFailure("[" + name + "] A replica was moved back to broker with broken disk.",
                                      underBrokers(1));
    std::vector<int> topics(m.T);
    for (int t = 0; t < m.T; ++t) topics[t] = t;
    std::sort(topics.begin(), topics.end(), [&m](int a, int c) { return m.topicNames[a] < m.topicNames[c]; });
    std::vector<std::vector<int32_t>> byTopic(m.T);
    for (int p = 0; p < m.P; ++p)
      for (int i = m.pOff[p]; i < m.pOff[p + 1]; ++i) byTopic[m.pTopic[p]].push_back(m.rBroker[m.pSlots[i]]);
    std::vector<int32_t> ids, order;
    for (int t : topics) {  // getPartitionsByTopic: a TreeMap by topic name
      if ((e.opt.anyExclTopic && e.opt.exclTopic[t]) || m.mustTopicSel[t]) continue;
      const auto& v = byTopic[t];  // the topic's brokers in partition / slot order
      const int set = v.empty() ? -1 : e.brokerSetOf[v[0]];
      bool one = true;
      for (int x : v) one &= e.brokerSetOf[x] == set;
      if (one) continue;
      ids.clear();  // first appearances (HashSet insertion order), then Collectors.toSet() iteration order
      for (int x : v)
        if (std::find(ids.begin(), ids.end(), x) == ids.end()) ids.push_back(x);
      javaHashSetOrder(ids, order);
      throw OptimizationFailure("[" + name + "] Topic " + m.topicNames[t] + " is not brokerSet-aware. brokers (" +
                                idList(m, order) + ").");
    }
    finished = true;
  }
  int compareStats(const ccmi_cluster_stats&, const ccmi_cluster_stats&) const override { return 0; }
};

std::unique_ptr<GoalImpl> makeMoreGoal(int kind) {
  switch (kind) {
    case CCMI_GOAL_RACK_AWARE: return std::make_unique<RackAware>();
    case CCMI_GOAL_MIN_TOPIC_LEADERS_PER_BROKER: return std::make_unique<MinTopicLeaders>();
    case CCMI_GOAL_REPLICA_CAPACITY: return std::make_unique<ReplicaCapacity>();
    case CCMI_GOAL_DISK_CAPACITY:
    case CCMI_GOAL_NW_IN_CAPACITY:
    case CCMI_GOAL_NW_OUT_CAPACITY:
    case CCMI_GOAL_CPU_CAPACITY: return std::make_unique<Capacity>(kind);
    case CCMI_GOAL_POTENTIAL_NW_OUT: return std::make_unique<PotentialNwOut>();
    case CCMI_GOAL_TOPIC_REPLICA_DISTRIBUTION: return std::make_unique<TopicReplicaDistribution>();
    case CCMI_GOAL_TOPIC_LEADER_REPLICA_DISTRIBUTION: return std::make_unique<TopicLeaderReplicaDistribution>();
    case CCMI_GOAL_KAFKA_ASSIGNER_EVEN_RACK_AWARE: return std::make_unique<KafkaAssignerEvenRackAware>();
    case CCMI_GOAL_KAFKA_ASSIGNER_DISK_USAGE_DISTRIBUTION: return std::make_unique<KafkaAssignerDiskUsageDistribution>();
    case CCMI_GOAL_LEADER_REPLICA_DISTRIBUTION: return std::make_unique<LeaderReplicaDistribution>();
    case CCMI_GOAL_LEADER_BYTES_IN_DISTRIBUTION: return std::make_unique<LeaderBytesIn>();
    case CCMI_GOAL_PREFERRED_LEADER_ELECTION: return std::make_unique<PreferredLeaderElection>();
    case CCMI_GOAL_RACK_AWARE_DISTRIBUTION: return std::make_unique<RackAwareDist>();
    case CCMI_GOAL_BROKER_SET_AWARE: return std::make_unique<BrokerSetAware>();
    default: throw Unsupported("goal kind " + std::to_string(kind) + " is not implemented in this build");
  }
}

}  // namespace ccmi
