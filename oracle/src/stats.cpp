// ORACLE — test infrastructure only (see jsem.h header).
// Line-by-line restatement of ClusterModelStats.populate (ClusterModelStats.java:84-511).
// Iteration orders: brokers() is id-ascending; aliveBrokers() (HashSet<Broker>) is id-ascending for
// dense ids; topics() is a HashSet<String> whose iteration order only perturbs the last bits of the
// topic AVG/ST_DEV sums (parity for stats is 1e-9 relative, BASELINE.json north_star).
#include "stats.h"

#include <chrono>

#include <climits>
#include <cmath>

namespace oracle {

double computeResourceUtilizationBalanceThreshold(double avg, int resource, const BalancingConstraint& bc,
                                                  bool triggered, double margin, bool isLower) {
  if (margin >= 1) throw std::invalid_argument("Balance margin must be less than 1.0");
  bool isLowUtilization = avg <= bc.lowUtilizationThreshold[resource];
  double bp = bc.resourceBalancePercentage[resource];
  if (triggered) bp *= bc.goalViolationDistributionThresholdMultiplier;
  double withMargin = (bp - 1) * margin;
  if (isLower) {
    if (isLowUtilization) return 0.0;
    return avg * jmax(0, (1 - withMargin));
  }
  double thr = avg * (1 + withMargin);
  if (isLowUtilization) return jmax(thr, bc.lowUtilizationThreshold[resource] * margin);
  return thr;
}

namespace {
struct StatsTimer {  // ClusterModel::statsSeconds += the time of one ClusterModelStats.populate
  const ClusterModel& cm;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  ~StatsTimer() { cm.statsSeconds += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); }
};
}  // namespace

ClusterModelStats computeStats(const ClusterModel& cm, const BalancingConstraint& bc, const OptimizationOptions& o) {
  StatsTimer timer{cm};
  ClusterModelStats s{};
  const int B = (int)cm.brokers.size();
  std::vector<int> alive = cm.aliveBrokers();
  std::vector<char> allowed(B, 0);
  int numAllowed = 0;
  for (int b : alive)
    if (!o.excludedBrokersForReplicaMove.count(cm.brokers[b].id)) {
      allowed[b] = 1;
      numAllowed++;
    }
  s.numBrokers = B;
  s.numTopics = cm.numTopics();
  // utilizationForResources
  for (int res = 0; res < NUM_RESOURCES; ++res) {
    double resourceUtilization = expectedUtil(cm.load, res, cm.W);
    double avgPct = resourceUtilization / cm.capacityWithAllowedReplicaMovesFor(res, o);
    double upper = computeResourceUtilizationBalanceThreshold(avgPct, res, bc, o.triggeredByGoalViolation, 0.9, false);
    double lower = computeResourceUtilizationBalanceThreshold(avgPct, res, bc, o.triggeredByGoalViolation, 0.9, true);
    double hottest = 0.0, coldest = 1.7976931348623157e308, varianceSum = 0.0;
    int numBalanced = 0;
    for (int b : alive) {
      double u = isHostResource(res) ? cm.hostUtil(b, res) : cm.brokerUtil(b, res);
      hottest = jmax(hottest, u);
      coldest = jmin(coldest, u);
      if (allowed[b]) {
        double cap = isHostResource(res) ? cm.hostCapacity(b, res) : cm.brokers[b].capacity[res];
        double pct = u / cap;
        if (pct >= lower && pct <= upper) numBalanced++;
        double d = u - avgPct * cap;
        varianceSum += d * d;
      }
    }
    s.numBalancedBrokersByResource[res] = numBalanced;
    s.resAvg[res] = resourceUtilization / numAllowed;
    s.resMax[res] = hottest;
    s.resMin[res] = coldest;
    s.resStd[res] = std::sqrt(varianceSum / numAllowed);
  }
  // utilizationForPotentialNwOut
  {
    double maxP = 0.0, minP = 1.7976931348623157e308, varianceSum = 0.0;
    JDoubleSum sum;
    for (int b : alive)
      if (allowed[b]) sum.add(expectedUtil(cm.potentialLeadershipLoad[b], NW_OUT, cm.W));
    double inCluster = sum.result();
    double capacity = cm.capacityWithAllowedReplicaMovesFor(NW_OUT, o);
    double avgPct = inCluster / capacity;
    double thr = bc.capacityThreshold[NW_OUT];
    s.numBrokersUnderPotentialNwOut = 0;
    for (int b : alive) {
      double u = expectedUtil(cm.potentialLeadershipLoad[b], NW_OUT, cm.W);
      double cap = cm.brokers[b].capacity[NW_OUT];
      maxP = jmax(maxP, u);
      minP = jmin(minP, u);
      if (allowed[b]) {
        if (u / cap <= thr) s.numBrokersUnderPotentialNwOut++;
        double d = u - avgPct * cap;
        varianceSum += d * d;
      }
    }
    s.pnwAvg = inCluster / numAllowed;
    s.pnwMax = maxP;
    s.pnwMin = minP;
    s.pnwStd = std::sqrt(varianceSum / numAllowed);
  }
  // populateReplicaStats for replicas and leaders
  auto replicaStats = [&](auto countFn, double& avgOut, int& maxOut, int& minOut, double& stdOut) {
    int mx = 0, mn = INT_MAX, total = 0;
    for (int b = 0; b < B; ++b) {
      int n = countFn(b);
      total += n;
      mx = std::max(mx, n);
      mn = std::min(mn, n);
    }
    double avg = ((double)total) / numAllowed;
    double variance = 0.0;
    for (int b : alive)
      if (allowed[b]) {
        double d = (double)countFn(b) - avg;
        variance += (d * d) / numAllowed;
      }
    avgOut = avg;
    maxOut = mx;
    minOut = mn;
    stdOut = std::sqrt(variance);
  };
  replicaStats([&](int b) { return (int)cm.brokers[b].replicas.size(); }, s.repAvg, s.repMax, s.repMin, s.repStd);
  s.numReplicasInCluster = cm.numReplicas();
  {
    std::set<int> parts;
    for (int r : cm.selfHealingEligibleReplicas) parts.insert(cm.replicas[r].partition);
    s.numPartitionsWithOfflineReplicas = (int)parts.size();
  }
  replicaStats([&](int b) { return cm.brokers[b].numLeaders; }, s.leadAvg, s.leadMax, s.leadMin, s.leadStd);
  // numForAvgTopicReplicas
  {
    double avgAcc = 0.0, stdAcc = 0.0;
    int mxAcc = 0, mnAcc = INT_MAX;
    for (int t = 0; t < cm.numTopics(); ++t) {
      int mx = 0, mn = INT_MAX;
      double avg = ((double)cm.numReplicasByTopic[t]) / numAllowed;
      double variance = 0.0;
      for (int b = 0; b < B; ++b) {
        auto it = cm.brokers[b].topicReplicaCount.find(t);
        int n = it == cm.brokers[b].topicReplicaCount.end() ? 0 : it->second;
        mx = std::max(mx, n);
        mn = std::min(mn, n);
        if (cm.brokers[b].isAlive() && allowed[b]) {
          double d = n - avg;
          variance += (d * d) / numAllowed;
        }
      }
      avgAcc += avg;
      mxAcc = std::max(mxAcc, mx);
      mnAcc = std::min(mnAcc, mn);
      stdAcc += std::sqrt(variance);
    }
    s.topicAvg = avgAcc / s.numTopics;
    s.topicMax = mxAcc;
    s.topicMin = mnAcc;
    s.topicStd = stdAcc / s.numTopics;
  }
  // populateStatsForDisks (ClusterModelStats.java:489-511)
  {
    double totalVariance = 0;
    int numAliveDisks = 0;
    s.numUnbalancedDisks = 0;
    s.diskUtilizationStDev = 0.0;
    for (int b : alive) {
      const double brokerPct = cm.averageDiskUtilizationPct(b);
      const double upper = brokerPct * bc.resourceBalancePercentage[DISK];
      const double lower = brokerPct * jmax(0, (2 - bc.resourceBalancePercentage[DISK]));
      for (int d : cm.brokers[b].disks) {
        if (!cm.disks[d].alive) continue;
        const double pct = cm.diskUtilizationPct(d);
        if (pct > upper || pct < lower) s.numUnbalancedDisks++;
        totalVariance += std::pow(pct - brokerPct, 2);
        numAliveDisks++;
      }
    }
    if (numAliveDisks > 0) s.diskUtilizationStDev = std::sqrt(totalVariance / numAliveDisks);
  }
  return s;
}

}  // namespace oracle
