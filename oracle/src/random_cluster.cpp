// ORACLE — test infrastructure only (see jsem.h header).
// RandomCluster.java:53-92 (generate), :119-336 (populate), :352-391 (dead broker marking),
// :465-478 (uniformlyRandom / exponentialRandom), JBOD placement :315-331 with src/test/resources/
// testCapacityConfigJBOD.json (BrokerCapacityConfigFileResolver: DISK = sum of the logdir capacities). Math.log is glibc log (HotSpot's intrinsic is
// within 1 ulp; a rare last-bit difference is a documented residual generator risk).
#include "random_cluster.h"

#include <cmath>
#include <stdexcept>
#include <string>

namespace oracle {

static const int64_t SEED_BASE = 3140, REPLICATION_SEED = 5234, LEADER_SEED = 72033, REPLICA_ASSIGNMENT_SEED = 1240,
                     TOPIC_POPULARITY_SEED = 7234;

static int uniformlyRandom(int min, int max, int64_t seed) { return JRandom(seed).nextInt((max - min) + 1) + min; }
static double exponentialRandom(double mean, JRandom& r) { return std::log(1.0 - r.nextDouble()) * (-mean); }

struct TopicMeta {
  std::string name;
  int rf, leaders;
  int total() const { return rf * leaders; }
};

static int totalReplicas(const std::vector<TopicMeta>& m) {
  int t = 0;
  for (const auto& x : m) t += x.total();
  return t;
}

void randomCluster(ClusterModel& cm, const ClusterProperties& p) {
  if (p.numRacks > p.numBrokers || p.numBrokers <= 0 || p.numRacks <= 0) throw std::invalid_argument("bad input");
  cm.W = 1;
  for (int i = 0; i < p.numRacks; ++i) cm.createRack(std::to_string(i));
  auto create = [&](int rack, int i) {
    double cap[NUM_RESOURCES] = {100.0, 300000.0, 200000.0, 300000.0};  // CPU, NW_IN, NW_OUT, DISK
    if (i == 1) {
      cap[NW_IN] = 150000.0;
      cap[NW_OUT] = 150000.0;
      cap[DISK] = 150000.0;
    }
    std::vector<std::pair<std::string, double>> logdirs;
    if (p.jbod == 1) {  // testCapacityConfigJBOD.json
      if (i == 0) {
        cap[CPU] = 200.0, cap[NW_IN] = 200000.0, cap[NW_OUT] = 200000.0;
        logdirs = {{"/tmp/kafka-logs", 2000000.0}};
      } else if (i == 1 || i == 2) {
        cap[CPU] = 300.0, cap[NW_IN] = 300000.0, cap[NW_OUT] = 200000.0;
        logdirs = {{"/tmp/kafka-logs-1", 350000.0}, {"/tmp/kafka-logs-2", 550000.0}};
        if (i == 2) logdirs.insert(logdirs.end(), {{"/tmp/kafka-logs-3", 750000.0}, {"/tmp/kafka-logs-4", 950000.0}});
      } else {
        cap[CPU] = 100.0, cap[NW_IN] = 100000.0, cap[NW_OUT] = 100000.0;
        for (int k = 1; k <= 10; ++k) logdirs.push_back({"/tmp/kafka-logs-" + std::to_string(k), k == 1 ? 400000.0 : 200000.0});
      }
    } else if (p.jbod == 2) {
      for (int k = 0; k < p.numLogdirs; ++k) logdirs.push_back({"/mnt/data-" + std::to_string(k + 1), p.logdirCapacity[k]});
    }
    if (p.jbod) {
      double total = 0.0;
      for (const auto& l : logdirs) total += l.second;
      cap[DISK] = total;
    }
    cm.createBroker(rack, i, cap);
    for (const auto& l : logdirs) cm.createDisk(i, l.first, l.second);
  };
  for (int i = 0; i < p.numRacks; ++i) create(i, i);
  for (int i = p.numRacks; i < p.numBrokers; ++i) create(uniformlyRandom(0, p.numRacks - 1, SEED_BASE + i), i);
  // populate
  const int numBrokers = p.numBrokers;
  if (p.numDeadBrokers < 0 || p.numBrokersWithBadDisk < 0 || numBrokers < p.numDeadBrokers + p.numBrokersWithBadDisk ||
      p.numTopics <= 0 || p.minReplication > p.maxReplication || (p.leaderInFirstPosition && p.minReplication < 2) ||
      p.maxReplication > numBrokers || p.numTopics > p.numReplicas ||
      (p.minReplication == p.maxReplication && p.numReplicas % p.minReplication != 0))
    throw std::invalid_argument("Random cluster population failed due to bad input.");
  std::vector<TopicMeta> meta;
  for (int i = 0; i < p.numTopics; ++i) meta.push_back({"T" + std::to_string(i), 1, 1});
  for (int i = 0; i < p.numTopics; ++i) {
    meta[i].rf = uniformlyRandom(p.minReplication, p.maxReplication, REPLICATION_SEED + i);
    if (totalReplicas(meta) > p.numReplicas) meta[i].rf = p.minReplication;
  }
  int maxRandomLeaders = p.numReplicas / p.numTopics;
  for (int i = 0; i < p.numTopics; ++i) {
    int old = meta[i].leaders;
    meta[i].leaders = uniformlyRandom(2, maxRandomLeaders, LEADER_SEED + i);
    if (totalReplicas(meta) > p.numReplicas) meta[i].leaders = old;
  }
  int total = totalReplicas(meta);
  while (total < p.numReplicas) {
    for (int i = 0; i < p.numTopics; ++i) {
      meta[i].leaders++;
      total += meta[i].rf;
      if (total > p.numReplicas) {
        meta[i].leaders--;
        total -= meta[i].rf;
      }
      if (total == p.numReplicas) break;
    }
  }
  JRandom rCpu(100000), rDisk(300000), rNwIn(500000), rNwOut(700000);
  JRandom rPop(TOPIC_POPULARITY_SEED);
  meta.push_back({"TopicWithOneLeaderPerBroker", 2, numBrokers});
  for (const auto& m : meta) cm.ensureTopic(m.name);
  int replicaIndex = 0;
  for (size_t ti = 0; ti < meta.size(); ++ti) {
    const TopicMeta& datum = meta[ti];
    double pop = exponentialRandom(1.0, rPop);
    for (int i = 1; i <= datum.leaders; ++i) {
      std::vector<int> usedBrokers, usedRacks;
      int resolver = 0;
      auto used = [&](int b) {
        for (int x : usedBrokers)
          if (x == b) return true;
        if (p.rackAware)
          for (int rk : usedRacks)
            if (rk == cm.brokers[b].rack) return true;
        return false;
      };
      auto binOf = [&](int v, bool linear) {
        for (int bin = 1; bin <= numBrokers; ++bin) {
          if (linear) {
            int bv = 2 * v;
            if (bv <= bin * (bin + 1) && bv > (bin - 1) * bin) return bin - 1;
          } else if (v <= bin * bin) {
            return bin - 1;
          }
        }
        return 0;
      };
      int partitionIdx = -1;
      for (int j = 1; j <= datum.rf; ++j) {
        int b;
        if (p.distribution == 0) {
          b = uniformlyRandom(0, numBrokers - 1, REPLICA_ASSIGNMENT_SEED + replicaIndex);
          while (used(b)) {
            resolver++;
            b = uniformlyRandom(0, numBrokers - 1, REPLICA_ASSIGNMENT_SEED + replicaIndex + resolver);
          }
        } else {
          bool linear = p.distribution == 1;
          int range = linear ? (numBrokers * (numBrokers + 1)) / 2 : numBrokers * numBrokers;
          int v = uniformlyRandom(1, range, REPLICA_ASSIGNMENT_SEED + replicaIndex);
          b = binOf(v, linear);
          while (used(b)) {
            resolver++;
            v = uniformlyRandom(1, range, REPLICA_ASSIGNMENT_SEED + replicaIndex + resolver);
            b = binOf(v, linear);
          }
        }
        Load amv;
        amv.mask = 0x3F;
        for (int k = 0; k < NUM_METRICS; ++k) mvZero(amv.m[k], 1);
        double cpu = exponentialRandom(p.meanCpu * pop, rCpu);
        mvSet(amv.m[M_CPU], 0, cpu);
        double nwIn = exponentialRandom(p.meanNwIn * pop, rNwIn);
        mvSet(amv.m[M_LBI], 0, nwIn);
        double disk = exponentialRandom(p.meanDisk * pop, rDisk);
        mvSet(amv.m[M_DISK], 0, disk);
        bool leader = (j == 1);
        if (leader) {
          double nwOut = exponentialRandom(p.meanNwOut * pop, rNwOut);
          mvSet(amv.m[M_LBO], 0, nwOut);
        } else {
          mvSet(amv.m[M_LBO], 0, 0.0);
        }
        // AggregatedMetricValues.add(id, metricValues) copies through MetricValues.add (float values only)
        Load staged;
        amvAdd(staged, amv, 1);
        if (j == 1) partitionIdx = cm.createPartition((int)ti, i - 1);
        int r = cm.createReplica(b, partitionIdx, j - 1, leader, !cm.brokers[b].isAlive());
        cm.setReplicaLoad(r, staged);
        usedBrokers.push_back(b);
        usedRacks.push_back(cm.brokers[b].rack);
        replicaIndex++;
      }
      if (!p.leaderInFirstPosition) {
        Partition& part = cm.partitions[partitionIdx];
        int lpos = 0;
        for (size_t k = 0; k < part.replicas.size(); ++k)
          if (part.replicas[k] == part.leader) lpos = (int)k;
        std::swap(part.replicas[1], part.replicas[lpos]);
      }
    }
  }
  cm.finalizeTopics();
  // Uniform-randomly assign replicas to disks (RandomCluster.java:315-331): brokers by id, Broker.replicas() HashSet
  // order, conflict resolver per broker
  if (p.jbod) {
    for (int b = 0; b < (int)cm.brokers.size(); ++b) {
      int resolver = 0, idx = 0;
      const std::vector<int> dl = cm.brokers[b].disks;
      const int n = (int)dl.size();
      for (int r : cm.brokers[b].replicaSet.order()) {
        const double du = cm.replicaUtil(r, DISK);
        int a = uniformlyRandom(0, n - 1, REPLICA_ASSIGNMENT_SEED + idx);
        while (cm.disks[dl[a]].capacity < cm.disks[dl[a]].utilization + du) {
          resolver++;
          a = uniformlyRandom(0, n - 1, REPLICA_ASSIGNMENT_SEED + idx + resolver);
        }
        cm.diskAddReplica(dl[a], r);
        cm.diskAssignLog.push_back({r, dl[a]});
        idx++;
      }
    }
  }
  // markBrokenBrokers: dead brokers (no excluded topics in scope)
  if (p.numDeadBrokers > 0) {
    int idx = 0;
    while (p.numDeadBrokers - idx > 0) {
      if (cm.brokers[idx].isAlive()) cm.setBrokerState(idx, BrokerState::DEAD);
      idx++;
    }
  }
  if (p.numBrokersWithBadDisk > 0) {
    if (!p.jbod) {
      // Without disk information (RandomCluster.java:409-449, no excluded topics): the first replica in
      // Broker.replicas() (HashSet) order of each of the first alive brokers with replicas becomes original-offline,
      // and the broker whose id is the running count is set to BAD_DISKS (the reference passes the count, not the id)
      if (p.numDeadBrokers > 0)
        throw std::invalid_argument("bad-disk brokers without disks next to dead brokers are outside the oracle scope");
      int idx = 0;
      for (int b = 0; b < (int)cm.brokers.size() && idx < p.numBrokersWithBadDisk; ++b) {
        const Broker& br = cm.brokers[b];
        if (br.replicas.empty() || !br.isAlive() || br.hasBadDisks()) continue;
        cm.markReplicaOriginalOffline(br.replicaSet.order().front());
        cm.setBrokerState(idx, BrokerState::BAD_DISKS);
        idx++;
      }
      return;
    }
    int marked = 0;  // one (the first, TreeMap order) disk of each of the first alive brokers
    for (int b = 0; b < (int)cm.brokers.size() && marked < p.numBrokersWithBadDisk; ++b) {
      if (!cm.brokers[b].isAlive()) continue;
      cm.markDiskDead(b, cm.brokers[b].disks.front());
      cm.setBrokerState(b, BrokerState::BAD_DISKS);
      marked++;
    }
  }
}

}  // namespace oracle
