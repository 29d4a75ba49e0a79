// Synthetic input generator: the reference's RandomCluster fixture (src/test/java/.../model/RandomCluster.java
// :53-92 generate, :119-336 populate, :352-391 dead-broker marking; seeds TestConstants.java:19-26; capacities
// src/test/resources/DefaultCapacityConfig.json) emitted directly in the flattened desc layout, so benches and
// tests can build the 10K-broker / 1M-replica configurations without a JVM. JBOD (POPULATE_REPLICA_PLACEMENT_INFO):
// logdirs from src/test/resources/testCapacityConfigJBOD.json (or the C4 layout), replicas placed on disks by
// RandomCluster.java:315-331 (Broker.replicas() HashSet order) and bad disks marked by :430-443.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "ccmi.h"
#include "jsem.h"

#include "buffers.h"

namespace ccmi {

namespace {
int uniform(int lo, int hi, int64_t seed) { return JavaRandom(seed).nextInt(hi - lo + 1) + lo; }
double expRandom(double mean, JavaRandom& r) { return std::log(1.0 - r.nextDouble()) * (-mean); }

// Replica.compareTo on the generated arrays (all replicas online at placement time)
struct GenReplicaOrder {
  const ccmi_cluster_buffers* o;
  const std::vector<int32_t>* topicRank;
  int cmp(int a, int b) const {
    const int na = o->partNumber[o->repPart[a]], nb = o->partNumber[o->repPart[b]];
    if (na != nb) return na > nb ? 1 : -1;
    const int ia = o->repBroker[a], ib = o->repBroker[b];
    if (ia != ib) return ia > ib ? 1 : -1;
    const int ta = (*topicRank)[o->partTopic[o->repPart[a]]], tb = (*topicRank)[o->partTopic[o->repPart[b]]];
    return ta == tb ? 0 : (ta < tb ? -1 : 1);
  }
};

// logdir -> capacity of broker b (BrokerCapacityConfigFileResolver; TreeMap order is applied by the model)
std::vector<std::pair<std::string, double>> logdirsOf(const ccmi_random_cluster_props& p, int b) {
  std::vector<std::pair<std::string, double>> v;
  if (p.jbod == 1) {  // testCapacityConfigJBOD.json
    if (b == 0) {
      v = {{"/tmp/kafka-logs", 2000000.0}};
    } else if (b == 1 || b == 2) {
      v = {{"/tmp/kafka-logs-1", 350000.0}, {"/tmp/kafka-logs-2", 550000.0}};
      if (b == 2) v.insert(v.end(), {{"/tmp/kafka-logs-3", 750000.0}, {"/tmp/kafka-logs-4", 950000.0}});
    } else {
      for (int k = 1; k <= 10; ++k) v.push_back({"/tmp/kafka-logs-" + std::to_string(k), k == 1 ? 400000.0 : 200000.0});
    }
  } else if (p.jbod == 2) {
    for (int k = 0; k < p.num_logdirs; ++k) v.push_back({"/mnt/data-" + std::to_string(k + 1), p.logdir_capacity[k]});
  }
  return v;
}
}  // namespace

ccmi_cluster_buffers* generateRandomCluster(const ccmi_random_cluster_props& p) {
  const int B = p.num_brokers;
  if (p.num_racks > B || B <= 0 || p.num_racks <= 0) throw std::invalid_argument("Random cluster generation failed due to bad input.");
  if (p.jbod < 0 || p.jbod > 2 || (p.jbod == 2 && (p.num_logdirs < 1 || p.num_logdirs > 8)))
    throw std::invalid_argument("jbod must be 0, 1 or 2 (2: 1..8 logdirs)");
  if (p.num_brokers_with_bad_disk != 0 && !p.jbod && p.num_dead_brokers != 0)
    throw std::invalid_argument("bad-disk brokers without disks next to dead brokers are not generated");
  if (p.num_dead_brokers < 0 || p.num_brokers_with_bad_disk < 0 ||
      B < p.num_dead_brokers + p.num_brokers_with_bad_disk || p.num_topics <= 0 ||
      p.min_replication > p.max_replication || (p.leader_in_first_position && p.min_replication < 2) ||
      p.max_replication > B || p.num_topics > p.num_replicas ||
      (p.min_replication == p.max_replication && p.num_replicas % p.min_replication != 0))
    throw std::invalid_argument("Random cluster population failed due to bad input.");
  auto* out = new ccmi_cluster_buffers();
  auto& o = *out;
  // generate(): brokers 0..racks-1 on their own racks, the rest on seeded random racks
  o.brokerId.resize(B);
  o.brokerRack.resize(B);
  o.brokerState.assign(B, CCMI_BROKER_ALIVE);
  o.brokerCap.resize((size_t)4 * B);
  for (int b = 0; b < B; ++b) {
    o.brokerId[b] = b;
    o.brokerRack[b] = b < p.num_racks ? b : uniform(0, p.num_racks - 1, 3140 + b);
    const bool small = (b == 1);  // DefaultCapacityConfig.json overrides broker 1
    o.brokerCap[4 * b + CCMI_CPU] = 100.0;
    o.brokerCap[4 * b + CCMI_NW_IN] = small ? 150000.0 : 300000.0;
    o.brokerCap[4 * b + CCMI_NW_OUT] = small ? 150000.0 : 200000.0;
    o.brokerCap[4 * b + CCMI_DISK] = small ? 150000.0 : 300000.0;
    if (p.jbod == 1) {
      const double cpu = b == 0 ? 200.0 : (b <= 2 ? 300.0 : 100.0);
      const double nin = b == 0 ? 200000.0 : (b <= 2 ? 300000.0 : 100000.0);
      const double nout = b == 0 ? 200000.0 : (b <= 2 ? 200000.0 : 100000.0);
      o.brokerCap[4 * b + CCMI_CPU] = cpu;
      o.brokerCap[4 * b + CCMI_NW_IN] = nin;
      o.brokerCap[4 * b + CCMI_NW_OUT] = nout;
    }
    if (p.jbod) {
      double total = 0.0;
      for (const auto& l : logdirsOf(p, b)) {
        total += l.second;
        o.diskBroker.push_back(b);
        o.diskStr.push_back(l.first);
        o.diskCap.push_back(l.second);
      }
      o.brokerCap[4 * b + CCMI_DISK] = total;
    }
  }
  // populate(): topic replication factors and leader counts
  const int T0 = p.num_topics;
  std::vector<int> rf(T0, 1), leaders(T0, 1);
  int64_t total = T0;  // every topic starts at rf 1 x 1 leader
  for (int i = 0; i < T0; ++i) {
    const int r = uniform(p.min_replication, p.max_replication, 5234 + i);
    total += (int64_t)(r - rf[i]) * leaders[i];
    rf[i] = r;
    if (total > p.num_replicas) {
      total += (int64_t)(p.min_replication - rf[i]) * leaders[i];
      rf[i] = p.min_replication;
    }
  }
  const int maxRandomLeaders = p.num_replicas / T0;
  for (int i = 0; i < T0; ++i) {
    const int old = leaders[i];
    const int l = uniform(2, maxRandomLeaders, 72033 + i);
    total += (int64_t)(l - old) * rf[i];
    leaders[i] = l;
    if (total > p.num_replicas) {
      total -= (int64_t)(l - old) * rf[i];
      leaders[i] = old;
    }
  }
  while (total < p.num_replicas) {
    for (int i = 0; i < T0; ++i) {
      leaders[i]++;
      total += rf[i];
      if (total > p.num_replicas) {
        leaders[i]--;
        total -= rf[i];
      }
      if (total == p.num_replicas) break;
    }
  }
  for (int i = 0; i < T0; ++i) o.topicStr.push_back("T" + std::to_string(i));
  o.topicStr.push_back("TopicWithOneLeaderPerBroker");
  rf.push_back(2);
  leaders.push_back(B);
  const int T = T0 + 1;
  JavaRandom rCpu(100000), rDisk(300000), rNwIn(500000), rNwOut(700000), rPop(7234);
  int64_t R = 0, P = 0;
  for (int t = 0; t < T; ++t) {
    R += (int64_t)rf[t] * leaders[t];
    P += leaders[t];
  }
  o.partTopic.reserve(P);
  o.partNumber.reserve(P);
  o.partOff.reserve(P + 1);
  o.repPart.reserve(R);
  o.repBroker.reserve(R);
  o.repLeader.reserve(R);
  o.repLoad.reserve((size_t)R * 6);
  std::vector<int> usedB, usedR;
  int64_t replicaIndex = 0;
  for (int t = 0; t < T; ++t) {
    const double pop = expRandom(1.0, rPop);
    for (int i = 1; i <= leaders[t]; ++i) {
      const int part = (int)o.partTopic.size();
      o.partTopic.push_back(t);
      o.partNumber.push_back(i - 1);
      o.partOff.push_back((int32_t)o.repPart.size());
      usedB.clear();
      usedR.clear();
      int resolver = 0;
      auto taken = [&](int b) {
        for (int x : usedB)
          if (x == b) return true;
        if (p.rack_aware)
          for (int x : usedR)
            if (x == o.brokerRack[b]) return true;
        return false;
      };
      auto pick = [&](int64_t seed) {
        if (p.distribution == 0) return uniform(0, B - 1, seed);
        if (p.distribution == 1) {
          const int v = uniform(1, (B * (B + 1)) / 2, seed);
          for (int bin = 1; bin <= B; ++bin)
            if (2 * v <= bin * (bin + 1) && 2 * v > (bin - 1) * bin) return bin - 1;
          return 0;
        }
        const int v = uniform(1, B * B, seed);
        for (int bin = 1; bin <= B; ++bin)
          if (v <= bin * bin) return bin - 1;
        return 0;
      };
      for (int j = 1; j <= rf[t]; ++j) {
        int b = pick(1240 + replicaIndex);
        while (taken(b)) {
          resolver++;
          b = pick(1240 + replicaIndex + resolver);
        }
        // KafkaCruiseControlUnitTestUtils.setValueForResource: the value goes to the first metric of the group,
        // stored as MetricValues float windows (W = 1)
        float load[6] = {0, 0, 0, 0, 0, 0};
        load[CCMI_M_CPU_USAGE] = (float)expRandom(p.mean_cpu * pop, rCpu);
        load[CCMI_M_LEADER_BYTES_IN] = (float)expRandom(p.mean_nw_in * pop, rNwIn);
        load[CCMI_M_DISK_USAGE] = (float)expRandom(p.mean_disk * pop, rDisk);
        if (j == 1) load[CCMI_M_LEADER_BYTES_OUT] = (float)expRandom(p.mean_nw_out * pop, rNwOut);
        o.repPart.push_back(part);
        o.repBroker.push_back(b);
        o.repLeader.push_back(j == 1 ? 1 : 0);
        o.repLoad.insert(o.repLoad.end(), load, load + 6);
        usedB.push_back(b);
        usedR.push_back(o.brokerRack[b]);
        replicaIndex++;
      }
    }
  }
  o.partOff.push_back((int32_t)o.repPart.size());
  o.partReplicas.resize(o.repPart.size());
  for (size_t r = 0; r < o.repPart.size(); ++r) o.partReplicas[r] = (int32_t)r;
  if (!p.leader_in_first_position) {
    for (size_t q = 0; q + 1 < o.partOff.size(); ++q) {
      const int a = o.partOff[q];
      // the leader was created first: Partition.swapReplicaPositions(1, indexOf(leader) = 0)
      std::swap(o.partReplicas[a + 1], o.partReplicas[a]);
    }
  }
  o.repOffline.assign(o.repPart.size(), 0);
  std::vector<int32_t> repDisk;
  if (!p.jbod && p.num_brokers_with_bad_disk > 0) {
    // markBrokenBrokers without disk information (RandomCluster.java:409-449, no excluded topics): the first replica
    // in Broker.replicas() (HashSet<Replica>) order of each of the first alive brokers with replicas becomes
    // original-offline, and the broker whose id is the running count becomes BAD_DISKS (the reference passes the
    // count, not the broker's id)
    std::vector<int32_t> topicRank(T), topicHash(T);
    {
      std::vector<int> idx(T);
      for (int t = 0; t < T; ++t) idx[t] = t;
      std::sort(idx.begin(), idx.end(), [&](int a, int b) { return o.topicStr[a] < o.topicStr[b]; });
      for (int i = 0; i < T; ++i) topicRank[idx[i]] = i;
    }
    for (int t = 0; t < T; ++t) topicHash[t] = jStringHash(o.topicStr[t].c_str());
    GenReplicaOrder ord{&o, &topicRank};
    std::vector<JHashSet<GenReplicaOrder>> sets(B, JHashSet<GenReplicaOrder>(&ord));
    for (size_t r = 0; r < o.repPart.size(); ++r) {
      const int part = o.repPart[r];
      const int32_t tp = jMix(jMix(1, o.partNumber[part]), topicHash[o.partTopic[part]]);
      sets[o.repBroker[r]].add((int)r, jMix(jMix(1, tp), o.repBroker[r]));
    }
    std::vector<int32_t> members;
    int idx = 0;
    for (int b = 0; b < B && idx < p.num_brokers_with_bad_disk; ++b) {
      if (sets[b].size() == 0 || o.brokerState[b] == CCMI_BROKER_BAD_DISKS) continue;
      sets[b].order(members);
      o.repOffline[members.front()] = 1;
      o.brokerState[idx] = CCMI_BROKER_BAD_DISKS;
      idx++;
    }
  }
  if (p.jbod) {
    // Uniform-randomly assign replicas to disks: brokers by id, Broker.replicas() (HashSet<Replica>) order, the
    // conflict resolver counting per broker (RandomCluster.java:315-331)
    std::vector<int32_t> topicRank(T);
    {
      std::vector<int> idx(T);
      for (int t = 0; t < T; ++t) idx[t] = t;
      std::sort(idx.begin(), idx.end(), [&](int a, int b) { return o.topicStr[a] < o.topicStr[b]; });
      for (int i = 0; i < T; ++i) topicRank[idx[i]] = i;
    }
    std::vector<int32_t> topicHash(T);
    for (int t = 0; t < T; ++t) topicHash[t] = jStringHash(o.topicStr[t].c_str());
    GenReplicaOrder ord{&o, &topicRank};
    std::vector<JHashSet<GenReplicaOrder>> sets(B, JHashSet<GenReplicaOrder>(&ord));
    for (size_t r = 0; r < o.repPart.size(); ++r) {
      const int part = o.repPart[r];
      const int32_t tp = jMix(jMix(1, o.partNumber[part]), topicHash[o.partTopic[part]]);
      sets[o.repBroker[r]].add((int)r, jMix(jMix(1, tp), o.repBroker[r]));
    }
    std::vector<std::vector<int32_t>> disksOf(B);  // logdir order
    for (size_t k = 0; k < o.diskBroker.size(); ++k) disksOf[o.diskBroker[k]].push_back((int32_t)k);
    for (int b = 0; b < B; ++b)
      std::sort(disksOf[b].begin(), disksOf[b].end(), [&](int x, int y) { return o.diskStr[x] < o.diskStr[y]; });
    std::vector<double> util(o.diskBroker.size(), 0.0);
    repDisk.assign(o.repPart.size(), -1);
    std::vector<int32_t> members;
    for (int b = 0; b < B; ++b) {
      const auto& dl = disksOf[b];
      const int n = (int)dl.size();
      int resolver = 0, idx = 0;
      sets[b].order(members);
      for (int r : members) {
        const double f = (double)o.repLoad[(size_t)r * 6 + CCMI_M_DISK_USAGE];
        const double du = f > 0.0 ? f : (f != f ? f : 0.0);  // expectedUtilizationFor(DISK)
        int a = uniform(0, n - 1, 1240 + idx);
        while (o.diskCap[dl[a]] < util[dl[a]] + du) {
          resolver++;
          a = uniform(0, n - 1, 1240 + idx + resolver);
        }
        util[dl[a]] += du;
        repDisk[r] = dl[a];
        o.diskAssignReplica.push_back(r);
        o.diskAssignDisk.push_back(dl[a]);
        idx++;
      }
    }
    // markBrokenBrokers with disks: the first disk (logdir order) of the first alive brokers dies
    // (ClusterModel.markDiskDead: broker DISK capacity -= disk capacity, the disk's replicas original-offline)
    int marked = 0;
    for (int b = 0; b < B && marked < p.num_brokers_with_bad_disk; ++b) {
      if (b < p.num_dead_brokers || disksOf[b].empty()) continue;
      const int d = disksOf[b].front();
      o.brokerCap[4 * (size_t)b + CCMI_DISK] -= o.diskCap[d];
      o.diskCap[d] = -1.0;
      for (size_t r = 0; r < repDisk.size(); ++r)
        if (repDisk[r] == d) o.repOffline[r] = 1;
      o.brokerState[b] = CCMI_BROKER_BAD_DISKS;
      marked++;
    }
  }
  // markBrokenBrokers: brokers 0..numDead-1 become DEAD
  // (Broker.setState(DEAD) also overwrites the capacity with DEAD_BROKER_CAPACITY, Broker.java:322-329, and kills
  // the broker's disks)
  for (int b = 0; b < p.num_dead_brokers; ++b) {
    o.brokerState[b] = CCMI_BROKER_DEAD;
    for (int k = 0; k < 4; ++k) o.brokerCap[4 * (size_t)b + k] = -1.0;
    for (size_t k = 0; k < o.diskBroker.size(); ++k)
      if (o.diskBroker[k] == b) o.diskCap[k] = -1.0;
  }
  for (auto& s : o.topicStr) o.topicPtr.push_back(s.c_str());
  ccmi_cluster_desc& d = o.desc;
  std::memset(&d, 0, sizeof(d));
  d.num_windows = 1;
  d.num_racks = p.num_racks;
  d.num_brokers = B;
  d.broker_id = o.brokerId.data();
  d.broker_rack = o.brokerRack.data();
  d.broker_state = o.brokerState.data();
  d.broker_capacity = o.brokerCap.data();
  d.num_topics = T;
  d.topic_names = o.topicPtr.data();
  d.num_partitions = (int32_t)o.partTopic.size();
  d.partition_topic = o.partTopic.data();
  d.partition_number = o.partNumber.data();
  d.partition_offset = o.partOff.data();
  d.partition_replicas = o.partReplicas.data();
  d.num_replicas = (int32_t)o.repPart.size();
  d.replica_partition = o.repPart.data();
  d.replica_broker = o.repBroker.data();
  d.replica_is_leader = o.repLeader.data();
  d.replica_offline = o.repOffline.data();
  d.replica_load = o.repLoad.data();
  if (p.jbod) {
    for (auto& x : o.diskStr) o.diskPtr.push_back(x.c_str());
    d.num_disks = (int32_t)o.diskBroker.size();
    d.disk_broker = o.diskBroker.data();
    d.disk_logdir = o.diskPtr.data();
    d.disk_capacity = o.diskCap.data();
    d.replica_disk = nullptr;  // created without a disk; placed by the disk_assign replay
    d.num_disk_assignments = (int32_t)o.diskAssignReplica.size();
    d.disk_assign_replica = o.diskAssignReplica.data();
    d.disk_assign_disk = o.diskAssignDisk.data();
  }
  return out;
}

}  // namespace ccmi
