// Synthetic input generator: the reference's RandomCluster fixture (src/test/java/.../model/RandomCluster.java
// :53-92 generate, :119-336 populate, :352-391 dead-broker marking; seeds TestConstants.java:19-26; capacities
// src/test/resources/DefaultCapacityConfig.json) emitted directly in the flattened desc layout, so benches and
// tests can build the 10K-broker / 1M-replica configurations without a JVM.
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
}  // namespace

ccmi_cluster_buffers* generateRandomCluster(const ccmi_random_cluster_props& p) {
  const int B = p.num_brokers;
  if (p.num_racks > B || B <= 0 || p.num_racks <= 0) throw std::invalid_argument("Random cluster generation failed due to bad input.");
  if (p.num_dead_brokers < 0 || p.num_brokers_with_bad_disk != 0 || B < p.num_dead_brokers || p.num_topics <= 0 ||
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
  // markBrokenBrokers: brokers 0..numDead-1 become DEAD
  // (Broker.setState(DEAD) also overwrites the capacity with DEAD_BROKER_CAPACITY, Broker.java:322-329)
  for (int b = 0; b < p.num_dead_brokers; ++b) {
    o.brokerState[b] = CCMI_BROKER_DEAD;
    for (int k = 0; k < 4; ++k) o.brokerCap[4 * (size_t)b + k] = -1.0;
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
  return out;
}

}  // namespace ccmi
