// Model ingestion: LoadMonitor.clusterModel's model-building calls flattened straight into a
// ccmi_cluster_desc. Restates:
//   LoadMonitor.populateClusterCapacity   monitor/LoadMonitor.java:563-600 (createRack + createBroker per live node)
//   ClusterModel.handleDeadBroker         model/ClusterModel.java:772-779
//   MonitorUtils.populatePartitionLoad    monitor/MonitorUtils.java:415-479 (createReplica + setReplicaLoad per replica)
//   MonitorUtils.getAggregatedMetricValues / adjustCpuUsage / fillInReplicationBytesOut / toFollowerMetricValues
//                                         monitor/MonitorUtils.java:83-107,198-265
//   ModelUtils.getFollowerCpuUtilFromLeaderLoad  model/ModelUtils.java:64-80 (static weights, ModelParameters.java:23-31)
//   MonitorUtils.setBadBrokerState        monitor/MonitorUtils.java:349-356
// MetricValues hold floats (every set() rounds a double to float); group sums (AggregatedMetricValues.valuesForGroup)
// add the group's metrics into a zeroed float array in metric-id order.
#include <algorithm>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "ccmi.h"
#include "errors.h"  // setLastError (ccmi_last_error)

namespace {

constexpr double kUnitIntervalToPercentage = 100.0;         // MonitorUtils.UNIT_INTERVAL_TO_PERCENTAGE
constexpr double kCpuWeightLeaderBytesIn = 0.7;             // ModelParameters defaults
constexpr double kCpuWeightLeaderBytesOut = 0.15;
constexpr double kCpuWeightFollowerBytesIn = 0.15;

struct BrokerIn {
  int32_t id;
  int32_t rack;
  double cap[4];
  int32_t state;
  std::string host;  // Rack._hosts key (handleDeadBroker: "UNKNOWN_HOST-<n>", a host of its own)
};
struct DiskIn {
  int32_t brokerId;
  std::string logdir;
  double cap;
  uint8_t demoted = 0;
};

}  // namespace

struct ccmi_model_builder {
  int32_t W = 1;
  std::vector<std::string> rackNames;
  std::map<std::string, int32_t> rackIndex;
  std::vector<BrokerIn> brokers;  // creation order
  std::map<int32_t, size_t> brokerById;
  std::vector<DiskIn> disks;
  std::vector<std::string> topics;
  std::map<std::string, int32_t> topicIndex;
  // partitions / replicas in populate order
  std::vector<int32_t> pTopic, pNumber, pOff{0};
  std::vector<int32_t> rBrokerId, rPartition;
  std::vector<uint8_t> rLeader, rOffline;
  std::vector<std::string> rLogdir;  // "" = none
  std::vector<float> rLoad;          // [R][6][W]
  // flattened output (ccmi_builder_desc)
  std::vector<int32_t> oBrokerId, oRack, oState, oRBroker, oPartReplicas, oDiskBroker, oRDisk, oHost;
  std::vector<uint8_t> oDiskDemoted;
  int32_t unknownHosts = 0;
  std::vector<double> oCap, oDiskCap;
  std::vector<const char*> oTopicNames, oDiskLogdir;
  std::vector<int32_t> sortedIds;
};

namespace {

template <class F>
ccmi_status run(F&& f) {
  try {
    f();
    return CCMI_OK;
  } catch (std::exception& e) {
    ccmi::setLastError(e.what());
    return CCMI_E_INVALID;
  }
}

int32_t rackOf(ccmi_model_builder* b, const std::string& rack) {  // ClusterModel.createRack (putIfAbsent)
  auto it = b->rackIndex.find(rack);
  if (it != b->rackIndex.end()) return it->second;
  const int32_t i = (int32_t)b->rackNames.size();
  b->rackNames.push_back(rack);
  b->rackIndex.emplace(rack, i);
  return i;
}

// AggregatedMetricValues.valuesForGroup: a zeroed float array plus each metric of the group in metric-id order
float groupSum(const float* agg, int W, int w, int m0, int m1) {
  float s = 0.0f;
  s += agg[m0 * W + w];
  s += agg[m1 * W + w];
  return s;
}

}  // namespace

extern "C" {

ccmi_status ccmi_builder_create(int32_t num_windows, ccmi_model_builder** out) {
  if (!out || num_windows < 1 || num_windows > 5) return CCMI_E_INVALID;
  *out = new ccmi_model_builder();
  (*out)->W = num_windows;
  return CCMI_OK;
}

void ccmi_builder_destroy(ccmi_model_builder* b) { delete b; }

ccmi_status ccmi_builder_create_broker(ccmi_model_builder* b, const char* rack, const char* host,
                                       int32_t broker_id, const double capacity[4], int32_t alive) {
  if (!b || !rack || !capacity || broker_id < 0) return CCMI_E_INVALID;
  return run([&] {
    const bool exists = b->brokerById.count(broker_id) != 0;
    if (exists) {
      if (alive) throw std::invalid_argument("broker " + std::to_string(broker_id) + " created twice");
      return;  // handleDeadBroker: nothing to do for a known broker
    }
    BrokerIn x;
    x.id = broker_id;
    x.rack = rackOf(b, rack);
    std::memcpy(x.cap, capacity, sizeof(x.cap));
    // handleDeadBroker creates the broker alive; setBadBrokerState marks it dead once the partitions are in — the
    // desc applies broker states after every replica is created, so the state is recorded now
    x.state = alive ? CCMI_BROKER_ALIVE : CCMI_BROKER_DEAD;
    // a live node's host (LoadMonitor.java:602); a dead one gets UNKNOWN_HOST-<n> (ClusterModel.java:776-777)
    x.host = alive && host ? std::string(host) : "UNKNOWN_HOST-" + std::to_string(b->unknownHosts++);
    b->brokerById.emplace(broker_id, b->brokers.size());
    b->brokers.push_back(x);
  });
}

ccmi_status ccmi_builder_add_disk(ccmi_model_builder* b, int32_t broker_id, const char* logdir, double capacity) {
  if (!b || !logdir) return CCMI_E_INVALID;
  return run([&] {
    if (!b->brokerById.count(broker_id)) throw std::invalid_argument("unknown broker");
    for (const DiskIn& d : b->disks)
      if (d.brokerId == broker_id && d.logdir == logdir) throw std::invalid_argument("duplicate logdir");
    b->disks.push_back(DiskIn{broker_id, logdir, capacity});
  });
}

ccmi_status ccmi_builder_populate_partition(ccmi_model_builder* b, const char* topic, int32_t partition,
                                            const int32_t* replica_broker_ids, int32_t num_replicas,
                                            int32_t leader_broker_id, const uint8_t* offline,
                                            const char* const* logdirs, const float* leader_metrics) {
  if (!b || !topic || !replica_broker_ids || num_replicas < 1 || num_replicas > 8 || !leader_metrics)
    return CCMI_E_INVALID;
  return run([&] {
    for (int i = 0; i < num_replicas; ++i) {
      if (!b->brokerById.count(replica_broker_ids[i]))
        throw std::invalid_argument("replica on unknown broker " + std::to_string(replica_broker_ids[i]) +
                                    " (create it first: ccmi_builder_create_broker with alive = 0)");
      for (int j = 0; j < i; ++j)
        if (replica_broker_ids[j] == replica_broker_ids[i]) throw std::invalid_argument("duplicate replica broker");
    }
    if (leader_broker_id < 0) return;  // offline partition: LoadMonitor skips its replicas
    int leaders = 0;
    for (int i = 0; i < num_replicas; ++i) leaders += replica_broker_ids[i] == leader_broker_id ? 1 : 0;
    if (leaders != 1)
      throw std::invalid_argument("partition " + std::string(topic) + "-" + std::to_string(partition) + ": leader broker " +
                                  std::to_string(leader_broker_id) + " is not one of its replica brokers");
    const int W = b->W;
    auto ti = b->topicIndex.find(topic);
    int32_t t;
    if (ti == b->topicIndex.end()) {
      t = (int32_t)b->topics.size();
      b->topics.push_back(topic);
      b->topicIndex.emplace(topic, t);
    } else {
      t = ti->second;
    }
    const int32_t p = (int32_t)b->pTopic.size();
    b->pTopic.push_back(t);
    b->pNumber.push_back(partition);
    // the partition's aggregated leader values, mutated in place as the reference does (one shared object)
    std::vector<float> agg(leader_metrics, leader_metrics + CCMI_NUM_METRICS * W);
    bool needToAdjustCpuUsage = true;
    for (int i = 0; i < num_replicas; ++i) {
      const bool isLeader = replica_broker_ids[i] == leader_broker_id;
      if (needToAdjustCpuUsage)  // adjustCpuUsage
        for (int w = 0; w < W; ++w)
          agg[CCMI_M_CPU_USAGE * W + w] = (float)((double)agg[CCMI_M_CPU_USAGE * W + w] * kUnitIntervalToPercentage);
      float load[CCMI_NUM_METRICS * 5];
      if (isLeader) {  // fillInReplicationBytesOut
        const int numFollowers = num_replicas - 1;
        for (int w = 0; w < W; ++w)
          agg[CCMI_M_REPLICATION_BYTES_OUT * W + w] = (float)((double)agg[CCMI_M_LEADER_BYTES_IN * W + w] * numFollowers);
        std::memcpy(load, agg.data(), sizeof(float) * CCMI_NUM_METRICS * W);
      } else {  // toFollowerMetricValues
        for (int w = 0; w < W; ++w) {
          const double lbi = groupSum(agg.data(), W, w, CCMI_M_LEADER_BYTES_IN, CCMI_M_REPLICATION_BYTES_IN);
          const double lbo = groupSum(agg.data(), W, w, CCMI_M_LEADER_BYTES_OUT, CCMI_M_REPLICATION_BYTES_OUT);
          const double cpu = agg[CCMI_M_CPU_USAGE * W + w];
          double f;
          if (lbi == 0.0 && lbo == 0.0) f = 0.0;
          else f = cpu * (kCpuWeightFollowerBytesIn * lbi) / (kCpuWeightLeaderBytesIn * lbi + kCpuWeightLeaderBytesOut * lbo);
          load[CCMI_M_CPU_USAGE * W + w] = (float)f;
          load[CCMI_M_DISK_USAGE * W + w] = agg[CCMI_M_DISK_USAGE * W + w];
          load[CCMI_M_LEADER_BYTES_IN * W + w] = agg[CCMI_M_LEADER_BYTES_IN * W + w];
          load[CCMI_M_REPLICATION_BYTES_IN * W + w] = agg[CCMI_M_REPLICATION_BYTES_IN * W + w];
          load[CCMI_M_LEADER_BYTES_OUT * W + w] = 0.0f;
          load[CCMI_M_REPLICATION_BYTES_OUT * W + w] = 0.0f;
        }
      }
      needToAdjustCpuUsage = false;
      b->rBrokerId.push_back(replica_broker_ids[i]);
      b->rPartition.push_back(p);
      b->rLeader.push_back(isLeader ? 1 : 0);
      b->rOffline.push_back(offline && offline[i] ? 1 : 0);
      b->rLogdir.push_back(logdirs && logdirs[i] ? logdirs[i] : "");
      b->rLoad.insert(b->rLoad.end(), load, load + CCMI_NUM_METRICS * W);
    }
    b->pOff.push_back((int32_t)b->rBrokerId.size());
  });
}

ccmi_status ccmi_builder_set_broker_state(ccmi_model_builder* b, int32_t broker_id, int32_t state) {
  if (!b || state < CCMI_BROKER_ALIVE || state > CCMI_BROKER_BAD_DISKS) return CCMI_E_INVALID;
  return run([&] {
    auto it = b->brokerById.find(broker_id);
    if (it == b->brokerById.end()) throw std::invalid_argument("unknown broker");
    BrokerIn& x = b->brokers[it->second];
    // setBadBrokerState: BAD_DISKS only for a broker that is still alive
    if (state == CCMI_BROKER_BAD_DISKS && x.state == CCMI_BROKER_DEAD) return;
    x.state = state;
  });
}

ccmi_status ccmi_builder_set_disk_state(ccmi_model_builder* b, int32_t broker_id, const char* logdir, int32_t state) {
  if (!b || !logdir || (state != CCMI_DISK_ALIVE && state != CCMI_DISK_DEMOTED)) return CCMI_E_INVALID;
  return run([&] {
    for (DiskIn& d : b->disks)
      if (d.brokerId == broker_id && d.logdir == logdir) {
        d.demoted = state == CCMI_DISK_DEMOTED ? 1 : 0;
        return;
      }
    // DemoteBrokerRunnable.java:144-146
    throw std::invalid_argument("Broker " + std::to_string(broker_id) + " does not have logdir " + logdir + ".");
  });
}

ccmi_status ccmi_builder_desc(ccmi_model_builder* b, ccmi_cluster_desc* out) {
  if (!b || !out) return CCMI_E_INVALID;
  return run([&] {
    const int B = (int)b->brokers.size(), R = (int)b->rBrokerId.size(), P = (int)b->pTopic.size();
    if (B == 0) throw std::invalid_argument("no brokers");
    b->sortedIds.clear();
    for (const BrokerIn& x : b->brokers) b->sortedIds.push_back(x.id);
    std::sort(b->sortedIds.begin(), b->sortedIds.end());
    std::map<int32_t, int32_t> indexOf;
    for (int i = 0; i < B; ++i) indexOf[b->sortedIds[i]] = i;
    b->oBrokerId.resize(B);
    b->oRack.resize(B);
    b->oState.resize(B);
    b->oCap.resize((size_t)B * 4);
    for (int i = 0; i < B; ++i) {
      const BrokerIn& x = b->brokers[b->brokerById.at(b->sortedIds[i])];
      b->oBrokerId[i] = i;
      b->oRack[i] = x.rack;
      b->oState[i] = x.state;
      for (int k = 0; k < 4; ++k) b->oCap[(size_t)i * 4 + k] = x.cap[k];
    }
    // hosts: one per (rack, host name) (Rack._hosts), indexed in first-broker order
    {
      std::map<std::pair<int32_t, std::string>, int32_t> hostIndex;
      b->oHost.resize(B);
      for (int i = 0; i < B; ++i) {
        const BrokerIn& x = b->brokers[b->brokerById.at(b->sortedIds[i])];
        auto it = hostIndex.emplace(std::make_pair(x.rack, x.host), (int32_t)hostIndex.size()).first;
        b->oHost[i] = it->second;
      }
    }
    b->oRBroker.resize(R);
    for (int r = 0; r < R; ++r) b->oRBroker[r] = indexOf.at(b->rBrokerId[r]);
    b->oPartReplicas.resize(R);
    for (int r = 0; r < R; ++r) b->oPartReplicas[r] = r;  // populate order is Partition._replicas order
    b->oTopicNames.clear();
    for (const std::string& s : b->topics) b->oTopicNames.push_back(s.c_str());
    // disks: broker index, then logdir String order (Broker._diskByLogdir is a TreeMap)
    std::vector<size_t> dOrder(b->disks.size());
    for (size_t i = 0; i < dOrder.size(); ++i) dOrder[i] = i;
    std::sort(dOrder.begin(), dOrder.end(), [&](size_t x, size_t y) {
      const int bx = indexOf.at(b->disks[x].brokerId), by = indexOf.at(b->disks[y].brokerId);
      return bx != by ? bx < by : b->disks[x].logdir < b->disks[y].logdir;
    });
    b->oDiskBroker.clear();
    b->oDiskCap.clear();
    b->oDiskLogdir.clear();
    b->oDiskDemoted.clear();
    for (size_t i : dOrder) {
      b->oDiskDemoted.push_back(b->disks[i].demoted);
      b->oDiskBroker.push_back(indexOf.at(b->disks[i].brokerId));
      b->oDiskCap.push_back(b->brokers[b->brokerById.at(b->disks[i].brokerId)].state == CCMI_BROKER_DEAD
                                ? -1.0
                                : b->disks[i].cap);
      b->oDiskLogdir.push_back(b->disks[i].logdir.c_str());
    }
    b->oRDisk.assign(R, -1);
    if (!b->disks.empty())
      for (int r = 0; r < R; ++r) {
        if (b->rLogdir[r].empty()) continue;
        for (size_t k = 0; k < dOrder.size(); ++k) {
          const DiskIn& d = b->disks[dOrder[k]];
          if (d.brokerId == b->rBrokerId[r] && d.logdir == b->rLogdir[r]) b->oRDisk[r] = (int32_t)k;
        }
        if (b->oRDisk[r] < 0) throw std::invalid_argument("replica on an unknown logdir " + b->rLogdir[r]);
      }
    std::memset(out, 0, sizeof(*out));
    out->num_windows = b->W;
    out->num_racks = (int32_t)b->rackNames.size();
    out->num_brokers = B;
    out->broker_id = b->oBrokerId.data();
    out->broker_rack = b->oRack.data();
    out->broker_state = b->oState.data();
    out->broker_capacity = b->oCap.data();
    out->num_topics = (int32_t)b->topics.size();
    out->topic_names = b->oTopicNames.data();
    out->num_partitions = P;
    out->partition_topic = b->pTopic.data();
    out->partition_number = b->pNumber.data();
    out->partition_offset = b->pOff.data();
    out->partition_replicas = b->oPartReplicas.data();
    out->num_replicas = R;
    out->replica_partition = b->rPartition.data();
    out->replica_broker = b->oRBroker.data();
    out->replica_is_leader = b->rLeader.data();
    out->replica_offline = b->rOffline.data();
    out->replica_load = b->rLoad.data();
    out->replica_load_order = nullptr;
    out->num_disks = (int32_t)b->oDiskBroker.size();
    if (out->num_disks) {
      out->disk_broker = b->oDiskBroker.data();
      out->disk_logdir = b->oDiskLogdir.data();
      out->disk_capacity = b->oDiskCap.data();
      out->replica_disk = b->oRDisk.data();
      out->disk_demoted = b->oDiskDemoted.data();
    }
    out->broker_host = b->oHost.data();
  });
}

ccmi_status ccmi_builder_broker_ids(const ccmi_model_builder* b, int32_t* out) {
  if (!b || !out) return CCMI_E_INVALID;
  if (b->sortedIds.size() != b->brokers.size()) return CCMI_E_STATE;  // call ccmi_builder_desc first
  std::copy(b->sortedIds.begin(), b->sortedIds.end(), out);
  return CCMI_OK;
}

}  // extern "C"
