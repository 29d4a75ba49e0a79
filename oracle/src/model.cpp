// ORACLE — test infrastructure only (see jsem.h header). Restates the reference model mutations:
//   ClusterModel.createBroker/createReplica/setReplicaLoad  ClusterModel.java (createReplica :395-446)
//   ClusterModel.relocateReplica/removeReplica              ClusterModel.java:380-396,546-564
//   ClusterModel.relocateLeadership                         ClusterModel.java:409-441
//   Broker.addReplica/removeReplica/makeFollower/makeLeader Broker.java:336-510
//   Replica.makeFollower/computeCpuLoadAsFollower/makeLeader Replica.java:210-310
//   ModelUtils.getFollowerCpuUtilFromLeaderLoad             ModelUtils.java:64-80 (weights 0.7/0.15/0.15)
//   Disk.addReplica/removeReplica/addReplicaLoad, Broker.moveReplicaBetweenDisks/markDiskDead
//                                                           Disk.java:113-146, Broker.java:519-543
#include "model.h"

#include <chrono>

#include <algorithm>
#include <stdexcept>

namespace oracle {

const char* resourceName(int r) {
  static const char* n[] = {"CPU", "NW_IN", "NW_OUT", "DISK"};
  return n[r];
}

// ------------------------------------------------------------------ sorted replicas
SortedReplicas::SortedReplicas(const ClusterModel* cm, SortSpec s, int broker)
    : spec(std::move(s)), set(ReplicaCmp{cm, nullptr}), owner(broker) {
  // rebind comparator to our own (stable) spec storage
  set = std::set<int, ReplicaCmp>(ReplicaCmp{cm, &spec});
}

int ReplicaCmp::compare(int a, int b) const {
  for (PrioFn p : spec->priority) {
    int p1, p2;
    if (p == PrioFn::IMMIGRANTS) {
      p1 = cm->isImmigrant(a) ? 0 : 1;
      p2 = cm->isImmigrant(b) ? 0 : 1;
    } else if (p == PrioFn::DISK_IMMIGRANTS) {  // r.originalDisk() != r.disk() ? 0 : 1
      p1 = cm->replicas[a].origDisk != cm->replicas[a].disk ? 0 : 1;
      p2 = cm->replicas[b].origDisk != cm->replicas[b].disk ? 0 : 1;
    } else {
      p1 = cm->isCurrentOffline(a) ? 0 : 1;
      p2 = cm->isCurrentOffline(b) ? 0 : 1;
    }
    if (p1 != p2) return p1 < p2 ? -1 : 1;
  }
  if (spec->score != ScoreFn::NONE) {
    double s1 = (double)groupAvg(cm->replicas[a].load, spec->scoreResource, cm->W);
    double s2 = (double)groupAvg(cm->replicas[b].load, spec->scoreResource, cm->W);
    if (spec->score == ScoreFn::REVERSE_BY_GROUP) {
      s1 = -s1;
      s2 = -s2;
    }
    int c = dcompare(s1, s2);
    if (c != 0) return c;
  }
  return cm->replicaCompareTo(a, b);
}
int ClusterModel::replicaCompareTo(int a, int b) const {
  bool o1 = isCurrentOffline(a), o2 = isCurrentOffline(b);
  if (o1 && !o2) return -1;
  if (!o1 && o2) return 1;
  const Replica& ra = replicas[a];
  const Replica& rb = replicas[b];
  const Partition& pa = partitions[ra.partition];
  const Partition& pb = partitions[rb.partition];
  if (pa.number != pb.number) return pa.number > pb.number ? 1 : -1;
  int ida = brokers[ra.origBroker].id, idb = brokers[rb.origBroker].id;
  if (ida != idb) return ida > idb ? 1 : -1;
  if ((int)topicRank.size() != numTopics()) {  // before finalizeTopics: String.compareTo on the names
    const int c = topicNames[pa.topic].compare(topicNames[pb.topic]);
    return c == 0 ? 0 : (c < 0 ? -1 : 1);
  }
  int ta = topicRank[pa.topic], tb = topicRank[pb.topic];
  return ta == tb ? 0 : (ta < tb ? -1 : 1);
}
bool ReplicaCmp::operator()(int a, int b) const { return compare(a, b) < 0; }

bool ClusterModel::passesSelection(const SortSpec& spec, int r) const {
  const Replica& rep = replicas[r];
  for (const Selection& s : spec.selection) {
    bool ok = true;
    switch (s.fn) {
      case SelFn::LEADERS: ok = rep.isLeader; break;
      case SelFn::FOLLOWERS: ok = !rep.isLeader; break;
      case SelFn::ONLINE: ok = !isCurrentOffline(r); break;
      case SelFn::OFFLINE: ok = isCurrentOffline(r); break;
      case SelFn::IMMIGRANTS: ok = isImmigrant(r); break;
      case SelFn::IMMIGRANT_OR_OFFLINE: ok = isImmigrant(r) || isCurrentOffline(r); break;
      case SelFn::EXCLUDED_TOPICS:  // r.isOriginalOffline() || !excludedTopics.contains(topic)
        ok = isOriginalOffline(r) ||
             !(s.topics ? *s.topics : excludedTopicsSel).count(partitions[rep.partition].topic);
        break;
      case SelFn::INCLUDED_TOPICS:  // includedTopics.contains(topic) (ReplicaSortFunctionFactory.java:153-155)
        ok = s.topics->count(partitions[rep.partition].topic) > 0;
        break;
      case SelFn::ABOVE_LIMIT: ok = replicaUtil(r, s.resource) > s.limit; break;
      case SelFn::BELOW_LIMIT: ok = replicaUtil(r, s.resource) < s.limit; break;
    }
    if (!ok) return false;
  }
  return true;
}

int ClusterModel::numLeadersFor(int b, int topic) const {
  const auto it = brokers[b].topicLeaderCount.find(topic);
  return it == brokers[b].topicLeaderCount.end() ? 0 : it->second;
}

// Broker.trackSortedReplicas (Broker.java:398-408): the broker's own set and one per disk
void ClusterModel::trackSortedReplicas(int b, const std::string& name, const SortSpec& spec) {
  auto& m = brokers[b].sorted;
  if (m.find(name) == m.end()) m.emplace(name, std::make_unique<SortedReplicas>(this, spec, b));  // putIfAbsent
  for (int d : brokers[b].disks) {
    auto& dm = disks[d].sorted;
    if (dm.find(name) == dm.end()) {
      auto sr = std::make_unique<SortedReplicas>(this, spec, b);
      sr->disk = d;
      dm.emplace(name, std::move(sr));
    }
  }
}
void ClusterModel::untrackSortedReplicas(const std::string& name) {
  for (auto& br : brokers) br.sorted.erase(name);
  for (auto& dk : disks) dk.sorted.erase(name);
}
void ClusterModel::brokerUntrackSortedReplicas(int b, const std::string& name) {
  brokers[b].sorted.erase(name);
  for (int d : brokers[b].disks) disks[d].sorted.erase(name);
}
void ClusterModel::clearSortedReplicas() {
  for (auto& br : brokers) br.sorted.clear();
  for (auto& dk : disks) dk.sorted.clear();
}
void ClusterModel::brokerClearSortedReplicas(int b) {
  brokers[b].sorted.clear();
  for (int d : brokers[b].disks) disks[d].sorted.clear();
}
SortedReplicas& ClusterModel::trackedDiskSortedReplicas(int d, const std::string& name) {
  auto it = disks[d].sorted.find(name);
  if (it == disks[d].sorted.end()) throw std::runtime_error("The sort name " + name + " is not found.");
  SortedReplicas& sr = *it->second;
  if (!sr.initialized) {  // SortedReplicas.ensureInitialize: _disk.replicas().forEach(this::add)
    sr.initialized = true;
    for (int r : disks[d].replicas)
      if (passesSelection(sr.spec, r)) sr.set.insert(r);
  }
  return sr;
}
std::vector<int> ClusterModel::diskSortedReplicasClone(int d, const std::string& name) {
  const auto& s = trackedDiskSortedReplicas(d, name).set;
  return std::vector<int>(s.begin(), s.end());
}

SortedReplicas& ClusterModel::trackedSortedReplicas(int b, const std::string& name) {
  auto it = brokers[b].sorted.find(name);
  if (it == brokers[b].sorted.end()) throw std::runtime_error("The sort name " + name + " is not found.");
  SortedReplicas& sr = *it->second;
  if (!sr.initialized) {  // SortedReplicas.ensureInitialize
    sr.initialized = true;
    for (int r : brokers[b].replicas)
      if (passesSelection(sr.spec, r)) sr.set.insert(r);
  }
  return sr;
}
const std::set<int, ReplicaCmp>& ClusterModel::sortedReplicasView(int b, const std::string& name) {
  return trackedSortedReplicas(b, name).set;
}
std::vector<int> ClusterModel::sortedReplicasClone(int b, const std::string& name) {
  const auto& s = trackedSortedReplicas(b, name).set;
  return std::vector<int>(s.begin(), s.end());
}
void ClusterModel::sortedAdd(int b, int r) {
  for (auto& kv : brokers[b].sorted) {
    SortedReplicas& sr = *kv.second;
    if (sr.initialized && passesSelection(sr.spec, r)) sr.set.insert(r);
  }
}
void ClusterModel::sortedRemove(int b, int r) {
  for (auto& kv : brokers[b].sorted) {
    SortedReplicas& sr = *kv.second;
    if (sr.initialized) sr.set.erase(r);
  }
}

// ------------------------------------------------------------------ construction
int ClusterModel::createRack(const std::string& id) {
  for (size_t i = 0; i < racks.size(); ++i)
    if (racks[i].id == id) return (int)i;
  racks.push_back({id, {}});
  return (int)racks.size() - 1;
}
int ClusterModel::createBroker(int rackIdx, int brokerId, const double cap[NUM_RESOURCES], int host) {
  if (brokerId != (int)brokers.size()) throw std::runtime_error("oracle requires dense broker ids 0..B-1");
  // Rack.createBroker -> Rack._hosts.computeIfAbsent(hostName) -> Host.createBroker (Host.java: _aliveBrokers++,
  // _hostCapacity += the broker's capacity)
  if (host < 0) host = (int)hosts.size();
  if ((int)hosts.size() <= host) hosts.resize(host + 1);
  Host& h = hosts[host];
  h.brokers.push_back(brokerId);
  h.aliveBrokers++;
  for (int r = 0; r < NUM_RESOURCES; ++r) h.capacity[r] += cap[r];
  brokerHost.push_back(host);
  Broker b;
  b.id = brokerId;
  b.rack = rackIdx;
  b.replicaSet.setComparator([this](int x, int y) { return replicaCompareTo(x, y); });
  b.leaderSet.setComparator([this](int x, int y) { return replicaCompareTo(x, y); });
  b.offlineSet.setComparator([this](int x, int y) { return replicaCompareTo(x, y); });
  b.topicKeys.setComparator([this](int x, int y) { return topicNames[x].compare(topicNames[y]); });
  for (int r = 0; r < NUM_RESOURCES; ++r) b.capacity[r] = cap[r];
  brokers.push_back(std::move(b));
  potentialLeadershipLoad.emplace_back();
  racks[rackIdx].brokers.push_back(brokerId);
  refreshCapacity();
  return brokerId;
}
int ClusterModel::ensureTopic(const std::string& name) {
  for (int i = (int)topicNames.size() - 1; i >= 0; --i)
    if (topicNames[i] == name) return i;
  topicNames.push_back(name);
  topicHash.push_back(jStringHash(name));
  numReplicasByTopic.push_back(0);
  replicationFactorByTopic.push_back(0);
  return (int)topicNames.size() - 1;
}
void ClusterModel::finalizeTopics() {
  std::vector<int> idx(topicNames.size());
  for (size_t i = 0; i < idx.size(); ++i) idx[i] = (int)i;
  std::sort(idx.begin(), idx.end(), [&](int a, int b) { return topicNames[a] < topicNames[b]; });
  topicRank.assign(topicNames.size(), 0);
  for (size_t i = 0; i < idx.size(); ++i) topicRank[idx[i]] = (int)i;
}

int ClusterModel::createPartition(int topic, int number) {
  Partition part;
  part.topic = topic;
  part.number = number;
  partitions.push_back(std::move(part));
  if (replicationFactorByTopic[topic] == 0) replicationFactorByTopic[topic] = 1;  // putIfAbsent(topic, 1)
  return (int)partitions.size() - 1;
}

int ClusterModel::createReplica(int brokerIdx, int p, int index, bool isLeader, bool isOffline, int disk) {
  int topic = partitions[p].topic;
  Replica rep;
  rep.broker = brokerIdx;
  rep.origBroker = brokerIdx;
  rep.disk = rep.origDisk = disk;
  rep.isLeader = isLeader;
  rep.origOfflineFlag = isOffline;
  int r = (int)replicas.size();
  rep.partition = p;
  replicas.push_back(std::move(rep));
  brokerAddReplica(brokerIdx, r);  // rack.addReplica -> host.addReplica -> broker.addReplica
  numReplicasByTopic[topic] += 1;
  Partition& part = partitions[p];
  if (isLeader) {
    if (part.leader >= 0) throw std::runtime_error("Partition already has a leader");
    part.leader = r;
    part.replicas.insert(part.replicas.begin() + index, r);
    return r;
  }
  part.replicas.insert(part.replicas.begin() + index, r);
  if (part.leader >= 0) loadAddLoad(potentialLeadershipLoad[brokerIdx], replicas[part.leader].load, W);
  int followers = 0;
  for (int x : part.replicas)
    if (!replicas[x].isLeader) followers++;
  int rf = std::max(replicationFactorByTopic[topic], followers + 1);
  replicationFactorByTopic[topic] = rf;
  maxReplicationFactor = std::max(maxReplicationFactor, rf);
  return r;
}

void ClusterModel::setReplicaLoad(int r, const Load& amv) {
  Replica& rep = replicas[r];
  if (!rep.load.empty()) throw std::runtime_error("load already set");
  int b = rep.broker;
  // Broker.setReplicaLoad
  amvAdd(rep.load, amv, W);  // Load.initializeMetricValues
  if (rep.isLeader) amvAdd(brokers[b].leadershipLoadForNwResources, amv, W);
  amvAdd(brokers[b].load, amv, W);
  amvAdd(hosts[brokerHost[b]].load, amv, W);  // Host.setReplicaLoad: _load.addMetricValues (rack load unused)
  amvAdd(load, amv, W);  // cluster
  if (rep.disk >= 0) disks[rep.disk].utilization += replicaUtil(r, DISK);  // Disk.addReplicaLoad
  const Partition& part = partitions[rep.partition];
  if (part.leader >= 0 && replicas[part.leader].broker == b) {
    for (int x : part.replicas) amvAdd(potentialLeadershipLoad[replicas[x].broker], amv, W);
  }
}

void ClusterModel::refreshCapacity() {
  for (int r = 0; r < NUM_RESOURCES; ++r) {
    double c = 0;
    for (const Broker& b : brokers)
      if (b.isAlive()) c += b.capacity[r];
    clusterCapacity[r] = c;
  }
}

void ClusterModel::setBrokerState(int b, BrokerState s) {
  Broker& br = brokers[b];
  {  // Host.setBrokerState: the capacity of a broker that dies leaves the host's, before Broker.setState
    Host& h = hosts[brokerHost[b]];
    if (br.isAlive() && s == BrokerState::DEAD) {
      for (int k = 0; k < NUM_RESOURCES; ++k) h.capacity[k] -= br.capacity[k];
      h.aliveBrokers--;
    } else if (!br.isAlive() && s != BrokerState::DEAD) {
      for (int k = 0; k < NUM_RESOURCES; ++k) h.capacity[k] += br.capacity[k];
      h.aliveBrokers++;
    }
  }
  br.state = s;
  if (!br.isAlive()) {  // Broker.setState: _currentOfflineReplicas.addAll(replicas())
    for (int r : br.replicaSet.order()) br.offlineSet.add(r, replicaHash(r));
    for (int r : br.replicas) {
      if (!replicas[r].inBrokerOffline) {
        replicas[r].inBrokerOffline = true;
        br.numOffline++;
      }
    }
    for (int k = 0; k < NUM_RESOURCES; ++k) br.capacity[k] = -1.0;
    for (int d : br.disks) {  // Disk.setState(DEAD)
      disks[d].alive = false;
      disks[d].capacity = -1.0;
    }
  }
  for (int r : br.replicas)
    if (replicas[r].inBrokerOffline) selfHealingEligibleReplicas.insert(r);
  refreshCapacity();
  switch (s) {
    case BrokerState::DEAD:
      deadBrokers.insert(b);
      brokersWithBadDisks.erase(b);
      break;
    case BrokerState::NEW:
      newBrokers.insert(b);
      deadBrokers.erase(b);
      brokersWithBadDisks.erase(b);
      break;
    case BrokerState::DEMOTED:
    case BrokerState::ALIVE:
      deadBrokers.erase(b);
      brokersWithBadDisks.erase(b);
      break;
    case BrokerState::BAD_DISKS:
      deadBrokers.erase(b);
      brokersWithBadDisks.insert(b);
      for (int r : br.replicas)
        if (replicas[r].inBrokerOffline) partitions[replicas[r].partition].ineligibleBrokers.insert(b);
      break;
  }
}

// ------------------------------------------------------------------ queries
int ClusterModel::replicaOnBroker(int partition, int b) const {
  for (int r : partitions[partition].replicas)
    if (replicas[r].broker == b) return r;
  return -1;
}
std::vector<int> ClusterModel::aliveBrokers() const {
  std::vector<int> out;
  out.reserve(brokers.size());
  for (size_t i = 0; i < brokers.size(); ++i)
    if (brokers[i].isAlive()) out.push_back((int)i);
  return out;
}
std::vector<int> ClusterModel::aliveBrokersUnderThreshold(int res, double thr) const {
  std::vector<int> out;
  for (size_t i = 0; i < brokers.size(); ++i) {
    const Broker& b = brokers[i];
    if (!b.isAlive()) continue;
    if (isBrokerResource(res)) {
      double lim = b.capacity[res] * thr;
      if (brokerUtil((int)i, res) >= lim) continue;
    }
    if (isHostResource(res)) {
      double lim = hostCapacity((int)i, res) * thr;
      if (hostUtil((int)i, res) >= lim) continue;
    }
    out.push_back((int)i);
  }
  return out;
}
std::vector<int> ClusterModel::aliveBrokersOverThreshold(int res, double thr) const {
  std::vector<int> out;
  for (size_t i = 0; i < brokers.size(); ++i) {
    const Broker& b = brokers[i];
    if (!b.isAlive()) continue;
    if (isBrokerResource(res)) {
      double lim = b.capacity[res] * thr;
      if (brokerUtil((int)i, res) <= lim) continue;
    }
    if (isHostResource(res)) {
      double lim = hostCapacity((int)i, res) * thr;
      if (hostUtil((int)i, res) <= lim) continue;
    }
    out.push_back((int)i);
  }
  return out;
}
double ClusterModel::capacityWithAllowedReplicaMovesFor(int res, const OptimizationOptions& o) const {
  double drop = 0.0;  // DoubleStream.sum over alive excluded brokers
  JDoubleSum s;
  for (size_t i = 0; i < brokers.size(); ++i)
    if (brokers[i].isAlive() && o.excludedBrokersForReplicaMove.count(brokers[i].id)) s.add(brokers[i].capacity[res]);
  drop = s.result();
  return clusterCapacity[res] - drop;
}
std::vector<int> ClusterModel::onlineFollowerBrokers(int p) const {
  std::vector<int> out;
  for (int r : partitions[p].replicas)
    if (!replicas[r].isLeader && !isCurrentOffline(r)) out.push_back(replicas[r].broker);
  return out;
}

std::vector<int> ClusterModel::replicaDistributionFlat() const {
  std::vector<int> out;
  for (const Partition& p : partitions)
    for (int r : p.replicas) out.push_back(replicas[r].broker);
  return out;
}
std::vector<int> ClusterModel::leaderDistribution() const {
  std::vector<int> out;
  out.reserve(partitions.size());
  for (const Partition& p : partitions) out.push_back(replicas[p.leader].broker);
  return out;
}

// ------------------------------------------------------------------ broker mutations
void ClusterModel::brokerAddReplica(int b, int r) {
  Broker& br = brokers[b];
  Replica& rep = replicas[r];
  rep.posInBroker = (int)br.replicas.size();
  br.replicas.push_back(r);
  br.replicaSet.add(r, replicaHash(r));
  br.topicKeys.add(partitions[rep.partition].topic, topicHash[partitions[rep.partition].topic]);
  rep.inBrokerImmigrants = rep.inBrokerOffline = rep.inBrokerLeaders = false;
  if (brokers[rep.origBroker].id != br.id) {
    rep.inBrokerImmigrants = true;
    br.numImmigrants++;
  } else if (isOriginalOffline(r)) {
    rep.inBrokerOffline = true;
    br.numOffline++;
    br.offlineSet.add(r, replicaHash(r));
  }
  br.topicReplicaCount[partitions[rep.partition].topic] += 1;
  if (rep.isLeader) {
    br.topicLeaderCount[partitions[rep.partition].topic] += 1;
    loadAddLoad(br.leadershipLoadForNwResources, rep.load, W);
    rep.inBrokerLeaders = true;
    br.numLeaders++;
    br.leaderSet.add(r, replicaHash(r));
  }
  loadAddLoad(br.load, rep.load, W);
  {  // Host.addReplica: _replicas.add, _load.addLoad(replica.load())
    Host& h = hosts[brokerHost[b]];
    h.numReplicas++;
    loadAddLoad(h.load, rep.load, W);
  }
  sortedAdd(b, r);
  if (rep.disk >= 0) {  // _diskByLogdir.get(replica.disk().logDir()).addReplica(replica)
    const int dd = diskOf(b, disks[rep.disk].logdir);
    if (dd < 0) throw std::runtime_error("NullPointerException: broker " + std::to_string(br.id) + " has no logdir " +
                                         disks[rep.disk].logdir);
    diskAddReplica(dd, r);
  }
}

int ClusterModel::brokerRemoveReplica(int b, int partition) {
  int r = replicaOnBroker(partition, b);
  if (r < 0) return -1;
  Broker& br = brokers[b];
  Replica& rep = replicas[r];
  // _replicas.remove (swap-remove keeps O(1); HashSet order is not semantically used)
  int pos = rep.posInBroker;
  int last = br.replicas.back();
  br.replicas[pos] = last;
  replicas[last].posInBroker = pos;
  br.replicas.pop_back();
  rep.posInBroker = -1;
  br.replicaSet.remove(r, replicaHash(r));
  br.offlineSet.remove(r, replicaHash(r));
  loadSubLoad(br.load, rep.load, W);
  {  // Host.removeReplica: _replicas.remove, _load.subtractLoad(replica.load())
    Host& h = hosts[brokerHost[b]];
    h.numReplicas--;
    loadSubLoad(h.load, rep.load, W);
  }
  br.topicReplicaCount[partitions[partition].topic] -= 1;
  if (rep.isLeader) {
    br.topicLeaderCount[partitions[partition].topic] -= 1;
    loadSubLoad(br.leadershipLoadForNwResources, rep.load, W);
    if (rep.inBrokerLeaders) br.numLeaders--;
    br.leaderSet.remove(r, replicaHash(r));
  }
  rep.inBrokerLeaders = false;
  if (rep.inBrokerImmigrants) br.numImmigrants--;
  if (rep.inBrokerOffline) br.numOffline--;
  rep.inBrokerImmigrants = rep.inBrokerOffline = false;
  sortedRemove(b, r);
  return r;
}

Load ClusterModel::replicaMakeFollower(int r) {
  Replica& rep = replicas[r];
  if (!rep.isLeader) throw std::runtime_error("makeFollower on non-leader");
  Load& L = rep.load;
  Load delta;
  // computeCpuLoadAsFollower
  MV chg;
  mvZero(chg, W);
  MV totOut, totIn;
  mvZero(totOut, W);
  mvAdd(totOut, L.m[M_LBO], W);
  mvAdd(totOut, L.m[M_RBO], W);
  mvZero(totIn, W);
  mvAdd(totIn, L.m[M_LBI], W);
  mvAdd(totIn, L.m[M_RBI], W);
  MV& cpu = L.m[M_CPU];
  for (int i = 0; i < W; ++i) {
    double in = (double)totIn.v[i], out = (double)totOut.v[i], c = (double)cpu.v[i];
    double newCpu;
    if (in == 0.0 && out == 0.0) newCpu = 0.0;
    else newCpu = c * (0.15 * in) / (0.7 * in + 0.15 * out);
    mvSet(chg, i, (double)cpu.v[i] - newCpu);
    mvSet(cpu, i, newCpu);
  }
  // leadershipLoadDelta.add(cpuMetricId, cpuLoadChange); leadershipLoadDelta.add(nwOutLoad)
  delta.mask = (uint8_t)((1u << M_CPU) | (1u << M_LBO) | (1u << M_RBO));
  mvZero(delta.m[M_CPU], W);
  mvAdd(delta.m[M_CPU], chg, W);
  mvZero(delta.m[M_LBO], W);
  mvAdd(delta.m[M_LBO], L.m[M_LBO], W);
  mvZero(delta.m[M_RBO], W);
  mvAdd(delta.m[M_RBO], L.m[M_RBO], W);
  // clearLoadFor(NW_OUT)
  mvZero(L.m[M_LBO], W);
  mvZero(L.m[M_RBO], W);
  rep.isLeader = false;
  return delta;
}

Load ClusterModel::brokerMakeFollower(int b, int partition) {
  int r = replicaOnBroker(partition, b);
  Broker& br = brokers[b];
  loadSubLoad(br.leadershipLoadForNwResources, replicas[r].load, W);
  sortedRemove(b, r);
  Load delta = replicaMakeFollower(r);
  br.topicLeaderCount[partitions[partition].topic] -= 1;
  loadSubDelta(br.load, delta, W);
  loadSubDelta(hosts[brokerHost[b]].load, delta, W);  // Host.makeFollower: _load.subtractLoad(leadershipLoadDelta)
  if (replicas[r].inBrokerLeaders) {
    replicas[r].inBrokerLeaders = false;
    br.numLeaders--;
  }
  br.leaderSet.remove(r, replicaHash(r));
  sortedAdd(b, r);
  return delta;
}

void ClusterModel::brokerMakeLeader(int b, int partition, const Load& delta) {
  int r = replicaOnBroker(partition, b);
  Broker& br = brokers[b];
  sortedRemove(b, r);
  if (!replicas[r].isLeader) br.topicLeaderCount[partitions[partition].topic] += 1;
  replicas[r].isLeader = true;
  loadAddDelta(replicas[r].load, delta, W);
  loadAddLoad(br.leadershipLoadForNwResources, replicas[r].load, W);
  loadAddDelta(br.load, delta, W);
  loadAddDelta(hosts[brokerHost[b]].load, delta, W);  // Host.makeLeader: _load.addLoad(leadershipLoadDelta)
  if (!replicas[r].inBrokerLeaders) {
    replicas[r].inBrokerLeaders = true;
    br.numLeaders++;
  }
  br.leaderSet.add(r, replicaHash(r));
  sortedAdd(b, r);
}

std::vector<int> ClusterModel::partitionBrokersSet(int p) const {
  JHashSet set;
  for (int r : partitions[p].replicas) set.add(replicas[r].broker, brokers[replicas[r].broker].id);
  return set.order();
}

// ------------------------------------------------------------------ cluster mutations
void ClusterModel::relocateReplica(int p, int src, int dst) {
  int r = brokerRemoveReplica(src, p);
  if (r < 0) throw std::runtime_error("Replica is not in the cluster.");
  int topic = partitions[p].topic;
  numReplicasByTopic[topic] -= 1;
  loadSubLoad(load, replicas[r].load, W);
  loadSubLoad(potentialLeadershipLoad[src], replicas[partitions[p].leader].load, W);
  replicas[r].broker = dst;
  brokerAddReplica(dst, r);
  numReplicasByTopic[topic] += 1;
  loadAddLoad(load, replicas[r].load, W);
  loadAddLoad(potentialLeadershipLoad[dst], replicas[partitions[p].leader].load, W);
  if (recordActions) actionLog.push_back({(int)ActionType::INTER_BROKER_REPLICA_MOVEMENT, p, src, dst, -1});
}

void ClusterModel::moveReplicaToEnd(int r) {
  std::vector<int>& v = partitions[replicas[r].partition].replicas;
  auto it = std::find(v.begin(), v.end(), r);
  if (it == v.end()) throw std::logic_error("Did not find replica for partition.");
  v.erase(it);
  v.push_back(r);
}

bool ClusterModel::relocateLeadership(int p, int src, int dst) {
  int sr = replicaOnBroker(p, src);
  if (!replicas[sr].isLeader) return false;
  int dr = replicaOnBroker(p, dst);
  if (replicas[dr].isLeader)  // IllegalArgumentException (ClusterModel.java:415-421)
    throw std::invalid_argument("Cannot relocate leadership of partition " + topicNames[partitions[p].topic] + "-" +
                                std::to_string(partitions[p].number) + "from broker " + std::to_string(brokers[src].id) +
                                " to broker " + std::to_string(brokers[dst].id) +
                                " because the destination replica is a leader.");
  Load delta = brokerMakeFollower(src, p);
  brokerMakeLeader(dst, p, delta);
  Partition& part = partitions[p];
  int pos = (int)(std::find(part.replicas.begin(), part.replicas.end(), dr) - part.replicas.begin());
  std::swap(part.replicas[0], part.replicas[pos]);
  part.leader = dr;
  if (recordActions) actionLog.push_back({(int)ActionType::LEADERSHIP_MOVEMENT, p, src, dst, -1});
  return true;
}

// ------------------------------------------------------------------ disks
int ClusterModel::createDisk(int b, const std::string& logdir, double capacity) {
  Disk dk;
  dk.broker = b;
  dk.logdir = logdir;
  dk.replicaSet.setComparator([this](int x, int y) { return replicaCompareTo(x, y); });
  if (capacity < 0) {  // Disk(logDir, broker, diskCapacity): negative capacity = dead disk
    dk.capacity = -1.0;
    dk.alive = false;
  } else {
    dk.capacity = capacity;
  }
  if (!brokers[b].isAlive()) {
    dk.capacity = -1.0;
    dk.alive = false;
  }
  const int d = (int)disks.size();
  disks.push_back(std::move(dk));
  auto& lst = brokers[b].disks;  // TreeMap<String, Disk>: String.compareTo order
  auto it = lst.begin();
  while (it != lst.end() && disks[*it].logdir < logdir) ++it;
  if (it != lst.end() && disks[*it].logdir == logdir) throw std::invalid_argument("duplicate logdir " + logdir);
  lst.insert(it, d);
  return d;
}
int ClusterModel::diskOf(int b, const std::string& logdir) const {
  for (int d : brokers[b].disks)
    if (disks[d].logdir == logdir) return d;
  return -1;
}
void ClusterModel::diskAddReplica(int d, int r) {
  Disk& dk = disks[d];
  if (dk.replicas.count(r)) throw std::logic_error("Disk " + dk.logdir + " already has replica " + topicNames[partitions[replicas[r].partition].topic] +
                                               "-" + std::to_string(partitions[replicas[r].partition].number));
  dk.utilization += replicaUtil(r, DISK);
  dk.replicas.insert(r);
  dk.replicaSet.add(r, replicaHash(r));
  replicas[r].disk = d;
  for (auto& kv : dk.sorted) {
    SortedReplicas& sr = *kv.second;
    if (sr.initialized && passesSelection(sr.spec, r)) sr.set.insert(r);
  }
}
void ClusterModel::diskRemoveReplica(int d, int r) {
  Disk& dk = disks[d];
  if (!dk.replicas.count(r)) throw std::logic_error("Disk " + dk.logdir + " does not has replica " + topicNames[partitions[replicas[r].partition].topic] +
                                               "-" + std::to_string(partitions[replicas[r].partition].number));
  dk.utilization -= replicaUtil(r, DISK);
  dk.replicas.erase(r);
  dk.replicaSet.remove(r, replicaHash(r));
  for (auto& kv : dk.sorted) {
    SortedReplicas& sr = *kv.second;
    if (sr.initialized) sr.set.erase(r);
  }
}
// Replica.markOriginalOffline (Replica.java:91-97)
void ClusterModel::markReplicaOriginalOffline(int r) {
  Replica& rep = replicas[r];
  if (rep.broker != rep.origBroker) throw std::logic_error("Cannot mark an immigrant replica as offline.");
  rep.origOfflineFlag = true;
  if (!rep.inBrokerOffline) {
    rep.inBrokerOffline = true;
    brokers[rep.origBroker].numOffline++;
    brokers[rep.origBroker].offlineSet.add(r, replicaHash(r));
  }
}
void ClusterModel::markDiskDead(int b, int d) {
  Broker& br = brokers[b];
  hosts[brokerHost[b]].capacity[DISK] -= disks[d].capacity;  // Host.markDiskDead
  br.capacity[DISK] -= disks[d].capacity;
  disks[d].alive = false;
  disks[d].capacity = -1.0;
  for (int r : disks[d].replicas) {  // Replica.markOriginalOffline
    Replica& rep = replicas[r];
    if (rep.broker != rep.origBroker) throw std::logic_error("Cannot mark an immigrant replica as offline.");
    rep.origOfflineFlag = true;
    if (!rep.inBrokerOffline) {
      rep.inBrokerOffline = true;
      brokers[rep.origBroker].numOffline++;
      brokers[rep.origBroker].offlineSet.add(r, replicaHash(r));
    }
  }
  for (int r : br.replicas)
    if (replicas[r].inBrokerOffline) selfHealingEligibleReplicas.insert(r);
  refreshCapacity();
}
double ClusterModel::averageDiskUtilizationPct(int b) const {
  double cap = 0, util = 0;
  for (int d : brokers[b].disks)
    if (disks[d].alive) {
      cap += disks[d].capacity;
      util += disks[d].utilization;
    }
  return cap > 0 ? util / cap : 1.0;
}
std::vector<int> ClusterModel::replicaDiskFlat() const {
  std::vector<int> out;
  for (const Partition& p : partitions)
    for (int r : p.replicas) out.push_back(replicas[r].disk);
  return out;
}
void ClusterModel::relocateReplicaToDisk(int p, int b, int dst) {
  const int r = replicaOnBroker(p, b);
  if (r < 0) throw std::runtime_error("Replica is not in the cluster.");
  const int src = diskOf(b, disks[replicas[r].disk].logdir);  // Broker.moveReplicaBetweenDisks
  if (src < 0 || disks[dst].broker != b) throw std::runtime_error("NullPointerException: logdir not on broker");
  diskRemoveReplica(src, r);
  diskAddReplica(dst, r);
  if (recordActions)
    actionLog.push_back({(int)ActionType::INTRA_BROKER_REPLICA_MOVEMENT, p, b, b, -1, src, dst});
}

void ClusterModel::checkDeadline() const {
  const double now = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  if (now > deadline) throw DeadlineReached();
}

}  // namespace oracle
