// Host model: build from the flattened desc, exact mutations, sorted-replica tracking, dirty rows.
#include "model.h"

#include <algorithm>
#include <cstring>
#include <stdexcept>

#include "device.h"
#include "hostpool.h"
#include "prof.h"

namespace ccmi {

// Replica.compareTo (Replica.java:349-377): offline first, then partition number, original broker id, topic
int ReplicaOrder::cmp(int a, int b) const {
  const bool oa = m->curOffline(a), ob = m->curOffline(b);
  if (oa != ob) return oa ? -1 : 1;
  const int na = m->pNumber[m->rPart[a]], nb = m->pNumber[m->rPart[b]];
  if (na != nb) return na > nb ? 1 : -1;
  const int ia = m->bId[m->rOrig[a]], ib = m->bId[m->rOrig[b]];
  if (ia != ib) return ia > ib ? 1 : -1;
  const int ta = m->topicRank[m->pTopic[m->rPart[a]]], tb = m->topicRank[m->pTopic[m->rPart[b]]];
  return ta == tb ? 0 : (ta < tb ? -1 : 1);
}
int TopicOrder::cmp(int a, int b) const {  // String.compareTo sign
  const int ra = m->topicRank[a], rb = m->topicRank[b];
  return ra == rb ? 0 : (ra < rb ? -1 : 1);
}

void Model::build(const ccmi_cluster_desc& d) {
  if (d.num_windows < 1 || d.num_windows > kMaxW) throw std::invalid_argument("num_windows must be in [1,5]");
  W = d.num_windows;
  ops = LoadOps(W);
  B = d.num_brokers;
  R = d.num_replicas;
  P = d.num_partitions;
  T = d.num_topics;
  bState.assign(B, BState::ALIVE);
  bRack.assign(d.broker_rack, d.broker_rack + B);
  for (int b = 0; b < B; ++b)
    if (bRack[b] < 0 || bRack[b] > 32767) throw std::invalid_argument("broker rack index must be in [0, 32767]");
  bId.assign(B, 0);
  for (int b = 0; b < B; ++b) {
    bId[b] = d.broker_id[b];
    if (bId[b] != b) throw std::invalid_argument("ABI v1 requires broker_id[b] == b");
  }
  bCap.assign(d.broker_capacity, d.broker_capacity + 4 * (size_t)B);
  // hosts: Rack._hosts.computeIfAbsent(name) with the brokers created in index order; Host.createBroker adds each
  // broker's capacity and counts it alive (Host.java)
  sharedHosts = false;
  bHost.assign(B, 0);
  {
    std::vector<int32_t> dense(d.broker_host ? (size_t)B : 0, -1), hostRack;
    H = 0;
    for (int b = 0; b < B; ++b) {
      int h;
      if (d.broker_host) {
        const int x = d.broker_host[b];
        if (x < 0 || x >= B) throw std::invalid_argument("broker_host out of range");
        if (dense[x] < 0) {
          dense[x] = H++;
          hostRack.push_back(bRack[b]);
        } else {
          if (hostRack[dense[x]] != bRack[b]) throw std::invalid_argument("brokers of one host in different racks");
          sharedHosts = true;
        }
        h = dense[x];
      } else {
        h = H++;
      }
      bHost[b] = h;
    }
    hBrokers.assign(H, {});
    hCap.assign((size_t)4 * H, 0.0);
    hAlive.assign(H, 0);
    hNrep.assign(H, 0);
    for (int b = 0; b < B; ++b) {
      const int h = bHost[b];
      hBrokers[h].push_back(b);
      hAlive[h]++;
      for (int k = 0; k < 4; ++k) hCap[4 * (size_t)h + k] += bCap[4 * (size_t)b + k];
    }
    hLoad.assign(sharedHosts ? H : 0, LoadVec());
    hUtilC.assign(sharedHosts ? (size_t)4 * H : 0, 0.0);
  }
  bRepl.assign(B, {});
  bNlead.assign(B, 0);
  bNimm.assign(B, 0);
  bNoff.assign(B, 0);
  bLoad.assign(B, LoadVec());
  bLnw.assign(B, LoadVec());
  bPot.assign(B, LoadVec());
  rPart.assign(d.replica_partition, d.replica_partition + R);
  rBroker.assign(d.replica_broker, d.replica_broker + R);
  rOrig = rBroker;
  rPos.assign(R, -1);
  rLeader.assign(d.replica_is_leader, d.replica_is_leader + R);
  rOrigOff.assign(d.replica_offline, d.replica_offline + R);
  rInImm.assign(R, 0);
  rInOff.assign(R, 0);
  rLoad.assign(R, LoadVec());
  pTopic.assign(d.partition_topic, d.partition_topic + P);
  pNumber.assign(d.partition_number, d.partition_number + P);
  pOff.assign(d.partition_offset, d.partition_offset + P + 1);
  pSlots.assign(d.partition_replicas, d.partition_replicas + R);
  pLeader.assign(P, -1);
  topicNames.clear();
  topicHash.assign(T, 0);
  for (int t = 0; t < T; ++t) {
    topicNames.emplace_back(d.topic_names[t]);
    topicHash[t] = jStringHash(d.topic_names[t]);
  }
  bReplicaSet.assign(B, ReplicaSet(&replicaOrder));
  bLeaderSet.assign(B, ReplicaSet(&replicaOrder));
  bOfflineSet.assign(B, ReplicaSet(&replicaOrder));
  bTopicKeys.assign(B, TopicSet(&topicOrder));
  {
    std::vector<int> idx(T);
    for (int t = 0; t < T; ++t) idx[t] = t;
    std::sort(idx.begin(), idx.end(), [&](int a, int b) { return topicNames[a] < topicNames[b]; });
    topicRank.assign(T, 0);
    for (int i = 0; i < T; ++i) topicRank[idx[i]] = i;
  }
  if (R >= (1 << 29)) throw std::invalid_argument("more than 2^29 replicas are not supported");
  topicNrep.assign(T, 0);
  selfHealing.assign(R, 0);
  tracked.assign(B, {});
  for (int p = 0; p < P; ++p)
    for (int i = pOff[p]; i < pOff[p + 1]; ++i) {
      const int r = pSlots[i];
      if (r < 0 || r >= R || rPart[r] != p) throw std::invalid_argument("partition CSR inconsistent with replica_partition");
    }
  // Replay createReplica + setReplicaLoad in replica index order (or: every createReplica, then setReplicaLoad in
  // replica_load_order).
  const int32_t* loadOrder = d.replica_load_order;
  const int nLoads = loadOrder && d.num_replica_loads > 0 ? d.num_replica_loads : R;
  if (loadOrder) {
    if (nLoads > R) throw std::invalid_argument("num_replica_loads above num_replicas");
    std::vector<uint8_t> seen(R, 0);
    for (int i = 0; i < nLoads; ++i) {
      if (loadOrder[i] < 0 || loadOrder[i] >= R || seen[loadOrder[i]])
        throw std::invalid_argument("replica_load_order repeats a replica or is out of range");
      seen[loadOrder[i]] = 1;
    }
  }
  std::vector<std::vector<int32_t>> created(P);
  auto setLoad = [&](int r) {  // ClusterModel.setReplicaLoad (ClusterModel.java:738-760)
    const int p = rPart[r], b = rBroker[r];
    LoadVec amv;
    amv.mask = 0x3F;
    for (int k = 0; k < 6; ++k) {
      ops.zero(amv.m[k]);
      for (int w = 0; w < W; ++w) {
        amv.m[k].v[w] = d.replica_load[((size_t)r * 6 + k) * W + w];
        amv.m[k].sum += (double)amv.m[k].v[w];
      }
    }
    ops.addAll(rLoad[r], amv);
    if (rLeader[r]) ops.addAll(bLnw[b], amv);
    ops.addAll(bLoad[b], amv);
    if (sharedHosts) ops.addAll(hLoad[bHost[b]], amv);  // Host.setReplicaLoad: _load.addMetricValues
    ops.addAll(cLoad, amv);
    if (pLeader[p] >= 0 && rBroker[pLeader[p]] == b)
      for (int x : created[p]) ops.addAll(bPot[rBroker[x]], amv);
  };
  for (int r = 0; r < R; ++r) {  // ClusterModel.createReplica (ClusterModel.java:822-880)
    const int p = rPart[r], b = rBroker[r];
    if (b < 0 || b >= B) throw std::invalid_argument("replica broker out of range");
    brokerAdd(b, r);  // load still empty: only sets/counters change
    topicNrep[pTopic[p]]++;
    if (rLeader[r]) {
      if (pLeader[p] >= 0) throw std::invalid_argument("partition has two leaders");
      pLeader[p] = r;
    } else if (pLeader[p] >= 0) {
      ops.addAll(bPot[b], rLoad[pLeader[p]]);
    }
    created[p].push_back(r);
    if ((int)created[p].size() > maxRf) maxRf = (int)created[p].size();
    if (!loadOrder) setLoad(r);
  }
  if (loadOrder)
    for (int i = 0; i < nLoads; ++i) setLoad(loadOrder[i]);
  if (maxRf > kMaxRf) throw std::invalid_argument("replication factor above 8 is not supported");
  for (int p = 0; p < P; ++p)
    if (pLeader[p] < 0) throw std::invalid_argument("partition without leader");
  // broker states (ClusterModel.setBrokerState)
  for (int b = 0; b < B; ++b) {
    const BState s = (BState)d.broker_state[b];
    if (s == BState::ALIVE) continue;
    if (s < BState::ALIVE || s > BState::BAD_DISKS) throw std::invalid_argument("unknown broker state");
    bState[b] = s;
    if (s == BState::BAD_DISKS) numBadDisk++;
    if (s == BState::DEAD) {
      numDead++;
      for (int r : bRepl[b])
        if (!rInOff[r]) {
          rInOff[r] = 1;
          bNoff[b]++;
        }
      // Broker.setState(DEAD): _currentOfflineReplicas.addAll(_replicas)
      std::vector<int32_t> order;
      bReplicaSet[b].order(order);
      for (int r : order) bOfflineSet[b].add(r, replicaHash(r));
      {  // Host.setBrokerState: a dying broker's capacity leaves its host before Broker.setState sets it to -1
        const int h = bHost[b];
        for (int k = 0; k < 4; ++k) hCap[4 * (size_t)h + k] -= bCap[4 * b + k];
        hAlive[h]--;
      }
      for (int k = 0; k < 4; ++k) bCap[4 * b + k] = -1.0;
    }
    if (s == BState::NEW) numNew++;
    for (int r : bRepl[b])
      if (rInOff[r] && !selfHealing[r]) {
        selfHealing[r] = 1;
        numSelfHealing++;
      }
  }
  {
    std::vector<std::vector<int32_t>> inel(P);
    for (int b = 0; b < B; ++b)
      if (bState[b] == BState::BAD_DISKS)
        for (int r : bRepl[b]) {
          auto& v = inel[rPart[r]];
          if (rInOff[r] && std::find(v.begin(), v.end(), b) == v.end()) v.push_back(b);
        }
    pIneligOff.assign(P + 1, 0);
    pIneligB.clear();
    for (int p = 0; p < P; ++p) {
      pIneligB.insert(pIneligB.end(), inel[p].begin(), inel[p].end());
      pIneligOff[p + 1] = (int32_t)pIneligB.size();
    }
  }
  for (int k = 0; k < 4; ++k) {
    double c = 0;
    for (int b = 0; b < B; ++b)
      if (alive(b)) c += bCap[4 * b + k];
    clusterCap[k] = c;
  }
  bVer.assign(B, 0);
  bDelta.assign(B, {});
  sortedCache.assign(B, {});
  filteredCache.assign(B, {});
  exclTopicSel.assign(T, 0);
  mustTopicSel.assign(T, 0);
  bUtilC.assign((size_t)4 * B, 0.0);
  bPctC.assign((size_t)4 * B, 0.0);
  rUtilC.assign((size_t)4 * R, 0.0);
  rScoreC.assign((size_t)4 * R, 0.f);
  for (int b = 0; b < B; ++b) refreshBroker(b);
  if (sharedHosts)
    for (int h = 0; h < H; ++h)
      for (int k = 0; k < 4; ++k) hUtilC[4 * (size_t)h + k] = ops.util(hLoad[h], k);
  for (int r = 0; r < R; ++r) refreshReplica(r);
  buildDisks(d);
  {
    // dense rank of the static tail of Replica.compareTo (partition number, original broker id, topic name)
    std::vector<int32_t> idx(R);
    for (int r = 0; r < R; ++r) idx[r] = r;
    auto tail = [&](int a, int b) {
      const int na = pNumber[rPart[a]], nb = pNumber[rPart[b]];
      if (na != nb) return na > nb ? 1 : -1;
      const int ia = bId[rOrig[a]], ib = bId[rOrig[b]];
      if (ia != ib) return ia > ib ? 1 : -1;
      const int ta = topicRank[pTopic[rPart[a]]], tb = topicRank[pTopic[rPart[b]]];
      return ta == tb ? 0 : (ta < tb ? -1 : 1);
    };
    std::sort(idx.begin(), idx.end(), [&](int a, int b) { return tail(a, b) < 0; });
    rStatic.assign(R, 0);
    for (int i = 1; i < R; ++i) rStatic[idx[i]] = rStatic[idx[i - 1]] + (tail(idx[i - 1], idx[i]) != 0);
  }
  ldB = (B + 3) & ~3;
  topicCountDense.assign((size_t)T * ldB, 0);
  for (int r = 0; r < R; ++r) topicCountDense[(size_t)pTopic[rPart[r]] * ldB + rBroker[r]]++;
  bDirty.assign(B, 0);
  rDirty.assign(R, 0);
  pDirty.assign(P, 0);
  cDirtyB.assign(B, 0);
  cDirtyR.assign(R, 0);
  cDirtyP.assign(P, 0);
  cDirtyH.assign(sharedHosts ? H : 0, 0);
}

// Disks (ccmi.h desc fields): created with their broker, logdir order per broker, replica_disk given to
// createReplica (utilization accumulates when the load is set: Disk.addReplicaLoad), then the disk_assign replay of
// Disk.addReplica (the fixture's placement step).
void Model::buildDisks(const ccmi_cluster_desc& d) {
  D = d.num_disks;
  if (D < 0) throw std::invalid_argument("num_disks < 0");
  dBroker.assign(D, 0);
  dLogdir.assign(D, std::string());
  dCap.assign(D, 0.0);
  dUtil.assign(D, 0.0);
  dAlive.assign(D, 1);
  dMembers.assign(D, {});
  rDisk.assign(R, -1);
  rOrigDisk.assign(R, -1);
  rDiskPos.assign(R, -1);
  std::vector<std::vector<int32_t>> per(B);
  for (int k = 0; k < D; ++k) {
    const int b = d.disk_broker[k];
    if (b < 0 || b >= B) throw std::invalid_argument("disk broker out of range");
    dBroker[k] = b;
    dLogdir[k] = d.disk_logdir[k] ? d.disk_logdir[k] : "";
    const double c = d.disk_capacity[k];
    dCap[k] = c < 0 ? -1.0 : c;  // Disk(logDir, broker, capacity): negative = dead
    dAlive[k] = c < 0 ? 0 : 1;
    per[b].push_back(k);
  }
  bDiskOff.assign(B + 1, 0);
  bDisks.clear();
  for (int b = 0; b < B; ++b) {
    auto& v = per[b];
    std::sort(v.begin(), v.end(), [&](int x, int y) { return dLogdir[x] < dLogdir[y]; });  // String.compareTo (ASCII)
    for (size_t i = 1; i < v.size(); ++i)
      if (dLogdir[v[i]] == dLogdir[v[i - 1]]) throw std::invalid_argument("duplicate logdir on a broker");
    if ((int)v.size() > kMaxDisksPerBroker) throw std::invalid_argument("more than 31 logdirs on a broker");
    bDiskOff[b] = (int)bDisks.size();
    bDisks.insert(bDisks.end(), v.begin(), v.end());
  }
  bDiskOff[B] = (int)bDisks.size();
  dDemoted.assign(D, 0);
  anyDemotedDisk = false;
  dReplicaSet.clear();
  if (d.disk_demoted)
    for (int k = 0; k < D; ++k)
      if (d.disk_demoted[k]) dDemoted[k] = 1, anyDemotedDisk = true;
  if (anyDemotedDisk) dReplicaSet.assign(D, ReplicaSet(&replicaOrder));
  for (int b = 0; b < B; ++b)
    if (!alive(b))
      for (int k = bDiskOff[b]; k < bDiskOff[b + 1]; ++k) {  // Broker.setState(DEAD): Disk.setState(DEAD)
        dAlive[bDisks[k]] = 0;
        dCap[bDisks[k]] = -1.0;
      }
  if (D == 0) return;
  if (d.replica_disk)
    for (int r = 0; r < R; ++r) {
      const int k = d.replica_disk[r];
      if (k < -1 || k >= D) throw std::invalid_argument("replica disk out of range");
      if (k >= 0 && dBroker[k] != rBroker[r]) throw std::invalid_argument("replica disk on another broker");
      if (k < 0) continue;
      rDisk[r] = rOrigDisk[r] = k;
      rDiskPos[r] = (int32_t)dMembers[k].size();
      dMembers[k].push_back(r);
      if (anyDemotedDisk) dReplicaSet[k].add(r, replicaHash(r));
      dUtil[k] += ru(r, R_DISK);  // Disk.addReplica (load still empty: += 0.0) then Disk.addReplicaLoad
    }
  for (int i = 0; i < d.num_disk_assignments; ++i) {
    const int r = d.disk_assign_replica[i], k = d.disk_assign_disk[i];
    if (r < 0 || r >= R || k < 0 || k >= D || dBroker[k] != rBroker[r])
      throw std::invalid_argument("disk assignment out of range");
    diskAdd(k, r);
  }
}

int Model::diskOf(int b, const std::string& logdir) const {
  for (int k = bDiskOff[b]; k < bDiskOff[b + 1]; ++k)
    if (dLogdir[bDisks[k]] == logdir) return bDisks[k];
  return -1;
}
double Model::avgDiskPct(int b) const {
  double cap = 0, util = 0;
  for (int k = bDiskOff[b]; k < bDiskOff[b + 1]; ++k) {
    const int d = bDisks[k];
    if (dAlive[d]) {
      cap += dCap[d];
      util += dUtil[d];
    }
  }
  return cap > 0 ? util / cap : 1.0;
}
// Membership: without ghosts (Disk._replicas entries left by inter-broker moves) a replica is a member of exactly
// its current disk, tracked by rDiskPos (O(1)); with ghosts the member lists are searched.
void Model::diskAdd(int d, int r) {
  auto& v = dMembers[d];
  const bool member = diskGhosts ? std::find(v.begin(), v.end(), r) != v.end() : (rDisk[r] == d && rDiskPos[r] >= 0);
  if (member)
    throw StateError("Disk " + dLogdir[d] + " already has replica " + topicNames[pTopic[rPart[r]]] + "-" +
                     std::to_string(pNumber[rPart[r]]));
  dUtil[d] += ru(r, R_DISK);
  rDisk[r] = d;
  rDiskPos[r] = (int32_t)v.size();
  v.push_back(r);
  if (anyDemotedDisk) dReplicaSet[d].add(r, replicaHash(r));
  diskDirty = true;
}
void Model::diskRemove(int d, int r) {
  auto& v = dMembers[d];
  int pos = -1;
  if (rDisk[r] == d && rDiskPos[r] >= 0 && rDiskPos[r] < (int)v.size() && v[rDiskPos[r]] == r) {
    pos = rDiskPos[r];
  } else if (diskGhosts) {
    auto it = std::find(v.begin(), v.end(), r);
    if (it != v.end()) pos = (int)(it - v.begin());
  }
  if (pos < 0)
    throw StateError("Disk " + dLogdir[d] + " does not has replica " + topicNames[pTopic[rPart[r]]] + "-" +
                     std::to_string(pNumber[rPart[r]]));
  dUtil[d] -= ru(r, R_DISK);
  const int last = v.back();
  v[pos] = last;
  if (rDisk[last] == d) rDiskPos[last] = pos;
  v.pop_back();
  if (rDisk[r] == d) rDiskPos[r] = -1;
  if (anyDemotedDisk) dReplicaSet[d].remove(r, replicaHash(r));
  diskDirty = true;
}
void Model::relocateReplicaToDisk(int p, int b, int dst) {
  const int r = replicaOn(p, b);
  if (r < 0 || rDisk[r] < 0) throw std::runtime_error("Replica is not in the cluster.");
  const int src = diskOf(b, dLogdir[rDisk[r]]);  // Broker.moveReplicaBetweenDisks(tp, replica.disk().logDir(), ...)
  if (src < 0 || dst < 0 || dBroker[dst] != b) throw std::runtime_error("NullPointerException: logdir not on broker");
  diskRemove(src, r);
  diskAdd(dst, r);
  ActionRec a{CCMI_INTRA_BROKER_REPLICA_MOVEMENT, p, b, b, -1};
  a.srcDisk = src;
  a.dstDisk = dst;
  log.push_back(a);
}
void Model::replayDiskMove(int r, int src, int dst) {
  diskRemove(src, r);
  diskAdd(dst, r);
  ActionRec a{CCMI_INTRA_BROKER_REPLICA_MOVEMENT, rPart[r], dBroker[src], dBroker[src], -1};
  a.srcDisk = src;
  a.dstDisk = dst;
  log.push_back(a);
}
std::vector<int32_t> Model::replicaDisks() const {
  std::vector<int32_t> v(R);
  for (int i = 0; i < R; ++i) v[i] = rDisk[pSlots[i]];
  return v;
}

void Model::refreshBroker(int b) {
  for (int k = 0; k < 4; ++k) {
    const double u = ops.util(bLoad[b], k), c = cap(b, k);
    bUtilC[4 * b + k] = u;
    bPctC[4 * b + k] = c > 0 ? u / c : 1.0;
    if (ordBuilt_[k] && !ordDirty_[k][b]) {
      ordDirty_[k][b] = 1;
      ordDirtyList_[k].push_back(b);
    }
  }
}

void Model::refreshHost(int b) {
  if (!sharedHosts) return;
  const int h = bHost[b];
  for (int k = 0; k < 4; ++k) hUtilC[4 * (size_t)h + k] = ops.util(hLoad[h], k);
  if (dev)  // the device keeps each broker's host utilization in its record (BrokerRec.hutil)
    for (int x : hBrokers[h]) markB(x);
}

const std::vector<int32_t>& Model::brokersByPct(int res) {
  PhaseScope ps(PH_ORDER);
  auto less = [this, res](int x, int y) { return cmpBrokerPct(res, x, y) < 0; };
  std::vector<int32_t>& ord = ordPct_[res];
  std::vector<int32_t>& dl = ordDirtyList_[res];
  std::vector<uint8_t>& df = ordDirty_[res];
  if (!ordBuilt_[res]) {
    ord.resize(B);
    for (int b = 0; b < B; ++b) ord[b] = b;
    std::sort(ord.begin(), ord.end(), less);
    df.assign(B, 0);
    dl.clear();
    ordBuilt_[res] = true;
    return ord;
  }
  if (dl.empty()) return ord;
  // drop the moved brokers (one compaction pass), then put them back at their new keys: binary-search
  // insertion for a few, a merge for many
  size_t w = 0;
  for (size_t i = 0; i < ord.size(); ++i)
    if (!df[ord[i]]) ord[w++] = ord[i];
  ord.resize(w);
  if (dl.size() <= 16) {
    for (int b : dl) ord.insert(std::lower_bound(ord.begin(), ord.end(), b, less), b);
  } else {
    std::sort(dl.begin(), dl.end(), less);
    ordScratch_.resize((size_t)B);
    std::merge(ord.begin(), ord.end(), dl.begin(), dl.end(), ordScratch_.begin(), less);
    ord.swap(ordScratch_);
  }
  for (int b : dl) df[b] = 0;
  dl.clear();
  return ord;
}
void Model::refreshReplica(int r) {
  for (int k = 0; k < 4; ++k) {
    rUtilC[4 * r + k] = ops.util(rLoad[r], k);
    rScoreC[4 * r + k] = rLoad[r].mask ? ops.groupAvg(rLoad[r], k) : 0.f;
  }
}

double Model::capacityWithAllowedReplicaMoves(int res, const std::vector<uint8_t>& excluded) const {
  // _clusterCapacity[res] - DoubleStream.sum(capacity of alive excluded brokers)
  double s0 = 0, s1 = 0, simple = 0;
  bool any = false;
  for (int b = 0; b < B; ++b)
    if (alive(b) && !excluded.empty() && excluded[b]) {
      const double v = cap(b, res);
      const double t = v - s1, vv = s0 + t;
      s1 = (vv - s0) - t;
      s0 = vv;
      simple += v;
      any = true;
    }
  double drop = any ? s0 + s1 : 0.0;
  if (std::isnan(drop) && std::isinf(simple)) drop = simple;
  return clusterCap[res] - drop;
}

// ------------------------------------------------------------------------------- broker membership
void Model::brokerAdd(int b, int r) {
  rPos[r] = (int)bRepl[b].size();
  bRepl[b].push_back(r);
  const int32_t h = replicaHash(r);
  bReplicaSet[b].add(r, h);
  const int t = pTopic[rPart[r]];
  bTopicKeys[b].add(t, topicHash[t]);
  rInImm[r] = rInOff[r] = 0;
  if (rOrig[r] != b) {
    rInImm[r] = 1;
    bNimm[b]++;
  } else if (origOffline(r)) {
    rInOff[r] = 1;
    bNoff[b]++;
    bOfflineSet[b].add(r, h);
  }
  if (rLeader[r]) {
    ops.addAll(bLnw[b], rLoad[r]);
    bNlead[b]++;
    bLeaderSet[b].add(r, h);
  }
  ops.addAll(bLoad[b], rLoad[r]);
  hNrep[bHost[b]]++;  // Host.addReplica: _replicas.add, _load.addLoad(replica.load())
  if (sharedHosts) ops.addAll(hLoad[bHost[b]], rLoad[r]);
  sortedInsert(b, r);
}

int Model::brokerRemove(int b, int p) {
  const int r = replicaOn(p, b);
  if (r < 0) return -1;
  auto& v = bRepl[b];
  const int pos = rPos[r];
  v[pos] = v.back();
  rPos[v[pos]] = pos;
  v.pop_back();
  rPos[r] = -1;
  const int32_t h = replicaHash(r);
  bReplicaSet[b].remove(r, h);
  bOfflineSet[b].remove(r, h);
  ops.subAll(bLoad[b], rLoad[r]);
  hNrep[bHost[b]]--;
  if (sharedHosts) ops.subAll(hLoad[bHost[b]], rLoad[r]);  // Host.removeReplica: _load.subtractLoad(replica.load())
  if (rLeader[r]) {
    ops.subAll(bLnw[b], rLoad[r]);
    bNlead[b]--;
    bLeaderSet[b].remove(r, h);
  }
  if (rInImm[r]) bNimm[b]--;
  if (rInOff[r]) bNoff[b]--;
  rInImm[r] = rInOff[r] = 0;
  sortedErase(b, r);
  return r;
}

static inline int64_t relocStampNs() {
  return prof().on ? (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                         std::chrono::steady_clock::now().time_since_epoch()).count()
                   : 0;
}

void Model::relocateReplica(int p, int src, int dst) {
  lastRelocNs = relocStampNs();
  PhaseScope ps(PH_RELOCATE);
  bVer[src]++;
  bVer[dst]++;
  verLog.push_back(src);
  verLog.push_back(dst);
  const int r = brokerRemove(src, p);
  if (r < 0) throw std::runtime_error("Replica is not in the cluster.");
  noteDelta(src, r);
  noteDelta(dst, r);
  ops.subAll(cLoad, rLoad[r]);
  ops.subAll(bPot[src], rLoad[pLeader[p]]);
  rBroker[r] = dst;
  brokerAdd(dst, r);
  if (rDisk[r] >= 0) {  // Broker.addReplica: _diskByLogdir.get(replica.disk().logDir()).addReplica(replica)
    const int dd = diskOf(dst, dLogdir[rDisk[r]]);
    if (dd < 0) throw std::runtime_error("NullPointerException: broker " + std::to_string(bId[dst]) + " has no logdir " +
                                         dLogdir[rDisk[r]]);
    diskGhosts++;  // the source disk keeps the replica (Broker.removeReplica does not touch disks)
    diskAdd(dd, r);
  }
  ops.addAll(cLoad, rLoad[r]);
  ops.addAll(bPot[dst], rLoad[pLeader[p]]);
  refreshBroker(src);
  refreshBroker(dst);
  refreshHost(src);
  refreshHost(dst);
  log.push_back({CCMI_INTER_BROKER_REPLICA_MOVEMENT, p, src, dst, -1});
  if (!topicCountDense.empty()) {
    topicCountDense[(size_t)pTopic[p] * ldB + src]--;
    topicCountDense[(size_t)pTopic[p] * ldB + dst]++;
  }
  const bool lead = rLeader[r] && !topicLeadDense.empty();
  if (lead) {
    topicLeadDense[(size_t)pTopic[p] * ldB + src]--;
    topicLeadDense[(size_t)pTopic[p] * ldB + dst]++;
  }
  if (dev && !replaying) {
    markChain(cDirtyB, cDirtyBList, src);
    markChain(cDirtyB, cDirtyBList, dst);
    if (sharedHosts) {
      markChain(cDirtyH, cDirtyHList, bHost[src]);
      markChain(cDirtyH, cDirtyHList, bHost[dst]);
    }
    markB(src);
    markB(dst);
    markR(r);
    markP(p);
    dev->tdeltas.push_back({pTopic[p], src, -1, 0});
    dev->tdeltas.push_back({pTopic[p], dst, +1, 0});
    if (lead) {
      dev->tdeltas.push_back({pTopic[p], src, -1, 1});
      dev->tdeltas.push_back({pTopic[p], dst, +1, 1});
    }
  }
}

void Model::enableTopicLeaders() {
  if (!topicLeadDense.empty()) return;
  topicLeadDense.assign((size_t)T * ldB, 0);
  for (int p = 0; p < P; ++p) topicLeadDense[(size_t)pTopic[p] * ldB + rBroker[pLeader[p]]]++;
  if (dev) {
    flushToDevice();  // pending rows first: the device table starts from the host's current state
    dev->flushOnly();
    dev->enableTopicLeaders(topicLeadDense.data());
  }
}

void Model::swapSlots(int p, int i, int j) {
  if (i == j) return;
  std::swap(pSlots[pOff[p] + i], pSlots[pOff[p] + j]);
  if (dev && !replaying) {
    markChain(cDirtyP, cDirtyPList, p);
    markP(p);
  }
}

void Model::moveReplicaToEnd(int r) {
  const int p = rPart[r];
  int pos = pOff[p];
  while (pos < pOff[p + 1] && pSlots[pos] != r) ++pos;
  if (pos == pOff[p + 1]) throw StateError("Did not find replica for partition.");
  for (int i = pos; i + 1 < pOff[p + 1]; ++i) pSlots[i] = pSlots[i + 1];
  pSlots[pOff[p + 1] - 1] = r;
  if (dev && !replaying) {
    markChain(cDirtyP, cDirtyPList, p);
    markP(p);
  }
}

bool Model::relocateLeadership(int p, int src, int dst) {
  lastRelocNs = relocStampNs();
  PhaseScope ps(PH_RELOCATE);
  const int sr = replicaOn(p, src);
  if (sr < 0 || !rLeader[sr]) return false;
  const int dr = replicaOn(p, dst);
  if (dr < 0) throw std::runtime_error("no destination replica");
  if (rLeader[dr])  // IllegalArgumentException (ClusterModel.java:415-421)
    throw std::invalid_argument("Cannot relocate leadership of partition " + topicNames[pTopic[p]] + "-" +
                                std::to_string(pNumber[p]) + "from broker " + std::to_string(bId[src]) + " to broker " +
                                std::to_string(bId[dst]) + " because the destination replica is a leader.");
  bVer[src]++;
  bVer[dst]++;
  verLog.push_back(src);
  verLog.push_back(dst);
  noteDelta(src, sr);
  noteDelta(dst, dr);
  // Broker.makeFollower(src)
  ops.subAll(bLnw[src], rLoad[sr]);
  sortedErase(src, sr);
  LoadVec& L = rLoad[sr];
  LoadVec delta;
  ldMakeFollower(L, delta, W);
  rLeader[sr] = 0;
  refreshReplica(sr);
  if (bLoad[src].mask) ops.subAll(bLoad[src], delta);
  if (sharedHosts && hLoad[bHost[src]].mask) ops.subAll(hLoad[bHost[src]], delta);  // Host.makeFollower
  bNlead[src]--;
  bLeaderSet[src].remove(sr, replicaHash(sr));
  sortedInsert(src, sr);
  // Broker.makeLeader(dst)
  sortedErase(dst, dr);
  rLeader[dr] = 1;
  if (rLoad[dr].mask) ops.addAll(rLoad[dr], delta);
  refreshReplica(dr);
  ops.addAll(bLnw[dst], rLoad[dr]);
  if (bLoad[dst].mask) ops.addAll(bLoad[dst], delta);
  if (sharedHosts && hLoad[bHost[dst]].mask) ops.addAll(hLoad[bHost[dst]], delta);  // Host.makeLeader
  bNlead[dst]++;
  bLeaderSet[dst].add(dr, replicaHash(dr));
  sortedInsert(dst, dr);
  // Partition.relocateLeadership: swap positions 0 and indexOf(dr)
  int pos = pOff[p];
  while (pSlots[pos] != dr) ++pos;
  std::swap(pSlots[pOff[p]], pSlots[pos]);
  pLeader[p] = dr;
  refreshBroker(src);
  refreshBroker(dst);
  refreshHost(src);
  refreshHost(dst);
  log.push_back({CCMI_LEADERSHIP_MOVEMENT, p, src, dst, -1});
  if (!topicLeadDense.empty()) {
    topicLeadDense[(size_t)pTopic[p] * ldB + src]--;
    topicLeadDense[(size_t)pTopic[p] * ldB + dst]++;
  }
  if (dev && !replaying) {
    if (!topicLeadDense.empty()) {
      dev->tdeltas.push_back({pTopic[p], src, -1, 1});
      dev->tdeltas.push_back({pTopic[p], dst, +1, 1});
    }
    markChain(cDirtyB, cDirtyBList, src);
    markChain(cDirtyB, cDirtyBList, dst);
    if (sharedHosts) {
      markChain(cDirtyH, cDirtyHList, bHost[src]);
      markChain(cDirtyH, cDirtyHList, bHost[dst]);
    }
    markChain(cDirtyR, cDirtyRList, sr);
    markChain(cDirtyR, cDirtyRList, dr);
    markChain(cDirtyP, cDirtyPList, p);
    markB(src);
    markB(dst);
    markR(sr);
    markR(dr);
    markP(p);
  }
  return true;
}

void Model::flushToDevice() {
  if (!dev) return;
  for (int b : bDirtyList) {
    BrokerRow row;
    row.b = b;
    row.nrep = nrep(b);
    row.nlead = bNlead[b];
    row.alive = alive(b) ? 1 : 0;
    for (int k = 0; k < 4; ++k) row.util[k] = bUtilC[4 * b + k];
    row.potNwOut = potNwOut(b);
    row.leadNwIn = leadNwIn(b);
    for (int k = 0; k < 3; ++k) row.hutil[k] = hu(b, k);
    dev->brows.push_back(row);
    bDirty[b] = 0;
  }
  bDirtyList.clear();
  for (int r : rDirtyList) {
    ReplicaRow row;
    row.r = r;
    row.broker = rBroker[r];
    row.flags = (rLeader[r] ? RF_LEADER : 0) | (rOrigOff[r] ? RF_ORIG_OFFLINE : 0) | (alive(rOrig[r]) ? 0 : RF_ORIG_DEAD);
    row.pad = 0;
    for (int k = 0; k < 4; ++k) row.util[k] = rUtilC[4 * r + k];
    dev->rrows.push_back(row);
    rDirty[r] = 0;
  }
  rDirtyList.clear();
  for (int p : pDirtyList) {
    PartitionRow row;
    row.p = p;
    row.n = pOff[p + 1] - pOff[p];
    for (int k = 0; k < kMaxRf; ++k) {
      row.brokers[k] = k < row.n ? rBroker[pSlots[pOff[p] + k]] : -1;
      row.racks[k] = (int16_t)(k < row.n ? bRack[row.brokers[k]] : -1);
    }
    row.leadNwOut = pLeadNwOut(p);
    dev->prows.push_back(row);
    pDirty[p] = 0;
  }
  pDirtyList.clear();
}

void Model::flushChainLoads() {
  if (!dev) return;
  for (int b : cDirtyBList) {
    dev->lrows.push_back({LR_BROKER, b, bLoad[b]});
    dev->lrows.push_back({LR_LEADERSHIP_NW, b, bLnw[b]});
    dev->lrows.push_back({LR_POTENTIAL, b, bPot[b]});
    cDirtyB[b] = 0;
  }
  cDirtyBList.clear();
  for (int r : cDirtyRList) {
    dev->lrows.push_back({LR_REPLICA, r, rLoad[r]});
    cDirtyR[r] = 0;
  }
  cDirtyRList.clear();
  for (int p : cDirtyPList) {
    SlotRow row;
    row.p = p;
    row.leader = pLeader[p];
    for (int k = 0; k < kMaxRf; ++k) row.slots[k] = k < pOff[p + 1] - pOff[p] ? pSlots[pOff[p] + k] : -1;
    dev->srows.push_back(row);
    cDirtyP[p] = 0;
  }
  cDirtyPList.clear();
  for (int h : cDirtyHList) {
    dev->lrows.push_back({LR_HOST, h, hLoad[h]});
    cDirtyH[h] = 0;
  }
  cDirtyHList.clear();
}

// ------------------------------------------------------------------------------- sorted replicas
bool Model::selects(const Spec& s, int r) const {
  if (s.selLeaders && !rLeader[r]) return false;
  if (s.selFollowers && rLeader[r]) return false;
  if (s.selImmigrants && !immigrant(r)) return false;
  if (s.selImmOrOffline && !(immigrant(r) || curOffline(r))) return false;
  if (s.selOffline && !curOffline(r)) return false;
  // ReplicaSortFunctionFactory.selectReplicasBasedOnExcludedTopics (:135-146)
  if (s.selExclTopics && !origOffline(r) && exclTopicSel[pTopic[rPart[r]]]) return false;
  if (s.selExclMust && !origOffline(r) && (exclTopicSel[pTopic[rPart[r]]] || mustTopicSel[pTopic[rPart[r]]])) return false;
  if (s.selMustTopics && !mustTopicSel[pTopic[rPart[r]]]) return false;  // ReplicaSortFunctionFactory.java:153-155
  if (s.selAboveRes >= 0 && !(ru(r, s.selAboveRes) > s.aboveLimit)) return false;
  if (s.selBelowRes >= 0 && !(ru(r, s.selBelowRes) < s.belowLimit)) return false;
  return true;
}

// SortedReplicas comparator (priority functions, score by Double.compare, Replica.compareTo) as one 64-bit key:
// [prioOffline | prioImmigrant | Double.compare-ordered float score | offline | static tail rank (29 bits)].
// Replica.compareTo's tail (partition number, original broker id, topic) never changes, so it is ranked once.
uint64_t Model::replicaKey(const Spec& s, int r) const {
  const bool off = curOffline(r);
  uint64_t k = 0;
  if (s.prioOffline && !off) k |= 1ull << 63;
  if (s.prioImmigrants && !immigrant(r)) k |= 1ull << 62;
  if (s.scoreRes >= 0) {
    // (double)float compared with Double.compare: -0.0 < 0.0, every NaN equal and above +Infinity
    const float f = rScoreC[4 * r + s.scoreRes];
    uint32_t u;
    if (f != f) {
      u = 0xFFFFFFFFu;
    } else {
      uint32_t bits;
      memcpy(&bits, &f, 4);
      u = (bits & 0x80000000u) ? ~bits : (bits | 0x80000000u);
      if (s.scoreReverse) u = ~u;  // Double.compare(-a, -b): exactly the reversed order for non-NaN a, b
    }
    k |= (uint64_t)u << 30;
  }
  if (!off) k |= 1ull << 29;
  return k | (uint64_t)rStatic[r];
}
int Model::cmpReplica(const Spec& s, int a, int b) const {
  const uint64_t ka = replicaKey(s, a), kb = replicaKey(s, b);
  return ka == kb ? 0 : (ka < kb ? -1 : 1);
}

void Model::track(int b, int nameId, const Spec& s) {
  for (auto& t : tracked[b])
    if (t.nameId == nameId) return;  // putIfAbsent
  tracked[b].push_back({nameId, s, false, {}});
}
void Model::untrackAll(int nameId) {
  for (int b = 0; b < B; ++b) untrack(b, nameId);
}
void Model::untrack(int b, int nameId) {
  auto& v = tracked[b];
  for (size_t i = 0; i < v.size(); ++i)
    if (v[i].nameId == nameId) {
      v.erase(v.begin() + i);
      return;
    }
}
void Model::clearTracked() {
  for (int b = 0; b < B; ++b) tracked[b].clear();
}
void Model::clearTracked(int b) { tracked[b].clear(); }

// Per-broker cache of a few snapshots (Spec -> sorted list), valid while the broker's version is unchanged.
static std::shared_ptr<const std::vector<int32_t>>* cacheFind(std::vector<Model::SortedCacheEntry>& cache,
                                                                uint32_t ver, const Model::Spec& s) {
  for (auto& c : cache)
    if (c.ver == ver && c.spec == s) return &c.v;
  return nullptr;
}
static void cachePut(std::vector<Model::SortedCacheEntry>& cache, uint32_t ver, const Model::Spec& s,
                     std::shared_ptr<const std::vector<int32_t>> v) {
  Model::SortedCacheEntry* slot = nullptr;
  for (auto& c : cache)
    if (c.spec == s || c.ver != ver) {
      slot = &c;
      break;
    }
  if (!slot) {
    if (cache.size() < 4) {
      cache.emplace_back();
      slot = &cache.back();
    } else {
      slot = &cache[ver & 3];
    }
  }
  slot->spec = s;
  slot->ver = ver;
  slot->v = std::move(v);
}

void Model::setMustTopicSelection(const std::vector<uint8_t>& t) {
  if (t == mustTopicSel) return;
  mustTopicSel = t;
  ++selEpoch;
  for (auto& c : sortedCache) c.clear();
  for (auto& c : filteredCache) c.clear();
}

void Model::setExcludedTopicSelection(const std::vector<uint8_t>& t) {
  if (t == exclTopicSel) return;
  exclTopicSel = t;
  ++selEpoch;
  for (auto& c : sortedCache) c.clear();
  for (auto& c : filteredCache) c.clear();
}

// The snapshot of version bVer[b] from the cached one of an earlier version with the same Spec: the replicas the
// version log names leave, and those still on b that the Spec selects re-enter at their (key, index) position —
// the order a full sort of (replicaKey, r) gives, since every other replica kept its key.
bool Model::snapshotFromPrevious(int b, const Spec& s, std::vector<SortedCacheEntry>& cache, std::vector<int32_t>& out) {
  static const bool off = std::getenv("CCMI_SNAPSHOT_FULL") != nullptr;  // diagnostics: always re-sort
  if (off) return false;
  const SortedCacheEntry* prev = nullptr;
  for (const auto& c : cache)
    if (c.spec == s && c.v && c.ver < bVer[b]) prev = &c;
  if (!prev || bVer[b] - prev->ver > kDeltaLog) return false;
  int32_t changed[kDeltaLog];
  int nc = 0;
  uint32_t covered = 0;
  for (const auto& d : bDelta[b])
    if (d.first > prev->ver && d.first <= bVer[b]) {
      ++covered;
      if (d.second >= 0) changed[nc++] = d.second;
    }
  if (covered != bVer[b] - prev->ver) return false;
  out.clear();
  out.reserve(prev->v->size() + nc);
  for (int r : *prev->v) {
    bool skip = false;
    for (int i = 0; i < nc; ++i) skip |= changed[i] == r;
    if (!skip) out.push_back(r);
  }
  for (int i = 0; i < nc; ++i) {
    const int x = changed[i];
    bool dup = false;
    for (int j = 0; j < i; ++j) dup |= changed[j] == x;
    if (dup || rBroker[x] != b || !selects(s, x)) continue;
    const uint64_t kx = replicaKey(s, x);
    auto at = std::lower_bound(out.begin(), out.end(), x, [&](int y, int) {
      const uint64_t ky = replicaKey(s, y);
      return ky != kx ? ky < kx : y < x;
    });
    out.insert(at, x);
  }
  return true;
}

std::shared_ptr<const std::vector<int32_t>> Model::snapshot(int b, const Spec& s) {
  const bool limited = s.selAboveRes >= 0 || s.selBelowRes >= 0;
  auto& cache = limited ? filteredCache[b] : sortedCache[b];
  if (auto* hit = cacheFind(cache, bVer[b], s)) return *hit;
  std::shared_ptr<std::vector<int32_t>> v = std::make_shared<std::vector<int32_t>>();
  if (limited) {
    // The utilization limit only filters: the limit-free snapshot (cached across limits) filtered in order.
    Spec base = s;
    base.selAboveRes = base.selBelowRes = -1;
    base.aboveLimit = base.belowLimit = 0;
    const auto v0 = snapshot(b, base);
    v->reserve(v0->size());
    for (int r : *v0)
      if ((s.selAboveRes < 0 || ru(r, s.selAboveRes) > s.aboveLimit) &&
          (s.selBelowRes < 0 || ru(r, s.selBelowRes) < s.belowLimit))
        v->push_back(r);
  } else {
    const bool derived = snapshotFromPrevious(b, s, cache, *v);
    static const bool check = std::getenv("CCMI_SNAPSHOT_CHECK") != nullptr;  // tests: derived == re-sorted
    if (!derived || check) {
      PhaseScope ps(PH_SORTED_INIT);
      std::vector<std::pair<uint64_t, int32_t>>& keyed = snapKeys_;
      keyed.clear();
      for (int r : bRepl[b])
        if (selects(s, r)) keyed.push_back({replicaKey(s, r), r});
      std::sort(keyed.begin(), keyed.end());
      std::vector<int32_t> full;
      full.reserve(keyed.size());
      for (const auto& kr : keyed) full.push_back(kr.second);
      if (derived && full != *v) throw std::logic_error("snapshot derived from the previous version differs");
      *v = std::move(full);
    }
  }
  cachePut(cache, bVer[b], s, v);
  return v;
}

void Model::snapshotMany(const Spec& s, const std::vector<int32_t>& bs,
                         std::vector<std::shared_ptr<const std::vector<int32_t>>>& out) {
  const int n = (int)bs.size();
  out.assign(n, nullptr);
  static const bool check = std::getenv("CCMI_SNAPSHOT_CHECK") != nullptr;
  HostPool& pool = HostPool::get();
  if (check || pool.threads() <= 1 || n < 8) {
    for (int i = 0; i < n; ++i) out[i] = snapshot(bs[i], s);
    return;
  }
  // A utilization limit only filters the limit-free snapshot (as snapshot() does): the base Spec is sorted, the
  // limited one filtered from it.
  const bool limited = s.selAboveRes >= 0 || s.selBelowRes >= 0;
  Spec base = s;
  base.selAboveRes = base.selBelowRes = -1;
  base.aboveLimit = base.belowLimit = 0;
  // read-only phase: cache hits, versions derived from a cached predecessor, full sorts of the rest
  std::vector<std::shared_ptr<const std::vector<int32_t>>> freshBase(limited ? n : 0);
  std::vector<uint8_t> fresh(n, 0);
  auto baseOf = [&](int b, bool& isFresh) {
    auto& cache = sortedCache[b];
    if (auto* hit = cacheFind(cache, bVer[b], base)) {
      isFresh = false;
      return *hit;
    }
    auto v = std::make_shared<std::vector<int32_t>>();
    if (!snapshotFromPrevious(b, base, cache, *v)) {
      std::vector<std::pair<uint64_t, int32_t>> keyed;
      for (int r : bRepl[b])
        if (selects(base, r)) keyed.push_back({replicaKey(base, r), r});
      std::sort(keyed.begin(), keyed.end());
      v->reserve(keyed.size());
      for (const auto& kr : keyed) v->push_back(kr.second);
    }
    isFresh = true;
    return std::shared_ptr<const std::vector<int32_t>>(std::move(v));
  };
  pool.parallelFor(n, [&](int i) {
    const int b = bs[i];
    if (!limited) {
      bool f = false;
      out[i] = baseOf(b, f);
      fresh[i] = f;
      return;
    }
    if (auto* hit = cacheFind(filteredCache[b], bVer[b], s)) {
      out[i] = *hit;
      return;
    }
    bool f = false;
    const auto v0 = baseOf(b, f);
    if (f) freshBase[i] = v0;
    auto v = std::make_shared<std::vector<int32_t>>();
    v->reserve(v0->size());
    for (int r : *v0)
      if ((s.selAboveRes < 0 || ru(r, s.selAboveRes) > s.aboveLimit) &&
          (s.selBelowRes < 0 || ru(r, s.selBelowRes) < s.belowLimit))
        v->push_back(r);
    out[i] = std::move(v);
    fresh[i] = 1;
  });
  for (int i = 0; i < n; ++i) {
    const int b = bs[i];
    if (limited && freshBase[i]) cachePut(sortedCache[b], bVer[b], base, freshBase[i]);
    if (fresh[i]) cachePut(limited ? filteredCache[b] : sortedCache[b], bVer[b], s, out[i]);
  }
}

const std::vector<int32_t>& Model::sorted(int b, int nameId) {
  for (auto& t : tracked[b])
    if (t.nameId == nameId) {
      if (!t.init) {
        t.init = true;
        t.owned = false;
        t.shared = snapshot(b, t.spec);
      }
      return t.view();
    }
  throw std::runtime_error("sorted replicas not tracked");
}

void Model::sortedInsert(int b, int r) {
  for (auto& t : tracked[b]) {
    if (!t.init || !selects(t.spec, r)) continue;
    const Spec& s = t.spec;
    const uint64_t kr = replicaKey(s, r);
    const auto& cv = t.view();
    auto cit = std::lower_bound(cv.begin(), cv.end(), kr, [&](int x, uint64_t k) { return replicaKey(s, x) < k; });
    if (cit != cv.end() && replicaKey(s, *cit) == kr) continue;  // TreeSet.add of an equal element
    const size_t pos = (size_t)(cit - cv.begin());
    auto& v = t.mut();
    v.insert(v.begin() + pos, r);
  }
}
void Model::sortedErase(int b, int r) {
  for (auto& t : tracked[b]) {
    if (!t.init) continue;
    const Spec& s = t.spec;
    const uint64_t kr = replicaKey(s, r);
    const auto& cv = t.view();
    auto cit = std::lower_bound(cv.begin(), cv.end(), kr, [&](int x, uint64_t k) { return replicaKey(s, x) < k; });
    if (cit != cv.end() && *cit == r) {
      const size_t pos = (size_t)(cit - cv.begin());
      auto& v = t.mut();
      v.erase(v.begin() + pos);
    }
  }
}

}  // namespace ccmi
