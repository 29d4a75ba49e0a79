// Host half of the engine's cluster model: structure-of-arrays state with the reference's exact load
// arithmetic, plus dirty-row tracking that feeds the device mirror (device.h).
//
// Numeric representation follows MetricValues (float window values + double running sum;
// cruise-control-core/.../aggregator/MetricValues.java:17-221) and ModelUtils.expectedUtilizationFor
// (model/ModelUtils.java:162-176). Mutations follow ClusterModel.relocateReplica / relocateLeadership
// (model/ClusterModel.java:380-441,546-564), Broker.add/removeReplica/makeFollower/makeLeader
// (model/Broker.java:336-510) and Replica.makeFollower/makeLeader (model/Replica.java:210-310), in the
// reference's operation order so every float/double rounding is reproduced.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <unordered_set>
#include <vector>

#include "ccmi.h"
#include "devtypes.h"
#include "errors.h"
#include "jsem.h"
#include "loadops.h"

namespace ccmi {

constexpr int kMaxDisksPerBroker = 31;  // intra.h kIntraMaxDisks (TimSort binary-insertion range)

class LoadOps {  // loadops.h arithmetic with the session's window count
 public:
  explicit LoadOps(int W) : W(W) {}
  int W;
  void zero(Window& x) const { ldZero(x, W); }
  void add(Window& a, const Window& b) const { ldAdd(a, b, W); }
  void sub(Window& a, const Window& b) const { ldSub(a, b, W); }
  void set(Window& a, int i, double x) const { ldSet(a, i, x); }
  float avg(const Window& a) const { return ldAvg(a, W); }
  void addAll(LoadVec& d, const LoadVec& s) const { ldAddAll(d, s, W); }
  void subAll(LoadVec& d, const LoadVec& s) const {
    for (int k = 0; k < 6; ++k)
      if ((s.mask >> k & 1) && !(d.mask >> k & 1)) throw std::runtime_error("subtract from a missing metric");
    ldSubAll(d, s, W);
  }
  double util(const LoadVec& l, int res) const { return ldUtil(l, res, W); }
  float groupAvg(const LoadVec& l, int res) const {  // valuesForGroup(group, def, shareValueArray=true).avg()
    if (res == R_CPU) return avg(l.m[M_CPU]);
    if (res == R_DISK) return avg(l.m[M_DISK]);
    Window acc;
    zero(acc);
    add(acc, l.m[res == R_NW_IN ? M_LBI : M_LBO]);
    add(acc, l.m[res == R_NW_IN ? M_RBI : M_RBO]);
    return avg(acc);
  }
};

enum class BState : int32_t { ALIVE = 0, DEAD = 1, NEW = 2, DEMOTED = 3, BAD_DISKS = 4 };

struct ActionRec {
  int32_t type, partition, src, dst, destPartition;
  int32_t srcDisk = -1, dstDisk = -1;  // intra-broker moves
};

class Device;
class Model;

// Element orders of the broker HashSets: Replica.compareTo (Replica.java:349-377) and String.compareTo.
struct ReplicaOrder {
  const Model* m;
  int cmp(int a, int b) const;
};
struct TopicOrder {
  const Model* m;
  int cmp(int a, int b) const;
};
using ReplicaSet = JHashSet<ReplicaOrder>;
using TopicSet = JHashSet<TopicOrder>;

class Model {
 public:
  int W = 1, B = 0, R = 0, P = 0, T = 0;
  LoadOps ops{1};
  // brokers
  std::vector<BState> bState;
  std::vector<int32_t> bRack, bId;
  std::vector<double> bCap;                 // [B][4]
  std::vector<std::vector<int32_t>> bRepl;  // replica ids hosted (HashSet contents; order unused)
  std::vector<int32_t> bNlead, bNimm, bNoff;
  std::vector<LoadVec> bLoad, bLnw, bPot;
  // Broker._replicas, _leaderReplicas, _currentOfflineReplicas (HashSet<Replica>) and _topicReplicas' key set
  // (HashMap<String, ...>), emulated for their iteration order
  std::vector<ReplicaSet> bReplicaSet, bLeaderSet, bOfflineSet;
  std::vector<TopicSet> bTopicKeys;
  ReplicaOrder replicaOrder{this};
  TopicOrder topicOrder{this};
  std::vector<int32_t> topicHash;           // String.hashCode of every topic name
  int32_t replicaHash(int r) const {        // Objects.hash(TopicPartition, originalBroker.id())
    const int p = rPart[r];
    const int32_t tp = jMix(jMix(1, pNumber[p]), topicHash[pTopic[p]]);  // TopicPartition.hashCode
    return jMix(jMix(1, tp), bId[rOrig[r]]);
  }
  std::vector<double> bUtilC;               // cache [B][4] of ops.util(bLoad[b], res)
  std::vector<double> bPctC;                // cache [B][4] of GoalUtils.utilization: util / cap, 1.0 if cap <= 0
  // All brokers ordered by (utilization %, id) per resource — the order every utilization-keyed TreeSet /
  // PriorityQueue of the ResourceDistribution drivers iterates in. Repaired lazily from a dirty list.
  const std::vector<int32_t>& brokersByPct(int res);
  int cmpBrokerPct(int res, int x, int y) const {
    const int c = jcmpDouble(pct(x, res), pct(y, res));
    return c ? c : jcmpInt(bId[x], bId[y]);
  }
  // replicas
  std::vector<int32_t> rPart, rBroker, rOrig, rPos;
  std::vector<uint8_t> rLeader, rOrigOff, rInImm, rInOff;
  std::vector<LoadVec> rLoad;
  std::vector<double> rUtilC;               // [R][4]
  std::vector<float> rScoreC;               // [R][4] groupAvg per resource (sorted-replica score)
  // partitions
  std::vector<int32_t> pTopic, pNumber, pOff, pSlots, pLeader;  // pSlots: replica ids, Partition._replicas order
  // topics
  std::vector<std::string> topicNames;
  std::vector<int32_t> topicRank, topicNrep;
  std::vector<std::pair<uint64_t, int32_t>> snapKeys_;  // snapshot() scratch
  std::vector<int32_t> rStatic;  // dense rank of (partition number, original broker id, topic) — Replica.compareTo tail
  std::vector<int32_t> topicCountDense;     // [T][ldB] live Broker.numReplicasOfTopicInBroker counts
  int ldB = 4;
  int tcount(int t, int b) const { return topicCountDense[(size_t)t * ldB + b]; }
  // [T][ldB] live Broker.numLeadersFor counts, kept (here and on the device) once a goal asked for them
  std::vector<int32_t> topicLeadDense;
  int tlead(int t, int b) const { return topicLeadDense[(size_t)t * ldB + b]; }
  void enableTopicLeaders();
  // disks: replica placement over logdirs (JBOD; Broker._diskByLogdir TreeMap, model/Disk.java)
  int D = 0;
  std::vector<int32_t> dBroker;
  std::vector<std::string> dLogdir;
  std::vector<double> dCap, dUtil;          // Disk._capacity (-1 dead), Disk._utilization
  std::vector<uint8_t> dAlive;
  std::vector<std::vector<int32_t>> dMembers;  // Disk._replicas (a HashSet; its order is never observed)
  std::vector<int32_t> bDiskOff, bDisks;    // CSR: each broker's disks in logdir order
  std::vector<int32_t> rDisk, rOrigDisk;    // Replica._disk / _originalDisk (-1 = null)
  std::vector<int32_t> rDiskPos;            // index of the replica in dMembers[rDisk[r]] (-1 = not a member)
  // Disk.State.DEMOTED (ccmi.h disk_demoted) and, when a disk is demoted, every disk's Disk._replicas as the Java
  // HashSet it is (PreferredLeaderElectionGoal iterates a demoted disk's replicas)
  std::vector<uint8_t> dDemoted;
  bool anyDemotedDisk = false;
  std::vector<ReplicaSet> dReplicaSet;
  // Disk._replicas entries left behind by inter-broker moves (Broker.removeReplica keeps the replica on its disk)
  int64_t diskGhosts = 0;
  bool diskDirty = true;                    // device copy of dUtil is stale
  int diskOf(int b, const std::string& logdir) const;
  double diskPct(int d) const { return dCap[d] > 0 ? dUtil[d] / dCap[d] : 1.0; }  // GoalUtils.diskUtilizationPercentage
  double avgDiskPct(int b) const;            // GoalUtils.averageDiskUtilizationPercentage
  void diskAdd(int d, int r);                // Disk.addReplica (Disk.java:113-121)
  void diskRemove(int d, int r);             // Disk.removeReplica (Disk.java:139-146)
  // ClusterModel.relocateReplica(tp, brokerId, destinationLogdir) (ClusterModel.java:362-366), logged
  void relocateReplicaToDisk(int p, int b, int dst);
  // the same relocation for a K6 record whose replica and source disk are known (replay of a device decision)
  void replayDiskMove(int r, int src, int dst);
  std::vector<int32_t> replicaDisks() const;  // [R] disk of every replica slot in partition order

  // cluster
  LoadVec cLoad;
  double clusterCap[4] = {0, 0, 0, 0};
  std::vector<uint8_t> selfHealing;         // per replica: in _selfHealingEligibleReplicas
  int64_t numSelfHealing = 0;
  int numDead = 0, numNew = 0, numBadDisk = 0;
  // hosts (ccmi.h broker_host; Rack._hosts, model/Host.java). sharedHosts: some host holds two or more brokers. Only
  // then is host state kept: the load of its brokers' replicas with every add / subtract in the reference's order,
  // the capacity of its alive brokers (Host.capacityFor: -1 without one) and its replica count. Otherwise every host
  // value is its broker's own, bit for bit.
  bool sharedHosts = false;
  int H = 0;
  std::vector<int32_t> bHost;                  // [B] dense host index
  std::vector<std::vector<int32_t>> hBrokers;  // [H] brokers of each host
  std::vector<LoadVec> hLoad;                  // [H] Host._load
  std::vector<double> hCap, hUtilC;            // [H][4] Host._hostCapacity, cached expectedUtilizationFor
  std::vector<int32_t> hAlive, hNrep;          // [H] Host._aliveBrokers, Host._replicas.size()
  bool hostMode() const { return sharedHosts; }  // hu / hcap differ from bu / bcap only when brokers share hosts
  double hu(int b, int res) const { return sharedHosts ? hUtilC[4 * (size_t)bHost[b] + res] : bu(b, res); }
  double hcap(int b, int res) const {
    if (!sharedHosts) return cap(b, res);
    const int h = bHost[b];
    return hAlive[h] > 0 ? hCap[4 * (size_t)h + res] : -1.0;
  }
  bool hostEmpty(int b) const { return sharedHosts ? hNrep[bHost[b]] == 0 : nrep(b) == 0; }
  // Partition._ineligibleBrokers: a BAD_DISKS broker holding an offline replica of the partition may not receive
  // one of its replicas (ClusterModel.setBrokerState :325-331); CSR over partitions, static
  std::vector<int32_t> pIneligOff, pIneligB;
  bool ineligible(int p, int b) const {
    for (int k = pIneligOff[p]; k < pIneligOff[p + 1]; ++k)
      if (pIneligB[k] == b) return true;
    return false;
  }
  int maxRf = 1;
  // action log + counters
  std::vector<ActionRec> log;
  int64_t candidates = 0;

  // device mirror
  Device* dev = nullptr;
  std::vector<uint8_t> bDirty, rDirty, pDirty;
  std::vector<int32_t> bDirtyList, rDirtyList, pDirtyList;
  void markB(int b) {
    if (!bDirty[b]) {
      bDirty[b] = 1;
      bDirtyList.push_back(b);
    }
  }
  void markR(int r) {
    if (!rDirty[r]) {
      rDirty[r] = 1;
      rDirtyList.push_back(r);
    }
  }
  void markP(int p) {
    if (!pDirty[p]) {
      pDirty[p] = 1;
      pDirtyList.push_back(p);
    }
  }
  void flushToDevice();  // turn dirty rows into Device::brows/rrows/prows
  // Chains (device.h): entities whose Java loads / slot order the host changed since the last chain launch, sent as
  // Device::lrows / srows before the next one. While `replaying` the host re-applies moves the device already made:
  // nothing is marked.
  bool replaying = false;
  std::vector<uint8_t> cDirtyB, cDirtyR, cDirtyP, cDirtyH;
  std::vector<int32_t> cDirtyBList, cDirtyRList, cDirtyPList, cDirtyHList;
  void markChain(std::vector<uint8_t>& f, std::vector<int32_t>& l, int x) {
    if (!f[x]) {
      f[x] = 1;
      l.push_back(x);
    }
  }
  void flushChainLoads();
  struct Replay {  // scope in which relocations re-apply moves a device chain already made
    Model& m;
    explicit Replay(Model& mm) : m(mm) { m.replaying = true; }
    ~Replay() { m.replaying = false; }
  };

  // ---- queries
  bool alive(int b) const { return bState[b] != BState::DEAD; }
  bool isNew(int b) const { return bState[b] == BState::NEW; }
  double cap(int b, int res) const { return bCap[4 * b + res]; }
  double bu(int b, int res) const { return bUtilC[4 * b + res]; }
  double ru(int r, int res) const { return rUtilC[4 * r + res]; }
  double pct(int b, int res) const { return bPctC[4 * b + res]; }  // GoalUtils.utilization (cached)
  int nrep(int b) const { return (int)bRepl[b].size(); }
  bool origOffline(int r) const { return rOrigOff[r] || !alive(rOrig[r]); }
  bool curOffline(int r) const { return (origOffline(r) && rBroker[r] == rOrig[r]) || !alive(rBroker[r]); }
  bool immigrant(int r) const { return rOrig[r] != rBroker[r]; }
  int replicaOn(int p, int b) const {
    for (int i = pOff[p]; i < pOff[p + 1]; ++i)
      if (rBroker[pSlots[i]] == b) return pSlots[i];
    return -1;
  }
  void onlineFollowerBrokers(int p, std::vector<int>& out) const {
    out.clear();
    for (int i = pOff[p]; i < pOff[p + 1]; ++i) {
      const int r = pSlots[i];
      if (!rLeader[r] && !curOffline(r)) out.push_back(rBroker[r]);
    }
  }
  double capacityWithAllowedReplicaMoves(int res, const std::vector<uint8_t>& excludedReplicaMove) const;
  double clusterUtil(int res) const { return ops.util(cLoad, res); }
  double potNwOut(int b) const { return ops.util(bPot[b], R_NW_OUT); }   // potentialLeadershipLoadFor(b) NW_OUT
  double leadNwIn(int b) const { return ops.util(bLnw[b], R_NW_IN); }    // leadershipLoadForNwResources NW_IN
  double pLeadNwOut(int p) const { return ru(pLeader[p], R_NW_OUT); }    // partition(tp).leader() NW_OUT
  int numLeaderReplicas() const { return P; }

  // ---- mutations (record into the action log, mark dirty rows)
  void relocateReplica(int p, int src, int dst);
  // Partition.swapReplicaPositions / swapFollowerPositions (Partition.java:162-186): slots i and j (0-based within p)
  void swapSlots(int p, int i, int j);
  bool relocateLeadership(int p, int src, int dst);
  void moveReplicaToEnd(int r);  // Partition.moveReplicaToEnd (Partition.java:192-197): slot order only

  // ---- sorted replica tracking (sorted-vector implementation of SortedReplicas)
  struct Spec {
    bool selLeaders = false, selFollowers = false, selImmigrants = false, selImmOrOffline = false;
    bool selOffline = false;
    bool selExclTopics = false;  // selectReplicasBasedOnExcludedTopics over exclTopicSel
    bool selExclMust = false;    // ... over exclTopicSel + mustTopicSel (BrokerSetAwareGoal._excludedTopics)
    bool selMustTopics = false;  // selectReplicasBasedOnIncludedTopics over mustTopicSel (MinTopicLeadersPerBrokerGoal)
    int selAboveRes = -1, selBelowRes = -1;
    double aboveLimit = 0, belowLimit = 0;
    bool prioOffline = false, prioImmigrants = false;
    int scoreRes = -1;  // -1 none
    bool scoreReverse = false;
    bool operator==(const Spec& o) const {
      return selLeaders == o.selLeaders && selFollowers == o.selFollowers && selImmigrants == o.selImmigrants &&
             selOffline == o.selOffline && selExclTopics == o.selExclTopics && selExclMust == o.selExclMust &&
             selMustTopics == o.selMustTopics &&
             selImmOrOffline == o.selImmOrOffline && selAboveRes == o.selAboveRes && selBelowRes == o.selBelowRes &&
             aboveLimit == o.aboveLimit && belowLimit == o.belowLimit && prioOffline == o.prioOffline &&
             prioImmigrants == o.prioImmigrants && scoreRes == o.scoreRes && scoreReverse == o.scoreReverse;
    }
  };
  struct Tracked {
    int nameId;
    Spec spec;
    bool init = false;
    std::shared_ptr<const std::vector<int32_t>> shared;  // initial contents shared with the cache
    std::vector<int32_t> own;                            // private copy once the live view diverges
    bool owned = false;
    const std::vector<int32_t>& view() const { return owned ? own : *shared; }
    std::vector<int32_t>& mut() {
      if (!owned) {
        own = *shared;
        owned = true;
        shared.reset();
      }
      return own;
    }
  };
  std::vector<std::vector<Tracked>> tracked;  // per broker
  // Initial contents of a SortedReplicas depend only on the broker's replicas (set, loads, leadership,
  // origin) and the Spec; bVer[b] changes whenever any of those change, so an initialisation can be reused
  // from a cache entry with the same Spec and version instead of re-sorting.
  struct SortedCacheEntry {
    Spec spec;
    uint32_t ver = 0;
    std::shared_ptr<const std::vector<int32_t>> v;
  };
  std::vector<uint32_t> bVer;
  // Every version bump in order (src and dst of each relocation): readers that keep per-broker state derived from
  // snapshots (the queue scans' snapshot directory) catch up from their position instead of re-checking every broker.
  std::vector<int32_t> verLog;
  // CCMI_PROFILE: when the last relocation happened (steady_clock nanoseconds; 0 before the first)
  int64_t lastRelocNs = 0;
  // bumped whenever the selection sets the Specs do not carry change (excluded / must topics)
  uint32_t selEpoch = 0;
  // The replica whose membership or sort key changed at each of a broker's last kDeltaLog version bumps (-1: none),
  // so a snapshot can be derived from the previous version's instead of re-sorting the broker.
  static constexpr size_t kDeltaLog = 8;
  std::vector<std::vector<std::pair<uint32_t, int32_t>>> bDelta;
  void noteDelta(int b, int r) {
    auto& d = bDelta[b];
    if (d.size() == kDeltaLog) d.erase(d.begin());
    d.push_back({bVer[b], r});
  }
  std::vector<std::vector<SortedCacheEntry>> sortedCache;    // per broker, a few limit-free Specs
  std::vector<std::vector<SortedCacheEntry>> filteredCache;  // per broker, a few Specs with a utilization limit
  // OptimizationOptions.excludedTopics as the selection function sees it ([T] flags); setting a different set
  // drops the cached snapshots (their Specs do not carry the set)
  std::vector<uint8_t> exclTopicSel;
  void setExcludedTopicSelection(const std::vector<uint8_t>& t);
  // MinTopicLeadersPerBrokerGoal's topics ([T] flags) as selMustTopics / selExclMust see them (same cache rule)
  std::vector<uint8_t> mustTopicSel;
  void setMustTopicSelection(const std::vector<uint8_t>& t);
  void track(int b, int nameId, const Spec& s);
  void untrackAll(int nameId);
  void untrack(int b, int nameId);
  void clearTracked();
  void clearTracked(int b);
  const std::vector<int32_t>& sorted(int b, int nameId);  // lazily initialized live view
  // Contents a SortedReplicas(b, s) initialised now would have (shared with the initialisation cache): equal to
  // the live view of a set tracked earlier, because every key change re-inserts the replica.
  std::shared_ptr<const std::vector<int32_t>> snapshot(int b, const Spec& s);
  bool snapshotFromPrevious(int b, const Spec& s, std::vector<SortedCacheEntry>& cache, std::vector<int32_t>& out);
  // snapshot(bs[i], s) into out[i] for every listed broker, the misses computed on the host pool (hostpool.h; the
  // model is only read while they run, the caches are filled afterwards on this thread). The contents snapshot()
  // returns.
  void snapshotMany(const Spec& s, const std::vector<int32_t>& bs,
                    std::vector<std::shared_ptr<const std::vector<int32_t>>>& out);
  // One Spec's snapshots of every broker, looked up by broker id and version (no per-call cache search or
  // reference counting): the drivers that poll many brokers per scan (moveIn, swap) keep one per Spec.
  struct SnapTable {
    Spec spec;
    const void* owner = nullptr;  // the Model the table was filled from
    bool bound = false;
    uint32_t epoch = 0;         // selEpoch when bound
    std::vector<uint32_t> ver;  // bVer[b] + 1 of the stored snapshot, 0 = none
    std::vector<std::shared_ptr<const std::vector<int32_t>>> v;
    // (bVer[b] + 1) << 32 | the snapshot's size, 0 = none: viewSize() without a snapshot
    std::vector<uint64_t> size;
  };
  void bindSnapTable(SnapTable& t, const Spec& s) {
    if (!t.bound || t.owner != this || !(t.spec == s) || t.epoch != selEpoch) {
      t.spec = s;
      t.owner = this;
      t.bound = true;
      t.epoch = selEpoch;
      t.ver.assign(B, 0);
      t.v.assign(B, nullptr);
      t.size.assign(B, 0);
    }
  }
  const std::vector<int32_t>& snapshotIn(SnapTable& t, int b, const Spec& s) { return *snapshotInShared(t, b, s); }
  const std::shared_ptr<const std::vector<int32_t>>& snapshotInShared(SnapTable& t, int b, const Spec& s) {
    bindSnapTable(t, s);
    if (t.ver[b] != bVer[b] + 1u) {
      t.v[b] = snapshot(b, s);
      t.ver[b] = bVer[b] + 1u;
      t.size[b] = ((uint64_t)t.ver[b] << 32) | (uint32_t)t.v[b]->size();
    }
    return t.v[b];
  }
  // snapshotInShared for every listed broker into out[i]: the table's current entries as they are, the rest computed
  // together (snapshotMany: on the host pool when there are many) and stored in the table
  void snapshotManyIn(SnapTable& t, const Spec& s, const std::vector<int32_t>& bs,
                      std::vector<std::shared_ptr<const std::vector<int32_t>>>& out) {
    bindSnapTable(t, s);
    missB_.clear();
    for (int b : bs)
      if (t.ver[b] != bVer[b] + 1u) missB_.push_back(b);
    if (!missB_.empty()) {
      snapshotMany(s, missB_, missV_);
      for (size_t i = 0; i < missB_.size(); ++i) {
        const int b = missB_[i];
        t.v[b] = std::move(missV_[i]);
        t.ver[b] = bVer[b] + 1u;
        t.size[b] = ((uint64_t)t.ver[b] << 32) | (uint32_t)t.v[b]->size();
      }
      missV_.clear();
    }
    out.resize(bs.size());
    for (size_t i = 0; i < bs.size(); ++i) out[i] = t.v[bs[i]];
  }
  // snapshotIn(t, b, s).size() — the replicas of b that s selects — counted instead of sorted when the table holds no
  // current snapshot of b (a polled broker's size is all a driver's visited count needs from it)
  size_t viewSize(SnapTable& t, int b, const Spec& s) {
    bindSnapTable(t, s);
    return viewSizeBound(t, b);
  }
  // viewSize on a table bindSnapTable(t, s) bound to the same Spec since the last selection change
  size_t viewSizeBound(SnapTable& t, int b) {
    const uint32_t v = bVer[b] + 1u;
    const uint64_t x = t.size[b];
    if ((uint32_t)(x >> 32) == v) return (size_t)(uint32_t)x;
    uint32_t n = 0;
    for (int r : bRepl[b]) n += selects(t.spec, r) ? 1u : 0u;
    t.size[b] = ((uint64_t)v << 32) | n;
    return n;
  }
  bool selects(const Spec& s, int r) const;
  uint64_t replicaKey(const Spec& s, int r) const;
  int cmpReplica(const Spec& s, int a, int b) const;

  // Replays the desc construction order documented in include/ccmi.h (ClusterModel.createReplica +
  // setReplicaLoad per replica, then partition list order, then broker states).
  void build(const ccmi_cluster_desc& d);

 private:
  void buildDisks(const ccmi_cluster_desc& d);
  void brokerAdd(int b, int r);
  int brokerRemove(int b, int p);
  void refreshBroker(int b);
  void refreshHost(int b);  // the host of broker b: cached utilization, and every broker of it dirty (BrokerRow.hutil)
  std::vector<int32_t> ordPct_[4], ordDirtyList_[4], ordScratch_;
  std::vector<int32_t> missB_;  // snapshotManyIn scratch
  std::vector<std::shared_ptr<const std::vector<int32_t>>> missV_;
  std::vector<uint8_t> ordDirty_[4];
  bool ordBuilt_[4] = {false, false, false, false};
  void refreshReplica(int r);
  void sortedInsert(int b, int r);
  void sortedErase(int b, int r);
};

}  // namespace ccmi
