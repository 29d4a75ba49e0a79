// Device side of a session: HBM tables, a host-coherent mapped staging area for row updates and scan
// requests, and the launch/readback protocol of one scan (no DMA copies, no stream synchronisation):
//   host  packs [row updates | request arrays] into the mapped staging area
//   K1/2  scan_cross / scan_pairs: when the update list fits the LDS overlay and the request is small, the
//         scan applies the rows itself and reads the request from the staging area (one launch);
//         otherwise K4 prep applies the rows and copies the request into HBM first
//   K5    scan_swap (+ visited sum) always after prep
//   the last workgroup writes one {seq, key} word into a host-mapped mailbox; the host spins on it
// Everything runs on one HIP stream per session, so HIP events on that stream time the kernels.
#pragma once
#include <functional>
#include <cstdint>
#include <string>
#include <unordered_map>
#include <memory>
#include <vector>

#include "devtypes.h"
#include "intra.h"
#include "shard_group.h"
#include "snapseg.h"

namespace ccmi {


// Algorithmic bytes per evaluated candidate: destination-broker record 4x f64 util, 4x f64 capacity,
// f64 potential NW_OUT, f64 leader NW_IN, i32 replica/leader/rack/topic-replica counts = 96 B.
constexpr int64_t kBytesPerCandidate = 96;
// K6 algorithmic bytes: per disk capacity + utilization + alive (17 B); per replica entry the replica id, disk,
// DISK utilization, score, Replica.compareTo rank, original disk and selection flag (29 B).
constexpr int64_t kIntraBytesPerDisk = 17;
constexpr int64_t kIntraBytesPerEntry = 29;

struct DevicePerf {
  int64_t scanLaunches = 0;
  int64_t scanPairs = 0;   // device-evaluated candidates (speculation included), pair-space size per launch
  double scanKernelMs = 0;
  int64_t scanBytes = 0;   // algorithmic bytes (96 B per evaluated candidate)
  int64_t statsLaunches = 0;
  double statsKernelMs = 0;
  int64_t statsBytes = 0;
  int64_t syncs = 0;
  int64_t singleLaunch = 0;  // scans that applied their rows in-kernel and read the request from host memory
  int64_t chainLaunches = 0; // K7 chains (several decisions per launch)
  int64_t scanRequired = 0;  // candidates the launches had to evaluate: each first-fit list up to its winner
  int64_t intraLaunches = 0;  // K6 intra-broker launches
  double intraKernelMs = 0;  // intra_brokers launches (HIP events, kernel timing on)
  double intraSortMs = 0;    // intra_sort launches (one per K6 call)
  int64_t intraSorts = 0;
  int64_t intraBytes = 0;     // algorithmic bytes of K6 (per broker record + per replica entry)
  int64_t combines = 0;       // shard-combiner calls (MIN allreduce of a scan's first-fit key)
  int64_t crossLaunches = 0;  // the scan_cross share of the scan counters
  int64_t crossRequired = 0;
  double crossKernelMs = 0;
  int64_t serverLaunches = 0;  // K8 scan_server launches (each serves many scans)
  int64_t serverIdleExits = 0;  // commands the server watchdog ended before it saw them (then launched)
  int64_t serverScans = 0;     // scans served by a running scan_server (no launch each)
  double serverBusyMs = 0;     // their device busy time (s_memrealtime, command seen -> result published)
  int64_t serverPayloadBytes = 0;  // command payload written through the BAR (program, rows, request arrays)
  int64_t serverRequired = 0;  // candidates those scans had to evaluate
  int64_t serverChains = 0;    // K7 chains the running server took as commands (no launch, no server restart)
  int64_t serverApplies = 0;   // apply-only server commands (topic-count deltas before a served scan that reads them)
  double serverResidentMs = 0;  // HIP-event time from each server launch to its exit (kernel timing on)
};

// K6 (kernels/intra.hip, intra.h): one intra-broker goal over every broker in one launch.
struct IntraRequest {
  int32_t goal;               // IntraGoal
  double capThr, margin;
  int32_t nPrior = 0;
  int32_t priorKind[4] = {0, 0, 0, 0};
  int32_t priorSlot[4] = {0, 0, 0, 0};  // threshold slots of prior IG_USAGE goals
  int32_t slot = 0;               // this goal's threshold slot (IG_USAGE)
  const int32_t* brokers = nullptr;  // ascending broker ids to rebalance
  int32_t nBrokers = 0;
  const int32_t* eOff = nullptr;  // [B+1] CSR of the replicas on each broker's disks
  const int32_t* eRep = nullptr;
  const int32_t* eDisk = nullptr;
  const uint8_t* rSel = nullptr;  // [R] tracked-sorted-replica selection
};
struct IntraResult {
  std::vector<int32_t> count, status;  // [B] records / IntraStatus per broker
  std::vector<int64_t> cand;           // [B]
  std::vector<int64_t> off;            // [B+1] compact record offsets (broker-id order)
  std::vector<int32_t> rep, src, dst;  // records
  std::vector<double> upper, lower;    // [B] this goal's thresholds (IG_USAGE)
};
struct DiskStatsOut {  // ClusterModelStats.populateStatsForDisks partials
  double varSum;
  int32_t unbalanced, numAlive;
};
constexpr int kDiskStatsBlocks = 256;  // stats_disks workgroups (partials folded by one wave)

class Device {
 public:
  Device(int ordinal, int B, int R, int P, int T, int maxGoalSlots);
  static int countGfx950();  // visible gfx950 devices
  ~Device();
  Device(const Device&) = delete;
  Device& operator=(const Device&) = delete;

  // Host work the engine hands over for the time a scan is in flight: called between polls of the result until it
  // returns false (each call a few microseconds of host-only work that touches no device state). Set around one
  // scan by its caller.
  std::function<bool()> idleWork;
  // Adds the last server command's busy time to perf (the kernel publishes it just after the result word); called
  // before every command and before perf is read.
  void collectServerBusy();
  struct IdleScope {  // clears idleWork when the scan returns or throws
    Device* d;
    ~IdleScope() { d->idleWork = nullptr; }
  };

  // initial upload (host arrays in device layout)
  void uploadStatic(const double* bCapRM, const int32_t* rPart, const int32_t* rOrig, const int32_t* pOff,
                    const int32_t* topicNrep, const int32_t* bRack, const int32_t* pTopic);
  // Partition._ineligibleBrokers as CSR (n = list length; nothing is uploaded for n == 0)
  void uploadIneligible(const int32_t* off, const int32_t* brokers, int n);
  void uploadDynamic(const double* bUtilRM, const int32_t* bNrep, const int32_t* bNlead, const double* bPot,
                     const double* bLeadNwIn, const uint8_t* bAlive, const double* rUtilRM, const int32_t* rBroker,
                     const uint8_t* rFlags, const int32_t* pBrokers, const double* pLeadNwOut,
                     const int32_t* topicCountDense /* [T][ldB] */);
  void setAllowed(int slot, const uint8_t* allowedB);
  // Brokers sharing hosts (Model::sharedHosts): every broker's host utilization [B][3] (CPU, NW_IN, NW_OUT) and its
  // host's capacity [B][3] (Host.capacityFor); from then on the predicates and stats read host values for those
  void uploadHosts(const double* hutil, const double* hcap);
  // The host model's replica -> broker, replica -> partition and partition -> topic arrays (stable for the session):
  // cross / pair scans send each row with its broker, partition and topic (RowRef).
  void setRowSource(const int32_t* rBroker, const int32_t* rPart, const int32_t* pTopic) {
    rowBroker_ = rBroker;
    rowPart_ = rPart;
    partTopic_ = pTopic;
  }
  // OptimizationOptions.excludedBrokersFor{Leadership,ReplicaMove} as bits kExclLeadBit / kExclMoveBit of every
  // broker's allowedBits
  void setExclusions(const uint8_t* exclLead, const uint8_t* exclMove, const uint8_t* isNew);
  // TopicReplicaDistributionGoal balance limits per topic (frozen at its initGoalState)
  void setTopicLimits(const int32_t* upper, const int32_t* lower);
  // BrokerSetAwareGoal: BrokerRec.bset [B] (broker set of every broker) and ReplicaRec.bset [R] (the set the mapping
  // policy gives every replica), strided writes that leave the rest of the records alone
  void setBrokerSets(const int32_t* brokerSet, const int32_t* replicaSet);
  // Broker.numLeadersFor counts [T][ldB] (the host model's dense table), kept on the device from now on (deltas of
  // kind 1 and the chain kernels update them); MinTopicLeadersPerBrokerGoal's minimum per topic [T] (-1 = not its topic)
  void enableTopicLeaders(const int32_t* topicLeadDense);
  void setMinLeaders(const int32_t* tMin);
  // TopicLeaderReplicaDistributionGoal's (upper, lower) leader limits per topic [T][2] (frozen at its initGoalState)
  void setTopicLeadLimits(const int32_t* lim);

  // pending row updates (flushed with the next launch)
  std::vector<BrokerRow> brows;
  std::vector<ReplicaRow> rrows;
  std::vector<PartitionRow> prows;
  std::vector<TopicCountDelta> tdeltas;

  // returns the winning key or -1. Cross: rows reps[0,K) x columns [c0,c1) of cands[0,N), key = k*N + j.
  // Pairs: pairs [p0,p1) of (pr, pb), key = pair index. Keys are global, so shards MIN-combine them.
  int64_t scanCross(const DevProgram& prog, const int32_t* reps, int K, const int32_t* cands, int N, int c0, int c1);
  int64_t scanSwap(const DevProgram& prog, const int32_t* srcs, int S, const int32_t* cbOff, int M,
                   const int32_t* cbRep, int nCand, const SwapLimit& lim, int64_t* visited);
  int64_t scanPairs(const DevProgram& prog, const int32_t* pr, const int32_t* pb, int p0, int p1);
  // A cross scan whose rows are snapshot segments: segment i contributes (*v)[skip, end) (replicas on broker cb, the
  // snapshot current for cb). Each snapshot is uploaded once into a device-resident pool and the scan sends only
  // the segment table; keys are those of scanCross over the concatenated rows. Falls back to scanCross.
  using SegIn = SnapSeg;
  int64_t scanSegs(const DevProgram& prog, const std::vector<SegIn>& segs, const int32_t* cands, int N, int c0,
                   int c1);
  bool segsUsable() const { return serverUsable_ && serverAllowed_; }

  // Queue scans (SOP_QUEUE, devtypes.h): the rows of a whole broker queue in one command. Each broker's rows are its
  // snapshot under ONE Spec, uploaded once per broker version into the snapshot pool and found through the snapshot
  // directory (QueueDirEntry[B] in fine-grained VRAM, written by the host only when a broker's snapshot changes). The
  // engine keeps the directory current (qdirSet after every version bump it has not yet seen); the device only reads.
  bool queueUsable() const;
  // entries belong to `key` (the engine's Spec + selection identity); another key drops every entry
  void qdirBind(uint64_t key);
  uint64_t qdirKey() const { return qdirKey_; }
  // bumped when the pool wraps: every directory entry then refers to overwritten rows and must be set again
  uint32_t poolEpoch() const { return poolEpoch_; }
  // upload broker b's snapshot and point its directory entry at it (false: larger than the pool)
  bool qdirSet(int b, std::shared_ptr<const std::vector<int32_t>> v);
  // qdirSet(bs[i], snaps[i]) for many brokers at once: the pool offsets are assigned here, the rows are written
  // through the BAR on the host pool (each row's RowRef gathers its partition and topic: random reads of the model,
  // most of a directory sync's time). false: a snapshot does not fit the pool.
  bool qdirSetMany(const std::vector<int32_t>& bs, const std::vector<std::shared_ptr<const std::vector<int32_t>>>& snaps);
  const std::vector<int32_t>& qdirRows(int b) const { return *qdirSnap_[b]; }
  int qdirLen(int b) const { return qdirSnap_[b] ? (int)qdirSnap_[b]->size() : 0; }
  // first accepted (row, column) over the queue entries [head (if >= 0)] ++ tail[0, nTail) (entry 0 from row skip0) x
  // cands[0, N); key = (i * span + row) * N + column with span = queueSpan(); -1 when none. Every entry must be set for
  // the bound key.
  int64_t scanQueue(const DevProgram& prog, int head, int skip0, const int32_t* tail, int nTail, const int32_t* cands,
                    int N);
  int queueSpan() const { return qdirSpan_; }
  // Shard groups (shard_group.h): the block every rank of the group maps, and the group's rank count. A served cross /
  // segment / pair scan is then combined by the server (takeDeviceCombined() reports it once); any other combine goes
  // through groupCombineHost on the same slot sequence.
  void attachGroup(CombineBlock* blk, int count, int rank);
  // armGroupCombine before the scan call Engine::combine wraps: the first served cross / segment / pair command after it
  // combines on the device (a scan the engine does not combine — a queue scan's flattened fallback — is never tagged)
  void armGroupCombine() { combineArmed_ = grpHost_ != nullptr; }
  bool takeDeviceCombined() {
    const bool x = devCombined_;
    devCombined_ = false;
    combineArmed_ = false;
    return x;
  }
  int64_t groupCombineHost(int64_t key);  // -1 = none, both ways
  static CombineBlock* allocCombineBlock();
  static void freeCombineBlock(CombineBlock* b);
  // the session's scans may (not) use the resident scan server (sessions whose scans wait on other ranks may not)
  // at most `blocks` server workgroups from the next server launch on (a multiple of 8, at least 8)
  void limitServerBlocks(int blocks);
  // an API call that may scan on this device begins / ends (the device's server budget is shared among its active
  // calls, ensureServer)
  void callBegin();
  void callEnd();
  void setServerAllowed(bool on) {
    if (!on) stopServer();
    serverAllowed_ = on;
  }
  void stats(const StatsParams& P, const uint8_t* allowedAliveHost, StatsOut* out);

  // Chains (K7, kernels/scan.hip): decisions applied on the device inside one launch. uploadLoads gives the device
  // the Java loads and partition slot order (once per session); lrows / srows carry the entities the host changed
  // without the device since the last chain and are sent first.
  void uploadLoads(int W, const LoadVec* rLoad, const LoadVec* bLoad, const LoadVec* bLnw, const LoadVec* bPot,
                   const int32_t* pSlots, const int32_t* pLeader);
  // brokers sharing hosts: Host._load per host, each broker's host and the hosts' brokers (CSR), once per session
  void uploadHostLoads(int H, const LoadVec* hLoad, const int32_t* bHost, const int32_t* hOff, const int32_t* hBrk);
  std::vector<LoadRow> lrows;
  std::vector<SlotRow> srows;
  struct ChainResult {
    int64_t accepts = 0, visited = 0, failRow = 0;
  };
  // PAIRS chain; log receives the accepted pair indices in order
  ChainResult chainPairs(const DevProgram& prog, const int32_t* pr, const int32_t* pb, const int32_t* next, int n,
                         int maxAccepts, std::vector<int32_t>& log);
  // RACK_ROWS chain; log receives (row, candidate index) per accepted row
  ChainResult chainRackRows(const DevProgram& prog, const int32_t* rows, int n, const int32_t* cands, int N,
                            std::vector<int32_t>& log);
  // RackAwareGoal's rows decided per partition group with no optimized goals (rackrows.h): rows[0, n) in loop order,
  // order[gOff[g], gOff[g + 1]) the row indices of group g in row order; res[k] receives the accepted candidate
  // index, kRackKeep or kRackFail. Nothing is applied on the device. Returns the candidates evaluated.
  int64_t rackRowsGroups(const DevProgram& prog, const int32_t* rows, int n, const int32_t* order, const int32_t* gOff,
                         int G, const int32_t* cands, int N, int32_t* res);
  void flushOnly();
  void flushPending();

  // Disks (JBOD): the static disk / replica tables once per session; setDiskUtil whenever the host changed a disk's
  // utilization; intraRun = one intra-broker goal (K6); statsDisks = the disk part of ClusterModelStats.
  void uploadDisks(int D, const int32_t* bDiskOff, const int32_t* bDisks, const double* dCap, const uint8_t* dAlive,
                   const uint8_t* bAlive, const int32_t* rOrigDisk, const double* rDu, const float* rScore,
                   const int32_t* rTie);
  void setDiskUtil(const double* dUtil);
  void intraRun(const IntraRequest& q, IntraResult& out);
  void statsDisks(double diskBalance, DiskStatsOut* out);

  DevicePerf perf;
  bool timing = false;  // record HIP events around kernels (bench/profiling)
  int ldB() const { return ldB_; }
  // K8 scan server (kernels/scan.hip scan_server): cross / pair scans are served by one persistent launch while it
  // runs; any other work on the session stream stops it first. CCMI_SERVER=0 turns it off (a launch per scan).
  void stopServer();

 private:
  int ordinal_, B_, R_, P_, T_, ldB_, G_;
  void* st_ = nullptr;  // hipStream_t
  // tables (records, devtypes.h) and the host copies used to assemble them
  BrokerRec* brokers_ = nullptr;
  ReplicaRec* replicas_ = nullptr;
  PartitionRec* parts_ = nullptr;
  int32_t *topicCount_ = nullptr, *topicNrep_ = nullptr, *tUpper_ = nullptr, *tLower_ = nullptr;
  int32_t *pIneligOff_ = nullptr, *pIneligB_ = nullptr;
  int32_t *topicLead_ = nullptr, *tMinLead_ = nullptr, *tLeadLim_ = nullptr;
  double* hostCap_ = nullptr;  // [B][3] Host.capacityFor of each broker's host (null: no shared hosts)
  uint8_t* allowedAlive_ = nullptr;
  std::vector<BrokerRec> hBrokers_;
  std::vector<PartitionRec> hParts_;
  std::vector<int32_t> hRPart_, hROrig_, hPOff_, bRackHost_;
  std::vector<uint32_t> allowedHost_;
  void *topicScratch_ = nullptr, *statsOut_ = nullptr, *statsPart_ = nullptr;
  // staging (host-coherent, mapped) and the request copy in HBM
  char* hStage_ = nullptr;
  char* hStageDev_ = nullptr;
  size_t stageCap_ = 0, stageUsed_ = 0;
  char* dReq_ = nullptr;
  size_t reqCap_ = 0;
  // result words in HBM, arrival counter, host mailbox {seq, value, extra}
  unsigned long long* dResult_ = nullptr;
  unsigned int* dDone_ = nullptr;
  unsigned long long* hResult_ = nullptr;
  unsigned long long* hResultDev_ = nullptr;
  unsigned long long seq_ = 0;
  alignas(16) unsigned char statsHost_[sizeof(StatsOut)];
  void *ev0_ = nullptr, *ev1_ = nullptr, *ev2_ = nullptr;  // hipEvent_t
  bool serverTimed_ = false;  // the running server launch has its start event recorded
  void *evS0_ = nullptr, *evS1_ = nullptr;  // hipEvent_t: a scan-server launch's residency (kernel timing on)
  struct Staged {
    int nb = 0, nr = 0, np = 0, nt = 0;
    size_t obr = 0, orr = 0, opr = 0, otd = 0, end = 0;
  };
  DevTables tables() const;
  size_t updatesBytes() const;
  Staged packUpdates(size_t extra);
  void unpackUpdates(const Staged& g);
  void ensureStage(size_t bytes);
  void ensureReq(size_t bytes);
  void launchPrepFor(const Staged& g, size_t reqBytes, bool scan);
  UpdateList stagedList(const Staged& g) const;
  UpdateList overlayFor(const Staged& g) const;
  MutTables mutTables() const;
  const char* stageScan(const Staged& g, size_t req, bool readsTopicCounts, UpdateList& u);
  bool waitMail(unsigned long long seq, bool serverCmd = false);
  int64_t finishScan();
  unsigned long long* stamps_ = nullptr;
  // scan server state: the fine-grained VRAM block [ServerCmd | payload] the host writes through the BAR
  char* fg_ = nullptr;
  size_t fgCap_ = 0;
  bool serverOn_ = false;
  bool serverUsable_ = false;  // set in the constructor (gfx950, CCMI_SERVER, fine-grained VRAM host-writable)
  bool serverAllowed_ = true;   // setServerAllowed
  CombineBlock* grpHost_ = nullptr;  // attachGroup: host pointer, this device's mapping, ranks, combines so far
  unsigned long long grpDev_ = 0;
  int grpCount_ = 0, grpRank_ = 0;
  uint64_t grpCalls_ = 0;
  uint32_t grpHostSeq_ = 0;  // host combines so far (their results arrive in mail[6] under this count)
  bool devCombined_ = false;
  bool combineArmed_ = false;
  std::vector<unsigned long long> groupMail_;  // the test emulation's shard-group mailbox (the product uses hResult_)
  int serverBlocks_ = 256;     // the running (or last) server launch's workgroups
  int serverBlocksCap_ = 256;  // at most this many (CU count, CCMI_SERVER_BLOCKS, limitServerBlocks)
  // goal-parallel server tiles (ServerCmd.goalParts): at most this many waves per candidate (CCMI_GOAL_SPLIT: 1, 2 or
  // 4) and only for scans whose split first sweep needs at most CCMI_GOAL_SPLIT_WGS workgroups
  int goalSplitMax_ = 4;
  bool applyViaServer_ = true;  // packForServer
  int goalSplitWgs_ = 256;
  // a server scan's first sweep sized from its site's last winner depth (serverRun; CCMI_SCAN_WIDTH=full: off)
  bool adaptiveWidth_ = true;
  // pair commands within one tile share their goals over several workgroups (serverRun; CCMI_WG_GOAL_SPLIT=0: off)
  bool wgGoalSplit_ = true;
  // Device::waitMail: polls of the result word before the first stream query (CCMI_QUERY_SPINS, default 16384)
  uint64_t spinsBeforeQuery_ = 16384;
  unsigned long long stuckTicks_ = 1000000000ull;  // 10 s of s_memrealtime: a command unpublished that long is stuck
  unsigned long long chainDelayTicks_ = 0;
  unsigned long long parkTicks_ = 100000ull;  // 1 ms: a shard-group scan waiting longer parks the server
  bool parkedPending_ = false;                // waitMail saw the server park with the awaited command
  size_t lrowsSent_ = 0, srowsSent_ = 0;      // CCMI_PROFILE: the last chain command's load / slot rows
  void retireParkedServer();
  bool claimServer();
  std::unordered_map<uint64_t, int64_t> lastDepth_;
  int progVer_ = 0;
  bool progSent_ = false;
  DevProgram lastProg_{};
  unsigned long long* dServerT0_ = nullptr;
  unsigned long long lastCmdSeq_ = 0;  // the sequence word the command block holds
  int32_t rowsEpoch_ = 0;              // server commands with rows so far (ServerCmd.rowsEpoch)
  double lastServerUse_ = 0;  // steady-clock seconds of the last served scan (the host restarts an idle server)
  bool serveScan(const DevProgram& prog, const Staged& g, bool readsTopicCounts);
  bool ensureServer();
  int serverProgram(const DevProgram& prog, char* pay);
  bool postCommand(ServerCmd& c, bool rowsSent);
  Staged packForServer(const DevProgram& prog, bool readsTc, bool& serve);
  bool busyPending_ = false;      // a completed command's busy time not yet collected
  unsigned long long busySeq_ = 0;
  // a K7 chain as a server command over the request arrays a0 | a1 | a2 (SOP_CHAIN); false = launch it instead
  bool serverChain(const DevProgram& prog, int mode, const int32_t* a0, int n0, const int32_t* a1, int n1,
                   const int32_t* a2, int n2, int n, int m, int maxAccepts);
  void streamWait(const char* what, double seconds);
  int32_t* dRackRes_ = nullptr;  // rackRowsGroups results (+ the evaluated-candidate counter after them)
  size_t rackResCap_ = 0;
  int32_t* dChainReq_ = nullptr;  // SOP_CHAIN request copy in HBM (the chain rereads it per decision)
  size_t chainReqCap_ = 0;
  const int32_t *rowBroker_ = nullptr, *rowPart_ = nullptr, *partTopic_ = nullptr;
  void writeRowRefs(char* dst, const int32_t* reps, size_t n) const;
  // A: replica ids sent as RowRefs (nA entries), or for SOP_SEGS the segment table (nA entries of SegEntry)
  int64_t serverRun(const DevProgram& prog, const Staged& g, int op, const void* A, size_t nA, const int32_t* C,
                    size_t nC, const int32_t params[6]);
  // snapshot pool (fine-grained VRAM, ring of RowRefs; a wrap restarts the server so no cache holds a reused line)
  RowRef* segPool_ = nullptr;
  size_t segCap_ = 0, segHead_ = 0;
  std::unordered_map<const void*, std::pair<std::shared_ptr<const std::vector<int32_t>>, uint32_t>> segCache_;
  std::vector<int32_t> segFlat_;
  std::vector<SegEntry> segTab_;
  int64_t segUpload(const SegIn& s);  // pool index of the snapshot's first entry, or -1 (does not fit)
  uint32_t poolEpoch_ = 0;
  uint64_t qdirKey_ = 0;
  int qdirSpan_ = 1;  // >= every set entry's length since the last bind
  QueueDirEntry* qdir_ = nullptr;  // fine-grained VRAM [B] (host-written through the BAR)
  std::vector<std::shared_ptr<const std::vector<int32_t>>> qdirSnap_;  // [B] the snapshot each entry points at
  void ensureFg(size_t bytes);
  int32_t* rowVisited_ = nullptr;
  size_t rowVisitedCap_ = 0;
  // chain state
  int W_ = 1;
  LoadVec *dRLoad_ = nullptr, *dBLoad_ = nullptr, *dBLnw_ = nullptr, *dBPot_ = nullptr, *dHLoad_ = nullptr;
  int32_t *dBHost_ = nullptr, *dHOff_ = nullptr, *dHBrk_ = nullptr;
  int32_t *dPOff_ = nullptr, *dPSlots_ = nullptr, *dPLeader_ = nullptr;
  // chain results in host-coherent mapped memory: the kernels write them, the host reads them after the stream sync
  // (no device-to-host copies per chain)
  int32_t* hChainLog_ = nullptr;
  int32_t* hChainLogDev_ = nullptr;
  size_t chainLogCap_ = 0;
  ChainResultDev* hChainOut_ = nullptr;
  ChainResultDev* hChainOutDev_ = nullptr;
  void ensureChainLog(size_t n);
  ChainTables chainTables() const;
  template <class F>
  size_t stageChainCopy(size_t reqBytes, Staged& g, size_t& oReq, F fill, void* stream);
  // disk state (K6)
  int D_ = 0;
  int32_t *dBDiskOff_ = nullptr, *dBDisks_ = nullptr, *dROrigDisk_ = nullptr, *dRTie_ = nullptr;
  double *dDCap_ = nullptr, *dDUtilIn_ = nullptr, *dDUtil_ = nullptr, *dRDu_ = nullptr;
  uint8_t *dDAlive_ = nullptr, *dBAlive_ = nullptr, *dRSel_ = nullptr;
  float* dRScore_ = nullptr;
  double *dUpper_ = nullptr, *dLower_ = nullptr;  // [G][B] usage-goal thresholds
  int32_t *dEOff_ = nullptr, *dERep_ = nullptr, *dEDiskIn_ = nullptr, *dEDisk_ = nullptr, *dSnapA_ = nullptr,
          *dSnapB_ = nullptr, *dOrdRev_ = nullptr, *dOrdFwd_ = nullptr, *dNSel_ = nullptr, *dHist_ = nullptr, *dBrokers_ = nullptr, *dLogCap_ = nullptr, *dCount_ = nullptr,
          *dStatus_ = nullptr, *dLogRep_ = nullptr, *dLogSrc_ = nullptr, *dLogDst_ = nullptr, *dCRep_ = nullptr,
          *dCSrc_ = nullptr, *dCDst_ = nullptr;
  int64_t *dLogOff_ = nullptr, *dCand_ = nullptr, *dCOff_ = nullptr;
  IntraRep* dRStat_ = nullptr;  // K6 packed static replica fields
  double* dEDu_ = nullptr;  // K6 entry-indexed gathers (IntraArgs.eDu / eOrig / eKeyRev / eKeyFwd)
  int32_t* dEOrig_ = nullptr;
  uint64_t *dEKeyRev_ = nullptr, *dEKeyFwd_ = nullptr;
  size_t entCap_ = 0, logCap_ = 0, compactCap_ = 0;
  DiskStatsOut* dDiskStats_ = nullptr;
  std::vector<void*> intraAllocs_;
  std::vector<int32_t> hBDiskOff_;
};


}  // namespace ccmi
