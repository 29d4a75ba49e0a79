// Device-resident structure-of-arrays mirror of the cluster model, and the scan request formats.
// Shared by host engine code and gfx950 kernels (plain POD, no HIP types).
//
// Layout in HBM (one session, B brokers, R replicas, P partitions, T topics) — the logical columns below are
// packed into per-entity records (BrokerRec / ReplicaRec / PartitionRec, further down):
//   broker rows   bUtil[4][B] f64 (expected utilization, ModelUtils.expectedUtilizationFor),
//                 bCap[4][B] f64, bNrep[B] i32, bNlead[B] i32, bPotNwOut[B] f64, bAlive[B] u8
//   replica rows  rUtil[4][R] f64, rPart/rBroker/rOrig[R] i32, rFlags[R] u8 (bit0 leader, bit1 orig-offline)
//   partitions    pOff[P+1] i32, pBrokers[R] i32 (current broker of every replica slot, Partition._replicas order)
//   topics        topicCount[T][B] i32 (dense Broker._topicReplicas sizes, for ClusterModelStats topic stats)
//   goal state    allowedBits[B] u32 (bit g: broker in goal slot g's _brokersAllowedReplicaMove, frozen at init)
//   more broker   bRack[B] i32 (static), bLeadNwIn[B] f64 (Broker._leadershipLoadForNwResources NW_IN)
//   more part.    pTopic[P] i32 (static), pLeadNwOut[P] f64 (NW_OUT utilization of the partition's leader)
//   topic limits  tUpper[T], tLower[T] i32 (TopicReplicaDistributionGoal balance limits, frozen at init)
// Resource-major broker columns make a candidate row (consecutive destination brokers) a coalesced read.
#pragma once
#include <stdint.h>

#include "loadops.h"

namespace ccmi {

constexpr int kMaxGoals = 20;     // goals in one program: the goal being optimized + its optimized goals
constexpr int kExclLeadBit = 31;  // allowedBits bit of a broker excluded for leadership (above every goal slot)
constexpr int kExclMoveBit = 30;  // allowedBits bit of a broker excluded for replica moves
constexpr int kNewBit = 29;       // allowedBits bit of a NEW broker (Broker.State.NEW)
// allowedBits goal slots [0, kMaxSlots): one per goal the session holds (one per goal kind) plus the running one
constexpr int kMaxSlots = 29;
static_assert(kMaxSlots <= kNewBit && kMaxGoals <= kMaxSlots, "goal slots overlap the broker flag bits");
constexpr int kMaxRf = 8;
// Dirty rows of each kind a cross/pair scan stages into its LDS overlay itself (kernels/scan.hip OverlayLds); a
// launch with more pending rows of any kind runs `prep` first (device.cpp stageScan). Shared by host and kernel.
constexpr int kOverlayRows = 32;

enum DevGoalKind : int32_t {
  DG_REPLICA_DISTRIBUTION = 0,
  DG_RESOURCE_DISTRIBUTION = 1,
  DG_ACCEPT_ALL = 2,  // MinTopicLeadersPerBrokerGoal without configured topics
  DG_RACK_AWARE = 3,
  DG_REPLICA_CAPACITY = 4,
  DG_CAPACITY = 5,
  DG_POTENTIAL_NW_OUT = 6,
  DG_TOPIC_REPLICA_DISTRIBUTION = 7,
  DG_LEADER_REPLICA_DISTRIBUTION = 8,
  DG_LEADER_BYTES_IN = 9,
  DG_RACK_AWARE_DISTRIBUTION = 10,
  DG_BROKER_SET_AWARE = 11,
  DG_MIN_TOPIC_LEADERS = 12,  // MinTopicLeadersPerBrokerGoal with configured topics
  DG_TOPIC_LEADER_DISTRIBUTION = 13  // TopicLeaderReplicaDistributionGoal
};
// ReplicaRec.bset flag of a replica of one of MinTopicLeadersPerBrokerGoal's topics: BrokerSetAwareGoal accepts every
// action on such a replica (BrokerSetAwareGoal.java:258-264) and leaves it out of its own moves (:136-151). Broker set
// indices stay below the flag; a negative bset is "none".
constexpr int32_t kBsetMust = 1 << 24;
// Operands a program's predicates read beyond the base broker/replica/partition record (DevProgram.needs).
enum DevNeed : uint32_t {
  NEED_RACK = 1, NEED_POT = 2, NEED_LEAD = 4, NEED_LBI = 8, NEED_TOPIC = 16, NEED_TLEAD = 32,
  NEED_TLLIM = 64  // TopicLeaderReplicaDistributionGoal's per-topic leader limits (with NEED_TLEAD)
};
// Resource.isHostResource / isBrokerResource (Resource.java:18-25): CPU both, NW_IN / NW_OUT host only, DISK broker only
constexpr bool isHostRes(int res) { return res != 3; }
constexpr bool isBrokerRes(int res) { return res == 0 || res == 3; }
// Candidate filters applied inside a CROSS scan before the predicate conjunction (the reference builds these
// candidate lists per replica; the kernel skips the excluded destinations instead).
enum DevFilter : int32_t {
  FILTER_NONE = 0,
  FILTER_RACK_AWARE = 1  // RackAwareGoal.rackAwareEligibleBrokers: rack not among the partition's other racks
};
enum DevAction : int32_t { DA_MOVE = 0, DA_LEADERSHIP = 1, DA_SWAP = 2 };
enum RFlag : uint8_t { RF_LEADER = 1, RF_ORIG_OFFLINE = 2, RF_ORIG_DEAD = 4 /* original broker dead (static) */ };

// Frozen per-goal state needed by selfSatisfied/actionAcceptance (a goal's initGoalState output).
struct DevGoal {
  int32_t kind;
  int32_t resource;
  int32_t upper, lower;        // ReplicaDistributionAbstractGoal._balanceUpperLimit/_balanceLowerLimit
  double upperThr, lowerThr;   // ResourceDistributionGoal._balanceUpperThreshold/_balanceLowerThreshold
  int32_t fixOffline;          // _fixOfflineReplicasOnly
  int32_t allowedSlot;         // bit of DevTables.allowedBits
  int32_t selfHealing;         // ReplicaCapacityGoal._isSelfHealingMode (unused by predicates; kept for parity)
  int32_t pad0;
  int64_t maxReplicas;         // BalancingConstraint.maxReplicasPerBroker (ReplicaCapacityGoal)
  double capThr;               // capacity threshold of `resource` (CapacityGoal, PotentialNwOutGoal: NW_OUT)
  double lbiMean;              // LeaderBytesInDistributionGoal._meanLeaderBytesIn (cached on first use)
  double lbiBalance;           // resource balance percentage of NW_IN
  double lbiLowUtil;           // low utilization threshold of NW_IN
};

// goals[0] is the goal being optimized (selfSatisfied); goals[1..n) are the optimized goals in the order
// AnalyzerUtils.isProposalAcceptableForOptimizedGoals visits them.
// A swap scan's candidate-row limit filter (sortedCandidateReplicas' selectReplicasBelowLimit / AboveLimit,
// ResourceDistributionGoal.java:543-569), applied on the device to limit-free candidate lists: res < 0 = none.
struct SwapLimit {
  int32_t res = -1;
  int32_t above = 0;  // 1: keep utilization > limit; 0: keep utilization < limit
  double limit = 0;
};

struct DevProgram {
  int32_t nGoals;
  int32_t action;
  uint32_t needs;   // DevNeed bits over all goals of the program
  int32_t filter;   // DevFilter of a CROSS scan
  int32_t exclLeadMove;  // replica moves: a leader replica may not go to a broker excluded for leadership
  int32_t swapExcl;      // swaps: GoalUtils.eligibleReplicasForSwap exclusion rules apply
  // new brokers in the cluster: moves / leadership go only to NEW brokers or the replica's original broker
  // (GoalUtils.eligibleBrokers :193-198); swaps follow eligibleReplicasForSwap's CASE#1/#3 (:276-297)
  int32_t newOnly;
  int32_t pad1;
  DevGoal goals[kMaxGoals];
};

// HBM records. One candidate pair reads one replica record, one partition record and two broker records, each
// a whole 64/128-byte line set fetched in one round trip: the dependency chain of a candidate is
// request -> replica + destination broker -> partition + source broker (-> topic counts for the topic goal).
struct alignas(64) BrokerRec {
  double util[4];         // ModelUtils.expectedUtilizationFor per resource
  double cap[4];          // capacity (-1 for dead brokers)
  double pot;             // potential leadership NW_OUT (ClusterModel.potentialLeadershipLoadFor)
  double lbi;             // leadership NW_IN (Broker.leadershipLoadForNwResources)
  int32_t nrep, nlead, rack;
  uint32_t allowedBits;   // bit g: in goal slot g's _brokersAllowedReplicaMove; bit 31: excluded for leadership
  int32_t alive;
  int32_t bset;           // broker set index (BrokerSetAwareGoal; static while a goal chain runs), -1 = none
  // Broker.host().load().expectedUtilizationFor(CPU, NW_IN, NW_OUT) — the host resources (Resource.isHostResource).
  // Equal to util[0..2] unless brokers share a host; read only when DevTables.hostCap is set.
  double hutil[3];
};
struct alignas(64) ReplicaRec {
  double util[4];
  int32_t broker, part, orig, flags;  // flags: RFlag bits
  int32_t bset;  // the broker set the replica belongs to (ReplicaToBrokerSetMappingPolicy) | kBsetMust, -1 = none
  int32_t pad[3];
};
struct alignas(64) PartitionRec {
  int32_t n, topic;
  int32_t brokers[kMaxRf];  // current broker of every replica slot (Partition._replicas order, leader first)
  double leadNwOut;         // NW_OUT utilization of the leader replica
  int16_t racks[kMaxRf];    // racks of `brokers`
};
static_assert(sizeof(BrokerRec) == 128 && sizeof(ReplicaRec) == 64 && sizeof(PartitionRec) == 64, "record sizes");

struct DevTables {
  const BrokerRec* brokers;
  const ReplicaRec* replicas;
  const PartitionRec* parts;
  const int32_t* topicCount;  // [T][ldB]
  const int32_t* tUpper;
  const int32_t* tLower;
  unsigned long long* stamps;  // diagnostics (CCMI_STAMPS=1): s_memrealtime stamps of workgroup 0, else null
  // Partition._ineligibleBrokers (BAD_DISKS brokers that held an offline replica of the partition, static):
  // CSR [P + 1] / list; null when the model has none
  const int32_t* pIneligOff;
  const int32_t* pIneligB;
  // Broker.numLeadersFor(topic) counts [T][ldB] (kept once a goal needs them, else null) and MinTopicLeadersPerBrokerGoal's
  // minimum per topic [T] (-1: not one of its topics; null when the goal has no topics)
  const int32_t* topicLead;
  const int32_t* tMinLead;
  // TopicLeaderReplicaDistributionGoal's _balanceUpperLimitByTopic / _balanceLowerLimitByTopic as [T][2] (upper,
  // lower) pairs, one 8-byte load per row; null until the goal runs
  const int32_t* tLeadLim;
  // Host.capacityFor(CPU, NW_IN, NW_OUT) of every broker's host [B][3] (static: -1 for a host without alive brokers);
  // null unless brokers share a host — then every host value is the broker's own and the predicates read those
  const double* hostCap;
  int32_t B, R, P, ldB;
  // scan server idle poll (CCMI_SERVER_POLL): 0 = back off (s_sleep 4, then 16 after 256 polls), 1 = spin, 2 = s_sleep 1
  int32_t pollMode;
  // 1: workgroup 0 re-reads the sequence word after copying a header (CCMI_SEQ_RECHECK=1); 0 (default): one read
  int32_t seqRecheck;
  // diagnostics (CCMI_CONJ_REPEAT=1): pair scans evaluate each candidate's conjunction twice (same result), so the
  // stamps show what the conjunction's arithmetic costs
  int32_t conjRepeat;
  // scan-server workgroups that poll the command word themselves (CCMI_DIRECT_POLLERS, default 8, the fewest workgroups
  // a scan command has; 1: workgroup 0 alone, the others wait for its doorbell)
  int32_t directPollers;
  // the scan server's stuck-command bound in s_memrealtime ticks (CCMI_SERVER_STUCK_MS, default 10 s) and a test-only
  // delay added to every chain command (CCMI_CHAIN_DELAY_US, default 0: a chain that outlasts a short bound)
  unsigned long long stuckTicks;
  unsigned long long chainDelayTicks;
  // a shard-group scan unpublished this long parks the server (CCMI_GROUP_PARK_US, default 1 ms; shard_group.h)
  unsigned long long parkTicks;
};

// Row updates the host flushes to the device before a scan (only rows touched since the last flush).
struct BrokerRow {
  int32_t b, nrep, nlead, alive;
  double util[4];
  double potNwOut;
  double leadNwIn;
  double hutil[3];  // BrokerRec.hutil (a host's load changes mark every broker of the host dirty)
};
struct ReplicaRow {
  int32_t r, broker, flags, pad;
  double util[4];
};
struct PartitionRow {
  int32_t p, n;
  int32_t brokers[kMaxRf];
  double leadNwOut;
  int16_t racks[kMaxRf];
};
// kind 0: topicCount (replicas of the topic on the broker), 1: topicLead (leaders of the topic on the broker)
struct TopicCountDelta {
  int32_t topic, broker, delta, kind;
};
// The LDS overlay of a scan workgroup (one copy of each row kind) stays well inside the 160 KB of a CU so four
// resident scan workgroups per CU still fit.
static_assert(kOverlayRows * (sizeof(BrokerRow) + sizeof(ReplicaRow) + sizeof(PartitionRow)) <= 16 * 1024,
              "overlay LDS budget");

// Writable views of the dynamic tables (row application inside a scan) and a staged update list.
struct MutTables {
  BrokerRec* brokers;
  ReplicaRec* replicas;
  PartitionRec* parts;
  int32_t* topicCount;
  int32_t* topicLead;  // null unless kept
  int32_t ldB;
};
// A scan row as the host knows it: the replica with its current broker, partition and topic, so the device loads
// the replica, partition, broker and topic-count records together (one dependent level after the request instead of
// three). K7 chains move replicas on the device and keep reading the broker from the replica record.
struct alignas(16) RowRef {
  int32_t r, src, p, topic;
};
static_assert(sizeof(RowRef) == 16, "RowRef is one 16-byte load");

struct UpdateList {
  const BrokerRow* brows;
  const ReplicaRow* rrows;
  const PartitionRow* prows;
  const TopicCountDelta* tdel;
  int32_t nb, nr, np, nt;
};

// Scan request modes.
//   CROSS : pairs (replicas[k], cands[j]) in k-major order; key = k * N + j
//   SWAP  : rows (m, s) = (candidate broker segment m, source replica s); a row's candidates are
//           cbRep[cbOff[m] .. cbOff[m+1]); key = ((m * S + s) << 24) | j of the row's FIRST terminal j,
//           kept only when that terminal is an ACCEPT (AbstractGoal.maybeApplySwapAction semantics).
enum ScanMode : int32_t { SM_CROSS = 0, SM_SWAP = 1 };

struct ScanHeader {
  int32_t mode;
  int32_t K;     // CROSS: number of replicas; SWAP: number of source replicas S
  int32_t N;     // CROSS: number of candidates; SWAP: number of segments M
  int32_t nCand; // SWAP: total candidate replicas
};

// Scan-server command (kernels/scan.hip scan_server), at the start of the fine-grained VRAM block the host writes;
// `seq` is written last, behind a store fence. Offsets are bytes from the payload base.
// SOP_CHAIN: a K7 chain (ChainMode) run by workgroup 0 of the server (nActive = 1) on the tables themselves: the
// command's rows, load rows (oL, nl) and slot rows (oS, ns) are applied first, the request is copied into chainReq,
// the decisions are logged to chainLog / chainOut (host-mapped), and the writes are released at system scope before
// the publish — no stop and relaunch of the server around a chain.
enum ServerOp : int32_t { SOP_CROSS = 0, SOP_PAIRS = 1, SOP_EXIT = 2, SOP_SEGS = 3, SOP_CHAIN = 4, SOP_QUEUE = 5 };
// SOP_QUEUE: a cross scan whose rows are the snapshots of a queue of brokers (ResourceDistributionGoal's move-in
// candidate queue, polled in order): queue entry i (broker id at oA) contributes rows [skip, len) of its snapshot in the
// device-resident snapshot pool, where {pool offset, len} is the broker's entry in the snapshot directory (fine-grained
// VRAM the host keeps current, ServerCmd.queueDir); skip = c0 for entry 0, 0 for the others. Columns are the N
// candidates at oC. Key = (i * span + row) * N + column (span = K >= every entry's len), so keys follow the poll order.
struct QueueDirEntry {
  uint32_t off;  // pool index of the broker's first snapshot row
  int32_t len;   // its snapshot length
};
// SOP_SEGS: a cross scan whose rows are the concatenation of nSegs segments of the device-resident snapshot pool
// (Device::scanSegs); the segment table at oA holds {first pool entry, first row} per segment plus {0, K} at the end.
constexpr int kMaxSegs = 1024;
struct SegEntry {
  uint32_t off;   // pool index of the segment's first row
  int32_t start;  // its row index in the concatenation
};
struct alignas(16) ServerCmd {
  unsigned long long seq;
  int32_t op;
  int32_t K, Nr, N, c0;  // SOP_CROSS: rows A[0, K) x columns C[0, Nr) of an N-column list starting at column c0
  int32_t n, keyBase;    // SOP_PAIRS: pairs (A[q], C[q]), q < n, key = keyBase + q
  int32_t sliced;
  int32_t progVer;       // the DevProgram at oProg changes only with its version
  int32_t nb, nr, np, nt;
  uint32_t oProg, oB, oR, oP, oT, oA, oC;
  int32_t nSegs;    // SOP_SEGS: entries of the segment table
  int32_t nActive;  // workgroups [0, nActive) take part (a multiple of 8); the others only follow the sequence
  // commands with rows before this one since the session started: a workgroup takes an agent acquire before it reads
  // the tables whenever this differs from the value it last acquired at (rows of commands it skipped included)
  int32_t rowsEpoch;
  // SOP_CHAIN: mode (ChainMode), n (pairs / rows), N (RACK_ROWS candidates), maxAccepts (PAIRS), load / slot rows
  int32_t chainMode, chainN, chainM, maxAccepts;
  int32_t nl, ns;
  uint32_t oL, oS;
  // SOP_CROSS / SOP_SEGS / SOP_PAIRS: wavefronts per candidate (1, 2 or 4), each evaluating a share of the goals
  // (moveCandidateAcceptedPart); a tile is then kBlock / goalParts candidates
  int32_t goalParts;
  unsigned long long chainReq;  // device addresses: HBM scratch for the request, host-mapped log and result
  unsigned long long chainLog;
  unsigned long long chainOut;
  unsigned long long queueDir;  // SOP_QUEUE: the snapshot directory (QueueDirEntry[B], fine-grained VRAM)
  // SOP_CROSS / SOP_SEGS / SOP_PAIRS of a session in a shard group (shard_group.h): the group's combine block (0: no
  // combine), this combine's slot, the rank and the rank count; the last workgroup folds the scan's key into the slot
  // instead of publishing it, and the group's last rank to arrive publishes the minimum to every rank
  unsigned long long combineBlock;
  int32_t combineSlot, combineRank, combineCount;
  // SOP_PAIRS within one tile: this many workgroups (each goalParts waves) share the tile's goals — workgroup w takes
  // parts w * goalParts + wave % goalParts of wgParts * goalParts — and AND their accept masks (1: one workgroup)
  int32_t wgParts;
};
// The sequence word: the host stores (next | kSeqBusy) before it rewrites the other fields and `next` after them, each
// behind a store fence; a workgroup copies the header once it reads a new sequence that is not busy (the fields landed
// first, and the host rewrites them only after that command's result). DevTables.seqRecheck adds the seqlock's second
// read of the word after the copy.
constexpr unsigned long long kSeqBusy = 1ull << 63;
// Set in the sequence word of a command every direct poller takes part in (ServerCmd.nActive >= DevTables.directPollers):
// those workgroups then know from the word alone that their header copy cannot tear (scan.hip scan_server).
constexpr unsigned long long kSeqAll = 1ull << 62;
static_assert(sizeof(ServerCmd) % 16 == 0, "ServerCmd words");

// Device-resident Java loads and partition slot order, so chain kernels can apply moves themselves (apply.h).
struct ChainTables {
  BrokerRec* brokers;
  ReplicaRec* replicas;
  PartitionRec* parts;
  int32_t* topicCount;
  int32_t* topicLead;  // null unless kept
  int32_t ldB;
  int32_t W;
  LoadVec* rLoad;    // [R]  Replica.load()
  LoadVec* bLoad;    // [B]  Broker.load()
  LoadVec* bLnw;     // [B]  Broker._leadershipLoadForNwResources
  LoadVec* bPot;     // [B]  ClusterModel._potentialLeadershipLoadByBrokerId
  const int32_t* pOff;  // [P+1]
  int32_t* pSlots;   // [R]  replica ids in Partition._replicas order (leader first)
  int32_t* pLeader;  // [P]
  // brokers sharing hosts (Model::sharedHosts; hLoad null otherwise): Host._load per host, each broker's host and every
  // host's brokers (CSR), so a chain move updates the host aggregates and every broker's BrokerRec.hutil of the host
  LoadVec* hLoad;         // [H]
  const int32_t* bHost;   // [B]
  const int32_t* hOff;    // [H+1]
  const int32_t* hBrk;    // [B]
};
// Host-side changes to those loads since the last chain launch (moves the host applied without the device).
enum LoadRowKind : int32_t { LR_REPLICA = 0, LR_BROKER = 1, LR_LEADERSHIP_NW = 2, LR_POTENTIAL = 3, LR_HOST = 4 };
struct LoadRow {
  int32_t kind, id;
  LoadVec v;
};
struct SlotRow {
  int32_t p, leader;
  int32_t slots[kMaxRf];
};
// Chain request: PAIRS = explicit (replica, destination) pairs in reference order with a group structure (after an
// accept the scan resumes at next[accepted]), stopping after maxAccepts; RACK_ROWS = RackAwareGoal's per-replica rows
// over one candidate list, each row re-checked against shouldKeepInTheCurrentBroker when reached.
enum ChainMode : int32_t { CM_PAIRS = 0, CM_RACK_ROWS = 1 };
struct ChainResultDev {
  unsigned long long accepts, visited, failRow;  // failRow: row + 1 of a RACK_ROWS row with no accepted candidate
};

// ClusterModelStats reduction (kernels/stats.hip)
struct TopicPartial {
  double avg, sd;
  int32_t mx, mn;
};
struct StatsParams {
  int32_t B, T;
  int32_t numAllowed;
  double clusterUtil[4];
  double avgPct[4];
  double upperThr[4], lowerThr[4];
  double potCapacity;  // capacityWithAllowedReplicaMovesFor(NW_OUT)
  double nwOutCapThreshold;
  double potSum;                 // sum of potential NW_OUT over alive allowed brokers (ClusterModelStats.java:334-340)
  int64_t repTotal, leadTotal;   // replicas / leaders over all brokers (populateReplicaStats totals)
  // brokers share hosts: the host resources' utilization and capacity are the host's (ClusterModelStats.java:297-303):
  // BrokerRec.hutil and this [B][3] table; null = the broker's own
  const double* hostCap;
};
// stats_partials record layout: double fields [0,4) hot, [4,8) cold, [8,12) variance sums per resource, then the
// named ones; int fields [0,4) balanced counts per resource, then the named ones.
enum : int { kSdPHot = 12, kSdPCold, kSdPVar, kSdRepVar, kSdLeadVar, kSdTAvg, kSdTSd, kStatD };
enum : int { kSiUnder = 4, kSiRepMx, kSiRepMn, kSiLeadMx, kSiLeadMn, kSiTMx, kSiTMn, kStatI };
constexpr int kStatsPartBlocks = 64;
struct StatsOut {
  double resAvg[4], resMax[4], resMin[4], resStd[4];
  int32_t numBalanced[4];
  double pnwAvg, pnwMax, pnwMin, pnwStd;
  int32_t numUnderPot;
  double repAvg, repStd;
  int32_t repMax, repMin;
  double leadAvg, leadStd;
  int32_t leadMax, leadMin;
  double topicAvg, topicStd;
  int32_t topicMax, topicMin;
};

}  // namespace ccmi
