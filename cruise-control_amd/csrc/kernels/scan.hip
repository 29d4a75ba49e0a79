// gfx950 kernels for the goal optimizer's candidate scans.
//
// K1+K2  scan_cross : first-fit over (replica k, destination broker j) pairs in k-major order — the
//                     candidate loop of AbstractGoal.maybeApplyBalancingAction (AbstractGoal.java:243-270)
//                     unrolled over the caller's replica loop. The answer is the SMALLEST pair index whose
//                     predicate conjunction holds, i.e. the deterministic argmin that breaks ties by the
//                     reference's iteration order; found with a wavefront ballot, an LDS block reduction and
//                     one 64-bit atomicMin per block (order-independent, so results are bitwise stable).
// K5     scan_swap  : one wavefront per (candidate broker m, source replica s) row walks that broker's
//                     candidate replicas (AbstractGoal.maybeApplySwapAction, AbstractGoal.java:287-338);
//                     the row's FIRST terminal outcome decides it, and the smallest row whose terminal is
//                     an ACCEPT wins.
// K4     prep       : scatters the host's dirty broker/replica/partition rows and topic-count deltas into
//                     the device tables, copies the scan request from the host-mapped staging area into HBM
//                     and resets the result words — one launch, no DMA copy.
// Cross/pair scans apply small update lists themselves (LDS overlay, see OverlayLds) and read small requests
// straight from the host-mapped staging area, so a scan is ONE launch. Results go back without a copy or a
// stream sync: the last workgroup to finish (arrival counter) writes one {seq, key} word into a host-mapped
// mailbox, and the host spins on it.
// Built with -ffp-contract=off: every predicate is the reference's IEEE double expression.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>

#include "../engine/apply.h"
#include "../engine/devtypes.h"
#include "../engine/predicates.h"
#include "../engine/rackrows.h"
#include "../engine/shard_group.h"

namespace ccmi {

struct DevView {
  DevTables t;
  __device__ __forceinline__ double bu(int b, int res) const { return t.brokers[b].util[res]; }
  __device__ __forceinline__ double bcap(int b, int res) const { return t.brokers[b].cap[res]; }
  __device__ __forceinline__ bool hostMode() const { return t.hostCap != nullptr; }
  __device__ __forceinline__ double hu(int b, int res) const { return t.hostCap ? t.brokers[b].hutil[res] : bu(b, res); }
  __device__ __forceinline__ double hcap(int b, int res) const {
    return t.hostCap ? t.hostCap[3 * (size_t)b + res] : bcap(b, res);
  }
  __device__ __forceinline__ int nrep(int b) const { return t.brokers[b].nrep; }
  __device__ __forceinline__ bool alive(int b) const { return t.brokers[b].alive != 0; }
  __device__ __forceinline__ bool allowed(int slot, int b) const { return (t.brokers[b].allowedBits >> slot) & 1u; }
  __device__ __forceinline__ double ru(int r, int res) const { return t.replicas[r].util[res]; }
  __device__ __forceinline__ int flags(int r) const { return t.replicas[r].flags; }
  __device__ __forceinline__ int rbroker(int r) const { return t.replicas[r].broker; }
  __device__ __forceinline__ int rorig(int r) const { return t.replicas[r].orig; }
  __device__ __forceinline__ bool origOff(int r) const {
    return (t.replicas[r].flags & (RF_ORIG_OFFLINE | RF_ORIG_DEAD)) != 0;
  }
  __device__ __forceinline__ int rpart(int r) const { return t.replicas[r].part; }
  __device__ __forceinline__ bool hosts(int p, int b) const {
    const PartitionRec& x = t.parts[p];
    bool has = false;
    for (int i = 0; i < x.n; ++i) has |= (x.brokers[i] == b);
    return has;
  }
  __device__ __forceinline__ int rack(int b) const { return t.brokers[b].rack; }
  __device__ __forceinline__ bool ineligible(int p, int b) const {
    if (!t.pIneligOff) return false;
    bool in = false;
    for (int k = t.pIneligOff[p]; k < t.pIneligOff[p + 1]; ++k) in |= t.pIneligB[k] == b;
    return in;
  }
  __device__ __forceinline__ bool otherOnRack(int p, int self, int rk) const {
    const PartitionRec& x = t.parts[p];
    bool any = false;
    for (int i = 0; i < x.n; ++i) any |= (x.brokers[i] != self) && (x.racks[i] == rk);
    return any;
  }
  __device__ __forceinline__ int slotRack(int /*p*/, int b) const { return t.brokers[b].rack; }
  __device__ __forceinline__ int rackCount(int p, int rk) const {
    const PartitionRec& x = t.parts[p];
    int c = 0;
    for (int i = 0; i < x.n; ++i) c += x.racks[i] == rk ? 1 : 0;
    return c;
  }
  __device__ __forceinline__ int nlead(int b) const { return t.brokers[b].nlead; }
  __device__ __forceinline__ double pot(int b) const { return t.brokers[b].pot; }
  __device__ __forceinline__ double lnwin(int b) const { return t.brokers[b].lbi; }
  __device__ __forceinline__ double pLeadNwOut(int p) const { return t.parts[p].leadNwOut; }
  __device__ __forceinline__ int ptopic(int p) const { return t.parts[p].topic; }
  __device__ __forceinline__ int tcount(int tp, int b) const { return t.topicCount[(size_t)tp * t.ldB + b]; }
  __device__ __forceinline__ int tUpper(int tp) const { return t.tUpper[tp]; }
  __device__ __forceinline__ int tLower(int tp) const { return t.tLower[tp]; }
  __device__ __forceinline__ int bset(int b) const { return t.brokers[b].bset; }
  __device__ __forceinline__ int rbset(int r) const { return t.replicas[r].bset; }
  __device__ __forceinline__ int tlead(int tp, int b) const { return t.topicLead[(size_t)tp * t.ldB + b]; }
  __device__ __forceinline__ int tMinLead(int tp) const { return t.tMinLead ? t.tMinLead[tp] : -1; }
  __device__ __forceinline__ int tLeadUpper(int tp) const { return t.tLeadLim[2 * tp]; }
  __device__ __forceinline__ int tLeadLower(int tp) const { return t.tLeadLim[2 * tp + 1]; }
};

// Row updates a cross/pair scan applies itself (instead of a separate launch): every workgroup stages the
// host's dirty rows from the host-mapped staging area into LDS and reads a dirty entity from there, while
// workgroup 0 writes the rows into the HBM tables for the next launch. Only dirty rows are written and no
// workgroup reads a dirty row from HBM during the launch, so there is no read/write race.
struct OverlayLds {  // kOverlayRows (devtypes.h): the host sends larger update lists through `prep`
  BrokerRow b[kOverlayRows];
  ReplicaRow r[kOverlayRows];
  PartitionRow p[kOverlayRows];
  int nb, nr, np;
  __device__ __forceinline__ int broker(int x) const {
    for (int i = 0; i < nb; ++i)
      if (b[i].b == x) return i;
    return -1;
  }
  __device__ __forceinline__ int replica(int x) const {
    for (int i = 0; i < nr; ++i)
      if (r[i].r == x) return i;
    return -1;
  }
  __device__ __forceinline__ int partition(int x) const {
    for (int i = 0; i < np; ++i)
      if (p[i].p == x) return i;
    return -1;
  }
};

// Copy n rows (whole 32-bit words) from the host-mapped staging area into LDS. The first word of every thread is
// loaded by the caller's single batch (stageLoad) so the three row kinds cost one PCIe round trip, not three.
template <class Row>
__device__ __forceinline__ int rowWords(int n) { return n * (int)(sizeof(Row) / 4); }
template <class Row>
__device__ __forceinline__ void stageRest(Row* dst, const Row* __restrict__ src, int n) {
  const int words = rowWords<Row>(n);
  for (int w = threadIdx.x + blockDim.x; w < words; w += blockDim.x)
    reinterpret_cast<int32_t*>(dst)[w] = reinterpret_cast<const int32_t*>(src)[w];
}

__device__ __forceinline__ void applyRowsBlock(const MutTables& M, const BrokerRow* brows, int nb,
                                               const ReplicaRow* rrows, int nr, const PartitionRow* prows, int np,
                                               const TopicCountDelta* tdel, int nt, int first, int stride) {
  for (int i = first; i < nb; i += stride) {
    const BrokerRow& x = brows[i];
    BrokerRec& d = M.brokers[x.b];
#pragma unroll
    for (int k = 0; k < 4; ++k) d.util[k] = x.util[k];
    d.nrep = x.nrep;
    d.nlead = x.nlead;
    d.pot = x.potNwOut;
    d.lbi = x.leadNwIn;
    d.alive = x.alive;
#pragma unroll
    for (int k = 0; k < 3; ++k) d.hutil[k] = x.hutil[k];
  }
  for (int i = first; i < nr; i += stride) {
    const ReplicaRow& x = rrows[i];
    ReplicaRec& d = M.replicas[x.r];
#pragma unroll
    for (int k = 0; k < 4; ++k) d.util[k] = x.util[k];
    d.broker = x.broker;
    d.flags = x.flags;
  }
  for (int i = first; i < np; i += stride) {
    const PartitionRow& x = prows[i];
    PartitionRec& d = M.parts[x.p];
#pragma unroll
    for (int k = 0; k < kMaxRf; ++k) {
      d.brokers[k] = x.brokers[k];
      d.racks[k] = x.racks[k];
    }
    d.leadNwOut = x.leadNwOut;
  }
  for (int i = first; i < nt; i += stride) {
    const TopicCountDelta d = tdel[i];
    atomicAdd(&(d.kind ? M.topicLead : M.topicCount)[(size_t)d.topic * M.ldB + d.broker], d.delta);
  }
}

// applyRowsBlock with device-scope stores (the scan server): each store is written through to memory, so the rows
// need no L2 write-back before workgroup 0 arrives — the next command's acquire (an L2 invalidate) is enough for every
// workgroup to read them.
__device__ __forceinline__ void stDev(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), __double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void stDev(int32_t* p, int32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void applyRowsCoherent(const MutTables& M, const BrokerRow* brows, int nb,
                                                  const ReplicaRow* rrows, int nr, const PartitionRow* prows, int np,
                                                  int first, int stride) {
  for (int i = first; i < nb; i += stride) {
    const BrokerRow& x = brows[i];
    BrokerRec& d = M.brokers[x.b];
#pragma unroll
    for (int k = 0; k < 4; ++k) stDev(&d.util[k], x.util[k]);
    stDev(&d.nrep, x.nrep);
    stDev(&d.nlead, x.nlead);
    stDev(&d.pot, x.potNwOut);
    stDev(&d.lbi, x.leadNwIn);
    stDev(&d.alive, x.alive);
#pragma unroll
    for (int k = 0; k < 3; ++k) stDev(&d.hutil[k], x.hutil[k]);
  }
  for (int i = first; i < nr; i += stride) {
    const ReplicaRow& x = rrows[i];
    ReplicaRec& d = M.replicas[x.r];
#pragma unroll
    for (int k = 0; k < 4; ++k) stDev(&d.util[k], x.util[k]);
    stDev(&d.broker, x.broker);
    stDev(&d.flags, x.flags);
  }
  for (int i = first; i < np; i += stride) {
    const PartitionRow& x = prows[i];
    PartitionRec& d = M.parts[x.p];
#pragma unroll
    for (int k = 0; k < kMaxRf; ++k) stDev(&d.brokers[k], x.brokers[k]);
    stDev(&d.leadNwOut, x.leadNwOut);
    int32_t* rk = reinterpret_cast<int32_t*>(d.racks);  // the int16 racks as whole words
    const int32_t* xr = reinterpret_cast<const int32_t*>(x.racks);
#pragma unroll
    for (int k = 0; k < kMaxRf / 2; ++k) stDev(&rk[k], xr[k]);
  }
}

// Stage the update list into LDS (every workgroup that evaluates pairs) and apply it to HBM (workgroup 0, which
// always evaluates the first chunk). Workgroups whose first chunk is already beaten exit without staging.
__device__ __forceinline__ void overlayStage(OverlayLds& ov, const UpdateList& U) {
  if (threadIdx.x == 0) {
    ov.nb = U.nb;
    ov.nr = U.nr;
    ov.np = U.np;
  }
  if (U.nb | U.nr | U.np) {
    // one batch of independent host reads (a thread's first word of each row kind), then the stores
    const int t = threadIdx.x;
    const int wb = rowWords<BrokerRow>(U.nb), wr = rowWords<ReplicaRow>(U.nr), wp = rowWords<PartitionRow>(U.np);
    int32_t xb = 0, xr = 0, xp = 0;
    if (t < wb) xb = reinterpret_cast<const int32_t*>(U.brows)[t];
    if (t < wr) xr = reinterpret_cast<const int32_t*>(U.rrows)[t];
    if (t < wp) xp = reinterpret_cast<const int32_t*>(U.prows)[t];
    if (t < wb) reinterpret_cast<int32_t*>(ov.b)[t] = xb;
    if (t < wr) reinterpret_cast<int32_t*>(ov.r)[t] = xr;
    if (t < wp) reinterpret_cast<int32_t*>(ov.p)[t] = xp;
    stageRest<BrokerRow>(ov.b, U.brows, U.nb);
    stageRest<ReplicaRow>(ov.r, U.rrows, U.nr);
    stageRest<PartitionRow>(ov.p, U.prows, U.np);
  }
  __syncthreads();
}
__device__ __forceinline__ void overlayApply(const OverlayLds& ov, const UpdateList& U, const MutTables& M,
                                             const DevTables& T) {
  if (blockIdx.x == 0 && (U.nb | U.nr | U.np | U.nt))
    applyRowsBlock(M, ov.b, ov.nb, ov.r, ov.nr, ov.p, ov.np, U.tdel, U.nt, threadIdx.x, blockDim.x);
}

// A move candidate's operands gathered up front with independent loads (row side: the replica, its broker,
// its partition's brokers; destination side: one broker record), so the predicate conjunction runs on
// registers instead of a chain of control-dependent loads. Accessors answer only for the ids a move
// predicate asks about (the replica r, its source/original broker, the destination, r's partition).
// Operands only some goals read (racks, potential NW_OUT, leader counts, leader bytes-in, topic counts) are
// loaded when the program's `needs` mask asks for them (a wave-uniform branch).
struct PreView {
  int r, src, orig, p, rflags, dst, snrep, dnrep;
  uint32_t aliveBits;   // bit 0 src, bit 2 dst (values, never addressed: keeps the view in VGPRs)
  uint32_t srcAllowed;  // allowedBits of src
  int pn, pb0, pb1, pb2, pb3, pb4, pb5, pb6, pb7;
  uint32_t dAllowed;    // allowedBits of dst (bit kExclLeadBit: excluded for leadership)
  double ru0, ru1, ru2, ru3, sbu0, sbu1, sbu2, sbu3, scap0, scap1, scap2, scap3;
  double dbu0, dbu1, dbu2, dbu3, dcap0, dcap1, dcap2, dcap3;
  // optional operands
  int drack, prk0, prk1, prk2, prk3, prk4, prk5, prk6, prk7;
  double spot, dpot, plno, slbi, dlbi;
  int snlead, dnlead, topic, stc, dtc, tup, tlo;
  int rbs, sbs, dbs;  // broker sets: the replica's (mapping policy), the source's, the destination's
  int stl, dtl, tmn;  // leaders of the row's topic on the source / destination, MinTopicLeaders' minimum of it
  int tlu, tll;       // TopicLeaderReplicaDistributionGoal's leader limits of the row's topic
  bool inelig;  // dst is one of the row's partition's ineligible brokers
  // host resources of the source's / destination's hosts (only when brokers share hosts: DevTables.hostCap set). The
  // view keeps where they are (the broker's record or its dirty overlay row, and the host capacity table) and the
  // predicates load them on use: no registers held for them on the common one-broker-per-host path.
  bool hmode;
  const double* shu;  // source's host utilization [3] (HBM record or LDS overlay row)
  const double* dhu;  // destination's
  const double* hcapT;  // DevTables.hostCap

  static __device__ __forceinline__ double sel(int k, double a, double b, double c, double d) {
    return k == 0 ? a : (k == 1 ? b : (k == 2 ? c : d));
  }
  __device__ __forceinline__ void setPartition(const PartitionRec& x) {  // x: LDS overlay row or HBM record
    pn = x.n;
    pb0 = x.brokers[0];
    pb1 = x.brokers[1];
    pb2 = x.brokers[2];
    pb3 = x.brokers[3];
    pb4 = x.brokers[4];
    pb5 = x.brokers[5];
    pb6 = x.brokers[6];
    pb7 = x.brokers[7];
    plno = x.leadNwOut;
    topic = x.topic;
    prk0 = x.racks[0];
    prk1 = x.racks[1];
    prk2 = x.racks[2];
    prk3 = x.racks[3];
    prk4 = x.racks[4];
    prk5 = x.racks[5];
    prk6 = x.racks[6];
    prk7 = x.racks[7];
  }
  // Every HBM field is loaded unconditionally (independent loads the compiler can issue together) and then
  // replaced from the LDS overlay when the entity is dirty in this launch.
  __device__ __forceinline__ void loadRow(const DevTables& t, const DevProgram& prog, int rr, const OverlayLds& ov) {
    r = rr;
    const ReplicaRec& rec = t.replicas[r];
    orig = rec.orig;
    p = rec.part;
    src = rec.broker;
    rflags = rec.flags;
    rbs = rec.bset;
    ru0 = rec.util[0];
    ru1 = rec.util[1];
    ru2 = rec.util[2];
    ru3 = rec.util[3];
    const int ri = ov.replica(r);
    if (ri >= 0) {
      const ReplicaRow& x = ov.r[ri];
      src = x.broker;
      rflags = x.flags;
      ru0 = x.util[0];
      ru1 = x.util[1];
      ru2 = x.util[2];
      ru3 = x.util[3];
    }
    setPartition(t.parts[p]);
    const BrokerRec& sb = t.brokers[src];
    bool aSrc = sb.alive != 0;
    snrep = sb.nrep;
    sbu0 = sb.util[0];
    sbu1 = sb.util[1];
    sbu2 = sb.util[2];
    sbu3 = sb.util[3];
    snlead = sb.nlead;
    spot = sb.pot;
    slbi = sb.lbi;
    scap0 = sb.cap[0];
    scap1 = sb.cap[1];
    scap2 = sb.cap[2];
    scap3 = sb.cap[3];
    srcAllowed = sb.allowedBits;
    sbs = sb.bset;
    loadSrcHost(t, sb, ov);
    const int pi = ov.partition(p);
    if (pi >= 0) {
      const PartitionRow& x = ov.p[pi];
      pn = x.n;
      pb0 = x.brokers[0];
      pb1 = x.brokers[1];
      pb2 = x.brokers[2];
      pb3 = x.brokers[3];
      pb4 = x.brokers[4];
      pb5 = x.brokers[5];
      pb6 = x.brokers[6];
      pb7 = x.brokers[7];
      plno = x.leadNwOut;
      prk0 = x.racks[0];
      prk1 = x.racks[1];
      prk2 = x.racks[2];
      prk3 = x.racks[3];
      prk4 = x.racks[4];
      prk5 = x.racks[5];
      prk6 = x.racks[6];
      prk7 = x.racks[7];
    }
    const int si = ov.broker(src);
    if (si >= 0) {
      const BrokerRow& x = ov.b[si];
      aSrc = x.alive != 0;
      snrep = x.nrep;
      sbu0 = x.util[0];
      sbu1 = x.util[1];
      sbu2 = x.util[2];
      sbu3 = x.util[3];
      snlead = x.nlead;
      spot = x.potNwOut;
      slbi = x.leadNwIn;
    }
    aliveBits = (aliveBits & 4u) | (aSrc ? 1u : 0u);
    inelig = false;
    if (t.pIneligOff)  // uniform: only models with BAD_DISKS brokers carry the table
      for (int k = t.pIneligOff[p]; k < t.pIneligOff[p + 1]; ++k) inelig |= t.pIneligB[k] == dst;
    if (prog.needs & NEED_TOPIC) {
      tup = t.tUpper[topic];
      tlo = t.tLower[topic];
      stc = t.topicCount[(size_t)topic * t.ldB + src];
      dtc = t.topicCount[(size_t)topic * t.ldB + dst];
    }
    if (prog.needs & NEED_TLEAD) {
      tmn = t.tMinLead ? t.tMinLead[topic] : -1;
      stl = t.topicLead[(size_t)topic * t.ldB + src];
      dtl = t.topicLead[(size_t)topic * t.ldB + dst];
    }
    if (prog.needs & NEED_TLLIM) {
      const int2 lim = reinterpret_cast<const int2*>(t.tLeadLim)[topic];
      tlu = lim.x;
      tll = lim.y;
    }
  }
  // A row whose broker, partition and topic the host sent (RowRef): every record load is independent.
  __device__ __forceinline__ void loadRowRef(const DevTables& t, const DevProgram& prog, const RowRef x,
                                             const OverlayLds& ov) {
    r = x.r;
    src = x.src;
    p = x.p;
    topic = x.topic;
    const ReplicaRec& rec = t.replicas[r];
    orig = rec.orig;
    rflags = rec.flags;
    rbs = rec.bset;
    ru0 = rec.util[0];
    ru1 = rec.util[1];
    ru2 = rec.util[2];
    ru3 = rec.util[3];
    const int ri = ov.replica(r);
    if (ri >= 0) {
      const ReplicaRow& y = ov.r[ri];
      rflags = y.flags;
      ru0 = y.util[0];
      ru1 = y.util[1];
      ru2 = y.util[2];
      ru3 = y.util[3];
    }
    setPartition(t.parts[p]);
    const BrokerRec& sb = t.brokers[src];
    bool aSrc = sb.alive != 0;
    snrep = sb.nrep;
    sbu0 = sb.util[0];
    sbu1 = sb.util[1];
    sbu2 = sb.util[2];
    sbu3 = sb.util[3];
    snlead = sb.nlead;
    spot = sb.pot;
    slbi = sb.lbi;
    scap0 = sb.cap[0];
    scap1 = sb.cap[1];
    scap2 = sb.cap[2];
    scap3 = sb.cap[3];
    srcAllowed = sb.allowedBits;
    sbs = sb.bset;
    loadSrcHost(t, sb, ov);
    if (prog.needs & NEED_TOPIC) {
      tup = t.tUpper[topic];
      tlo = t.tLower[topic];
      stc = t.topicCount[(size_t)topic * t.ldB + src];
      dtc = t.topicCount[(size_t)topic * t.ldB + dst];
    }
    if (prog.needs & NEED_TLEAD) {
      tmn = t.tMinLead ? t.tMinLead[topic] : -1;
      stl = t.topicLead[(size_t)topic * t.ldB + src];
      dtl = t.topicLead[(size_t)topic * t.ldB + dst];
    }
    if (prog.needs & NEED_TLLIM) {
      const int2 lim = reinterpret_cast<const int2*>(t.tLeadLim)[topic];
      tlu = lim.x;
      tll = lim.y;
    }
    inelig = false;
    if (t.pIneligOff)  // uniform: only models with BAD_DISKS brokers carry the table
      for (int k = t.pIneligOff[p]; k < t.pIneligOff[p + 1]; ++k) inelig |= t.pIneligB[k] == dst;
    const int pi = ov.partition(p);
    if (pi >= 0) {
      const PartitionRow& y = ov.p[pi];
      pn = y.n;
      pb0 = y.brokers[0];
      pb1 = y.brokers[1];
      pb2 = y.brokers[2];
      pb3 = y.brokers[3];
      pb4 = y.brokers[4];
      pb5 = y.brokers[5];
      pb6 = y.brokers[6];
      pb7 = y.brokers[7];
      plno = y.leadNwOut;
      prk0 = y.racks[0];
      prk1 = y.racks[1];
      prk2 = y.racks[2];
      prk3 = y.racks[3];
      prk4 = y.racks[4];
      prk5 = y.racks[5];
      prk6 = y.racks[6];
      prk7 = y.racks[7];
    }
    const int si = ov.broker(src);
    if (si >= 0) {
      const BrokerRow& y = ov.b[si];
      aSrc = y.alive != 0;
      snrep = y.nrep;
      sbu0 = y.util[0];
      sbu1 = y.util[1];
      sbu2 = y.util[2];
      sbu3 = y.util[3];
      snlead = y.nlead;
      spot = y.potNwOut;
      slbi = y.leadNwIn;
    }
    aliveBits = (aliveBits & 4u) | (aSrc ? 1u : 0u);
  }
  // The source broker's host values (src is set; a dirty source row in the overlay wins)
  __device__ __forceinline__ void loadSrcHost(const DevTables& t, const BrokerRec& sb, const OverlayLds& ov) {
    hmode = t.hostCap != nullptr;
    if (!hmode) return;  // uniform per launch
    const int si = ov.broker(src);
    shu = si >= 0 ? ov.b[si].hutil : sb.hutil;
  }
  // The destination side, loaded BEFORE the row (it depends only on the destination id); the destination's
  // topic count needs the row's topic and is read in loadRow.
  __device__ __forceinline__ void loadDst(const DevTables& t, int d, const OverlayLds& ov) {
    dst = d;
    const BrokerRec& db = t.brokers[d];
    bool aDst = db.alive != 0;
    dnrep = db.nrep;
    dbu0 = db.util[0];
    dbu1 = db.util[1];
    dbu2 = db.util[2];
    dbu3 = db.util[3];
    dnlead = db.nlead;
    dpot = db.pot;
    dlbi = db.lbi;
    dcap0 = db.cap[0];
    dcap1 = db.cap[1];
    dcap2 = db.cap[2];
    dcap3 = db.cap[3];
    drack = db.rack;
    dAllowed = db.allowedBits;
    dbs = db.bset;
    const int di = ov.broker(d);
    if (di >= 0) {
      const BrokerRow& x = ov.b[di];
      aDst = x.alive != 0;
      dnrep = x.nrep;
      dbu0 = x.util[0];
      dbu1 = x.util[1];
      dbu2 = x.util[2];
      dbu3 = x.util[3];
      dnlead = x.nlead;
      dpot = x.potNwOut;
      dlbi = x.leadNwIn;
    }
    aliveBits = aDst ? 4u : 0u;
    hmode = t.hostCap != nullptr;
    if (hmode) {  // uniform per launch
      dhu = di >= 0 ? ov.b[di].hutil : db.hutil;
      hcapT = t.hostCap;
    }
  }
  __device__ __forceinline__ double bu(int b, int k) const {
    return b == dst ? sel(k, dbu0, dbu1, dbu2, dbu3) : sel(k, sbu0, sbu1, sbu2, sbu3);
  }
  __device__ __forceinline__ double bcap(int b, int k) const {
    return b == dst ? sel(k, dcap0, dcap1, dcap2, dcap3) : sel(k, scap0, scap1, scap2, scap3);
  }
  __device__ __forceinline__ bool hostMode() const { return hmode; }
  __device__ __forceinline__ double hu(int b, int k) const {  // k < 3 (host resources)
    if (!hmode) return bu(b, k);
    return (b == dst ? dhu : shu)[k];
  }
  __device__ __forceinline__ double hcap(int b, int k) const {
    if (!hmode) return bcap(b, k);
    return hcapT[3 * (size_t)(b == dst ? dst : src) + k];
  }
  __device__ __forceinline__ int nrep(int b) const { return b == dst ? dnrep : snrep; }
  // asked for src and dst only (the original broker's liveness is folded into origOff)
  __device__ __forceinline__ bool alive(int b) const { return (aliveBits & (b == dst ? 4u : 1u)) != 0; }
  __device__ __forceinline__ bool allowed(int slot, int /*b == src*/) const { return (srcAllowed >> slot) & 1u; }
  __device__ __forceinline__ double ru(int /*r*/, int k) const { return sel(k, ru0, ru1, ru2, ru3); }
  __device__ __forceinline__ int flags(int) const { return rflags; }
  __device__ __forceinline__ int rbroker(int) const { return src; }
  __device__ __forceinline__ int rorig(int) const { return orig; }
  __device__ __forceinline__ bool origOff(int) const { return (rflags & (RF_ORIG_OFFLINE | RF_ORIG_DEAD)) != 0; }
  __device__ __forceinline__ int rpart(int) const { return p; }
  __device__ __forceinline__ bool hosts(int /*p*/, int b) const {
    return (pb0 == b) | (pb1 == b) | (pb2 == b) | (pb3 == b) | (pb4 == b) | (pb5 == b) | (pb6 == b) | (pb7 == b);
  }
  __device__ __forceinline__ int rack(int /*b == dst*/) const { return drack; }
  __device__ __forceinline__ bool ineligible(int /*p*/, int /*b == dst*/) const { return inelig; }
  // GoalUtils.eligibleBrokers' replica-dependent filters: filterOutBrokersExcludedForLeadership for a leader
  // replica's move (GoalUtils.java:170-180), and with NEW brokers only new brokers or the replica's original broker
  // (:193-198)
  __device__ __forceinline__ bool exclLeadBlocked(const DevProgram& prog) const {
    if (prog.exclLeadMove && (rflags & RF_LEADER) && ((dAllowed >> kExclLeadBit) & 1u)) return true;
    return prog.newOnly && !((dAllowed >> kNewBit) & 1u) && dst != orig;
  }
  __device__ __forceinline__ bool otherOnRack(int /*p*/, int self, int rk) const {
    return (pb0 >= 0 && pb0 != self && prk0 == rk) | (pb1 >= 0 && pb1 != self && prk1 == rk) |
           (pb2 >= 0 && pb2 != self && prk2 == rk) | (pb3 >= 0 && pb3 != self && prk3 == rk) |
           (pb4 >= 0 && pb4 != self && prk4 == rk) | (pb5 >= 0 && pb5 != self && prk5 == rk) |
           (pb6 >= 0 && pb6 != self && prk6 == rk) | (pb7 >= 0 && pb7 != self && prk7 == rk);
  }
  // rack of the partition's slot on broker b (b hosts the partition: the replica's own broker)
  // (exactly one slot holds b; every term selects a value against a constant, so the compiler cannot turn the
  // chain into a select of field addresses — that would keep the whole view in scratch memory)
  __device__ __forceinline__ int slotRack(int /*p*/, int b) const {
    return (pb0 == b ? prk0 : 0) | (pb1 == b ? prk1 : 0) | (pb2 == b ? prk2 : 0) | (pb3 == b ? prk3 : 0) |
           (pb4 == b ? prk4 : 0) | (pb5 == b ? prk5 : 0) | (pb6 == b ? prk6 : 0) | (pb7 == b ? prk7 : 0);
  }
  __device__ __forceinline__ int rackCount(int /*p*/, int rk) const {
    return (pb0 >= 0 && prk0 == rk) + (pb1 >= 0 && prk1 == rk) + (pb2 >= 0 && prk2 == rk) + (pb3 >= 0 && prk3 == rk) +
           (pb4 >= 0 && prk4 == rk) + (pb5 >= 0 && prk5 == rk) + (pb6 >= 0 && prk6 == rk) + (pb7 >= 0 && prk7 == rk);
  }
  __device__ __forceinline__ int nlead(int b) const { return b == dst ? dnlead : snlead; }
  __device__ __forceinline__ double pot(int b) const { return b == dst ? dpot : spot; }
  __device__ __forceinline__ double lnwin(int b) const { return b == dst ? dlbi : slbi; }
  __device__ __forceinline__ double pLeadNwOut(int) const { return plno; }
  __device__ __forceinline__ int ptopic(int) const { return topic; }
  __device__ __forceinline__ int tcount(int, int b) const { return b == dst ? dtc : stc; }
  __device__ __forceinline__ int tUpper(int) const { return tup; }
  __device__ __forceinline__ int tLower(int) const { return tlo; }
  __device__ __forceinline__ int bset(int b) const { return b == dst ? dbs : sbs; }
  __device__ __forceinline__ int rbset(int) const { return rbs; }
  __device__ __forceinline__ int tlead(int, int b) const { return b == dst ? dtl : stl; }
  __device__ __forceinline__ int tMinLead(int) const { return tmn; }
  __device__ __forceinline__ int tLeadUpper(int) const { return tlu; }
  __device__ __forceinline__ int tLeadLower(int) const { return tll; }

  // RackAwareGoal.rackAwareEligibleBrokers: the destination's rack is not in the partition's rack list with
  // one occurrence of the replica's own rack removed (RackAwareGoal.java:193-211).
  __device__ __forceinline__ bool rackEligible() const {
    int srk = -1;
    if (pb0 == src) srk = prk0;
    else if (pb1 == src) srk = prk1;
    else if (pb2 == src) srk = prk2;
    else if (pb3 == src) srk = prk3;
    else if (pb4 == src) srk = prk4;
    else if (pb5 == src) srk = prk5;
    else if (pb6 == src) srk = prk6;
    else if (pb7 == src) srk = prk7;
    int cnt = 0;
    cnt += (pb0 >= 0 && prk0 == drack);
    cnt += (pb1 >= 0 && prk1 == drack);
    cnt += (pb2 >= 0 && prk2 == drack);
    cnt += (pb3 >= 0 && prk3 == drack);
    cnt += (pb4 >= 0 && prk4 == drack);
    cnt += (pb5 >= 0 && prk5 == drack);
    cnt += (pb6 >= 0 && prk6 == drack);
    cnt += (pb7 >= 0 && prk7 == drack);
    if (srk == drack) cnt -= 1;
    return cnt == 0;
  }
};

constexpr int kBlock = 256;
constexpr uint32_t kXcds = 8;                // MI355X: 8 XCDs, each with its own L2
// Scans with at least this many destination columns are XCD-sliced (narrower scans keep the plain k-major tiling).
// CCMI_XCD_SLICE_MIN_COLS overrides it (diagnostics and the parity tests that force slicing on small clusters).
static uint32_t xcdSliceMinCols() {
  static const uint32_t v = [] {
    const char* e = std::getenv("CCMI_XCD_SLICE_MIN_COLS");
    const unsigned long x = e ? std::strtoul(e, nullptr, 10) : 0ul;
    return x ? (uint32_t)x : 2048u;
  }();
  return v;
}

// The slicing rule, for the scan server's host side (device.cpp)
uint32_t scanXcdSliceMinCols() { return xcdSliceMinCols(); }

// Diagnostics: workgroup 0 / thread 0 records s_memrealtime (100 MHz) at fixed points of a launch.
#define CCMI_STAMP(T, seq, i)                                                                         \
  do {                                                                                               \
    if ((T).stamps && blockIdx.x == 0 && threadIdx.x == 0) {                                          \
      __builtin_amdgcn_s_waitcnt(0); /* outstanding loads of this lane land before the stamp */        \
      (T).stamps[((seq)&1023ull) * 8 + (i)] = __builtin_amdgcn_s_memrealtime();                       \
    }                                                                                                 \
  } while (0)
// Scan-server phase stamps (CCMI_STAMPS): workgroup 0's thread 0 notes when it saw a command (0), had it copied (1),
// was ready for its first tile (2), finished its first tile (3, rows staged with it) and arrived (4); the deltas are
// summed at stamps[8192 + i].
#define SRV_STAMP(T, i)                                                                               \
  do {                                                                                               \
    if ((T).stamps && blockIdx.x == 0 && threadIdx.x == 0) {                                          \
      __builtin_amdgcn_s_waitcnt(0);                                                                  \
      srvT[i] = __builtin_amdgcn_s_memrealtime();                                                     \
    }                                                                                                 \
  } while (0)
constexpr unsigned long long kNone = ~0ull;
// Register budgets. A candidate's view (PreView: the replica, partition and both brokers' fields) has to stay in
// VGPRs — a spilled view sends every predicate operand through scratch. The server and the one-workgroup chains
// run one workgroup (4 waves) per CU, so one wave per SIMD and the whole register file; the launched scans keep two.
constexpr int kServerWaves = 1;
constexpr int kScanWaves = 2;

__device__ __forceinline__ unsigned long long waveMin(unsigned long long v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    unsigned long long o = __shfl_xor(v, off, 64);
    v = o < v ? o : v;
  }
  return v;
}

__device__ __forceinline__ unsigned long long blockMin(unsigned long long v) {
  __shared__ unsigned long long part[kBlock / 64];
  v = waveMin(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) part[wave] = v;
  __syncthreads();
  unsigned long long r = part[0];
#pragma unroll
  for (int w = 1; w < kBlock / 64; ++w) r = part[w] < r ? part[w] : r;
  __syncthreads();
  return r;
}

// Current best key, read once per block so the early exit is uniform across the block's waves.
__device__ __forceinline__ unsigned long long blockBest(const unsigned long long* result) {
  __shared__ unsigned long long sBest;
  if (threadIdx.x == 0) sBest = __hip_atomic_load(result, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const unsigned long long b = sBest;
  __syncthreads();
  return b;
}

// First accepted candidate slot of a scan-server tile, or -1. The block's waves form kBlock / 64 / parts groups of
// `parts` waves; group g evaluates slots [64 g, 64 g + 64), each of its waves a share of the goals, and a slot is
// accepted when every wave of its group accepted it (parts = 1: every wave is its own group). Slots are in key order.
__device__ __forceinline__ int tileFirst(bool ok, int parts) {
  __shared__ unsigned long long sBal[kBlock / 64];
  const unsigned long long bal = __ballot(ok);
  if ((threadIdx.x & 63) == 0) sBal[threadIdx.x >> 6] = bal;
  __syncthreads();
  int first = -1;
  const int groups = (kBlock / 64) / parts;
  for (int g = 0; g < groups; ++g) {
    unsigned long long pass = ~0ull;
    for (int p = 0; p < parts; ++p) pass &= sBal[g * parts + p];
    if (pass) {
      first = g * 64 + __builtin_ctzll(pass);
      break;
    }
  }
  __syncthreads();
  return first;
}

// The accept mask of a scan-server tile's first group (slots 0..63): the AND of its `parts` waves' ballots.
__device__ __forceinline__ unsigned long long tileMask(bool ok, int parts) {
  __shared__ unsigned long long sBalM[kBlock / 64];
  const unsigned long long bal = __ballot(ok);
  if ((threadIdx.x & 63) == 0) sBalM[threadIdx.x >> 6] = bal;
  __syncthreads();
  unsigned long long pass = ~0ull;
  for (int p = 0; p < parts; ++p) pass &= sBalM[p];
  __syncthreads();
  return pass;
}

// Last-arriver publish: every workgroup arrives once (after its final atomicMin); the last one reads the
// winning key and writes ONE 64-bit word {seq:32 | key+1:32} (0 in the low half = no winner) to the host
// mailbox — a single aligned 8-byte store, so the host never sees a sequence number without its key and
// no system-scope fence (an L2 writeback) is needed. Keys of cross/pair scans are < 2^31 (host-checked).
__device__ __forceinline__ void publishLast(unsigned long long* __restrict__ result, unsigned int* __restrict__ done,
                                            unsigned long long* __restrict__ mail, unsigned long long seq) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // this workgroup's atomicMin before its arrival
    const unsigned int prev = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      const unsigned long long v = __hip_atomic_load(&result[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long lo = v == kNone ? 0ull : (v + 1) & 0xffffffffull;
      result[0] = kNone;  // self-cleaning: the next scan starts from a reset result and counter
      *done = 0;
      __hip_atomic_store(&mail[0], ((seq & 0xffffffffull) << 32) | lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// Rows reps[0, K) x candidate columns [c0, c0 + Nr) of an N-column candidate list; key = k * N + c0 + jj. A sharded
// session scans only its own column range; keys stay global, so a MIN over shards is the global first fit.
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, kScanWaves))) void scan_cross(DevTables T, MutTables Mt, UpdateList U, DevProgram prog,
                                                     const RowRef* __restrict__ reps,
                                                     const int32_t* __restrict__ cands, int K, int Nr, int N, int c0,
                                                     int sliced, unsigned long long* __restrict__ result,
                                                     unsigned int* __restrict__ done,
                                                     unsigned long long* __restrict__ mail, unsigned long long seq) {
  __shared__ OverlayLds ov;
  CCMI_STAMP(T, seq, 0);
  bool staged = false;
  // XCD-sliced tiling for wide scans: workgroups are dispatched round-robin over the 8 XCDs, so workgroup w
  // (XCD w % 8) sweeps only destination columns [s*W, s*W + Ws) of slice s = w % 8, k-major within the slice.
  // Each XCD's L2 then holds 1/8 of the destination broker records instead of all of them. Keys stay global
  // and increase along every workgroup's tile sequence, so the early exits below remain exact. The launcher
  // decides (`sliced`) and then guarantees gridDim.x % kXcds == 0.
  uint32_t colStart = 0, Ws = (uint32_t)Nr, wg = blockIdx.x, wgs = gridDim.x;
  if (sliced) {
    const uint32_t W = ((uint32_t)Nr + kXcds - 1) / kXcds;
    const uint32_t sl = blockIdx.x % kXcds;
    colStart = sl * W;
    Ws = colStart < (uint32_t)Nr ? min(W, (uint32_t)Nr - colStart) : 0u;
    wg = blockIdx.x / kXcds;
    wgs = gridDim.x / kXcds;
  }
  const uint32_t total = (uint32_t)K * Ws;
  for (uint32_t base = wg * kBlock; base < total; base += wgs * kBlock) {
    const uint32_t kb = base / Ws;
    const unsigned long long keyBase = (unsigned long long)kb * N + c0 + colStart + (base - kb * Ws);
    if (blockBest(result) <= keyBase) break;  // an earlier pair already won: nothing later can (block-uniform)
    // the request's indices (host-mapped) are read before the overlay is staged: both round trips overlap
    const uint32_t q = base + threadIdx.x;
    const uint32_t k = q / Ws;
    const uint32_t j = colStart + (q - k * Ws);
    RowRef rq{0, 0, 0, 0};
    int dq = 0;
    if (q < total) {
      rq = reps[k];
      dq = cands[j];
    }
    if (!staged) {
      overlayStage(ov, U);
      overlayApply(ov, U, Mt, T);
      staged = true;
      CCMI_STAMP(T, seq, 1);
    }
    unsigned long long local = kNone;
    if (q < total) {
      PreView v;
      v.loadDst(T, dq, ov);
      v.loadRowRef(T, prog, rq, ov);
      CCMI_STAMP(T, seq, 6);  // the view's loads landed (diagnostics split loads from predicate time)
      const bool inList = (prog.filter != FILTER_RACK_AWARE || v.rackEligible()) && !v.exclLeadBlocked(prog);
      if (inList && moveCandidateAccepted(prog, v, v.r, v.dst)) local = (unsigned long long)k * N + c0 + j;
    }
    CCMI_STAMP(T, seq, 2);
    const unsigned long long m = blockMin(local);
    CCMI_STAMP(T, seq, 3);
    if (m != kNone) {
      if (threadIdx.x == 0) atomicMin(result, m);
      break;
    }
  }
  CCMI_STAMP(T, seq, 4);
  publishLast(result, done, mail, seq);
  CCMI_STAMP(T, seq, 5);
}

// ------------------------------------------------------------------------------------------------ scan server
// K8 scan_server: ONE persistent launch serves a stream of cross / pair scans. The host writes each command (rows,
// program, request arrays, then the sequence word behind a store fence) into fine-grained VRAM that the CPU writes
// through the BAR; every workgroup polls the sequence word, evaluates its tiles exactly as scan_cross / scan_pairs
// do, and the last workgroup to arrive publishes {seq, key} to the host mailbox. No launch and no PCIe read of the
// request per scan. Everything the host wrote is read with system-scope loads (never from a cache line of an earlier
// command); workgroup 0 writes the command's dirty rows to HBM and releases them before it arrives, and every
// workgroup takes an agent-scope acquire when it sees the next command (MI355X_MICROARCH.md, inter-workgroup
// visibility). The launch exits on SOP_EXIT or after kServerIdleTicks without a command (watchdog; the host stops the
// server before any other work on the session stream and at the end of every API call, so it never relies on it).
__device__ __forceinline__ int32_t ldSys(const int32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// Up to three [src, src + words) -> dst copies in one pass: every thread issues its system-scope loads (at most
// kCopyBatch per thread per pass) before it stores any, so a command's tables cost one memory round trip, not one
// per word a thread copies.
constexpr int kCopyBatch = 12;
__device__ __forceinline__ void copySys3(int32_t* d0, const int32_t* s0, int n0, int32_t* d1, const int32_t* s1,
                                         int n1, int32_t* d2, const int32_t* s2, int n2) {
  const int total = n0 + n1 + n2;
  for (int base = 0; base < total; base += kBlock * kCopyBatch) {
    int32_t v[kCopyBatch];
#pragma unroll
    for (int u = 0; u < kCopyBatch; ++u) {
      const int w = base + u * kBlock + (int)threadIdx.x;
      if (w < n0) v[u] = ldSys(s0 + w);
      else if (w < n0 + n1) v[u] = ldSys(s1 + (w - n0));
      else if (w < total) v[u] = ldSys(s2 + (w - n0 - n1));
    }
#pragma unroll
    for (int u = 0; u < kCopyBatch; ++u) {
      const int w = base + u * kBlock + (int)threadIdx.x;
      if (w < n0) d0[w] = v[u];
      else if (w < n0 + n1) d1[w - n0] = v[u];
      else if (w < total) d2[w - n0 - n1] = v[u];
    }
  }
}
__device__ __forceinline__ void copySys(void* dst, const void* src, int bytes) {  // whole 32-bit words, all threads
  copySys3(reinterpret_cast<int32_t*>(dst), reinterpret_cast<const int32_t*>(src), bytes / 4, nullptr, nullptr, 0,
           nullptr, nullptr, 0);
}
__device__ __forceinline__ RowRef ldSysRow(const int32_t* p) {  // four independent system-scope loads
  return RowRef{ldSys(p), ldSys(p + 1), ldSys(p + 2), ldSys(p + 3)};
}
template <class X>
__device__ __forceinline__ void copySysOneThread(X* dst, const X* src) {  // all loads issued, then the stores
  static_assert(sizeof(X) % 4 == 0, "whole words");
  constexpr int n = (int)(sizeof(X) / 4);
  int32_t v[n];
#pragma unroll
  for (int w = 0; w < n; ++w) v[w] = ldSys(reinterpret_cast<const int32_t*>(src) + w);
#pragma unroll
  for (int w = 0; w < n; ++w) reinterpret_cast<int32_t*>(dst)[w] = v[w];
}
constexpr unsigned long long kServerIdleTicks = 200000000ull;  // 2 s of s_memrealtime (100 MHz)
constexpr int kMaskTiles = 4;  // tiles of a shared-goal pair command (ServerCmd.wgParts; the server's mask words)
// scan-server doorbell word: valid and exit flags, nActive (bits 32-61), the command sequence's low 32 bits
constexpr unsigned long long kBellValid = 1ull << 63, kBellExit = 1ull << 62;
constexpr unsigned long long kParkBit = 1ull << 62;  // mail[7]: the server parked after this command (shard groups)

// thread 0's record writes become visible to the whole workgroup (one CU: workgroup scope; the next launch sees them
// through the kernel boundary)
__device__ __forceinline__ void chainSync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// The accepted pair of a chain decision as its evaluating lane saw it (LDS): the apply starts from these instead of
// re-reading the request, the replica record and the partition record (three dependent loads on its critical path).
struct ChainWin {
  int r, dst, src, p, flags;
  int spos, dpos;  // src's and dst's positions in the partition's broker list (-1: not in it)
};

// K7 chain bodies (defined with the chain kernels below; SOP_CHAIN runs them inside the server)
__device__ __forceinline__ void chainPairsRun(const DevTables& T, const ChainTables& C, const DevProgram& prog, const OverlayLds& ov,
                              LoadVec* sc, const RowRef* __restrict__ pr, const int32_t* __restrict__ pb,
                              const int32_t* __restrict__ next, int n, int maxAccepts, int32_t* __restrict__ log,
                              ChainResultDev* __restrict__ out, ChainWin* win);
__device__ __forceinline__ void chainRackRowsRun(const DevTables& T, const ChainTables& C, const DevProgram& prog,
                                 const OverlayLds& ov, LoadVec* sc, const int32_t* __restrict__ rows, int n,
                                 const int32_t* __restrict__ cands, int N, int32_t* __restrict__ log,
                                 ChainResultDev* __restrict__ out);

// The scan server's LDS objects at namespace scope: the kernel and its out-of-line chain body name the same objects
// directly, so no LDS address is passed across the call.
__shared__ OverlayLds gSrvOv;
__shared__ DevProgram gSrvProg;
__shared__ ChainWin gSrvWin;  // a chain decision's winner, from its evaluating lane to the apply
alignas(8) __shared__ unsigned char gSrvScRaw[2 * sizeof(LoadVec)];  // a chain's leadership hand-over (LoadVec has a
                                                                      // member initializer)

// SOP_CHAIN on workgroup 0: the command's rows and the host's load / slot rows into the tables, the request into HBM
// (the chain rereads it per decision), then the chain itself on an empty overlay. Every write of the chain is a plain
// store of this workgroup; the caller releases them (system scope: the log is host-mapped) before the publish.
// Out of line (noinline): the chain bodies (K7 evaluation + apply) are several times the size of the scan paths, and
// inlined they made the server's code ~3.5x larger and its scan commands ~50 % slower on gfx950 (same-box A/B).
__device__ __attribute__((noinline)) void serverChain(const DevTables T, const ChainTables C, const MutTables Mt,
                                                      const ServerCmd c, const char* __restrict__ pay) {
  OverlayLds& ov = gSrvOv;
  const DevProgram& prog = gSrvProg;
  LoadVec* sc = reinterpret_cast<LoadVec*>(gSrvScRaw);
  UpdateList U;
  U.tdel = (const TopicCountDelta*)(pay + c.oT);
  U.nt = c.nt;
  const LoadRow* lrows = (const LoadRow*)(pay + c.oL);
  const SlotRow* srows = (const SlotRow*)(pay + c.oS);
  int32_t* req = reinterpret_cast<int32_t*>(c.chainReq);
  const int32_t* reqIn = reinterpret_cast<const int32_t*>(pay + c.oA);
  // CM_PAIRS request: [RowRef pr[n] | pb[n] | next[n]] (the rows' broker, partition and topic as the host knows them:
  // a leadership chain moves no replica, so they stay valid through the chain); RACK_ROWS: [rows[n] | cands[N]]
  const int words = c.chainMode == CM_PAIRS ? 6 * c.chainN : c.chainN + c.chainM;
  auto putLoad = [&](const LoadRow& x) {
    LoadVec* dst = x.kind == LR_REPLICA ? C.rLoad
                   : (x.kind == LR_BROKER       ? C.bLoad
                      : (x.kind == LR_LEADERSHIP_NW ? C.bLnw : (x.kind == LR_HOST ? C.hLoad : C.bPot)));
    dst[x.id] = x.v;
  };
  auto putSlots = [&](const SlotRow& x) {
    const int o = C.pOff[x.p], n = C.pOff[x.p + 1] - o;
    for (int k = 0; k < n; ++k) C.pSlots[o + k] = x.slots[k];
    C.pLeader[x.p] = x.leader;
  };
  // First pass: each thread's first topic delta, load row, slot row and request words are loaded together (one
  // fine-grained round trip for the lot instead of one per kind), then written; the rare remainders follow.
  {
    const int t = (int)threadIdx.x, nt = (int)blockDim.x;
    TopicCountDelta d;
    LoadRow xl;
    SlotRow xs;
    int32_t w4[4];
    if (t < U.nt) copySysOneThread(&d, &U.tdel[t]);
    if (t < c.nl) copySysOneThread(&xl, &lrows[t]);
    if (t < c.ns) copySysOneThread(&xs, &srows[t]);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (t + k * nt < words) w4[k] = ldSys(reqIn + t + k * nt);
    applyRowsCoherent(Mt, ov.b, ov.nb, ov.r, ov.nr, ov.p, ov.np, threadIdx.x, blockDim.x);
    if (t < U.nt) atomicAdd(&(d.kind ? Mt.topicLead : Mt.topicCount)[(size_t)d.topic * Mt.ldB + d.broker], d.delta);
    if (t < c.nl) putLoad(xl);
    if (t < c.ns) putSlots(xs);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (t + k * nt < words) req[t + k * nt] = w4[k];
  }
  for (int i = threadIdx.x + blockDim.x; i < U.nt; i += blockDim.x) {
    TopicCountDelta d;
    copySysOneThread(&d, &U.tdel[i]);
    atomicAdd(&(d.kind ? Mt.topicLead : Mt.topicCount)[(size_t)d.topic * Mt.ldB + d.broker], d.delta);
  }
  for (int i = threadIdx.x + blockDim.x; i < c.nl; i += blockDim.x) {
    LoadRow x;
    copySysOneThread(&x, &lrows[i]);
    putLoad(x);
  }
  for (int i = threadIdx.x + blockDim.x; i < c.ns; i += blockDim.x) {
    SlotRow x;
    copySysOneThread(&x, &srows[i]);
    putSlots(x);
  }
  for (int w = threadIdx.x + 4 * blockDim.x; w < words; w += blockDim.x) req[w] = ldSys(reqIn + w);
  if (threadIdx.x == 0) ov.nb = ov.nr = ov.np = 0;  // the tables hold the rows now
  __builtin_amdgcn_s_waitcnt(0);
  chainSync();
  int32_t* log = reinterpret_cast<int32_t*>(c.chainLog);
  ChainResultDev* out = reinterpret_cast<ChainResultDev*>(c.chainOut);
  if (c.chainMode == CM_PAIRS)
    chainPairsRun(T, C, prog, ov, sc, reinterpret_cast<const RowRef*>(req), req + 4 * c.chainN, req + 5 * c.chainN,
                  c.chainN, c.maxAccepts, log, out,
                  &gSrvWin);
  else
    chainRackRowsRun(T, C, prog, ov, sc, req, c.chainN, req + c.chainN, c.chainM, log, out);
}

// Shard groups (engine/shard_group.h): this rank's first-fit key into the combine slot with system-scope atomics (the
// block is pinned host memory every device of the process maps), its result tag (the command's sequence, mail[0]),
// and its arrival. No wait: the group's LAST rank to arrive — this workgroup, another rank's server or a rank's host
// thread — publishes the minimum into every rank's mailbox and resets the slot.
__device__ __attribute__((noinline)) void groupArrive(unsigned long long blockAddr, int slot, int rank, int count,
                                                      unsigned long long v, unsigned long long seq) {
  CombineBlock* b = reinterpret_cast<CombineBlock*>(blockAddr);
  CombineSlot* s = &b->slot[slot];
  __hip_atomic_store(&s->tag[rank], kTagServer | (seq & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  unsigned long long cur = __hip_atomic_load(&s->minKey, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  while (v < cur && !__hip_atomic_compare_exchange_weak(&s->minKey, &cur, v, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_SYSTEM)) {
  }
  if (__hip_atomic_fetch_add(&s->arrived, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM) != (unsigned)count - 1) return;
  const unsigned long long g = __hip_atomic_load(&s->minKey, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
  const unsigned long long lo = g == kCombineNone ? 0ull : (g + 1) & 0xffffffffull;
  for (int r = 0; r < count; ++r) {
    const unsigned long long t = __hip_atomic_load(&s->tag[r], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    unsigned long long* mail =
        reinterpret_cast<unsigned long long*>(__hip_atomic_load(&b->mail[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    __hip_atomic_store(&mail[(t >> 62) == 1 ? 0 : 6], ((t & 0xffffffffull) << 32) | lo, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __hip_atomic_store(&s->minKey, kCombineNone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&s->arrived, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, kServerWaves))) void scan_server(DevTables T, MutTables Mt, ChainTables Ch, const ServerCmd* __restrict__ cmd,
                                                      const char* __restrict__ pay, const RowRef* __restrict__ pool,
                                                      unsigned long long* __restrict__ result,
                                                      unsigned int* __restrict__ done,
                                                      unsigned long long* __restrict__ mail,
                                                      unsigned long long* __restrict__ t0,
                                                      unsigned long long* __restrict__ bell,
                                                      unsigned long long startSeq) {
  OverlayLds& ov = gSrvOv;
  DevProgram& prog = gSrvProg;
  __shared__ ServerCmd c;
  __shared__ int sExit;
  __shared__ SegEntry sSeg[kMaxSegs + 1];
  unsigned long long last = startSeq;
  int progVer = -1;
  int acqEpoch = -1;  // ServerCmd.rowsEpoch of this workgroup's last acquire (-1: none since the launch)
  // The acquire an epoch change needs is taken early when possible: once this workgroup's last command is published
  // (the last arriver stores its sequence into pub, a device word beside the doorbell, after every participant's
  // writes completed), the workgroup invalidates its L1 while it idles, so the next command's loads need no acquire
  // of their own (an agent acquire is ~1.7 us of its first tile otherwise, MI355X_MICROARCH.md). acqFresh: no device
  // write was published since that acquire.
  unsigned long long* const pub = bell + 4;
  unsigned long long* const maskWord = t0 + 4;  // a shared-goal pair command's tile accept masks [kMaskTiles] (all ones
                                                // between commands)
  bool acqFresh = false;
  unsigned long long idleSince = __builtin_amdgcn_s_memrealtime();
  bool participated = false;  // this workgroup took part in its last command (thread 0's view)
  bool lastGrouped = false;   // ... and that command was a shard group's scan
  unsigned long long srvT[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // (6: the first tile's request landed, 7: rows staged)
  unsigned long long qBatch = 0, qTiles = 0;  // CCMI_STAMPS, SOP_QUEUE: workgroup 0's batch-loaded stamp and tiles
  for (;;) {
    if (threadIdx.x == 0) {
      int ex = 0;
      // The idle clock starts once this workgroup sees its last command published: until then a workgroup that was
      // dispatched late (the GPU busy with other sessions' kernels) is still working on it and the host is waiting.
      bool published = last == startSeq;
      // Workgroups 0 .. T.directPollers - 1 (8) poll the host-written command word (fine-grained VRAM: every poll is a memory
      // read) and copy the header themselves, so a small command's workgroups all start together; workgroup 0 then
      // rings a doorbell in device memory with the command's {valid, exit, nActive, seq} for the others, which poll it
      // with agent-scope loads the XCD's L2 serves until it changes (MI355X_MICROARCH.md hand-off table: one lane's sc1
      // store, sc1 load polls) — 256 workgroups polling the command word would be most of the server's memory traffic.
      // Only the command's participants copy its header.
      for (int spin = 0;; ++spin) {
        if (!acqFresh && last != startSeq &&
            __hip_atomic_load(pub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == last) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          acqFresh = true;
        }
        if ((uint32_t)blockIdx.x < (uint32_t)T.directPollers) {
          const unsigned long long s = __hip_atomic_load(&cmd->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          const unsigned long long sp = s & ~kSeqAll;
          if (sp != last && !(s & kSeqBusy)) {
            // The host stores the header's other fields, a store fence, then the new sequence (Device::postCommand),
            // so they landed before it did, and it rewrites them only after this command's result — which waits for
            // every participant, so a participant's copy cannot tear. Workgroup 0 always takes part, and so does every
            // direct poller when the word carries kSeqAll: one read suffices. Otherwise (a chain, one participant)
            // another poller may be no participant while the host already rewrites the header for the next command:
            // its copy counts only when the word still reads `s` after it (the seqlock's second read), unless the copy
            // says it does not take part (then it does not, whatever the rest of a torn copy says: a participant's copy
            // cannot tear). T.seqRecheck: the second read always.
            copySysOneThread(&c, cmd);
            c.seq = sp;
            const bool recheck = T.seqRecheck || (blockIdx.x != 0 && !(s & kSeqAll) &&
                                                  (uint32_t)blockIdx.x < (uint32_t)c.nActive);
            if (!recheck || __hip_atomic_load(&cmd->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == s) {
              if (blockIdx.x == 0) {  // the doorbell is for the workgroups past the direct pollers
                const unsigned long long ring = kBellValid | (c.op == SOP_EXIT ? kBellExit : 0ull) |
                                                ((unsigned long long)(uint32_t)c.nActive << 32) | (sp & 0xffffffffull);
                __hip_atomic_store(bell, ring, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              }
              break;
            }
            continue;
          }
        } else {
          const unsigned long long b = __hip_atomic_load(bell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((b & kBellValid) && (b & 0xffffffffull) != (last & 0xffffffffull)) {
            const uint32_t nAct = (uint32_t)(b >> 32) & 0x3fffffffu;
            if ((b & kBellExit) || (uint32_t)blockIdx.x >= nAct) {
              // not taking part (or the exit command): the doorbell says all this workgroup needs
              c.op = (b & kBellExit) ? SOP_EXIT : SOP_CROSS;
              c.nActive = (int32_t)nAct;
              c.seq = b & 0xffffffffull;
              break;
            }
            // a participant: the host rewrites the header only after this command's result, which waits for this
            // workgroup, so one copy is stable
            copySysOneThread(&c, cmd);
            break;
          }
        }
        if ((spin & 63) == 63) {
          if (!published) {
            const unsigned long long mw = __hip_atomic_load(&mail[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if ((mw >> 32) == (last & 0xffffffffull)) {
              published = true;
              idleSince = __builtin_amdgcn_s_memrealtime();
            } else {
              const unsigned long long waited = __builtin_amdgcn_s_memrealtime() - idleSince;
              // A shard group's scan waits for the other ranks' arrivals (shard_group.h). Past T.parkTicks workgroup 0
              // parks the server — it ends the launch so nothing of this device waits behind it (a rank sharing the
              // GPU may need it for a launch of its own) — unless the host has posted a newer command meanwhile: the
              // compare-and-swap on mail[7] (the last posted sequence, which the host moves forward with its own
              // compare-and-swap before every command) decides between the two. The result still arrives in mail[0].
              if (blockIdx.x == 0 && lastGrouped && waited > T.parkTicks) {
                unsigned long long expect = last;
                if (__hip_atomic_compare_exchange_strong(&mail[7], &expect, last | kParkBit, __ATOMIC_ACQ_REL,
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
                  ex = 5;
                  break;
                }
              }
              // a command this workgroup took part in never completed (a participant never arrived), 10 s after this
              // workgroup took it: leave instead of spinning forever
              if (participated && waited > T.stuckTicks) {
                ex = 3;
                break;
              }
              // a non-participant (the command may run as long as it needs: a K7 chain on workgroup 0) or a participant
              // of a parked group scan leaves with workgroup 0's exit record for that command
              const unsigned long long xr = __hip_atomic_load(&mail[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
              if (((xr >> 32) == 3ull || (xr >> 32) == 5ull) && (xr & 0xffffffffull) == (last & 0xffffffffull)) {
                ex = (int)(xr >> 32);
                break;
              }
            }
          } else if (__builtin_amdgcn_s_memrealtime() - idleSince > kServerIdleTicks) {
            ex = 1;
            break;
          }
        }
        // back off once the host has been away for a while (its own phases between commands): fewer polls of the
        // command word from every workgroup, at most ~0.4 us more latency for the command that ends the wait
        if (T.pollMode == 1) continue;
        if (T.pollMode == 2) __builtin_amdgcn_s_sleep(1);
        else if (spin < 256) __builtin_amdgcn_s_sleep(4);
        else __builtin_amdgcn_s_sleep(16);
      }
      SRV_STAMP(T, 0);
      participated = !ex && c.op != SOP_EXIT && (uint32_t)blockIdx.x < (uint32_t)c.nActive;
      lastGrouped = participated && c.combineBlock != 0;
      idleSince = __builtin_amdgcn_s_memrealtime();  // a stuck command is timed from when this workgroup took it
      // the rows workgroup 0 wrote for earlier commands (released before its arrivals) become visible with an agent
      // acquire; a command no earlier one wrote rows before needs none
      if (!ex && (uint32_t)blockIdx.x < (uint32_t)c.nActive) {
        if (acqFresh) {
          acqEpoch = c.rowsEpoch;  // acquired after the previous command's publication: nothing newer to see
        } else if (c.rowsEpoch != acqEpoch) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          acqEpoch = c.rowsEpoch;
        }
      }
      acqFresh = false;  // this command may write (its rows, a chain's moves) before the next one
      SRV_STAMP(T, 1);
      if (blockIdx.x == 0)  // busy-time stamp, read by the last workgroup to arrive
        __hip_atomic_store(t0, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      sExit = ex;
    }
    __syncthreads();
    if (sExit || c.op == SOP_EXIT) {
      // exit record for the host's diagnostics: mail[3] = {reason (1 watchdog, 2 exit command, 3 stuck command, 5 parked
      // waiting for a shard group) : 32 | last seq : 32}
      if (blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_store(&mail[3], ((unsigned long long)(sExit ? sExit : 2) << 32) | (last & 0xffffffffull),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
    const bool rows = (c.nb | c.nr | c.np | c.nt) != 0;
    const uint32_t nAct = (uint32_t)c.nActive;
    if (blockIdx.x >= nAct) {  // not taking part: only the sequence moves on
      last = c.seq;
      __syncthreads();
      continue;
    }
    if (c.progVer != progVer) {
      copySys(&prog, pay + c.oProg, (int)sizeof(DevProgram));
      progVer = c.progVer;
    }
    UpdateList U;
    U.brows = (const BrokerRow*)(pay + c.oB);
    U.rrows = (const ReplicaRow*)(pay + c.oR);
    U.prows = (const PartitionRow*)(pay + c.oP);
    U.tdel = (const TopicCountDelta*)(pay + c.oT);
    U.nb = c.nb;
    U.nr = c.nr;
    U.np = c.np;
    U.nt = c.nt;
    __syncthreads();
    bool staged = false;
    auto stage = [&]() {
      if (threadIdx.x == 0) {
        ov.nb = U.nb;
        ov.nr = U.nr;
        ov.np = U.np;
      }
      copySys3(reinterpret_cast<int32_t*>(ov.b), reinterpret_cast<const int32_t*>(U.brows),
               U.nb * (int)(sizeof(BrokerRow) / 4), reinterpret_cast<int32_t*>(ov.r),
               reinterpret_cast<const int32_t*>(U.rrows), U.nr * (int)(sizeof(ReplicaRow) / 4),
               reinterpret_cast<int32_t*>(ov.p), reinterpret_cast<const int32_t*>(U.prows),
               U.np * (int)(sizeof(PartitionRow) / 4));
      __syncthreads();
      staged = true;
    };
    // The command's rows go into the tables (for the next commands) from the last active workgroup, which has the
    // fewest tiles (none on a short command), so the row writes run next to workgroup 0's tiles instead of after
    // them; every workgroup stages the rows into its LDS overlay with its first tile (overlapping that tile's
    // request loads).
    const bool writer = blockIdx.x == nAct - 1;
    SRV_STAMP(T, 2);
    bool firstTile = true;
    const int32_t* A = (const int32_t*)(pay + c.oA);
    const int32_t* C = (const int32_t*)(pay + c.oC);
    if (c.op == SOP_CHAIN) {
      const unsigned long long tc0 = T.stamps ? __builtin_amdgcn_s_memrealtime() : 0;
      stage();
      serverChain(T, Ch, Mt, c, pay);
      if (T.chainDelayTicks) {  // tests: a chain that outlasts a short stuck bound (the other workgroups must wait)
        const unsigned long long t = __builtin_amdgcn_s_memrealtime();
        while (__builtin_amdgcn_s_memrealtime() - t < T.chainDelayTicks) __builtin_amdgcn_s_sleep(8);
      }
      const unsigned long long tc1 = T.stamps ? __builtin_amdgcn_s_memrealtime() : 0;
      // every wave's stores complete, then one system-scope release: the records and loads for the other XCDs' next
      // acquire, the log and result for the host (MI355X_MICROARCH.md, inter-workgroup visibility)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (T.stamps) {  // CCMI_STAMPS, chain commands: [8230] count, [8231] ready -> chain start (rows, request),
                         // [8232] the chain (rows into the tables + decisions), [8233] the release
          const unsigned long long tc2 = __builtin_amdgcn_s_memrealtime();
          atomicAdd(&T.stamps[8230], 1ull);
          atomicAdd(&T.stamps[8231], tc0 - srvT[2]);
          atomicAdd(&T.stamps[8232], tc1 - tc0);
          atomicAdd(&T.stamps[8233], tc2 - tc1);
          atomicAdd(&T.stamps[8234], tc0 - srvT[0]);
        }
      }
    } else if (c.op == SOP_CROSS || c.op == SOP_SEGS) {
      const bool segs = c.op == SOP_SEGS;
      bool segsLoaded = false;
      const int nSegs = c.nSegs;
      const int K = c.K, Nr = c.Nr, N = c.N, c0 = c.c0;
      uint32_t colStart = 0, Ws = (uint32_t)Nr, wg = blockIdx.x, wgs = nAct;
      if (c.sliced) {
        const uint32_t W = ((uint32_t)Nr + kXcds - 1) / kXcds;
        const uint32_t sl = blockIdx.x % kXcds;
        colStart = sl * W;
        Ws = colStart < (uint32_t)Nr ? min(W, (uint32_t)Nr - colStart) : 0u;
        wg = blockIdx.x / kXcds;
        wgs = nAct / kXcds;
      }
      // goal-parallel tiles: `parts` waves per candidate, tile = kBlock / parts candidates (slot = group * 64 + lane)
      const int parts = (c.goalParts == 2 || c.goalParts == 4) ? c.goalParts : 1;
      const uint32_t tile = (uint32_t)(kBlock / parts);
      const int wave = (int)(threadIdx.x >> 6);
      const int part = wave % parts;
      const uint32_t slot = (uint32_t)(wave / parts) * 64u + (threadIdx.x & 63u);
      const uint32_t total = (uint32_t)K * Ws;
      for (uint32_t base = wg * tile; base < total; base += wgs * tile) {
        const uint32_t kb = base / Ws;
        const unsigned long long keyBase = (unsigned long long)kb * N + c0 + colStart + (base - kb * Ws);
        // (the first tile skips the early-exit check: a winner can hardly exist yet, and its round trip would delay
        // the tile's request loads; a superfluous tile only loses to the smaller key in atomicMin)
        if (!firstTile && blockBest(result) <= keyBase) break;
        const uint32_t q = base + slot;
        const uint32_t k = q / Ws;
        const uint32_t j = colStart + (q - k * Ws);
        RowRef rq{0, 0, 0, 0};
        int dq = 0;
        if (segs) {
          if (!segsLoaded) {  // the segment table (written for this command: system-scope loads) into LDS
            copySys(sSeg, A, (nSegs + 1) * (int)sizeof(SegEntry));
            __syncthreads();
            segsLoaded = true;
          }
          if (q < total) {
            int lo = 0, hi = nSegs - 1;  // the last segment starting at or before row k
            while (lo < hi) {
              const int mid = (lo + hi + 1) >> 1;
              if (sSeg[mid].start <= (int)k) lo = mid;
              else hi = mid - 1;
            }
            rq = pool[sSeg[lo].off + (k - (uint32_t)sSeg[lo].start)];  // written before any command read it
            dq = ldSys(C + j);
          }
        } else if (q < total) {
          rq = ldSysRow(A + 4 * (size_t)k);
          dq = ldSys(C + j);
        }
        if (firstTile) SRV_STAMP(T, 6);
        if (!staged) stage();
        if (firstTile) SRV_STAMP(T, 7);
        bool ok = false;
        if (q < total) {
          PreView v;
          v.loadDst(T, dq, ov);
          v.loadRowRef(T, prog, rq, ov);
          if (firstTile) SRV_STAMP(T, 5);  // the first tile's view loads landed
          const bool inList = (prog.filter != FILTER_RACK_AWARE || v.rackEligible()) && !v.exclLeadBlocked(prog);
          ok = inList && moveCandidateAcceptedPart(prog, v, v.r, v.dst, part, parts);
        }
        const int f = tileFirst(ok, parts);
        if (firstTile) {
          SRV_STAMP(T, 3);
          firstTile = false;
        }
        if (T.stamps && threadIdx.x == 0)  // CCMI_STAMPS: pairs evaluated per op ([8220 + op])
          atomicAdd(&T.stamps[8220 + c.op], (unsigned long long)min(tile, total - base));
        if (f >= 0) {  // keys grow with q inside a workgroup's range (row-major over its columns)
          if (threadIdx.x == 0) {
            const uint32_t qf = base + (uint32_t)f, kf = qf / Ws;
            atomicMin(result, (unsigned long long)kf * N + c0 + colStart + (qf - kf * Ws));
          }
          break;
        }
      }
    } else if (c.op == SOP_QUEUE) {
      // Brokers in queue order over the workgroups (entry i on workgroup i % nAct). A workgroup loads the directory
      // entries of all its brokers up front (two fine-grained round trips for the command, not per broker) and walks
      // their rows as ONE range — its brokers' (row, column) pairs back to back, a prefix sum in LDS — in tiles of
      // kBlock / parts slots, so a tile spans several short snapshots. Keys grow with (entry, row, column) along that
      // range, so the early exits keep the first fit exact.
      const int n = c.n, N = c.N, span = c.K, skip0 = c.c0;
      const int parts = (c.goalParts == 2 || c.goalParts == 4) ? c.goalParts : 1;
      const uint32_t tile = (uint32_t)(kBlock / parts);
      const int wave = (int)(threadIdx.x >> 6);
      const int part = wave % parts;
      const uint32_t slot = (uint32_t)(wave / parts) * 64u + (threadIdx.x & 63u);
      const int32_t* Q = (const int32_t*)(pay + c.oA);
      const QueueDirEntry* dir = reinterpret_cast<const QueueDirEntry*>(c.queueDir);
      __shared__ uint32_t sOff[kBlock];        // pool offset of each batch entry's first scanned row
      __shared__ uint32_t sPre[kBlock + 1];    // pair prefix over the batch's entries
      __shared__ int32_t sCand[kBlock];
      const bool candsLds = N <= kBlock;
      if (candsLds && (int)threadIdx.x < N) sCand[threadIdx.x] = ldSys(C + threadIdx.x);
      const int wgI = (int)blockIdx.x;
      const int mine = wgI < n ? (n - wgI + (int)nAct - 1) / (int)nAct : 0;  // entries wgI, wgI + nAct, ...
      bool found = false;
      for (int kb = 0; kb < mine && !found; kb += kBlock) {
        const int nb = mine - kb < kBlock ? mine - kb : kBlock;
        uint32_t cnt = 0;
        if ((int)threadIdx.x < nb) {
          const int i = wgI + (kb + (int)threadIdx.x) * (int)nAct;
          const int b = ldSys(Q + i);
          const unsigned long long e = __hip_atomic_load(reinterpret_cast<const unsigned long long*>(dir + b),
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          const int len = (int)(uint32_t)(e >> 32), r0 = i == 0 ? skip0 : 0;
          cnt = len > r0 ? (uint32_t)(len - r0) * (uint32_t)N : 0u;
          sOff[threadIdx.x] = (uint32_t)(e & 0xffffffffull) + (uint32_t)r0;
        }
        // exclusive prefix of cnt over the block (wave scans, then the wave totals)
        {
          __shared__ uint32_t sWave[kBlock / 64];
          uint32_t x = cnt;
          const int lane = (int)(threadIdx.x & 63u);
#pragma unroll
          for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, (unsigned)d, 64);
            if (lane >= d) x += y;
          }
          if (lane == 63) sWave[threadIdx.x >> 6] = x;
          __syncthreads();
          uint32_t add = 0;
          for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) add += sWave[w];
          sPre[threadIdx.x + 1] = x + add;
          if (threadIdx.x == 0) sPre[0] = 0;
          __syncthreads();
        }
        const uint32_t total = sPre[nb];
        if (T.stamps && blockIdx.x == 0 && threadIdx.x == 0 && kb == 0) qBatch = __builtin_amdgcn_s_memrealtime();
        // this slot's pair of the NEXT tile, loaded while the current one is evaluated (software pipelining of the
        // fine-grained pool reads: a tile's critical path is then its record loads and the conjunction)
        RowRef nextRq{0, 0, 0, 0};
        int nextK = 0;
        bool haveNext = false;
        auto rowAt = [&](uint32_t v, int& k) {  // the pool row of pair v (k: its entry, advanced from the caller's)
          while (k + 1 < nb && sPre[k + 1] <= v) ++k;
          return pool[sOff[k] + (v - sPre[k]) / (uint32_t)N];  // written before any command read it (a ring)
        };
        for (uint32_t base = 0; base < total; base += tile) {
          // the tile's first pair: its key bounds every key of the tile from below
          int kf = 0;
          {
            int lo = 0, hi = nb - 1;  // last entry whose range starts at or before `base`
            while (lo < hi) {
              const int mid = (lo + hi + 1) >> 1;
              if (sPre[mid] <= base) lo = mid;
              else hi = mid - 1;
            }
            kf = lo;
          }
          auto keyOf = [&](int k, uint32_t v) {  // key of pair v of the range, inside batch entry k
            const int i = wgI + (kb + k) * (int)nAct;
            const uint32_t w = v - sPre[k];
            const uint32_t row = (uint32_t)(i == 0 ? skip0 : 0) + w / (uint32_t)N;
            return ((unsigned long long)i * (unsigned long long)span + row) * (unsigned long long)N + w % (uint32_t)N;
          };
          if (!firstTile && blockBest(result) <= keyOf(kf, base)) {
            found = true;  // a smaller key exists: nothing later in this workgroup's range can win
            break;
          }
          const uint32_t v = base + slot;
          RowRef rq{0, 0, 0, 0};
          int dq = 0;
          int k = kf;
          if (v < total) {
            if (haveNext) {
              rq = nextRq;
              k = nextK;
            } else {
              rq = rowAt(v, k);
            }
            const uint32_t w = v - sPre[k];
            dq = candsLds ? sCand[w % (uint32_t)N] : ldSys(C + w % (uint32_t)N);
          }
          haveNext = false;
          if (v + tile < total) {  // the next tile's row of this slot (a tile spans a few entries)
            nextK = k;
            nextRq = rowAt(v + tile, nextK);
            haveNext = true;
          }
          if (!staged) stage();
          bool ok = false;
          if (v < total) {
            PreView pv;
            pv.loadDst(T, dq, ov);
            pv.loadRowRef(T, prog, rq, ov);
            if (firstTile) SRV_STAMP(T, 5);
            ok = !pv.exclLeadBlocked(prog) && moveCandidateAcceptedPart(prog, pv, pv.r, pv.dst, part, parts);
          }
          const int f = tileFirst(ok, parts);
          if (firstTile) {
            SRV_STAMP(T, 3);
            firstTile = false;
          }
          ++qTiles;
          if (T.stamps && threadIdx.x == 0)
            atomicAdd(&T.stamps[8220 + SOP_QUEUE], (unsigned long long)min(tile, total - base));
          if (f >= 0) {
            if (threadIdx.x == (unsigned)(f % 64) + (unsigned)((f / 64) * parts * 64)) atomicMin(result, keyOf(k, v));
            found = true;
            break;
          }
        }
        __syncthreads();  // the batch arrays are rewritten by the next batch
      }
    } else if (c.wgParts > 1) {  // SOP_PAIRS of at most kMaskTiles tiles of 64, each tile's goals shared by wgParts WGs
      // Workgroup w takes tile w / wgParts (slots 64 t .. 64 t + 63 of the pairs, one group of `parts` waves) and share
      // w % wgParts of its goal conjunction, and ANDs its accept mask into the tile's mask word; the last workgroup to
      // arrive takes the first set bit of the first tile (moveCandidateAcceptedPart: the same conjunction whatever the
      // split, and every tile is evaluated, so the first fit is exact).
      const int n = c.n;
      const int parts = (c.goalParts == 2 || c.goalParts == 4) ? c.goalParts : 1;
      const int wave = (int)(threadIdx.x >> 6);
      const int tileI = (int)blockIdx.x / c.wgParts, share = (int)blockIdx.x % c.wgParts;
      const int q = tileI * 64 + (wave / parts) * 64 + (int)(threadIdx.x & 63);
      if (tileI * 64 < n && tileI < kMaskTiles) {
        RowRef rq{0, 0, 0, 0};
        int dq = 0;
        if (q < n) {
          rq = ldSysRow(A + 4 * (size_t)q);
          dq = ldSys(C + q);
        }
        if (!staged) stage();
        bool ok = false;
        if (q < n) {
          PreView v;
          v.loadDst(T, dq, ov);
          v.loadRowRef(T, prog, rq, ov);
          ok = !v.exclLeadBlocked(prog) &&
               moveCandidateAcceptedPart(prog, v, v.r, v.dst, share * parts + wave % parts, c.wgParts * parts);
        }
        const unsigned long long m = tileMask(ok, parts);
        if (firstTile) {
          SRV_STAMP(T, 3);
          firstTile = false;
        }
        if (threadIdx.x == 0 && m != ~0ull)
          __hip_atomic_fetch_and(maskWord + tileI, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    } else {  // SOP_PAIRS
      const int n = c.n, keyBase = c.keyBase;
      const int parts = (c.goalParts == 2 || c.goalParts == 4) ? c.goalParts : 1;
      const int tile = kBlock / parts;
      const int wave = (int)(threadIdx.x >> 6);
      const int part = wave % parts;
      const int slot = (wave / parts) * 64 + (int)(threadIdx.x & 63);
      for (int base = blockIdx.x * tile; base < n; base += (int)nAct * tile) {
        if (!firstTile && blockBest(result) <= (unsigned long long)(keyBase + base)) break;
        const int q = base + slot;
        RowRef rq{0, 0, 0, 0};
        int dq = 0;
        if (q < n) {
          rq = ldSysRow(A + 4 * (size_t)q);
          dq = ldSys(C + q);
        }
        if (firstTile) SRV_STAMP(T, 6);
        if (!staged) stage();
        if (firstTile) SRV_STAMP(T, 7);
        bool ok = false;
        if (q < n) {
          PreView v;
          v.loadDst(T, dq, ov);
          v.loadRowRef(T, prog, rq, ov);
          if (firstTile) SRV_STAMP(T, 5);
          ok = !v.exclLeadBlocked(prog) && moveCandidateAcceptedPart(prog, v, v.r, v.dst, part, parts);
          if (T.conjRepeat)  // diagnostics: the same conjunction again (the part index is opaque to the compiler)
            ok = ok & moveCandidateAcceptedPart(prog, v, v.r, v.dst, part + T.conjRepeat - 1, parts);
        }
        const int f = tileFirst(ok, parts);
        if (firstTile) {
          SRV_STAMP(T, 3);
          firstTile = false;
        }
        if (T.stamps && threadIdx.x == 0)
          atomicAdd(&T.stamps[8220 + SOP_PAIRS], (unsigned long long)min(tile, n - base));
        if (f >= 0) {
          if (threadIdx.x == 0) atomicMin(result, (unsigned long long)(keyBase + base + f));
          break;
        }
      }
    }
    if (firstTile) SRV_STAMP(T, 3);
    // The writer workgroup writes the command's rows into the tables for the next commands (no workgroup reads them
    // from the tables in this one: the LDS overlay has them) after its tiles, with write-through device-scope stores,
    // and applies the topic-count deltas with device-scope atomics.
    if (writer && rows && c.op != SOP_CHAIN) {
      if (!staged) stage();
      applyRowsCoherent(Mt, ov.b, ov.nb, ov.r, ov.nr, ov.p, ov.np, threadIdx.x, blockDim.x);
      for (int i = threadIdx.x; i < U.nt; i += blockDim.x) {
        TopicCountDelta d;
        copySysOneThread(&d, &U.tdel[i]);
        atomicAdd(&(d.kind ? Mt.topicLead : Mt.topicCount)[(size_t)d.topic * Mt.ldB + d.broker], d.delta);
      }
    }
    // arrival: every store and atomic of the command is device-scope, so waiting for them to complete orders them
    // before the arrival (no cache write-back). The last workgroup publishes and resets with device-scope atomics.
    __syncthreads();
    if (threadIdx.x == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned int prev = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (T.stamps && blockIdx.x == 0 && c.op == SOP_QUEUE) {  // queue commands: [8210..8215]
        const unsigned long long tA = __builtin_amdgcn_s_memrealtime();
        const unsigned long long tb = qBatch ? qBatch : srvT[2];
        atomicAdd(&T.stamps[8210], 1ull);
        atomicAdd(&T.stamps[8211], srvT[2] - srvT[0]);
        atomicAdd(&T.stamps[8212], tb - srvT[2]);
        atomicAdd(&T.stamps[8213], srvT[3] > tb ? srvT[3] - tb : 0ull);
        atomicAdd(&T.stamps[8214], tA - (srvT[3] > tb ? srvT[3] : tb));
        atomicAdd(&T.stamps[8215], qTiles);
        qBatch = 0;
        qTiles = 0;
      }
      if (T.stamps && blockIdx.x == 0 && c.op != SOP_CHAIN) {  // scan commands (chains have their own stamps)
        srvT[4] = __builtin_amdgcn_s_memrealtime();
        atomicAdd(&T.stamps[8192 + 0], 1ull);
        for (int i = 0; i < 4; ++i) atomicAdd(&T.stamps[8192 + 1 + i], srvT[i + 1] - srvT[i]);
        if (srvT[5] > srvT[2] && srvT[5] <= srvT[3] && c.op != SOP_PAIRS) {  // cross / segment: ready -> views landed
          atomicAdd(&T.stamps[8197], srvT[5] - srvT[2]);
          atomicAdd(&T.stamps[8198], 1ull);
        }
        // the first tile in four parts, pair commands at [8256..8260], cross commands at [8261..8265]: ready -> the
        // request landed (6), -> rows staged (7), -> view loads landed (5), -> the tile's first slot (3)
        if ((c.op == SOP_PAIRS || c.op == SOP_CROSS) && srvT[2] < srvT[6] && srvT[6] <= srvT[7] && srvT[7] <= srvT[5] &&
            srvT[5] <= srvT[3]) {
          const int o = c.op == SOP_PAIRS ? 8256 : 8261;
          atomicAdd(&T.stamps[o], 1ull);
          atomicAdd(&T.stamps[o + 1], srvT[6] - srvT[2]);
          atomicAdd(&T.stamps[o + 2], srvT[7] - srvT[6]);
          atomicAdd(&T.stamps[o + 3], srvT[5] - srvT[7]);
          atomicAdd(&T.stamps[o + 4], srvT[3] - srvT[5]);
        }
      }
      if (prev == nAct - 1) {
        // the result and workgroup 0's start stamp in one batch of loads (a pair command with shared goals: the first
        // slot its mask word kept, the word reset to all ones)
        unsigned long long v = __hip_atomic_load(&result[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long tStart = __hip_atomic_load(t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (c.op == SOP_PAIRS && c.wgParts > 1) {
          unsigned long long m[kMaskTiles];
          const int tiles = min((c.n + 63) / 64, kMaskTiles);
#pragma unroll
          for (int t = 0; t < kMaskTiles; ++t)
            m[t] = t < tiles ? __hip_atomic_load(maskWord + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
          v = kNone;
#pragma unroll
          for (int t = kMaskTiles - 1; t >= 0; --t)
            if (t < tiles) {
              if (m[t]) v = (unsigned long long)c.keyBase + (unsigned long long)(t * 64 + __builtin_ctzll(m[t]));
              __hip_atomic_store(maskWord + t, ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __hip_atomic_store(&result[0], kNone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long lo = v == kNone ? 0ull : (v + 1) & 0xffffffffull;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned long long busy = __builtin_amdgcn_s_memrealtime() - tStart;
        if (T.stamps && c.op != SOP_CHAIN) {  // CCMI_STAMPS: busy time of scans with / without rows, the writer last
          atomicAdd(&T.stamps[rows ? 8236 : 8238], 1ull);
          atomicAdd(&T.stamps[rows ? 8237 : 8239], busy);
          if (rows && writer) atomicAdd(&T.stamps[8235], 1ull);
        }
        if (c.combineBlock)  // a shard group's scan: the group's last rank publishes mail[0] (shard_group.h)
          groupArrive(c.combineBlock, c.combineSlot, c.combineRank, c.combineCount, v, c.seq);
        else
          __hip_atomic_store(&mail[0], ((c.seq & 0xffffffffull) << 32) | lo, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
        // mail[5]: the command's busy time (100 MHz ticks from workgroup 0 seeing it to the publish, low 40 bits)
        // tagged with the sequence's low 24 bits, stored after the word with no wait in between: the host collects it
        // before its next command (Device::collectServerBusy) instead of the publish waiting for a second PCIe write
        __hip_atomic_store(&mail[5], ((c.seq & 0xffffffull) << 40) | (busy & ((1ull << 40) - 1)), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        // every participant arrived after its writes completed: the idle workgroups may take their acquire now
        __hip_atomic_store(pub, c.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    last = c.seq;
    idleSince = __builtin_amdgcn_s_memrealtime();
    __syncthreads();
  }
}

// One wavefront per row (m, s). rowsPerBlock = kBlock / 64.
// With a SwapLimit the candidate lists are limit-free: rows failing the limit are not candidates (not evaluated,
// not counted), exactly as if the host had filtered them; keys still index the unfiltered list.
__global__ __launch_bounds__(kBlock) void scan_swap(DevTables T, DevProgram prog, const int32_t* __restrict__ srcs, int S,
                                                    const int32_t* __restrict__ cbOff, const int32_t* __restrict__ cbRep,
                                                    int M, SwapLimit lim, unsigned long long* __restrict__ result,
                                                    int32_t* __restrict__ rowVisited) {
  const DevView v{T};
  const int lane = threadIdx.x & 63;
  const int waveInBlock = threadIdx.x >> 6;
  const long long rows = (long long)M * S;
  for (long long row = (long long)blockIdx.x * (kBlock / 64) + waveInBlock; row < rows;
       row += (long long)gridDim.x * (kBlock / 64)) {
    const unsigned long long best = __hip_atomic_load(result, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((best >> 24) < (unsigned long long)row) return;
    const int m = (int)(row / S);
    const int s = (int)(row - (long long)m * S);
    const int sr = srcs[s];
    const int c0 = cbOff[m], c1 = cbOff[m + 1];
    if (c0 == c1) {
      if (lane == 0) rowVisited[row] = 0;
      continue;
    }
    const int db = v.rbroker(cbRep[c0]);  // every row's candidates live on one broker
    if (swapRowExcluded(prog, v, sr, db)) {
      if (lane == 0) rowVisited[row] = 0;
      continue;
    }
    int visited = 0;
    for (int base = c0; base < c1; base += 64) {
      const int idx = base + lane;
      bool in = idx < c1;
      if (in && lim.res >= 0) {
        const double u = v.ru(cbRep[idx], lim.res);
        in = lim.above ? u > lim.limit : u < lim.limit;
      }
      int outcome = 0;
      if (in) outcome = swapCandidateOutcome(prog, v, sr, cbRep[idx], db);
      const unsigned long long passing = __ballot(in);
      const unsigned long long term = __ballot(outcome != 0);
      if (term) {
        const int first = __ffsll((long long)term) - 1;
        const int firstOutcome = __shfl(outcome, first, 64);
        if (firstOutcome == 1 && lane == 0)
          atomicMin(result, ((unsigned long long)row << 24) | (unsigned long long)(base + first - c0));
        visited += __popcll(passing & (first == 63 ? ~0ull : ((2ull << first) - 1)));
        break;
      }
      visited += __popcll(passing);
    }
    if (lane == 0) rowVisited[row] = visited;
  }
}

// Reference-equivalent candidate count of a swap scan: every row before the winning row ran to its first
// terminal (or its end), plus the winning row up to its accepted candidate.
__global__ __launch_bounds__(1024) void swap_visited_sum(const int32_t* __restrict__ rowVisited, long long rows,
                                                         unsigned long long* __restrict__ result,
                                                         unsigned long long* __restrict__ mail, unsigned long long seq) {
  __shared__ long long part[16];
  const unsigned long long best = result[0];
  const long long lim = best == kNone ? rows : (long long)(best >> 24) + 1;
  long long s = 0;
  for (long long i = threadIdx.x; i < lim; i += blockDim.x) s += rowVisited[i];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    long long t = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += part[w];
    result[1] = (unsigned long long)t;
    // rare path (swap scans): values first, then the sequence word behind a system-scope release
    __hip_atomic_store(&mail[1], best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&mail[2], (unsigned long long)t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    result[0] = kNone;
    result[1] = 0;
    __hip_atomic_store(&mail[0], (seq & 0xffffffffull) << 32, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// PAIRS: explicit (replica, broker) list in iteration order (leadership moves: per-replica follower lists).
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, kScanWaves))) void scan_pairs(DevTables T, MutTables Mt, UpdateList U, DevProgram prog,
                                                     const RowRef* __restrict__ pr,
                                                     const int32_t* __restrict__ pb, int n, int keyBase,
                                                     unsigned long long* __restrict__ result,
                                                     unsigned int* __restrict__ done,
                                                     unsigned long long* __restrict__ mail, unsigned long long seq) {
  __shared__ OverlayLds ov;
  CCMI_STAMP(T, seq, 0);
  bool staged = false;
  for (int base = blockIdx.x * kBlock; base < n; base += gridDim.x * kBlock) {
    if (blockBest(result) <= (unsigned long long)(keyBase + base)) break;
    const int q = base + threadIdx.x;
    RowRef rq{0, 0, 0, 0};
    int dq = 0;
    if (q < n) {  // request reads overlap the overlay staging (see scan_cross)
      rq = pr[q];
      dq = pb[q];
    }
    if (!staged) {
      overlayStage(ov, U);
      overlayApply(ov, U, Mt, T);
      staged = true;
      CCMI_STAMP(T, seq, 1);
    }
    unsigned long long local = kNone;
    if (q < n) {
      PreView v;
      v.loadDst(T, dq, ov);
      v.loadRowRef(T, prog, rq, ov);
      if (!v.exclLeadBlocked(prog) && moveCandidateAccepted(prog, v, v.r, v.dst))
        local = (unsigned long long)(keyBase + q);
    }
    CCMI_STAMP(T, seq, 2);
    const unsigned long long m = blockMin(local);
    CCMI_STAMP(T, seq, 3);
    if (m != kNone) {
      if (threadIdx.x == 0) atomicMin(result, m);
      break;
    }
  }
  CCMI_STAMP(T, seq, 4);
  publishLast(result, done, mail, seq);
  CCMI_STAMP(T, seq, 5);
}

// ------------------------------------------------------------------------------------------------ chains
// K7: first-fit decisions applied on the device, one after the other, inside ONE launch. One workgroup: every
// decision evaluates the remaining candidates in blocks of kBlock (first accepted = block minimum), thread 0 applies
// the winning move to the device records and loads (apply.h, the host model's exact arithmetic), and the workgroup
// continues with the state the next decision of the reference loop would see. The host replays the logged moves
// into its own model afterwards.
template <int WC>  // WC > 0: the window count as a compile-time constant (the lanes' copies stay in registers)
struct DevApply {
  ChainTables c;
  LoadVec* sc;  // two LoadVecs in LDS: the leadership steps' hand-over
  static constexpr int W = WC;
  __device__ __forceinline__ LoadVec& rLoad(int r) { return c.rLoad[r]; }
  __device__ __forceinline__ LoadVec& bLoad(int b) { return c.bLoad[b]; }
  __device__ __forceinline__ LoadVec& bLnw(int b) { return c.bLnw[b]; }
  __device__ __forceinline__ LoadVec& bPot(int b) { return c.bPot[b]; }
  __device__ __forceinline__ LoadVec& scratch(int i) { return sc[i]; }
  __device__ __forceinline__ ReplicaRec& rep(int r) { return c.replicas[r]; }
  __device__ __forceinline__ BrokerRec& brk(int b) { return c.brokers[b]; }
  __device__ __forceinline__ PartitionRec& part(int p) { return c.parts[p]; }
  __device__ __forceinline__ int& slot(int p, int i) { return c.pSlots[c.pOff[p] + i]; }
  __device__ __forceinline__ int& leader(int p) { return c.pLeader[p]; }
  __device__ __forceinline__ void topicAdd(int t, int b, int d) { c.topicCount[(size_t)t * c.ldB + b] += d; }
  __device__ __forceinline__ void topicLeadAdd(int t, int b, int d) {
    if (c.topicLead) c.topicLead[(size_t)t * c.ldB + b] += d;
  }
  __device__ __forceinline__ bool hostsOn() const { return c.hLoad != nullptr; }
  __device__ __forceinline__ int host(int b) const { return c.bHost[b]; }
  __device__ __forceinline__ LoadVec& hLoad(int h) { return c.hLoad[h]; }
  __device__ __forceinline__ int hostBegin(int h) const { return c.hOff[h]; }
  __device__ __forceinline__ int hostEnd(int h) const { return c.hOff[h + 1]; }
  __device__ __forceinline__ int hostBroker(int i) const { return c.hBrk[i]; }
};


// The finish fields of a replica move (apply.h finish lanes) spread over waves 1..3 — a wave runs only lanes that take
// the same code path (the source and destination sides by address), so no wave serializes divergent paths of loads:
//   wave 1 lanes 0/1: broker counts of src / dst; 2/3: topic counts; 4/5: topic leader counts
//   wave 2 lane 0: the replica's broker;   wave 3 lane 0: its partition slot
template <class S>
__device__ __forceinline__ void replicaFinishWaves(S& s, int t, int r, int p, int src, int dst, bool lead) {
  const int w = t >> 6, l = t & 63;
  if (w == 1 && l < 2) {
    BrokerRec& b = s.brk(l == 0 ? src : dst);
    b.nrep += l == 0 ? -1 : 1;
    if (lead) b.nlead += l == 0 ? -1 : 1;
  } else if (w == 1 && l < 4) {
    s.topicAdd(s.part(p).topic, l == 2 ? src : dst, l == 2 ? -1 : 1);
  } else if (w == 1 && l < 6) {
    if (lead) s.topicLeadAdd(s.part(p).topic, l == 4 ? src : dst, l == 4 ? -1 : 1);
  } else if (w == 2 && l == 0) {
    applyReplicaFinishLane(s, 2, r, p, src, dst, lead);  // the replica's broker
  } else if (w == 3 && l == 0) {
    applyReplicaFinishLane(s, 3, r, p, src, dst, lead);  // its partition slot
  }
}

// Apply one move with the whole workgroup; every thread calls it. Replica move: the apply.h lanes on threads 0..5
// (broker, potential and leadership-NW loads) and the host lanes on 6..7, one step, beside the finish lanes (counts,
// replica, partition slots, topic counts) on waves 1-3; then the host utilizations. Leadership: the finish fields no
// step touches (leader / topic leader counts, slots) run on waves 1-2 from the start, the partition record on wave 3
// after step 1; every aggregate of the move has its own lane, which loads it into registers at the first step (one
// memory round trip for all of them):
//   lane 0 leadership NW load of src (-= sr's old load)        lane 1 sr's load (makeFollower -> delta, new load)
//   lane 2 Broker.load() of src (-= delta)                     lane 3 Broker.load() of dst (+= delta)
//   lane 4 dr's load (+= delta, -> scratch for lane 5)         lane 5 leadership NW load of dst (+= dr's new load)
//   lanes 6, 7 the hosts (Host.makeFollower / makeLeader)
// the same operations on the same values, in the order apply.h's sequential form (the emulation) runs them.
// CCMI_STAMPS: thread 0's time points inside an apply ([8240] applies, [8241..8244] leadership: loads landed, step 0
// done, step 1 done, end; [8245..8246] replica move: lanes done, end), each summed from the previous point
__device__ __forceinline__ void applyStamp(unsigned long long* st, unsigned long long& t, int slot, bool drain) {
  if (!st || threadIdx.x != 0) return;
  if (drain) __builtin_amdgcn_s_waitcnt(0);
  const unsigned long long u = __builtin_amdgcn_s_memrealtime();
  atomicAdd(&st[slot], u - t);
  t = u;
}
template <int WC>
__device__ void chainApply(const ChainTables& C, LoadVec* sc, int action, int r, int dst, const ChainWin* win,
                           unsigned long long* st) {
  unsigned long long tS = st ? __builtin_amdgcn_s_memrealtime() : 0;
  if (st && threadIdx.x == 0) atomicAdd(&st[8240], 1ull);
  DevApply<WC> S{C, sc};
  int src, p, rflags;
  if (win) {  // the evaluating lane's view of the winner (same records, read in this decision's evaluation)
    src = win->src;
    p = win->p;
    rflags = win->flags;
  } else {
    const ReplicaRec rr = C.replicas[r];
    src = rr.broker;
    p = rr.part;
    rflags = rr.flags;
  }
  const int t = threadIdx.x;
  constexpr int W = WC;
  if (action == DA_LEADERSHIP) {
    int sr, dr, dpos;
    if (win && win->spos >= 0 && win->dpos >= 0) {  // the two slots directly (leadershipReplicas' result)
      const int o = C.pOff[p];
      sr = C.pSlots[o + win->spos];
      dr = C.pSlots[o + win->dpos];
      dpos = win->dpos;
    } else {
      leadershipReplicas(S, p, src, dst, sr, dr, dpos);
    }
    // lane -> its aggregate, chosen by address (one load / store instruction stream for all lanes, no divergence)
    const bool hosts = S.hostsOn();
    const int hs = hosts ? S.host(src) : 0, hd = hosts ? S.host(dst) : 0;
    const bool hostLane = t >= 6 && t < 6 + kHostLanes && hosts && !(t == 7 && hs == hd);
    const bool active = t < 6 || hostLane;
    LoadVec* agg = t == 0   ? &S.bLnw(src)
                   : t == 1 ? &S.rLoad(sr)
                   : t == 2 ? &S.bLoad(src)
                   : t == 3 ? &S.bLoad(dst)
                   : t == 4 ? &S.rLoad(dr)
                   : t == 5 ? &S.bLnw(dst)
                            : (hosts ? &S.hLoad(t == 6 ? hs : hd) : &S.bLnw(src));
    // The finish fields that no step reads or writes run from the start on waves 1 and 2, beside the steps: the leader
    // and topic leader counts of src and dst (wave 1, one lane per side) and the partition's slots and leader (wave 2).
    // Wave 3 loads the partition record's broker and rack pairs now and writes the swap after step 1, with the leader
    // NW_OUT the record keeps: dr's new load (scratch(1), the value lane 4 stores into dr's record).
    const int w = t >> 6, l = t & 63;
    if (w == 1 && l < 2) S.brk(l == 0 ? src : dst).nlead += l == 0 ? -1 : 1;
    else if (w == 1 && l < 4) S.topicLeadAdd(S.part(p).topic, l == 2 ? src : dst, l == 2 ? -1 : 1);
    else if (w == 2 && l == 0) applyLeadershipFinishLane(S, 2, p, dr, dpos, src, dst);
    const bool recLane = w == 3 && l == 0;
    int b0 = 0, bd = 0;
    int16_t k0 = 0, kd = 0;
    if (recLane) {
      const PartitionRec& prc = S.part(p);
      b0 = prc.brokers[0];
      bd = prc.brokers[dpos];
      k0 = prc.racks[0];
      kd = prc.racks[dpos];
    }
    LoadVec x, o;
    // step 0: every lane's aggregate into registers (lane 0 also sr's load, lanes 1 and 4 their replica's flags);
    // lanes 0 and 1 compute
    if (active) ldCopy(x, *agg, W);
    if (t == 0) ldCopy(o, S.rLoad(sr), W);
    const int32_t flags0 = (t == 1 || t == 4) ? S.rep(t == 1 ? sr : dr).flags : 0;
    applyStamp(st, tS, 8241, true);
    if (t == 0) {
      ldAddSignedAll(x, o, W, true);
      ldCopy(*agg, x, W);
      S.brk(src).lbi = ldUtil(x, R_NW_IN, W);
    } else if (t == 1) {
      ldMakeFollower(x, o, W);
      ldCopy(S.scratch(0), o, W);  // delta
    }
    chainSync();
    applyStamp(st, tS, 8242, false);
    // step 1: the delta everywhere it goes (lanes 2, 3, 4 and the hosts: one add or subtract each)
    const bool takesDelta = (t >= 2 && t <= 4) || hostLane;
    if (takesDelta && x.mask) {
      ldCopy(o, S.scratch(0), W);
      ldAddSignedAll(x, o, W, t == 2 || t == 6);
      if (t == 6 && hs == hd) ldAddSignedAll(x, o, W, false);  // Host.makeFollower then makeLeader on one host
    }
    if (active && t >= 1 && t != 5) ldCopy(*agg, x, W);  // lane 1: sr's new load (makeFollower's result)
    if (t == 1 || t == 4) {
      ReplicaRec& rec = S.rep(t == 1 ? sr : dr);
      rec.flags = t == 1 ? (flags0 & ~(int32_t)RF_LEADER) : (flags0 | (int32_t)RF_LEADER);
      for (int k = 0; k < 4; ++k) rec.util[k] = ldUtil(x, k, W);
      if (t == 4) ldCopy(S.scratch(1), x, W);  // dr's new load, for lane 5
    } else if (t == 2 || t == 3) {
      BrokerRec& rec = S.brk(t == 2 ? src : dst);
      for (int k = 0; k < 4; ++k) rec.util[k] = ldUtil(x, k, W);
      if (!hosts)
        for (int k = 0; k < 3; ++k) rec.hutil[k] = rec.util[k];
    }
    chainSync();
    applyStamp(st, tS, 8243, false);
    // step 2: dst's leadership NW load; the partition record (wave 3); the host utilizations
    if (t == 5) {
      ldCopy(o, S.scratch(1), W);
      ldAddSignedAll(x, o, W, false);
      ldCopy(*agg, x, W);
      S.brk(dst).lbi = ldUtil(x, R_NW_IN, W);
    } else if (recLane) {
      PartitionRec& prc = S.part(p);
      prc.brokers[0] = bd;
      prc.brokers[dpos] = b0;
      prc.racks[0] = kd;
      prc.racks[dpos] = k0;
      ldCopy(o, S.scratch(1), W);
      prc.leadNwOut = ldUtil(o, R_NW_OUT, W);
    }
    if (hosts) applyHostUtil(S, src, dst, t, (int)blockDim.x);
    chainSync();
    applyStamp(st, tS, 8244, false);
  } else {
    const bool lead = (rflags & RF_LEADER) != 0;
    const int lr = C.pLeader[p];
    if (t < kReplicaLanes) applyReplicaLane(S, t, r, src, dst, lr, lead);
    else if (t < kReplicaLanes + kHostLanes) applyHostReplicaLane(S, t - kReplicaLanes, r, src, dst);
    else
      replicaFinishWaves(S, t, r, p, src, dst, lead);  // independent of the load lanes (counts, slots, topic counts)
    applyStamp(st, tS, 8245, true);
    if (S.hostsOn()) {
      chainSync();
      applyHostUtil(S, src, dst, t, (int)blockDim.x);
    }
    chainSync();
    applyStamp(st, tS, 8246, false);
  }
}
__device__ __forceinline__ void chainApplyAny(const ChainTables& C, LoadVec* sc, int action, int r, int dst,
                                              const ChainWin* win = nullptr, unsigned long long* st = nullptr) {
  switch (C.W) {  // block-uniform
    case 1: chainApply<1>(C, sc, action, r, dst, win, st); break;
    case 2: chainApply<2>(C, sc, action, r, dst, win, st); break;
    case 3: chainApply<3>(C, sc, action, r, dst, win, st); break;
    case 4: chainApply<4>(C, sc, action, r, dst, win, st); break;
    default: chainApply<5>(C, sc, action, r, dst, win, st); break;
  }
}

// First accepted pair q in [start, n) on the current state (kNone if none), block-uniform. When the rest of the list
// fits a tile of 64 or 128 pairs, 4 or 2 waves share each pair's goals (goal-parallel tiles, tileFirst): the same
// single tile, with the conjunction's latency split over the SIMDs.
__device__ __forceinline__ unsigned long long chainFirstPair(const DevTables& T, const DevProgram& prog,
                                                             const OverlayLds& ov, const RowRef* pr,
                                                             const int32_t* pb, int start, int n, ChainWin* win) {
  const int nGoals = prog.nGoals;
  for (int base = start; base < n;) {
    const int rest = n - base;
    const int parts = (rest <= 64 && nGoals >= 4) ? 4 : ((rest <= 128 && nGoals >= 2) ? 2 : 1);  // block-uniform
    const int wave = (int)(threadIdx.x >> 6);
    const int part = wave % parts;
    const int slot = (wave / parts) * 64 + (int)(threadIdx.x & 63);
    const int q = base + slot;
    bool ok = false;
    PreView v;
    // CCMI_STAMPS: [8250] tiles, thread 0's view loads [8251], conjunction [8252], tile reduction [8253]
    unsigned long long tE = T.stamps ? __builtin_amdgcn_s_memrealtime() : 0;
    if (T.stamps && threadIdx.x == 0) atomicAdd(&T.stamps[8250], 1ull);
    if (q < n) {
      v.loadDst(T, pb[q], ov);
      v.loadRowRef(T, prog, pr[q], ov);  // one dependent level: the row's records and the destination's together
      applyStamp(T.stamps, tE, 8251, true);
      ok = !v.exclLeadBlocked(prog) && moveCandidateAcceptedPart(prog, v, v.r, v.dst, part, parts);
      applyStamp(T.stamps, tE, 8252, true);
    }
    const int f = tileFirst(ok, parts);
    applyStamp(T.stamps, tE, 8253, false);
    if (f >= 0) {
      if (slot == f && part == 0) {  // the winner's lane hands its view of the pair to the apply
        int sp = -1, dp = -1;
        const int bs[8] = {v.pb0, v.pb1, v.pb2, v.pb3, v.pb4, v.pb5, v.pb6, v.pb7};
#pragma unroll
        for (int i = 0; i < 8; ++i)
          if (i < v.pn) {
            if (bs[i] == v.src) sp = i;
            if (bs[i] == v.dst) dp = i;
          }
        *win = ChainWin{v.r, v.dst, v.src, v.p, v.rflags, sp, dp};
      }
      __syncthreads();
      return (unsigned long long)(base + f);
    }
    base += kBlock / parts;
  }
  return kNone;
}

// A chain's decision log is kept in LDS while the chain runs and copied to the host-mapped log once at the end: a store
// to host memory completes only after its PCIe round trip, and a wave's later loads wait for its older stores (vmcnt
// counts both in issue order), so a per-decision store there stalled the next apply's loads by several microseconds.
constexpr int kChainLogLds = 1024;
__shared__ int32_t gChainLog[kChainLogLds];
__device__ __forceinline__ void chainLogPut(int32_t* __restrict__ log, int i, int32_t v) {  // thread 0
  if (i < kChainLogLds) gChainLog[i] = v;
  else log[i] = v;  // (a longer log than the LDS copy holds goes out directly)
}
__device__ __forceinline__ void chainLogFlush(int32_t* __restrict__ log, int n) {  // every thread
  __syncthreads();
  for (int i = (int)threadIdx.x; i < n && i < kChainLogLds; i += (int)blockDim.x) log[i] = gChainLog[i];
}

// PAIRS: pairs (pr[q], pb[q]) in reference order; after accepting q the loop resumes at next[q]; at most
// maxAccepts moves (the callers' stop counts). visited = reference-equivalent candidates of the sequence of scans.
// The body runs in its own launch (chain_pairs) or inside the scan server (SOP_CHAIN); `ov` is an empty overlay.
__device__ __forceinline__ void chainPairsRun(const DevTables& T, const ChainTables& C, const DevProgram& prog,
                                              const OverlayLds& ov, LoadVec* sc, const RowRef* __restrict__ pr,
                                              const int32_t* __restrict__ pb, const int32_t* __restrict__ next, int n,
                                              int maxAccepts, int32_t* __restrict__ log,
                                              ChainResultDev* __restrict__ out, ChainWin* win) {
  int start = 0, acc = 0;
  unsigned long long visited = 0;
  // CCMI_STAMPS: thread 0 sums the time in candidate evaluation and in applying moves (stamps[8200 .. 8203])
  const bool st = T.stamps && threadIdx.x == 0;
  unsigned long long tEval = 0, tApply = 0, t = st ? __builtin_amdgcn_s_memrealtime() : 0;
  const unsigned long long tStart = t;
  while (start < n && acc < maxAccepts) {
    const unsigned long long best = chainFirstPair(T, prog, ov, pr, pb, start, n, win);
    if (st) {
      const unsigned long long u = __builtin_amdgcn_s_memrealtime();
      tEval += u - t;
      t = u;
    }
    if (best == kNone) {
      visited += (unsigned long long)(n - start);
      break;
    }
    visited += best - (unsigned long long)start + 1;
    const int q = (int)best;
    if (threadIdx.x == 0) chainLogPut(log, acc, q);
    chainApplyAny(C, sc, prog.action, win->r, win->dst, win, T.stamps);
    if (st) {
      __builtin_amdgcn_s_waitcnt(0);
      const unsigned long long u = __builtin_amdgcn_s_memrealtime();
      tApply += u - t;
      t = u;
    }
    ++acc;
    start = next[q];
  }
  if (st) {
    atomicAdd(&T.stamps[8200], 1ull);
    atomicAdd(&T.stamps[8201], (unsigned long long)acc);
    atomicAdd(&T.stamps[8202], tEval);
    atomicAdd(&T.stamps[8203], tApply);
    atomicAdd(&T.stamps[8204], __builtin_amdgcn_s_memrealtime() - tStart);
  }
  chainLogFlush(log, acc);
  if (threadIdx.x == 0) {
    out->accepts = (unsigned long long)acc;
    out->visited = visited;
    out->failRow = 0;
  }
}

__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, kServerWaves))) void chain_pairs(DevTables T, ChainTables C, DevProgram prog,
                                                      const RowRef* __restrict__ pr, const int32_t* __restrict__ pb,
                                                      const int32_t* __restrict__ next, int n, int maxAccepts,
                                                      int32_t* __restrict__ log, ChainResultDev* __restrict__ out) {
  __shared__ OverlayLds ov;
  __shared__ alignas(8) unsigned char scRaw[2 * sizeof(LoadVec)];  // LoadVec has a member initializer
  __shared__ ChainWin win;
  if (threadIdx.x == 0) ov.nb = ov.nr = ov.np = 0;
  __syncthreads();
  chainPairsRun(T, C, prog, ov, reinterpret_cast<LoadVec*>(scRaw), pr, pb, next, n, maxAccepts, log, out, &win);
}

// RACK_ROWS: AbstractRackAwareGoal.rebalanceForBroker (AbstractRackAwareGoal.java:144-170) over the rows of every
// broker in order. A row is skipped when its broker is alive, the replica online and shouldKeepInTheCurrentBroker
// holds on the CURRENT partition state (RackAwareGoal.java:214-225); otherwise the first candidate in cands[0, N)
// that rackAwareEligibleBrokers keeps and the predicate conjunction accepts wins. No winner: failRow = row + 1.
__device__ __forceinline__ void chainRackRowsRun(const DevTables& T, const ChainTables& C, const DevProgram& prog,
                                                 const OverlayLds& ov, LoadVec* sc, const int32_t* __restrict__ rows,
                                                 int n, const int32_t* __restrict__ cands, int N,
                                                 int32_t* __restrict__ log, ChainResultDev* __restrict__ out) {
  int acc = 0;
  unsigned long long fail = 0;
  for (int k = 0; k < n; ++k) {
    const int r = rows[k];
    const ReplicaRec rr = C.replicas[r];
    const BrokerRec& sb = C.brokers[rr.broker];
    const bool off = ((rr.flags & (RF_ORIG_OFFLINE | RF_ORIG_DEAD)) && rr.broker == rr.orig) || !sb.alive;
    const PartitionRec& pp = C.parts[rr.part];
    bool keep = true;
    for (int i = 0; i < pp.n; ++i) keep &= !(pp.brokers[i] != rr.broker && pp.racks[i] == sb.rack);
    if (sb.alive && !off && keep) continue;
    unsigned long long best = kNone;
    for (int base = 0; base < N; base += kBlock) {
      const int j = base + threadIdx.x;
      unsigned long long local = kNone;
      if (j < N) {
        PreView v;
        v.loadDst(T, cands[j], ov);
        v.loadRow(T, prog, r, ov);
        if (v.rackEligible() && !v.exclLeadBlocked(prog) && moveCandidateAccepted(prog, v, v.r, v.dst))
          local = (unsigned long long)j;
      }
      const unsigned long long m = blockMin(local);
      if (m != kNone) {
        best = m;
        break;
      }
    }
    if (best == kNone) {
      fail = (unsigned long long)k + 1;
      break;
    }
    if (threadIdx.x == 0) {
      chainLogPut(log, 2 * acc, k);
      chainLogPut(log, 2 * acc + 1, (int)best);
    }
    chainApplyAny(C, sc, DA_MOVE, r, cands[best]);
    ++acc;
  }
  chainLogFlush(log, 2 * acc);
  if (threadIdx.x == 0) {
    out->accepts = (unsigned long long)acc;
    out->visited = 0;
    out->failRow = fail;
  }
}

__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, kServerWaves))) void chain_rack_rows(DevTables T, ChainTables C, DevProgram prog,
                                                          const int32_t* __restrict__ rows, int n,
                                                          const int32_t* __restrict__ cands, int N,
                                                          int32_t* __restrict__ log, ChainResultDev* __restrict__ out) {
  __shared__ OverlayLds ov;
  __shared__ alignas(8) unsigned char scRaw[2 * sizeof(LoadVec)];  // LoadVec has a member initializer
  if (threadIdx.x == 0) ov.nb = ov.nr = ov.np = 0;
  __syncthreads();
  chainRackRowsRun(T, C, prog, ov, reinterpret_cast<LoadVec*>(scRaw), rows, n, cands, N, log, out);
}

// RackAwareGoal's rows with no optimized goals (rackrows.h): one lane per partition group, every group at once.
struct RackRowsView {
  DevTables t;
  __device__ __forceinline__ int rack(int b) const { return t.brokers[b].rack; }
  __device__ __forceinline__ bool alive(int b) const { return t.brokers[b].alive != 0; }
  __device__ __forceinline__ uint32_t bits(int b) const { return t.brokers[b].allowedBits; }
  __device__ __forceinline__ int flags(int r) const { return t.replicas[r].flags; }
  __device__ __forceinline__ int rorig(int r) const { return t.replicas[r].orig; }
  __device__ __forceinline__ int rbroker(int r) const { return t.replicas[r].broker; }
  __device__ __forceinline__ int rpart(int r) const { return t.replicas[r].part; }
  __device__ __forceinline__ int pn(int p) const { return t.parts[p].n; }
  __device__ __forceinline__ int pbroker(int p, int i) const { return t.parts[p].brokers[i]; }
  __device__ __forceinline__ bool ineligible(int p, int b) const {
    if (!t.pIneligOff) return false;
    bool in = false;
    for (int k = t.pIneligOff[p]; k < t.pIneligOff[p + 1]; ++k) in |= t.pIneligB[k] == b;
    return in;
  }
};
__global__ __launch_bounds__(256) void rack_rows_groups(DevTables T, DevProgram prog, const int32_t* __restrict__ rows,
                                                        const int32_t* __restrict__ order,
                                                        const int32_t* __restrict__ gOff, int G,
                                                        const int32_t* __restrict__ cands, int N,
                                                        int32_t* __restrict__ res,
                                                        unsigned long long* __restrict__ evaluated) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long ev = 0;
  if (g < G) ev = (unsigned long long)rackRowsGroup(RackRowsView{T}, prog, rows, order, gOff[g], gOff[g + 1], cands, N, res);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) ev += __shfl_xor(ev, off, 64);
  if ((threadIdx.x & 63) == 0 && ev) atomicAdd(evaluated, ev);
}

// Host-side load changes since the last chain (LoadRow / SlotRow lists staged in host-mapped memory).
__global__ __launch_bounds__(256) void sync_loads(ChainTables C, const LoadRow* __restrict__ lrows, int nl,
                                                  const SlotRow* __restrict__ srows, int ns) {
  const int stride = gridDim.x * blockDim.x;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nl; i += stride) {
    const LoadRow& x = lrows[i];
    LoadVec* dst = x.kind == LR_REPLICA ? C.rLoad
                   : (x.kind == LR_BROKER       ? C.bLoad
                      : (x.kind == LR_LEADERSHIP_NW ? C.bLnw : (x.kind == LR_HOST ? C.hLoad : C.bPot)));
    dst[x.id] = x.v;
  }
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < ns; i += stride) {
    const SlotRow& x = srows[i];
    const int o = C.pOff[x.p], n = C.pOff[x.p + 1] - o;
    for (int k = 0; k < n; ++k) C.pSlots[o + k] = x.slots[k];
    C.pLeader[x.p] = x.leader;
  }
}

__global__ __launch_bounds__(256) void prep(MutTables M,
                                            const BrokerRow* __restrict__ brows, int nb,
                                            const ReplicaRow* __restrict__ rrows, int nr,
                                            const PartitionRow* __restrict__ prows, int np,
                                            const TopicCountDelta* __restrict__ tdel, int nt,
                                            const int4* __restrict__ req, int4* __restrict__ dReq, int nReq4,
                                            unsigned long long* __restrict__ result, unsigned int* __restrict__ done) {
  const int stride = gridDim.x * blockDim.x;
  const int first = blockIdx.x * blockDim.x + threadIdx.x;
  applyRowsBlock(M, brows, nb, rrows, nr, prows, np, tdel, nt, first, stride);
  for (int i = first; i < nReq4; i += stride) dReq[i] = req[i];
  if (blockIdx.x == 0 && threadIdx.x == 0 && result) {
    result[0] = kNone;
    result[1] = 0;
    *done = 0;
  }
}

// ------------------------------------------------------------------------------------------------ launchers
// First-fit scans cap their grid at what the chip holds resident at once (256 CUs x 4 workgroups of 256 threads
// at the scan kernels' register budget): the blocks then sweep the pair space in order, chunk c in iteration
// c / grid, and each chunk start is checked against the current best before any work — a launch whose winner
// is early costs one chunk per block, and no workgroup is dispatched only to exit.
static uint64_t residentBlocks() {  // CCMI_GRID_CAP overrides (diagnostics)
  static const uint64_t v = [] {
    const char* e = std::getenv("CCMI_GRID_CAP");
    return e ? (uint64_t)std::strtoull(e, nullptr, 10) : (uint64_t)1024;
  }();
  return v;
}
static unsigned gridFor(uint64_t work, uint64_t perBlock, uint64_t cap = 4096) {
  if (cap >= kXcds) cap -= cap % kXcds;  // an XCD-sliced grid rounds up to a multiple of 8 and stays under the cap
  uint64_t blocks = (work + perBlock - 1) / perBlock;
  if (blocks > cap) blocks = cap;
  if (blocks == 0) blocks = 1;
  return (unsigned)blocks;
}

hipError_t launchScanCross(const DevTables& T, const MutTables& M, const UpdateList& U, const DevProgram& prog,
                           const RowRef* reps, const int32_t* cands, int K, int Nr, int N, int c0,
                           unsigned long long* result, unsigned int* done, unsigned long long* mail,
                           unsigned long long seq, hipStream_t st) {
  unsigned blocks = gridFor((uint64_t)K * (uint64_t)Nr, (uint64_t)kBlock, residentBlocks());
  // wide scans: one slice of destination columns per XCD
  const int sliced = (uint32_t)Nr >= xcdSliceMinCols() ? 1 : 0;
  if (sliced) blocks = (blocks + kXcds - 1) / kXcds * kXcds;
  hipLaunchKernelGGL(scan_cross, dim3(blocks), dim3(kBlock), 0, st, T, M, U, prog, reps, cands, K, Nr, N, c0, sliced,
                     result, done, mail, seq);
  return hipGetLastError();
}

hipError_t launchScanSwap(const DevTables& T, const DevProgram& prog, const int32_t* srcs, int S, const int32_t* cbOff,
                          const int32_t* cbRep, int M, const SwapLimit& lim, unsigned long long* result, int32_t* rowVisited,
                          unsigned long long* mail, unsigned long long seq, hipStream_t st, hipEvent_t ev0,
                          hipEvent_t ev1) {
  const uint64_t rows = (uint64_t)M * (uint64_t)S;
  const unsigned blocks = gridFor(rows, kBlock / 64);
  if (ev0) (void)hipEventRecord(ev0, st);
  hipLaunchKernelGGL(scan_swap, dim3(blocks), dim3(kBlock), 0, st, T, prog, srcs, S, cbOff, cbRep, M, lim, result,
                     rowVisited);
  if (ev1) (void)hipEventRecord(ev1, st);
  hipLaunchKernelGGL(swap_visited_sum, dim3(1), dim3(1024), 0, st, rowVisited, (long long)rows, result, mail, seq);
  return hipGetLastError();
}

hipError_t launchScanPairs(const DevTables& T, const MutTables& M, const UpdateList& U, const DevProgram& prog,
                           const RowRef* pr, const int32_t* pb, int n, int keyBase, unsigned long long* result,
                           unsigned int* done, unsigned long long* mail, unsigned long long seq, hipStream_t st) {
  const unsigned blocks = gridFor((uint64_t)n, (uint64_t)kBlock, residentBlocks());
  hipLaunchKernelGGL(scan_pairs, dim3(blocks), dim3(kBlock), 0, st, T, M, U, prog, pr, pb, n, keyBase, result, done,
                     mail, seq);
  return hipGetLastError();
}

// One workgroup per CU slot: `blocks` workgroups of kBlock threads, all resident (the launcher caps it at 2 per CU).
hipError_t launchScanServer(const DevTables& T, const MutTables& M, const ChainTables& C, const ServerCmd* cmd,
                            const char* pay, const RowRef* pool, unsigned long long* result, unsigned int* done,
                            unsigned long long* mail, unsigned long long* t0, unsigned long long* bell,
                            unsigned long long startSeq, int blocks, hipStream_t st) {
  if (blocks < (int)kXcds || blocks % (int)kXcds != 0 || blocks > 512) return hipErrorInvalidValue;
  hipLaunchKernelGGL(scan_server, dim3(blocks), dim3(kBlock), 0, st, T, M, C, cmd, pay, pool, result, done, mail, t0,
                     bell, startSeq);
  return hipGetLastError();
}

hipError_t launchChainPairs(const DevTables& T, const ChainTables& C, const DevProgram& prog, const RowRef* pr,
                            const int32_t* pb, const int32_t* next, int n, int maxAccepts, int32_t* log,
                            ChainResultDev* out, hipStream_t st) {
  hipLaunchKernelGGL(chain_pairs, dim3(1), dim3(kBlock), 0, st, T, C, prog, pr, pb, next, n, maxAccepts, log, out);
  return hipGetLastError();
}

hipError_t launchChainRackRows(const DevTables& T, const ChainTables& C, const DevProgram& prog, const int32_t* rows,
                               int n, const int32_t* cands, int N, int32_t* log, ChainResultDev* out, hipStream_t st) {
  hipLaunchKernelGGL(chain_rack_rows, dim3(1), dim3(kBlock), 0, st, T, C, prog, rows, n, cands, N, log, out);
  return hipGetLastError();
}

hipError_t launchRackRowsGroups(const DevTables& T, const DevProgram& prog, const int32_t* rows, const int32_t* order,
                                const int32_t* gOff, int G, const int32_t* cands, int N, int32_t* res,
                                unsigned long long* evaluated, hipStream_t st) {
  if (G <= 0) return hipSuccess;
  hipLaunchKernelGGL(rack_rows_groups, dim3((unsigned)((G + 255) / 256)), dim3(256), 0, st, T, prog, rows, order, gOff,
                     G, cands, N, res, evaluated);
  return hipGetLastError();
}

hipError_t launchSyncLoads(const ChainTables& C, const LoadRow* lrows, int nl, const SlotRow* srows, int ns,
                           hipStream_t st) {
  if (nl + ns == 0) return hipSuccess;
  const unsigned blocks = gridFor((uint64_t)(nl > ns ? nl : ns), 256, 1024);
  hipLaunchKernelGGL(sync_loads, dim3(blocks), dim3(256), 0, st, C, lrows, nl, srows, ns);
  return hipGetLastError();
}

hipError_t launchPrep(const MutTables& M, const UpdateList& U, const int4* req,
                      int4* dReq, int nReq4, unsigned long long* result, unsigned int* done, hipStream_t st) {
  int n = U.nb;
  if (U.nr > n) n = U.nr;
  if (U.np > n) n = U.np;
  if (U.nt > n) n = U.nt;
  if (nReq4 > n) n = nReq4;
  if (n == 0 && !result) return hipSuccess;
  const unsigned blocks = gridFor((uint64_t)(n ? n : 1), 256);
  hipLaunchKernelGGL(prep, dim3(blocks), dim3(256), 0, st, M, U.brows, U.nb, U.rrows, U.nr, U.prows, U.np,
                     U.tdel, U.nt, req, dReq, nReq4, result, done);
  return hipGetLastError();
}

}  // namespace ccmi
