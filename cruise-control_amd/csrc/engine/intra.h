// K6: the intra-broker (JBOD) goals, one broker per device wavefront. Disks belong to one broker and the intra-broker
// goals never move a replica between brokers, so every broker's rebalance is independent of every other broker's:
// the reference's sequential broker loop (AbstractGoal.optimize :98-101) runs as B independent programs and the host
// concatenates their action logs in broker-id order. Written once for the gfx950 kernel (kernels/intra.hip) and the
// test-only sequential emulation (tests/emu), so both make the same decisions with the same arithmetic.
//
// Reference restated (paths under cruise-control/src/main/java/com/linkedin/kafka/cruisecontrol/):
//   IntraBrokerDiskCapacityGoal.rebalanceForBroker          analyzer/goals/IntraBrokerDiskCapacityGoal.java:187-221
//   IntraBrokerDiskUsageDistributionGoal (init :78-104, acceptance :175-243, rebalance :254-481)
//   AbstractGoal.maybeMoveReplicaBetweenDisks / maybeSwapReplicaBetweenDisks   analyzer/goals/AbstractGoal.java:351-430
//   GoalUtils.legitMoveBetweenDisks :237-244, diskUtilizationPercentage :397-400, averageDiskUtilizationPercentage
//   :379-389; Disk.addReplica / removeReplica (model/Disk.java:113-146); java.util.PriorityQueue siftUp/siftDown;
//   java.util.TimSort binary insertion sort (< 32 elements); SortedReplicas ordering with
//   ReplicaSortFunctionFactory.prioritizeDiskImmigrants + (reverse)sortByMetricGroupValue(DISK) + Replica.compareTo.
// Kept reference behaviours (see oracle/src/goals_intra.cpp): the swap applies only the source replica's move plus a
// remove/add of the destination replica on its own disk; the capacity goal's non-transitive candidate comparator;
// the swap phases end when their disk queue repeats a state after passes without a swap (the reference spins there
// until its 500 ms per-disk timeout).
#pragma once
#include <stdint.h>

#include "loadops.h"  // CCMI_LD

namespace ccmi {

constexpr int kIntraMaxDisks = 31;  // TimSort's binary-insertion path (MIN_MERGE = 32) covers every broker
constexpr int kIntraHist = 16;      // queue states remembered per swap phase (cycle detection)
constexpr int kIntraMaxPrior = 4;   // optimized intra-broker goals a session can hold
enum IntraGoal : int32_t { IG_CAPACITY = 0, IG_USAGE = 1 };
enum IntraStatus : int32_t { IS_OK = 0, IS_LOG_FULL = 1, IS_CYCLE = 2 };

struct IntraPrior {  // an optimized intra-broker goal whose actionAcceptance every action must pass
  int32_t kind;        // IntraGoal
  const double* upper; // [B] frozen IntraBrokerDiskUsageDistributionGoal thresholds (IG_USAGE)
  const double* lower;
};

// A replica's static K6 fields in one 32-byte record (intra_sort gathers one line per entry instead of one per field)
struct alignas(32) IntraRep {
  double du;         // expectedUtilizationFor(DISK)
  float score;       // valuesForGroup(DISK).avg()
  int32_t tie;       // Replica.compareTo rank among online replicas
  int32_t origDisk;  // Replica._originalDisk (-1 = null)
  int32_t pad[3];
};
static_assert(sizeof(IntraRep) == 32, "one aligned 32-byte record per replica");

struct IntraArgs {
  int32_t goal;    // IntraGoal being optimized
  double capThr;   // BalancingConstraint.capacityThreshold(DISK)
  double margin;   // (resourceBalancePercentage(DISK) - 1) * BALANCE_MARGIN (0.9)
  int32_t nPrior;
  IntraPrior prior[kIntraMaxPrior];
  const int32_t* brokers;  // brokers to run (alive brokers, or the ones whose log overflowed)
  int32_t nBrokers;
  const int32_t* bDiskOff;  // [B+1] CSR of bDisks: a broker's disks in logdir order (TreeMap)
  const int32_t* bDisks;
  const double* dCap;
  const uint8_t* dAlive;
  const double* dUtilIn;  // [D] initial Disk._utilization
  double* dUtil;          // [D] working copy
  const int32_t* eOff;    // [B+1] CSR of the broker's replicas
  const int32_t* eRep;
  const int32_t* eDiskIn;  // initial disk of each entry
  int32_t* eDisk;          // working copy
  const double* rDu;       // [R] expectedUtilizationFor(DISK)
  const float* rScore;     // [R] valuesForGroup(DISK).avg()
  const int32_t* rTie;     // [R] Replica.compareTo rank among online replicas
  const int32_t* rOrigDisk;  // [R] Replica._originalDisk (-1 = null)
  const uint8_t* rSel;     // [R] selectOnlineReplicas && selectReplicasBasedOnExcludedTopics
  const IntraRep* rStat;   // [R] rDu / rScore / rTie / rOrigDisk packed (device; the emulation reads the arrays)
  // entry-indexed copies of the replica fields the program reads per entry (filled by intra_sort / the emulation
  // once per launch): a broker's entries are one contiguous range, so its snapshots and candidate checks read a few
  // lines instead of one 128-B replica-table line per entry per pass
  double* eDu;             // [entries] rDu[eRep[i]]
  int32_t* eOrig;          // [entries] rOrigDisk[eRep[i]]
  uint64_t* eKeyRev;       // [entries] intraSortKey(.., reverse) of selected entries, ~0 for the others
  uint64_t* eKeyFwd;       // [entries] intraSortKey(.., forward), ~0 for the others
  int32_t* snapA;          // [entries] scratch (the broker's CSR range)
  int32_t* snapB;
  int32_t* ordRev;         // [entries] the broker's selected entries in reverse-score order (intraSortKeys)
  int32_t* ordFwd;         //           and in score order
  int32_t* nSel;           // [B] selected entries per broker
  int32_t* hist;           // [B][kIntraHist][kIntraMaxDisks + 1] scratch
  double* upperOut;        // [B] thresholds of this goal (IG_USAGE)
  double* lowerOut;
  const int64_t* logOff;   // [B] first log record of the broker
  const int32_t* logCap;   // [B] records available
  int32_t* logRep;         // records: replica, source disk, destination disk
  int32_t* logSrc;
  int32_t* logDst;
  int32_t* logCount;       // [B] out
  int32_t* status;         // [B] out: IntraStatus
  int64_t* cand;           // [B] out: candidates evaluated (reference-equivalent)
};

// Double.compare
CCMI_LD int intraDcmp(double a, double b) {
  if (a < b) return -1;
  if (a > b) return 1;
  const bool na = a != a, nb = b != b;
  if (na || nb) return na == nb ? 0 : (na ? 1 : -1);
  const bool sa = __builtin_signbit(a) != 0, sb = __builtin_signbit(b) != 0;  // -0.0 < 0.0
  return sa == sb ? 0 : (sa ? -1 : 1);
}
// ((Double) x).intValue()
CCMI_LD int32_t intraD2I(double x) {
  if (x != x) return 0;
  if (x >= 2147483647.0) return 2147483647;
  if (x <= -2147483648.0) return (int32_t)0x80000000;
  return (int32_t)x;
}

// The SortedReplicas comparator without its priority function as one unique 64-bit key: the score
// ((double) DISK average, negated for the reverse order) in Double.compare order, then Replica.compareTo's static
// tail rank (online replicas). Double.compare(-a, -b) is exactly the reversed order for non-NaN a, b; NaN is the
// largest score in both orders.
CCMI_LD uint64_t intraSortKey(float score, int32_t tie, bool reverse) {
  uint32_t bits;
  __builtin_memcpy(&bits, &score, 4);
  uint32_t u;
  if (score != score) {
    u = 0xFFFFFFFFu;
  } else {
    u = (bits & 0x80000000u) ? ~bits : (bits | 0x80000000u);
    if (reverse) u = ~u;
  }
  return ((uint64_t)u << 32) | (uint32_t)tie;
}

class IntraBroker {
 public:
  // snapA / snapB: the two snapshot buffers (nullptr = the broker's CSR range of A.snapA / A.snapB); the kernel passes
  // LDS buffers when the broker's selected entries fit
  CCMI_LD IntraBroker(const IntraArgs& a, int broker, int32_t* snapA = nullptr, int32_t* snapB = nullptr)
      : A(a), b(broker) {
    e0 = A.eOff[b];
    sa = snapA ? snapA : A.snapA + e0;
    sb = snapB ? snapB : A.snapB + e0;
    e1 = A.eOff[b + 1];
    d0 = A.bDiskOff[b];
    d1 = A.bDiskOff[b + 1];
    logBase = A.logOff[b];
    logCap = A.logCap[b];
  }

  // ordRev / ordFwd / nSel hold the broker's selected entries sorted by intraSortKey (kernels/intra.hip intra_sort,
  // or the emulation's sort): every key of the SortedReplicas comparator but the disk-immigrant priority is fixed
  // while the goal runs (intra-broker moves change neither loads nor offline status), so a snapshot of disk d is
  // two passes over that order (immigrants of d first, then the others).
  CCMI_LD void run() {
    for (int k = d0; k < d1; ++k) A.dUtil[A.bDisks[k]] = A.dUtilIn[A.bDisks[k]];
    for (int i = e0; i < e1; ++i) A.eDisk[i] = A.eDiskIn[i];
    nSel = A.nSel[b];
    if (A.goal == IG_CAPACITY) capacityRebalance();
    else usageRebalance();
    A.logCount[b] = nLog;
    A.status[b] = status;
    A.cand[b] = cand;
  }

 private:
  const IntraArgs& A;
  int b, e0, e1, d0, d1;
  int64_t logBase;
  int logCap, nLog = 0;
  int32_t status = IS_OK;
  int64_t cand = 0;
  double up = 0, lo = 0;  // this goal's thresholds (IG_USAGE)
  int nSel = 0;           // selected entries (ordRev / ordFwd length)
  int32_t* sa;            // snapshot buffers
  int32_t* sb;

  CCMI_LD double pct(int d) const { return A.dCap[d] > 0 ? A.dUtil[d] / A.dCap[d] : 1.0; }
  CCMI_LD double avgPct() const {
    double cap = 0, util = 0;
    for (int k = d0; k < d1; ++k) {
      const int d = A.bDisks[k];
      if (A.dAlive[d]) {
        cap += A.dCap[d];
        util += A.dUtil[d];
      }
    }
    return cap > 0 ? util / cap : 1.0;
  }
  CCMI_LD double du(int i) const { return A.eDu[i]; }

  // the disk's tracked sorted replicas (a clone), as entry indices into out[0..n): prioritizeDiskImmigrants puts the
  // replicas whose original disk is not d first, each group in the static order. On the device the broker's wavefront
  // runs the program redundantly on every lane (uniform control flow, identical stores) and only this filter is split
  // over the lanes: 64 entries per step, the kept ones compacted in order by a ballot prefix count.
#if defined(__HIP_DEVICE_COMPILE__)
  __device__ int snapshot(int d, bool reverse, int32_t* out) const {
    const int32_t* ord = (reverse ? A.ordRev : A.ordFwd) + e0;
    const int lane = threadIdx.x & 63;
    const uint64_t below = (1ull << lane) - 1;
    int n = 0;
    for (int pass = 0; pass < 2; ++pass)
      for (int k0 = 0; k0 < nSel; k0 += 64) {
        const int k = k0 + lane;
        bool keep = false;
        int i = 0;
        if (k < nSel) {
          i = ord[k];
          keep = A.eDisk[i] == d && ((A.eOrig[i] != d) == (pass == 0));
        }
        const uint64_t m = __ballot(keep);
        if (keep) out[n + __popcll(m & below)] = i;
        n += __popcll(m);
      }
    __syncthreads();  // the block is this one wavefront: every lane sees the compacted list (LDS or global)
    return n;
  }
#else
  int snapshot(int d, bool reverse, int32_t* out) const {
    const int32_t* ord = (reverse ? A.ordRev : A.ordFwd) + e0;
    int n = 0;
    for (int pass = 0; pass < 2; ++pass)
      for (int k = 0; k < nSel; ++k) {
        const int i = ord[k];
        if (A.eDisk[i] == d && ((A.eOrig[i] != d) == (pass == 0))) out[n++] = i;
      }
    return n;
  }
#endif

  CCMI_LD void record(int r, int src, int dst) {
    if (nLog >= logCap) {
      status = IS_LOG_FULL;
      return;
    }
    A.logRep[logBase + nLog] = r;
    A.logSrc[logBase + nLog] = src;
    A.logDst[logBase + nLog] = dst;
    ++nLog;
  }
  // ClusterModel.relocateReplica(tp, broker, logdir): Disk.removeReplica then Disk.addReplica
  CCMI_LD void relocate(int i, int dst) {
    const int src = A.eDisk[i];
    const double u = du(i);
    A.dUtil[src] -= u;
    A.dUtil[dst] += u;
    A.eDisk[i] = dst;
    record(A.eRep[i], src, dst);
  }

  // IntraBrokerDiskUsageDistributionGoal.actionAcceptance with thresholds (u, l); delta = sourceUtilizationDelta
  CCMI_LD bool usageAccept(double u, double l, int s, int t, double delta) const {
    if (delta == 0) return true;
    const double srcAllow = delta > 0 ? A.dCap[s] * u - A.dUtil[s] : A.dUtil[s] - A.dCap[s] * l;
    const double dstAllow = delta > 0 ? A.dUtil[t] - A.dCap[t] * l : A.dCap[t] * u - A.dUtil[t];
    const double ad = delta < 0 ? -delta : delta;
    if ((srcAllow >= 0 && srcAllow < ad) || (dstAllow >= 0 && dstAllow < ad)) return false;
    const double prev = pct(s) - pct(t);
    const double next = prev + delta / A.dCap[s] + delta / A.dCap[t];
    return (next < 0 ? -next : next) < (prev < 0 ? -prev : prev);
  }
  CCMI_LD bool underCap(int d, double add) const { return A.dUtil[d] + add < A.dCap[d] * A.capThr; }
  // AnalyzerUtils.isProposalAcceptableForOptimizedGoals for a move of entry i to disk t
  CCMI_LD bool priorsAcceptMove(int i, int t) const {
    for (int k = 0; k < A.nPrior; ++k) {
      const IntraPrior& p = A.prior[k];
      if (p.kind == IG_CAPACITY) {
        if (!underCap(t, du(i))) return false;
      } else if (!usageAccept(p.upper[b], p.lower[b], A.eDisk[i], t, -du(i))) {
        return false;
      }
    }
    return true;
  }
  CCMI_LD bool priorsAcceptSwap(int i, int j) const {
    const double delta = du(j) - du(i);
    for (int k = 0; k < A.nPrior; ++k) {
      const IntraPrior& p = A.prior[k];
      if (p.kind == IG_CAPACITY) {
        if (!(delta > 0 ? underCap(A.eDisk[i], delta) : underCap(A.eDisk[j], -delta))) return false;
      } else if (!usageAccept(p.upper[b], p.lower[b], A.eDisk[i], A.eDisk[j], delta)) {
        return false;
      }
    }
    return true;
  }

  // One candidate of AbstractGoal.maybeMoveReplicaBetweenDisks: entry i to disk t accepted on the current state
  CCMI_LD bool moveOk(int i, int t) const {
    if (!A.dAlive[t]) return false;  // legitMoveBetweenDisks (same broker by construction)
    bool self;
    if (A.goal == IG_CAPACITY) {
      self = du(i) > 0 && underCap(t, du(i));
    } else {
      const double delta = -du(i);
      self = delta != 0 && usageAccept(up, lo, A.eDisk[i], t, delta);
    }
    return self && priorsAcceptMove(i, t);
  }
  // One candidate of AbstractGoal.maybeSwapReplicaBetweenDisks (usage goal): 0 continue, 1 swap, 2 return false
  CCMI_LD int swapOutcome(int i, int j) const {
    if (!A.dAlive[A.eDisk[j]]) return 2;
    if (!A.dAlive[A.eDisk[i]]) return 0;
    const double delta = du(j) - du(i);
    if (!(delta != 0 && usageAccept(up, lo, A.eDisk[i], A.eDisk[j], delta))) return 2;
    return priorsAcceptSwap(i, j) ? 1 : 0;
  }
  // The first q in [q0, n) whose candidate decides (moves: accepted; swaps: any outcome but 0), evaluated on the
  // current state, or n; `out` = that outcome. On the device the broker's wavefront evaluates 64 candidates per step
  // and a ballot picks the first (every lane then holds the same answer); on the host one at a time. Nothing changes
  // state, so either way it is the candidate the sequential loop would stop at.
#if defined(__HIP_DEVICE_COMPILE__)
  template <class F>
  __device__ int firstDeciding(int q0, int n, F outcome, int& out) const {
    const int lane = threadIdx.x & 63;
    for (int k0 = q0; k0 < n; k0 += 64) {
      const int k = k0 + lane;
      const int o = k < n ? outcome(k) : 0;
      const uint64_t any = __ballot(o != 0);
      if (any) {
        const int first = __builtin_ctzll(any);
        out = (__ballot(o == 1) >> first) & 1ull ? 1 : 2;
        return k0 + first;
      }
    }
    out = 0;
    return n;
  }
#else
  template <class F>
  int firstDeciding(int q0, int n, F outcome, int& out) const {
    for (int k = q0; k < n; ++k) {
      const int o = outcome(k);
      if (o != 0) {
        out = o;
        return k;
      }
    }
    out = 0;
    return n;
  }
#endif
  // AbstractGoal.maybeMoveReplicaBetweenDisks: the first accepted candidate disk in cands[0, n)
  CCMI_LD int maybeMove(int i, const int32_t* cands, int n) {
    int o;
    const int k = firstDeciding(0, n, [&](int q) { return moveOk(i, cands[q]) ? 1 : 0; }, o);
    cand += k < n ? k + 1 : n;
    if (k == n) return -1;
    relocate(i, cands[k]);
    return cands[k];
  }
  // The rows rows[s0, m) each tried against the single disk t (moveLoadIn / moveLoadOut): the first accepted row,
  // moved, or m; one candidate per row visited
  CCMI_LD int moveFirstRow(const int32_t* rows, int s0, int m, int t) {
    int o;
    const int s = firstDeciding(s0, m, [&](int q) { return moveOk(rows[q], t) ? 1 : 0; }, o);
    cand += s < m ? s - s0 + 1 : m - s0;
    if (s < m) relocate(rows[s], t);
    return s;
  }
  // AbstractGoal.maybeSwapReplicaBetweenDisks (usage goal only)
  CCMI_LD bool maybeSwap(int i, const int32_t* cands, int n) {
    int o;
    const int k = firstDeciding(0, n, [&](int q) { return swapOutcome(i, cands[q]); }, o);
    cand += k < n ? k + 1 : n;
    if (o != 1) return false;
    const int j = cands[k];
    const int t = A.eDisk[j];
    relocate(i, t);
    // the destination replica goes to sourceReplica.disk(), read after the first relocation: its own disk
    const double u = du(j);
    A.dUtil[t] -= u;
    A.dUtil[t] += u;
    record(A.eRep[j], t, t);
    return true;
  }

  // ---------------------------------------------------------------- IntraBrokerDiskCapacityGoal
  CCMI_LD bool over(int d) const { return A.dUtil[d] > A.dCap[d] * A.capThr; }
  CCMI_LD void capacityRebalance() {
    int32_t overD[kIntraMaxDisks], cands[kIntraMaxDisks];
    int nOver = 0, nC = 0;
    for (int k = d0; k < d1; ++k) {
      const int d = A.bDisks[k];
      if (A.dAlive[d] && over(d)) overD[nOver++] = d;
      else cands[nC++] = d;
    }
    if (nOver == 0) return;
    timSortSmall(cands, nC);
    for (int k = 0; k < nOver; ++k) {
      const int d = overD[k];
      const int n = snapshot(d, true, sa);
      for (int q = 0; q < n; ++q) {
        maybeMove(sa[q], cands, nC);
        if (!over(d)) break;
      }
    }
  }
  CCMI_LD int allowanceCmp(int d1, int d2) const {  // ((Double) (allowance2 - allowance1)).intValue()
    const double a1 = A.dCap[d1] * A.capThr - A.dUtil[d1];
    const double a2 = A.dCap[d2] * A.capThr - A.dUtil[d2];
    return intraD2I(a2 - a1);
  }
  CCMI_LD void timSortSmall(int32_t* a, int n) const {  // TimSort.sort, n < MIN_MERGE
    if (n < 2) return;
    int runHi = 1;
    if (allowanceCmp(a[runHi++], a[0]) < 0) {
      while (runHi < n && allowanceCmp(a[runHi], a[runHi - 1]) < 0) runHi++;
      for (int x = 0, y = runHi - 1; x < y; ++x, --y) {
        const int32_t t = a[x];
        a[x] = a[y];
        a[y] = t;
      }
    } else {
      while (runHi < n && allowanceCmp(a[runHi], a[runHi - 1]) >= 0) runHi++;
    }
    for (int start = runHi; start < n; ++start) {
      const int32_t pivot = a[start];
      int left = 0, right = start;
      while (left < right) {
        const int mid = (left + right) >> 1;
        if (allowanceCmp(pivot, a[mid]) < 0) right = mid;
        else left = mid + 1;
      }
      for (int k = start; k > left; --k) a[k] = a[k - 1];
      a[left] = pivot;
    }
  }

  // ---------------------------------------------------------------- java.util.PriorityQueue<Disk> on live pct
  CCMI_LD int pqCmp(int x, int y, bool desc) const { return desc ? intraDcmp(pct(y), pct(x)) : intraDcmp(pct(x), pct(y)); }
  CCMI_LD void pqAdd(int32_t* q, int& n, int x, bool desc) const {
    int k = n++;
    while (k > 0) {
      const int parent = (k - 1) >> 1;
      const int e = q[parent];
      if (pqCmp(x, e, desc) >= 0) break;
      q[k] = e;
      k = parent;
    }
    q[k] = x;
  }
  CCMI_LD int pqPoll(int32_t* q, int& n, bool desc) const {
    const int result = q[0];
    const int m = --n;
    const int x = q[m];
    if (m > 0) {
      int k = 0;
      const int half = m >> 1;
      while (k < half) {
        int child = (k << 1) + 1;
        int c = q[child];
        const int right = child + 1;
        if (right < m && pqCmp(c, q[right], desc) > 0) c = q[child = right];
        if (pqCmp(x, c, desc) <= 0) break;
        q[k] = c;
        k = child;
      }
      q[k] = x;
    }
    return result;
  }
  // queue-state history of a swap phase since its last swap: true when (q, n) was seen (the reference spins)
  CCMI_LD bool seenBefore(const int32_t* q, int n, int& nHist) {
    int32_t* H = A.hist + (int64_t)b * kIntraHist * (kIntraMaxDisks + 1);
    for (int h = 0; h < nHist; ++h) {
      const int32_t* s = H + h * (kIntraMaxDisks + 1);
      if (s[0] != n) continue;
      bool eq = true;
      for (int k = 0; k < n && eq; ++k) eq = s[1 + k] == q[k];
      if (eq) return true;
    }
    if (nHist == kIntraHist) {
      status = IS_CYCLE;
      return true;
    }
    int32_t* s = H + nHist * (kIntraMaxDisks + 1);
    s[0] = n;
    for (int k = 0; k < n; ++k) s[1 + k] = q[k];
    ++nHist;
    return false;
  }

  // ---------------------------------------------------------------- IntraBrokerDiskUsageDistributionGoal
  CCMI_LD void usageRebalance() {
    const double avg = avgPct();
    up = avg * (1 + A.margin);
    const double lm = 1 - A.margin;
    lo = avg * (lm > 0 ? lm : 0.0);
    A.upperOut[b] = up;
    A.lowerOut[b] = lo;
    for (int k = d0; k < d1 && status == IS_OK; ++k) {
      const int d = A.bDisks[k];
      if (!A.dAlive[d]) continue;
      if (pct(d) > up) {
        if (moveLoadOut(d)) swapLoadOut(d);
      }
      if (pct(d) < lo) {
        if (moveLoadIn(d)) swapLoadIn(d);
      }
    }
  }
  CCMI_LD bool moveLoadIn(int disk) {
    const double brokerUtil = avgPct();
    int32_t q[kIntraMaxDisks];
    int n = 0;
    for (int k = d0; k < d1; ++k) {
      const int cd = A.bDisks[k];
      if (A.dAlive[cd] && pct(cd) > brokerUtil) pqAdd(q, n, cd, true);
    }
    while (n > 0) {
      const int cd = pqPoll(q, n, true);
      const int m = snapshot(cd, true, sa);
      for (int s = moveFirstRow(sa, 0, m, disk); s < m; s = moveFirstRow(sa, s + 1, m, disk)) {
        if (pct(disk) > lo) return false;
        if (n > 0 && pct(cd) < pct(q[0])) {
          pqAdd(q, n, cd, true);
          break;
        }
      }
    }
    return true;
  }
  CCMI_LD bool moveLoadOut(int disk) {
    const double brokerUtil = avgPct();
    int32_t q[kIntraMaxDisks];
    int n = 0;
    for (int k = d0; k < d1; ++k) {
      const int cd = A.bDisks[k];
      if (A.dAlive[cd] && pct(cd) < brokerUtil) pqAdd(q, n, cd, false);
    }
    // the disk's snapshot is re-taken only after a move left it (between polls without a move it is unchanged:
    // entry disks, original disks and the static order are all it reads)
    int m = 0;
    bool fresh = false;
    while (n > 0) {
      const int cd = pqPoll(q, n, false);
      if (!fresh) m = snapshot(disk, true, sa);
      fresh = true;
      for (int s = moveFirstRow(sa, 0, m, cd); s < m; s = moveFirstRow(sa, s + 1, m, cd)) {
        fresh = false;
        if (pct(disk) < up) return false;
        if (n > 0 && pct(cd) > pct(q[0])) {
          pqAdd(q, n, cd, false);
          break;
        }
      }
    }
    return true;
  }
  // rebalanceBySwappingLoadOut (desc = false, source sorted reverse, candidates ascending) and
  // rebalanceBySwappingLoadIn (desc = true, source ascending, candidates reverse)
  CCMI_LD void swapPhase(int disk, bool in) {
    int32_t q[kIntraMaxDisks];
    int n = 0;
    for (int k = d0; k < d1; ++k) {
      const int cd = A.bDisks[k];
      if (A.dAlive[cd] && (in ? pct(cd) > lo : pct(cd) < up)) pqAdd(q, n, cd, in);
    }
    int nHist = 0;
    int m = 0;
    bool fresh = false;  // sa holds the disk's snapshot of the current state (re-taken only after a swap)
    while (n > 0) {
      const int cd = pqPoll(q, n, in);
      bool swapped = false;
      if (!fresh) m = snapshot(disk, !in, sa);
      fresh = true;
      const int c = snapshot(cd, in, sb);  // the candidate view cannot change before a swap
      for (int s = 0; s < m; ++s) {
        if (maybeSwap(sa[s], sb, c)) {
          if (in ? pct(disk) > lo : pct(disk) < up) return;
          swapped = true;
          fresh = false;
          break;
        }
      }
      if (in ? pct(cd) > lo : pct(cd) < up) pqAdd(q, n, cd, in);
      if (swapped) nHist = 0;
      else if (seenBefore(q, n, nHist)) return;
    }
  }
  CCMI_LD void swapLoadOut(int disk) { swapPhase(disk, false); }
  CCMI_LD void swapLoadIn(int disk) { swapPhase(disk, true); }
};

}  // namespace ccmi
