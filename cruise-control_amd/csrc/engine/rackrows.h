// RackAwareGoal's broker loop decided per partition (host emulation and gfx950 kernel share this code).
//
// AbstractRackAwareGoal.rebalanceForBroker (AbstractRackAwareGoal.java:144-170) visits, broker by broker, the replicas
// that violate rack awareness (shouldKeepInTheCurrentBroker, RackAwareGoal.java:214-225) or are offline, and moves each
// to the first broker of rackAwareEligibleBrokers (RackAwareGoal.java:193-211) that maybeApplyBalancingAction accepts.
// With no optimized goals (RackAwareGoal first in the chain) a candidate's acceptance reads only the replica's own
// partition (GoalUtils.legitMove, the rack filter) and static broker state (racks, liveness, exclusion / NEW bits):
// the decisions of one partition's rows depend on each other, in row order, and on nothing else. So every partition's
// rows are decided by one lane, all partitions at once, on a private copy of the partition's slots; the host then
// applies the accepted moves in row order, which fixes the floating-point order of every aggregate.
#pragma once
#include <stdint.h>

#include "devtypes.h"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define CCMI_RR __host__ __device__ __forceinline__
#else
#define CCMI_RR inline
#endif

namespace ccmi {

// res[k] for row k: the accepted candidate index, kRackKeep (the row holds when reached), kRackFail (no candidate)
constexpr int32_t kRackKeep = -1;
constexpr int32_t kRackFail = -2;

// V: rack(b) alive(b) bits(b) (BrokerRec.allowedBits) flags(r) rorig(r) rbroker(r) rpart(r) pn(p) pbroker(p, i)
// ineligible(p, b)
template <class V>
CCMI_RR int64_t rackRowsGroup(const V& v, const DevProgram& prog, const int32_t* rows, const int32_t* order, int i0,
                              int i1, const int32_t* cands, int N, int32_t* res) {
  if (i0 >= i1) return 0;
  const int p = v.rpart(rows[order[i0]]);
  const int n = v.pn(p);
  int pb[kMaxRf], prk[kMaxRf];
  for (int i = 0; i < kMaxRf; ++i) {
    pb[i] = i < n ? v.pbroker(p, i) : -1;
    prk[i] = i < n ? v.rack(pb[i]) : -1;
  }
  int64_t evaluated = 0;
  for (int q = i0; q < i1; ++q) {
    const int k = order[q];
    const int r = rows[k];
    const int src = v.rbroker(r), orig = v.rorig(r), fl = v.flags(r);
    const int srk = v.rack(src);
    const bool srcAlive = v.alive(src);
    const bool off = ((fl & (RF_ORIG_OFFLINE | RF_ORIG_DEAD)) && src == orig) || !srcAlive;
    bool keep = true;
    for (int i = 0; i < n; ++i) keep &= !(pb[i] != src && prk[i] == srk);
    if (srcAlive && !off && keep) {
      res[k] = kRackKeep;
      continue;
    }
    int best = kRackFail;
    for (int j = 0; j < N; ++j) {
      const int d = cands[j];
      const int drk = v.rack(d);
      ++evaluated;
      int cnt = 0;  // the partition's racks with one occurrence of the replica's own removed
      for (int i = 0; i < n; ++i) cnt += prk[i] == drk ? 1 : 0;
      if (srk == drk) cnt -= 1;
      if (cnt != 0) continue;
      const uint32_t bits = v.bits(d);
      if (prog.exclLeadMove && (fl & RF_LEADER) && ((bits >> kExclLeadBit) & 1u)) continue;
      if (prog.newOnly && !((bits >> kNewBit) & 1u) && d != orig) continue;
      bool hosts = false;
      for (int i = 0; i < n; ++i) hosts |= pb[i] == d;
      if (hosts || v.ineligible(p, d)) continue;  // GoalUtils.legitMove
      best = j;
      break;
    }
    res[k] = best;
    if (best < 0) continue;  // the host stops at the first failing row; later rows of this lane are unused
    for (int i = 0; i < n; ++i)
      if (pb[i] == src) {
        pb[i] = cands[best];
        prk[i] = v.rack(cands[best]);
        break;
      }
  }
  return evaluated;
}

}  // namespace ccmi
