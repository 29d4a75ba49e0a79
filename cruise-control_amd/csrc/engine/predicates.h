// Goal predicates (legitMove / selfSatisfied / actionAcceptance) written once for host and device.
//
// Every comparison reproduces the reference's IEEE double expression exactly (no FMA: the library is
// built with -ffp-contract=off for host and gfx950):
//   ReplicaDistributionGoal.actionAcceptance      ReplicaDistributionGoal.java:119-138
//   ReplicaDistributionAbstractGoal limits        ReplicaDistributionAbstractGoal.java:79-104 (…AfterChange)
//   ReplicaDistributionAbstractGoal.selfSatisfied ReplicaDistributionAbstractGoal.java:160-170
//   ResourceDistributionGoal.actionAcceptance     ResourceDistributionGoal.java:101-156 (+ Disk/NwIn overrides)
//   ResourceDistributionGoal.selfSatisfied        ResourceDistributionGoal.java:199-224
//   isLoad{Above,Under}Balance…AfterChange        ResourceDistributionGoal.java:880-927
//   isGettingMoreBalanced / isSwapViolating…      ResourceDistributionGoal.java:943-1037
//   GoalUtils.legitMove                           GoalUtils.java:213-226
// One broker per host (RandomCluster names hosts after brokers), so the host-resource branch equals the
// broker branch bit for bit and is folded into it.
#pragma once
#include <stdint.h>

#include "devtypes.h"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define CCMI_HD __host__ __device__ __forceinline__
#else
#define CCMI_HD inline
#endif

namespace ccmi {

// V must provide: bu(b,res) bcap(b,res) nrep(b) alive(b) allowed(slot,b) ru(r,res) flags(r) rbroker(r)
// rorig(r) rpart(r) and, for partition membership, hosts(p,b) — or pbegin(p) pend(p) pbroker(i) through
// hostsPartition's generic form.
template <class V>
CCMI_HD bool currentOffline(const V& v, int r) {
  const int orig = v.rorig(r), br = v.rbroker(r);
  const bool origOffline = (v.flags(r) & RF_ORIG_OFFLINE) || !v.alive(orig);
  return (origOffline && br == orig) || !v.alive(br);
}

template <class V>
CCMI_HD bool hostsPartition(const V& v, int p, int b) {
  return v.hosts(p, b);
}

template <class V>
CCMI_HD bool legitMove(const V& v, int r, int dst, int action) {
  const bool has = hostsPartition(v, v.rpart(r), dst);
  if (action == DA_MOVE) return !has;  // no broken-disk ineligibility in ABI v1 (no BAD_DISKS brokers)
  if (action == DA_LEADERSHIP) return (v.flags(r) & RF_LEADER) && has;
  return false;
}

// ---------------------------------------------------------------- ReplicaDistributionGoal
template <class V>
CCMI_HD bool rdAccept(const DevGoal& g, const V& v, int action, int src, int dst) {
  if (action != DA_MOVE) return true;  // swaps and leadership moves are accepted
  const int upperDst = v.alive(dst) ? g.upper : 0;
  if (!(v.nrep(dst) + 1 <= upperDst)) return false;
  if (!v.allowed(g.allowedSlot, src)) return true;
  const int lowerSrc = v.alive(src) ? g.lower : 0;
  return v.nrep(src) - 1 >= lowerSrc;
}

// ---------------------------------------------------------------- ResourceDistributionGoal
template <class V>
CCMI_HD bool resAboveLowerAfter(const DevGoal& g, const V& v, int b, double delta, bool add) {
  const double lim = v.bcap(b, g.resource) * g.lowerThr;
  const double u = v.bu(b, g.resource);
  return add ? (u + delta >= lim) : (u - delta >= lim);
}
template <class V>
CCMI_HD bool resUnderUpperAfter(const DevGoal& g, const V& v, int b, double delta, bool add, double thr) {
  const double lim = v.bcap(b, g.resource) * thr;
  const double u = v.bu(b, g.resource);
  return add ? (u + delta <= lim) : (u - delta <= lim);
}
template <class V>
CCMI_HD bool resGettingMoreBalanced(const DevGoal& g, const V& v, int sb, double delta, int db) {
  const int res = g.resource;
  const double sc = v.bcap(sb, res), dc = v.bcap(db, res);
  const double prevDiff = (v.bu(sb, res) / sc) - (v.bu(db, res) / dc);
  const double nextDiff = prevDiff + (delta / sc) + (delta / dc);
  return __builtin_fabs(nextDiff) < __builtin_fabs(prevDiff);
}
// isSwapViolatingContainerLimit for the broker container (host container identical)
template <class V>
CCMI_HD bool resSwapViolating(const DevGoal& g, const V& v, double delta, int sb, int db) {
  const int res = g.resource;
  const double su = v.bu(sb, res), du = v.bu(db, res);
  bool underUpper;
  if (delta > 0) underUpper = su + delta <= v.bcap(sb, res) * g.upperThr;
  else underUpper = du - delta <= v.bcap(db, res) * g.upperThr;
  if (!underUpper) return true;
  bool aboveLower;
  if (delta < 0) aboveLower = su + delta >= v.bcap(sb, res) * g.lowerThr;
  else aboveLower = du - delta >= v.bcap(db, res) * g.lowerThr;
  return !aboveLower;
}

template <class V>
CCMI_HD bool resAcceptMove(const DevGoal& g, const V& v, int action, int r, int src, int dst) {
  if (action == DA_LEADERSHIP && (g.resource == 3 /*DISK*/ || g.resource == 1 /*NW_IN*/)) return true;
  const double ru = v.ru(r, g.resource);
  const bool srcExcluded = !v.allowed(g.allowedSlot, src);
  const bool srcAboveLower = resAboveLowerAfter(g, v, src, 0.0, true);
  const bool dstUnderUpper = resUnderUpperAfter(g, v, dst, 0.0, false, g.upperThr);
  if ((srcExcluded || srcAboveLower) && dstUnderUpper) {
    return resUnderUpperAfter(g, v, dst, ru, true, g.upperThr) &&
           (srcExcluded || resAboveLowerAfter(g, v, src, ru, false));
  } else if (srcExcluded) {
    return ru == 0.0;
  }
  return resGettingMoreBalanced(g, v, src, -ru, dst);
}

// swap: source replica sr on sb, destination replica dr on db. Returns ccmi_acceptance (0 accept, 1 replica reject).
template <class V>
CCMI_HD int resAcceptSwap(const DevGoal& g, const V& v, int sr, int sb, int dr, int db) {
  const double delta = v.ru(dr, g.resource) - v.ru(sr, g.resource);
  if (delta == 0) return 0;
  const bool both = delta > 0
                        ? (resAboveLowerAfter(g, v, db, 0.0, true) && resUnderUpperAfter(g, v, sb, 0.0, false, g.upperThr))
                        : (resAboveLowerAfter(g, v, sb, 0.0, true) && resUnderUpperAfter(g, v, db, 0.0, false, g.upperThr));
  if (both) return resSwapViolating(g, v, delta, sb, db) ? 1 : 0;
  return resGettingMoreBalanced(g, v, sb, delta, db) ? 0 : 1;
}

// ---------------------------------------------------------------- dispatch
template <class V>
CCMI_HD bool goalAcceptMove(const DevGoal& g, const V& v, int action, int r, int src, int dst) {
  if (g.kind == DG_REPLICA_DISTRIBUTION) return rdAccept(g, v, action, src, dst);
  return resAcceptMove(g, v, action, r, src, dst);
}
template <class V>
CCMI_HD bool goalSelfSatisfiedMove(const DevGoal& g, const V& v, int action, int r, int src, int dst) {
  if (g.kind == DG_REPLICA_DISTRIBUTION) {
    if (g.fixOffline && currentOffline(v, r)) return true;
    return rdAccept(g, v, action, src, dst);
  }
  if (g.fixOffline && currentOffline(v, r)) return action == DA_MOVE;
  const double ru = v.ru(r, g.resource);
  return resUnderUpperAfter(g, v, dst, ru, true, g.upperThr) && resAboveLowerAfter(g, v, src, ru, false);
}
// returns 0 ACCEPT, 1 REPLICA_REJECT, 2 BROKER_REJECT
template <class V>
CCMI_HD int goalAcceptSwap(const DevGoal& g, const V& v, int sr, int sb, int dr, int db) {
  if (g.kind == DG_REPLICA_DISTRIBUTION) return 0;
  return resAcceptSwap(g, v, sr, sb, dr, db);
}
template <class V>
CCMI_HD bool goalSelfSatisfiedSwap(const DevGoal& g, const V& v, int sr, int sb, int dr, int db) {
  if (g.kind == DG_REPLICA_DISTRIBUTION) {
    if (g.fixOffline && currentOffline(v, sr)) return true;
    return true;  // rdAccept(SWAP) == ACCEPT
  }
  if (g.fixOffline && currentOffline(v, sr)) return false;  // action != INTER_BROKER_REPLICA_MOVEMENT
  const double delta = v.ru(dr, g.resource) - v.ru(sr, g.resource);
  return delta != 0 && !resSwapViolating(g, v, delta, sb, db);
}

// Full candidate predicate of AbstractGoal.maybeApplyBalancingAction's loop body for one (replica, dest):
// legit && selfSatisfied && every optimized goal ACCEPTs.
template <class V>
CCMI_HD bool moveCandidateAccepted(const DevProgram& prog, const V& v, int r, int dst) {
  const int action = prog.action;
  const int src = v.rbroker(r);
  if (!legitMove(v, r, dst, action)) return false;
  if (!goalSelfSatisfiedMove(prog.goals[0], v, action, r, src, dst)) return false;
  for (int i = 1; i < prog.nGoals; ++i)
    if (!goalAcceptMove(prog.goals[i], v, action, r, src, dst)) return false;
  return true;
}

// One step of AbstractGoal.maybeApplySwapAction's loop for (source sr, destination replica dr on db):
// returns 0 = continue, 1 = terminal ACCEPT, 2 = terminal null (return null).
template <class V>
CCMI_HD int swapCandidateOutcome(const DevProgram& prog, const V& v, int sr, int dr, int db) {
  const int sb = v.rbroker(sr);
  if (!legitMove(v, sr, db, DA_MOVE)) return 2;
  if (!legitMove(v, dr, sb, DA_MOVE)) return 0;
  if (!goalSelfSatisfiedSwap(prog.goals[0], v, sr, sb, dr, db)) return 2;
  for (int i = 1; i < prog.nGoals; ++i) {
    const int acc = goalAcceptSwap(prog.goals[i], v, sr, sb, dr, db);
    if (acc == 1) return 0;
    if (acc == 2) return 2;
  }
  return 1;
}

}  // namespace ccmi
