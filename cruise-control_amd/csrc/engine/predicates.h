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
//   RackAwareGoal / AbstractRackAwareGoal         RackAwareGoal.java:57-66, AbstractRackAwareGoal.java:76-117
//   ReplicaCapacityGoal                           ReplicaCapacityGoal.java:69-82,165-168
//   CapacityGoal (+ Disk/NwIn leadership ACCEPT)  CapacityGoal.java:75-133,431-475, DiskCapacityGoal.java:40-43
//   PotentialNwOutGoal                            PotentialNwOutGoal.java:73-113,152-183
//   TopicReplicaDistributionGoal                  TopicReplicaDistributionGoal.java:153-214,300-314
//   LeaderReplicaDistributionGoal                 LeaderReplicaDistributionGoal.java:91-123
//   LeaderBytesInDistributionGoal                 LeaderBytesInDistributionGoal.java:69-127,264-271
//   TopicLeaderReplicaDistributionGoal            TopicLeaderReplicaDistributionGoal.java:181-256,359-374
// Host resources (CPU, NW_IN, NW_OUT; Resource.java:18-25) are checked against the broker's host as the reference
// does (V::hu / V::hcap: Broker.host().load() / Host.capacityFor); when every host holds one broker those equal the
// broker's own values bit for bit, and V::hostMode() is false: the host checks are then the broker checks and are skipped
// (the same booleans, without evaluating both).
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

// A value every lane holds alike (program and goal fields): on gfx950 it goes to a scalar register, so the goal
// dispatch below branches on a scalar (the scan server keeps the program in LDS, where the compiler cannot prove the
// value uniform and would otherwise build the switch from per-lane compares).
CCMI_HD int uniform(int x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_readfirstlane(x);
#else
  return x;
#endif
}

// V must provide: bu(b,res) bcap(b,res) hostMode() hu(b,res) hcap(b,res) nrep(b) alive(b) allowed(slot,b) ru(r,res) flags(r) rbroker(r)
// rorig(r) origOff(r) rpart(r) hosts(p,b), and for the goals that read them: rack(b) otherOnRack(p,self,rack)
// slotRack(p,b) (rack of partition p's replica on b) rackCount(p,rack) nlead(b)
// pot(b) lnwin(b) pLeadNwOut(p) ptopic(p) tcount(t,b) tUpper(t) tLower(t) bset(b) rbset(r) (broker sets)
// tlead(t,b) (Broker.numLeadersFor) tMinLead(t) (MinTopicLeadersPerBrokerGoal's minimum, -1 = not its topic)
// tLeadUpper(t) tLeadLower(t) (TopicLeaderReplicaDistributionGoal's limits).
// Replica.isCurrentOffline; V::origOff(r) = isOriginalOffline || original broker dead
template <class V>
CCMI_HD bool currentOffline(const V& v, int r) {
  const int orig = v.rorig(r), br = v.rbroker(r);
  return (v.origOff(r) && br == orig) || !v.alive(br);
}

template <class V>
CCMI_HD bool hostsPartition(const V& v, int p, int b) {
  return v.hosts(p, b);
}

template <class V>
CCMI_HD bool legitMove(const V& v, int r, int dst, int action) {
  const bool has = hostsPartition(v, v.rpart(r), dst);
  // Partition.canAssignReplicaToBroker: not one of the partition's ineligible (broken-disk) brokers
  if (action == DA_MOVE) return !has && !v.ineligible(v.rpart(r), dst);
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
// isLoadAboveBalanceLowerLimitAfterChange / isLoadUnderBalanceUpperLimitAfterChange (:880-927): a host resource is
// within the limit when the host or the broker is
template <class V>
CCMI_HD bool resAboveLowerAfter(const DevGoal& g, const V& v, int b, double delta, bool add) {
  const int res = uniform(g.resource);
  const double lim = v.bcap(b, res) * g.lowerThr;
  const double u = v.bu(b, res);
  const bool brokerAbove = add ? (u + delta >= lim) : (u - delta >= lim);
  if (!isHostRes(res) || !v.hostMode()) return brokerAbove;
  const double hlim = v.hcap(b, res) * g.lowerThr;
  const double hu = v.hu(b, res);
  const bool hostAbove = add ? (hu + delta >= hlim) : (hu - delta >= hlim);
  return hostAbove || brokerAbove;
}
template <class V>
CCMI_HD bool resUnderUpperAfter(const DevGoal& g, const V& v, int b, double delta, bool add, double thr) {
  const int res = uniform(g.resource);
  const double lim = v.bcap(b, res) * thr;
  const double u = v.bu(b, res);
  const bool brokerUnder = add ? (u + delta <= lim) : (u - delta <= lim);
  if (!isHostRes(res) || !v.hostMode()) return brokerUnder;
  const double hlim = v.hcap(b, res) * thr;
  const double hu = v.hu(b, res);
  const bool hostUnder = add ? (hu + delta <= hlim) : (hu - delta <= hlim);
  return hostUnder || brokerUnder;
}
template <class V>
CCMI_HD bool resGettingMoreBalanced(const DevGoal& g, const V& v, int sb, double delta, int db) {
  const int res = uniform(g.resource);
  const double sc = v.bcap(sb, res), dc = v.bcap(db, res);
  const double prevDiff = (v.bu(sb, res) / sc) - (v.bu(db, res) / dc);
  const double nextDiff = prevDiff + (delta / sc) + (delta / dc);
  return __builtin_fabs(nextDiff) < __builtin_fabs(prevDiff);
}
// isSwapViolatingContainerLimit (:1005-1037) for the broker container, or with `host` the brokers' hosts
template <class V>
CCMI_HD bool resSwapContainerViolating(const DevGoal& g, const V& v, double delta, int sb, int db, bool host) {
  const int res = uniform(g.resource);
  const double su = host ? v.hu(sb, res) : v.bu(sb, res), du = host ? v.hu(db, res) : v.bu(db, res);
  const double sc = host ? v.hcap(sb, res) : v.bcap(sb, res), dc = host ? v.hcap(db, res) : v.bcap(db, res);
  bool underUpper;
  if (delta > 0) underUpper = su + delta <= sc * g.upperThr;
  else underUpper = du - delta <= dc * g.upperThr;
  if (!underUpper) return true;
  bool aboveLower;
  if (delta < 0) aboveLower = su + delta >= sc * g.lowerThr;
  else aboveLower = du - delta >= dc * g.lowerThr;
  return !aboveLower;
}
// isSwapViolatingLimit (:982-1003): the broker check, then for a host resource the host check
template <class V>
CCMI_HD bool resSwapViolating(const DevGoal& g, const V& v, double delta, int sb, int db) {
  const bool broker = resSwapContainerViolating(g, v, delta, sb, db, false);
  if (!broker || !isHostRes(uniform(g.resource)) || !v.hostMode()) return broker;
  return resSwapContainerViolating(g, v, delta, sb, db, true);
}

template <class V>
CCMI_HD bool resAcceptMove(const DevGoal& g, const V& v, int action, int r, int src, int dst) {
  if (action == DA_LEADERSHIP && (uniform(g.resource) == 3 /*DISK*/ || uniform(g.resource) == 1 /*NW_IN*/)) return true;
  const double ru = v.ru(r, uniform(g.resource));
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
  const double delta = v.ru(dr, uniform(g.resource)) - v.ru(sr, uniform(g.resource));
  if (delta == 0) return 0;
  const bool both = delta > 0
                        ? (resAboveLowerAfter(g, v, db, 0.0, true) && resUnderUpperAfter(g, v, sb, 0.0, false, g.upperThr))
                        : (resAboveLowerAfter(g, v, sb, 0.0, true) && resUnderUpperAfter(g, v, db, 0.0, false, g.upperThr));
  if (both) return resSwapViolating(g, v, delta, sb, db) ? 1 : 0;
  return resGettingMoreBalanced(g, v, sb, delta, db) ? 0 : 1;
}

// ---------------------------------------------------------------- RackAwareGoal
// doesReplicaMoveViolateActionAcceptance: another broker of the partition sits on the destination's rack
template <class V>
CCMI_HD bool rackViolates(const V& v, int r, int dst) {
  return v.otherOnRack(v.rpart(r), v.rbroker(r), v.rack(dst));
}

// ---------------------------------------------------------------- RackAwareDistributionGoal
// doesReplicaMoveViolateActionAcceptance (RackAwareDistributionGoal.java:88-104): a move to another rack may not
// leave the destination rack with at least as many of the partition's replicas as the source rack had
template <class V>
CCMI_HD bool rackDistViolates(const V& v, int r, int dst) {
  const int p = v.rpart(r);
  const int srk = v.slotRack(p, v.rbroker(r)), drk = v.rack(dst);
  if (srk == drk) return false;
  return v.rackCount(p, drk) >= v.rackCount(p, srk);
}

// ---------------------------------------------------------------- BrokerSetAwareGoal
CCMI_HD bool bsetMust(int e) { return e >= 0 && (e & kBsetMust) != 0; }
CCMI_HD int bsetIndex(int e) { return e >= 0 ? (e & (kBsetMust - 1)) : e; }
// doesReplicaMoveViolateActionAcceptance (BrokerSetAwareGoal.java:266-279): the destination's broker set differs from
// the set the mapping policy gives the replica
template <class V>
CCMI_HD bool bsetViolates(const V& v, int r, int dst) {
  return bsetIndex(v.rbset(r)) != v.bset(dst);
}
// actionAcceptance (:256-283): a MinTopicLeadersPerBrokerGoal topic of the (source) replica is accepted whatever the
// action; otherwise the source replica's side is a BROKER_REJECT and the swapped replica's side a REPLICA_REJECT
template <class V>
CCMI_HD bool bsetAcceptMove(const V& v, int action, int r, int dst) {
  if (bsetMust(v.rbset(r)) || action == DA_LEADERSHIP) return true;
  return !bsetViolates(v, r, dst);
}
template <class V>
CCMI_HD int bsetAcceptSwap(const V& v, int sr, int sb, int dr, int db) {
  if (bsetMust(v.rbset(sr))) return 0;
  if (bsetViolates(v, sr, db)) return 2;
  return bsetViolates(v, dr, sb) ? 1 : 0;
}

// ---------------------------------------------------------------- MinTopicLeadersPerBrokerGoal
// doesLeaderRemoveViolateOptimizedGoal for replica r on broker b (MinTopicLeadersPerBrokerGoal.java:141-153)
template <class V>
CCMI_HD bool minLeadRemoveViolates(const V& v, int r, int b) {
  if (!(v.flags(r) & RF_LEADER)) return false;
  const int t = v.ptopic(v.rpart(r));
  const int mn = v.tMinLead(t);
  return mn >= 0 && v.tlead(t, b) <= mn;
}
// actionAcceptance (:97-131): actions on other topics are accepted (actionAffectsRelevantTopics :265-271); a move or
// leadership move may not take the source below its minimum; acceptReplicaSwap (:116-131)
template <class V>
CCMI_HD bool minLeadAcceptMove(const V& v, int r, int src) {
  return v.tMinLead(v.ptopic(v.rpart(r))) < 0 || !minLeadRemoveViolates(v, r, src);
}
template <class V>
CCMI_HD int minLeadAcceptSwap(const V& v, int sr, int sb, int dr, int db) {
  const int ts = v.ptopic(v.rpart(sr)), td = v.ptopic(v.rpart(dr));
  if (v.tMinLead(ts) < 0 && v.tMinLead(td) < 0) return 0;
  const bool sl = (v.flags(sr) & RF_LEADER) != 0, dl = (v.flags(dr) & RF_LEADER) != 0;
  if (!sl && !dl) return 0;
  if (sl && dl && ts == td) return 0;
  return (minLeadRemoveViolates(v, sr, sb) || minLeadRemoveViolates(v, dr, db)) ? 1 : 0;
}

// ---------------------------------------------------------------- CapacityGoal
// isUtilizationUnderLimitAfterAddingLoad (CapacityGoal.java:455-475): the host check for a host resource, the broker
// check for a broker resource
template <class V>
CCMI_HD bool capUnderAfterAdding(const DevGoal& g, const V& v, int b, double u) {
  const int res = uniform(g.resource);
  if (!v.hostMode()) {  // one check: the host check of a host-only resource keeps its NaN behaviour
    const double x = v.bu(b, res) + u, lim = v.bcap(b, res) * g.capThr;
    return isBrokerRes(res) ? x < lim : !(x >= lim);
  }
  if (isHostRes(res) && v.hu(b, res) + u >= v.hcap(b, res) * g.capThr) return false;
  if (isBrokerRes(res)) return v.bu(b, res) + u < v.bcap(b, res) * g.capThr;
  return true;
}

// ---------------------------------------------------------------- PotentialNwOutGoal
template <class V>
CCMI_HD bool potSelfSatisfiedMove(const DevGoal& g, const V& v, int action, int r, int dst) {
  if (g.fixOffline && currentOffline(v, r)) return action == DA_MOVE;
  const double destCap = v.bcap(dst, 2) * g.capThr;
  return destCap >= v.pot(dst) + v.pLeadNwOut(v.rpart(r));
}
template <class V>
CCMI_HD bool potAcceptMove(const DevGoal& g, const V& v, int action, int r, int src, int dst) {
  if (action == DA_LEADERSHIP) return true;
  if (potSelfSatisfiedMove(g, v, action, r, dst)) return true;
  const double du = v.pot(dst), su = v.pot(src);
  const double mx = du >= su ? (du == su && du == 0.0 ? (__builtin_signbit(du) ? su : du) : du) : su;  // Math.max
  return du + v.pLeadNwOut(v.rpart(r)) <= mx;
}

// ---------------------------------------------------------------- TopicReplicaDistributionGoal
template <class V>
CCMI_HD bool topicUnderUpperAfterAdd(const V& v, int t, int b) {
  return v.tcount(t, b) + 1 <= (v.alive(b) ? v.tUpper(t) : 0);
}
template <class V>
CCMI_HD bool topicAboveLowerAfterRemove(const V& v, int t, int b) {
  return v.tcount(t, b) - 1 >= (v.alive(b) ? v.tLower(t) : 0);
}
template <class V>
CCMI_HD bool topicAcceptMove(const DevGoal& g, const V& v, int action, int r, int src, int dst) {
  if (action == DA_LEADERSHIP) return true;
  const int t = v.ptopic(v.rpart(r));
  return topicUnderUpperAfterAdd(v, t, dst) && (!v.allowed(g.allowedSlot, src) || topicAboveLowerAfterRemove(v, t, src));
}

// ---------------------------------------------------------------- LeaderReplicaDistributionGoal
template <class V>
CCMI_HD bool leaderMovementSatisfiable(const DevGoal& g, const V& v, int src, int dst) {
  if (!(v.nlead(dst) + 1 <= (v.alive(dst) ? g.upper : 0))) return false;
  if (!v.allowed(g.allowedSlot, src)) return true;
  return v.nlead(src) - 1 >= (v.alive(src) ? g.lower : 0);
}
template <class V>
CCMI_HD bool leadAcceptMove(const DevGoal& g, const V& v, int action, int r, int src, int dst) {
  if (action == DA_MOVE && !(v.flags(r) & RF_LEADER)) return true;
  return leaderMovementSatisfiable(g, v, src, dst);
}

// ---------------------------------------------------------------- TopicLeaderReplicaDistributionGoal
// isLeadershipGoalSatisfiable (:231-256): one more leader of topic t on dst stays within its upper limit, and one
// fewer on src stays within its lower limit unless src is excluded for replica moves
template <class V>
CCMI_HD bool tlSatisfiable(const DevGoal& g, const V& v, int t, int src, int dst) {
  if (!(v.tlead(t, dst) + 1 <= (v.alive(dst) ? v.tLeadUpper(t) : 0))) return false;
  if (!v.allowed(g.allowedSlot, src)) return true;
  return v.tlead(t, src) - 1 >= (v.alive(src) ? v.tLeadLower(t) : 0);
}
// actionAcceptance (:181-229): a follower's replica move is accepted; a leader's move and a leadership move are not
// if they unbalance the topic's leaders
template <class V>
CCMI_HD bool tlAcceptMove(const DevGoal& g, const V& v, int action, int r, int src, int dst) {
  if (action == DA_MOVE && !(v.flags(r) & RF_LEADER)) return true;
  return tlSatisfiable(g, v, v.ptopic(v.rpart(r)), src, dst);
}
template <class V>
CCMI_HD int tlAcceptSwap(const DevGoal& g, const V& v, int sr, int sb, int dr, int db) {
  const int st = v.ptopic(v.rpart(sr)), dt = v.ptopic(v.rpart(dr));
  const bool sl = (v.flags(sr) & RF_LEADER) != 0, dl = (v.flags(dr) & RF_LEADER) != 0;
  if ((st == dt && sl && dl) || (!sl && !dl)) return 0;
  if (sl && !dl) return tlSatisfiable(g, v, st, sb, db) ? 0 : 1;
  if (!sl && dl) return tlSatisfiable(g, v, dt, db, sb) ? 0 : 1;
  return (tlSatisfiable(g, v, st, sb, db) && tlSatisfiable(g, v, dt, db, sb)) ? 0 : 1;
}

// ---------------------------------------------------------------- LeaderBytesInDistributionGoal
template <class V>
CCMI_HD double lbiThreshold(const DevGoal& g, const V& v, int b) {
  const double low = g.lbiLowUtil * v.bcap(b, 1);
  const double m = g.lbiMean * g.lbiBalance;
  return m >= low ? (m == low && m == 0.0 ? (__builtin_signbit(m) ? low : m) : m) : low;  // Math.max
}
template <class V>
CCMI_HD bool lbiAcceptMove(const DevGoal& g, const V& v, int action, int r, int dst) {
  if (!(v.flags(r) & RF_LEADER)) return true;  // replica move of a follower (leadership moves start at a leader)
  const double newDest = v.lnwin(dst) + v.ru(r, 1);
  return !(newDest > lbiThreshold(g, v, dst));
}

// ---------------------------------------------------------------- dispatch
template <class V>
CCMI_HD bool goalAcceptMove(const DevGoal& g, const V& v, int action, int r, int src, int dst) {
  switch (uniform(g.kind)) {
    case DG_REPLICA_DISTRIBUTION: return rdAccept(g, v, action, src, dst);
    case DG_RESOURCE_DISTRIBUTION: return resAcceptMove(g, v, action, r, src, dst);
    case DG_RACK_AWARE: return action == DA_LEADERSHIP || !rackViolates(v, r, dst);
    case DG_RACK_AWARE_DISTRIBUTION: return action == DA_LEADERSHIP || !rackDistViolates(v, r, dst);
    case DG_BROKER_SET_AWARE: return bsetAcceptMove(v, action, r, dst);
    case DG_MIN_TOPIC_LEADERS: return minLeadAcceptMove(v, r, src);
    case DG_REPLICA_CAPACITY: return action == DA_LEADERSHIP || (int64_t)v.nrep(dst) < g.maxReplicas;
    case DG_CAPACITY:
      if (action == DA_LEADERSHIP && (uniform(g.resource) == 3 /*DISK*/ || uniform(g.resource) == 1 /*NW_IN*/)) return true;
      return capUnderAfterAdding(g, v, dst, v.ru(r, uniform(g.resource)));
    case DG_POTENTIAL_NW_OUT: return potAcceptMove(g, v, action, r, src, dst);
    case DG_TOPIC_REPLICA_DISTRIBUTION: return topicAcceptMove(g, v, action, r, src, dst);
    case DG_LEADER_REPLICA_DISTRIBUTION: return leadAcceptMove(g, v, action, r, src, dst);
    case DG_LEADER_BYTES_IN: return lbiAcceptMove(g, v, action, r, dst);
    case DG_TOPIC_LEADER_DISTRIBUTION: return tlAcceptMove(g, v, action, r, src, dst);
    default: return true;  // DG_ACCEPT_ALL
  }
}
template <class V>
CCMI_HD bool goalSelfSatisfiedMove(const DevGoal& g, const V& v, int action, int r, int src, int dst) {
  switch (uniform(g.kind)) {
    case DG_REPLICA_DISTRIBUTION:
      if (g.fixOffline && currentOffline(v, r)) return true;
      return rdAccept(g, v, action, src, dst);
    case DG_RESOURCE_DISTRIBUTION: break;
    case DG_RACK_AWARE:
    case DG_RACK_AWARE_DISTRIBUTION:
    case DG_BROKER_SET_AWARE: return true;
    case DG_ACCEPT_ALL: return action == DA_MOVE;  // MinTopicLeadersPerBrokerGoal moves offline replicas only
    case DG_MIN_TOPIC_LEADERS: {  // selfSatisfied (MinTopicLeadersPerBrokerGoal.java:252-263)
      if (currentOffline(v, r)) return action == DA_MOVE;
      const int t = v.ptopic(v.rpart(r));
      return v.tlead(t, src) > v.tMinLead(t);
    }
    case DG_REPLICA_CAPACITY: return (int64_t)v.nrep(dst) < g.maxReplicas;
    case DG_CAPACITY: return capUnderAfterAdding(g, v, dst, v.ru(r, uniform(g.resource)));
    case DG_POTENTIAL_NW_OUT: return potSelfSatisfiedMove(g, v, action, r, dst);
    case DG_TOPIC_REPLICA_DISTRIBUTION:
      if (g.fixOffline && currentOffline(v, r)) return action == DA_MOVE;
      return topicAcceptMove(g, v, DA_MOVE, r, src, dst);
    case DG_LEADER_REPLICA_DISTRIBUTION:
      if (g.fixOffline && currentOffline(v, r)) return true;
      return leadAcceptMove(g, v, action, r, src, dst);
    case DG_LEADER_BYTES_IN: return lbiAcceptMove(g, v, action, r, dst);
    case DG_TOPIC_LEADER_DISTRIBUTION:  // selfSatisfied (:359-374)
      if (g.fixOffline && currentOffline(v, r)) return action == DA_MOVE;
      return tlSatisfiable(g, v, v.ptopic(v.rpart(r)), src, dst);
    default: return true;
  }
  if (g.fixOffline && currentOffline(v, r)) return action == DA_MOVE;
  const double ru = v.ru(r, uniform(g.resource));
  return resUnderUpperAfter(g, v, dst, ru, true, g.upperThr) && resAboveLowerAfter(g, v, src, ru, false);
}
// returns 0 ACCEPT, 1 REPLICA_REJECT, 2 BROKER_REJECT
template <class V>
CCMI_HD int goalAcceptSwap(const DevGoal& g, const V& v, int sr, int sb, int dr, int db) {
  switch (uniform(g.kind)) {
    case DG_RESOURCE_DISTRIBUTION: return resAcceptSwap(g, v, sr, sb, dr, db);
    case DG_RACK_AWARE:
      if (rackViolates(v, sr, db)) return 2;
      return rackViolates(v, dr, sb) ? 1 : 0;
    case DG_RACK_AWARE_DISTRIBUTION:
      if (rackDistViolates(v, sr, db)) return 2;
      return rackDistViolates(v, dr, sb) ? 1 : 0;
    case DG_BROKER_SET_AWARE: return bsetAcceptSwap(v, sr, sb, dr, db);
    case DG_MIN_TOPIC_LEADERS: return minLeadAcceptSwap(v, sr, sb, dr, db);
    case DG_CAPACITY: {
      const double su = v.ru(sr, uniform(g.resource)), du = v.ru(dr, uniform(g.resource));
      const double delta = du - su;
      return (delta > 0 ? capUnderAfterAdding(g, v, sb, delta) : capUnderAfterAdding(g, v, db, -delta)) ? 0 : 1;
    }
    case DG_POTENTIAL_NW_OUT: {
      // selfSatisfied (swap form) first, then the max-utilization bound
      const double sU = v.pLeadNwOut(v.rpart(sr)), dU = v.pLeadNwOut(v.rpart(dr));
      const double destU = v.pot(db), srcU = v.pot(sb);
      bool self;
      if (g.fixOffline && currentOffline(v, sr)) {
        self = false;
      } else {
        const double destCap = v.bcap(db, 2) * g.capThr, srcCap = v.bcap(sb, 2) * g.capThr;
        self = !(destCap < destU + sU - dU) && srcCap >= srcU + dU - sU;
      }
      if (self) return 0;
      const double mx = destU >= srcU ? (destU == srcU && destU == 0.0 ? (__builtin_signbit(destU) ? srcU : destU) : destU)
                                      : srcU;
      if (srcU + dU - sU > mx) return 1;
      return destU + sU - dU <= mx ? 0 : 1;
    }
    case DG_TOPIC_REPLICA_DISTRIBUTION: {
      const int st = v.ptopic(v.rpart(sr)), dt = v.ptopic(v.rpart(dr));
      if (st == dt) return 0;
      const bool s2d = topicUnderUpperAfterAdd(v, st, db) && topicAboveLowerAfterRemove(v, st, sb);
      return (s2d && topicUnderUpperAfterAdd(v, dt, sb) && topicAboveLowerAfterRemove(v, dt, db)) ? 0 : 1;
    }
    case DG_LEADER_REPLICA_DISTRIBUTION: {
      const bool sl = (v.flags(sr) & RF_LEADER) != 0, dl = (v.flags(dr) & RF_LEADER) != 0;
      if (sl && !dl) return leaderMovementSatisfiable(g, v, sb, db) ? 0 : 1;
      if (!sl && dl) return leaderMovementSatisfiable(g, v, db, sb) ? 0 : 1;
      return 0;
    }
    case DG_LEADER_BYTES_IN: {
      const bool sl = (v.flags(sr) & RF_LEADER) != 0, dl = (v.flags(dr) & RF_LEADER) != 0;
      if (!sl && !dl) return 0;
      const double srU = v.ru(sr, 1), drU = v.ru(dr, 1);
      const double newDest = v.lnwin(db) + srU - drU;
      const double newSrc = v.lnwin(sb) + drU - srU;
      if (newSrc > lbiThreshold(g, v, sb)) return 1;
      return !(newDest > lbiThreshold(g, v, db)) ? 0 : 1;
    }
    case DG_TOPIC_LEADER_DISTRIBUTION: return tlAcceptSwap(g, v, sr, sb, dr, db);
    default: return 0;  // ReplicaDistribution, ReplicaCapacity, MinTopicLeaders accept swaps
  }
}
template <class V>
CCMI_HD bool goalSelfSatisfiedSwap(const DevGoal& g, const V& v, int sr, int sb, int dr, int db) {
  if (uniform(g.kind) == DG_REPLICA_DISTRIBUTION) {
    if (g.fixOffline && currentOffline(v, sr)) return true;
    return true;  // rdAccept(SWAP) == ACCEPT
  }
  if (g.fixOffline && currentOffline(v, sr)) return false;  // action != INTER_BROKER_REPLICA_MOVEMENT
  const double delta = v.ru(dr, uniform(g.resource)) - v.ru(sr, uniform(g.resource));
  return delta != 0 && !resSwapViolating(g, v, delta, sb, db);
}

// Full candidate predicate of AbstractGoal.maybeApplyBalancingAction's loop body for one (replica, dest):
// legit && selfSatisfied && every optimized goal ACCEPTs.
template <class V>
CCMI_HD bool moveCandidateAccepted(const DevProgram& prog, const V& v, int r, int dst) {
  const int action = uniform(prog.action);
  const int src = v.rbroker(r);
  if (!legitMove(v, r, dst, action)) return false;
  if (!goalSelfSatisfiedMove(prog.goals[0], v, action, r, src, dst)) return false;
  const int nGoals = uniform(prog.nGoals);
  for (int i = 1; i < nGoals; ++i)
    if (!goalAcceptMove(prog.goals[i], v, action, r, src, dst)) return false;
  return true;
}
// moveCandidateAccepted split over `parts` evaluators of the same candidate (the scan server's goal-parallel tiles,
// one wavefront per part): part 0 takes the legitimacy check and the optimizing goal, the prior goals go round robin
// (goal i to part i % parts). The candidate is accepted iff every part accepts it — the same conjunction, since every
// check is a pure function of the view; only the order of evaluation (and the early exit) differs.
template <class V>
CCMI_HD bool moveCandidateAcceptedPart(const DevProgram& prog, const V& v, int r, int dst, int part, int parts) {
  const int action = uniform(prog.action);
  const int src = v.rbroker(r);
  part = uniform(part);
  if (part == 0) {
    if (!legitMove(v, r, dst, action)) return false;
    if (!goalSelfSatisfiedMove(prog.goals[0], v, action, r, src, dst)) return false;
  }
  const int nGoals = uniform(prog.nGoals);
  for (int i = part == 0 ? parts : part; i < nGoals; i += parts)
    if (!goalAcceptMove(prog.goals[i], v, action, r, src, dst)) return false;
  return true;
}

// GoalUtils.eligibleReplicasForSwap (GoalUtils.java:258-274): a swap row is empty when the destination broker is
// excluded for leadership and the (originally online) source replica is a leader, or the destination is excluded
// for replica moves and the source replica is originally online.
// GoalUtils.eligibleBrokers' replica-dependent filters for a (replica, destination) candidate of a move or
// leadership scan: a leader replica's move skips brokers excluded for leadership (GoalUtils.java:170-180), and with
// NEW brokers only new brokers or the replica's original broker are eligible (:193-198). (PreView, which caches the
// destination's bits, has its own copy: exclLeadBlocked.)
template <class V>
CCMI_HD bool candidateBlocked(const DevProgram& prog, const V& v, int r, int db) {
  if (prog.exclLeadMove && (v.flags(r) & RF_LEADER) && v.allowed(kExclLeadBit, db)) return true;
  return prog.newOnly && !v.allowed(kNewBit, db) && db != v.rorig(r);
}

// With NEW brokers, a row is kept only when the source broker is new and the destination is new or the source
// replica's original broker (CASE#1); the CASE#2 rows (old source, new destination) are the host's (Engine::swapScan).
template <class V>
CCMI_HD bool swapRowExcluded(const DevProgram& prog, const V& v, int sr, int db) {
  if (prog.swapExcl && !v.origOff(sr)) {
    if (v.allowed(kExclMoveBit, db)) return true;
    if ((v.flags(sr) & RF_LEADER) && v.allowed(kExclLeadBit, db)) return true;
  }
  if (prog.newOnly) {
    const int sb = v.rbroker(sr);
    if (!(v.allowed(kNewBit, sb) && (v.allowed(kNewBit, db) || v.rorig(sr) == db))) return true;
  }
  return false;
}

// One step of AbstractGoal.maybeApplySwapAction's loop for (source sr, destination replica dr on db):
// returns 0 = continue, 1 = terminal ACCEPT, 2 = terminal null (return null).
template <class V>
CCMI_HD int swapCandidateOutcome(const DevProgram& prog, const V& v, int sr, int dr, int db) {
  const int sb = v.rbroker(sr);
  if (!legitMove(v, sr, db, DA_MOVE)) return 2;
  if (!legitMove(v, dr, sb, DA_MOVE)) return 0;
  if (!goalSelfSatisfiedSwap(prog.goals[0], v, sr, sb, dr, db)) return 2;
  const int nGoals = uniform(prog.nGoals);
  for (int i = 1; i < nGoals; ++i) {
    const int acc = goalAcceptSwap(prog.goals[i], v, sr, sb, dr, db);
    if (acc == 1) return 0;
    if (acc == 2) return 2;
  }
  return 1;
}

}  // namespace ccmi
