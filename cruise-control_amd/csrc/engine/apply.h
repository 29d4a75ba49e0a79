// Move application written once for the gfx950 chain kernels (kernels/scan.hip) and the test-only sequential
// device emulation (tests/emu): the device-resident records a scan reads (BrokerRec / ReplicaRec / PartitionRec /
// topic counts, devtypes.h) are recomputed from the device copies of the Java loads exactly as the host model does it
// (model.cpp relocateReplica / relocateLeadership), so a chain kernel can apply a move and go on scanning, and the
// host replays the same moves into its own model afterwards.
//   ClusterModel.relocateReplica     model/ClusterModel.java:380-396 (removeReplica :546-564)
//   ClusterModel.relocateLeadership  model/ClusterModel.java:409-441
//   Broker.addReplica / removeReplica / makeFollower / makeLeader  model/Broker.java:336-510
//   Replica.makeFollower / makeLeader model/Replica.java:210-310
//   Partition.relocateLeadership     model/Partition.java:243-247
//
// A move changes up to six load aggregates, each by exactly one add or subtract, so the aggregates are updated by
// "lanes" that run in parallel on the device (one wavefront, lane-dependent addresses, one memory round trip) and one
// after the other in the emulation. Steps separate the lanes that depend on each other (leadership: the follower
// CPU delta first). The record fields each lane writes are disjoint.
#pragma once
#include "devtypes.h"
#include "loadops.h"

namespace ccmi {

CCMI_LD void ldCopy(LoadVec& d, const LoadVec& s, int W) {  // the W live windows of every metric
  d.mask = s.mask;
  for (int k = 0; k < 6; ++k) {
    for (int i = 0; i < W; ++i) d.m[k].v[i] = s.m[k].v[i];
    d.m[k].sum = s.m[k].sum;
  }
}
// ldAddAll (neg = false) / ldSubAll (neg = true): x - y is x + (-y) in IEEE arithmetic, so one instruction stream
// serves both; a missing metric is created only by an add (a subtract always finds it)
CCMI_LD void ldAddSignedAll(LoadVec& d, const LoadVec& s, int W, bool neg) {
  for (int k = 0; k < 6; ++k)
    if (s.mask >> k & 1) {
      if (!(d.mask >> k & 1)) {
        ldZero(d.m[k], W);
        d.mask |= (uint8_t)(1 << k);
      }
      for (int i = 0; i < W; ++i) {
        const double x = neg ? -(double)s.m[k].v[i] : (double)s.m[k].v[i];
        d.m[k].v[i] = (float)((double)d.m[k].v[i] + x);
        d.m[k].sum += x;
      }
    }
}

// S provides: W; LoadVec& rLoad(r), bLoad(b), bLnw(b), bPot(b), scratch(i) (i = 0, 1: step-to-step values);
// ReplicaRec& rep(r); BrokerRec& brk(b); PartitionRec& part(p); int& slot(p, i) (replica id of partition slot i);
// int& leader(p); void topicAdd(t, b, d); void topicLeadAdd(t, b, d) (a no-op unless leader counts are kept);
// bool hostsOn() (brokers share hosts), int host(b), LoadVec& hLoad(h), int hostBegin(h), hostEnd(h), hostBroker(i).
//
// Hosts (Model::sharedHosts): Host.addReplica / removeReplica add / subtract the replica's load (model/Host.java), and
// Host.makeFollower / makeLeader the leadership CPU / NW_OUT delta when the host has metrics. Each host aggregate gets
// one operation per broker of the move, in the reference's order (the source's first): two hosts take one lane each,
// one host shared by source and destination takes both operations on one lane. Every broker of a touched host then
// reads its host utilization (BrokerRec.hutil) again; without shared hosts hutil is the broker's own util.

// ---- relocateReplica(tp, src, dst) of replica r: lanes 0..5, then applyReplicaFinish
//   lane 0/1 Broker.load() of src (-= r) / dst (+= r)         -> util[4]
//   lane 2/3 potential leadership load of src / dst (+-= leader of p) -> pot
//   lane 4/5 leadership NW load of src / dst (+-= r, leaders only)    -> lbi
constexpr int kReplicaLanes = 6;
template <class S>
CCMI_LD void applyReplicaLane(S& s, int lane, int r, int src, int dst, int lr, bool lead) {
  if (lane >= kReplicaLanes || (lane >= 4 && !lead)) return;
  const int b = (lane & 1) ? dst : src;
  LoadVec& t = lane < 2 ? s.bLoad(b) : (lane < 4 ? s.bPot(b) : s.bLnw(b));
  LoadVec x, o;
  ldCopy(x, t, s.W);
  ldCopy(o, (lane == 2 || lane == 3) ? s.rLoad(lr) : s.rLoad(r), s.W);
  ldAddSignedAll(x, o, s.W, !(lane & 1));
  ldCopy(t, x, s.W);
  BrokerRec& rec = s.brk(b);
  if (lane < 2) {
    for (int k = 0; k < 4; ++k) rec.util[k] = ldUtil(x, k, s.W);
    if (!s.hostsOn())  // one broker per host: the host values are the broker's
      for (int k = 0; k < 3; ++k) rec.hutil[k] = rec.util[k];
  } else if (lane < 4) {
    rec.pot = ldUtil(x, R_NW_OUT, s.W);
  } else {
    rec.lbi = ldUtil(x, R_NW_IN, s.W);
  }
}
// counts, the replica's broker, its partition slot and the topic counts, after the lanes: independent fields, one
// finish lane each (kReplicaFinishLanes, in parallel on the device)
constexpr int kReplicaFinishLanes = 8;
template <class S>
CCMI_LD void applyReplicaFinishLane(S& s, int lane, int r, int p, int src, int dst, bool lead) {
  switch (lane) {
    case 0:
      s.brk(src).nrep -= 1;
      if (lead) s.brk(src).nlead -= 1;
      break;
    case 1:
      s.brk(dst).nrep += 1;
      if (lead) s.brk(dst).nlead += 1;
      break;
    case 2: s.rep(r).broker = dst; break;
    case 3: {
      PartitionRec& pr = s.part(p);
      const int16_t rk = (int16_t)s.brk(dst).rack;
      for (int i = 0; i < kMaxRf; ++i)
        if (i < pr.n && s.slot(p, i) == r) {
          pr.brokers[i] = dst;
          pr.racks[i] = rk;
        }
      break;
    }
    case 4: s.topicAdd(s.part(p).topic, src, -1); break;
    case 5: s.topicAdd(s.part(p).topic, dst, +1); break;
    case 6:
      if (lead) s.topicLeadAdd(s.part(p).topic, src, -1);
      break;
    case 7:
      if (lead) s.topicLeadAdd(s.part(p).topic, dst, +1);
      break;
    default: break;
  }
}
template <class S>
CCMI_LD void applyReplicaFinish(S& s, int r, int src, int dst, bool lead) {
  const int p = s.rep(r).part;
  for (int l = 0; l < kReplicaFinishLanes; ++l) applyReplicaFinishLane(s, l, r, p, src, dst, lead);
}

// ---- relocateLeadership(tp, src, dst) of the leader sr (on src) to the follower dr (on dst)
//   step 0: lane 0 leadership NW load of src -= sr (its load before makeFollower)            -> src lbi
//           lane 1 makeFollower on a copy of sr's load: scratch(0) = delta, scratch(1) = new load of sr
//   step 1: lane 0 Broker.load() of src -= delta (when it has metrics)                          -> src util
//           lane 1 Broker.load() of dst += delta (when it has metrics)                          -> dst util
//           lane 2 dr's load += delta (when it has metrics)                                    -> dr util, leader flag
//           lane 3 sr's load = scratch(1)                                                       -> sr util, leader flag
//   step 2: lane 0 leadership NW load of dst += dr's new load                                  -> dst lbi
// then applyLeadershipFinish: leader counts, Partition.relocateLeadership and the partition record
constexpr int kLeadershipSteps = 3;
template <class S>
CCMI_LD void applyLeadershipLane(S& s, int step, int lane, int sr, int dr, int src, int dst) {
  LoadVec x, o;
  if (step == 0) {
    if (lane == 0) {
      ldCopy(x, s.bLnw(src), s.W);
      ldCopy(o, s.rLoad(sr), s.W);
      ldAddSignedAll(x, o, s.W, true);
      ldCopy(s.bLnw(src), x, s.W);
      s.brk(src).lbi = ldUtil(x, R_NW_IN, s.W);
    } else if (lane == 1) {
      ldCopy(x, s.rLoad(sr), s.W);
      ldMakeFollower(x, o, s.W);
      ldCopy(s.scratch(0), o, s.W);
      ldCopy(s.scratch(1), x, s.W);
    }
  } else if (step == 1) {
    if (lane > 3) return;
    if (lane == 3) {
      ldCopy(x, s.scratch(1), s.W);
      ldCopy(s.rLoad(sr), x, s.W);
      ReplicaRec& rec = s.rep(sr);
      rec.flags &= ~(int32_t)RF_LEADER;
      for (int k = 0; k < 4; ++k) rec.util[k] = ldUtil(x, k, s.W);
      return;
    }
    LoadVec& t = lane == 0 ? s.bLoad(src) : (lane == 1 ? s.bLoad(dst) : s.rLoad(dr));
    ldCopy(x, t, s.W);
    if (x.mask) {
      ldCopy(o, s.scratch(0), s.W);
      ldAddSignedAll(x, o, s.W, lane == 0);
      ldCopy(t, x, s.W);
    }
    if (lane < 2) {
      BrokerRec& rec = s.brk(lane == 0 ? src : dst);
      for (int k = 0; k < 4; ++k) rec.util[k] = ldUtil(x, k, s.W);
      if (!s.hostsOn())
        for (int k = 0; k < 3; ++k) rec.hutil[k] = rec.util[k];
    } else {
      ReplicaRec& rec = s.rep(dr);
      rec.flags |= (int32_t)RF_LEADER;
      for (int k = 0; k < 4; ++k) rec.util[k] = ldUtil(x, k, s.W);
    }
  } else if (lane == 0) {
    ldCopy(x, s.bLnw(dst), s.W);
    ldCopy(o, s.rLoad(dr), s.W);
    ldAddSignedAll(x, o, s.W, false);
    ldCopy(s.bLnw(dst), x, s.W);
    s.brk(dst).lbi = ldUtil(x, R_NW_IN, s.W);
  }
}
// leader counts, Partition.relocateLeadership (slots and leader), the partition record and the topic leader counts:
// independent fields, one finish lane each (kLeadershipFinishLanes, in parallel on the device)
constexpr int kLeadershipFinishLanes = 6;
template <class S>
CCMI_LD void applyLeadershipFinishLane(S& s, int lane, int p, int dr, int dpos, int src, int dst) {
  switch (lane) {
    case 0: s.brk(src).nlead -= 1; break;
    case 1: s.brk(dst).nlead += 1; break;
    case 2: {
      const int first = s.slot(p, 0);
      s.slot(p, 0) = dr;
      s.slot(p, dpos) = first;
      s.leader(p) = dr;
      break;
    }
    case 3: {
      PartitionRec& pr = s.part(p);
      const int b0 = pr.brokers[0];
      pr.brokers[0] = pr.brokers[dpos];
      pr.brokers[dpos] = b0;
      const int16_t k0 = pr.racks[0];
      pr.racks[0] = pr.racks[dpos];
      pr.racks[dpos] = k0;
      pr.leadNwOut = s.rep(dr).util[R_NW_OUT];
      break;
    }
    case 4: s.topicLeadAdd(s.part(p).topic, src, -1); break;
    case 5: s.topicLeadAdd(s.part(p).topic, dst, +1); break;
    default: break;
  }
}
template <class S>
CCMI_LD void applyLeadershipFinish(S& s, int p, int dr, int dpos, int src, int dst) {
  for (int l = 0; l < kLeadershipFinishLanes; ++l) applyLeadershipFinishLane(s, l, p, dr, dpos, src, dst);
}
// the two replicas of p on src and dst, and dr's slot
template <class S>
CCMI_LD void leadershipReplicas(S& s, int p, int src, int dst, int& sr, int& dr, int& dpos) {
  const PartitionRec& pr = s.part(p);
  sr = dr = -1;
  dpos = 0;
  for (int i = 0; i < kMaxRf; ++i) {
    if (i >= pr.n) break;
    if (pr.brokers[i] == src) sr = s.slot(p, i);
    if (pr.brokers[i] == dst) {
      dr = s.slot(p, i);
      dpos = i;
    }
  }
}

// ---- host aggregates (S::hostsOn()): lane 0 the source's host, lane 1 the destination's when it is another host
//   replica move: Host.removeReplica (src host -= r), Host.addReplica (dst host += r)
constexpr int kHostLanes = 2;
template <class S>
CCMI_LD void applyHostReplicaLane(S& s, int lane, int r, int src, int dst) {
  if (!s.hostsOn() || lane >= kHostLanes) return;
  const int hs = s.host(src), hd = s.host(dst);
  if (lane == 1 && hs == hd) return;
  LoadVec& t = s.hLoad(lane == 0 ? hs : hd);
  LoadVec x, o;
  ldCopy(x, t, s.W);
  ldCopy(o, s.rLoad(r), s.W);
  ldAddSignedAll(x, o, s.W, lane == 0);
  if (lane == 0 && hs == hd) ldAddSignedAll(x, o, s.W, false);
  ldCopy(t, x, s.W);
}
//   leadership (step 1, delta = scratch(0)): Host.makeFollower (src host -= delta), Host.makeLeader (dst host += delta),
//   each only when the host has metrics
template <class S>
CCMI_LD void applyHostLeadershipLane(S& s, int lane, int src, int dst) {
  if (!s.hostsOn() || lane >= kHostLanes) return;
  const int hs = s.host(src), hd = s.host(dst);
  if (lane == 1 && hs == hd) return;
  LoadVec& t = s.hLoad(lane == 0 ? hs : hd);
  LoadVec x, o;
  ldCopy(x, t, s.W);
  if (!x.mask) return;
  ldCopy(o, s.scratch(0), s.W);
  ldAddSignedAll(x, o, s.W, lane == 0);
  if (lane == 0 && hs == hd) ldAddSignedAll(x, o, s.W, false);
  ldCopy(t, x, s.W);
}
// every broker of the move's host(s): BrokerRec.hutil from the host load (ClusterModel.host(...).load()); lanes
// [lane0, ...) stepping by `step` share the brokers
template <class S>
CCMI_LD void applyHostUtil(S& s, int src, int dst, int lane, int step) {
  if (!s.hostsOn()) return;
  const int hs = s.host(src), hd = s.host(dst);
  for (int pass = 0; pass < 2; ++pass) {
    const int h = pass == 0 ? hs : hd;
    if (pass == 1 && hd == hs) break;
    const LoadVec& L = s.hLoad(h);
    for (int i = s.hostBegin(h) + lane; i < s.hostEnd(h); i += step) {
      BrokerRec& rec = s.brk(s.hostBroker(i));
      for (int k = 0; k < 3; ++k) rec.hutil[k] = ldUtil(L, k, s.W);
    }
  }
}

// Sequential form (emulation): every lane of every step in order.
template <class S>
inline void applyRelocateReplica(S& s, int r, int dst) {
  const int src = s.rep(r).broker, lr = s.leader(s.rep(r).part);
  const bool lead = (s.rep(r).flags & RF_LEADER) != 0;
  for (int l = 0; l < kReplicaLanes; ++l) applyReplicaLane(s, l, r, src, dst, lr, lead);
  for (int l = 0; l < kHostLanes; ++l) applyHostReplicaLane(s, l, r, src, dst);
  applyHostUtil(s, src, dst, 0, 1);
  applyReplicaFinish(s, r, src, dst, lead);
}
template <class S>
inline void applyRelocateLeadership(S& s, int p, int src, int dst) {
  int sr, dr, dpos;
  leadershipReplicas(s, p, src, dst, sr, dr, dpos);
  for (int st = 0; st < kLeadershipSteps; ++st) {
    for (int l = 0; l < 4; ++l) applyLeadershipLane(s, st, l, sr, dr, src, dst);
    if (st == 1)
      for (int l = 0; l < kHostLanes; ++l) applyHostLeadershipLane(s, l, src, dst);
  }
  applyHostUtil(s, src, dst, 0, 1);
  applyLeadershipFinish(s, p, dr, dpos, src, dst);
}

}  // namespace ccmi
