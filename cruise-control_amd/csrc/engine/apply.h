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
#pragma once
#include "devtypes.h"
#include "loadops.h"

namespace ccmi {

// S provides: W; LoadVec& rLoad(r), bLoad(b), bLnw(b), bPot(b); ReplicaRec& rep(r); BrokerRec& brk(b);
// PartitionRec& part(p); int& slot(p, i) (replica id of partition slot i); int& leader(p); void topicAdd(t, b, d).
template <class S>
CCMI_LD void applyRefreshBroker(S& s, int b) {
  BrokerRec& x = s.brk(b);
  for (int k = 0; k < 4; ++k) x.util[k] = ldUtil(s.bLoad(b), k, s.W);
  x.pot = ldUtil(s.bPot(b), R_NW_OUT, s.W);
  x.lbi = ldUtil(s.bLnw(b), R_NW_IN, s.W);
}
template <class S>
CCMI_LD void applyRefreshReplica(S& s, int r) {
  for (int k = 0; k < 4; ++k) s.rep(r).util[k] = ldUtil(s.rLoad(r), k, s.W);
}

// relocateReplica(tp, src, dst) of replica r (its broker is the source)
template <class S>
CCMI_LD void applyRelocateReplica(S& s, int r, int dst) {
  ReplicaRec& rr = s.rep(r);
  const int src = rr.broker, p = rr.part;
  const bool lead = (rr.flags & RF_LEADER) != 0;
  // Broker.removeReplica(src)
  ldSubAll(s.bLoad(src), s.rLoad(r), s.W);
  if (lead) {
    ldSubAll(s.bLnw(src), s.rLoad(r), s.W);
    s.brk(src).nlead -= 1;
  }
  s.brk(src).nrep -= 1;
  // _potentialLeadershipLoadByBrokerId
  const int lr = s.leader(p);
  ldSubAll(s.bPot(src), s.rLoad(lr), s.W);
  rr.broker = dst;
  // Broker.addReplica(dst)
  if (lead) {
    ldAddAll(s.bLnw(dst), s.rLoad(r), s.W);
    s.brk(dst).nlead += 1;
  }
  ldAddAll(s.bLoad(dst), s.rLoad(r), s.W);
  s.brk(dst).nrep += 1;
  ldAddAll(s.bPot(dst), s.rLoad(lr), s.W);
  applyRefreshBroker(s, src);
  applyRefreshBroker(s, dst);
  PartitionRec& pr = s.part(p);
  for (int i = 0; i < pr.n; ++i)
    if (s.slot(p, i) == r) {
      pr.brokers[i] = dst;
      pr.racks[i] = (int16_t)s.brk(dst).rack;
    }
  s.topicAdd(pr.topic, src, -1);
  s.topicAdd(pr.topic, dst, +1);
}

// relocateLeadership(tp, src, dst): src's replica of p must be the leader, dst's a follower
template <class S>
CCMI_LD void applyRelocateLeadership(S& s, int p, int src, int dst) {
  PartitionRec& pr = s.part(p);
  int sr = -1, dr = -1, dpos = 0;
  for (int i = 0; i < pr.n; ++i) {
    const int x = s.slot(p, i);
    if (s.rep(x).broker == src) sr = x;
    if (s.rep(x).broker == dst) {
      dr = x;
      dpos = i;
    }
  }
  // Broker.makeFollower(src)
  ldSubAll(s.bLnw(src), s.rLoad(sr), s.W);
  LoadVec delta;
  ldMakeFollower(s.rLoad(sr), delta, s.W);
  s.rep(sr).flags &= ~(int32_t)RF_LEADER;
  applyRefreshReplica(s, sr);
  if (s.bLoad(src).mask) ldSubAll(s.bLoad(src), delta, s.W);
  s.brk(src).nlead -= 1;
  // Broker.makeLeader(dst)
  s.rep(dr).flags |= (int32_t)RF_LEADER;
  if (s.rLoad(dr).mask) ldAddAll(s.rLoad(dr), delta, s.W);
  applyRefreshReplica(s, dr);
  ldAddAll(s.bLnw(dst), s.rLoad(dr), s.W);
  if (s.bLoad(dst).mask) ldAddAll(s.bLoad(dst), delta, s.W);
  s.brk(dst).nlead += 1;
  // Partition.relocateLeadership: swap positions 0 and indexOf(dr)
  const int first = s.slot(p, 0);
  s.slot(p, 0) = dr;
  s.slot(p, dpos) = first;
  s.leader(p) = dr;
  const int b0 = pr.brokers[0];
  pr.brokers[0] = pr.brokers[dpos];
  pr.brokers[dpos] = b0;
  const int16_t k0 = pr.racks[0];
  pr.racks[0] = pr.racks[dpos];
  pr.racks[dpos] = k0;
  pr.leadNwOut = s.rep(dr).util[R_NW_OUT];
  applyRefreshBroker(s, src);
  applyRefreshBroker(s, dst);
}

}  // namespace ccmi
