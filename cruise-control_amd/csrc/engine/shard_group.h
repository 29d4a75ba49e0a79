// Shard groups (ccmi_shard_group_*, ABI v11): the ranks of one destination-sharded proposal driven from ONE process —
// one host thread per session, typically one session per GPU of the node — MIN-combine each scan's first-fit key in a
// block of pinned host memory that every device of the process maps. A scan the rank's resident scan server ran is
// combined by the server itself (its last workgroup to finish the scan folds the rank's key into the slot, waits for
// the other ranks' arrivals with system-scope atomics — PCIe / xGMI atomics on host memory — and publishes the group's
// minimum as the scan's result, kernels/scan.hip); a scan that ran as a launch is combined by the rank's host thread
// with the same protocol on the same slot (groupHostMin). Every rank makes the same sequence of combines (identical
// host drivers), so the two slots are used alternately: a slot's last rank out resets it, and no rank reaches that
// slot again before every rank has arrived at the other one, which the resetting rank does only after its reset.
#pragma once
#include <cstdint>

namespace ccmi {

// One slot per combine parity, on lines of their own. minKey: ~0 = no accepted candidate.
struct alignas(64) CombineSlot {
  unsigned long long minKey;
  unsigned int arrived;
  unsigned int departed;
  char pad[48];
};
struct CombineBlock {
  CombineSlot slot[2];
};
static_assert(sizeof(CombineSlot) == 64, "one line per slot");

constexpr unsigned long long kCombineNone = ~0ull;

// The host side of one combine on `slot` (host pointer), for `count` ranks: fold key (-1 = none) in, wait for every
// rank, return the group minimum (-1 = none). Throws std::runtime_error after `timeoutSeconds` without every rank.
int64_t groupHostMin(CombineSlot* slot, int count, int64_t key, double timeoutSeconds);
void initCombineBlock(CombineBlock* b);

}  // namespace ccmi
