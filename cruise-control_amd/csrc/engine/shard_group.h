// Shard groups (ccmi_shard_group_*, ABI v11): the ranks of one destination-sharded proposal driven from ONE process —
// one host thread per session, typically one session per GPU of the node — MIN-combine each scan's first-fit key in a
// block of pinned host memory that every device of the process maps.
//
// A combine never waits inside a kernel. Each rank folds its key into the combine slot (system-scope compare-and-swap
// minimum), leaves a tag saying where its result goes, and counts itself in; the LAST rank to arrive reads the group
// minimum and publishes it to every rank's host mailbox, then resets the slot. A scan the rank's resident scan server
// ran arrives from the server's last workgroup (kernels/scan.hip) and its result goes to mail[0] under the command's
// sequence, where the host already waits for the command; a scan that ran as a launch arrives from the rank's host
// thread (groupHostMin) and its result goes to mail[6] under the rank's combine count. So no rank's GPU is ever held
// waiting for another rank (ranks sharing a GPU, whose launches may queue behind each other's servers, cannot
// deadlock), and whichever side arrives last does the publishing. Every rank makes the same sequence of combines
// (identical host drivers); the two slots alternate, and a slot's resetter arrives at the other slot only after its
// reset, so no rank reaches a slot again before it is clean.
#pragma once
#include <cstdint>

namespace ccmi {

constexpr int kGroupMaxRanks = 16;
constexpr unsigned long long kCombineNone = ~0ull;
// tag of a rank's pending result: kind (1 = server command -> mail[0], 2 = host combine -> mail[6]) << 62 | seq (32 bits)
constexpr unsigned long long kTagServer = 1ull << 62, kTagHost = 2ull << 62;

struct alignas(64) CombineSlot {
  unsigned long long minKey;
  unsigned int arrived;
  unsigned int pad;
  unsigned long long tag[kGroupMaxRanks];
};
struct CombineBlock {
  CombineSlot slot[2];
  unsigned long long mail[kGroupMaxRanks];  // each rank's mailbox (pinned, portable host memory; the same address on
                                            // every device of the process)
};

void initCombineBlock(CombineBlock* b);
// The host side of one combine of rank `rank` on slot `s` (groupCalls & 1): fold key (-1 = none) in; the last rank
// publishes and resets; the others wait for mail[6] of their own mailbox to carry `seq`. Returns the group minimum
// (-1 = none); throws std::runtime_error after `timeoutSeconds` without it.
int64_t groupHostMin(CombineBlock* b, int slot, int rank, int count, int64_t key, uint32_t seq, double timeoutSeconds);

}  // namespace ccmi
