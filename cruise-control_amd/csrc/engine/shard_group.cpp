// Host side of the shard-group combine (shard_group.h).
#include "shard_group.h"

#include <sched.h>

#include <chrono>
#include <stdexcept>

namespace ccmi {

namespace {
double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
}  // namespace

void initCombineBlock(CombineBlock* b) {
  for (CombineSlot& s : b->slot) {
    __atomic_store_n(&s.minKey, kCombineNone, __ATOMIC_RELAXED);
    for (auto& t : s.tag) __atomic_store_n(&t, 0ull, __ATOMIC_RELAXED);
    __atomic_store_n(&s.arrived, 0u, __ATOMIC_RELEASE);
  }
  for (auto& m : b->mail) __atomic_store_n(&m, 0ull, __ATOMIC_RELEASE);
}

int64_t groupHostMin(CombineBlock* b, int slot, int rank, int count, int64_t key, uint32_t seq, double timeoutSeconds) {
  CombineSlot& s = b->slot[slot];
  const unsigned long long k = key < 0 ? kCombineNone : (unsigned long long)key;
  __atomic_store_n(&s.tag[rank], kTagHost | seq, __ATOMIC_RELAXED);
  unsigned long long cur = __atomic_load_n(&s.minKey, __ATOMIC_RELAXED);
  while (k < cur && !__atomic_compare_exchange_n(&s.minKey, &cur, k, true, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED)) {
  }
  if (__atomic_fetch_add(&s.arrived, 1u, __ATOMIC_ACQ_REL) == (unsigned)count - 1) {
    // the last rank in: publish the minimum to every rank's mailbox, then reset the slot
    const unsigned long long g = __atomic_load_n(&s.minKey, __ATOMIC_ACQUIRE);
    const unsigned long long lo = g == kCombineNone ? 0ull : (g + 1) & 0xffffffffull;
    for (int r = 0; r < count; ++r) {
      const unsigned long long t = __atomic_load_n(&s.tag[r], __ATOMIC_ACQUIRE);
      auto* mail = reinterpret_cast<unsigned long long*>(__atomic_load_n(&b->mail[r], __ATOMIC_ACQUIRE));
      if (r == rank) continue;
      __atomic_store_n(&mail[(t >> 62) == 1 ? 0 : 6], ((t & 0xffffffffull) << 32) | lo, __ATOMIC_RELEASE);
    }
    __atomic_store_n(&s.minKey, kCombineNone, __ATOMIC_RELAXED);
    __atomic_store_n(&s.arrived, 0u, __ATOMIC_RELEASE);
    return g == kCombineNone ? -1 : (int64_t)g;
  }
  auto* mine = reinterpret_cast<unsigned long long*>(__atomic_load_n(&b->mail[rank], __ATOMIC_ACQUIRE));
  const double t0 = now();
  for (uint64_t spins = 0;; ++spins) {
    const unsigned long long w = __atomic_load_n(&mine[6], __ATOMIC_ACQUIRE);
    if ((w >> 32) == seq) {
      const unsigned long long lo = w & 0xffffffffull;
      return lo == 0 ? -1 : (int64_t)(lo - 1);
    }
    if ((spins & 4095) == 4095 && now() - t0 > timeoutSeconds)
      throw std::runtime_error("shard group combine: not every rank arrived");
    if (spins > (1u << 16)) sched_yield();
    else __builtin_ia32_pause();
  }
}

}  // namespace ccmi
