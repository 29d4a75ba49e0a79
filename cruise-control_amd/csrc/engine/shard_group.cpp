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
    __atomic_store_n(&s.arrived, 0u, __ATOMIC_RELAXED);
    __atomic_store_n(&s.departed, 0u, __ATOMIC_RELEASE);
  }
}

int64_t groupHostMin(CombineSlot* s, int count, int64_t key, double timeoutSeconds) {
  const unsigned long long k = key < 0 ? kCombineNone : (unsigned long long)key;
  unsigned long long cur = __atomic_load_n(&s->minKey, __ATOMIC_RELAXED);
  while (k < cur && !__atomic_compare_exchange_n(&s->minKey, &cur, k, true, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED)) {
  }
  __atomic_fetch_add(&s->arrived, 1u, __ATOMIC_ACQ_REL);
  const double t0 = now();
  for (uint64_t spins = 0; __atomic_load_n(&s->arrived, __ATOMIC_ACQUIRE) < (unsigned)count; ++spins) {
    if ((spins & 4095) == 4095 && now() - t0 > timeoutSeconds)
      throw std::runtime_error("shard group combine: not every rank arrived");
    if (spins > (1u << 16)) sched_yield();
    else __builtin_ia32_pause();
  }
  const unsigned long long g = __atomic_load_n(&s->minKey, __ATOMIC_ACQUIRE);
  if (__atomic_fetch_add(&s->departed, 1u, __ATOMIC_ACQ_REL) == (unsigned)count - 1) {
    __atomic_store_n(&s->minKey, kCombineNone, __ATOMIC_RELAXED);
    __atomic_store_n(&s->arrived, 0u, __ATOMIC_RELAXED);
    __atomic_store_n(&s->departed, 0u, __ATOMIC_RELEASE);
  }
  return g == kCombineNone ? -1 : (int64_t)g;
}

}  // namespace ccmi
