// Host shared-memory MIN combiner (shard_shm.h).
#include "shard_shm.h"

#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstring>
#include <stdexcept>
#include <string>

namespace ccmi {

namespace {
constexpr uint64_t kMagic = 0x63636d6973686d31ull;  // "ccmishm1"

struct alignas(64) Line64 {
  std::atomic<int64_t> v;
  char pad[56];
};
struct alignas(64) Line32 {
  std::atomic<uint32_t> v;
  char pad[60];
};
struct Slot {
  Line64 minKey;
  Line32 arrived;
  Line32 departed;
};
struct Block {
  Line64 magic;    // written last by rank 0 (release): the block is initialised
  Line64 created;  // CLOCK_REALTIME ns when rank 0 initialised it (before the magic)
  Line64 nonce;    // the job's nonce (shmCreate), written before the magic
  Line32 count;
  Line32 attached;
  Slot slot[2];
};
static_assert(std::atomic<int64_t>::is_always_lock_free && std::atomic<uint32_t>::is_always_lock_free,
              "lock-free atomics in shared memory");

double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int64_t wallNs() {
  return (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::system_clock::now().time_since_epoch()).count();
}
inline void relax(uint64_t spins) {
  if (spins > (1u << 16)) sched_yield();  // past ~1 ms another rank is far behind: give the core away between polls
  else __builtin_ia32_pause();
}
}  // namespace

struct ShmShard {
  Block* blk = nullptr;
  int rank = 0, count = 1;
  uint64_t calls = 0;
  double timeout = 120.0;
  bool broken = false;  // a combine timed out: its slot counters are inconsistent, every later call fails fast
};

ShmShard* shmCreate(const char* name, int rank, int count, double timeoutSeconds, uint64_t nonce) {
  if (!name || name[0] != '/' || std::strchr(name + 1, '/')) throw std::invalid_argument("shm name must be \"/name\"");
  if (count < 1 || rank < 0 || rank >= count) throw std::invalid_argument("shard rank out of range");
  int fd = -1;
  const double t0 = now();
  const int64_t joinNs = wallNs();
  auto* s = new ShmShard();
  s->rank = rank;
  s->count = count;
  s->timeout = timeoutSeconds;
  if (rank == 0) {
    shm_unlink(name);  // a block left by an earlier run of the same job name
    fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0 || ftruncate(fd, sizeof(Block)) != 0) {
      const std::string err = std::strerror(errno);
      if (fd >= 0) close(fd);
      delete s;
      throw std::runtime_error("shm_open(create) / ftruncate failed: " + err);
    }
    void* p = mmap(nullptr, sizeof(Block), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) {
      delete s;
      throw std::runtime_error(std::string("mmap failed: ") + std::strerror(errno));
    }
    s->blk = static_cast<Block*>(p);
    Block& b = *s->blk;
    for (Slot& x : b.slot) {
      x.minKey.v.store(INT64_MAX, std::memory_order_relaxed);
      x.arrived.v.store(0, std::memory_order_relaxed);
      x.departed.v.store(0, std::memory_order_relaxed);
    }
    b.count.v.store((uint32_t)count, std::memory_order_relaxed);
    b.attached.v.store(0, std::memory_order_relaxed);
    b.created.v.store(wallNs(), std::memory_order_relaxed);
    b.nonce.v.store((int64_t)nonce, std::memory_order_relaxed);
    b.magic.v.store((int64_t)kMagic, std::memory_order_release);
  } else {
    // A block a crashed run left under the same name can be opened before rank 0 replaces it. With a job nonce it is
    // told apart by the nonce, whatever its age. Without one (nonce 0) its creation stamp gives it away: rank 0 of a
    // block waits at most `timeoutSeconds` for its ranks, so a block created longer than that before this rank arrived
    // has no rank 0 left. Either way it is dropped and the name polled again.
    for (;;) {
      if (now() - t0 > timeoutSeconds) {
        shmDestroy(s);
        throw std::runtime_error("shm combiner: rank 0's block never appeared (or was never initialised)");
      }
      fd = shm_open(name, O_RDWR, 0600);
      if (fd >= 0) {
        struct stat st;
        if (fstat(fd, &st) == 0 && (size_t)st.st_size >= sizeof(Block)) {
          void* p = mmap(nullptr, sizeof(Block), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
          close(fd);
          fd = -1;
          if (p == MAP_FAILED) {
            shmDestroy(s);
            throw std::runtime_error(std::string("mmap failed: ") + std::strerror(errno));
          }
          Block* b = static_cast<Block*>(p);
          if (b->magic.v.load(std::memory_order_acquire) == (int64_t)kMagic) {
            const int64_t created = b->created.v.load(std::memory_order_relaxed);
            const bool current = nonce != 0 ? (uint64_t)b->nonce.v.load(std::memory_order_relaxed) == nonce
                                            : created + (int64_t)(timeoutSeconds * 1e9) >= joinNs;
            if (current) {
              s->blk = b;
              break;
            }
          }
          munmap(p, sizeof(Block));  // not initialised yet, or stale: look again
        } else {
          close(fd);
          fd = -1;
        }
      }
      usleep(1000);
    }
    if (s->blk->count.v.load(std::memory_order_relaxed) != (uint32_t)count) {
      shmDestroy(s);
      throw std::invalid_argument("shm combiner: ranks disagree on the shard count");
    }
  }
  Block& b = *s->blk;
  b.attached.v.fetch_add(1, std::memory_order_acq_rel);
  for (uint64_t spins = 0; b.attached.v.load(std::memory_order_acquire) < (uint32_t)count; ++spins) {
    if (now() - t0 > timeoutSeconds) {
      shmDestroy(s);
      throw std::runtime_error("shm combiner: not every rank attached");
    }
    relax(spins);
  }
  if (rank == 0) shm_unlink(name);  // every rank has it mapped: the name is no longer needed
  return s;
}

void shmDestroy(ShmShard* s) {
  if (!s) return;
  if (s->blk) munmap(s->blk, sizeof(Block));
  delete s;
}

int shmMin(void* ctx, int64_t* key) {
  auto* s = static_cast<ShmShard*>(ctx);
  if (s->broken) return 1;
  Slot& x = s->blk->slot[s->calls & 1];
  ++s->calls;
  int64_t cur = x.minKey.v.load(std::memory_order_relaxed);
  while (*key < cur && !x.minKey.v.compare_exchange_weak(cur, *key, std::memory_order_acq_rel)) {
  }
  x.arrived.v.fetch_add(1, std::memory_order_acq_rel);
  const double t0 = now();
  for (uint64_t spins = 0; x.arrived.v.load(std::memory_order_acquire) < (uint32_t)s->count; ++spins) {
    if ((spins & 4095) == 4095 && now() - t0 > s->timeout) {
      s->broken = true;  // this slot's arrival count now disagrees with the other ranks': never combine again
      return 1;
    }
    relax(spins);
  }
  *key = x.minKey.v.load(std::memory_order_acquire);
  // the last rank out resets the slot; no rank reaches it again before every rank arrived at the next call (the
  // other slot), which this rank does only after the reset
  if (x.departed.v.fetch_add(1, std::memory_order_acq_rel) == (uint32_t)s->count - 1) {
    x.minKey.v.store(INT64_MAX, std::memory_order_relaxed);
    x.arrived.v.store(0, std::memory_order_relaxed);
    x.departed.v.store(0, std::memory_order_release);
  }
  return 0;
}

}  // namespace ccmi
