// Host shared-memory combiner for destination-sharded sessions on one node (ccmi_session_attach_shm).
//
// Every rank of a sharded proposal runs the same host drivers, so the ranks make the same sequence of combine calls.
// Each call MIN-combines one int64 key per rank in a POSIX shared-memory block: an atomic fetch-min into the call's
// slot, an arrival count every rank spins on, and a departure count whose last rank resets the slot (two slots used
// alternately, so a rank never reaches a slot before its previous use was reset). No GPU work: the scan server stays
// resident on every rank, and the key never leaves host memory (the server already publishes it there).
#pragma once
#include <stdint.h>

namespace ccmi {

struct ShmShard;

// rank 0 creates the block `name` (a POSIX shared-memory name, e.g. "/ccmi_<job>"), the others open it; every rank
// waits until all `count` ranks are attached (then rank 0 unlinks the name). Throws std::runtime_error on failure or
// after `timeoutSeconds` without every rank. `nonce` (the same nonzero value on every rank of the job, e.g. rank 0's
// start time broadcast over the process group) is stamped into the block by rank 0, and the other ranks attach only
// to a block carrying it, so a block a crashed run left under the same name is refused however recent; with nonce 0 a
// block is taken as stale only when it was created more than `timeoutSeconds` before the rank arrived.
ShmShard* shmCreate(const char* name, int rank, int count, double timeoutSeconds = 120.0, uint64_t nonce = 0);
void shmDestroy(ShmShard* s);
// ccmi_allreduce_min_fn: *key = MIN over ranks (INT64_MAX = none); 0 on success, nonzero after a timeout
int shmMin(void* ctx, int64_t* key);

}  // namespace ccmi
