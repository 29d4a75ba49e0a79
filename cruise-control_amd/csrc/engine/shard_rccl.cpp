// RCCL combiner for destination-sharded sessions (shard_rccl.h). The key travels host -> HBM -> allreduce(MIN)
// -> host on a dedicated stream; the scan that produced it has already completed (its mailbox was read).
#include "shard_rccl.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <stdexcept>
#include <string>

namespace ccmi {

struct RcclShard {
  ncclComm_t comm = nullptr;
  hipStream_t st = nullptr;
  int64_t* dKey = nullptr;
  int64_t* hKey = nullptr;
};

static void ck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error in ") + what + ": " + hipGetErrorString(e));
}
static void ckn(ncclResult_t e, const char* what) {
  if (e != ncclSuccess) throw std::runtime_error(std::string("RCCL device error in ") + what + ": " + ncclGetErrorString(e));
}

bool rcclUniqueId(uint8_t out[128]) {
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return false;
  std::memcpy(out, &id, 128);
  return true;
}

RcclShard* rcclCreate(int device, int rank, int count, const uint8_t idBytes[128]) {
  ck(hipSetDevice(device), "hipSetDevice");
  auto* r = new RcclShard();
  ncclUniqueId id;
  std::memcpy(&id, idBytes, 128);
  ckn(ncclCommInitRank(&r->comm, count, id, rank), "ncclCommInitRank");
  ck(hipStreamCreateWithFlags(&r->st, hipStreamNonBlocking), "hipStreamCreate");
  ck(hipMalloc((void**)&r->dKey, sizeof(int64_t)), "hipMalloc");
  ck(hipHostMalloc((void**)&r->hKey, sizeof(int64_t), hipHostMallocDefault), "hipHostMalloc");
  return r;
}

void rcclDestroy(RcclShard* r) {
  if (!r) return;
  if (r->st) (void)hipStreamSynchronize(r->st);
  if (r->comm) (void)ncclCommDestroy(r->comm);
  if (r->dKey) (void)hipFree(r->dKey);
  if (r->hKey) (void)hipHostFree(r->hKey);
  if (r->st) (void)hipStreamDestroy(r->st);
  delete r;
}

int rcclMin(void* ctx, int64_t* key) {
  auto* r = static_cast<RcclShard*>(ctx);
  *r->hKey = *key;
  if (hipMemcpyAsync(r->dKey, r->hKey, sizeof(int64_t), hipMemcpyHostToDevice, r->st) != hipSuccess) return 1;
  if (ncclAllReduce(r->dKey, r->dKey, 1, ncclInt64, ncclMin, r->comm, r->st) != ncclSuccess) return 2;
  if (hipMemcpyAsync(r->hKey, r->dKey, sizeof(int64_t), hipMemcpyDeviceToHost, r->st) != hipSuccess) return 3;
  if (hipStreamSynchronize(r->st) != hipSuccess) return 4;
  *key = *r->hKey;
  return 0;
}

}  // namespace ccmi
