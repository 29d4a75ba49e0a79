// Built-in combiner of destination-sharded sessions: one int64 MIN allreduce over RCCL (xGMI) per scan.
#pragma once
#include <cstdint>

namespace ccmi {

struct RcclShard;
bool rcclUniqueId(uint8_t out[128]);
RcclShard* rcclCreate(int device, int rank, int count, const uint8_t id[128]);
void rcclDestroy(RcclShard* r);
int rcclMin(void* ctx, int64_t* key);  // ccmi_allreduce_min_fn

}  // namespace ccmi
