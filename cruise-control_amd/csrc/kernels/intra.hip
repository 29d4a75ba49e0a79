// K6: intra-broker (JBOD) goals on gfx950 (engine/intra.h holds the per-broker program) and the disk part of the
// ClusterModelStats reduction (model/ClusterModelStats.java:489-511).
//
// intra_sort    : one wavefront per broker: its replicas' fixed sort orders (reverse / forward DISK score, then
//                 Replica.compareTo) by rank counting over LDS tiles.
// intra_brokers : one wavefront per broker. A broker's rebalance touches only its own disks and replicas, so the B
//                 programs of a goal are independent; each reads its replicas' records (contiguous CSR range) and its
//                 disks, and writes its ordered action records into its own log range. The decisions are sequential
//                 (first fit, Java order), so every lane runs them redundantly; the O(entries) disk snapshots, which
//                 dominate, are filtered 64 entries per step into LDS (global scratch for brokers over kIntraLdsSnap).
// intra_compact : packs the per-broker log ranges into one array in broker-id order (the reference's action order).
// stats_disks   : per alive broker (one thread each, up to kDiskStatsBlocks workgroups) the average disk utilization
//                 percentage and its disks' deviations; unbalanced-disk count and variance sum folded per workgroup,
//                 then the workgroup partials in block order by one wave (deterministic; the stats parity bar is 1e-9
//                 relative).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../engine/device.h"
#include "../engine/intra.h"

namespace ccmi {

// One wavefront per broker. Pass 1 gathers each entry's replica fields ONCE (one replica-table line per entry) into
// the entry-indexed arrays the program reads (eDu, eOrig) and the two sort keys (eKeyRev / eKeyFwd, ~0 = not
// selected); pass 2 ranks every selected entry under both orders (ranks are a permutation: keys are unique) over key
// tiles staged from those contiguous arrays through LDS; ordRev / ordFwd[e0 + rank] = entry.
constexpr int kSortTile = 512;
__global__ __launch_bounds__(64) void intra_sort(IntraArgs A) {
  __shared__ uint64_t kRev[kSortTile], kFwd[kSortTile];
  const int b = A.brokers[blockIdx.x];
  const int e0 = A.eOff[b], n = A.eOff[b + 1] - e0;
  const int lane = threadIdx.x;
  int selCount = 0;
  for (int i = lane; i < n; i += 64) {
    const int r = A.eRep[e0 + i];
    const bool sel = A.rSel[r] != 0;
    const IntraRep x = A.rStat[r];
    A.eDu[e0 + i] = x.du;
    A.eOrig[e0 + i] = x.origDisk;
    A.eKeyRev[e0 + i] = sel ? intraSortKey(x.score, x.tie, true) : ~0ull;
    A.eKeyFwd[e0 + i] = sel ? intraSortKey(x.score, x.tie, false) : ~0ull;
    selCount += __popcll(__ballot(sel));
  }
  __syncthreads();  // this wavefront's own stores (one wavefront per workgroup) before its loads below
  for (int ic = 0; ic < n; ic += 64) {
    const int i = ic + lane;
    uint64_t rev = ~0ull, fwd = ~0ull;
    if (i < n) {
      rev = A.eKeyRev[e0 + i];
      fwd = A.eKeyFwd[e0 + i];
    }
    const bool mine = rev != ~0ull;
    int rankRev = 0, rankFwd = 0;
    for (int jt = 0; jt < n; jt += kSortTile) {
      const int m = n - jt < kSortTile ? n - jt : kSortTile;
      if (ic == 0 || n > kSortTile) {  // a broker of at most kSortTile entries stages its keys once
        __syncthreads();
        for (int j = lane; j < m; j += 64) {
          kRev[j] = A.eKeyRev[e0 + jt + j];
          kFwd[j] = A.eKeyFwd[e0 + jt + j];
        }
        __syncthreads();
      }
      if (mine)
        for (int j = 0; j < m; ++j) {  // unselected entries carry ~0: never below a selected key
          rankRev += kRev[j] < rev ? 1 : 0;
          rankFwd += kFwd[j] < fwd ? 1 : 0;
        }
    }
    if (mine) {
      A.ordRev[e0 + rankRev] = e0 + i;
      A.ordFwd[e0 + rankFwd] = e0 + i;
    }
  }
  if (lane == 0) A.nSel[b] = selCount;
}

constexpr int kIntraLdsSnap = 2048;
__global__ __launch_bounds__(64) void intra_brokers(IntraArgs A) {
  __shared__ int32_t sA[kIntraLdsSnap], sB[kIntraLdsSnap];
  const int b = A.brokers[blockIdx.x];
  const bool lds = A.nSel[b] <= kIntraLdsSnap;  // a snapshot holds at most the broker's selected entries
  IntraBroker ib(A, b, lds ? sA : nullptr, lds ? sB : nullptr);
  ib.run();
}

__global__ __launch_bounds__(256) void intra_compact(const int32_t* __restrict__ brokers, int n,
                                                     const int64_t* __restrict__ logOff,
                                                     const int32_t* __restrict__ count,
                                                     const int64_t* __restrict__ cOff, const int32_t* __restrict__ rep,
                                                     const int32_t* __restrict__ src, const int32_t* __restrict__ dst,
                                                     int32_t* __restrict__ cRep, int32_t* __restrict__ cSrc,
                                                     int32_t* __restrict__ cDst) {
  // one wavefront per broker, lanes over its records (coalesced)
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  if (wave >= n) return;
  const int b = brokers[wave];
  const int64_t s = logOff[b], d = cOff[b];
  for (int k = lane; k < count[b]; k += 64) {
    cRep[d + k] = rep[s + k];
    cSrc[d + k] = src[s + k];
    cDst[d + k] = dst[s + k];
  }
}

// stats_disks_partials: one thread per broker over a grid of up to kDiskStatsBlocks workgroups; each workgroup folds
// its brokers' unbalanced-disk counts and variance terms (wave shuffle, then the waves in order) into partial[block].
// stats_disks_combine: one wave folds the partials in block order (deterministic: the parity bar is 1e-9 relative).
__global__ __launch_bounds__(256) void stats_disks_partials(const int32_t* __restrict__ bDiskOff,
                                                            const int32_t* __restrict__ bDisks,
                                                            const double* __restrict__ dCap,
                                                            const uint8_t* __restrict__ dAlive,
                                                            const double* __restrict__ dUtil,
                                                            const uint8_t* __restrict__ bAlive, int B, double balance,
                                                            DiskStatsOut* __restrict__ partial) {
  __shared__ double sv[4];
  __shared__ int su[4], sa[4];
  double var = 0.0;
  int unb = 0, na = 0;
  for (int b = blockIdx.x * blockDim.x + threadIdx.x; b < B; b += gridDim.x * blockDim.x) {
    if (!bAlive[b]) continue;
    const int k0 = bDiskOff[b], k1 = bDiskOff[b + 1];
    double cap = 0, util = 0;
    for (int k = k0; k < k1; ++k) {
      const int d = bDisks[k];
      if (dAlive[d]) {
        cap += dCap[d];
        util += dUtil[d];
      }
    }
    const double avg = cap > 0 ? util / cap : 1.0;  // GoalUtils.averageDiskUtilizationPercentage
    const double upper = avg * balance;
    const double lm = 2 - balance;
    const double lower = avg * (lm > 0 ? lm : 0.0);
    for (int k = k0; k < k1; ++k) {
      const int d = bDisks[k];
      if (!dAlive[d]) continue;
      const double pct = dCap[d] > 0 ? dUtil[d] / dCap[d] : 1.0;
      if (pct > upper || pct < lower) unb++;
      const double x = pct - avg;
      var += x * x;
      na++;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    var += __shfl_xor(var, off, 64);
    unb += __shfl_xor(unb, off, 64);
    na += __shfl_xor(na, off, 64);
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    sv[w] = var;
    su[w] = unb;
    sa[w] = na;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double v = 0;
    int u = 0, a = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) {
      v += sv[k];
      u += su[k];
      a += sa[k];
    }
    partial[blockIdx.x] = DiskStatsOut{v, u, a};
  }
}

__global__ __launch_bounds__(64) void stats_disks_combine(const DiskStatsOut* __restrict__ partial, int n,
                                                          DiskStatsOut* __restrict__ out) {
  // lane l folds partials l, l + 64, ... in order; then the lanes in order (lane 0 reads them back through LDS)
  __shared__ DiskStatsOut s[64];
  DiskStatsOut acc{0.0, 0, 0};
  for (int i = threadIdx.x; i < n; i += 64) {
    acc.varSum += partial[i].varSum;
    acc.unbalanced += partial[i].unbalanced;
    acc.numAlive += partial[i].numAlive;
  }
  s[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    DiskStatsOut t{0.0, 0, 0};
    for (int l = 0; l < 64; ++l) {
      t.varSum += s[l].varSum;
      t.unbalanced += s[l].unbalanced;
      t.numAlive += s[l].numAlive;
    }
    *out = t;
  }
}

hipError_t launchIntraSort(const IntraArgs& A, hipStream_t st) {
  if (A.nBrokers <= 0) return hipSuccess;
  hipLaunchKernelGGL(intra_sort, dim3(A.nBrokers), dim3(64), 0, st, A);
  return hipGetLastError();
}

hipError_t launchIntra(const IntraArgs& A, hipStream_t st) {
  if (A.nBrokers <= 0) return hipSuccess;
  hipLaunchKernelGGL(intra_brokers, dim3(A.nBrokers), dim3(64), 0, st, A);
  return hipGetLastError();
}

hipError_t launchIntraCompact(const int32_t* brokers, int n, const int64_t* logOff, const int32_t* count,
                              const int64_t* cOff, const int32_t* rep, const int32_t* src, const int32_t* dst,
                              int32_t* cRep, int32_t* cSrc, int32_t* cDst, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(intra_compact, dim3((n + 3) / 4), dim3(256), 0, st, brokers, n, logOff, count, cOff, rep, src, dst,
                     cRep, cSrc, cDst);
  return hipGetLastError();
}

hipError_t launchStatsDisks(const int32_t* bDiskOff, const int32_t* bDisks, const double* dCap, const uint8_t* dAlive,
                            const double* dUtil, const uint8_t* bAlive, int B, double balance, DiskStatsOut* out,
                            hipStream_t st) {
  // out[0]: the result; out[1 .. kDiskStatsBlocks]: the workgroup partials
  int blocks = (B + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > kDiskStatsBlocks ? kDiskStatsBlocks : blocks);
  hipLaunchKernelGGL(stats_disks_partials, dim3(blocks), dim3(256), 0, st, bDiskOff, bDisks, dCap, dAlive, dUtil, bAlive,
                     B, balance, out + 1);
  hipLaunchKernelGGL(stats_disks_combine, dim3(1), dim3(64), 0, st, out + 1, blocks, out);
  return hipGetLastError();
}

}  // namespace ccmi
