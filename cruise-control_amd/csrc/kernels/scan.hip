// gfx950 kernels for the goal optimizer's candidate scans.
//
// K1+K2  scan_cross : first-fit over (replica k, destination broker j) pairs in k-major order — the
//                     candidate loop of AbstractGoal.maybeApplyBalancingAction (AbstractGoal.java:243-270)
//                     unrolled over the caller's replica loop. The answer is the SMALLEST pair index whose
//                     predicate conjunction holds, i.e. the deterministic argmin that breaks ties by the
//                     reference's iteration order; found with a wavefront ballot, an LDS block reduction and
//                     one 64-bit atomicMin per block (order-independent, so results are bitwise stable).
// K5     scan_swap  : one wavefront per (candidate broker m, source replica s) row walks that broker's
//                     candidate replicas (AbstractGoal.maybeApplySwapAction, AbstractGoal.java:287-338);
//                     the row's FIRST terminal outcome decides it, and the smallest row whose terminal is
//                     an ACCEPT wins.
// K4     apply_rows : scatters the host's dirty broker/replica/partition rows and topic-count deltas into
//                     the device tables before a scan or a stats pass.
// Built with -ffp-contract=off: every predicate is the reference's IEEE double expression.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../engine/devtypes.h"
#include "../engine/predicates.h"

namespace ccmi {

struct DevView {
  DevTables t;
  __device__ __forceinline__ double bu(int b, int res) const { return t.bUtil[(size_t)res * t.B + b]; }
  __device__ __forceinline__ double bcap(int b, int res) const { return t.bCap[(size_t)res * t.B + b]; }
  __device__ __forceinline__ int nrep(int b) const { return t.bNrep[b]; }
  __device__ __forceinline__ bool alive(int b) const { return t.bAlive[b] != 0; }
  __device__ __forceinline__ bool allowed(int slot, int b) const { return t.allowed[(size_t)slot * t.B + b] != 0; }
  __device__ __forceinline__ double ru(int r, int res) const { return t.rUtil[(size_t)res * t.R + r]; }
  __device__ __forceinline__ int flags(int r) const { return t.rFlags[r]; }
  __device__ __forceinline__ int rbroker(int r) const { return t.rBroker[r]; }
  __device__ __forceinline__ int rorig(int r) const { return t.rOrig[r]; }
  __device__ __forceinline__ int rpart(int r) const { return t.rPart[r]; }
  __device__ __forceinline__ int pbegin(int p) const { return t.pOff[p]; }
  __device__ __forceinline__ int pend(int p) const { return t.pOff[p + 1]; }
  __device__ __forceinline__ int pbroker(int i) const { return t.pBrokers[i]; }
};

constexpr int kBlock = 256;
constexpr int kItems = 4;
constexpr unsigned long long kNone = ~0ull;

__device__ __forceinline__ unsigned long long waveMin(unsigned long long v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    unsigned long long o = __shfl_xor(v, off, 64);
    v = o < v ? o : v;
  }
  return v;
}

__device__ __forceinline__ unsigned long long blockMin(unsigned long long v) {
  __shared__ unsigned long long part[kBlock / 64];
  v = waveMin(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) part[wave] = v;
  __syncthreads();
  unsigned long long r = part[0];
#pragma unroll
  for (int w = 1; w < kBlock / 64; ++w) r = part[w] < r ? part[w] : r;
  __syncthreads();
  return r;
}

// Current best key, read once per block so the early exit is uniform across the block's waves.
__device__ __forceinline__ unsigned long long blockBest(const unsigned long long* result) {
  __shared__ unsigned long long sBest;
  if (threadIdx.x == 0) sBest = __hip_atomic_load(result, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const unsigned long long b = sBest;
  __syncthreads();
  return b;
}

__global__ __launch_bounds__(kBlock) void scan_cross(DevTables T, DevProgram prog, const int32_t* __restrict__ reps,
                                                     const int32_t* __restrict__ cands, int K, int N,
                                                     unsigned long long* __restrict__ result) {
  const DevView v{T};
  const uint32_t total = (uint32_t)K * (uint32_t)N;
  const uint32_t chunk = kBlock * kItems;
  for (uint32_t base = blockIdx.x * chunk; base < total; base += gridDim.x * chunk) {
    if (blockBest(result) <= base) return;  // an earlier pair already won: nothing later can (block-uniform)
    unsigned long long local = kNone;
#pragma unroll
    for (int it = 0; it < kItems; ++it) {
      const uint32_t q = base + it * kBlock + threadIdx.x;
      if (q < total && local == kNone) {
        const uint32_t k = q / (uint32_t)N;
        const uint32_t j = q - k * (uint32_t)N;
        if (moveCandidateAccepted(prog, v, reps[k], cands[j])) local = q;
      }
    }
    const unsigned long long m = blockMin(local);
    if (m != kNone) {
      if (threadIdx.x == 0) atomicMin(result, m);
      return;
    }
  }
}

// One wavefront per row (m, s). rowsPerBlock = kBlock / 64.
__global__ __launch_bounds__(kBlock) void scan_swap(DevTables T, DevProgram prog, const int32_t* __restrict__ srcs, int S,
                                                    const int32_t* __restrict__ cbOff, const int32_t* __restrict__ cbRep,
                                                    int M, unsigned long long* __restrict__ result,
                                                    int32_t* __restrict__ rowVisited) {
  const DevView v{T};
  const int lane = threadIdx.x & 63;
  const int waveInBlock = threadIdx.x >> 6;
  const long long rows = (long long)M * S;
  for (long long row = (long long)blockIdx.x * (kBlock / 64) + waveInBlock; row < rows;
       row += (long long)gridDim.x * (kBlock / 64)) {
    const unsigned long long best = __hip_atomic_load(result, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((best >> 24) < (unsigned long long)row) return;
    const int m = (int)(row / S);
    const int s = (int)(row - (long long)m * S);
    const int sr = srcs[s];
    const int c0 = cbOff[m], c1 = cbOff[m + 1];
    if (c0 == c1) {
      if (lane == 0) rowVisited[row] = 0;
      continue;
    }
    const int db = v.rbroker(cbRep[c0]);
    int visited = c1 - c0;
    for (int base = c0; base < c1; base += 64) {
      const int idx = base + lane;
      int outcome = 0;
      if (idx < c1) outcome = swapCandidateOutcome(prog, v, sr, cbRep[idx], db);
      const unsigned long long term = __ballot(outcome != 0);
      if (term) {
        const int first = __ffsll((long long)term) - 1;
        const int firstOutcome = __shfl(outcome, first, 64);
        if (firstOutcome == 1 && lane == 0)
          atomicMin(result, ((unsigned long long)row << 24) | (unsigned long long)(base + first - c0));
        visited = base + first - c0 + 1;
        break;
      }
    }
    if (lane == 0) rowVisited[row] = visited;
  }
}

// Reference-equivalent candidate count of a swap scan: every row before the winning row ran to its first
// terminal (or its end), plus the winning row up to its accepted candidate.
__global__ __launch_bounds__(1024) void swap_visited_sum(const int32_t* __restrict__ rowVisited, long long rows,
                                                         unsigned long long* __restrict__ result) {
  __shared__ long long part[16];
  const unsigned long long best = result[0];
  const long long lim = best == kNone ? rows : (long long)(best >> 24) + 1;
  long long s = 0;
  for (long long i = threadIdx.x; i < lim; i += blockDim.x) s += rowVisited[i];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    long long t = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += part[w];
    result[1] = (unsigned long long)t;
  }
}

// PAIRS: explicit (replica, broker) list in iteration order (leadership moves: per-replica follower lists).
__global__ __launch_bounds__(kBlock) void scan_pairs(DevTables T, DevProgram prog, const int32_t* __restrict__ pr,
                                                     const int32_t* __restrict__ pb, int n,
                                                     unsigned long long* __restrict__ result) {
  const DevView v{T};
  const int chunk = kBlock * kItems;
  for (int base = blockIdx.x * chunk; base < n; base += gridDim.x * chunk) {
    if (blockBest(result) <= (unsigned long long)base) return;
    unsigned long long local = kNone;
#pragma unroll
    for (int it = 0; it < kItems; ++it) {
      const int q = base + it * kBlock + threadIdx.x;
      if (q < n && local == kNone && moveCandidateAccepted(prog, v, pr[q], pb[q])) local = (unsigned long long)q;
    }
    const unsigned long long m = blockMin(local);
    if (m != kNone) {
      if (threadIdx.x == 0) atomicMin(result, m);
      return;
    }
  }
}

__global__ void apply_rows(double* bUtil, int32_t* bNrep, int32_t* bNlead, double* bPot, uint8_t* bAlive, int B,
                           const BrokerRow* __restrict__ brows, int nb, double* rUtil, int32_t* rBroker, uint8_t* rFlags,
                           int R, const ReplicaRow* __restrict__ rrows, int nr, const int32_t* __restrict__ pOff,
                           int32_t* pBrokers, const PartitionRow* __restrict__ prows, int np, int32_t* topicCount,
                           int ldB, const TopicCountDelta* __restrict__ tdel, int nt) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nb) {
    const BrokerRow& x = brows[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) bUtil[(size_t)k * B + x.b] = x.util[k];
    bNrep[x.b] = x.nrep;
    bNlead[x.b] = x.nlead;
    bPot[x.b] = x.potNwOut;
    bAlive[x.b] = (uint8_t)x.alive;
  }
  if (i < nr) {
    const ReplicaRow& x = rrows[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) rUtil[(size_t)k * R + x.r] = x.util[k];
    rBroker[x.r] = x.broker;
    rFlags[x.r] = (uint8_t)x.flags;
  }
  if (i < np) {
    const PartitionRow& x = prows[i];
    const int o = pOff[x.p];
    for (int k = 0; k < x.n; ++k) pBrokers[o + k] = x.brokers[k];
  }
  if (i < nt) {
    const TopicCountDelta& d = tdel[i];
    atomicAdd(&topicCount[(size_t)d.topic * ldB + d.broker], d.delta);
  }
}

// ------------------------------------------------------------------------------------------------ launchers
hipError_t launchScanCross(const DevTables& T, const DevProgram& prog, const int32_t* reps, const int32_t* cands, int K,
                           int N, unsigned long long* result, hipStream_t st) {
  const uint64_t total = (uint64_t)K * (uint64_t)N;
  const uint64_t chunk = kBlock * kItems;
  uint64_t blocks = (total + chunk - 1) / chunk;
  if (blocks > 4096) blocks = 4096;
  if (blocks == 0) blocks = 1;
  hipLaunchKernelGGL(scan_cross, dim3((unsigned)blocks), dim3(kBlock), 0, st, T, prog, reps, cands, K, N, result);
  return hipGetLastError();
}

hipError_t launchScanSwap(const DevTables& T, const DevProgram& prog, const int32_t* srcs, int S, const int32_t* cbOff,
                          const int32_t* cbRep, int M, unsigned long long* result, int32_t* rowVisited, hipStream_t st,
                          hipEvent_t ev0, hipEvent_t ev1) {
  const uint64_t rows = (uint64_t)M * (uint64_t)S;
  uint64_t blocks = (rows + (kBlock / 64) - 1) / (kBlock / 64);
  if (blocks > 4096) blocks = 4096;
  if (blocks == 0) blocks = 1;
  if (ev0) (void)hipEventRecord(ev0, st);
  hipLaunchKernelGGL(scan_swap, dim3((unsigned)blocks), dim3(kBlock), 0, st, T, prog, srcs, S, cbOff, cbRep, M, result,
                     rowVisited);
  if (ev1) (void)hipEventRecord(ev1, st);
  hipLaunchKernelGGL(swap_visited_sum, dim3(1), dim3(1024), 0, st, rowVisited, (long long)rows, result);
  return hipGetLastError();
}

hipError_t launchScanPairs(const DevTables& T, const DevProgram& prog, const int32_t* pr, const int32_t* pb, int n,
                           unsigned long long* result, hipStream_t st) {
  const int chunk = kBlock * kItems;
  int blocks = (n + chunk - 1) / chunk;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(scan_pairs, dim3(blocks), dim3(kBlock), 0, st, T, prog, pr, pb, n, result);
  return hipGetLastError();
}

hipError_t launchApplyRows(double* bUtil, int32_t* bNrep, int32_t* bNlead, double* bPot, uint8_t* bAlive, int B,
                           const BrokerRow* brows, int nb, double* rUtil, int32_t* rBroker, uint8_t* rFlags, int R,
                           const ReplicaRow* rrows, int nr, const int32_t* pOff, int32_t* pBrokers,
                           const PartitionRow* prows, int np, int32_t* topicCount, int ldB, const TopicCountDelta* tdel,
                           int nt, hipStream_t st) {
  int n = nb;
  if (nr > n) n = nr;
  if (np > n) n = np;
  if (nt > n) n = nt;
  if (n == 0) return hipSuccess;
  const int threads = 256;
  const int blocks = (n + threads - 1) / threads;
  hipLaunchKernelGGL(apply_rows, dim3(blocks), dim3(threads), 0, st, bUtil, bNrep, bNlead, bPot, bAlive, B, brows, nb,
                     rUtil, rBroker, rFlags, R, rrows, nr, pOff, pBrokers, prows, np, topicCount, ldB, tdel, nt);
  return hipGetLastError();
}

}  // namespace ccmi
