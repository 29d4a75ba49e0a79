// K3: fused ClusterModelStats reduction (model/ClusterModelStats.java:84-511) on gfx950.
//
// stats_topics : one workgroup per topic row of the dense topicCount[T][B] matrix — the O(T x B)
//                numForAvgTopicReplicas loop (ClusterModelStats.java:446-476), the dominant HBM stream.
//                Rows are read 16 B per lane (int4), max/min/variance reduced through LDS, one record
//                per topic written out.
// stats_partials / stats_combine : per-resource utilization stats (:267-322), potential NW_OUT (:332-362),
//                replica / leader count stats (:371-436) over the broker columns, plus the reduction of the
//                per-topic records: a grid of up to kStatsPartBlocks workgroups, then one wave folding their
//                partials in block order. Sums are tree-ordered (parity bar for stats: 1e-9 relative).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../engine/devtypes.h"

namespace ccmi {

constexpr int kTB = 256;

template <typename T, typename Op>
__device__ __forceinline__ T blockReduce(T v, Op op, T* scratch) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = op(v, __shfl_xor(v, off, 64));
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) scratch[wave] = v;
  __syncthreads();
  T r = scratch[0];
  const int nw = blockDim.x >> 6;
  for (int w = 1; w < nw; ++w) r = op(r, scratch[w]);
  return r;
}

struct OpAdd {
  template <typename T>
  __device__ T operator()(T a, T b) const { return a + b; }
};
struct OpMax {
  template <typename T>
  __device__ T operator()(T a, T b) const { return a > b ? a : b; }
};
struct OpMin {
  template <typename T>
  __device__ T operator()(T a, T b) const { return a < b ? a : b; }
};

// allowedAlive[b]: broker alive and allowed for replica moves (ClusterModelStats._brokersAllowedReplicaMove)
__global__ __launch_bounds__(kTB) void stats_topics(const int32_t* __restrict__ tc, const int32_t* __restrict__ topicNrep,
                                                    const uint8_t* __restrict__ allowedAlive, int B, int ldB,
                                                    int T, int numAllowed, TopicPartial* __restrict__ out) {
  __shared__ double sd[kTB / 64];
  __shared__ int si[kTB / 64];
  for (int t = blockIdx.x; t < T; t += gridDim.x) {
    const int32_t* row = tc + (size_t)t * ldB;
    const double avg = ((double)topicNrep[t]) / numAllowed;
    double var = 0.0;
    int mx = 0, mn = 0x7fffffff;
    // rows are padded to ldB (multiple of 4) so every lane loads 16 B; padding columns are skipped
    const int n4 = ldB >> 2;
    const int4* row4 = reinterpret_cast<const int4*>(row);
    const uint32_t* al4 = reinterpret_cast<const uint32_t*>(allowedAlive);
    for (int i = threadIdx.x; i < n4; i += kTB) {
      const int4 c = row4[i];
      const uint32_t a = al4[i];
      const int cs[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (4 * i + k >= B) break;
        const int n = cs[k];
        mx = n > mx ? n : mx;
        mn = n < mn ? n : mn;
        if ((a >> (8 * k)) & 0xff) {
          const double d = n - avg;
          var += (d * d) / numAllowed;
        }
      }
    }
    var = blockReduce(var, OpAdd(), sd);
    mx = blockReduce(mx, OpMax(), si);
    mn = blockReduce(mn, OpMin(), si);
    if (threadIdx.x == 0) out[t] = {avg, sqrt(var), mx, mn};
    __syncthreads();
  }
}

// stats_partials + stats_combine: the broker-column and topic-record reductions as a grid of kPartBlocks
// workgroups, each writing one StatsPartial, then one wave folding the partials in block order (deterministic).
// The two averages a variance needs (potential NW_OUT sum, replica / leader totals) come from the host in
// StatsParams, so every quantity is a single pass.
struct StatsPartial {
  double d[kStatD];
  int32_t i[kStatI];
};

__device__ __forceinline__ double dOp(int k, double a, double b) {
  return k < 4 || k == kSdPHot ? (a > b ? a : b) : (k < 8 || k == kSdPCold) ? (a < b ? a : b) : a + b;
}
__device__ __forceinline__ int32_t iOp(int k, int32_t a, int32_t b) {
  return (k == kSiRepMx || k == kSiLeadMx || k == kSiTMx) ? (a > b ? a : b)
         : (k == kSiRepMn || k == kSiLeadMn || k == kSiTMn) ? (a < b ? a : b)
                                                              : a + b;
}
__device__ __forceinline__ double dInit(int k) {
  return (k >= 4 && k < 8) || k == kSdPCold ? 1.7976931348623157e308 : 0.0;
}
__device__ __forceinline__ int32_t iInit(int k) {
  return (k == kSiRepMn || k == kSiLeadMn || k == kSiTMn) ? 0x7fffffff : 0;
}

template <int N>
__device__ __forceinline__ void waveFoldD(double (&v)[N]) {
#pragma unroll
  for (int k = 0; k < N; ++k)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v[k] = dOp(k, v[k], __shfl_xor(v[k], off, 64));
}
template <int N>
__device__ __forceinline__ void waveFoldI(int32_t (&v)[N]) {
#pragma unroll
  for (int k = 0; k < N; ++k)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v[k] = iOp(k, v[k], __shfl_xor(v[k], off, 64));
}

__global__ __launch_bounds__(kTB) void stats_partials(StatsParams P, const BrokerRec* __restrict__ br,
                                                      const uint8_t* __restrict__ allowedAlive,
                                                      const TopicPartial* __restrict__ topics,
                                                      StatsPartial* __restrict__ part) {
  double d[kStatD];
  int32_t iv[kStatI];
#pragma unroll
  for (int k = 0; k < kStatD; ++k) d[k] = dInit(k);
#pragma unroll
  for (int k = 0; k < kStatI; ++k) iv[k] = iInit(k);
  const int na = P.numAllowed;
  const double repAvg = (double)P.repTotal / na, leadAvg = (double)P.leadTotal / na;
  const double potPct = P.potSum / P.potCapacity;
  const int stride = gridDim.x * kTB;
  for (int b = blockIdx.x * kTB + threadIdx.x; b < P.B; b += stride) {
    const BrokerRec x = br[b];
    const bool allowed = allowedAlive[b] != 0;
    // replica / leader counts: max/min over every broker, variance over alive allowed ones
    iv[kSiRepMx] = max(iv[kSiRepMx], x.nrep);
    iv[kSiRepMn] = min(iv[kSiRepMn], x.nrep);
    iv[kSiLeadMx] = max(iv[kSiLeadMx], x.nlead);
    iv[kSiLeadMn] = min(iv[kSiLeadMn], x.nlead);
    if (!x.alive) continue;
    // host resources are the host's when brokers share hosts (ClusterModelStats.java:297-303)
    const bool hostVals = P.hostCap != nullptr;
#pragma unroll
    for (int res = 0; res < 4; ++res) {
      const double u = hostVals && res < 3 ? x.hutil[res] : x.util[res];
      d[res] = u > d[res] ? u : d[res];
      d[4 + res] = u < d[4 + res] ? u : d[4 + res];
      if (allowed) {
        const double cap = hostVals && res < 3 ? P.hostCap[3 * (size_t)b + res] : x.cap[res];
        const double pct = u / cap;
        if (pct >= P.lowerThr[res] && pct <= P.upperThr[res]) iv[res]++;
        const double dv = u - P.avgPct[res] * cap;
        d[8 + res] += dv * dv;
      }
    }
    const double u = x.pot;
    d[kSdPHot] = u > d[kSdPHot] ? u : d[kSdPHot];
    d[kSdPCold] = u < d[kSdPCold] ? u : d[kSdPCold];
    if (allowed) {
      const double cap = x.cap[2];
      if (u / cap <= P.nwOutCapThreshold) iv[kSiUnder]++;
      const double dv = u - potPct * cap;
      d[kSdPVar] += dv * dv;
      const double dr = (double)x.nrep - repAvg, dl = (double)x.nlead - leadAvg;
      d[kSdRepVar] += (dr * dr) / na;
      d[kSdLeadVar] += (dl * dl) / na;
    }
  }
  for (int t = blockIdx.x * kTB + threadIdx.x; t < P.T; t += stride) {
    const TopicPartial x = topics[t];
    d[kSdTAvg] += x.avg;
    d[kSdTSd] += x.sd;
    iv[kSiTMx] = max(iv[kSiTMx], x.mx);
    iv[kSiTMn] = min(iv[kSiTMn], x.mn);
  }
  waveFoldD(d);
  waveFoldI(iv);
  __shared__ double sd[kTB / 64][kStatD];
  __shared__ int32_t si[kTB / 64][kStatI];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < kStatD; ++k) sd[wave][k] = d[k];
#pragma unroll
    for (int k = 0; k < kStatI; ++k) si[wave][k] = iv[k];
  }
  __syncthreads();
  if (threadIdx.x < kStatD) {
    const int k = threadIdx.x;
    double r = sd[0][k];
    for (int w = 1; w < kTB / 64; ++w) r = dOp(k, r, sd[w][k]);
    part[blockIdx.x].d[k] = r;
  } else if (threadIdx.x >= 64 && threadIdx.x < 64 + kStatI) {
    const int k = threadIdx.x - 64;
    int32_t r = si[0][k];
    for (int w = 1; w < kTB / 64; ++w) r = iOp(k, r, si[w][k]);
    part[blockIdx.x].i[k] = r;
  }
}

// one wave; lane g folds partial g (G <= 64)
__global__ __launch_bounds__(64) void stats_combine(StatsParams P, const StatsPartial* __restrict__ part, int G,
                                                    StatsOut* __restrict__ out) {
  double d[kStatD];
  int32_t iv[kStatI];
  const int g = threadIdx.x;
#pragma unroll
  for (int k = 0; k < kStatD; ++k) d[k] = g < G ? part[g].d[k] : dInit(k);
#pragma unroll
  for (int k = 0; k < kStatI; ++k) iv[k] = g < G ? part[g].i[k] : iInit(k);
  waveFoldD(d);
  waveFoldI(iv);
  if (threadIdx.x != 0) return;
  const int na = P.numAllowed;
  for (int res = 0; res < 4; ++res) {
    out->numBalanced[res] = iv[res];
    out->resAvg[res] = P.clusterUtil[res] / na;
    out->resMax[res] = d[res];
    out->resMin[res] = d[4 + res];
    out->resStd[res] = sqrt(d[8 + res] / na);
  }
  out->pnwAvg = P.potSum / na;
  out->pnwMax = d[kSdPHot];
  out->pnwMin = d[kSdPCold];
  out->pnwStd = sqrt(d[kSdPVar] / na);
  out->numUnderPot = iv[kSiUnder];
  out->repAvg = (double)P.repTotal / na;
  out->repStd = sqrt(d[kSdRepVar]);
  out->repMax = iv[kSiRepMx];
  out->repMin = iv[kSiRepMn];
  out->leadAvg = (double)P.leadTotal / na;
  out->leadStd = sqrt(d[kSdLeadVar]);
  out->leadMax = iv[kSiLeadMx];
  out->leadMin = iv[kSiLeadMn];
  out->topicAvg = d[kSdTAvg] / P.T;
  out->topicStd = d[kSdTSd] / P.T;
  out->topicMax = iv[kSiTMx];
  out->topicMin = iv[kSiTMn];
}

hipError_t launchStats(const StatsParams& P, const int32_t* tc, const int32_t* topicNrep, const BrokerRec* brokers,
                       const uint8_t* allowedAlive, TopicPartial* scratch, void* partials, StatsOut* out, int ldB,
                       hipStream_t st,
                       hipEvent_t evTopic0, hipEvent_t evTopic1) {
  int blocks = P.T < 8192 ? P.T : 8192;
  if (blocks < 1) blocks = 1;
  if (evTopic0) (void)hipEventRecord(evTopic0, st);
  hipLaunchKernelGGL(stats_topics, dim3(blocks), dim3(kTB), 0, st, tc, topicNrep, allowedAlive, P.B, ldB, P.T,
                     P.numAllowed, scratch);
  if (evTopic1) (void)hipEventRecord(evTopic1, st);
  const int work = (P.B > P.T ? P.B : P.T);
  int G = (work + kTB - 1) / kTB;
  G = G < 1 ? 1 : (G > kStatsPartBlocks ? kStatsPartBlocks : G);
  StatsPartial* part = reinterpret_cast<StatsPartial*>(partials);
  hipLaunchKernelGGL(stats_partials, dim3(G), dim3(kTB), 0, st, P, brokers, allowedAlive, scratch, part);
  hipLaunchKernelGGL(stats_combine, dim3(1), dim3(64), 0, st, P, part, G, out);
  return hipGetLastError();
}

}  // namespace ccmi
