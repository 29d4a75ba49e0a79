// K3: fused ClusterModelStats reduction (model/ClusterModelStats.java:84-511) on gfx950.
//
// stats_topics : one workgroup per topic row of the dense topicCount[T][B] matrix — the O(T x B)
//                numForAvgTopicReplicas loop (ClusterModelStats.java:446-476), the dominant HBM stream.
//                Rows are read 16 B per lane (int4), max/min/variance reduced through LDS, one record
//                per topic written out.
// stats_final  : one workgroup: per-resource utilization stats (:267-322), potential NW_OUT (:332-362),
//                replica / leader count stats (:371-436) over the broker columns, plus the reduction of
//                the per-topic records. Sums are tree-ordered (parity bar for stats: 1e-9 relative).
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

__global__ __launch_bounds__(1024) void stats_final(StatsParams P, const BrokerRec* __restrict__ br,
                                                    const uint8_t* __restrict__ allowedAlive,
                                                    const TopicPartial* __restrict__ topics, StatsOut* __restrict__ out) {
  __shared__ double sd[16];
  __shared__ int si[16];
  const int B = P.B;
  const int na = P.numAllowed;
  for (int res = 0; res < 4; ++res) {
    double hot = 0.0, cold = 1.7976931348623157e308, varSum = 0.0;
    int bal = 0;
    for (int b = threadIdx.x; b < B; b += blockDim.x) {
      if (!br[b].alive) continue;
      const double u = br[b].util[res];
      hot = u > hot ? u : hot;
      cold = u < cold ? u : cold;
      if (allowedAlive[b]) {
        const double cap = br[b].cap[res];
        const double pct = u / cap;
        if (pct >= P.lowerThr[res] && pct <= P.upperThr[res]) bal++;
        const double d = u - P.avgPct[res] * cap;
        varSum += d * d;
      }
    }
    hot = blockReduce(hot, OpMax(), sd);
    cold = blockReduce(cold, OpMin(), sd);
    varSum = blockReduce(varSum, OpAdd(), sd);
    bal = blockReduce(bal, OpAdd(), si);
    if (threadIdx.x == 0) {
      out->numBalanced[res] = bal;
      out->resAvg[res] = P.clusterUtil[res] / na;
      out->resMax[res] = hot;
      out->resMin[res] = cold;
      out->resStd[res] = sqrt(varSum / na);
    }
  }
  // potential NW_OUT
  {
    double s = 0.0;
    for (int b = threadIdx.x; b < B; b += blockDim.x)
      if (br[b].alive && allowedAlive[b]) s += br[b].pot;
    s = blockReduce(s, OpAdd(), sd);
    const double avgPct = s / P.potCapacity;
    double hot = 0.0, cold = 1.7976931348623157e308, varSum = 0.0;
    int under = 0;
    for (int b = threadIdx.x; b < B; b += blockDim.x) {
      if (!br[b].alive) continue;
      const double u = br[b].pot;
      const double cap = br[b].cap[2];
      hot = u > hot ? u : hot;
      cold = u < cold ? u : cold;
      if (allowedAlive[b]) {
        if (u / cap <= P.nwOutCapThreshold) under++;
        const double d = u - avgPct * cap;
        varSum += d * d;
      }
    }
    hot = blockReduce(hot, OpMax(), sd);
    cold = blockReduce(cold, OpMin(), sd);
    varSum = blockReduce(varSum, OpAdd(), sd);
    under = blockReduce(under, OpAdd(), si);
    if (threadIdx.x == 0) {
      out->pnwAvg = s / na;
      out->pnwMax = hot;
      out->pnwMin = cold;
      out->pnwStd = sqrt(varSum / na);
      out->numUnderPot = under;
    }
  }
  // replica and leader counts (populateReplicaStats: totals/max/min over all brokers, variance over allowed)
  for (int which = 0; which < 2; ++which) {
    int total = 0, mx = 0, mn = 0x7fffffff;
    for (int b = threadIdx.x; b < B; b += blockDim.x) {
      const int n = which == 0 ? br[b].nrep : br[b].nlead;
      total += n;
      mx = n > mx ? n : mx;
      mn = n < mn ? n : mn;
    }
    total = blockReduce(total, OpAdd(), si);
    mx = blockReduce(mx, OpMax(), si);
    mn = blockReduce(mn, OpMin(), si);
    const double avg = ((double)total) / na;
    double var = 0.0;
    for (int b = threadIdx.x; b < B; b += blockDim.x)
      if (br[b].alive && allowedAlive[b]) {
        const double d = (double)(which == 0 ? br[b].nrep : br[b].nlead) - avg;
        var += (d * d) / na;
      }
    var = blockReduce(var, OpAdd(), sd);
    if (threadIdx.x == 0) {
      if (which == 0) {
        out->repAvg = avg;
        out->repStd = sqrt(var);
        out->repMax = mx;
        out->repMin = mn;
      } else {
        out->leadAvg = avg;
        out->leadStd = sqrt(var);
        out->leadMax = mx;
        out->leadMin = mn;
      }
    }
  }
  // topic records
  {
    double avgSum = 0.0, sdSum = 0.0;
    int mx = 0, mn = 0x7fffffff;
    for (int t = threadIdx.x; t < P.T; t += blockDim.x) {
      const TopicPartial x = topics[t];
      avgSum += x.avg;
      sdSum += x.sd;
      mx = x.mx > mx ? x.mx : mx;
      mn = x.mn < mn ? x.mn : mn;
    }
    avgSum = blockReduce(avgSum, OpAdd(), sd);
    sdSum = blockReduce(sdSum, OpAdd(), sd);
    mx = blockReduce(mx, OpMax(), si);
    mn = blockReduce(mn, OpMin(), si);
    if (threadIdx.x == 0) {
      out->topicAvg = avgSum / P.T;
      out->topicStd = sdSum / P.T;
      out->topicMax = mx;
      out->topicMin = mn;
    }
  }
}

hipError_t launchStats(const StatsParams& P, const int32_t* tc, const int32_t* topicNrep, const BrokerRec* brokers,
                       const uint8_t* allowedAlive, TopicPartial* scratch, StatsOut* out, int ldB, hipStream_t st,
                       hipEvent_t evTopic0, hipEvent_t evTopic1) {
  int blocks = P.T < 8192 ? P.T : 8192;
  if (blocks < 1) blocks = 1;
  if (evTopic0) (void)hipEventRecord(evTopic0, st);
  hipLaunchKernelGGL(stats_topics, dim3(blocks), dim3(kTB), 0, st, tc, topicNrep, allowedAlive, P.B, ldB, P.T,
                     P.numAllowed, scratch);
  if (evTopic1) (void)hipEventRecord(evTopic1, st);
  hipLaunchKernelGGL(stats_final, dim3(1), dim3(1024), 0, st, P, brokers, allowedAlive, scratch, out);
  return hipGetLastError();
}

}  // namespace ccmi
