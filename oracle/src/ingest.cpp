// ORACLE — test infrastructure only (see jsem.h header). Restatement of the per-partition load derivation of
// LoadMonitor.clusterModel: MonitorUtils.populatePartitionLoad (monitor/MonitorUtils.java:415-479) with
// getAggregatedMetricValues (:215-226), adjustCpuUsage (:198-205), fillInReplicationBytesOut (:241-257),
// toFollowerMetricValues (:83-107) and ModelUtils.getFollowerCpuUtilFromLeaderLoad (model/ModelUtils.java:64-80),
// over the reference's float MetricValues (MetricValues.set rounds to float; valuesForGroup adds into zeros).
#include <cstdint>
#include <cstring>
#include <vector>

namespace {
enum { CPU = 0, DISK = 1, LBI = 2, LBO = 3, RBI = 4, RBO = 5, NM = 6 };
}

extern "C" {

// leader_metrics[6*W] (metric-major, newest window first) -> out[n][6*W] for the replicas in PartitionInfo.replicas()
// order; is_leader[i] marks the leader. Returns 0.
int32_t oc_ingest_partition(int32_t W, int32_t n, const uint8_t* is_leader, const float* leader_metrics, float* out) {
  std::vector<float> agg(leader_metrics, leader_metrics + NM * W);  // ValuesAndExtrapolations.metricValues()
  bool needToAdjustCpuUsage = true;
  for (int i = 0; i < n; ++i) {
    float* o = out + (size_t)i * NM * W;
    if (needToAdjustCpuUsage) {
      for (int w = 0; w < W; ++w) agg[CPU * W + w] = (float)(agg[CPU * W + w] * 100.0);
    }
    if (is_leader[i]) {
      for (int w = 0; w < W; ++w) agg[RBO * W + w] = (float)(agg[LBI * W + w] * (double)(n - 1));
      std::memcpy(o, agg.data(), sizeof(float) * NM * W);
    } else {
      for (int w = 0; w < W; ++w) {
        float in = 0.0f, outb = 0.0f;  // valuesForGroup(NW_IN) / valuesForGroup(NW_OUT)
        in += agg[LBI * W + w];
        in += agg[RBI * W + w];
        outb += agg[LBO * W + w];
        outb += agg[RBO * W + w];
        const double bi = in, bo = outb, cpu = agg[CPU * W + w];
        const double f = (bi == 0.0 && bo == 0.0) ? 0.0 : cpu * (0.15 * bi) / (0.7 * bi + 0.15 * bo);
        o[CPU * W + w] = (float)f;
        o[DISK * W + w] = agg[DISK * W + w];
        o[LBI * W + w] = agg[LBI * W + w];
        o[RBI * W + w] = agg[RBI * W + w];
        o[LBO * W + w] = 0.0f;
        o[RBO * W + w] = 0.0f;
      }
    }
    needToAdjustCpuUsage = false;
  }
  return 0;
}

}  // extern "C"
