// MetricValues / AggregatedMetricValues arithmetic shared by the host model and the gfx950 kernels that apply moves
// on the device, so both produce the same bits (built with -ffp-contract=off everywhere):
//   MetricValues.add / subtract / set / avg      cruise-control-core/.../aggregator/MetricValues.java:39-45,100-160
//   AggregatedMetricValues.add / subtract        cruise-control-core/.../aggregator/AggregatedMetricValues.java
//   ModelUtils.expectedUtilizationFor            model/ModelUtils.java:162-176
//   Replica.makeFollower / computeCpuLoadAsFollower, ModelUtils.getFollowerCpuUtilFromLeaderLoad
//                                                model/Replica.java:210-305, model/ModelUtils.java:64-80
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define CCMI_LD __host__ __device__ __forceinline__
#else
#define CCMI_LD inline
#endif

namespace ccmi {

enum Res { R_CPU = 0, R_NW_IN = 1, R_NW_OUT = 2, R_DISK = 3 };
enum Met { M_CPU = 0, M_DISK = 1, M_LBI = 2, M_LBO = 3, M_RBI = 4, M_RBO = 5 };
constexpr int kMaxW = 5;

struct Window {  // one MetricValues: float window values (newest first) + double running sum
  float v[kMaxW];
  double sum;
};
struct LoadVec {  // AggregatedMetricValues over the 6 resource metrics (bit k of mask: metric k present)
  uint8_t mask = 0;
  Window m[6];
};
static_assert(sizeof(Window) == 32 && sizeof(LoadVec) == 200, "LoadVec layout is shared with the device");

CCMI_LD double ldMax0(double a) {  // Math.max(a, 0.0): NaN stays NaN, -0.0 becomes +0.0
  if (a != a) return a;
  return a > 0.0 ? a : 0.0;
}
CCMI_LD void ldZero(Window& x, int W) {
  for (int i = 0; i < W; ++i) x.v[i] = 0.f;
  x.sum = 0.0;
}
CCMI_LD void ldAdd(Window& a, const Window& b, int W) {
  for (int i = 0; i < W; ++i) {
    const double d = (double)b.v[i];
    a.v[i] = (float)((double)a.v[i] + d);
    a.sum += d;
  }
}
CCMI_LD void ldSub(Window& a, const Window& b, int W) {
  for (int i = 0; i < W; ++i) {
    const double d = (double)b.v[i];
    a.v[i] = (float)((double)a.v[i] - d);
    a.sum -= d;
  }
}
CCMI_LD void ldSet(Window& a, int i, double x) {
  a.sum += x - (double)a.v[i];
  a.v[i] = (float)x;
}
CCMI_LD float ldAvg(const Window& a, int W) { return (float)(a.sum / W); }
// AggregatedMetricValues.add: a missing metric is created (zeroed) first
CCMI_LD void ldAddAll(LoadVec& d, const LoadVec& s, int W) {
  for (int k = 0; k < 6; ++k)
    if (s.mask >> k & 1) {
      if (!(d.mask >> k & 1)) {
        ldZero(d.m[k], W);
        d.mask |= (uint8_t)(1 << k);
      }
      ldAdd(d.m[k], s.m[k], W);
    }
}
// AggregatedMetricValues.subtract (the caller guarantees every metric of s is present in d)
CCMI_LD void ldSubAll(LoadVec& d, const LoadVec& s, int W) {
  for (int k = 0; k < 6; ++k)
    if (s.mask >> k & 1) ldSub(d.m[k], s.m[k], W);
}
CCMI_LD double ldUtil(const LoadVec& l, int res, int W) {  // ModelUtils.expectedUtilizationFor
  if (!l.mask) return 0.0;
  double r = 0;
  switch (res) {
    case R_CPU: r += (double)ldAvg(l.m[M_CPU], W); break;
    case R_DISK: r += (double)l.m[M_DISK].v[0]; break;
    case R_NW_IN:
      r += (double)ldAvg(l.m[M_LBI], W);
      r += (double)ldAvg(l.m[M_RBI], W);
      break;
    default:
      r += (double)ldAvg(l.m[M_LBO], W);
      r += (double)ldAvg(l.m[M_RBO], W);
      break;
  }
  return ldMax0(r);
}

// Replica.makeFollower's load change (Replica.java:221-305): the replica keeps the follower CPU
// (ModelUtils.getFollowerCpuUtilFromLeaderLoad, weights 0.7 / 0.15 / 0.15) and drops its NW_OUT; returns the delta
// (CPU, LEADER_BYTES_OUT, REPLICATION_BYTES_OUT) that moves to the new leader.
CCMI_LD void ldMakeFollower(LoadVec& L, LoadVec& delta, int W) {
  Window totOut, totIn, chg;
  ldZero(totOut, W);
  ldAdd(totOut, L.m[M_LBO], W);
  ldAdd(totOut, L.m[M_RBO], W);
  ldZero(totIn, W);
  ldAdd(totIn, L.m[M_LBI], W);
  ldAdd(totIn, L.m[M_RBI], W);
  ldZero(chg, W);
  for (int i = 0; i < W; ++i) {
    const double in = (double)totIn.v[i], out = (double)totOut.v[i], c = (double)L.m[M_CPU].v[i];
    const double follower = (in == 0.0 && out == 0.0) ? 0.0 : c * (0.15 * in) / (0.7 * in + 0.15 * out);
    ldSet(chg, i, (double)L.m[M_CPU].v[i] - follower);
    ldSet(L.m[M_CPU], i, follower);
  }
  delta.mask = (1 << M_CPU) | (1 << M_LBO) | (1 << M_RBO);
  ldZero(delta.m[M_CPU], W);
  ldAdd(delta.m[M_CPU], chg, W);
  ldZero(delta.m[M_LBO], W);
  ldAdd(delta.m[M_LBO], L.m[M_LBO], W);
  ldZero(delta.m[M_RBO], W);
  ldAdd(delta.m[M_RBO], L.m[M_RBO], W);
  ldZero(L.m[M_LBO], W);
  ldZero(L.m[M_RBO], W);
}

}  // namespace ccmi
