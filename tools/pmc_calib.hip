// FETCH_SIZE / WRITE_SIZE calibration on scan_cross's own access pattern (MI355X_MICROARCH.md, HBM section:
// "Other access widths are uncalibrated: calibrate on a known byte count in your own access pattern").
//
// Each kernel touches every byte it is credited with exactly once, from a table 4x the Infinity Cache, so the
// memory-side counters see misses only:
//   stream16  : 16 B per lane coalesced streaming read of the table (the guide's calibrated x2 case: the control)
//   gather128 : one lane per BrokerRec at a random permutation index, reading the fields PreView::loadDst reads
//               (scan.hip) — scan_cross's destination-record gather
//   gather64  : one lane per 64 B record (ReplicaRec / PartitionRec size) at a random index, all 8 dwordx2 fields
//   gather8   : one lane per 128 B record reading only its 8 B `pot` field (a partial line)
// Each kernel writes one double per lane (coalesced, 8 B/lane) so WRITE_SIZE can be checked too.
//
// Prints one JSON line with the algorithmic bytes per dispatch of each kernel; tools/pmc_summary.py --calib pairs
// it with the --pmc FETCH_SIZE / WRITE_SIZE passes of the same binary.
//
//   hipcc -O3 --offload-arch=gfx950 tools/pmc_calib.hip -o tools/pmc_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#include "../cruise-control_amd/csrc/engine/devtypes.h"

using ccmi::BrokerRec;

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

__global__ __launch_bounds__(256) void stream16(const int4* __restrict__ t, size_t n4, double* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const int4 v = t[i];
  out[i] = (double)(v.x ^ v.y ^ v.z ^ v.w);
}

__global__ __launch_bounds__(256) void gather128(const BrokerRec* __restrict__ t, const int32_t* __restrict__ idx,
                                                 int n, double* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const BrokerRec& b = t[idx[i]];
  double s = b.util[0] + b.util[1] + b.util[2] + b.util[3] + b.cap[0] + b.cap[1] + b.cap[2] + b.cap[3] + b.pot + b.lbi;
  s += (double)(b.nrep + b.nlead + b.rack + (int)b.allowedBits + b.alive);
  out[i] = s;
}

struct Rec64 {
  double f[8];
};

__global__ __launch_bounds__(256) void gather64(const Rec64* __restrict__ t, const int32_t* __restrict__ idx, int n,
                                                double* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const Rec64& r = t[idx[i]];
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += r.f[k];
  out[i] = s;
}

__global__ __launch_bounds__(256) void gather8(const BrokerRec* __restrict__ t, const int32_t* __restrict__ idx, int n,
                                               double* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  out[i] = t[idx[i]].pot;
}

int main() {
  const size_t tableBytes = (size_t)1 << 30;  // 1 GiB: 4x the 256 MiB Infinity Cache
  const int n128 = (int)(tableBytes / sizeof(BrokerRec)), n64 = (int)(tableBytes / sizeof(Rec64));
  const size_t n4 = tableBytes / 16;
  void* table = nullptr;
  int32_t *idx128 = nullptr, *idx64 = nullptr;
  double* out = nullptr;
  CK(hipMalloc(&table, tableBytes));
  CK(hipMemset(table, 1, tableBytes));
  CK(hipMalloc(&idx128, (size_t)n128 * 4));
  CK(hipMalloc(&idx64, (size_t)n64 * 4));
  CK(hipMalloc(&out, n4 * 8));
  std::mt19937 rng(20261016u);
  {
    std::vector<int32_t> p(n128);
    std::iota(p.begin(), p.end(), 0);
    std::shuffle(p.begin(), p.end(), rng);
    CK(hipMemcpy(idx128, p.data(), p.size() * 4, hipMemcpyHostToDevice));
  }
  {
    std::vector<int32_t> p(n64);
    std::iota(p.begin(), p.end(), 0);
    std::shuffle(p.begin(), p.end(), rng);
    CK(hipMemcpy(idx64, p.data(), p.size() * 4, hipMemcpyHostToDevice));
  }
  // flush the Infinity Cache of the index uploads by streaming the table once first
  hipLaunchKernelGGL(stream16, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, 0, (const int4*)table, n4, out);
  hipLaunchKernelGGL(stream16, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, 0, (const int4*)table, n4, out);
  hipLaunchKernelGGL(gather128, dim3((n128 + 255) / 256), dim3(256), 0, 0, (const BrokerRec*)table, idx128, n128, out);
  hipLaunchKernelGGL(gather64, dim3((n64 + 255) / 256), dim3(256), 0, 0, (const Rec64*)table, idx64, n64, out);
  hipLaunchKernelGGL(gather8, dim3((n128 + 255) / 256), dim3(256), 0, 0, (const BrokerRec*)table, idx128, n128, out);
  CK(hipDeviceSynchronize());
  // algorithmic bytes per dispatch: every line of the table the kernel touches, plus index reads and output writes
  std::printf(
      "{\"table_bytes\": %zu, \"kernels\": {"
      "\"stream16\": {\"read\": %zu, \"write\": %zu, \"dispatches_counted\": \"second\"}, "
      "\"gather128\": {\"read\": %zu, \"write\": %zu, \"useful_read\": %zu}, "
      "\"gather64\": {\"read\": %zu, \"write\": %zu}, "
      "\"gather8\": {\"read\": %zu, \"write\": %zu, \"useful_read\": %zu}}}\n",
      tableBytes, tableBytes, n4 * 8, tableBytes + (size_t)n128 * 4, (size_t)n128 * 8,
      (size_t)n128 * 100 + (size_t)n128 * 4, tableBytes + (size_t)n64 * 4, (size_t)n64 * 8,
      tableBytes + (size_t)n128 * 4, (size_t)n128 * 8, (size_t)n128 * 12);
  CK(hipFree(table));
  CK(hipFree(idx128));
  CK(hipFree(idx64));
  CK(hipFree(out));
  return 0;
}
