// Round-trip latency probe for the scan protocol (measurement tool, not product code).
// Each case: host prepares a small payload, launches one kernel that consumes it and publishes a sequence
// number into host-coherent memory, host spins until it sees it. Reports the average host wall time per
// round trip over many iterations.
//
//   hipcc --offload-arch=gfx950 -O2 tools/latency_probe.hip -o tools/latency_probe && ./tools/latency_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));          \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

struct Args2K {
  int v[500];
};

__device__ __forceinline__ void publish(unsigned long long* mail, unsigned long long word) {
  __hip_atomic_store(mail, word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_empty(unsigned long long* mail, unsigned long long seq) {
  if (threadIdx.x == 0 && blockIdx.x == 0) publish(mail, seq << 32);
}
__global__ void k_read(const int* __restrict__ src, unsigned long long* mail, unsigned long long seq) {
  if (threadIdx.x == 0 && blockIdx.x == 0) publish(mail, (seq << 32) | (unsigned)src[0]);
}
__global__ void k_read_chain(const int* __restrict__ src, unsigned long long* mail, unsigned long long seq) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    int a = src[0];
    int b = src[1 + (a & 7)];
    publish(mail, (seq << 32) | (unsigned)(a + b));
  }
}
__global__ void k_args(Args2K a, unsigned long long* mail, unsigned long long seq) {
  if (threadIdx.x == 0 && blockIdx.x == 0) publish(mail, (seq << 32) | (unsigned)(a.v[0] + a.v[499]));
}
__global__ void k_wide(const int* __restrict__ src, int n, unsigned long long* mail, unsigned long long seq,
                       unsigned int* done) {
  __shared__ int s;
  int acc = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) acc += src[i];
  if (threadIdx.x == 0) s = 0;
  __syncthreads();
  atomicAdd(&s, acc);
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    unsigned prev = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {
      *done = 0;
      publish(mail, (seq << 32) | (unsigned)s);
    }
  }
}

static unsigned long long g_seq = 0;

static void spin(volatile unsigned long long* mail, unsigned long long seq) {
  while ((__atomic_load_n(mail, __ATOMIC_ACQUIRE) >> 32) != (seq & 0xffffffffull)) __builtin_ia32_pause();
}

template <class F>
static double timeit(const char* name, int iters, F&& f) {
  for (int i = 0; i < 50; ++i) f();
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < iters; ++i) f();
  const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / iters;
  std::printf("%-58s %8.2f us\n", name, us);
  return us;
}

int main() {
  CK(hipSetDevice(0));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  unsigned long long* mail;
  CK(hipHostMalloc((void**)&mail, 4096, hipHostMallocMapped | hipHostMallocCoherent));
  std::memset(mail, 0, 4096);
  unsigned long long* mailDev;
  CK(hipHostGetDevicePointer((void**)&mailDev, mail, 0));
  int* hcoh;
  CK(hipHostMalloc((void**)&hcoh, 1 << 20, hipHostMallocMapped | hipHostMallocCoherent));
  int* hcohDev;
  CK(hipHostGetDevicePointer((void**)&hcohDev, hcoh, 0));
  int* hnc;
  CK(hipHostMalloc((void**)&hnc, 1 << 20, hipHostMallocMapped | hipHostMallocNonCoherent));
  int* hncDev;
  CK(hipHostGetDevicePointer((void**)&hncDev, hnc, 0));
  int* dmem;
  CK(hipMalloc((void**)&dmem, 1 << 20));
  unsigned int* done;
  CK(hipMalloc((void**)&done, 64));
  CK(hipMemset(done, 0, 64));
  for (int i = 0; i < 1024; ++i) hcoh[i] = hnc[i] = i;
  const int N = 2000;

  timeit("launch + hipStreamSynchronize (empty kernel)", N, [&] {
    ++g_seq;
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st, mailDev, g_seq);
    CK(hipStreamSynchronize(st));
  });
  timeit("launch + mailbox spin (empty kernel)", N, [&] {
    ++g_seq;
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st, mailDev, g_seq);
    spin(mail, g_seq);
  });
  timeit("read 1 int from host-coherent memory + mailbox", N, [&] {
    ++g_seq;
    hcoh[0] = (int)g_seq;
    hipLaunchKernelGGL(k_read, dim3(1), dim3(64), 0, st, hcohDev, mailDev, g_seq);
    spin(mail, g_seq);
  });
  timeit("2 dependent reads from host-coherent memory + mailbox", N, [&] {
    ++g_seq;
    hipLaunchKernelGGL(k_read_chain, dim3(1), dim3(64), 0, st, hcohDev, mailDev, g_seq);
    spin(mail, g_seq);
  });
  timeit("2 dependent reads from host non-coherent memory + mailbox", N, [&] {
    ++g_seq;
    hipLaunchKernelGGL(k_read_chain, dim3(1), dim3(64), 0, st, hncDev, mailDev, g_seq);
    spin(mail, g_seq);
  });
  timeit("2 dependent reads from HBM + mailbox", N, [&] {
    ++g_seq;
    hipLaunchKernelGGL(k_read_chain, dim3(1), dim3(64), 0, st, dmem, mailDev, g_seq);
    spin(mail, g_seq);
  });
  timeit("2 KB kernel-argument payload + mailbox", N, [&] {
    ++g_seq;
    Args2K a;
    a.v[0] = (int)g_seq;
    a.v[499] = 1;
    hipLaunchKernelGGL(k_args, dim3(1), dim3(64), 0, st, a, mailDev, g_seq);
    spin(mail, g_seq);
  });
  timeit("hipMemcpyAsync 4 KB H2D (pinned) + read kernel + mailbox", N, [&] {
    ++g_seq;
    CK(hipMemcpyAsync(dmem, hcoh, 4096, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_read, dim3(1), dim3(64), 0, st, dmem, mailDev, g_seq);
    spin(mail, g_seq);
  });
  timeit("two kernels back to back + mailbox", N, [&] {
    ++g_seq;
    hipLaunchKernelGGL(k_read, dim3(1), dim3(64), 0, st, dmem, mailDev, g_seq - 1);
    hipLaunchKernelGGL(k_read, dim3(1), dim3(64), 0, st, dmem, mailDev, g_seq);
    spin(mail, g_seq);
  });
  for (int n : {4096, 65536, 262144}) {
    char name[96];
    std::snprintf(name, sizeof name, "wide read of %d ints from host-coherent (64 blocks) + mailbox", n);
    timeit(name, 500, [&] {
      ++g_seq;
      hipLaunchKernelGGL(k_wide, dim3(64), dim3(256), 0, st, hcohDev, n, mailDev, g_seq, done);
      spin(mail, g_seq);
    });
    std::snprintf(name, sizeof name, "wide read of %d ints from HBM (64 blocks) + mailbox", n);
    timeit(name, 500, [&] {
      ++g_seq;
      hipLaunchKernelGGL(k_wide, dim3(64), dim3(256), 0, st, dmem, n, mailDev, g_seq, done);
      spin(mail, g_seq);
    });
  }
  // fine-grained device memory written by the CPU through the BAR (posted writes), read by the kernel from HBM
  int* fg = nullptr;
  if (hipExtMallocWithFlags((void**)&fg, 1 << 20, hipDeviceMallocFinegrained) == hipSuccess) {
    hipPointerAttribute_t attr;
    const bool ok = hipPointerGetAttributes(&attr, fg) == hipSuccess;
    std::printf("fine-grained VRAM allocated (attr ok=%d, type=%d)\n", (int)ok, ok ? (int)attr.type : -1);
    std::fflush(stdout);
    // host store into it: only when the pointer is host-accessible (large BAR); a fault here ends the probe
    volatile int* hv = fg;
    hv[0] = 7;
    std::printf("host store to fine-grained VRAM ok, readback %d\n", hv[0]);
    std::fflush(stdout);
    timeit("host writes 1 int to fine-grained VRAM + 2 dependent reads + mailbox", N, [&] {
      ++g_seq;
      hv[0] = (int)g_seq;
      hipLaunchKernelGGL(k_read_chain, dim3(1), dim3(64), 0, st, fg, mailDev, g_seq);
      spin(mail, g_seq);
    });
    static int buf[16384];
    for (int n : {256, 4096, 16384}) {
      char name[112];
      std::snprintf(name, sizeof name, "host memcpy %d ints to fine-grained VRAM + wide read (64 blocks) + mailbox", n);
      timeit(name, 500, [&] {
        ++g_seq;
        buf[0] = (int)g_seq;
        std::memcpy(fg, buf, (size_t)n * 4);
        hipLaunchKernelGGL(k_wide, dim3(64), dim3(256), 0, st, fg, n, mailDev, g_seq, done);
        spin(mail, g_seq);
      });
      std::snprintf(name, sizeof name, "host memcpy %d ints to host-coherent + wide read (64 blocks) + mailbox", n);
      timeit(name, 500, [&] {
        ++g_seq;
        buf[0] = (int)g_seq;
        std::memcpy(hcoh, buf, (size_t)n * 4);
        hipLaunchKernelGGL(k_wide, dim3(64), dim3(256), 0, st, hcohDev, n, mailDev, g_seq, done);
        spin(mail, g_seq);
      });
    }
  } else {
    std::printf("fine-grained VRAM allocation failed\n");
  }
  std::printf("done\n");
  return 0;
}
