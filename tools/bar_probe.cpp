// Host-side write bandwidth into fine-grained VRAM through the BAR (the scan server's command block and snapshot pool
// are written this way) against a DMA copy from pinned host memory: memcpy, 16/32-byte non-temporal stores, 1.6 KB
// pieces as the snapshot uploads write them. Prints one line per variant.
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int main() {
  const size_t bytes = 16u << 20, piece = 1600;
  char* fg = nullptr;
  CK(hipExtMallocWithFlags((void**)&fg, bytes, hipDeviceMallocFinegrained));
  char* coarse = nullptr;
  CK(hipMalloc((void**)&coarse, bytes));
  char* pinned = nullptr;
  CK(hipHostMalloc((void**)&pinned, bytes, hipHostMallocDefault));
  std::vector<char> src(bytes, 1);
  for (size_t i = 0; i < bytes; ++i) src[i] = (char)i;
  auto report = [&](const char* what, double s, size_t n) { std::printf("%-44s %8.2f ms  %8.1f MB/s\n", what, s * 1e3, n / s / 1e6); };
  for (int rep = 0; rep < 2; ++rep) {
    double t = now();
    std::memcpy(fg, src.data(), bytes);
    _mm_sfence();
    report("memcpy 16 MB into fine-grained VRAM", now() - t, bytes);
    t = now();
    for (size_t o = 0; o + piece <= bytes; o += piece) std::memcpy(fg + o, src.data() + o, piece);
    _mm_sfence();
    report("memcpy 1.6 KB pieces", now() - t, bytes / piece * piece);
    t = now();
    for (size_t o = 0; o < bytes; o += 16)
      _mm_stream_si128((__m128i*)(fg + o), _mm_loadu_si128((const __m128i*)(src.data() + o)));
    _mm_sfence();
    report("16-byte non-temporal stores", now() - t, bytes);
    t = now();
    for (size_t o = 0; o < bytes; o += 32)
      _mm256_stream_si256((__m256i*)(fg + o), _mm256_loadu_si256((const __m256i*)(src.data() + o)));
    _mm_sfence();
    report("32-byte non-temporal stores", now() - t, bytes);
    t = now();
    for (size_t o = 0; o < bytes; o += 8) *(volatile unsigned long long*)(fg + o) = *(const unsigned long long*)(src.data() + o);
    _mm_sfence();
    report("8-byte volatile stores", now() - t, bytes);
    std::memcpy(pinned, src.data(), bytes);
    t = now();
    CK(hipMemcpy(coarse, pinned, bytes, hipMemcpyHostToDevice));
    report("hipMemcpy pinned -> VRAM (DMA) 16 MB", now() - t, bytes);
    t = now();
    CK(hipMemcpy(fg, pinned, piece, hipMemcpyHostToDevice));
    report("hipMemcpy pinned -> fine-grained 1.6 KB", now() - t, piece);
  }
  return 0;
}
