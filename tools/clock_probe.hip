// Shader-clock probe: a v_mad_u64_u32 issue loop (8 independent chains per lane, as in
// tools/valu_peak.hip) with s_memtime (shader cycles) and s_memrealtime (100 MHz) stamps per wave,
// so the clock the SIMDs ran at during the loop is Δmemtime / Δrealtime · 100 MHz.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/clock_probe.hip -o tools/clock_probe
//   ./tools/clock_probe [blocks]      (256 threads per block; 16384 = the full-chip case of valu_peak)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <unistd.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int ITERS = 4096;

__global__ __launch_bounds__(256) void k_mad_clock(uint64_t* out, unsigned long long* stamps, uint32_t seed, int iters) {
  uint32_t a = seed + threadIdx.x, b = seed * 3u + blockIdx.x;
  uint64_t acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = (uint64_t)(a + k) << 7;
  const unsigned long long c0 = __builtin_readcyclecounter(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      uint64_t cy;
      asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[k]), "=s"(cy) : "v"(a), "v"(b));
    }
  }
  const unsigned long long c1 = __builtin_readcyclecounter(), r1 = __builtin_amdgcn_s_memrealtime();
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) {
    unsigned long long* p = stamps + ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 2;
    p[0] = c1 - c0;
    p[1] = r1 - r0;
  }
}

int main(int argc, char** argv) {
  // clock_probe [blocks] [threads per block] [idle ms before each timed launch] [launches] [iterations]
  const int blocks = argc > 1 ? atoi(argv[1]) : 16384;
  const int threads = argc > 2 ? atoi(argv[2]) : 256;
  const int idle_ms = argc > 3 ? atoi(argv[3]) : 0;
  const int reps = argc > 4 ? atoi(argv[4]) : 1;
  const int iters = argc > 5 ? atoi(argv[5]) : ITERS;
  const int wpb = (threads + 63) / 64;
  uint64_t* out;
  unsigned long long* st;
  CHECK(hipMalloc(&out, (size_t)blocks * 256 * 8));
  CHECK(hipMalloc(&st, (size_t)blocks * 4 * 2 * 8));
  hipLaunchKernelGGL(k_mad_clock, dim3(blocks), dim3(threads), 0, 0, out, st, 7u, iters);
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int r = 0; r < reps; ++r) {
    if (idle_ms) usleep(1000 * idle_ms);
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k_mad_clock, dim3(blocks), dim3(threads), 0, 0, out, st, 9u, iters);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> h((size_t)blocks * 8);
    CHECK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
    double cyc = 0, rt = 0;
    for (int b = 0; b < blocks; ++b)
      for (int w = 0; w < wpb; ++w) { cyc += (double)h[((size_t)b * 4 + w) * 2]; rt += (double)h[((size_t)b * 4 + w) * 2 + 1]; }
    const double macs = (double)blocks * threads * iters * 8;
    printf("{\"blocks\": %d, \"threads\": %d, \"idle_ms\": %d, \"ms\": %.4f, \"mad_Tops\": %.3f, \"s_memtime_ghz\": %.3f, "
           "\"cycles_per_mad_per_wave\": %.3f}\n", blocks, threads, idle_ms, ms, macs / (ms * 1e-3) / 1e12, cyc / (rt * 10.0),
           (cyc / ((double)blocks * wpb)) / (iters * 8.0));
  }
  return 0;
}
