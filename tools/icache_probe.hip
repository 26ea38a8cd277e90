// Does a lone wave pay for instruction fetch on long straight-line code?  A v_mad_u64_u32 stream
// as one straight-line body of BODY instructions (8 bytes each), run ITERS times, against the same
// number of MACs in a small loop; one wave alone, two or four waves of one workgroup (one CU), and
// one wave in each of two workgroups.  HISTORY.md, round 5 (latency).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/icache_probe.hip -o tools/icache_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

#define STR2(x) #x
#define STR(x) STR2(x)
#define MACS(N) asm volatile(".rept " STR(N) "\n\tv_mad_u64_u32 v[4:5], s[20:21], v2, v3, v[4:5]\n\t.endr" ::: "v2", "v3", "v4", "v5", "s20", "s21")

template <int BIG>
__global__ __launch_bounds__(256) void k_fetch(uint64_t* out, int iters) {
  asm volatile("v_mov_b32 v2, %0\n\tv_mov_b32 v3, %0\n\tv_mov_b32 v4, 0\n\tv_mov_b32 v5, 0" : : "v"(threadIdx.x) : "v2", "v3", "v4", "v5");
  for (int i = 0; i < iters; ++i) {
    if (BIG) MACS(12288);     // 96 KiB of code per pass
    else MACS(256);           // 2 KiB, resident in the instruction cache
  }
  uint32_t r;
  asm volatile("v_mov_b32 %0, v4" : "=v"(r) : : "v4");
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int BIG>
static void run(uint64_t* out, int blocks, int threads, int iters) {
  hipLaunchKernelGGL((k_fetch<BIG>), dim3(blocks), dim3(threads), 0, 0, out, iters);
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int rep = 0; rep < 3; ++rep) {
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL((k_fetch<BIG>), dim3(blocks), dim3(threads), 0, 0, out, iters);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double macs_per_wave = (double)iters * (BIG ? 12288 : 256);
    printf("{\"body\": \"%s\", \"blocks\": %d, \"threads\": %d, \"ms\": %.4f, \"ns_per_mac_per_wave\": %.3f}\n",
           BIG ? "96KiB straight-line" : "2KiB loop", blocks, threads, ms, 1e6 * ms / macs_per_wave);
  }
}

int main() {
  uint64_t* out;
  CHECK(hipMalloc(&out, 1024 * 256 * 8));
  const int cfg[][2] = {{1, 64}, {1, 128}, {1, 256}, {2, 64}, {1, 64}};
  for (auto& c : cfg) {
    run<1>(out, c[0], c[1], 16);
    run<0>(out, c[0], c[1], 1024);
  }
  return 0;
}
