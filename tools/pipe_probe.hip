// Which instruction classes compete with v_mad_u64_u32 for issue on gfx950.  Every lane runs
// 8 independent MAC chains; each loop iteration adds K extra instructions of one class per MAC
// (independent of the chains).  Two waves per SIMD (2,048 waves), as the verify kernels run.
// If an op class co-issues beside the MACs, the time stays at the MAC-only time; if it takes
// the MAC's issue slot, each extra op costs what a MAC costs.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/pipe_probe.hip -o tools/pipe_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int ITERS = 16384;

template <int OP, int K>
__global__ __launch_bounds__(256) void k_probe(uint64_t* out, uint32_t seed) {
  uint32_t a = seed + threadIdx.x, b = seed * 3u + blockIdx.x;
  uint64_t acc[8];
  uint32_t x[8];
  uint64_t y[4];
#pragma unroll
  for (int k = 0; k < 8; ++k) { acc[k] = (uint64_t)(a + k) << 7; x[k] = a * (k + 1); }
#pragma unroll
  for (int k = 0; k < 4; ++k) y[k] = (uint64_t)(b + k) << 9;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      uint64_t cy;
      asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[k]), "=s"(cy) : "v"(a), "v"(b));
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const int t = (k * K + j) & 7;
        if (OP == 1) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(x[t]) : "v"(a));
        if (OP == 2) asm volatile("v_alignbit_b32 %0, %1, %0, 28" : "+v"(x[t]) : "v"(b));
        if (OP == 3) asm volatile("v_lshrrev_b64 %0, 28, %0" : "+v"(y[t & 3]));
        if (OP == 4) asm volatile("v_lshl_add_u64 %0, %1, 0, %0" : "+v"(y[t & 3]) : "v"(y[(t + 1) & 3]));
        if (OP == 5) asm volatile("v_mul_lo_u32 %0, %1, %0" : "+v"(x[t]) : "v"(a));
        if (OP == 6) asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=v"(x[t]) : "v"(x[(t + 1) & 7]));
        if (OP == 7) asm volatile("v_add_co_u32 %0, vcc, %1, %0\n\tv_addc_co_u32 %2, vcc, %3, %2, vcc" : "+v"(x[t]), "+v"(x[(t + 4) & 7]) : "v"(a), "v"(b) : "vcc");
        if (OP == 8) asm volatile("v_and_b32 %0, 0xfffffff, %0" : "+v"(x[t]));
        if (OP == 9) asm volatile("v_add3_u32 %0, %1, %2, %0" : "+v"(x[t]) : "v"(a), "v"(b));
      }
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s ^= acc[k] ^ x[k];
#pragma unroll
  for (int k = 0; k < 4; ++k) s ^= y[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OP, int K>
static void run(const char* name, uint64_t* out, int blocks, double base_ms) {
  hipLaunchKernelGGL((k_probe<OP, K>), dim3(blocks), dim3(256), 0, 0, out, 7u);
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0, 0));
  hipLaunchKernelGGL((k_probe<OP, K>), dim3(blocks), dim3(256), 0, 0, out, 9u);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  // SIMD cycles per extra op relative to one MAC: (t - t_mac) / t_mac * (MACs / extra ops)
  const double rel = base_ms > 0 ? (ms - base_ms) / base_ms / K : 0.0;
  printf("{\"op\": \"%s\", \"per_mac\": %d, \"ms\": %.4f, \"extra_cost_in_macs\": %.3f}\n", name, K, ms, rel);
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 512;   // 512 x 256 lanes = 2,048 waves = 2 per SIMD
  uint64_t* out;
  CHECK(hipMalloc(&out, (size_t)blocks * 256 * 8));
  // baseline: MACs only
  hipLaunchKernelGGL((k_probe<0, 0>), dim3(blocks), dim3(256), 0, 0, out, 7u);
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0, 0));
  hipLaunchKernelGGL((k_probe<0, 0>), dim3(blocks), dim3(256), 0, 0, out, 9u);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float base = 0;
  CHECK(hipEventElapsedTime(&base, e0, e1));
  const double macs = (double)blocks * 256 * ITERS * 8;
  printf("{\"op\": \"mac only\", \"blocks\": %d, \"ms\": %.4f, \"mad_Tops\": %.2f}\n", blocks, base, macs / (base * 1e-3) / 1e12);
  run<1, 1>("v_xor_b32", out, blocks, base);
  run<1, 2>("v_xor_b32", out, blocks, base);
  run<8, 1>("v_and_b32 (literal)", out, blocks, base);
  run<9, 1>("v_add3_u32", out, blocks, base);
  run<2, 1>("v_alignbit_b32", out, blocks, base);
  run<3, 1>("v_lshrrev_b64", out, blocks, base);
  run<4, 1>("v_lshl_add_u64", out, blocks, base);
  run<5, 1>("v_mul_lo_u32", out, blocks, base);
  run<6, 1>("v_mov_b32_dpp", out, blocks, base);
  run<7, 1>("v_add_co_u32 + v_addc_co_u32", out, blocks, base);
  return 0;
}
