// Phase profile of the throughput final exponentiation (final_exp<fp2p_t>, the body of
// k_final_exp_verdict): s_memtime cycle stamps at the BLS_FE_MARK points of bls381_pairing.hpp,
// accumulated per wave in LDS by lane 0 and averaged over the waves.  Full occupancy (2^16 items,
// two waves per SIMD) or one item (a lone wave).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I consensus-specs_amd/csrc tools/fe_phases.hip -o tools/fe_phases
//   ./tools/fe_phases [items]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__shared__ unsigned long long fe_acc[2][8];
__shared__ unsigned long long fe_last[2];
__device__ __forceinline__ void fe_mark(int k) {
  if ((threadIdx.x & 63) == 0) {
    const int w = threadIdx.x >> 6;
    const unsigned long long now = __builtin_readcyclecounter();
    fe_acc[w][k] += now - fe_last[w];
    fe_last[w] = now;
  }
}
#define BLS_FE_MARK(k) fe_mark(k)
#include "bls381_pair.hpp"

using namespace bls381;
using fp12p = fp12_g<fp2p_t>;

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

__device__ __forceinline__ fp_t ld(const uint32_t* p, size_t nl, size_t lane, int c) {
  fp_t r;
#pragma unroll
  for (int k = 0; k < 14; ++k) r.w[k] = p[(size_t)(c * 14 + k) * nl + lane] & FP_MASK;
  r.w[13] &= 0x7ffff;
  return r;
}

__global__ void __launch_bounds__(128, 2) k_fe_phases(size_t nl, const uint32_t* in, uint32_t* out,
                                                      unsigned long long* prof) {
  const size_t lane = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    for (int k = 0; k < 8; ++k) fe_acc[w][k] = 0;
    fe_last[w] = __builtin_readcyclecounter();
  }
  if (lane >= nl) return;
  fp12p f;
  f.c0.c0.v = ld(in, nl, lane, 0); f.c0.c1.v = ld(in, nl, lane, 1); f.c0.c2.v = ld(in, nl, lane, 2);
  f.c1.c0.v = ld(in, nl, lane, 3); f.c1.c1.v = ld(in, nl, lane, 4); f.c1.c2.v = ld(in, nl, lane, 5);
  const unsigned long long t0 = __builtin_readcyclecounter(), r0 = __builtin_amdgcn_s_memrealtime();
  f = final_exp(f);
  const unsigned long long t1 = __builtin_readcyclecounter(), r1 = __builtin_amdgcn_s_memrealtime();
#pragma unroll
  for (int k = 0; k < 14; ++k) out[k * nl + lane] = f.c0.c0.v.w[k];
  if ((threadIdx.x & 63) == 0) {
    unsigned long long* p = prof + ((size_t)blockIdx.x * 2 + w) * 10;
    for (int k = 0; k < 8; ++k) p[k] = fe_acc[w][k];
    p[8] = t1 - t0;
    p[9] = r1 - r0;   // s_memrealtime: constant 100 MHz
  }
}

int main(int argc, char** argv) {
  const size_t items = argc > 1 ? strtoull(argv[1], 0, 0) : 65536;
  const size_t nl = 2 * items, words = 6 * 14 * nl;
  std::vector<uint32_t> h(words);
  uint64_t s = 0x9E3779B97F4A7C15ull;
  for (auto& x : h) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; x = (uint32_t)s; }
  uint32_t *din, *dout;
  unsigned long long* dprof;
  const size_t blocks = (nl + 127) / 128;
  CHECK(hipMalloc(&din, words * 4));
  CHECK(hipMalloc(&dout, 14 * nl * 4));
  CHECK(hipMalloc(&dprof, blocks * 2 * 10 * 8));
  CHECK(hipMemcpy(din, h.data(), words * 4, hipMemcpyHostToDevice));
  CHECK(hipMemset(dprof, 0, blocks * 2 * 10 * 8));
  hipLaunchKernelGGL(k_fe_phases, dim3(blocks), dim3(128), 0, 0, nl, din, dout, dprof);   // warm-up
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0, 0));
  hipLaunchKernelGGL(k_fe_phases, dim3(blocks), dim3(128), 0, 0, nl, din, dout, dprof);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned long long> p(blocks * 2 * 10);
  CHECK(hipMemcpy(p.data(), dprof, p.size() * 8, hipMemcpyDeviceToHost));
  const char* names[9] = {"csqr runs (57 per x-power, x5)", "shared inversion + denominators (x5)",
                          "3 decompressions + 2 Fp12 products (x5)", "GS tail squarings (6 per x-power, x5)",
                          "GS tail Fp12 products (3 per x-power, x5)", "easy part (inverse, 2 products, Frobenius)",
                          "chain tail (c, t^3, result: 5 products, GS square)", "between x-powers (products, Frobenius)",
                          "final_exp total"};
  double sum[10] = {0};
  size_t waves = 0;
  for (size_t b = 0; b < blocks; ++b)
    for (int w = 0; w < 2; ++w) {
      const unsigned long long* q = &p[(b * 2 + w) * 10];
      if (q[8] == 0) continue;
      ++waves;
      for (int k = 0; k < 10; ++k) sum[k] += (double)q[k];
    }
  printf("{\"items\": %zu, \"kernel_ms\": %.4f, \"waves\": %zu, \"phases_cycles_per_wave\": {", items, ms, waves);
  for (int k = 0; k < 9; ++k) printf("%s\"%s\": %.0f", k ? ", " : "", names[k], sum[k] / (waves ? waves : 1));
  printf("}, \"s_memtime_ghz\": %.3f}\n", sum[9] > 0 ? sum[8] / (sum[9] * 10.0) : 0.0);
  return 0;
}
