// Latency of one compressed-squaring chain for a single item: the quad form (cq_sqr, 4 lanes) against
// the octet form (co_sqr, 8 lanes), REPS dependent squarings in one wave with every lane active
// (lanes past the item recompute it), as k_final_exp_verdict_q / _o run them for single calls.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I consensus-specs_amd/csrc tools/csqr_lat.hip -o tools/csqr_lat
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "bls381.h"
#include "bls381_kernels.hpp"

using namespace bls381;

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

__device__ __forceinline__ fp2p_t ldp(const uint32_t* p, int c) {
  fp_t r;
  const int lane = threadIdx.x & 1;
#pragma unroll
  for (int k = 0; k < 14; ++k) r.w[k] = p[(c * 2 + lane) * 14 + k] & FP_MASK;
  r.w[13] &= 0x7ffff;
  return pr_make(r);
}

__global__ void __launch_bounds__(64) k_quad(int reps, const uint32_t* in, uint32_t* out, unsigned long long* cyc) {
  cq_t g;
  g.x = ldp(in, qd_hi() ? 1 : 0);
  g.y = ldp(in, qd_hi() ? 3 : 2);
  const unsigned long long c0 = __builtin_readcyclecounter();
  for (int i = 0; i < reps; ++i) g = cq_sqr(g);
  const unsigned long long c1 = __builtin_readcyclecounter();
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < 14; ++k) s ^= g.x.v.w[k] ^ g.y.v.w[k];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[0] = c1 - c0;
}

__global__ void __launch_bounds__(64) k_oct(int reps, const uint32_t* in, uint32_t* out, unsigned long long* cyc) {
  cq_t q;
  q.x = ldp(in, qd_hi() ? 1 : 0);
  q.y = ldp(in, qd_hi() ? 3 : 2);
  fp2p_t g = co_enter(q);
  const unsigned long long c0 = __builtin_readcyclecounter();
  for (int i = 0; i < reps; ++i) g = co_sqr(g);
  const unsigned long long c1 = __builtin_readcyclecounter();
  const cq_t r = co_exit(g);
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < 14; ++k) s ^= r.x.v.w[k] ^ r.y.v.w[k];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[0] = c1 - c0;
}

int main() {
  std::vector<uint32_t> h(8 * 14);
  uint64_t st = 0x9E3779B97F4A7C15ull;
  for (auto& x : h) { st ^= st << 13; st ^= st >> 7; st ^= st << 17; x = (uint32_t)st; }
  uint32_t *din, *dout;
  unsigned long long* dc;
  CHECK(hipMalloc(&din, h.size() * 4));
  CHECK(hipMalloc(&dout, 64 * 4));
  CHECK(hipMalloc(&dc, 8));
  CHECK(hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  const int reps = 315;
  for (int r = 0; r < 3; ++r) {
    for (int v = 0; v < 2; ++v) {
      hipEvent_t e0, e1;
      CHECK(hipEventCreate(&e0));
      CHECK(hipEventCreate(&e1));
      CHECK(hipEventRecord(e0, 0));
      if (v == 0) hipLaunchKernelGGL(k_quad, dim3(1), dim3(64), 0, 0, reps, din, dout, dc);
      else hipLaunchKernelGGL(k_oct, dim3(1), dim3(64), 0, 0, reps, din, dout, dc);
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      unsigned long long c = 0;
      CHECK(hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost));
      printf("{\"form\": \"%s\", \"squarings\": %d, \"ms\": %.4f, \"cycles_per_squaring\": %.0f}\n",
             v ? "octet co_sqr" : "quad cq_sqr", reps, ms, (double)c / reps);
    }
  }
  return 0;
}
