// Microbenchmark of the final exponentiation's compressed squaring on 2^16 items
// (lane pairs, two waves per SIMD like k_final_exp_verdict):
//   k_csqr_gs    the Fp2-squaring form (6 fp2_sqr calls + reduced combinations)
//   k_csqr_lazy  the lazily reduced form (bls381_lazy.hpp, cyc_csqr_lazy)
// plus the signed / unsigned 64-bit multiply-add issue rates.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I consensus-specs_amd/csrc tools/csqr_bench.hip -o tools/csqr_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "bls381_pair.hpp"

using namespace bls381;

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

__device__ __forceinline__ fp_t ld(const uint32_t* p, size_t nl, size_t lane, int c) {
  fp_t r;
#pragma unroll
  for (int k = 0; k < 14; ++k) r.w[k] = p[(size_t)(c * 14 + k) * nl + lane] & FP_MASK;
  r.w[13] &= 0x7ffff;
  return r;
}
__device__ __forceinline__ void st(uint32_t* p, size_t nl, size_t lane, int c, const fp_t& a) {
#pragma unroll
  for (int k = 0; k < 14; ++k) p[(size_t)(c * 14 + k) * nl + lane] = a.w[k];
}

__device__ __forceinline__ cyc_bc<fp2p_t> csqr_gs(const cyc_bc<fp2p_t>& g) {
  cyc_bc<fp2p_t> r;
  {
    const fp2p_t t0 = fp2_sqr(g.g4), t1 = fp2_sqr(g.g5), t2 = fp2_sqr(fp2_add(g.g4, g.g5));
    r.g2 = fp2_3p2(fp2_mul_xi(fp2_sub2(t2, t0, t1)), g.g2);
    r.g3 = fp2_3m2(fp2_add_mul_xi(t0, t1), g.g3);
  }
  const fp2p_t t3 = fp2_sqr(g.g2), t4 = fp2_sqr(g.g3), t5 = fp2_sqr(fp2_add(g.g2, g.g3));
  r.g4 = fp2_3m2(fp2_add_mul_xi(t3, t4), g.g4);
  r.g5 = fp2_3p2(fp2_sub2(t5, t3, t4), g.g5);
  return r;
}

#define KHEAD                                                        \
  const size_t lane = (size_t)blockIdx.x * blockDim.x + threadIdx.x; \
  if (lane >= nl) return;                                            \
  cyc_bc<fp2p_t> g;                                                  \
  g.g2 = pr_make(ld(in, nl, lane, 0)); g.g3 = pr_make(ld(in, nl, lane, 1)); \
  g.g4 = pr_make(ld(in, nl, lane, 2)); g.g5 = pr_make(ld(in, nl, lane, 3));
#define KTAIL \
  st(out, nl, lane, 0, g.g2.v); st(out, nl, lane, 1, g.g3.v); st(out, nl, lane, 2, g.g4.v); st(out, nl, lane, 3, g.g5.v);

__global__ void __launch_bounds__(128, 2) k_csqr_gs(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  KHEAD
  for (int i = 0; i < reps; ++i) g = csqr_gs(g);
  KTAIL
}
__global__ void __launch_bounds__(128, 2) k_csqr_lazy(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  KHEAD
  for (int i = 0; i < reps; ++i) g = cyc_csqr_lazy(g);
  KTAIL
}
// the lazy form with the scheduler fenced between outputs (live range of one wide value)
__global__ void __launch_bounds__(128, 2) k_csqr_lazy_fenced(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  KHEAD
  for (int i = 0; i < reps; ++i) {
    const bool p = pr_odd();
    cyc_bc<fp2p_t> r;
    const fp_t e4 = pr_dpp<DPP_EVEN>(g.g4.v), o4 = pr_dpp<DPP_ODD>(g.g4.v);
    const fp_t e5 = pr_dpp<DPP_EVEN>(g.g5.v), o5 = pr_dpp<DPP_ODD>(g.g5.v);
    r.g2 = pr_make(fp_6p2(lz_xi_mul(p, e4, o4, e5, o5), g.g2.v));
    BLS_PHASE();
    r.g3 = pr_make(fp_3m2(lz_sqr_xisqr(p, e4, o4, e5, o5), g.g3.v));
    BLS_PHASE();
    const fp_t e2 = pr_dpp<DPP_EVEN>(g.g2.v), o2 = pr_dpp<DPP_ODD>(g.g2.v);
    const fp_t e3 = pr_dpp<DPP_EVEN>(g.g3.v), o3 = pr_dpp<DPP_ODD>(g.g3.v);
    r.g4 = pr_make(fp_3m2(lz_sqr_xisqr(p, e2, o2, e3, o3), g.g4.v));
    BLS_PHASE();
    r.g5 = pr_make(fp_6p2(lz_mul(p, e2, o2, e3, o3), g.g5.v));
    BLS_PHASE();
    g = r;
  }
  KTAIL
}
// one lazy output only (2 products + 1 reduction per lane) vs one fp2 product
__global__ void __launch_bounds__(128, 2) k_lz_mul(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  KHEAD
  for (int i = 0; i < reps; ++i) {
    const fp_t e = pr_dpp<DPP_EVEN>(g.g2.v), o = pr_dpp<DPP_ODD>(g.g2.v);
    const fp_t e3 = pr_dpp<DPP_EVEN>(g.g3.v), o3 = pr_dpp<DPP_ODD>(g.g3.v);
    g.g2 = pr_make(lz_mul(pr_odd(), e, o, e3, o3));
  }
  KTAIL
}
__global__ void __launch_bounds__(128, 2) k_fp2_mul(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  KHEAD
  for (int i = 0; i < reps; ++i) g.g2 = fp2_mul(g.g2, g.g3);
  KTAIL
}

// whole exponentiation by x / whole final exponentiation, one per item
__device__ __forceinline__ fp12_g<fp2p_t> ld12(const uint32_t* p, size_t nl, size_t lane) {
  fp12_g<fp2p_t> f;
  f.c0.c0.v = ld(p, nl, lane, 0); f.c0.c1.v = ld(p, nl, lane, 1); f.c0.c2.v = ld(p, nl, lane, 2);
  f.c1.c0.v = ld(p, nl, lane, 3); f.c1.c1.v = ld(p, nl, lane, 4); f.c1.c2.v = ld(p, nl, lane, 5);
  return f;
}
__device__ __forceinline__ void st12(uint32_t* p, size_t nl, size_t lane, const fp12_g<fp2p_t>& f) {
  st(p, nl, lane, 0, f.c0.c0.v); st(p, nl, lane, 1, f.c0.c1.v); st(p, nl, lane, 2, f.c0.c2.v);
  st(p, nl, lane, 3, f.c1.c0.v); st(p, nl, lane, 4, f.c1.c1.v); st(p, nl, lane, 5, f.c1.c2.v);
}
__global__ void __launch_bounds__(128, 2) k_cyc_exp_x(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  const size_t lane = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= nl) return;
  fp12_g<fp2p_t> f = ld12(in, nl, lane);
  for (int i = 0; i < reps; ++i) f = cyc_exp_x(f);
  st12(out, nl, lane, f);
}
__global__ void __launch_bounds__(128, 2) k_final_exp(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  const size_t lane = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= nl) return;
  fp12_g<fp2p_t> f = ld12(in, nl, lane);
  for (int i = 0; i < reps; ++i) f = final_exp(f);
  st12(out, nl, lane, f);
}
__global__ void __launch_bounds__(128, 2) k_fp12_mul(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  const size_t lane = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= nl) return;
  fp12_g<fp2p_t> f = ld12(in, nl, lane), g = ld12(in + 6 * 14 * nl / 2, nl / 2, lane / 2);
  for (int i = 0; i < reps; ++i) f = fp12_mul_inl(f, g);
  st12(out, nl, lane, f);
}

constexpr int ITERS = 4096;
__global__ __launch_bounds__(256) void k_mad_u64(uint64_t* o, uint32_t seed) {
  uint32_t a = seed + threadIdx.x, b = seed * 3u + blockIdx.x;
  uint64_t acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = (uint64_t)(a + k) << 7;
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      uint64_t cy;
      asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[k]), "=s"(cy) : "v"(a), "v"(b));
    }
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s ^= acc[k];
  o[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_mad_i64(uint64_t* o, uint32_t seed) {
  uint32_t a = seed + threadIdx.x, b = seed * 3u + blockIdx.x;
  uint64_t acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = (uint64_t)(a + k) << 7;
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      uint64_t cy;
      asm volatile("v_mad_i64_i32 %0, %1, %2, %3, %0" : "+v"(acc[k]), "=s"(cy) : "v"(a), "v"(b));
    }
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s ^= acc[k];
  o[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  const size_t n = 1 << 16, nl = 2 * n;
  std::vector<uint32_t> h(12 * 14 * nl);
  uint64_t x = 88172645463325252ull;
  for (auto& v : h) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = (uint32_t)x; }
  uint32_t *in, *out;
  CHECK(hipMalloc(&in, h.size() * 4));
  CHECK(hipMalloc(&out, h.size() * 4));
  CHECK(hipMemcpy(in, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const dim3 grid((unsigned)(nl / 128)), blk(128);
  auto time = [&](const char* name, void (*k)(size_t, int, const uint32_t*, uint32_t*), int reps) {
    hipLaunchKernelGGL(k, grid, blk, 0, 0, nl, reps, in, out);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(k, grid, blk, 0, 0, nl, reps, in, out);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"kernel\": \"%s\", \"reps\": %d, \"ms\": %.3f, \"us_per_op\": %.3f}\n", name, reps, ms, 1e3 * ms / reps);
  };
  time("csqr_gs", k_csqr_gs, 63);
  time("csqr_lazy", k_csqr_lazy, 63);
  time("csqr_lazy_fenced", k_csqr_lazy_fenced, 63);
  time("lz_mul", k_lz_mul, 63);
  time("fp2_mul", k_fp2_mul, 63);
  time("cyc_exp_x", k_cyc_exp_x, 1);
  time("fp12_mul", k_fp12_mul, 16);
  time("final_exp", k_final_exp, 1);
  uint64_t* o;
  CHECK(hipMalloc(&o, 1024 * 256 * 8 * 8));
  auto rate = [&](const char* name, void (*k)(uint64_t*, uint32_t)) {
    const dim3 g(1024 * 8), b(256);
    hipLaunchKernelGGL(k, g, b, 0, 0, o, 7u);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(k, g, b, 0, 0, o, 7u);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double ops = (double)g.x * b.x * ITERS * 8;
    printf("{\"instr\": \"%s\", \"Tops\": %.3f}\n", name, ops / (ms * 1e-3) / 1e12);
  };
  rate("v_mad_u64_u32", k_mad_u64);
  rate("v_mad_i64_i32", k_mad_i64);
  return 0;
}
