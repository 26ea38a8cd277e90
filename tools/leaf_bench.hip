// Issue efficiency of the lane-pair Fp2 product (the leaf every G2 / Fp12 kernel calls),
// 2^16 items (2,048 waves, two per SIMD unless a kernel says otherwise): time per product
// and the share of the v_mad issue bound it reaches.  Parts timed separately: the 2x14x14
// column product, the Montgomery reduction, and the whole product as a call or inlined.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I consensus-specs_amd/csrc tools/leaf_bench.hip -o tools/leaf_bench
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
#define KHEAD const size_t lane = (size_t)blockIdx.x * blockDim.x + threadIdx.x; if (lane >= nl) return;

// the 2x14x14 columns only (the product half of fp2p_mul_body), folded to 14 words
__device__ __forceinline__ fp_t prod_only(const fp_t& a, const fp_t& b) {
  const bool odd = pr_odd();
  const fp_t ao = pr_dpp<DPP_SWAP>(a), b0 = pr_dpp<DPP_EVEN>(b), b1 = pr_dpp<DPP_ODD>(b);
  uint32_t w[14];
#pragma unroll
  for (int k = 0; k < 14; ++k) w[k] = odd ? b1.w[k] : Q8S_LIMBS[k] - b1.w[k];
  uint64_t T[28];
#pragma unroll
  for (int k = 0; k < 28; ++k) T[k] = 0;
#pragma unroll
  for (int i = 0; i < 14; ++i)
#pragma unroll
    for (int j = 0; j < 14; ++j) { T[i + j] += (uint64_t)a.w[i] * b0.w[j]; T[i + j] += (uint64_t)ao.w[i] * w[j]; }
  fp_t r;
#pragma unroll
  for (int k = 0; k < 14; ++k) r.w[k] = ((uint32_t)T[k] ^ (uint32_t)(T[k + 14] >> 20)) & FP_MASK;
  return r;
}
// the Montgomery reduction only, of a wide value built from a, b without products
__device__ __forceinline__ fp_t redc_only(const fp_t& a, const fp_t& b) {
  uint64_t T[28];
#pragma unroll
  for (int k = 0; k < 14; ++k) { T[k] = ((uint64_t)a.w[k] << 30) + b.w[k]; T[k + 14] = ((uint64_t)b.w[k] << 30) + a.w[k]; }
  return fp_redc_wide(T);
}
__device__ __noinline__ fpv_t prod_call(fpv_t a, fpv_t b) { return fp_pack(prod_only(fp_unpack(a), fp_unpack(b))); }
__device__ __noinline__ fpv_t redc_call(fpv_t a, fpv_t b) { return fp_pack(redc_only(fp_unpack(a), fp_unpack(b))); }

template <int W>
__global__ void __launch_bounds__(128, W) k_call(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  KHEAD
  fp2p_t x = pr_make(ld(in, nl, lane, 0)), y = pr_make(ld(in, nl, lane, 1));
  for (int i = 0; i < reps; ++i) x = fp2_mul(x, y);
  st(out, nl, lane, 0, x.v);
}
// two independent chains, each product a call
__global__ void __launch_bounds__(128, 2) k_call2(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  KHEAD
  fp2p_t x = pr_make(ld(in, nl, lane, 0)), y = pr_make(ld(in, nl, lane, 1));
  fp2p_t z = pr_make(ld(in, nl, lane, 2)), w = pr_make(ld(in, nl, lane, 3));
  for (int i = 0; i < reps; i += 2) { x = fp2_mul(x, y); z = fp2_mul(z, w); }
  st(out, nl, lane, 0, x.v); st(out, nl, lane, 1, z.v);
}
__global__ void __launch_bounds__(128, 2) k_inl(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  KHEAD
  fp_t x = ld(in, nl, lane, 0), y = ld(in, nl, lane, 1);
  for (int i = 0; i < reps; ++i) x = fp2p_mul_body(x, y);
  st(out, nl, lane, 0, x);
}
__global__ void __launch_bounds__(128, 2) k_prod(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  KHEAD
  fpv_t x = fp_pack(ld(in, nl, lane, 0)), y = fp_pack(ld(in, nl, lane, 1));
  for (int i = 0; i < reps; ++i) x = prod_call(x, y);
  st(out, nl, lane, 0, fp_unpack(x));
}
__global__ void __launch_bounds__(128, 2) k_redc(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  KHEAD
  fpv_t x = fp_pack(ld(in, nl, lane, 0)), y = fp_pack(ld(in, nl, lane, 1));
  for (int i = 0; i < reps; ++i) x = redc_call(x, y);
  st(out, nl, lane, 0, fp_unpack(x));
}

typedef void (*kfn)(size_t, int, const uint32_t*, uint32_t*);
struct Bench { const char* name; kfn k; int reps; int macs; };

int main(int argc, char** argv) {
  const size_t items = argc > 1 ? strtoull(argv[1], 0, 0) : 65536;
  const double ghz = argc > 2 ? atof(argv[2]) : 2.1;
  const size_t nl = 2 * items, words = 4 * 14 * nl;
  std::vector<uint32_t> h(words);
  uint64_t s = 0x9E3779B97F4A7C15ull;
  for (auto& x : h) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; x = (uint32_t)s; }
  uint32_t *din, *dout;
  CHECK(hipMalloc(&din, words * 4));
  CHECK(hipMalloc(&dout, words * 4));
  CHECK(hipMemcpy(din, h.data(), words * 4, hipMemcpyHostToDevice));
  const Bench B[] = {
      {"fp2 product, call, 2 waves/SIMD", k_call<2>, 512, 588},
      {"fp2 product, call, 4 waves/SIMD", k_call<4>, 512, 588},
      {"fp2 product, two chains of calls", k_call2, 512, 588},
      {"fp2 product, inlined", k_inl, 512, 588},
      {"column product only (2x14x14), call", k_prod, 512, 392},
      {"Montgomery reduction only, call", k_redc, 512, 196},
  };
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const dim3 blk(128), grid((unsigned)((nl + 127) / 128));
  printf("{\"items\": %zu, \"ghz_assumed\": %.2f, \"results\": [\n", items, ghz);
  for (size_t b = 0; b < sizeof(B) / sizeof(B[0]); ++b) {
    hipLaunchKernelGGL(B[b].k, grid, blk, 0, 0, nl, B[b].reps, din, dout);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(B[b].k, grid, blk, 0, 0, nl, B[b].reps, din, dout);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    // v_mad issue bound: 4 cycles per wave64 MAC on a SIMD; nl / 64 waves over 1,024 SIMDs
    const double waves = (double)nl / 64.0, simd_cycles = waves / 1024.0 * B[b].macs * 4.0 * B[b].reps;
    const double bound_ms = simd_cycles / (ghz * 1e6);
    printf("%s  {\"kernel\": \"%s\", \"us_per_op_2^16\": %.4f, \"mac_issue_frac\": %.3f}", b ? ",\n" : "", B[b].name,
           1e3 * ms / B[b].reps * 65536.0 / items, bound_ms / ms);
  }
  printf("\n]}\n");
  return 0;
}
