// Component microbenchmarks of the gfx950 pipeline kernels: each kernel runs one
// building block of the verify pipeline on 2^16 items (lane pairs, two waves per
// SIMD like the production kernels) so the per-item time of every block can be
// compared with its instruction count ("where the time goes").
// Inputs are random field elements; only timing is reported.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I consensus-specs_amd/csrc tools/micro_bench.hip -o tools/micro_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "bls381_pair.hpp"

using namespace bls381;

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

using fp12p = fp12_g<fp2p_t>;

__device__ __forceinline__ fp_t ld(const uint32_t* p, size_t nl, size_t lane, int c) {
  fp_t r;
#pragma unroll
  for (int k = 0; k < 14; ++k) r.w[k] = p[(size_t)(c * 14 + k) * nl + lane] & FP_MASK;
  r.w[13] &= 0x7ffff;   // value < 2^383 / 16 < q
  return r;
}
__device__ __forceinline__ void st(uint32_t* p, size_t nl, size_t lane, int c, const fp_t& a) {
#pragma unroll
  for (int k = 0; k < 14; ++k) p[(size_t)(c * 14 + k) * nl + lane] = a.w[k];
}
__device__ __forceinline__ fp12p ld12(const uint32_t* p, size_t nl, size_t lane) {
  fp12p f;
  f.c0.c0.v = ld(p, nl, lane, 0); f.c0.c1.v = ld(p, nl, lane, 1); f.c0.c2.v = ld(p, nl, lane, 2);
  f.c1.c0.v = ld(p, nl, lane, 3); f.c1.c1.v = ld(p, nl, lane, 4); f.c1.c2.v = ld(p, nl, lane, 5);
  return f;
}
__device__ __forceinline__ void st12(uint32_t* p, size_t nl, size_t lane, const fp12p& f) {
  st(p, nl, lane, 0, f.c0.c0.v); st(p, nl, lane, 1, f.c0.c1.v); st(p, nl, lane, 2, f.c0.c2.v);
  st(p, nl, lane, 3, f.c1.c0.v); st(p, nl, lane, 4, f.c1.c1.v); st(p, nl, lane, 5, f.c1.c2.v);
}

#define KHEAD                                                        \
  const size_t lane = (size_t)blockIdx.x * blockDim.x + threadIdx.x; \
  if (lane >= nl) return;

__global__ void __launch_bounds__(128, 2) k_fp2mul(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  KHEAD
  fp2p_t x = pr_make(ld(in, nl, lane, 0)), y = pr_make(ld(in, nl, lane, 1));
  for (int i = 0; i < reps; ++i) x = fp2_mul(x, y);
  st(out, nl, lane, 0, x.v);
}
// two independent products per step, bodies inlined (ILP inside one call boundary)
__global__ void __launch_bounds__(128, 2) k_fp2mul_x2(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  KHEAD
  fp_t x = ld(in, nl, lane, 0), y = ld(in, nl, lane, 1), z = ld(in, nl, lane, 2), w = ld(in, nl, lane, 3);
  for (int i = 0; i < reps; i += 2) {
    x = fp2p_mul_body(x, y);
    z = fp2p_mul_body(z, w);
  }
  st(out, nl, lane, 0, x); st(out, nl, lane, 1, z);
}
// the call loop at 3 and 4 waves per SIMD
__global__ void __launch_bounds__(128, 3) k_fp2mul_o3(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  KHEAD
  fp2p_t x = pr_make(ld(in, nl, lane, 0)), y = pr_make(ld(in, nl, lane, 1));
  for (int i = 0; i < reps; ++i) x = fp2_mul(x, y);
  st(out, nl, lane, 0, x.v);
}
__global__ void __launch_bounds__(128, 4) k_fp2mul_o4(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  KHEAD
  fp2p_t x = pr_make(ld(in, nl, lane, 0)), y = pr_make(ld(in, nl, lane, 1));
  for (int i = 0; i < reps; ++i) x = fp2_mul(x, y);
  st(out, nl, lane, 0, x.v);
}
__global__ void __launch_bounds__(128, 1) k_fp2mul_o1(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  KHEAD
  fp2p_t x = pr_make(ld(in, nl, lane, 0)), y = pr_make(ld(in, nl, lane, 1));
  for (int i = 0; i < reps; ++i) x = fp2_mul(x, y);
  st(out, nl, lane, 0, x.v);
}
__global__ void __launch_bounds__(128, 2) k_fp2sqr(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  KHEAD
  fp2p_t x = pr_make(ld(in, nl, lane, 0));
  for (int i = 0; i < reps; ++i) x = fp2_sqr(x);
  st(out, nl, lane, 0, x.v);
}
__global__ void __launch_bounds__(128, 2) k_fpmul(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  KHEAD
  fp_t x = ld(in, nl, lane, 0), y = ld(in, nl, lane, 1);
  for (int i = 0; i < reps; ++i) x = fp_mul(x, y);
  st(out, nl, lane, 0, x);
}
__global__ void __launch_bounds__(128, 2) k_fp2add(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  KHEAD
  fp2p_t x = pr_make(ld(in, nl, lane, 0)), y = pr_make(ld(in, nl, lane, 1));
  for (int i = 0; i < reps; ++i) x = fp2_add_mul_xi(x, y);
  st(out, nl, lane, 0, x.v);
}
__global__ void __launch_bounds__(128, 2) k_inv(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  KHEAD
  fp_t x = ld(in, nl, lane, 0);
  for (int i = 0; i < reps; ++i) x = fp_inv(x);
  st(out, nl, lane, 0, x);
}
__global__ void __launch_bounds__(128, 2) k_csqr(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  KHEAD
  cyc_bc<fp2p_t> g;
  g.g2.v = ld(in, nl, lane, 0); g.g3.v = ld(in, nl, lane, 1); g.g4.v = ld(in, nl, lane, 2); g.g5.v = ld(in, nl, lane, 3);
  for (int i = 0; i < reps; ++i) g = cyc_csqr(g);
  st(out, nl, lane, 0, g.g2.v); st(out, nl, lane, 1, g.g3.v); st(out, nl, lane, 2, g.g4.v); st(out, nl, lane, 3, g.g5.v);
}
__global__ void __launch_bounds__(128, 2) k_fp12mul(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  KHEAD
  fp12p f = ld12(in, nl, lane), g = ld12(in + 6 * 14 * nl, nl, lane);
  for (int i = 0; i < reps; ++i) f = fp12_mul(f, g);
  st12(out, nl, lane, f);
}
__global__ void __launch_bounds__(128, 2) k_fp12mul_inl(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  KHEAD
  fp12p f = ld12(in, nl, lane), g = ld12(in + 6 * 14 * nl, nl, lane);
  for (int i = 0; i < reps; ++i) f = fp12_mul_inl(f, g);
  st12(out, nl, lane, f);
}
__global__ void __launch_bounds__(128, 2) k_decomp(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  KHEAD
  cyc_bc<fp2p_t> g;
  g.g2.v = ld(in, nl, lane, 0); g.g3.v = ld(in, nl, lane, 1); g.g4.v = ld(in, nl, lane, 2); g.g5.v = ld(in, nl, lane, 3);
  fp2p_t inv = pr_make(ld(in, nl, lane, 4));
  fp12p f = fp12_one<fp2p_t>();
  for (int i = 0; i < reps; ++i) {
    const fp12p x = cyc_decompress(g, inv);
    g.g2 = x.c0.c0; inv = x.c1.c1;
  }
  st(out, nl, lane, 0, g.g2.v); st(out, nl, lane, 1, inv.v);
}
__global__ void __launch_bounds__(128, 2) k_ml1(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  KHEAD
  aff_t<fp2p_t> Q;
  Q.x.v = ld(in, nl, lane, 0); Q.y.v = ld(in, nl, lane, 1);
  aff_t<fp_t> p; p.x = ld(in, nl, lane, 2); p.y = ld(in, nl, lane, 3);
  const g1_line_pre P = g1_prepare(p);
  fp12p f = fp12_one<fp2p_t>();
  bool degen = false;
  for (int i = 0; i < reps; ++i) {
    const fp12p g = miller_loop_n<1>(&Q, &P, degen);
    f.c0.c0 = fp2_add(f.c0.c0, g.c0.c0);
  }
  st12(out, nl, lane, f);
}
__global__ void __launch_bounds__(128, 2) k_cycexp(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  KHEAD
  fp12p f = ld12(in, nl, lane);
  for (int i = 0; i < reps; ++i) f = cyc_exp_x(f);
  st12(out, nl, lane, f);
}
__global__ void __launch_bounds__(128, 2) k_fe(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  KHEAD
  fp12p f = ld12(in, nl, lane);
  for (int i = 0; i < reps; ++i) f = final_exp(f);
  st12(out, nl, lane, f);
}
__global__ void __launch_bounds__(128, 2) k_ml2(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  KHEAD
  aff_t<fp2p_t> Q[2];
  g1_line_pre P[2];
  for (int k = 0; k < 2; ++k) {
    Q[k].x.v = ld(in, nl, lane, 4 * k); Q[k].y.v = ld(in, nl, lane, 4 * k + 1);
    aff_t<fp_t> p; p.x = ld(in, nl, lane, 4 * k + 2); p.y = ld(in, nl, lane, 4 * k + 3);
    P[k] = g1_prepare(p);
  }
  fp12p f = fp12_one<fp2p_t>();
  bool degen = false;
  for (int i = 0; i < reps; ++i) {
    const fp12p g = miller_loop_n<2>(Q, P, degen);
    f.c0.c0 = fp2_add(f.c0.c0, g.c0.c0);
  }
  st12(out, nl, lane, f);
}
__global__ void __launch_bounds__(128, 2) k_bp(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  KHEAD
  aff_t<fp2p_t> p;
  p.x.v = ld(in, nl, lane, 0); p.y.v = ld(in, nl, lane, 1);
  for (int i = 0; i < reps; ++i) {
    const jac_t<fp2p_t> r = g2_mul_bp(p);
    p.x = r.x; p.y = r.y;
  }
  st(out, nl, lane, 0, p.x.v); st(out, nl, lane, 1, p.y.v);
}
__global__ void __launch_bounds__(128, 2) k_fp2inv(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  KHEAD
  fp2p_t x = pr_make(ld(in, nl, lane, 0));
  for (int i = 0; i < reps; ++i) x = fp2_inv(x);
  st(out, nl, lane, 0, x.v);
}
__global__ void __launch_bounds__(128, 2) k_candidate(size_t nl, int reps, const uint32_t* in, uint32_t* out) {
  KHEAD
  uint8_t msg[32], dom[8] = {0, 0, 0, 0, 0, 0, 0, 3};
  for (int k = 0; k < 8; ++k) {
    const uint32_t w = in[(size_t)k * nl + (lane & ~(size_t)1)];
    msg[4 * k] = (uint8_t)w; msg[4 * k + 1] = (uint8_t)(w >> 8); msg[4 * k + 2] = (uint8_t)(w >> 16);
    msg[4 * k + 3] = (uint8_t)(w >> 24);
  }
  aff_t<fp2p_t> c;
  for (int i = 0; i < reps; ++i) { hash_to_g2_candidate(c, msg, 32, dom); msg[0] ^= (uint8_t)c.x.v.w[0]; }
  st(out, nl, lane, 0, c.x.v); st(out, nl, lane, 1, c.y.v);
}

typedef void (*kfn)(size_t, int, const uint32_t*, uint32_t*);
struct Bench { const char* name; kfn k; int reps; const char* unit; };

int main(int argc, char** argv) {
  const size_t items = argc > 1 ? strtoull(argv[1], 0, 0) : 65536;
  const size_t nl = 2 * items;
  const size_t words = 12 * 14 * nl;
  std::vector<uint32_t> h(words);
  uint64_t s = 0x9E3779B97F4A7C15ull;
  for (auto& w : h) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; w = (uint32_t)s; }
  uint32_t *din, *dout;
  CHECK(hipMalloc(&din, words * 4));
  CHECK(hipMalloc(&dout, words * 4));
  CHECK(hipMemcpy(din, h.data(), words * 4, hipMemcpyHostToDevice));
  const Bench B[] = {
      {"fp_mul (one lane)", k_fpmul, 256, "op"},
      {"fp2_mul (pair)", k_fp2mul, 256, "op"},
      {"fp2_mul x2 inlined (pair)", k_fp2mul_x2, 256, "op"},
      {"fp2_mul 1 wave/SIMD (pair)", k_fp2mul_o1, 256, "op"},
      {"fp2_mul 3 waves/SIMD (pair)", k_fp2mul_o3, 256, "op"},
      {"fp2_mul 4 waves/SIMD (pair)", k_fp2mul_o4, 256, "op"},
      {"fp2_sqr (pair)", k_fp2sqr, 256, "op"},
      {"fp2_add_mul_xi (pair)", k_fp2add, 1024, "op"},
      {"fp_inv (xgcd)", k_inv, 8, "op"},
      {"fp12_mul_inl (pair)", k_fp12mul_inl, 16, "op"},
      {"cyc_decompress (pair)", k_decomp, 16, "op"},
      {"miller_loop_n<1> (pair)", k_ml1, 1, "op"},
      {"fp2_inv (pair)", k_fp2inv, 8, "op"},
      {"cyc_csqr (pair)", k_csqr, 315, "op"},
      {"fp12_mul (pair)", k_fp12mul, 16, "op"},
      {"cyc_exp_x (pair)", k_cycexp, 5, "op"},
      {"final_exp (pair)", k_fe, 1, "op"},
      {"miller_loop_n<2> (pair)", k_ml2, 1, "op"},
      {"g2_mul_bp (pair)", k_bp, 1, "op"},
      {"hash candidate (pair)", k_candidate, 1, "op"},
  };
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const dim3 blk(128), grid((unsigned)((nl + 127) / 128));
  printf("{\"items\": %zu, \"results\": [\n", items);
  bool first = true;
  for (const auto& b : B) {
    hipLaunchKernelGGL(b.k, grid, blk, 0, 0, nl, b.reps, din, dout);   // warm-up
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(b.k, grid, blk, 0, 0, nl, b.reps, din, dout);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    printf("%s  {\"block\": \"%s\", \"reps\": %d, \"ms\": %.4f, \"ms_per_rep_2^16_items\": %.5f}", first ? "" : ",\n",
           b.name, b.reps, ms, ms / b.reps * 65536.0 / items);
    first = false;
    fflush(stdout);
  }
  printf("\n]}\n");
  CHECK(hipFree(din));
  CHECK(hipFree(dout));
  return 0;
}
