// Fp multiplication microbenchmark on gfx950: current 12x32-bit CIOS vs a
// 14x28-bit radix (every partial product accumulates in place into a 64-bit
// column with one v_mad_u64_u32; no carry chain inside the product).
// Each lane runs 4 independent multiplication chains; reports Fp muls/s.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "bls381_field.hpp"

using namespace bls381;

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

struct f28 { uint32_t l[14]; };
constexpr uint32_t M28 = (1u << 28) - 1;
__device__ __host__ constexpr uint32_t Q28[14] = {
#include "q28.inc"
};
__device__ __host__ constexpr uint32_t QINV28 =
#include "qinv28.inc"
;

__device__ __host__ __attribute__((noinline)) f28 mul28(f28 a, f28 b) {
  uint64_t T[28];
#pragma unroll
  for (int k = 0; k < 28; ++k) T[k] = 0;
#pragma unroll
  for (int i = 0; i < 14; ++i)
#pragma unroll
    for (int j = 0; j < 14; ++j) T[i + j] += (uint64_t)a.l[i] * b.l[j];
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    const uint32_t m = ((uint32_t)T[i] * QINV28) & M28;
#pragma unroll
    for (int j = 0; j < 14; ++j) T[i + j] += (uint64_t)m * Q28[j];
    T[i + 1] += T[i] >> 28;
  }
  f28 r;
  uint64_t c = 0;
#pragma unroll
  for (int j = 0; j < 14; ++j) {
    const uint64_t v = T[14 + j] + c;
    r.l[j] = (uint32_t)v & M28;
    c = v >> 28;
  }
  // conditional subtract q (canonical output < q)
  f28 d;
  int32_t br = 0;
#pragma unroll
  for (int j = 0; j < 14; ++j) {
    int32_t t = (int32_t)r.l[j] - (int32_t)Q28[j] + br;
    d.l[j] = (uint32_t)t & M28;
    br = t >> 28;   // arithmetic: -1 on borrow
  }
#pragma unroll
  for (int j = 0; j < 14; ++j) r.l[j] = br ? r.l[j] : d.l[j];
  return r;
}

__device__ __host__ __attribute__((noinline)) f28 sqr28(f28 a) {
  uint64_t T[28];
  uint32_t a2[14];
#pragma unroll
  for (int k = 0; k < 28; ++k) T[k] = 0;
#pragma unroll
  for (int i = 0; i < 14; ++i) a2[i] = a.l[i] << 1;
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    T[2 * i] += (uint64_t)a.l[i] * a.l[i];
#pragma unroll
    for (int j = i + 1; j < 14; ++j) T[i + j] += (uint64_t)a2[i] * a.l[j];
  }
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    const uint32_t m = ((uint32_t)T[i] * QINV28) & M28;
#pragma unroll
    for (int j = 0; j < 14; ++j) T[i + j] += (uint64_t)m * Q28[j];
    T[i + 1] += T[i] >> 28;
  }
  f28 r;
  uint64_t c = 0;
#pragma unroll
  for (int j = 0; j < 14; ++j) {
    const uint64_t v = T[14 + j] + c;
    r.l[j] = (uint32_t)v & M28;
    c = v >> 28;
  }
  f28 d;
  int32_t br = 0;
#pragma unroll
  for (int j = 0; j < 14; ++j) {
    int32_t t = (int32_t)r.l[j] - (int32_t)Q28[j] + br;
    d.l[j] = (uint32_t)t & M28;
    br = t >> 28;
  }
#pragma unroll
  for (int j = 0; j < 14; ++j) r.l[j] = br ? r.l[j] : d.l[j];
  return r;
}

constexpr int ITERS = 256;

__global__ __launch_bounds__(256) void k_v0(uint32_t* out, const uint32_t* in) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  fp_t x[4];
  for (int c = 0; c < 4; ++c)
    for (int k = 0; k < 12; ++k) x[c].w[k] = in[(c * 12 + k) % 48] ^ (k == 0 ? (uint32_t)t : 0u);
  for (int c = 0; c < 4; ++c) x[c].w[11] &= 0x0fffffff;
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int c = 0; c < 4; ++c) x[c] = fp_mul(x[c], x[(c + 1) & 3]);
  uint32_t s = 0;
  for (int c = 0; c < 4; ++c) for (int k = 0; k < 12; ++k) s ^= x[c].w[k];
  out[t] = s;
}

template <bool SQR>
__global__ __launch_bounds__(256) void k_v1(uint32_t* out, const uint32_t* in) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  f28 x[4];
  for (int c = 0; c < 4; ++c)
    for (int k = 0; k < 14; ++k) x[c].l[k] = (in[(c * 14 + k) % 48] ^ (k == 0 ? (uint32_t)t : 0u)) & M28;
  for (int c = 0; c < 4; ++c) x[c].l[13] &= 0xffff;
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int c = 0; c < 4; ++c) x[c] = SQR ? sqr28(x[c]) : mul28(x[c], x[(c + 1) & 3]);
  uint32_t s = 0;
  for (int c = 0; c < 4; ++c) for (int k = 0; k < 14; ++k) s ^= x[c].l[k];
  out[t] = s;
}

// correctness: x*y for given inputs, 28-bit vs reference via host
__global__ void k_check(const uint32_t* a, const uint32_t* b, uint32_t* o, int n) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  f28 x, y;
  for (int k = 0; k < 14; ++k) { x.l[k] = a[t * 14 + k]; y.l[k] = b[t * 14 + k]; }
  f28 r = mul28(x, y);
  f28 s = sqr28(x);
  for (int k = 0; k < 14; ++k) { o[t * 28 + k] = r.l[k]; o[t * 28 + 14 + k] = s.l[k]; }
}

template <typename K>
double run(K k, uint32_t* d_out, uint32_t* d_in, int blocks) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d_out, d_in);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  const int reps = 3;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d_out, d_in);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main(int argc, char** argv) {
  // correctness inputs from file (host-generated): n, a[n*14], b[n*14], expect[n*28]
  FILE* f = fopen(argc > 1 ? argv[1] : "tools/fpmul_check.bin", "rb");
  if (!f) { printf("no check file\n"); return 1; }
  int n; if (fread(&n, 4, 1, f) != 1) return 1;
  uint32_t* h = (uint32_t*)malloc(sizeof(uint32_t) * n * 56);
  if (fread(h, 4, (size_t)n * 56, f) != (size_t)n * 56) return 1;
  fclose(f);
  uint32_t *d_a, *d_b, *d_o;
  CHECK(hipMalloc(&d_a, n * 56)); CHECK(hipMalloc(&d_b, n * 56)); CHECK(hipMalloc(&d_o, n * 112));
  CHECK(hipMemcpy(d_a, h, n * 56, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_b, h + n * 14, n * 56, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_check, dim3((n + 63) / 64), dim3(64), 0, 0, d_a, d_b, d_o, n);
  uint32_t* o = (uint32_t*)malloc(n * 112);
  CHECK(hipMemcpy(o, d_o, n * 112, hipMemcpyDeviceToHost));
  int bad = memcmp(o, h + n * 28, n * 112) != 0;
  printf("{\"check_ok\": %s", bad ? "false" : "true");
  hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, 0));
  const int blocks = p.multiProcessorCount * 4;   // 4 x 256 lanes per CU
  uint32_t* d_out; uint32_t* d_in;
  CHECK(hipMalloc(&d_out, blocks * 256 * 4)); CHECK(hipMalloc(&d_in, 48 * 4));
  CHECK(hipMemcpy(d_in, h, 48 * 4, hipMemcpyHostToDevice));
  const double muls = (double)blocks * 256 * ITERS * 4;
  double t0 = run(k_v0, d_out, d_in, blocks);
  double t1 = run(k_v1<false>, d_out, d_in, blocks);
  double t2 = run(k_v1<true>, d_out, d_in, blocks);
  printf(", \"v0_cios32_Gmul_s\": %.2f, \"v1_radix28_mul_Gmul_s\": %.2f, \"v1_radix28_sqr_Gmul_s\": %.2f}\n",
         muls / t0 / 1e6, muls / t1 / 1e6, muls / t2 / 1e6);
  return 0;
}
