// Integer-VALU peak microbenchmark for gfx950 (MI355X).
// Measures the sustained rate of the instructions the BLS12-381 field
// arithmetic is built from: v_mad_u64_u32 (32x32+64 -> 64 MAC),
// v_add_co_u32 / v_addc_co_u32 (carry chain) and v_mul_lo/hi_u32.
// The measured v_mad_u64_u32 rate is the roofline denominator reported by
// bench.py (DESIGN.md "Roofline"). Each thread runs 8 independent chains so
// the SIMD is issue-bound, not latency-bound.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int ITERS = 4096;

__global__ __launch_bounds__(256) void k_mad64(uint64_t* out, uint32_t seed) {
  uint32_t a = seed + threadIdx.x, b = seed * 3u + blockIdx.x;
  uint64_t acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = (uint64_t)(a + k) << 7;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      uint64_t cy;
      asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[k]), "=s"(cy) : "v"(a), "v"(b));
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_addc(uint64_t* out, uint32_t seed) {
  uint32_t a = seed + threadIdx.x;
  uint32_t lo[8], hi[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { lo[k] = a + k; hi[k] = a ^ k; }
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      // one v_add_co_u32 + one v_addc_co_u32 per step: 2 VALU ops
      asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %2, vcc"
                   : "+v"(lo[k]), "+v"(hi[k]) : "v"(a) : "vcc");
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s ^= ((uint64_t)hi[k] << 32) | lo[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_mullo(uint64_t* out, uint32_t seed) {
  uint32_t a = seed + threadIdx.x;
  uint32_t x[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) x[k] = a + k;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[k]) : "v"(a));
  }
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s ^= x[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_add(uint64_t* out, uint32_t seed) {
  uint32_t a = seed + threadIdx.x;
  uint32_t x[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) x[k] = a + k;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[k]) : "v"(a));
  }
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s ^= x[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// one instruction template per kernel: 8 independent chains of 32-bit values
#define K32(NAME, ASM, ...)                                                               \
  __global__ __launch_bounds__(256) void NAME(uint64_t* out, uint32_t seed) {             \
    uint32_t a = seed + threadIdx.x, b = seed * 7u + 3u;                                  \
    uint32_t x[8];                                                                        \
    _Pragma("unroll") for (int k = 0; k < 8; ++k) x[k] = a + k;                          \
    for (int i = 0; i < ITERS; ++i) {                                                     \
      _Pragma("unroll") for (int k = 0; k < 8; ++k) asm volatile(ASM : "+v"(x[k]) : "v"(a), "v"(b) __VA_ARGS__); \
    }                                                                                     \
    uint64_t s = 0;                                                                       \
    _Pragma("unroll") for (int k = 0; k < 8; ++k) s ^= x[k];                             \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                       \
  }
K32(k_alignbit, "v_alignbit_b32 %0, %1, %0, 28")
K32(k_add3, "v_add3_u32 %0, %0, %1, %2")
K32(k_and, "v_and_b32 %0, %0, %1")
K32(k_cndmask, "v_cmp_lt_u32 vcc, %1, %2\n\tv_cndmask_b32 %0, %0, %1, vcc", : "vcc")
K32(k_dpp, "v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")
K32(k_lshl_add, "v_lshl_add_u32 %0, %0, 4, %1")
// 64-bit shift / shift-add on 8 independent 64-bit chains
__global__ __launch_bounds__(256) void k_shr64(uint64_t* out, uint32_t seed) {
  uint64_t x[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) x[k] = ((uint64_t)(seed + k) << 40) | threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) asm volatile("v_lshrrev_b64 %0, 1, %0" : "+v"(x[k]));
  }
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s ^= x[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_lshladd64(uint64_t* out, uint32_t seed) {
  uint64_t x[8], y = ((uint64_t)seed << 20) | threadIdx.x;
#pragma unroll
  for (int k = 0; k < 8; ++k) x[k] = ((uint64_t)(seed + k) << 30) | threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(x[k]) : "v"(y));
  }
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s ^= x[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
static double time_kernel(K kern, uint64_t* d, int blocks, int reps) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, 1u);   // warm-up launch
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, (uint32_t)r);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0; CHECK(hipEventElapsedTime(&ms, e0, e1));
  CHECK(hipEventDestroy(e0)); CHECK(hipEventDestroy(e1));
  return ms / reps;
}

// Each instruction is timed at three launch shapes -- one round of 32 waves per CU repeated 5
// times, and single launches of 8,192 and 16,384 blocks (tools/csqr_bench.hip's shape) -- and
// the JSON gives every rate and the best ("<instr>_Tops").  bench.py prices the integer-VALU
// roofline with these and takes as the v_mad_u64_u32 peak the larger of the best rate and the
// issue-model bound of 39.3 T/s (256 CU x 4 SIMD x 16 lanes/clk x 2.4 GHz for a 4-cycle op).
struct Shape { int blocks, reps; };

template <typename K>
static void report(const char* name, K kern, uint64_t* d, const Shape* shapes, int ns, double ops_per_lane) {
  double best = 0;
  printf(", \"%s_Tops_by_shape\": [", name);
  for (int i = 0; i < ns; ++i) {
    const double t = time_kernel(kern, d, shapes[i].blocks, shapes[i].reps);
    const double r = (double)shapes[i].blocks * 256.0 * ops_per_lane / (t * 1e-3) / 1e12;
    if (r > best) best = r;
    printf("%s{\"blocks\": %d, \"reps\": %d, \"Tops\": %.3f}", i ? ", " : "", shapes[i].blocks, shapes[i].reps, r);
  }
  printf("], \"%s_Tops\": %.3f", name, best);
}

int main() {
  hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  const Shape shapes[3] = {{cus * 8, 5}, {8192, 1}, {16384, 1}};
  const int max_blocks = 16384;
  uint64_t* d; CHECK(hipMalloc(&d, (size_t)max_blocks * 256 * 8));
  const double o = (double)ITERS * 8.0;   // instructions per lane
  printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d", p.gcnArchName, cus, p.clockRate);
  report("v_mad_u64_u32", k_mad64, d, shapes, 3, o);
  report("v_add_co+v_addc_co", k_addc, d, shapes, 3, 2 * o);
  report("v_mul_lo_u32", k_mullo, d, shapes, 3, o);
  report("v_add_u32", k_add, d, shapes, 3, o);
  report("v_alignbit_b32", k_alignbit, d, shapes, 3, o);
  report("v_add3_u32", k_add3, d, shapes, 3, o);
  report("v_and_b32", k_and, d, shapes, 3, o);
  report("v_cmp+v_cndmask", k_cndmask, d, shapes, 3, 2 * o);
  report("v_mov_b32_dpp", k_dpp, d, shapes, 3, o);
  report("v_lshl_add_u32", k_lshl_add, d, shapes, 3, o);
  report("v_lshrrev_b64", k_shr64, d, shapes, 3, o);
  report("v_lshl_add_u64", k_lshladd64, d, shapes, 3, o);
  printf("}\n");
  CHECK(hipFree(d));
  return 0;
}
