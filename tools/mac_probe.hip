// v_mad_u64_u32 issue rate against register banks, chain count and the carry-out SGPR, at two
// waves per SIMD (the verify kernels' occupancy).  Explicit registers (one asm block per step):
//   conflict-free: multiplicands in v2 (bank 2) and v3 (bank 3), accumulators in v[4k:4k+1]
//   (banks 0, 1); conflicting: multiplicands in v1 / v5 (banks 1, 1).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mac_probe.hip -o tools/mac_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int ITERS = 8192;
#define CLOB "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", \
  "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", \
  "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", \
  "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", \
  "v66", "v67", "v68", "v69", "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27", "s28", "s29", "s30", "s31", "s40", "s41", "s42", "s43"

#define M8(A, B, S0, S1, S2, S3, S4, S5, S6, S7) \
  "v_mad_u64_u32 v[4:5], " S0 ", " A ", " B ", v[4:5]\n\t" \
  "v_mad_u64_u32 v[8:9], " S1 ", " A ", " B ", v[8:9]\n\t" \
  "v_mad_u64_u32 v[12:13], " S2 ", " A ", " B ", v[12:13]\n\t" \
  "v_mad_u64_u32 v[16:17], " S3 ", " A ", " B ", v[16:17]\n\t" \
  "v_mad_u64_u32 v[20:21], " S4 ", " A ", " B ", v[20:21]\n\t" \
  "v_mad_u64_u32 v[24:25], " S5 ", " A ", " B ", v[24:25]\n\t" \
  "v_mad_u64_u32 v[28:29], " S6 ", " A ", " B ", v[28:29]\n\t" \
  "v_mad_u64_u32 v[32:33], " S7 ", " A ", " B ", v[32:33]\n\t"
#define M8B(A, B, S0) \
  "v_mad_u64_u32 v[36:37], " S0 ", " A ", " B ", v[36:37]\n\t" \
  "v_mad_u64_u32 v[40:41], " S0 ", " A ", " B ", v[40:41]\n\t" \
  "v_mad_u64_u32 v[44:45], " S0 ", " A ", " B ", v[44:45]\n\t" \
  "v_mad_u64_u32 v[48:49], " S0 ", " A ", " B ", v[48:49]\n\t" \
  "v_mad_u64_u32 v[52:53], " S0 ", " A ", " B ", v[52:53]\n\t" \
  "v_mad_u64_u32 v[56:57], " S0 ", " A ", " B ", v[56:57]\n\t" \
  "v_mad_u64_u32 v[60:61], " S0 ", " A ", " B ", v[60:61]\n\t" \
  "v_mad_u64_u32 v[64:65], " S0 ", " A ", " B ", v[64:65]\n\t"
#define SS "s[20:21]"

template <int V>
__global__ __launch_bounds__(256) void k_mac(uint64_t* out, uint32_t seed) {
  uint32_t r = 0;
  asm volatile("v_mov_b32 v1, %0\n\tv_mov_b32 v2, %0\n\tv_mov_b32 v3, %1\n\tv_mov_b32 v5, %1" : : "v"(seed + threadIdx.x), "v"(seed ^ blockIdx.x) : CLOB);
  for (int i = 0; i < ITERS; ++i) {
    if (V == 0) asm volatile(M8("v2", "v3", SS, SS, SS, SS, SS, SS, SS, SS) : : : CLOB);                 // conflict-free, 8 chains
    if (V == 1) asm volatile(M8("v1", "v5", SS, SS, SS, SS, SS, SS, SS, SS) : : : CLOB);                 // bank conflict (v1, v5, acc bank 1)
    if (V == 2) asm volatile(M8("v2", "v3", "s[20:21]", "s[22:23]", "s[24:25]", "s[26:27]", "s[28:29]", "s[30:31]", "s[40:41]", "s[42:43]") : : : CLOB);
    if (V == 3) asm volatile(M8("v2", "v3", SS, SS, SS, SS, SS, SS, SS, SS) M8B("v2", "v3", SS) : : : CLOB);   // 16 chains
    if (V == 4) asm volatile("v_mad_u64_u32 v[4:5], s[20:21], v2, v3, v[4:5]\n\tv_mad_u64_u32 v[8:9], s[20:21], v2, v3, v[8:9]\n\t"
                             "v_mad_u64_u32 v[12:13], s[20:21], v2, v3, v[12:13]\n\tv_mad_u64_u32 v[16:17], s[20:21], v2, v3, v[16:17]\n\t"
                             "v_mad_u64_u32 v[4:5], s[20:21], v2, v3, v[4:5]\n\tv_mad_u64_u32 v[8:9], s[20:21], v2, v3, v[8:9]\n\t"
                             "v_mad_u64_u32 v[12:13], s[20:21], v2, v3, v[12:13]\n\tv_mad_u64_u32 v[16:17], s[20:21], v2, v3, v[16:17]" : : : CLOB);   // 4 chains
    if (V == 5) asm volatile("v_mad_u64_u32 v[4:5], s[20:21], v2, v3, v[4:5]\n\tv_mad_u64_u32 v[4:5], s[20:21], v2, v3, v[4:5]\n\t"
                             "v_mad_u64_u32 v[4:5], s[20:21], v2, v3, v[4:5]\n\tv_mad_u64_u32 v[4:5], s[20:21], v2, v3, v[4:5]\n\t"
                             "v_mad_u64_u32 v[4:5], s[20:21], v2, v3, v[4:5]\n\tv_mad_u64_u32 v[4:5], s[20:21], v2, v3, v[4:5]\n\t"
                             "v_mad_u64_u32 v[4:5], s[20:21], v2, v3, v[4:5]\n\tv_mad_u64_u32 v[4:5], s[20:21], v2, v3, v[4:5]" : : : CLOB);   // 1 chain
  }
  asm volatile("v_xor_b32 %0, v4, v8\n\tv_xor_b32 %0, %0, v12\n\tv_xor_b32 %0, %0, v36" : "=v"(r) : : CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int V>
static void run(const char* name, uint64_t* out, int blocks, int threads, int macs_per_iter) {
  hipLaunchKernelGGL((k_mac<V>), dim3(blocks), dim3(threads), 0, 0, out, 7u);
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0, 0));
  hipLaunchKernelGGL((k_mac<V>), dim3(blocks), dim3(threads), 0, 0, out, 9u);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double macs = (double)blocks * threads * ITERS * macs_per_iter;
  const double waves = (double)blocks * ((threads + 63) / 64);
  printf("{\"variant\": \"%s\", \"blocks\": %d, \"threads\": %d, \"ms\": %.4f, \"mad_Tops\": %.3f, \"frac_of_39.32\": %.3f, \"us_per_1k_mac_per_wave\": %.3f}\n", name, blocks, threads, ms,
         macs / (ms * 1e-3) / 1e12, macs / (ms * 1e-3) / 1e12 / 39.32, 1e3 * ms / (ITERS * (double)macs_per_iter) * 1e3 * (waves > 0 ? 1.0 : 0.0));
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 512;
  const int threads = argc > 2 ? atoi(argv[2]) : 256;
  const int only = argc > 3 ? atoi(argv[3]) : 0;
  uint64_t* out;
  CHECK(hipMalloc(&out, (size_t)blocks * 256 * 8));
  run<0>("8 chains, conflict-free, one carry SGPR", out, blocks, threads, 8);
  if (only) return 0;
  run<1>("8 chains, bank conflicts", out, blocks, threads, 8);
  run<2>("8 chains, conflict-free, eight carry SGPRs", out, blocks, threads, 8);
  run<3>("16 chains, conflict-free", out, blocks, threads, 16);
  run<4>("4 chains, conflict-free", out, blocks, threads, 8);
  run<5>("1 chain", out, blocks, threads, 8);
  return 0;
}
