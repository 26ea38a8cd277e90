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
#include <algorithm>

__shared__ unsigned long long fe_acc[2][8];
__shared__ unsigned long long fe_last[2];
#ifndef FE_PRIO_TOGGLE
#define FE_PRIO_TOGGLE 0
#endif
__shared__ unsigned fe_cnt[2];
__device__ __forceinline__ void fe_mark(int k) {
#if FE_PRIO_TOGGLE
  // alternate the issue priority of the SIMD's two waves at every mark (wave slot parity)
  {
    const unsigned slot = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4) & 1u;
    const int w = threadIdx.x >> 6;
    const unsigned c = fe_cnt[w] + 1;
    if ((threadIdx.x & 63) == 0) fe_cnt[w] = c;
    // scalar (uniform) branch: s_setprio ignores exec, so a divergent if would run both
    const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)((c + slot) & 1u));
    if (hi) __builtin_amdgcn_s_setprio(2); else __builtin_amdgcn_s_setprio(0);
  }
#endif
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
    fe_cnt[w] = 0;
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
    unsigned long long* p = prof + ((size_t)blockIdx.x * 2 + w) * 14;
    for (int k = 0; k < 8; ++k) p[k] = fe_acc[w][k];
    p[8] = t1 - t0;
    p[9] = r1 - r0;   // s_memrealtime: constant 100 MHz
    p[10] = r0;
    p[11] = r1;
    p[12] = (unsigned long long)__builtin_amdgcn_s_getreg((3 << 11) | 20);   // HW_REG_XCC_ID[3:0]
    p[13] = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
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
  CHECK(hipMalloc(&dprof, blocks * 2 * 14 * 8));
  CHECK(hipMemcpy(din, h.data(), words * 4, hipMemcpyHostToDevice));
  CHECK(hipMemset(dprof, 0, blocks * 2 * 14 * 8));
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
  std::vector<unsigned long long> p(blocks * 2 * 14);
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
      const unsigned long long* q = &p[(b * 2 + w) * 14];
      if (q[8] == 0) continue;
      ++waves;
      for (int k = 0; k < 10; ++k) sum[k] += (double)q[k];
    }
  printf("{\"items\": %zu, \"kernel_ms\": %.4f, \"waves\": %zu, \"phases_cycles_per_wave\": {", items, ms, waves);
  for (int k = 0; k < 9; ++k) printf("%s\"%s\": %.0f", k ? ", " : "", names[k], sum[k] / (waves ? waves : 1));
  // wave start / end spread (s_memrealtime, 10 ns ticks): late starts mean a second round of waves
  unsigned long long smin = ~0ull, smax = 0, emin = ~0ull, emax = 0;
  std::vector<unsigned long long> starts;
  for (size_t b = 0; b < blocks; ++b)
    for (int w = 0; w < 2; ++w) {
      const unsigned long long* q = &p[(b * 2 + w) * 14];
      if (q[8] == 0) continue;
      smin = std::min(smin, q[10]); smax = std::max(smax, q[10]);
      emin = std::min(emin, q[11]); emax = std::max(emax, q[11]);
      starts.push_back(q[10]);
    }
  // per XCD: waves, mean FE cycles, mean and max end (ms after the first start)
  double xw[16] = {0}, xc[16] = {0}, xe[16] = {0}, xm[16] = {0};
  for (size_t b = 0; b < blocks; ++b)
    for (int w = 0; w < 2; ++w) {
      const unsigned long long* q = &p[(b * 2 + w) * 14];
      if (q[8] == 0) continue;
      const int x = (int)(q[12] & 15);
      const double e = (q[11] - smin) * 1e-5;
      xw[x] += 1; xc[x] += (double)q[8]; xe[x] += e; xm[x] = std::max(xm[x], e);
    }
  fprintf(stderr, "xcd waves mean_fe_Mcycles mean_end_ms max_end_ms\n");
  for (int x = 0; x < 16; ++x)
    if (xw[x] > 0) fprintf(stderr, "%d %.0f %.2f %.3f %.3f\n", x, xw[x], xc[x] / xw[x] / 1e6, xe[x] / xw[x], xm[x]);
  // per SIMD (XCC, SE, CU, SIMD from HW_ID): the two waves' end times
  {
    std::vector<std::pair<unsigned long long, std::pair<unsigned long long, int>>> v;   // (simd key, (end, slot))
    for (size_t b = 0; b < blocks; ++b)
      for (int w = 0; w < 2; ++w) {
        const unsigned long long* q = &p[(b * 2 + w) * 14];
        if (q[8] == 0) continue;
        const unsigned long long hw = q[13];
        const unsigned long long key = (q[12] << 32) | (hw & 0x6F30);   // SE 14:13, SH 12, CU 11:8, SIMD 5:4
        v.push_back({key, {q[11], (int)(hw & 15)}});
      }
    std::sort(v.begin(), v.end());
    double early = 0, late2 = 0; size_t pairs = 0, lone = 0, more = 0, older_first = 0;
    for (size_t i = 0; i < v.size();) {
      size_t j = i;
      while (j < v.size() && v[j].first == v[i].first) ++j;
      if (j - i == 2) {
        const auto& a = v[i].second; const auto& c = v[i + 1].second;
        const double ea = (a.first - smin) * 1e-5, ec = (c.first - smin) * 1e-5;
        early += std::min(ea, ec); late2 += std::max(ea, ec); ++pairs;
        older_first += ((ea < ec) == (a.second < c.second)) ? 1 : 0;
        if (pairs <= 4) fprintf(stderr, "pair slots %d %d ends %.3f %.3f\n", a.second, c.second, ea, ec);
      } else if (j - i == 1) ++lone; else ++more;
      i = j;
    }
    fprintf(stderr, "simds with 2 waves %zu, 1 wave %zu, >2 %zu; mean early end %.3f ms, mean late end %.3f ms; "
            "lower slot finishes first in %zu\n", pairs, lone, more, pairs ? early / pairs : 0, pairs ? late2 / pairs : 0,
            older_first);
  }
  size_t late = 0;
  for (auto x : starts) late += (x - smin) > 50000 ? 1 : 0;   // started > 0.5 ms after the first wave
  printf("}, \"s_memtime_ghz\": %.3f, \"start_spread_ms\": %.3f, \"end_spread_ms\": %.3f, "
         "\"first_start_to_last_end_ms\": %.3f, \"waves_started_late\": %zu}\n",
         sum[9] > 0 ? sum[8] / (sum[9] * 10.0) : 0.0, (smax - smin) * 1e-5, (emax - emin) * 1e-5, (emax - smin) * 1e-5, late);
  return 0;
}
