// gfx950 kernels of the BLS12-381 engine.  G1 work runs one item per lane; all
// G2 / Fp12 work runs one item per adjacent lane pair (bls381_pair.hpp).  Every
// intermediate lives in HBM in structure-of-arrays, limb-major layout so that
// each limb load/store of a wavefront is one contiguous 256-byte access
// (DESIGN.md "Data layout in HBM"):
//   one-lane items:  limb k of Fp component c of item i at base[(c*14 + k) * n + i]
//   lane-pair items: limb k of Fp2 component c of item i, coefficient p, at
//                    base[(c*14 + k) * 2n + 2i + p]   (lane index 2i + p)
#pragma once
#include "bls381_pair.hpp"
#include "bls381_quad.hpp"
#include "bls381_ssz.hpp"

namespace bls381 {

// ST_NOSUB: decodes, but is not in G2 (randomized batching routes it to the per-item path)
enum : uint8_t { ST_OK = 0, ST_INF = 1, ST_BAD = 2, ST_NOSUB = 3 };

// Subgroup policy (include/bls381.h BLS381_POLICY_*; DESIGN.md "Subgroup policy").
//   PYECC:  py_ecc 1.7.0's checks only -- on-curve decoding, no subgroup test; the
//           reduced pairing then ignores torsion of order prime to r in a pubkey,
//           and a degenerate Miller loop (miller_loop_n) yields verdict False.
//   STRICT: every pubkey and signature must lie in G1 / G2
//           (specs/bls_signature.md:135-136,143-144).  Aggregates never check.
// The kernels take the policy as a flags word `check` / `check_subgroup`: bits 0-1 the
// subgroup mode (0 none; 1 a point outside the subgroup is ST_BAD; 2 it is ST_NOSUB),
// bit 2 (CHK_LAX) the codec -- set: py_ecc 1.7.0's lax decoder (the PYECC policy), clear:
// the spec's strict one (bls381_curve.hpp "Codecs").
enum : int { CHK_SUB_MASK = 3, CHK_LAX = 4 };
// Registry entry status bit: the key decodes (lax) but is not a canonical encoding, so
// the strict codec rejects it (k_reg_decode, agg_accumulate).
constexpr uint8_t ST_NONCANON = 0x80;

constexpr int KBLOCK = 128;   // lanes per workgroup for the per-item kernels
// minimum waves per SIMD requested from the register allocator for the heavy
// per-item kernels (1 = up to 512 VGPR+AGPR per lane, 2 = up to 256).  Two:
// one wave alone issues a VALU op every 4 cycles, a second fills the other 2.
#ifndef BLS_WAVES_PER_EU
#define BLS_WAVES_PER_EU 2
#endif
#ifndef BLS_ML_WAVES_PER_EU
#define BLS_ML_WAVES_PER_EU BLS_WAVES_PER_EU
#endif
#ifndef BLS_FE_WAVES_PER_EU
#define BLS_FE_WAVES_PER_EU BLS_WAVES_PER_EU
#endif
// the fused C2 prologue (k_prologue_1<0>): 3 waves per SIMD (168 VGPRs; scratch 5,040 -> 5,808 B/lane)
// measured 2.68 ms against 2.90 ms at 2 (profiles/ab_r06h_prologue_waves.txt, same box, alternating):
// its one-lane code is latency-bound, and a third wave hides more than the larger frame costs.
// The randomized prologue (k_prologue_1<1>) does not fit 3 and stays at BLS_WAVES_PER_EU.
#ifndef BLS_PROLOGUE_WAVES_PER_EU
#define BLS_PROLOGUE_WAVES_PER_EU 3
#endif
// aggregation kernels (k_agg_chunks, k_agg_lanes): measurement knob
#ifndef BLS_AGG_WAVES_PER_EU
#define BLS_AGG_WAVES_PER_EU BLS_WAVES_PER_EU
#endif

// ------------------------------------------------------------ SoA access --
// Every SoA buffer is device global memory: the accesses go through global-address-space
// pointers, so they compile to global_load / global_store even inside a non-inlined function
// whose pointer parameter the compiler cannot trace to a kernel argument (a generic pointer
// would make them flat accesses, which also count against lgkmcnt and wait with LDS traffic).
typedef __attribute__((address_space(1))) const uint32_t g_cu32;
typedef __attribute__((address_space(1))) uint32_t g_u32;
__device__ __forceinline__ fp_t soa_ld(const uint32_t* __restrict__ p, size_t n, size_t i, int c) {
  g_cu32* g = (g_cu32*)p;
  fp_t r;
#pragma unroll
  for (int k = 0; k < FP_LIMBS; ++k) r.w[k] = g[(size_t)(c * FP_LIMBS + k) * n + i];
  return r;
}
__device__ __forceinline__ void soa_st(uint32_t* __restrict__ p, size_t n, size_t i, int c, const fp_t& a) {
  g_u32* g = (g_u32*)p;
#pragma unroll
  for (int k = 0; k < FP_LIMBS; ++k) g[(size_t)(c * FP_LIMBS + k) * n + i] = a.w[k];
}
__device__ __forceinline__ aff_t<fp_t> soa_ld_g1(const uint32_t* p, size_t n, size_t i) {
  aff_t<fp_t> a; a.x = soa_ld(p, n, i, 0); a.y = soa_ld(p, n, i, 1); return a;
}
__device__ __forceinline__ void soa_st_g1(uint32_t* p, size_t n, size_t i, const aff_t<fp_t>& a) {
  soa_st(p, n, i, 0, a.x); soa_st(p, n, i, 1, a.y);
}
// lane-pair items: n items, item i, Fp2 component c (this lane's coefficient)
__device__ __forceinline__ fp2p_t soa_ld2p(const uint32_t* p, size_t n, size_t i, int c) {
  return pr_make(soa_ld(p, 2 * n, 2 * i + (pr_odd() ? 1 : 0), c));
}
__device__ __forceinline__ void soa_st2p(uint32_t* p, size_t n, size_t i, int c, const fp2p_t& a) {
  soa_st(p, 2 * n, 2 * i + (pr_odd() ? 1 : 0), c, a.v);
}
__device__ __forceinline__ aff_t<fp2p_t> soa_ld_g2(const uint32_t* p, size_t n, size_t i) {
  aff_t<fp2p_t> a; a.x = soa_ld2p(p, n, i, 0); a.y = soa_ld2p(p, n, i, 1); return a;
}
__device__ __forceinline__ void soa_st_g2(uint32_t* p, size_t n, size_t i, const aff_t<fp2p_t>& a) {
  soa_st2p(p, n, i, 0, a.x); soa_st2p(p, n, i, 1, a.y);
}
using fp12p_t = fp12_g<fp2p_t>;
__device__ __forceinline__ fp12p_t soa_ld12(const uint32_t* p, size_t n, size_t i) {
  fp12p_t f;
  f.c0.c0 = soa_ld2p(p, n, i, 0); f.c0.c1 = soa_ld2p(p, n, i, 1); f.c0.c2 = soa_ld2p(p, n, i, 2);
  f.c1.c0 = soa_ld2p(p, n, i, 3); f.c1.c1 = soa_ld2p(p, n, i, 4); f.c1.c2 = soa_ld2p(p, n, i, 5);
  return f;
}
__device__ __forceinline__ void soa_st12(uint32_t* p, size_t n, size_t i, const fp12p_t& f) {
  soa_st2p(p, n, i, 0, f.c0.c0); soa_st2p(p, n, i, 1, f.c0.c1); soa_st2p(p, n, i, 2, f.c0.c2);
  soa_st2p(p, n, i, 3, f.c1.c0); soa_st2p(p, n, i, 4, f.c1.c1); soa_st2p(p, n, i, 5, f.c1.c2);
}
template <class F> struct soa_jac;
template <> struct soa_jac<fp_t> {
  static constexpr int NC = 3;
  __device__ static jac_t<fp_t> ld(const uint32_t* p, size_t n, size_t i) {
    jac_t<fp_t> r; r.x = soa_ld(p, n, i, 0); r.y = soa_ld(p, n, i, 1); r.z = soa_ld(p, n, i, 2); return r;
  }
  __device__ static void st(uint32_t* p, size_t n, size_t i, const jac_t<fp_t>& a) {
    soa_st(p, n, i, 0, a.x); soa_st(p, n, i, 1, a.y); soa_st(p, n, i, 2, a.z);
  }
};
template <> struct soa_jac<fp2p_t> {
  static constexpr int NC = 6;   // words: 3 Fp2 x 2 lanes
  __device__ static jac_t<fp2p_t> ld(const uint32_t* p, size_t n, size_t i) {
    jac_t<fp2p_t> r; r.x = soa_ld2p(p, n, i, 0); r.y = soa_ld2p(p, n, i, 1); r.z = soa_ld2p(p, n, i, 2); return r;
  }
  __device__ static void st(uint32_t* p, size_t n, size_t i, const jac_t<fp2p_t>& a) {
    soa_st2p(p, n, i, 0, a.x); soa_st2p(p, n, i, 1, a.y); soa_st2p(p, n, i, 2, a.z);
  }
};

// The latency kernels' lane assignment: units (items or pair tasks) of LPI lanes each.  A wave that
// holds at least one unit keeps all 64 lanes active -- lanes past the last unit recompute it with
// their stores masked (`live` false) -- and a wave with no unit exits.  Partially filled waves of these
// spill-heavy kernels ran erratically slower (r05, HISTORY.md round 5: the quad FE took 2.86-3.87 ms
// with 8 of 64 lanes in use and 2.87-2.91 ms with all 64; 1-item calls 9.3-9.5 against 8.4 ms).
template <int LPI>
__device__ __forceinline__ bool lat_unit(size_t n_units, size_t& u, bool& live) {
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (((g & ~(size_t)63) / LPI) >= n_units) return false;   // the wave's first unit
  const size_t raw = g / LPI;
  live = raw < n_units;
  u = live ? raw : n_units - 1;
  return true;
}

__device__ __forceinline__ void ld_bytes(uint8_t* dst, const uint8_t* __restrict__ src, int len) {
  for (int k = 0; k < len; ++k) dst[k] = src[k];
}

// lanes per item: 1 for G1 (fp_t), 2 for G2 (fp2p_t)
template <class F> struct lanes_per;
template <> struct lanes_per<fp_t> { static constexpr int N = 1; };
template <> struct lanes_per<fp2p_t> { static constexpr int N = 2; };

// grid helper for kernels: item index of this lane (pair kernels: lane / 2)
template <int LPI>
__device__ __forceinline__ size_t item_index() {
  return ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / LPI;
}

// --------------------------------------------------------- decode kernels --
// pubkeys -> affine G1 (SoA 2 Fp) + status; optional subgroup check
__device__ __forceinline__ void dev_decode_g1(size_t i, size_t n, const uint8_t* __restrict__ pks,
                                              uint32_t* __restrict__ out, uint8_t* __restrict__ st,
                                              int check_subgroup) {
  if (i >= n) return;
  uint8_t b[48];
  ld_bytes(b, pks + 48 * i, 48);
  aff_t<fp_t> a;
  int s = g1_decompress(a, b, (check_subgroup & CHK_LAX) != 0);
  if (s == PT_OK && (check_subgroup & CHK_SUB_MASK) && !g1_in_subgroup(a)) s = PT_BAD;
  st[i] = (uint8_t)s;
  if (s == PT_OK) soa_st_g1(out, n, i, a);
}
__global__ void __launch_bounds__(KBLOCK, BLS_WAVES_PER_EU) k_decode_g1(size_t n, const uint8_t* __restrict__ pks,
                                                     uint32_t* __restrict__ out, uint8_t* __restrict__ st,
                                                     int check_subgroup) {
  dev_decode_g1(item_index<1>(), n, pks, out, st, check_subgroup);
}

// signatures -> affine G2 (pair SoA, 2 Fp2) + status; check_subgroup: 0 none,
// 1 a point outside G2 is ST_BAD, 2 it is ST_NOSUB (and its point is stored)
__global__ void __launch_bounds__(KBLOCK, BLS_WAVES_PER_EU) k_decode_g2(size_t n, const uint8_t* __restrict__ sigs,
                                                     uint32_t* __restrict__ out, uint8_t* __restrict__ st,
                                                     int check_subgroup) {
  const size_t i = item_index<2>();
  if (i >= n) return;
  aff_t<fp2p_t> a;
  const int sub = check_subgroup & CHK_SUB_MASK;
  int s = g2_decompress(a, sigs + 96 * i, (check_subgroup & CHK_LAX) != 0);
  if (s == PT_OK && sub && !g2_in_subgroup(a)) s = sub == 2 ? ST_NOSUB : PT_BAD;
  if (!pr_odd()) st[i] = (uint8_t)s;
  if (s == PT_OK || s == ST_NOSUB) soa_st_g2(out, n, i, a);
}

// (msg, dom8) -> the verification hash BP(H0) = [3(x^2-1)] hash_to_G2(msg, dom)
// affine (pair SoA; g2_mul_bp: every verify kernel pairs it with the pubkey and
// the signature with -[3(x^2-1)] g1, G1_VGEN_*).  dom_stride 0 = one shared domain.
// koff != nullptr: the try-and-increment offsets k_hash_search found (no search here).
// prio != 0: raise the waves' issue priority (s_setprio) -- the latency path, where a few
// hash waves share SIMDs with a full-chip side launch (a grouped call's committee sums).
__global__ void __launch_bounds__(KBLOCK, BLS_WAVES_PER_EU) k_hash_g2(size_t n, const uint8_t* __restrict__ msgs, uint32_t mlen,
                                                   const uint8_t* __restrict__ doms, int dom_stride,
                                                   uint32_t* __restrict__ out, uint8_t* __restrict__ st,
                                                   const uint32_t* __restrict__ koff, int prio) {
  if (prio) __builtin_amdgcn_s_setprio(2);
  const size_t i = item_index<2>();
  if (i >= n) return;
  uint8_t dom[8];
  ld_bytes(dom, doms + (size_t)dom_stride * i, 8);
  aff_t<fp2p_t> c;
  hash_to_g2_candidate(c, msgs + (size_t)mlen * i, mlen, dom, koff ? (int)koff[i] : -1);
  aff_t<fp2p_t> h;
  const bool fin = jac_to_aff(h, g2_mul_bp(c));
  if (st && !pr_odd()) st[i] = fin ? ST_OK : ST_INF;
  if (fin) soa_st_g2(out, n, i, h);
}

// k_hash_g2 on lane quads (the latency form for small batches): the candidate on both halves as in
// the pair kernel, the cofactor map with its independent products split over the halves
// (g2_mul_bp_q, bls381_quad.hpp); the lo pair stores the point.
__global__ void __launch_bounds__(KBLOCK, BLS_WAVES_PER_EU) k_hash_g2_q(size_t n, const uint8_t* __restrict__ msgs, uint32_t mlen,
                                                     const uint8_t* __restrict__ doms, int dom_stride,
                                                     uint32_t* __restrict__ out, uint8_t* __restrict__ st,
                                                     const uint32_t* __restrict__ koff, int prio) {
  if (prio) __builtin_amdgcn_s_setprio(2);
  size_t i;
  bool live;
  if (!lat_unit<4>(n, i, live)) return;
  uint8_t dom[8];
  ld_bytes(dom, doms + (size_t)dom_stride * i, 8);
  aff_t<fp2p_t> c;
  hash_to_g2_candidate(c, msgs + (size_t)mlen * i, mlen, dom, koff ? (int)koff[i] : -1);
  aff_t<fp2p_t> h;
  const bool fin = jac_to_aff(h, g2_mul_bp_q(c));
  if (qd_hi() || !live) return;
  if (st && !pr_odd()) st[i] = fin ? ST_OK : ST_INF;
  if (fin) soa_st_g2(out, n, i, h);
}

// k_hash_g2_q with the cofactor map's doublings on lane octets (g2_mul_bp_o); quad A's lo pair stores
__global__ void __launch_bounds__(KBLOCK, BLS_WAVES_PER_EU) k_hash_g2_o(size_t n, const uint8_t* __restrict__ msgs, uint32_t mlen,
                                                     const uint8_t* __restrict__ doms, int dom_stride,
                                                     uint32_t* __restrict__ out, uint8_t* __restrict__ st,
                                                     const uint32_t* __restrict__ koff, int prio) {
  if (prio) __builtin_amdgcn_s_setprio(2);
  size_t i;
  bool live;
  if (!lat_unit<8>(n, i, live)) return;
  uint8_t dom[8];
  ld_bytes(dom, doms + (size_t)dom_stride * i, 8);
  aff_t<fp2p_t> c;
  hash_to_g2_candidate(c, msgs + (size_t)mlen * i, mlen, dom, koff ? (int)koff[i] : -1);
  aff_t<fp2p_t> h;
  const bool fin = jac_to_aff(h, g2_mul_bp_o(c));
  if (oc_b() || qd_hi() || !live) return;
  if (st && !pr_odd()) st[i] = fin ? ST_OK : ST_INF;
  if (fin) soa_st_g2(out, n, i, h);
}

// One-lane forms of decode_g2 and hash_to_g2 (fp2_t arithmetic on one lane per item:
// Karatsuba Fp2 products, and the Fp-only square roots computed once per item instead of
// on both lanes of a pair).  They write the lane-pair SoA layout the pair kernels read.
__device__ __forceinline__ void soa_st_g2_1(uint32_t* p, size_t n, size_t i, const aff_t<fp2_t>& a) {
  soa_st(p, 2 * n, 2 * i, 0, a.x.c0); soa_st(p, 2 * n, 2 * i + 1, 0, a.x.c1);
  soa_st(p, 2 * n, 2 * i, 1, a.y.c0); soa_st(p, 2 * n, 2 * i + 1, 1, a.y.c1);
}
__device__ __forceinline__ void dev_decode_g2_1(size_t i, size_t n, const uint8_t* __restrict__ sigs,
                                                uint32_t* __restrict__ out, uint8_t* __restrict__ st,
                                                int check_subgroup) {
  if (i >= n) return;
  aff_t<fp2_t> a;
  const int sub = check_subgroup & CHK_SUB_MASK;
  int s = g2_decompress(a, sigs + 96 * i, (check_subgroup & CHK_LAX) != 0);
  if (s == PT_OK && sub && !g2_in_subgroup(a)) s = sub == 2 ? ST_NOSUB : PT_BAD;
  st[i] = (uint8_t)s;
  if (s == PT_OK || s == ST_NOSUB) soa_st_g2_1(out, n, i, a);
}
__global__ void __launch_bounds__(KBLOCK, BLS_WAVES_PER_EU) k_decode_g2_1(size_t n, const uint8_t* __restrict__ sigs,
                                                       uint32_t* __restrict__ out, uint8_t* __restrict__ st,
                                                       int check_subgroup) {
  dev_decode_g2_1(item_index<1>(), n, sigs, out, st, check_subgroup);
}

// hash_to_G2 in two launches (the throughput path): the try-and-increment search and the
// square root on one lane per item (k_hash_cand_1: the root's two Fp exponentiations once
// per item, where the pair form computes them on both lanes), then the cofactor map BP and
// the affine conversion on lane pairs (k_hash_bp, in place over the candidate points).
//
// BLS_HASH_COMPACT=1: the try-and-increment search runs over the whole wave as a pool.
// A lane-per-item loop runs until the wave's slowest item has found its square (~7 rounds
// for 64 items at success probability 1/2, against a mean of 2).  Here, each round,
// the wave's unresolved items share all 64 lanes: with m items left, item t (the r-th
// unresolved) takes the lanes j = r, r + m, r + 2m, ... and tests its offsets k_t, k_t + 1,
// ... one per lane; its square is the lowest successful offset (the spec's candidate
// order), else k_t advances past all of them.  ~3 rounds per wave.
#ifndef BLS_HASH_COMPACT
#define BLS_HASH_COMPACT 1
#endif

// the r-th set bit (r < popcount(m)) of a 64-bit mask
__device__ __forceinline__ uint32_t nth_set_bit64(uint64_t m, uint32_t r) {
  uint32_t pos = 0;
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {
    const uint64_t lo = m & ((1ull << w) - 1ull);
    const uint32_t c = (uint32_t)__builtin_popcountll(lo);
    if (r >= c) { r -= c; m >>= w; pos += w; }
    else m = lo;
  }
  return pos;
}

__device__ __forceinline__ uint32_t lane_shfl(uint32_t v, uint32_t src) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v);
}

__device__ __forceinline__ void dev_hash_cand_1(size_t i, size_t n, const uint8_t* __restrict__ msgs, uint32_t mlen,
                                                const uint8_t* __restrict__ doms, int dom_stride,
                                                uint32_t* __restrict__ out) {
#if BLS_HASH_COMPACT
  // every lane of the wave takes part in the pooled search: no early return before it
  const bool valid = i < n;
  fp2_t x;
  if (valid) {
    uint8_t dom[8];
    ld_bytes(dom, doms + (size_t)dom_stride * i, 8);
    const uint8_t* msg = msgs + (size_t)mlen * i;
    uint32_t d[8];
    sha256_msg_dom_tag(d, msg, mlen, dom, 1);
    x.c0 = fp_to_mont(fp_plain_from_digest(d));
    sha256_msg_dom_tag(d, msg, mlen, dom, 2);
    x.c1 = fp_to_mont(fp_plain_from_digest(d));
  } else {
    x.c0 = fp_zero(); x.c1 = fp_zero();
  }
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t k = 0;            // this lane's item: next offset to test
  int32_t found = valid ? -1 : 0;
  while (true) {
    const uint64_t P = __builtin_amdgcn_ballot_w64(found < 0);
    if (P == 0) break;
    const uint32_t m = (uint32_t)__builtin_popcountll(P);
    const uint32_t t = nth_set_bit64(P, lane % m);        // the item this lane tests for
    const uint32_t off = lane_shfl(k, t) + lane / m;
    fp2_t y;
#pragma unroll
    for (int w = 0; w < FP_LIMBS; ++w) { y.c0.w[w] = lane_shfl(x.c0.w[w], t); y.c1.w[w] = lane_shfl(x.c1.w[w], t); }
    fp_t o = fp_zero();
    o.w[0] = off;
    y.c0 = fp_add(y.c0, fp_to_mont(o));
    const fp2_t rhs = fp2_add(fp2_mul(fp2_sqr(y), y), G2_B_M);
    const bool sq = fp_legendre(fp_add(fp_sqr(rhs.c0), fp_sqr(rhs.c1))) >= 0;
    const uint64_t B = __builtin_amdgcn_ballot_w64(sq);
    if (found < 0) {
      // this lane owns an unresolved item: its lanes are r, r + m, ... (r = its rank in P)
      const uint32_t r = (uint32_t)__builtin_popcountll(P & ((1ull << lane) - 1ull));
      int32_t first = -1;
      uint32_t cnt = 0;
      for (uint32_t j = r; j < 64; j += m, ++cnt)
        if (first < 0 && ((B >> j) & 1ull)) first = (int32_t)cnt;
      if (first >= 0) found = (int32_t)(k + (uint32_t)first);
      else k += cnt;
    }
  }
  if (!valid) return;
  {
    fp_t o = fp_zero();
    o.w[0] = (uint32_t)found;
    x.c0 = fp_add(x.c0, fp_to_mont(o));
  }
  const fp2_t rhs = fp2_add(fp2_mul(fp2_sqr(x), x), G2_B_M);
  fp2_t y;
  fp2_sqrt(y, rhs);   // succeeds: rhs is a square
  aff_t<fp2_t> c;
  c.x = x;
  c.y = g2_select_root(y);
  soa_st_g2_1(out, n, i, c);
#else
  if (i >= n) return;
  uint8_t dom[8];
  ld_bytes(dom, doms + (size_t)dom_stride * i, 8);
  aff_t<fp2_t> c;
  hash_to_g2_candidate(c, msgs + (size_t)mlen * i, mlen, dom);
  soa_st_g2_1(out, n, i, c);
#endif
}
__global__ void __launch_bounds__(KBLOCK, BLS_WAVES_PER_EU) k_hash_cand_1(size_t n, const uint8_t* __restrict__ msgs,
                                                       uint32_t mlen, const uint8_t* __restrict__ doms,
                                                       int dom_stride, uint32_t* __restrict__ out) {
  dev_hash_cand_1(item_index<1>(), n, msgs, mlen, doms, dom_stride, out);
}
__global__ void __launch_bounds__(KBLOCK, BLS_WAVES_PER_EU) k_hash_bp(size_t n, uint32_t* __restrict__ pts,
                                                   uint8_t* __restrict__ st) {
  const size_t i = item_index<2>();
  if (i >= n) return;
  const aff_t<fp2p_t> c = soa_ld_g2(pts, n, i);
  aff_t<fp2p_t> h;
  const bool fin = jac_to_aff(h, g2_mul_bp(c));
  if (st && !pr_odd()) st[i] = fin ? ST_OK : ST_INF;
  if (fin) soa_st_g2(pts, n, i, h);
}

// The latency form of the try-and-increment search (bls_signature.md:74-86): W lanes per
// message test candidates x + k, x + k + 1, ..., one Legendre symbol each (one-lane Fp2
// arithmetic), and the item's lowest square offset is taken from a ballot; with W = 16 a
// round fails with probability 2^-16, so a batch no longer waits for its slowest item's
// ~6 sequential rounds.  koff[i] = the offset of the first square (the spec's point).
template <int W>
__global__ void __launch_bounds__(KBLOCK) k_hash_search(size_t n, const uint8_t* __restrict__ msgs, uint32_t mlen,
                                                       const uint8_t* __restrict__ doms, int dom_stride,
                                                       uint32_t* __restrict__ koff) {
  static_assert(W == 16, "lane groups of 16 within a wave");
  const size_t i = item_index<W>();
  if (i >= n) return;
  const uint32_t j = threadIdx.x % W;
  uint8_t dom[8];
  ld_bytes(dom, doms + (size_t)dom_stride * i, 8);
  const uint8_t* msg = msgs + (size_t)mlen * i;
  uint32_t d[8];
  fp2_t x;
  sha256_msg_dom_tag(d, msg, mlen, dom, 1);
  x.c0 = fp_to_mont(fp_plain_from_digest(d));
  sha256_msg_dom_tag(d, msg, mlen, dom, 2);
  x.c1 = fp_to_mont(fp_plain_from_digest(d));
  for (uint32_t t = 0; t < j; ++t) x.c0 = fp_add(x.c0, FP_ONE_M);
  const fp_t step8 = fp_mul_small(FP_ONE_M, 8);
  const uint32_t sh = (threadIdx.x & 63u) & ~(uint32_t)(W - 1);
  for (uint32_t base = 0;; base += W) {
    const fp2_t rhs = fp2_add(fp2_mul(fp2_sqr(x), x), G2_B_M);
    const bool sq = fp_legendre(fp_add(fp_sqr(rhs.c0), fp_sqr(rhs.c1))) >= 0;
    const uint32_t m = (uint32_t)(__builtin_amdgcn_ballot_w64(sq) >> sh) & ((1u << W) - 1u);
    if (m) {
      if (j == 0) koff[i] = base + (uint32_t)__builtin_ctz(m);
      break;
    }
    x.c0 = fp_add(fp_add(x.c0, step8), step8);
  }
}

// --------------------------------------------------------- verify kernels --
// One bls_verify per lane pair: FE( ML(sig, -g1) * ML(H(m), pk) ) == 1, with the
// infinity short-circuit of py_ecc's pairing (a pair with an infinite point is 1).
// sig_check (STRICT policy): the signature's G2 membership is tested here, on the loop's
// final running point T = [|x|] sig (psi(sig) == -T), instead of by 64 more doublings in
// k_decode_g2; a signature outside G2 makes the verdict False either way.
__global__ void __launch_bounds__(KBLOCK, BLS_ML_WAVES_PER_EU) k_miller_verify(size_t n, const uint32_t* __restrict__ sig_aff,
                                                         const uint8_t* __restrict__ sig_st,
                                                         const uint32_t* __restrict__ pk_aff,
                                                         const uint8_t* __restrict__ pk_st,
                                                         const uint32_t* __restrict__ h_aff,
                                                         uint32_t* __restrict__ f_out, uint8_t* __restrict__ st_out,
                                                         int sig_check) {
  const size_t i = item_index<2>();
  if (i >= n) return;
  const bool lead = !pr_odd();
  const uint8_t ss = sig_st[i], ps = pk_st[i];
  if (ss == ST_BAD || ps == ST_BAD) { if (lead) st_out[i] = ST_BAD; return; }
  aff_t<fp2p_t> Q[2];
  g1_line_pre P[2];
  int np = 0;
  if (ss == ST_OK) {
    Q[np] = soa_ld_g2(sig_aff, n, i);
    aff_t<fp_t> ng; ng.x = G1_VGEN_X_M; ng.y = G1_VGEN_NEGY_M;
    P[np] = g1_prepare(ng);
    ++np;
  }
  if (ps == ST_OK) {
    Q[np] = soa_ld_g2(h_aff, n, i);
    P[np] = g1_prepare(soa_ld_g1(pk_aff, n, i));
    ++np;
  }
  fp12p_t f;
  bool degen = false;
  g2_proj<fp2p_t> T0;
  g2_proj<fp2p_t>* t0 = (sig_check && ss == ST_OK) ? &T0 : nullptr;
  if (np == 2) f = miller_loop_n<2>(Q, P, degen, t0);
  else if (np == 1) f = miller_loop_n<1>(Q, P, degen, t0);
  else f = fp12_one<fp2p_t>();
  bool bad = degen;   // a degenerate loop is py_ecc's zero pairing value: verdict False
  if (t0 && !degen) bad = !g2_psi_matches_neg(Q[0], T0);
  soa_st12(f_out, n, i, f);
  if (lead) st_out[i] = bad ? ST_BAD : ST_OK;
}

// ----------------------------------------- split Miller loop (throughput path) --
// The two-pair Miller loop of k_miller_verify in two kernels, so that neither holds the
// other's state (DESIGN.md §6 "Split Miller loop"):
//   k_ml_lines   one item per lane quad.  The lo half runs the running point of the pair
//                (sig, -[c]g1), the hi half that of (BP(H0), pk).  At each of the 68 Miller
//                steps the two halves' lines l (lo) and l' (hi) are multiplied on the quad
//                into L = l l' (6 Fp2 products, 3 per half) and L is written to HBM.
//   k_ml_accum   one item per lane pair: f <- f^2 L (doubling steps) or f L (addition
//                steps), f^2 and the sparse product f L (17 Fp2 products) with f in registers.
// Per doubling step this is 12 + 17 + 6 = 35 Fp2 products of f arithmetic instead of the
// 12 + 2 x 13 = 38 of miller_loop_n<2>, and the doubling kernel's live set is one running
// point per lane instead of f plus two points.  The product is the same field element.
// L layout (per item i of a chunk of cnt items, step j, Fp2 component c, this lane's
// coefficient p): limb k at L[((j * ML_LC + c) * 14 + k) * 2 cnt + 2 i + p], c = 0..2 the
// w^0 half (L00, L01, L02), c = 3..4 (L11, L12) -- L10 is always zero.
constexpr int ML_STEPS = 68;   // 63 doubling + 5 addition steps over |x|
constexpr int ML_LC = 5;
constexpr size_t ML_L_WORDS_PER_ITEM = (size_t)ML_STEPS * ML_LC * FP_LIMBS * 2;
enum : uint8_t { ML_ST_ONE = 4 };   // both pairs infinite: the item's Miller value is 1

// L = l l' of the lo half's line l = x (c0, c1, c2) and the hi half's l' (d0, d1, d2), on a quad:
//   t0 = c0 d0, t1 = c1 d1, s = c2 d2 (lo: t0, t1, (c0+c1)(d0+d1); hi: s, (c0+c2)(d0+d2), (c1+c2)(d1+d2))
//   lo: L00 = t0 + xi s, L01 = m01 - t0 - t1, L02 = t1;   hi: L11 = m02 - t0 - s, L12 = m12 - t1 - s
// (line_pair_product in bls381_pairing.hpp, with the products split over the halves).  Each
// lane's x is its own half's line; on return lo holds (L00, L01, L02), hi (L11, L12, -).
__device__ __forceinline__ void quad_line_pair(const fp2p_t& x0, const fp2p_t& x1, const fp2p_t& x2, fp2p_t& o0,
                                               fp2p_t& o1, fp2p_t& o2) {
  const bool hi = qd_hi();
  const fp2p_t y0 = qd_swap(x0), y1 = qd_swap(x1), y2 = qd_swap(x2);
  // products are symmetric in (c, d), so each half pairs its own line with the other's
  const fp2p_t p0 = fp2_mul(qd_sel(hi, x2, x0), qd_sel(hi, y2, y0));                   // t0 | s
  const fp2p_t p1 = fp2_mul(qd_sel(hi, fp2_add_lazy(x0, x2), x1), qd_sel(hi, fp2_add_lazy(y0, y2), y1));   // t1 | m02
  const fp2p_t p2 = fp2_mul(qd_sel(hi, fp2_add_lazy(x1, x2), fp2_add_lazy(x0, x1)),
                            qd_sel(hi, fp2_add_lazy(y1, y2), fp2_add_lazy(y0, y1)));   // m01 | m12
  const fp2p_t q0 = qd_swap(p0), q1 = qd_swap(p1);   // lo: s, m02;  hi: t0, t1
  // lo: L00 = p0 + xi q0, L01 = p2 - p0 - p1, L02 = p1;  hi: L11 = p1 - q0 - p0, L12 = p2 - q1 - p0
  o0 = qd_sel(hi, fp2_sub2(p1, q0, p0), fp2_add_mul_xi(p0, q0));
  o1 = fp2_sub2(p2, qd_sel(hi, q1, p0), qd_sel(hi, p0, p1));
  o2 = p1;
}

// BLS_ML_L_NT=1 (default): the line products are stored non-temporally -- they stream through HBM
// to k_ml_accum, and the lines kernel's own scratch keeps the caches.  r04e, one box, two runs each:
// k_ml_lines 6.69 / 6.70 -> 6.59 / 6.61 ms, k_ml_accum 7.29 / 7.30 -> 7.17 / 7.25 ms.
#ifndef BLS_ML_L_NT
#define BLS_ML_L_NT 1
#endif
__device__ __forceinline__ void soa_st_L(uint32_t* __restrict__ p, size_t n, size_t i, int c, const fp_t& a) {
#if BLS_ML_L_NT
#pragma unroll
  for (int k = 0; k < FP_LIMBS; ++k) __builtin_nontemporal_store(a.w[k], &((g_u32*)p)[(size_t)(c * FP_LIMBS + k) * n + i]);
#else
  soa_st(p, n, i, c, a);
#endif
}
__device__ __forceinline__ void ml_store_L(uint32_t* __restrict__ L, size_t cnt, size_t i, int j, bool hi,
                                           const fp2p_t& o0, const fp2p_t& o1, const fp2p_t& o2) {
  const size_t col = 2 * i + (pr_odd() ? 1 : 0);
  const int c = j * ML_LC + (hi ? 3 : 0);
  soa_st_L(L, 2 * cnt, col, c + 0, o0.v);
  soa_st_L(L, 2 * cnt, col, c + 1, o1.v);
  if (!hi) soa_st_L(L, 2 * cnt, col, c + 2, o2.v);
}

// the 68 steps of one half's running point, with the quad's line products written to L
__device__ __noinline__ g2_proj<fp2p_t> ml_lines_run(const aff_t<fp2p_t> Q, const g1_line_pre pre, bool active,
                                                    uint32_t* __restrict__ L, size_t cnt, size_t li) {
  const bool hi = qd_hi();
  const fp2p_t one = e2_one<fp2p_t>(), zero = e2_zero<fp2p_t>();
  g2_proj<fp2p_t> T;
  T.x = Q.x; T.y = Q.y; T.z = one;
  int j = 0;
  for (int b = 62; b >= 0; --b) {
    fp2p_t c0, c1, c2, o0, o1, o2;
    line_dbl(T, pre, c0, c1, c2);
    quad_line_pair(qd_sel(active, c0, one), qd_sel(active, c1, zero), qd_sel(active, c2, zero), o0, o1, o2);
    ml_store_L(L, cnt, li, j++, hi, o0, o1, o2);
    if ((BLS_X_ABS >> b) & 1) {
      line_add(T, Q, pre, c0, c1, c2);
      quad_line_pair(qd_sel(active, c0, one), qd_sel(active, c1, zero), qd_sel(active, c2, zero), o0, o1, o2);
      ml_store_L(L, cnt, li, j++, hi, o0, o1, o2);
    }
  }
  return T;
}

// BLS_ML_LINES_LDS=1: the doubling steps' line constants (-3 xp, 2 yp: 28 words per lane) live in
// LDS (14 KB per workgroup of 128 lanes), and Q and the addition steps' constants (-xp, yp) are
// re-read from their SoA rows at each of the five addition steps.  Without it the loop keeps
// all of them in the kernel's scratch frame (its live set is over the VGPR budget) and re-reads
// them through flat loads at every step: most of k_ml_lines' HBM traffic beyond L itself.
#ifndef BLS_ML_LINES_LDS
#define BLS_ML_LINES_LDS 1
#endif
typedef __attribute__((address_space(3))) uint32_t lds_u32;
// where a half's pair lives: Q (pair SoA of nq2 lanes, lane lp), P (G1 SoA of np items, item
// ip) or, with p == nullptr, -[c] g1 (the constant G1_VGEN)
struct ml_src {
  const uint32_t* q;
  size_t nq2, lp;
  const uint32_t* p;
  size_t np, ip;
};
__device__ __forceinline__ aff_t<fp2p_t> ml_src_q(const ml_src& s) {
  aff_t<fp2p_t> Q;
  Q.x = pr_make(soa_ld(s.q, s.nq2, s.lp, 0));
  Q.y = pr_make(soa_ld(s.q, s.nq2, s.lp, 1));
  return Q;
}
__device__ __forceinline__ aff_t<fp_t> ml_src_p(const ml_src& s) {
  aff_t<fp_t> P;
  if (s.p) {
    P = soa_ld_g1(s.p, s.np, s.ip);
  } else {
    P.x = G1_VGEN_X_M; P.y = G1_VGEN_NEGY_M;
  }
  return P;
}
// this lane's column of the LDS line constants: word k of -3 xp at col[k KBLOCK], of 2 yp at
// col[(14 + k) KBLOCK] (lane-major: conflict-free)
struct g1_dbl_lds { const lds_u32* col; };
__device__ __forceinline__ fp_t pre_n3x(const g1_dbl_lds& p) {
  fp_t r;
#pragma unroll
  for (int k = 0; k < FP_LIMBS; ++k) r.w[k] = p.col[k * KBLOCK];
  return r;
}
__device__ __forceinline__ fp_t pre_y2(const g1_dbl_lds& p) {
  fp_t r;
#pragma unroll
  for (int k = 0; k < FP_LIMBS; ++k) r.w[k] = p.col[(FP_LIMBS + k) * KBLOCK];
  return r;
}
constexpr int ML_LDS_WORDS = 2 * FP_LIMBS * KBLOCK;
__device__ __forceinline__ void ml_lds_put(lds_u32* col, const g1_line_pre& pre) {
#pragma unroll
  for (int k = 0; k < FP_LIMBS; ++k) {
    col[k * KBLOCK] = pre.n3x.w[k];
    col[(FP_LIMBS + k) * KBLOCK] = pre.y2.w[k];
  }
}
// src by value: the L stores cannot alias it (a by-reference src would be re-read from the
// caller's frame after every store)
// (the final running point is returned by value: no pointer into the caller's frame)
// bal: the launch is one round of two-wave slots (the host's choice, bls381_capi.hip): the
// steps alternate the priority by the clock (BLS_WAVE_BALANCE=2), else by step parity
__device__ __noinline__ g2_proj<fp2p_t> ml_lines_run_lds(const ml_src src, const lds_u32* col, bool active,
                                                        uint32_t* __restrict__ L, size_t cnt, size_t li,
                                                        int bal) {
  const bool hi = qd_hi();
  const fp2p_t one = e2_one<fp2p_t>(), zero = e2_zero<fp2p_t>();
  g2_proj<fp2p_t> T;
  {
    const aff_t<fp2p_t> Q = ml_src_q(src);
    T.x = Q.x; T.y = Q.y; T.z = one;
  }
  const g1_dbl_lds dp{col};
  int j = 0;
  for (int b = 62; b >= 0; --b) {
#if BLS_WAVE_BALANCE == 2
    if (bal) wave_prio(balance_clock());
    else wave_balance_lds((unsigned)b);
#else
    (void)bal;
    wave_balance_lds((unsigned)b);
#endif
    fp2p_t c0, c1, c2, o0, o1, o2;
    line_dbl(T, dp, c0, c1, c2);
    quad_line_pair(qd_sel(active, c0, one), qd_sel(active, c1, zero), qd_sel(active, c2, zero), o0, o1, o2);
    ml_store_L(L, cnt, li, j++, hi, o0, o1, o2);
    if ((BLS_X_ABS >> b) & 1) {
      const aff_t<fp2p_t> Q = ml_src_q(src);
      const aff_t<fp_t> P = ml_src_p(src);
      g1_line_pre pre;
      pre.nx = fp_neg(P.x);
      pre.y = P.y;
      pre.n3x = pre.nx;   // unused by line_add
      pre.y2 = P.y;
      line_add(T, Q, pre, c0, c1, c2);
      quad_line_pair(qd_sel(active, c0, one), qd_sel(active, c1, zero), qd_sel(active, c2, zero), o0, o1, o2);
      ml_store_L(L, cnt, li, j++, hi, o0, o1, o2);
    }
  }
  return T;
}

// items i0 .. i0 + cnt - 1 of the batch (SoA inputs of n items); L and st_out are chunk-local
__global__ void __launch_bounds__(KBLOCK, BLS_ML_WAVES_PER_EU) k_ml_lines(size_t n, size_t i0, size_t cnt,
                                                    const uint32_t* __restrict__ sig_aff,
                                                    const uint8_t* __restrict__ sig_st,
                                                    const uint32_t* __restrict__ pk_aff,
                                                    const uint8_t* __restrict__ pk_st,
                                                    const uint32_t* __restrict__ h_aff,
                                                    uint32_t* __restrict__ L, uint8_t* __restrict__ st_out,
                                                    int sig_check, size_t l0, size_t lcnt, int bal) {
  // this launch: items l0 .. l0 + lcnt - 1 of the chunk (L strided by the chunk's cnt)
  const size_t li = l0 + item_index<4>();
  if (li >= l0 + lcnt || li >= cnt) return;
  const size_t i = i0 + li;
  const bool hi = qd_hi();
  const bool lead = (threadIdx.x & 3u) == 0;
  const size_t lp = 2 * i + (pr_odd() ? 1 : 0);
  const uint8_t ss = sig_st[i], ps = pk_st[i];
  if (ss == ST_BAD || ps == ST_BAD) { if (lead) st_out[li] = ST_BAD; return; }
  const bool sig_ok = ss == ST_OK, pk_ok = ps == ST_OK;
  if (!sig_ok && !pk_ok) { if (lead) st_out[li] = ML_ST_ONE; return; }
  // an inactive half (infinite point) runs the other half's pair with its lines masked to 1
  const bool active = hi ? pk_ok : sig_ok;
  const bool use_pk = hi ? pk_ok : !sig_ok;
  const uint32_t* qsrc = use_pk ? h_aff : sig_aff;
  g2_proj<fp2p_t> T;
#if BLS_ML_LINES_LDS
  __shared__ uint32_t lds_pre[ML_LDS_WORDS];
  lds_u32* col = (lds_u32*)lds_pre + threadIdx.x;
  const ml_src src{qsrc, 2 * n, lp, use_pk ? pk_aff : nullptr, n, i};
  ml_lds_put(col, g1_prepare(ml_src_p(src)));   // each lane writes and reads only its own column
  T = ml_lines_run_lds(src, col, active, L, cnt, li, bal);
  const aff_t<fp2p_t> Q = ml_src_q(src);
#else
  aff_t<fp2p_t> Q;
  Q.x = pr_make(soa_ld(qsrc, 2 * n, lp, 0));
  Q.y = pr_make(soa_ld(qsrc, 2 * n, lp, 1));
  aff_t<fp_t> P;
  if (use_pk) {
    P = soa_ld_g1(pk_aff, n, i);
  } else {
    P.x = G1_VGEN_X_M; P.y = G1_VGEN_NEGY_M;
  }
  const g1_line_pre pre = g1_prepare(P);
  T = ml_lines_run(Q, pre, active, L, cnt, li);
#endif
  // py_ecc's zero pairing value for a degenerate loop; the strict policy's G2 test of the
  // signature on the lo half's final point (psi(sig) == -[|x|] sig)
  bool bad = active && fp2_is_zero(T.z);
  if (sig_check && !hi && sig_ok && !bad) bad = !g2_psi_matches_neg(Q, T);
  bad = !qd_all(!bad);
  if (lead) st_out[li] = bad ? ST_BAD : ST_OK;
}

__device__ __forceinline__ fp12p_t ml_load_L(const uint32_t* __restrict__ L, size_t cnt, size_t i, int j) {
  const size_t col = 2 * i + (pr_odd() ? 1 : 0);
  const int c = j * ML_LC;
  fp12p_t r;
  r.c0.c0 = pr_make(soa_ld(L, 2 * cnt, col, c + 0));
  r.c0.c1 = pr_make(soa_ld(L, 2 * cnt, col, c + 1));
  r.c0.c2 = pr_make(soa_ld(L, 2 * cnt, col, c + 2));
  r.c1.c0 = e2_zero<fp2p_t>();
  r.c1.c1 = pr_make(soa_ld(L, 2 * cnt, col, c + 3));
  r.c1.c2 = pr_make(soa_ld(L, 2 * cnt, col, c + 4));
  return r;
}

// BLS_ML_ACCUM_LDS=1: k_ml_accum stages each step's L (5 Fp per lane) in LDS -- each lane its
// own column, 35 KB per workgroup -- and reads every coefficient at its use, instead of holding
// all five (70 VGPRs) beside f through the step's 29 Fp2 products.
#ifndef BLS_ML_ACCUM_LDS
#define BLS_ML_ACCUM_LDS 0
#endif
constexpr int ML_ACC_LDS_WORDS = ML_LC * FP_LIMBS * KBLOCK;
// volatile: within one lane the compiler would otherwise forward the staged values from the
// registers that stored them (no other lane reads the column) and drop LDS altogether
__device__ __forceinline__ fp2p_t ml_lds_c(const lds_u32* col, int c) {
  const volatile lds_u32* v = col;
  fp_t r;
#pragma unroll
  for (int k = 0; k < FP_LIMBS; ++k) r.w[k] = v[(c * FP_LIMBS + k) * KBLOCK];
  return pr_make(r);
}
// step j's L from HBM into this lane's LDS column, one coefficient at a time
__device__ __forceinline__ void ml_stage_L(lds_u32* col, const uint32_t* __restrict__ L, size_t cnt, size_t i, int j) {
  const size_t lane = 2 * i + (pr_odd() ? 1 : 0);
#pragma unroll
  for (int c = 0; c < ML_LC; ++c) {
    const fp_t v = soa_ld(L, 2 * cnt, lane, j * ML_LC + c);
    volatile lds_u32* d = col;
#pragma unroll
    for (int k = 0; k < FP_LIMBS; ++k) d[(c * FP_LIMBS + k) * KBLOCK] = v.w[k];
  }
}
// fp12_mul_by_line_pair_inl (bls381_pairing.hpp) with L read from LDS at each use:
// L = (L00 + L01 v + L02 v^2) + (L11 v + L12 v^2) w, coefficients 0..4 of the column
__device__ __forceinline__ fp12p_t fp12_mul_by_line_pair_lds(const fp12p_t& f, const lds_u32* col) {
  const fp6p_t& a = f.c0;
  const fp6p_t& b = f.c1;
  fp6p_t aP;
  {
    const fp2p_t t0 = fp2_mul(a.c0, ml_lds_c(col, 0));
    const fp2p_t t1 = fp2_mul(a.c1, ml_lds_c(col, 1));
    const fp2p_t t2 = fp2_mul(a.c2, ml_lds_c(col, 2));
    aP.c0 = fp2_add_mul_xi(t0, fp2_sub2(fp2_mul(fp2_add_lazy(a.c1, a.c2),
                                                fp2_add_lazy(ml_lds_c(col, 1), ml_lds_c(col, 2))), t1, t2));
    aP.c1 = fp2_add_mul_xi(fp2_sub2(fp2_mul(fp2_add_lazy(a.c0, a.c1),
                                            fp2_add_lazy(ml_lds_c(col, 0), ml_lds_c(col, 1))), t0, t1), t2);
    aP.c2 = fp2_add(fp2_sub2(fp2_mul(fp2_add_lazy(a.c0, a.c2),
                                     fp2_add_lazy(ml_lds_c(col, 0), ml_lds_c(col, 2))), t0, t2), t1);
  }
  fp6p_t bQ;
  {
    const fp2p_t t1 = fp2_mul(b.c1, ml_lds_c(col, 3));
    const fp2p_t t2 = fp2_mul(b.c2, ml_lds_c(col, 4));
    bQ.c0 = fp2_mul_xi(fp2_sub2(fp2_mul(fp2_add_lazy(b.c1, b.c2), fp2_add_lazy(ml_lds_c(col, 3), ml_lds_c(col, 4))),
                                t1, t2));
    bQ.c1 = fp2_add_mul_xi(fp2_mul(b.c0, ml_lds_c(col, 3)), t2);
    bQ.c2 = fp2_add(fp2_mul(b.c0, ml_lds_c(col, 4)), t1);
  }
  fp6p_t pq;
  pq.c0 = ml_lds_c(col, 0);
  pq.c1 = fp2_add(ml_lds_c(col, 1), ml_lds_c(col, 3));
  pq.c2 = fp2_add(ml_lds_c(col, 2), ml_lds_c(col, 4));
  const fp6p_t m = fp6_mul_inl(fp6_add(a, b), pq);
  fp12p_t r;
  r.c0 = fp6_add_mul_by_v(aP, bQ);
  r.c1 = fp6_sub2(m, aP, bQ);
  return r;
}

// f = conj(prod_j L_j^(2^(later doublings))) for items i0 .. i0 + cnt - 1; writes f (SoA over n
// items, the layout k_final_exp_verdict reads) and the item status.  grp > 0 (randomized
// batches): item i's value goes to slot (i / grp) (grp + 1) + i % grp of n slots, so every
// group of grp values leaves a slot free after it (the signature-sum value of a sub-batch).
__global__ void __launch_bounds__(KBLOCK, BLS_ML_WAVES_PER_EU) k_ml_accum(size_t n, size_t i0, size_t cnt,
                                                    const uint32_t* __restrict__ L,
                                                    const uint8_t* __restrict__ st_in,
                                                    uint32_t* __restrict__ f_out, uint8_t* __restrict__ st_out,
                                                    size_t grp) {
  const size_t li = item_index<2>();
  if (li >= cnt) return;
  const size_t i = grp ? ((i0 + li) / grp) * (grp + 1) + (i0 + li) % grp : i0 + li;
  const bool lead = !pr_odd();
  const uint8_t s = st_in[li];
  if (s == ST_BAD) { if (lead) st_out[i] = ST_BAD; return; }
  fp12p_t f;
  if (s == ML_ST_ONE) {
    f = fp12_one<fp2p_t>();
  } else {
#if BLS_ML_ACCUM_LDS
    __shared__ uint32_t lds_L[ML_ACC_LDS_WORDS];
    lds_u32* col = (lds_u32*)lds_L + threadIdx.x;   // each lane writes and reads only its own column
    f = ml_load_L(L, cnt, li, 0);
    int j = 1;
    if ((BLS_X_ABS >> 62) & 1) {
      ml_stage_L(col, L, cnt, li, j++);
      f = fp12_mul_by_line_pair_lds(f, col);
    }
    for (int b = 61; b >= 0; --b) {
      ml_stage_L(col, L, cnt, li, j++);
      f = fp12_mul_by_line_pair_lds(fp12_sqr_inl(f), col);
      if ((BLS_X_ABS >> b) & 1) {
        ml_stage_L(col, L, cnt, li, j++);
        f = fp12_mul_by_line_pair_lds(f, col);
      }
    }
#else
    f = ml_load_L(L, cnt, li, 0);
    int j = 1;
    if ((BLS_X_ABS >> 62) & 1) f = fp12_mul_by_line_pair_inl(f, ml_load_L(L, cnt, li, j++));
    for (int b = 61; b >= 0; --b) {
      wave_balance((unsigned)b);
      f = fp12_mul_by_line_pair_inl(fp12_sqr_inl(f), ml_load_L(L, cnt, li, j++));
      if ((BLS_X_ABS >> b) & 1) f = fp12_mul_by_line_pair_inl(f, ml_load_L(L, cnt, li, j++));
    }
#endif
    f = fp12_conj(f);
  }
  soa_st12(f_out, n, i, f);
  if (lead) st_out[i] = ST_OK;
}

// k_ml_accum on lane quads (bls381_quad.hpp: lo holds f's Fp6 half c0, hi c1), for launches
// with too few accumulators to fill the chip on lane pairs (randomized sub-batches: two
// items per accumulator, so 2^16 items give 2^15 of them -- 1,024 pair waves, one per
// SIMD, against 2,048 quad waves).  Same L input, same output layout (pair SoA), same grp.
__device__ __noinline__ fq12_t ml_accum_q_run(const uint32_t* __restrict__ L, size_t cnt, size_t li) {
  const bool hi = qd_hi();
  const size_t col = 2 * li + (pr_odd() ? 1 : 0);
  auto load = [&](int j) {
    const int c = j * ML_LC;
    fq12_t r;
    r.h.c0 = hi ? e2_zero<fp2p_t>() : pr_make(soa_ld(L, 2 * cnt, col, c + 0));
    r.h.c1 = pr_make(soa_ld(L, 2 * cnt, col, c + (hi ? 3 : 1)));
    r.h.c2 = pr_make(soa_ld(L, 2 * cnt, col, c + (hi ? 4 : 2)));
    return r;
  };
  fq12_t f = load(0);
  int j = 1;
  if ((BLS_X_ABS >> 62) & 1) f = fq12_mul(f, load(j++));
  for (int b = 61; b >= 0; --b) {
    f = fq12_mul(fq12_sqr(f), load(j++));
    if ((BLS_X_ABS >> b) & 1) f = fq12_mul(f, load(j++));
  }
  return fq12_conj(f);
}

__global__ void __launch_bounds__(KBLOCK, BLS_ML_WAVES_PER_EU) k_ml_accum_q(size_t n, size_t i0, size_t cnt,
                                                      const uint32_t* __restrict__ L,
                                                      const uint8_t* __restrict__ st_in,
                                                      uint32_t* __restrict__ f_out, uint8_t* __restrict__ st_out,
                                                      size_t grp) {
  const size_t li = item_index<4>();
  if (li >= cnt) return;
  const size_t i = grp ? ((i0 + li) / grp) * (grp + 1) + (i0 + li) % grp : i0 + li;
  const bool lead = (threadIdx.x & 3u) == 0;
  const uint8_t s = st_in[li];
  if (s == ST_BAD) { if (lead) st_out[i] = ST_BAD; return; }
  // the quad's lanes: lo pair reads L's lane-pair slot li (both halves read slot li)
  const fq12_t f = (s == ML_ST_ONE) ? fq12_one() : ml_accum_q_run(L, cnt, li);
  const int p = pr_odd() ? 1 : 0;
  const int c0 = qd_hi() ? 3 : 0;
  soa_st(f_out, 2 * n, 2 * i + p, c0 + 0, f.h.c0.v);
  soa_st(f_out, 2 * n, 2 * i + p, c0 + 1, f.h.c1.v);
  soa_st(f_out, 2 * n, 2 * i + p, c0 + 2, f.h.c2.v);
  if (lead) st_out[i] = ST_OK;
}

// The same verify on a lane quad (bls381_quad.hpp): the lo half runs the pair
// (sig, -g1), the hi half (H(m), pk), side by side; a single finite pair runs on
// lo with the hi half idle.  f is stored in the layout of k_miller_verify (each
// half writes its three Fp2 components), so the final exponentiation is shared.
__global__ void __launch_bounds__(KBLOCK, BLS_ML_WAVES_PER_EU) k_miller_verify_q(size_t n, const uint32_t* __restrict__ sig_aff,
                                                           const uint8_t* __restrict__ sig_st,
                                                           const uint32_t* __restrict__ pk_aff,
                                                           const uint8_t* __restrict__ pk_st,
                                                           const uint32_t* __restrict__ h_aff,
                                                           uint32_t* __restrict__ f_out, uint8_t* __restrict__ st_out) {
  size_t i;
  bool live;
  if (!lat_unit<4>(n, i, live)) return;
  const bool hi = qd_hi();
  const bool lead = (threadIdx.x & 3u) == 0 && live;
  const size_t lp = 2 * i + (pr_odd() ? 1 : 0);   // this lane's coefficient slot of item i
  const uint8_t ss = sig_st[i], ps = pk_st[i];
  if (ss == ST_BAD || ps == ST_BAD) { if (lead) st_out[i] = ST_BAD; return; }
  const bool sig_ok = ss == ST_OK, pk_ok = ps == ST_OK;
  fq12_t f;
  bool degen = false;
  if (sig_ok || pk_ok) {
    // lo: the signature pair if finite, else the pubkey pair; hi: the pubkey pair when both are
    // finite, else an idle copy of lo's pair (valid operands, its lines masked to 1)
    const bool active = hi ? (sig_ok && pk_ok) : true;
    const bool use_pk = (hi && active) || !sig_ok;
    aff_t<fp2p_t> Q;
    aff_t<fp_t> P;
    const uint32_t* qsrc = use_pk ? h_aff : sig_aff;
    Q.x = pr_make(soa_ld(qsrc, 2 * n, lp, 0));
    Q.y = pr_make(soa_ld(qsrc, 2 * n, lp, 1));
    if (use_pk) {
      P = soa_ld_g1(pk_aff, n, i);
    } else {
      P.x = G1_VGEN_X_M; P.y = G1_VGEN_NEGY_M;
    }
    f = miller_loop_quad(Q, g1_prepare(P), active, degen);
  } else {
    f = fq12_one();
  }
  if (!live) return;
  const int c0 = hi ? 3 : 0;
  soa_st(f_out, 2 * n, lp, c0 + 0, f.h.c0.v);
  soa_st(f_out, 2 * n, lp, c0 + 1, f.h.c1.v);
  soa_st(f_out, 2 * n, lp, c0 + 2, f.h.c2.v);
  if (lead) st_out[i] = degen ? ST_BAD : ST_OK;
}

// The latency form of k_miller_verify: one quad per Miller pair (miller_loop_q1).
// Pair task t = 2i + k of item i runs on lanes 4t..4t+3: k = 0 the pair
// (sig, -[c]g1), k = 1 (BP(H0), pk).  Each task writes its own Fp12 (pair SoA over
// 2n values) and status; an inactive pair (infinite operand) writes f = 1.
// k_final_exp_verdict_q<2> multiplies the two.
__global__ void __launch_bounds__(KBLOCK, BLS_ML_WAVES_PER_EU) k_miller_verify_o(size_t n, const uint32_t* __restrict__ sig_aff,
                                                           const uint8_t* __restrict__ sig_st,
                                                           const uint32_t* __restrict__ pk_aff,
                                                           const uint8_t* __restrict__ pk_st,
                                                           const uint32_t* __restrict__ h_aff,
                                                           uint32_t* __restrict__ f_out, uint8_t* __restrict__ st_out) {
  size_t t;
  bool live;
  if (!lat_unit<4>(2 * n, t, live)) return;
  const size_t i = t >> 1;
  const bool hpair = (t & 1) != 0;
  const bool lead = (threadIdx.x & 3u) == 0 && live;
  const int p = pr_odd() ? 1 : 0;
  const uint8_t ss = sig_st[i], ps = pk_st[i];
  if (ss == ST_BAD || ps == ST_BAD) { if (lead) st_out[t] = ST_BAD; return; }
  fq12_t f;
  bool degen = false;
  if (hpair ? ps == ST_OK : ss == ST_OK) {
    const uint32_t* qsrc = hpair ? h_aff : sig_aff;
    aff_t<fp2p_t> Q;
    Q.x = pr_make(soa_ld(qsrc, 2 * n, 2 * i + p, 0));
    Q.y = pr_make(soa_ld(qsrc, 2 * n, 2 * i + p, 1));
    aff_t<fp_t> P;
    if (hpair) {
      P = soa_ld_g1(pk_aff, n, i);
    } else {
      P.x = G1_VGEN_X_M; P.y = G1_VGEN_NEGY_M;
    }
    f = miller_loop_q1(Q, g1_prepare(P), degen);
  } else {
    f = fq12_one();
  }
  if (!live) return;
  const size_t lp = 2 * t + p;
  const int c0 = qd_hi() ? 3 : 0;
  soa_st(f_out, 4 * n, lp, c0 + 0, f.h.c0.v);
  soa_st(f_out, 4 * n, lp, c0 + 1, f.h.c1.v);
  soa_st(f_out, 4 * n, lp, c0 + 2, f.h.c2.v);
  if (lead) st_out[t] = degen ? ST_BAD : ST_OK;
}

// k_miller_verify_o with one octet per Miller pair (miller_loop_o1_run, bls381_quad.hpp): pair task
// t = 2i + k of item i on lanes 8t..8t+7; quad A stores f in the layout k_miller_verify_o writes.
__global__ void __launch_bounds__(KBLOCK, BLS_ML_WAVES_PER_EU) k_miller_verify_oo(size_t n, const uint32_t* __restrict__ sig_aff,
                                                            const uint8_t* __restrict__ sig_st,
                                                            const uint32_t* __restrict__ pk_aff,
                                                            const uint8_t* __restrict__ pk_st,
                                                            const uint32_t* __restrict__ h_aff,
                                                            uint32_t* __restrict__ f_out, uint8_t* __restrict__ st_out) {
  size_t t;
  bool live;
  if (!lat_unit<8>(2 * n, t, live)) return;
  const size_t i = t >> 1;
  const bool hpair = (t & 1) != 0;
  const bool lead = (threadIdx.x & 7u) == 0 && live;
  const int p = pr_odd() ? 1 : 0;
  const uint8_t ss = sig_st[i], ps = pk_st[i];
  if (ss == ST_BAD || ps == ST_BAD) { if (lead) st_out[t] = ST_BAD; return; }
  fq12_t f;
  bool degen = false;
  if (hpair ? ps == ST_OK : ss == ST_OK) {
    const uint32_t* qsrc = hpair ? h_aff : sig_aff;
    aff_t<fp2p_t> Q;
    Q.x = pr_make(soa_ld(qsrc, 2 * n, 2 * i + p, 0));
    Q.y = pr_make(soa_ld(qsrc, 2 * n, 2 * i + p, 1));
    aff_t<fp_t> P;
    if (hpair) {
      P = soa_ld_g1(pk_aff, n, i);
    } else {
      P.x = G1_VGEN_X_M; P.y = G1_VGEN_NEGY_M;
    }
    const fq12_ml r = miller_loop_o1_run(Q, g1_prepare(P));
    f = r.f;
    degen = r.degenerate;
  } else {
    f = fq12_one();
  }
  if (!live || oc_b()) return;
  const size_t lp = 2 * t + p;
  const int c0 = qd_hi() ? 3 : 0;
  soa_st(f_out, 4 * n, lp, c0 + 0, f.h.c0.v);
  soa_st(f_out, 4 * n, lp, c0 + 1, f.h.c1.v);
  soa_st(f_out, 4 * n, lp, c0 + 2, f.h.c2.v);
  if (lead) st_out[t] = degen ? ST_BAD : ST_OK;
}

// The throughput final exponentiation (lane pairs).  It runs cyc_exp_x without its exact
// fallback (final_exp_check<.., 0>): the items of a wave that met a snapshot with g2 = 0 get
// verdict FE_REDO, and k_final_exp_redo, queued right behind it, recomputes exactly those with
// the fallback in its call tree.  Nothing reads the verdicts between the two launches.
constexpr uint8_t FE_REDO = 0xFF;
__global__ void __launch_bounds__(KBLOCK, BLS_FE_WAVES_PER_EU) k_final_exp_verdict(size_t n, const uint32_t* __restrict__ f_in,
                                                             const uint8_t* __restrict__ st,
                                                             uint8_t* __restrict__ verdict) {
  const size_t i = item_index<2>();
  if (i >= n) return;
  const bool lead = !pr_odd();
  if (st[i] != ST_OK) { if (lead) verdict[i] = 0; return; }
  const fp12p_t f = soa_ld12(f_in, n, i);
  const int v = final_exp_check<fp2p_t, 0>(f);
  if (lead) verdict[i] = v == 2 ? FE_REDO : (uint8_t)v;
}

// the exact pass over k_final_exp_verdict's FE_REDO items (a wave without one exits at once)
__global__ void __launch_bounds__(KBLOCK, BLS_FE_WAVES_PER_EU) k_final_exp_redo(size_t n, const uint32_t* __restrict__ f_in,
                                                          uint8_t* __restrict__ verdict) {
  const size_t i = item_index<2>();
  if (i >= n || verdict[i] != FE_REDO) return;
  const bool lead = !pr_odd();
  const fp12p_t f = soa_ld12(f_in, n, i);
  const int v = final_exp_check<fp2p_t, 1>(f);
  if (lead) verdict[i] = (uint8_t)v;
}

// The same verdict on a lane quad (final_exp_q: each half holds one Fp6 half of
// f and runs half of every Fp12 step): half the per-item latency, for batches
// that leave SIMDs idle.  Item i's f is the product of NF values NF i + k of the
// pair-SoA layout k_final_exp_verdict reads (NF = 2: the two Miller pairs of
// k_miller_verify_o); any value not ST_OK makes the verdict False.
template <int NF>
__global__ void __launch_bounds__(KBLOCK, BLS_FE_WAVES_PER_EU) k_final_exp_verdict_q(size_t n, const uint32_t* __restrict__ f_in,
                                                               const uint8_t* __restrict__ st,
                                                               uint8_t* __restrict__ verdict) {
  size_t i;
  bool live;
  if (!lat_unit<4>(n, i, live)) return;
  const bool lead = (threadIdx.x & 3u) == 0 && live;
  bool ok = true;
  for (int k = 0; k < NF; ++k) ok = ok && st[NF * i + k] == ST_OK;
  if (!ok) { if (lead) verdict[i] = 0; return; }
  const int p = pr_odd() ? 1 : 0;
  const int c0 = qd_hi() ? 3 : 0;
  const size_t nv = NF * n;
  auto load = [&](size_t v) {
    fq12_t g;
    g.h.c0 = pr_make(soa_ld(f_in, 2 * nv, 2 * v + p, c0 + 0));
    g.h.c1 = pr_make(soa_ld(f_in, 2 * nv, 2 * v + p, c0 + 1));
    g.h.c2 = pr_make(soa_ld(f_in, 2 * nv, 2 * v + p, c0 + 2));
    return g;
  };
  fq12_t f = load(NF * i);
  for (int k = 1; k < NF; ++k) f = fq12_mul(f, load(NF * i + k));
  const bool one = fq12_is_one(final_exp_q(f));
  if (lead) verdict[i] = one ? 1 : 0;
}

// k_final_exp_verdict_q on an octet with the Fp12 products split four ways (final_exp_oq):
// both quads hold f; quad A's lead lane writes the verdict
// SQ = 1: the compressed squarings on the octet too (final_exp_oo, BLS381_FE_OCT=3)
template <int NF, int SQ = 0>
__global__ void __launch_bounds__(KBLOCK, BLS_FE_WAVES_PER_EU) k_final_exp_verdict_oq(size_t n, const uint32_t* __restrict__ f_in,
                                                                const uint8_t* __restrict__ st,
                                                                uint8_t* __restrict__ verdict) {
  size_t i;
  bool live;
  if (!lat_unit<8>(n, i, live)) return;
  const bool lead = (threadIdx.x & 7u) == 0 && live;
  bool ok = true;
  for (int k = 0; k < NF; ++k) ok = ok && st[NF * i + k] == ST_OK;
  if (!ok) { if (lead) verdict[i] = 0; return; }
  const int p = pr_odd() ? 1 : 0;
  const int c0 = qd_hi() ? 3 : 0;
  const size_t nv = NF * n;
  auto load = [&](size_t v) {
    fq12_t g;
    g.h.c0 = pr_make(soa_ld(f_in, 2 * nv, 2 * v + p, c0 + 0));
    g.h.c1 = pr_make(soa_ld(f_in, 2 * nv, 2 * v + p, c0 + 1));
    g.h.c2 = pr_make(soa_ld(f_in, 2 * nv, 2 * v + p, c0 + 2));
    return g;
  };
  fq12_t f = load(NF * i);
  for (int k = 1; k < NF; ++k) f = fq12_mul_oct(f, load(NF * i + k));
  const bool one = fq12_is_one(SQ ? final_exp_oo(f) : final_exp_oq(f));
  if (lead) verdict[i] = one ? 1 : 0;
}


// ------------------------------------- randomized batch verification (opt-in) --
// Small-exponent batch test (SURVEY.md §7 "Verdict semantics under batching"):
// a sub-batch of items verifies when
//   prod_i e(H(m_i), [r_i] pk_i) * e(sum_i [r_i] sig_i, -g1) == 1
// with independent 64-bit r_i; one final exponentiation per sub-batch.  Only
// items whose signature lies in G2 enter a sub-batch (the pairing is linear in
// that argument only on G2); the others, and every item of a failing sub-batch,
// are verified one by one.
enum : uint8_t { RB_BAD = 0, RB_BATCH = 1, RB_SINGLE = 2 };

// The weight of item i is r_i = k0 + mu k1 (mod r) with mu = -x^2 and (k1, k0) the first
// 8 bytes of SHA-256(seed || i), i as 8 little-endian bytes (never both 0).  The 2^64
// pairs give 2^64 distinct weights (|k0 - k0'| < 2^32 < x^2), the small-exponent test's
// error bound.  mu acts through cheap endomorphisms, so [r_i] P is a joint 32-bit
// multiplication (jac_mul_2x32): on G1 sigma(x, y) = (beta x, y) = [-x^2] P (a torsion
// component of a py_ecc-policy pubkey is multiplied differently, but the reduced pairing
// is trivial on it, as in the per-item path); on G2 -psi^2(Q) = [-x^2] Q (batched
// signatures are in G2).
struct rb_weight { uint32_t k0, k1; };
__device__ __forceinline__ rb_weight rb_scalar(const uint8_t* seed32, uint64_t i) {
  uint8_t buf[40];
  for (int k = 0; k < 32; ++k) buf[k] = seed32[k];
  for (int k = 0; k < 8; ++k) buf[32 + k] = (uint8_t)(i >> (8 * k));
  uint32_t d[8];
  sha256(d, buf, 40);
  rb_weight w{d[1], d[0]};
  if ((w.k0 | w.k1) == 0) w.k0 = 1;
  return w;
}

// The randomized prologue (round 6), in the default path's shape: the one-lane roles -- decode +
// [r_i] pk_i (dev_rb_decode_g1), the codec-only signature decode and the hash's search + root -- in
// one launch (k_prologue_1<1>), then the pair launches k_rb_g2_test and k_hash_bp.
// dev_rb_decode_g1: one lane per item; the pubkey decoded under the call's codec and subgroup mode
// (as k_decode_g1), and for a finite key R1 = [r_i] pk_i affine (status OK / INF).  The class waits
// for the signature's G2 test (k_rb_g2_test).
__device__ __forceinline__ void dev_rb_decode_g1(size_t i, size_t n, const uint8_t* __restrict__ pks,
                                                 const uint8_t* __restrict__ seed32,
                                                 uint32_t* __restrict__ pk_aff, uint8_t* __restrict__ pk_st,
                                                 uint32_t* __restrict__ r1_aff, uint8_t* __restrict__ r1_st,
                                                 int check_subgroup) {
  if (i >= n) return;
  uint8_t b[48];
  ld_bytes(b, pks + 48 * i, 48);
  aff_t<fp_t> p;
  int s = g1_decompress(p, b, (check_subgroup & CHK_LAX) != 0);
  if (s == PT_OK && (check_subgroup & CHK_SUB_MASK) && !g1_in_subgroup(p)) s = PT_BAD;
  pk_st[i] = (uint8_t)s;
  uint8_t st = ST_INF;
  if (s == PT_OK) {
    soa_st_g1(pk_aff, n, i, p);
    aff_t<fp_t> sp;                       // sigma(p) = [-x^2] p
    sp.x = fp_mul(G1_BETA_M, p.x);
    sp.y = p.y;
    const rb_weight w = rb_scalar(seed32, i);
    aff_t<fp_t> a;
    if (jac_to_aff(a, jac_mul_2x32(p, sp, w.k0, w.k1))) {
      soa_st_g1(r1_aff, n, i, a);
      st = ST_OK;
    }
  }
  r1_st[i] = st;
}

// The one-lane prologue as ONE launch (r06): the workgroups take the three roles in dispatch order --
// first the hash's search + root (the longest), then the pubkey decode (RB: + [r_i] pk_i), then the
// signature decode, nb workgroups each.  As three launches on three streams the order in which their
// waves took the SIMD slots varied from step to step: with the hash search first the prologue took
// 2.8-2.9 ms, with the pubkey decode first the search waited for slots and it took 3.2-3.7 ms
// (profiles/prologue_spans_r06c.txt).  Interleaving the roles (workgroup b: role b % 3) measured
// 3.17-3.19 ms (r06d); this order fixes the fast one.
template <int RB>
__global__ void __launch_bounds__(KBLOCK, RB ? BLS_WAVES_PER_EU : BLS_PROLOGUE_WAVES_PER_EU) k_prologue_1(
    size_t n, const uint8_t* __restrict__ pks, const uint8_t* __restrict__ sigs, const uint8_t* __restrict__ msgs,
    uint32_t mlen, const uint8_t* __restrict__ doms, int dom_stride, const uint8_t* __restrict__ seed32,
    uint32_t* __restrict__ pk_aff, uint8_t* __restrict__ pk_st, uint32_t* __restrict__ sig_aff,
    uint8_t* __restrict__ sig_st, uint32_t* __restrict__ h_aff, uint32_t* __restrict__ r1_aff,
    uint8_t* __restrict__ r1_st, int chk_g1, int chk_g2) {
  const uint32_t nb = gridDim.x / 3u;
  const uint32_t role = blockIdx.x / nb;
  const size_t i = (size_t)(blockIdx.x - role * nb) * blockDim.x + threadIdx.x;
  if (role == 0) {
    dev_hash_cand_1(i, n, msgs, mlen, doms, dom_stride, h_aff);
  } else if (role == 1) {
    if (RB) dev_rb_decode_g1(i, n, pks, seed32, pk_aff, pk_st, r1_aff, r1_st, chk_g1);
    else dev_decode_g1(i, n, pks, pk_aff, pk_st, chk_g1);
  } else {
    dev_decode_g2_1(i, n, sigs, sig_aff, sig_st, chk_g2);
  }
}

// k_rb_g2_test: one lane pair per item; the signature's G2 membership (psi(Q) == [x] Q) after the
// one-lane codec-only decode, and the item's class: outside G2 the signature is ST_BAD (strict) or
// ST_NOSUB (py_ecc: the item goes to the per-item path, where it is an ordinary point).
__global__ void __launch_bounds__(KBLOCK, BLS_WAVES_PER_EU) k_rb_g2_test(size_t n, const uint32_t* __restrict__ sig_aff,
                                                      uint8_t* __restrict__ sig_st,
                                                      const uint8_t* __restrict__ pk_st,
                                                      uint8_t* __restrict__ cls, int strict) {
  const size_t i = item_index<2>();
  if (i >= n) return;
  uint8_t ss = sig_st[i];
  if (ss == ST_OK && !g2_in_subgroup(soa_ld_g2(sig_aff, n, i))) ss = strict ? ST_BAD : ST_NOSUB;
  if (pr_odd()) return;
  const uint8_t ps = pk_st[i];
  sig_st[i] = ss;
  cls[i] = (ps == ST_BAD || ss == ST_BAD) ? RB_BAD : (ss == ST_NOSUB ? RB_SINGLE : RB_BATCH);
}

// per item, one lane pair: R2 = [r_i] sig_i (Jacobian SoA; infinity when the item is not
// batched: a bad pubkey, or a signature that is not a finite point of G2 -- the class
// k_rb_g2_test assigns, recomputed from the statuses)
__global__ void __launch_bounds__(KBLOCK, BLS_WAVES_PER_EU) k_rb_scale_g2(size_t n, const uint8_t* __restrict__ seed32,
                                                       const uint32_t* __restrict__ sig_aff,
                                                       const uint8_t* __restrict__ sig_st,
                                                       const uint8_t* __restrict__ pk_st,
                                                       uint32_t* __restrict__ r2_jac) {
  const size_t i = item_index<2>();
  if (i >= n) return;
  jac_t<fp2p_t> r = jac_infinity<fp2p_t>();
  if (pk_st[i] != ST_BAD && sig_st[i] == ST_OK) {
    const aff_t<fp2p_t> q = soa_ld_g2(sig_aff, n, i);
    aff_t<fp2p_t> sq = g2_psi(g2_psi(q));   // -psi^2(q) = [-x^2] q
    sq.y = fp2_neg(sq.y);
    const rb_weight w = rb_scalar(seed32, i);
    r = jac_mul_2x32(q, sq, w.k0, w.k1);
  }
  soa_jac<fp2p_t>::st(r2_jac, n, i, r);
}

// per sub-batch: sum of the R2 -> affine + status
__global__ void __launch_bounds__(KBLOCK, BLS_WAVES_PER_EU) k_agg_g2_affine(size_t ng, const uint32_t* __restrict__ jac,
                                                         const uint8_t* __restrict__ bad,
                                                         uint32_t* __restrict__ out_aff, uint8_t* __restrict__ st) {
  const size_t g = item_index<2>();
  if (g >= ng) return;
  const bool lead = !pr_odd();
  if (bad[g]) { if (lead) st[g] = ST_BAD; return; }
  aff_t<fp2p_t> a;
  if (!jac_to_aff(a, soa_jac<fp2p_t>::ld(jac, ng, g))) { if (lead) st[g] = ST_INF; return; }
  soa_st_g2(out_aff, ng, g, a);
  if (lead) st[g] = ST_OK;
}

// ---- the sub-batch signature sums S_b = sum_i [r_i] sig_i as a bucket MSM (Pippenger) ----
// With r_i = k0 + mu k1 and phi(Q) = -psi^2(Q) = (zeta x, y) = [mu] Q on G2, S_b is a multi-
// scalar product over the 2B points Q_i, phi(Q_i) of sub-batch b with 32-bit scalars k0_i,
// k1_i: RB_MSM_W windows of RB_MSM_C bits.  Point p of a sub-batch is item p / 2 of it, phi
// applied when p is odd.  An item outside the batch (bad pubkey, signature not a finite G2
// point) has scalars 0 and never enters a bucket -- the same items k_rb_scale_g2 leaves at
// infinity.  Per item this is ~2 x 8 x 15/16 mixed additions instead of a 32-doubling joint
// ladder per item; the per-sub-batch bucket and window sums are shared.
//   k_rb_msm_sort    one workgroup per sub-batch: digits, counting sort by (window, digit)
//   k_rb_msm_bucket  one lane pair per (sub-batch, window, digit): its points summed
//   k_rb_msm_window  one lane pair per (sub-batch, window): sum_d d B_d by running sums
//   k_rb_msm_combine one lane pair per sub-batch: sum_w 2^(C w) S_w (Horner), Jacobian out
constexpr int RB_MSM_C = 4, RB_MSM_W = 32 / RB_MSM_C, RB_MSM_D = 1 << RB_MSM_C;

// off: per (b, w) RB_MSM_D + 1 list starts (digit d's points at [off[d], off[d+1]) of the
// (b, w) list); idx: per (b, w) 2B point numbers (uint16: B < 2^15).  The scalars are
// recomputed in each pass (rb_scalar: one SHA-256 compression per item).
__device__ __forceinline__ void rb_msm_scalars(const uint8_t* seed32, const uint8_t* sig_st, const uint8_t* pk_st,
                                               size_t i, uint32_t& k0, uint32_t& k1) {
  k0 = k1 = 0;
  if (pk_st[i] != ST_BAD && sig_st[i] == ST_OK) {
    const rb_weight w = rb_scalar(seed32, i);
    k0 = w.k0; k1 = w.k1;
  }
}

__global__ void __launch_bounds__(KBLOCK) k_rb_msm_sort(size_t n, size_t B, const uint8_t* __restrict__ seed32,
                                                        const uint8_t* __restrict__ sig_st,
                                                        const uint8_t* __restrict__ pk_st,
                                                        uint32_t* __restrict__ off, uint16_t* __restrict__ idx) {
  __shared__ uint32_t cnt[RB_MSM_W][RB_MSM_D];
  const size_t b = blockIdx.x, base = b * B;
  if (base >= n) return;
  const uint32_t m = (uint32_t)(n - base < B ? n - base : B);
  for (uint32_t t = threadIdx.x; t < RB_MSM_W * RB_MSM_D; t += blockDim.x) cnt[t / RB_MSM_D][t % RB_MSM_D] = 0;
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < m; t += blockDim.x) {
    uint32_t k[2];
    rb_msm_scalars(seed32, sig_st, pk_st, base + t, k[0], k[1]);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int w = 0; w < RB_MSM_W; ++w) {
        const uint32_t d = (k[h] >> (RB_MSM_C * w)) & (RB_MSM_D - 1);
        if (d) atomicAdd(&cnt[w][d], 1u);
      }
  }
  __syncthreads();
  if (threadIdx.x < RB_MSM_W) {
    const int w = threadIdx.x;
    uint32_t* o = off + (b * RB_MSM_W + w) * (RB_MSM_D + 1);
    uint32_t run = 0;
    o[0] = 0;
    for (int d = 1; d < RB_MSM_D; ++d) { o[d] = run; const uint32_t c = cnt[w][d]; cnt[w][d] = run; run += c; }
    o[RB_MSM_D] = run;
  }
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < m; t += blockDim.x) {
    uint32_t k[2];
    rb_msm_scalars(seed32, sig_st, pk_st, base + t, k[0], k[1]);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int w = 0; w < RB_MSM_W; ++w) {
        const uint32_t d = (k[h] >> (RB_MSM_C * w)) & (RB_MSM_D - 1);
        if (d) idx[(b * RB_MSM_W + w) * 2 * B + atomicAdd(&cnt[w][d], 1u)] = (uint16_t)(2 * t + h);
      }
  }
}

// bucket (b, w, d), d >= 1: the sum of its points (Jacobian SoA over nb * W * D slots;
// slot (b W + w) D + d, digit-0 slots unused)
__global__ void __launch_bounds__(KBLOCK, BLS_WAVES_PER_EU) k_rb_msm_bucket(size_t n, size_t B, size_t nb,
                                                         const uint32_t* __restrict__ sig_aff,
                                                         const uint32_t* __restrict__ off,
                                                         const uint16_t* __restrict__ idx,
                                                         uint32_t* __restrict__ bucket) {
  const size_t t = item_index<2>();
  constexpr size_t TPB = RB_MSM_W * (RB_MSM_D - 1);   // tasks per sub-batch
  if (t >= nb * TPB) return;
  const size_t b = t / TPB, r = t % TPB, w = r / (RB_MSM_D - 1), d = r % (RB_MSM_D - 1) + 1;
  const uint32_t* o = off + (b * RB_MSM_W + w) * (RB_MSM_D + 1);
  const uint16_t* li = idx + (b * RB_MSM_W + w) * 2 * B;
  jac_t<fp2p_t> acc = jac_infinity<fp2p_t>();
  for (uint32_t k = o[d], e = o[d + 1]; k < e; ++k) {
    const uint32_t p = li[k];
    aff_t<fp2p_t> Q = soa_ld_g2(sig_aff, n, b * B + (p >> 1));
    if (p & 1u) Q.x.v = fp_mul(Q.x.v, G2_ZETA_M);   // phi(Q) = (zeta x, y)
    acc = jac_add_aff(acc, Q);
  }
  soa_jac<fp2p_t>::st(bucket, nb * RB_MSM_W * RB_MSM_D, (b * RB_MSM_W + w) * RB_MSM_D + d, acc);
}

// window (b, w): sum_d d B_d = sum over d of the running sums of B_15 .. B_d
__global__ void __launch_bounds__(KBLOCK, BLS_WAVES_PER_EU) k_rb_msm_window(size_t nb, const uint32_t* __restrict__ bucket,
                                                         uint32_t* __restrict__ win) {
  const size_t t = item_index<2>();
  if (t >= nb * RB_MSM_W) return;
  const size_t ns = nb * RB_MSM_W * RB_MSM_D;
  jac_t<fp2p_t> run = jac_infinity<fp2p_t>(), sum = jac_infinity<fp2p_t>();
  for (int d = RB_MSM_D - 1; d >= 1; --d) {
    run = jac_add(run, soa_jac<fp2p_t>::ld(bucket, ns, t * RB_MSM_D + d));
    sum = jac_add(sum, run);
  }
  soa_jac<fp2p_t>::st(win, nb * RB_MSM_W, t, sum);
}

// sub-batch b: S_b = sum_w 2^(C w) S_(b,w), Horner from the top window
__global__ void __launch_bounds__(KBLOCK, BLS_WAVES_PER_EU) k_rb_msm_combine(size_t nb, const uint32_t* __restrict__ win,
                                                          uint32_t* __restrict__ out_jac) {
  const size_t b = item_index<2>();
  if (b >= nb) return;
  const size_t nw = nb * RB_MSM_W;
  jac_t<fp2p_t> acc = soa_jac<fp2p_t>::ld(win, nw, b * RB_MSM_W + RB_MSM_W - 1);
  for (int w = RB_MSM_W - 2; w >= 0; --w) {
#pragma unroll 1
    for (int k = 0; k < RB_MSM_C; ++k) acc = jac_dbl(acc);
    acc = jac_add(acc, soa_jac<fp2p_t>::ld(win, nw, b * RB_MSM_W + w));
  }
  soa_jac<fp2p_t>::st(out_jac, nb, b, acc);
}

// Randomized batches, split Miller loop (the C2 kernels' layout): quad q runs the pairs
// (BP(H_i), [r_i] pk_i) of items i = 2q (lo half) and 2q + 1 (hi half) and writes their line
// products L = l l' for k_ml_accum, so two batched items share one f and its squarings.  A
// half whose item is not batched (not RB_BATCH, an infinite [r_i] pk_i or hash) idles with its
// lines masked to 1.  Status per quad: ML_ST_ONE (both idle), ST_BAD (a degenerate loop: the
// sub-batch then fails and its items go one by one), else ST_OK.
__global__ void __launch_bounds__(KBLOCK, BLS_ML_WAVES_PER_EU) k_rb_ml_lines(size_t n, size_t q0, size_t cnt,
                                                       const uint32_t* __restrict__ h_aff,
                                                       const uint8_t* __restrict__ h_st,
                                                       const uint32_t* __restrict__ r1_aff,
                                                       const uint8_t* __restrict__ r1_st,
                                                       const uint8_t* __restrict__ cls,
                                                       uint32_t* __restrict__ L, uint8_t* __restrict__ st_out) {
  const size_t lq = item_index<4>();
  if (lq >= cnt) return;
  const size_t q = q0 + lq;
  const bool hi = qd_hi();
  const bool lead = (threadIdx.x & 3u) == 0;
  const size_t ia = 2 * q, ib = 2 * q + 1;
  const bool a_ok = ia < n && cls[ia] == RB_BATCH && r1_st[ia] == ST_OK && h_st[ia] == ST_OK;
  const bool b_ok = ib < n && cls[ib] == RB_BATCH && r1_st[ib] == ST_OK && h_st[ib] == ST_OK;
  if (!a_ok && !b_ok) { if (lead) st_out[lq] = ML_ST_ONE; return; }
  // an idle half runs the other half's pair with its lines masked to 1
  const bool active = hi ? b_ok : a_ok;
  const size_t i = (hi ? b_ok : !a_ok) ? ib : ia;
  const size_t lp = 2 * i + (pr_odd() ? 1 : 0);
  g2_proj<fp2p_t> T;
#if BLS_ML_LINES_LDS
  __shared__ uint32_t lds_pre[ML_LDS_WORDS];
  lds_u32* col = (lds_u32*)lds_pre + threadIdx.x;
  const ml_src src{h_aff, 2 * n, lp, r1_aff, n, i};
  ml_lds_put(col, g1_prepare(ml_src_p(src)));
  T = ml_lines_run_lds(src, col, active, L, cnt, lq, 0);
#else
  aff_t<fp2p_t> Q;
  Q.x = pr_make(soa_ld(h_aff, 2 * n, lp, 0));
  Q.y = pr_make(soa_ld(h_aff, 2 * n, lp, 1));
  const g1_line_pre pre = g1_prepare(soa_ld_g1(r1_aff, n, i));
  T = ml_lines_run(Q, pre, active, L, cnt, lq);
#endif
  bool bad = active && fp2_is_zero(T.z);
  bad = !qd_all(!bad);
  if (lead) st_out[lq] = bad ? ST_BAD : ST_OK;
}

// the signature-sum slot of every sub-batch: (sum_i [r_i] sig_i, -[c] g1), one lane quad
// per sub-batch (miller_loop_q1, the latency form: nb is small and this branch runs
// beside the per-item work)
// (slot_per: the item value slots per sub-batch; the sum's slot follows them)
__global__ void __launch_bounds__(KBLOCK, BLS_ML_WAVES_PER_EU) k_rb_miller_sig(size_t nb, size_t slot_per,
                                                         const uint32_t* __restrict__ s_aff,
                                                         const uint8_t* __restrict__ s_st, size_t nslots,
                                                         uint32_t* __restrict__ f_out, uint8_t* __restrict__ st_out) {
  const size_t b = item_index<4>();
  if (b >= nb) return;
  const size_t slot = b * (slot_per + 1) + slot_per;
  const int p = pr_odd() ? 1 : 0;
  fq12_t f = fq12_one();
  bool degen = false;
  const uint8_t st = s_st[b];
  if (st == ST_OK) {
    aff_t<fp2p_t> Q;
    Q.x = pr_make(soa_ld(s_aff, 2 * nb, 2 * b + p, 0));
    Q.y = pr_make(soa_ld(s_aff, 2 * nb, 2 * b + p, 1));
    aff_t<fp_t> ng; ng.x = G1_VGEN_X_M; ng.y = G1_VGEN_NEGY_M;
    f = miller_loop_q1(Q, g1_prepare(ng), degen);
  }
  const int c0 = qd_hi() ? 3 : 0;
  soa_st(f_out, 2 * nslots, 2 * slot + p, c0 + 0, f.h.c0.v);
  soa_st(f_out, 2 * nslots, 2 * slot + p, c0 + 1, f.h.c1.v);
  soa_st(f_out, 2 * nslots, 2 * slot + p, c0 + 2, f.h.c2.v);
  if ((threadIdx.x & 3u) == 0) st_out[slot] = (st == ST_BAD || degen) ? ST_BAD : ST_OK;
}

// ---------------------------------------------------- aggregation kernels --
// A chunk is a contiguous range [begin, end) of inputs belonging to one group.
// Each workgroup sums one chunk: item slots (one lane, or one lane pair for G2)
// stride over the chunk, then a tree reduction of Jacobian partials staged in
// LDS.  The input is either compressed points (level 1: decode + sum) or
// Jacobian SoA partials.
struct agg_chunk { uint32_t begin, end; };

template <class F> struct pt_traits;
template <> struct pt_traits<fp_t> {
  static constexpr int BYTES = 48;
  __device__ static int decode(aff_t<fp_t>& a, const uint8_t* b, bool lax) { return g1_decompress(a, b, lax); }
  __device__ static bool in_subgroup(const aff_t<fp_t>& a) { return g1_in_subgroup(a); }
};
template <> struct pt_traits<fp2p_t> {
  static constexpr int BYTES = 96;
  __device__ static int decode(aff_t<fp2p_t>& a, const uint8_t* b, bool lax) { return g2_decompress(a, b, lax); }
  __device__ static bool in_subgroup(const aff_t<fp2p_t>& a) { return g2_in_subgroup(a); }
};

// Registry points are entry-major (AoS): entry r's affine x and y limbs are the 28
// consecutive words at aff + 28 r (112 B, 16-byte aligned).  Members are read by
// validator index, i.e. at random entries: an entry is one contiguous 112-byte read
// (seven 16-byte loads) instead of 28 limb loads that each touch their own cache line,
// as a limb-major (SoA) layout would give for a random index.
constexpr int REG_WORDS = 2 * FP_LIMBS;
__device__ __forceinline__ void reg_st_g1(uint32_t* aff, size_t r, const aff_t<fp_t>& a) {
  uint4* p = reinterpret_cast<uint4*>(aff + (size_t)REG_WORDS * r);
  uint32_t w[REG_WORDS];
#pragma unroll
  for (int k = 0; k < FP_LIMBS; ++k) { w[k] = a.x.w[k]; w[FP_LIMBS + k] = a.y.w[k]; }
#pragma unroll
  for (int q = 0; q < REG_WORDS / 4; ++q) p[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}
template <class F> __device__ aff_t<F> reg_ld_aff(const uint32_t* aff, size_t r);
template <> __device__ __forceinline__ aff_t<fp_t> reg_ld_aff<fp_t>(const uint32_t* aff, size_t r) {
  const uint4* p = reinterpret_cast<const uint4*>(aff + (size_t)REG_WORDS * r);
  uint32_t w[REG_WORDS];
#pragma unroll
  for (int q = 0; q < REG_WORDS / 4; ++q) {
    const uint4 v = p[q];
    w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
  }
  aff_t<fp_t> a;
#pragma unroll
  for (int k = 0; k < FP_LIMBS; ++k) { a.x.w[k] = w[k]; a.y.w[k] = w[FP_LIMBS + k]; }
  return a;
}
template <> __device__ __forceinline__ aff_t<fp2p_t> reg_ld_aff<fp2p_t>(const uint32_t*, size_t) {
  __builtin_trap();   // the registry holds G1 pubkeys only; never instantiated with entries
}

// Inputs of a level-1 chunk sum: compressed bytes, or (AGG_REGISTRY, G1 only) a
// registry entry per input -- entry >= 0 reads the registry's decoded point,
// entry < 0 decodes the input's own bytes (a cache miss).
enum : int { AGG_BYTES = 0, AGG_JAC = 1, AGG_REGISTRY = 2 };
struct agg_reg_src {
  const int32_t* entry;   // per input: registry entry or -1
  const uint32_t* aff;    // registry affine points, entry-major (reg_ld_aff)
  const uint8_t* st;      // registry entry status: ST_OK / ST_INF / ST_BAD
  size_t cap;             // entries allocated
  size_t size;            // entries in use: an entry >= size is an error (BAD), never read
};

// adds level-1 input e (compressed bytes, or a registry entry) to acc.  `check` flags
// (CHK_*): the codec, and (STRICT policy, verify_multiple) a point outside the subgroup is bad
template <class F, int MODE>
__device__ __forceinline__ void agg_accumulate(jac_t<F>& acc, bool& bad, uint32_t e, const uint8_t* in_bytes,
                                               const agg_reg_src& reg, int check) {
  const bool lax = (check & CHK_LAX) != 0;
  const int sub = check & CHK_SUB_MASK;
  if (MODE == AGG_REGISTRY) {
    const int32_t r = reg.entry ? reg.entry[e] : -1;
    if ((r >= 0 && (size_t)r >= reg.size) || (r < 0 && !in_bytes)) { bad = true; return; }
    if (r >= 0) {
      const uint8_t rs0 = reg.st[r];
      const uint8_t rs = (rs0 & ST_NONCANON) && !lax ? (uint8_t)ST_BAD : (uint8_t)(rs0 & ~ST_NONCANON);
      if (rs == ST_BAD) {
        bad = true;
      } else if (rs == ST_OK) {
        const aff_t<F> a = reg_ld_aff<F>(reg.aff, (size_t)r);
        if (sub && !pt_traits<F>::in_subgroup(a)) bad = true;
        else acc = jac_add_aff(acc, a);
      }
      return;
    }
  }
  aff_t<F> a;
  int s = pt_traits<F>::decode(a, in_bytes + (size_t)pt_traits<F>::BYTES * e, lax);
  if (s == PT_OK && sub && !pt_traits<F>::in_subgroup(a)) s = PT_BAD;
  if (s == PT_BAD) bad = true;
  else if (s == PT_OK) acc = jac_add_aff(acc, a);
}

// Level 1 for small G1 chunks: one lane sums one chunk in sequence.  Used when
// chunks average a few inputs (bls_verify_multiple's per-message groups, often
// one key each), where a workgroup per chunk would leave 127 of 128 lanes idle.
template <int MODE>
__global__ void __launch_bounds__(KBLOCK, BLS_AGG_WAVES_PER_EU) k_agg_lanes(size_t nchunks, const agg_chunk* __restrict__ chunks,
                                                     const uint8_t* __restrict__ in_bytes,
                                                     uint32_t* __restrict__ out_jac, uint8_t* __restrict__ out_bad,
                                                     agg_reg_src reg, int check) {
  const size_t c = item_index<1>();
  if (c >= nchunks) return;
  const agg_chunk ch = chunks[c];
  jac_t<fp_t> acc = jac_infinity<fp_t>();
  bool bad = false;
  for (uint32_t e = ch.begin; e < ch.end; ++e) agg_accumulate<fp_t, MODE>(acc, bad, e, in_bytes, reg, check);
  soa_jac<fp_t>::st(out_jac, nchunks, c, acc);
  out_bad[c] = bad ? 1 : 0;
}

template <class F, int MODE>
__global__ void __launch_bounds__(KBLOCK, BLS_AGG_WAVES_PER_EU) k_agg_chunks(size_t nchunks, const agg_chunk* __restrict__ chunks,
                                                      const uint8_t* __restrict__ in_bytes,
                                                      const uint32_t* __restrict__ in_jac, size_t n_in,
                                                      const uint8_t* __restrict__ in_bad,
                                                      uint32_t* __restrict__ out_jac, uint8_t* __restrict__ out_bad,
                                                      agg_reg_src reg, int check) {
  constexpr int LPI = lanes_per<F>::N;
  constexpr int NW = sizeof(jac_t<F>) / 4;   // words per lane
  __shared__ uint32_t lds[KBLOCK * NW];
  __shared__ int bad_any;
  const size_t c = blockIdx.x;
  if (c >= nchunks) return;
  const agg_chunk ch = chunks[c];
  if (threadIdx.x == 0) bad_any = 0;
  __syncthreads();
  jac_t<F> acc = jac_infinity<F>();
  bool bad = false;
  const uint32_t slot = threadIdx.x / LPI;
  for (uint32_t e = ch.begin + slot; e < ch.end; e += KBLOCK / LPI) {
    if (MODE == AGG_JAC) {
      if (in_bad[e]) bad = true;
      acc = jac_add(acc, soa_jac<F>::ld(in_jac, n_in, e));
      continue;
    }
    agg_accumulate<F, MODE>(acc, bad, e, in_bytes, reg, check);
  }
  if (bad) bad_any = 1;
  // tree reduction through LDS (lane-major words: conflict-free stride-1 access);
  // s counts lanes and stays a multiple of LPI, so item slots move whole
  uint32_t* mine = lds;
  for (int s = KBLOCK / 2; s >= LPI; s >>= 1) {
    __syncthreads();
    if (threadIdx.x >= s && threadIdx.x < 2 * s) {
      const uint32_t* src = reinterpret_cast<const uint32_t*>(&acc);
      for (int w = 0; w < NW; ++w) mine[w * KBLOCK + (threadIdx.x - s)] = src[w];
    }
    __syncthreads();
    if (threadIdx.x < s) {
      jac_t<F> o;
      uint32_t* dst = reinterpret_cast<uint32_t*>(&o);
      for (int w = 0; w < NW; ++w) dst[w] = mine[w * KBLOCK + threadIdx.x];
      acc = jac_add(acc, o);
    }
  }
  __syncthreads();
  if (threadIdx.x < LPI) {
    soa_jac<F>::st(out_jac, nchunks, c, acc);
    if (threadIdx.x == 0) out_bad[c] = (uint8_t)bad_any;
  }
}

__device__ __forceinline__ void pt_compress(uint8_t* out, const jac_t<fp_t>& p) { g1_compress(out, p); }
__device__ __forceinline__ void pt_compress(uint8_t* out, const jac_t<fp2p_t>& p) { g2_compress(out, p); }

// per group: Jacobian sum -> compressed bytes + status
template <class F>
__global__ void __launch_bounds__(KBLOCK, BLS_WAVES_PER_EU) k_agg_compress(size_t ng, const uint32_t* __restrict__ jac,
                                                        const uint8_t* __restrict__ bad,
                                                        uint8_t* __restrict__ out, int32_t* __restrict__ status) {
  constexpr int LPI = lanes_per<F>::N;
  const size_t g = item_index<LPI>();
  if (g >= ng) return;
  const bool lead = (threadIdx.x % LPI) == 0;
  if (bad[g]) { if (lead) status[g] = BLS381_EINVAL_POINT; return; }
  const jac_t<F> p = soa_jac<F>::ld(jac, ng, g);
  pt_compress(out + (size_t)pt_traits<F>::BYTES * g, p);
  if (lead) status[g] = 0;
}

// per group: Jacobian G1 sum -> affine + status (OK / INF / BAD).  The members'
// subgroup checks (STRICT policy) ran when they were decoded; py_ecc checks none.
__global__ void __launch_bounds__(KBLOCK, BLS_WAVES_PER_EU) k_agg_g1_affine(size_t ng, const uint32_t* __restrict__ jac,
                                                         const uint8_t* __restrict__ bad,
                                                         uint32_t* __restrict__ out_aff, uint8_t* __restrict__ st) {
  const size_t g = item_index<1>();
  if (g >= ng) return;
  if (bad[g]) { st[g] = ST_BAD; return; }
  aff_t<fp_t> a;
  if (!jac_to_aff(a, soa_jac<fp_t>::ld(jac, ng, g))) { st[g] = ST_INF; return; }
  soa_st_g1(out_aff, ng, g, a);
  st[g] = ST_OK;
}

// -------------------------------------------------------- pubkey registry --
// Device-resident registry of decoded pubkeys: entry j
// holds the 48-byte key, its status and its affine point (entry-major, reg_st_g1); an
// open-addressing table (u32 entry per slot, REG_EMPTY when free, linear
// probing, power-of-two size) maps key bytes to entries.
constexpr uint32_t REG_EMPTY = 0xFFFFFFFFu;

// 48 key bytes -> 32-bit hash (all 12 words mixed; the x bytes are uniform)
__device__ __forceinline__ uint32_t reg_hash(const uint8_t* k) {
  uint32_t h = 0x9E3779B9u;
  for (int w = 0; w < 12; ++w) {
    const uint32_t v = (uint32_t)k[4 * w] | ((uint32_t)k[4 * w + 1] << 8) | ((uint32_t)k[4 * w + 2] << 16) |
                       ((uint32_t)k[4 * w + 3] << 24);
    h = (h ^ v) * 0x85EBCA6Bu;
    h ^= h >> 15;
  }
  return h;
}
__device__ __forceinline__ bool reg_key_eq(const uint8_t* a, const uint8_t* b) {
  uint32_t d = 0;
  for (int i = 0; i < 48; ++i) d |= (uint32_t)(a[i] ^ b[i]);
  return d == 0;
}

// decode keys [first, first + n) in place (status + affine point).  Entries serve calls
// under either policy: a key is decoded with the lax codec, and one the strict codec
// rejects is marked ST_NONCANON (its lax point is the only point either codec gives it).
__global__ void __launch_bounds__(KBLOCK, BLS_WAVES_PER_EU) k_reg_decode(size_t first, size_t n, size_t cap,
                                                      const uint8_t* __restrict__ keys,
                                                      uint32_t* __restrict__ aff, uint8_t* __restrict__ st) {
  const size_t t = item_index<1>();
  if (t >= n) return;
  const size_t j = first + t;
  aff_t<fp_t> a;
  const uint8_t* k = keys + 48 * j;
  const int s = g1_decompress(a, k, true);
  if (s == PT_OK) reg_st_g1(aff, j, a);
  const uint8_t nc = s != PT_BAD && !g1_canonical(k) ? ST_NONCANON : (uint8_t)0;
  st[j] = (uint8_t)((s == PT_OK ? ST_OK : (s == PT_INF ? ST_INF : ST_BAD)) | nc);
}

// insert entries [first, first + n) that decoded.  Equal keys share one slot,
// which ends up holding the smallest of their entries (atomicMin), whatever
// the order the lanes run in; the caller then resolves each key with
// k_reg_lookup once the table has settled.
__global__ void __launch_bounds__(KBLOCK) k_reg_insert(size_t first, size_t n, const uint8_t* __restrict__ keys,
                                                       const uint8_t* __restrict__ st, uint32_t* table, uint32_t mask) {
  const size_t t = item_index<1>();
  if (t >= n) return;
  const uint32_t j = (uint32_t)(first + t);
  if (st[j] == ST_BAD) return;
  const uint8_t* k = keys + 48 * (size_t)j;
  uint32_t slot = reg_hash(k) & mask;
  for (uint32_t probe = 0; probe <= mask; ++probe, slot = (slot + 1) & mask) {
    uint32_t cur = __atomic_load_n(&table[slot], __ATOMIC_RELAXED);
    if (cur == REG_EMPTY) {
      cur = atomicCAS(&table[slot], REG_EMPTY, j);
      if (cur == REG_EMPTY) return;
    }
    if (reg_key_eq(keys + 48 * (size_t)cur, k)) { atomicMin(&table[slot], j); return; }
  }
}

// content-addressed lookup of n compressed keys: entry or -1 (not registered)
__global__ void __launch_bounds__(KBLOCK) k_reg_lookup(size_t n, const uint8_t* __restrict__ q,
                                                       const uint8_t* __restrict__ keys,
                                                       const uint32_t* __restrict__ table, uint32_t mask,
                                                       int32_t* __restrict__ entry) {
  const size_t t = item_index<1>();
  if (t >= n) return;
  const uint8_t* k = q + 48 * t;
  uint32_t slot = reg_hash(k) & mask;
  int32_t r = -1;
  for (uint32_t probe = 0; probe <= mask; ++probe, slot = (slot + 1) & mask) {
    const uint32_t cur = table[slot];
    if (cur == REG_EMPTY) break;
    if (reg_key_eq(keys + 48 * (size_t)cur, k)) { r = (int32_t)cur; break; }
  }
  entry[t] = r;
}

// ------------------------------------------------------ SSZ roots (§8(f)2) --
// roots of n serialized fixed-size items (item i at items + i * stride); the
// program (bls381_ssz.hpp) is uniform, so every lane runs the same ops
__global__ void __launch_bounds__(KBLOCK) k_ssz_root(size_t n, const uint8_t* __restrict__ items, size_t stride,
                                                     const uint32_t* __restrict__ prog, uint32_t plen,
                                                     uint8_t* __restrict__ roots, int32_t* __restrict__ err) {
  const size_t i = item_index<1>();
  if (i >= n) return;
  uint32_t stk[SSZ_STACK][8];
  uint32_t r[8];
  if (!ssz_run(r, items + i * stride, prog, plen, stk)) { *err = 1; return; }
  uint8_t* o = roots + 32 * i;
  for (int w = 0; w < 8; ++w)
    for (int b = 0; b < 4; ++b) o[4 * w + b] = (uint8_t)(r[w] >> (24 - 8 * b));
}

// gather a byte field [off, off + len) of n strided items into a packed array
__global__ void __launch_bounds__(KBLOCK) k_gather_field(size_t n, const uint8_t* __restrict__ items, size_t stride,
                                                         uint32_t off, uint32_t len, uint8_t* __restrict__ out) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * len) return;
  const size_t i = t / len, b = t % len;
  out[t] = items[i * stride + off + b];
}

// ------------------------------------------------------- sign / privtopub --
__device__ __forceinline__ scalar_t scalar_from_be32(const uint8_t* b) {
  scalar_t k;
  for (int i = 0; i < 8; ++i) {
    const uint8_t* p = b + 28 - 4 * i;
    k.w[i] = ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
  }
  for (int i = 8; i < 16; ++i) k.w[i] = 0;
  return k;
}

// sign = [sk] hash_to_G2(m, d), compressed; one lane pair per item
__global__ void __launch_bounds__(KBLOCK, BLS_WAVES_PER_EU) k_sign(size_t n, const uint8_t* __restrict__ msgs, uint32_t mlen,
                                                const uint8_t* __restrict__ sks, const uint8_t* __restrict__ doms,
                                                uint8_t* __restrict__ out) {
  const size_t i = item_index<2>();
  if (i >= n) return;
  uint8_t dom[8];
  ld_bytes(dom, doms + 8 * i, 8);
  aff_t<fp2p_t> c;
  hash_to_g2_candidate(c, msgs + (size_t)mlen * i, mlen, dom);
  aff_t<fp2p_t> h;
  if (!jac_to_aff(h, g2_mul_cofactor(c))) {
    g2_compress(out + 96 * i, jac_infinity<fp2p_t>());
  } else {
    g2_compress(out + 96 * i, jac_mul_limbs(h, scalar_from_be32(sks + 32 * i), 256));
  }
}

__global__ void __launch_bounds__(KBLOCK, BLS_WAVES_PER_EU) k_privtopub(size_t n, const uint8_t* __restrict__ sks, uint8_t* __restrict__ out) {
  const size_t i = item_index<1>();
  if (i >= n) return;
  aff_t<fp_t> g; g.x = G1_GEN_X_M; g.y = G1_GEN_Y_M;
  uint8_t pk[48];
  g1_compress(pk, jac_mul_limbs(g, scalar_from_be32(sks + 32 * i), 256));
  for (int b = 0; b < 48; ++b) out[48 * i + b] = pk[b];
}

// hash_to_G2 -> compressed (96 B) + affine (192 B: x_re, x_im, y_re, y_im) per item
__global__ void __launch_bounds__(KBLOCK, BLS_WAVES_PER_EU) k_hash_g2_out(size_t n, const uint8_t* __restrict__ msgs, uint32_t mlen,
                                                       const uint8_t* __restrict__ doms,
                                                       uint8_t* __restrict__ comp, uint8_t* __restrict__ affb) {
  const size_t i = item_index<2>();
  if (i >= n) return;
  const int p = pr_odd() ? 1 : 0;
  uint8_t dom[8];
  ld_bytes(dom, doms + 8 * i, 8);
  aff_t<fp2p_t> c;
  hash_to_g2_candidate(c, msgs + (size_t)mlen * i, mlen, dom);
  aff_t<fp2p_t> h;
  if (!jac_to_aff(h, g2_mul_cofactor(c))) {
    g2_compress(comp + 96 * i, jac_infinity<fp2p_t>());
    for (int b = 0; b < 96; ++b) affb[192 * i + 96 * p + b] = 0;
    return;
  }
  g2_compress_aff(comp + 96 * i, h);
  fp_plain_to_be48(affb + 192 * i + 48 * p, fp_from_mont(h.x.v));
  fp_plain_to_be48(affb + 192 * i + 96 + 48 * p, fp_from_mont(h.y.v));
}

// ------------------------------------- py_ecc-exact projective hash_to_G2 --
// Mirrors py_ecc optimized_bls12_381 homogeneous `double`/`add` and the
// recursive `multiply` so the un-normalised triple
// printed by test_generators/bls/main.py:66-72 is reproduced bit for bit.
template <class E> struct proj2 { E x, y, z; };

template <class E>
__device__ __forceinline__ proj2<E> pyecc_double(const proj2<E>& p) {
  const E W = fp2_mul_small(fp2_sqr(p.x), 3);
  const E S = fp2_mul(p.y, p.z);
  const E B = fp2_mul(fp2_mul(p.x, p.y), S);
  const E H = fp2_sub(fp2_sqr(W), fp2_mul_small(B, 8));
  const E S2 = fp2_sqr(S);
  proj2<E> r;
  r.x = fp2_mul_small(fp2_mul(H, S), 2);
  r.y = fp2_sub(fp2_mul(W, fp2_sub(fp2_mul_small(B, 4), H)), fp2_mul_small(fp2_mul(fp2_sqr(p.y), S2), 8));
  r.z = fp2_mul_small(fp2_mul(S, S2), 8);
  return r;
}

template <class E>
__device__ __forceinline__ proj2<E> pyecc_add(const proj2<E>& p1, const proj2<E>& p2) {
  if (fp2_is_zero(p1.z) || fp2_is_zero(p2.z)) return fp2_is_zero(p2.z) ? p1 : p2;
  const E U1 = fp2_mul(p2.y, p1.z);
  const E U2 = fp2_mul(p1.y, p2.z);
  const E V1 = fp2_mul(p2.x, p1.z);
  const E V2 = fp2_mul(p1.x, p2.z);
  if (fp2_eq(V1, V2) && fp2_eq(U1, U2)) return pyecc_double(p1);
  if (fp2_eq(V1, V2)) { proj2<E> r; r.x = e2_one<E>(); r.y = e2_one<E>(); r.z = e2_zero<E>(); return r; }
  const E U = fp2_sub(U1, U2);
  const E V = fp2_sub(V1, V2);
  const E V_sq = fp2_sqr(V);
  const E V_sq_V2 = fp2_mul(V_sq, V2);
  const E V_cu = fp2_mul(V, V_sq);
  const E W = fp2_mul(p1.z, p2.z);
  const E A = fp2_sub(fp2_sub(fp2_mul(fp2_sqr(U), W), V_cu), fp2_mul_small(V_sq_V2, 2));
  proj2<E> r;
  r.x = fp2_mul(V, A);
  r.y = fp2_sub(fp2_mul(U, fp2_sub(V_sq_V2, A)), fp2_mul(V_cu, U2));
  r.z = fp2_mul(V_cu, W);
  return r;
}

// scratch: per item H2_BITS proj2 slots (pair SoA over n * H2_BITS items, 3 Fp2 each)
__global__ void __launch_bounds__(64, BLS_WAVES_PER_EU) k_hash_g2_pyecc(size_t n, const uint8_t* __restrict__ msgs,
                                                     const uint8_t* __restrict__ doms,
                                                     uint32_t* __restrict__ scratch, uint8_t* __restrict__ out288) {
  const size_t i = item_index<2>();
  if (i >= n) return;
  const int p = pr_odd() ? 1 : 0;
    uint8_t dom[8];
  ld_bytes(dom, doms + 8 * i, 8);
  aff_t<fp2p_t> c;
  hash_to_g2_candidate(c, msgs + 32 * i, 32, dom);
  const size_t ns = n * (size_t)H2_BITS;
  auto slot = [&](int b) { return i * (size_t)H2_BITS + b; };
  proj2<fp2p_t> cur;
  cur.x = c.x; cur.y = c.y; cur.z = e2_one<fp2p_t>();
  // doublings P_b = double^b(P) for b < top, stored; P_top is the accumulator start
  for (int b = 0; b < H2_BITS - 1; ++b) {
    const size_t s = slot(b);
    soa_st2p(scratch, ns, s, 0, cur.x); soa_st2p(scratch, ns, s, 1, cur.y); soa_st2p(scratch, ns, s, 2, cur.z);
    cur = pyecc_double(cur);
  }
  proj2<fp2p_t> acc = cur;
  for (int b = H2_BITS - 2; b >= 0; --b) {
    if ((H2_LIMBS[b >> 5] >> (b & 31)) & 1u) {
      const size_t s = slot(b);
      proj2<fp2p_t> pb;
      pb.x = soa_ld2p(scratch, ns, s, 0); pb.y = soa_ld2p(scratch, ns, s, 1); pb.z = soa_ld2p(scratch, ns, s, 2);
      acc = pyecc_add(acc, pb);
    }
  }
  uint8_t* o = out288 + 288 * i;
  fp_plain_to_be48(o + 48 * p, fp_from_mont(acc.x.v));
  fp_plain_to_be48(o + 96 + 48 * p, fp_from_mont(acc.y.v));
  fp_plain_to_be48(o + 192 + 48 * p, fp_from_mont(acc.z.v));
}

// -------------------------------------------------------- Fp12 byte codec --
// 576 B per item = a0, a1, a2, b0, b1, b2, each Fp2 as re || im (48 B each)
__global__ void __launch_bounds__(KBLOCK, BLS_WAVES_PER_EU) k_fp12_to_bytes(size_t n, const uint32_t* __restrict__ f,
                                                         uint8_t* __restrict__ out) {
  const size_t i = item_index<2>();
  if (i >= n) return;
  const int p = pr_odd() ? 1 : 0;
  const fp12p_t a = soa_ld12(f, n, i);
  const fp2p_t* cs[6] = {&a.c0.c0, &a.c0.c1, &a.c0.c2, &a.c1.c0, &a.c1.c1, &a.c1.c2};
  for (int k = 0; k < 6; ++k) fp_plain_to_be48(out + 576 * i + 96 * k + 48 * p, fp_from_mont(cs[k]->v));
}

__global__ void __launch_bounds__(KBLOCK, BLS_WAVES_PER_EU) k_fp12_from_bytes(size_t n, const uint8_t* __restrict__ in, uint32_t* __restrict__ f) {
  const size_t i = item_index<2>();
  if (i >= n) return;
  const int p = pr_odd() ? 1 : 0;
  fp12p_t a;
  fp2p_t* cs[6] = {&a.c0.c0, &a.c0.c1, &a.c0.c2, &a.c1.c0, &a.c1.c1, &a.c1.c2};
  for (int k = 0; k < 6; ++k) cs[k]->v = fp_to_mont(fp_plain_from_be48(in + 576 * i + 96 * k + 48 * p));
  soa_st12(f, n, i, a);
}

}  // namespace bls381
