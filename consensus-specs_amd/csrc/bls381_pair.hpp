// Fp2 on an adjacent lane pair -- the representation the gfx950 kernels use.
//
// Lane 2i+p of a wavefront holds coefficient p of item i's Fp2 values (p = 0:
// real part c0, p = 1: imaginary part c1).  Every Fp2 operation is one Fp
// operation per lane plus DPP exchanges inside the pair (v_mov_b32_dpp
// quad_perm, full-rate VALU, no LDS), so:
//   * an item's Fp12 is 6 Fp per lane (84 VGPRs) instead of 12 (168), which is
//     what lets the Miller-loop and final-exponentiation kernels run two waves
//     per SIMD without spilling;
//   * a batch of n items launches 2n lanes: C2's 2^16 verifications fill 2048
//     waves, two per SIMD of the 1024 on an MI355X, instead of one;
//   * Fp2 products fold the subtraction of a0 b0 - a1 b1 into one Montgomery
//     reduction per lane (lane 0: a0 b0 + a1 (8q - b1); lane 1: a1 b0 + a0 b1).
// The tower, curve, hash and pairing formulas above this file are templates
// over the Fp2 representation and are shared with the one-lane fp2_t that the
// host unit-test build checks against the oracle.
//
// Control flow must stay uniform within a pair (both lanes take every branch
// together; DPP reads the partner's registers): every predicate on an Fp2 value
// is combined across the pair before it is returned.
#pragma once
#include <hip/hip_runtime.h>

// Issue priority of the two waves a SIMD holds (s_setprio).  Without it the older wave takes most
// issue slots and finishes first, and the younger runs the rest of its work alone at a lone wave's
// issue rate: in k_final_exp_verdict's shape the older wave of every SIMD ends at 6.2 ms, the
// younger at 9.4 (tools/fe_phases.hip, profiles/fe_balance_r06.txt).
//   BLS_WAVE_BALANCE=2 (default, round 6): in a launch that puts two waves on every SIMD, all resident
//     from the start (one round of two-wave slots), the priority alternates with the real-time clock
//     (windows of 2^BLS_BALANCE_SHIFT ticks of s_memrealtime's 100 MHz), so both waves hold it for
//     equal times: 8.5 / 9.0 ms.  It is updated before every lane-pair Fp2 product call and at the
//     loops' steps.  The host picks those launches (bls381_capi.hip, balance_lds) and marks every
//     other one with an LDS allocation, which the device reads with one s_getreg; those keep the
//     step-parity form of 1 at the loops' steps.  Same box, alternating (profiles/ab_r06p_balance.txt):
//     C2 +1.0 to +2.3 %; k_final_exp_verdict 8.79-8.94 -> 8.45-8.51 ms, k_ml_accum 6.88-6.96 ->
//     6.61-6.64, k_hash_bp 3.27-3.31 -> 3.19; k_ml_lines 6.03-6.08 -> 6.32-6.38 (its loop function's
//     allocation around the calls came out with more spill traffic).  k_ml_lines has static LDS, so
//     the switch is off in it; its launches are one round each and pass the choice as an argument
//     (bls381_kernels.hpp, ml_lines_run_lds).
//   BLS_WAVE_BALANCE=1 (round 4): alternate by step parity at the loops' steps only.  It does not
//     balance: a wave one step ahead has the same priority as the other, which the older wins.
#ifndef BLS_WAVE_BALANCE
#define BLS_WAVE_BALANCE 2
#endif
// 2^16 ticks = 655 us: against 2^14 (164 us), same box, C2 -0.2 to +2.3 %, k_ml_lines 6.21-6.32 ->
// 6.05-6.16 ms, FE 8.38-8.42 -> 8.27-8.33 (profiles/ab_r06st_balance_window.txt; 2^13 and 2^15 too)
#ifndef BLS_BALANCE_SHIFT
#define BLS_BALANCE_SHIFT 16
#endif
namespace bls381 {
__device__ __forceinline__ unsigned wave_slot() {
  return (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4) & 1u;   // HW_ID[3:0]: the wave's slot
}
// s_setprio ignores exec: the condition is made wave-uniform and the branch is a scalar one
__device__ __forceinline__ void wave_prio(unsigned x) {
  const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)((x + wave_slot()) & 1u));
  if (hi) __builtin_amdgcn_s_setprio(2); else __builtin_amdgcn_s_setprio(0);
}
__device__ __forceinline__ bool wave_has_lds() {
  return ((unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 6) >> 12) & 0x1ffu;   // HW_REG_LDS_ALLOC size
}
__device__ __forceinline__ unsigned balance_clock() {
  return (unsigned)(__builtin_amdgcn_s_memrealtime() >> BLS_BALANCE_SHIFT);
}
// at a loop step
__device__ __forceinline__ void wave_balance(unsigned step) {
#if BLS_WAVE_BALANCE == 2
  if (!wave_has_lds()) wave_prio(balance_clock());
  else wave_prio(step);
#elif BLS_WAVE_BALANCE == 1
  wave_prio(step);
#else
  (void)step;
#endif
}
// at a loop step of a kernel that always has an LDS allocation (the line loop): the step-parity form
__device__ __forceinline__ void wave_balance_lds(unsigned step) {
#if BLS_WAVE_BALANCE
  wave_prio(step);
#else
  (void)step;
#endif
}
// at an Fp2 product call
__device__ __forceinline__ void wave_balance_call() {
#if BLS_WAVE_BALANCE == 2
  if (!wave_has_lds()) wave_prio(balance_clock());
#endif
}
}  // namespace bls381
#if BLS_WAVE_BALANCE && !defined(BLS_FE_STEP)
#define BLS_FE_STEP(j) ::bls381::wave_balance((unsigned)(j))
#endif
#include "bls381_hash.hpp"
#include "bls381_pairing.hpp"

namespace bls381 {

// ------------------------------------------------------------ pair plumbing --
__device__ __forceinline__ bool pr_odd() { return (threadIdx.x & 1u) != 0; }

// DPP quad_perm controls: lane selects within each group of four lanes
enum : int {
  DPP_SWAP = 0xB1,   // [1,0,3,2]: the partner's value
  DPP_EVEN = 0xA0,   // [0,0,2,2]: the even lane's value (coefficient c0)
  DPP_ODD = 0xF5,    // [1,1,3,3]: the odd lane's value (coefficient c1)
};

template <int CTRL>
__device__ __forceinline__ uint32_t pr_dpp(uint32_t x) {
  // mov_dpp: no old value to initialise (every lane of the quad is a valid source)
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ fp_t pr_dpp(const fp_t& a) {
  fp_t r;
#pragma unroll
  for (int k = 0; k < FP_LIMBS; ++k) r.w[k] = pr_dpp<CTRL>(a.w[k]);
  return r;
}
// a predicate true on both lanes of the pair
__device__ __forceinline__ bool pr_both(bool b) { return (pr_dpp<DPP_SWAP>((uint32_t)b) & (uint32_t)b) != 0; }

__device__ __forceinline__ fp_t fp_sel(bool c, const fp_t& a, const fp_t& b) {
  fp_t r;
#pragma unroll
  for (int k = 0; k < FP_LIMBS; ++k) r.w[k] = c ? a.w[k] : b.w[k];
  return r;
}

// ------------------------------------------------------ Fp2 multiplication --
// lane 0: a0 b0 + a1 (8q - b1) = Re(ab);  lane 1: a1 b0 + a0 b1 = Im(ab).
// Operands may be lazy sums (limbs < 2^29, values < 4q).  Column k holds <= 14
// products < 2^58 plus <= 14 products < 2^59 and the reduction's 14 products
// < 2^56: < 2^63.5.  The sum is < 48 q^2 < q R, so the result is < 2q.
__device__ __forceinline__ fp_t fp2p_mul_body(const fp_t& a, const fp_t& b) {
  const bool odd = pr_odd();
  const fp_t ao = pr_dpp<DPP_SWAP>(a);
  const fp_t b0 = pr_dpp<DPP_EVEN>(b);
  const fp_t b1 = pr_dpp<DPP_ODD>(b);
  uint32_t w[14];
#pragma unroll
  for (int k = 0; k < 14; ++k) w[k] = odd ? b1.w[k] : Q8S_LIMBS[k] - b1.w[k];
  uint64_t T[28];
#pragma unroll
  for (int k = 0; k < 28; ++k) T[k] = 0;
#pragma unroll
  for (int i = 0; i < 14; ++i)
#pragma unroll
    for (int j = 0; j < 14; ++j) {
      T[i + j] += (uint64_t)a.w[i] * b0.w[j];
      T[i + j] += (uint64_t)ao.w[i] * w[j];
    }
  return fp_redc_wide(T);
}

// lane 0: (a0 + a1)(a0 + 8q - a1) = a0^2 - a1^2;  lane 1: (a0 + a0) a1 = 2 a0 a1.
// Operand normalized (< 2q); the factors stay within fp_mul_body's bounds
// (limbs < 2^29 and < 2^30.4, values < 4q and < 10q).
__device__ __forceinline__ fp_t fp2p_sqr_body(const fp_t& a) {
  const bool odd = pr_odd();
  const fp_t ao = pr_dpp<DPP_SWAP>(a);
  fp_t x, y;
#pragma unroll
  for (int k = 0; k < 14; ++k) {
    x.w[k] = ao.w[k] + (odd ? ao.w[k] : a.w[k]);
    y.w[k] = odd ? a.w[k] : a.w[k] + Q8S_LIMBS[k] - ao.w[k];
  }
  return fp_mul_body(x, y);
}

// The lane-pair Fp2 products are calls (operands and result in VGPRs, no frame): inlining them
// everywhere (round 2's BLS_FP2_INLINE=1) grew the callers' live sets, Miller 14.7-15.0 -> 16.9 ms;
// round 5's scheduling-fenced inlined form (BLS_FP2_INLINE=2) faulted.
// Both knobs were removed in round 6.
#define BLS_FP2_CALL __device__ __attribute__((noinline))
BLS_FP2_CALL fpv_t fp2p_mul_call(fpv_t a, fpv_t b) {
  return fp_pack(fp2p_mul_body(fp_unpack(a), fp_unpack(b)));
}
BLS_FP2_CALL fpv_t fp2p_sqr_call(fpv_t a) {
  return fp_pack(fp2p_sqr_body(fp_unpack(a)));
}

// ------------------------------------------------------------ Fp2 on a pair --
__device__ __forceinline__ fp2p_t pr_make(const fp_t& v) { fp2p_t r; r.v = v; return r; }

template <> BLS_INLINE fp2p_t e2_zero<fp2p_t>() { return pr_make(fp_zero()); }
template <> BLS_INLINE fp2p_t e2_one<fp2p_t>() { return pr_make(fp_sel(pr_odd(), fp_zero(), FP_ONE_M)); }
template <> BLS_INLINE fp2p_t e2_k<fp2p_t>(const fp2_t& k) { return pr_make(fp_sel(pr_odd(), k.c1, k.c0)); }

__device__ __forceinline__ fp2p_t fp2_add(const fp2p_t& a, const fp2p_t& b) { return pr_make(fp_add(a.v, b.v)); }
__device__ __forceinline__ fp2p_t fp2_sub(const fp2p_t& a, const fp2p_t& b) { return pr_make(fp_sub(a.v, b.v)); }
__device__ __forceinline__ fp2p_t fp2_neg(const fp2p_t& a) { return pr_make(fp_neg(a.v)); }
__device__ __forceinline__ fp2p_t fp2_dbl(const fp2p_t& a) { return pr_make(fp_dbl(a.v)); }
__device__ __forceinline__ fp2p_t fp2_half(const fp2p_t& a) { return pr_make(fp_half(a.v)); }
__device__ __forceinline__ fp2p_t fp2_add_lazy(const fp2p_t& a, const fp2p_t& b) { return pr_make(fp_add_lazy(a.v, b.v)); }
__device__ __forceinline__ fp2p_t fp2_mul_fp(const fp2p_t& a, const fp_t& s) { return pr_make(fp_mul(a.v, s)); }
__device__ __forceinline__ fp2p_t fp2_mul_small(const fp2p_t& a, int k) { return pr_make(fp_mul_small(a.v, k)); }
__device__ __forceinline__ fp2p_t fp2_conj(const fp2p_t& a) { return pr_make(fp_sel(pr_odd(), fp_neg(a.v), a.v)); }
// xi = 1 + u:  (a0 - a1) + (a0 + a1) u -- lane 0: a0 + (2q - a1), lane 1: a1 + a0
__device__ __forceinline__ fp2p_t fp2_mul_xi(const fp2p_t& a) {
  const bool odd = pr_odd();
  const fp_t ao = pr_dpp<DPP_SWAP>(a.v);
  uint32_t s[14];
#pragma unroll
  for (int i = 0; i < 14; ++i) s[i] = a.v.w[i] + (odd ? ao.w[i] : Q2B_LIMBS[i] - ao.w[i]);
  return pr_make(fp_reduce_lc<2>(s));
}
// a + xi b -- lane 0: a0 + b0 + (2q - b1), lane 1: a1 + b1 + b0 (one reduction)
__device__ __forceinline__ fp2p_t fp2_add_mul_xi(const fp2p_t& a, const fp2p_t& b) {
  const bool odd = pr_odd();
  const fp_t bo = pr_dpp<DPP_SWAP>(b.v);
  uint32_t s[14];
#pragma unroll
  for (int i = 0; i < 14; ++i) s[i] = a.v.w[i] + b.v.w[i] + (odd ? bo.w[i] : Q2B_LIMBS[i] - bo.w[i]);
  return pr_make(fp_reduce_lc<3>(s));
}
__device__ __forceinline__ fp2p_t fp2_sub2(const fp2p_t& a, const fp2p_t& b, const fp2p_t& c) {
  return pr_make(fp_sub2(a.v, b.v, c.v));
}
__device__ __forceinline__ fp2p_t fp2_3m2(const fp2p_t& X, const fp2p_t& x) { return pr_make(fp_3m2(X.v, x.v)); }
__device__ __forceinline__ fp2p_t fp2_3p2(const fp2p_t& X, const fp2p_t& x) { return pr_make(fp_3p2(X.v, x.v)); }
__device__ __forceinline__ fp2p_t fp2_3pm2(const fp2p_t& X, const fp2p_t& x, bool minus) {
  return pr_make(fp_3pm2(X.v, x.v, minus));
}
__device__ __forceinline__ fp2p_t fp2_mul(const fp2p_t& a, const fp2p_t& b) {
  // at the call site, not in the callee: k_final_exp_verdict 8.42-8.54 -> 8.31-8.33 ms, its scratch
  // frame 7,824 -> 7,440 B/lane (profiles/ab_r06q_balance_site.txt)
  wave_balance_call();
  return pr_make(fp_unpack(fp2p_mul_call(fp_pack(a.v), fp_pack(b.v))));
}
__device__ __forceinline__ fp2p_t fp2_sqr(const fp2p_t& a) {
  wave_balance_call();
  return pr_make(fp_unpack(fp2p_sqr_call(fp_pack(a.v))));
}
__device__ __forceinline__ bool fp2_is_zero(const fp2p_t& a) { return pr_both(fp_is_zero(a.v)); }
__device__ __forceinline__ bool fp2_eq(const fp2p_t& a, const fp2p_t& b) { return pr_both(fp_eq(a.v, b.v)); }

// Karabina compressed squaring with lazy reduction (bls381_lazy.hpp): lane p computes
// coefficient p of every output from both coefficients of the inputs (DPP).  The (g4, g5)
// outputs come first so only one input pair is read across the lanes at a time.
__device__ __forceinline__ cyc_bc<fp2p_t> cyc_csqr_lazy(const cyc_bc<fp2p_t>& g) {
  const bool p = pr_odd();
  cyc_bc<fp2p_t> r;
  {
    const fp_t e4 = pr_dpp<DPP_EVEN>(g.g4.v), o4 = pr_dpp<DPP_ODD>(g.g4.v);
    const fp_t e5 = pr_dpp<DPP_EVEN>(g.g5.v), o5 = pr_dpp<DPP_ODD>(g.g5.v);
    r.g2 = pr_make(fp_6p2(lz_xi_mul(p, e4, o4, e5, o5), g.g2.v));
    r.g3 = pr_make(fp_3m2(lz_sqr_xisqr(p, e4, o4, e5, o5), g.g3.v));
  }
  const fp_t e2 = pr_dpp<DPP_EVEN>(g.g2.v), o2 = pr_dpp<DPP_ODD>(g.g2.v);
  const fp_t e3 = pr_dpp<DPP_EVEN>(g.g3.v), o3 = pr_dpp<DPP_ODD>(g.g3.v);
  r.g4 = pr_make(fp_3m2(lz_sqr_xisqr(p, e2, o2, e3, o3), g.g4.v));
  r.g5 = pr_make(fp_6p2(lz_mul(p, e2, o2, e3, o3), g.g5.v));
  return r;
}

// 1/x for an x both lanes of the pair hold (the norm of an Fp2 inverse): fp_inv's optimized
// binary GCD (bls381_field.hpp) with each round's two row updates split over the pair.  Both
// lanes run the same 30-step inner loop on the same approximations; lane 0 then applies the row
// (f0, g0) -- the new a and u -- and lane 1 the row (f1, g1) -- the new b and v -- and each reads
// the other's row by DPP.  Lane-relative: X = this lane's row, Y = the partner's, so lane 0 has
// (X, Y, U, V) = (a, b, u, v) and lane 1 (b, a, v, u), and both apply the same code with
// (cX, cY) = (f0, g0) on lane 0 and (g1, f1) on lane 1.  Half of fp_inv's full-width work per lane.
#ifndef BLS_INV_PAIR
#define BLS_INV_PAIR 1
#endif
__device__ inline fp_t fp_inv_pair(const fp_t am) {
  const bool odd = pr_odd();
  uint32_t w[12];
  fp_plain_to_words(w, fp_reduce_once(am));
  uint32_t z = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) z |= w[i];
  if (z == 0) return fp_zero();   // both lanes of the pair hold the same x
  int32_t A[INV_L], X[INV_L], Y[INV_L], U[INV_L], V[INV_L];
  inv_to_l30(A, w);
#pragma unroll
  for (int i = 0; i < INV_L; ++i) {
    X[i] = odd ? Q_L30[i] : A[i];
    Y[i] = odd ? A[i] : Q_L30[i];
    U[i] = 0;
    V[i] = 0;
  }
  if (odd) V[0] = 1; else U[0] = 1;   // u = 1, v = 0
  for (int round = 0; round < 26; ++round) {
    int t = 2;
    uint32_t top = 0;
#pragma unroll
    for (int i = 2; i < INV_L; ++i) {
      const uint32_t c = (uint32_t)(X[i] | Y[i]);
      if (c) { t = i; top = c; }
    }
    const int bl = top ? 32 - __builtin_clz(top) : 2;
    uint32_t x2 = 0, x1 = 0, x0 = 0, y2 = 0, y1 = 0, y0 = 0;
#pragma unroll
    for (int i = 2; i < INV_L; ++i) {
      const bool s = i == t;
      x2 = s ? (uint32_t)X[i] : x2; x1 = s ? (uint32_t)X[i - 1] : x1; x0 = s ? (uint32_t)X[i - 2] : x0;
      y2 = s ? (uint32_t)Y[i] : y2; y1 = s ? (uint32_t)Y[i - 1] : y1; y0 = s ? (uint32_t)Y[i - 2] : y0;
    }
    // a = lane 0's X / lane 1's Y, b the other
    const uint32_t a2 = odd ? y2 : x2, a1 = odd ? y1 : x1, a0 = odd ? y0 : x0;
    const uint32_t b2 = odd ? x2 : y2, b1 = odd ? x1 : y1, b0 = odd ? x0 : y0;
    const uint32_t al0 = (uint32_t)(odd ? Y[0] : X[0]), bl0 = (uint32_t)(odd ? X[0] : Y[0]);
    const uint32_t al1 = (uint32_t)(odd ? Y[1] : X[1]), bl1 = (uint32_t)(odd ? X[1] : Y[1]);
    const uint32_t al2 = (uint32_t)(odd ? Y[2] : X[2]), bl2 = (uint32_t)(odd ? X[2] : Y[2]);
    const uint64_t wa = ((uint64_t)a2 << 31) | ((uint64_t)a1 << 1) | (a0 >> 29);
    const uint64_t wb = ((uint64_t)b2 << 31) | ((uint64_t)b1 << 1) | (b0 >> 29);
    uint64_t xa = ((wa >> (bl - 1)) << 30) | al0;
    uint64_t xb = ((wb >> (bl - 1)) << 30) | bl0;
    if (t == 2 && bl <= 2) {
      xa = al0 | ((uint64_t)al1 << 30) | ((uint64_t)al2 << 60);
      xb = bl0 | ((uint64_t)bl1 << 30) | ((uint64_t)bl2 << 60);
    }
    int32_t f0 = 1, g0 = 0, f1 = 0, g1 = 1;
#pragma unroll 10
    for (int j = 0; j < 30; ++j) {
      const bool od = (xa & 1) != 0;
      const bool sw = od && xa < xb;
      const uint64_t ta = sw ? xb : xa, tb = sw ? xa : xb;
      const int32_t tf0 = sw ? f1 : f0, tg0 = sw ? g1 : g0, tf1 = sw ? f0 : f1, tg1 = sw ? g0 : g1;
      xa = (od ? ta - tb : ta) >> 1;
      xb = tb;
      f0 = od ? tf0 - tf1 : tf0;
      g0 = od ? tg0 - tg1 : tg0;
      f1 = tf1 + tf1;
      g1 = tg1 + tg1;
    }
    int32_t cX = odd ? g1 : f0, cY = odd ? f1 : g0;
    int32_t nX[INV_L], nU[INV_L];
    inv_lin_shift(nX, X, Y, cX, cY);
    if (nX[INV_L - 1] < 0) { inv_neg(nX); cX = -cX; cY = -cY; }
    inv_lin_modq(nU, U, V, cX, cY);
#pragma unroll
    for (int i = 0; i < INV_L; ++i) {
      X[i] = nX[i];
      Y[i] = (int32_t)pr_dpp<DPP_SWAP>((uint32_t)nX[i]);
      U[i] = nU[i];
      V[i] = (int32_t)pr_dpp<DPP_SWAP>((uint32_t)nU[i]);
    }
  }
  // done when a == 0 and b == 1; the inverse is v (lane 0's V, lane 1's U)
  uint32_t bad = 0;
#pragma unroll
  for (int i = 0; i < INV_L; ++i) {
    const uint32_t a = (uint32_t)(odd ? Y[i] : X[i]), b = (uint32_t)(odd ? X[i] : Y[i]);
    bad |= a | (i ? b : b ^ 1u);
  }
  if (BLS_ANY(bad != 0)) return fp_inv_xgcd(am);
  fp_t r;
#pragma unroll
  for (int k = 0; k < 14; ++k) {
    const int bit = 28 * k, i = bit / 30, sh = bit % 30;
    uint64_t x = (uint64_t)(uint32_t)(odd ? U[i] : V[i]) >> sh;
    if (i + 1 < INV_L) x |= (uint64_t)(uint32_t)(odd ? U[i + 1] : V[i + 1]) << (30 - sh);
    r.w[k] = (uint32_t)x & FP_MASK;
  }
  return fp_mul(r, FP_R3);
}

// 1/a = conj(a) / (a0^2 + a1^2); the norm (the same on both lanes) is inverted by the pair
__device__ inline fp2p_t fp2_inv(const fp2p_t a) {
  const fp_t t = fp_sqr(a.v);
#if BLS_INV_PAIR
  const fp_t ni = fp_inv_pair(fp_add(t, pr_dpp<DPP_SWAP>(t)));
#else
  const fp_t ni = fp_inv(fp_add(t, pr_dpp<DPP_SWAP>(t)));
#endif
  const fp_t r = fp_mul(a.v, ni);
  return pr_make(fp_sel(pr_odd(), fp_neg(r), r));
}

// a^((q-3)/4) = a^(q >> 2) for an a held on both lanes of the pair, right to left: the even lane
// squares a^(2^i), the odd lane multiplies the set bits' powers (broadcast by DPP) into the
// product, so each of the 379 exponent bits costs one product time, against 375 squarings + 86
// products when both lanes run fp_pow_qm3d4's window chain (BLS_POW_PAIR=0).  The exponent is a
// constant: the bit tests are wave-uniform (scalar branches).  Result on both lanes.
#ifndef BLS_POW_PAIR
#define BLS_POW_PAIR 1
#endif
__device__ __noinline__ fp_t fp_pow_qm3d4_pair(const fp_t a) {
#if BLS_POW_PAIR
  const bool odd = pr_odd();
  fp_t r = odd ? FP_ONE_M : a;   // even lane: a^(2^i); odd lane: the running product
#pragma unroll 1
  for (int i = 0; i < 379; ++i) {
    const int b = i + 2;
    const fp_t pw = pr_dpp<DPP_EVEN>(r);
    if ((Q_LIMBS[b / 28] >> (b % 28)) & 1u)
      r = fp_mul(odd ? r : pw, pw);
    else
      r = fp_sel(odd, r, fp_sqr(r));
  }
  return pr_dpp<DPP_ODD>(r);
#else
  return fp_pow_qm3d4(a);
#endif
}

__device__ __forceinline__ bool fp_sqrt_pair(fp_t& r, const fp_t& a) {
  r = fp_mul(fp_pow_qm3d4_pair(a), a);
  return fp_eq(fp_sqr(r), a);
}

// Complex-method square root (same steps as the one-lane fp2_sqrt, so the
// spec's selection rule picks the same root).  With gamma = sqrt(a0^2 + a1^2)
// and delta = (a0 + gamma)/2 (both lanes), t = delta^((q+1)/4) and 1/t come
// from one power of delta; the root is (t, a1/(2t)) when t^2 = delta and
// (a1/(2t), t) otherwise.
__device__ __forceinline__ bool fp2_sqrt(fp2p_t& r, const fp2p_t& a) {
  const bool odd = pr_odd();
  const fp_t a0 = pr_dpp<DPP_EVEN>(a.v);
  const fp_t a1 = pr_dpp<DPP_ODD>(a.v);
  if (fp_is_zero(a1)) {
    // even lane: sqrt(a0) -> (s, 0);  odd lane: sqrt(-a0) -> (0, s)
    fp_t s;
    const bool ok = fp_sqrt(s, odd ? fp_neg(a0) : a0);
    const bool ok0 = pr_dpp<DPP_EVEN>((uint32_t)ok) != 0;
    const bool ok1 = pr_dpp<DPP_ODD>((uint32_t)ok) != 0;
    if (ok0) { r.v = odd ? fp_zero() : s; return true; }
    if (ok1) { r.v = odd ? s : fp_zero(); return true; }
    return false;
  }
  const fp_t t2 = fp_sqr(a.v);
  const fp_t alpha = fp_add(t2, pr_dpp<DPP_SWAP>(t2));
  fp_t gamma;
  if (!fp_sqrt_pair(gamma, alpha)) return false;
  const fp_t delta = fp_half(fp_add(a0, gamma));
  const fp_t u = fp_pow_qm3d4_pair(delta);
  const fp_t t = fp_mul(u, delta);                                   // delta^((q+1)/4)
  const fp_t other = fp_mul(a1, fp_half(fp_mul(fp_sqr(u), t)));     // a1 / (2t)
  const bool sq = fp_eq(fp_sqr(t), delta);
  r.v = (sq != odd) ? t : other;
  return true;
}

// curve-generic helpers (bls381_curve.hpp) for the pair representation
__device__ __forceinline__ fp2p_t f_add(const fp2p_t& a, const fp2p_t& b) { return fp2_add(a, b); }
__device__ __forceinline__ fp2p_t f_sub(const fp2p_t& a, const fp2p_t& b) { return fp2_sub(a, b); }
__device__ __forceinline__ fp2p_t f_mul(const fp2p_t& a, const fp2p_t& b) { return fp2_mul(a, b); }
__device__ __forceinline__ fp2p_t f_sqr(const fp2p_t& a) { return fp2_sqr(a); }
__device__ __forceinline__ fp2p_t f_dbl(const fp2p_t& a) { return fp2_dbl(a); }
__device__ __forceinline__ fp2p_t f_neg(const fp2p_t& a) { return fp2_neg(a); }
__device__ __forceinline__ fp2p_t f_sub2(const fp2p_t& a, const fp2p_t& b, const fp2p_t& c) { return fp2_sub2(a, b, c); }
__device__ __forceinline__ fp2p_t f_mul_small(const fp2p_t& a, int k) { return fp2_mul_small(a, k); }
__device__ __forceinline__ bool f_is_zero(const fp2p_t& a) { return fp2_is_zero(a); }
__device__ __forceinline__ bool f_eq(const fp2p_t& a, const fp2p_t& b) { return fp2_eq(a, b); }
__device__ __forceinline__ fp2p_t f_inv(const fp2p_t& a) { return fp2_inv(a); }
__device__ __forceinline__ void f_set_zero(fp2p_t& a) { a = e2_zero<fp2p_t>(); }
__device__ __forceinline__ void f_set_one(fp2p_t& a) { a = e2_one<fp2p_t>(); }

// --------------------------------------------------------------- G2 codec --
// a_flag rule of py_ecc compress/decompress_G2: from y_im, or y_re if y_im == 0
__device__ __forceinline__ int g2_y_flag(const fp2p_t& y_mont) {
  const fp_t yc = fp_from_mont(y_mont.v);
  const uint32_t up = fp_plain_is_upper_half(yc) ? 1u : 0u;
  const uint32_t z = fp_is_zero(yc) ? 1u : 0u;
  const uint32_t up0 = pr_dpp<DPP_EVEN>(up), up1 = pr_dpp<DPP_ODD>(up), z1 = pr_dpp<DPP_ODD>(z);
  return (int)(z1 ? up0 : up1);
}

// G2 decompress (bls_signature.md:54-64 / py_ecc decompress_G2, bls381_curve.hpp):
// z1 = flags | x_im (odd lane), z2 = x_re (even lane; lax: all 384 bits, reduced mod q)
__device__ __forceinline__ int g2_decompress(aff_t<fp2p_t>& out, const uint8_t* b96, bool lax) {
  const bool odd = pr_odd();
  const uint8_t top = b96[0];
  const int b1 = (top >> 6) & 1, a1 = (top >> 5) & 1;
  if (!lax && !g2_canonical(b96)) return PT_BAD;
  if (b1) return PT_INF;
  uint8_t tmp[48];
  const uint8_t* src = b96 + (odd ? 0 : 48);
  for (int i = 0; i < 48; ++i) tmp[i] = src[i];
  if (odd) tmp[0] &= 0x1f;
  const fp_t xc = fp_plain_from_be48(tmp);
  fp2p_t x;
  x.v = fp_to_mont(xc);
  const fp2p_t rhs = fp2_add(fp2_mul(fp2_sqr(x), x), e2_k<fp2p_t>(G2_B_M));
  fp2p_t y;
  if (!fp2_sqrt(y, rhs)) return PT_BAD;
  if (g2_y_flag(y) != a1) y = fp2_neg(y);
  out.x = x;
  out.y = y;
  return PT_OK;
}

// each lane writes its 48-byte half of the 96-byte encoding at out96
__device__ __forceinline__ void g2_compress_aff(uint8_t* out96, const aff_t<fp2p_t>& a) {
  const bool odd = pr_odd();
  const int flag = g2_y_flag(a.y);
  uint8_t b[48];
  fp_plain_to_be48(b, fp_from_mont(a.x.v));
  if (odd) b[0] |= 0x80 | (flag ? 0x20 : 0);
  uint8_t* dst = out96 + (odd ? 0 : 48);
  for (int i = 0; i < 48; ++i) dst[i] = b[i];
}

__device__ __forceinline__ void g2_compress(uint8_t* out96, const jac_t<fp2p_t>& p) {
  aff_t<fp2p_t> a;
  if (!jac_to_aff(a, p)) {
    const bool odd = pr_odd();
    uint8_t* dst = out96 + (odd ? 0 : 48);
    for (int i = 0; i < 48; ++i) dst[i] = 0;
    if (odd) dst[0] = 0xc0;
    return;
  }
  g2_compress_aff(out96, a);
}

// ------------------------------------------------------------ hash_to_G2 --
// try-and-increment (bls_signature.md:74-86) before the cofactor: the even lane
// hashes m || dom8 || 0x01 (x_re), the odd lane m || dom8 || 0x02 (x_im).
// known_k >= 0: the candidate offset is already known (k_hash_search found the first
// square, x + known_k), so the Legendre search is skipped.
__device__ __forceinline__ int hash_to_g2_candidate(aff_t<fp2p_t>& out, const uint8_t* msg, uint32_t mlen,
                                           const uint8_t dom8[8], int known_k = -1) {
  const bool odd = pr_odd();
  uint32_t d[8];
  sha256_msg_dom_tag(d, msg, mlen, dom8, odd ? 2 : 1);
  fp2p_t x;
  x.v = fp_to_mont(fp_plain_from_digest(d));
  const fp_t inc = fp_sel(odd, fp_zero(), FP_ONE_M);   // x += 1 (real part)
  // Search with the cheap Legendre test only, then take one square root after
  // the loop: inside the loop the root's exponentiations would run (under a
  // partial exec mask) in every trial in which any lane of the wave succeeds.
  // rhs is a square in Fp2 iff its norm is a square in Fp.  Each round tests two
  // consecutive candidates, one Legendre symbol per lane (lane 0: x, lane 1: x + 1),
  // and keeps the first square in candidate order: the spec's x, in half the
  // sequential Legendre evaluations.
  int trials = 0;
  fp2p_t rhs;
  if (known_k >= 0) {
    for (int j = 0; j < known_k; ++j) x.v = fp_add(x.v, inc);
    rhs = fp2_add(fp2_mul(fp2_sqr(x), x), e2_k<fp2p_t>(G2_B_M));
    trials = known_k + 1;
  }
  while (known_k < 0) {
    trials += 2;
    const fp2p_t x1 = pr_make(fp_add(x.v, inc));
    const fp2p_t r0 = fp2_add(fp2_mul(fp2_sqr(x), x), e2_k<fp2p_t>(G2_B_M));
    const fp2p_t r1 = fp2_add(fp2_mul(fp2_sqr(x1), x1), e2_k<fp2p_t>(G2_B_M));
    const fp_t t0 = fp_sqr(r0.v), t1 = fp_sqr(r1.v);
    const fp_t n0 = fp_add(t0, pr_dpp<DPP_SWAP>(t0)), n1 = fp_add(t1, pr_dpp<DPP_SWAP>(t1));
    const uint32_t sq = fp_legendre(odd ? n1 : n0) >= 0 ? 1u : 0u;
    const bool ok0 = pr_dpp<DPP_EVEN>(sq) != 0, ok1 = pr_dpp<DPP_ODD>(sq) != 0;
    if (ok0) { rhs = r0; break; }
    if (ok1) { x = x1; rhs = r1; break; }
    x.v = fp_add(x1.v, inc);
  }
  fp2p_t y;
  fp2_sqrt(y, rhs);   // succeeds: rhs is a square
  out.x = x;
  out.y = g2_select_root(y);
  return trials;
}

}  // namespace bls381
