// Lazy reduction: sums of Fp products accumulated in one signed double-width value
// and reduced once (DESIGN.md §5 "Lazy reduction").
//
// A wide value is 28 signed 64-bit columns, T = sum_k T[k] 2^(28k).  Products of
// signed 28/29-bit limbs accumulate in place (one v_mad_i64_i32 each), so a
// linear combination of products -- e.g. Re(a b) = a0 b0 - a1 b1, or a whole Fp2
// coefficient of an Fp6 product -- costs its products plus ONE Montgomery
// reduction, instead of one reduction per product plus a reduction per addition.
//
// wredc(T) requires -q 2^386 <= T < 2^390 q (checked by the callers' bounds):
// the columns 13..26 start at 2^22 q_j (an offset of q 2^386, a multiple of q, so
// the result is unchanged mod q) which makes the reduced value non-negative, and
// the result is normalized with value < q + (T + q 2^386) / 2^392.  Column
// bound: every column stays below 2^63 in magnitude (each caller states its sum).
//
// The per-lane functions below take the lane parity p and both coefficients of
// each Fp2 operand (e = c0, o = c1): the gfx950 kernels call them with p = the
// lane's parity in its pair and (e, o) read across the pair by DPP, the host build
// (fp2_t) calls them once per coefficient -- one source for both.
#pragma once
#include "bls381_field.hpp"

namespace bls381 {

struct wide_t { int64_t c[28]; };
typedef int32_t lv_t[14];   // a signed limb vector (|limb| < 2^30)

constexpr int WIDE_OFF_SHIFT = 22;   // offset q 2^(364 + 22) in columns 13..26

BLS_INLINE void wz_init(wide_t& T) {
#pragma unroll
  for (int k = 0; k < 28; ++k) T.c[k] = 0;
#pragma unroll
  for (int j = 0; j < 14; ++j) T.c[13 + j] = (int64_t)Q_LIMBS[j] << WIDE_OFF_SHIFT;
}

// BLS_LAZY_CSQR_V2 (default 1; 0 = the round-4 form, measurement knob): the compressed
// squaring's column offsets ride on each column's first product (wmac_init) and u = b0 -+ b1
// of lz_sqr_xisqr is squared unreduced (signed limbs)
#ifndef BLS_LAZY_CSQR_V2
#define BLS_LAZY_CSQR_V2 1
#endif

// T += x y  (signed limbs)
BLS_INLINE void wmac(wide_t& T, const lv_t& x, const lv_t& y) {
  BLS_COUNT_MACS(196);
#pragma unroll
  for (int i = 0; i < 14; ++i)
#pragma unroll
    for (int j = 0; j < 14; ++j) T.c[i + j] += (int64_t)x[i] * (int64_t)y[j];
}

// T = x y + the offset of wz_init: each column's first product takes the column's initial
// value as its addend (one v_mad with a scalar operand) instead of a separate move
BLS_INLINE void wmac_init(wide_t& T, const lv_t& x, const lv_t& y) {
#if !BLS_LAZY_CSQR_V2
  wz_init(T);
  wmac(T, x, y);
  return;
#endif
  BLS_COUNT_MACS(196);
#pragma unroll
  for (int i = 0; i < 14; ++i)
#pragma unroll
    for (int j = 0; j < 14; ++j) {
      const int k = i + j;
      const int64_t p = (int64_t)x[i] * (int64_t)y[j];
      if (i == 0 || j == 13)   // column k's first product in this order
        T.c[k] = p + ((k >= 13) ? ((int64_t)Q_LIMBS[k - 13] << WIDE_OFF_SHIFT) : 0);
      else
        T.c[k] += p;
    }
  T.c[27] = 0;
}

// T += k x^2 for a small signed k (105 products: cross terms doubled in the multiplier)
BLS_INLINE void wsqr_k(wide_t& T, const lv_t& x, int32_t k) {
  BLS_COUNT_MACS(105);
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    const int32_t d = k * x[i], c = 2 * k * x[i];
    T.c[2 * i] += (int64_t)d * (int64_t)x[i];
#pragma unroll
    for (int j = i + 1; j < 14; ++j) T.c[i + j] += (int64_t)c * (int64_t)x[j];
  }
}

// signed Montgomery reduction T 2^-392 mod q (see the header for the bounds)
BLS_INLINE fp_t wredc(wide_t& T) {
  BLS_COUNT_MACS(196);
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    const uint32_t m = ((uint32_t)T.c[i] * Q_INV28) & FP_MASK;
#pragma unroll
    for (int j = 0; j < 14; ++j) T.c[i + j] = (int64_t)((uint64_t)T.c[i + j] + (uint64_t)m * Q_LIMBS[j]);
    T.c[i + 1] += T.c[i] >> 28;
  }
  fp_t r;
  int64_t c = 0;
#pragma unroll
  for (int j = 0; j < 14; ++j) {
    const int64_t v = T.c[14 + j] + c;
    r.w[j] = (uint32_t)v & FP_MASK;
    c = v >> 28;
  }
  return r;
}

BLS_INLINE void lv_from(lv_t& r, const fp_t& a) {
#pragma unroll
  for (int k = 0; k < 14; ++k) r[k] = (int32_t)a.w[k];
}

// 6X + 2x (X < 1.03q and x < 2q normalized: < 10.2q, limbs <= 8 (2^28 - 1))
BLS_INLINE fp_t fp_6p2(const fp_t& X, const fp_t& x) {
  uint32_t s[14];
#pragma unroll
  for (int i = 0; i < 14; ++i) s[i] = 6u * X.w[i] + (x.w[i] << 1);
  return fp_reduce_lc<6>(s);
}

// six: 6 P + 2 x, else 3 S - 2 x (+ 4q), chosen per lane in one reduction (same bounds)
BLS_INLINE fp_t fp_6p2_3m2(bool six, const fp_t& P, const fp_t& S, const fp_t& x) {
  uint32_t s[14];
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    const uint32_t x2 = x.w[i] << 1;
    s[i] = six ? 6u * P.w[i] + x2 : 3u * S.w[i] + Q4B_LIMBS[i] - x2;
  }
  return fp_reduce_lc<6>(s);
}

// ---- Karabina compressed squaring, one output coefficient per call ----------
// (g2..g5) -> (g2'..g5') of cyc_csqr (bls381_pairing.hpp):
//   g2' = 6 xi g4 g5 + 2 g2          g3' = 3 (g4^2 + xi g5^2) - 2 g3
//   g4' = 3 (g2^2 + xi g3^2) - 2 g4  g5' = 6 g2 g3 + 2 g5
// with the products of each output summed in one wide value (lane p = coefficient p):
//   Re(xi a b) = a0 (b0 - b1) - a1 (b0 + b1)      Im(xi a b) = a0 (b0 + b1) + a1 (b0 - b1)
//   Re(a b) = a0 b0 - a1 b1                        Im(a b) = a0 b1 + a1 b0
//   a^2 + xi b^2: lz_sqr_xisqr below
// Inputs normalized (limbs < 2^28, values < 2q).  Column sums: xi a b and a b hold 28
// products < 2^57 (2^61.8); the reduction adds < 2^59.8.  Values: |X| < 16 q^2.

// Re/Im of xi a b
BLS_INLINE fp_t lz_xi_mul(bool p, const fp_t& a0, const fp_t& a1, const fp_t& b0, const fp_t& b1) {
  lv_t x1, y1, x2, y2;
#pragma unroll
  for (int k = 0; k < 14; ++k) {
    const int32_t s = (int32_t)b0.w[k] + (int32_t)b1.w[k];
    const int32_t d = (int32_t)b0.w[k] - (int32_t)b1.w[k];
    x1[k] = (int32_t)a0.w[k];
    x2[k] = (int32_t)a1.w[k];
    y1[k] = p ? s : d;
    y2[k] = p ? d : -s;
  }
  wide_t T;
  wmac_init(T, x1, y1);
  wmac(T, x2, y2);
  return wredc(T);
}

// Re/Im of a b
BLS_INLINE fp_t lz_mul(bool p, const fp_t& a0, const fp_t& a1, const fp_t& b0, const fp_t& b1) {
  lv_t x1, y1, x2, y2;
#pragma unroll
  for (int k = 0; k < 14; ++k) {
    x1[k] = (int32_t)a0.w[k];
    x2[k] = (int32_t)a1.w[k];
    y1[k] = (int32_t)(p ? b1.w[k] : b0.w[k]);
    y2[k] = p ? (int32_t)b0.w[k] : -(int32_t)b1.w[k];
  }
  wide_t T;
  wmac_init(T, x1, y1);
  wmac(T, x2, y2);
  return wredc(T);
}

// Re/Im of a^2 + xi b^2, with the xi b^2 part as squares:
//   Re(xi b^2) = (b0 - b1)^2 - 2 b1^2,  Im(xi b^2) = (b0 + b1)^2 - 2 b1^2
// 196 + 105 + 105 products per lane instead of 3 x 196.  u = b0 -+ b1 is squared as signed
// limbs, unreduced (round 5; it was reduced mod 2q first): |u_k| < 2^28 (lane 0) or
// u_k < 2^29 (lane 1).  Columns, lane 1 (all terms but 2 b1^2 non-negative): a-term
// 14 x 2^57 + u^2 15 x 2^58 + reduction 14 x 2^56 < 2^62.7, and -2 b1^2 > -2^60.9; lane 0 is
// smaller.  Values: lane 0 in (-16 q^2, 12 q^2), lane 1 in (-8 q^2, 24 q^2) (u < 4q), inside
// wredc's (-q 2^386, 2^390 q) ~ (-42 q^2, 675 q^2).
BLS_INLINE fp_t lz_sqr_xisqr(bool p, const fp_t& a0, const fp_t& a1, const fp_t& b0, const fp_t& b1) {
  lv_t x1, y1, u, v;
#pragma unroll
  for (int k = 0; k < 14; ++k) {
    const int32_t e = (int32_t)a0.w[k], o = (int32_t)a1.w[k];
    x1[k] = e + (p ? e : o);
    y1[k] = p ? o : e - o;
    const int32_t c = (int32_t)b0.w[k], d = (int32_t)b1.w[k];
    u[k] = p ? c + d : c - d;
    v[k] = d;
  }
#if !BLS_LAZY_CSQR_V2
  {
    uint32_t s[14];
#pragma unroll
    for (int k = 0; k < 14; ++k) s[k] = b0.w[k] + (p ? b1.w[k] : Q2B_LIMBS[k] - b1.w[k]);
    lv_from(u, fp_reduce_lc<2>(s));
  }
#endif
  wide_t T;
  wmac_init(T, x1, y1);
  wsqr_k(T, u, 1);
  wsqr_k(T, v, -2);
  return wredc(T);
}

}  // namespace bls381
