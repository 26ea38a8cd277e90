// BLS12-381 base field Fp and the tower Fp2 / Fp6 / Fp12.
//
// Fp: 14 limbs x 28 bits, Montgomery form R = 2^392.  Every 28x28-bit partial
// product accumulates in place into a 64-bit column (one v_mad_u64_u32, no
// carry chain); carries are resolved once per reduction row.
// Tower (DESIGN.md "Data layout"):  Fp2 = Fp[u]/(u^2+1),
// Fp6 = Fp2[v]/(v^3 - (1+u)),  Fp12 = Fp6[w]/(w^2 - v)  (w^6 = 1+u).
// Algorithms are mirrored 1:1 by oracle/tower_model.py (test infrastructure).
#pragma once
#include "bls381_defs.hpp"
#include "bls381_consts.hpp"

namespace bls381 {

#if defined(BLS_COUNT_OPS) && !defined(__HIP_DEVICE_COMPILE__)
// host op-count build (bench.py roofline): the 28x28-bit partial products (MACs) of the
// Fp products executed, each counted by the MACs it issues -- fp_mul 392 (196 product +
// 196 reduction), fp_sqr 301 (105 + 196), and in the lazy forms (bls381_lazy.hpp) wmac
// 196, wsqr_k 105, wredc 196.  bench.py divides by 392 for Fp-product equivalents.
inline thread_local uint64_t g_fp_macs = 0;
#define BLS_COUNT_MACS(k) (g_fp_macs += (k))
#else
#define BLS_COUNT_MACS(k) ((void)0)
#endif
#if !defined(__HIP_DEVICE_COMPILE__) && !defined(__HIP__)
// host build: inversions that took fp_inv's fallback (tests assert none do)
inline uint64_t g_inv_fallbacks = 0;
#define BLS_COUNT_INV_FALLBACK() (++g_inv_fallbacks)
#else
#define BLS_COUNT_INV_FALLBACK() ((void)0)
#endif

// ----------------------------------------------------------------- Fp -----
// Invariant for every fp_t crossing a function boundary: limbs < 2^28
// ("normalized") and value < 2q ("weakly reduced").  Canonical (< q) form is
// produced only where bits matter (codecs, comparisons).
BLS_INLINE fp_t fp_zero() { fp_t r; for (int i = 0; i < 14; ++i) r.w[i] = 0; return r; }
BLS_INLINE fp_t fp_one() { return FP_ONE_M; }

// signed carry propagation: limbs -> [0, 2^28) except the top limb, which
// keeps the (possibly negative) high part
BLS_INLINE void fp_carry(int32_t (&t)[14]) {
#pragma unroll
  for (int i = 0; i < 13; ++i) {
    t[i + 1] += t[i] >> 28;
    t[i] &= (int32_t)FP_MASK;
  }
}

// One reduction per linear combination (DESIGN.md "Arithmetic").  s is a
// non-negative combination of normalized values -- limbs 0..12 in [0, 2^31 - 8],
// the top limb >= -2 (a subtracted top limb may exceed the borrowed constant's by
// up to 2), value in [0, KMAX * 2q) with KMAX <= 8 -- and the result is s mod 2q,
// normalized: the unique value in [0, 2q), so bit-identical to any chain of
// two-operand additions and subtractions over the same terms.
//   k = floor(s13 / (Q2_13 + 1)) is at most floor(s / 2q) (no carry has been
//   propagated into limb 13 yet, and 2q < (Q2_13 + 1) 2^364) and at least
//   floor(s / 2q) - 1 (the carries into limb 13 are <= 8), so after s - k 2q and
//   one carry pass the value is in [0, 4q).  A value >= 2q has top limb >= Q2_13;
//   that (about one lane in 2^14) takes the exact conditional subtraction under a
//   wave-uniform branch.
template <int KMAX>
BLS_INLINE fp_t fp_reduce_lc(const uint32_t (&s)[14]) {
  static_assert(KMAX >= 1 && KMAX <= 8, "value bound");
  int32_t t[14];
  if (KMAX <= 2) {          // k in {0, 1}
    const uint32_t m = (int32_t)s[13] > (int32_t)Q2_LIMBS[13] ? ~0u : 0u;
#pragma unroll
    for (int i = 0; i < 14; ++i) t[i] = (int32_t)(s[i] - (Q2_LIMBS[i] & m));
  } else {                  // k <= 7: s_i - k q2_i < 2^31 in magnitude
    const int32_t top = (int32_t)s[13] > 0 ? (int32_t)s[13] : 0;   // < 0: value < 2q, k = 0
    const uint32_t k = (uint32_t)(((uint64_t)(uint32_t)top * LC_DIV_MAGIC) >> 40);
#pragma unroll
    for (int i = 0; i < 14; ++i) t[i] = (int32_t)(s[i] + k * NQ2_LIMBS[i]);
  }
  fp_carry(t);
  if (BLS_ANY(t[13] >= (int32_t)Q2_LIMBS[13])) {
    int32_t e[14];
#pragma unroll
    for (int i = 0; i < 14; ++i) e[i] = t[i] - (int32_t)Q2_LIMBS[i];
    fp_carry(e);
    const bool ge = e[13] >= 0;
#pragma unroll
    for (int i = 0; i < 14; ++i) t[i] = ge ? e[i] : t[i];
  }
  fp_t r;
#pragma unroll
  for (int i = 0; i < 14; ++i) r.w[i] = (uint32_t)t[i];
  return r;
}

// a + b (< 4q)
BLS_INLINE fp_t fp_add(const fp_t& a, const fp_t& b) {
  uint32_t s[14];
#pragma unroll
  for (int i = 0; i < 14; ++i) s[i] = a.w[i] + b.w[i];
  return fp_reduce_lc<2>(s);
}

// a - b + 2q (in (0, 4q)); Q2B's limbs are >= 2^28 - 1 >= b's, so no limb goes negative
BLS_INLINE fp_t fp_sub(const fp_t& a, const fp_t& b) {
  uint32_t s[14];
#pragma unroll
  for (int i = 0; i < 14; ++i) s[i] = a.w[i] + Q2B_LIMBS[i] - b.w[i];
  return fp_reduce_lc<2>(s);
}

BLS_INLINE fp_t fp_neg(const fp_t& a) {
  uint32_t s[14];
#pragma unroll
  for (int i = 0; i < 14; ++i) s[i] = Q2B_LIMBS[i] - a.w[i];
  return fp_reduce_lc<2>(s);
}

BLS_INLINE fp_t fp_dbl(const fp_t& a) {
  uint32_t s[14];
#pragma unroll
  for (int i = 0; i < 14; ++i) s[i] = a.w[i] << 1;
  return fp_reduce_lc<2>(s);
}

// a + b - c (< 6q)
BLS_INLINE fp_t fp_add_sub(const fp_t& a, const fp_t& b, const fp_t& c) {
  uint32_t s[14];
#pragma unroll
  for (int i = 0; i < 14; ++i) s[i] = a.w[i] + b.w[i] + Q2B_LIMBS[i] - c.w[i];
  return fp_reduce_lc<3>(s);
}

// a + b + c (< 6q)
BLS_INLINE fp_t fp_add3(const fp_t& a, const fp_t& b, const fp_t& c) {
  uint32_t s[14];
#pragma unroll
  for (int i = 0; i < 14; ++i) s[i] = a.w[i] + b.w[i] + c.w[i];
  return fp_reduce_lc<3>(s);
}

// a - b - c + 4q (in (0, 6q)); Q4B's limbs are >= 2^29 - 2 >= b_i + c_i
BLS_INLINE fp_t fp_sub2(const fp_t& a, const fp_t& b, const fp_t& c) {
  uint32_t s[14];
#pragma unroll
  for (int i = 0; i < 14; ++i) s[i] = a.w[i] + Q4B_LIMBS[i] - b.w[i] - c.w[i];
  return fp_reduce_lc<3>(s);
}

// 3X - 2x + 4q (in (0, 10q)) and 3X + 2x (< 10q): Granger-Scott outputs
BLS_INLINE fp_t fp_3m2(const fp_t& X, const fp_t& x) {
  uint32_t s[14];
#pragma unroll
  for (int i = 0; i < 14; ++i) s[i] = 3u * X.w[i] + Q4B_LIMBS[i] - (x.w[i] << 1);
  return fp_reduce_lc<5>(s);
}
BLS_INLINE fp_t fp_3p2(const fp_t& X, const fp_t& x) {
  uint32_t s[14];
#pragma unroll
  for (int i = 0; i < 14; ++i) s[i] = 3u * X.w[i] + (x.w[i] << 1);
  return fp_reduce_lc<5>(s);
}
// 3X - 2x (minus) or 3X + 2x, chosen per lane (same bounds as fp_3m2 / fp_3p2)
BLS_INLINE fp_t fp_3pm2(const fp_t& X, const fp_t& x, bool minus) {
  uint32_t s[14];
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    const uint32_t x2 = x.w[i] << 1;
    s[i] = 3u * X.w[i] + (minus ? Q4B_LIMBS[i] - x2 : x2);
  }
  return fp_reduce_lc<5>(s);
}

// lazy sum for a multiplication operand only: limbs < 2^29, value < 4q
BLS_INLINE fp_t fp_add_lazy(const fp_t& a, const fp_t& b) {
  fp_t r;
#pragma unroll
  for (int i = 0; i < 14; ++i) r.w[i] = a.w[i] + b.w[i];
  return r;
}

// value < 2q -> value < q (canonical)
BLS_INLINE fp_t fp_reduce_once(const fp_t& s) {
  int32_t b[14];
#pragma unroll
  for (int i = 0; i < 14; ++i) b[i] = (int32_t)s.w[i] - (int32_t)Q_LIMBS[i];
  fp_carry(b);
  const bool neg = b[13] < 0;
  fp_t r;
#pragma unroll
  for (int i = 0; i < 14; ++i) r.w[i] = neg ? s.w[i] : (uint32_t)b[i];
  return r;
}

// value < 2q: zero mod q  <=>  value == 0 or value == q
BLS_INLINE bool fp_is_zero(const fp_t& a) {
  uint32_t z = 0, e = 0;
#pragma unroll
  for (int i = 0; i < 14; ++i) { z |= a.w[i]; e |= a.w[i] ^ Q_LIMBS[i]; }
  return z == 0 || e == 0;
}

BLS_INLINE bool fp_eq(const fp_t& a, const fp_t& b) { return fp_is_zero(fp_sub(a, b)); }

// a / 2 mod q (value < 2q in, value < 1.5q out)
BLS_INLINE fp_t fp_half(const fp_t& a) {
  const uint32_t odd = a.w[0] & 1u;
  int32_t s[14];
#pragma unroll
  for (int i = 0; i < 14; ++i) s[i] = (int32_t)(a.w[i] + (odd ? Q_LIMBS[i] : 0u));
  fp_carry(s);
  fp_t r;
#pragma unroll
  for (int i = 0; i < 13; ++i) r.w[i] = ((uint32_t)s[i] >> 1) | (((uint32_t)s[i + 1] & 1u) << 27);
  r.w[13] = (uint32_t)s[13] >> 1;
  return r;
}

// Montgomery product a * b * 2^-392 mod q.  Inputs: limbs < 2^30 and
// value(a) * value(b) < 2900 q^2 (e.g. both < 4q lazily summed).  Output:
// normalized, value < 2q.  Column k accumulates <= 14 products < 2^60 plus
// <= 14 reduction products < 2^56 and a carry < 2^36: < 2^64.
BLS_INLINE fp_t fp_mul_body(const fp_t& a, const fp_t& b) {
  uint64_t T[28];
#pragma unroll
  for (int k = 0; k < 28; ++k) T[k] = 0;
#pragma unroll
  for (int i = 0; i < 14; ++i)
#pragma unroll
    for (int j = 0; j < 14; ++j) T[i + j] += (uint64_t)a.w[i] * b.w[j];
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    const uint32_t m = ((uint32_t)T[i] * Q_INV28) & FP_MASK;
#pragma unroll
    for (int j = 0; j < 14; ++j) T[i + j] += (uint64_t)m * Q_LIMBS[j];
    T[i + 1] += T[i] >> 28;
  }
  fp_t r;
  uint64_t c = 0;
#pragma unroll
  for (int j = 0; j < 14; ++j) {
    const uint64_t v = T[14 + j] + c;
    r.w[j] = (uint32_t)v & FP_MASK;
    c = v >> 28;
  }
  return r;
}

// squaring: 105 products instead of 196 (cross products doubled via 2a_i)
BLS_INLINE fp_t fp_sqr_body(const fp_t& a) {
  uint64_t T[28];
  uint32_t a2[14];
#pragma unroll
  for (int k = 0; k < 28; ++k) T[k] = 0;
#pragma unroll
  for (int i = 0; i < 14; ++i) a2[i] = a.w[i] << 1;
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    T[2 * i] += (uint64_t)a.w[i] * a.w[i];
#pragma unroll
    for (int j = i + 1; j < 14; ++j) T[i + j] += (uint64_t)a2[i] * a.w[j];
  }
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    const uint32_t m = ((uint32_t)T[i] * Q_INV28) & FP_MASK;
#pragma unroll
    for (int j = 0; j < 14; ++j) T[i + j] += (uint64_t)m * Q_LIMBS[j];
    T[i + 1] += T[i] >> 28;
  }
  fp_t r;
  uint64_t c = 0;
#pragma unroll
  for (int j = 0; j < 14; ++j) {
    const uint64_t v = T[14 + j] + c;
    r.w[j] = (uint32_t)v & FP_MASK;
    c = v >> 28;
  }
  return r;
}

// Call boundary.  clang passes an aggregate argument in registers only while the
// aggregates of a call fit 16 VGPRs, so a second fp_t operand would travel
// through scratch; 14-lane vectors are passed in v0..v27 and returned in v0..v13.
#if defined(__clang__)
typedef uint32_t fpv_t __attribute__((ext_vector_type(14)));
BLS_INLINE fpv_t fp_pack(const fp_t& a) {
  fpv_t v;
#pragma unroll
  for (int k = 0; k < 14; ++k) v[k] = a.w[k];
  return v;
}
BLS_INLINE fp_t fp_unpack(const fpv_t& v) {
  fp_t a;
#pragma unroll
  for (int k = 0; k < 14; ++k) a.w[k] = v[k];
  return a;
}
BLS_NOINLINE fpv_t fp_mul_call(fpv_t a, fpv_t b) { return fp_pack(fp_mul_body(fp_unpack(a), fp_unpack(b))); }
BLS_NOINLINE fpv_t fp_sqr_call(fpv_t a) { return fp_pack(fp_sqr_body(fp_unpack(a))); }
BLS_INLINE fp_t fp_mul(const fp_t& a, const fp_t& b) { return fp_unpack(fp_mul_call(fp_pack(a), fp_pack(b))); }
BLS_INLINE fp_t fp_sqr(const fp_t& a) { return fp_unpack(fp_sqr_call(fp_pack(a))); }
#else
BLS_NOINLINE fp_t fp_mul(fp_t a, fp_t b) { BLS_COUNT_MACS(392); return fp_mul_body(a, b); }
BLS_NOINLINE fp_t fp_sqr(fp_t a) { BLS_COUNT_MACS(301); return fp_sqr_body(a); }
#endif

// k * a for a small constant k: one reduction for k <= 8 (k a < 16q, limbs < 2^31)
BLS_INLINE fp_t fp_mul_small(const fp_t& a, int k) {
  if (k <= 8) {
    uint32_t s[14];
#pragma unroll
    for (int i = 0; i < 14; ++i) s[i] = (uint32_t)k * a.w[i];
    return fp_reduce_lc<8>(s);
  }
  fp_t r = a;
  fp_t acc = fp_zero();
  bool first = true;
  while (k) {
    if (k & 1) { acc = first ? r : fp_add(acc, r); first = false; }
    k >>= 1;
    if (k) r = fp_dbl(r);
  }
  return acc;
}

// left-to-right square-and-multiply over a 12-word little-endian (u32) exponent
BLS_DEV_INLINE fp_t fp_pow_limbs(const fp_t& a, const uint32_t* e, int nbits) {
  fp_t r = FP_ONE_M;
  for (int i = nbits - 1; i >= 0; --i) {
    r = fp_sqr(r);
    if ((e[i >> 5] >> (i & 31)) & 1u) r = fp_mul(r, a);
  }
  return r;
}

// u = a^((q-3)/4) by a 4-bit sliding window over the generated schedule
// (375 squarings + 78 multiplications + 8 for the odd-power table, against 605
// for plain square-and-multiply).  Every square root and inversion is built
// from this one power: sqrt(a) = u a, 1/a = u^4 a, 1/sqrt(a) = u^3 a.
BLS_HD inline fp_t fp_pow_qm3d4(const fp_t a) {
  const fp_t a2 = fp_sqr(a);
  const fp_t t1 = a, t3 = fp_mul(t1, a2), t5 = fp_mul(t3, a2), t7 = fp_mul(t5, a2);
  const fp_t t9 = fp_mul(t7, a2), t11 = fp_mul(t9, a2), t13 = fp_mul(t11, a2), t15 = fp_mul(t13, a2);
  fp_t r = FP_ONE_M;
  for (int k = 0; k < POW_QM3D4_NSTEPS; ++k) {
    for (int j = POW_QM3D4_SQR[k]; j > 0; --j) r = fp_sqr(r);
    switch (POW_QM3D4_DIG[k]) {   // uniform digit: a scalar branch, the table stays in registers
      case 1: r = fp_mul(r, t1); break;
      case 3: r = fp_mul(r, t3); break;
      case 5: r = fp_mul(r, t5); break;
      case 7: r = fp_mul(r, t7); break;
      case 9: r = fp_mul(r, t9); break;
      case 11: r = fp_mul(r, t11); break;
      case 13: r = fp_mul(r, t13); break;
      case 15: r = fp_mul(r, t15); break;
      default: break;
    }
  }
  return r;
}

// (fp_inv: optimized binary GCD, below the word helpers)
BLS_HD inline fp_t fp_inv(const fp_t am);

// returns true and sets r when a is a square; r = a^((q+1)/4)
BLS_DEV_INLINE bool fp_sqrt(fp_t& r, const fp_t& a) {
  r = fp_mul(fp_pow_qm3d4(a), a);
  return fp_eq(fp_sqr(r), a);
}

BLS_INLINE fp_t fp_to_mont(const fp_t& plain) { return fp_mul(plain, FP_R2); }
// Montgomery -> canonical plain value (< q)
BLS_INLINE fp_t fp_from_mont(const fp_t& m) {
  fp_t one = fp_zero();
  one.w[0] = 1;
  return fp_reduce_once(fp_mul(m, one));
}

// ---- plain (canonical, normalized) values: comparisons and byte codecs
// a < q
BLS_INLINE bool fp_plain_lt_q(const fp_t& a) {
  int32_t b[14];
#pragma unroll
  for (int i = 0; i < 14; ++i) b[i] = (int32_t)a.w[i] - (int32_t)Q_LIMBS[i];
  fp_carry(b);
  return b[13] < 0;
}

// a == 0 exactly (plain value; fp_is_zero would also accept a == q)
BLS_INLINE bool fp_plain_is_zero(const fp_t& a) {
  uint32_t z = 0;
#pragma unroll
  for (int i = 0; i < 14; ++i) z |= a.w[i];
  return z == 0;
}

// a > b
BLS_INLINE bool fp_plain_gt(const fp_t& a, const fp_t& b) {
  int32_t d[14];
#pragma unroll
  for (int i = 0; i < 14; ++i) d[i] = (int32_t)b.w[i] - (int32_t)a.w[i];
  fp_carry(d);
  return d[13] < 0;
}

// (2*y) // q == 1  <=>  2y >= q, for plain y < q (spec a_flag, bls_signature.md:52)
BLS_INLINE bool fp_plain_is_upper_half(const fp_t& y) {
  int32_t b[14];
#pragma unroll
  for (int i = 0; i < 14; ++i) b[i] = (int32_t)(2 * y.w[i]) - (int32_t)Q_LIMBS[i];
  fp_carry(b);
  return b[13] >= 0;
}

// 48 big-endian bytes -> plain limbs (no reduction; value < 2^384)
BLS_INLINE fp_t fp_plain_from_be48(const uint8_t* p) {
  uint32_t w[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const uint8_t* b = p + 44 - 4 * i;
    w[i] = ((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3];
  }
  fp_t r;
#pragma unroll
  for (int k = 0; k < 14; ++k) {
    const int bit = 28 * k, wi = bit >> 5, sh = bit & 31;
    uint64_t v = (uint64_t)w[wi] >> sh;
    if (wi + 1 < 12) v |= (uint64_t)w[wi + 1] << (32 - sh);
    r.w[k] = (uint32_t)v & FP_MASK;
  }
  return r;
}

// plain canonical value -> 48 big-endian bytes
BLS_INLINE void fp_plain_to_be48(uint8_t* p, const fp_t& a) {
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const int bit = 32 * i, k = bit / 28, sh = bit % 28;
    uint64_t v = (uint64_t)a.w[k] >> sh;
    if (k + 1 < 14) v |= (uint64_t)a.w[k + 1] << (28 - sh);
    if (k + 2 < 14 && 56 - sh < 32) v |= (uint64_t)a.w[k + 2] << (56 - sh);
    const uint32_t w = (uint32_t)v;
    uint8_t* b = p + 44 - 4 * i;
    b[0] = (uint8_t)(w >> 24);
    b[1] = (uint8_t)(w >> 16);
    b[2] = (uint8_t)(w >> 8);
    b[3] = (uint8_t)w;
  }
}

// plain canonical value -> 12 little-endian u32 words
BLS_INLINE void fp_plain_to_words(uint32_t w[12], const fp_t& a) {
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const int bit = 32 * i, k = bit / 28, sh = bit % 28;
    uint64_t v = (uint64_t)a.w[k] >> sh;
    if (k + 1 < 14) v |= (uint64_t)a.w[k + 1] << (28 - sh);
    if (k + 2 < 14 && 56 - sh < 32) v |= (uint64_t)a.w[k + 2] << (56 - sh);
    w[i] = (uint32_t)v;
  }
}

// word-level borrow chain step: a - b - bin, borrow out
BLS_INLINE uint32_t sub_borrow(uint32_t a, uint32_t b, uint32_t bin, uint32_t& bout) {
#if defined(__clang__)
  unsigned int bo;
  const uint32_t r = __builtin_subc(a, b, bin, &bo);
  bout = bo;
  return r;
#else
  const uint64_t v = (uint64_t)a - b - bin;
  bout = (uint32_t)(v >> 63);
  return (uint32_t)v;
#endif
}

// a >>= k (1 <= k <= 31) across 12 words; funnel shifts
BLS_INLINE void words_shr(uint32_t a[12], uint32_t k) {
#pragma unroll
  for (int i = 0; i < 11; ++i) a[i] = (uint32_t)((((uint64_t)a[i + 1] << 32) | a[i]) >> k);
  a[11] >>= k;
}

// strip the factors of two of a (a != 0); returns the parity of their number
BLS_INLINE uint32_t words_strip_twos(uint32_t a[12]) {
  uint32_t par = 0;
  while (a[0] == 0) {   // a whole zero word: probability ~2^-32 per step
#pragma unroll
    for (int i = 0; i < 11; ++i) a[i] = a[i + 1];
    a[11] = 0;
  }
  const uint32_t k = (uint32_t)__builtin_ctz(a[0]);
  if (k) {
    words_shr(a, k);
    par = k & 1u;
  }
  return par;
}

// Legendre symbol (a/q) of a Montgomery-form a: 1 (nonzero square), -1
// (non-square) or 0.  Binary Jacobi algorithm on 12 x 32-bit words, written
// branch-free per step (one subtraction, a conditional swap via the sign, one
// funnel shift): about 270 steps of ~80 word ops, an order of magnitude below
// Euler's criterion a^((q-1)/2), so the try-and-increment loop of hash_to_G2
// pays a full square root only for the candidate that succeeds.
BLS_HD inline int fp_legendre(const fp_t am) {
  uint32_t a[12], n[12];
  fp_plain_to_words(a, fp_from_mont(am));
  fp_plain_to_words(n, FP_Q_PLAIN);
  uint32_t z = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) z |= a[i];
  if (z == 0) return 0;
  // (2/n) = -1 iff n = 3, 5 mod 8 (n = q here)
  uint32_t t = words_strip_twos(a) & (((n[0] & 7u) == 3u || (n[0] & 7u) == 5u) ? 1u : 0u);
  while (true) {
    // a, n odd: d = a - n; when a < n swap (reciprocity: flip if both are 3 mod 4)
    uint32_t d[12], br = 0;
#pragma unroll
    for (int i = 0; i < 12; ++i) d[i] = sub_borrow(a[i], n[i], br, br);
    t ^= br & ((a[0] & n[0] & 2u) >> 1);
    uint32_t nb = 0, nz = 0;
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      const uint32_t nd = sub_borrow(0u, d[i], nb, nb);   // |a - n| when a < n
      const uint32_t an = a[i];
      a[i] = br ? nd : d[i];
      n[i] = br ? an : n[i];
      nz |= a[i];
    }
    if (nz == 0) break;                                   // a == n: n = gcd
    const uint32_t n8 = n[0] & 7u;
    t ^= words_strip_twos(a) & ((n8 == 3u || n8 == 5u) ? 1u : 0u);
  }
  uint32_t one = n[0] ^ 1u;
#pragma unroll
  for (int i = 1; i < 12; ++i) one |= n[i];
  if (one != 0) return 0;
  return t ? -1 : 1;
}

// ------------------------------------------------ inversion (binary xgcd) --
BLS_INLINE uint32_t add_carry(uint32_t a, uint32_t b, uint32_t cin, uint32_t& cout) {
#if defined(__clang__)
  unsigned int co;
  const uint32_t r = __builtin_addc(a, b, cin, &co);
  cout = co;
  return r;
#else
  const uint64_t v = (uint64_t)a + b + cin;
  cout = (uint32_t)(v >> 32);
  return (uint32_t)v;
#endif
}

// x / 2^k mod q for x < 2q and 1 <= k <= 31: (x + m q) / 2^k with
// m = -x q^-1 mod 2^k, an exact shift; the result stays < 2q
BLS_INLINE void words_div2k_modq(uint32_t x[12], uint32_t k) {
  const uint32_t m = (x[0] * Q_NINV32) & ((1u << k) - 1u);
  uint32_t t[13];
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    c += (uint64_t)m * Q_WORDS[i] + x[i];
    t[i] = (uint32_t)c;
    c >>= 32;
  }
  t[12] = (uint32_t)c;
#pragma unroll
  for (int i = 0; i < 12; ++i) x[i] = (uint32_t)((((uint64_t)t[i + 1] << 32) | t[i]) >> k);
}

// d = a - b mod 2q for a, b < 2q; d in [0, 2q)
BLS_INLINE void words_sub_mod2q(uint32_t d[12], const uint32_t a[12], const uint32_t b[12]) {
  uint32_t br = 0, c = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) d[i] = sub_borrow(a[i], b[i], br, br);
  const uint32_t mask = 0u - br;
#pragma unroll
  for (int i = 0; i < 12; ++i) d[i] = add_carry(d[i], Q2_WORDS[i] & mask, c, c);
}

// u >>= (its factors of two), x /= 2^(the same count) mod q
BLS_INLINE void xgcd_strip(uint32_t u[12], uint32_t x[12]) {
  while (u[0] == 0) {   // a whole zero word: probability ~2^-32 per step
#pragma unroll
    for (int i = 0; i < 11; ++i) u[i] = u[i + 1];
    u[11] = 0;
    words_div2k_modq(x, 16);
    words_div2k_modq(x, 16);
  }
  const uint32_t k = (uint32_t)__builtin_ctz(u[0]);
  if (k) {
    words_shr(u, k);
    words_div2k_modq(x, k);
  }
}

// 12 x 32-bit words (value < 2^381) -> 14 x 28-bit limbs
BLS_INLINE fp_t fp_from_words(const uint32_t w[12]) {
  fp_t r;
#pragma unroll
  for (int k = 0; k < 14; ++k) {
    const int bit = 28 * k, i = bit / 32, sh = bit % 32;
    uint32_t v = w[i] >> sh;
    if (sh > 4 && i + 1 < 12) v |= w[i + 1] << (32 - sh);
    r.w[k] = v & FP_MASK;
  }
  return r;
}

// 1/a (0 -> 0), variable-time binary extended gcd on the integer A = aR mod q
// (one subtraction, a conditional swap, one strip of twos per step, ~270 steps
// of ~150 word ops, the slowest lane of a wave setting the count), then
// A^-1 R^3 R^-1 = a^-1 R by one Montgomery product.  The safety net of fp_inv.
// Invariants: x1 A = u, x2 A = v (mod q); u, v odd after each strip; x1, x2 < 2q.
BLS_HD inline fp_t fp_inv_xgcd(const fp_t am) {
  uint32_t u[12], v[12], x1[12], x2[12];
  fp_plain_to_words(u, fp_reduce_once(am));
  uint32_t z = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) z |= u[i];
  if (z == 0) return fp_zero();
#pragma unroll
  for (int i = 0; i < 12; ++i) { v[i] = Q_WORDS[i]; x1[i] = 0; x2[i] = 0; }
  x1[0] = 1;
  xgcd_strip(u, x1);
  while (true) {
    uint32_t d[12], br = 0, nz = 0;
#pragma unroll
    for (int i = 0; i < 12; ++i) { d[i] = sub_borrow(u[i], v[i], br, br); nz |= d[i]; }
    if (nz == 0) break;                 // u == v == gcd == 1
    // u > v: (u, x1) <- (u - v, x1 - x2);  u < v: (u, v, x1, x2) <- (v - u, u, x2 - x1, x1)
    // x2 - x1 = 2q - xd: u != v here, so x1 != x2 (mod q) and xd lies in (0, 2q) \ {q}
    uint32_t xd[12], nb = 0, xb = 0;
    words_sub_mod2q(xd, x1, x2);
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      const uint32_t nd = sub_borrow(0u, d[i], nb, nb);
      const uint32_t xn = sub_borrow(Q2_WORDS[i], xd[i], xb, xb);
      const uint32_t uo = u[i], xo = x1[i];
      u[i] = br ? nd : d[i];
      v[i] = br ? uo : v[i];
      x1[i] = br ? xn : xd[i];
      x2[i] = br ? xo : x2[i];
    }
    xgcd_strip(u, x1);
  }
  // x1 < 2q -> canonical
  uint32_t e[12], bq = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) e[i] = sub_borrow(x1[i], Q_WORDS[i], bq, bq);
#pragma unroll
  for (int i = 0; i < 12; ++i) x1[i] = bq ? x1[i] : e[i];
  return fp_mul(fp_from_words(x1), FP_R3);
}

// ------------------------------- inversion (optimized binary GCD, Pornin) --
// 1/a (0 -> 0) by the optimized binary GCD of T. Pornin ("Optimized Binary GCD
// for Modular Inversion", 2020): a = A (the integer aR mod q), b = q, with
// a = u A and b = v A (mod q) throughout.  Each of 26 outer rounds runs 30
// binary-GCD steps on 62-bit approximations of a and b (their low 30 bits and
// their top 32 bits at the common length), collecting the steps in a 2x2 matrix
// (|f| + |g| <= 2^30), then applies it to the full values:
//   a, b <- (f0 a + g0 b) / 2^30, (f1 a + g1 b) / 2^30     (exact; signs fixed)
//   u, v <- (f0 u + g0 v) / 2^30, (f1 u + g1 v) / 2^30     (mod q, Montgomery-style)
// 26 x 30 = 780 >= 2 len(q) - 1 steps bring b to gcd = 1 and v to A^-1.  Every
// lane runs the same instruction stream (no data-dependent trip count), and a
// value is 13 signed 30-bit limbs, so the matrix products are 32x32 -> 64-bit
// multiply-adds with signed carries.  If b != 1 at the end (not expected: the
// step bound is the paper's), the wave falls back to fp_inv_xgcd.
constexpr int INV_L = 13;                 // 30-bit limbs
constexpr uint32_t INV_M30 = (1u << 30) - 1;

BLS_INLINE void inv_to_l30(int32_t r[INV_L], const uint32_t w[12]) {
#pragma unroll
  for (int k = 0; k < INV_L; ++k) {
    const int bit = 30 * k, i = bit / 32, sh = bit % 32;
    uint64_t v = (uint64_t)w[i] >> sh;
    if (i + 1 < 12) v |= (uint64_t)w[i + 1] << (32 - sh);
    r[k] = (int32_t)((uint32_t)v & INV_M30);
  }
}

// (f x + g y) / 2^30 for x, y of 13 limbs (exact division: the low limb cancels);
// the result's limbs are normalized (30 bits) except the top one, which is signed
BLS_INLINE void inv_lin_shift(int32_t r[INV_L], const int32_t x[INV_L], const int32_t y[INV_L], int32_t f, int32_t g) {
  int64_t acc = (int64_t)f * x[0] + (int64_t)g * y[0];
  acc >>= 30;
#pragma unroll
  for (int i = 1; i < INV_L; ++i) {
    acc += (int64_t)f * x[i] + (int64_t)g * y[i];
    r[i - 1] = (int32_t)((uint32_t)acc & INV_M30);
    acc >>= 30;
  }
  r[INV_L - 1] = (int32_t)acc;
}

// (f x + g y) / 2^30 mod q for x, y in [0, q): one Montgomery-style step with the
// low limb's multiple of q, then the result in (-q, 2q) is brought into [0, q)
BLS_INLINE void inv_lin_modq(int32_t r[INV_L], const int32_t x[INV_L], const int32_t y[INV_L], int32_t f, int32_t g) {
  const int64_t lo = (int64_t)f * x[0] + (int64_t)g * y[0];
  const int32_t k = (int32_t)(((uint32_t)lo * Q_NINV32) & INV_M30);
  int64_t acc = lo + (int64_t)k * Q_L30[0];
  acc >>= 30;
#pragma unroll
  for (int i = 1; i < INV_L; ++i) {
    acc += (int64_t)f * x[i] + (int64_t)g * y[i] + (int64_t)k * Q_L30[i];
    r[i - 1] = (int32_t)((uint32_t)acc & INV_M30);
    acc >>= 30;
  }
  r[INV_L - 1] = (int32_t)acc;
  // r in (-q, 2q): add q when negative, then subtract q when >= q
  const int32_t addq = r[INV_L - 1] < 0 ? 1 : 0;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < INV_L; ++i) {
    const int32_t t = r[i] + (addq ? Q_L30[i] : 0) + c;
    r[i] = (i < INV_L - 1) ? (int32_t)((uint32_t)t & INV_M30) : t;
    c = t >> 30;
  }
  int32_t d[INV_L];
  c = 0;
#pragma unroll
  for (int i = 0; i < INV_L; ++i) {
    const int32_t t = r[i] - Q_L30[i] + c;
    d[i] = (i < INV_L - 1) ? (int32_t)((uint32_t)t & INV_M30) : t;
    c = t >> 30;
  }
  const bool ge = d[INV_L - 1] >= 0;
#pragma unroll
  for (int i = 0; i < INV_L; ++i) r[i] = ge ? d[i] : r[i];
}

// x <- -x (limbs normalized, top limb signed)
BLS_INLINE void inv_neg(int32_t x[INV_L]) {
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < INV_L; ++i) {
    const int32_t t = c - x[i];
    x[i] = (i < INV_L - 1) ? (int32_t)((uint32_t)t & INV_M30) : t;
    c = t >> 30;
  }
}

BLS_HD inline fp_t fp_inv(const fp_t am) {
  uint32_t w[12];
  fp_plain_to_words(w, fp_reduce_once(am));
  uint32_t z = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) z |= w[i];
  if (z == 0) return fp_zero();
  int32_t a[INV_L], b[INV_L], u[INV_L], v[INV_L];
  inv_to_l30(a, w);
#pragma unroll
  for (int i = 0; i < INV_L; ++i) { b[i] = Q_L30[i]; u[i] = 0; v[i] = 0; }
  u[0] = 1;
  for (int round = 0; round < 26; ++round) {
    // approximations: low 30 bits, and the 32 bits below the common length n >= 62
    int t = 2;
    uint32_t top = 0;
#pragma unroll
    for (int i = 2; i < INV_L; ++i) {
      const uint32_t c = (uint32_t)(a[i] | b[i]);
      if (c) { t = i; top = c; }
    }
    const int bl = top ? 32 - __builtin_clz(top) : 2;   // bits of the top limb (n = 30 t + bl)
    uint32_t a2 = 0, a1 = 0, a0 = 0, b2 = 0, b1 = 0, b0 = 0;
#pragma unroll
    for (int i = 2; i < INV_L; ++i) {
      const bool s = i == t;
      a2 = s ? (uint32_t)a[i] : a2; a1 = s ? (uint32_t)a[i - 1] : a1; a0 = s ? (uint32_t)a[i - 2] : a0;
      b2 = s ? (uint32_t)b[i] : b2; b1 = s ? (uint32_t)b[i - 1] : b1; b0 = s ? (uint32_t)b[i - 2] : b0;
    }
    const uint64_t wa = ((uint64_t)a2 << 31) | ((uint64_t)a1 << 1) | (a0 >> 29);
    const uint64_t wb = ((uint64_t)b2 << 31) | ((uint64_t)b1 << 1) | (b0 >> 29);
    uint64_t xa = ((wa >> (bl - 1)) << 30) | (uint32_t)a[0];
    uint64_t xb = ((wb >> (bl - 1)) << 30) | (uint32_t)b[0];
    if (t == 2 && bl <= 2) {   // n <= 62: the exact values (the paper's requirement for n <= 2k)
      xa = (uint32_t)a[0] | ((uint64_t)(uint32_t)a[1] << 30) | ((uint64_t)(uint32_t)a[2] << 60);
      xb = (uint32_t)b[0] | ((uint64_t)(uint32_t)b[1] << 30) | ((uint64_t)(uint32_t)b[2] << 60);
    }
    int32_t f0 = 1, g0 = 0, f1 = 0, g1 = 1;
#pragma unroll 10
    for (int j = 0; j < 30; ++j) {
      const bool odd = (xa & 1) != 0;
      const bool sw = odd && xa < xb;
      const uint64_t ta = sw ? xb : xa, tb = sw ? xa : xb;
      const int32_t tf0 = sw ? f1 : f0, tg0 = sw ? g1 : g0, tf1 = sw ? f0 : f1, tg1 = sw ? g0 : g1;
      xa = (odd ? ta - tb : ta) >> 1;
      xb = tb;
      f0 = odd ? tf0 - tf1 : tf0;
      g0 = odd ? tg0 - tg1 : tg0;
      f1 = tf1 + tf1;
      g1 = tg1 + tg1;
    }
    int32_t na[INV_L], nb[INV_L];
    inv_lin_shift(na, a, b, f0, g0);
    inv_lin_shift(nb, a, b, f1, g1);
    if (na[INV_L - 1] < 0) { inv_neg(na); f0 = -f0; g0 = -g0; }
    if (nb[INV_L - 1] < 0) { inv_neg(nb); f1 = -f1; g1 = -g1; }
    int32_t nu[INV_L], nv[INV_L];
    inv_lin_modq(nu, u, v, f0, g0);
    inv_lin_modq(nv, u, v, f1, g1);
#pragma unroll
    for (int i = 0; i < INV_L; ++i) { a[i] = na[i]; b[i] = nb[i]; u[i] = nu[i]; v[i] = nv[i]; }
  }
  uint32_t bad = (uint32_t)b[0] ^ 1u;
#pragma unroll
  for (int i = 1; i < INV_L; ++i) bad |= (uint32_t)b[i];
#pragma unroll
  for (int i = 0; i < INV_L; ++i) bad |= (uint32_t)a[i];
  if (BLS_ANY(bad != 0)) {
    BLS_COUNT_INV_FALLBACK();
    return fp_inv_xgcd(am);
  }
  // v = A^-1 (canonical, 30-bit limbs) -> 28-bit limbs, then A^-1 R^3 / R
  fp_t r;
#pragma unroll
  for (int k = 0; k < 14; ++k) {
    const int bit = 28 * k, i = bit / 30, sh = bit % 30;
    uint64_t x = (uint64_t)(uint32_t)v[i] >> sh;
    if (i + 1 < INV_L) x |= (uint64_t)(uint32_t)v[i + 1] << (30 - sh);
    r.w[k] = (uint32_t)x & FP_MASK;
  }
  return fp_mul(r, FP_R3);
}

// ---------------------------------------------------------------- Fp2 -----
BLS_INLINE fp2_t fp2_zero() { fp2_t r; r.c0 = fp_zero(); r.c1 = fp_zero(); return r; }
BLS_INLINE fp2_t fp2_one() { fp2_t r; r.c0 = FP_ONE_M; r.c1 = fp_zero(); return r; }
BLS_INLINE bool fp2_is_zero(const fp2_t& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
BLS_INLINE bool fp2_eq(const fp2_t& a, const fp2_t& b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }
BLS_INLINE fp2_t fp2_add(const fp2_t& a, const fp2_t& b) { fp2_t r; r.c0 = fp_add(a.c0, b.c0); r.c1 = fp_add(a.c1, b.c1); return r; }
BLS_INLINE fp2_t fp2_sub(const fp2_t& a, const fp2_t& b) { fp2_t r; r.c0 = fp_sub(a.c0, b.c0); r.c1 = fp_sub(a.c1, b.c1); return r; }
BLS_INLINE fp2_t fp2_neg(const fp2_t& a) { fp2_t r; r.c0 = fp_neg(a.c0); r.c1 = fp_neg(a.c1); return r; }
BLS_INLINE fp2_t fp2_dbl(const fp2_t& a) { fp2_t r; r.c0 = fp_dbl(a.c0); r.c1 = fp_dbl(a.c1); return r; }
BLS_INLINE fp2_t fp2_half(const fp2_t& a) { fp2_t r; r.c0 = fp_half(a.c0); r.c1 = fp_half(a.c1); return r; }
BLS_INLINE fp2_t fp2_conj(const fp2_t& a) { fp2_t r; r.c0 = a.c0; r.c1 = fp_neg(a.c1); return r; }
BLS_INLINE fp2_t fp2_mul_fp(const fp2_t& a, const fp_t& b) { fp2_t r; r.c0 = fp_mul(a.c0, b); r.c1 = fp_mul(a.c1, b); return r; }

// ---- double-width (28-column) helpers for lazy reduction
// T[k] += sum_{i+j=k} a_i b_j   (operand limbs < 2^30)
BLS_INLINE void wide_mac(uint64_t (&T)[28], const fp_t& a, const fp_t& b) {
#pragma unroll
  for (int i = 0; i < 14; ++i)
#pragma unroll
    for (int j = 0; j < 14; ++j) T[i + j] += (uint64_t)a.w[i] * b.w[j];
}

// T[k] += columns of a^2 (operand limbs < 2^29)
BLS_INLINE void wide_sqr(uint64_t (&T)[28], const fp_t& a) {
  uint32_t a2[14];
#pragma unroll
  for (int i = 0; i < 14; ++i) a2[i] = a.w[i] << 1;
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    T[2 * i] += (uint64_t)a.w[i] * a.w[i];
#pragma unroll
    for (int j = i + 1; j < 14; ++j) T[i + j] += (uint64_t)a2[i] * a.w[j];
  }
}

// Montgomery reduction of a double-width value: columns < 2^63.2 and value
// < 2^773 (= q R) -> normalized, value < 2q.
BLS_INLINE fp_t fp_redc_wide(uint64_t (&T)[28]) {
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    const uint32_t m = ((uint32_t)T[i] * Q_INV28) & FP_MASK;
#pragma unroll
    for (int j = 0; j < 14; ++j) T[i + j] += (uint64_t)m * Q_LIMBS[j];
    T[i + 1] += T[i] >> 28;
  }
  fp_t r;
  uint64_t c = 0;
#pragma unroll
  for (int j = 0; j < 14; ++j) {
    const uint64_t v = T[14 + j] + c;
    r.w[j] = (uint32_t)v & FP_MASK;
    c = v >> 28;
  }
  return r;
}

// Fp2 product with one REDC per output coefficient (Karatsuba, lazy reduction):
//   c0 = REDC(a0 b0 + W - a1 b1),  c1 = REDC((a0+a1)(b0+b1) - a0 b0 - a1 b1)
// W = WIDE_QMULT, a multiple of q whose columns dominate any product column.
// Inputs may be lazy sums: limbs < 2^29, values < 4q.  Output normalized, < 2q.
// Fp2 multiplication: three Montgomery products (Karatsuba).  Kept inline so the
// only call boundary is fp_mul (two 14-word operands in argument registers);
// measured on MI355X, noinline Fp2-level functions (56-word arguments through
// the stack plus callee-saved spills) were 15-25 % slower end to end.
// Operands may be lazy sums (limbs < 2^29, values < 4q): the products see
// limbs < 2^30 and values < 8q.
BLS_INLINE fp2_t fp2_mul(const fp2_t& a, const fp2_t& b) {
  const fp_t t0 = fp_mul(a.c0, b.c0);
  const fp_t t1 = fp_mul(a.c1, b.c1);
  const fp_t t2 = fp_mul(fp_add_lazy(a.c0, a.c1), fp_add_lazy(b.c0, b.c1));
  fp2_t r;
  r.c0 = fp_sub(t0, t1);
  r.c1 = fp_sub2(t2, t0, t1);
  return r;
}

// Fp2 squaring: c0 = (a0 + a1)(a0 - a1), c1 = 2 a0 a1 (operands weakly reduced, < 2q)
BLS_INLINE fp2_t fp2_sqr(const fp2_t& a) {
  fp2_t r;
  r.c0 = fp_mul(fp_add_lazy(a.c0, a.c1), fp_sub(a.c0, a.c1));
  const fp_t t = fp_mul(a.c0, a.c1);
  r.c1 = fp_add(t, t);
  return r;
}

// lazy Fp2 sum for a multiplication operand only (limbs < 2^29, values < 4q)
BLS_INLINE fp2_t fp2_add_lazy(const fp2_t& a, const fp2_t& b) {
  fp2_t r; r.c0 = fp_add_lazy(a.c0, b.c0); r.c1 = fp_add_lazy(a.c1, b.c1); return r;
}

// multiply by xi = 1 + u
BLS_INLINE fp2_t fp2_mul_xi(const fp2_t& a) {
  fp2_t r;
  r.c0 = fp_sub(a.c0, a.c1);
  r.c1 = fp_add(a.c0, a.c1);
  return r;
}

BLS_INLINE fp2_t fp2_mul_small(const fp2_t& a, int k) {
  fp2_t r; r.c0 = fp_mul_small(a.c0, k); r.c1 = fp_mul_small(a.c1, k); return r;
}

// one-reduction combinations (fp_reduce_lc), shared names with the lane-pair type:
// a + xi b = (a0 + b0 - b1) + (a1 + b0 + b1) u
BLS_INLINE fp2_t fp2_add_mul_xi(const fp2_t& a, const fp2_t& b) {
  fp2_t r; r.c0 = fp_add_sub(a.c0, b.c0, b.c1); r.c1 = fp_add3(a.c1, b.c0, b.c1); return r;
}
// a - b - c
BLS_INLINE fp2_t fp2_sub2(const fp2_t& a, const fp2_t& b, const fp2_t& c) {
  fp2_t r; r.c0 = fp_sub2(a.c0, b.c0, c.c0); r.c1 = fp_sub2(a.c1, b.c1, c.c1); return r;
}
// 3X - 2x and 3X + 2x
BLS_INLINE fp2_t fp2_3m2(const fp2_t& X, const fp2_t& x) {
  fp2_t r; r.c0 = fp_3m2(X.c0, x.c0); r.c1 = fp_3m2(X.c1, x.c1); return r;
}
BLS_INLINE fp2_t fp2_3p2(const fp2_t& X, const fp2_t& x) {
  fp2_t r; r.c0 = fp_3p2(X.c0, x.c0); r.c1 = fp_3p2(X.c1, x.c1); return r;
}

BLS_HD inline fp2_t fp2_inv(const fp2_t a) {
  const fp_t n = fp_add(fp_sqr(a.c0), fp_sqr(a.c1));
  const fp_t ni = fp_inv(n);
  fp2_t r;
  r.c0 = fp_mul(a.c0, ni);
  r.c1 = fp_neg(fp_mul(a.c1, ni));
  return r;
}

// Complex-method square root for q = 3 mod 4 (DESIGN.md "Square roots").
// Returns false when a is a non-square.  Which of the two roots is returned
// is unspecified; callers apply the spec's selection rule.
BLS_DEV_INLINE bool fp2_sqrt(fp2_t& r, const fp2_t& a) {
  if (fp_is_zero(a.c1)) {
    fp_t s;
    if (fp_sqrt(s, a.c0)) { r.c0 = s; r.c1 = fp_zero(); return true; }
    if (fp_sqrt(s, fp_neg(a.c0))) { r.c0 = fp_zero(); r.c1 = s; return true; }
    return false;
  }
  const fp_t alpha = fp_add(fp_sqr(a.c0), fp_sqr(a.c1));
  fp_t gamma;
  if (!fp_sqrt(gamma, alpha)) return false;
  const fp_t delta = fp_half(fp_add(a.c0, gamma));
  // t = delta^((q+1)/4) and 1/t = delta^((3q-5)/4) from one power u = delta^((q-3)/4):
  // t = u delta, 1/t = u^2 t (delta != 0 here because a1 != 0)
  const fp_t u = fp_pow_qm3d4(delta);
  const fp_t t = fp_mul(u, delta);
  const fp_t other = fp_mul(a.c1, fp_half(fp_mul(fp_sqr(u), t)));   // a1 / (2t)
  if (fp_eq(fp_sqr(t), delta)) { r.c0 = t; r.c1 = other; }
  else { r.c0 = other; r.c1 = t; }
  return true;
}

// ------------------------------------------- representation-generic tower --
// Fp6 / Fp12 and everything above them are templates over the Fp2
// representation E: fp2_t (both coefficients in one lane; the host unit-test
// build) or fp2p_t (bls381_pair.hpp: the two coefficients in the two lanes of
// an adjacent lane pair; the gfx950 kernels).  Both provide the same fp2_*
// operations, so the formulas below exist once.
template <class E> BLS_INLINE E e2_zero();
template <class E> BLS_INLINE E e2_one();
template <class E> BLS_INLINE E e2_k(const fp2_t& k);   // a compile-time Fp2 constant
template <> BLS_INLINE fp2_t e2_zero<fp2_t>() { return fp2_zero(); }
template <> BLS_INLINE fp2_t e2_one<fp2_t>() { return fp2_one(); }
template <> BLS_INLINE fp2_t e2_k<fp2_t>(const fp2_t& k) { return k; }

// ---------------------------------------------------------------- Fp6 -----
template <class E> BLS_INLINE fp6_g<E> fp6_zero() { fp6_g<E> r; r.c0 = e2_zero<E>(); r.c1 = e2_zero<E>(); r.c2 = e2_zero<E>(); return r; }
template <class E> BLS_INLINE fp6_g<E> fp6_one() { fp6_g<E> r; r.c0 = e2_one<E>(); r.c1 = e2_zero<E>(); r.c2 = e2_zero<E>(); return r; }
template <class E> BLS_INLINE fp6_g<E> fp6_add(const fp6_g<E>& a, const fp6_g<E>& b) { fp6_g<E> r; r.c0 = fp2_add(a.c0, b.c0); r.c1 = fp2_add(a.c1, b.c1); r.c2 = fp2_add(a.c2, b.c2); return r; }
template <class E> BLS_INLINE fp6_g<E> fp6_sub(const fp6_g<E>& a, const fp6_g<E>& b) { fp6_g<E> r; r.c0 = fp2_sub(a.c0, b.c0); r.c1 = fp2_sub(a.c1, b.c1); r.c2 = fp2_sub(a.c2, b.c2); return r; }
template <class E> BLS_INLINE fp6_g<E> fp6_neg(const fp6_g<E>& a) { fp6_g<E> r; r.c0 = fp2_neg(a.c0); r.c1 = fp2_neg(a.c1); r.c2 = fp2_neg(a.c2); return r; }
template <class E> BLS_INLINE bool fp6_is_zero(const fp6_g<E>& a) { return fp2_is_zero(a.c0) && fp2_is_zero(a.c1) && fp2_is_zero(a.c2); }

template <class E>
BLS_INLINE fp6_g<E> fp6_mul_inl(const fp6_g<E>& a, const fp6_g<E>& b) {
  const E t0 = fp2_mul(a.c0, b.c0);
  const E t1 = fp2_mul(a.c1, b.c1);
  const E t2 = fp2_mul(a.c2, b.c2);
  fp6_g<E> r;
  r.c0 = fp2_add_mul_xi(t0, fp2_sub2(fp2_mul(fp2_add_lazy(a.c1, a.c2), fp2_add_lazy(b.c1, b.c2)), t1, t2));
  r.c1 = fp2_add_mul_xi(fp2_sub2(fp2_mul(fp2_add_lazy(a.c0, a.c1), fp2_add_lazy(b.c0, b.c1)), t0, t1), t2);
  r.c2 = fp2_add(fp2_sub2(fp2_mul(fp2_add_lazy(a.c0, a.c2), fp2_add_lazy(b.c0, b.c2)), t0, t2), t1);
  return r;
}

template <class E>
BLS_NOINLINE fp6_g<E> fp6_mul(const fp6_g<E> a, const fp6_g<E> b) { return fp6_mul_inl(a, b); }

template <class E>
BLS_INLINE fp6_g<E> fp6_mul_by_v(const fp6_g<E>& a) {
  fp6_g<E> r; r.c0 = fp2_mul_xi(a.c2); r.c1 = a.c0; r.c2 = a.c1; return r;
}

// a - b - c,  a + v b,  2a: one reduction per coefficient
template <class E>
BLS_INLINE fp6_g<E> fp6_sub2(const fp6_g<E>& a, const fp6_g<E>& b, const fp6_g<E>& c) {
  fp6_g<E> r; r.c0 = fp2_sub2(a.c0, b.c0, c.c0); r.c1 = fp2_sub2(a.c1, b.c1, c.c1); r.c2 = fp2_sub2(a.c2, b.c2, c.c2); return r;
}
template <class E>
BLS_INLINE fp6_g<E> fp6_add_mul_by_v(const fp6_g<E>& a, const fp6_g<E>& b) {
  fp6_g<E> r; r.c0 = fp2_add_mul_xi(a.c0, b.c2); r.c1 = fp2_add(a.c1, b.c0); r.c2 = fp2_add(a.c2, b.c1); return r;
}
template <class E>
BLS_INLINE fp6_g<E> fp6_dbl(const fp6_g<E>& a) {
  fp6_g<E> r; r.c0 = fp2_dbl(a.c0); r.c1 = fp2_dbl(a.c1); r.c2 = fp2_dbl(a.c2); return r;
}

template <class E>
BLS_HD inline fp6_g<E> fp6_inv(const fp6_g<E> a) {
  const E c0 = fp2_sub(fp2_sqr(a.c0), fp2_mul_xi(fp2_mul(a.c1, a.c2)));
  const E c1 = fp2_sub(fp2_mul_xi(fp2_sqr(a.c2)), fp2_mul(a.c0, a.c1));
  const E c2 = fp2_sub(fp2_sqr(a.c1), fp2_mul(a.c0, a.c2));
  const E t = fp2_add(fp2_mul(a.c0, c0), fp2_mul_xi(fp2_add(fp2_mul(a.c2, c1), fp2_mul(a.c1, c2))));
  const E ti = fp2_inv(t);
  fp6_g<E> r;
  r.c0 = fp2_mul(c0, ti);
  r.c1 = fp2_mul(c1, ti);
  r.c2 = fp2_mul(c2, ti);
  return r;
}

// ---------------------------------------------------------------- Fp12 ----
template <class E> BLS_INLINE fp12_g<E> fp12_one() { fp12_g<E> r; r.c0 = fp6_one<E>(); r.c1 = fp6_zero<E>(); return r; }

template <class E>
BLS_INLINE bool fp12_is_one(const fp12_g<E>& a) {
  return fp2_eq(a.c0.c0, e2_one<E>()) && fp2_is_zero(a.c0.c1) && fp2_is_zero(a.c0.c2) && fp6_is_zero(a.c1);
}

template <class E>
BLS_INLINE bool fp12_eq(const fp12_g<E>& a, const fp12_g<E>& b) {
  return fp2_eq(a.c0.c0, b.c0.c0) && fp2_eq(a.c0.c1, b.c0.c1) && fp2_eq(a.c0.c2, b.c0.c2) &&
         fp2_eq(a.c1.c0, b.c1.c0) && fp2_eq(a.c1.c1, b.c1.c1) && fp2_eq(a.c1.c2, b.c1.c2);
}

template <class E>
BLS_INLINE fp12_g<E> fp12_mul_inl(const fp12_g<E>& a, const fp12_g<E>& b) {
  const fp6_g<E> ac = fp6_mul_inl(a.c0, b.c0);
  const fp6_g<E> bd = fp6_mul_inl(a.c1, b.c1);
  fp12_g<E> r;
  r.c1 = fp6_sub2(fp6_mul_inl(fp6_add(a.c0, a.c1), fp6_add(b.c0, b.c1)), ac, bd);
  r.c0 = fp6_add_mul_by_v(ac, bd);
  return r;
}

// call version (loops of products, e.g. the segmented Fp12 products): its 84-word
// operands go through the stack, so the final exponentiation inlines instead
template <class E>
BLS_NOINLINE fp12_g<E> fp12_mul(const fp12_g<E> a, const fp12_g<E> b) {
  const fp6_g<E> ac = fp6_mul(a.c0, b.c0);
  const fp6_g<E> bd = fp6_mul(a.c1, b.c1);
  fp12_g<E> r;
  r.c1 = fp6_sub2(fp6_mul(fp6_add(a.c0, a.c1), fp6_add(b.c0, b.c1)), ac, bd);
  r.c0 = fp6_add_mul_by_v(ac, bd);
  return r;
}

// complex squaring: (a + b w)^2 = (a^2 + v b^2) + 2ab w
//   = ((a + b)(a + v b) - ab - v ab) + 2ab w
template <class E>
BLS_INLINE fp12_g<E> fp12_sqr_inl(const fp12_g<E>& f) {
  const fp6_g<E> ab = fp6_mul_inl(f.c0, f.c1);
  const fp6_g<E> t = fp6_mul_inl(fp6_add(f.c0, f.c1), fp6_add_mul_by_v(f.c0, f.c1));
  fp12_g<E> r;
  r.c0 = fp6_sub2(t, ab, fp6_mul_by_v(ab));
  r.c1 = fp6_dbl(ab);
  return r;
}

template <class E>
BLS_NOINLINE fp12_g<E> fp12_sqr(const fp12_g<E> f) { return fp12_sqr_inl(f); }

template <class E>
BLS_INLINE fp12_g<E> fp12_conj(const fp12_g<E>& a) { fp12_g<E> r; r.c0 = a.c0; r.c1 = fp6_neg(a.c1); return r; }

template <class E>
BLS_HD inline fp12_g<E> fp12_inv(const fp12_g<E> f) {
  const fp6_g<E> t = fp6_sub(fp6_mul(f.c0, f.c0), fp6_mul_by_v(fp6_mul(f.c1, f.c1)));
  const fp6_g<E> ti = fp6_inv(t);
  fp12_g<E> r;
  r.c0 = fp6_mul(f.c0, ti);
  r.c1 = fp6_neg(fp6_mul(f.c1, ti));
  return r;
}

// f^(q^p), p in {1,2,3}; coefficient of w^k picks up gamma[p][k] (and conj for odd p)
template <class E>
BLS_HD inline fp12_g<E> fp12_frob(const fp12_g<E> f, int p) {
  const fp2_t* g = FROB_GAMMA_M[p - 1];
  const bool odd = (p & 1) != 0;
  auto fr = [&](const E& c, int k) -> E {
    const E cc = odd ? fp2_conj(c) : c;
    return k == 0 ? cc : fp2_mul(cc, e2_k<E>(g[k]));
  };
  fp12_g<E> r;
  r.c0.c0 = fr(f.c0.c0, 0);
  r.c0.c1 = fr(f.c0.c1, 2);
  r.c0.c2 = fr(f.c0.c2, 4);
  r.c1.c0 = fr(f.c1.c0, 1);
  r.c1.c1 = fr(f.c1.c1, 3);
  r.c1.c2 = fr(f.c1.c2, 5);
  return r;
}

// sparse product f * (c0 + c1 v + c2 v w): 13 Fp2 multiplications
template <class E>
BLS_INLINE fp12_g<E> fp12_mul_by_line_inl(const fp12_g<E>& f, const E& c0, const E& c1, const E& c2) {
  const fp6_g<E>& a = f.c0;
  const fp6_g<E>& b = f.c1;
  // aA, A = c0 + c1 v
  fp6_g<E> aA;
  {
    const E t0 = fp2_mul(a.c0, c0);
    const E t1 = fp2_mul(a.c1, c1);
    aA.c0 = fp2_add_mul_xi(t0, fp2_mul(a.c2, c1));
    aA.c1 = fp2_sub2(fp2_mul(fp2_add_lazy(a.c0, a.c1), fp2_add_lazy(c0, c1)), t0, t1);
    aA.c2 = fp2_add(t1, fp2_mul(a.c2, c0));
  }
  // bB, B = c2 v
  fp6_g<E> bB;
  bB.c0 = fp2_mul_xi(fp2_mul(b.c2, c2));
  bB.c1 = fp2_mul(b.c0, c2);
  bB.c2 = fp2_mul(b.c1, c2);
  // (a + b)(A + B), A + B = c0 + (c1 + c2) v
  const fp6_g<E> s = fp6_add(a, b);
  const E d1 = fp2_add(c1, c2);
  fp6_g<E> m;
  {
    const E t0 = fp2_mul(s.c0, c0);
    const E t1 = fp2_mul(s.c1, d1);
    m.c0 = fp2_add_mul_xi(t0, fp2_mul(s.c2, d1));
    m.c1 = fp2_sub2(fp2_mul(fp2_add_lazy(s.c0, s.c1), fp2_add_lazy(c0, d1)), t0, t1);
    m.c2 = fp2_add(t1, fp2_mul(s.c2, c0));
  }
  fp12_g<E> r;
  r.c0 = fp6_add_mul_by_v(aA, bB);
  r.c1 = fp6_sub2(m, aA, bB);
  return r;
}

template <class E>
BLS_NOINLINE fp12_g<E> fp12_mul_by_line(const fp12_g<E> f, const E c0, const E c1, const E c2) {
  return fp12_mul_by_line_inl(f, c0, c1, c2);
}

// Granger-Scott squaring in the cyclotomic subgroup.  View Fp12 as
// Fp4[w]/(w^3 - z), Fp4 = Fp2[z]/(z^2 - xi), z = w^3:
//   f = A + B w + C w^2,  A = a0 + b1 z,  B = b0 + a2 z,  C = a1 + b2 z
//   A' = 3A^2 - 2 conj(A),  B' = 3 z C^2 + 2 conj(B),  C' = 3 B^2 - 2 conj(C)
template <class E>
BLS_INLINE fp12_g<E> fp12_cyclotomic_sqr_inl(const fp12_g<E>& f) {
  auto sq4 = [](const E& x0, const E& x1, E& r0, E& r1) {
    const E t0 = fp2_sqr(x0);
    const E t1 = fp2_sqr(x1);
    r0 = fp2_add_mul_xi(t0, t1);
    r1 = fp2_sub2(fp2_sqr(fp2_add(x0, x1)), t0, t1);
  };
  // 3X - 2x and 3X + 2x, one reduction each
  auto m3s2 = [](const E& X, const E& x) { return fp2_3m2(X, x); };
  auto m3a2 = [](const E& X, const E& x) { return fp2_3p2(X, x); };
  // Each group's outputs are formed as soon as its squares exist, so few Fp2
  // values stay live across the squaring calls (register pressure, not math).
  fp12_g<E> r;
  E X0, X1;
  // A' = 3A^2 - 2 conj(A), A = a0 + b1 z
  sq4(f.c0.c0, f.c1.c1, X0, X1);
  r.c0.c0 = m3s2(X0, f.c0.c0);
  r.c1.c1 = m3a2(X1, f.c1.c1);
  // B' = 3 z C^2 + 2 conj(B), C = a1 + b2 z, B = b0 + a2 z;  z (C0 + C1 z) = xi C1 + C0 z
  sq4(f.c0.c1, f.c1.c2, X0, X1);
  r.c1.c0 = m3a2(fp2_mul_xi(X1), f.c1.c0);
  r.c0.c2 = m3s2(X0, f.c0.c2);
  // C' = 3B^2 - 2 conj(C)
  sq4(f.c1.c0, f.c0.c2, X0, X1);
  r.c0.c1 = m3s2(X0, f.c0.c1);
  r.c1.c2 = m3a2(X1, f.c1.c2);
  return r;
}

template <class E>
BLS_NOINLINE fp12_g<E> fp12_cyclotomic_sqr(const fp12_g<E> f) { return fp12_cyclotomic_sqr_inl(f); }

}  // namespace bls381
