// G1 = E(Fp): y^2 = x^3 + 4 and G2 = E'(Fp2): y^2 = x^3 + 4(1+u).
// Jacobian coordinates, a = 0 formulas; compressed codecs following
// specs/bls_signature.md:36-64 (strict) or py_ecc 1.7.0 (lax);
// endomorphism subgroup checks; scalar multiplication.
#pragma once
#include "bls381_field.hpp"

namespace bls381 {

// ---- field-generic helpers so one set of curve formulas serves G1 and G2
BLS_INLINE fp_t f_add(const fp_t& a, const fp_t& b) { return fp_add(a, b); }
BLS_INLINE fp2_t f_add(const fp2_t& a, const fp2_t& b) { return fp2_add(a, b); }
BLS_INLINE fp_t f_sub(const fp_t& a, const fp_t& b) { return fp_sub(a, b); }
BLS_INLINE fp2_t f_sub(const fp2_t& a, const fp2_t& b) { return fp2_sub(a, b); }
BLS_INLINE fp_t f_mul(const fp_t& a, const fp_t& b) { return fp_mul(a, b); }
BLS_INLINE fp2_t f_mul(const fp2_t& a, const fp2_t& b) { return fp2_mul(a, b); }
BLS_INLINE fp_t f_sqr(const fp_t& a) { return fp_sqr(a); }
BLS_INLINE fp2_t f_sqr(const fp2_t& a) { return fp2_sqr(a); }
BLS_INLINE fp_t f_dbl(const fp_t& a) { return fp_dbl(a); }
BLS_INLINE fp2_t f_dbl(const fp2_t& a) { return fp2_dbl(a); }
BLS_INLINE fp_t f_neg(const fp_t& a) { return fp_neg(a); }
BLS_INLINE fp2_t f_neg(const fp2_t& a) { return fp2_neg(a); }
BLS_INLINE fp_t f_sub2(const fp_t& a, const fp_t& b, const fp_t& c) { return fp_sub2(a, b, c); }
BLS_INLINE fp2_t f_sub2(const fp2_t& a, const fp2_t& b, const fp2_t& c) { return fp2_sub2(a, b, c); }
BLS_INLINE fp_t f_mul_small(const fp_t& a, int k) { return fp_mul_small(a, k); }
BLS_INLINE fp2_t f_mul_small(const fp2_t& a, int k) { return fp2_mul_small(a, k); }
BLS_INLINE bool f_is_zero(const fp_t& a) { return fp_is_zero(a); }
BLS_INLINE bool f_is_zero(const fp2_t& a) { return fp2_is_zero(a); }
BLS_INLINE bool f_eq(const fp_t& a, const fp_t& b) { return fp_eq(a, b); }
BLS_INLINE bool f_eq(const fp2_t& a, const fp2_t& b) { return fp2_eq(a, b); }
BLS_INLINE fp_t f_inv(const fp_t& a) { return fp_inv(a); }
BLS_INLINE fp2_t f_inv(const fp2_t& a) { return fp2_inv(a); }
BLS_INLINE void f_set_zero(fp_t& a) { a = fp_zero(); }
BLS_INLINE void f_set_zero(fp2_t& a) { a = fp2_zero(); }
BLS_INLINE void f_set_one(fp_t& a) { a = fp_one(); }
BLS_INLINE void f_set_one(fp2_t& a) { a = fp2_one(); }

template <class F> struct jac_t { F x, y, z; };
template <class F> struct aff_t { F x, y; };

template <class F>
BLS_INLINE jac_t<F> jac_infinity() {
  jac_t<F> r;
  f_set_one(r.x); f_set_one(r.y); f_set_zero(r.z);
  return r;
}

template <class F>
BLS_INLINE bool jac_is_inf(const jac_t<F>& p) { return f_is_zero(p.z); }

template <class F>
BLS_INLINE jac_t<F> jac_from_aff(const aff_t<F>& a) {
  jac_t<F> r; r.x = a.x; r.y = a.y; f_set_one(r.z); return r;
}

template <class F>
BLS_INLINE jac_t<F> jac_neg(const jac_t<F>& p) { jac_t<F> r = p; r.y = f_neg(p.y); return r; }

// dbl-2009-l (a = 0): 2M + 5S
template <class F>
BLS_DEV_INLINE jac_t<F> jac_dbl(const jac_t<F>& p) {
  const F A = f_sqr(p.x);
  const F B = f_sqr(p.y);
  const F C = f_sqr(B);
  const F xb = f_add(p.x, B);
  const F D = f_dbl(f_sub2(f_sqr(xb), A, C));
  const F E = f_mul_small(A, 3);
  const F Fv = f_sqr(E);
  jac_t<F> r;
  r.x = f_sub2(Fv, D, D);
  r.y = f_sub(f_mul(E, f_sub(D, r.x)), f_mul_small(C, 8));
  r.z = f_dbl(f_mul(p.y, p.z));
  return r;   // Z = 0 stays 0 (infinity doubles to infinity)
}

// add-2007-bl full Jacobian addition with the exceptional cases
template <class F>
BLS_DEV_INLINE jac_t<F> jac_add(const jac_t<F>& p, const jac_t<F>& q) {
  if (jac_is_inf(p)) return q;
  if (jac_is_inf(q)) return p;
  const F Z1Z1 = f_sqr(p.z);
  const F Z2Z2 = f_sqr(q.z);
  const F U1 = f_mul(p.x, Z2Z2);
  const F U2 = f_mul(q.x, Z1Z1);
  const F S1 = f_mul(f_mul(p.y, q.z), Z2Z2);
  const F S2 = f_mul(f_mul(q.y, p.z), Z1Z1);
  const F H = f_sub(U2, U1);
  const F R = f_sub(S2, S1);
  if (f_is_zero(H)) {
    if (f_is_zero(R)) return jac_dbl(p);
    return jac_infinity<F>();
  }
  const F HH = f_sqr(H);
  const F HHH = f_mul(H, HH);
  const F V = f_mul(U1, HH);
  jac_t<F> r;
  r.x = f_sub2(f_sqr(R), HHH, f_dbl(V));
  r.y = f_sub(f_mul(R, f_sub(V, r.x)), f_mul(S1, HHH));
  r.z = f_mul(f_mul(p.z, q.z), H);
  return r;
}

// mixed addition p + (x2, y2) with an affine, finite second operand
template <class F>
BLS_DEV_INLINE jac_t<F> jac_add_aff(const jac_t<F>& p, const aff_t<F>& q) {
  if (jac_is_inf(p)) return jac_from_aff(q);
  const F Z1Z1 = f_sqr(p.z);
  const F U2 = f_mul(q.x, Z1Z1);
  const F S2 = f_mul(f_mul(q.y, p.z), Z1Z1);
  const F H = f_sub(U2, p.x);
  const F R = f_sub(S2, p.y);
  if (f_is_zero(H)) {
    if (f_is_zero(R)) return jac_dbl(p);
    return jac_infinity<F>();
  }
  const F HH = f_sqr(H);
  const F HHH = f_mul(H, HH);
  const F V = f_mul(p.x, HH);
  jac_t<F> r;
  r.x = f_sub2(f_sqr(R), HHH, f_dbl(V));
  r.y = f_sub(f_mul(R, f_sub(V, r.x)), f_mul(p.y, HHH));
  r.z = f_mul(p.z, H);
  return r;
}

template <class F>
BLS_DEV_INLINE bool jac_to_aff(aff_t<F>& out, const jac_t<F>& p) {
  if (jac_is_inf(p)) return false;
  const F zi = f_inv(p.z);
  const F zi2 = f_sqr(zi);
  out.x = f_mul(p.x, zi2);
  out.y = f_mul(f_mul(p.y, zi2), zi);
  return true;
}

// Scalar multiplications are one (non-inlined) function each, with the point
// formulas inlined into the loop, so the running point stays in registers.
// [k] a for a 64-bit scalar, affine base, left-to-right (the body, for callers that inline it)
template <class F>
BLS_DEV_INLINE jac_t<F> jac_mul_u64_body(const aff_t<F>& a, uint64_t k) {
  jac_t<F> r = jac_from_aff(a);
  int top = 63;
  while (top > 0 && !((k >> top) & 1)) --top;
  for (int i = top - 1; i >= 0; --i) {
    r = jac_dbl(r);
    if ((k >> i) & 1) r = jac_add_aff(r, a);
  }
  return r;
}
template <class F>
BLS_NOINLINE jac_t<F> jac_mul_u64(const aff_t<F> a, uint64_t k) { return jac_mul_u64_body(a, k); }

// [k0] a + [k1] s for 32-bit k0, k1 (Shamir's trick: one doubling chain, mixed additions);
// with s = endo(a) for an endomorphism acting as [mu] this is [k0 + mu k1] a at half the
// doublings of a 64-bit multiplication (the randomized-batch weights)
template <class F>
BLS_NOINLINE jac_t<F> jac_mul_2x32(const aff_t<F> a, const aff_t<F> s, uint32_t k0, uint32_t k1) {
  jac_t<F> r = jac_infinity<F>();
  const uint32_t any = k0 | k1;
  int top = 31;
  while (top > 0 && !((any >> top) & 1u)) --top;
  for (int i = top; i >= 0; --i) {
    if (i != top) r = jac_dbl(r);
    if ((k0 >> i) & 1u) r = jac_add_aff(r, a);
    if ((k1 >> i) & 1u) r = jac_add_aff(r, s);
  }
  return r;
}

// [k] p for a 64-bit scalar, Jacobian base
template <class F>
BLS_DEV_INLINE jac_t<F> jac_mul_u64_jac_body(const jac_t<F>& p, uint64_t k) {
  jac_t<F> r = p;
  int top = 63;
  while (top > 0 && !((k >> top) & 1)) --top;
  for (int i = top - 1; i >= 0; --i) {
    r = jac_dbl(r);
    if ((k >> i) & 1) r = jac_add(r, p);
  }
  return r;
}
template <class F>
BLS_NOINLINE jac_t<F> jac_mul_u64_jac(const jac_t<F> p, uint64_t k) { return jac_mul_u64_jac_body(p, k); }

// a scalar of up to 512 bits, little-endian 32-bit words, passed by value (no pointer into the
// caller's private memory crosses a call: DESIGN.md §10.8)
struct scalar_t { uint32_t w[16]; };

// [k] a for a little-endian multi-limb scalar (nbits <= 512 significant bits)
template <class F>
BLS_NOINLINE jac_t<F> jac_mul_limbs(const aff_t<F> a, const scalar_t k, int nbits) {
  jac_t<F> r = jac_infinity<F>();
  for (int i = nbits - 1; i >= 0; --i) {
    r = jac_dbl(r);
    if ((k.w[i >> 5] >> (i & 31)) & 1u) r = jac_add_aff(r, a);
  }
  return r;
}

// ------------------------------------------------------------- codecs -----
enum : int { PT_OK = 0, PT_INF = 1, PT_BAD = 2 };

// Codecs.  Two decoders share one body, selected per call by the policy
// (include/bls381.h BLS381_POLICY_*; DESIGN.md §3 "Codec"):
//   strict (lax == false): specs/bls_signature.md:47-52,58-64 -- c_flag set, x < q,
//     infinity only as the canonical 0xc0 || 00.. encoding, G2's z2 flags clear;
//   lax (lax == true): py_ecc 1.7.0 decompress_G1 / decompress_G2 --
//     b_flag set means infinity whatever the other bits; otherwise x = z mod 2^381
//     (G1, G2's imaginary part) or the whole 384-bit z2 (G2's real part), reduced
//     mod q; c_flag and x < q are never looked at.
// Both accept every canonical encoding with the same point; the lax decoder also
// accepts non-canonical encodings (strict PT_BAD).  g1_canonical tells them apart.
BLS_DEV_INLINE bool g1_canonical(const uint8_t* b48) {
  const uint8_t top = b48[0];
  const int c_flag = (top >> 7) & 1, b_flag = (top >> 6) & 1, a_flag = (top >> 5) & 1;
  uint8_t tmp[48];
  for (int i = 0; i < 48; ++i) tmp[i] = b48[i];
  tmp[0] &= 0x1f;
  const fp_t x = fp_plain_from_be48(tmp);
  if (!c_flag) return false;
  if (b_flag) return a_flag == 0 && fp_plain_is_zero(x);
  return fp_plain_lt_q(x);
}

// G1 decompress (bls_signature.md:36-52 / py_ecc decompress_G1).  PT_OK / PT_INF / PT_BAD.
BLS_DEV_INLINE int g1_decompress(aff_t<fp_t>& out, const uint8_t* b48, bool lax) {
  const uint8_t top = b48[0];
  const int b_flag = (top >> 6) & 1, a_flag = (top >> 5) & 1;
  if (!lax && !g1_canonical(b48)) return PT_BAD;
  if (b_flag) return PT_INF;
  uint8_t tmp[48];
  for (int i = 0; i < 48; ++i) tmp[i] = b48[i];
  tmp[0] &= 0x1f;
  const fp_t x = fp_plain_from_be48(tmp);          // < 2^381; lax: may be >= q
  const fp_t xm = fp_to_mont(x);                   // reduces mod q
  const fp_t rhs = fp_add(fp_mul(fp_sqr(xm), xm), G1_B_M);
  fp_t y;
  if (!fp_sqrt(y, rhs)) return PT_BAD;
  if ((int)fp_plain_is_upper_half(fp_from_mont(y)) != a_flag) y = fp_neg(y);
  out.x = xm;
  out.y = y;
  return PT_OK;
}

BLS_DEV_INLINE void g1_compress(uint8_t* b48, const jac_t<fp_t>& p) {
  aff_t<fp_t> a;
  if (!jac_to_aff(a, p)) {
    for (int i = 0; i < 48; ++i) b48[i] = 0;
    b48[0] = 0xc0;
    return;
  }
  const fp_t x = fp_from_mont(a.x);
  const fp_t y = fp_from_mont(a.y);
  fp_plain_to_be48(b48, x);
  b48[0] |= 0x80 | (fp_plain_is_upper_half(y) ? 0x20 : 0);
}

// a_flag rule of py_ecc compress/decompress_G2: from y_im, or y_re if y_im == 0
BLS_INLINE int g2_y_flag(const fp2_t& y_mont) {
  const fp_t yi = fp_from_mont(y_mont.c1);
  if (!fp_is_zero(yi)) return fp_plain_is_upper_half(yi) ? 1 : 0;
  return fp_plain_is_upper_half(fp_from_mont(y_mont.c0)) ? 1 : 0;
}

// strict-codec acceptance of a G2 encoding (bls_signature.md:58-64)
BLS_DEV_INLINE bool g2_canonical(const uint8_t* b96) {
  const uint8_t top = b96[0];
  const int c1 = (top >> 7) & 1, b1 = (top >> 6) & 1, a1 = (top >> 5) & 1;
  if (b96[48] & 0xe0) return false;               // a_flag2 == b_flag2 == c_flag2 == 0
  uint8_t tmp[48];
  for (int i = 0; i < 48; ++i) tmp[i] = b96[i];
  tmp[0] &= 0x1f;
  const fp_t x_im = fp_plain_from_be48(tmp);
  const fp_t x_re = fp_plain_from_be48(b96 + 48);
  if (!c1) return false;
  if (b1) return a1 == 0 && fp_plain_is_zero(x_im) && fp_plain_is_zero(x_re);
  return fp_plain_lt_q(x_im) && fp_plain_lt_q(x_re);
}

// G2 decompress (bls_signature.md:54-64 / py_ecc decompress_G2): z1 = flags | x_im,
// z2 = x_re (lax: all 384 bits of z2, flags included, reduced mod q)
BLS_DEV_INLINE int g2_decompress(aff_t<fp2_t>& out, const uint8_t* b96, bool lax) {
  const uint8_t top = b96[0];
  const int b1 = (top >> 6) & 1, a1 = (top >> 5) & 1;
  if (!lax && !g2_canonical(b96)) return PT_BAD;
  if (b1) return PT_INF;
  uint8_t tmp[48];
  for (int i = 0; i < 48; ++i) tmp[i] = b96[i];
  tmp[0] &= 0x1f;
  const fp_t x_im = fp_plain_from_be48(tmp);
  const fp_t x_re = fp_plain_from_be48(b96 + 48);
  fp2_t x;
  x.c0 = fp_to_mont(x_re);
  x.c1 = fp_to_mont(x_im);
  const fp2_t rhs = fp2_add(fp2_mul(fp2_sqr(x), x), G2_B_M);
  fp2_t y;
  if (!fp2_sqrt(y, rhs)) return PT_BAD;
  if (g2_y_flag(y) != a1) y = fp2_neg(y);
  out.x = x;
  out.y = y;
  return PT_OK;
}

BLS_DEV_INLINE void g2_compress_aff(uint8_t* b96, const aff_t<fp2_t>& a) {
  fp_plain_to_be48(b96, fp_from_mont(a.x.c1));
  fp_plain_to_be48(b96 + 48, fp_from_mont(a.x.c0));
  b96[0] |= 0x80 | (g2_y_flag(a.y) ? 0x20 : 0);
}

BLS_DEV_INLINE void g2_compress(uint8_t* b96, const jac_t<fp2_t>& p) {
  aff_t<fp2_t> a;
  if (!jac_to_aff(a, p)) {
    for (int i = 0; i < 96; ++i) b96[i] = 0;
    b96[0] = 0xc0;
    return;
  }
  g2_compress_aff(b96, a);
}

// ---------------------------------------------------- subgroup checks -----
// G1: sigma(P) = (beta x, y) acts on G1 as [-x^2]; P in G1 iff sigma(P) == -[x^2]P.
BLS_DEV_INLINE bool g1_in_subgroup(const aff_t<fp_t>& p) {
  const jac_t<fp_t> t = jac_mul_u64_jac(jac_mul_u64(p, BLS_X_ABS), BLS_X_ABS);  // [x^2] P
  if (jac_is_inf(t)) return false;
  const fp_t zz = fp_sqr(t.z);
  const fp_t zzz = fp_mul(zz, t.z);
  // sigma(P) == -T  <=>  beta*x*Z^2 == X  and  y*Z^3 == -Y
  return fp_eq(fp_mul(fp_mul(G1_BETA_M, p.x), zz), t.x) && fp_eq(fp_mul(p.y, zzz), fp_neg(t.y));
}

// psi(x, y) = (cx * conj(x), cy * conj(y)) on E'(Fp2)
template <class E>
BLS_INLINE aff_t<E> g2_psi(const aff_t<E>& a) {
  aff_t<E> r;
  r.x = fp2_mul(e2_k<E>(PSI_CX_M), fp2_conj(a.x));
  r.y = fp2_mul(e2_k<E>(PSI_CY_M), fp2_conj(a.y));
  return r;
}

// G2: Q in G2 iff psi(Q) == [x]Q = -[|x|]Q
template <class E>
BLS_DEV_INLINE bool g2_in_subgroup(const aff_t<E>& q) {
  const jac_t<E> t = jac_mul_u64(q, BLS_X_ABS);
  if (jac_is_inf(t)) return false;
  const aff_t<E> s = g2_psi(q);
  const E zz = fp2_sqr(t.z);
  const E zzz = fp2_mul(zz, t.z);
  return fp2_eq(fp2_mul(s.x, zz), t.x) && fp2_eq(fp2_mul(s.y, zzz), fp2_neg(t.y));
}

}  // namespace bls381
