// Fp12 on a lane quad -- the Miller-loop representation of the gfx950 kernels.
//
// Item i owns lanes 4i..4i+3.  Lanes 4i+{0,1} ("lo") hold the Fp6 half c0 of
// every Fp12 value, lanes 4i+{2,3} ("hi") the half c1, each as the lane-pair
// Fp2 of bls381_pair.hpp (lane 4i+2h+p: coefficient p).  So an item's Fp12 is
// 3 Fp per lane (42 VGPRs) instead of 6 on a lane pair, and every Fp12 product
// runs its two Fp6 halves side by side:
//   * square     (a + bw)^2:  lo a*b, hi (a+b)(a+vb)            6 Fp2-product steps
//   * product    (a + bw)(c + dw): lo a*c, hi b*d, then the three
//                Karatsuba products of (a+b)(c+d) split 3 + 3   9 steps
//   * two lines  l_lo * l_hi (one per half, sparse): 8 products,  4 steps
// against 12 / 18 / 26 sequential Fp2 products on a lane pair: the same lane
// work, half the per-lane state and half the latency per item.  The two halves
// also carry the two Miller-loop pairs of a bls_verify (lo: (sig, -g1), hi:
// (H(m), pk)), whose line functions then run in parallel.
//
// Cross-half moves are DPP quad_perm (full-rate VALU, no LDS).  Control flow
// must be uniform within a quad: every half-dependent choice below is a
// per-lane select, never a branch.
#pragma once
#include "bls381_pair.hpp"

namespace bls381 {

enum : int {
  DPP_HSWAP = 0x4E,   // [2,3,0,1]: the other half's value
};

__device__ __forceinline__ bool qd_hi() { return (threadIdx.x & 2u) != 0; }

using fp6p_t = fp6_g<fp2p_t>;

__device__ __forceinline__ fp2p_t qd_swap(const fp2p_t& a) { return pr_make(pr_dpp<DPP_HSWAP>(a.v)); }
__device__ __forceinline__ fp6p_t qd_swap(const fp6p_t& a) {
  fp6p_t r; r.c0 = qd_swap(a.c0); r.c1 = qd_swap(a.c1); r.c2 = qd_swap(a.c2); return r;
}
__device__ __forceinline__ fp2p_t qd_sel(bool c, const fp2p_t& a, const fp2p_t& b) { return pr_make(fp_sel(c, a.v, b.v)); }
__device__ __forceinline__ fp6p_t qd_sel(bool c, const fp6p_t& a, const fp6p_t& b) {
  fp6p_t r; r.c0 = qd_sel(c, a.c0, b.c0); r.c1 = qd_sel(c, a.c1, b.c1); r.c2 = qd_sel(c, a.c2, b.c2); return r;
}
// a predicate true on all four lanes of the quad
__device__ __forceinline__ bool qd_all(bool b) { return (pr_dpp<DPP_HSWAP>((uint32_t)b) & (uint32_t)b) != 0; }

// this lane's half of an Fp12: lo -> c0, hi -> c1
struct fq12_t { fp6p_t h; };

__device__ __forceinline__ fq12_t fq12_one() {
  fq12_t r;
  r.h = qd_sel(qd_hi(), fp6_zero<fp2p_t>(), fp6_one<fp2p_t>());
  return r;
}

__device__ __forceinline__ fq12_t fq12_conj(const fq12_t& f) {
  fq12_t r;
  r.h = qd_sel(qd_hi(), fp6_neg(f.h), f.h);
  return r;
}

// (s0 + s1 v + s2 v^2)(t0 + t1 v + t2 v^2) with the six Karatsuba products split
// between the halves (lo: s_k t_k, hi: the three cross sums), three steps; the
// result is formed on both halves.  s, t are the same on both halves.
__device__ __forceinline__ fp6p_t fp6_mul_split(const fp6p_t& s, const fp6p_t& t) {
  const bool hi = qd_hi();
  fp2p_t p[3];
  p[0] = fp2_mul(qd_sel(hi, fp2_add_lazy(s.c1, s.c2), s.c0), qd_sel(hi, fp2_add_lazy(t.c1, t.c2), t.c0));
  p[1] = fp2_mul(qd_sel(hi, fp2_add_lazy(s.c0, s.c1), s.c1), qd_sel(hi, fp2_add_lazy(t.c0, t.c1), t.c1));
  p[2] = fp2_mul(qd_sel(hi, fp2_add_lazy(s.c0, s.c2), s.c2), qd_sel(hi, fp2_add_lazy(t.c0, t.c2), t.c2));
  fp2p_t o[3];
  for (int k = 0; k < 3; ++k) o[k] = qd_swap(p[k]);
  // t0..t2 = s_k t_k, t3..t5 = cross products, whichever half computed them
  const fp2p_t t0 = qd_sel(hi, o[0], p[0]), t1 = qd_sel(hi, o[1], p[1]), t2 = qd_sel(hi, o[2], p[2]);
  const fp2p_t t3 = qd_sel(hi, p[0], o[0]), t4 = qd_sel(hi, p[1], o[1]), t5 = qd_sel(hi, p[2], o[2]);
  fp6p_t r;
  r.c0 = fp2_add_mul_xi(t0, fp2_sub2(t3, t1, t2));
  r.c1 = fp2_add_mul_xi(fp2_sub2(t4, t0, t1), t2);
  r.c2 = fp2_add(fp2_sub2(t5, t0, t2), t1);
  return r;
}

// (a + b w)(c + d w) = (ac + v bd) + ((a+b)(c+d) - ac - bd) w
__device__ __forceinline__ fq12_t fq12_mul(const fq12_t& f, const fq12_t& g) {
  const bool hi = qd_hi();
  const fp6p_t yf = qd_swap(f.h), yg = qd_swap(g.h);
  const fp6p_t p = fp6_mul_inl(f.h, g.h);            // lo: ac, hi: bd
  const fp6p_t m = fp6_mul_split(fp6_add(f.h, yf), fp6_add(g.h, yg));
  const fp6p_t o = qd_swap(p);                        // lo: bd, hi: ac
  fq12_t r;
  r.h = qd_sel(hi, fp6_sub2(m, o, p), fp6_add_mul_by_v(p, o));
  return r;
}

// (a + b w)^2 = ((a+b)(a+vb) - ab - v ab) + 2ab w
__device__ __forceinline__ fq12_t fq12_sqr(const fq12_t& f) {
  const bool hi = qd_hi();
  const fp6p_t y = qd_swap(f.h);                      // lo: b, hi: a
  const fp6p_t u = qd_sel(hi, fp6_add(f.h, y), f.h);  // lo: a, hi: a + b
  const fp6p_t v = qd_sel(hi, fp6_add_mul_by_v(y, f.h), y);   // lo: b, hi: a + v b
  const fp6p_t p = fp6_mul_inl(u, v);                 // lo: ab, hi: (a+b)(a+vb)
  const fp6p_t o = qd_swap(p);                        // lo: (a+b)(a+vb), hi: ab
  fq12_t r;
  r.h = qd_sel(hi, fp6_dbl(o), fp6_sub2(o, p, fp6_mul_by_v(p)));
  return r;
}

// The product of the two halves' sparse lines l = c0 + c1 v + c2 v w (lo: the
// lo pair's line, hi: the hi pair's line, (1, 0, 0) when that pair is idle):
//   l * l' = (c0d0 + xi c2d2 + (c0d1 + c1d0) v + c1d1 v^2)
//          + ((c0d2 + c2d0) v + (c1d2 + c2d1) v^2) w,
// eight products in four steps (lo takes the w^0 half's, hi the w^1 half's).
__device__ __forceinline__ fq12_t fq12_two_lines(const fp2p_t& x0, const fp2p_t& x1, const fp2p_t& x2) {
  const bool hi = qd_hi();
  const fp2p_t y0 = qd_swap(x0), y1 = qd_swap(x1), y2 = qd_swap(x2);
  // c = lo's line, d = hi's line, on every lane
  const fp2p_t c0 = qd_sel(hi, y0, x0), c1 = qd_sel(hi, y1, x1), c2 = qd_sel(hi, y2, x2);
  const fp2p_t d0 = qd_sel(hi, x0, y0), d1 = qd_sel(hi, x1, y1), d2 = qd_sel(hi, x2, y2);
  const fp2p_t p0 = fp2_mul(c0, qd_sel(hi, d2, d0));                                        // c0d0 | c0d2
  const fp2p_t p1 = fp2_mul(qd_sel(hi, c2, c1), qd_sel(hi, d0, d1));                        // c1d1 | c2d0
  const fp2p_t p2 = fp2_mul(qd_sel(hi, c1, fp2_add_lazy(c0, c1)), qd_sel(hi, d2, fp2_add_lazy(d0, d1)));
  const fp2p_t p3 = fp2_mul(c2, qd_sel(hi, d1, d2));                                        // c2d2 | c2d1
  fq12_t r;
  r.h.c0 = qd_sel(hi, e2_zero<fp2p_t>(), fp2_add_mul_xi(p0, p3));
  r.h.c1 = qd_sel(hi, fp2_add(p0, p1), fp2_sub2(p2, p0, p1));
  r.h.c2 = qd_sel(hi, fp2_add(p2, p3), p1);
  return r;
}

// Miller loop of two pairs at once, one per half: this lane's half runs
// (Q, P); `active` = this half's pair takes part (an idle half's line is 1).
// Returns conj(f_lo f_hi) (x < 0) in quad form.  `degenerate` (same on all four
// lanes) is set when an active pair's running point reached infinity
// (miller_loop_n: py_ecc's zero pairing value).
#ifndef BLS_ML_QUAD_INLINE
#define BLS_ML_QUAD_INLINE 0
#endif
// (operands and results by value: no pointer into the caller's private memory crosses the
// call; the reference form below is a force-inlined wrapper)
struct fq12_ml { fq12_t f; bool degenerate; };
#if BLS_ML_QUAD_INLINE
__device__ __forceinline__
#else
__device__ __noinline__
#endif
fq12_ml miller_loop_quad_run(const aff_t<fp2p_t> Q, const g1_line_pre P, bool active) {
  g2_proj<fp2p_t> T;
  T.x = Q.x; T.y = Q.y; T.z = e2_one<fp2p_t>();
  const fp2p_t one = e2_one<fp2p_t>(), zero = e2_zero<fp2p_t>();
  fq12_t f;
  bool first = true;
  for (int i = 62; i >= 0; --i) {
    fp2p_t c0, c1, c2;
    line_dbl(T, P, c0, c1, c2);
    const fq12_t L = fq12_two_lines(qd_sel(active, c0, one), qd_sel(active, c1, zero), qd_sel(active, c2, zero));
    f = first ? L : fq12_mul(fq12_sqr(f), L);
    first = false;
    if ((BLS_X_ABS >> i) & 1) {
      line_add(T, Q, P, c0, c1, c2);
      f = fq12_mul(f, fq12_two_lines(qd_sel(active, c0, one), qd_sel(active, c1, zero), qd_sel(active, c2, zero)));
    }
  }
  const bool deg = active && fp2_is_zero(T.z);
  fq12_ml r;
  r.degenerate = !qd_all(!deg);
  r.f = fq12_conj(f);
  return r;
}

__device__ __forceinline__ fq12_t miller_loop_quad(const aff_t<fp2p_t>& Q, const g1_line_pre& P, bool active,
                                                   bool& degenerate) {
  const fq12_ml r = miller_loop_quad_run(Q, P, active);
  degenerate = r.degenerate;
  return r.f;
}

// ------------------------------------------------ one Miller pair per quad --
// The latency form of the Miller loop: one pair per quad, T held on both halves,
// and the independent products of every step split over the halves:
//   doubling (line_dbl)       11 products -> 6 steps
//   addition (line_add)       15 products -> 8 steps
//   f * line (sparse)         13 products -> 7 steps
//   f^2                       12 products -> 6 steps (fq12_sqr)
// so a doubling iteration is 19 product steps against 30 for the two-pair quad
// loop above (and 36 for one pair on a lane pair).  Values computed on both
// halves from the same inputs stay bit-identical, so T needs no exchange.

// line_dbl with its products split: lo X^2 | hi Y^2, lo Z^2 | hi YZ, XY (both);
// then lo XX(-3xp) | hi YZ(2yp), lo XY(YY - 9b'Z^2) | hi YY YZ, lo h^2 | hi (3b'Z^2)^2
__device__ __forceinline__ void line_dbl_q1(g2_proj<fp2p_t>& T, const g1_line_pre& P, fp2p_t& c0, fp2p_t& c1,
                                            fp2p_t& c2) {
  const bool hi = qd_hi();
  const fp2p_t s1 = fp2_sqr(qd_sel(hi, T.y, T.x));
  const fp2p_t m1 = fp2_mul(T.z, qd_sel(hi, T.y, T.z));
  const fp2p_t XY = fp2_mul(T.x, T.y);
  const fp2p_t s1o = qd_swap(s1), m1o = qd_swap(m1);
  const fp2p_t XX = qd_sel(hi, s1o, s1), YY = qd_sel(hi, s1, s1o);
  const fp2p_t ZZ = qd_sel(hi, m1o, m1), YZ = qd_sel(hi, m1, m1o);
  const fp2p_t b3 = fp2_mul_small(fp2_mul_small(fp2_mul_xi(ZZ), 3), 4);   // 3 b' Z^2
  const fp2p_t b9 = fp2_mul_small(b3, 3);
  c0 = fp2_sub(YY, b3);
  const fp2p_t e = fp2_mul_fp(qd_sel(hi, YZ, XX), fp_sel(hi, P.y2, P.n3x));
  const fp2p_t h = fp2_half(fp2_add(YY, b9));
  const fp2p_t m2 = fp2_mul(qd_sel(hi, YY, XY), qd_sel(hi, YZ, fp2_sub(YY, b9)));
  const fp2p_t s2 = fp2_sqr(qd_sel(hi, b3, h));
  const fp2p_t eo = qd_swap(e), m2o = qd_swap(m2), s2o = qd_swap(s2);
  c1 = qd_sel(hi, eo, e);
  c2 = qd_sel(hi, e, eo);
  T.x = fp2_half(qd_sel(hi, m2o, m2));
  T.y = fp2_sub(qd_sel(hi, s2o, s2), fp2_mul_small(qd_sel(hi, s2, s2o), 3));
  T.z = fp2_dbl(qd_sel(hi, m2, m2o));
}

// ------------------------------------------- G2 point arithmetic on a quad --
// The latency form of hash_to_G2's cofactor map (k_hash_g2_q): the running point is held on both
// halves and the independent products of each step run on the two halves at once, as in
// line_dbl_q1.  Every value is the same on both halves after each step, so the exceptional-case
// branches of the point formulas stay uniform within the quad.  The same formulas as
// bls381_curve.hpp (dbl-2009-l, add-2007-bl, mixed addition); a square paired with a product runs
// as a product of the value with itself (the same field element; representations < 2q).
//   jac_dbl 7 products -> 4 steps, jac_add_aff 11 -> 6, jac_add 16 -> 8, psi 2 -> 1.
// lo's value and hi's value of a split step, on both halves
__device__ __forceinline__ void qd_both(const fp2p_t& mine, fp2p_t& lo_v, fp2p_t& hi_v) {
  const bool hi = qd_hi();
  const fp2p_t o = qd_swap(mine);
  lo_v = qd_sel(hi, o, mine);
  hi_v = qd_sel(hi, mine, o);
}

__device__ __forceinline__ jac_t<fp2p_t> jac_dbl_q(const jac_t<fp2p_t>& p) {
  const bool hi = qd_hi();
  fp2p_t A, B, C, XB2, Fv, YZ;
  qd_both(fp2_sqr(qd_sel(hi, p.y, p.x)), A, B);                                   // X^2 | Y^2
  qd_both(fp2_sqr(qd_sel(hi, fp2_add(p.x, B), B)), C, XB2);                       // B^2 | (X + B)^2
  const fp2p_t D = fp2_dbl(fp2_sub2(XB2, A, C));
  const fp2p_t E = fp2_mul_small(A, 3);
  qd_both(fp2_mul(qd_sel(hi, p.y, E), qd_sel(hi, p.z, E)), Fv, YZ);              // E^2 | Y Z
  jac_t<fp2p_t> r;
  r.x = fp2_sub2(Fv, D, D);
  r.y = fp2_sub(fp2_mul(E, fp2_sub(D, r.x)), fp2_mul_small(C, 8));
  r.z = fp2_dbl(YZ);
  return r;   // Z = 0 stays 0
}

__device__ __forceinline__ jac_t<fp2p_t> jac_add_aff_q(const jac_t<fp2p_t>& p, const aff_t<fp2p_t>& q) {
  if (jac_is_inf(p)) return jac_from_aff(q);
  const bool hi = qd_hi();
  fp2p_t Z1Z1, Y2Z1, U2, S2;
  qd_both(fp2_mul(p.z, qd_sel(hi, q.y, p.z)), Z1Z1, Y2Z1);                       // Z1^2 | y2 Z1
  qd_both(fp2_mul(Z1Z1, qd_sel(hi, Y2Z1, q.x)), U2, S2);                         // x2 Z1Z1 | y2 Z1 Z1Z1
  const fp2p_t H = fp2_sub(U2, p.x);
  const fp2p_t R = fp2_sub(S2, p.y);
  if (fp2_is_zero(H)) {
    if (fp2_is_zero(R)) return jac_dbl_q(p);
    return jac_infinity<fp2p_t>();
  }
  fp2p_t HH, Z3, HHH, V, RR, YH;
  qd_both(fp2_mul(H, qd_sel(hi, p.z, H)), HH, Z3);                               // H^2 | Z1 H
  qd_both(fp2_mul(HH, qd_sel(hi, p.x, H)), HHH, V);                              // H HH | X1 HH
  qd_both(fp2_mul(qd_sel(hi, p.y, R), qd_sel(hi, HHH, R)), RR, YH);              // R^2 | Y1 HHH
  jac_t<fp2p_t> r;
  r.x = fp2_sub2(RR, HHH, fp2_dbl(V));
  r.y = fp2_sub(fp2_mul(R, fp2_sub(V, r.x)), YH);
  r.z = Z3;
  return r;
}

__device__ __forceinline__ jac_t<fp2p_t> jac_add_q(const jac_t<fp2p_t>& p, const jac_t<fp2p_t>& q) {
  if (jac_is_inf(p)) return q;
  if (jac_is_inf(q)) return p;
  const bool hi = qd_hi();
  fp2p_t Z1Z1, Z2Z2, U1, U2, Y1Z2, Y2Z1, S1, S2;
  qd_both(fp2_sqr(qd_sel(hi, q.z, p.z)), Z1Z1, Z2Z2);                            // Z1^2 | Z2^2
  qd_both(fp2_mul(qd_sel(hi, q.x, p.x), qd_sel(hi, Z1Z1, Z2Z2)), U1, U2);       // X1 Z2Z2 | X2 Z1Z1
  qd_both(fp2_mul(qd_sel(hi, q.y, p.y), qd_sel(hi, p.z, q.z)), Y1Z2, Y2Z1);     // Y1 Z2 | Y2 Z1
  qd_both(fp2_mul(qd_sel(hi, Y2Z1, Y1Z2), qd_sel(hi, Z1Z1, Z2Z2)), S1, S2);     // Y1 Z2 Z2Z2 | Y2 Z1 Z1Z1
  const fp2p_t H = fp2_sub(U2, U1);
  const fp2p_t R = fp2_sub(S2, S1);
  if (fp2_is_zero(H)) {
    if (fp2_is_zero(R)) return jac_dbl_q(p);
    return jac_infinity<fp2p_t>();
  }
  fp2p_t HH, Z1Z2, HHH, V, RR, SH;
  qd_both(fp2_mul(qd_sel(hi, p.z, H), qd_sel(hi, q.z, H)), HH, Z1Z2);           // H^2 | Z1 Z2
  qd_both(fp2_mul(HH, qd_sel(hi, U1, H)), HHH, V);                               // H HH | U1 HH
  qd_both(fp2_mul(qd_sel(hi, S1, R), qd_sel(hi, HHH, R)), RR, SH);               // R^2 | S1 HHH
  jac_t<fp2p_t> r;
  r.x = fp2_sub2(RR, HHH, fp2_dbl(V));
  fp2p_t RV, Z3;
  qd_both(fp2_mul(qd_sel(hi, Z1Z2, R), qd_sel(hi, H, fp2_sub(V, r.x))), RV, Z3); // R (V - X3) | Z1 Z2 H
  r.y = fp2_sub(RV, SH);
  r.z = Z3;
  return r;
}

// psi on Jacobian coordinates: (cx conj(X), cy conj(Y), conj(Z)), the two products at once
__device__ __forceinline__ jac_t<fp2p_t> g2_psi_jac_q(const jac_t<fp2p_t>& p) {
  const bool hi = qd_hi();
  jac_t<fp2p_t> r;
  const fp2p_t k = qd_sel(hi, e2_k<fp2p_t>(PSI_CY_M), e2_k<fp2p_t>(PSI_CX_M));
  qd_both(fp2_mul(k, fp2_conj(qd_sel(hi, p.y, p.x))), r.x, r.y);
  r.z = fp2_conj(p.z);
  return r;
}

// [k] a (affine base) and [k] p (Jacobian base) for a 64-bit k, left to right
__device__ __noinline__ jac_t<fp2p_t> jac_mul_u64_q(const aff_t<fp2p_t> a, uint64_t k) {
  jac_t<fp2p_t> r = jac_from_aff(a);
  int top = 63;
  while (top > 0 && !((k >> top) & 1)) --top;
  for (int i = top - 1; i >= 0; --i) {
    r = jac_dbl_q(r);
    if ((k >> i) & 1) r = jac_add_aff_q(r, a);
  }
  return r;
}
__device__ __noinline__ jac_t<fp2p_t> jac_mul_u64_jac_q(const jac_t<fp2p_t> p, uint64_t k) {
  jac_t<fp2p_t> r = p;
  int top = 63;
  while (top > 0 && !((k >> top) & 1)) --top;
  for (int i = top - 1; i >= 0; --i) {
    r = jac_dbl_q(r);
    if ((k >> i) & 1) r = jac_add_q(r, p);
  }
  return r;
}

// g2_mul_bp (bls381_hash.hpp) on a quad: BP(P) = [x^2 - x - 1]P + [x - 1]psi(P) + 2 psi^2(P)
__device__ __noinline__ jac_t<fp2p_t> g2_mul_bp_q(const aff_t<fp2p_t> p) {
  aff_t<fp2p_t> np;
  np.x = p.x;
  np.y = fp2_neg(p.y);
  const jac_t<fp2p_t> t1 = jac_mul_u64_q(p, BLS_X_ABS);                                   // [|x|]P
  jac_t<fp2p_t> Q0 = jac_add_aff_q(jac_add_q(jac_mul_u64_jac_q(t1, BLS_X_ABS), t1), np);  // [x^2 - x - 1]P
  Q0 = jac_add_q(Q0, g2_psi_jac_q(jac_add_aff_q(jac_neg(t1), np)));                      // + psi([x - 1]P)
  return jac_add_q(Q0, g2_psi_jac_q(g2_psi_jac_q(jac_dbl_q(jac_from_aff(p)))));          // + psi^2(2P)
}

// line_add with its products split (lo | hi per step)
__device__ __forceinline__ void line_add_q1(g2_proj<fp2p_t>& T, const aff_t<fp2p_t>& Q, const g1_line_pre& P,
                                            fp2p_t& c0, fp2p_t& c1, fp2p_t& c2) {
  const bool hi = qd_hi();
  auto both = [&](const fp2p_t& mine, fp2p_t& lo_v, fp2p_t& hi_v) {
    const fp2p_t o = qd_swap(mine);
    lo_v = qd_sel(hi, o, mine);
    hi_v = qd_sel(hi, mine, o);
  };
  fp2p_t a, b;
  both(fp2_mul(T.z, qd_sel(hi, Q.x, Q.y)), a, b);                        // yq Z | xq Z
  const fp2p_t u = fp2_sub(a, T.y), v = fp2_sub(b, T.x);
  both(fp2_mul(qd_sel(hi, v, u), qd_sel(hi, Q.y, Q.x)), a, b);           // u xq | v yq
  c0 = fp2_sub(a, b);
  both(fp2_mul_fp(qd_sel(hi, v, u), fp_sel(hi, P.y, P.nx)), c1, c2);     // -u xp | v yp
  fp2p_t vv, uu;
  both(fp2_sqr(qd_sel(hi, u, v)), vv, uu);
  fp2p_t vvv, vvX;
  both(fp2_mul(vv, qd_sel(hi, T.x, v)), vvv, vvX);
  fp2p_t uuZ, vvvZ;
  both(fp2_mul(T.z, qd_sel(hi, vvv, uu)), uuZ, vvvZ);
  const fp2p_t A = fp2_sub2(uuZ, vvv, fp2_dbl(vvX));
  fp2p_t vvvY, vA;
  both(fp2_mul(qd_sel(hi, v, vvv), qd_sel(hi, A, T.y)), vvvY, vA);
  T.y = fp2_sub(fp2_mul(u, fp2_sub(vvX, A)), vvvY);
  T.x = vA;
  T.z = vvvZ;
}

// f * (c0 + c1 v + c2 v w) with the 13 products split 7 | 6 (lo: a = f.c0, hi: b = f.c1):
//   lo: aA (5 products of fp12_mul_by_line_inl), s2 d1, s2 c0
//   hi: bB (3), s0 c0, s1 d1, (s0 + s1)(c0 + d1)     with s = a + b, d1 = c1 + c2
__device__ __forceinline__ fq12_t fq12_mul_by_line_q1(const fq12_t& f, const fp2p_t& c0, const fp2p_t& c1,
                                                      const fp2p_t& c2) {
  const bool hi = qd_hi();
  const fp6p_t& h = f.h;
  fp6p_t s = fp6_add(h, qd_swap(h));
  const fp2p_t d1 = fp2_add(c1, c2);
  const fp2p_t p0 = fp2_mul(qd_sel(hi, h.c2, h.c0), qd_sel(hi, c2, c0));                    // a0c0 | b2c2
  const fp2p_t p1 = fp2_mul(qd_sel(hi, h.c0, h.c1), qd_sel(hi, c2, c1));                    // a1c1 | b0c2
  const fp2p_t p2 = fp2_mul(qd_sel(hi, h.c1, h.c2), qd_sel(hi, c2, c1));                    // a2c1 | b1c2
  const fp2p_t p3 = fp2_mul(qd_sel(hi, s.c0, fp2_add_lazy(h.c0, h.c1)), qd_sel(hi, c0, fp2_add_lazy(c0, c1)));  // (a0+a1)(c0+c1) | s0c0
  const fp2p_t p4 = fp2_mul(qd_sel(hi, s.c1, h.c2), qd_sel(hi, d1, c0));                    // a2c0 | s1d1
  const fp2p_t p5 = fp2_mul(qd_sel(hi, fp2_add_lazy(s.c0, s.c1), s.c2),
                            qd_sel(hi, fp2_add_lazy(c0, d1), d1));                          // s2d1 | (s0+s1)(c0+d1)
  const fp2p_t p6 = fp2_mul(s.c2, c0);                                                      // s2c0 (lo)
  // lo: aA;  hi: bB = (xi b2c2, b0c2, b1c2)
  fp6p_t X;
  X.c0 = qd_sel(hi, fp2_mul_xi(p0), fp2_add_mul_xi(p0, p2));
  X.c1 = qd_sel(hi, p1, fp2_sub2(p3, p0, p1));
  X.c2 = qd_sel(hi, p2, fp2_add(p1, p4));
  const fp6p_t Y = qd_swap(X);                       // lo: bB, hi: aA
  const fp2p_t q5 = qd_swap(p5), q6 = qd_swap(p6);    // hi: s2d1, s2c0 (lo's)
  fq12_t r;
  // lo: aA + v bB
  const fp6p_t lo = fp6_add_mul_by_v(X, Y);
  // hi: m - aA - bB,  m = (s0c0 + xi s2d1, (s0+s1)(c0+d1) - s0c0 - s1d1, s1d1 + s2c0)
  fp6p_t m;
  m.c0 = fp2_add_mul_xi(p3, q5);
  m.c1 = fp2_sub2(p5, p3, p4);
  m.c2 = fp2_add(p4, q6);
  r.h = qd_sel(hi, fp6_sub2(m, Y, X), lo);
  return r;
}

// Miller loop of one pair on a quad; returns conj(f) (x < 0).  degenerate as in miller_loop_n.
__device__ __noinline__ fq12_ml miller_loop_q1_run(const aff_t<fp2p_t> Q, const g1_line_pre P) {
  g2_proj<fp2p_t> T;
  T.x = Q.x; T.y = Q.y; T.z = e2_one<fp2p_t>();
  fq12_t f = fq12_one();
  bool first = true;
  for (int i = 62; i >= 0; --i) {
    fp2p_t c0, c1, c2;
    line_dbl_q1(T, P, c0, c1, c2);
    if (!first) f = fq12_sqr(f);
    f = fq12_mul_by_line_q1(f, c0, c1, c2);
    first = false;
    if ((BLS_X_ABS >> i) & 1) {
      line_add_q1(T, Q, P, c0, c1, c2);
      f = fq12_mul_by_line_q1(f, c0, c1, c2);
    }
  }
  fq12_ml r;
  r.degenerate = fp2_is_zero(T.z);   // T is the same on all four lanes
  r.f = fq12_conj(f);
  return r;
}

__device__ __forceinline__ fq12_t miller_loop_q1(const aff_t<fp2p_t>& Q, const g1_line_pre& P, bool& degenerate) {
  const fq12_ml r = miller_loop_q1_run(Q, P);
  degenerate = r.degenerate;
  return r.f;
}

// ----------------------------------------------- one Miller pair per octet --
// The lowest-latency Miller loop: one pair on 8 lanes, two quads (A = lanes 8t..8t+3, B = 8t+4..8t+7)
// that both hold T and f in the quad layout above.  Each step's independent products run on all
// four lane pairs at once and are exchanged between the quads (lane ^ 4, ds_swizzle):
//   line_dbl  11 products -> 3 steps (quad: 6),  f^2  12 -> 3 (6),  f * line  13 -> 4 (7)
// so a doubling iteration is 10 product steps against 19 on a quad.  The five additions of the loop
// run in the quad form on both quads.  A square paired with a product runs as a product of the value
// with itself, and an Fp x Fp2 product as an Fp2 product with (x, 0): the same field elements (all
// values stay < 2q), so the quads stay bit-identical and T and f need no exchange.
__device__ __forceinline__ bool oc_b() { return (threadIdx.x & 4u) != 0; }
__device__ __forceinline__ fp2p_t oc_swap(const fp2p_t& a) {
  fp2p_t r;
#pragma unroll
  for (int k = 0; k < FP_LIMBS; ++k)   // bitmask mode: and 0x1f, or 0, xor 4
    r.v.w[k] = (uint32_t)__builtin_amdgcn_ds_swizzle((int)a.v.w[k], 0x101F);
  return r;
}
// quad A's and quad B's value of a split step, on both quads
__device__ __forceinline__ void oc_both(const fp2p_t& mine, fp2p_t& a_v, fp2p_t& b_v) {
  const bool b = oc_b();
  const fp2p_t o = oc_swap(mine);
  a_v = qd_sel(b, o, mine);
  b_v = qd_sel(b, mine, o);
}

// ----------------------------------------- G2 doubling on an octet (k_hash_g2_o) --
// The point on both quads; the doubling's independent products on the octet's four lane pairs
// (slot = 2 * quad B + hi): X^2 | Y^2 | Y Z, then B^2 | (X + B)^2 | E^2, then E (D - X3) -- 3 product
// times against jac_dbl_q's 4.  The additions stay in the quad form (both quads compute them).
// The value of each of the first `nv` slots, on every lane of the octet
template <int NV>
__device__ __forceinline__ void oc_slots(const fp2p_t& mine, fp2p_t (&v)[NV]) {
  const bool b = oc_b(), hi = qd_hi();
  const fp2p_t oq = qd_swap(mine), oo = oc_swap(mine), oqo = oc_swap(oq);
#pragma unroll
  for (int t = 0; t < NV; ++t) {
    const bool bb = b != (bool)(t >> 1), hh = hi != (bool)(t & 1);
    v[t] = qd_sel(bb, qd_sel(hh, oqo, oo), qd_sel(hh, oq, mine));
  }
}
__device__ __forceinline__ fp2p_t oc_pick(const fp2p_t& a0, const fp2p_t& a1, const fp2p_t& a2, const fp2p_t& a3) {
  const bool b = oc_b(), hi = qd_hi();
  return qd_sel(b, qd_sel(hi, a3, a2), qd_sel(hi, a1, a0));
}

__device__ __forceinline__ jac_t<fp2p_t> jac_dbl_o(const jac_t<fp2p_t>& p) {
  fp2p_t v[3];
  oc_slots<3>(fp2_mul(oc_pick(p.x, p.y, p.y, p.x), oc_pick(p.x, p.y, p.z, p.x)), v);   // X^2 | Y^2 | Y Z
  const fp2p_t A = v[0], B = v[1], YZ = v[2];
  const fp2p_t E = fp2_mul_small(A, 3);
  const fp2p_t XpB = fp2_add(p.x, B);
  oc_slots<3>(fp2_mul(oc_pick(B, XpB, E, B), oc_pick(B, XpB, E, B)), v);             // B^2 | (X + B)^2 | E^2
  const fp2p_t C = v[0], XB2 = v[1], Fv = v[2];
  const fp2p_t D = fp2_dbl(fp2_sub2(XB2, A, C));
  jac_t<fp2p_t> r;
  r.x = fp2_sub2(Fv, D, D);
  r.y = fp2_sub(fp2_mul(E, fp2_sub(D, r.x)), fp2_mul_small(C, 8));
  r.z = fp2_dbl(YZ);
  return r;   // Z = 0 stays 0
}

__device__ __noinline__ jac_t<fp2p_t> jac_mul_u64_o(const aff_t<fp2p_t> a, uint64_t k) {
  jac_t<fp2p_t> r = jac_from_aff(a);
  int top = 63;
  while (top > 0 && !((k >> top) & 1)) --top;
  for (int i = top - 1; i >= 0; --i) {
    r = jac_dbl_o(r);
    if ((k >> i) & 1) r = jac_add_aff_q(r, a);
  }
  return r;
}
__device__ __noinline__ jac_t<fp2p_t> jac_mul_u64_jac_o(const jac_t<fp2p_t> p, uint64_t k) {
  jac_t<fp2p_t> r = p;
  int top = 63;
  while (top > 0 && !((k >> top) & 1)) --top;
  for (int i = top - 1; i >= 0; --i) {
    r = jac_dbl_o(r);
    if ((k >> i) & 1) r = jac_add_q(r, p);
  }
  return r;
}

// g2_mul_bp_q with the ladders' doublings on the octet
__device__ __noinline__ jac_t<fp2p_t> g2_mul_bp_o(const aff_t<fp2p_t> p) {
  aff_t<fp2p_t> np;
  np.x = p.x;
  np.y = fp2_neg(p.y);
  const jac_t<fp2p_t> t1 = jac_mul_u64_o(p, BLS_X_ABS);                                   // [|x|]P
  jac_t<fp2p_t> Q0 = jac_add_aff_q(jac_add_q(jac_mul_u64_jac_o(t1, BLS_X_ABS), t1), np);  // [x^2 - x - 1]P
  Q0 = jac_add_q(Q0, g2_psi_jac_q(jac_add_aff_q(jac_neg(t1), np)));                      // + psi([x - 1]P)
  return jac_add_q(Q0, g2_psi_jac_q(g2_psi_jac_q(jac_dbl_o(jac_from_aff(p)))));          // + psi^2(2P)
}

// fp6_mul_inl with its six Karatsuba products split A | B (the same formula, bit-identical)
__device__ __forceinline__ fp6p_t fp6_mul_oct(const fp6p_t& s, const fp6p_t& t) {
  const bool b = oc_b();
  fp2p_t t0, t1, t2, t3, t4, t5;
  oc_both(fp2_mul(qd_sel(b, fp2_add_lazy(s.c1, s.c2), s.c0), qd_sel(b, fp2_add_lazy(t.c1, t.c2), t.c0)), t0, t3);
  oc_both(fp2_mul(qd_sel(b, fp2_add_lazy(s.c0, s.c1), s.c1), qd_sel(b, fp2_add_lazy(t.c0, t.c1), t.c1)), t1, t4);
  oc_both(fp2_mul(qd_sel(b, fp2_add_lazy(s.c0, s.c2), s.c2), qd_sel(b, fp2_add_lazy(t.c0, t.c2), t.c2)), t2, t5);
  fp6p_t r;
  r.c0 = fp2_add_mul_xi(t0, fp2_sub2(t3, t1, t2));
  r.c1 = fp2_add_mul_xi(fp2_sub2(t4, t0, t1), t2);
  r.c2 = fp2_add(fp2_sub2(t5, t0, t2), t1);
  return r;
}

__device__ __forceinline__ fq12_t fq12_sqr_oct(const fq12_t& f) {
  const bool hi = qd_hi();
  const fp6p_t y = qd_swap(f.h);
  const fp6p_t u = qd_sel(hi, fp6_add(f.h, y), f.h);
  const fp6p_t v = qd_sel(hi, fp6_add_mul_by_v(y, f.h), y);
  const fp6p_t p = fp6_mul_oct(u, v);                 // lo: ab, hi: (a+b)(a+vb)
  const fp6p_t o = qd_swap(p);
  fq12_t r;
  r.h = qd_sel(hi, fp6_dbl(o), fp6_sub2(o, p, fp6_mul_by_v(p)));
  return r;
}

// fq12_mul_by_line_q1 with its seven product calls split A: p0..p3 | B: p4..p6 (p3 on both)
__device__ __forceinline__ fq12_t fq12_mul_by_line_oct(const fq12_t& f, const fp2p_t& c0, const fp2p_t& c1,
                                                       const fp2p_t& c2) {
  const bool hi = qd_hi(), b = oc_b();
  const fp6p_t& h = f.h;
  fp6p_t s = fp6_add(h, qd_swap(h));
  const fp2p_t d1 = fp2_add(c1, c2);
  fp2p_t p0, p1, p2, p3, p4, p5, p6;
  oc_both(fp2_mul(qd_sel(b, qd_sel(hi, s.c1, h.c2), qd_sel(hi, h.c2, h.c0)),
                  qd_sel(b, qd_sel(hi, d1, c0), qd_sel(hi, c2, c0))), p0, p4);            // a0c0 | b2c2 ; a2c0 | s1d1
  oc_both(fp2_mul(qd_sel(b, qd_sel(hi, fp2_add_lazy(s.c0, s.c1), s.c2), qd_sel(hi, h.c0, h.c1)),
                  qd_sel(b, qd_sel(hi, fp2_add_lazy(c0, d1), d1), qd_sel(hi, c2, c1))), p1, p5);   // a1c1 | b0c2 ; ...
  oc_both(fp2_mul(qd_sel(b, s.c2, qd_sel(hi, h.c1, h.c2)), qd_sel(b, c0, qd_sel(hi, c2, c1))), p2, p6);
  p3 = fp2_mul(qd_sel(hi, s.c0, fp2_add_lazy(h.c0, h.c1)), qd_sel(hi, c0, fp2_add_lazy(c0, c1)));
  fp6p_t X;
  X.c0 = qd_sel(hi, fp2_mul_xi(p0), fp2_add_mul_xi(p0, p2));
  X.c1 = qd_sel(hi, p1, fp2_sub2(p3, p0, p1));
  X.c2 = qd_sel(hi, p2, fp2_add(p1, p4));
  const fp6p_t Y = qd_swap(X);                       // lo: bB, hi: aA
  const fp2p_t q5 = qd_swap(p5), q6 = qd_swap(p6);
  fq12_t r;
  const fp6p_t lo = fp6_add_mul_by_v(X, Y);
  fp6p_t m;
  m.c0 = fp2_add_mul_xi(p3, q5);
  m.c1 = fp2_sub2(p5, p3, p4);
  m.c2 = fp2_add(p4, q6);
  r.h = qd_sel(hi, fp6_sub2(m, Y, X), lo);
  return r;
}

// line_dbl_q1 in three steps: A (X^2 | Y^2) with B (Z^2 | YZ); A (h^2 | b3^2) with B (XY | XY);
// A (XY(YY - 9b'Z^2) | YY YZ) with B (XX(-3xp) | YZ(2yp))
__device__ __forceinline__ void line_dbl_oct(g2_proj<fp2p_t>& T, const g1_line_pre& P, fp2p_t& c0, fp2p_t& c1,
                                             fp2p_t& c2) {
  const bool hi = qd_hi(), b = oc_b();
  fp2p_t s1, m1;
  {
    const fp2p_t xa = qd_sel(hi, T.y, T.x);
    oc_both(fp2_mul(qd_sel(b, T.z, xa), qd_sel(b, qd_sel(hi, T.y, T.z), xa)), s1, m1);
  }
  const fp2p_t s1o = qd_swap(s1), m1o = qd_swap(m1);
  const fp2p_t XX = qd_sel(hi, s1o, s1), YY = qd_sel(hi, s1, s1o);
  const fp2p_t ZZ = qd_sel(hi, m1o, m1), YZ = qd_sel(hi, m1, m1o);
  const fp2p_t b3 = fp2_mul_small(fp2_mul_small(fp2_mul_xi(ZZ), 3), 4);   // 3 b' Z^2
  const fp2p_t b9 = fp2_mul_small(b3, 3);
  c0 = fp2_sub(YY, b3);
  const fp2p_t h = fp2_half(fp2_add(YY, b9));
  fp2p_t s2, XY;
  {
    const fp2p_t xs = qd_sel(hi, b3, h);   // lo h^2 | hi (3b'Z^2)^2, as line_dbl_q1
    oc_both(fp2_mul(qd_sel(b, T.x, xs), qd_sel(b, T.y, xs)), s2, XY);
  }
  fp2p_t m2, e;
  {
    const fp2p_t pe = pr_make(fp_sel(pr_odd(), fp_zero(), fp_sel(hi, P.y2, P.n3x)));   // (y2 | n3x, 0)
    oc_both(fp2_mul(qd_sel(b, qd_sel(hi, YZ, XX), qd_sel(hi, YY, XY)),
                    qd_sel(b, pe, qd_sel(hi, YZ, fp2_sub(YY, b9)))), m2, e);
  }
  const fp2p_t eo = qd_swap(e), m2o = qd_swap(m2), s2o = qd_swap(s2);
  c1 = qd_sel(hi, eo, e);
  c2 = qd_sel(hi, e, eo);
  T.x = fp2_half(qd_sel(hi, m2o, m2));
  T.y = fp2_sub(qd_sel(hi, s2o, s2), fp2_mul_small(qd_sel(hi, s2, s2o), 3));
  T.z = fp2_dbl(qd_sel(hi, m2, m2o));
}

// Miller loop of one pair on an octet; returns conj(f) (x < 0) in the quad form on both quads.
__device__ __noinline__ fq12_ml miller_loop_o1_run(const aff_t<fp2p_t> Q, const g1_line_pre P) {
  g2_proj<fp2p_t> T;
  T.x = Q.x; T.y = Q.y; T.z = e2_one<fp2p_t>();
  fq12_t f = fq12_one();
  bool first = true;
  for (int i = 62; i >= 0; --i) {
    fp2p_t c0, c1, c2;
    line_dbl_oct(T, P, c0, c1, c2);
    if (!first) f = fq12_sqr_oct(f);
    f = fq12_mul_by_line_oct(f, c0, c1, c2);
    first = false;
    if ((BLS_X_ABS >> i) & 1) {
      line_add_q1(T, Q, P, c0, c1, c2);
      f = fq12_mul_by_line_oct(f, c0, c1, c2);
    }
  }
  fq12_ml r;
  r.degenerate = fp2_is_zero(T.z);   // T is the same on all eight lanes
  r.f = fq12_conj(f);
  return r;
}

// ------------------------------------------- final exponentiation on quads --
// The latency form of final_exp (bls381_pairing.hpp): the same chain, with every
// Fp12 step split over the two halves, for batches too small to fill the GPU
// (single calls, verify_multiple batches, randomized sub-batches).

// f^(q^p): lo holds the coefficients of w^0, w^2, w^4, hi those of w^1, w^3, w^5
__device__ __forceinline__ fq12_t fq12_frob(const fq12_t& f, int p) {
  const fp2_t* g = FROB_GAMMA_M[p - 1];
  const bool hi = qd_hi();
  const bool odd = (p & 1) != 0;
  auto fr = [&](const fp2p_t& c, int j) -> fp2p_t {
    const fp2p_t cc = odd ? fp2_conj(c) : c;
    return fp2_mul(cc, qd_sel(hi, e2_k<fp2p_t>(g[2 * j + 1]), e2_k<fp2p_t>(g[2 * j])));
  };
  fq12_t r;
  r.h.c0 = fr(f.h.c0, 0);
  r.h.c1 = fr(f.h.c1, 1);
  r.h.c2 = fr(f.h.c2, 2);
  return r;
}

// 1/(a + b w) = (a - b w) / (a^2 - v b^2): lo squares a, hi b; the Fp6 inverse
// runs on both halves
__device__ __forceinline__ fq12_t fq12_inv(const fq12_t& f) {
  const bool hi = qd_hi();
  const fp6p_t p = fp6_mul_inl(f.h, f.h);
  const fp6p_t o = qd_swap(p);
  const fp6p_t t = fp6_sub(qd_sel(hi, o, p), fp6_mul_by_v(qd_sel(hi, p, o)));
  const fp6p_t r = fp6_mul_inl(f.h, fp6_inv(t));
  fq12_t out;
  out.h = qd_sel(hi, fp6_neg(r), r);
  return out;
}

__device__ __forceinline__ bool fq12_is_one(const fq12_t& f) {
  const bool hi = qd_hi();
  const bool a = fp2_eq(f.h.c0, qd_sel(hi, e2_zero<fp2p_t>(), e2_one<fp2p_t>()));
  const bool b = fp2_is_zero(f.h.c1);
  const bool c = fp2_is_zero(f.h.c2);
  return qd_all(a & b & c);
}

// Karabina compressed squaring (cyc_csqr) on a quad.  lo holds (x, y) = (g4, g5)
// and squares them (t0, t1, t2 of cyc_csqr), hi holds (g2, g3) (t3, t4, t5); each
// half's outputs update the other half's pair, so one exchange per squaring:
// three Fp2 squarings per lane instead of six.
struct cq_t { fp2p_t x, y; };

__device__ __forceinline__ cq_t cq_compress(const fq12_t& f) {
  // g2 = b0 (hi c0), g3 = a2 (lo c2), g4 = a1 (lo c1), g5 = b2 (hi c2)
  cq_t g;
  g.x = qd_sel(qd_hi(), f.h.c0, f.h.c1);
  g.y = qd_swap(f.h.c2);
  return g;
}

__device__ __forceinline__ cq_t cq_sqr(const cq_t& g) {
  const bool hi = qd_hi();
#if BLS_LAZY_CSQR
  // lazy reduction (bls381_lazy.hpp): each half forms its two outputs from its own (x, y)
  // as wide sums -- S = x^2 + xi y^2 and lo: xi x y, hi: x y -- one reduction each
  const bool p = pr_odd();
  const fp_t ex = pr_dpp<DPP_EVEN>(g.x.v), ox = pr_dpp<DPP_ODD>(g.x.v);
  const fp_t ey = pr_dpp<DPP_EVEN>(g.y.v), oy = pr_dpp<DPP_ODD>(g.y.v);
  const fp_t S = lz_sqr_xisqr(p, ex, ox, ey, oy);
  fp_t P;
  {
    lv_t x1, y1, x2, y2;
#pragma unroll
    for (int k = 0; k < 14; ++k) {
      const int32_t b0 = (int32_t)ey.w[k], b1 = (int32_t)oy.w[k];
      const int32_t s = b0 + b1, d = b0 - b1;
      x1[k] = (int32_t)ex.w[k];
      x2[k] = (int32_t)ox.w[k];
      y1[k] = hi ? (p ? b1 : b0) : (p ? s : d);     // hi: Re/Im(x y), lo: Re/Im(xi x y)
      y2[k] = hi ? (p ? b0 : -b1) : (p ? d : -s);
    }
    wide_t T;
    wz_init(T);
    wmac(T, x1, y1);
    wmac(T, x2, y2);
    P = wredc(T);
  }
  // lo <- hi's (S, x y): g4' = 3 S - 2 g4, g5' = 6 x y + 2 g5;
  // hi <- lo's (xi x y, S): g2' = 6 xi x y + 2 g2, g3' = 3 S - 2 g3
  const fp_t So = pr_dpp<DPP_HSWAP>(S), Po = pr_dpp<DPP_HSWAP>(P);
  cq_t r;
  r.x = pr_make(fp_6p2_3m2(hi, Po, So, g.x.v));
  r.y = pr_make(fp_6p2_3m2(!hi, Po, So, g.y.v));
  return r;
#else
  const fp2p_t s0 = fp2_sqr(g.x), s1 = fp2_sqr(g.y), s2 = fp2_sqr(fp2_add(g.x, g.y));
  const fp2p_t D = fp2_sub2(s2, s0, s1);       // 2 x y
  const fp2p_t S = fp2_add_mul_xi(s0, s1);     // x^2 + xi y^2
  const fp2p_t U = qd_swap(qd_sel(hi, S, fp2_mul_xi(D)));   // lo <- S(hi), hi <- xi D(lo)
  const fp2p_t V = qd_swap(qd_sel(hi, D, S));               // lo <- D(hi), hi <- S(lo)
  cq_t r;
  r.x = fp2_3pm2(U, g.x, !hi);   // lo: g4' = 3 (g2^2 + xi g3^2) - 2 g4;  hi: g2' = 6 xi g4 g5 + 2 g2
  r.y = fp2_3pm2(V, g.y, hi);    // lo: g5' = 6 g2 g3 + 2 g5;             hi: g3' = 3 (g4^2 + xi g5^2) - 2 g3
  return r;
#endif
}

// g2 of a compressed value, on all four lanes
__device__ __forceinline__ fp2p_t cq_g2(const cq_t& g) { return qd_sel(qd_hi(), g.x, qd_swap(g.x)); }

// cyc_decompress on a quad; inv = 1 / (4 g2) on all lanes
__device__ __forceinline__ fq12_t cq_decompress(const cq_t& g, const fp2p_t& inv) {
  const bool hi = qd_hi();
  const fp2p_t xo = qd_swap(g.x), yo = qd_swap(g.y);
  const fp2p_t G2 = qd_sel(hi, g.x, xo), G3 = qd_sel(hi, g.y, yo);
  const fp2p_t G4 = qd_sel(hi, xo, g.x), G5 = qd_sel(hi, yo, g.y);
  const fp2p_t sq = fp2_sqr(qd_sel(hi, G5, G4));             // lo: g4^2, hi: g5^2
  const fp2p_t sqo = qd_swap(sq);
  const fp2p_t num = fp2_sub2(fp2_add_mul_xi(fp2_mul_small(qd_sel(hi, sqo, sq), 3), qd_sel(hi, sq, sqo)), G3, G3);
  const fp2p_t p1 = fp2_mul(qd_sel(hi, G3, num), qd_sel(hi, G4, inv));   // lo: b1, hi: g3 g4
  const fp2p_t p2 = fp2_mul(qd_sel(hi, G2, p1), qd_sel(hi, G5, p1));     // lo: b1^2, hi: g2 g5
  const fp2p_t p1o = qd_swap(p1), p2o = qd_swap(p2);
  const fp2p_t u = fp2_sub(fp2_add(fp2_dbl(p2), p2o), fp2_mul_small(p1o, 3));   // lo: 2 b1^2 + g2 g5 - 3 g3 g4
  fq12_t f;
  f.h.c0 = qd_sel(hi, G2, fp2_add(fp2_mul_xi(u), e2_one<fp2p_t>()));   // b0 | a0
  f.h.c1 = qd_sel(hi, p1o, G4);                                        // b1 | a1
  f.h.c2 = qd_sel(hi, G5, G3);                                         // b2 | a2
  return f;
}

// exact fallback (cyc_exp_x_gs): generic squarings, valid for every element
__device__ __noinline__ fq12_t cyc_exp_x_gs_q(const fq12_t f) {
  fq12_t r = f;
  for (int s = 0; s < 6; ++s) {
    for (int j = CYC_X_RUNS[s]; j > 0; --j) r = fq12_sqr(r);
    if (s < 5) r = fq12_mul(r, f);
  }
  return fq12_conj(r);
}

// f^x (cyc_exp_x): compressed squarings, six snapshots, one shared inversion
__device__ __noinline__ fq12_t cyc_exp_x_q(const fq12_t f) {
  const bool hi = qd_hi();
  cq_t snap[6];
  cq_t g = cq_compress(f);
  bool zero = false;
  for (int s = 0; s < 6; ++s) {
    for (int j = CYC_X_RUNS_RTL[s]; j > 0; --j) g = cq_sqr(g);
    snap[s] = g;
    zero = zero | fp2_is_zero(cq_g2(g));
  }
  if (BLS_ANY(zero)) return cyc_exp_x_gs_q(f);
  fp2p_t pre[6];
  pre[0] = fp2_mul_small(cq_g2(snap[0]), 4);
  for (int s = 1; s < 6; ++s) pre[s] = fp2_mul(pre[s - 1], fp2_mul_small(cq_g2(snap[s]), 4));
  fp2p_t inv = fp2_inv(pre[5]);
  fq12_t r;
  for (int s = 5; s >= 0; --s) {
    fp2p_t is = inv;
    if (s) {
      // lo: inv * pre[s-1] (this snapshot's 1/(4 g2)), hi: inv * 4 g2 (the next inv)
      const fp2p_t p = fp2_mul(inv, qd_sel(hi, fp2_mul_small(cq_g2(snap[s]), 4), pre[s - 1]));
      const fp2p_t po = qd_swap(p);
      is = qd_sel(hi, po, p);
      inv = qd_sel(hi, p, po);
    }
    const fq12_t x = cq_decompress(snap[s], is);
    r = (s == 5) ? x : fq12_mul(r, x);
  }
  return fq12_conj(r);
}

// f^(3 (q^12 - 1)/r), the chain of final_exp
__device__ inline fq12_t final_exp_q(const fq12_t f) {
  fq12_t t = fq12_mul(fq12_conj(f), fq12_inv(f));          // f^(q^6 - 1)
  t = fq12_mul(fq12_frob(t, 2), t);                        // ^(q^2 + 1)
  fq12_t a = fq12_mul(cyc_exp_x_q(t), fq12_conj(t));       // t^(x-1)
  a = fq12_mul(cyc_exp_x_q(a), fq12_conj(a));              // t^((x-1)^2)
  const fq12_t b = fq12_mul(cyc_exp_x_q(a), fq12_frob(a, 1));          // a^(x+q)
  const fq12_t bx2 = cyc_exp_x_q(cyc_exp_x_q(b));
  const fq12_t c = fq12_mul(fq12_mul(bx2, fq12_frob(b, 2)), fq12_conj(b));   // b^(x^2+q^2-1)
  const fq12_t t3 = fq12_mul(fq12_sqr(t), t);
  return fq12_mul(c, t3);
}


// ---- the final exponentiation on an octet, products split (k_final_exp_verdict_oq) ----
// The compressed squarings stay in the quad form on both quads (BLS381_FE_OCT=2; the default
// splits them four ways as well, cyc_exp_x_oo below); every Fp12 product runs its Fp6
// products over the four lane pairs: fq12_mul 9 product steps -> 5.
// fp6_mul_split with its three products per half split A: 0, 2 | B: 1, 2 (the same values)
__device__ __forceinline__ fp6p_t fp6_mul_split_oct(const fp6p_t& s, const fp6p_t& t) {
  const bool hi = qd_hi(), b = oc_b();
  const fp2p_t x0 = qd_sel(hi, fp2_add_lazy(s.c1, s.c2), s.c0), y0 = qd_sel(hi, fp2_add_lazy(t.c1, t.c2), t.c0);
  const fp2p_t x1 = qd_sel(hi, fp2_add_lazy(s.c0, s.c1), s.c1), y1 = qd_sel(hi, fp2_add_lazy(t.c0, t.c1), t.c1);
  const fp2p_t x2 = qd_sel(hi, fp2_add_lazy(s.c0, s.c2), s.c2), y2 = qd_sel(hi, fp2_add_lazy(t.c0, t.c2), t.c2);
  fp2p_t p[3];
  oc_both(fp2_mul(qd_sel(b, x1, x0), qd_sel(b, y1, y0)), p[0], p[1]);
  p[2] = fp2_mul(x2, y2);
  fp2p_t o[3];
  for (int k = 0; k < 3; ++k) o[k] = qd_swap(p[k]);
  const fp2p_t t0 = qd_sel(hi, o[0], p[0]), t1 = qd_sel(hi, o[1], p[1]), t2 = qd_sel(hi, o[2], p[2]);
  const fp2p_t t3 = qd_sel(hi, p[0], o[0]), t4 = qd_sel(hi, p[1], o[1]), t5 = qd_sel(hi, p[2], o[2]);
  fp6p_t r;
  r.c0 = fp2_add_mul_xi(t0, fp2_sub2(t3, t1, t2));
  r.c1 = fp2_add_mul_xi(fp2_sub2(t4, t0, t1), t2);
  r.c2 = fp2_add(fp2_sub2(t5, t0, t2), t1);
  return r;
}

__device__ __forceinline__ fq12_t fq12_mul_oct(const fq12_t& f, const fq12_t& g) {
  const bool hi = qd_hi();
  const fp6p_t yf = qd_swap(f.h), yg = qd_swap(g.h);
  const fp6p_t p = fp6_mul_oct(f.h, g.h);            // lo: ac, hi: bd
  const fp6p_t m = fp6_mul_split_oct(fp6_add(f.h, yf), fp6_add(g.h, yg));
  const fp6p_t o = qd_swap(p);
  fq12_t r;
  r.h = qd_sel(hi, fp6_sub2(m, o, p), fp6_add_mul_by_v(p, o));
  return r;
}

__device__ __noinline__ fq12_t cyc_exp_x_gs_oq(const fq12_t f) {
  fq12_t r = f;
  for (int s = 0; s < 6; ++s) {
    for (int j = CYC_X_RUNS[s]; j > 0; --j) r = fq12_sqr_oct(r);
    if (s < 5) r = fq12_mul_oct(r, f);
  }
  return fq12_conj(r);
}

__device__ __noinline__ fq12_t cyc_exp_x_oq(const fq12_t f) {
  const bool hi = qd_hi();
  cq_t snap[6];
  cq_t g = cq_compress(f);
  bool zero = false;
  for (int s = 0; s < 6; ++s) {
    for (int j = CYC_X_RUNS_RTL[s]; j > 0; --j) g = cq_sqr(g);
    snap[s] = g;
    zero = zero | fp2_is_zero(cq_g2(g));
  }
  if (BLS_ANY(zero)) return cyc_exp_x_gs_oq(f);
  fp2p_t pre[6];
  pre[0] = fp2_mul_small(cq_g2(snap[0]), 4);
  for (int s = 1; s < 6; ++s) pre[s] = fp2_mul(pre[s - 1], fp2_mul_small(cq_g2(snap[s]), 4));
  fp2p_t inv = fp2_inv(pre[5]);
  fq12_t r;
  for (int s = 5; s >= 0; --s) {
    fp2p_t is = inv;
    if (s) {
      const fp2p_t p = fp2_mul(inv, qd_sel(hi, fp2_mul_small(cq_g2(snap[s]), 4), pre[s - 1]));
      const fp2p_t po = qd_swap(p);
      is = qd_sel(hi, po, p);
      inv = qd_sel(hi, p, po);
    }
    const fq12_t x = cq_decompress(snap[s], is);
    r = (s == 5) ? x : fq12_mul_oct(r, x);
  }
  return fq12_conj(r);
}

__device__ inline fq12_t final_exp_oq(const fq12_t f) {
  fq12_t t = fq12_mul_oct(fq12_conj(f), fq12_inv(f));
  t = fq12_mul_oct(fq12_frob(t, 2), t);
  fq12_t a = fq12_mul_oct(cyc_exp_x_oq(t), fq12_conj(t));
  a = fq12_mul_oct(cyc_exp_x_oq(a), fq12_conj(a));
  const fq12_t b = fq12_mul_oct(cyc_exp_x_oq(a), fq12_frob(a, 1));
  const fq12_t bx2 = cyc_exp_x_oq(cyc_exp_x_oq(b));
  const fq12_t c = fq12_mul_oct(fq12_mul_oct(bx2, fq12_frob(b, 2)), fq12_conj(b));
  const fq12_t t3 = fq12_mul_oct(fq12_sqr_oct(t), t);
  return fq12_mul_oct(c, t3);
}

// ------------------------------------- compressed squarings on a lane octet --
// The lowest-latency form of cyc_exp_x for single calls: an item's FE runs on 8 lanes,
// two quads holding the same fq12_t (every Fp12 step is computed on both, identically),
// and only the 63 Karabina squarings per x-power -- most of the FE -- are split four ways:
// each lane pair of the octet holds one of (g4, g2, g5, g3) (pairs 0..3) and computes that
// coefficient's update as ONE lazily reduced sum of three products,
//   pair 0  g4' = 3 (g2^2 + xi g3^2) - 2 g4     pair 1  g2' = 6 xi g4 g5 + 2 g2
//   pair 2  g5' = 6 g2 g3 + 2 g5                pair 3  g3' = 3 (g4^2 + xi g5^2) - 2 g3
// (the product outputs leave their third product zero, so every lane runs the same
// instruction stream): 3 half-products and 1 reduction per lane per squaring, against 5
// and 2 on a quad.  The two operands come from the same quad's other pair (DPP quad_perm)
// and the other quad (DPP row_shl/row_shr by 4).
__device__ __forceinline__ bool od_upper() { return (threadIdx.x & 4u) != 0; }
// the same lane of the other quad of the octet
__device__ __forceinline__ fp_t od_cross(const fp_t& a) {
  return fp_sel(od_upper(), pr_dpp<0x114>(a), pr_dpp<0x104>(a));   // row_shr:4 | row_shl:4
}
// quad compressed value (both quads equal) -> this pair's coefficient: lower quad x, upper y
__device__ __forceinline__ fp2p_t co_enter(const cq_t& g) { return qd_sel(od_upper(), g.y, g.x); }
__device__ __forceinline__ cq_t co_exit(const fp2p_t& s) {
  const bool up = od_upper();
  const fp2p_t o = pr_make(od_cross(s.v));
  cq_t g;
  g.x = qd_sel(up, o, s);
  g.y = qd_sel(up, s, o);
  return g;
}

__device__ __forceinline__ fp2p_t co_sqr(const fp2p_t& g) {
  const bool up = od_upper(), p = pr_odd();
  const uint32_t pair = (threadIdx.x >> 1) & 3u;
  // the pair's role as opaque lane masks: on the plain comparisons the compiler rebuilt the operand
  // selects below as a branch tree over `pair` (268 exec-mask branches per squaring; r05
  // tools/csqr_lat.hip, one item: 15.0k -> 11.9k cycles per squaring with the masks; the operand prep
  // below as word blends instead of selects: 7.2k, against 10.1k for the quad form -> BLS381_FE_OCT=3)
  uint32_t sqm = ((pair ^ (pair >> 1)) & 1u) - 1u;            // pairs 0, 3: all ones
  uint32_t xpm = 0u - ((((pair ^ 1u) - 1u) >> 31) & 1u);      // pair 1: all ones
  asm volatile("" : "+v"(sqm), "+v"(xpm));
  const bool sq = sqm != 0, xp = xpm != 0;
  const fp_t a = pr_dpp<DPP_HSWAP>(g.v);
  const fp_t b = pr_dpp<DPP_HSWAP>(od_cross(g.v));
  const fp_t X = fp_sel(up, b, a), Y = fp_sel(up, a, b);     // (g2, g3) or (g4, g5)
  const fp_t X0 = pr_dpp<DPP_EVEN>(X), X1 = pr_dpp<DPP_ODD>(X);
  const fp_t Y0 = pr_dpp<DPP_EVEN>(Y), Y1 = pr_dpp<DPP_ODD>(Y);
  lv_t u;
  {
    uint32_t us[14];
#pragma unroll
    for (int k = 0; k < 14; ++k) us[k] = Y0.w[k] + (p ? Y1.w[k] : Q2B_LIMBS[k] - Y1.w[k]);
    lv_from(u, fp_reduce_lc<2>(us));   // Y0 -+ Y1 reduced (the square's operand)
  }
  lv_t a1, b1, a2, b2, a3, b3;
  const uint32_t pm = 0u - (uint32_t)p;
#pragma unroll
  for (int k = 0; k < 14; ++k) {
    const uint32_t x0 = X0.w[k], x1 = X1.w[k], y0 = Y0.w[k], y1 = Y1.w[k];
    const uint32_t ys = y0 + y1, yd = y0 - y1;
    // SQ:    Re (x0+x1)(x0-x1) + u^2 - 2 y1^2,  Im 2 x0 x1 + u^2 - 2 y1^2   (lz_sqr_xisqr)
    // XPROD: Re x0 (y0-y1) - x1 (y0+y1),        Im x0 (y0+y1) + x1 (y0-y1) (lz_xi_mul)
    // PROD:  Re x0 y0 - x1 y1,                  Im x0 y1 + x1 y0           (lz_mul)
    // (two's-complement words blended with the lane masks: no per-lane branches)
    auto blend = [](uint32_t m, uint32_t a, uint32_t b) { return b ^ (m & (a ^ b)); };   // m ? a : b
    const uint32_t t_sq = blend(pm, x1, x0 - x1), t_xp = blend(pm, ys, yd), t_pr = blend(pm, y1, y0);
    const uint32_t u_xp = blend(pm, yd, 0u - ys), u_pr = blend(pm, y0, 0u - y1);
    a1[k] = (int32_t)(x0 + (sqm & blend(pm, x0, x1)));
    b1[k] = (int32_t)blend(sqm, t_sq, blend(xpm, t_xp, t_pr));
    a2[k] = (int32_t)blend(sqm, (uint32_t)u[k], x1);
    b2[k] = (int32_t)blend(sqm, (uint32_t)u[k], blend(xpm, u_xp, u_pr));
    a3[k] = (int32_t)(sqm & (0u - 2u * y1));
    b3[k] = (int32_t)(sqm & y1);
  }
  // columns: 3 x 14 products < 2^57 (< 2^62.4) plus the reduction's < 2^59.8; values in
  // (-16 q^2, 12 q^2) as for lz_sqr_xisqr (the product outputs: |X| < 16 q^2)
  wide_t T;
  wz_init(T);
  wmac(T, a1, b1);
  wmac(T, a2, b2);
  wmac(T, a3, b3);
  const fp_t R = wredc(T);
  return pr_make(fp_6p2_3m2(!sq, R, R, g.v));
}

// cyc_exp_x_oq with the squarings on the octet as well (co_sqr) -- the single-call FE (BLS381_FE_OCT=3)
__device__ __noinline__ fq12_t cyc_exp_x_oo(const fq12_t f) {
  const bool hi = qd_hi();
  cq_t snap[6];
  fp2p_t g = co_enter(cq_compress(f));
  bool zero = false;
  for (int s = 0; s < 6; ++s) {
    for (int j = CYC_X_RUNS_RTL[s]; j > 0; --j) g = co_sqr(g);
    snap[s] = co_exit(g);
    zero = zero | fp2_is_zero(cq_g2(snap[s]));
  }
  if (BLS_ANY(zero)) return cyc_exp_x_gs_oq(f);
  fp2p_t pre[6];
  pre[0] = fp2_mul_small(cq_g2(snap[0]), 4);
  for (int s = 1; s < 6; ++s) pre[s] = fp2_mul(pre[s - 1], fp2_mul_small(cq_g2(snap[s]), 4));
  fp2p_t inv = fp2_inv(pre[5]);
  fq12_t r;
  for (int s = 5; s >= 0; --s) {
    fp2p_t is = inv;
    if (s) {
      const fp2p_t p = fp2_mul(inv, qd_sel(hi, fp2_mul_small(cq_g2(snap[s]), 4), pre[s - 1]));
      const fp2p_t po = qd_swap(p);
      is = qd_sel(hi, po, p);
      inv = qd_sel(hi, p, po);
    }
    const fq12_t x = cq_decompress(snap[s], is);
    r = (s == 5) ? x : fq12_mul_oct(r, x);
  }
  return fq12_conj(r);
}

__device__ inline fq12_t final_exp_oo(const fq12_t f) {
  fq12_t t = fq12_mul_oct(fq12_conj(f), fq12_inv(f));
  t = fq12_mul_oct(fq12_frob(t, 2), t);
  fq12_t a = fq12_mul_oct(cyc_exp_x_oo(t), fq12_conj(t));
  a = fq12_mul_oct(cyc_exp_x_oo(a), fq12_conj(a));
  const fq12_t b = fq12_mul_oct(cyc_exp_x_oo(a), fq12_frob(a, 1));
  const fq12_t bx2 = cyc_exp_x_oo(cyc_exp_x_oo(b));
  const fq12_t c = fq12_mul_oct(fq12_mul_oct(bx2, fq12_frob(b, 2)), fq12_conj(b));
  const fq12_t t3 = fq12_mul_oct(fq12_sqr_oct(t), t);
  return fq12_mul_oct(c, t3);
}

}  // namespace bls381
