// Optimal-ate Miller loop on the M-type sextic twist and the final
// exponentiation.  Formulas are mirrored by oracle/tower_model.py
// (line_dbl / line_add / miller_loop_multi / final_exp) and tested there
// against the reference restatement (oracle/bls_oracle.py).
//
// Lines are evaluated at P = (xp, yp) in E(Fp) and scaled by Fp2 factors,
// which the final exponentiation kills:  l = c0 + c1 v + c2 v w  with
//   tangent at T = (X:Y:Z):  c0 = Y^2 - 3b'Z^2, c1 = -3 X^2 xp, c2 = 2 Y Z yp
//   chord T,Q (Q affine):   c0 = u xq - v yq, c1 = -u xp, c2 = v yp,
//                           u = yq Z - Y, v = xq Z - X.
#pragma once
#include "bls381_curve.hpp"

namespace bls381 {

// Per-G1-point line-evaluation constants
struct g1_line_pre {
  fp_t n3x;   // -3 xp
  fp_t y2;    // 2 yp
  fp_t nx;    // -xp
  fp_t y;     // yp
};

BLS_INLINE g1_line_pre g1_prepare(const aff_t<fp_t>& p) {
  g1_line_pre r;
  r.nx = fp_neg(p.x);
  r.n3x = fp_add(fp_dbl(r.nx), r.nx);
  r.y = p.y;
  r.y2 = fp_dbl(p.y);
  return r;
}

// homogeneous-projective T on E'(Fp2)
template <class E> struct g2_proj { E x, y, z; };

template <class E>
BLS_INLINE E fp2_mul_b(const E& a) {
  // b' = 4(1+u): a * b' = 4 * xi * a
  const E t = fp2_mul_xi(a);
  return fp2_dbl(fp2_dbl(t));
}

// doubling step: T <- 2T, returns the tangent line at the old T evaluated at P
template <class E>
BLS_HD inline void line_dbl(g2_proj<E>& T, const g1_line_pre& P, E& c0, E& c1, E& c2) {
  const E XX = fp2_sqr(T.x);
  const E YY = fp2_sqr(T.y);
  const E ZZ = fp2_sqr(T.z);
  const E YZ = fp2_mul(T.y, T.z);
  const E bZZ = fp2_mul_b(ZZ);
  const E b3 = fp2_add(fp2_dbl(bZZ), bZZ);        // 3 b' Z^2
  const E b9 = fp2_add(fp2_dbl(b3), b3);          // 9 b' Z^2
  c0 = fp2_sub(YY, b3);
  c1 = fp2_mul_fp(XX, P.n3x);
  c2 = fp2_mul_fp(YZ, P.y2);
  const E XY = fp2_mul(T.x, T.y);
  const E h = fp2_half(fp2_add(YY, b9));
  const E b3sq = fp2_sqr(b3);                      // 9 b'^2 Z^4
  g2_proj<E> R;
  R.x = fp2_half(fp2_mul(XY, fp2_sub(YY, b9)));
  R.y = fp2_sub(fp2_sqr(h), fp2_add(fp2_dbl(b3sq), b3sq));  // h^2 - 27 b'^2 Z^4
  R.z = fp2_dbl(fp2_mul(YY, YZ));
  T = R;
}

// addition step: T <- T + Q, returns the chord through T and Q evaluated at P
template <class E>
BLS_HD inline void line_add(g2_proj<E>& T, const aff_t<E>& Q, const g1_line_pre& P, E& c0, E& c1, E& c2) {
  const E u = fp2_sub(fp2_mul(Q.y, T.z), T.y);
  const E v = fp2_sub(fp2_mul(Q.x, T.z), T.x);
  c0 = fp2_sub(fp2_mul(u, Q.x), fp2_mul(v, Q.y));
  c1 = fp2_mul_fp(u, P.nx);
  c2 = fp2_mul_fp(v, P.y);
  const E vv = fp2_sqr(v);
  const E vvv = fp2_mul(vv, v);
  const E vvX = fp2_mul(vv, T.x);
  const E A = fp2_sub(fp2_sub(fp2_mul(fp2_sqr(u), T.z), vvv), fp2_dbl(vvX));
  g2_proj<E> R;
  R.x = fp2_mul(v, A);
  R.y = fp2_sub(fp2_mul(u, fp2_sub(vvX, A)), fp2_mul(vvv, T.y));
  R.z = fp2_mul(vvv, T.z);
  T = R;
}

// Multi-Miller loop over n pairs (Q_k affine in G2, P_k affine in G1), all finite.
// Returns conj(prod_k f_{|x|,Q_k}(P_k)) = prod_k f_{x,Q_k}(P_k) up to factors the
// final exponentiation removes.  Squarings of f are shared by all pairs.
// One function per pair count; inside it the Fp12 squaring and line products
// are inlined so f stays in registers for the whole loop.
template <int N, class E>
BLS_NOINLINE fp12_g<E> miller_loop_n(const aff_t<E>* Q, const g1_line_pre* P) {
  g2_proj<E> T[N];
  for (int k = 0; k < N; ++k) { T[k].x = Q[k].x; T[k].y = Q[k].y; T[k].z = e2_one<E>(); }
  fp12_g<E> f = fp12_one<E>();
  bool first = true;
  for (int i = 62; i >= 0; --i) {
    if (!first) f = fp12_sqr_inl(f);
    for (int k = 0; k < N; ++k) {
      E c0, c1, c2;
      line_dbl(T[k], P[k], c0, c1, c2);
      f = fp12_mul_by_line_inl(f, c0, c1, c2);
    }
    first = false;
    if ((BLS_X_ABS >> i) & 1) {
      for (int k = 0; k < N; ++k) {
        E c0, c1, c2;
        line_add(T[k], Q[k], P[k], c0, c1, c2);
        f = fp12_mul_by_line_inl(f, c0, c1, c2);
      }
    }
  }
  return fp12_conj(f);
}

// runtime pair count (for verify_multiple chunks); pairs processed one at a time
template <class E>
BLS_HD inline fp12_g<E> miller_loop_1(const aff_t<E>& Q, const g1_line_pre& P) {
  return miller_loop_n<1>(&Q, &P);
}

// f^|x| in the cyclotomic subgroup, then conjugate for x < 0.
// |x| = 0xd201000000010000 has bits 63, 62, 60, 57, 48, 16: after r = f the
// squarings come in runs of 1, 2, 3, 9, 32 (each followed by r *= f) and a
// final 16.  One call per exponentiation; the runs are tight loops of inlined
// cyclotomic squarings, so r stays in registers (only the five products pass
// it through memory).
BLS_CONST int CYC_X_RUNS[6] = {1, 2, 3, 9, 32, 16};

template <class E>
BLS_NOINLINE fp12_g<E> cyc_exp_x(const fp12_g<E>& f) {
  fp12_g<E> r = f;
  for (int s = 0; s < 6; ++s) {
    for (int j = CYC_X_RUNS[s]; j > 0; --j) r = fp12_cyclotomic_sqr_inl(r);
    if (s < 5) r = fp12_mul(r, f);
  }
  return fp12_conj(r);
}

// f^(3 (q^12 - 1)/r).  3 is coprime to r, so the result is 1 exactly when the
// reduced pairing value is 1 (DESIGN.md "Final exponentiation").
// Hard part: 3 (q^4 - q^2 + 1)/r = (x-1)^2 (x+q) (x^2+q^2-1) + 3.
template <class E>
BLS_HD inline fp12_g<E> final_exp(const fp12_g<E>& f) {
  fp12_g<E> t = fp12_mul(fp12_conj(f), fp12_inv(f));     // f^(q^6 - 1)
  t = fp12_mul(fp12_frob(t, 2), t);                     // ^(q^2 + 1)
  fp12_g<E> a = fp12_mul(cyc_exp_x(t), fp12_conj(t));     // t^(x-1)
  a = fp12_mul(cyc_exp_x(a), fp12_conj(a));            // t^((x-1)^2)
  const fp12_g<E> b = fp12_mul(cyc_exp_x(a), fp12_frob(a, 1));            // a^(x+q)
  const fp12_g<E> bx2 = cyc_exp_x(cyc_exp_x(b));
  const fp12_g<E> c = fp12_mul(fp12_mul(bx2, fp12_frob(b, 2)), fp12_conj(b));  // b^(x^2+q^2-1)
  const fp12_g<E> t3 = fp12_mul(fp12_cyclotomic_sqr(t), t);
  return fp12_mul(c, t3);
}

}  // namespace bls381
