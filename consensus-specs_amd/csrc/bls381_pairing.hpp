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
#include "bls381_lazy.hpp"

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
  r.n3x = fp_mul_small(r.nx, 3);
  r.y = p.y;
  r.y2 = fp_dbl(p.y);
  return r;
}

// homogeneous-projective T on E'(Fp2)
template <class E> struct g2_proj { E x, y, z; };

// the doubling step reads only -3 xp and 2 yp, through these accessors: a kernel may keep
// them elsewhere than in a g1_line_pre (k_ml_lines: in LDS)
BLS_DEV_INLINE const fp_t& pre_n3x(const g1_line_pre& p) { return p.n3x; }
BLS_DEV_INLINE const fp_t& pre_y2(const g1_line_pre& p) { return p.y2; }

// doubling step: T <- 2T, returns the tangent line at the old T evaluated at P
template <class E, class PRE>
BLS_DEV_INLINE void line_dbl(g2_proj<E>& T, const PRE& P, E& c0, E& c1, E& c2) {
  const E XX = fp2_sqr(T.x);
  const E YY = fp2_sqr(T.y);
  const E ZZ = fp2_sqr(T.z);
  const E YZ = fp2_mul(T.y, T.z);
  const E b3 = fp2_mul_small(fp2_mul_small(fp2_mul_xi(ZZ), 3), 4);   // 3 b' Z^2 = 12 xi Z^2
  const E b9 = fp2_mul_small(b3, 3);                                 // 9 b' Z^2
  c0 = fp2_sub(YY, b3);
  c1 = fp2_mul_fp(XX, pre_n3x(P));
  c2 = fp2_mul_fp(YZ, pre_y2(P));
  const E XY = fp2_mul(T.x, T.y);
  const E h = fp2_half(fp2_add(YY, b9));
  const E b3sq = fp2_sqr(b3);                      // 9 b'^2 Z^4
  g2_proj<E> R;
  R.x = fp2_half(fp2_mul(XY, fp2_sub(YY, b9)));
  R.y = fp2_sub(fp2_sqr(h), fp2_mul_small(b3sq, 3));  // h^2 - 27 b'^2 Z^4
  R.z = fp2_dbl(fp2_mul(YY, YZ));
  T = R;
}

// addition step: T <- T + Q, returns the chord through T and Q evaluated at P
template <class E>
BLS_DEV_INLINE void line_add(g2_proj<E>& T, const aff_t<E>& Q, const g1_line_pre& P, E& c0, E& c1, E& c2) {
  const E u = fp2_sub(fp2_mul(Q.y, T.z), T.y);
  const E v = fp2_sub(fp2_mul(Q.x, T.z), T.x);
  c0 = fp2_sub(fp2_mul(u, Q.x), fp2_mul(v, Q.y));
  c1 = fp2_mul_fp(u, P.nx);
  c2 = fp2_mul_fp(v, P.y);
  const E vv = fp2_sqr(v);
  const E vvv = fp2_mul(vv, v);
  const E vvX = fp2_mul(vv, T.x);
  const E A = fp2_sub2(fp2_mul(fp2_sqr(u), T.z), vvv, fp2_dbl(vvX));
  g2_proj<E> R;
  R.x = fp2_mul(v, A);
  R.y = fp2_sub(fp2_mul(u, fp2_sub(vvX, A)), fp2_mul(vvv, T.y));
  R.z = fp2_mul(vvv, T.z);
  T = R;
}

// Two lines of one Miller step multiplied together before they meet f:
//   l = (c0 + c1 v) + (c2 v) w,  l' = (d0 + d1 v) + (d2 v) w
//   l l' = (t0 + xi s + m v + t1 v^2) + ((u - t0 - s) v + (u' - t1 - s) v^2) w
// with t0 = c0 d0, t1 = c1 d1, s = c2 d2, m = (c0 + c1)(d0 + d1) - t0 - t1,
// u = (c0 + c2)(d0 + d2), u' = (c1 + c2)(d1 + d2): 6 Fp2 products, and the product
// has no w v^0 coefficient (fp12_mul_by_line_pair_inl uses that).
template <class E>
BLS_INLINE fp12_g<E> line_pair_product(const E& c0, const E& c1, const E& c2,
                                       const E& d0, const E& d1, const E& d2) {
  const E t0 = fp2_mul(c0, d0);
  const E t1 = fp2_mul(c1, d1);
  const E s = fp2_mul(c2, d2);
  fp12_g<E> L;
  L.c0.c0 = fp2_add_mul_xi(t0, s);
  L.c0.c1 = fp2_sub2(fp2_mul(fp2_add_lazy(c0, c1), fp2_add_lazy(d0, d1)), t0, t1);
  L.c0.c2 = t1;
  L.c1.c0 = e2_zero<E>();
  L.c1.c1 = fp2_sub2(fp2_mul(fp2_add_lazy(c0, c2), fp2_add_lazy(d0, d2)), t0, s);
  L.c1.c2 = fp2_sub2(fp2_mul(fp2_add_lazy(c1, c2), fp2_add_lazy(d1, d2)), t1, s);
  return L;
}

// f * L for L = P + Q w with Q = q1 v + q2 v^2 (line_pair_product's shape): 6 + 5 + 6 = 17
// Fp2 products, against 2 x 13 for the two lines one at a time.
template <class E>
BLS_INLINE fp12_g<E> fp12_mul_by_line_pair_inl(const fp12_g<E>& f, const fp12_g<E>& L) {
  const fp6_g<E>& a = f.c0;
  const fp6_g<E>& b = f.c1;
  const fp6_g<E> aP = fp6_mul_inl(a, L.c0);
  // b Q: v^0 xi (b1 q2 + b2 q1), v^1 b0 q1 + xi b2 q2, v^2 b0 q2 + b1 q1
  fp6_g<E> bQ;
  {
    const E t1 = fp2_mul(b.c1, L.c1.c1);
    const E t2 = fp2_mul(b.c2, L.c1.c2);
    bQ.c0 = fp2_mul_xi(fp2_sub2(fp2_mul(fp2_add_lazy(b.c1, b.c2), fp2_add_lazy(L.c1.c1, L.c1.c2)), t1, t2));
    bQ.c1 = fp2_add_mul_xi(fp2_mul(b.c0, L.c1.c1), t2);
    bQ.c2 = fp2_add(fp2_mul(b.c0, L.c1.c2), t1);
  }
  fp6_g<E> pq;
  pq.c0 = L.c0.c0;
  pq.c1 = fp2_add(L.c0.c1, L.c1.c1);
  pq.c2 = fp2_add(L.c0.c2, L.c1.c2);
  const fp6_g<E> m = fp6_mul_inl(fp6_add(a, b), pq);
  fp12_g<E> r;
  r.c0 = fp6_add_mul_by_v(aP, bQ);
  r.c1 = fp6_sub2(m, aP, bQ);
  return r;
}

// (Round 2 measured multiplying the lines of pairs k, k+1 together first, 23 instead of 26 Fp2
// products per step, on this loop: 14.15 against 13.97 ms, the product's live set adds spills;
// the knob BLS_ML_LINE_PAIR was removed in round 6.  The split Miller loop's k_ml_lines / k_ml_accum
// do form L = l l' -- there each kernel holds only its own half of the state.)

// Multi-Miller loop over n pairs (Q_k affine in G2, P_k affine in G1), all finite.
// Returns conj(prod_k f_{|x|,Q_k}(P_k)) = prod_k f_{x,Q_k}(P_k) up to factors the
// final exponentiation removes.  Squarings of f are shared by all pairs.
// One function per pair count; inside it the Fp12 squaring and line products
// are inlined so f stays in registers for the whole loop.
//
// `degenerate` is set when some running point T_k reached infinity (Z = 0).
// That happens only for a Q_k with no G2 component whose small order divides a
// prefix of |x| (an order-13 point of E'(Fp2); DESIGN.md "Subgroup policy"):
// T = -Q in an addition step gives Z = 0, and Z = 0 stays 0 through every later
// step.  py_ecc's Miller loop then doubles the point at infinity, whose line
// has a zero denominator, so its pairing value is 0 and the verdict False; the
// kernels map the flag to that verdict.  Points of G2 never reach it.
// T0_out != nullptr: receives the first pair's final running point, [|x|] Q[0] in
// homogeneous projective coordinates (the signature's G2 membership test rides on it,
// g2_psi_matches_neg).
// The loop itself takes its pairs and returns its results by value (miller_loop_run): no
// pointer into the caller's private memory crosses the call; the pointer
// form below is a force-inlined wrapper over the caller's own arrays.
template <int N, class E> struct ml_pairs { aff_t<E> Q[N]; g1_line_pre P[N]; };
template <class E> struct ml_result { fp12_g<E> f; g2_proj<E> T0; bool degenerate; };

template <int N, class E>
BLS_NOINLINE ml_result<E> miller_loop_run(const ml_pairs<N, E> in) {
  const aff_t<E>* Q = in.Q;
  const g1_line_pre* P = in.P;
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
  bool deg = false;
  for (int k = 0; k < N; ++k) deg = deg | fp2_is_zero(T[k].z);   // no short circuit: pair-uniform DPP
  ml_result<E> r;
  r.f = fp12_conj(f);
  r.T0 = T[0];
  r.degenerate = deg;
  return r;
}

template <int N, class E>
BLS_DEV_INLINE fp12_g<E> miller_loop_n(const aff_t<E>* Q, const g1_line_pre* P, bool& degenerate,
                                   g2_proj<E>* T0_out = nullptr) {
  ml_pairs<N, E> in;
  for (int k = 0; k < N; ++k) { in.Q[k] = Q[k]; in.P[k] = P[k]; }
  const ml_result<E> r = miller_loop_run<N, E>(in);
  degenerate = r.degenerate;
  if (T0_out) *T0_out = r.T0;
  return r.f;
}

// G2 membership from a Miller loop's by-product: Q in G2 iff psi(Q) == [x] Q = -[|x|] Q, and
// the loop's final running point T (homogeneous projective, Z != 0) is [|x|] Q.
template <class E>
BLS_DEV_INLINE bool g2_psi_matches_neg(const aff_t<E>& q, const g2_proj<E>& T) {
  const aff_t<E> s = g2_psi(q);
  const bool a = fp2_eq(fp2_mul(s.x, T.z), T.x);
  const bool b = fp2_eq(fp2_mul(s.y, T.z), fp2_neg(T.y));
  return a & b;
}

// runtime pair count (for verify_multiple chunks); pairs processed one at a time
template <class E>
BLS_DEV_INLINE fp12_g<E> miller_loop_1(const aff_t<E>& Q, const g1_line_pre& P, bool& degenerate) {
  return miller_loop_n<1>(&Q, &P, degenerate);
}

// f^|x| in the cyclotomic subgroup by Granger-Scott squarings, then conjugate
// for x < 0.  |x| = 0xd201000000010000 has bits 63, 62, 60, 57, 48, 16: after
// r = f the squarings come in runs of 1, 2, 3, 9, 32 (each followed by r *= f)
// and a final 16.  The runs are tight loops of inlined cyclotomic squarings, so
// r stays in registers.  This is the exact fallback of cyc_exp_x below.
BLS_CONST int CYC_X_RUNS[6] = {1, 2, 3, 9, 32, 16};

template <class E>
BLS_NOINLINE fp12_g<E> cyc_exp_x_gs(const fp12_g<E> f) {
  fp12_g<E> r = f;
  for (int s = 0; s < 6; ++s) {
    for (int j = CYC_X_RUNS[s]; j > 0; --j) r = fp12_cyclotomic_sqr_inl(r);
    if (s < 5) r = fp12_mul(r, f);
  }
  return fp12_conj(r);
}

// Karabina compressed squaring.  With z = w^3, f = A + B w + C w^2 over
// Fp4 = Fp2[z]; the Granger-Scott outputs B' = 3 z C^2 + 2 conj(B) and
// C' = 3 B^2 - 2 conj(C) depend on B and C only, so
//   (g2, g3, g4, g5) = (B0, B1, C0, C1) = (b0, a2, a1, b2)
// squares on its own with six Fp2 squarings (Granger-Scott: nine), and
// A = (a0, b1) comes back from the norm condition f conj(f) = 1:
//   b1 = (xi g5^2 + 3 g4^2 - 2 g3) / (4 g2),  a0 = xi (2 b1^2 + g2 g5 - 3 g3 g4) + 1.
// Mirrored by oracle/tower_model.py (cyc_csqr / cyc_decompress).
template <class E> struct cyc_bc { E g2, g3, g4, g5; };

template <class E>
BLS_INLINE cyc_bc<E> cyc_compress(const fp12_g<E>& f) {
  cyc_bc<E> g; g.g2 = f.c1.c0; g.g3 = f.c0.c2; g.g4 = f.c0.c1; g.g5 = f.c1.c2; return g;
}

// BLS_LAZY_CSQR=1: each output coefficient is one lazily reduced sum of products
// (bls381_lazy.hpp): 10 products and 4 reductions per lane instead of 6 Fp2 squarings
// (12 reductions) and 11 reduced linear combinations.
#ifndef BLS_LAZY_CSQR
#define BLS_LAZY_CSQR 1
#endif

// the one-lane representation: the per-lane functions once per coefficient
BLS_INLINE cyc_bc<fp2_t> cyc_csqr_lazy(const cyc_bc<fp2_t>& g) {
  cyc_bc<fp2_t> r;
  for (int p = 0; p < 2; ++p) {
    fp_t& o2 = p ? r.g2.c1 : r.g2.c0;
    fp_t& o3 = p ? r.g3.c1 : r.g3.c0;
    fp_t& o4 = p ? r.g4.c1 : r.g4.c0;
    fp_t& o5 = p ? r.g5.c1 : r.g5.c0;
    o2 = fp_6p2(lz_xi_mul(p, g.g4.c0, g.g4.c1, g.g5.c0, g.g5.c1), p ? g.g2.c1 : g.g2.c0);
    o3 = fp_3m2(lz_sqr_xisqr(p, g.g4.c0, g.g4.c1, g.g5.c0, g.g5.c1), p ? g.g3.c1 : g.g3.c0);
    o4 = fp_3m2(lz_sqr_xisqr(p, g.g2.c0, g.g2.c1, g.g3.c0, g.g3.c1), p ? g.g4.c1 : g.g4.c0);
    o5 = fp_6p2(lz_mul(p, g.g2.c0, g.g2.c1, g.g3.c0, g.g3.c1), p ? g.g5.c1 : g.g5.c0);
  }
  return r;
}

template <class E>
BLS_INLINE cyc_bc<E> cyc_csqr(const cyc_bc<E>& g) {
#if BLS_LAZY_CSQR
  return cyc_csqr_lazy(g);   // fp2p_t: bls381_pair.hpp
#else
  cyc_bc<E> r;
  {
    const E t0 = fp2_sqr(g.g4), t1 = fp2_sqr(g.g5), t2 = fp2_sqr(fp2_add(g.g4, g.g5));
    r.g2 = fp2_3p2(fp2_mul_xi(fp2_sub2(t2, t0, t1)), g.g2);   // 6 xi g4 g5 + 2 g2
    r.g3 = fp2_3m2(fp2_add_mul_xi(t0, t1), g.g3);             // 3 (g4^2 + xi g5^2) - 2 g3
  }
  const E t3 = fp2_sqr(g.g2), t4 = fp2_sqr(g.g3), t5 = fp2_sqr(fp2_add(g.g2, g.g3));
  r.g4 = fp2_3m2(fp2_add_mul_xi(t3, t4), g.g4);               // 3 (g2^2 + xi g3^2) - 2 g4
  r.g5 = fp2_3p2(fp2_sub2(t5, t3, t4), g.g5);                 // 6 g2 g3 + 2 g5
  return r;
#endif
}

// the full element from (g2..g5) and 1 / (4 g2)
template <class E>
BLS_INLINE fp12_g<E> cyc_decompress(const cyc_bc<E>& g, const E& inv4g2) {
  const E num = fp2_sub2(fp2_add_mul_xi(fp2_mul_small(fp2_sqr(g.g4), 3), fp2_sqr(g.g5)), g.g3, g.g3);
  const E b1 = fp2_mul(num, inv4g2);
  const E u = fp2_sub(fp2_add(fp2_dbl(fp2_sqr(b1)), fp2_mul(g.g2, g.g5)), fp2_mul_small(fp2_mul(g.g3, g.g4), 3));
  fp12_g<E> f;
  f.c0.c0 = fp2_add(fp2_mul_xi(u), e2_one<E>());
  f.c0.c1 = g.g4; f.c0.c2 = g.g3;
  f.c1.c0 = g.g2; f.c1.c1 = b1; f.c1.c2 = g.g5;
  return f;
}

// f^x, right to left: f^|x| = prod over the six set bits b of f^(2^b).  The 63
// squarings run compressed; the six snapshots share one Fp2 inversion
// (Montgomery's trick) and are multiplied together.  A snapshot with g2 = 0 (f = 1,
// or a point of measure zero) cannot be decompressed this way: if any lane of the
// wave has one, the wave takes the Granger-Scott path instead (uniform branch).
BLS_CONST int CYC_X_RUNS_RTL[6] = {16, 32, 9, 3, 2, 1};

// Only the snapshots after 16, 48 and 57 squarings are compressed ones.  The last six
// squarings (runs 3, 2, 1) continue from the decompressed f^(2^57) with Granger-Scott squarings
// on the full element: three decompressions and their shares of the shared inversion (~30 Fp2
// products) against six dearer squarings (~6 x 1.3 Fp2 products).  (r03q: the all-compressed
// form with six snapshots measured the same time with a 480 B larger frame; removed in r06.)

// BLS_FE_MARK(k): phase marks for tools/fe_phases.hip (no code in the library)
#ifndef BLS_FE_MARK
#define BLS_FE_MARK(k)
#endif
#ifndef BLS_FE_STEP
#define BLS_FE_STEP(j)
#endif

// the final exponentiation's Fp12 products are inlined (r04r: as calls, fp12_mul with its
// operands through the stack, 9.79-9.83 against 9.16-9.20 ms per 2^16 launch)
#define FE_MUL12 fp12_mul_inl

template <class E>
BLS_INLINE fp12_g<E> fp12_zero() { fp12_g<E> r; r.c0 = fp6_zero<E>(); r.c1 = fp6_zero<E>(); return r; }

// FB: what a wave does when a snapshot has g2 = 0 (f = 1 from the infinity/infinity verify, or a
// point of measure zero), where the compressed form cannot be decompressed:
//   1: the exact Granger-Scott chain cyc_exp_x_gs, in this call (host build, latency kernels);
//   0: the wave returns 0 instead.  0 propagates through final_exp's chain (every later value is
//      a product with it, or an exponentiation of it), so final_exp_check reports the wave's items
//      as to be redone and k_final_exp_redo recomputes them with FB = 1.  The throughput kernel
//      then has neither cyc_exp_x_gs nor the called fp12_mul it uses in its call tree: the
//      fallback's 1,360 B + fp12_mul's 2,000 B frames leave every wave's scratch segment
//      (VERDICT r05 next #2).
template <class E, int FB = 1>
BLS_NOINLINE fp12_g<E> cyc_exp_x(const fp12_g<E> f) {
  BLS_FE_MARK(7);
  cyc_bc<E> snap[3];
  cyc_bc<E> g = cyc_compress(f);
  bool zero = false;
  for (int s = 0; s < 3; ++s) {
    for (int j = CYC_X_RUNS_RTL[s]; j > 0; --j) {
      g = cyc_csqr(g);
      BLS_FE_STEP(j);
    }
    snap[s] = g;
    const bool zs = fp2_is_zero(g.g2);   // evaluated on both lanes of a pair
    zero = zero | zs;
  }
  BLS_FE_MARK(0);
  if (BLS_ANY(zero)) {
    if constexpr (FB != 0) return cyc_exp_x_gs(f);
    else return fp12_zero<E>();
  }
  const E d0 = fp2_mul_small(snap[0].g2, 4), d1 = fp2_mul_small(snap[1].g2, 4);
  const E p01 = fp2_mul(d0, d1);
  E inv = fp2_inv(fp2_mul(p01, fp2_mul_small(snap[2].g2, 4)));   // 1 / (d0 d1 d2)
  BLS_FE_MARK(1);
  fp12_g<E> x = cyc_decompress(snap[2], fp2_mul(inv, p01));       // f^(2^57)
  inv = fp2_mul(inv, fp2_mul_small(snap[2].g2, 4));               // 1 / (d0 d1)
  fp12_g<E> r = FE_MUL12(x, cyc_decompress(snap[1], fp2_mul(inv, d0)));
  r = FE_MUL12(r, cyc_decompress(snap[0], fp2_mul(inv, d1)));
  BLS_FE_MARK(2);
  for (int s = 3; s < 6; ++s) {
    for (int j = CYC_X_RUNS_RTL[s]; j > 0; --j) x = fp12_cyclotomic_sqr_inl(x);
    BLS_FE_MARK(3);
    r = FE_MUL12(r, x);
    BLS_FE_MARK(4);
  }
  return fp12_conj(r);
}

// f^(3 (q^12 - 1)/r).  3 is coprime to r, so the result is 1 exactly when the
// reduced pairing value is 1 (DESIGN.md "Final exponentiation").
// Hard part: 3 (q^4 - q^2 + 1)/r = (x-1)^2 (x+q) (x^2+q^2-1) + 3, computed as c * t^3 with
// c = t^((x-1)^2 (x+q) (x^2+q^2-1)) (final_exp_ct returns the two factors).
template <class E> struct fe_ct { fp12_g<E> c, t3; };

template <class E, int FB = 1>
BLS_HD inline fe_ct<E> final_exp_ct(const fp12_g<E> f) {
  fp12_g<E> t = FE_MUL12(fp12_conj(f), fp12_inv(f));     // f^(q^6 - 1)
  t = FE_MUL12(fp12_frob(t, 2), t);                     // ^(q^2 + 1)
  BLS_FE_MARK(5);
  fp12_g<E> a = FE_MUL12(cyc_exp_x<E, FB>(t), fp12_conj(t));     // t^(x-1)
  a = FE_MUL12(cyc_exp_x<E, FB>(a), fp12_conj(a));              // t^((x-1)^2)
  const fp12_g<E> b = FE_MUL12(cyc_exp_x<E, FB>(a), fp12_frob(a, 1));            // a^(x+q)
  const fp12_g<E> bx2 = cyc_exp_x<E, FB>(cyc_exp_x<E, FB>(b));
  fe_ct<E> r;
  r.c = FE_MUL12(FE_MUL12(bx2, fp12_frob(b, 2)), fp12_conj(b));  // b^(x^2+q^2-1)
  r.t3 = FE_MUL12(fp12_cyclotomic_sqr(t), t);
  BLS_FE_MARK(6);
  return r;
}

template <class E>
BLS_HD inline fp12_g<E> final_exp(const fp12_g<E> f) {
  const fe_ct<E> r = final_exp_ct<E, 1>(f);
  return FE_MUL12(r.c, r.t3);
}

// The verdict form: 1 when f^(3(q^12-1)/r) == 1, else 0.  c t^3 == 1 is tested as c == conj(t^3)
// (t^3 is in the cyclotomic subgroup, where the inverse is the conjugate): one Fp12 product
// fewer than final_exp.  FB = 0 (cyc_exp_x): 2 when the item's wave returned the zero marker,
// i.e. c = 0 -- tested on two coefficients, so a genuine c with both zero (a measure-zero event)
// is merely recomputed by the exact launch too.
template <class E, int FB = 1>
BLS_HD inline int final_exp_check(const fp12_g<E> f) {
  const fe_ct<E> r = final_exp_ct<E, FB>(f);
  if (FB == 0 && fp2_is_zero(r.c.c0.c0) && fp2_is_zero(r.c.c1.c0)) return 2;
  return fp12_eq(r.c, fp12_conj(r.t3)) ? 1 : 0;
}

}  // namespace bls381
