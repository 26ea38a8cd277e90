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
#if BLS_ML_QUAD_INLINE
__device__ __forceinline__
#else
__device__ __noinline__
#endif
fq12_t miller_loop_quad(const aff_t<fp2p_t>& Q, const g1_line_pre& P, bool active,
                                                bool& degenerate) {
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
  degenerate = !qd_all(!deg);
  return fq12_conj(f);
}

}  // namespace bls381
