// SHA-256 (specs/core/0_beacon-chain.md:591-595) and the spec's try-and-increment
// hash_to_G2 (specs/bls_signature.md:68-87) on the device.
#pragma once
#include "bls381_curve.hpp"

namespace bls381 {

BLS_CONST uint32_t SHA256_K[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

BLS_INLINE uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

// one compression of a 16-word big-endian block into state h[8]
BLS_DEV_INLINE void sha256_compress(uint32_t h[8], const uint32_t blk[16]) {
  uint32_t w[64];
  for (int i = 0; i < 16; ++i) w[i] = blk[i];
  for (int i = 16; i < 64; ++i) {
    const uint32_t s0 = rotr32(w[i - 15], 7) ^ rotr32(w[i - 15], 18) ^ (w[i - 15] >> 3);
    const uint32_t s1 = rotr32(w[i - 2], 17) ^ rotr32(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 64; ++i) {
    const uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
    const uint32_t ch = (e & f) ^ (~e & g);
    const uint32_t t1 = hh + S1 + ch + SHA256_K[i] + w[i];
    const uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
    const uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    const uint32_t t2 = S0 + mj;
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

// SHA-256 of an arbitrary byte string (multi-block), digest as 8 big-endian words
BLS_DEV_INLINE void sha256(uint32_t out[8], const uint8_t* msg, uint32_t len) {
  uint32_t h[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                   0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  const uint64_t bitlen = (uint64_t)len * 8;
  const uint32_t nblocks = (len + 9 + 63) / 64;
  for (uint32_t bi = 0; bi < nblocks; ++bi) {
    uint32_t blk[16];
    for (int wi = 0; wi < 16; ++wi) {
      uint32_t word = 0;
      for (int k = 0; k < 4; ++k) {
        const uint64_t pos = (uint64_t)bi * 64 + wi * 4 + k;
        uint8_t byte;
        if (pos < len) byte = msg[pos];
        else if (pos == len) byte = 0x80;
        else if (pos >= (uint64_t)nblocks * 64 - 8) byte = (uint8_t)(bitlen >> (8 * (nblocks * 64 - 1 - pos)));
        else byte = 0;
        word = (word << 8) | byte;
      }
      blk[wi] = word;
    }
    sha256_compress(h, blk);
  }
  for (int i = 0; i < 8; ++i) out[i] = h[i];
}

// SHA-256 of msg || dom8 || tag (mlen + 9 bytes), the input of hash_to_G2's two
// coordinate hashes (bls_signature.md:76-77), read straight from msg: no copy,
// no per-lane buffer, so the message may be any length.
BLS_DEV_INLINE void sha256_msg_dom_tag(uint32_t out[8], const uint8_t* msg, uint32_t mlen, const uint8_t dom8[8],
                                      uint8_t tag) {
  uint32_t h[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                   0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  const uint64_t len = (uint64_t)mlen + 9;
  const uint64_t bitlen = len * 8;
  const uint64_t nblocks = (len + 9 + 63) / 64;
  for (uint64_t bi = 0; bi < nblocks; ++bi) {
    uint32_t blk[16];
    for (int wi = 0; wi < 16; ++wi) {
      uint32_t word = 0;
      for (int k = 0; k < 4; ++k) {
        const uint64_t pos = bi * 64 + wi * 4 + k;
        uint8_t byte;
        if (pos < mlen) byte = msg[pos];
        else if (pos < (uint64_t)mlen + 8) byte = dom8[pos - mlen];
        else if (pos == (uint64_t)mlen + 8) byte = tag;
        else if (pos == len) byte = 0x80;
        else if (pos >= nblocks * 64 - 8) byte = (uint8_t)(bitlen >> (8 * (nblocks * 64 - 1 - pos)));
        else byte = 0;
        word = (word << 8) | byte;
      }
      blk[wi] = word;
    }
    sha256_compress(h, blk);
  }
  for (int i = 0; i < 8; ++i) out[i] = h[i];
}

// 8 big-endian digest words -> plain Fp limbs (256-bit value < q)
BLS_INLINE fp_t fp_plain_from_digest(const uint32_t d[8]) {
  uint8_t b[48];
  for (int i = 0; i < 16; ++i) b[i] = 0;
  for (int i = 0; i < 8; ++i) {
    b[16 + 4 * i] = (uint8_t)(d[i] >> 24); b[17 + 4 * i] = (uint8_t)(d[i] >> 16);
    b[18 + 4 * i] = (uint8_t)(d[i] >> 8); b[19 + 4 * i] = (uint8_t)d[i];
  }
  return fp_plain_from_be48(b);
}

// spec root selection (bls_signature.md:91,107): keep the root whose imaginary
// part is the larger of {y_im, q - y_im}, ties (y_im == 0) broken on the real part.
template <class E>
BLS_INLINE E g2_select_root(const E& y) {
  return g2_y_flag(y) ? y : fp2_neg(y);
}

// try-and-increment part of hash_to_G2 (bls_signature.md:74-86), before the cofactor.
// msg may be any length (py_ecc hashes any bytes); dom8 = 8 domain bytes.
BLS_DEV_INLINE int hash_to_g2_candidate(aff_t<fp2_t>& out, const uint8_t* msg, uint32_t mlen,
                                       const uint8_t dom8[8]) {
  uint32_t d[8];
  sha256_msg_dom_tag(d, msg, mlen, dom8, 1);
  fp2_t x;
  x.c0 = fp_to_mont(fp_plain_from_digest(d));
  sha256_msg_dom_tag(d, msg, mlen, dom8, 2);
  x.c1 = fp_to_mont(fp_plain_from_digest(d));
  // rhs is a square in Fp2 iff its norm is a square in Fp: the cheap Legendre
  // test finds the candidate, then one square root is taken
  int trials = 0;
  fp2_t rhs;
  while (true) {
    ++trials;
    rhs = fp2_add(fp2_mul(fp2_sqr(x), x), G2_B_M);
    if (fp_legendre(fp_add(fp_sqr(rhs.c0), fp_sqr(rhs.c1))) >= 0) break;
    x.c0 = fp_add(x.c0, FP_ONE_M);
  }
  fp2_t y;
  fp2_sqrt(y, rhs);   // succeeds: rhs is a square
  out.x = x;
  out.y = g2_select_root(y);
  return trials;
}

// psi on Jacobian coordinates: (cx conj(X), cy conj(Y), conj(Z))
template <class E>
BLS_INLINE jac_t<E> g2_psi_jac(const jac_t<E>& p) {
  jac_t<E> r;
  r.x = fp2_mul(e2_k<E>(PSI_CX_M), fp2_conj(p.x));
  r.y = fp2_mul(e2_k<E>(PSI_CY_M), fp2_conj(p.y));
  r.z = fp2_conj(p.z);
  return r;
}

// [h2] P for the spec's full G2_cofactor h2 (bls_signature.md:71), exactly.
// With c = 3(x^2 - 1), the Budroni-Pintore combination
//   BP(P) = [x^2 - x - 1]P + [x - 1]psi(P) + 2 psi^2(P)  equals  [c h2]P
// for every P in E'(Fp2), and BP(P) lies in G2 where psi acts as [x].  Hence
// [h2]P = [c^-1 mod r] BP(P), and c^-1 mod r = sum_i e_i |x|^i with
// e0 = (|x|+1)/3, e1 = 2e0 - 1, e2 = 2e0 - 2, e3 = e0 - 1, which collapses to
//   [h2]P = [e0] S - T,  S = Q0 + 2Q1 + 2Q2 + Q3,  T = Q1 + 2Q2 + Q3,
//   Q_i = (-psi)^i BP(P).
// ~190 doublings + ~45 additions instead of the 508-doubling ladder; the
// identity is checked in oracle/tower_model.py and tests/test_tower_model.py.
// [e0] S by the NAF of e0 (leading digit +1); one call, loop body inlined.  S is
// made affine first (one Fp2 inversion, a binary-xgcd Fp inverse): each of the
// NAF's additions is then a mixed addition (7M + 4S instead of 11M + 5S).
template <class E>
BLS_NOINLINE jac_t<E> g2_mul_e0(const jac_t<E> S) {
  aff_t<E> a;
  if (!jac_to_aff(a, S)) return S;   // S = O: [e0] O = O
  aff_t<E> na;
  na.x = a.x;
  na.y = f_neg(a.y);
  jac_t<E> R = jac_from_aff(a);
  for (int i = 1; i < E0_NAF_LEN; ++i) {
    R = jac_dbl(R);
    const int dg = E0_NAF[i];
    if (dg > 0) R = jac_add_aff(R, a);
    else if (dg < 0) R = jac_add_aff(R, na);
  }
  return R;
}

// BP(P) = [c h2]P, c = 3(x^2 - 1): the verification hash.  The verify paths pair
// BP(H0) with the pubkey and the signature with -[c]g1 (G1_VGEN_*) instead of
// H = [h2]H0 with pk and sig with -g1: both pairing products are the original
// one raised to c, which is coprime to r, so "== 1" is unchanged (the reduced
// pairing is bilinear in its G2 argument for any G1-side point; tested against
// every torsion fixture).  Skips the [e0]S - T step of g2_mul_cofactor.
// BLS_BP_INLINE_LADDERS=1 (measurement knob): the two [|x|] ladders inlined into g2_mul_bp instead
// of calls.  r05: k_hash_bp's private segment 1,376 -> 1,808 B (the ladders' spills share one frame
// with the rest of the map), so the calls stay
#ifndef BLS_BP_INLINE_LADDERS
#define BLS_BP_INLINE_LADDERS 0
#endif
template <class E>
BLS_NOINLINE jac_t<E> g2_mul_bp(const aff_t<E> p) {
  aff_t<E> np;
  np.x = p.x;
  np.y = fp2_neg(p.y);
#if BLS_BP_INLINE_LADDERS
  const jac_t<E> t1 = jac_mul_u64_body(p, BLS_X_ABS);             // [|x|]P = -[x]P
  jac_t<E> Q0 = jac_add_aff(jac_add(jac_mul_u64_jac_body(t1, BLS_X_ABS), t1), np);   // [x^2 - x - 1]P
#else
  const jac_t<E> t1 = jac_mul_u64(p, BLS_X_ABS);                  // [|x|]P = -[x]P
  jac_t<E> Q0 = jac_add_aff(jac_add(jac_mul_u64_jac(t1, BLS_X_ABS), t1), np);   // [x^2 - x - 1]P
#endif
  Q0 = jac_add(Q0, g2_psi_jac(jac_add_aff(jac_neg(t1), np)));          // + psi([x - 1]P)
  return jac_add(Q0, g2_psi_jac(g2_psi_jac(jac_dbl(jac_from_aff(p)))));  // + psi^2(2P)
}

template <class E>
BLS_NOINLINE jac_t<E> g2_mul_cofactor(const aff_t<E> p) {
  const jac_t<E> Q0 = g2_mul_bp(p);
  const jac_t<E> Q1 = jac_neg(g2_psi_jac(Q0));
  const jac_t<E> Q2 = jac_neg(g2_psi_jac(Q1));
  const jac_t<E> T = jac_add(jac_add(jac_dbl(Q2), Q1), jac_neg(g2_psi_jac(Q2)));   // Q1 + 2Q2 + Q3
  const jac_t<E> S = jac_add(jac_add(T, Q1), Q0);
  return jac_add(g2_mul_e0(S), jac_neg(T));
}

// full hash_to_G2 for a 32-byte message; returns false only if the result is infinity
BLS_DEV_INLINE bool hash_to_g2_aff(aff_t<fp2_t>& out, const uint8_t msg[32], const uint8_t dom8[8]) {
  aff_t<fp2_t> c;
  hash_to_g2_candidate(c, msg, 32, dom8);
  return jac_to_aff(out, g2_mul_cofactor(c));
}

}  // namespace bls381
