// Host unit-test build of the device arithmetic headers -- TEST INFRASTRUCTURE.
//
// g++ compiles the exact headers the gfx950 kernels use so that, in a container
// with no GPU, every layer (Fp ... Fp12, codecs, subgroup checks, hash_to_G2,
// Miller loop, final exponentiation) can be checked against oracle/ by
// tests/test_host_arith.py.  This library is loaded only by tests; it is not a
// fallback and the product library (libbls381.so) never links it.
//
// Byte conventions (all big-endian, plain / non-Montgomery values):
//   Fp 48 B;  Fp2 96 B = re || im;  Fp12 576 B = a0,a1,a2,b0,b1,b2 (each Fp2)
//   G1 affine 96 B = x || y;  G2 affine 192 B = x || y (each Fp2)
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "bls381_hash.hpp"
#include "bls381_pairing.hpp"
#include "bls381_ssz.hpp"

using namespace bls381;

namespace {
fp_t ld(const uint8_t* p) { return fp_to_mont(fp_plain_from_be48(p)); }
void st(uint8_t* p, const fp_t& a) { fp_plain_to_be48(p, fp_from_mont(a)); }
fp2_t ld2(const uint8_t* p) { fp2_t r; r.c0 = ld(p); r.c1 = ld(p + 48); return r; }
void st2(uint8_t* p, const fp2_t& a) { st(p, a.c0); st(p + 48, a.c1); }
fp12_t ld12(const uint8_t* p) {
  fp12_t r;
  r.c0.c0 = ld2(p); r.c0.c1 = ld2(p + 96); r.c0.c2 = ld2(p + 192);
  r.c1.c0 = ld2(p + 288); r.c1.c1 = ld2(p + 384); r.c1.c2 = ld2(p + 480);
  return r;
}
void st12(uint8_t* p, const fp12_t& a) {
  st2(p, a.c0.c0); st2(p + 96, a.c0.c1); st2(p + 192, a.c0.c2);
  st2(p + 288, a.c1.c0); st2(p + 384, a.c1.c1); st2(p + 480, a.c1.c2);
}
aff_t<fp_t> ldg1(const uint8_t* p) { aff_t<fp_t> a; a.x = ld(p); a.y = ld(p + 48); return a; }
aff_t<fp2_t> ldg2(const uint8_t* p) { aff_t<fp2_t> a; a.x = ld2(p); a.y = ld2(p + 96); return a; }
}  // namespace

extern "C" {

// one-reduction combinations on raw normalized limbs (14 x u32, values < 2q, Montgomery
// or not -- the reduction is mod 2q only): op 0 a+b, 1 a-b, 2 -a, 3 2a, 4 a+b-c, 5 a+b+c,
// 6 a-b-c, 7 3a-2b, 8 3a+2b, 9..16 k*a for k = op-8 (k = 1..8)
void hc_fp_lc_raw(int op, const uint32_t* a, const uint32_t* b, const uint32_t* c, uint32_t* o) {
  fp_t x, y, z, r;
  for (int i = 0; i < 14; ++i) { x.w[i] = a[i]; y.w[i] = b[i]; z.w[i] = c[i]; }
  switch (op) {
    case 0: r = fp_add(x, y); break;
    case 1: r = fp_sub(x, y); break;
    case 2: r = fp_neg(x); break;
    case 3: r = fp_dbl(x); break;
    case 4: r = fp_add_sub(x, y, z); break;
    case 5: r = fp_add3(x, y, z); break;
    case 6: r = fp_sub2(x, y, z); break;
    case 7: r = fp_3m2(x, y); break;
    case 8: r = fp_3p2(x, y); break;
    default: r = fp_mul_small(x, op - 8); break;
  }
  for (int i = 0; i < 14; ++i) o[i] = r.w[i];
}

void hc_fp_mul(const uint8_t* a, const uint8_t* b, uint8_t* o) { st(o, fp_mul(ld(a), ld(b))); }
void hc_fp_add(const uint8_t* a, const uint8_t* b, uint8_t* o) { st(o, fp_add(ld(a), ld(b))); }
void hc_fp_sub(const uint8_t* a, const uint8_t* b, uint8_t* o) { st(o, fp_sub(ld(a), ld(b))); }
void hc_fp_half(const uint8_t* a, uint8_t* o) { st(o, fp_half(ld(a))); }
void hc_fp_inv(const uint8_t* a, uint8_t* o) { st(o, fp_inv(ld(a))); }
void hc_fp_inv_xgcd(const uint8_t* a, uint8_t* o) { st(o, fp_inv_xgcd(ld(a))); }
uint64_t hc_inv_fallbacks() { return g_inv_fallbacks; }
int hc_fp_sqrt(const uint8_t* a, uint8_t* o) {
  fp_t r;
  const bool ok = fp_sqrt(r, ld(a));
  st(o, r);
  return ok;
}
int hc_fp_legendre(const uint8_t* a) { return fp_legendre(ld(a)); }
// raw Montgomery multiply on plain limbs (checks fp_mul's bound handling directly)
void hc_fp_mont_mul_raw(const uint8_t* a, const uint8_t* b, uint8_t* o) {
  fp_plain_to_be48(o, fp_mul(fp_plain_from_be48(a), fp_plain_from_be48(b)));
}

void hc_fp2_mul(const uint8_t* a, const uint8_t* b, uint8_t* o) { st2(o, fp2_mul(ld2(a), ld2(b))); }
void hc_fp2_sqr(const uint8_t* a, uint8_t* o) { st2(o, fp2_sqr(ld2(a))); }
void hc_fp2_inv(const uint8_t* a, uint8_t* o) { st2(o, fp2_inv(ld2(a))); }
int hc_fp2_sqrt_select(const uint8_t* a, uint8_t* o) {
  fp2_t r;
  if (!fp2_sqrt(r, ld2(a))) return 0;
  st2(o, g2_select_root(r));
  return 1;
}

// lazy-operand stress: raw (Montgomery-domain) limbs in, operands are the lazy
// sums X+Y and Z+U (each summand < 2^384 as given); returns raw weakly-reduced limbs
static fp2_t ldraw2(const uint8_t* p) { fp2_t r; r.c0 = fp_plain_from_be48(p); r.c1 = fp_plain_from_be48(p + 48); return r; }
static void straw2(uint8_t* p, const fp2_t& a) { fp_plain_to_be48(p, a.c0); fp_plain_to_be48(p + 48, a.c1); }
void hc_fp2_mul_lazy_raw(const uint8_t* x, const uint8_t* y, const uint8_t* z, const uint8_t* u, uint8_t* o) {
  straw2(o, fp2_mul(fp2_add_lazy(ldraw2(x), ldraw2(y)), fp2_add_lazy(ldraw2(z), ldraw2(u))));
}

// Karabina compressed squaring (lazy reduction, bls381_lazy.hpp) on raw Montgomery-domain
// limbs: in/out = (g2, g3, g4, g5) as 4 x 96 bytes, inputs any values < 2q
void hc_cyc_csqr_raw(const uint8_t* in, uint8_t* out) {
  cyc_bc<fp2_t> g;
  g.g2 = ldraw2(in); g.g3 = ldraw2(in + 96); g.g4 = ldraw2(in + 192); g.g5 = ldraw2(in + 288);
  const cyc_bc<fp2_t> r = cyc_csqr(g);
  straw2(out, r.g2); straw2(out + 96, r.g3); straw2(out + 192, r.g4); straw2(out + 288, r.g5);
}

void hc_fp12_mul(const uint8_t* a, const uint8_t* b, uint8_t* o) { st12(o, fp12_mul(ld12(a), ld12(b))); }
void hc_fp12_sqr(const uint8_t* a, uint8_t* o) { st12(o, fp12_sqr(ld12(a))); }
void hc_fp12_inv(const uint8_t* a, uint8_t* o) { st12(o, fp12_inv(ld12(a))); }
void hc_fp12_frob(const uint8_t* a, int p, uint8_t* o) { st12(o, fp12_frob(ld12(a), p)); }
void hc_fp12_cyc_sqr(const uint8_t* a, uint8_t* o) { st12(o, fp12_cyclotomic_sqr(ld12(a))); }
void hc_fp12_mul_by_line(const uint8_t* f, const uint8_t* c0, const uint8_t* c1, const uint8_t* c2, uint8_t* o) {
  st12(o, fp12_mul_by_line(ld12(f), ld2(c0), ld2(c1), ld2(c2)));
}
void hc_final_exp(const uint8_t* a, uint8_t* o) { st12(o, final_exp(ld12(a))); }
// the verdict form (final_exp_check): 1 / 0, or 2 with fb = 0 when a snapshot had g2 = 0
int hc_final_exp_check(const uint8_t* a, int fb) {
  return fb ? final_exp_check<fp2_t, 1>(ld12(a)) : final_exp_check<fp2_t, 0>(ld12(a));
}

// lax != 0: py_ecc 1.7.0's codec, else the spec's strict one
int hc_g1_decompress(const uint8_t* b48, uint8_t* aff96, int lax) {
  aff_t<fp_t> a;
  const int s = g1_decompress(a, b48, lax != 0);
  if (s == PT_OK) { st(aff96, a.x); st(aff96 + 48, a.y); }
  return s;
}
int hc_g2_decompress(const uint8_t* b96, uint8_t* aff192, int lax) {
  aff_t<fp2_t> a;
  const int s = g2_decompress(a, b96, lax != 0);
  if (s == PT_OK) { st2(aff192, a.x); st2(aff192 + 96, a.y); }
  return s;
}
void hc_g1_compress_aff(const uint8_t* aff96, uint8_t* b48) { g1_compress(b48, jac_from_aff(ldg1(aff96))); }
void hc_g2_compress_aff(const uint8_t* aff192, uint8_t* b96) { g2_compress_aff(b96, ldg2(aff192)); }
int hc_g1_in_subgroup(const uint8_t* aff96) { return g1_in_subgroup(ldg1(aff96)); }
int hc_g2_in_subgroup(const uint8_t* aff192) { return g2_in_subgroup(ldg2(aff192)); }

int hc_hash_to_g2(const uint8_t* msg, uint32_t mlen, const uint8_t* dom8, uint8_t* aff192, uint8_t* comp96) {
  aff_t<fp2_t> c;
  const int trials = hash_to_g2_candidate(c, msg, mlen, dom8);
  aff_t<fp2_t> h;
  if (!jac_to_aff(h, g2_mul_cofactor(c))) return -2;
  st2(aff192, h.x); st2(aff192 + 96, h.y);
  g2_compress_aff(comp96, h);
  return trials;
}
void hc_sha256(const uint8_t* msg, uint32_t len, uint8_t* out32) {
  uint32_t d[8];
  sha256(d, msg, len);
  for (int i = 0; i < 8; ++i) {
    out32[4 * i] = (uint8_t)(d[i] >> 24); out32[4 * i + 1] = (uint8_t)(d[i] >> 16);
    out32[4 * i + 2] = (uint8_t)(d[i] >> 8); out32[4 * i + 3] = (uint8_t)d[i];
  }
}

// Miller loop of n <= 4 pairs (G2 affine 192 B each, G1 affine 96 B each)
int hc_miller_loop(int n, const uint8_t* q192, const uint8_t* p96, uint8_t* o576) {
  aff_t<fp2_t> Q[4];
  g1_line_pre P[4];
  if (n < 1 || n > 4) return -1;
  for (int k = 0; k < n; ++k) { Q[k] = ldg2(q192 + 192 * k); P[k] = g1_prepare(ldg1(p96 + 96 * k)); }
  fp12_t f;
  bool degen = false;
  switch (n) {
    case 1: f = miller_loop_n<1>(Q, P, degen); break;
    case 2: f = miller_loop_n<2>(Q, P, degen); break;
    case 3: f = miller_loop_n<3>(Q, P, degen); break;
    default: f = miller_loop_n<4>(Q, P, degen); break;
  }
  st12(o576, f);
  return degen ? 1 : 0;
}

// ---- whole-call semantics of the gfx950 pipelines, same headers, one thread
// (bls381_capi.hip run_verify_batch / run_vm_batch): decode, the subgroup
// policy (strict != 0: BLS381_POLICY_STRICT, the spec's codec and subgroup checks; else
// py_ecc 1.7.0's lax codec and no subgroup check), py_ecc's infinity short circuit
// (a pair with an infinite point is 1), a degenerate Miller loop -> False,
// one final exponentiation.  Returns 1 / 0.
static bool g1_in(const aff_t<fp_t>& a) { return g1_in_subgroup(a); }
static bool g2_in(const aff_t<fp2_t>& a) { return g2_in_subgroup(a); }

static int verify_pairs(int np, const aff_t<fp2_t>* Q, const aff_t<fp_t>* Pa) {
  // pairs one Miller loop each (products of f), as k_miller_pairs_batch
  fp12_t f = fp12_one<fp2_t>();
  for (int k = 0; k < np; ++k) {
    bool degen = false;
    g1_line_pre P = g1_prepare(Pa[k]);
    f = fp12_mul(f, miller_loop_n<1>(&Q[k], &P, degen));
    if (degen) return 0;
  }
  return fp12_is_one(final_exp(f)) ? 1 : 0;
}

int hc_verify(const uint8_t* pk48, const uint8_t* msg, uint32_t mlen, const uint8_t* sig96, const uint8_t* dom8,
              int strict) {
  aff_t<fp_t> P;
  aff_t<fp2_t> S;
  const int sp = g1_decompress(P, pk48, !strict);
  const int ss = g2_decompress(S, sig96, !strict);
  if (sp == PT_BAD || ss == PT_BAD) return 0;
  if (strict && ((sp == PT_OK && !g1_in(P)) || (ss == PT_OK && !g2_in(S)))) return 0;
  aff_t<fp2_t> Q[2];
  aff_t<fp_t> Pa[2];
  int np = 0;
  if (ss == PT_OK) {
    Q[np] = S;
    Pa[np].x = G1_VGEN_X_M;   // -[3(x^2-1)] g1, paired with the signature (k_hash_g2)
    Pa[np].y = G1_VGEN_NEGY_M;
    ++np;
  }
  if (sp == PT_OK) {
    aff_t<fp2_t> c;
    hash_to_g2_candidate(c, msg, mlen, dom8);
    if (jac_to_aff(Q[np], g2_mul_bp(c))) { Pa[np] = P; ++np; }
  }
  return verify_pairs(np, Q, Pa);
}

// n pubkeys / messages (mlen bytes each); pubkeys grouped by distinct message
int hc_verify_multiple(size_t n, const uint8_t* pks, const uint8_t* msgs, uint32_t mlen, const uint8_t* sig96,
                       const uint8_t* dom8, int strict) {
  std::map<std::string, jac_t<fp_t>> groups;
  for (size_t i = 0; i < n; ++i) {
    const std::string key((const char*)msgs + mlen * i, mlen);
    auto it = groups.find(key);
    if (it == groups.end()) it = groups.emplace(key, jac_infinity<fp_t>()).first;
    aff_t<fp_t> a;
    const int s = g1_decompress(a, pks + 48 * i, !strict);
    if (s == PT_BAD || (s == PT_OK && strict && !g1_in(a))) return 0;
    if (s == PT_OK) it->second = jac_add_aff(it->second, a);
  }
  aff_t<fp2_t> S;
  const int ss = g2_decompress(S, sig96, !strict);
  if (ss == PT_BAD || (ss == PT_OK && strict && !g2_in(S))) return 0;
  std::vector<aff_t<fp2_t>> Q;
  std::vector<aff_t<fp_t>> Pa;
  for (auto& g : groups) {
    aff_t<fp_t> a;
    if (!jac_to_aff(a, g.second)) continue;
    aff_t<fp2_t> c, h;
    hash_to_g2_candidate(c, (const uint8_t*)g.first.data(), mlen, dom8);
    if (!jac_to_aff(h, g2_mul_bp(c))) continue;
    Q.push_back(h);
    Pa.push_back(a);
  }
  if (ss == PT_OK) {
    aff_t<fp_t> ng;
    ng.x = G1_VGEN_X_M;
    ng.y = G1_VGEN_NEGY_M;
    Q.push_back(S);
    Pa.push_back(ng);
  }
  return verify_pairs((int)Q.size(), Q.data(), Pa.data());
}

// n independent bls_verify calls (32-byte messages) on `threads` host threads:
// the C++ CPU baseline line of bench.py (same arithmetic headers, g++ -O2)
int hc_verify_batch_mt(size_t n, const uint8_t* pks, const uint8_t* msgs32, const uint8_t* sigs, const uint8_t* dom8s,
                       int strict, int threads, uint8_t* verdicts) {
  if (threads < 1) threads = 1;
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t)
    pool.emplace_back([=] {
      for (size_t i = (size_t)t; i < n; i += (size_t)threads)
        verdicts[i] = (uint8_t)hc_verify(pks + 48 * i, msgs32 + 32 * i, 32, sigs + 96 * i, dom8s + 8 * i, strict);
    });
  for (auto& th : pool) th.join();
  return 0;
}

// G1 / G2 scalar multiplication with the same curve code (fixture helpers)
static scalar_t hc_scalar(const uint32_t* k_limbs, int nbits) {
  scalar_t k{};
  for (int i = 0; i < (nbits + 31) / 32 && i < 16; ++i) k.w[i] = k_limbs[i];
  return k;
}
void hc_g1_mul(const uint8_t* aff96, const uint32_t* k_limbs, int nbits, uint8_t* b48) {
  g1_compress(b48, jac_mul_limbs(ldg1(aff96), hc_scalar(k_limbs, nbits), nbits));
}
void hc_g2_mul(const uint8_t* aff192, const uint32_t* k_limbs, int nbits, uint8_t* b96) {
  g2_compress(b96, jac_mul_limbs(ldg2(aff192), hc_scalar(k_limbs, nbits), nbits));
}

// SSZ root program (bls381_ssz.hpp) over one serialized item: 1 ok, 0 malformed program
int hc_ssz_root(const uint8_t* item, const uint32_t* prog, uint32_t plen, uint8_t* out32) {
  static uint32_t stk[SSZ_STACK][8];
  uint32_t r[8];
  if (!ssz_run(r, item, prog, plen, stk)) return 0;
  for (int w = 0; w < 8; ++w)
    for (int b = 0; b < 4; ++b) out32[4 * w + b] = (uint8_t)(r[w] >> (24 - 8 * b));
  return 1;
}

#if defined(BLS_COUNT_OPS)
// Per-stage MAC counts (BLS_COUNT_MACS: partial products of the Fp products, 392 per
// fp_mul) of one bls_verify exactly as the gfx950
// kernels of bls381_capi.hip stage it (decode_g1 [+ subgroup check when strict],
// decode_g2 [+ subgroup check], hash_to_g2, miller_loop_2, final_exp).  out[5]
// receives the counts.
int hc_count_verify_stages(const uint8_t* pk48, const uint8_t* msg32, const uint8_t* sig96, const uint8_t* dom8,
                           int strict, uint64_t* out) {
  aff_t<fp_t> P;
  aff_t<fp2_t> S, H;
  g_fp_macs = 0;
  int sp = g1_decompress(P, pk48, !strict);
  if (strict && sp == PT_OK && !g1_in_subgroup(P)) sp = PT_BAD;
  out[0] = g_fp_macs;
  g_fp_macs = 0;
  int ss = g2_decompress(S, sig96, !strict);
  if (strict && ss == PT_OK && !g2_in_subgroup(S)) ss = PT_BAD;
  out[1] = g_fp_macs;
  g_fp_macs = 0;
  aff_t<fp2_t> c;
  hash_to_g2_candidate(c, msg32, 32, dom8);
  jac_to_aff(H, g2_mul_bp(c));
  out[2] = g_fp_macs;
  if (sp != PT_OK || ss != PT_OK) { out[3] = out[4] = 0; return -1; }
  g_fp_macs = 0;
  aff_t<fp2_t> Q[2] = {S, H};
  aff_t<fp_t> ng; ng.x = G1_VGEN_X_M; ng.y = G1_VGEN_NEGY_M;
  g1_line_pre Pp[2] = {g1_prepare(ng), g1_prepare(P)};
  bool degen = false;
  const fp12_t f = miller_loop_n<2>(Q, Pp, degen);
  out[3] = g_fp_macs;
  g_fp_macs = 0;
  const bool ok = final_exp_check<fp2_t, 1>(f) == 1;   // the kernel's verdict form (one product fewer)
  out[4] = g_fp_macs;
  // the split Miller loop of the throughput path, per kernel (bls381_kernels.hpp):
  // out[5] k_ml_lines (both running points, L = l l'), out[6] k_ml_accum (f^2 L)
  uint64_t lines = 0, accum = 0;
  g2_proj<fp2_t> T[2];
  for (int k = 0; k < 2; ++k) { T[k].x = Q[k].x; T[k].y = Q[k].y; T[k].z = fp2_one(); }
  fp12_t g;
  int step = 0;
  auto run_step = [&](bool add) {
    fp2_t c[3], d[3];
    g_fp_macs = 0;
    if (add) { line_add(T[0], Q[0], Pp[0], c[0], c[1], c[2]); line_add(T[1], Q[1], Pp[1], d[0], d[1], d[2]); }
    else { line_dbl(T[0], Pp[0], c[0], c[1], c[2]); line_dbl(T[1], Pp[1], d[0], d[1], d[2]); }
    const fp12_t L = line_pair_product(c[0], c[1], c[2], d[0], d[1], d[2]);
    lines += g_fp_macs;
    g_fp_macs = 0;
    if (step == 0) g = L;
    else if (add || step == 1) g = fp12_mul_by_line_pair_inl(g, L);
    else g = fp12_mul_by_line_pair_inl(fp12_sqr_inl(g), L);
    accum += g_fp_macs;
    ++step;
  };
  for (int b = 62; b >= 0; --b) {
    run_step(false);
    if ((BLS_X_ABS >> b) & 1) run_step(true);
  }
  out[5] = lines;
  out[6] = accum;
  return ok ? 1 : 0;
}

// MACs of the randomized path's per-item and per-sub-batch stages (bench.py rb roofline):
// out[0] [r] pk = sigma(pk) + the joint 32-bit ladder + affine (k_rb_decode_g1's scalar part),
// out[1] the signature's G2 test (k_rb_g2_test), out[2] one mixed G2 addition (the MSM's unit:
// ~15 per item at 4-bit windows), out[3] the joint 32-bit G2 ladder [r] sig (k_rb_scale_g2, the
// path above the MSM's sub-batch cap), out[4] one Miller pair (S, -[c] g1) (k_rb_miller_sig).
int hc_count_rb_item(const uint8_t* pk48, const uint8_t* sig96, uint32_t k0, uint32_t k1, uint64_t* out) {
  aff_t<fp_t> P;
  aff_t<fp2_t> S;
  if (g1_decompress(P, pk48, true) != PT_OK || g2_decompress(S, sig96, true) != PT_OK) return -1;
  g_fp_macs = 0;
  aff_t<fp_t> sp;
  sp.x = fp_mul(G1_BETA_M, P.x);
  sp.y = P.y;
  aff_t<fp_t> r1;
  jac_to_aff(r1, jac_mul_2x32(P, sp, k0, k1));
  out[0] = g_fp_macs;
  g_fp_macs = 0;
  (void)g2_in_subgroup(S);
  out[1] = g_fp_macs;
  g_fp_macs = 0;
  const jac_t<fp2_t> j = jac_mul_2x32(S, g2_psi(S), 3u, 5u);   // a generic Jacobian point
  g_fp_macs = 0;
  (void)jac_add_aff(j, S);
  out[2] = g_fp_macs;
  aff_t<fp2_t> sq = g2_psi(g2_psi(S));
  sq.y = fp2_neg(sq.y);
  g_fp_macs = 0;
  (void)jac_mul_2x32(S, sq, k0, k1);
  out[3] = g_fp_macs;
  aff_t<fp_t> ng; ng.x = G1_VGEN_X_M; ng.y = G1_VGEN_NEGY_M;
  const g1_line_pre pre = g1_prepare(ng);
  bool degen = false;
  g_fp_macs = 0;
  (void)miller_loop_n<1>(&S, &pre, degen);
  out[4] = g_fp_macs;
  return 0;
}

// MACs (BLS_COUNT_MACS) of one committee aggregation of n pubkeys (decode + adds)
int hc_count_aggregate(size_t n, const uint8_t* pks, uint64_t* out) {
  g_fp_macs = 0;
  jac_t<fp_t> acc = jac_infinity<fp_t>();
  for (size_t i = 0; i < n; ++i) {
    aff_t<fp_t> a;
    const int s = g1_decompress(a, pks + 48 * i, true);
    if (s == PT_BAD) return -1;
    if (s == PT_OK) acc = jac_add_aff(acc, a);
  }
  uint8_t b[48];
  g1_compress(b, acc);
  *out = g_fp_macs;
  return 0;
}
#endif

}  // extern "C"
