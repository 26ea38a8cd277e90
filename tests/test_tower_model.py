"""oracle/tower_model.py (our device algorithms) vs oracle/bls_oracle.py (reference)."""
import random

import bls_oracle as O
import tower_model as M

q = O.q


def _r2(rng):
    return (rng.randrange(q), rng.randrange(q))


def test_tower_is_isomorphic_to_pyecc_fq12():
    rng = random.Random(1)
    f = tuple(_r2(rng) for _ in range(6))
    g = tuple(_r2(rng) for _ in range(6))
    assert M.to_pyecc12(M.mul12(f, g)) == O.f12_mul(M.to_pyecc12(f), M.to_pyecc12(g))
    assert M.to_pyecc12(M.frob12(f, 1)) == O.f12_pow(M.to_pyecc12(f), q)
    assert M.mul12(M.inv12(f), f) == M.ONE12


def test_cyclotomic_square_and_final_exp_chain():
    rng = random.Random(2)
    f = tuple(_r2(rng) for _ in range(6))
    t = M.mul12(M.conj12(f), M.inv12(f))
    t = M.mul12(M.frob12(t, 2), t)
    assert M.cyclotomic_sqr(t) == M.mul12(t, t)
    assert M.to_pyecc12(M.final_exp(f)) == O.f12_pow(M.to_pyecc12(f), 3 * (q ** 12 - 1) // O.r)


def test_karabina_compressed_exponentiation():
    """Compressed squarings of (g2..g5) track Granger-Scott squarings exactly, the
    decompression recovers the full element, and f^|x| right to left equals the
    square-and-multiply chain (bls381_pairing.hpp cyc_exp_x)."""
    rng = random.Random(3)
    f = tuple(_r2(rng) for _ in range(6))
    t = M.mul12(M.conj12(f), M.inv12(f))
    t = M.mul12(M.frob12(t, 2), t)
    x, g = t, M.cyc_compress(t)
    for _ in range(4):
        x, g = M.cyclotomic_sqr(x), M.cyc_csqr(g)
        assert M.cyc_compress(x) == g and M.cyc_decompress(g) == x
    assert M.cyc_exp_abs_x_compressed(t) == M.cyc_exp_abs_x(t)


def test_pairing_bilinear_and_relation_to_oracle():
    rng = random.Random(3)
    g1 = (O.g_x, O.g_y)
    g2 = (O.G2_gen_x, O.G2_gen_y)
    e = M.pairing(g2, g1)
    a, b = rng.randrange(O.r), rng.randrange(O.r)
    aP = O.pt_normalize(O.FqOps, O.pt_multiply(O.FqOps, O.G1, a))
    bQ = O.pt_normalize(O.Fq2Ops, O.pt_multiply(O.Fq2Ops, O.G2, b))
    assert M.pairing(bQ, aP) == M.pow12(e, a * b % O.r)
    # ours = oracle^-3 (conjugation for x < 0, factor 3 in the hard part)
    assert M.to_pyecc12(e) == O.f12_pow(O.pairing(O.G2, O.G1), (-3) % O.r)


def test_cofactor_clearing_identity():
    """[h2]P == [e0]S - T (device hash_to_G2 cofactor) on points outside G2; and the
    Budroni-Pintore combination equals [3(x^2-1) h2]P."""
    F = M.Fq2
    for s in range(3):
        x, y = M.map_candidate(bytes([s]) * 32, b"\x07" * 8)
        P = (x, y, M.ONE2)
        want = M.jac_to_affine(F, M.jac_mul(F, P, O.G2_cofactor))
        assert M.jac_to_affine(F, M.clear_cofactor_h2(P)) == want
    k = pow(3 * (O.BLS_X ** 2 - 1), -1, O.r)
    e0 = (M.X_ABS + 1) // 3
    assert k == e0 + (2 * e0 - 1) * M.X_ABS + (2 * e0 - 2) * M.X_ABS ** 2 + (e0 - 1) * M.X_ABS ** 3


def _header_fp(name):
    """A Montgomery-form fp_t constant of bls381_consts.hpp as an integer."""
    import os
    import re
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        "consensus-specs_amd", "csrc", "bls381_consts.hpp")
    m = re.search(r"fp_t %s = \{\{([^}]*)\}\}" % name, open(path).read())
    limbs = [int(w.strip().rstrip("u"), 16) for w in m.group(1).split(",")]
    v = sum(l << (28 * i) for i, l in enumerate(limbs))
    return v * pow(2, -392, q) % q


def test_verification_hash_scaling():
    """The verify kernels pair BP(H0) = [c h2]H0 with the pubkey and the signature with
    -[c]g1 (G1_VGEN_*), c = 3(x^2-1): the pairing product is the original one to the
    power c, coprime to r, so the verdict is unchanged (bls381_hash.hpp g2_mul_bp)."""
    F = M.Fq2
    c = 3 * (M.X_ABS ** 2 - 1)
    assert c % O.r and O.r % 3
    cg = O.pt_normalize(O.FqOps, O.pt_multiply(O.FqOps, O.G1, c % O.r))
    assert _header_fp("G1_VGEN_X_M") == cg[0] and _header_fp("G1_VGEN_NEGY_M") == (-cg[1]) % q
    ncg = (cg[0], (-cg[1]) % q)
    sk, msg, dom8 = 0x1234567, b"\x5a" * 32, (3).to_bytes(8, "big")
    x, y = M.map_candidate(msg, dom8)
    H0 = (x, y, M.ONE2)
    bp = M.jac_to_affine(F, M.g2_bp(H0))
    assert bp == M.jac_to_affine(F, M.jac_mul(F, M.clear_cofactor_h2(H0), c))
    H = M.jac_to_affine(F, M.clear_cofactor_h2(H0))
    pk = O.pt_normalize(O.FqOps, O.pt_multiply(O.FqOps, O.G1, sk))
    sig = O.pt_normalize(O.Fq2Ops, O.pt_multiply(O.Fq2Ops, (H[0], H[1], M.ONE2), sk))
    f_scaled = M.final_exp(M.miller_loop_multi([(sig, ncg), (bp, pk)]))
    assert f_scaled == M.ONE12
    pk2 = O.pt_normalize(O.FqOps, O.pt_multiply(O.FqOps, O.G1, sk + 1))
    ng = (O.g_x, (-O.g_y) % q)
    f_plain = M.final_exp(M.miller_loop_multi([(sig, ng), (H, pk2)]))
    assert M.final_exp(M.miller_loop_multi([(sig, ncg), (bp, pk2)])) == M.pow12(f_plain, c % O.r) != M.ONE12


def test_hash_sqrt_subgroup_models():
    rng = random.Random(4)
    for i in range(60):
        v = _r2(rng) if i % 4 else (rng.randrange(q), 0)
        a, b = O.modular_squareroot(v), M.sqrt_fp2(v)
        assert (a is None) == (b is None)
        if a is not None:
            assert M.choose_root(b) == a
    msg, dom = bytes(range(32)), 77
    H = M.hash_to_g2_affine(msg, dom.to_bytes(8, "big"))
    assert H == O.g2_affine(O.hash_to_G2(msg, dom))
    assert M.g2_in_subgroup((H[0], H[1], M.ONE2))
    x, y = M.map_candidate(msg, b"abcdefgh")
    assert not M.g2_in_subgroup((x, y, M.ONE2))
    pk = O.pt_normalize(O.FqOps, O.pubkey_to_G1(O.privtopub(99)))
    assert M.g1_in_subgroup((pk[0], pk[1], 1))
    s = M.sqrt_fp((5 ** 3 + 4) % q)
    assert not M.g1_in_subgroup((5, s, 1))
