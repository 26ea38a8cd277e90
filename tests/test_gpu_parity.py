"""GPU parity: the gfx950 engine (through the C ABI) vs the oracle.

Bit-exact for every byte output; identical verdicts.  Fixtures were produced
by tests/golden/make_vectors.py from oracle/bls_oracle.py (py_ecc 1.7.0
restatement).  Larger sizes are covered by size-independent properties
(sign -> verify round trips, tamper -> False, aggregation linearity).
"""
import os
import random
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import bls_oracle as O  # noqa: E402


def _dom(c):
    return int(c["input"]["domain"], 16)


def _hex(s):
    return bytes.fromhex(s[2:] if s.startswith("0x") else s)


# ---------------------------------------------------------------- C1 vectors
def test_priv_to_pub_vectors(native, golden):
    from bls381_amd import bls
    vec, _ = golden
    for c in vec["priv_to_pub"]:
        assert bls.privtopub(int(c["input"], 16)) == _hex(c["output"])


def test_msg_hash_compressed_vectors(native, golden):
    from bls381_amd import bls
    vec, _ = golden
    for c in vec["msg_hash_g2_compressed"]:
        out = bls.hash_to_G2_compressed(_hex(c["input"]["message"]), _dom(c))
        assert out == _hex(c["output"][0]) + _hex(c["output"][1])


def test_msg_hash_uncompressed_vectors_pyecc_projective(native, golden):
    from bls381_amd import bls
    vec, _ = golden
    for c in vec["msg_hash_g2_uncompressed"]:
        X, Y, Z = bls.hash_to_G2_pyecc_projective(_hex(c["input"]["message"]), _dom(c))
        want = [[int(a, 16), int(b, 16)] for a, b in c["output"]]
        assert [list(X), list(Y), list(Z)] == want


def test_sign_vectors(native, golden):
    from bls381_amd import bls
    vec, _ = golden
    for c in vec["sign_msg"]:
        i = c["input"]
        sig = bls.bls_sign(_hex(i["message"]), int(i["privkey"], 16), int(i["domain"], 16))
        assert sig == _hex(c["output"])


def test_aggregate_vectors(native, golden):
    from bls381_amd import bls
    vec, _ = golden
    for c in vec["aggregate_sigs"]:
        assert bls.bls_aggregate_signatures([_hex(s) for s in c["input"]]) == _hex(c["output"])
    for c in vec["aggregate_pubkeys"]:
        assert bls.bls_aggregate_pubkeys([_hex(s) for s in c["input"]]) == _hex(c["output"])


# ------------------------------------------------------------ golden batches
def test_golden_verify_single_and_batch(native, golden):
    from bls381_amd import bls
    _, gb = golden
    items = gb["verify"]
    for it in items:
        got = bls.bls_verify(bytes.fromhex(it["pubkey"]), bytes.fromhex(it["message"]),
                             bytes.fromhex(it["signature"]), int(it["domain"]))
        assert got == it["expected"], it["kind"]
    pks = b"".join(bytes.fromhex(it["pubkey"]) for it in items)
    msgs = b"".join(bytes.fromhex(it["message"]) for it in items)
    sigs = b"".join(bytes.fromhex(it["signature"]) for it in items)
    doms = b"".join(int(it["domain"]).to_bytes(8, "big") for it in items)
    v = native.verify_batch(pks, msgs, sigs, doms)
    assert list(v) == [it["expected"] for it in items]


def test_golden_verify_multiple(native, golden):
    from bls381_amd import bls
    _, gb = golden
    for it in gb["verify_multiple"]:
        got = bls.bls_verify_multiple([bytes.fromhex(p) for p in it["pubkeys"]],
                                      [bytes.fromhex(m) for m in it["messages"]],
                                      bytes.fromhex(it["signature"]), int(it["domain"]))
        assert got == it["expected"], it["kind"]


def test_golden_aggregates(native, golden):
    from bls381_amd import bls
    _, gb = golden
    for it in gb["aggregate_pubkeys"]:
        assert bls.bls_aggregate_pubkeys([bytes.fromhex(p) for p in it["input"]]).hex() == it["output"], it["kind"]
    for it in gb["aggregate_sigs"]:
        assert bls.bls_aggregate_signatures([bytes.fromhex(s) for s in it["input"]]).hex() == it["output"], it["kind"]


def test_survey_abi_names(native, golden):
    """SURVEY §8(b)'s names: bls381_init_devices(n) and bls381_aggregate_g1/_g2 behave as
    bls381_init / bls381_aggregate_pubkeys / _signatures."""
    import ctypes
    L = native.lib()
    assert L.bls381_init_devices(1) == 0
    assert L.bls381_init_devices(0) != 0
    _, gb = golden
    for it in gb["aggregate_pubkeys"]:
        pks = b"".join(bytes.fromhex(p) for p in it["input"])
        out = ctypes.create_string_buffer(48)
        assert L.bls381_aggregate_g1(len(it["input"]), pks, out) == 0
        assert out.raw.hex() == it["output"], it["kind"]
    for it in gb["aggregate_sigs"]:
        sigs = b"".join(bytes.fromhex(p) for p in it["input"])
        out = ctypes.create_string_buffer(96)
        assert L.bls381_aggregate_g2(len(it["input"]), sigs, out) == 0
        assert out.raw.hex() == it["output"], it["kind"]


def test_golden_hash_to_g2(native, golden):
    from bls381_amd import bls
    _, gb = golden
    for it in gb["hash_to_g2"]:
        m, d = bytes.fromhex(it["message"]), int(it["domain"])
        assert bls.hash_to_G2_compressed(m, d).hex() == it["compressed"]
        (xr, xi), (yr, yi) = bls.hash_to_G2_affine(m, d)
        assert [hex(xr), hex(xi), hex(yr), hex(yi)] == it["affine"]


@pytest.mark.parametrize("policy", ["pyecc", "strict"])
def test_invalid_encodings_raise_in_aggregate(native, golden, policy):
    """Encodings neither codec can decode (no square root) raise under both policies."""
    from bls381_amd import bls
    _, gb = golden
    old = bls.SUBGROUP_POLICY
    bls.SUBGROUP_POLICY = policy
    try:
        for h in gb["invalid_g1"]:
            with pytest.raises(ValueError):
                bls.bls_aggregate_pubkeys([bytes.fromhex(h)])
        for h in gb["invalid_g2"]:
            with pytest.raises(ValueError):
                bls.bls_aggregate_signatures([bytes.fromhex(h)])
    finally:
        bls.SUBGROUP_POLICY = old


def _codec_variant_cases():
    """(pk, msg, sig) triples from valid signatures with their encodings mutated: flags cleared
    or flipped, x + q (and G2's real part + q, which sets z2's flag bits), infinity with and
    without junk, a changed x.  Expected verdict per policy from the oracle's decoders: True iff
    both inputs decode to the signed points, or both to infinity (py_ecc's pairing with an
    infinite point is 1) -- a different point fails the pairing check.  A subset is re-checked
    with the oracle's full verify in the test."""
    Q = O.q
    cases = []
    for sk in (7, 0x1234567, 0x2f3e4d5c6b7a8990a1b2c3d4e5f60718293a4b5c6d7e8f9):
        msg = bytes([sk % 251]) * 32
        pk, sig = O.privtopub(sk), O.sign(msg, sk, 3)
        z = int.from_bytes(pk, "big")
        x, fl = z & ((1 << 381) - 1), z >> 381
        pks = [z, z & ~(1 << 383), z ^ (1 << 381), (fl << 381) | (x ^ 1), x,
               (1 << 383) | (1 << 382), (1 << 383) | (1 << 382) | 12345, (1 << 382) | x]
        if x + Q < (1 << 381):
            pks += [(fl << 381) | (x + Q), ((fl & 3) << 381) | (x + Q)]
        z1, z2 = int.from_bytes(sig[:48], "big"), int.from_bytes(sig[48:], "big")
        x1, f1 = z1 & ((1 << 381) - 1), z1 >> 381
        sigs = [(z1, z2), (z1 & ~(1 << 383), z2), (z1 ^ (1 << 381), z2), (z1, z2 + Q), (z1, z2 | (1 << 383)),
                ((1 << 383) | (1 << 382), 0), ((1 << 383) | (1 << 382) | 99, 7), (z1, z2 ^ 1)]
        if x1 + Q < (1 << 381):
            sigs += [((f1 << 381) | (x1 + Q), z2), (((f1 & 3) << 381) | (x1 + Q), z2)]
        enc_pk = lambda v: v.to_bytes(48, "big")
        enc_sig = lambda t: t[0].to_bytes(48, "big") + t[1].to_bytes(48, "big")
        combos = [(p, sigs[0]) for p in pks] + [(pks[0], t) for t in sigs[1:]]
        combos += [(p, t) for p in pks[5:7] for t in sigs[5:7]]     # both at infinity
        P0, S0 = O.pubkey_to_G1(pk), O.signature_to_G2(sig)
        for p, t in combos:
            want = {}
            for pol in ("pyecc", "strict"):
                try:
                    P = O.decompress_G1(p, pol == "strict")
                    S = O.decompress_G2(t, pol == "strict")
                    both_inf = O.pt_is_inf(O._FqOps, P) and O.pt_is_inf(O._Fq2Ops, S)
                    want[pol] = both_inf or (O.pt_eq(O._FqOps, P, P0) and O.pt_eq(O._Fq2Ops, S, S0))
                except ValueError:
                    want[pol] = False
            cases.append((enc_pk(p), msg, enc_sig(t), want))
    return cases


@pytest.mark.parametrize("n", [64, 20000, (1 << 16) + 3])
def test_verify_codec_variants_both_policies(native, n):
    """bls_verify over mutated encodings of valid signatures (_codec_variant_cases), tiled to n
    items so the quad, pair and split-loop layouts all see them, under both policies; a subset
    against the oracle's full verify (py_ecc) and verify_strict."""
    cases = _codec_variant_cases()
    if n == 64:
        for pk, msg, sig, want in cases[::9]:
            assert O.verify(msg, pk, sig, 3) == want["pyecc"], pk.hex()
            assert O.verify_strict(msg, pk, sig, 3) == want["strict"], pk.hex()
    reps = (n + len(cases) - 1) // len(cases)
    tiled = (cases * reps)[:n]
    pks = b"".join(c[0] for c in tiled)
    msgs = b"".join(c[1] for c in tiled)
    sigs = b"".join(c[2] for c in tiled)
    doms = (3).to_bytes(8, "big") * n
    try:
        for pol in ("pyecc", "strict"):
            native.set_subgroup_policy(pol)
            got = list(native.verify_batch(pks, msgs, sigs, doms))
            assert got == [c[3][pol] for c in tiled], pol
        assert any(c[3]["pyecc"] != c[3]["strict"] for c in cases)
    finally:
        native.set_subgroup_policy("pyecc")


@pytest.mark.parametrize("policy", ["pyecc", "strict"])
def test_codec_fuzz_aggregates_both_policies(native, policy):
    """The device decoders on seeded structured encodings (tests/codec_fuzz.py: all flag
    combinations, x >= q, x = 0, junk under b_flag, G2 real parts with top bits set), each as a
    one-key aggregate: the oracle's bytes under the call's policy, or ValueError where its codec
    rejects.  G1 through one batch call (one group per key, the one-lane level-1 kernel), G2 per
    call through the shim's native entry point."""
    from codec_fuzz import g1_encodings, g2_encodings
    strict = policy == "strict"
    native.set_subgroup_policy(policy)
    try:
        keys = g1_encodings(0xC0DEC3, 1500)
        want = []
        for b in keys:
            try:
                want.append(O.aggregate_pubkeys([b], strict).hex())
            except ValueError:
                want.append(None)
        off = np.arange(len(keys) + 1, dtype=np.uint32)
        outs, st = native.aggregate_pubkeys_batch(off, b"".join(keys))
        got = [o.hex() if s == 0 else None for o, s in zip(outs, st)]
        assert got == want
        assert any(w is None for w in want) and any(w is not None for w in want)
        for b in g2_encodings(0xC0DEC4, 300):
            try:
                w = O.aggregate_signatures([b], strict).hex()
            except ValueError:
                w = None
            try:
                g = native.aggregate_signatures(b).hex()
            except ValueError:
                g = None
            assert g == w, (b.hex(), policy)
    finally:
        native.set_subgroup_policy("pyecc")


@pytest.mark.parametrize("policy", ["pyecc", "strict"])
def test_noncanonical_aggregates_both_policies(native, noncanon, policy):
    """bls_aggregate_pubkeys / _signatures over non-canonical encodings (bls_noncanonical.json):
    py_ecc 1.7.0's bytes under "pyecc" (e.g. [00 * 48] -> 0x80 || 00*47, the order-3 point),
    ValueError where the spec's codec rejects an input under "strict" -- through the shim,
    the batch entry point (one group per case), the registry and the SURVEY names."""
    import ctypes
    from bls381_amd import bls
    from bls381_amd.registry import PubkeyRegistry
    col = "output_" + policy
    h = bytes.fromhex
    old = bls.SUBGROUP_POLICY
    bls.SUBGROUP_POLICY = policy
    native.set_subgroup_policy(policy)
    reg = PubkeyRegistry(256)
    try:
        for c in noncanon["aggregate_pubkeys"]:
            keys = [h(p) for p in c["input"]]
            if c[col] is None:
                with pytest.raises(ValueError):
                    bls.bls_aggregate_pubkeys(keys)
            else:
                assert bls.bls_aggregate_pubkeys(keys).hex() == c[col], (c["kind"], policy)
        for c in noncanon["aggregate_sigs"]:
            sigs = [h(s) for s in c["input"]]
            if c[col] is None:
                with pytest.raises(ValueError):
                    bls.bls_aggregate_signatures(sigs)
            else:
                assert bls.bls_aggregate_signatures(sigs).hex() == c[col], (c["kind"], policy)
        # one batch, one group per case
        groups = [[h(p) for p in c["input"]] for c in noncanon["aggregate_pubkeys"]]
        off = np.cumsum([0] + [len(g) for g in groups]).astype(np.uint32)
        outs, st = native.aggregate_pubkeys_batch(off, b"".join(b"".join(g) for g in groups))
        for c, o, s in zip(noncanon["aggregate_pubkeys"], outs, st):
            assert (o.hex() if s == 0 else None) == c[col], (c["kind"], policy)
        # the registry decodes laxly once and serves both policies (ST_NONCANON entries)
        ent = reg.add([k for g in groups for k in g])
        for i, c in enumerate(noncanon["aggregate_pubkeys"]):
            members = [int(ent[j]) for j in range(off[i], off[i + 1])]
            if any(m < 0 for m in members):          # a key neither codec decodes is never an entry
                assert c["output_pyecc"] is None
                continue
            if c[col] is None:
                with pytest.raises(ValueError):
                    reg.aggregate_indices([members])
            else:
                assert reg.aggregate_indices([members])[0].hex() == c[col], (c["kind"], policy)
        L = native.lib()
        for c in noncanon["aggregate_sigs"]:
            sigs = b"".join(h(s) for s in c["input"])
            out = ctypes.create_string_buffer(96)
            rc = L.bls381_aggregate_g2(len(c["input"]), sigs, out)
            assert (out.raw.hex() if rc == 0 else None) == c[col], (c["kind"], policy)
    finally:
        reg.close()
        bls.SUBGROUP_POLICY = old
        native.set_subgroup_policy("pyecc")


# ----------------------------------------------------- edge cases (§4, A.5-7)
def test_empty_aggregates_and_lists(native):
    from bls381_amd import bls
    assert bls.bls_aggregate_pubkeys([]) == bytes([0xC0]) + b"\x00" * 47
    assert bls.bls_aggregate_signatures([]) == bytes([0xC0]) + b"\x00" * 95
    inf_sig = bytes([0xC0]) + b"\x00" * 95
    assert bls.bls_verify_multiple([], [], inf_sig, 0) is True
    with pytest.raises(ValueError):
        bls.bls_verify_multiple([b"\x00" * 48], [], inf_sig, 0)


def test_non32_message_length(native):
    from bls381_amd import bls
    sk = 12345
    for msg in (b"", b"abc", bytes(range(100))):
        sig = bls.bls_sign(msg, sk, 77)
        assert sig == O.sign(msg, sk, 77)
        assert bls.bls_verify(bls.privtopub(sk), msg, sig, 77) is True
        assert bls.bls_verify(bls.privtopub(sk), msg + b"x", sig, 77) is False


# ------------------------------------------ synthetic batches (seeded, C2 shape)
def _make_batch(n, seed, tamper_every=4):
    """n signed items from the engine itself (sign), a fraction tampered."""
    from bls381_amd import bls
    rng = random.Random(seed)
    pks, msgs, sigs, doms, exp = [], [], [], [], []
    for i in range(n):
        sk = rng.randrange(1, O.r)
        m = bytes(rng.getrandbits(8) for _ in range(32))
        d = rng.getrandbits(64)
        pk = bls.privtopub(sk)
        sig = bls.bls_sign(m, sk, d)
        ok = True
        if i % tamper_every == 1:
            m = bytes([m[0] ^ 1]) + m[1:]
            ok = False
        elif i % tamper_every == 2 and i > 2:
            sig = sigs[-1]
            ok = False
        pks.append(pk); msgs.append(m); sigs.append(sig); doms.append(d); exp.append(ok)
    return pks, msgs, sigs, doms, exp


def test_batch_against_oracle_small(native):
    pks, msgs, sigs, doms, exp = _make_batch(12, 0xB15_0001)
    # oracle check of the engine-made signatures and verdicts
    for pk, m, s, d, e in list(zip(pks, msgs, sigs, doms, exp))[:6]:
        assert O.verify(m, pk, s, d) == e
    v = native.verify_batch(b"".join(pks), b"".join(msgs), b"".join(sigs),
                            b"".join(d.to_bytes(8, "big") for d in doms))
    assert list(v) == exp


@pytest.mark.parametrize("policy", ["pyecc", "strict"])
@pytest.mark.parametrize("n", [100, 8193, 12000, 20000, 60000, (1 << 18) + 3])
def test_verify_layouts_tiled_special_cases(native, golden, torsion, policy, n):
    """The golden and torsion bls_verify cases (infinite keys and signatures, bad encodings,
    small-order components, a degenerate Miller loop) tiled to n items, so every Miller /
    final-exponentiation layout sees them: n <= 8192 one quad per Miller pair + the 2-value
    quad FE, n <= 49152 both pairs on one quad + the quad FE, above that lane pairs (60,000: the
    FE, the cofactor map and the Miller accumulation are one-round launches of two waves per
    SIMD, which run with the clock-based wave balance; 2^18 + 3: launches of several rounds of
    waves with a ragged last wave).  From 8,193 items on the py_ecc
    policy runs the one-launch prologue (k_prologue_1: each of its three roles ends in a ragged
    workgroup at 8,193).  The tiled verdicts equal the untiled batch's, which equal the fixtures'
    column for the policy."""
    _, gb = golden
    gcol = "expected" if policy == "pyecc" else "expected_strict"
    cases = [(c, c[gcol]) for c in gb["verify"] if len(bytes.fromhex(c["message"])) == 32]
    cases += [(c, c["expected_" + policy]) for c in torsion["verify"]]
    assert all(len(bytes.fromhex(c["message"])) == 32 for c, _ in cases)

    def run(items):
        return list(native.verify_batch(b"".join(bytes.fromhex(c["pubkey"]) for c in items),
                                        b"".join(bytes.fromhex(c["message"]) for c in items),
                                        b"".join(bytes.fromhex(c["signature"]) for c in items),
                                        b"".join(int(c["domain"]).to_bytes(8, "big") for c in items)))
    native.set_subgroup_policy(policy)
    try:
        base = run([c for c, _ in cases])
        tiled = run([cases[i % len(cases)][0] for i in range(n)])
    finally:
        native.set_subgroup_policy("pyecc")
    assert base == [e for _, e in cases]
    # strict, n > 49152: the signature's G2 test runs on the Miller loop's final point
    assert tiled == [base[i % len(cases)] for i in range(n)]


@pytest.mark.parametrize("policy", ["pyecc", "strict"])
def test_latency_batches_every_small_size(native, golden, torsion, policy):
    """The latency kernels keep whole waves active and mask the stores of lanes past the last item
    (lat_unit, bls381_kernels.hpp): batches of every size around the wave boundaries of their layouts
    (16 items per wave on quads, 8 on octets, 4 per wave for the octet Miller pairs), at rotating
    offsets into the golden + torsion verify cases, give each case's fixture verdict."""
    _, gb = golden
    gcol = "expected" if policy == "pyecc" else "expected_strict"
    cases = [(c, c[gcol]) for c in gb["verify"] if len(bytes.fromhex(c["message"])) == 32]
    cases += [(c, c["expected_" + policy]) for c in torsion["verify"]]
    native.set_subgroup_policy(policy)
    try:
        for n in (1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 31, 33):
            for off in (0, 5):
                items = [cases[(off + i) % len(cases)] for i in range(n)]
                got = list(native.verify_batch(b"".join(bytes.fromhex(c["pubkey"]) for c, _ in items),
                                               b"".join(bytes.fromhex(c["message"]) for c, _ in items),
                                               b"".join(bytes.fromhex(c["signature"]) for c, _ in items),
                                               b"".join(int(c["domain"]).to_bytes(8, "big") for c, _ in items)))
                assert got == [e for _, e in items], (n, off)
    finally:
        native.set_subgroup_policy("pyecc")


@pytest.mark.parametrize("n", [4096, 12000, 20000])
def test_batch_full_size_roundtrip(native, n):
    """Signed items (sign -> verify round trip), 1/4 tampered, at sizes that run each Miller /
    final-exponentiation layout: size-independent check."""
    from bls381_amd import bls
    rng = np.random.default_rng(7)
    # one key, many messages: signing cost stays small, verify work per item is full
    sk = 0x1234567890ABCDEF
    pk = bls.privtopub(sk)
    msgs = [bytes(rng.integers(0, 256, 32, dtype=np.uint8)) for _ in range(64)]
    sigs = [bls.bls_sign(m, sk, 3) for m in msgs]
    idx = rng.integers(0, 64, n)
    tam = (np.arange(n) % 4) == 3
    m_all = [msgs[i] for i in idx]
    s_all = [sigs[(i + 1) % 64] if t else sigs[i] for i, t in zip(idx, tam)]
    v = native.verify_batch(pk * n, b"".join(m_all), b"".join(s_all), (3).to_bytes(8, "big") * n)
    assert v.sum() == n - tam.sum()
    assert not v[tam].any()


def test_committee_aggregate_batch(native):
    """C3 shape: 128-member committees; batch aggregation == per-group oracle sum."""
    keys = [O.privtopub(k) for k in range(1, 129)]
    offsets = np.array([0, 128, 128 + 64, 128 + 64 + 1, 128 + 64 + 1], dtype=np.uint32)
    pks = b"".join(keys) + b"".join(keys[:64]) + keys[5]
    outs, st = native.aggregate_pubkeys_batch(offsets, pks)
    assert list(st) == [0, 0, 0, 0]
    assert outs[0] == O.aggregate_pubkeys(keys)
    assert outs[1] == O.aggregate_pubkeys(keys[:64])
    assert outs[2] == keys[5]
    assert outs[3] == bytes([0xC0]) + b"\x00" * 47


def test_large_aggregation_multilevel(native):
    """> CHUNK (512) keys exercises the multi-level reduction: sum_{k=1..N} [k]G = [N(N+1)/2]G."""
    n = 3000
    keys = [O.privtopub(k) for k in range(1, 41)]
    pks = b"".join(keys[i % 40] for i in range(n))
    # sum of (i % 40) + 1 for i < n
    total = sum((i % 40) + 1 for i in range(n))
    from bls381_amd import bls
    assert bls.bls_aggregate_pubkeys([pks[48 * i:48 * i + 48] for i in range(n)]) == O.privtopub(total)


def test_verify_multiple_many_messages(native):
    """C5 shape (small L): L distinct messages, aggregated signature, product tree of Miller loops."""
    from bls381_amd import bls
    rng = random.Random(0xB15_0005)
    L = 37
    sks = [rng.randrange(1, O.r) for _ in range(L)]
    msgs = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(L)]
    pks = [bls.privtopub(k) for k in sks]
    sig = bls.bls_aggregate_signatures([bls.bls_sign(m, k, 1) for m, k in zip(msgs, sks)])
    assert bls.bls_verify_multiple(pks, msgs, sig, 1) is True
    assert bls.bls_verify_multiple(pks[1:] + pks[:1], msgs, sig, 1) is False
    assert bls.bls_verify_multiple(pks, msgs, sig, 2) is False


def test_partial_products_combine(native):
    """Sharded verify_multiple: per-shard Fp12 partials combine to the single-call verdict."""
    from bls381_amd import bls
    rng = random.Random(11)
    L = 6
    sks = [rng.randrange(1, O.r) for _ in range(L)]
    msgs = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(L)]
    pks = [bls.privtopub(k) for k in sks]
    sig = bls.bls_aggregate_signatures([bls.bls_sign(m, k, 9) for m, k in zip(msgs, sks)])
    d8 = (9).to_bytes(8, "big")
    parts = []
    for r in range(3):
        sel = [i for i in range(L) if i % 3 == r]
        rc, p = native.miller_partial(b"".join(pks[i] for i in sel), b"".join(msgs[i] for i in sel), 32,
                                      sig, r == 0, d8)
        assert rc == 0
        parts.append(p)
    assert native.final_verify(b"".join(parts)) is True
    assert native.final_verify(b"".join(parts[:2])) is False


def test_deterministic_replay(native):
    """Same batch twice -> identical verdict bytes (device race check)."""
    pks, msgs, sigs, doms, exp = _make_batch(8, 3)
    args = (b"".join(pks), b"".join(msgs), b"".join(sigs), b"".join(d.to_bytes(8, "big") for d in doms))
    a = native.verify_batch(*args)
    b = native.verify_batch(*args)
    assert (a == b).all() and list(a) == exp


# ---------------------------------- batched bls_verify_multiple (C3 / C5 shapes)
def test_verify_multiple_batch_golden(native, golden):
    """All golden verify_multiple cases as ONE batch: per-call verdicts == py_ecc's."""
    _, gb = golden
    cases = [c for c in gb["verify_multiple"] if len(c["pubkeys"]) == len(c["messages"])]
    off, pks, msgs, sigs, doms = [0], b"", b"", b"", b""
    for c in cases:
        pks += b"".join(bytes.fromhex(p) for p in c["pubkeys"])
        msgs += b"".join(bytes.fromhex(m) for m in c["messages"])
        sigs += bytes.fromhex(c["signature"])
        doms += int(c["domain"]).to_bytes(8, "big")
        off.append(off[-1] + len(c["pubkeys"]))
    v = native.verify_multiple_batch(off, pks, msgs, 32, sigs, doms)
    assert list(v) == [c["expected"] for c in cases]


@pytest.mark.parametrize("reps", [1, 700])
def test_verify_multiple_batch_layouts_tiled(native, golden, torsion, reps):
    """Golden + torsion verify_multiple cases repeated `reps` times in one batch: reps = 1 runs
    one lane quad per Miller pair (k_miller_tasks_q1, <= 8192 pairs), reps = 700 two pairs
    per quad (k_miller_quads).  Per-call verdicts == the fixtures' py_ecc column."""
    _, gb = golden
    cases = [(c, c["expected"]) for c in gb["verify_multiple"] if len(c["pubkeys"]) == len(c["messages"])]
    cases += [(c, c["expected_pyecc"]) for c in torsion["verify_multiple"]]
    off, pks, msgs, sigs, doms, want = [0], [], [], [], [], []
    for _ in range(reps):
        for c, e in cases:
            pks += [bytes.fromhex(p) for p in c["pubkeys"]]
            msgs += [bytes.fromhex(m) for m in c["messages"]]
            sigs.append(bytes.fromhex(c["signature"]))
            doms.append(int(c["domain"]).to_bytes(8, "big"))
            off.append(off[-1] + len(c["pubkeys"]))
            want.append(e)
    assert all(len(m) == 32 for m in msgs)
    v = native.verify_multiple_batch(off, b"".join(pks), b"".join(msgs), 32, b"".join(sigs), b"".join(doms))
    assert list(v) == want


def _committee_calls(rng, n_calls, max_keys, sks):
    """Calls of 0..max_keys members over 1..3 distinct messages, signed with the engine."""
    from bls381_amd import bls
    calls = []
    for c in range(n_calls):
        k = rng.randrange(0, max_keys + 1)
        members = [rng.randrange(len(sks)) for _ in range(k)]
        cand = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(rng.randrange(1, 4))]
        msgs = [cand[rng.randrange(len(cand))] for _ in range(k)]
        dom = rng.getrandbits(64)
        sig = bls.bls_aggregate_signatures([bls.bls_sign(m, sks[i], dom) for i, m in zip(members, msgs)])
        calls.append([members, msgs, sig, dom, True])
    return calls


def test_verify_multiple_batch_committees(native):
    """C3 shape: many calls, ragged sizes (incl. empty), tampered calls; == single-call API."""
    from bls381_amd import bls
    rng = random.Random(0xB15_0C03)
    sks = [rng.randrange(1, O.r) for _ in range(24)]
    pubs = [bls.privtopub(k) for k in sks]
    calls = _committee_calls(rng, 40, 12, sks)
    for j, cl in enumerate(calls):
        if j % 5 == 1:                     # other call's signature
            cl[2] = calls[j - 1][2]
            cl[4] = len(cl[0]) == 0 and len(calls[j - 1][0]) == 0
        elif j % 5 == 2:                   # wrong domain
            cl[3] ^= 1
            cl[4] = len(cl[0]) == 0
        elif j % 5 == 3 and cl[0]:         # one member swapped for another key
            cl[0] = [(cl[0][0] + 1) % len(sks)] + cl[0][1:]
            cl[4] = False
    off, pks, msgs, sigs, doms = [0], b"", b"", b"", b""
    for members, ms, sig, dom, _ in calls:
        pks += b"".join(pubs[i] for i in members)
        msgs += b"".join(ms)
        sigs += sig
        doms += dom.to_bytes(8, "big")
        off.append(off[-1] + len(members))
    v = native.verify_multiple_batch(off, pks, msgs, 32, sigs, doms)
    single = [bls.bls_verify_multiple([pubs[i] for i in m], ms, s, d) for m, ms, s, d, _ in calls]
    assert list(v) == single
    assert list(v) == [c[4] for c in calls]


def test_verify_multiple_batch_many_messages(native):
    """C5 shape: calls with 70 and 9 distinct messages (multi-pass segmented product) beside small ones."""
    from bls381_amd import bls
    rng = random.Random(0xB15_0C05)
    calls = []
    for L in (70, 1, 9, 8, 2):
        sks = [rng.randrange(1, O.r) for _ in range(L)]
        ms = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(L)]
        pks = native.privtopub_batch(b"".join(k.to_bytes(32, "big") for k in sks))
        sig = bls.bls_aggregate_signatures(
            [native.sign_batch(b"".join(ms), b"".join(k.to_bytes(32, "big") for k in sks),
                               (5).to_bytes(8, "big") * L)[96 * i:96 * i + 96] for i in range(L)])
        calls.append((pks, b"".join(ms), sig))
    off = np.cumsum([0] + [len(p) // 48 for p, _, _ in calls])
    good = native.verify_multiple_batch(off, b"".join(p for p, _, _ in calls), b"".join(m for _, m, _ in calls), 32,
                                        b"".join(s for _, _, s in calls), (5).to_bytes(8, "big") * len(calls))
    assert list(good) == [True] * len(calls)
    # rotate signatures between calls: every call fails
    sigs = [s for _, _, s in calls]
    sigs = sigs[1:] + sigs[:1]
    bad = native.verify_multiple_batch(off, b"".join(p for p, _, _ in calls), b"".join(m for _, m, _ in calls), 32,
                                       b"".join(sigs), (5).to_bytes(8, "big") * len(calls))
    assert not bad.any()


def test_aggregate_batch_device_async_back_to_back(native):
    """Device-pointer aggregation returns before its copies run: two different plans queued
    back to back on one stream, with host churn in between, must both land intact."""
    import ctypes
    import torch
    L = native.lib()
    dev = torch.device("cuda", 0)
    keys = [O.privtopub(k) for k in range(1, 33)]
    stream = torch.cuda.current_stream(dev)
    runs = []
    for ng, cs in ((2048, 3), (700, 5)):
        # groups alternate: cs keys, then an empty group
        sizes = [cs if g % 2 == 0 else 0 for g in range(ng)]
        offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint32)
        idx = [(g * 7 + j) % 32 for g in range(ng) for j in range(sizes[g])]
        d_pks = torch.frombuffer(bytearray(b"".join(keys[i] for i in idx)), dtype=torch.uint8).to(dev)
        d_out = torch.zeros(ng * 48, dtype=torch.uint8, device=dev)
        d_st = torch.full((ng,), -7, dtype=torch.int32, device=dev)
        ws = torch.empty(L.bls381_aggregate_pubkeys_batch_workspace_size(ng, len(idx)), dtype=torch.uint8,
                         device=dev)
        native.check(L.bls381_aggregate_pubkeys_batch_device(
            ng, offs.ctypes.data_as(ctypes.c_void_p), len(idx), d_pks.data_ptr(), d_out.data_ptr(), d_st.data_ptr(),
            ws.data_ptr(), ctypes.c_void_p(stream.cuda_stream)))
        del offs                                      # the caller's offsets may die right away
        _ = [bytearray(1 << 16) for _ in range(64)]   # host allocation churn
        runs.append((ng, sizes, idx, d_out, d_st, d_pks, ws))
    torch.cuda.synchronize()
    cache = {}
    for ng, sizes, idx, d_out, d_st, _, _ in runs:
        assert int(d_st.abs().sum().item()) == 0
        out = d_out.cpu().numpy().tobytes()
        pos = 0
        for g in range(ng):
            members = idx[pos:pos + sizes[g]]
            pos += sizes[g]
            k = sum(i + 1 for i in members)
            if k not in cache:
                cache[k] = O.privtopub(k) if k else bytes([0xC0]) + bytes(47)
            want = cache[k]
            assert out[48 * g:48 * g + 48] == want, (ng, g)


def test_device_entry_points_order_on_torch_default_stream(native):
    """stream=NULL (torch's default stream) means the HIP null stream: a torch read of the
    output right after the call (no device-wide synchronize) must see the finished result."""
    import ctypes
    import torch
    L = native.lib()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    keys = [O.privtopub(k) for k in range(1, 17)]
    ng = 512
    sizes = [128 if g % 2 == 0 else 0 for g in range(ng)]
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint32)
    idx = [(g * 5 + j) % 16 for g in range(ng) for j in range(sizes[g])]
    host_pks = b"".join(keys[i] for i in idx)
    d_pks = torch.frombuffer(bytearray(host_pks), dtype=torch.uint8).to(dev)
    d_out = torch.zeros(ng * 48, dtype=torch.uint8, device=dev)
    d_st = torch.zeros(ng, dtype=torch.int32, device=dev)
    ws = torch.empty(L.bls381_aggregate_pubkeys_batch_workspace_size(ng, len(idx)), dtype=torch.uint8, device=dev)
    native.check(L.bls381_aggregate_pubkeys_batch_device(
        ng, offs.ctypes.data_as(ctypes.c_void_p), len(idx), d_pks.data_ptr(), d_out.data_ptr(), d_st.data_ptr(),
        ws.data_ptr(), ctypes.c_void_p(stream.cuda_stream)))
    got = d_out.cpu().numpy().tobytes()            # torch-stream ordered read only
    ref, rst = native.aggregate_pubkeys_batch(offs, host_pks)
    assert got == b"".join(ref) and not np.any(rst)
    # verify_batch_device likewise
    sks = [3, 5, 7, 11]
    msg = bytes(range(32))
    pks = b"".join(O.privtopub(k) for k in sks)
    sigs = bytearray(native.sign_batch(msg * 4, b"".join(k.to_bytes(32, "big") for k in sks),
                                       (3).to_bytes(8, "big") * 4))
    sigs[96 * 2:96 * 3] = sigs[0:96]
    t = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)
    d_v = torch.zeros(4, dtype=torch.uint8, device=dev)
    vws = torch.empty(L.bls381_verify_batch_workspace_size(4), dtype=torch.uint8, device=dev)
    keep = [t(pks), t(msg * 4), t(bytes(sigs)), t((3).to_bytes(8, "big") * 4)]   # alive across the call
    native.check(L.bls381_verify_batch_device(4, *[x.data_ptr() for x in keep], d_v.data_ptr(),
                                              vws.data_ptr(), ctypes.c_void_p(stream.cuda_stream)))
    assert d_v.cpu().tolist() == [1, 1, 0, 1]


# ------------------------------------------ pubkey registry (§8(f) rank 1)
def test_registry_matches_aggregate_pubkeys(native, golden):
    """Registry aggregation (by index and by content lookup) == bls_aggregate_pubkeys bytes."""
    from bls381_amd import bls
    from bls381_amd.registry import PubkeyRegistry
    _, gb = golden
    inf = bytes([0xC0]) + b"\x00" * 47
    keys = [O.privtopub(k) for k in range(1, 201)] + [inf]
    bad = [bytes.fromhex(h) for h in gb["invalid_g1"]]
    reg = PubkeyRegistry(1024)
    ent = reg.add(keys + bad + keys[:3])            # bad keys -> -1, duplicates -> earlier entry
    assert list(ent[:201]) == list(range(201))
    assert all(e == -1 for e in ent[201:201 + len(bad)])
    assert list(ent[201 + len(bad):]) == [0, 1, 2]
    assert len(reg) == 201 + len(bad) + 3
    assert list(reg.lookup([keys[7], keys[200], O.privtopub(999), bad[0]])) == [7, 200, -1, -1]
    rng = random.Random(0xB15_0006)
    groups = [rng.sample(range(201), 128) for _ in range(6)] + [[], [200], [3, 3, 3], list(range(201))]
    got = reg.aggregate_indices(groups)
    for g, out in zip(groups, got):
        assert out == O.aggregate_pubkeys([keys[i] for i in g])
    # content-addressed: registered, unregistered and infinity members mixed
    extra = [O.privtopub(k) for k in range(1000, 1010)]
    byte_groups = [[keys[i] for i in groups[0]] + extra, extra, [keys[5], inf], []]
    got = reg.aggregate_pubkeys_batch(byte_groups)
    for g, out in zip(byte_groups, got):
        assert out == O.aggregate_pubkeys(g)
    # the bls shim routed through the registry: same bytes, same errors
    bls.use_pubkey_registry(reg)
    try:
        assert bls.bls_aggregate_pubkeys(byte_groups[0]) == O.aggregate_pubkeys(byte_groups[0])
        for b in bad:
            with pytest.raises(ValueError):
                bls.bls_aggregate_pubkeys([keys[0], b])
        assert bls.bls_aggregate_pubkeys([]) == inf
    finally:
        bls.use_pubkey_registry(None)
    # a bad or out-of-range entry fails its group only
    with pytest.raises(ValueError):
        reg.aggregate_indices([[0, 201]])            # entry 201 holds an undecodable key
    with pytest.raises(ValueError):
        reg.aggregate_indices([[0, len(reg)]])       # past the end: never read
    reg.close()


def test_registry_large_multilevel(native):
    """3000-member group through the registry (multi-level tree): sum [k]G = [sum k]G."""
    from bls381_amd.registry import PubkeyRegistry
    keys = [O.privtopub(k) for k in range(1, 41)]
    reg = PubkeyRegistry(64)
    reg.add(keys)
    n = 3000
    idx = [i % 40 for i in range(n)]
    out = reg.aggregate_indices([idx, idx[:513]])
    assert out[0] == O.privtopub(sum(i + 1 for i in idx))
    assert out[1] == O.privtopub(sum(i + 1 for i in idx[:513]))
    with pytest.raises(ValueError):
        reg.add([keys[0]] * 100)                     # capacity 64 exceeded
    reg.close()


# ---------------------------------------- YAML `bls` suites (§8(f) rank 4)
def test_yaml_vectors_generate_and_run(native, golden, tmp_path):
    """The engine regenerates all 94 generator cases bit-exact, and the runner passes them."""
    from bls381_amd import bls, vector_runner as V
    vec, _ = golden
    cases = V.generate_cases(bls)
    assert cases == vec
    V.write_suites(str(tmp_path), cases)
    res = V.run(str(tmp_path), bls)
    assert sum(ok for ok, _ in res.values()) == 94 and not any(f for _, f in res.values())


# ------------------------------------------------ SSZ roots (§8(f) rank 2)
def test_ssz_roots_match_fixtures(native, golden):
    import json
    from bls381_amd import ssz
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ssz_roots.json")) as f:
        fx = json.load(f)
    types = {"DepositData": ssz.DepositData, "AttestationDataAndCustodyBit": ssz.AttestationDataAndCustodyBit,
             "AttestationData": ssz.AttestationData, "Crosslink": ssz.Crosslink,
             "BeaconBlockHeader": ssz.BeaconBlockHeader}
    for name, typ in types.items():
        cases = [c for c in fx["roots"] if c["type"] == name]
        items = [bytes.fromhex(c["serialized"]) for c in cases] * 50          # a batch of several waves
        got = ssz.hash_tree_root_batch(typ, items)
        assert [g.hex() for g in got] == [c["hash_tree_root"] for c in cases] * 50, name
        got = ssz.signing_root_batch(typ, items)
        assert [g.hex() for g in got] == [c["signing_root"] for c in cases] * 50, name


def test_verify_deposits_pipeline(native):
    """process_deposit's PoP check with signing roots made on the device == oracle verdicts."""
    import ssz_oracle as S
    from bls381_amd import bls, ssz
    rng = random.Random(0xB15_0008)
    dom = 3
    items, want = [], []
    for j in range(300):
        sk = rng.randrange(1, 1 << 250)
        v = {"pubkey": bls.privtopub(sk), "withdrawal_credentials": bytes(rng.randrange(256) for _ in range(32)),
             "amount": 32 * 10 ** 9 + j, "signature": b"\x00" * 96}
        root = S.signing_root(S.DepositData, v)
        v["signature"] = bls.bls_sign(root, sk, dom)
        ok = True
        if j % 7 == 3:
            v["amount"] += 1; ok = False             # signed data changed
        elif j % 7 == 5:
            v["signature"] = b"\x00" * 96; ok = False
        items.append(S.serialize(S.DepositData, v))
        want.append(ok)
    got = ssz.verify_deposits(items, dom)
    assert list(got) == want
    for k in (0, 3, 5):                                # the oracle's own verify on a few
        v = items[k]
        assert O.verify(S.signing_root(S.DepositData, {"pubkey": v[:48], "withdrawal_credentials": v[48:80],
                                                       "amount": int.from_bytes(v[80:88], "little"),
                                                       "signature": v[88:]}), v[:48], v[88:], dom) == want[k]


# ------------------------------- subgroup policy on torsion points
def _vm_args(c):
    return ([bytes.fromhex(p) for p in c["pubkeys"]], [bytes.fromhex(m) for m in c["messages"]],
            bytes.fromhex(c["signature"]), int(c["domain"]))


@pytest.mark.parametrize("policy", ["pyecc", "strict"])
def test_torsion_verdicts_both_policies(native, torsion, policy):
    """Points with small-order components: py_ecc's verdicts under SUBGROUP_POLICY="pyecc"
    (incl. the degenerate Miller loop of an order-13 signature), the spec-strict ones under
    "strict" -- through the shim, the verify batch, the verify_multiple batch and the
    sharded partial products."""
    from bls381_amd import bls
    col = "expected_" + policy
    old = bls.SUBGROUP_POLICY
    bls.SUBGROUP_POLICY = policy
    try:
        vs = torsion["verify"]
        for c in vs:
            got = bls.bls_verify(bytes.fromhex(c["pubkey"]), bytes.fromhex(c["message"]),
                                 bytes.fromhex(c["signature"]), int(c["domain"]))
            assert got == c[col], (c["kind"], policy)
        native.set_subgroup_policy(policy)
        v = native.verify_batch(b"".join(bytes.fromhex(c["pubkey"]) for c in vs),
                                b"".join(bytes.fromhex(c["message"]) for c in vs),
                                b"".join(bytes.fromhex(c["signature"]) for c in vs),
                                b"".join(int(c["domain"]).to_bytes(8, "big") for c in vs))
        assert list(v) == [c[col] for c in vs]
        vms = torsion["verify_multiple"]
        for c in vms:
            assert bls.bls_verify_multiple(*_vm_args(c)) == c[col], (c["kind"], policy)
        native.set_subgroup_policy(policy)
        off, pks, msgs, sigs, doms = [0], b"", b"", b"", b""
        for c in vms:
            p, m, s, d = _vm_args(c)
            pks += b"".join(p); msgs += b"".join(m); sigs += s; doms += d.to_bytes(8, "big")
            off.append(off[-1] + len(p))
        assert list(native.verify_multiple_batch(off, pks, msgs, 32, sigs, doms)) == [c[col] for c in vms]
        for c in vms:                                  # two-shard partial products
            p, m, s, d = _vm_args(c)
            d8 = d.to_bytes(8, "big")
            rc0, a = native.miller_partial(b"".join(p[:1]), b"".join(m[:1]), 32, s, True, d8)
            rc1, b = native.miller_partial(b"".join(p[1:]), b"".join(m[1:]), 32, s, False, d8)
            got = (rc0 == 0 and rc1 == 0) and native.final_verify(a + b)
            if len(set(m)) == len(m):                  # shards split whole message groups only
                assert got == c[col], (c["kind"], policy)
    finally:
        bls.SUBGROUP_POLICY = old
        native.set_subgroup_policy(old)


def test_torsion_aggregates(native, torsion):
    """Aggregation never checks subgroups: sums with torsion components are py_ecc's bytes."""
    from bls381_amd import bls
    for c in torsion["aggregate_pubkeys"]:
        assert bls.bls_aggregate_pubkeys([bytes.fromhex(p) for p in c["input"]]).hex() == c["output"], c["kind"]
    for c in torsion["aggregate_sigs"]:
        assert bls.bls_aggregate_signatures([bytes.fromhex(s) for s in c["input"]]).hex() == c["output"], c["kind"]


def test_long_and_mixed_length_messages(native):
    """py_ecc hashes messages of any length: > 256 bytes (streamed SHA-256, multi-block), and
    a verify_multiple mixing lengths (per-length partial products, one final exponentiation)."""
    from bls381_amd import bls
    sk = 4242
    for n in (257, 1000, 4096):
        msg = bytes((7 * i) & 0xFF for i in range(n))
        sig = bls.bls_sign(msg, sk, 11)
        assert sig == O.sign(msg, sk, 11)
        assert bls.bls_verify(bls.privtopub(sk), msg, sig, 11) is True
        assert bls.bls_verify(bls.privtopub(sk), msg[:-1], sig, 11) is False
    sks = [5, 6, 7, 8]
    msgs = [b"\x01" * 32, b"\x02" * 300, b"", b"\x01" * 32]
    pks = [bls.privtopub(k) for k in sks]
    sig = bls.bls_aggregate_signatures([bls.bls_sign(m, k, 2) for m, k in zip(msgs, sks)])
    assert O.verify_multiple(pks, msgs, sig, 2) is True
    assert bls.bls_verify_multiple(pks, msgs, sig, 2) is True
    assert bls.bls_verify_multiple(pks[::-1], msgs, sig, 2) is False
    with pytest.raises(ValueError):
        bls.bls_verify(pks[0], bytes((1 << 20) + 1), sig, 2)


# ---------------------------------------------- C4 / C5 at full size
def test_c4_aggregate_2p20_keys_eight_shards(native):
    """C4: 2^20 pubkeys aggregated as 8 shards (sharding.shard_range, one per GPU of a node),
    each a device partial, the partials summed: equals [sum k]G in closed form (the keys are
    [(i mod 64) + 1]G), and equals the unsharded aggregation."""
    from bls381_amd.sharding import shard_range
    n, world = 1 << 20, 8
    base = native.privtopub_batch(b"".join(k.to_bytes(32, "big") for k in range(1, 65)))
    keys = np.frombuffer(base, dtype=np.uint8).reshape(64, 48)[np.arange(n) % 64].tobytes()
    parts = []
    for r in range(world):
        lo, hi = shard_range(n, r, world)
        parts.append(native.aggregate_pubkeys(keys[48 * lo:48 * hi]))
    total = native.aggregate_pubkeys(b"".join(parts))
    want = sum((i % 64) + 1 for i in range(n)) % O.r
    assert total == O.privtopub(want)
    assert native.aggregate_pubkeys(keys) == total


def test_c4_verify_multiple_batch_eight_shards(native, golden):
    """C4 second half: independent verify_multiple calls split into 8 contiguous call ranges
    (sharding.shard_range); the per-shard batch verdicts, concatenated, equal the oracle's."""
    from bls381_amd.sharding import shard_range
    _, gb = golden
    cases = [c for c in gb["verify_multiple"] if len(c["pubkeys"]) == len(c["messages"])] * 9
    world = 8
    got = []
    for r in range(world):
        lo, hi = shard_range(len(cases), r, world)
        off, pks, msgs, sigs, doms = [0], b"", b"", b"", b""
        for c in cases[lo:hi]:
            pks += b"".join(bytes.fromhex(p) for p in c["pubkeys"])
            msgs += b"".join(bytes.fromhex(m) for m in c["messages"])
            sigs += bytes.fromhex(c["signature"])
            doms += int(c["domain"]).to_bytes(8, "big")
            off.append(off[-1] + len(c["pubkeys"]))
        got.extend(native.verify_multiple_batch(off, pks, msgs, 32, sigs, doms))
    assert got == [c["expected"] for c in cases]


def test_c5_verify_multiple_4096_messages(native):
    """C5 at L = 4096: signatures from the engine spot-checked against the oracle, the
    aggregate signature over all 4096 (message, key) pairs verifies, a swapped key, a changed
    message or domain does not; the two-shard partial products agree."""
    from bls381_amd import bls
    rng = random.Random(0xB15_C5)
    L = 4096
    sks = [rng.randrange(1, O.r) for _ in range(L)]
    msgs = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(L)]
    skb = b"".join(k.to_bytes(32, "big") for k in sks)
    pks = native.privtopub_batch(skb)
    sigs = native.sign_batch(b"".join(msgs), skb, (1).to_bytes(8, "big") * L)
    for j in (0, 1777, L - 1):
        assert sigs[96 * j:96 * j + 96] == O.sign(msgs[j], sks[j], 1)
        assert pks[48 * j:48 * j + 48] == O.privtopub(sks[j])
    sig = native.aggregate_signatures(sigs)
    pk_list = [pks[48 * j:48 * j + 48] for j in range(L)]
    assert bls.bls_verify_multiple(pk_list, msgs, sig, 1) is True
    assert bls.bls_verify_multiple(pk_list, msgs, sig, 2) is False
    swapped = pk_list[:]
    swapped[5], swapped[6] = swapped[6], swapped[5]
    assert bls.bls_verify_multiple(swapped, msgs, sig, 1) is False
    changed = msgs[:]
    changed[4000] = bytes([changed[4000][0] ^ 1]) + changed[4000][1:]
    assert bls.bls_verify_multiple(pk_list, changed, sig, 1) is False
    d8 = (1).to_bytes(8, "big")
    rc0, a = native.miller_partial(pks[:48 * 2048], b"".join(msgs[:2048]), 32, sig, True, d8)
    rc1, b = native.miller_partial(pks[48 * 2048:], b"".join(msgs[2048:]), 32, sig, False, d8)
    assert rc0 == 0 and rc1 == 0 and native.final_verify(a + b) is True


def test_verify_multiple_batch_device_entry(native, golden, torsion):
    """bls381_verify_multiple_batch_device (keys, signatures, domains in HBM; plan from host
    offsets + messages): golden and torsion calls in one batch, verdicts == oracle columns."""
    import ctypes
    import torch
    L = native.lib()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    _, gb = golden
    cases = [(c, c["expected"]) for c in gb["verify_multiple"] if len(c["pubkeys"]) == len(c["messages"])]
    cases += [(c, c["expected_pyecc"]) for c in torsion["verify_multiple"]]
    off, pks, msgs, sigs, doms = [0], b"", b"", b"", b""
    for c, _ in cases:
        pks += b"".join(bytes.fromhex(p) for p in c["pubkeys"])
        msgs += b"".join(bytes.fromhex(m) for m in c["messages"])
        sigs += bytes.fromhex(c["signature"])
        doms += int(c["domain"]).to_bytes(8, "big")
        off.append(off[-1] + len(c["pubkeys"]))
    off = np.array(off, dtype=np.uint32)
    t = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)
    d_pks, d_sigs, d_doms = t(pks), t(sigs), t(doms)
    d_v = torch.full((len(cases),), 7, dtype=torch.uint8, device=dev)
    ws = torch.empty(L.bls381_verify_multiple_batch_workspace_size(len(cases), len(pks) // 48, 32),
                     dtype=torch.uint8, device=dev)
    native.set_subgroup_policy("pyecc")
    native.check(L.bls381_verify_multiple_batch_device(
        len(cases), off.ctypes.data_as(ctypes.c_void_p), msgs, 32, d_pks.data_ptr(), d_sigs.data_ptr(),
        d_doms.data_ptr(), d_v.data_ptr(), ws.data_ptr(), ctypes.c_void_p(stream.cuda_stream)))
    del off, msgs                                   # the plan is the engine's own copy
    got = d_v.cpu().tolist()
    assert got == [int(e) for _, e in cases]


@pytest.mark.parametrize("policy", ["pyecc", "strict"])
def test_verify_multiple_grouped_device(native, golden, torsion, policy):
    """bls381_verify_multiple_grouped_device (validate_indexed_attestation's
    verify_multiple-of-aggregates, aggregation fused): golden + torsion calls regrouped by
    message, with one group split in two under the same message (merged again) and an empty
    group per call (the infinite aggregate); per-call verdicts == the fixtures' column for the
    subgroup policy (py_ecc's, or the strict one), directly and through the registry."""
    import ctypes
    import torch
    from bls381_amd import bls
    L = native.lib()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    h = bytes.fromhex
    _, gb = golden
    gcol = "expected" if policy == "pyecc" else "expected_strict"
    cases = [([h(p) for p in c["pubkeys"]], [h(m) for m in c["messages"]], h(c["signature"]), int(c["domain"]),
              c[gcol]) for c in gb["verify_multiple"] if len(c["pubkeys"]) == len(c["messages"])]
    cases += [([h(p) for p in c["pubkeys"]], [h(m) for m in c["messages"]], h(c["signature"]), int(c["domain"]),
               c["expected_" + policy]) for c in torsion["verify_multiple"]]
    rng = random.Random(0xB15_0C0D)
    sks = [rng.randrange(1, O.r) for _ in range(24)]
    pubs = [bls.privtopub(k) for k in sks]
    for members, ms, sig, dom, ok in _committee_calls(rng, 30, 10, sks):
        cases.append(([pubs[i] for i in members], ms, sig, dom, ok))

    def run(calls, reg=None):
        cgo, gko, gmsgs, keys, sigs, doms = [0], [0], [], [], b"", b""
        for pks, ms, sig, dom, _ in calls:
            order = []
            for m in ms:
                if m not in order:
                    order.append(m)
            groups = [[p for p, mm in zip(pks, ms) if mm == m] for m in order]
            gm = list(order)
            if groups and len(groups[0]) >= 2:            # split: two groups, same message
                groups = [groups[0][:1], groups[0][1:]] + groups[1:]
                gm = [gm[0], gm[0]] + gm[1:]
            groups.append([])                             # the empty aggregate
            gm.append(bytes(rng.getrandbits(8) for _ in range(32)))
            for g, m in zip(groups, gm):
                keys += g
                gmsgs.append(m)
                gko.append(gko[-1] + len(g))
            cgo.append(cgo[-1] + len(groups))
            sigs += sig
            doms += dom.to_bytes(8, "big")
        cgo = np.array(cgo, dtype=np.uint32)
        gko = np.array(gko, dtype=np.uint32)
        t = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)
        d_pks, d_sigs, d_doms = t(b"".join(keys) + b"\0"), t(sigs), t(doms)
        d_v = torch.full((len(calls),), 7, dtype=torch.uint8, device=dev)
        ws = torch.empty(L.bls381_verify_multiple_grouped_workspace_size(len(calls), len(gmsgs), len(keys), 32),
                         dtype=torch.uint8, device=dev)
        if reg is None:
            native.check(L.bls381_verify_multiple_grouped_device(
                len(calls), cgo.ctypes.data_as(ctypes.c_void_p), len(gmsgs), gko.ctypes.data_as(ctypes.c_void_p),
                b"".join(gmsgs), 32, d_pks.data_ptr(), d_sigs.data_ptr(), d_doms.data_ptr(), d_v.data_ptr(),
                ws.data_ptr(), ctypes.c_void_p(stream.cuda_stream)))
        else:
            # members as registry entries (an undecodable key's entry holds a BAD status)
            ent = reg.add(keys) if keys else np.zeros(0, dtype=np.int32)
            d_ent = t(ent.astype(np.int32).tobytes() + b"\0\0\0\0")
            native.check(L.bls381_registry_verify_multiple_grouped_device(
                reg._h, len(calls), cgo.ctypes.data_as(ctypes.c_void_p), len(gmsgs),
                gko.ctypes.data_as(ctypes.c_void_p), b"".join(gmsgs), 32, d_ent.data_ptr(), d_sigs.data_ptr(),
                d_doms.data_ptr(), d_v.data_ptr(), ws.data_ptr(), ctypes.c_void_p(stream.cuda_stream)))
        return [bool(x) for x in d_v.cpu().tolist()]

    native.set_subgroup_policy(policy)
    from bls381_amd.registry import PubkeyRegistry
    reg = PubkeyRegistry(4096)
    try:
        assert run(cases) == [bool(c[4]) for c in cases]
        # one call per attestation, as an epoch: the same verdicts in a batch of 600 (task path)
        many = [cases[i % len(cases)] for i in range(600)]
        assert run(many) == [bool(c[4]) for c in many]
        assert run(cases, reg) == [bool(c[4]) for c in cases]
    finally:
        reg.close()
        native.set_subgroup_policy("pyecc")


# ------------------------------------ native multi-GPU ABI over RCCL
def _comm_checks(native, golden, torsion, noncanon):
    from bls381_amd import comm
    _, gb = golden
    h = bytes.fromhex
    native.set_subgroup_policy("pyecc")
    vms = [(c, c["expected"]) for c in gb["verify_multiple"] if len(c["pubkeys"]) == len(c["messages"])]
    vms += [(c, c["expected_pyecc"]) for c in torsion["verify_multiple"]]
    for c, want in vms:
        got = comm.verify_multiple([h(p) for p in c["pubkeys"]], [h(m) for m in c["messages"]], h(c["signature"]),
                                   int(c["domain"]))
        assert got == want, c["kind"]
    for c in gb["aggregate_pubkeys"] + torsion["aggregate_pubkeys"]:
        assert comm.aggregate_pubkeys([h(p) for p in c["input"]]).hex() == c["output"], c["kind"]
    for c in noncanon["aggregate_pubkeys"]:       # py_ecc's lax codec on every rank's slice
        if c["output_pyecc"] is None:
            with pytest.raises(ValueError):
                comm.aggregate_pubkeys([h(p) for p in c["input"]])
        else:
            assert comm.aggregate_pubkeys([h(p) for p in c["input"]]).hex() == c["output_pyecc"], c["kind"]
    keys = [O.privtopub(k) for k in range(1, 41)]
    assert comm.aggregate_pubkeys([keys[i % 40] for i in range(1000)]) == O.privtopub(
        sum((i % 40) + 1 for i in range(1000)))
    with pytest.raises(ValueError):
        comm.aggregate_pubkeys(keys[:7] + [h(gb["invalid_g1"][1])])
    # the device-resident form (one process holds the whole call: world 1, or every virtual rank)
    import torch

    def dev_agg(pk_list):
        blob = b"".join(pk_list)
        d_pks = torch.frombuffer(bytearray(blob + b"\0"), dtype=torch.uint8)[:len(blob)].cuda()
        d_out = torch.zeros(48, dtype=torch.uint8, device="cuda")
        d_st = torch.full((1,), -1, dtype=torch.int32, device="cuda")
        d_ws = torch.empty(comm.aggregate_pubkeys_device_workspace_size(len(pk_list)), dtype=torch.uint8, device="cuda")
        s = torch.cuda.current_stream()
        comm.aggregate_pubkeys_device(len(pk_list), d_pks.data_ptr(), d_out.data_ptr(), d_st.data_ptr(),
                                      d_ws.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize()
        return bytes(d_out.cpu().numpy()), int(d_st.item())
    for c in gb["aggregate_pubkeys"] + torsion["aggregate_pubkeys"]:
        assert dev_agg([h(p) for p in c["input"]]) == (bytes.fromhex(c["output"]), 0), c["kind"]
    assert dev_agg([keys[i % 40] for i in range(1000)]) == (O.privtopub(sum((i % 40) + 1 for i in range(1000))), 0)
    assert dev_agg(keys[:7] + [h(gb["invalid_g1"][1])])[1] == native.EINVAL_POINT
    off, pks, msgs, sigs, doms = [0], b"", b"", b"", b""
    for c, _ in vms * 2:
        pks += b"".join(h(p) for p in c["pubkeys"]); msgs += b"".join(h(m) for m in c["messages"])
        sigs += h(c["signature"]); doms += int(c["domain"]).to_bytes(8, "big")
        off.append(off[-1] + len(c["pubkeys"]))
    assert comm.verify_multiple_batch(off, pks, msgs, 32, sigs, doms) == [w for _, w in vms * 2]


def test_native_comm_rccl_world1(native, golden, torsion, noncanon):
    """The library's own RCCL communicator (ncclCommInitRank through dlopen), one rank: the
    collective entry points give the single-GPU verdicts and bytes.  Multi-rank RCCL on a
    one-GPU box is refused by RCCL itself (duplicate GPU), see the virtual-rank test."""
    from bls381_amd import comm
    comm.init(1, 0, comm.unique_id())
    try:
        assert comm.size() == 1 and comm.rank() == 0
        _comm_checks(native, golden, torsion, noncanon)
    finally:
        comm.destroy()
    assert comm.size() == 0


@pytest.mark.parametrize("virtual", [False, True])
def test_native_comm_destroy_after_device_call(native, virtual):
    """bls381_comm_destroy right after the device-resident aggregation, with its collectives still
    queued on the caller's stream and no synchronisation in between: the destroy waits
    for them, and the aggregate and status written afterwards are the right ones."""
    import torch
    from bls381_amd import comm
    keys = [O.privtopub(k) for k in range(1, 41)]
    blob = b"".join(keys[i % 40] for i in range(4096))
    want = O.privtopub(sum((i % 40) + 1 for i in range(4096)))
    d_pks = torch.frombuffer(bytearray(blob), dtype=torch.uint8).cuda()
    d_out = torch.zeros(48, dtype=torch.uint8, device="cuda")
    d_st = torch.full((1,), -1, dtype=torch.int32, device="cuda")
    if virtual:
        comm.init_virtual(3)
    else:
        comm.init(1, 0, comm.unique_id())
    try:
        d_ws = torch.empty(comm.aggregate_pubkeys_device_workspace_size(4096), dtype=torch.uint8, device="cuda")
        s = torch.cuda.current_stream()
        comm.aggregate_pubkeys_device(4096, d_pks.data_ptr(), d_out.data_ptr(), d_st.data_ptr(), d_ws.data_ptr(),
                                      s.cuda_stream)
    finally:
        comm.destroy()
    assert comm.size() == 0
    torch.cuda.synchronize()
    assert int(d_st.item()) == 0
    assert bytes(d_out.cpu().numpy()) == want


@pytest.mark.parametrize("world", [2, 3, 8])
def test_native_comm_virtual_ranks(native, golden, torsion, noncanon, world):
    """N ranks on one GPU (bls381_comm_init_virtual): per-rank partials by distinct message,
    rank-0 product + single final exponentiation, contiguous aggregation ranges -- no PyTorch."""
    from bls381_amd import comm
    comm.init_virtual(world)
    try:
        assert comm.size() == world
        _comm_checks(native, golden, torsion, noncanon)
    finally:
        comm.destroy()


# ------------------------- opt-in randomized batch verification (north star)
@pytest.mark.parametrize("policy", ["pyecc", "strict"])
def test_randomized_batch_matches_per_item_verdicts(native, golden, torsion, policy):
    """Golden + torsion verify items (bad encodings, infinities, torsion in keys and signatures)
    through bls381_verify_batch_randomized at several sub-batch sizes: the same verdicts as
    the default per-item pipeline (py_ecc's, or the strict column)."""
    import os as _os
    _, gb = golden
    gcol = "expected" if policy == "pyecc" else "expected_strict"
    items = [(c, c[gcol]) for c in gb["verify"]]
    items += [(c, c["expected_" + policy]) for c in torsion["verify"]]
    pks = b"".join(bytes.fromhex(c["pubkey"]) for c, _ in items)
    msgs = b"".join(bytes.fromhex(c["message"]) for c, _ in items)
    sigs = b"".join(bytes.fromhex(c["signature"]) for c, _ in items)
    doms = b"".join(int(c["domain"]).to_bytes(8, "big") for c, _ in items)
    native.set_subgroup_policy(policy)
    try:
        want = list(native.verify_batch(pks, msgs, sigs, doms))
        assert want == [e for _, e in items]
        for B in (2, 8, 64):
            got = native.verify_batch_randomized(pks, msgs, sigs, doms, _os.urandom(32), B)
            assert list(got) == want, B
    finally:
        native.set_subgroup_policy("pyecc")


@pytest.mark.parametrize("n", [4096, 5003, 65536])
def test_randomized_batch_clean_and_tampered(native, n):
    """n valid items: every sub-batch passes (no per-item re-verification); the same batch
    with 1/16 tampered: identical verdicts to the default pipeline, failing sub-batches
    re-verified.  The re-verification runs the per-item pairings over the call's own decoded
    points and hashes; at 2^16 items sub-batches of 64 (every one fails: 2^16 items, the split
    Miller loop) and of 8 (~40 % fail: the quad loops) cover its layouts."""
    import ctypes
    import os as _os
    import torch
    L = native.lib()
    rng = np.random.default_rng(17)
    sk = 0xC0FFEE
    pk = O.privtopub(sk)
    ms = [bytes(rng.integers(0, 256, 32, dtype=np.uint8)) for _ in range(64)]
    ss = native.sign_batch(b"".join(ms), sk.to_bytes(32, "big") * 64, (3).to_bytes(8, "big") * 64)
    idx = rng.integers(0, 64, n)
    msgs = b"".join(ms[i] for i in idx)
    sigs = bytearray(b"".join(ss[96 * i:96 * i + 96] for i in idx))
    doms = (3).to_bytes(8, "big") * n
    dev = torch.device("cuda", 0)
    t = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)
    stream = torch.cuda.current_stream(dev)

    def run(sig_bytes, B):
        d = [t(pk * n), t(msgs), t(bytes(sig_bytes)), t(doms)]
        v = torch.zeros(n, dtype=torch.uint8, device=dev)
        ws = torch.empty(L.bls381_verify_batch_randomized_workspace_size(n, B), dtype=torch.uint8, device=dev)
        st = (ctypes.c_uint64 * 3)()
        native.check(L.bls381_verify_batch_randomized_device(n, *[x.data_ptr() for x in d], _os.urandom(32), B,
                                                             v.data_ptr(), ws.data_ptr(),
                                                             ctypes.c_void_p(stream.cuda_stream), st))
        return v.cpu().numpy().astype(bool), list(st)

    for B in ((64, 2, 256) if n == 5003 else (64,)):   # ragged last sub-batch; every MSM sub-batch passes
        v, st = run(sigs, B)
        assert v.all() and st == [n, 0, 0], B
    for i in range(5, n, 16):
        j = (i + 1) % n
        if idx[j] != idx[i]:
            sigs[96 * i:96 * i + 96] = sigs[96 * j:96 * j + 96]
    want = native.verify_batch(pk * n, msgs, bytes(sigs), doms)
    assert not want.all()
    for B in ((64, 8) if n > 4096 else (64,)):
        v, st = run(sigs, B)
        assert np.array_equal(v, want) and st[2] > 0 and st[0] + st[1] == n, B


def test_randomized_batch_largest_sub_batches(native):
    """The largest sub-batches: B = 32,768, the 16-bit point-number limit of the MSM
    lists, which now takes the per-item ladder and the tree sum, and B = 256, the largest MSM
    sub-batch, over 2^16 + 3 items (a ragged 3-item last sub-batch).  Clean: every sub-batch
    passes; one tampered item in the first sub-batch: exactly that sub-batch fails and its
    items are re-verified to the default path's verdicts."""
    import ctypes
    import os as _os
    import torch
    L = native.lib()
    n = (1 << 16) + 3
    rng = np.random.default_rng(23)
    sk = 0xBA7C4
    pk = O.privtopub(sk)
    ms = [bytes(rng.integers(0, 256, 32, dtype=np.uint8)) for _ in range(32)]
    ss = native.sign_batch(b"".join(ms), sk.to_bytes(32, "big") * 32, (3).to_bytes(8, "big") * 32)
    idx = rng.integers(0, 32, n)
    msgs = b"".join(ms[i] for i in idx)
    sigs = bytearray(b"".join(ss[96 * i:96 * i + 96] for i in idx))
    doms = (3).to_bytes(8, "big") * n
    dev = torch.device("cuda", 0)
    t = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)
    stream = torch.cuda.current_stream(dev)

    def run(sig_bytes, B):
        d = [t(pk * n), t(msgs), t(bytes(sig_bytes)), t(doms)]
        v = torch.zeros(n, dtype=torch.uint8, device=dev)
        ws = torch.empty(L.bls381_verify_batch_randomized_workspace_size(n, B), dtype=torch.uint8, device=dev)
        st = (ctypes.c_uint64 * 3)()
        native.check(L.bls381_verify_batch_randomized_device(n, *[x.data_ptr() for x in d], _os.urandom(32), B,
                                                             v.data_ptr(), ws.data_ptr(),
                                                             ctypes.c_void_p(stream.cuda_stream), st))
        return v.cpu().numpy().astype(bool), list(st)

    for B in (32768, 256):
        v, st = run(sigs, B)
        assert v.all() and st == [n, 0, 0], B
    j = next(k for k in range(1, 32) if idx[k] != idx[0])
    sigs[0:96] = sigs[96 * j:96 * j + 96]
    for B in (32768, 256):
        v, st = run(sigs, B)
        assert not v[0] and v[1:].all() and st[2] == 1 and st[1] == B, (B, st)


# ---------------------------- octet-layout final exponentiation (latency knob)
_OCT_SCRIPT = r"""
import json, os, sys
root = sys.argv[1]
sys.path[:0] = [root, os.path.join(root, "consensus-specs_amd")]
import numpy as np
from bls381_amd import _native as native
native.init(0)
gb = json.load(open(os.path.join(root, "tests", "golden", "bls_golden_batches.json")))
tor = json.load(open(os.path.join(root, "tests", "golden", "bls_torsion.json")))
items = [(c, c["expected"]) for c in gb["verify"] if len(bytes.fromhex(c["message"])) == 32]
items += [(c, c["expected_pyecc"]) for c in tor["verify"]]
for n in (len(items), 3000):
    sel = [items[i % len(items)] for i in range(n)]
    got = native.verify_batch(b"".join(bytes.fromhex(c["pubkey"]) for c, _ in sel),
                              b"".join(bytes.fromhex(c["message"]) for c, _ in sel),
                              b"".join(bytes.fromhex(c["signature"]) for c, _ in sel),
                              b"".join(int(c["domain"]).to_bytes(8, "big") for c, _ in sel))
    assert list(got) == [e for _, e in sel], n
vms = [(c, c["expected"]) for c in gb["verify_multiple"] if len(c["pubkeys"]) == len(c["messages"])]
vms += [(c, c["expected_pyecc"]) for c in tor["verify_multiple"]]
off, pks, msgs, sigs, doms = [0], b"", b"", b"", b""
for c, _ in vms:
    pks += b"".join(bytes.fromhex(p) for p in c["pubkeys"]); msgs += b"".join(bytes.fromhex(m) for m in c["messages"])
    sigs += bytes.fromhex(c["signature"]); doms += int(c["domain"]).to_bytes(8, "big")
    off.append(off[-1] + len(c["pubkeys"]))
assert list(native.verify_multiple_batch(np.array(off, dtype=np.uint32), pks, msgs, 32, sigs, doms)) == [e for _, e in vms]
print("octet fe ok")
"""


@pytest.mark.parametrize("knob", ["BLS381_FE_OCT=2", "BLS381_ML_OCTET=0", "BLS381_HASH_OCT=0"])
def test_octet_final_exponentiation_knob(knob):
    """The latency path's non-default layouts, each read once per process (so in a child
    process), give the fixture verdicts for bls_verify batches (one and two values per item) and
    verify_multiple batches: BLS381_FE_OCT=2 (k_final_exp_verdict_oq<.., 0>: products split over
    the octet, squarings on quads), BLS381_ML_OCTET=0 (the quad Miller kernels k_miller_verify_o
    and k_miller_tasks<4> for small nf), BLS381_HASH_OCT=0 (k_hash_g2_q, the cofactor map on
    quads).  The defaults (FE_OCT=3, ML_OCTET=1, HASH_OCT=1) run in every other test."""
    import subprocess
    var, val = knob.split("=")
    env = dict(os.environ, **{var: val})
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _OCT_SCRIPT, root], env=env, capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0 and "octet fe ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


# ------------------------------- full-size C3 epoch
def test_c3_full_epoch_three_forms_agree(native):
    """The mainnet-preset epoch at full size: 1,024 committees x 128 members drawn from 8,192
    validators (privkeys 1..8192, helpers/keys.py's small-integer keys), each attestation checked
    the way validate_indexed_attestation does it (0_beacon-chain.md:1023-1034):
    bls_aggregate_pubkeys(committee), bls_aggregate_pubkeys([]) (custody bit 1 is always empty in
    phase 0) and bls_verify_multiple([agg, agg_inf], [m0, m1], sig, DOMAIN_ATTESTATION), with
    1/16 of the attestations signed over a different m0.  The two-call form (aggregates left in
    HBM, then the verify batch), the grouped call and the grouped call over a registry must agree
    call by call with the construction; the oracle re-derives the aggregates and the verdicts of
    four attestations: a valid one, a tampered one, and the infinity aggregate of the empty group."""
    import ctypes
    import torch
    from bls381_amd.registry import PubkeyRegistry
    L = native.lib()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    t = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)
    nv, nc, cs = 8192, 1024, 128
    sk = list(range(1, nv + 1))
    pks = native.privtopub_batch(b"".join(k.to_bytes(32, "big") for k in sk))
    rng = np.random.default_rng(0xB15_0003)
    idx = np.stack([rng.choice(nv, cs, replace=False) for _ in range(nc)]).reshape(-1)
    pk_arr = np.frombuffer(pks, dtype=np.uint8).reshape(nv, 48)
    offsets = np.repeat(np.arange(0, nc * cs + 1, cs, dtype=np.uint32), 2)[1:]   # groups 2c, 2c+1 (empty)
    m0 = bytearray(rng.bytes(32 * nc))
    m1 = rng.bytes(32 * nc)
    ssum = [int(sum(sk[j] for j in idx[c * cs:(c + 1) * cs])) % O.r for c in range(nc)]
    sigs = native.sign_batch(bytes(m0), b"".join(k.to_bytes(32, "big") for k in ssum), (2).to_bytes(8, "big") * nc)
    expected = np.ones(nc, dtype=bool)
    for c in range(5, nc, 16):
        m0[32 * c + 7] ^= 0x80
        expected[c] = False
    msgs = b"".join(bytes(m0[32 * c:32 * c + 32]) + m1[32 * c:32 * c + 32] for c in range(nc))
    call_off = np.arange(0, 2 * nc + 1, 2, dtype=np.uint32)
    doms = (2).to_bytes(8, "big") * nc
    d_cpks, d_sigs, d_doms = t(pk_arr[idx].tobytes()), t(sigs), t(doms)
    cvp = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    sp = ctypes.c_void_p(stream.cuda_stream)
    # two calls: aggregates in HBM, then the verify_multiple batch over them
    d_out = torch.zeros(2 * nc * 48, dtype=torch.uint8, device=dev)
    d_st = torch.zeros(2 * nc, dtype=torch.int32, device=dev)
    aws = torch.empty(L.bls381_aggregate_pubkeys_batch_workspace_size(2 * nc, nc * cs), dtype=torch.uint8, device=dev)
    native.check(L.bls381_aggregate_pubkeys_batch_device(2 * nc, cvp(offsets), nc * cs, d_cpks.data_ptr(),
                                                         d_out.data_ptr(), d_st.data_ptr(), aws.data_ptr(), sp))
    d_v1 = torch.zeros(nc, dtype=torch.uint8, device=dev)
    vws = torch.empty(L.bls381_verify_multiple_batch_workspace_size(nc, 2 * nc, 32), dtype=torch.uint8, device=dev)
    native.check(L.bls381_verify_multiple_batch_device(nc, cvp(call_off), msgs, 32, d_out.data_ptr(), d_sigs.data_ptr(),
                                                       d_doms.data_ptr(), d_v1.data_ptr(), vws.data_ptr(), sp))
    # one grouped call, and the same over a registry of the 8,192 keys
    gws = torch.empty(L.bls381_verify_multiple_grouped_workspace_size(nc, 2 * nc, nc * cs, 32), dtype=torch.uint8,
                      device=dev)
    d_v2 = torch.zeros(nc, dtype=torch.uint8, device=dev)
    native.check(L.bls381_verify_multiple_grouped_device(nc, cvp(call_off), 2 * nc, cvp(offsets), msgs, 32,
                                                         d_cpks.data_ptr(), d_sigs.data_ptr(), d_doms.data_ptr(),
                                                         d_v2.data_ptr(), gws.data_ptr(), sp))
    reg = PubkeyRegistry(nv)
    try:
        ent = reg.add([pks[48 * i:48 * i + 48] for i in range(nv)])
        assert np.all(ent >= 0)
        d_ent = t(ent[idx].astype(np.uint32).tobytes())
        d_v3 = torch.zeros(nc, dtype=torch.uint8, device=dev)
        native.check(L.bls381_registry_verify_multiple_grouped_device(
            reg._h, nc, cvp(call_off), 2 * nc, cvp(offsets), msgs, 32, d_ent.data_ptr(), d_sigs.data_ptr(),
            d_doms.data_ptr(), d_v3.data_ptr(), gws.data_ptr(), sp))
        torch.cuda.synchronize()
        v3 = d_v3.cpu().numpy().astype(bool)
    finally:
        reg.close()
    torch.cuda.synchronize()
    assert int(d_st.abs().sum().item()) == 0
    v1, v2 = d_v1.cpu().numpy().astype(bool), d_v2.cpu().numpy().astype(bool)
    assert np.array_equal(v1, expected) and np.array_equal(v2, expected) and np.array_equal(v3, expected)
    aggs = d_out.cpu().numpy().tobytes()
    inf = bytes([0xC0]) + bytes(47)
    for c in (0, 5, 21, 1023):            # valid, tampered (c % 16 == 5), tampered, valid
        agg, agg1 = aggs[96 * c:96 * c + 48], aggs[96 * c + 48:96 * c + 96]
        members = [pks[48 * j:48 * j + 48] for j in idx[c * cs:(c + 1) * cs]]
        assert agg == O.aggregate_pubkeys(members) and agg1 == O.aggregate_pubkeys([]) == inf, c
        want = O.verify_multiple([agg, agg1], [msgs[64 * c:64 * c + 32], msgs[64 * c + 32:64 * c + 64]],
                                 sigs[96 * c:96 * c + 96], 2)
        assert want == bool(expected[c]), c


# ------------------------------ the boundary's residual py_ecc behaviours
@pytest.mark.parametrize("policy", ["pyecc", "strict"])
def test_shim_lengths_and_domain_order(native, noncanon, policy):
    """bls_noncanonical.json shim_* cases through the bls shim under each policy: pubkeys and
    signatures of other lengths (py_ecc reads them as integers; strict: Bytes48 / Bytes96), and
    an out-of-range domain, which py_ecc serialises after the decodes preceding hash_to_G2."""
    from bls381_amd import bls
    col, ocol = "expected_" + policy, "output_" + policy

    def outcome(fn, *a):
        try:
            return fn(*a)
        except (OverflowError, bls.ValidationError) as e:
            return type(e).__name__

    old = bls.SUBGROUP_POLICY
    bls.SUBGROUP_POLICY = policy
    try:
        for c in noncanon["shim_verify"]:
            got = outcome(bls.bls_verify, bytes.fromhex(c["pubkey"]), bytes.fromhex(c["message"]),
                          bytes.fromhex(c["signature"]), int(c["domain"]))
            assert got == c[col], (c["kind"], got)
        for c in noncanon["shim_verify_multiple"]:
            got = outcome(bls.bls_verify_multiple, [bytes.fromhex(p) for p in c["pubkeys"]],
                          [bytes.fromhex(m) for m in c["messages"]], bytes.fromhex(c["signature"]), int(c["domain"]))
            assert got == c[col], (c["kind"], got)
            if col == "expected_pyecc" and "pyecc_order_dependent" in c:
                # py_ecc itself may give either outcome (set order); the shim's is one of them
                assert got in c["pyecc_order_dependent"], (c["kind"], got)
        for name, fn in (("shim_aggregate_pubkeys", bls.bls_aggregate_pubkeys),
                         ("shim_aggregate_sigs", bls.bls_aggregate_signatures)):
            for c in noncanon[name]:
                try:
                    got = fn([bytes.fromhex(x) for x in c["input"]]).hex()
                except ValueError:
                    got = None
                assert got == c[ocol], (name, c["kind"])
    finally:
        bls.SUBGROUP_POLICY = old


def test_shim_call_keeps_process_policy(native):
    """a process-wide 'strict' policy set by another front end survives a shim call
    that reaches the device (the shim stays on 'pyecc' and scopes it to the call)."""
    from bls381_amd import _native, bls
    msg = bytes(range(32))
    sk = 0x1234567
    pk, sig = bls.privtopub(sk), bls.bls_sign(msg, sk, 3)
    assert bls.SUBGROUP_POLICY == "pyecc"
    _native.set_subgroup_policy("strict")
    try:
        assert bls.bls_verify(pk, msg, sig, 3) is True
        assert bls.bls_verify_multiple([pk], [msg], sig, 3) is True
        assert _native.get_subgroup_policy() == "strict"
        assert _native.get_thread_subgroup_policy() == "strict"
    finally:
        _native.set_subgroup_policy("pyecc")
