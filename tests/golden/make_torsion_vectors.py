"""Generate tests/golden/bls_torsion.json: on-curve points outside G1 / G2.

py_ecc 1.7.0 decodes a pubkey or signature onto the curve and never checks its
subgroup (the reference calls it through eth2spec/utils/bls.py:24-31).  The
spec asks for "a valid G1 point" / "a valid G2 point"
(specs/bls_signature.md:135-136,143-144).  The two behaviours differ exactly on
the inputs built here -- points with a component of small order:

* G1 = E(Fp) has cofactor 3 * 11^2 * 10177^2 * 859267^2 * 52437899^2; the
  pubkey 0x80 || 00*47 decodes to (0, 2), a point of order 3.
* G2 = E'(Fp2) has cofactor 13^2 * 23^2 * 2713 * 11953 * 262069 * p; its 13-
  and 23-parts are Z13 x Z13 and Z23 x Z23.

Every case carries two verdict columns:
  expected_pyecc  -- oracle/bls_oracle.py verify / verify_multiple (py_ecc);
  expected_strict -- the same, and False unless every point is in G1 / G2.
Aggregates never check subgroups; their bytes are the oracle's.

Run:  python tests/golden/make_torsion_vectors.py   (about two minutes on one core)
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import bls_oracle as o  # noqa: E402

q, r = o.q, o.r
H1 = (o.BLS_X - 1) ** 2 // 3
N1 = H1 * r                      # #E(Fp)
N2 = o.G2_cofactor * r           # #E'(Fp2)
F1, F2 = o.FqOps, o.Fq2Ops


def _strip(n, p):
    while n % p == 0:
        n //= p
    return n


def _rand_g1(rng):
    while True:
        x = rng.randrange(q)
        rhs = (x ** 3 + 4) % q
        y = pow(rhs, (q + 1) // 4, q)
        if y * y % q == rhs:
            return (x, y, 1)


def _rand_g2(rng):
    while True:
        x = (rng.randrange(q), rng.randrange(q))
        y = o.modular_squareroot(o.f2_add(o.f2_mul(o.f2_sqr(x), x), o.B2))
        if y is not None:
            return (x, y, o.FQ2_ONE)


def torsion_point(F, rand, N, p, rng):
    """A point of order exactly p (prime): a random point times N with p stripped,
    then times p until one more multiple by p would give infinity."""
    while True:
        t = o.pt_multiply(F, rand(rng), _strip(N, p))
        if o.pt_is_inf(F, t):
            continue
        while not o.pt_is_inf(F, o.pt_multiply(F, t, p)):
            t = o.pt_multiply(F, t, p)
        return t


def main():
    rng = random.Random(0xB15_7013)
    d = 3
    m = bytes(rng.getrandbits(8) for _ in range(32))
    m2 = bytes(rng.getrandbits(8) for _ in range(32))
    G = o.G1
    pk_of = lambda pt: o.G1_to_pubkey(pt)
    sig_of = lambda pt: o.G2_to_signature(pt)
    add1 = lambda a, b: o.pt_add(F1, a, b)
    add2 = lambda a, b: o.pt_add(F2, a, b)
    T3 = (0, 2, 1)                                   # pubkey 0x80 || 00*47
    assert pk_of(T3) == bytes([0x80]) + bytes(47)
    T11 = torsion_point(F1, _rand_g1, N1, 11, rng)
    T10177 = torsion_point(F1, _rand_g1, N1, 10177, rng)
    T13 = [torsion_point(F2, _rand_g2, N2, 13, rng) for _ in range(3)]
    T23 = [torsion_point(F2, _rand_g2, N2, 23, rng) for _ in range(2)]
    T2713 = torsion_point(F2, _rand_g2, N2, 2713, rng)
    P = lambda k: o.pt_multiply(F1, G, k)
    S = lambda k, msg=m: o.signature_to_G2(o.sign(msg, k, d))
    inf_pk, inf_sig = pk_of(o.Z1), sig_of(o.Z2)

    verify_cases = [
        ("pk_order3_sig_inf", pk_of(T3), m, inf_sig),
        ("pk_order3_sig_valid", pk_of(T3), m, sig_of(S(1))),
        ("pk_G_plus_T3", pk_of(add1(G, T3)), m, sig_of(S(1))),
        ("pk_5G_plus_T11", pk_of(add1(P(5), T11)), m, sig_of(S(5))),
        ("pk_7G_plus_T10177", pk_of(add1(P(7), T10177)), m, sig_of(S(7))),
        ("pk_T11_sig_inf", pk_of(T11), m, inf_sig),
        ("pk_G_plus_T3_wrong_msg", pk_of(add1(G, T3)), m2, sig_of(S(1))),
        ("pk_5G_plus_T3_sig_plus_T13", pk_of(add1(P(5), T3)), m, sig_of(add2(S(5), T13[0]))),
        ("sig_plus_T13_a", o.privtopub(5), m, sig_of(add2(S(5), T13[0]))),
        ("sig_plus_T13_b", o.privtopub(5), m, sig_of(add2(S(5), T13[1]))),
        ("sig_plus_T23", o.privtopub(5), m, sig_of(add2(S(5), T23[0]))),
        ("sig_plus_T2713", o.privtopub(5), m, sig_of(add2(S(5), T2713))),
        ("sig_T13_pk_inf", inf_pk, m, sig_of(T13[0])),          # degenerate Miller loop
        ("sig_T13c_pk_inf", inf_pk, m, sig_of(T13[2])),
        ("sig_T13_pk_valid", o.privtopub(5), m, sig_of(T13[1])),
        ("sig_T23_pk_inf", inf_pk, m, sig_of(T23[0])),
        ("sig_T23_pk_valid", o.privtopub(5), m, sig_of(T23[1])),
        ("sig_T2713_pk_inf", inf_pk, m, sig_of(T2713)),
        ("sig_T13_plus_T23_pk_inf", inf_pk, m, sig_of(add2(T13[0], T23[0]))),
        ("pk_T3_sig_T13", pk_of(T3), m, sig_of(T13[0])),
        ("control_valid", o.privtopub(5), m, sig_of(S(5))),
        ("control_inf_inf", inf_pk, m, inf_sig),
    ]
    out = {"verify": [], "verify_multiple": [], "aggregate_pubkeys": [], "aggregate_sigs": []}
    for kind, pk, msg, sig in verify_cases:
        out["verify"].append({"kind": kind, "pubkey": pk.hex(), "message": msg.hex(), "signature": sig.hex(),
                              "domain": str(d), "expected_pyecc": o.verify(msg, pk, sig, d),
                              "expected_strict": o.verify_strict(msg, pk, sig, d)})
        print("verify", kind, out["verify"][-1]["expected_pyecc"], out["verify"][-1]["expected_strict"], flush=True)

    agg_sig_11 = o.aggregate_signatures([o.sign(m, 11, d), o.sign(m, 12, d)])
    agg_sig_2m = o.aggregate_signatures([o.sign(m, 11, d), o.sign(m2, 12, d)])
    vm_cases = [
        ("one_key_G_plus_T3", [pk_of(add1(G, T3))], [m], sig_of(S(1))),
        ("one_key_order3_sig_inf", [pk_of(T3)], [m], inf_sig),
        # torsion cancels in the group sum: py_ecc True, strict False (per-key check)
        ("group_torsion_cancels", [pk_of(add1(P(11), T3)), pk_of(add1(P(12), o.pt_neg(F1, T3)))], [m, m],
         agg_sig_11),
        ("group_torsion_remains", [pk_of(add1(P(11), T3)), pk_of(add1(P(12), T3))], [m, m], agg_sig_11),
        ("two_msgs_one_torsion_key", [pk_of(add1(P(11), T11)), o.privtopub(12)], [m, m2], agg_sig_2m),
        ("attestation_agg_plus_T11", [pk_of(add1(add1(P(11), P(12)), T11)), inf_pk], [m, m2], agg_sig_11),
        ("sig_plus_T13", [o.privtopub(11), o.privtopub(12)], [m, m],
         sig_of(add2(o.signature_to_G2(agg_sig_11), T13[0]))),
        ("empty_sig_T13", [], [], sig_of(T13[0])),            # degenerate Miller loop
        ("empty_sig_T23", [], [], sig_of(T23[0])),
        ("control_valid", [o.privtopub(11), o.privtopub(12)], [m, m], agg_sig_11),
    ]
    for kind, pks, msgs, sig in vm_cases:
        out["verify_multiple"].append({
            "kind": kind, "pubkeys": [p.hex() for p in pks], "messages": [x.hex() for x in msgs],
            "signature": sig.hex(), "domain": str(d),
            "expected_pyecc": o.verify_multiple(pks, msgs, sig, d),
            "expected_strict": o.verify_multiple_strict(pks, msgs, sig, d)})
        c = out["verify_multiple"][-1]
        print("verify_multiple", kind, c["expected_pyecc"], c["expected_strict"], flush=True)

    aggp = [("T3_and_G", [pk_of(T3), pk_of(G)]), ("T3_x3_is_inf", [pk_of(T3)] * 3),
            ("G_plus_T11_and_T11", [pk_of(add1(G, T11)), pk_of(T11), o.privtopub(9)]),
            ("T10177", [pk_of(T10177)])]
    for kind, pks in aggp:
        out["aggregate_pubkeys"].append({"kind": kind, "input": [p.hex() for p in pks],
                                         "output": o.aggregate_pubkeys(pks).hex()})
    aggs = [("sig_plus_T13_and_T13", [sig_of(add2(S(5), T13[0])), sig_of(T13[0])]),
            ("T13_x13_is_inf", [sig_of(T13[1])] * 13),
            ("T23_and_sig", [sig_of(T23[0]), sig_of(S(3))]), ("T2713", [sig_of(T2713)])]
    for kind, sigs in aggs:
        out["aggregate_sigs"].append({"kind": kind, "input": [s.hex() for s in sigs],
                                      "output": o.aggregate_signatures(sigs).hex()})
    with open(os.path.join(HERE, "bls_torsion.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("bls_torsion.json:", {k: len(v) for k, v in out.items()})


if __name__ == "__main__":
    main()
