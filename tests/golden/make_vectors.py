"""Generate the committed golden fixtures under tests/golden/ from the oracle.

* bls_vectors.json -- the 94 `test_generators/bls` cases (reference
  `test_generators/bls/main.py:33-158`): same DOMAINS (:33-39), MESSAGES (:41-45),
  PRIVKEYS (:47-53), same case loops and the same hex encodings
  (`int_to_hex`, :19-23; 48-byte coordinates, :68-69,85).  py_ecc is absent, so
  outputs come from oracle/bls_oracle.py (a restatement of py_ecc 1.7.0).
* bls_golden_batches.json -- small synthetic verify / verify_multiple /
  aggregate sets with verdicts and edge cases (SURVEY.md §8c "Fixtures to commit").

Run:  python tests/golden/make_vectors.py   (about a minute on one core)
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import bls_oracle as o  # noqa: E402

DOMAINS = [0, 1, 1234, 2 ** 32 - 1, 2 ** 64 - 1]
MESSAGES = [b"\x00" * 32, b"\x56" * 32, b"\xab" * 32]
PRIVKEYS = [
    0x263dbd792f5b1be47ed85f8938c0f29586af0d3ac7b977f21c278fe1462040e3,
    0x47b8192d77bf871b62e87859d653922725724a5c031afeabc60bcef5ff665138,
    0x328388aff0d4a5b7dc9205abd374e7e98f3cd9f3418edb4eafda5fb16473d216,
]


def int_to_hex(n, byte_length=None):
    # eth_utils.int_to_big_endian: minimal big-endian, b'\x00' for zero
    bv = n.to_bytes(max(1, (n.bit_length() + 7) // 8), "big")
    if byte_length:
        bv = bv.rjust(byte_length, b"\x00")
    return "0x" + bv.hex()


def gen_reference_cases():
    cases = {"msg_hash_g2_uncompressed": [], "msg_hash_g2_compressed": [], "priv_to_pub": [],
             "sign_msg": [], "aggregate_sigs": [], "aggregate_pubkeys": []}
    hashes = {}
    for msg in MESSAGES:
        for domain in DOMAINS:
            h = o.hash_to_G2(msg, domain)
            hashes[(msg, domain)] = h
            cases["msg_hash_g2_uncompressed"].append({
                "input": {"message": "0x" + msg.hex(), "domain": int_to_hex(domain)},
                "output": o.g2_projective_to_hex(h)})
    for msg in MESSAGES:
        for domain in DOMAINS:
            z1, z2 = o.compress_G2(hashes[(msg, domain)])
            cases["msg_hash_g2_compressed"].append({
                "input": {"message": "0x" + msg.hex(), "domain": int_to_hex(domain)},
                "output": [int_to_hex(z1, 48), int_to_hex(z2, 48)]})
    pubkeys = [o.privtopub(k) for k in PRIVKEYS]
    for k, pk in zip(PRIVKEYS, pubkeys):
        cases["priv_to_pub"].append({"input": int_to_hex(k), "output": "0x" + pk.hex()})
    sigs = {}
    for k in PRIVKEYS:
        for msg in MESSAGES:
            for domain in DOMAINS:
                s = o.sign(msg, k, domain)
                sigs[(k, msg, domain)] = s
                cases["sign_msg"].append({
                    "input": {"privkey": int_to_hex(k), "message": "0x" + msg.hex(),
                              "domain": int_to_hex(domain)},
                    "output": "0x" + s.hex()})
    for domain in DOMAINS:
        for msg in MESSAGES:
            ss = [sigs[(k, msg, domain)] for k in PRIVKEYS]
            cases["aggregate_sigs"].append({
                "input": ["0x" + s.hex() for s in ss],
                "output": "0x" + o.aggregate_signatures(ss).hex()})
    cases["aggregate_pubkeys"].append({
        "input": ["0x" + p.hex() for p in pubkeys],
        "output": "0x" + o.aggregate_pubkeys(pubkeys).hex()})
    return cases


def gen_golden_batches(seed=0xB15_0001):
    rng = random.Random(seed)
    out = {"verify": [], "verify_multiple": [], "aggregate_pubkeys": [], "aggregate_sigs": [],
           "hash_to_g2": [], "invalid_g1": [], "invalid_g2": []}
    # --- bls_verify: valid items and tampered variants (SURVEY §8d C2 tamper classes)
    base = []
    for i in range(16):
        sk = rng.randrange(1, o.r)
        msg = bytes(rng.getrandbits(8) for _ in range(32))
        dom = rng.choice([0, 1, 2, 3, 2 ** 32 - 1, 2 ** 64 - 1, rng.getrandbits(64)])
        pk = o.privtopub(sk)
        sig = o.sign(msg, sk, dom)
        base.append((sk, msg, dom, pk, sig))
    items = []
    for i, (sk, msg, dom, pk, sig) in enumerate(base):
        items.append(("valid", pk, msg, sig, dom))
    for i, (sk, msg, dom, pk, sig) in enumerate(base[:12]):
        kind = i % 6
        if kind == 0:
            m2 = bytearray(msg); m2[rng.randrange(32)] ^= 1 << rng.randrange(8)
            items.append(("msg_bitflip", pk, bytes(m2), sig, dom))
        elif kind == 1:
            items.append(("sig_swap", pk, msg, base[(i + 1) % len(base)][4], dom))
        elif kind == 2:
            items.append(("zero_sig", pk, msg, b"\x00" * 96, dom))
        elif kind == 3:
            items.append(("domain_change", pk, msg, sig, (dom + 1) % 2 ** 64))
        elif kind == 4:
            items.append(("pk_swap", base[(i + 1) % len(base)][3], msg, sig, dom))
        else:
            s2 = bytearray(sig); s2[95] ^= 0x01
            items.append(("sig_bitflip", pk, msg, bytes(s2), dom))
    inf_pk = bytes([0xC0]) + b"\x00" * 47
    inf_sig = bytes([0xC0]) + b"\x00" * 95
    items.append(("inf_pk_inf_sig", inf_pk, base[0][1], inf_sig, 5))
    items.append(("inf_pk_valid_sig", inf_pk, base[0][1], base[0][4], base[0][2]))
    items.append(("valid_pk_inf_sig", base[0][3], base[0][1], inf_sig, base[0][2]))
    items.append(("stub_pk_stub_sig", b"\x22" * 48, base[0][1], b"\x11" * 96, 0))
    items.append(("zero_pk", b"\x00" * 48, base[0][1], base[0][4], base[0][2]))
    pk_x_ge_q = (0x80 | (o.q >> 376)).to_bytes(1, "big") + (o.q % 2 ** 376).to_bytes(47, "big")
    items.append(("pk_x_eq_q", pk_x_ge_q, base[0][1], base[0][4], base[0][2]))
    for kind, pk, msg, sig, dom in items:
        out["verify"].append({"kind": kind, "pubkey": pk.hex(), "message": msg.hex(),
                              "signature": sig.hex(), "domain": str(dom),
                              "expected": o.verify(msg, pk, sig, dom),
                              "expected_strict": o.verify_strict(msg, pk, sig, dom)})
    # --- bls_verify_multiple
    vm = []
    # attestation shape: [agg(committee), inf], [m0, m1]
    sks = [rng.randrange(1, o.r) for _ in range(5)]
    pks = [o.privtopub(k) for k in sks]
    m0 = bytes(rng.getrandbits(8) for _ in range(32))
    m1 = bytes(rng.getrandbits(8) for _ in range(32))
    d = 2
    agg_sig = o.aggregate_signatures([o.sign(m0, k, d) for k in sks])
    agg_pk = o.aggregate_pubkeys(pks)
    vm.append(("attestation", [agg_pk, inf_pk], [m0, m1], agg_sig, d))
    vm.append(("attestation_bad_domain", [agg_pk, inf_pk], [m0, m1], agg_sig, 3))
    # distinct messages, one key each
    msgs = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(4)]
    sig4 = o.aggregate_signatures([o.sign(m, k, 1) for m, k in zip(msgs, sks[:4])])
    vm.append(("distinct_4", pks[:4], msgs, sig4, 1))
    vm.append(("distinct_4_swapped_pks", [pks[1], pks[0], pks[2], pks[3]], msgs, sig4, 1))
    # repeated message groups (grouping by message)
    msgs_r = [msgs[0], msgs[1], msgs[0], msgs[1], msgs[0]]
    sig_r = o.aggregate_signatures([o.sign(m, k, 7) for m, k in zip(msgs_r, sks)])
    vm.append(("grouped_5", pks, msgs_r, sig_r, 7))
    vm.append(("empty_inf_sig", [], [], inf_sig, 0))
    vm.append(("empty_valid_sig", [], [], base[0][4], 0))
    vm.append(("zero_sig", pks[:2], msgs[:2], b"\x00" * 96, 1))
    vm.append(("bad_pk", [pks[0], b"\x00" * 48], msgs[:2], sig4, 1))
    for kind, pkl, ml, sig, dom in vm:
        out["verify_multiple"].append({
            "kind": kind, "pubkeys": [p.hex() for p in pkl], "messages": [m.hex() for m in ml],
            "signature": sig.hex(), "domain": str(dom),
            "expected": o.verify_multiple(pkl, ml, sig, dom),
            "expected_strict": (o.verify_multiple_strict(pkl, ml, sig, dom) if len(pkl) == len(ml) else None)})
    # --- aggregates, including cancellation to infinity and doubling
    g1 = o.privtopub(1)
    neg_g1 = o.G1_to_pubkey(o.pt_neg(o.FqOps, o.G1))
    agg_cases = [("empty", []), ("single", [pks[0]]), ("five", pks), ("cancel", [g1, neg_g1]),
                 ("double", [pks[0], pks[0]]), ("with_inf", [pks[0], inf_pk, pks[1]]),
                 ("all_inf", [inf_pk, inf_pk])]
    for kind, pkl in agg_cases:
        out["aggregate_pubkeys"].append({"kind": kind, "input": [p.hex() for p in pkl],
                                         "output": o.aggregate_pubkeys(pkl).hex()})
    sigs5 = [o.sign(m0, k, d) for k in sks]
    neg_s = o.G2_to_signature(o.pt_neg(o.Fq2Ops, o.signature_to_G2(sigs5[0])))
    sagg = [("empty", []), ("single", sigs5[:1]), ("five", sigs5), ("cancel", [sigs5[0], neg_s]),
            ("double", [sigs5[1], sigs5[1]]), ("with_inf", [sigs5[0], inf_sig])]
    for kind, sl in sagg:
        out["aggregate_sigs"].append({"kind": kind, "input": [s.hex() for s in sl],
                                      "output": o.aggregate_signatures(sl).hex()})
    # --- extra hash_to_G2 points (affine + compressed), random messages/domains
    for i in range(16):
        msg = bytes(rng.getrandbits(8) for _ in range(32))
        dom = rng.getrandbits(64)
        x, y, trials = o.hash_to_G2_affine_candidate(msg, dom)
        h = o.hash_to_G2(msg, dom)
        (xr, xi), (yr, yi) = o.g2_affine(h)
        out["hash_to_g2"].append({"message": msg.hex(), "domain": str(dom), "trials": trials,
                                  "affine": [hex(xr), hex(xi), hex(yr), hex(yi)],
                                  "compressed": o.G2_to_signature(h).hex()})
    # --- encodings both codecs reject (aggregate raises under either policy); the
    # encodings only the strict codec rejects are in bls_noncanonical.json
    bad_g1 = []
    # x with no square root: search deterministically
    xx = 1
    while True:
        rhs = (xx ** 3 + 4) % o.q
        if pow(rhs, (o.q - 1) // 2, o.q) != 1:
            break
        xx += 1
    bad_g1.append((2 ** 383 + xx).to_bytes(48, "big"))
    bad_g1.append((xx).to_bytes(48, "big"))                 # c_flag clear as well
    if xx + o.q < 2 ** 381:
        bad_g1.append((2 ** 383 + xx + o.q).to_bytes(48, "big"))   # x + q: the same x mod q
    for b in bad_g1:
        out["invalid_g1"].append(b.hex())
    # G2: an x whose x^3 + 4(1 + i) has no square root in Fp2, canonical and not
    xi = 1
    while o.modular_squareroot(o.f2_add(o.f2_mul(o.f2_sqr((0, xi)), (0, xi)), o.B2)) is not None:
        xi += 1
    bad_g2 = [(2 ** 383 + xi).to_bytes(48, "big") + b"\x00" * 48,
              (xi).to_bytes(48, "big") + (o.q).to_bytes(48, "big")]
    for b in bad_g2:
        for strict in (False, True):
            try:
                o.signature_to_G2(b, strict)
                raise AssertionError("expected undecodable")
            except ValueError:
                pass
        out["invalid_g2"].append(b.hex())
    return out


def main():
    ref = gen_reference_cases()
    with open(os.path.join(HERE, "bls_vectors.json"), "w") as f:
        json.dump(ref, f, indent=1)
    print("bls_vectors.json:", {k: len(v) for k, v in ref.items()},
          "total", sum(len(v) for v in ref.values()))
    gb = gen_golden_batches()
    with open(os.path.join(HERE, "bls_golden_batches.json"), "w") as f:
        json.dump(gb, f, indent=1)
    print("bls_golden_batches.json:", {k: len(v) for k, v in gb.items()})


if __name__ == "__main__":
    main()
