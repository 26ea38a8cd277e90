"""Generate tests/golden/ssz_roots.json (SSZ roots).

Roots come from oracle/ssz_oracle.py.  When /root/reference is present, the
reference's own test_libs/pyspec/eth2spec/utils/merkle_minimal.py (pure, hashlib
only) is imported and must agree with the oracle on every merkleize case, and its
zerohashes table is written as the known answers.  (The reference's
ssz_typing.py raises TypeError at import on Python 3.10, so the type layer is
the oracle's restatement of the 0_beacon-chain.md containers.)

Run: python tests/golden/make_ssz_vectors.py
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import ssz_oracle as S  # noqa: E402

REF = "/root/reference/test_libs/pyspec"


def ref_merkle():
    if not os.path.isdir(REF):
        return None
    sys.path.insert(0, REF)
    from eth2spec.utils import merkle_minimal   # pure: hashlib via eth2spec.utils.hash_function
    return merkle_minimal


def rand_value(rng, typ):
    k = typ[0]
    if k == "uint":
        return rng.randrange(1 << (8 * typ[1]))
    if k == "bool":
        return rng.random() < 0.5
    if k == "bytes":
        return bytes(rng.randrange(256) for _ in range(typ[1]))
    return {name: rand_value(rng, t) for name, t in typ[1]}


def main():
    rng = random.Random(0xB15_0007)
    mm = ref_merkle()
    out = {"pinned_by_reference_merkle_minimal": mm is not None}
    zh = [S.ZERO]
    for _ in range(1, 8):
        zh.append(S.merkleize_chunks([zh[-1], zh[-1]]))
    if mm is not None:
        assert [bytes(h) for h in mm.zerohashes[:8]] == zh
    out["zerohashes"] = [h.hex() for h in zh]
    out["merkleize"] = []
    for n in list(range(1, 10)) + [16, 17]:
        chunks = [bytes(rng.randrange(256) for _ in range(32)) for _ in range(n)]
        root = S.merkleize_chunks(chunks)
        if mm is not None:
            assert mm.merkleize_chunks(chunks) == root
        out["merkleize"].append({"chunks": [c.hex() for c in chunks], "root": root.hex()})
    types = {"DepositData": S.DepositData, "AttestationDataAndCustodyBit": S.AttestationDataAndCustodyBit,
             "AttestationData": S.AttestationData, "Crosslink": S.Crosslink, "BeaconBlockHeader": S.BeaconBlockHeader}
    out["roots"] = []
    for name, typ in types.items():
        for j in range(4):
            v = rand_value(rng, typ)
            if j == 0:   # an all-zero value
                v = S_zero(typ)
            case = {"type": name, "serialized": S.serialize(typ, v).hex(),
                    "hash_tree_root": S.hash_tree_root(typ, v).hex()}
            case["signing_root"] = S.signing_root(typ, v).hex()
            out["roots"].append(case)
    with open(os.path.join(HERE, "ssz_roots.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote ssz_roots.json; pinned by reference merkle_minimal:", mm is not None)


def S_zero(typ):
    k = typ[0]
    if k == "uint":
        return 0
    if k == "bool":
        return False
    if k == "bytes":
        return b"\x00" * typ[1]
    return {name: S_zero(t) for name, t in typ[1]}


if __name__ == "__main__":
    main()
