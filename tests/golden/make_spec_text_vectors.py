"""Pin the oracle's hash_to_G2 / modular_squareroot to the reference's own spec text.

The reference holds no BLS vectors and py_ecc 1.7.0 is absent, so the oracle
(oracle/bls_oracle.py) is a restatement.  This script takes the executable part of the
reference's text mechanically: the ```python blocks of specs/bls_signature.md:68-108 (the
`hash_to_G2` and `modular_squareroot` sections), pulled by the reference's own extractor,
scripts/function_puller.py:12-83 (get_spec), and runs them unmodified over a minimal Fq2
(the spec's `Fq2([re, im])` with `**`, `*`, `/`, `+`, `-`, `==`, `.coeffs`).  What the text
leaves undefined is supplied here and named in the output:
  * hash      = SHA-256 (specs/core/0_beacon-chain.md:591-595)
  * bytes8    = int.to_bytes(8, DOMAIN_BYTEORDER): the spec does not say which byte order;
                SURVEY.md A.2 (py_ecc 1.7.0) says big-endian, the oracle's single switch
  * multiply_in_G2(P, k) = [k]P on E'(Fp2) (normalised affine out; the oracle's projective
                formulas, so only the point is compared, not py_ecc's raw triple)
  * coerce_to_int = the canonical integer of an Fq element (bls_signature.md:94)

get_spec() itself stops on this file: every block of bls_signature.md opens with constants
(`G2_cofactor = ...`, `Fq2_order = ...`) before its `def`, and get_spec reads `is_ssz`
before its first `def` / `class` line sets it (UnboundLocalError at function_puller.py:63).
The script then applies get_spec's own fence rule (lines starting '```python' open a block,
'```' closes it, function_puller.py:40-44) and records that it did.

Output: tests/golden/spec_text_hash.json -- for the 15 test_generators/bls message x domain
inputs (main.py:33-45) and the golden-batch messages: the spec text's hash_to_G2 point
(affine, both byte orders), and modular_squareroot outputs on fixed inputs.  The CPU test
tests/test_oracle_known_answers.py::test_oracle_matches_spec_text compares the oracle with
it; nothing at test time reads /root/reference.

Run (in the build container, where /root/reference exists):
    python tests/golden/make_spec_text_vectors.py
"""
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("BLS381_REFERENCE", "/root/reference")
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import bls_oracle as o  # noqa: E402

SPEC = os.path.join(REF, "specs", "bls_signature.md")
DOMAINS = [0, 1, 1234, 2 ** 32 - 1, 2 ** 64 - 1]          # test_generators/bls/main.py:33-39
MESSAGES = [b"\x00" * 32, b"\x56" * 32, b"\xab" * 32]       # main.py:41-45


def pull_blocks():
    """The spec's python blocks, by the reference's extractor (or its fence rule, see above)."""
    sys.path.insert(0, os.path.join(REF, "scripts"))
    import function_puller
    try:
        functions, constants, _, _ = function_puller.get_spec(SPEC)
        return "\n".join(functions.values()), "function_puller.get_spec"
    except UnboundLocalError as e:
        note = "function_puller.get_spec raised UnboundLocalError (%s); its fence rule applied" % e
    blocks, cur = [], None
    for line in open(SPEC).readlines():
        line = line.rstrip()
        if line[:9] == "```python":
            cur = []
        elif line[:3] == "```":
            if cur is not None:
                blocks.append("\n".join(cur))
            cur = None
        elif cur is not None:
            cur.append(line)
    return "\n\n".join(blocks), note


class Fq2:
    """Minimal Fq2 = Fq[i]/(i^2 + 1) with the interface the spec text uses."""
    def __init__(self, coeffs):
        self.coeffs = (coeffs[0] % o.q, coeffs[1] % o.q)

    def _t(self):
        return self.coeffs

    def __add__(self, b):
        return Fq2(o.f2_add(self.coeffs, b.coeffs))

    def __sub__(self, b):
        return Fq2(o.f2_sub(self.coeffs, b.coeffs))

    def __neg__(self):
        return Fq2(o.f2_neg(self.coeffs))

    def __mul__(self, b):
        return Fq2(o.f2_mul(self.coeffs, b.coeffs))

    def __truediv__(self, b):
        return Fq2(o.f2_mul(self.coeffs, o.f2_inv(b.coeffs)))

    def __pow__(self, e):
        return Fq2(o.f2_pow(self.coeffs, e))

    def __eq__(self, b):
        return isinstance(b, Fq2) and self.coeffs == b.coeffs

    def __hash__(self):
        return hash(self.coeffs)


def run_spec(code, byteorder):
    ns = {
        "Fq2": Fq2, "Bytes32": bytes, "uint64": int, "uint384": int,
        "hash": lambda b: hashlib.sha256(b).digest(),
        "bytes8": lambda d: int(d).to_bytes(8, byteorder),
        "coerce_to_int": lambda e: int(e),
    }

    def multiply_in_G2(pt, k):
        x, y = pt
        p = o.pt_multiply(o.Fq2Ops, (x.coeffs, y.coeffs, o.FQ2_ONE), k)
        return o.pt_normalize(o.Fq2Ops, p)

    ns["multiply_in_G2"] = multiply_in_G2
    exec(compile(code, SPEC, "exec"), ns)   # noqa: S102 -- the reference's own spec text
    return ns


def main():
    code, how = pull_blocks()
    golden = json.load(open(os.path.join(HERE, "bls_golden_batches.json")))
    msgs = MESSAGES + sorted({bytes.fromhex(c["message"]) for c in golden["verify"]
                              if len(bytes.fromhex(c["message"])) == 32})[:12]
    out = {"source": "specs/bls_signature.md:68-108 python blocks (%s)" % how,
           "supplied": {"hash": "sha256", "bytes8": "int.to_bytes(8, byteorder), both orders recorded",
                        "multiply_in_G2": "[k]P, affine out", "coerce_to_int": "canonical integer"},
           "hash_to_G2": [], "modular_squareroot": []}
    spec = {bo: run_spec(code, bo) for bo in ("big", "little")}
    for m in msgs:
        for d in DOMAINS:
            row = {"message": m.hex(), "domain": str(d)}
            for bo, ns in spec.items():
                (xr, xi), (yr, yi) = ns["hash_to_G2"](m, d)
                row["affine_" + bo] = [hex(xr), hex(xi), hex(yr), hex(yi)]
            out["hash_to_G2"].append(row)
            print("hash_to_G2", m.hex()[:8], d, row["affine_big"][0][:12], flush=True)
    rng = random.Random(0xB15_5EC7)
    for _ in range(24):
        v = (rng.randrange(o.q), rng.randrange(o.q))
        r = spec["big"]["modular_squareroot"](Fq2(v))
        out["modular_squareroot"].append({"input": [hex(v[0]), hex(v[1])],
                                          "output": None if r is None else [hex(r.coeffs[0]), hex(r.coeffs[1])]})
    with open(os.path.join(HERE, "spec_text_hash.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("spec_text_hash.json:", len(out["hash_to_G2"]), "hash cases,", len(out["modular_squareroot"]), "roots;", how)


if __name__ == "__main__":
    main()
