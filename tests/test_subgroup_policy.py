"""Subgroup policy on the CPU: torsion fixtures vs the oracle, and the whole-call
semantics of the device headers (host g++ build) under both policies.

py_ecc 1.7.0 (reference path: eth2spec/utils/bls.py:24-31) never checks that a
point lies in G1 / G2; the spec asks for valid group points
(specs/bls_signature.md:135-136,143-144).  tests/golden/bls_torsion.json holds
both verdict columns; the engine's BLS381_POLICY_PYECC must give the first and
BLS381_POLICY_STRICT the second.  The GPU side of the same check is
tests/test_gpu_parity.py::test_torsion_*.
"""
import ctypes
import os
import subprocess
import sys

import pytest

import bls_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def L():
    import build_native
    return ctypes.CDLL(os.environ.get("BLS381_HOSTCHECK_LIB") or build_native.build_hostcheck())


def _h(s):
    return bytes.fromhex(s)


def test_torsion_fixtures_match_oracle(torsion):
    """Recompute a spread of the committed verdicts (one in three verify cases, every
    verify_multiple case) and every aggregate with the oracle."""
    for c in torsion["verify"][::3]:
        a = (_h(c["message"]), _h(c["pubkey"]), _h(c["signature"]), int(c["domain"]))
        assert O.verify(*a) == c["expected_pyecc"], c["kind"]
        assert O.verify_strict(*a) == c["expected_strict"], c["kind"]
    for c in torsion["verify_multiple"]:
        a = ([_h(p) for p in c["pubkeys"]], [_h(m) for m in c["messages"]], _h(c["signature"]), int(c["domain"]))
        assert O.verify_multiple(*a) == c["expected_pyecc"], c["kind"]
        assert O.verify_multiple_strict(*a) == c["expected_strict"], c["kind"]
    for c in torsion["aggregate_pubkeys"]:
        assert O.aggregate_pubkeys([_h(p) for p in c["input"]]).hex() == c["output"], c["kind"]
    for c in torsion["aggregate_sigs"]:
        assert O.aggregate_signatures([_h(s) for s in c["input"]]).hex() == c["output"], c["kind"]


def test_torsion_fixtures_cover_both_divergences(torsion):
    """The file pins each way the policies differ: True under py_ecc and False under
    strict (G1 torsion), and the degenerate Miller loop of an order-13 signature."""
    kinds = {c["kind"]: c for c in torsion["verify"]}
    assert kinds["pk_order3_sig_inf"]["expected_pyecc"] and not kinds["pk_order3_sig_inf"]["expected_strict"]
    assert kinds["pk_G_plus_T3"]["expected_pyecc"] and not kinds["pk_G_plus_T3"]["expected_strict"]
    assert not kinds["sig_T13_pk_inf"]["expected_pyecc"]
    vm = {c["kind"]: c for c in torsion["verify_multiple"]}
    assert vm["group_torsion_cancels"]["expected_pyecc"] and not vm["group_torsion_cancels"]["expected_strict"]


def _host_verify(L, c, strict):
    m = _h(c["message"])
    return L.hc_verify(_h(c["pubkey"]), m, len(m), _h(c["signature"]), int(c["domain"]).to_bytes(8, "big"), strict)


def _host_verify_multiple(L, c, strict):
    pks = b"".join(_h(p) for p in c["pubkeys"])
    msgs = b"".join(_h(m) for m in c["messages"])
    return L.hc_verify_multiple(len(c["pubkeys"]), pks or None, msgs or None, 32, _h(c["signature"]),
                                int(c["domain"]).to_bytes(8, "big"), strict)


@pytest.mark.parametrize("strict", [0, 1])
def test_host_pipeline_torsion_verdicts(L, torsion, strict):
    """The device headers' pipeline semantics (policy, degenerate loop -> False) on the host."""
    col = "expected_strict" if strict else "expected_pyecc"
    for c in torsion["verify"]:
        assert _host_verify(L, c, strict) == int(c[col]), (c["kind"], strict)
    for c in torsion["verify_multiple"]:
        assert _host_verify_multiple(L, c, strict) == int(c[col]), (c["kind"], strict)


@pytest.mark.parametrize("strict", [0, 1])
def test_host_pipeline_golden_verdicts(L, golden, strict):
    """The golden batches' verdict column of each policy (they differ only on the
    non-canonical encodings the batches hold: the zero key, x = q, the stub encodings)."""
    _, gb = golden
    col = "expected_strict" if strict else "expected"
    for c in gb["verify"]:
        assert _host_verify(L, c, strict) == int(c[col]), c["kind"]
    for c in gb["verify_multiple"]:
        if len(c["pubkeys"]) != len(c["messages"]):
            continue
        assert _host_verify_multiple(L, c, strict) == int(c[col]), c["kind"]


def test_noncanonical_fixtures_match_oracle(noncanon):
    """bls_noncanonical.json recomputed by the oracle: py_ecc's lax codec
    and the spec's strict one (bls_signature.md:47-52,58-64), verdicts and aggregate bytes."""
    for c in noncanon["verify"][::2]:
        a = (_h(c["message"]), _h(c["pubkey"]), _h(c["signature"]), int(c["domain"]))
        assert O.verify(*a) == c["expected_pyecc"], c["kind"]
        assert O.verify_strict(*a) == c["expected_strict"], c["kind"]
    for name, fn in (("aggregate_pubkeys", O.aggregate_pubkeys), ("aggregate_sigs", O.aggregate_signatures)):
        for c in noncanon[name]:
            for strict, col in ((False, "output_pyecc"), (True, "output_strict")):
                try:
                    got = fn([_h(x) for x in c["input"]], strict).hex()
                except ValueError:
                    got = None
                assert got == c[col], (name, c["kind"], col)
    kinds = {c["kind"]: c for c in noncanon["aggregate_pubkeys"]}
    assert kinds["zero_key"]["output_pyecc"] == "80" + "00" * 47 and kinds["zero_key"]["output_strict"] is None
    v = {c["kind"]: c for c in noncanon["verify"]}
    assert v["deposit_pk_c0"]["expected_pyecc"] and not v["deposit_pk_c0"]["expected_strict"]


def test_host_codecs_noncanonical(L, noncanon):
    """The device headers' two decoders (host build) on every non-canonical encoding:
    the lax one gives py_ecc's point (oracle), the strict one rejects what the spec rejects."""
    buf = ctypes.create_string_buffer(192)
    i48 = lambda b: int.from_bytes(b, "big")
    pks = {p for c in noncanon["verify"] for p in [c["pubkey"]]}
    pks |= {p for c in noncanon["aggregate_pubkeys"] for p in c["input"]}
    for hx in sorted(pks):
        b = _h(hx)
        for strict in (False, True):
            try:
                want = O.pubkey_to_G1(b, strict)
                ws = 1 if want[2] == 0 else 0
            except ValueError:
                want, ws = None, 2
            s = L.hc_g1_decompress(b, buf, 0 if strict else 1)
            assert s == ws, (hx, strict)
            if s == 0:
                assert (i48(buf.raw[:48]), i48(buf.raw[48:96])) == (want[0], want[1]), hx
    sigs = {c["signature"] for c in noncanon["verify"]} | {s for c in noncanon["aggregate_sigs"] for s in c["input"]}
    for hx in sorted(sigs):
        b = _h(hx)
        for strict in (False, True):
            try:
                want = O.signature_to_G2(b, strict)
                ws = 1 if want[2] == O.FQ2_ZERO else 0
            except ValueError:
                want, ws = None, 2
            s = L.hc_g2_decompress(b, buf, 0 if strict else 1)
            assert s == ws, (hx, strict)
            if s == 0:
                got = ((i48(buf.raw[:48]), i48(buf.raw[48:96])), (i48(buf.raw[96:144]), i48(buf.raw[144:192])))
                assert got == (want[0], want[1]), hx


def test_host_codecs_fuzz(L):
    """Both host-built decoders against the oracle's codecs on seeded structured encodings
    (tests/codec_fuzz.py: every flag combination, x >= q, x = 0, junk under b_flag, G2 real
    parts with their own top bits set): same status and the same point, both policies."""
    from codec_fuzz import g1_encodings, g2_encodings
    buf = ctypes.create_string_buffer(192)
    i48 = lambda b: int.from_bytes(b, "big")
    seen = set()
    for b in g1_encodings(0xC0DEC1, 2000):
        for strict in (False, True):
            try:
                want = O.pubkey_to_G1(b, strict)
                ws = 1 if want[2] == 0 else 0
            except ValueError:
                want, ws = None, 2
            seen.add(("g1", strict, ws))
            s = L.hc_g1_decompress(b, buf, 0 if strict else 1)
            assert s == ws, (b.hex(), strict)
            if s == 0:
                assert (i48(buf.raw[:48]), i48(buf.raw[48:96])) == (want[0], want[1]), b.hex()
    for b in g2_encodings(0xC0DEC2, 600):
        for strict in (False, True):
            try:
                want = O.signature_to_G2(b, strict)
                ws = 1 if want[2] == O.FQ2_ZERO else 0
            except ValueError:
                want, ws = None, 2
            seen.add(("g2", strict, ws))
            s = L.hc_g2_decompress(b, buf, 0 if strict else 1)
            assert s == ws, (b.hex(), strict)
            if s == 0:
                got = ((i48(buf.raw[:48]), i48(buf.raw[48:96])), (i48(buf.raw[96:144]), i48(buf.raw[144:192])))
                assert got == (want[0], want[1]), b.hex()
    # every outcome (point, infinity, rejected) occurs for both groups under both codecs
    assert len(seen) == 12, sorted(seen)


_ASAN_RUNNER = r"""
import ctypes, json, sys
L = ctypes.CDLL(sys.argv[1])
with open(sys.argv[2]) as f: gb = json.load(f)
with open(sys.argv[3]) as f: tor = json.load(f)
h = bytes.fromhex
bad = 0
nc = json.load(open(sys.argv[4]))
for src, col in ((gb, "expected"), (tor, "expected_pyecc"), (nc, "expected_pyecc")):
    for c in src["verify"]:
        m = h(c["message"])
        v = L.hc_verify(h(c["pubkey"]), m, len(m), h(c["signature"]), int(c["domain"]).to_bytes(8, "big"), 0)
        bad += v != int(c[col])
    for c in src["verify_multiple"]:
        if len(c["pubkeys"]) != len(c["messages"]):
            continue
        pks = b"".join(h(p) for p in c["pubkeys"]) or None
        ms = b"".join(h(x) for x in c["messages"]) or None
        v = L.hc_verify_multiple(len(c["pubkeys"]), pks, ms, 32, h(c["signature"]),
                                 int(c["domain"]).to_bytes(8, "big"), 0)
        bad += v != int(c[col])
print("mismatches", bad)
sys.exit(1 if bad else 0)
"""


def test_sanitized_host_build_over_golden_batches(tmp_path):
    """ASan + UBSan build of the device headers (host) over every golden and torsion
    verify / verify_multiple case: no sanitizer report, same verdicts."""
    import build_native
    lib = build_native.build_hostcheck(sanitize=True)
    asan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    ubsan = subprocess.run(["gcc", "-print-file-name=libubsan.so"], capture_output=True, text=True).stdout.strip()
    if not os.path.isabs(asan) or not os.path.exists(asan):
        pytest.skip("libasan runtime not found")
    runner = tmp_path / "run.py"
    runner.write_text(_ASAN_RUNNER)
    env = dict(os.environ, LD_PRELOAD=" ".join(p for p in (asan, ubsan) if os.path.isabs(p)),
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    g = os.path.join(ROOT, "tests", "golden")
    res = subprocess.run([sys.executable, str(runner), lib, os.path.join(g, "bls_golden_batches.json"),
                          os.path.join(g, "bls_torsion.json"), os.path.join(g, "bls_noncanonical.json")],
                         env=env, capture_output=True, text=True,
                         timeout=600)
    assert res.returncode == 0, res.stdout[-2000:] + res.stderr[-4000:]
    assert "ERROR: AddressSanitizer" not in res.stderr and "runtime error" not in res.stderr, res.stderr[-4000:]
    assert "mismatches 0" in res.stdout


def _outcome(fn, *a):
    try:
        return fn(*a)
    except (OverflowError, O.ValidationError) as e:
        return type(e).__name__


def test_shim_boundary_fixtures_match_oracle(noncanon):
    """bls_noncanonical.json's shim_* sections (VERDICT r04 missing #4) recomputed by the
    oracle: py_ecc 1.7.0 reads pubkeys and signatures of any length as big-endian integers,
    and serialises the domain after the decodes that precede hash_to_G2; the strict policy
    takes Bytes48 / Bytes96 and a uint64 domain first."""
    for c in noncanon["shim_verify"]:
        a = (_h(c["message"]), _h(c["pubkey"]), _h(c["signature"]), int(c["domain"]))
        assert _outcome(O.verify, *a) == c["expected_pyecc"], c["kind"]
        assert _outcome(O.verify_strict, *a) == c["expected_strict"], c["kind"]
    for c in noncanon["shim_verify_multiple"]:
        a = ([_h(p) for p in c["pubkeys"]], [_h(m) for m in c["messages"]], _h(c["signature"]), int(c["domain"]))
        assert _outcome(O.verify_multiple, *a) == c["expected_pyecc"], c["kind"]
        assert _outcome(O.verify_multiple_strict, *a) == c["expected_strict"], c["kind"]
    for name, fn in (("shim_aggregate_pubkeys", O.aggregate_pubkeys), ("shim_aggregate_sigs", O.aggregate_signatures)):
        for c in noncanon[name]:
            for strict, col in ((False, "output_pyecc"), (True, "output_strict")):
                try:
                    got = fn([_h(x) for x in c["input"]], strict).hex()
                except ValueError:
                    got = None
                assert got == c[col], (name, c["kind"], col)
    v = {c["kind"]: c for c in noncanon["shim_verify"]}
    assert v["pk_leading_junk_byte"]["expected_pyecc"] is True
    assert v["domain_2_64_bad_sig"]["expected_pyecc"] is False
    assert v["domain_2_64_valid"]["expected_pyecc"] == "OverflowError"


def test_shim_length_normalisation_is_py_ecc_decoding(noncanon):
    """The shim hands odd-length pubkeys / signatures to the engine as the 48 / 96-byte
    encodings py_ecc's lax decoders read identically (bls._lax_pubkey / _lax_signature):
    the oracle decodes both to the same point, or rejects both."""
    from bls381_amd import bls

    def dec(fn, b):
        try:
            return fn(b)
        except ValueError:
            return None
    pks = {_h(p) for c in noncanon["shim_verify"] for p in [c["pubkey"]]}
    pks |= {_h(p) for c in noncanon["shim_aggregate_pubkeys"] for p in c["input"]}
    for b in pks:
        n = bls._lax_pubkey(b)
        assert len(n) == 48 and dec(O.pubkey_to_G1, n) == dec(O.pubkey_to_G1, b), b.hex()
    sigs = {_h(c["signature"]) for c in noncanon["shim_verify"]}
    sigs |= {_h(s) for c in noncanon["shim_aggregate_sigs"] for s in c["input"]}
    for b in sigs:
        n = bls._lax_signature(b)
        assert len(n) == 96 and dec(O.signature_to_G2, n) == dec(O.signature_to_G2, b), b.hex()
