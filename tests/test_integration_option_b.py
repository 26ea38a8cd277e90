"""INTEGRATION.md option B (tests/integration_option_b.py): the reference module
test_libs/pyspec/eth2spec/utils/bls.py:1-46 with its py_ecc calls replaced by ctypes
calls into libbls381.so.  The CPU tests check its flag/stub behaviour and error mapping;
the GPU test runs the golden and torsion batches through it."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "consensus-specs_amd", "lib", "libbls381.so")


@pytest.fixture(scope="module")
def B():
    if not os.path.exists(LIB):
        pytest.skip("libbls381.so not built")
    os.environ["BLS381_LIB"] = LIB
    spec = importlib.util.spec_from_file_location("integration_option_b",
                                                  os.path.join(ROOT, "tests", "integration_option_b.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _has_device(B):
    return B._L.bls381_device_count() > 0


def test_option_b_flag_stubs_and_errors(B):
    """bls.py:3-21 semantics (flag read at call time, stub returns) and the error mapping
    that holds without a device: length mismatch -> ValidationError (a ValueError),
    bad domain -> OverflowError, wrong sizes -> False / ValueError."""
    assert issubclass(B.ValidationError, ValueError)
    with pytest.raises(B.ValidationError):
        B.bls_verify_multiple([b"\x00" * 48], [], b"\x00" * 96, 0)
    with pytest.raises(OverflowError):
        B.bls_verify(b"\x00" * 48, b"\x00" * 32, b"\x00" * 96, 1 << 64)
    assert B.bls_verify(b"\x00" * 47, b"\x00" * 32, b"\x00" * 96, 0) is False
    with pytest.raises(ValueError):
        B.bls_aggregate_pubkeys([b"\x00" * 47])
    B.bls_active = False
    try:
        assert B.bls_verify(b"", b"", b"", 0) is True
        assert B.bls_verify_multiple([], [], b"", 0) is True
        assert B.bls_aggregate_pubkeys([]) == B.STUB_PUBKEY
        assert B.bls_aggregate_signatures([]) == B.STUB_SIGNATURE
        assert B.bls_sign(b"", 1, 0) == B.STUB_SIGNATURE
    finally:
        B.bls_active = True


def test_option_b_no_device_fails_loudly(B):
    """Without a gfx950 device the engine's BLS381_ENODEV raises, never a verdict."""
    if _has_device(B):
        pytest.skip("a device is present")
    with pytest.raises(B.NativeUnavailable):
        B.bls_verify(b"\xc0" + b"\x00" * 47, b"\x00" * 32, b"\xc0" + b"\x00" * 95, 0)
    with pytest.raises(B.NativeUnavailable):
        B.bls_aggregate_pubkeys([b"\xc0" + b"\x00" * 47])


@pytest.mark.gpu
def test_option_b_golden_and_torsion(B, golden, torsion):
    vec, gb = golden
    for it in gb["verify"]:
        assert B.bls_verify(bytes.fromhex(it["pubkey"]), bytes.fromhex(it["message"]),
                            bytes.fromhex(it["signature"]), int(it["domain"])) == it["expected"], it["kind"]
    for it in gb["verify_multiple"]:
        assert B.bls_verify_multiple([bytes.fromhex(p) for p in it["pubkeys"]],
                                     [bytes.fromhex(m) for m in it["messages"]],
                                     bytes.fromhex(it["signature"]), int(it["domain"])) == it["expected"], it["kind"]
    for it in gb["aggregate_pubkeys"]:
        assert B.bls_aggregate_pubkeys([bytes.fromhex(p) for p in it["input"]]).hex() == it["output"], it["kind"]
    for it in gb["aggregate_sigs"]:
        assert B.bls_aggregate_signatures([bytes.fromhex(s) for s in it["input"]]).hex() == it["output"], it["kind"]
    for k in gb["invalid_g1"]:
        with pytest.raises(ValueError):
            B.bls_aggregate_pubkeys([bytes.fromhex(k)])
    for c in vec["sign_msg"]:
        i = c["input"]
        assert B.bls_sign(bytes.fromhex(i["message"][2:]), int(i["privkey"], 16),
                          int(i["domain"], 16)).hex() == c["output"][2:]
    # torsion fixtures: the engine's process-wide policy is the default ("pyecc")
    for c in torsion["verify"]:
        assert B.bls_verify(bytes.fromhex(c["pubkey"]), bytes.fromhex(c["message"]),
                            bytes.fromhex(c["signature"]), int(c["domain"])) == c["expected_pyecc"], c["kind"]
    for c in torsion["verify_multiple"]:
        assert B.bls_verify_multiple([bytes.fromhex(p) for p in c["pubkeys"]],
                                     [bytes.fromhex(m) for m in c["messages"]],
                                     bytes.fromhex(c["signature"]), int(c["domain"])) == c["expected_pyecc"], c["kind"]
    # mixed message lengths in one call: one final exponentiation over per-length partials
    from bls381_amd import bls as pkg
    sks, ms = [7, 11], [b"\x01" * 32, b"\x02" * 40]
    pks = [pkg.privtopub(k) for k in sks]
    sig = B.bls_aggregate_signatures([B.bls_sign(m, k, 5) for m, k in zip(ms, sks)])
    assert B.bls_verify_multiple(pks, ms, sig, 5) is True
    assert B.bls_verify_multiple(pks, [ms[0], ms[1] + b"x"], sig, 5) is False
    assert B.bls_verify_multiple(pks, ms, sig, 6) is False
