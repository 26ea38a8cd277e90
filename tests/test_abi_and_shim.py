"""CPU-side checks of the boundary: the C-ABI library loads and exports every
symbol include/bls381.h declares; the Python mirror keeps the reference's
module semantics (bls.py:3-46); with no device the product fails loudly (no
CPU fallback)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    txt = open(os.path.join(ROOT, "include", "bls381.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(bls381_\w+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    import build_native
    from bls381_amd import _native
    lib_path = build_native.build_hip()
    L = ctypes.CDLL(lib_path)
    names = header_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(L, n), n
    assert sorted(_native._SIGS) == names, "ctypes binding table out of sync with include/bls381.h"
    _native.load_library()   # binds all signatures


def test_kernels_are_gfx950_code_objects():
    import build_native
    blob = open(build_native.build_hip(), "rb").read()
    # the offload bundle carries exactly one device target: gfx950
    assert b"hipv4-amdgcn-amd-amdhsa--gfx950" in blob
    assert b"amdhsa--gfx942" not in blob and b"amdhsa--gfx90a" not in blob


def test_no_device_fails_loudly():
    from bls381_amd import _native
    L = _native.load_library()
    if L.bls381_device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(_native.NativeUnavailable):
        _native.lib()
    assert L.bls381_verify(b"\x00" * 48, b"\x00" * 32, 32, b"\x00" * 96, b"\x00" * 8) == _native.ENODEV


def test_stub_mode_mirrors_reference():
    from bls381_amd import bls
    assert bls.STUB_SIGNATURE == b"\x11" * 96 and bls.STUB_PUBKEY == b"\x22" * 48
    old = bls.bls_active
    try:
        bls.bls_active = False
        assert bls.bls_verify(b"", b"", b"", 0) is True
        assert bls.bls_verify_multiple([], [], b"", 0) is True
        assert bls.bls_aggregate_pubkeys([b"x"]) == bls.STUB_PUBKEY
        assert bls.bls_aggregate_signatures([]) == bls.STUB_SIGNATURE
        assert bls.bls_sign(b"m", 1, 0) == bls.STUB_SIGNATURE
    finally:
        bls.bls_active = old


def test_errors_raised_before_the_engine():
    from bls381_amd import bls
    with pytest.raises(ValueError):
        bls.bls_verify_multiple([b"\x00" * 48], [], b"\x00" * 96, 0)
    with pytest.raises(bls.ValidationError):
        bls.bls_verify_multiple([], [b"\x00" * 32], b"\x00" * 96, 0)
    with pytest.raises(OverflowError):
        bls.bls_verify(b"\x00" * 48, b"\x00" * 32, b"\x00" * 96, 2 ** 64)
    with pytest.raises(OverflowError):
        bls.bls_verify(b"\x00" * 48, b"\x00" * 32, b"\x00" * 96, -1)
    # wrong-length encodings are invalid inputs -> False without reaching the device
    assert bls.bls_verify(b"\x00" * 47, b"\x00" * 32, b"\x00" * 96, 0) is False
    with pytest.raises(ValueError):
        bls.bls_aggregate_pubkeys([b"\x00" * 47])


def test_keyword_names_match_reference():
    import inspect
    from bls381_amd import bls
    # reference bls.py:25,30,35,40,45 (callers pass kwargs, 0_beacon-chain.md:1024-1033)
    want = {"bls_verify": ["pubkey", "message_hash", "signature", "domain"],
            "bls_verify_multiple": ["pubkeys", "message_hashes", "signature", "domain"],
            "bls_aggregate_pubkeys": ["pubkeys"],
            "bls_aggregate_signatures": ["signatures"],
            "bls_sign": ["message_hash", "privkey", "domain"]}
    for name, params in want.items():
        fn = getattr(bls, name)
        inner = next(c.cell_contents for c in fn.__closure__ if callable(c.cell_contents))
        assert list(inspect.signature(inner).parameters) == params, name


def test_registry_shim_hook_is_opt_in():
    from bls381_amd import bls
    assert bls._pubkey_registry is None
    bls.use_pubkey_registry(None)
    assert bls._pubkey_registry is None
