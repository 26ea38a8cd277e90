"""SSZ roots (§8(f) rank 2): oracle vs fixtures, and the root-program interpreter
(csrc/bls381_ssz.hpp, host build) vs the oracle on CPU.  GPU half: test_gpu_parity.py."""
import ctypes
import json
import os
import random

import pytest

import ssz_oracle as S
from bls381_amd import ssz

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TYPES = {"DepositData": (S.DepositData, ssz.DepositData),
         "AttestationDataAndCustodyBit": (S.AttestationDataAndCustodyBit, ssz.AttestationDataAndCustodyBit),
         "AttestationData": (S.AttestationData, ssz.AttestationData),
         "Crosslink": (S.Crosslink, ssz.Crosslink),
         "BeaconBlockHeader": (S.BeaconBlockHeader, ssz.BeaconBlockHeader)}


@pytest.fixture(scope="module")
def fx():
    with open(os.path.join(ROOT, "tests", "golden", "ssz_roots.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def L():
    import build_native
    return ctypes.CDLL(os.environ.get("BLS381_HOSTCHECK_LIB") or build_native.build_hostcheck())


def test_merkleize_known_answers(fx):
    # zero hashes of merkle_minimal.py (pinned by the fixture script against the reference module)
    z = S.ZERO
    for h in fx["zerohashes"][:6]:
        assert S.merkleize_chunks([S.ZERO] * (1 << fx["zerohashes"].index(h))) == bytes.fromhex(h)
    assert S.merkleize_chunks([z]) == z
    for case in fx["merkleize"]:
        assert S.merkleize_chunks([bytes.fromhex(c) for c in case["chunks"]]).hex() == case["root"]


def test_oracle_matches_fixtures(fx):
    for case in fx["roots"]:
        typ = TYPES[case["type"]][0]
        ser = bytes.fromhex(case["serialized"])
        assert S.serialize(typ, S_unpack(typ, ser)) == ser
        v = S_unpack(typ, ser)
        assert S.hash_tree_root(typ, v).hex() == case["hash_tree_root"]
        if typ[0] == "container":
            assert S.signing_root(typ, v).hex() == case["signing_root"]


def S_unpack(typ, b):
    """serialized bytes -> oracle value (fixed-size types)."""
    k = typ[0]
    if k == "uint":
        return int.from_bytes(b, "little")
    if k == "bool":
        return b == b"\x01"
    if k == "bytes":
        return b
    out, off = {}, 0
    for name, t in typ[1]:
        n = ssz.item_size(t)
        out[name] = S_unpack(t, b[off:off + n])
        off += n
    return out


def test_programs_on_host_interpreter(L, fx):
    buf = ctypes.create_string_buffer(32)
    for case in fx["roots"]:
        typ = TYPES[case["type"]][1]
        ser = bytes.fromhex(case["serialized"])
        for signing, key in ((False, "hash_tree_root"), (True, "signing_root")):
            if signing and typ[0] != "container":
                continue
            prog = ssz.compile_root(typ, signing)
            assert L.hc_ssz_root(ser, prog.ctypes.data_as(ctypes.c_void_p), len(prog), buf) == 1
            assert buf.raw.hex() == case[key], (case["type"], key)


def test_deposit_program_is_the_engines():
    # csrc/bls381_capi.hip DEPOSIT_SIGNING_PROG == the compiler's signing_root(DepositData)
    assert list(ssz.compile_root(ssz.DepositData, True)) == [1, 0, 32, 1, 32, 16, 2, 2, 1, 48, 32, 1, 80, 8, 2, 3]
    assert ssz.item_size(ssz.DepositData) == 184


def test_malformed_program_rejected_on_host(L):
    buf = ctypes.create_string_buffer(32)
    import numpy as np
    for prog in ([2, 1], [1, 0, 33], [1, 0, 8, 1, 0, 8], [9]):
        p = np.asarray(prog, dtype=np.uint32)
        assert L.hc_ssz_root(b"\x00" * 64, p.ctypes.data_as(ctypes.c_void_p), len(p), buf) == 0
