"""SSZ hash_tree_root / signing_root of fixed-size containers on the GPU -- the
message_hash producer in front of bls_verify.

The reference computes every BLS message with SSZ merkleization on the CPU:
``signing_root(deposit.data)`` for deposits (specs/core/0_beacon-chain.md:1755-1758)
and ``hash_tree_root(AttestationDataAndCustodyBit(...))`` for attestations
(:1029-1030), through test_libs/pyspec/eth2spec/utils/ssz/ssz_impl.py:143-163.
Here a fixed-size type compiles into a short program over the item's SSZ
serialization (csrc/bls381_ssz.hpp), and the engine runs it for a whole batch,
one lane per item.  The bytes equal ssz_impl's for the same values.

Types: ``uint(nbytes)``, ``BOOL``, ``Bytes(n)``, ``Container((name, type), ...)``;
the beacon-chain containers on the BLS path are predefined below.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native

SSZ_CHUNK = 1
SSZ_MERKLE = 2


def uint(n: int):
    return ("uint", n)


BOOL = ("bool",)


def Bytes(n: int):
    return ("bytes", n)


def Container(*fields):
    return ("container", list(fields))


# specs/core/0_beacon-chain.md containers whose roots are BLS messages
Crosslink = Container(("shard", uint(8)), ("start_epoch", uint(8)), ("end_epoch", uint(8)),
                      ("parent_root", Bytes(32)), ("data_root", Bytes(32)))
AttestationData = Container(("beacon_block_root", Bytes(32)), ("source_epoch", uint(8)),
                            ("source_root", Bytes(32)), ("target_epoch", uint(8)), ("target_root", Bytes(32)),
                            ("crosslink", Crosslink))
AttestationDataAndCustodyBit = Container(("data", AttestationData), ("custody_bit", BOOL))
DepositData = Container(("pubkey", Bytes(48)), ("withdrawal_credentials", Bytes(32)), ("amount", uint(8)),
                        ("signature", Bytes(96)))
BeaconBlockHeader = Container(("slot", uint(8)), ("parent_root", Bytes(32)), ("state_root", Bytes(32)),
                              ("body_root", Bytes(32)), ("signature", Bytes(96)))


def item_size(typ) -> int:
    k = typ[0]
    if k == "uint":
        return typ[1]
    if k == "bool":
        return 1
    if k == "bytes":
        return typ[1]
    return sum(item_size(t) for _, t in typ[1])


def serialize(typ, v) -> bytes:
    """SSZ serialization of a fixed-size value (ssz_impl.py:21-30 for basics; fields concatenated)."""
    k = typ[0]
    if k == "uint":
        return int(v).to_bytes(typ[1], "little")
    if k == "bool":
        return b"\x01" if v else b"\x00"
    if k == "bytes":
        v = bytes(v)
        if len(v) != typ[1]:
            raise ValueError("expected %d bytes" % typ[1])
        return v
    return b"".join(serialize(t, v[name]) for name, t in typ[1])


def _emit(typ, off: int, prog: list) -> int:
    k = typ[0]
    if k in ("uint", "bool"):
        n = item_size(typ)
        prog += [SSZ_CHUNK, off, n]
        return off + n
    if k == "bytes":
        n = typ[1]
        pieces = max(1, (n + 31) // 32)
        for j in range(pieces):
            prog += [SSZ_CHUNK, off + 32 * j, min(32, n - 32 * j)]
        if pieces > 1:
            prog += [SSZ_MERKLE, pieces]
        return off + n
    for _, t in typ[1]:
        off = _emit(t, off, prog)
    prog += [SSZ_MERKLE, len(typ[1])]
    return off


def compile_root(typ, signing: bool = False) -> np.ndarray:
    """The root program of `typ` (signing=True: signing_root, the last field left out)."""
    prog: list = []
    if signing:
        if typ[0] != "container" or len(typ[1]) < 2:
            raise ValueError("signing_root needs a container with at least two fields")
        off = 0
        for _, t in typ[1][:-1]:
            off = _emit(t, off, prog)
        prog += [SSZ_MERKLE, len(typ[1]) - 1]
    else:
        _emit(typ, 0, prog)
    return np.asarray(prog, dtype=np.uint32)


def _roots(typ, items, signing: bool) -> list:
    size = item_size(typ)
    blob = b"".join(bytes(x) for x in items)
    n = len(blob) // size
    if n * size != len(blob):
        raise ValueError("items must be %d-byte serializations" % size)
    if n == 0:
        return []
    prog = compile_root(typ, signing)
    out = ctypes.create_string_buffer(32 * n)
    _native.check(_native.lib().bls381_ssz_root_batch(n, blob, size, prog.ctypes.data_as(ctypes.c_void_p),
                                                      len(prog), out))
    raw = out.raw
    return [raw[32 * i:32 * i + 32] for i in range(n)]


def hash_tree_root_batch(typ, serialized_items) -> list:
    """hash_tree_root of each serialized item (ssz_impl.py:143-155)."""
    return _roots(typ, serialized_items, False)


def signing_root_batch(typ, serialized_items) -> list:
    """signing_root of each serialized container (ssz_impl.py:158-163)."""
    return _roots(typ, serialized_items, True)


def verify_deposits(deposit_datas, domain) -> np.ndarray:
    """process_deposit's check for each serialized DepositData (0_beacon-chain.md:1755-1758):
    bls_verify(pubkey, signing_root(deposit.data), signature, domain), roots computed on the device."""
    blob = b"".join(bytes(x) for x in deposit_datas)
    n = len(blob) // 184
    if n * 184 != len(blob):
        raise ValueError("DepositData serializations are 184 bytes")
    out = np.zeros(n, dtype=np.uint8)
    if n:
        dom = int(domain).to_bytes(8, "big") * n
        _native.check(_native.lib().bls381_verify_deposits(n, blob, dom, out.ctypes.data_as(ctypes.c_void_p)))
    return out.astype(bool)
