"""CPU restatement of the reference's SSZ hash_tree_root / signing_root for
fixed-size types -- TEST INFRASTRUCTURE ONLY (tests/ and the fixture script may
import it; the product path never does).

Follows test_libs/pyspec/eth2spec/utils/ssz/ssz_impl.py:
  serialize_basic :21-30 (uints little-endian, bool 0x00/0x01)
  pack / chunkify :110-119 (zero-pad to a 32-byte multiple)
  hash_tree_root  :143-155 (bottom-layer kinds chunkify their serialization;
                   containers merkleize their field roots)
  signing_root    :158-163 (the last field left out)
and utils/merkle_minimal.py merkleize_chunks (zero chunks up to a power of two;
a single chunk is its own root) with utils/hash_function.py hash = SHA-256.
Parity pin: tests/golden/make_ssz_vectors.py checks merkleize_chunks against the
reference's own merkle_minimal.py when /root/reference is present; the reference's
ssz_typing.py does not import on Python 3.10 (an ordinary TypeError at import
time), so the type layer is restated here from 0_beacon-chain.md's containers.

Types: ("uint", nbytes) | ("bool",) | ("bytes", n) | ("container", [(name, type), ...]).
Values: int | bool | bytes | dict name -> value.
"""
from hashlib import sha256

ZERO = b"\x00" * 32


def uint(n):
    return ("uint", n)


BOOL = ("bool",)


def Bytes(n):
    return ("bytes", n)


def Container(*fields):
    return ("container", list(fields))


def merkleize_chunks(chunks):
    """merkle_minimal.merkleize_chunks."""
    n = len(chunks)
    p = 1 if n == 0 else 1 << (n - 1).bit_length()
    layer = list(chunks) + [ZERO] * (p - n)
    while len(layer) > 1:
        layer = [sha256(layer[i] + layer[i + 1]).digest() for i in range(0, len(layer), 2)]
    return layer[0]


def chunkify(b):
    b = b + b"\x00" * (-len(b) % 32)
    return [b[i:i + 32] for i in range(0, len(b), 32)] or [ZERO]


def serialize(typ, v):
    k = typ[0]
    if k == "uint":
        return int(v).to_bytes(typ[1], "little")
    if k == "bool":
        return b"\x01" if v else b"\x00"
    if k == "bytes":
        v = bytes(v)
        assert len(v) == typ[1]
        return v
    return b"".join(serialize(t, v[name]) for name, t in typ[1])


def hash_tree_root(typ, v):
    k = typ[0]
    if k in ("uint", "bool", "bytes"):
        return merkleize_chunks(chunkify(serialize(typ, v)))
    return merkleize_chunks([hash_tree_root(t, v[name]) for name, t in typ[1]])


def signing_root(typ, v):
    assert typ[0] == "container"
    return merkleize_chunks([hash_tree_root(t, v[name]) for name, t in typ[1][:-1]])


# 0_beacon-chain.md containers on the BLS path
Crosslink = Container(("shard", uint(8)), ("start_epoch", uint(8)), ("end_epoch", uint(8)),
                      ("parent_root", Bytes(32)), ("data_root", Bytes(32)))                       # :303-312
AttestationData = Container(("beacon_block_root", Bytes(32)), ("source_epoch", uint(8)),
                            ("source_root", Bytes(32)), ("target_epoch", uint(8)), ("target_root", Bytes(32)),
                            ("crosslink", Crosslink))                                            # :318-329
AttestationDataAndCustodyBit = Container(("data", AttestationData), ("custody_bit", BOOL))      # :335-339
DepositData = Container(("pubkey", Bytes(48)), ("withdrawal_credentials", Bytes(32)), ("amount", uint(8)),
                        ("signature", Bytes(96)))                                                 # :394-402
BeaconBlockHeader = Container(("slot", uint(8)), ("parent_root", Bytes(32)), ("state_root", Bytes(32)),
                              ("body_root", Bytes(32)), ("signature", Bytes(96)))                # :406-413
