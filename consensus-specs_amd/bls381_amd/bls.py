"""Drop-in replacement for the reference's `eth2spec.utils.bls`
(test_libs/pyspec/eth2spec/utils/bls.py:1-46), backed by the gfx950 engine.

Same module attributes (`bls_active`, `STUB_SIGNATURE`, `STUB_PUBKEY`,
`only_with_bls`), same function names and keyword names, same return types and
the same error behaviour as the py_ecc 1.7.0 calls they replace
(SURVEY.md Appendix A):

* bls_verify / bls_verify_multiple return False for undecodable or invalid
  inputs (py_ecc catches ValidationError/ValueError/AssertionError);
* bls_verify_multiple raises ValidationError (a ValueError) on a length mismatch;
* bls_aggregate_* raise ValueError on an invalid point encoding;
* a domain outside [0, 2^64) raises OverflowError (int.to_bytes).

Inputs py_ecc reads as integers (VERDICT r04 missing #4), under the "pyecc" policy:
* a pubkey of any length is decompress_G1(big_endian_to_int(pubkey)), and a signature
  of any length decompress_G2((int(sig[:48]), int(sig[48:]))): such inputs are passed to
  the engine as the 48 / 96-byte encodings the lax decoder reads identically (_lax_pubkey,
  _lax_signature);
* the domain is serialised inside hash_to_G2, after the decodes that come before it:
  bls_verify returns False for an undecodable signature before an out-of-range domain
  raises OverflowError; bls_verify_multiple decodes the first message group's pubkeys
  (sorted message order) first and never serialises the domain of an empty call.
The "strict" policy takes the spec's types: Bytes48 / Bytes96 only (other lengths are
False, or ValueError from the aggregates) and a uint64 domain, checked first.
Fixtures: tests/golden/bls_noncanonical.json "shim_*" sections, both columns.

Divergences from that contract (tested in tests/test_gpu_parity.py):
* a message longer than _native.MSG_MAX (1 MiB) raises ValueError from bls_verify,
  bls_verify_multiple and bls_sign, where py_ecc would hash it and return a verdict.
  The spec's message_hash is Bytes32, so no spec call reaches the limit; raising
  keeps a verdict from ever being guessed for an input the engine did not hash.
* bls_verify_multiple with a domain outside [0, 2^64) and an undecodable pubkey in one
  of several message groups: py_ecc 1.7.0 walks set(message_hashes), so whether it
  decodes that group first (False) or serialises the domain first (OverflowError)
  depends on the process's hash seed.  This module takes the sorted order; the
  fixtures mark both cases as order-dependent (pyecc_order_dependent).
Messages up to the limit may have any length, and one bls_verify_multiple call may
mix lengths (each length group becomes a partial Miller product; one final
exponentiation decides the call).

Two switches mirror behaviour the reference leaves to py_ecc:
* DOMAIN_BYTEORDER -- how the int domain becomes 8 bytes;
* SUBGROUP_POLICY  -- "pyecc" (default): py_ecc 1.7.0's behaviour -- its lax codec
  (b_flag set means infinity whatever the other bits, x taken mod
  2^381 and reduced mod q, no c_flag or x < q check) and no subgroup test, only the
  on-curve test; "strict": the spec's codec (bls_signature.md:47-52,58-64: c_flag
  set, x < q, canonical infinity) and every pubkey / signature must also lie in
  G1 / G2 (:135-136,143-144).  The verdicts and aggregate bytes differ only on
  points with a small-order component (tests/golden/bls_torsion.json) and on
  non-canonical encodings (tests/golden/bls_noncanonical.json); both files carry
  both columns.
  The switch applies to this module's calls only: each call runs inside a
  thread-local policy scope (_native.subgroup_policy_scope), so the process-wide
  policy other front ends read (_native.set_subgroup_policy) is never rewritten.
"""
from . import _native

# Flag to make BLS active or not (bls.py:3-4).  Tests flip it through the
# module attribute (eth2spec/test/context.py:79-90).
bls_active = True

STUB_SIGNATURE = b'\x11' * 96
STUB_PUBKEY = b'\x22' * 48

# py_ecc 1.7.0 serialises the int domain big-endian; one switch.
DOMAIN_BYTEORDER = "big"

# Codec and subgroup checks: "pyecc" (py_ecc 1.7.0, the reference's behaviour) or
# "strict" (the spec's point format and valid-G1/G2-point rule).  One switch.
SUBGROUP_POLICY = "pyecc"


class ValidationError(ValueError):
    """Mirror of eth_utils.ValidationError raised by py_ecc.verify_multiple."""


def only_with_bls(alt_return=None):
    """
    Decorator factory to make a function only run when BLS is active. Otherwise return the default.
    (bls.py:10-21; the flag is read at call time from this module.)
    """
    def runner(fn):
        def entry(*args, **kw):
            if bls_active:
                return fn(*args, **kw)
            else:
                return alt_return
        return entry
    return runner


def _dom8(domain) -> bytes:
    return int(domain).to_bytes(8, DOMAIN_BYTEORDER)


def _sk32(privkey) -> bytes:
    k = int(privkey)
    if k < 0:
        raise ValueError("negative private key")
    # [k]P == [k mod r]P on the prime-order groups; py_ecc multiplies by k itself
    r = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
    if k >= 1 << 256:
        k %= r
    return k.to_bytes(32, "big")


_Q = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab


def _lax_pubkey(p: bytes) -> bytes:
    """The 48-byte encoding py_ecc 1.7.0's lax decode_G1 reads like big_endian_to_int(p): it
    looks at bits 381-382 and z mod 2^381 only (bit 383 and up are ignored)."""
    if len(p) == 48:
        return p
    return (int.from_bytes(p, "big") % (1 << 384)).to_bytes(48, "big")


def _lax_signature(sig: bytes) -> bytes:
    """The 96-byte encoding py_ecc 1.7.0's lax decode_G2 reads like (int(sig[:48]),
    int(sig[48:])): z1 (at most 48 bytes), and z2 of any length, of which only z2 mod q
    is used (the real part of x)."""
    if len(sig) == 96:
        return sig
    z1 = int.from_bytes(sig[:48], "big")
    z2 = int.from_bytes(sig[48:], "big") % _Q
    return z1.to_bytes(48, "big") + z2.to_bytes(48, "big")


def _strict() -> bool:
    return SUBGROUP_POLICY == "strict"


def _signature_decodes(sig: bytes) -> bool:
    """Whether the call's codec decodes `sig` (a valid encoding under the policy)."""
    try:
        with _native.subgroup_policy_scope(SUBGROUP_POLICY):
            _native.aggregate_signatures(sig)
        return True
    except ValueError:
        return False


def _pubkeys_decode(pks) -> bool:
    try:
        with _native.subgroup_policy_scope(SUBGROUP_POLICY):
            _native.aggregate_pubkeys(b"".join(pks))
        return True
    except ValueError:
        return False


def _check_len(message_hash: bytes) -> None:
    if len(message_hash) > _native.MSG_MAX:
        raise ValueError("message of %d bytes is longer than the engine's %d-byte limit"
                         % (len(message_hash), _native.MSG_MAX))


@only_with_bls(alt_return=True)
def bls_verify(pubkey, message_hash, signature, domain):
    if _strict():
        dom8 = _dom8(domain)       # uint64 (the spec's type), before anything else
    pubkey, message_hash, signature = bytes(pubkey), bytes(message_hash), bytes(signature)
    _check_len(message_hash)
    if _strict():
        if len(pubkey) != 48 or len(signature) != 96:
            return False
    else:
        pubkey, signature = _lax_pubkey(pubkey), _lax_signature(signature)
        try:
            dom8 = _dom8(domain)
        except OverflowError:
            # py_ecc: signature_to_G2 runs before hash_to_G2 serialises the domain (A.5)
            if not _signature_decodes(signature):
                return False
            raise
    with _native.subgroup_policy_scope(SUBGROUP_POLICY):
        return _native.verify(pubkey, message_hash, signature, dom8)


@only_with_bls(alt_return=True)
def bls_verify_multiple(pubkeys, message_hashes, signature, domain):
    if len(pubkeys) != len(message_hashes):
        raise ValidationError(
            "len(pubkeys) (%s) should be equal to len(message_hashes) (%s)" % (len(pubkeys), len(message_hashes)))
    if _strict():
        dom8 = _dom8(domain)
    pks = [bytes(p) for p in pubkeys]
    msgs = [bytes(m) for m in message_hashes]
    signature = bytes(signature)
    for m in msgs:
        _check_len(m)
    if _strict():
        if any(len(p) != 48 for p in pks) or len(signature) != 96:
            return False
    else:
        pks, signature = [_lax_pubkey(p) for p in pks], _lax_signature(signature)
        try:
            dom8 = _dom8(domain)
        except OverflowError:
            if not pks:
                dom8 = bytes(8)    # py_ecc never serialises the domain of an empty call (A.6)
            else:
                # the first message group's pubkeys are decoded before hash_to_G2 serialises it
                first = min(msgs)
                if not _pubkeys_decode([p for p, m in zip(pks, msgs) if m == first]):
                    return False
                raise
    with _native.subgroup_policy_scope(SUBGROUP_POLICY):
        return verify_multiple_bytes(pks, msgs, signature, dom8)


def verify_multiple_bytes(pks, msgs, signature: bytes, dom8: bytes) -> bool:
    """bls_verify_multiple on validated bytes (48-byte keys, 96-byte signature, messages
    of any lengths <= MSG_MAX) under the policy already set."""
    lens = sorted({len(m) for m in msgs})
    if len(lens) <= 1:
        mlen = lens[0] if lens else 32
        return _native.verify_multiple(b"".join(pks), b"".join(msgs), mlen, signature, dom8)
    # mixed lengths: one partial Miller product per length (the signature pair in
    # the first), multiplied and finally exponentiated once -- py_ecc's product
    parts = []
    for j, mlen in enumerate(lens):
        sel = [i for i, m in enumerate(msgs) if len(m) == mlen]
        rc, part = _native.miller_partial(b"".join(pks[i] for i in sel), b"".join(msgs[i] for i in sel), mlen,
                                          signature, j == 0, dom8)
        if rc != 0:
            return False
        parts.append(part)
    return _native.final_verify(b"".join(parts))


# Optional device-resident pubkey registry (registry.PubkeyRegistry): when set,
# bls_aggregate_pubkeys reads registered members' decoded points from HBM
# instead of decompressing them.  Same bytes and errors either way.
_pubkey_registry = None


def use_pubkey_registry(registry) -> None:
    """Route bls_aggregate_pubkeys through `registry` (None switches it off)."""
    global _pubkey_registry
    _pubkey_registry = registry


@only_with_bls(alt_return=STUB_PUBKEY)
def bls_aggregate_pubkeys(pubkeys):
    pks = [bytes(p) for p in pubkeys]
    if _strict():
        if any(len(p) != 48 for p in pks):
            raise ValueError("pubkeys must be 48 bytes")
    else:
        pks = [_lax_pubkey(p) for p in pks]
    with _native.subgroup_policy_scope(SUBGROUP_POLICY):
        if _pubkey_registry is not None:
            return _pubkey_registry.aggregate_pubkeys(pks)
        return _native.aggregate_pubkeys(b"".join(pks))


@only_with_bls(alt_return=STUB_SIGNATURE)
def bls_aggregate_signatures(signatures):
    sigs = [bytes(s) for s in signatures]
    if _strict():
        if any(len(s) != 96 for s in sigs):
            raise ValueError("signatures must be 96 bytes")
    else:
        sigs = [_lax_signature(s) for s in sigs]
    with _native.subgroup_policy_scope(SUBGROUP_POLICY):
        return _native.aggregate_signatures(b"".join(sigs))


@only_with_bls(alt_return=STUB_SIGNATURE)
def bls_sign(message_hash, privkey, domain):
    message_hash = bytes(message_hash)
    _check_len(message_hash)
    return _native.sign(message_hash, _sk32(privkey), _dom8(domain))


# ---- py_ecc.bls extras used by the reference's helpers / vector generator
def privtopub(privkey) -> bytes:
    """py_ecc bls.privtopub (eth2spec/test/helpers/keys.py:5, test_generators/bls/main.py:114)."""
    return _native.privtopub(_sk32(privkey))


def hash_to_G2_compressed(message_hash, domain) -> bytes:
    """compress_G2(hash_to_G2(m, d)) as 96 bytes (test_generators/bls/main.py:84-85)."""
    comp, _ = _native.hash_to_g2(bytes(message_hash), _dom8(domain))
    return comp


def hash_to_G2_affine(message_hash, domain):
    """Normalised affine ((x_re, x_im), (y_re, y_im)) as ints."""
    _, aff = _native.hash_to_g2(bytes(message_hash), _dom8(domain))
    v = [int.from_bytes(aff[48 * k:48 * k + 48], "big") for k in range(4)]
    return (v[0], v[1]), (v[2], v[3])


def hash_to_G2_pyecc_projective(message_hash, domain):
    """py_ecc's un-normalised projective triple (test_generators/bls/main.py:66-72)."""
    out = _native.hash_to_g2_pyecc_projective(bytes(message_hash), _dom8(domain))
    v = [int.from_bytes(out[48 * k:48 * k + 48], "big") for k in range(6)]
    return ((v[0], v[1]), (v[2], v[3]), (v[4], v[5]))
