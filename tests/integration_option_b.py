"""INTEGRATION.md option B as a runnable module: the reference's
`test_libs/pyspec/eth2spec/utils/bls.py` (bls.py:1-46) with its five py_ecc calls
replaced by ctypes calls into libbls381.so, and nothing else from this repository.

A maintainer pastes this file over the reference module; tests/test_integration_option_b.py
runs it against the golden and torsion batches on the GPU (and its error mapping on the
CPU).  Behaviour kept from py_ecc 1.7.0:
  * verifies return a bool; an undecodable input is False;
  * bls_verify_multiple raises ValidationError (a ValueError) on a length mismatch;
  * aggregates raise ValueError on an invalid encoding;
  * a domain outside [0, 2^64) raises OverflowError.
Engine errors are never turned into verdicts: BLS381_ENODEV raises NativeUnavailable,
BLS381_EARG ValueError, BLS381_EHIP NativeError.
"""
import ctypes
import os

_L = ctypes.CDLL(os.environ.get("BLS381_LIB", "libbls381.so"))
_vp, _sz, _i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
_L.bls381_device_count.restype = _i
_L.bls381_verify.argtypes = [ctypes.c_char_p, ctypes.c_char_p, _sz, ctypes.c_char_p, ctypes.c_char_p]
_L.bls381_verify_multiple.argtypes = [_sz, ctypes.c_char_p, ctypes.c_char_p, _sz, ctypes.c_char_p,
                                      ctypes.c_char_p]
_L.bls381_miller_partial.argtypes = [_sz, ctypes.c_char_p, ctypes.c_char_p, _sz, ctypes.c_char_p, _i,
                                     ctypes.c_char_p, ctypes.c_char_p]
_L.bls381_final_verify.argtypes = [_sz, ctypes.c_char_p]
_L.bls381_aggregate_pubkeys.argtypes = [_sz, ctypes.c_char_p, ctypes.c_char_p]
_L.bls381_aggregate_signatures.argtypes = [_sz, ctypes.c_char_p, ctypes.c_char_p]
_L.bls381_sign.argtypes = [ctypes.c_char_p, _sz, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
for _f in ("bls381_verify", "bls381_verify_multiple", "bls381_miller_partial", "bls381_final_verify",
           "bls381_aggregate_pubkeys", "bls381_aggregate_signatures", "bls381_sign"):
    getattr(_L, _f).restype = _i

# include/bls381.h return codes
_EINVAL_POINT, _EARG, _ENODEV, _EHIP = -1, -2, -3, -4


class NativeUnavailable(RuntimeError):
    """No gfx950 device (the engine has no CPU fallback)."""


class NativeError(RuntimeError):
    """A HIP runtime error inside the engine."""


class ValidationError(ValueError):
    """eth_utils.ValidationError, as py_ecc's verify_multiple raises it."""


def _rc(rc):
    if rc == _ENODEV:
        raise NativeUnavailable("no gfx950 device for the BLS engine")
    if rc == _EHIP:
        raise NativeError("HIP error in the BLS engine")
    if rc == _EARG:
        raise ValueError("invalid argument to the BLS engine")
    return rc


# ---- the reference module's own definitions (bls.py:3-21), unchanged
bls_active = True

STUB_SIGNATURE = b'\x11' * 96
STUB_PUBKEY = b'\x22' * 48


def only_with_bls(alt_return=None):
    """
    Decorator factory to make a function only run when BLS is active. Otherwise return the default.
    """
    def runner(fn):
        def entry(*args, **kw):
            if bls_active:
                return fn(*args, **kw)
            else:
                return alt_return
        return entry
    return runner


def _d8(domain):
    return int(domain).to_bytes(8, 'big')    # py_ecc 1.7.0 domain serialisation


# ---- the five bodies (bls.py:24-46) on the engine
@only_with_bls(alt_return=True)
def bls_verify(pubkey, message_hash, signature, domain):
    d8 = _d8(domain)
    pubkey, m, signature = bytes(pubkey), bytes(message_hash), bytes(signature)
    if len(pubkey) != 48 or len(signature) != 96:
        return False
    return _rc(_L.bls381_verify(pubkey, m, len(m), signature, d8)) == 1


@only_with_bls(alt_return=True)
def bls_verify_multiple(pubkeys, message_hashes, signature, domain):
    if len(pubkeys) != len(message_hashes):
        raise ValidationError("len(pubkeys) (%d) should be equal to len(message_hashes) (%d)"
                              % (len(pubkeys), len(message_hashes)))
    d8 = _d8(domain)
    pks = [bytes(p) for p in pubkeys]
    msgs = [bytes(m) for m in message_hashes]
    signature = bytes(signature)
    if any(len(p) != 48 for p in pks) or len(signature) != 96:
        return False
    lens = sorted({len(m) for m in msgs}) or [32]
    if len(lens) == 1:
        return _rc(_L.bls381_verify_multiple(len(pks), b"".join(pks), b"".join(msgs), lens[0], signature,
                                             d8)) == 1
    # mixed message lengths: one Miller product per length, one final exponentiation
    parts = []
    for j, ml in enumerate(lens):
        sel = [i for i, m in enumerate(msgs) if len(m) == ml]
        out = ctypes.create_string_buffer(576)
        rc = _rc(_L.bls381_miller_partial(len(sel), b"".join(pks[i] for i in sel), b"".join(msgs[i] for i in sel),
                                          ml, signature, 1 if j == 0 else 0, d8, out))
        if rc != 0:
            return False
        parts.append(out.raw)
    return _rc(_L.bls381_final_verify(len(parts), b"".join(parts))) == 1


@only_with_bls(alt_return=STUB_PUBKEY)
def bls_aggregate_pubkeys(pubkeys):
    pks = [bytes(p) for p in pubkeys]
    if any(len(p) != 48 for p in pks):
        raise ValueError("pubkeys must be 48 bytes")
    out = ctypes.create_string_buffer(48)
    if _rc(_L.bls381_aggregate_pubkeys(len(pks), b"".join(pks), out)) == _EINVAL_POINT:
        raise ValueError("invalid pubkey encoding")
    return out.raw


@only_with_bls(alt_return=STUB_SIGNATURE)
def bls_aggregate_signatures(signatures):
    sigs = [bytes(s) for s in signatures]
    if any(len(s) != 96 for s in sigs):
        raise ValueError("signatures must be 96 bytes")
    out = ctypes.create_string_buffer(96)
    if _rc(_L.bls381_aggregate_signatures(len(sigs), b"".join(sigs), out)) == _EINVAL_POINT:
        raise ValueError("invalid signature encoding")
    return out.raw


@only_with_bls(alt_return=STUB_SIGNATURE)
def bls_sign(message_hash, privkey, domain):
    k = int(privkey)
    if k < 0:
        raise ValueError("negative private key")
    if k >= 1 << 256:
        k %= 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
    out = ctypes.create_string_buffer(96)
    m = bytes(message_hash)
    _rc(_L.bls381_sign(m, len(m), k.to_bytes(32, 'big'), _d8(domain), out))
    return out.raw
