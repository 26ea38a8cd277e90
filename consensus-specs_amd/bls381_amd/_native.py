"""ctypes binding of lib/libbls381.so (include/bls381.h).  No PyTorch.

The product path has no CPU fallback: if the library cannot be loaded, or no
gfx950 device is visible, every call raises `NativeUnavailable`.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BLS381_LIB", os.path.join(_HERE, "..", "lib", "libbls381.so"))

OK = 0
EINVAL_POINT = -1
EARG = -2
ENODEV = -3
EHIP = -4
MSG_MAX = 1 << 20           # BLS381_MSG_MAX
POLICY = {"pyecc": 0, "strict": 1}   # BLS381_POLICY_PYECC / _STRICT

# every symbol include/bls381.h declares, with its ctypes signature
_u8p = ctypes.c_void_p
_SIGS = {
    "bls381_device_count": (ctypes.c_int, []),
    "bls381_init": (ctypes.c_int, [ctypes.c_int]),
    "bls381_init_devices": (ctypes.c_int, [ctypes.c_int]),
    "bls381_shutdown": (None, []),
    "bls381_last_error": (ctypes.c_char_p, []),
    "bls381_set_subgroup_policy": (ctypes.c_int, [ctypes.c_int]),
    "bls381_get_subgroup_policy": (ctypes.c_int, []),
    "bls381_set_thread_subgroup_policy": (ctypes.c_int, [ctypes.c_int]),
    "bls381_get_thread_subgroup_policy": (ctypes.c_int, []),
    "bls381_profile_enable": (ctypes.c_int, [ctypes.c_int]),
    "bls381_profile_read": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t]),
    "bls381_verify": (ctypes.c_int, [_u8p, _u8p, ctypes.c_size_t, _u8p, _u8p]),
    "bls381_verify_multiple": (ctypes.c_int, [ctypes.c_size_t, _u8p, _u8p, ctypes.c_size_t, _u8p, _u8p]),
    "bls381_aggregate_pubkeys": (ctypes.c_int, [ctypes.c_size_t, _u8p, _u8p]),
    "bls381_aggregate_signatures": (ctypes.c_int, [ctypes.c_size_t, _u8p, _u8p]),
    "bls381_aggregate_g1": (ctypes.c_int, [ctypes.c_size_t, _u8p, _u8p]),
    "bls381_aggregate_g2": (ctypes.c_int, [ctypes.c_size_t, _u8p, _u8p]),
    "bls381_sign": (ctypes.c_int, [_u8p, ctypes.c_size_t, _u8p, _u8p, _u8p]),
    "bls381_privtopub": (ctypes.c_int, [_u8p, _u8p]),
    "bls381_sign_batch": (ctypes.c_int, [ctypes.c_size_t, _u8p, _u8p, _u8p, _u8p]),
    "bls381_privtopub_batch": (ctypes.c_int, [ctypes.c_size_t, _u8p, _u8p]),
    "bls381_hash_to_g2": (ctypes.c_int, [_u8p, ctypes.c_size_t, _u8p, _u8p, _u8p]),
    "bls381_hash_to_g2_pyecc_projective": (ctypes.c_int, [ctypes.c_size_t, _u8p, _u8p, _u8p]),
    "bls381_verify_batch": (ctypes.c_int, [ctypes.c_size_t, _u8p, _u8p, _u8p, _u8p, _u8p]),
    "bls381_verify_batch_workspace_size": (ctypes.c_size_t, [ctypes.c_size_t]),
    "bls381_verify_batch_device": (ctypes.c_int, [ctypes.c_size_t, _u8p, _u8p, _u8p, _u8p, _u8p, _u8p, _u8p]),
    "bls381_verify_batch_randomized": (ctypes.c_int, [ctypes.c_size_t, _u8p, _u8p, _u8p, _u8p, _u8p, ctypes.c_size_t,
                                                      _u8p]),
    "bls381_verify_batch_randomized_workspace_size": (ctypes.c_size_t, [ctypes.c_size_t, ctypes.c_size_t]),
    "bls381_verify_batch_randomized_device": (ctypes.c_int, [ctypes.c_size_t, _u8p, _u8p, _u8p, _u8p, _u8p,
                                                             ctypes.c_size_t, _u8p, _u8p, _u8p, _u8p]),
    "bls381_aggregate_pubkeys_batch": (ctypes.c_int, [ctypes.c_size_t, _u8p, _u8p, _u8p, _u8p]),
    "bls381_aggregate_pubkeys_batch_workspace_size": (ctypes.c_size_t, [ctypes.c_size_t, ctypes.c_size_t]),
    "bls381_aggregate_pubkeys_batch_device": (ctypes.c_int, [ctypes.c_size_t, _u8p, ctypes.c_size_t, _u8p, _u8p,
                                                             _u8p, _u8p, _u8p]),
    "bls381_verify_multiple_batch": (ctypes.c_int, [ctypes.c_size_t, _u8p, _u8p, _u8p, ctypes.c_size_t, _u8p,
                                                    _u8p, _u8p]),
    "bls381_verify_multiple_batch_workspace_size": (ctypes.c_size_t, [ctypes.c_size_t, ctypes.c_size_t,
                                                                      ctypes.c_size_t]),
    "bls381_verify_multiple_batch_device": (ctypes.c_int, [ctypes.c_size_t, _u8p, _u8p, ctypes.c_size_t, _u8p, _u8p,
                                                           _u8p, _u8p, _u8p, _u8p]),
    "bls381_verify_multiple_grouped_workspace_size": (ctypes.c_size_t, [ctypes.c_size_t, ctypes.c_size_t,
                                                                        ctypes.c_size_t, ctypes.c_size_t]),
    "bls381_verify_multiple_grouped_device": (ctypes.c_int, [ctypes.c_size_t, _u8p, ctypes.c_size_t, _u8p, _u8p,
                                                             ctypes.c_size_t, _u8p, _u8p, _u8p, _u8p, _u8p, _u8p]),
    "bls381_miller_partial": (ctypes.c_int, [ctypes.c_size_t, _u8p, _u8p, ctypes.c_size_t, _u8p, ctypes.c_int,
                                             _u8p, _u8p]),
    "bls381_final_verify": (ctypes.c_int, [ctypes.c_size_t, _u8p]),
    "bls381_comm_unique_id": (ctypes.c_int, [_u8p]),
    "bls381_comm_rccl_path": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t]),
    "bls381_comm_init": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _u8p]),
    "bls381_comm_init_virtual": (ctypes.c_int, [ctypes.c_int]),
    "bls381_comm_size": (ctypes.c_int, []),
    "bls381_comm_rank": (ctypes.c_int, []),
    "bls381_comm_destroy": (None, []),
    "bls381_verify_multiple_sharded": (ctypes.c_int, [ctypes.c_size_t, _u8p, _u8p, ctypes.c_size_t, _u8p, _u8p]),
    "bls381_aggregate_pubkeys_sharded": (ctypes.c_int, [ctypes.c_size_t, _u8p, _u8p]),
    "bls381_aggregate_pubkeys_sharded_device_workspace_size": (ctypes.c_size_t, [ctypes.c_size_t]),
    "bls381_aggregate_pubkeys_sharded_device": (ctypes.c_int, [ctypes.c_size_t, _u8p, _u8p, _u8p, _u8p, _u8p]),
    "bls381_verify_multiple_batch_sharded": (ctypes.c_int, [ctypes.c_size_t, _u8p, _u8p, _u8p, ctypes.c_size_t,
                                                            _u8p, _u8p, _u8p]),
    "bls381_ssz_root_batch": (ctypes.c_int, [ctypes.c_size_t, _u8p, ctypes.c_size_t, _u8p, ctypes.c_uint32, _u8p]),
    "bls381_ssz_root_workspace_size": (ctypes.c_size_t, []),
    "bls381_ssz_root_batch_device": (ctypes.c_int, [ctypes.c_size_t, _u8p, ctypes.c_size_t, ctypes.c_size_t, _u8p,
                                                    ctypes.c_uint32, _u8p, _u8p, _u8p]),
    "bls381_verify_deposits": (ctypes.c_int, [ctypes.c_size_t, _u8p, _u8p, _u8p]),
    "bls381_verify_deposits_workspace_size": (ctypes.c_size_t, [ctypes.c_size_t]),
    "bls381_verify_deposits_device": (ctypes.c_int, [ctypes.c_size_t, _u8p, _u8p, _u8p, _u8p, _u8p]),
    "bls381_registry_create": (ctypes.c_int, [ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)]),
    "bls381_registry_destroy": (None, [ctypes.c_void_p]),
    "bls381_registry_size": (ctypes.c_size_t, [ctypes.c_void_p]),
    "bls381_registry_add": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, _u8p, _u8p]),
    "bls381_registry_verify_multiple_grouped_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, _u8p,
                                                                      ctypes.c_size_t, _u8p, _u8p, ctypes.c_size_t,
                                                                      _u8p, _u8p, _u8p, _u8p, _u8p, _u8p]),
    "bls381_registry_lookup": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, _u8p, _u8p]),
    "bls381_registry_aggregate_indices": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, _u8p, _u8p, _u8p,
                                                         _u8p]),
    "bls381_registry_aggregate_pubkeys_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, _u8p, _u8p,
                                                               _u8p, _u8p]),
    "bls381_registry_aggregate_workspace_size": (ctypes.c_size_t, [ctypes.c_size_t, ctypes.c_size_t]),
    "bls381_registry_aggregate_indices_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, _u8p,
                                                                ctypes.c_size_t, _u8p, _u8p, _u8p, _u8p, _u8p]),
}


class NativeUnavailable(RuntimeError):
    """The HIP engine is not usable (library missing, or no gfx950 device)."""


class NativeError(RuntimeError):
    pass


_lib = None
_lock = threading.Lock()
_checked_device = False


def load_library(path: str = LIB_PATH):
    """Load the shared library and bind every exported symbol (no device needed)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(path):
                raise NativeUnavailable(
                    "libbls381.so not found at %s -- build it with __graft_entry__.build()" % path)
            lib = ctypes.CDLL(path)
            for name, (res, args) in _SIGS.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


def lib():
    """The library, after checking that a device is present (fails loudly)."""
    global _checked_device
    L = load_library()
    if not _checked_device:
        if L.bls381_device_count() <= 0:
            raise NativeUnavailable("no HIP device visible: the gfx950 BLS engine has no CPU fallback")
        _checked_device = True
    return L


def last_error() -> str:
    e = load_library().bls381_last_error()
    return e.decode() if e else ""


def check(rc: int) -> int:
    if rc == ENODEV:
        raise NativeUnavailable("gfx950 device unavailable: " + last_error())
    if rc == EHIP:
        raise NativeError("HIP error: " + last_error())
    if rc == EARG:
        raise ValueError("invalid argument to bls381 engine")
    return rc


def _buf(b: bytes):
    return ctypes.c_char_p(b) if b else None


def init(device: int = 0) -> None:
    check(lib().bls381_init(device))


def set_subgroup_policy(name: str) -> None:
    """'pyecc' or 'strict' (include/bls381.h BLS381_POLICY_*); process-wide."""
    if name not in POLICY:
        raise ValueError("unknown subgroup policy %r (expected one of %s)" % (name, sorted(POLICY)))
    check(load_library().bls381_set_subgroup_policy(POLICY[name]))


def get_subgroup_policy() -> str:
    code = load_library().bls381_get_subgroup_policy()
    return {v: k for k, v in POLICY.items()}[code]


class subgroup_policy_scope:
    """Context manager: calls queued from this thread inside the block use `name`
    (bls381_set_thread_subgroup_policy); the process-wide policy is left alone and the
    thread's previous override is restored on exit."""

    def __init__(self, name: str):
        if name not in POLICY:
            raise ValueError("unknown subgroup policy %r (expected one of %s)" % (name, sorted(POLICY)))
        self.code = POLICY[name]

    def __enter__(self):
        lib_ = load_library()
        self.prev = _thread_override.get()
        check(lib_.bls381_set_thread_subgroup_policy(self.code))
        _thread_override.set(self.code)
        return self

    def __exit__(self, *exc):
        check(load_library().bls381_set_thread_subgroup_policy(self.prev))
        _thread_override.set(self.prev)
        return False


class _Override:
    """This thread's override as the library holds it (-1: none); mirrored here so a
    nested scope can restore it without another call."""
    _tls = __import__("threading").local()

    def get(self) -> int:
        return getattr(self._tls, "code", -1)

    def set(self, code: int) -> None:
        self._tls.code = code


_thread_override = _Override()


def get_thread_subgroup_policy() -> str:
    code = load_library().bls381_get_thread_subgroup_policy()
    return {v: k for k, v in POLICY.items()}[code]


def verify(pk: bytes, msg: bytes, sig: bytes, dom8: bytes) -> bool:
    rc = check(lib().bls381_verify(_buf(pk), _buf(msg), len(msg), _buf(sig), _buf(dom8)))
    return rc == 1


def verify_multiple(pks: bytes, msgs: bytes, msg_len: int, sig: bytes, dom8: bytes) -> bool:
    n = len(pks) // 48
    rc = check(lib().bls381_verify_multiple(n, _buf(pks), _buf(msgs), msg_len, _buf(sig), _buf(dom8)))
    return rc == 1


def aggregate_pubkeys(pks: bytes) -> bytes:
    out = ctypes.create_string_buffer(48)
    rc = check(lib().bls381_aggregate_pubkeys(len(pks) // 48, _buf(pks), out))
    if rc == EINVAL_POINT:
        raise ValueError("invalid G1 point encoding in aggregate_pubkeys")
    return out.raw


def aggregate_signatures(sigs: bytes) -> bytes:
    out = ctypes.create_string_buffer(96)
    rc = check(lib().bls381_aggregate_signatures(len(sigs) // 96, _buf(sigs), out))
    if rc == EINVAL_POINT:
        raise ValueError("invalid G2 point encoding in aggregate_signatures")
    return out.raw


def sign(msg: bytes, sk32: bytes, dom8: bytes) -> bytes:
    out = ctypes.create_string_buffer(96)
    check(lib().bls381_sign(_buf(msg), len(msg), _buf(sk32), _buf(dom8), out))
    return out.raw


def privtopub(sk32: bytes) -> bytes:
    out = ctypes.create_string_buffer(48)
    check(lib().bls381_privtopub(_buf(sk32), out))
    return out.raw


def sign_batch(msgs32: bytes, sks32: bytes, dom8s: bytes) -> bytes:
    n = len(msgs32) // 32
    out = ctypes.create_string_buffer(96 * max(n, 1))
    check(lib().bls381_sign_batch(n, _buf(msgs32), _buf(sks32), _buf(dom8s), out))
    return out.raw[:96 * n]


def privtopub_batch(sks32: bytes) -> bytes:
    n = len(sks32) // 32
    out = ctypes.create_string_buffer(48 * max(n, 1))
    check(lib().bls381_privtopub_batch(n, _buf(sks32), out))
    return out.raw[:48 * n]


def hash_to_g2(msg: bytes, dom8: bytes):
    comp = ctypes.create_string_buffer(96)
    aff = ctypes.create_string_buffer(192)
    check(lib().bls381_hash_to_g2(_buf(msg), len(msg), _buf(dom8), comp, aff))
    return comp.raw, aff.raw


def hash_to_g2_pyecc_projective(msgs32: bytes, dom8s: bytes) -> bytes:
    n = len(msgs32) // 32
    out = ctypes.create_string_buffer(288 * max(n, 1))
    check(lib().bls381_hash_to_g2_pyecc_projective(n, _buf(msgs32), _buf(dom8s), out))
    return out.raw[:288 * n]


def verify_batch(pks: bytes, msgs32: bytes, sigs: bytes, dom8s: bytes) -> np.ndarray:
    n = len(pks) // 48
    out = np.zeros(n, dtype=np.uint8)
    if n:
        check(lib().bls381_verify_batch(n, _buf(pks), _buf(msgs32), _buf(sigs), _buf(dom8s),
                                        out.ctypes.data_as(ctypes.c_void_p)))
    return out.astype(bool)


def verify_batch_randomized(pks: bytes, msgs32: bytes, sigs: bytes, dom8s: bytes, seed: bytes,
                            batch: int = 64) -> np.ndarray:
    """Opt-in randomized batch verification (bls381_verify_batch_randomized); per-item verdicts."""
    n = len(pks) // 48
    out = np.zeros(n, dtype=np.uint8)
    if n:
        check(lib().bls381_verify_batch_randomized(n, _buf(pks), _buf(msgs32), _buf(sigs), _buf(dom8s), _buf(seed),
                                                   batch, out.ctypes.data_as(ctypes.c_void_p)))
    return out.astype(bool)


def aggregate_pubkeys_batch(offsets: np.ndarray, pks: bytes):
    offsets = np.ascontiguousarray(offsets, dtype=np.uint32)
    ng = len(offsets) - 1
    out = ctypes.create_string_buffer(48 * max(ng, 1))
    status = np.zeros(max(ng, 1), dtype=np.int32)
    check(lib().bls381_aggregate_pubkeys_batch(ng, offsets.ctypes.data_as(ctypes.c_void_p), _buf(pks), out,
                                               status.ctypes.data_as(ctypes.c_void_p)))
    return [out.raw[48 * g:48 * g + 48] for g in range(ng)], status[:ng]


def verify_multiple_batch(call_off, pks: bytes, msgs: bytes, msg_len: int, sigs: bytes, dom8s: bytes) -> np.ndarray:
    """Batch of bls_verify_multiple calls; call c owns items [call_off[c], call_off[c+1])."""
    call_off = np.ascontiguousarray(call_off, dtype=np.uint32)
    nc = len(call_off) - 1
    out = np.zeros(max(nc, 1), dtype=np.uint8)
    check(lib().bls381_verify_multiple_batch(nc, call_off.ctypes.data_as(ctypes.c_void_p), _buf(pks), _buf(msgs),
                                             msg_len, _buf(sigs), _buf(dom8s), out.ctypes.data_as(ctypes.c_void_p)))
    return out[:nc].astype(bool)


def miller_partial(pks: bytes, msgs: bytes, msg_len: int, sig: bytes, include_sig: bool, dom8: bytes):
    out = ctypes.create_string_buffer(576)
    n = len(pks) // 48
    rc = check(lib().bls381_miller_partial(n, _buf(pks), _buf(msgs), msg_len, _buf(sig), int(include_sig),
                                           _buf(dom8), out))
    return rc, out.raw


def final_verify(parts: bytes) -> bool:
    k = len(parts) // 576
    return check(lib().bls381_final_verify(k, _buf(parts))) == 1


def profile_enable(on: bool) -> None:
    lib().bls381_profile_enable(int(on))


def profile_read() -> dict:
    import json
    buf = ctypes.create_string_buffer(1 << 16)
    n = lib().bls381_profile_read(buf, len(buf))
    if n < 0:
        raise NativeError("profile_read failed")
    return json.loads(buf.value.decode())
