"""Device-resident registry of decoded validator pubkeys.

The reference aggregates committee pubkeys out of the validator registry on every
attestation (specs/core/0_beacon-chain.md:1025-1026:
``bls_aggregate_pubkeys([state.validator_registry[i].pubkey for i in indices])``),
and py_ecc decompresses every member each time (an Fp square root per key).
Validator pubkeys never change, so the engine decodes each one once into HBM
(include/bls381.h ``bls381_registry_*``) and aggregates by validator index, or by
content lookup of the compressed bytes.  Results are byte-identical to
``bls_aggregate_pubkeys`` over the same encodings, with the same error behaviour
(an undecodable member raises ValueError).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native


class PubkeyRegistry:
    """Append-only table of decoded pubkeys on the current device.

    Entry ``e`` is the ``e``-th key ever added, so adding
    ``state.validator_registry`` in order makes entries validator indices.
    """

    def __init__(self, capacity: int):
        L = _native.lib()
        h = ctypes.c_void_p()
        _native.check(L.bls381_registry_create(int(capacity), ctypes.byref(h)))
        self._h = h
        self.capacity = int(capacity)

    def close(self) -> None:
        if getattr(self, "_h", None):
            _native.lib().bls381_registry_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self) -> int:
        return int(_native.lib().bls381_registry_size(self._h))

    def add(self, pubkeys) -> np.ndarray:
        """Append keys; returns per key the entry holding its bytes (-1: does not decode)."""
        blob = _join48(pubkeys)
        n = len(blob) // 48
        out = np.zeros(n, dtype=np.int32)
        if n:
            rc = _native.lib().bls381_registry_add(self._h, n, blob, out.ctypes.data_as(ctypes.c_void_p))
            _native.check(rc)
        return out

    def lookup(self, pubkeys) -> np.ndarray:
        blob = _join48(pubkeys)
        n = len(blob) // 48
        out = np.zeros(n, dtype=np.int32)
        if n:
            _native.check(_native.lib().bls381_registry_lookup(self._h, n, blob,
                                                               out.ctypes.data_as(ctypes.c_void_p)))
        return out

    def aggregate_indices(self, groups) -> list:
        """bls_aggregate_pubkeys over registry entries, one result per group (list of index lists)."""
        groups = [np.asarray(g, dtype=np.int64) for g in groups]
        if any(g.size and (g.min() < 0 or g.max() >= 1 << 32) for g in groups):
            raise ValueError("registry index out of range")
        off = np.zeros(len(groups) + 1, dtype=np.uint32)
        off[1:] = np.cumsum([g.size for g in groups])
        idx = np.concatenate(groups).astype(np.uint32) if groups and off[-1] else np.zeros(1, np.uint32)
        return self._run(_native.lib().bls381_registry_aggregate_indices, off, idx.ctypes.data_as(ctypes.c_void_p))

    def aggregate_pubkeys_batch(self, groups) -> list:
        """bls_aggregate_pubkeys per group of compressed keys; registered members are not re-decoded."""
        blobs = [_join48(g) for g in groups]
        off = np.zeros(len(groups) + 1, dtype=np.uint32)
        off[1:] = np.cumsum([len(b) // 48 for b in blobs])
        data = b"".join(blobs)
        return self._run(_native.lib().bls381_registry_aggregate_pubkeys_batch, off, data if data else None)

    def aggregate_pubkeys(self, pubkeys) -> bytes:
        return self.aggregate_pubkeys_batch([pubkeys])[0]

    def _run(self, fn, off, src):
        ng = len(off) - 1
        if ng == 0:
            return []
        out = ctypes.create_string_buffer(48 * ng)
        st = np.zeros(ng, dtype=np.int32)
        _native.check(fn(self._h, ng, off.ctypes.data_as(ctypes.c_void_p), src, out,
                         st.ctypes.data_as(ctypes.c_void_p)))
        if np.any(st == _native.EINVAL_POINT):
            raise ValueError("invalid pubkey encoding in aggregate")
        raw = out.raw
        return [raw[48 * g:48 * g + 48] for g in range(ng)]


def _join48(keys) -> bytes:
    ks = [bytes(k) for k in keys]
    if any(len(k) != 48 for k in ks):
        raise ValueError("pubkeys must be 48 bytes")
    return b"".join(ks)
