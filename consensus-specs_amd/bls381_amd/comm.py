"""Native multi-GPU calls over the library's own RCCL communicator -- ctypes only, no PyTorch.

One process per GPU.  Rank 0 makes RCCL's 128-byte unique id;
`exchange_unique_id` hands it to the other ranks over a plain TCP socket at
MASTER_ADDR:port (the address torchrun-style launchers export; 127.0.0.1 on
one node), then every rank calls `init`.  The collective entry points mirror
the single-GPU ones (include/bls381.h "native multi-GPU over RCCL"):

* verify_multiple(pubkeys, message_hashes, signature, domain) -- one call split
  over the ranks by distinct message, one final exponentiation on rank 0;
* aggregate_pubkeys(pubkeys) -- contiguous ranges, partials summed on rank 0;
* verify_multiple_batch(calls) -- independent calls, contiguous call ranges.

bls381_amd.sharding holds the same protocols over torch.distributed, used by
the CPU (gloo) tests of the partition / gather / single-FE logic.
"""
from __future__ import annotations

import ctypes
import socket
import struct
import time
from typing import List, Sequence

import numpy as np

from . import _native

UID_BYTES = 128


def unique_id() -> bytes:
    out = ctypes.create_string_buffer(UID_BYTES)
    _native.check(_native.load_library().bls381_comm_unique_id(out))
    return out.raw


def exchange_unique_id(rank: int, world: int, addr: str = "127.0.0.1", port: int = 29517,
                       timeout: float = 120.0, make_id=None) -> bytes:
    """Rank 0 makes the id and serves it to world - 1 peers; the others fetch it.

    make_id: the id factory (default: RCCL's, through bls381_comm_unique_id).  The CPU
    tests pass a stub, so the rendezvous runs without a GPU (tests/test_sharding.py)."""
    make_id = make_id or unique_id
    if world == 1:
        return make_id()
    if rank == 0:
        uid = make_id()
        if len(uid) != UID_BYTES:
            raise ValueError("unique id must be %d bytes" % UID_BYTES)
        srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        srv.bind((addr, port))
        srv.listen(world)
        srv.settimeout(timeout)
        try:
            for _ in range(world - 1):
                conn, _ = srv.accept()
                with conn:
                    conn.sendall(struct.pack("!I", UID_BYTES) + uid)
        finally:
            srv.close()
        return uid
    deadline = time.time() + timeout
    while True:
        try:
            with socket.create_connection((addr, port), timeout=5.0) as s:
                data = b""
                while len(data) < 4 + UID_BYTES:
                    chunk = s.recv(4 + UID_BYTES - len(data))
                    if not chunk:
                        break
                    data += chunk
            if len(data) == 4 + UID_BYTES and struct.unpack("!I", data[:4])[0] == UID_BYTES:
                return data[4:]
        except OSError:
            pass
        if time.time() > deadline:
            raise TimeoutError("no unique id from rank 0 at %s:%d" % (addr, port))
        time.sleep(0.05)


def rccl_path() -> str:
    """The RCCL shared object the library's communicator uses (bls381_comm_rccl_path)."""
    buf = ctypes.create_string_buffer(4096)
    _native.check(_native.load_library().bls381_comm_rccl_path(buf, len(buf)))
    return buf.value.decode()


def loaded_rccl_paths() -> List[str]:
    """Every librccl mapped into this process (from /proc/self/maps), resolved."""
    import os
    out = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                parts = line.split()
                if len(parts) >= 6 and "librccl" in os.path.basename(parts[-1]):
                    out.add(os.path.realpath(parts[-1]))
    except OSError:
        pass
    return sorted(out)


def init(world: int, rank: int, uid: bytes) -> None:
    """Create this process's communicator on the device chosen with _native.init."""
    _native.check(_native.lib().bls381_comm_init(world, rank, uid))


def init_virtual(world: int) -> None:
    """This process plays all `world` ranks on its GPU (the N-rank protocol on one GPU)."""
    _native.check(_native.lib().bls381_comm_init_virtual(world))


def size() -> int:
    return _native.load_library().bls381_comm_size()


def rank() -> int:
    return _native.load_library().bls381_comm_rank()


def destroy() -> None:
    _native.load_library().bls381_comm_destroy()


def verify_multiple(pubkeys: Sequence[bytes], message_hashes: Sequence[bytes], signature: bytes,
                    domain: int, byteorder: str = "big") -> bool:
    """Collective bls_verify_multiple; every rank passes the same call and gets the verdict."""
    if len(pubkeys) != len(message_hashes):
        raise ValueError("len(pubkeys) (%s) should be equal to len(message_hashes) (%s)"
                         % (len(pubkeys), len(message_hashes)))
    pks = [bytes(p) for p in pubkeys]
    msgs = [bytes(m) for m in message_hashes]
    lens = {len(m) for m in msgs}
    if any(len(p) != 48 for p in pks) or len(bytes(signature)) != 96 or len(lens) > 1:
        raise ValueError("collective verify_multiple takes 48-byte keys, a 96-byte signature, equal-length messages")
    mlen = lens.pop() if lens else 32
    rc = _native.check(_native.lib().bls381_verify_multiple_sharded(
        len(pks), _native._buf(b"".join(pks)), _native._buf(b"".join(msgs)), mlen, _native._buf(bytes(signature)),
        _native._buf(int(domain).to_bytes(8, byteorder))))
    return rc == 1


def aggregate_pubkeys(pubkeys: Sequence[bytes]) -> bytes:
    """Collective bls_aggregate_pubkeys; ValueError on every rank for an invalid encoding."""
    blob = b"".join(bytes(p) for p in pubkeys)
    if len(blob) != 48 * len(pubkeys):
        raise ValueError("pubkeys must be 48 bytes")
    out = ctypes.create_string_buffer(48)
    rc = _native.check(_native.lib().bls381_aggregate_pubkeys_sharded(len(pubkeys), _native._buf(blob), out))
    if rc == _native.EINVAL_POINT:
        raise ValueError("invalid G1 point encoding in aggregate_pubkeys")
    return out.raw


def aggregate_pubkeys_device_workspace_size(n_local: int) -> int:
    return int(_native.lib().bls381_aggregate_pubkeys_sharded_device_workspace_size(n_local))


def aggregate_pubkeys_device(n_local: int, d_pks: int, d_out48: int, d_status: int, d_workspace: int,
                             stream: int = 0) -> None:
    """Collective bls_aggregate_pubkeys over device-resident keys (device pointers as ints): this
    rank's n_local keys in, the aggregate (48 B) and the status (int32, 0 or EINVAL_POINT) out on every
    rank, queued on `stream`; no host copy, no synchronisation."""
    _native.check(_native.lib().bls381_aggregate_pubkeys_sharded_device(
        n_local, ctypes.c_void_p(d_pks), ctypes.c_void_p(d_out48), ctypes.c_void_p(d_status),
        ctypes.c_void_p(d_workspace), ctypes.c_void_p(stream)))


def verify_multiple_batch(call_off, pks: bytes, msgs: bytes, msg_len: int, sigs: bytes, dom8s: bytes) -> List[bool]:
    """Independent calls over the ranks (same arguments on every rank); all verdicts on every rank."""
    call_off = np.ascontiguousarray(call_off, dtype=np.uint32)
    nc = len(call_off) - 1
    out = np.zeros(max(nc, 1), dtype=np.uint8)
    _native.check(_native.lib().bls381_verify_multiple_batch_sharded(
        nc, call_off.ctypes.data_as(ctypes.c_void_p), _native._buf(pks), _native._buf(msgs), msg_len,
        _native._buf(sigs), _native._buf(dom8s), out.ctypes.data_as(ctypes.c_void_p)))
    return [bool(v) for v in out[:nc]]
