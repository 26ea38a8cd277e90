"""Multi-GPU bls_verify_multiple: one Fp12 partial per rank.

The distinct messages of a call are dealt round-robin to ranks (a message's
pubkey group never straddles two ranks, so each rank's group sums and subgroup
checks are the single-GPU ones).  Each rank computes the Miller-loop product
of its pairs (rank 0 also the (signature, -g1) pair) with
`bls381_miller_partial`; the 576-byte partials and their status bytes are
all-gathered (RCCL over xGMI with backend "nccl", or gloo on CPU); rank 0
multiplies them and runs ONE final exponentiation (`bls381_final_verify`),
exactly py_ecc's single-FE semantics; the verdict is broadcast.

`partial_fn` / `final_fn` default to the native engine; tests substitute the
CPU model of the same tower to exercise the protocol without a GPU.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence

PART_BYTES = 576


class ValidationError(ValueError):
    pass


def partition_messages(message_hashes: Sequence[bytes], world: int) -> List[List[int]]:
    """Indices of the items each rank handles: distinct message k -> rank k % world."""
    order = {}
    for m in message_hashes:
        if m not in order:
            order[m] = len(order)
    shards: List[List[int]] = [[] for _ in range(world)]
    for i, m in enumerate(message_hashes):
        shards[order[m] % world].append(i)
    return shards


def _native_partial(pks: bytes, msgs: bytes, mlen: int, sig: bytes, include_sig: bool, dom8: bytes):
    from . import _native
    return _native.miller_partial(pks, msgs, mlen, sig, include_sig, dom8)


def _native_final(parts: bytes) -> bool:
    from . import _native
    return _native.final_verify(parts)


def sharded_verify_multiple(pubkeys, message_hashes, signature, domain, *, rank: int, world: int,
                            group=None, device=None, partial_fn: Optional[Callable] = None,
                            final_fn: Optional[Callable] = None, byteorder: str = "big") -> bool:
    import torch
    import torch.distributed as dist
    if len(pubkeys) != len(message_hashes):
        raise ValidationError("len(pubkeys) (%s) should be equal to len(message_hashes) (%s)"
                              % (len(pubkeys), len(message_hashes)))
    partial_fn = partial_fn or _native_partial
    final_fn = final_fn or _native_final
    dom8 = int(domain).to_bytes(8, byteorder)
    msgs = [bytes(m) for m in message_hashes]
    pks = [bytes(p) for p in pubkeys]
    mlen = len(msgs[0]) if msgs else 32
    bad_shape = any(len(p) != 48 for p in pks) or len(bytes(signature)) != 96 or any(len(m) != mlen for m in msgs)
    mine = partition_messages(msgs, world)[rank]
    if bad_shape:
        st, part = 1, bytes(PART_BYTES)
    else:
        st, part = partial_fn(b"".join(pks[i] for i in mine), b"".join(msgs[i] for i in mine), mlen,
                              bytes(signature), rank == 0, dom8)
    dev = device if device is not None else torch.device("cpu")
    payload = torch.tensor(list(bytes([1 if st else 0]) + part), dtype=torch.uint8, device=dev)
    gathered = [torch.empty_like(payload) for _ in range(world)]
    dist.all_gather(gathered, payload, group=group)
    verdict = torch.zeros(1, dtype=torch.uint8, device=dev)
    if rank == 0:
        rows = [bytes(g.cpu().tolist()) for g in gathered]
        if all(r[0] == 0 for r in rows):
            verdict[0] = 1 if final_fn(b"".join(r[1:] for r in rows)) else 0
    dist.broadcast(verdict, src=0, group=group)
    return bool(verdict.item())
