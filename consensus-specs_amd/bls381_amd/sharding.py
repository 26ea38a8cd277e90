"""Multi-GPU bls_verify_multiple: one Fp12 partial per rank.

The distinct messages of a call are dealt round-robin to ranks (a message's
pubkey group never straddles two ranks, so each rank's group sums and subgroup
checks are the single-GPU ones).  Each rank computes the Miller-loop product
of its pairs (rank 0 also the (signature, -g1) pair) with
`bls381_miller_partial`; the 576-byte partials and their status bytes are
all-gathered (RCCL over xGMI with backend "nccl", or gloo on CPU); rank 0
multiplies them and runs ONE final exponentiation (`bls381_final_verify`),
exactly py_ecc's single-FE semantics; the verdict is broadcast.

Also here:

* `sharded_aggregate_pubkeys`: contiguous pubkey ranges per rank; each rank
  aggregates its range to one compressed partial (48 B + status), the
  partials are all-gathered and rank 0 sums them (G1 addition is associative,
  and compress/decompress of a partial is exact); the result is broadcast.
  Any invalid encoding on any rank raises ValueError on every rank, as
  py_ecc's aggregate_pubkeys does.
* `sharded_verify_multiple_batch`: many independent verify_multiple calls,
  contiguous call ranges per rank (a call's final exponentiation is never
  split); verdict bytes are all-gathered so every rank returns all of them.

`partial_fn` / `final_fn` / `agg_fn` / `batch_fn` default to the native
engine; tests substitute CPU models to exercise the protocols without a GPU.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence

PART_BYTES = 576
MSG_MAX = 1 << 20   # BLS381_MSG_MAX


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
    if any(len(m) > MSG_MAX for m in msgs):
        raise ValueError("message longer than the engine's %d-byte limit" % MSG_MAX)
    bad_shape = any(len(p) != 48 for p in pks) or len(bytes(signature)) != 96
    mine = partition_messages(msgs, world)[rank]
    # one partial per distinct message length (the batch ABI takes one length
    # per launch); every rank sends one per length of the whole call, so the
    # all-gathered payloads have equal sizes.  The signature pair rides in rank
    # 0's first partial.
    lens = sorted({len(m) for m in msgs}) or [32]
    st, parts = 0, []
    for j, mlen in enumerate(lens):
        sel = [i for i in mine if len(msgs[i]) == mlen]
        if bad_shape:
            s, part = 1, bytes(PART_BYTES)
        else:
            s, part = partial_fn(b"".join(pks[i] for i in sel), b"".join(msgs[i] for i in sel), mlen,
                                 bytes(signature), rank == 0 and j == 0, dom8)
        st |= 1 if s else 0
        parts.append(part)
    dev = device if device is not None else torch.device("cpu")
    payload = torch.tensor(list(bytes([st]) + b"".join(parts)), dtype=torch.uint8, device=dev)
    gathered = [torch.empty_like(payload) for _ in range(world)]
    dist.all_gather(gathered, payload, group=group)
    verdict = torch.zeros(1, dtype=torch.uint8, device=dev)
    if rank == 0:
        rows = [bytes(g.cpu().tolist()) for g in gathered]
        if all(r[0] == 0 for r in rows):
            verdict[0] = 1 if final_fn(b"".join(r[1:] for r in rows)) else 0
    dist.broadcast(verdict, src=0, group=group)
    return bool(verdict.item())


def shard_range(n: int, rank: int, world: int):
    """Contiguous [lo, hi) of n units for `rank` (sizes differ by at most one)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def _native_agg(pks: bytes) -> bytes:
    """Aggregate -> compressed 48 B; ValueError on an invalid encoding."""
    from . import _native
    return _native.aggregate_pubkeys(pks)


def _gather_bytes(payload: bytes, world: int, group, dev):
    import torch
    import torch.distributed as dist
    t = torch.tensor(list(payload), dtype=torch.uint8, device=dev)
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t, group=group)
    return [bytes(o.cpu().tolist()) for o in out]


def sharded_aggregate_pubkeys(pubkeys, *, rank: int, world: int, group=None, device=None,
                              agg_fn: Optional[Callable] = None) -> bytes:
    """bls_aggregate_pubkeys over `world` ranks; every rank passes the same list."""
    import torch
    import torch.distributed as dist
    agg_fn = agg_fn or _native_agg
    dev = device if device is not None else torch.device("cpu")
    lo, hi = shard_range(len(pubkeys), rank, world)
    try:
        part, st = agg_fn(b"".join(bytes(p) for p in pubkeys[lo:hi])), 0
        if len(part) != 48:
            raise ValueError("partial aggregate is not 48 bytes")
    except ValueError:
        part, st = bytes(48), 1
    rows = _gather_bytes(bytes([st]) + part, world, group, dev)
    res = torch.zeros(49, dtype=torch.uint8, device=dev)
    if rank == 0:
        if any(r[0] for r in rows):
            res[0] = 1
        else:
            res[1:] = torch.tensor(list(agg_fn(b"".join(r[1:] for r in rows))), dtype=torch.uint8)
    dist.broadcast(res, src=0, group=group)
    out = bytes(res.cpu().tolist())
    if out[0]:
        raise ValueError("invalid pubkey encoding in aggregate")
    return out[1:]


def _native_batch(call_off, pks: bytes, msgs: bytes, mlen: int, sigs: bytes, dom8s: bytes):
    from . import _native
    return [bool(v) for v in _native.verify_multiple_batch(call_off, pks, msgs, mlen, sigs, dom8s)]


def _native_mixed(pks, msgs, sig: bytes, dom8: bytes) -> bool:
    from . import bls
    return bls.verify_multiple_bytes(pks, msgs, sig, dom8)


def sharded_verify_multiple_batch(calls, *, rank: int, world: int, group=None, device=None,
                                  batch_fn: Optional[Callable] = None, mixed_fn: Optional[Callable] = None,
                                  byteorder: str = "big") -> List[bool]:
    """Independent calls (pubkeys, message_hashes, signature, domain), contiguous ranges per rank.

    Every rank passes the same call list and gets every verdict back.  A call
    whose list lengths differ raises ValidationError on every rank, before any
    collective, as the single-call API does.
    """
    import torch
    batch_fn = batch_fn or _native_batch
    for pks, msgs, _, _ in calls:
        if len(pks) != len(msgs):
            raise ValidationError("len(pubkeys) (%s) should be equal to len(message_hashes) (%s)"
                                  % (len(pks), len(msgs)))
    dev = device if device is not None else torch.device("cpu")
    lo, hi = shard_range(len(calls), rank, world)
    mine = calls[lo:hi]
    for _, msgs, _, _ in calls:
        if any(len(bytes(m)) > MSG_MAX for m in msgs):
            raise ValueError("message longer than the engine's %d-byte limit" % MSG_MAX)
    # the batch ABI takes one message length per launch: bucket calls by it;
    # bad sizes -> False, as bls.bls_verify_multiple; a call mixing message
    # lengths goes through mixed_fn (per-length partial products, one FE)
    mixed_fn = mixed_fn or _native_mixed
    verdicts = [False] * len(mine)
    buckets = {}
    for j, (pks, msgs, s, d) in enumerate(mine):
        if any(len(bytes(p)) != 48 for p in pks) or len(bytes(s)) != 96:
            continue
        lens = {len(bytes(m)) for m in msgs}
        if len(lens) > 1:
            verdicts[j] = bool(mixed_fn([bytes(p) for p in pks], [bytes(m) for m in msgs], bytes(s),
                                        int(d).to_bytes(8, byteorder)))
            continue
        buckets.setdefault(lens.pop() if lens else 32, []).append(j)
    for mlen, idx in buckets.items():
        run = [mine[j] for j in idx]
        off = [0]
        for pks, _, _, _ in run:
            off.append(off[-1] + len(pks))
        got = batch_fn(off, b"".join(bytes(p) for c in run for p in c[0]),
                       b"".join(bytes(m) for c in run for m in c[1]), mlen,
                       b"".join(bytes(c[2]) for c in run),
                       b"".join(int(c[3]).to_bytes(8, byteorder) for c in run))
        for j, v in zip(idx, got):
            verdicts[j] = bool(v)
    width = shard_range(len(calls), 0, world)[1]   # rank 0 holds the largest range
    pad = bytes(1 if v else 0 for v in verdicts) + bytes(width - len(verdicts))
    rows = _gather_bytes(pad, world, group, dev) if world > 1 else [pad]
    out: List[bool] = []
    for r in range(world):
        a, b = shard_range(len(calls), r, world)
        out.extend(bool(x) for x in rows[r][:b - a])
    return out
