"""Multi-rank bls_verify_multiple protocol (bls381_amd.sharding) on CPU/gloo.

World size 2, gloo backend, 127.0.0.1.  The per-rank partial product and the
final exponentiation use the CPU model of the engine's tower
(oracle/tower_model.py) in place of the GPU, so the partition / all-gather /
single-final-exponentiation protocol is checked here; the GPU-side partials
are checked by tests/test_gpu_parity.py::test_partial_products_combine.
"""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def model_partial(pks, msgs, mlen, sig, include_sig, dom8):
    import bls_oracle as O
    import tower_model as M
    pairs = []
    n = len(pks) // 48
    groups = {}
    order = []
    for i in range(n):
        m = msgs[mlen * i:mlen * (i + 1)]
        if m not in groups:
            groups[m] = O.Z1
            order.append(m)
        groups[m] = O.pt_add(O.FqOps, groups[m], O.pubkey_to_G1(pks[48 * i:48 * (i + 1)]))
    dom = int.from_bytes(dom8, "big")
    for m in order:
        if O.pt_is_inf(O.FqOps, groups[m]):
            continue
        pairs.append((O.g2_affine(O.hash_to_G2(m, dom)), O.pt_normalize(O.FqOps, groups[m])))
    if include_sig:
        s = O.signature_to_G2(sig)
        if not O.pt_is_inf(O.Fq2Ops, s):
            pairs.append((O.g2_affine(s), (O.g_x, (-O.g_y) % O.q)))
    f = M.miller_loop_multi(pairs) if pairs else M.ONE12
    return 0, b"".join(c[0].to_bytes(48, "big") + c[1].to_bytes(48, "big") for c in f)


def model_final(parts):
    import tower_model as M
    f = M.ONE12
    for k in range(len(parts) // 576):
        p = parts[576 * k:576 * (k + 1)]
        g = tuple((int.from_bytes(p[96 * i:96 * i + 48], "big"), int.from_bytes(p[96 * i + 48:96 * i + 96], "big"))
                  for i in range(6))
        f = M.mul12(f, g)
    return M.final_exp(f) == M.ONE12


def model_batch(call_off, pks, msgs, mlen, sigs, dom8s):
    """CPU stand-in for bls381_verify_multiple_batch: the oracle, call by call."""
    import bls_oracle as O
    out = []
    for c in range(len(call_off) - 1):
        a, b = call_off[c], call_off[c + 1]
        out.append(O.verify_multiple([pks[48 * i:48 * i + 48] for i in range(a, b)],
                                     [msgs[mlen * i:mlen * i + mlen] for i in range(a, b)],
                                     sigs[96 * c:96 * c + 96], int.from_bytes(dom8s[8 * c:8 * c + 8], "big")))
    return out


def model_mixed(pks, msgs, sig, dom8):
    """CPU stand-in for one mixed-length call (bls.verify_multiple_bytes)."""
    import bls_oracle as O
    return O.verify_multiple(pks, msgs, sig, int.from_bytes(dom8, "big"))


def _oracle_agg(pks):
    import bls_oracle as O
    return O.aggregate_pubkeys([pks[48 * i:48 * i + 48] for i in range(len(pks) // 48)])


def _worker(rank, world, port, case, q, kind="vm"):
    sys.path.insert(0, os.path.join(ROOT, "consensus-specs_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch.distributed as dist
    from bls381_amd import sharding
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    if kind == "vm":
        pks, msgs, sig, dom = case
        v = sharding.sharded_verify_multiple(pks, msgs, sig, dom, rank=rank, world=world,
                                             partial_fn=model_partial, final_fn=model_final)
    elif kind == "agg":
        try:
            v = sharding.sharded_aggregate_pubkeys(case, rank=rank, world=world, agg_fn=_oracle_agg)
        except ValueError:
            v = "ValueError"
    else:
        v = sharding.sharded_verify_multiple_batch(case, rank=rank, world=world, batch_fn=model_batch,
                                                   mixed_fn=model_mixed)
    q.put((rank, v))
    dist.barrier()
    dist.destroy_process_group()


def _run(case, world=2, kind="vm"):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, q, kind)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
        assert p.exitcode == 0
    res = dict(q.get() for _ in range(world))
    return res


@pytest.fixture(scope="module")
def case():
    import bls_oracle as O
    sks = [11, 22, 33, 44]
    msgs = [b"\x01" * 32, b"\x02" * 32, b"\x01" * 32, b"\x03" * 32]
    pks = [O.privtopub(k) for k in sks]
    sig = O.aggregate_signatures([O.sign(m, k, 5) for m, k in zip(msgs, sks)])
    return pks, msgs, sig, 5


def test_partition_keeps_message_groups_on_one_rank():
    from bls381_amd.sharding import partition_messages
    msgs = [b"a", b"b", b"a", b"c", b"b", b"d"]
    sh = partition_messages(msgs, 2)
    assert sorted(sh[0] + sh[1]) == list(range(6))
    for r in range(2):
        for m in {msgs[i] for i in sh[r]}:
            assert all(i in sh[r] for i in range(6) if msgs[i] == m)


def test_sharded_verify_multiple_gloo_world2(case):
    import bls_oracle as O
    pks, msgs, sig, dom = case
    assert O.verify_multiple(pks, msgs, sig, dom) is True
    res = _run(case)
    assert res == {0: True, 1: True}
    bad = (pks[::-1], msgs, sig, dom)
    res = _run(bad)
    assert res == {0: False, 1: False}


def test_sharded_verify_multiple_mixed_lengths_gloo_world2():
    """Messages of several lengths in one call: one partial per length per rank, one FE."""
    import bls_oracle as O
    sks = [11, 22, 33, 44, 55]
    msgs = [b"\x01" * 32, b"\x02" * 20, b"\x01" * 32, b"\x03" * 40, b""]
    pks = [O.privtopub(k) for k in sks]
    sig = O.aggregate_signatures([O.sign(m, k, 5) for m, k in zip(msgs, sks)])
    assert O.verify_multiple(pks, msgs, sig, 5) is True
    assert _run((pks, msgs, sig, 5)) == {0: True, 1: True}
    assert _run((pks, msgs[:4] + [b"x"], sig, 5)) == {0: False, 1: False}


def test_shard_range_covers_everything():
    from bls381_amd.sharding import shard_range
    for n in (0, 1, 5, 8, 1 << 20):
        for world in (1, 2, 3, 8):
            rs = [shard_range(n, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[r][1] == rs[r + 1][0] for r in range(world - 1))
            assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1


def test_sharded_aggregate_pubkeys_gloo_world2():
    """C4 protocol: per-rank compressed partials, summed on rank 0 == one aggregate over all keys."""
    import bls_oracle as O
    keys = [O.privtopub(k) for k in range(1, 8)]
    res = _run(keys, kind="agg")
    want = O.privtopub(sum(range(1, 8)))
    assert res == {0: want, 1: want}
    # an encoding neither codec decodes (x^3 + 4 not a square) on rank 1's half raises on both ranks
    x = next(x for x in range(1, 100) if pow((x ** 3 + 4) % O.q, (O.q - 1) // 2, O.q) != 1)
    res = _run(keys[:6] + [(2 ** 383 + x).to_bytes(48, "big")], kind="agg")
    assert res == {0: "ValueError", 1: "ValueError"}
    # fewer keys than ranks: the empty shard contributes infinity
    res = _run(keys[:1], kind="agg")
    assert res == {0: keys[0], 1: keys[0]}


def test_sharded_verify_multiple_batch_gloo_world2(case):
    """C4 second half: independent calls sharded by call; every rank gets all verdicts in order."""
    import bls_oracle as O
    pks, msgs, sig, dom = case
    inf_sig = O.aggregate_signatures([])
    calls = [
        (pks[:1], msgs[:1], O.sign(msgs[0], 11, 5), 5),        # True
        ([], [], inf_sig, 7),                                   # True (empty product)
        (pks[:1], msgs[:1], O.sign(msgs[0], 11, 5), 6),        # wrong domain
        ([], [], O.sign(msgs[0], 11, 5), 7),                    # empty call, non-infinite signature
        (pks[:1], [b"\x01" * 31], O.sign(msgs[0], 11, 5), 5),  # other message length
        (pks[:2], [msgs[0], b"\x07" * 7],                      # mixed lengths in one call
         O.aggregate_signatures([O.sign(msgs[0], 11, 5), O.sign(b"\x07" * 7, 22, 5)]), 5),
    ]
    want = [True, True, False, False, False, True]
    res = _run(calls, kind="batch")
    assert res == {0: want, 1: want}


# ---------------------------------------- native communicator rendezvous (comm.py)
def _uid_worker(rank, world, port, q):
    sys.path.insert(0, os.path.join(ROOT, "consensus-specs_amd"))
    from bls381_amd import comm
    stub = bytes((7 * k + 3) % 256 for k in range(comm.UID_BYTES))
    got = comm.exchange_unique_id(rank, world, "127.0.0.1", port, timeout=60.0, make_id=lambda: stub)
    q.put((rank, got))


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_unique_id_tcp(world):
    """comm.exchange_unique_id over real sockets at 127.0.0.1: rank 0 serves a stub 128-byte id
    (RCCL's would need a GPU) and every rank ends with the same bytes.  The non-zero ranks may
    start before rank 0 listens; they retry until it does."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_uid_worker, args=(r, world, port, q)) for r in reversed(range(world))]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(out) == list(range(world))
    assert len({v for v in out.values()}) == 1 and len(out[0]) == 128


def test_exchange_unique_id_times_out_without_rank0():
    sys.path.insert(0, os.path.join(ROOT, "consensus-specs_amd"))
    from bls381_amd import comm
    with pytest.raises(TimeoutError):
        comm.exchange_unique_id(1, 2, "127.0.0.1", _free_port(), timeout=0.5, make_id=lambda: b"\0" * 128)


def test_exchange_unique_id_rejects_wrong_size():
    sys.path.insert(0, os.path.join(ROOT, "consensus-specs_amd"))
    from bls381_amd import comm
    with pytest.raises(ValueError):
        comm.exchange_unique_id(0, 2, "127.0.0.1", _free_port(), timeout=0.5, make_id=lambda: b"\0" * 5)
