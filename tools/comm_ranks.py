"""N processes, one RCCL rank each, through the library's native communicator
(bls381_amd.comm, ctypes only): collective verify_multiple / aggregate_pubkeys /
verify_multiple_batch on the golden fixtures, every rank checking the verdicts.

    python tools/comm_ranks.py N [port]      (spawns N ranks; all on device 0 when
                                              only one GPU is visible)
"""
import json
import multiprocessing as mp
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "consensus-specs_amd"))


def worker(rank, world, port, q):
    try:
        from bls381_amd import _native, comm
        ndev = _native.load_library().bls381_device_count()
        _native.init(rank % max(ndev, 1))
        uid = comm.exchange_unique_id(rank, world, "127.0.0.1", port)
        comm.init(world, rank, uid)
        gb = json.load(open(os.path.join(ROOT, "tests", "golden", "bls_golden_batches.json")))
        h = bytes.fromhex
        vms = [c for c in gb["verify_multiple"] if len(c["pubkeys"]) == len(c["messages"])]
        got = [comm.verify_multiple([h(p) for p in c["pubkeys"]], [h(m) for m in c["messages"]], h(c["signature"]),
                                    int(c["domain"])) for c in vms]
        ok_vm = got == [c["expected"] for c in vms]
        agg = [comm.aggregate_pubkeys([h(p) for p in c["input"]]).hex() == c["output"] for c in gb["aggregate_pubkeys"]]
        try:
            comm.aggregate_pubkeys([h(gb["aggregate_pubkeys"][2]["input"][0]), h(gb["invalid_g1"][1])])
            raised = False
        except ValueError:
            raised = True
        off, pks, msgs, sigs, doms = [0], b"", b"", b"", b""
        for c in vms * 3:
            pks += b"".join(h(p) for p in c["pubkeys"]); msgs += b"".join(h(m) for m in c["messages"])
            sigs += h(c["signature"]); doms += int(c["domain"]).to_bytes(8, "big")
            off.append(off[-1] + len(c["pubkeys"]))
        bv = comm.verify_multiple_batch(off, pks, msgs, 32, sigs, doms)
        ok_batch = bv == [c["expected"] for c in vms * 3]
        comm.destroy()
        q.put((rank, {"verify_multiple": ok_vm, "aggregate": all(agg), "invalid_raises": raised,
                      "batch": ok_batch, "size": world}))
    except Exception as e:  # reported to the parent, which fails
        q.put((rank, {"error": "%s: %s" % (type(e).__name__, e)}))


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    port = int(sys.argv[2]) if len(sys.argv) > 2 else 29517
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    ps = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(180)
    res = dict(q.get() for _ in range(world)) if all(p.exitcode == 0 for p in ps) else {}
    print(json.dumps({"world": world, "exitcodes": [p.exitcode for p in ps], "ranks": res}))
    good = len(res) == world and all(v.get("verify_multiple") and v.get("aggregate") and v.get("invalid_raises")
                                     and v.get("batch") for v in res.values())
    sys.exit(0 if good else 1)


if __name__ == "__main__":
    main()
