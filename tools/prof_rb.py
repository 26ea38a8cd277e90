"""One clean randomized batch (2^16 items, sub-batch 64) through the host-buffer C ABI,
run twice; for rocprofv3 --kernel-trace + tools/timeline.py (stream overlap of the
signature branch).  python tools/prof_rb.py [n] [B]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "consensus-specs_amd"))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 16
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    import bench
    from bls381_amd import _native as native
    native.init(0)
    pks, _, _, doms, _, _ = bench.make_workload(native, n, 0xB15_0007)
    msgs, sigs = bench.make_workload.clean
    seed = bytes(range(32))
    for _ in range(2):
        v = native.verify_batch_randomized(pks, msgs, sigs, doms, seed, B)
    assert v.all()
    print("ok", n, B)


if __name__ == "__main__":
    main()
