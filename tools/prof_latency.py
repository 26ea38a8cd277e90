"""Per-kernel HIP-event times of small verify batches (latency path): n items of
bls_verify through the host-buffer C ABI, wall time vs the sum of kernel times.

Usage: python tools/prof_latency.py [n ...]   (default 1 64 1024)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "consensus-specs_amd"))
import numpy as np  # noqa: E402
from bls381_amd import _native as native  # noqa: E402

R = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001


def main():
    native.init(0)
    sizes = [int(a) for a in sys.argv[1:]] or [1, 64, 1024]
    rng = np.random.default_rng(7)
    for n in sizes:
        skb = b"".join((int.from_bytes(rng.bytes(32), "big") % (R - 1) + 1).to_bytes(32, "big") for _ in range(n))
        msgs = rng.bytes(32 * n)
        doms = (3).to_bytes(8, "big") * n
        pks = native.privtopub_batch(skb)
        sigs = native.sign_batch(msgs, skb, doms)
        assert native.verify_batch(pks, msgs, sigs, doms).all()
        walls = []
        for _ in range(5):
            t0 = time.perf_counter()
            native.verify_batch(pks, msgs, sigs, doms)
            walls.append(1e3 * (time.perf_counter() - t0))
        native.profile_enable(True)
        native.verify_batch(pks, msgs, sigs, doms)
        prof = native.profile_read()
        native.profile_enable(False)
        print("n=%d wall ms median %.2f min %.2f" % (n, sorted(walls)[2], min(walls)))
        for k, v in sorted(prof.items(), key=lambda kv: -kv[1]["total_ms"]):
            print("  %-24s %3d launches %9.3f ms" % (k, v["count"], v["total_ms"]))
        sys.stdout.flush()


if __name__ == "__main__":
    main()
