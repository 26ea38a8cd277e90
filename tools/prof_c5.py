"""Per-kernel HIP-event times of one batched C5 call (16 calls x L=4096), for tuning the multi-pairing path."""
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
    Lm, nc = int(sys.argv[1]) if len(sys.argv) > 1 else 4096, int(sys.argv[2]) if len(sys.argv) > 2 else 16
    rng = np.random.default_rng(5)
    skb = b"".join((int.from_bytes(rng.bytes(32), "big") % (R - 1) + 1).to_bytes(32, "big") for _ in range(Lm))
    pks = native.privtopub_batch(skb)
    msgs, sigs = [], []
    for _ in range(nc):
        m = rng.bytes(32 * Lm)
        msgs.append(m)
        sigs.append(native.aggregate_signatures(native.sign_batch(m, skb, (1).to_bytes(8, "big") * Lm)))
    off = np.arange(0, nc * Lm + 1, Lm, dtype=np.uint32)
    args = (off, pks * nc, b"".join(msgs), 32, b"".join(sigs), (1).to_bytes(8, "big") * nc)
    assert native.verify_multiple_batch(*args).all()
    native.profile_enable(True)
    t0 = time.perf_counter()
    native.verify_multiple_batch(*args)
    dt = time.perf_counter() - t0
    prof = native.profile_read()
    native.profile_enable(False)
    print("wall ms %.2f" % (1e3 * dt))
    for k, v in sorted(prof.items(), key=lambda kv: -kv[1]["total_ms"]):
        print("%-24s %3d launches %9.3f ms" % (k, v["count"], v["total_ms"]))


if __name__ == "__main__":
    main()
