"""Single bls_verify latency through the shim (host bytes in, bool out), REPS calls over distinct
items, median / min ms -- for same-box A/B of latency knobs run as separate processes.
Usage: python tools/lat_ab.py [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "consensus-specs_amd"))
import numpy as np  # noqa: E402
from bls381_amd import _native as native, bls  # noqa: E402

R = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    native.init(0)
    rng = np.random.default_rng(11)
    skb = b"".join((int.from_bytes(rng.bytes(32), "big") % (R - 1) + 1).to_bytes(32, "big") for _ in range(reps))
    msgs = rng.bytes(32 * reps)
    doms = (3).to_bytes(8, "big") * reps
    pks = native.privtopub_batch(skb)
    sigs = native.sign_batch(msgs, skb, doms)
    bls.bls_verify(pks[:48], msgs[:32], sigs[:96], 3)   # warm-up
    t = []
    for i in range(reps):
        t0 = time.perf_counter()
        ok = bls.bls_verify(pks[48 * i:48 * i + 48], msgs[32 * i:32 * i + 32], sigs[96 * i:96 * i + 96], 3)
        t.append(1e3 * (time.perf_counter() - t0))
        assert ok
    inf = bytes([0xC0]) + bytes(47)
    u = []
    for i in range(reps):
        t0 = time.perf_counter()
        ok = bls.bls_verify_multiple([pks[48 * i:48 * i + 48], inf], [msgs[32 * i:32 * i + 32], bytes(32)],
                                     sigs[96 * i:96 * i + 96], 3)
        u.append(1e3 * (time.perf_counter() - t0))
        assert ok
    print("pad %s: bls_verify median %.2f min %.2f ms; attestation verify_multiple median %.2f min %.2f ms"
          % (os.environ.get("BLS381_LAT_PAD", "1"), float(np.median(t)), min(t), float(np.median(u)), min(u)))


if __name__ == "__main__":
    main()
