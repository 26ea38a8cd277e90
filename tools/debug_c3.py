"""Small-scale replay of bench.py's C3 construction with per-stage diagnostics."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "consensus-specs_amd"))
from bls381_amd import _native as native

R = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
INF = bytes([0xC0]) + bytes(47)
nc, cs, n = int(sys.argv[1]), int(sys.argv[2]), 256
rng = np.random.default_rng(5)
sks = [int.from_bytes(rng.bytes(32), "big") % (R - 1) + 1 for _ in range(n)]
pks = native.privtopub_batch(b"".join(k.to_bytes(32, "big") for k in sks))
idx = rng.integers(0, n, nc * cs)
pk_arr = np.frombuffer(pks, dtype=np.uint8).reshape(n, 48)
offsets = np.repeat(np.arange(0, nc * cs + 1, cs, dtype=np.uint32), 2)[1:]
aggs, st = native.aggregate_pubkeys_batch(offsets, pk_arr[idx].tobytes())
print("agg status nonzero:", int(np.count_nonzero(st)))
ssum = [sum(sks[j] for j in idx[c * cs:(c + 1) * cs]) % R for c in range(nc)]
want = native.privtopub_batch(b"".join(k.to_bytes(32, "big") for k in ssum))
bad_agg = [c for c in range(nc) if aggs[2 * c] != want[48 * c:48 * c + 48]]
bad_inf = [c for c in range(nc) if aggs[2 * c + 1] != INF]
print("committee agg mismatches:", bad_agg[:10], len(bad_agg), " empty-agg != INF:", bad_inf[:10], len(bad_inf))
m0 = rng.bytes(32 * nc)
m1 = rng.bytes(32 * nc)
sigs = native.sign_batch(m0, b"".join(k.to_bytes(32, "big") for k in ssum), (2).to_bytes(8, "big") * nc)
msgs = b"".join(m0[32 * c:32 * c + 32] + m1[32 * c:32 * c + 32] for c in range(nc))
off = np.arange(0, 2 * nc + 1, 2, dtype=np.uint32)
flat = b"".join(aggs)
v = native.verify_multiple_batch(off, flat, msgs, 32, sigs, (2).to_bytes(8, "big") * nc)
print("batch verdicts true:", int(v.sum()), "of", nc)
single = [native.verify_multiple(flat[96 * c:96 * c + 96], msgs[64 * c:64 * c + 64], 32, sigs[96 * c:96 * c + 96],
                                 (2).to_bytes(8, "big")) for c in range(min(nc, 8))]
print("single (first 8):", single)
# without the INF pubkey
v1 = [native.verify(want[48 * c:48 * c + 48], m0[32 * c:32 * c + 32], sigs[96 * c:96 * c + 96], (2).to_bytes(8, "big"))
      for c in range(min(nc, 8))]
print("plain verify (first 8):", v1)
