"""Replays bench.py's C3 construction exactly and reports which verdicts differ (diagnostic tool)."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "consensus-specs_amd"))
import torch
import bench
from bls381_amd import _native as native

native.init(0)
L = native.lib()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 16
pks, msgs, sigs, doms, expected, sk_ints = bench.make_workload(native, n, 0xB15_0001)
dev = torch.device("cuda", 0)
t_u8 = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)
nc, cs = 1024, 128
rng = np.random.default_rng(0xB15_0003)
idx = rng.integers(0, n, nc * cs)
pk_arr = np.frombuffer(pks, dtype=np.uint8).reshape(n, 48)
offsets = np.repeat(np.arange(0, nc * cs + 1, cs, dtype=np.uint32), 2)[1:]
d_cpks = t_u8(pk_arr[idx].tobytes())
d_out = torch.zeros(2 * nc * 48, dtype=torch.uint8, device=dev)
d_st = torch.zeros(2 * nc, dtype=torch.int32, device=dev)
aws = torch.empty(L.bls381_aggregate_pubkeys_batch_workspace_size(2 * nc, nc * cs), dtype=torch.uint8, device=dev)
stream = torch.cuda.current_stream(dev)
native.check(L.bls381_aggregate_pubkeys_batch_device(
    2 * nc, offsets.ctypes.data_as(ctypes.c_void_p), nc * cs, d_cpks.data_ptr(), d_out.data_ptr(),
    d_st.data_ptr(), aws.data_ptr(), ctypes.c_void_p(stream.cuda_stream)))
aggs = d_out.cpu().numpy().tobytes()
ref, rst = native.aggregate_pubkeys_batch(offsets, pk_arr[idx].tobytes())
print("device agg == host agg:", aggs == b"".join(ref), "status", int(d_st.abs().sum().item()), int(np.count_nonzero(rst)))
ssum = [sum(sk_ints[j] for j in idx[c * cs:(c + 1) * cs]) % bench.R_ORDER for c in range(nc)]
want = native.privtopub_batch(b"".join(k.to_bytes(32, "big") for k in ssum))
bad = [c for c in range(nc) if aggs[96 * c:96 * c + 48] != want[48 * c:48 * c + 48]]
print("agg vs privtopub(sum) mismatches:", len(bad), bad[:10])
m0 = bytearray(rng.bytes(32 * nc))
m1 = rng.bytes(32 * nc)
sigs3 = native.sign_batch(bytes(m0), b"".join(k.to_bytes(32, "big") for k in ssum), (2).to_bytes(8, "big") * nc)
expected = np.ones(nc, dtype=bool)
for c in range(5, nc, 16):
    m0[32 * c + 7] ^= 0x80
    expected[c] = False
msgs3 = b"".join(bytes(m0[32 * c:32 * c + 32]) + m1[32 * c:32 * c + 32] for c in range(nc))
call_off = np.arange(0, 2 * nc + 1, 2, dtype=np.uint32)
got = native.verify_multiple_batch(call_off, aggs, msgs3, 32, sigs3, (2).to_bytes(8, "big") * nc)
diff = np.nonzero(got != expected)[0]
print("verdict mismatches:", len(diff), diff[:20].tolist(), "got", got[diff[:20]].tolist())
for c in diff[:4].tolist():
    one = native.verify_multiple_batch(np.array([0, 2], dtype=np.uint32), aggs[96 * c:96 * c + 96],
                                       msgs3[64 * c:64 * c + 64], 32, sigs3[96 * c:96 * c + 96], (2).to_bytes(8, "big"))
    pv = native.verify(want[48 * c:48 * c + 48], bytes(m0[32 * c:32 * c + 32]), sigs3[96 * c:96 * c + 96], (2).to_bytes(8, "big"))
    print(" call", c, "alone:", bool(one[0]), "plain verify:", pv, "expected", bool(expected[c]))
