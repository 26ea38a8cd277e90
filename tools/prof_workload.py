"""Minimal profiling workload: one C2 verify batch (device-resident), run twice.

Used under rocprofv3 (kernel trace or --pmc passes) so counter rows map to one
launch of each pipeline kernel.  python tools/prof_workload.py [n]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "consensus-specs_amd"))

import numpy as np  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 16
    import bench
    import torch
    from bls381_amd import _native as native
    native.init(0)
    L = native.lib()
    pks, msgs, sigs, doms, expected, _ = bench.make_workload(native, n, 0xB15_0001)
    dev = torch.device("cuda", 0)
    t = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)
    d = [t(pks), t(msgs), t(sigs), t(doms)]
    ver = torch.zeros(n, dtype=torch.uint8, device=dev)
    ws = torch.empty(L.bls381_verify_batch_workspace_size(n), dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream(dev)
    for _ in range(2):
        native.check(L.bls381_verify_batch_device(n, d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(),
                                                  d[3].data_ptr(), ver.data_ptr(), ws.data_ptr(),
                                                  ctypes.c_void_p(s.cuda_stream)))
    torch.cuda.synchronize()
    assert np.array_equal(ver.cpu().numpy().astype(bool), expected)
    # C3 committee aggregation (1024 x 128 keys drawn from the batch): k_agg_chunks + k_agg_compress
    nc, cs = 1024, 128
    idx = np.random.default_rng(3).integers(0, n, nc * cs)
    cpks = np.frombuffer(pks, dtype=np.uint8).reshape(n, 48)[idx].tobytes()
    off = np.arange(0, nc * cs + 1, cs, dtype=np.uint32)
    d_c = t(cpks)
    d_out = torch.zeros(nc * 48, dtype=torch.uint8, device=dev)
    d_st = torch.zeros(nc, dtype=torch.int32, device=dev)
    aws = torch.empty(L.bls381_aggregate_pubkeys_batch_workspace_size(nc, nc * cs), dtype=torch.uint8, device=dev)
    for _ in range(2):
        native.check(L.bls381_aggregate_pubkeys_batch_device(nc, off.ctypes.data_as(ctypes.c_void_p), nc * cs,
                                                             d_c.data_ptr(), d_out.data_ptr(), d_st.data_ptr(),
                                                             aws.data_ptr(), ctypes.c_void_p(s.cuda_stream)))
    torch.cuda.synchronize()
    assert int(d_st.abs().sum().item()) == 0
    # the same committees from the device pubkey registry (validator indices): k_agg_chunks<fp_t,1> reads
    # decoded SoA limbs by index and has no scratch frame -- its HBM bytes against the algorithmic
    # 112 B + 4 B per member show whether the limb loads are coalesced
    from bls381_amd.registry import PubkeyRegistry
    ref = d_out.clone()
    reg = PubkeyRegistry(n)
    ent = reg.add([pks[48 * i:48 * i + 48] for i in range(n)])
    d_idx = t(ent[idx].astype(np.uint32).tobytes())
    d_out.zero_()
    rws = torch.empty(L.bls381_registry_aggregate_workspace_size(nc, nc * cs), dtype=torch.uint8, device=dev)
    for _ in range(2):
        native.check(L.bls381_registry_aggregate_indices_device(
            reg._h, nc, off.ctypes.data_as(ctypes.c_void_p), nc * cs, d_idx.data_ptr(), d_out.data_ptr(),
            d_st.data_ptr(), rws.data_ptr(), ctypes.c_void_p(s.cuda_stream)))
    torch.cuda.synchronize()
    assert torch.equal(d_out, ref) and int(d_st.abs().sum().item()) == 0
    reg.close()
    print("prof workload ok", n)


if __name__ == "__main__":
    main()
