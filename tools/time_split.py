"""Kernel times of one C2 verify batch for a given libbls381 build (BLS381_LIB), verdicts unchecked.

Profiling aid for variant builds that deliberately skip work (stage-cost splits).
python tools/time_split.py [n]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "consensus-specs_amd"))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 16
    import bench
    import torch
    from bls381_amd import _native as native
    native.init(0)
    L = native.lib()
    pks, msgs, sigs, doms, _, _ = bench.make_workload(native, n, 0xB15_0001)
    dev = torch.device("cuda", 0)
    t = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)
    d = [t(pks), t(msgs), t(sigs), t(doms)]
    ver = torch.zeros(n, dtype=torch.uint8, device=dev)
    ws = torch.empty(L.bls381_verify_batch_workspace_size(n), dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream(dev)
    run = lambda: native.check(L.bls381_verify_batch_device(n, d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(),
                                                             d[3].data_ptr(), ver.data_ptr(), ws.data_ptr(),
                                                             ctypes.c_void_p(s.cuda_stream)))
    run()
    torch.cuda.synchronize()
    native.profile_enable(True)
    for _ in range(2):
        run()
    torch.cuda.synchronize()
    prof = native.profile_read()
    print(os.path.basename(os.environ.get("BLS381_LIB", "libbls381.so")),
          {k: round(v["total_ms"] / v["count"], 2) for k, v in prof.items()})


if __name__ == "__main__":
    main()
