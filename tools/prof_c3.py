"""One C3 epoch step (bench.py bench_c3: 1024 committees x 128, two device aggregations +
one device verify_multiple batch), run three times; for rocprofv3 --kernel-trace +
tools/timeline.py.  python tools/prof_c3.py
"""
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "consensus-specs_amd"))


def main():
    import bench
    import torch
    from bls381_amd import _native as native
    native.init(0)
    L = native.lib()
    n = 1 << 14
    pks, _, _, _, _, sk_ints = bench.make_workload(native, n, 0xB15_0001)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    t_u8 = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)
    args = types.SimpleNamespace(committees=1024, committee_size=128, steps=3)
    r = bench.bench_c3(native, L, args, pks, sk_ints, 1, 0, dev, stream, t_u8, None)
    print(r["ms_per_epoch_step"])


if __name__ == "__main__":
    main()
