"""Benchmark: BLS signature verifications/s on MI355X (BASELINE.json `metric`).

Workload (BASELINE.json configs[1]): 2^16 independent
`bls_verify` deposit proof-of-possession checks -- random secret keys, random
32-byte messages, domain = bls_domain(DOMAIN_DEPOSIT) = 3 -- with 1/16 of the
items tampered (message bit flip or signature swap: full work, verdict False).
One step = one `bls381_verify_batch_device` over the whole batch (decode G1 +
subgroup, decode G2 + subgroup, hash_to_G2, 2-pair Miller loop, final
exponentiation, verdict), inputs resident in HBM.

Multi-GPU: every rank verifies its own 2^16 batch (independent items shard with
no data-path collective; weak scaling); barrier + synchronize around the timed
steps, max over ranks.  Launched either by `torch.distributed.run --nproc-per-node
N ... bench.py --gpus N` (WORLD_SIZE set: this process is one rank) or as plain
`bench.py --gpus N` with WORLD_SIZE unset: the process then only launches N child
ranks (subprocesses with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set; it never
touches the GPU itself) and relays rank 0's JSON line.  Either way a world that is
not N ranks is an error, and the line carries `rccl_world` and every rank's
ms_per_step.

Also reported (secondary lines in the same JSON object):
- "aggregation": committee pubkey aggregation alone (1024 committees x 128);
- "c3_epoch": one epoch of attestations per GPU -- per committee
  bls_aggregate_pubkeys(128 pks) + bls_aggregate_pubkeys([]) +
  bls_verify_multiple([agg, inf], [m0, m1], sig, 2): the aggregation and the
  1024 verify_multiple calls as two batched device calls (aggregates stay in
  HBM); "grouped": the same epoch as one bls381_verify_multiple_grouped_device
  call (validate_indexed_attestation's pattern, the sums beside hash_to_G2);
  "grouped_registry": the same with members as registry entries;
- "c4_aggregate": 2^17 pubkeys per GPU aggregated to one partial, partials
  all-gathered over RCCL and summed on rank 0 (2^20 keys at 8 GPUs);
- "c5_multi_pairing": bls_verify_multiple with L distinct messages;
plus the dominant kernel's roofline against the measured v_mad_u64_u32
peak, and a CPU baseline (the oracle's py_ecc-algorithm restatement on the
host cores, bounded sample of the same items).
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "consensus-specs_amd"))

VALU_PEAK_FILE = os.path.join(ROOT, "profiles", "valu_peak_r04.json")
# Algorithmic work unit: one 381-bit Montgomery product = 300 32x32->64 MACs
# (12x12 product + 12x12 reduction + 12 quotient digits at 32-bit limbs).  The
# engine's radix-2^28 product issues 392 MACs; the excess is implementation
# overhead and is deliberately not credited.
MACS_PER_FP_MUL = 300
# The op-count host build counts the 28x28-bit MACs each Fp product issues (fp_mul 392,
# fp_sqr 301, lazy half-products 196 / 105, wide reductions 196; bls381_field.hpp
# BLS_COUNT_MACS); Fp-product equivalents = MACs / 392, so a squaring or a lazy square
# is credited by its products, not as a full product.
ISSUED_MACS_PER_FP_MUL = 392
# Integer-VALU peak: v_mad_u64_u32 issues over 4 cycles per wave64 on a SIMD (16 lanes per
# clock; MI355X_MICROARCH.md: a full-rate VALU op takes 2), so 256 CUs x 4 SIMDs x 16 x 2.4 GHz.
# The denominator is the larger of this bound and the best rate tools/valu_peak measures.
MAD_ISSUE_BOUND_TOPS = 256 * 4 * 16 * 2.4e9 / 1e12
DOMAIN_DEPOSIT = 3


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=1 << 16, help="verifies per rank per step")
    ap.add_argument("--committees", type=int, default=1024)
    ap.add_argument("--committee-size", type=int, default=128)
    ap.add_argument("--cpu-sample", type=int, default=256)
    ap.add_argument("--cpu-procs", type=int, default=16)
    ap.add_argument("--cpp-sample", type=int, default=2048, help="items for the C++ host-build CPU line")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-aggregate", action="store_true")
    ap.add_argument("--no-secondary", action="store_true", help="skip the C3/C4/C5 lines")
    ap.add_argument("--inflight", type=int, default=1,
                    help="headline: consecutive steps alternate over this many streams (independent batches)")
    ap.add_argument("--secondary-timeout", type=int, default=360,
                    help="with several ranks: end the secondary lines after this many seconds (the headline is kept)")
    ap.add_argument("--sections", type=str, default="",
                    help="comma list: run only these secondary lines (host, deposits, randomized, c3, c4, c5, rccl, latency)")
    ap.add_argument("--rb-batch", type=str, default="64,8",
                    help="randomized sub-batch sizes (comma list; the first is the line's own, r06: 64 the best clean, 8 the best with 1/16 tampered)")
    ap.add_argument("--c4-keys", type=int, default=1 << 17, help="pubkeys per GPU in the C4 aggregation")
    ap.add_argument("--c5", type=str, default="16,128,1024,4096", help="C5 distinct-message counts")
    ap.add_argument("--policy", choices=["pyecc", "strict"], default="pyecc",
                    help="subgroup policy of the headline line (bls.SUBGROUP_POLICY)")
    ap.add_argument("--fail-on-secondary-error", action="store_true",
                    help="exit 3 when a secondary line failed (recorded as secondary_error / {\"error\": ...}); "
                         "default: the line is printed and the exit code is 0")
    ap.add_argument("--dry-run-fail-rank", type=int, default=-1, help=argparse.SUPPRESS)   # launcher test hook
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check without a GPU: the ranks join a gloo world, report it and exit")
    return ap.parse_args()


def _free_port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(args):
    """`bench.py --gpus N` without WORLD_SIZE: start N rank processes and relay rank 0's line.
    This process never initialises the GPU (device_count() does not, on this image), and the
    ranks are children, not an exec of this process."""
    import subprocess
    n = args.gpus
    if not args.dry_run:
        import torch
        have = torch.cuda.device_count()
        if have < n:
            sys.stderr.write("bench.py --gpus %d: only %d device(s) visible\n" % (n, have))
            return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    # rank 0's stdout is drained on a thread; if any rank fails the others are ended (a rank left
    # waiting in a collective for a dead peer would never return)
    import threading
    buf = []
    reader = threading.Thread(target=lambda: buf.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    failed = False
    while any(p.poll() is None for p in procs):
        if not failed and any(p.poll() not in (None, 0) for p in procs):
            failed = True
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            deadline = time.time() + 30
            while time.time() < deadline and any(p.poll() is None for p in procs):
                time.sleep(0.5)
            for p in procs:
                if p.poll() is None:
                    p.kill()
        time.sleep(0.5)
    reader.join(timeout=30)
    out = (buf[0] if buf else b"").decode()
    rcs = [p.returncode for p in procs]
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    if lines:
        print(lines[-1], flush=True)
    bad = [rc for rc in rcs if rc != 0]
    if bad or not lines:
        sys.stderr.write("bench.py --gpus %d: rank exit codes %s\n" % (n, rcs))
        return bad[0] if bad else 1
    return 0


def dry_run(args, world, rank):
    """The rank side of the launcher check: a gloo world on the CPU, no device touched."""
    import torch
    import torch.distributed as dist
    if rank == args.dry_run_fail_rank:
        raise SystemExit("dry run: rank %d fails before joining the world" % rank)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        got = dist.get_world_size()
        ranks = [None] * got
        dist.all_gather_object(ranks, rank)
        dist.destroy_process_group()
    else:
        got, ranks = 1, [0]
    if got != args.gpus:
        raise SystemExit("world is %d ranks, --gpus %d" % (got, args.gpus))
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": args.gpus, "rccl_world": got, "ranks": ranks}))


def make_workload(native, n, seed):
    """2^16 signed deposit items built on the GPU (untimed), 1/16 tampered."""
    rng = np.random.default_rng(seed)
    r = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
    sks = bytearray()
    for _ in range(n):
        k = int.from_bytes(rng.bytes(32), "big") % (r - 1) + 1
        sks += k.to_bytes(32, "big")
    sks = bytes(sks)
    msgs = bytearray(rng.bytes(32 * n))
    doms = DOMAIN_DEPOSIT.to_bytes(8, "big") * n
    pks = native.privtopub_batch(sks)
    sigs = bytearray(native.sign_batch(bytes(msgs), sks, doms))
    sk_ints = [int.from_bytes(sks[32 * i:32 * i + 32], "big") for i in range(n)]
    make_workload.clean = (bytes(msgs), bytes(sigs))     # before tampering (randomized-batch line)
    expected = np.ones(n, dtype=bool)
    for i in range(3, n, 16):              # 1/16 tampered, full verification work
        if (i // 16) % 2 == 0:
            msgs[32 * i] ^= 0x01           # message bit flip
        else:
            j = (i + 1) % n
            sigs[96 * i:96 * i + 96] = sigs[96 * j:96 * j + 96]   # signature of another item
        expected[i] = False
    return pks, bytes(msgs), bytes(sigs), doms, expected, sk_ints


def load_valu_peak():
    """(peak T MAC/s, source): max(the measured best v_mad_u64_u32 rate, the 39.3 T/s issue bound)."""
    try:
        with open(VALU_PEAK_FILE) as f:
            d = json.load(f)
        meas = float(d["v_mad_u64_u32_Tops"])
    except Exception:
        return MAD_ISSUE_BOUND_TOPS, "issue bound (no measurement file)"
    src = "max(issue bound %.2f, measured %.2f in %s)" % (MAD_ISSUE_BOUND_TOPS, meas, os.path.relpath(VALU_PEAK_FILE, ROOT))
    return max(meas, MAD_ISSUE_BOUND_TOPS), src


# profile key (bls381_profile_read) -> kernel symbol in rocprofv3 / PMC output
PROFILE_KERNEL = {"decode_g1": "k_decode_g1", "decode_g2": "k_decode_g2", "decode_g2_1": "k_decode_g2_1",
                  "hash_to_g2": "k_hash_g2",
                  "miller_loop_2": "k_miller_verify", "final_exp": "k_final_exp_verdict",
                  "miller_lines": "k_ml_lines", "miller_accum": "k_ml_accum",
                  "hash_cand": "k_hash_cand_1", "hash_bp": "k_hash_bp",
                  "final_exp_q": "k_final_exp_verdict_q<1>", "miller_loop_2q": "k_miller_verify_q",
                  "prologue": "k_prologue_1<0>", "final_exp_redo": "k_final_exp_redo"}
# the C2 batch (2^16 items) runs the split Miller loop: the monolithic count is not part of its pipeline
PIPELINE_STAGES = ["decode_g1", "decode_g2", "hash_to_g2", "miller_lines", "miller_accum", "final_exp"]


def stage_times(prof, steps):
    """ms per step of each pipeline stage from the profile (the final exponentiation's exact pass
    over its rare g2 = 0 waves, k_final_exp_redo, is part of the final_exp stage)"""
    ms = {k: v["total_ms"] / steps for k, v in prof.items()}
    # the one-lane signature decode (profile key "decode_g2_1") is the C2 pipeline's decode_g2 stage
    if "decode_g2_1" in ms:
        ms["decode_g2"] = ms.pop("decode_g2_1") + ms.get("decode_g2", 0.0)
    if "final_exp_redo" in ms:
        ms["final_exp"] = ms.get("final_exp", 0.0) + ms.pop("final_exp_redo")
    return ms


def stage_kernels(prof_key, prof):
    """[(kernel symbol, launches per step)] of a stage"""
    if prof_key == "decode_g2" and "decode_g2_1" in prof:
        return [(PROFILE_KERNEL["decode_g2_1"], 1)]
    return [(PROFILE_KERNEL.get(prof_key, "k_" + prof_key), 1)]


def load_pmc_traffic(kernels, n):
    """HBM bytes per step of the dominant stage's kernels ([(symbol, launches)]) from the newest committed PMC pass
    (profiles/pmc_<tag>_counters.json, written by tools/pmc_summary.py from separate rocprofv3 --pmc
    runs of tools/prof_workload.py at the same n; FETCH_SIZE doubled per MI355X_MICROARCH.md "HBM").
    PMC counters cannot be read inside the timed run, so this is the last profiled build's figure."""
    import glob
    # newest by round tag (pmc_r01a < pmc_r01h ...): file mtimes are not preserved by a checkout
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*_counters.json")))
    for f in reversed(files):
        try:
            d = json.load(open(f))
            tot = 0.0
            for sym, launches in kernels:
                k = d["kernels"][sym]
                if int(k.get("waves", 0)) * 64 not in (n, 2 * n):   # lanes = n (G1) or 2n (lane-pair)
                    raise KeyError(sym)
                tot += launches * k["hbm_bytes_per_launch"]
            return tot, os.path.relpath(f, ROOT)
        except Exception:
            continue
    return None, None


def issue_roofline(kernels, n, measured_ms):
    """Instruction-issue roofline of a kernel: its VALU instructions per launch from the
    newest committed PMC pass (SQ_INSTS_VALU, _INT64, _INT32; wave instructions), each class priced at
    its best measured chip-wide issue rate from one tools/valu_peak run (VALU_PEAK_FILE: v_mad_u64_u32
    for INT64, v_add_u32 for INT32, the median VOP3 rate for the rest), against the launch's live
    HIP-event time.  frac < 1 is time the kernel did not issue VALU work (stalls: SQ_WAIT_ANY)."""
    import glob
    try:
        rates = json.load(open(VALU_PEAK_FILE))
    except Exception:
        return None
    vop3 = sorted(v for k, v in rates.items() if k.endswith("_Tops") and k not in (
        "v_mad_u64_u32_Tops", "v_add_u32_Tops", "v_and_b32_Tops", "v_cmp+v_cndmask_Tops"))
    r_other = vop3[len(vop3) // 2]
    for f in reversed(sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*_counters.json")))):
        try:
            d = json.load(open(f))["kernels"]
            i64 = i32 = allv = 0.0
            for sym, launches in kernels:
                k = d[sym]
                if int(k.get("waves", 0)) * 64 not in (n, 2 * n) or k.get("valu_int64_insts") is None:
                    raise KeyError(sym)
                i64 += launches * k["valu_int64_insts"]
                i32 += launches * k["valu_int32_insts"]
                allv += launches * k["valu_insts"]
            other = allv - i64 - i32
            model_ms = 64e3 * (i64 / (rates["v_mad_u64_u32_Tops"] * 1e12) + i32 / (rates["v_add_u32_Tops"] * 1e12) +
                               other / (r_other * 1e12))
            return {"kernels": [k for k, _ in kernels], "valu_int64_insts": i64, "valu_int32_insts": i32,
                    "valu_other_insts": other, "issue_time_ms": round(model_ms, 3),
                    "measured_ms": round(measured_ms, 3), "frac": round(model_ms / measured_ms, 4),
                    "rates_Tops": {"int64": rates["v_mad_u64_u32_Tops"], "int32": rates["v_add_u32_Tops"],
                                   "other (median VOP3)": r_other},
                    "source": os.path.relpath(f, ROOT)}
        except Exception:
            continue
    return None


def count_fp_muls(pks, msgs, sigs, doms, strict=0, k=8):
    """Per-stage Fp-product equivalents per verify (MACs issued / 392), counted by the -DBLS_COUNT_OPS
    host build (strict = 1: with the subgroup checks of BLS381_POLICY_STRICT)."""
    import build_native
    path = build_native.build_hostcheck(count_ops=True)
    L = ctypes.CDLL(path)
    tot = np.zeros(7)
    done = 0
    for i in range(64):
        out = (ctypes.c_uint64 * 7)()
        if L.hc_count_verify_stages(pks[48 * i:48 * i + 48], msgs[32 * i:32 * i + 32],
                                    sigs[96 * i:96 * i + 96], doms[8 * i:8 * i + 8], strict, out) == 1:
            tot += np.array(list(out), dtype=float)
            done += 1
            if done == k:
                break
    names = ["decode_g1", "decode_g2", "hash_to_g2", "miller_loop_2", "final_exp", "miller_lines", "miller_accum"]
    return {nm: tot[j] / done / ISSUED_MACS_PER_FP_MUL for j, nm in enumerate(names)}


MAC_PROBE_FILE = os.path.join(ROOT, "profiles", "mac_probe_r05k.txt")


def mac_stream_ceiling(achieved, peak):
    """The rate a pure v_mad_u64_u32 stream reaches at the verify kernels' occupancy (two waves per
    SIMD, tools/mac_probe.hip, measured once per build round): the ceiling any kernel at that occupancy
    can approach, beside the issue-bound peak the frac is priced against (HISTORY.md, round 5 "What bounds the products")."""
    try:
        rates = []
        block = None
        for ln in open(MAC_PROBE_FILE):
            if ln.startswith("# blocks"):
                block = int(ln.split()[-1])
            elif ln.startswith("{") and block == 512:
                rates.append(json.loads(ln)["mad_Tops"])
        if not rates or not peak:
            return None
        top = max(rates)
        return {"waves_per_simd": 2, "mac_only_Tops": top, "frac_of_peak": round(top / peak, 4),
                "achieved_frac_of_ceiling": round(achieved / top, 4), "source": os.path.relpath(MAC_PROBE_FILE, ROOT)}
    except (OSError, ValueError, KeyError):
        return None


def agg_roofline(aprof, sample_pks, k, keys):
    """Roofline of the committee aggregation's dominant kernel: Fp multiplications per key of
    decode + add (the -DBLS_COUNT_OPS host build, hc_count_aggregate over one committee) x keys x
    300 MACs, over that kernel's HIP-event time; the same integer-VALU peak as the C2 line."""
    import build_native
    L = ctypes.CDLL(build_native.build_hostcheck(count_ops=True))
    out = ctypes.c_uint64()
    if L.hc_count_aggregate(ctypes.c_size_t(k), sample_pks, ctypes.byref(out)) != 0:
        return None
    per_key = out.value / k / ISSUED_MACS_PER_FP_MUL
    ms = {kk: v["total_ms"] / v["count"] for kk, v in aprof.items()}
    dom = max(ms, key=ms.get)
    peak, _ = load_valu_peak()
    ach = per_key * MACS_PER_FP_MUL * keys / (ms[dom] * 1e-3) / 1e12
    return {"kernel": dom, "fp_mul_per_key": round(per_key, 1), "kernel_avg_ms": ms,
            "achieved": round(ach, 3), "peak": peak, "unit": "T MAC/s (v_mad_u64_u32, 32x32+64)",
            "frac": round(ach / peak, 4) if peak else None}


def _cpu_verify(args):
    import bls_oracle as O
    pk, m, s, d = args
    return O.verify(m, pk, s, d)


def cpu_baseline(pks, msgs, sigs, sample, procs):
    """Oracle (py_ecc 1.7.0 algorithm restatement) verify on host cores, bounded sample."""
    import multiprocessing as mp
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    items = [(pks[48 * i:48 * i + 48], msgs[32 * i:32 * i + 32], sigs[96 * i:96 * i + 96], DOMAIN_DEPOSIT)
             for i in range(sample)]
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    with ctx.Pool(procs) as pool:
        res = pool.map(_cpu_verify, items, chunksize=1)
    dt = time.perf_counter() - t0
    return sample / dt, res, dt


def cpu_baseline_cpp(pks, msgs, sigs, doms, sample, threads):
    """The g++ build of the engine's own arithmetic headers (host_check.cpp hc_verify: same
    decode / hash_to_G2 / Miller loop / final exponentiation code as the kernels, scalar
    x86-64) on `threads` host threads, bounded sample: the stronger CPU line."""
    import build_native
    L = ctypes.CDLL(build_native.build_hostcheck())
    out = (ctypes.c_uint8 * sample)()
    t0 = time.perf_counter()
    L.hc_verify_batch_mt(ctypes.c_size_t(sample), pks, msgs, sigs, doms, 0, threads, out)
    dt = time.perf_counter() - t0
    return sample / dt, [bool(v) for v in out], dt


R_ORDER = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
INF_G1 = bytes([0xC0]) + bytes(47)


def _max_time(t, world, dist, dev):
    if world > 1:
        import torch
        x = torch.tensor([t], dtype=torch.float64, device=dev)
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        t = float(x.item())
    return t


def bench_c3(native, L, args, pks, sk_ints, world, rank, dev, stream, t_u8, dist):
    """C3: 1024 committees x 128, per committee 2 aggregates + 1 verify_multiple."""
    import torch
    nc, cs, n = args.committees, args.committee_size, len(sk_ints)
    rng = np.random.default_rng(0xB15_0003 + rank)
    idx = rng.integers(0, n, nc * cs)
    pk_arr = np.frombuffer(pks, dtype=np.uint8).reshape(n, 48)
    # groups 2c (the committee) and 2c+1 (empty: bls_aggregate_pubkeys([]))
    offsets = np.repeat(np.arange(0, nc * cs + 1, cs, dtype=np.uint32), 2)[1:]
    d_cpks = t_u8(pk_arr[idx].tobytes())
    d_out = torch.zeros(2 * nc * 48, dtype=torch.uint8, device=dev)
    d_st = torch.zeros(2 * nc, dtype=torch.int32, device=dev)
    aws = torch.empty(L.bls381_aggregate_pubkeys_batch_workspace_size(2 * nc, nc * cs), dtype=torch.uint8, device=dev)
    m0 = bytearray(rng.bytes(32 * nc))
    m1 = rng.bytes(32 * nc)
    # aggregate signature of a committee on m0 == signature with the summed key
    ssum = [sum(sk_ints[j] for j in idx[c * cs:(c + 1) * cs]) % R_ORDER for c in range(nc)]
    sigs = native.sign_batch(bytes(m0), b"".join(k.to_bytes(32, "big") for k in ssum), (2).to_bytes(8, "big") * nc)
    expected = np.ones(nc, dtype=bool)
    for c in range(5, nc, 16):             # 1/16 of the attestations carry a wrong message
        m0[32 * c + 7] ^= 0x80
        expected[c] = False
    msgs = b"".join(bytes(m0[32 * c:32 * c + 32]) + m1[32 * c:32 * c + 32] for c in range(nc))
    call_off = np.arange(0, 2 * nc + 1, 2, dtype=np.uint32)
    doms = (2).to_bytes(8, "big") * nc
    d_sigs, d_doms = t_u8(sigs), t_u8(doms)
    d_ver = torch.zeros(nc, dtype=torch.uint8, device=dev)
    vws = torch.empty(L.bls381_verify_multiple_batch_workspace_size(nc, 2 * nc, 32), dtype=torch.uint8, device=dev)

    def step():
        # aggregates stay in HBM: bls_aggregate_pubkeys -> bls_verify_multiple on device buffers, one stream
        native.check(L.bls381_aggregate_pubkeys_batch_device(
            2 * nc, offsets.ctypes.data_as(ctypes.c_void_p), nc * cs, d_cpks.data_ptr(), d_out.data_ptr(),
            d_st.data_ptr(), aws.data_ptr(), ctypes.c_void_p(stream.cuda_stream)))
        native.check(L.bls381_verify_multiple_batch_device(
            nc, call_off.ctypes.data_as(ctypes.c_void_p), msgs, 32, d_out.data_ptr(), d_sigs.data_ptr(),
            d_doms.data_ptr(), d_ver.data_ptr(), vws.data_ptr(), ctypes.c_void_p(stream.cuda_stream)))

    step()
    torch.cuda.synchronize()
    assert np.array_equal(d_ver.cpu().numpy().astype(bool), expected), "C3 verdict mismatch"
    assert int(d_st.abs().sum().item()) == 0
    host = native.verify_multiple_batch(call_off, d_out.cpu().numpy().tobytes(), msgs, 32, sigs, doms)
    assert np.array_equal(host, expected), "C3 host-path verdict mismatch"
    steps = max(args.steps, 3)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    t = _max_time(time.perf_counter() - t0, world, dist, dev)
    # the same epoch as one grouped call (bls381_verify_multiple_grouped_device): the committee
    # sums run beside hash_to_G2 instead of before it
    call_groups = np.arange(0, 2 * nc + 1, 2, dtype=np.uint32)
    gws = torch.empty(L.bls381_verify_multiple_grouped_workspace_size(nc, 2 * nc, nc * cs, 32), dtype=torch.uint8,
                      device=dev)
    d_ver2 = torch.zeros(nc, dtype=torch.uint8, device=dev)

    def fused():
        native.check(L.bls381_verify_multiple_grouped_device(
            nc, call_groups.ctypes.data_as(ctypes.c_void_p), 2 * nc, offsets.ctypes.data_as(ctypes.c_void_p), msgs,
            32, d_cpks.data_ptr(), d_sigs.data_ptr(), d_doms.data_ptr(), d_ver2.data_ptr(), gws.data_ptr(),
            ctypes.c_void_p(stream.cuda_stream)))

    fused()
    torch.cuda.synchronize()
    assert np.array_equal(d_ver2.cpu().numpy().astype(bool), expected), "C3 grouped verdict mismatch"
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(steps):
        fused()
    torch.cuda.synchronize()
    tf = _max_time(time.perf_counter() - t1, world, dist, dev)
    # and with the members as validator indices into a device pubkey registry (a node keeps the
    # registry decoded; 0_beacon-chain.md:1025-1026 reads state.validator_registry[i].pubkey)
    from bls381_amd.registry import PubkeyRegistry
    reg = PubkeyRegistry(n)
    ent = reg.add([pks[48 * i:48 * i + 48] for i in range(n)])
    assert np.all(ent >= 0)
    d_ent = t_u8(ent[idx].astype(np.uint32).tobytes())
    d_ver3 = torch.zeros(nc, dtype=torch.uint8, device=dev)

    def fused_reg():
        native.check(L.bls381_registry_verify_multiple_grouped_device(
            reg._h, nc, call_groups.ctypes.data_as(ctypes.c_void_p), 2 * nc, offsets.ctypes.data_as(ctypes.c_void_p),
            msgs, 32, d_ent.data_ptr(), d_sigs.data_ptr(), d_doms.data_ptr(), d_ver3.data_ptr(), gws.data_ptr(),
            ctypes.c_void_p(stream.cuda_stream)))

    fused_reg()
    torch.cuda.synchronize()
    assert np.array_equal(d_ver3.cpu().numpy().astype(bool), expected), "C3 registry grouped verdict mismatch"
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    for _ in range(steps):
        fused_reg()
    torch.cuda.synchronize()
    tr = _max_time(time.perf_counter() - t2, world, dist, dev)
    reg.close()
    return {"workload": "C3: %d committees x %d per GPU: 2 x bls_aggregate_pubkeys + bls_verify_multiple([agg, inf], "
                        "[m0, m1], sig, 2) each, 1/16 wrong message; device-resident (aggregates never leave HBM)"
                        % (nc, cs),
            "attestations_per_s": nc * steps * world / t, "ms_per_epoch_step": 1e3 * t / steps, "n_gpus": world,
            "grouped": {"api": "bls381_verify_multiple_grouped_device (aggregation fused beside hash_to_G2)",
                        "attestations_per_s": nc * steps * world / tf, "ms_per_epoch_step": 1e3 * tf / steps},
            "grouped_registry": {"api": "bls381_registry_verify_multiple_grouped_device (members as registry "
                                        "entries of the %d keys)" % n,
                                 "attestations_per_s": nc * steps * world / tr, "ms_per_epoch_step": 1e3 * tr / steps}}


def bench_deposits(native, L, args, pks, sk_ints, world, dist, dev, stream, t_u8):
    """C2 end to end from serialized DepositData: signing_root(deposit.data) on the
    device feeding the verify pipeline (process_deposit, 0_beacon-chain.md:1755-1758), same keys as C2."""
    import torch
    from bls381_amd import ssz
    n = len(pks) // 48
    rng = np.random.default_rng(0xB15_0009)
    wc = rng.bytes(32 * n)
    amt = (32 * 10 ** 9 + np.arange(n, dtype=np.uint64)).astype("<u8").tobytes()
    items = [pks[48 * i:48 * i + 48] + wc[32 * i:32 * i + 32] + amt[8 * i:8 * i + 8] + b"\x00" * 96 for i in range(n)]
    roots = b"".join(ssz.signing_root_batch(ssz.DepositData, items))
    sks = b"".join(k.to_bytes(32, "big") for k in sk_ints)
    doms = DOMAIN_DEPOSIT.to_bytes(8, "big") * n
    sigs = native.sign_batch(roots, sks, doms)
    blob = bytearray(b"".join(items[i][:88] + sigs[96 * i:96 * i + 96] for i in range(n)))
    expected = np.ones(n, dtype=bool)
    for i in range(5, n, 16):              # 1/16 tampered: amount changed after signing
        blob[184 * i + 80] ^= 0x01
        expected[i] = False
    d_dd, d_dom = t_u8(bytes(blob)), t_u8(doms)
    d_ver = torch.zeros(n, dtype=torch.uint8, device=dev)
    ws = torch.empty(L.bls381_verify_deposits_workspace_size(n), dtype=torch.uint8, device=dev)

    def step():
        native.check(L.bls381_verify_deposits_device(n, d_dd.data_ptr(), d_dom.data_ptr(), d_ver.data_ptr(),
                                                     ws.data_ptr(), ctypes.c_void_p(stream.cuda_stream)))
    step()
    torch.cuda.synchronize()
    assert np.array_equal(d_ver.cpu().numpy().astype(bool), expected), "deposit verdict mismatch"
    steps = max(args.steps, 3)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    t = _max_time(time.perf_counter() - t0, world, dist, dev)
    return {"workload": "C2 from %d serialized DepositData per GPU: device signing_root + bls_verify" % n,
            "deposits_per_s": n * steps * world / t, "ms_per_step": 1e3 * t / steps, "n_gpus": world}


def bench_registry_c3(native, L, args, pks, idx, offsets, d_ref_out, world, dist, dev, stream, t_u8):
    """C3 committees aggregated from the device-resident pubkey registry: the
    same 1024 x 128 members as validator indices into a registry of the 2^16 keys (the reference reads
    state.validator_registry[i].pubkey, 0_beacon-chain.md:1025-1026).  Output bytes must equal the
    decode-every-key path's."""
    import torch
    from bls381_amd.registry import PubkeyRegistry
    n = len(pks) // 48
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reg = PubkeyRegistry(n)
    ent = reg.add([pks[48 * i:48 * i + 48] for i in range(n)])
    build_s = time.perf_counter() - t0
    assert np.all(ent >= 0)
    nc = len(offsets) - 1
    ent_idx = ent[idx].astype(np.uint32)          # duplicate keys resolve to their first entry
    d_idx = t_u8(ent_idx.tobytes())
    d_out = torch.zeros(nc * 48, dtype=torch.uint8, device=dev)
    d_st = torch.zeros(nc, dtype=torch.int32, device=dev)
    ws = torch.empty(L.bls381_registry_aggregate_workspace_size(nc, len(idx)), dtype=torch.uint8, device=dev)

    def step():
        native.check(L.bls381_registry_aggregate_indices_device(
            reg._h, nc, offsets.ctypes.data_as(ctypes.c_void_p), len(idx), d_idx.data_ptr(), d_out.data_ptr(),
            d_st.data_ptr(), ws.data_ptr(), ctypes.c_void_p(stream.cuda_stream)))
    step()
    torch.cuda.synchronize()
    assert torch.equal(d_out, d_ref_out) and int(d_st.abs().sum().item()) == 0, "registry aggregation mismatch"
    steps = max(args.steps, 3) * 4
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    t = _max_time(time.perf_counter() - t0, world, dist, dev)
    reg.close()
    return {"workload": "C3 committees by validator index from a registry of %d decoded pubkeys" % n,
            "committee_aggregations_per_s": nc * steps * world / t,
            "pubkeys_aggregated_per_s": nc * (len(idx) // nc) * steps * world / t,
            "ms_per_step": 1e3 * t / steps, "registry_build_ms": 1e3 * build_s,
            "registry_build_keys_per_s": n / build_s}


def bench_c4(native, L, args, world, rank, dev, stream, t_u8, dist):
    """C4: 2^17 pubkeys/GPU -> one partial per GPU, RCCL all-gather, rank 0 sums."""
    import torch
    k = args.c4_keys
    # keys [1..64] * G cycled: the expected sum is known in closed form
    base = native.privtopub_batch(b"".join(j.to_bytes(32, "big") for j in range(1, 65)))
    pk = np.frombuffer(base, dtype=np.uint8).reshape(64, 48)[np.arange(k) % 64].tobytes()
    d_pk = t_u8(pk)
    off = np.array([0, k], dtype=np.uint32)
    d_out = torch.zeros(48, dtype=torch.uint8, device=dev)
    d_st = torch.zeros(1, dtype=torch.int32, device=dev)
    aws = torch.empty(L.bls381_aggregate_pubkeys_batch_workspace_size(1, k), dtype=torch.uint8, device=dev)

    def step():
        native.check(L.bls381_aggregate_pubkeys_batch_device(
            1, off.ctypes.data_as(ctypes.c_void_p), k, d_pk.data_ptr(), d_out.data_ptr(), d_st.data_ptr(),
            aws.data_ptr(), ctypes.c_void_p(stream.cuda_stream)))
        if world > 1:
            parts = [torch.empty_like(d_out) for _ in range(world)]
            dist.all_gather(parts, d_out)
            allp = torch.cat(parts).cpu().numpy().tobytes()
        else:
            # one rank: its partial is the aggregate (no partials to sum on rank 0)
            return d_out.cpu().numpy().tobytes()
        return native.aggregate_pubkeys(allp) if rank == 0 else None

    res = step()
    if rank == 0:
        want_scalar = world * sum((i % 64) + 1 for i in range(k)) % R_ORDER
        assert res == native.privtopub_batch(want_scalar.to_bytes(32, "big")), "C4 aggregate mismatch"
    steps = max(args.steps, 3)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    t = _max_time(time.perf_counter() - t0, world, dist, dev)
    # per-kernel times from two extra, untimed steps (profiling events stay out of the timed loop)
    native.profile_enable(True)
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    cprof = native.profile_read()
    native.profile_enable(False)
    cprof = {kk: {"count": v["count"] / 2 * steps, "total_ms": v["total_ms"] / 2 * steps} for kk, v in cprof.items()}
    out = {"workload": "C4: %d pubkeys per GPU (%d total) -> one bls_aggregate_pubkeys; per-GPU partial, "
                       "all-gather, sum on rank 0 (one rank: the partial is the aggregate)" % (k, k * world),
           "pubkeys_aggregated_per_s": k * world * steps / t, "ms_per_aggregate": 1e3 * t / steps,
           "n_gpus": world, "roofline": agg_roofline(cprof, pk[:48 * 128], 128, k)}
    out["registry"] = bench_c4_registry(native, L, args, world, rank, dev, stream, t_u8, dist)
    return out


def bench_c4_registry(native, L, args, world, rank, dev, stream, t_u8, dist):
    """C4 from the device-resident registry: this rank's shard of the validator registry (k distinct keys,
    decoded once) aggregated by validator index; partial per GPU, all-gather, sum on rank 0."""
    import torch
    from bls381_amd.registry import PubkeyRegistry
    k = args.c4_keys
    rng = np.random.default_rng(0xB15_0004 + rank)
    sks = [int.from_bytes(rng.bytes(32), "big") % (R_ORDER - 1) + 1 for _ in range(k)]
    pks = native.privtopub_batch(b"".join(x.to_bytes(32, "big") for x in sks))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reg = PubkeyRegistry(k)
    ent = reg.add([pks[48 * i:48 * i + 48] for i in range(k)])
    build = time.perf_counter() - t0
    assert np.all(ent == np.arange(k))
    off = np.array([0, k], dtype=np.uint32)
    d_idx = t_u8(np.arange(k, dtype=np.uint32).tobytes())
    d_out = torch.zeros(48, dtype=torch.uint8, device=dev)
    d_st = torch.zeros(1, dtype=torch.int32, device=dev)
    ws = torch.empty(L.bls381_registry_aggregate_workspace_size(1, k), dtype=torch.uint8, device=dev)
    want_local = native.privtopub_batch((sum(sks) % R_ORDER).to_bytes(32, "big"))

    def step():
        native.check(L.bls381_registry_aggregate_indices_device(
            reg._h, 1, off.ctypes.data_as(ctypes.c_void_p), k, d_idx.data_ptr(), d_out.data_ptr(), d_st.data_ptr(),
            ws.data_ptr(), ctypes.c_void_p(stream.cuda_stream)))
        if world > 1:
            parts = [torch.empty_like(d_out) for _ in range(world)]
            dist.all_gather(parts, d_out)
            allp = torch.cat(parts).cpu().numpy().tobytes()
        else:
            allp = d_out.cpu().numpy().tobytes()
        return allp, (native.aggregate_pubkeys(allp) if rank == 0 else None)

    allp, _ = step()
    assert allp[48 * rank:48 * rank + 48] == want_local, "C4 registry aggregate mismatch"
    steps = max(args.steps, 3) * 4
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    t = _max_time(time.perf_counter() - t0, world, dist, dev)
    reg.close()
    return {"workload": "C4 from per-GPU registry shards of %d decoded pubkeys, aggregated by index" % k,
            "pubkeys_aggregated_per_s": k * world * steps / t, "ms_per_aggregate": 1e3 * t / steps,
            "registry_build_ms": 1e3 * build}


def bench_c5(native, args, world, rank, dist, dev):
    """C5: one bls_verify_multiple with L distinct messages (L+1 Miller loops, 1 FE)."""
    import torch
    out = []
    rng = np.random.default_rng(0xB15_0005 + rank)
    for Lm in [int(x) for x in args.c5.split(",") if x]:
        sks = [int.from_bytes(rng.bytes(32), "big") % (R_ORDER - 1) + 1 for _ in range(Lm)]
        skb = b"".join(s.to_bytes(32, "big") for s in sks)
        msgs = rng.bytes(32 * Lm)
        pks = native.privtopub_batch(skb)
        sig = native.aggregate_signatures(native.sign_batch(msgs, skb, (1).to_bytes(8, "big") * Lm))
        off = np.array([0, Lm], dtype=np.uint32)
        d1 = (1).to_bytes(8, "big")
        assert native.verify_multiple_batch(off, pks, msgs, 32, sig, d1)[0]
        assert not native.verify_multiple_batch(off, pks, msgs, 32, sig, (2).to_bytes(8, "big"))[0]
        steps = max(args.steps, 3)
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            native.verify_multiple_batch(off, pks, msgs, 32, sig, d1)
        t = _max_time(time.perf_counter() - t0, world, dist, dev)
        out.append({"L": Lm, "ms_per_call": 1e3 * t / steps, "pairings_per_s": (Lm + 1) * steps * world / t})
    # throughput: many such calls in one batch (each call keeps its own single final exponentiation)
    Lm, nc = 4096, 16
    sks = [int.from_bytes(rng.bytes(32), "big") % (R_ORDER - 1) + 1 for _ in range(Lm)]
    skb = b"".join(s.to_bytes(32, "big") for s in sks)
    pks = native.privtopub_batch(skb)
    msgs_all, sigs = [], []
    for c in range(nc):
        m = rng.bytes(32 * Lm)
        msgs_all.append(m)
        sigs.append(native.aggregate_signatures(native.sign_batch(m, skb, (1).to_bytes(8, "big") * Lm)))
    off = np.arange(0, nc * Lm + 1, Lm, dtype=np.uint32)
    pk_all, msg_all, sig_all, dom_all = pks * nc, b"".join(msgs_all), b"".join(sigs), (1).to_bytes(8, "big") * nc
    assert native.verify_multiple_batch(off, pk_all, msg_all, 32, sig_all, dom_all).all()
    steps = max(args.steps, 3)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        native.verify_multiple_batch(off, pk_all, msg_all, 32, sig_all, dom_all)
    t = _max_time(time.perf_counter() - t0, world, dist, dev)
    batched = {"calls": nc, "L": Lm, "ms_per_batch": 1e3 * t / steps,
               "pairings_per_s": nc * (Lm + 1) * steps * world / t}
    return {"workload": "C5: one bls_verify_multiple per GPU with L distinct messages, one key each, aggregated "
                        "signature, domain 1 (host buffers)", "n_gpus": world, "points": out,
            "batched": batched}


def bench_native_comm(native, args, world, rank, dist, dev):
    """The library's own RCCL communicator (bls381_amd.comm, no torch in the data path; torch only
    hands the 128-byte unique id around here): C4 as ONE collective bls_aggregate_pubkeys over all
    ranks' keys, and one C5 bls_verify_multiple (L = 4096) split across the ranks by message with a
    single final exponentiation on rank 0."""
    import torch
    from bls381_amd import comm
    if world > 1:
        box = [comm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        uid = box[0]
    else:
        uid = comm.unique_id()
    comm.init(world, rank, uid)
    # one RCCL in the process: the library reuses the one torch.distributed loaded (if any)
    import os
    out = {"n_gpus": world, "rccl": {"library": os.path.realpath(comm.rccl_path()),
                                     "mapped": comm.loaded_rccl_paths()}}
    out["rccl"]["single_copy"] = len(out["rccl"]["mapped"]) <= 1
    # the communicator as the library sees it (bls381_comm_size / _rank): the sharded lines below run
    # through it, not through torch.distributed
    out["rccl"]["world"], out["rccl"]["rank"] = comm.size(), comm.rank()
    if out["rccl"]["world"] != world:
        raise RuntimeError("library communicator has %d ranks, expected %d" % (out["rccl"]["world"], world))
    try:
        k = args.c4_keys * world
        base = native.privtopub_batch(b"".join(j.to_bytes(32, "big") for j in range(1, 65)))
        keys = np.frombuffer(base, dtype=np.uint8).reshape(64, 48)[np.arange(k) % 64]
        key_list = [bytes(r) for r in keys]
        want = native.privtopub_batch((sum((i % 64) + 1 for i in range(k)) % R_ORDER).to_bytes(32, "big"))
        assert comm.aggregate_pubkeys(key_list) == want, "native C4 aggregate mismatch"
        steps = max(args.steps, 3)
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            comm.aggregate_pubkeys(key_list)
        t = _max_time(time.perf_counter() - t0, world, dist, dev)
        out["c4_aggregate"] = {"pubkeys": k, "pubkeys_aggregated_per_s": k * steps / t, "ms_per_aggregate": 1e3 * t / steps,
                               "note": "host keys in (PCIe copies inside the time), one collective call"}
        # the same collective over device-resident keys: each rank's contiguous slice already in HBM
        base, extra = divmod(k, world)
        lo = rank * base + min(rank, extra)
        cnt = base + (1 if rank < extra else 0)
        d_keys = torch.from_numpy(np.ascontiguousarray(keys[lo:lo + cnt]).reshape(-1)).to(dev)
        d_out = torch.zeros(48, dtype=torch.uint8, device=dev)
        d_st = torch.zeros(1, dtype=torch.int32, device=dev)
        d_ws = torch.empty(comm.aggregate_pubkeys_device_workspace_size(cnt), dtype=torch.uint8, device=dev)
        cs = torch.cuda.current_stream(dev).cuda_stream

        def dstep():
            comm.aggregate_pubkeys_device(cnt, d_keys.data_ptr(), d_out.data_ptr(), d_st.data_ptr(), d_ws.data_ptr(), cs)
        dstep()
        torch.cuda.synchronize()
        assert bytes(d_out.cpu().numpy()) == want and int(d_st.item()) == 0, "native C4 device aggregate mismatch"
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            dstep()
        torch.cuda.synchronize()
        t = _max_time(time.perf_counter() - t0, world, dist, dev)
        out["c4_aggregate_device"] = {"pubkeys": k, "pubkeys_aggregated_per_s": k * steps / t,
                                      "ms_per_aggregate": 1e3 * t / steps,
                                      "note": "device-resident keys (each rank its slice), result in HBM on every rank"}
        # C3-shaped epoch through the library's communicator: 1,024 attestations
        # verify_multiple([agg_pk, inf], [m0, m1], sig), contiguous call ranges per rank, every verdict
        # on every rank (bls381_verify_multiple_batch_sharded: no data-path collective)
        rng3 = np.random.default_rng(0xB15_0006)
        nc = args.committees
        sk3 = [int.from_bytes(rng3.bytes(32), "big") % (R_ORDER - 1) + 1 for _ in range(nc)]
        skb3 = b"".join(x.to_bytes(32, "big") for x in sk3)
        m0 = bytearray(rng3.bytes(32 * nc))
        m1 = rng3.bytes(32 * nc)
        apk = native.privtopub_batch(skb3)
        sig3 = native.sign_batch(bytes(m0), skb3, (2).to_bytes(8, "big") * nc)
        want3 = np.ones(nc, dtype=bool)
        for c in range(5, nc, 16):
            m0[32 * c + 7] ^= 0x80
            want3[c] = False
        inf = bytes([0xC0]) + bytes(47)
        pks3 = b"".join(apk[48 * c:48 * c + 48] + inf for c in range(nc))
        msgs3 = b"".join(bytes(m0[32 * c:32 * c + 32]) + m1[32 * c:32 * c + 32] for c in range(nc))
        off3 = np.arange(0, 2 * nc + 1, 2, dtype=np.uint32)
        doms3 = (2).to_bytes(8, "big") * nc
        got3 = comm.verify_multiple_batch(off3, pks3, msgs3, 32, sig3, doms3)
        assert np.array_equal(np.array(got3, dtype=bool), want3), "native C3 sharded verdict mismatch"
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            comm.verify_multiple_batch(off3, pks3, msgs3, 32, sig3, doms3)
        t = _max_time(time.perf_counter() - t0, world, dist, dev)
        out["c3_epoch_sharded"] = {"attestations": nc, "attestations_per_s": nc * steps / t,
                                   "ms_per_epoch": 1e3 * t / steps,
                                   "note": "committee aggregates given (privtopub of the summed key), host buffers in, "
                                           "contiguous call ranges per rank, verdicts on every rank"}
        rng = np.random.default_rng(0xB15_0005)
        Lm = 4096
        sks = [int.from_bytes(rng.bytes(32), "big") % (R_ORDER - 1) + 1 for _ in range(Lm)]
        skb = b"".join(x.to_bytes(32, "big") for x in sks)
        m = rng.bytes(32 * Lm)
        pkb = native.privtopub_batch(skb)
        sig = native.aggregate_signatures(native.sign_batch(m, skb, (1).to_bytes(8, "big") * Lm))
        pk_list = [pkb[48 * j:48 * j + 48] for j in range(Lm)]
        m_list = [m[32 * j:32 * j + 32] for j in range(Lm)]
        assert comm.verify_multiple(pk_list, m_list, sig, 1) is True
        assert comm.verify_multiple(pk_list, m_list, sig, 2) is False
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            comm.verify_multiple(pk_list, m_list, sig, 1)
        t = _max_time(time.perf_counter() - t0, world, dist, dev)
        out["c5_split_call"] = {"L": Lm, "ms_per_call": 1e3 * t / steps, "pairings_per_s": (Lm + 1) * steps / t}
    finally:
        comm.destroy()
    return out


def bench_randomized(native, L, args, pks, msgs, sigs, doms, expected, world, dist, dev, stream, t_u8):
    """Opt-in randomized batch verification (bls381_verify_batch_randomized_device): sub-batches
    of 32 items (--rb-batch) share one final exponentiation; per-item verdicts (failing sub-batches are
    re-verified item by item).  On the clean C2 batch, and on the bench's 1/16-tampered one
    (nearly every sub-batch then fails: the fallback cost)."""
    import torch
    n = len(pks) // 48
    sizes = [int(x) for x in args.rb_batch.split(",") if x]
    res = {}
    for B in sizes:
        res[str(B)] = _bench_randomized_b(native, L, args, pks, msgs, sigs, doms, expected, world, dist, dev,
                                          stream, t_u8, n, B)
    out = dict(res[str(sizes[0])])
    if len(sizes) > 1:
        out["by_sub_batch"] = res
    return out


def _bench_randomized_b(native, L, args, pks, msgs, sigs, doms, expected, world, dist, dev, stream, t_u8, n, B):
    import torch
    clean_msgs, clean_sigs = make_workload.clean
    out = {"sub_batch": B}
    ws = torch.empty(L.bls381_verify_batch_randomized_workspace_size(n, B), dtype=torch.uint8, device=dev)
    d_v = torch.zeros(n, dtype=torch.uint8, device=dev)
    for name, m, sg, want in (("clean", clean_msgs, clean_sigs, np.ones(n, dtype=bool)),
                              ("tampered_1_in_16", msgs, sigs, expected)):
        d = [t_u8(pks), t_u8(m), t_u8(sg), t_u8(doms)]
        st = (ctypes.c_uint64 * 3)()

        def step():
            native.check(L.bls381_verify_batch_randomized_device(
                n, *[x.data_ptr() for x in d], os.urandom(32), B, d_v.data_ptr(), ws.data_ptr(),
                ctypes.c_void_p(stream.cuda_stream), st))
        step()
        assert np.array_equal(d_v.cpu().numpy().astype(bool), want), "randomized verdict mismatch (%s)" % name
        steps = max(args.steps, 3)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        t = _max_time(time.perf_counter() - t0, world, dist, dev)
        out[name] = {"verifications_per_s": n * steps * world / t, "ms_per_step": 1e3 * t / steps,
                     "accepted_in_batches": int(st[0]), "verified_singly": int(st[1]), "failed_sub_batches": int(st[2])}
        if name == "clean":
            # the path's own roofline: per-kernel HIP-event times from two extra,
            # untimed steps, and its algorithmic work per item against the clean step's time
            native.profile_enable(True)
            for _ in range(2):
                step()
            torch.cuda.synchronize()
            prof = native.profile_read()
            native.profile_enable(False)
            out["roofline"] = rb_roofline(pks, msgs, sigs, doms, B, n, {k: v["total_ms"] / 2 for k, v in prof.items()},
                                          1e-3 * out["clean"]["ms_per_step"])
    return out


def rb_roofline(pks, msgs, sigs, doms, B, n, kern_ms, step_s):
    """Algorithmic work of the randomized path (Fp-product equivalents per item, MAC-weighted as the
    headline's) over the clean step's wall time, and the item Miller accumulation (k_ml_accum_q, its
    largest kernel) against its own launch time."""
    import build_native
    c = count_fp_muls(pks, msgs, sigs, doms)
    L = ctypes.CDLL(build_native.build_hostcheck(count_ops=True))
    rb = np.zeros(5)
    for i in range(4):
        o = (ctypes.c_uint64 * 5)()
        if L.hc_count_rb_item(pks[48 * i:48 * i + 48], sigs[96 * i:96 * i + 96], 0x9E3779B9 ^ i, 0x7F4A7C15 + i, o) == 0:
            rb += np.array(list(o), dtype=float)
    rb /= 4 * ISSUED_MACS_PER_FP_MUL
    sig_sum = 15 * rb[2] if B <= 256 else rb[3]   # bucket MSM (2 x 8 windows x 15/16 adds) or the ladder
    per_item = {"decode_g1": c["decode_g1"], "scale_g1": rb[0], "decode_g2": c["decode_g2"], "g2_test": rb[1],
                "hash_to_g2": c["hash_to_g2"], "item_miller_lines": c["miller_lines"] / 2,
                "item_miller_accum": c["miller_accum"] / 2, "signature_sum": sig_sum,
                "sub_batch_products": 54 * 0.5, "sub_batch_miller": rb[4] / B, "sub_batch_final_exp": c["final_exp"] / B}
    peak, _ = load_valu_peak()
    work = sum(per_item.values())
    whole = work * MACS_PER_FP_MUL * n / step_s / 1e12
    res = {"fp_mul_per_item": {k: round(v, 1) for k, v in per_item.items()}, "fp_mul_per_item_total": round(work, 1),
           "default_path_fp_mul_per_item": round(sum(c[k] for k in PIPELINE_STAGES), 1),
           "pipeline_achieved": round(whole, 3), "pipeline_frac": round(whole / peak, 4) if peak else None,
           "peak": peak, "unit": "T MAC/s", "kernel_avg_ms": {k: round(v, 3) for k, v in kern_ms.items()}}
    acc_ms = kern_ms.get("rb_miller_accum")
    if acc_ms:
        a = c["miller_accum"] * MACS_PER_FP_MUL * (n / 2) / (1e-3 * acc_ms) / 1e12
        res["dominant"] = {"kernel": "rb_miller_accum (k_ml_accum_q)", "achieved": round(a, 3),
                           "frac": round(a / peak, 4) if peak else None}
    return res


def bench_latency(native, pks, msgs, sigs, expected):
    """Single-call latency through the drop-in shim (the reference calls BLS one signature at a
    time: 0_beacon-chain.md:1594,1603,1664,1756,1796,1824): bls_verify and an attestation-shaped
    bls_verify_multiple, host bytes in, bool out (PCIe copies, launches and the sync included);
    plus small device batches, where the quad Miller loop halves the per-item latency."""
    from bls381_amd import bls
    reps = 15
    out = {}
    times = []
    for i in range(reps):
        t0 = time.perf_counter()
        v = bls.bls_verify(pks[48 * i:48 * i + 48], msgs[32 * i:32 * i + 32], sigs[96 * i:96 * i + 96], DOMAIN_DEPOSIT)
        times.append(time.perf_counter() - t0)
        assert v == bool(expected[i])
    out["bls_verify_ms"] = {"median": 1e3 * float(np.median(times)), "min": 1e3 * min(times)}
    inf = bytes([0xC0]) + bytes(47)
    times = []
    for i in range(reps):
        t0 = time.perf_counter()
        bls.bls_verify_multiple([pks[48 * i:48 * i + 48], inf], [msgs[32 * i:32 * i + 32], bytes(32)],
                                sigs[96 * i:96 * i + 96], DOMAIN_DEPOSIT)
        times.append(time.perf_counter() - t0)
    out["bls_verify_multiple_attestation_ms"] = {"median": 1e3 * float(np.median(times)), "min": 1e3 * min(times)}
    for k in (64, 1024, 16384):
        native.verify_batch(pks[:48 * k], msgs[:32 * k], sigs[:96 * k], DOMAIN_DEPOSIT.to_bytes(8, "big") * k)
        t0 = time.perf_counter()
        v = native.verify_batch(pks[:48 * k], msgs[:32 * k], sigs[:96 * k], DOMAIN_DEPOSIT.to_bytes(8, "big") * k)
        dt = time.perf_counter() - t0
        assert np.array_equal(v, expected[:k])
        out["verify_batch_%d" % k] = {"ms": 1e3 * dt, "verifications_per_s": k / dt}
    return out


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("WORLD_SIZE=%d but --gpus %d" % (world, args.gpus))
    if args.dry_run:
        dry_run(args, world, rank)
        return
    import torch
    import torch.distributed as dist
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local_rank))
        if dist.get_world_size() != args.gpus:
            raise SystemExit("RCCL world is %d ranks, --gpus %d" % (dist.get_world_size(), args.gpus))
    torch.cuda.set_device(local_rank)
    from bls381_amd import _native as native
    native.init(local_rank)
    L = native.lib()
    native.set_subgroup_policy(args.policy)

    # ---------------- workload, device-resident
    n = args.n
    pks, msgs, sigs, doms, expected, sk_ints = make_workload(native, n, 0xB15_0001 + rank)
    dev = torch.device("cuda", local_rank)
    t_u8 = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)
    d_pks, d_msgs, d_sigs, d_doms = t_u8(pks), t_u8(msgs), t_u8(sigs), t_u8(doms)
    stream = torch.cuda.current_stream(dev)
    # --inflight K: consecutive steps alternate over K streams, each with its own workspace and verdict
    # buffer, so a step's first launches need not wait for the previous step's last ones (independent
    # batches, as a node verifying a stream of them would run them); every step still does the whole
    # pipeline over its batch and every step's verdicts are checked below
    kin = max(1, args.inflight)
    streams = [stream] + [torch.cuda.Stream(dev) for _ in range(kin - 1)]
    wss = [torch.empty(L.bls381_verify_batch_workspace_size(n), dtype=torch.uint8, device=dev) for _ in range(kin)]
    vers = [torch.zeros(n, dtype=torch.uint8, device=dev) for _ in range(kin)]
    d_ver, ws = vers[0], wss[0]
    counter = [0]

    def step():
        j = counter[0] % kin
        counter[0] += 1
        rc = L.bls381_verify_batch_device(n, d_pks.data_ptr(), d_msgs.data_ptr(), d_sigs.data_ptr(),
                                          d_doms.data_ptr(), vers[j].data_ptr(), wss[j].data_ptr(),
                                          ctypes.c_void_p(streams[j].cuda_stream))
        native.check(rc)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    for v in vers:
        v.zero_()
    torch.cuda.synchronize()
    native.profile_enable(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    prof = native.profile_read()
    native.profile_enable(False)
    for j, v in enumerate(vers[:min(kin, args.steps)]):
        got = v.cpu().numpy().astype(bool)
        if not np.array_equal(got, expected):
            raise SystemExit("verdict mismatch on rank %d (stream %d): %d wrong" % (rank, j, int((got != expected).sum())))
    counter[0] = 0
    rank_ms = [1e3 * elapsed / args.steps]
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        allt = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(allt, t)
        rank_ms = [1e3 * float(x.item()) / args.steps for x in allt]
        elapsed = max(float(x.item()) for x in allt)
    total_items = n * args.steps * world
    value = total_items / elapsed
    # the same K steps again with the per-launch HIP events off (the headline keeps
    # the events, which the roofline's kernel times come from; this shows what they cost)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    quiet = _max_time(time.perf_counter() - t0, world, dist, dev)
    counter[0] = 0
    no_events = {"ms_per_step": round(1e3 * quiet / args.steps, 3), "value": round(total_items / quiet, 2)}

    def bench_other_policy():
        # the same batch under the other subgroup policy (same verdicts: no torsion points in it)
        pol = "strict" if args.policy == "pyecc" else "pyecc"
        native.set_subgroup_policy(pol)
        try:
            step()
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
            ot = _max_time(time.perf_counter() - t0, world, dist, dev)
            assert np.array_equal(d_ver.cpu().numpy().astype(bool), expected), "verdict mismatch under " + pol
        finally:
            native.set_subgroup_policy(args.policy)
        return {"subgroup_policy": pol, "verifications_per_s": n * args.steps * world / ot,
                "ms_per_step": 1e3 * ot / args.steps}

    def bench_aggregation():
        # committee aggregation (C3 shape), device-resident
        nc, cs = args.committees, args.committee_size
        # distinct committees drawn from the 2^16 generated keys (131072 member slots)
        rng = np.random.default_rng(0xB15_0003 + rank)
        idx = rng.integers(0, n, nc * cs)
        pk_arr = np.frombuffer(pks, dtype=np.uint8).reshape(n, 48)
        cpks = pk_arr[idx].tobytes()
        offsets = np.arange(0, nc * cs + 1, cs, dtype=np.uint32)
        d_cpks = t_u8(cpks)
        d_out = torch.zeros(nc * 48, dtype=torch.uint8, device=dev)
        d_st = torch.zeros(nc, dtype=torch.int32, device=dev)
        aws = torch.empty(L.bls381_aggregate_pubkeys_batch_workspace_size(nc, nc * cs), dtype=torch.uint8, device=dev)

        def astep():
            native.check(L.bls381_aggregate_pubkeys_batch_device(
                nc, offsets.ctypes.data_as(ctypes.c_void_p), nc * cs, d_cpks.data_ptr(), d_out.data_ptr(),
                d_st.data_ptr(), aws.data_ptr(), ctypes.c_void_p(stream.cuda_stream)))
        astep()
        torch.cuda.synchronize()
        ref_out, ref_st = native.aggregate_pubkeys_batch(offsets, cpks)   # host-buffer path, same engine
        assert d_out.cpu().numpy().tobytes() == b"".join(ref_out) and not np.any(ref_st), "aggregation mismatch"
        if world > 1:
            dist.barrier()
        a_steps = max(args.steps, 3)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a_steps):
            astep()
        torch.cuda.synchronize()
        at = time.perf_counter() - t0
        # per-kernel HIP-event times for the roofline from extra, untimed steps (the
        # headline rate carries no profiling events)
        native.profile_enable(True)
        for _ in range(2):
            astep()
        torch.cuda.synchronize()
        aprof = native.profile_read()
        native.profile_enable(False)
        if world > 1:
            t = torch.tensor([at], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            at = float(t.item())
        assert int(d_st.abs().sum().item()) == 0
        agg = {"workload": "C3: %d committees x %d pubkeys, bls_aggregate_pubkeys each" % (nc, cs),
               "committee_aggregations_per_s": nc * a_steps * world / at,
               "pubkeys_aggregated_per_s": nc * cs * a_steps * world / at,
               "ms_per_step": 1e3 * at / a_steps,
               "roofline": agg_roofline(aprof, cpks[:48 * cs], cs, nc * cs)}
        agg["registry"] = bench_registry_c3(native, L, args, pks, idx, offsets, d_out, world, dist, dev, stream, t_u8)
        return agg

    # ---------------- the headline's line (rank 0): roofline of the dominant kernel from the timed
    # steps' own HIP-event profile
    line = None
    if rank == 0:
        counts = count_fp_muls(pks, msgs, sigs, doms, strict=int(args.policy == "strict"))
        kern_ms = stage_times(prof, args.steps)   # ms per step of each stage (each kernel once per step)
        dom_k = max(kern_ms, key=kern_ms.get)
        dom_kernels = stage_kernels(dom_k, prof)
        peak, peak_src = load_valu_peak()
        launch_macs = counts.get(dom_k, 0.0) * MACS_PER_FP_MUL * n
        achieved = launch_macs / (kern_ms[dom_k] * 1e-3) / 1e12
        traffic, traffic_src = load_pmc_traffic(dom_kernels, n)
        roofline = {"bound": "valu-int32", "kernel": dom_k, "kernels": [k for k, _ in dom_kernels],
                    "achieved": round(achieved, 3),
                    "peak": peak, "unit": "T MAC/s (v_mad_u64_u32, 32x32+64)",
                    "frac": round(achieved / peak, 4) if peak else None, "traffic": traffic,
                    "traffic_unit": "HBM bytes per step of the stage's launches (PMC FETCH_SIZE x2 + WRITE_SIZE)", "traffic_source": traffic_src,
                    "macs_per_launch": launch_macs,
                    "fp_mul_per_item": counts, "kernel_avg_ms": kern_ms,
                    "peak_source": peak_src}
        # the whole pipeline's work over the timed step's wall time (kernels on the side stream overlap
        # the main stream, so the sum of kernel times would double-count them)
        whole = sum(counts[k] for k in PIPELINE_STAGES) * MACS_PER_FP_MUL * n / (elapsed / args.steps) / 1e12
        roofline["pipeline_achieved"] = round(whole, 3)
        roofline["pipeline_frac"] = round(whole / peak, 4) if peak else None
        roofline["issue"] = issue_roofline(dom_kernels, n, kern_ms[dom_k])
        roofline["occupancy_ceiling"] = mac_stream_ceiling(achieved, peak)
        line = {
            "metric": "BLS sig verifications/sec (whole node)",
            "value": round(value, 2),
            "unit": "verifications/s",
            "n_gpus": world,
            "rccl_world": dist.get_world_size() if world > 1 else 1,
            "rank_ms_per_step": [round(x, 3) for x in rank_ms],
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32 (381-bit Montgomery, 14x28-bit limbs in u32 words)",
            "data": "synthetic (random keys/messages, signatures made on device)",
            "config": {"workload": "C2: %d independent bls_verify deposit PoP checks per GPU (domain=3, 1/16 tampered)" % n,
                       "global_batch": n * world, "parallelism": "dp%d (independent items, no collective)" % world,
                       "batches_in_flight": kin,
                       "subgroup_policy": args.policy},
            "roofline": roofline,
            "no_profiling_events": no_events,
        }

    # ---------------- secondary lines (other policy, C3 aggregation, deposits, randomized, C3-C5,
    # RCCL, latency), after the headline and guarded: an error is recorded in the line instead of
    # losing it.  With several ranks a rank that fails inside a collective would leave the others
    # waiting in it, so any error ends the phase, and a watchdog on every rank ends it after
    # --secondary-timeout s: rank 0 prints the headline with the lines that finished, every rank
    # exits 0 (3 with --fail-on-secondary-error, which tools/gpu_final.sh passes).
    sec = {"c2_host_buffers": None, "other_policy": None, "cpu_baseline": None, "cpu_baseline_cpp": None,
           "aggregation": None}
    import threading
    state = {"printed": False}
    emit_lock = threading.Lock()

    def emit(extra=None):
        with emit_lock:
            if rank == 0 and not state["printed"]:
                state["printed"] = True
                out = dict(line)
                out.update(sec)
                out.update(extra or {})
                print(json.dumps(out), flush=True)

    def stop_phase(msg):
        emit({"secondary_error": msg})
        sys.stdout.flush()
        sys.stderr.write("bench.py rank %d: %s\n" % (rank, msg))
        os._exit(3 if args.fail_on_secondary_error else 0)

    watchdog = None
    if world > 1:
        watchdog = threading.Timer(args.secondary_timeout, stop_phase,
                                   ["secondary lines stopped by the %d s watchdog" % args.secondary_timeout])
        watchdog.daemon = True
        watchdog.start()

    def guarded(key, fn):
        try:
            r = fn()
            if r is not None:
                sec[key] = r
        except Exception as ex:   # noqa: BLE001 -- recorded in the line
            msg = "%s: %s: %s" % (key, type(ex).__name__, ex)
            if world > 1:
                stop_phase(msg)
            sec[key] = {"error": msg}

    def bench_host_buffers():
        # the same C2 batch through the host-buffer entry point (bls381_verify_batch: 184 B per item
        # copied in over PCIe, verdicts copied out, both inside the time) beside the device-resident
        # headline
        native.verify_batch(pks, msgs, sigs, doms)
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            got = native.verify_batch(pks, msgs, sigs, doms)
        ht = _max_time(time.perf_counter() - t0, world, dist, dev)
        assert np.array_equal(got, expected), "host-buffer verdict mismatch"
        return {"entry_point": "bls381_verify_batch (host buffers in, verdicts out)",
                "verifications_per_s": n * args.steps * world / ht, "ms_per_step": 1e3 * ht / args.steps,
                "bytes_in_per_step": 184 * n, "bytes_out_per_step": n}

    only = set(x for x in args.sections.split(",") if x)
    want = lambda k: (not args.no_secondary and not only) or k in only
    if want("host"):
        guarded("c2_host_buffers", bench_host_buffers)
    if not args.no_secondary:
        guarded("other_policy", bench_other_policy)
    if not args.no_aggregate:
        guarded("aggregation", bench_aggregation)
    if want("deposits"):
        guarded("c2_deposits", lambda: bench_deposits(native, L, args, pks, sk_ints, world, dist, dev, stream, t_u8))
    if want("randomized"):
        guarded("c2_randomized_batch", lambda: bench_randomized(native, L, args, pks, msgs, sigs, doms, expected, world,
                                                                dist, dev, stream, t_u8))
    if want("c3"):
        guarded("c3_epoch", lambda: bench_c3(native, L, args, pks, sk_ints, world, rank, dev, stream, t_u8, dist))
    if want("c4"):
        guarded("c4_aggregate", lambda: bench_c4(native, L, args, world, rank, dev, stream, t_u8, dist))
    if want("c5"):
        guarded("c5_multi_pairing", lambda: bench_c5(native, args, world, rank, dist, dev))
    if want("rccl"):
        guarded("native_rccl", lambda: bench_native_comm(native, args, world, rank, dist, dev))
    if want("latency") and rank == 0:
        guarded("latency", lambda: bench_latency(native, pks, msgs, sigs, expected))
    if watchdog is not None:
        watchdog.cancel()

    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:
            rate, res, dt = cpu_baseline(pks, msgs, sigs, args.cpu_sample, args.cpu_procs)
            assert list(res) == list(expected[:args.cpu_sample]), "CPU oracle disagrees with GPU verdicts"
            sec["cpu_baseline"] = {
                "value": round(rate, 3), "unit": "verifications/s", "cores": args.cpu_procs, "kind": "port",
                "sample": "first %d items of the same C2 batch, oracle/bls_oracle.py verify (py_ecc 1.7.0 "
                          "algorithm restatement: Fq12-coordinate Miller loop, naive final exponentiation), "
                          "multiprocessing.Pool(%d), %.1f s wall" % (args.cpu_sample, args.cpu_procs, dt)}
            k = min(args.cpp_sample, n)
            rate, res, dt = cpu_baseline_cpp(pks[:48 * k], msgs[:32 * k], sigs[:96 * k], doms[:8 * k], k, args.cpu_procs)
            assert res == list(expected[:k]), "C++ host build disagrees with GPU verdicts"
            sec["cpu_baseline_cpp"] = {
                "value": round(rate, 3), "unit": "verifications/s", "cores": args.cpu_procs, "kind": "port",
                "sample": "first %d items of the same C2 batch, C++ host build of the engine's arithmetic headers "
                          "(g++ -O2, host_check.cpp hc_verify_batch_mt), %d std::threads, %.1f s wall"
                          % (k, args.cpu_procs, dt)}

        emit()
    if world > 1:
        dist.destroy_process_group()
    failed = [k for k, v in sec.items() if isinstance(v, dict) and "error" in v]
    if failed and args.fail_on_secondary_error:
        sys.stderr.write("bench.py rank %d: secondary lines failed: %s\n" % (rank, ", ".join(failed)))
        sys.exit(3)


if __name__ == "__main__":
    main()
