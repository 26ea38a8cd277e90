"""YAML test-vector generator and runner for the `bls` test format.

Generator: the layout test_generators/bls/main.py writes through gen_base.gen_runner
(test_libs/gen_helpers/gen_base/gen_runner.py:97-111: `<out>/<handler dir>/<name>.yaml`)
and gen_suite.render_suite (gen_suite.py:7-22: title, summary, forks_timeline, forks,
config, runner, handler, test_cases), with the same inputs (main.py:30-53: DOMAINS,
MESSAGES, PRIVKEYS) and the same encodings (main.py:19-23 int_to_hex, coordinates
zero-padded to 48 bytes, main.py:68-69,85).  Outputs are computed by the gfx950 engine
in place of py_ecc.

Runner: reads any directory of such suites (specs/test_formats/bls/*.md) and checks
every case against the engine, handler by handler.

    python -m bls381_amd.vector_runner generate OUT_DIR
    python -m bls381_amd.vector_runner run DIR
"""
from __future__ import annotations

import os
import sys

import yaml

# test_generators/bls/main.py:30-53
DOMAINS = [0, 1, 1234, 2 ** 32 - 1, 2 ** 64 - 1]
MESSAGES = [bytes(b"\x00" * 32), bytes(b"\x56" * 32), bytes(b"\xab" * 32)]
PRIVKEYS = [
    0x263dbd792f5b1be47ed85f8938c0f29586af0d3ac7b977f21c278fe1462040e3,
    0x47b8192d77bf871b62e87859d653922725724a5c031afeabc60bcef5ff665138,
    0x328388aff0d4a5b7dc9205abd374e7e98f3cd9f3418edb4eafda5fb16473d216,
]

# (output file name, handler directory, suite title, suite handler) -- main.py:164-238
SUITES = [
    ("g2_uncompressed", "msg_hash_g2_uncompressed", "BLS G2 Uncompressed msg hash", "msg_hash_uncompressed"),
    ("g2_compressed", "msg_hash_g2_compressed", "BLS G2 Compressed msg hash", "msg_hash_compressed"),
    ("priv_to_pub", "priv_to_pub", "BLS private key to pubkey", "priv_to_pub"),
    ("sign_msg", "sign_msg", "BLS sign msg", "sign_msg"),
    ("aggregate_sigs", "aggregate_sigs", "BLS aggregate sigs", "aggregate_sigs"),
    ("aggregate_pubkeys", "aggregate_pubkeys", "BLS aggregate pubkeys", "aggregate_pubkeys"),
]
SUMMARIES = {
    "priv_to_pub": "BLS Convert private key to public key",
    "sign_msg": "BLS Sign a message",
    "aggregate_sigs": "BLS Aggregate signatures",
    "aggregate_pubkeys": "BLS Aggregate public keys",
}


def int_to_hex(n: int, byte_length: int = None) -> str:
    """main.py:19-23 (eth_utils int_to_big_endian: minimal big-endian, 0 -> 0x00)."""
    b = n.to_bytes(max(1, (n.bit_length() + 7) // 8), "big")
    if byte_length:
        b = b.rjust(byte_length, b"\x00")
    return "0x" + b.hex()


def _h(b: bytes) -> str:
    return "0x" + bytes(b).hex()


def _unhex(s: str) -> bytes:
    return bytes.fromhex(s[2:] if s.startswith("0x") else s)


# ------------------------------------------------------------------ cases --
def generate_cases(bls) -> dict:
    """All 94 cases of main.py's six suites, outputs from `bls` (the engine's bls module)."""
    cases = {h: [] for _, h, _, _ in SUITES}
    for msg in MESSAGES:                                               # case01 (main.py:85-96)
        for d in DOMAINS:
            X, Y, Z = bls.hash_to_G2_pyecc_projective(msg, d)
            cases["msg_hash_g2_uncompressed"].append({
                "input": {"message": _h(msg), "domain": int_to_hex(d)},
                "output": [[int_to_hex(c, 48) for c in pt] for pt in (X, Y, Z)]})
    for msg in MESSAGES:                                               # case02 (main.py:99-109)
        for d in DOMAINS:
            comp = bls.hash_to_G2_compressed(msg, d)
            cases["msg_hash_g2_compressed"].append({
                "input": {"message": _h(msg), "domain": int_to_hex(d)},
                "output": [_h(comp[:48]), _h(comp[48:])]})
    for sk in PRIVKEYS:                                                # case03 (main.py:112-119)
        cases["priv_to_pub"].append({"input": int_to_hex(sk), "output": _h(bls.privtopub(sk))})
    for sk in PRIVKEYS:                                                # case04 (main.py:122-135)
        for msg in MESSAGES:
            for d in DOMAINS:
                cases["sign_msg"].append({
                    "input": {"privkey": int_to_hex(sk), "message": _h(msg), "domain": int_to_hex(d)},
                    "output": _h(bls.bls_sign(msg, sk, d))})
    for d in DOMAINS:                                                  # case06 (main.py:142-149)
        for msg in MESSAGES:
            sigs = [bls.bls_sign(msg, sk, d) for sk in PRIVKEYS]
            cases["aggregate_sigs"].append({"input": [_h(s) for s in sigs],
                                            "output": _h(bls.bls_aggregate_signatures(sigs))})
    pks = [bls.privtopub(sk) for sk in PRIVKEYS]                       # case07 (main.py:152-158)
    cases["aggregate_pubkeys"].append({"input": [_h(p) for p in pks], "output": _h(bls.bls_aggregate_pubkeys(pks))})
    return cases


def write_suites(out_dir: str, cases: dict) -> list:
    """gen_runner.py:97-111 layout; returns the written paths."""
    paths = []
    for name, hdir, title, handler in SUITES:
        suite = {"title": title, "summary": SUMMARIES.get(hdir, title), "forks_timeline": "mainnet",
                 "forks": ["phase0"], "config": "mainnet", "runner": "bls", "handler": handler,
                 "test_cases": cases[hdir]}
        d = os.path.join(out_dir, hdir)
        os.makedirs(d, exist_ok=True)
        p = os.path.join(d, name + ".yaml")
        with open(p, "w") as f:
            yaml.safe_dump(suite, f, sort_keys=False, default_flow_style=None)
        paths.append(p)
    return paths


def load_suites(root: str) -> list:
    """Every *.yaml suite under root whose runner is `bls` (yaml.safe_load: data only)."""
    out = []
    for dp, _, files in sorted(os.walk(root)):
        for fn in sorted(files):
            if fn.endswith((".yaml", ".yml")):
                with open(os.path.join(dp, fn)) as f:
                    s = yaml.safe_load(f)
                if isinstance(s, dict) and s.get("runner") == "bls":
                    out.append((os.path.join(dp, fn), s))
    return out


# ---------------------------------------------------------------- handlers --
# specs/test_formats/bls/<handler>.md "Condition" sections
def _case_msg_hash_uncompressed(bls, c):
    i = c["input"]
    X, Y, Z = bls.hash_to_G2_pyecc_projective(_unhex(i["message"]), int(i["domain"], 16))
    return [[int(a, 16), int(b, 16)] for a, b in c["output"]] == [list(X), list(Y), list(Z)]


def _case_msg_hash_compressed(bls, c):
    i = c["input"]
    comp = bls.hash_to_G2_compressed(_unhex(i["message"]), int(i["domain"], 16))
    return comp == _unhex(c["output"][0]) + _unhex(c["output"][1])


def _case_priv_to_pub(bls, c):
    return bls.privtopub(int(c["input"], 16)) == _unhex(c["output"])


def _case_sign_msg(bls, c):
    i = c["input"]
    return bls.bls_sign(_unhex(i["message"]), int(i["privkey"], 16), int(i["domain"], 16)) == _unhex(c["output"])


def _case_aggregate_sigs(bls, c):
    return bls.bls_aggregate_signatures([_unhex(s) for s in c["input"]]) == _unhex(c["output"])


def _case_aggregate_pubkeys(bls, c):
    return bls.bls_aggregate_pubkeys([_unhex(p) for p in c["input"]]) == _unhex(c["output"])


HANDLERS = {
    "msg_hash_uncompressed": _case_msg_hash_uncompressed,
    "msg_hash_g2_uncompressed": _case_msg_hash_uncompressed,
    "msg_hash_compressed": _case_msg_hash_compressed,
    "msg_hash_g2_compressed": _case_msg_hash_compressed,
    "priv_to_pub": _case_priv_to_pub,
    "sign_msg": _case_sign_msg,
    "aggregate_sigs": _case_aggregate_sigs,
    "aggregate_pubkeys": _case_aggregate_pubkeys,
}


def run(root: str, bls=None) -> dict:
    """Check every case of every bls suite under root; {path: (passed, failed_case_indices)}."""
    if bls is None:
        from . import bls as _bls
        bls = _bls
    res = {}
    for path, suite in load_suites(root):
        fn = HANDLERS.get(suite["handler"])
        if fn is None:
            raise ValueError("unknown bls handler %r in %s" % (suite["handler"], path))
        failed = [k for k, c in enumerate(suite["test_cases"]) if not fn(bls, c)]
        res[path] = (len(suite["test_cases"]) - len(failed), failed)
    return res


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if len(argv) != 2 or argv[0] not in ("generate", "run"):
        print(__doc__)
        return 2
    from . import _native, bls
    _native.init(0)
    if argv[0] == "generate":
        for p in write_suites(argv[1], generate_cases(bls)):
            print(p)
        return 0
    bad = 0
    for path, (ok, failed) in run(argv[1], bls).items():
        print("%-60s %4d passed %4d failed" % (path, ok, len(failed)))
        bad += len(failed)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
