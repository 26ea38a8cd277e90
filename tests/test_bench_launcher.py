"""bench.py's rank launcher on the CPU (no GPU touched): `bench.py --gpus N` with WORLD_SIZE
unset starts N rank processes, which join one world (gloo in --dry-run) and report it; a world
that is not N ranks is an error (BASELINE.json `metric`: verifications/s at 1/2/4/8 GPUs)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=240)


def test_launcher_two_ranks_dry_run():
    r = _bench(["--gpus", "2", "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line == {"dry_run": True, "n_gpus": 2, "rccl_world": 2, "ranks": [0, 1]}


def test_launcher_one_rank_dry_run():
    r = _bench(["--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["rccl_world"] == 1


def test_world_size_must_match_gpus():
    r = _bench(["--gpus", "2", "--dry-run"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=1 but --gpus 2" in r.stderr


def test_launcher_ends_the_other_ranks_when_one_fails():
    """A rank that dies leaves its peers waiting in the rendezvous: the launcher ends them and fails
    instead of hanging (the driver's scaling run must not wait on a dead world)."""
    import time
    t0 = time.time()
    r = _bench(["--gpus", "3", "--dry-run", "--dry-run-fail-rank", "1"])
    assert r.returncode != 0
    assert "rank exit codes" in r.stderr
    assert time.time() - t0 < 120
