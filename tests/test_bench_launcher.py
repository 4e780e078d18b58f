"""bench.py's N-rank path on CPU: `python bench.py --gpus N` with no RANK in
the environment spawns N rank processes itself (no external launcher, no
exec), the control plane runs its barrier and max-over-ranks, rank 0 prints
the one JSON line, and a rank that dies fails the whole run instead of
hanging it.  --dry-run skips everything that touches a GPU."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(*args, timeout=120):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT")}
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args],
                          capture_output=True, text=True, timeout=timeout, env=env)


def test_self_launch_spawns_ranks_and_prints_one_line():
    p = run("--gpus", "3", "--dry-run")
    assert p.returncode == 0, p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 3 and d["max_over_ranks"] == 2.0
    assert d["allgather"] == ["r0", "r1", "r2"]  # the handle exchange of the xGMI transport


def test_dead_rank_fails_fast():
    t0 = time.time()
    p = run("--gpus", "2", "--dry-run", "--dry-run-fail-rank", "1")
    assert p.returncode != 0
    assert time.time() - t0 < 60  # rank 0 is killed, not left waiting on accept()


def test_world_size_mismatch_rejected():
    env = dict(os.environ, RANK="0", WORLD_SIZE="2")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4",
                        "--dry-run"], capture_output=True, text=True, timeout=60, env=env)
    assert p.returncode != 0 and "WORLD_SIZE" in p.stderr
