"""bench.py's rank bookkeeping (CPU): --gpus N starts N ranks itself when no
launcher did, refuses a launcher that started a different number, and the
JSON line's n_gpus / parallelism come from the ranks that actually ran
(`--dry-run`: the same launch path, gloo on the CPU, no GPU work)."""
from __future__ import annotations

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    env["OMP_NUM_THREADS"] = "1"
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True, timeout=240)


def _line(p):
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    return json.loads(lines[0])


def test_gpus_flag_starts_that_many_ranks():
    """The default N > 1 headline is north_star's design: one lego scene
    sharded by spatial slab over the N ranks (strong scaling)."""
    out = _line(_run(["--gpus", "2", "--dry-run"]))
    assert out["n_gpus"] == 2 and out["scaling"] == "strong"
    assert out["config"]["parallelism"] == "slab2"


def test_gpus_flag_slab_mode():
    for flag in (["--slab"], ["--multi", "slab"]):
        out = _line(_run(["--gpus", "2", "--dry-run"] + flag))
        assert out["n_gpus"] == 2 and out["scaling"] == "strong"
        assert out["config"]["parallelism"] == "slab2"
    out = _line(_run(["--gpus", "2", "--dp", "--dry-run"]))
    assert out["scaling"] == "weak" and out["config"]["parallelism"].startswith("dp2")


def test_default_is_one_rank():
    out = _line(_run(["--dry-run"]))
    assert out["n_gpus"] == 1 and out["config"]["parallelism"] == "single"


def test_launcher_rank_count_must_match_flag():
    p = _run(["--gpus", "8", "--dry-run"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0
    assert "--gpus 8" in p.stderr and "WORLD_SIZE=1" in p.stderr
