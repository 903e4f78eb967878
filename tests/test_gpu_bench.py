"""bench.py end to end on the GPU (the driver runs it at round end): the JSON
line's contract, and the render worker thread (the default) rendering the
same frames as the frame loop's own thread."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*extra):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
           "--no-extra-configs", *extra]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_line_contract_and_render_thread():
    d = _bench()
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["value"] > 0 and d["higher_is_better"] is True
    assert d["config"]["render_thread"] is True and d["config"]["render_overlap"] is True
    r = d["roofline"]
    assert r["bound"] == "hbm" and 0 < r["frac"] < 1 and r["peak"] == 8000.0
    # the loop's own thread renders the same frames: the same pair count for the last frame
    d0 = _bench("--render-thread", "0")
    assert d0["config"]["render_thread"] is False
    assert d0["num_rendered"] == d["num_rendered"] > 0


def test_bench_two_ranks_on_one_gpu_multi_fields():
    """--gpus 2 rehearsed on one GPU (GSMPM_SHARE_GPU=1: both ranks on cuda:0,
    RCCL over its socket transport): the default dp headline (weak scaling)
    and the multi_gpu side measurements -- lego through 2 slabs with the
    render-aware re-cut (per-rank sim ms, rank-0 render / gather ms, rank 0's
    weight below 1 and its share of the particles below half) and the sim /
    render split."""
    env = dict(os.environ, GSMPM_SHARE_GPU="1")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--multi-configs", "lego,split"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["config"]["parallelism"].startswith("dp2")
    assert d["value"] > 0 and d["config"]["particles_total"] > d["config"]["particles_per_gpu"]
    m = d["multi_gpu"]
    s = m["B_lego_slab"]
    assert len(s["per_rank_sim_ms"]) == 2 and all(v > 0 for v in s["per_rank_sim_ms"])
    assert s["rank0_render_ms"] > 0 and s["rank0_gather_ms"] >= 0 and 0 < s["rank0_weight"] < 1
    assert sum(s["per_rank_particles"]) == s["particles"]
    assert s["per_rank_particles"][0] < s["particles"] / 2  # the render-aware re-cut moved rank 0's share
    sp = m["B_lego_sim_render_split"]
    assert sp["frame_ms"] > 0 and sp["rank1_sim_ms"] > 0 and sp["rank0_render_ms"] > 0
    assert sp["num_rendered"] > 0
    print(json.dumps(m))
