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
    # the headline is the live-byte basis: achieved = bytes per launch / average launch time
    assert abs(r["achieved"] - r["algorithmic_bytes_per_launch"] / r["avg_launch_us"] / 1e3) < 0.01 * r["achieved"]
    assert 0 < r["substep"]["frac"] < 1 and 0 < r["frac_dense_contract"]
    # no fraction above 1 anywhere in the line (the dense n^3 basis is only a labelled contract figure)
    for k, v in d["kernels_roofline"].items():
        assert 0 < v["frac"] < 1, (k, v)
        assert "dense_rate_GBps" not in v
    # the loop's own thread renders the same frames: the same pair count for the last frame
    d0 = _bench("--render-thread", "0")
    assert d0["config"]["render_thread"] is False
    assert d0["num_rendered"] == d["num_rendered"] > 0


def test_bench_two_ranks_on_one_gpu_multi_fields():
    """--gpus 2 rehearsed on one GPU (GSMPM_SHARE_GPU=1: both ranks on cuda:0,
    RCCL over its socket transport): the default slab headline (one lego
    scene through 2 slabs, strong scaling) with its per-rank fields -- sim ms,
    particles (rank 0's share below half: the render-aware re-cut), the
    window-exchange bytes per substep, migrations, rank-0 render / gather ms --
    and the side measurements: the replicas form (one scene per rank) and the
    sim / render split."""
    env = dict(os.environ, GSMPM_SHARE_GPU="1")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "3",
           "--multi-configs", "dp,split"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["config"]["parallelism"] == "slab2"
    assert d["value"] > 0 and d["steps"] == 2 and d["ms_per_step"] > 0
    s = d["slab"]
    assert s["frames"] == 2 and s["substeps_per_frame"] == 100
    assert len(s["per_rank_sim_ms"]) == 2 and all(v > 0 for v in s["per_rank_sim_ms"])
    assert s["rank0_render_ms"] > 0 and s["rank0_gather_ms"] >= 0 and 0 < s["rank0_weight"] < 1
    assert sum(s["per_rank_particles"]) == s["particles"] == d["config"]["particles_total"]
    assert s["per_rank_particles"][0] < s["particles"] / 2  # the render-aware re-cut moved rank 0's share
    # both ranks share one bound: each sends the same window rect (float4 x planes x rect) every substep
    eb = s["per_rank_exchange_bytes_per_substep"]
    assert eb[0] == eb[1] > 0 and eb[0] % 16 == 0
    assert len(s["per_rank_migrations_per_frame"]) == 2
    m = d["multi_gpu"]
    dp = m["B_lego_dp"]
    assert dp["particles_total"] > s["particles"] and dp["frame_ms"] > 0 and dp["scaling"] == "weak"
    sp = m["B_lego_sim_render_split"]
    assert sp["frame_ms"] > 0 and sp["rank1_sim_ms"] > 0 and sp["rank0_render_ms"] > 0
    assert sp["num_rendered"] > 0
    print(json.dumps(d))
