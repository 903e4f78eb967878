#!/usr/bin/env python3
"""bench_fit.py -- config 5 (extra.py system identification) on one MI355X.

One step = one extra.py training iteration of the differentiable MPM
(extra.py:205-241 without the renderer): 30 x p2g2p_forward(0.03/30, s),
postprocess_forward, set_grads, postprocess_backward, 30 x p2g2p_backward,
learn, cycle_init -- on n_grid 50 (extra.py:57), sticky ground, SURVEY §8(d)
config E: 20,000 torus Gaussians (R = 0.3, r = 0.1; models_extra/torus is not
in the reference, so the torus and its initial velocity are synthetic).

Prints one JSON line like bench.py: value = particle-substeps/s counting the
forward and backward substeps (2 x 30 per particle per iteration); a
cpu_baseline of the serial oracle (oracle/diff_oracle.c) on a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting-mpm_amd")]

NG, EXT, DT, NSUB = 50, 2.0, 0.03 / 30, 30
MAT = dict(E=2e5, nu=0.3, density=1000.0)
GRAV = (0.0, -9.8, 0.0)


def torus(n, seed=0):
    rng = np.random.default_rng(seed)
    th, ph = rng.uniform(0, 2 * np.pi, n), rng.uniform(0, 2 * np.pi, n)
    r, R = 0.1 * np.sqrt(rng.uniform(0, 1, n)), 0.3
    x = np.stack([1.0 + (R + r * np.cos(ph)) * np.cos(th), 0.85 + r * np.sin(ph),
                  1.0 + (R + r * np.cos(ph)) * np.sin(th)], 1).astype(np.float32)
    cov = np.tile(np.array([4e-6, 1e-6, 0, 4e-6, 5e-7, 4e-6], np.float32), (n, 1))
    v = np.stack([np.zeros(n), -np.full(n, 1.5), 0.5 * np.cos(th)], 1).astype(np.float32)
    return x, cov, v


def volumes(x):
    # get_particle_volume (filling.py:27-42): grid_dx^3 / particles in the cell
    cell = np.floor(x * (NG / EXT)).astype(np.int64)
    key = (cell[:, 0] * NG + cell[:, 1]) * NG + cell[:, 2]
    _, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
    return ((EXT / NG) ** 3 / cnt[inv]).astype(np.float32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--particles", type=int, default=20_000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--cpu-particles", type=int, default=4000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    a = ap.parse_args()
    import torch
    from gsmpm.fit import FitSimulator
    dev = torch.device("cuda:0")
    n = a.particles
    x, cov, v = torus(n)
    vol = volumes(x)
    t = lambda arr: torch.from_numpy(np.ascontiguousarray(arr)).to(dev)
    g = FitSimulator(n, n_grid=NG, grid_extent=EXT, gravity=GRAV, **MAT)
    g.set_particles(t(x), t(cov), t(vol), t(v))
    g.set_bc_ground_only()
    gx = t(np.random.default_rng(1).normal(0, 1, (n, 3)).astype(np.float32))
    gc = t(np.full(n * 6, 10.0, np.float32))
    st = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]

    def iteration(split=False):
        if split:
            ev[0].record(st)
        for s in range(NSUB):
            g.forward(DT, s)
        g.postprocess_forward()
        if split:
            ev[1].record(st)
        g.clear_grads()
        g.set_grads(gx, gc)
        g.postprocess_backward()
        for s in reversed(range(NSUB)):
            g.backward(DT, s)
        g.learn()
        g.cycle_init()
        if split:
            ev[2].record(st)

    for _ in range(a.warmup):
        iteration()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        iteration()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    iteration(split=True)
    torch.cuda.synchronize()
    fwd_ms, bwd_ms = ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])
    ms = el / a.steps * 1e3
    cpu = None
    if not a.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        m = a.cpu_particles
        xc, cc, vc = torus(m, 2)
        o = O.OracleDiff(xc, cc, volumes(xc), n_grid=NG, grid_extent=EXT, gravity=GRAV, init_v=vc,
                         ground_only=True, **MAT)
        c0 = time.perf_counter()
        for s in range(NSUB):
            o.p2g2p_forward(DT, s)
        o.postprocess_forward()
        o.clear_grads()
        o.set_grads(np.ones((m, 3), np.float32), np.ones(m * 6, np.float32))
        o.postprocess_backward()
        for s in reversed(range(NSUB)):
            o.p2g2p_backward(DT, s)
        o.learn()
        o.cycle_init()
        cs = time.perf_counter() - c0
        cpu = {"value": 2 * NSUB * m / cs, "unit": "particle-substeps/s", "cores": 1, "kind": "port",
               "sample": f"one iteration (30 fwd + 30 bwd substeps) of {m} torus particles, serial oracle"}
    print(json.dumps({
        "metric": "extra.py fit iterations/s (config 5, differentiable MPM fwd+bwd)",
        "value": 2 * NSUB * n / (ms / 1e3), "unit": "particle-substeps/s (fwd+bwd)", "n_gpus": 1,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": ms, "iterations_per_s": 1e3 / ms,
        "forward_ms": fwd_ms, "backward_ms": bwd_ms, "higher_is_better": True, "dtype": "f32",
        "data": "synthetic torus", "config": {"workload": "config 5 (extra.py), n_grid 50, 30 substeps",
                                              "particles": n}, "cpu_baseline": cpu}))


if __name__ == "__main__":
    main()
