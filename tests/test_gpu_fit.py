"""Differentiable MPM on the GPU (gsmpm_fit_* through gsmpm/fit.py and the
MPM_Simulator(fitting=True) drop-in) against the oracle (oracle/diff_oracle.c,
itself checked by finite differences in test_oracle_diff.py).

Scene: the config-5 shape of extra.py (n_grid 50, extent 2, 30 substeps of
0.03/30, sticky ground, initial velocity), synthetic torus-like blob.
Tolerances (max-abs error over the reference's max-abs value):
  forward  x, F, v, C, stress, cov 1e-4 (measured <= 5e-6 at config E's
  shape; P2G sums in a different order: exact fixed-point sums per chunk
  window, f32 sums of <= 8 windows per node);
  backward adjoints: `_adjoint_close` -- per particle 5e-3 of its own
  magnitude (+1e-3 of the max) for all but 0.1 % of particles, and 5e-2 of the
  max for every particle.  The reference algorithm is ill-conditioned at
  grid nodes of tiny mass (v_out = v_in / m with stress forces that do not
  vanish with the weight), so a particle's logE adjoint can reach 1e10 and
  move by ~2 % with the atomic summation order alone: tools/fit_probe3.py
  measured GPU-vs-GPU run-to-run spreads of up to 2.07e-2 there (12 runs),
  equal to the GPU-vs-oracle maximum, with medians of 2e-6.
  learn: logE/y 1e-5 absolute after one step.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from conftest import rel_err

pytestmark = pytest.mark.gpu

NG, EXT, DT, NSUB = 50, 2.0, 0.03 / 30, 30
MAT = dict(E=2e5, nu=0.3, density=1000.0)
GRAV = (0.0, -9.8, 0.0)


def _scene(n=4000, seed=0):
    rng = np.random.default_rng(seed)
    th = rng.uniform(0, 2 * np.pi, n)
    ph = rng.uniform(0, 2 * np.pi, n)
    r = 0.08 * np.sqrt(rng.uniform(0, 1, n))
    R = 0.25
    x = np.stack([1.0 + (R + r * np.cos(ph)) * np.cos(th), 0.80 + r * np.sin(ph),
                  1.0 + (R + r * np.cos(ph)) * np.sin(th)], 1).astype(np.float32)
    cov = np.tile(np.array([4e-6, 1e-6, 0, 4e-6, 5e-7, 4e-6], np.float32), (n, 1))
    cov *= rng.uniform(0.5, 1.5, (n, 1)).astype(np.float32)
    v = np.stack([np.zeros(n), -np.full(n, 1.5), 0.5 * np.cos(th)], 1).astype(np.float32)
    return x, cov, v


def _adjoint_close(a, b, what, later_iteration=False):
    """Per-element rule above.  later_iteration: the second training iteration
    starts from a state in ground contact where a few particles sit on a
    branch (m > 1e-15, |J| clamp) that summation order can flip;
    tools/fit_probe3.py (12 GPU runs) measured there, GPU-vs-GPU exactly as
    GPU-vs-oracle: 3.4 % of entries beyond 5e-3, 1.7 % beyond 2e-2, 0.4 %
    beyond 5e-2, median 2e-6.  The rule then is: <= 1 % beyond 5e-2, median
    < 1e-4, max 5e-2 of the largest entry."""
    a = np.asarray(a, np.float64).reshape(-1)
    b = np.asarray(b, np.float64).reshape(-1)
    r = np.abs(a - b) / (np.abs(b) + 1e-3 * np.abs(b).max() + 1e-30)
    e = rel_err(a, b)
    med = float(np.median(r))
    if later_iteration:
        frac = float((r > 5e-2).mean())
        assert frac <= 1e-2 and med < 1e-4 and e < 5e-2, (what, frac, e, med)
        return
    frac = float((r > 5e-3).mean())
    assert frac <= 1e-3 and e < 5e-2, (what, frac, e, med)


def _pair(dev, n=4000, seed=0):
    import oracle as O
    from gsmpm.fit import FitSimulator
    x, cov, v = _scene(n, seed)
    vol = O.particle_volume(x, NG, EXT)
    o = O.OracleDiff(x, cov, vol, n_grid=NG, grid_extent=EXT, gravity=GRAV, init_v=v, ground_only=True, **MAT)
    g = FitSimulator(n, n_grid=NG, grid_extent=EXT, gravity=GRAV, **MAT)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    g.set_particles(t(x), t(cov), t(vol), t(v))
    g.set_bc_ground_only()
    return o, g


def _forward(o, g):
    for s in range(NSUB):
        o.p2g2p_forward(DT, s)
        g.forward(DT, s)
    o.postprocess_forward()
    g.postprocess_forward()


def test_fit_forward_matches_oracle(dev):
    o, g = _pair(dev)
    _forward(o, g)
    n = o.n
    for lvl in (1, 10, NSUB):
        for k, tol in (("x", 1e-4), ("F", 1e-4), ("v", 1e-4), ("C", 1e-4)):
            e = rel_err(g.get(k, lvl).cpu().numpy(), getattr(o, k)[lvl])
            assert e < tol, (k, lvl, e)
    for lvl in (0, NSUB - 1):
        e = rel_err(g.get("stress", lvl).cpu().numpy(), o.stress[lvl])
        assert e < 1e-4, ("stress", lvl, e)
    assert rel_err(g.get("cov").cpu().numpy(), o.cov.reshape(n, 6)) < 1e-4
    np.testing.assert_allclose(g.get("mass").cpu().numpy(), o.mass, rtol=1e-6)
    np.testing.assert_allclose(g.get("mu").cpu().numpy(), o.mu, rtol=1e-5)
    np.testing.assert_allclose(g.get("lam").cpu().numpy(), o.lam, rtol=1e-5)
    # the ground BC bit: some particles must have been stopped by the sticky cube
    assert (o.v[NSUB][:, 1] > -0.5).any()


def test_fit_backward_learn_cycle_match_oracle(dev):
    o, g = _pair(dev, n=3000, seed=1)
    _forward(o, g)
    rng = np.random.default_rng(7)
    gx = rng.normal(0, 1, (o.n, 3)).astype(np.float32)
    gc = (rng.normal(0, 1, o.n * 6) * 1e3).astype(np.float32)
    o.clear_grads(); o.set_grads(gx, gc); o.postprocess_backward()
    g.clear_grads(); g.set_grads(torch.from_numpy(gx), torch.from_numpy(gc)); g.postprocess_backward()
    np.testing.assert_array_equal(g.get("gx", NSUB).cpu().numpy(), gx)
    for s in reversed(range(NSUB)):
        o.p2g2p_backward(DT, s)
        g.backward(DT, s)
    for k in ("glogE", "gy", "gmu", "glam"):
        _adjoint_close(g.get(k).cpu().numpy(), getattr(o, k), k)
    for k in ("gx", "gv", "gF", "gC"):
        for lvl in (0, NSUB // 2):
            _adjoint_close(g.get(k, lvl).cpu().numpy(), getattr(o, k)[lvl], (k, lvl))
    o.learn(); g.learn()
    assert np.abs(g.get("logE").cpu().numpy() - o.logE).max() < 1e-5
    assert np.abs(g.get("y").cpu().numpy() - o.y).max() < 1e-5
    o.cycle_init(); g.cycle_init()
    for k in ("x", "v", "F", "C"):
        assert rel_err(g.get(k, 0).cpu().numpy(), getattr(o, k)[0]) < 2e-3, k
    # a second forward pass from the cycled state (bins of level 0 rebuilt)
    for s in range(3):
        o.p2g2p_forward(DT, s)
        g.forward(DT, s)
    assert rel_err(g.get("x", 3).cpu().numpy(), o.x[3]) < 1e-4


def test_fit_grid_levels_equal_recompute(dev):
    """The backward pass reading the grid its forward pass stored per level
    (the default) gives bit-identical adjoints to recomputing P2G + the grid
    update as the reference's p2g2p_backward does: one simulator, one forward
    pass and its bins, the backward pass run twice from the same adjoint seed,
    the second time after mu_lam() (same mu/lam bits) dropped the stored
    grids.  Then a state change between the passes (set x at a level) is seen
    by that level's backward (its grid is recomputed)."""
    import oracle as O
    from gsmpm.fit import FitSimulator
    x, cov, v = _scene(3000, 3)
    vol = O.particle_volume(x, NG, EXT)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    g = FitSimulator(len(x), n_grid=NG, grid_extent=EXT, gravity=GRAV, **MAT)
    g.set_particles(t(x), t(cov), t(vol), t(v))
    g.set_bc_ground_only()
    rng = np.random.default_rng(5)
    gx = t(rng.normal(0, 1, (len(x), 3)).astype(np.float32))
    gc = t((rng.normal(0, 1, len(x) * 6) * 1e3).astype(np.float32))
    for s in range(NSUB):
        g.forward(DT, s)
    g.postprocess_forward()
    keys = [(k, None) for k in ("glogE", "gy", "gmu", "glam")] + \
           [(k, lvl) for k in ("gx", "gv", "gF", "gC") for lvl in (0, 7, NSUB - 1)]
    runs = []
    for drop in (False, True):
        if drop:
            g.mu_lam()
        g.clear_grads(); g.set_grads(gx, gc); g.postprocess_backward()
        for s in reversed(range(NSUB)):
            g.backward(DT, s)
        r = {(k, l): (g.get(k) if l is None else g.get(k, l)).cpu().numpy() for k, l in keys}
        r.update({w: g.get_grid(w).cpu().numpy() for w in ("mass", "v_in", "v_out")})  # level 0's
        runs.append(r)
    for key in runs[0]:
        np.testing.assert_array_equal(runs[0][key], runs[1][key], err_msg=str(key))
    # x changed at level 4 after the forward pass: backward(4) recomputes level 4's grid
    m_before = g.get_grid("mass").cpu().numpy()
    g.set("x", g.get("x", 4) + 2e-2, 4)
    g.clear_grads(); g.set_grads(gx, gc)
    g.backward(DT, 4)
    assert not np.array_equal(g.get_grid("mass").cpu().numpy(), m_before)


def test_fit_ragged_and_tiny(dev):
    """n not a multiple of 256, a handful of particles, a small grid."""
    import oracle as O
    from gsmpm.fit import FitSimulator
    for n, ng in ((37, 16), (1000 + 3, 24)):
        rng = np.random.default_rng(n)
        x = rng.uniform(0.7, 1.3, (n, 3)).astype(np.float32)
        cov = np.tile(np.array([1e-4, 0, 0, 1e-4, 0, 1e-4], np.float32), (n, 1))
        v = rng.normal(0, 0.3, (n, 3)).astype(np.float32)
        vol = O.particle_volume(x, ng, EXT)
        o = O.OracleDiff(x, cov, vol, n_grid=ng, grid_extent=EXT, gravity=GRAV, init_v=v, levels=6,
                         ground_only=True, **MAT)
        g = FitSimulator(n, n_grid=ng, grid_extent=EXT, levels=6, gravity=GRAV, **MAT)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        g.set_particles(t(x), t(cov), t(vol), t(v))
        g.set_bc_ground_only()
        for s in range(5):
            o.p2g2p_forward(1e-3, s)
            g.forward(1e-3, s)
        assert rel_err(g.get("x", 5).cpu().numpy(), o.x[5]) < 1e-4
        assert rel_err(g.get("F", 5).cpu().numpy(), o.F[5]) < 1e-4


def test_fit_binning_paths(dev):
    """The binning bookkeeping (csrc/fit.hip bin_level): a grid of more than
    8,192 tiles (k_scan + k_place instead of the fused k_scanplace), a level
    stepped forward twice (its counters were already consumed), and x set at a
    level between forward steps (counts taken again by k_count); the oracle
    runs the same call sequence."""
    import oracle as O
    from gsmpm.fit import FitSimulator
    # 176: 22^3 = 10,648 tiles (dense enough blob, dt under the CFL limit of dx = 0.011)
    for n, ng, lo, hi, dt in ((3000, 24, 0.8, 1.2, 1e-3), (3000, 176, 0.95, 1.05, 1e-4)):
        rng = np.random.default_rng(ng)
        x = rng.uniform(lo, hi, (n, 3)).astype(np.float32)
        cov = np.tile(np.array([1e-4, 0, 0, 1e-4, 0, 1e-4], np.float32), (n, 1))
        v = rng.normal(0, 0.05, (n, 3)).astype(np.float32)
        vol = O.particle_volume(x, ng, EXT)
        o = O.OracleDiff(x, cov, vol, n_grid=ng, grid_extent=EXT, gravity=GRAV, init_v=v, levels=8,
                         ground_only=True, **MAT)
        g = FitSimulator(n, n_grid=ng, grid_extent=EXT, levels=8, gravity=GRAV, **MAT)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        g.set_particles(t(x), t(cov), t(vol), t(v))
        g.set_bc_ground_only()
        seq = [0, 1, 2, 2, 3]  # level 2 twice
        for s in seq:
            o.p2g2p_forward(dt, s)
            g.forward(dt, s)
        assert rel_err(g.get("x", 4).cpu().numpy(), o.x[4]) < 1e-4, ng
        # x of level 4 moved between forward steps
        xs = o.x[4] + np.float32(1e-3)
        o.x[4][:] = xs
        g.set("x", t(xs), 4)
        for s in (4, 5, 6):
            o.p2g2p_forward(dt, s)
            g.forward(dt, s)
        assert rel_err(g.get("x", 7).cpu().numpy(), o.x[7]) < 1e-4, ng
        assert rel_err(g.get("F", 7).cpu().numpy(), o.F[7]) < 1e-4, ng


def test_fit_dropin_extra_py_loop(dev):
    """The extra.py train loop (extra.py:189-241) through the drop-in API."""
    import oracle as O
    from arguments import MPMParams
    from argparse import ArgumentParser
    from mpm_solver.solver import MPM_Simulator
    x, cov, v = _scene(2000, 3)
    vol = O.particle_volume(x, NG, EXT)
    parser = ArgumentParser()
    group = MPMParams(parser, {"n_grid": NG, "grid_extent": EXT, "E": MAT["E"], "nu": MAT["nu"],
                               "density": MAT["density"], "gravity": list(GRAV)})
    args = group.extract(parser.parse_args([]))
    args.fitting = True
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    sim = MPM_Simulator(t(x), t(cov), t(vol), args, init_v=t(v))
    sim.set_bc_ground_only()
    o = O.OracleDiff(x, cov, vol, n_grid=NG, grid_extent=EXT, gravity=GRAV, init_v=v, ground_only=True, **MAT)
    for it in range(2):
        for s in range(NSUB):
            sim.p2g2p(DT, s)   # extra.py:207's call, routed to p2g2p_forward
            o.p2g2p_forward(DT, s)
        sim.postprocess_forward()
        o.postprocess_forward()
        means = sim.mpm_state.particle_xyz.to_torch()[30]
        covs = sim.mpm_state.particle_cov.to_torch()
        assert means.shape == (2000, 3) and covs.shape == (2000 * 6,)
        assert rel_err(means.cpu().numpy(), o.x[30]) < 1e-4
        gx = (means - means.mean(0)).detach()
        gc = torch.ones_like(covs) * 10
        sim.clear_grads()
        o.clear_grads()
        sim.mpm_state.set_grads(gx, gc)
        o.set_grads(gx.cpu().numpy(), gc.cpu().numpy())
        sim.postprocess_backward()
        o.postprocess_backward()
        for s in reversed(range(NSUB)):
            sim.p2g2p_backward(DT, s)
            o.p2g2p_backward(DT, s)
        _adjoint_close(sim.mpm_model.logE.grad.to_torch().cpu().numpy(), o.glogE, ("glogE", it), it > 0)
        _adjoint_close(sim.mpm_model.y.grad.to_torch().cpu().numpy(), o.gy, ("gy", it), it > 0)
        sim.learn()
        o.learn()
        sim.mpm_state.cycle_init()
        o.cycle_init()
    # learn() clips each adjoint to +-1: a particle whose (ill-conditioned, see
    # _adjoint_close) adjoint changes sign moves by 2 x 0.8; allow 1 % of them
    logE = sim.mpm_model.logE.to_torch().cpu().numpy()
    assert (np.abs(logE - o.logE) > 1e-4).mean() <= 1e-2
    E_opt = 10 ** sim.mpm_model.logE.to_torch().mean().item()
    assert abs(np.log10(E_opt) - o.logE.astype(np.float64).mean()) < 1.6 * 1e-2
    with pytest.raises(TypeError):
        sim.postprocess()



def test_extra_py_synthetic_training_loop(dev, tmp_path):
    """extra.py's SystemIndentifier end to end on a synthetic torus (config E shape,
    smaller): differentiable MPM + rasterizer forward/backward + learn, 1 iteration
    of 20 frames.  Checks the loop runs, losses stay finite, and the physical
    parameters move under the gradients."""
    import math as _m
    from argparse import ArgumentParser
    import extra
    from arguments import MPMParams
    parser = ArgumentParser()
    sim_args = MPMParams(parser)
    sim_args.fitting = True
    sim_args.E, sim_args.nu = 3e5, 0.3

    class A:
        iters = 1
    si = extra.SystemIndentifier("", "", sim_args, A(), synthetic=dict(n=3000, E_true=1e5, size=64, n_cams=2))
    assert len(si.cameras_all) == extra.train_num_frames + extra.test_num_frames
    gt0, gt10 = si.cameras_all[0][0].original_image, si.cameras_all[10][0].original_image
    assert float((gt0 - gt10).abs().max()) > 0.05  # the torus moved between frames
    hist = si.train(log=lambda *_: None)
    assert len(hist) == extra.train_num_frames
    assert all(_m.isfinite(h[2]) and _m.isfinite(h[3]) and _m.isfinite(h[4]) for h in hist)
    assert hist[-1][3] != 3e5  # learn() moved E
