"""The folded grid update (fused.h FOLD, GSMPM_FOLD=1; an A/B form, off by
default since it measured slower): k_fused stages the
previous substep's grid update from the chunk windows itself, so a substep
is one launch instead of k_fused + k_grid_f (k_grid_f stays only after a
re-binning).  The staged node values are summed in k_grid_f's fixed order and
updated by the same node_update, so the folded pipeline must reproduce the
unfolded one (GSMPM_FOLD=0) BIT FOR BIT whenever no particle leaves its
chunk window -- the lego scene with a fixed cube and the ground collider, a
stress-bearing material, multi-chunk tiles, several step calls (graph
replays) -- as long as the run is deterministic: every tile one chunk, no
escapes.  Which chunk of a multi-chunk tile a particle lands in follows the
binning's atomics, and escaping scatters go through float atomics in both
forms (as the reference's Taichi atomics, utils.py:89-134), so there the two
forms agree to the run-to-run spread (multi-chunk tiles: 1e-6) or within
the parity bar (a swirl leaving the windows -- the slow path that evaluates
a particle's stencil nodes on demand -- and particles outside the grid,
where every launch escapes).  Parity with
the CPU oracle is the rest of the GPU suite, which runs the default
two-launch pipeline that these tests compare against.

Reference: the substep being folded is /root/reference/mpm_solver/solver.py:27-52
(p2g -> grid_normalization_and_gravity -> grid_postprocess -> g2p),
utils.py:89-134, 177-183, 218-282."""
import os

import numpy as np
import pytest

from scenarios import lego_problem

pytestmark = pytest.mark.gpu

FIELDS = ("x", "v", "C", "F_trial")


def _run(dev, fold, x, cov, vol, v=None, calls=1, nsub=100, rebin=None, bcs=True, impulse=0.0, **kw):
    import torch
    from gsmpm.sim import Simulator
    old = os.environ.get("GSMPM_FOLD")
    os.environ["GSMPM_FOLD"] = "1" if fold else "0"
    try:
        sim = Simulator(len(x), **kw)
    finally:
        if old is None:
            os.environ.pop("GSMPM_FOLD")
        else:
            os.environ["GSMPM_FOLD"] = old
    if rebin:
        sim.set_rebin_interval(rebin)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    sim.set_particles(t(x), t(cov), t(vol), None if v is None else t(v))
    masks = [0] * nsub
    if bcs:
        b0 = sim.add_fixed_cube([1.0, 1.0, 0.9], [0.2, 0.2, 0.1])
        sim.add_plane_collider([0.0, 0.0, 0.4], [0.0, 0.0, 1.0], 0.0)
        masks = [1 << b0] * nsub
        if impulse:
            b1 = sim.add_impulse([1.0, 1.0, 1.1], [0.3, 0.3, 0.2], [0.0, 0.0, -impulse], 1e-4)
            masks = [m | ((1 << b1) if s % 7 < 3 else 0) for s, m in enumerate(masks)]
    for _ in range(calls):
        sim.step(1e-4, masks)
    torch.cuda.synchronize()
    out = {k: sim.get(k).cpu().numpy() for k in FIELDS}
    out["stats"] = sim.debug_stats()
    out["escapes"] = sim.escapes()
    out["folded"] = sim.folded
    return out


def _assert_identical(a, b):
    assert a["folded"] and not b["folded"]
    assert a["escapes"] == b["escapes"] == 0, (a["escapes"], b["escapes"])
    for k in FIELDS:
        assert a[k].shape == b[k].shape
        d = np.abs(a[k].astype(np.float64) - b[k].astype(np.float64)).max()
        assert np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32)), f"{k}: max |diff| {d:.3e}"


# the GPU suite's parity bounds (tests/test_gpu_mpm.py): x, F_trial 1e-4; v, C (grid-velocity gradients,
# which a stress model or the float-atomic escape path amplifies by ~1/dx) 2e-3 / 5e-3
TOL = {"x": 1e-4, "F_trial": 1e-4, "v": 2e-3, "C": 5e-3}


def _assert_close(a, b, tol=None):
    """Within `tol` (default: the parity bounds) of each other, relative to the field's max."""
    assert a["folded"] and not b["folded"]
    for k in FIELDS:
        scale = max(float(np.abs(b[k]).max()), 1e-30)
        e = float(np.abs(a[k].astype(np.float64) - b[k]).max()) / scale
        bound = tol if tol is not None else TOL[k]
        assert e < bound, (k, e)


def _lego(n, ng, material="jelly", seed=0):
    prob = lego_problem(n, ng, seed=seed)
    cfg = prob["cfg"]
    kw = dict(n_grid=ng, grid_extent=cfg["grid_extent"], material=material, E=cfg["E"], nu=cfg["nu"],
              density=cfg["density"], gravity=cfg["gravity"])
    return prob["x"].astype(np.float32), prob["cov"], prob["vol"], kw


@pytest.mark.parametrize("material", ["jelly", "metal"])
def test_fold_bit_identical_lego(dev, material):
    """lego-like scene, 5k particles at 64^3 (every tile one chunk: the
    fixed-point window sums are exact whatever order the binning's atomics
    put the particles in, so both forms are deterministic), fixed cube +
    ground collider, 100 substeps (5 re-binnings), two step calls: folded ==
    unfolded, bit for bit."""
    x, cov, vol, kw = _lego(5_000, 64, material)
    a = _run(dev, True, x, cov, vol, calls=2, **kw)
    b = _run(dev, False, x, cov, vol, calls=2, **kw)
    assert np.abs(a["x"] - x).max() > 0  # it moved
    assert a["stats"]["max_per_tile"] <= 256 and b["stats"]["max_per_tile"] <= 256
    _assert_identical(a, b)


def test_fold_lego_20k_multi_chunk(dev):
    """20k particles at 64^3: some tiles hold several chunks, and which chunk a
    particle lands in follows the binning's atomics (the chunks' f32 window
    sums then differ in the last bits from run to run, in either form), so
    folded and unfolded agree to the run-to-run spread: 1e-5 of the field's
    max."""
    x, cov, vol, kw = _lego(20_000, 64)
    a = _run(dev, True, x, cov, vol, calls=2, **kw)
    b = _run(dev, False, x, cov, vol, calls=2, **kw)
    assert a["escapes"] == 0 and b["escapes"] == 0
    _assert_close(a, b, tol=1e-5)


def test_fold_escapes(dev):
    """A swirl (~0.3 cells a substep) with the bins kept for 50 substeps, 30
    substeps (test_gpu_mpm.py::test_fused_margin_escapes' scene, which holds
    the same run to the oracle): most particles leave their chunk window,
    scatter through the escape accumulators (three rotating buffers) and
    gather through the on-demand node evaluation; the unfolded pipeline
    sweeps every tile instead."""
    x, cov, vol, kw = _lego(3000, 48)
    c = x.mean(0)
    r = x - c
    v0 = (200.0 * np.stack([-r[:, 1], r[:, 0], 0.3 * r[:, 0]], 1)).astype(np.float32)
    a = _run(dev, True, x, cov, vol, v=v0, nsub=30, rebin=50, **kw)
    b = _run(dev, False, x, cov, vol, v=v0, nsub=30, rebin=50, **kw)
    assert a["escapes"] > 1000 and b["escapes"] > 1000
    _assert_close(a, b)


def test_fold_outside_grid(dev):
    """60 particles outside the grid (the "outside" chunk: every launch
    escapes) beside 1,500 inside, 45 substeps."""
    rng = np.random.default_rng(5)
    ng, ext = 32, 2.0
    xin = rng.uniform(0.3, 0.9, size=(1500, 3))
    xout = np.stack([rng.uniform(2.05, 2.3, 60), rng.uniform(0.4, 0.8, 60), rng.uniform(0.4, 0.8, 60)], 1)
    x = np.concatenate([xin, xout]).astype(np.float32)
    v = rng.normal(0, 0.5, size=x.shape).astype(np.float32)
    cov = np.tile(np.array([1e-4, 0, 0, 1e-4, 0, 1e-4], np.float32), (len(x), 1))
    vol = np.full(len(x), (ext / ng) ** 3 / 8, np.float32)
    kw = dict(n_grid=ng, grid_extent=ext, material="metal", E=2e4, nu=0.3, density=200.0, gravity=(0.0, -9.8, 0.0))
    a = _run(dev, True, x, cov, vol, v=v, nsub=45, bcs=False, **kw)
    b = _run(dev, False, x, cov, vol, v=v, nsub=45, bcs=False, **kw)
    assert a["escapes"] >= 60 * 45
    _assert_close(a, b)


def test_fold_multi_chunk_tiles(dev):
    """30k particles in a small box: tiles of several 256-particle chunks (the
    second and further chunks of a covering tile, summed after the first
    ones); within the run-to-run spread of the binning order (1e-5)."""
    rng = np.random.default_rng(3)
    ng, ext = 64, 2.0
    x = rng.uniform(0.8, 1.2, size=(30_000, 3)).astype(np.float32)
    cov = np.tile(np.array([1e-5, 0, 0, 1e-5, 0, 1e-5], np.float32), (len(x), 1))
    vol = np.full(len(x), 1e-7, np.float32)
    kw = dict(n_grid=ng, grid_extent=ext, material="jelly", E=2e4, nu=0.3, density=200.0, gravity=(0.0, 0.0, -9.8))
    a = _run(dev, True, x, cov, vol, nsub=40, **kw)
    b = _run(dev, False, x, cov, vol, nsub=40, **kw)
    assert a["stats"]["max_per_tile"] > 512  # third chunks too
    assert a["escapes"] == 0 and b["escapes"] == 0
    _assert_close(a, b, tol=1e-5)


def test_fold_profile_counts_grid_launches(dev):
    """The profile's kernel_ms[3] is the number of k_grid_f launches of the
    profiled substeps: one per re-binning when folded, one per substep
    otherwise (what bench.py divides k_grid_f's time by)."""
    import torch
    from gsmpm.sim import Simulator
    x, cov, vol, kw = _lego(5000, 48)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    got = {}
    old = os.environ.get("GSMPM_FOLD")
    for fold in (True, False):
        os.environ["GSMPM_FOLD"] = "1" if fold else "0"
        try:
            sim = Simulator(len(x), **kw)
        finally:
            if old is None:
                os.environ.pop("GSMPM_FOLD")
            else:
                os.environ["GSMPM_FOLD"] = old
        sim.set_particles(t(x), t(cov), t(vol))
        got[fold] = sim.profile(1e-4, [0] * 100)
    assert got[False][3] == 100
    assert 1 <= got[True][3] <= 10 and got[True][1] < got[False][1]
