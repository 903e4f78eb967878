"""MPM parity: HIP path (through the drop-in MPM_Simulator / C-ABI) vs the CPU oracle.

Tolerance (BASELINE north_star): 1e-4 relative on particle positions and
covariances, err = max|gpu - oracle| / max|oracle| per field.  Float atomics
make the HIP sum order differ from the oracle's serial order, so other fields
are checked at the same scale-relative bound.
"""
import numpy as np
import pytest

from conftest import rel_err
from scenarios import build_oracle_sim, lego_problem, oracle_run

pytestmark = pytest.mark.gpu

# both substep pipelines: the fused G2P2G one (default) and the per-phase one
# (slabs, KEEP_GRID); the fused one re-bins every 10 substeps by default, the
# "fused_r1" case every substep, "fused_r50" almost never (margin escapes)
PIPES = ["fused", "phased"]


def _pipe_over(pipe):
    return {"phased": pipe == "phased"}


def _set_rebin(s, pipe):
    if pipe.startswith("fused_r"):
        s._sim.set_rebin_interval(int(pipe[len("fused_r"):]))

TOL = 1e-4
# Every field of a stress-free run (jelly as written) is held to the
# north_star 1e-4 (measured: v, C <= 3e-6).  With a stiff stress model v and C
# (C = sum v_i dpos^T w 4/dx^2) amplify the summation-order difference of the
# grid sums by ~1/dx, so stress-bearing runs (FCR jelly, metal, sand, foam) get
# their own bound for those two (measured on these 48^3 scenes: v <= 1.8e-3,
# C <= 3.2e-3); x / F_trial / cov carry 1e-4 everywhere.
TOL_DERIVED = {"v": 2e-3, "C": 5e-3}


# Two reference-algorithm conditioning limits (documented in DESIGN.md §Parity):
#  * metal yield_stress grows by 2*mu*xi*dgamma with dgamma from log(sigma),
#    sigma ~ 1 + 1e-4: f32 log near 1 carries ~1e-3 relative noise;
#  * foam's F = U * diag * V^T is element-wise (constitutive_models.py:256, F13):
#    it depends on the SVD basis itself, which is ill-defined for F ~ I, so
#    F_trial (not x) inherits the float-atomic noise amplified.
MATERIAL_TOL = {"metal": {"yield": 5e-3}, "foam": {"F_trial": 2e-2}}


def _compare(s, ref, fields=("x", "v", "C", "F_trial"), tol=TOL, extra=None, stress=False):
    st = s.mpm_state
    got = {
        "x": st.particle_xyz.to_torch().cpu().numpy(),
        "v": st.particle_vel.to_torch().cpu().numpy(),
        "C": st.particle_C.to_torch().cpu().numpy().reshape(-1, 9),
        "F_trial": st.particle_F_trial.to_torch().cpu().numpy().reshape(-1, 9),
    }
    exp = {"x": ref.x, "v": ref.v, "C": ref.C, "F_trial": ref.F_trial}
    errs = {k: rel_err(got[k], exp[k]) for k in fields}
    if __import__('os').environ.get('GSMPM_PRINT_ERRS'):
        print('ERRS', __import__('os').environ.get('PYTEST_CURRENT_TEST', '').split(' ')[0], {k: f'{e:.2e}' for k, e in errs.items()})
    for k, e in errs.items():
        bound = (extra or {}).get(k, TOL_DERIVED.get(k, tol) if stress else tol)
        assert e < bound, f"{k}: rel err {e:.3e} > {bound} (all: {errs})"
    return errs


@pytest.mark.parametrize("pipe", PIPES + ["fused_r1", "fused_r50"])
def test_lego_config_A_parity(dev, pipe):
    """configs[0]: lego.json jelly (as written), 5k Gaussians, 64^3, 50 substeps."""
    from gpu_helpers import dropin_sim
    prob = lego_problem(5000, 64)
    ref, imps, ops = build_oracle_sim(prob)
    dt = prob["cfg"]["substep_dt"]
    s, args = dropin_sim(prob, dev, **_pipe_over(pipe))
    _set_rebin(s, pipe)
    assert s._sim.pipeline == ("phased" if pipe == "phased" else "fused")
    t = oracle_run(ref, imps, ops, dt, 50)
    for _ in range(50):
        s.p2g2p(dt)
    assert abs(s.time - t) == 0.0
    _compare(s, ref)
    s.postprocess()
    ref.postprocess()
    cov = s.mpm_state.particle_cov.to_torch().cpu().numpy().reshape(-1, 6)
    R = s.mpm_state.particle_R.to_torch().cpu().numpy().reshape(-1, 9)
    assert rel_err(cov, ref.cov) < TOL
    assert rel_err(R, ref.R) < TOL


@pytest.mark.parametrize("pipe", PIPES)
@pytest.mark.parametrize("material,quirk", [("metal", True), ("sand", True), ("foam", True), ("jelly", False)])
def test_materials_parity(dev, material, quirk, pipe):
    """Return maps + SVD stress (metal/sand/foam) and FCR jelly (F3 fixed), 30 substeps."""
    from gpu_helpers import dropin_sim
    prob = lego_problem(4000, 48)
    ref, imps, ops = build_oracle_sim(prob, material=material, jelly_quirk=quirk)
    dt = prob["cfg"]["substep_dt"]
    s, _ = dropin_sim(prob, dev, material=material, jelly_fcr=not quirk, **_pipe_over(pipe))
    oracle_run(ref, imps, ops, dt, 30)
    for _ in range(30):
        s.p2g2p(dt)
    extra = MATERIAL_TOL.get(material, {})
    _compare(s, ref, extra=extra, stress=True)  # every case here carries stress
    if material == "metal":
        y = s.mpm_model.yield_stress.to_torch().cpu().numpy()
        assert rel_err(y, ref.yield_stress) < extra["yield"]


@pytest.mark.parametrize("pipe", PIPES)
def test_impulse_window(dev, pipe):
    """ImpulseBC active on a host-decided window mid-run (boundary_conditions.py:41-45)."""
    from gpu_helpers import dropin_sim
    prob = lego_problem(3000, 48)
    for d in prob["cfg"]["boundary_conditions"]:
        if d["type"] == "impulse":
            d["start_time"] = 0.0015
            d["force"] = [-80.0, 0.0, 30.0]
    ref, imps, ops = build_oracle_sim(prob)
    dt = prob["cfg"]["substep_dt"]
    s, _ = dropin_sim(prob, dev, **_pipe_over(pipe))
    oracle_run(ref, imps, ops, dt, 40)
    for _ in range(40):
        s.p2g2p(dt)
    _compare(s, ref)


@pytest.mark.parametrize("pipe", PIPES)
def test_eager_equals_graph(dev, pipe):
    """Per-substep launches and the cached hipGraph replay give identical state,
    over four step calls with the same key: the graph's two instances
    (GSMPM_GRAPH_COPIES, launched in turn) both run."""
    import torch
    from gsmpm.sim import Simulator
    prob = lego_problem(3000, 48)
    cfg = prob["cfg"]
    outs = []
    for graph in (False, True):
        sim = Simulator(len(prob["x"]), n_grid=48, material="metal", E=cfg["E"], nu=cfg["nu"],
                        density=cfg["density"], gravity=cfg["gravity"], use_graph=graph, phased=pipe == "phased")
        t = lambda a: torch.from_numpy(a).to(dev)
        sim.set_particles(t(prob["x"]), t(prob["cov"]), t(prob["vol"]))
        b = sim.add_fixed_cube([1.0, 1.2, 0.5], [1.0, 0.8, 0.3])
        sim.add_plane_collider([0, 0, 0.4], [0, 0, 1])
        for _ in range(4):
            sim.step(1e-4, [1 << b] * 20)
        outs.append(sim.get("x").cpu().numpy())
    assert rel_err(outs[0], outs[1]) < 1e-6


@pytest.mark.parametrize("pipe", PIPES)
def test_resort_keeps_caller_order(dev, pipe):
    """Device Morton re-sorts between substeps only permute storage: fields read
    back in caller order and still match the oracle."""
    from gpu_helpers import dropin_sim
    prob = lego_problem(3000, 48)
    ref, imps, ops = build_oracle_sim(prob)
    dt = prob["cfg"]["substep_dt"]
    s, _ = dropin_sim(prob, dev, **_pipe_over(pipe))
    s._sim.resort(interval=7)
    oracle_run(ref, imps, ops, dt, 60)
    for k in range(60):
        s.p2g2p(dt)
        if k % 9 == 0:
            s.flush()
    _compare(s, ref)
    s.postprocess()
    ref.postprocess()
    cov = s.mpm_state.particle_cov.to_torch().cpu().numpy().reshape(-1, 6)
    assert rel_err(cov, ref.cov) < TOL


@pytest.mark.parametrize("pipe", PIPES)
def test_large_grid_binning_path(dev, pipe):
    """> 8192 tiles (176^3 -> 10,648 8^3 tiles, 10,672 8x8x7 tiles) takes the
    multi-workgroup scan + scatter binning instead of the fused one; same parity bar."""
    from gpu_helpers import dropin_sim
    prob = lego_problem(3000, 176)
    ref, imps, ops = build_oracle_sim(prob)
    dt = prob["cfg"]["substep_dt"]
    s, _ = dropin_sim(prob, dev, **_pipe_over(pipe))
    oracle_run(ref, imps, ops, dt, 12)
    for _ in range(12):
        s.p2g2p(dt)
    _compare(s, ref)


@pytest.mark.parametrize("material", ["jelly", "metal"])
def test_fused_margin_escapes(dev, material):
    """Fused pipeline with bins kept for 50 substeps while a swirl moves
    particles ~0.3 cells per substep (9 cells over the run): most particles
    leave their chunk's one-cell window margin and take the global gather /
    float-atomic scatter path, and every grid update sweeps all tiles.  Same
    parity bar as the binned path."""
    import torch
    import oracle as O
    from gsmpm.sim import Simulator
    prob = lego_problem(3000, 48)
    cfg = prob["cfg"]
    x = prob["x"].astype(np.float32)
    c = x.mean(0)
    r = x - c
    v0 = (200.0 * np.stack([-r[:, 1], r[:, 0], 0.3 * r[:, 0]], 1)).astype(np.float32)
    dt = 1e-4
    dx = cfg["grid_extent"] / 48
    assert np.abs(v0).max() * dt * 30 > 2 * dx  # beyond the margin within the run
    kw = dict(n_grid=48, grid_extent=cfg["grid_extent"], material=material, E=cfg["E"], nu=cfg["nu"],
              density=cfg["density"], gravity=cfg["gravity"])
    ref = O.OracleMPM(x, prob["cov"], prob["vol"], v=v0, **kw)
    ref.add_collider([0.0, 0.0, 0.4], [0.0, 0.0, 1.0], 0.0)
    sim = Simulator(len(x), **kw)
    sim.set_rebin_interval(50)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    sim.set_particles(t(x), t(prob["cov"]), t(prob["vol"]), t(v0))
    sim.add_plane_collider([0.0, 0.0, 0.4], [0.0, 0.0, 1.0], 0.0)
    assert sim.pipeline == "fused"
    for _ in range(30):
        ref.substep(dt, [], [1])
    sim.step(dt, [0xFFFFFFFF] * 30)
    got = {"x": sim.get("x"), "v": sim.get("v"), "C": sim.get("C"), "F_trial": sim.get("F_trial")}
    exp = {"x": ref.x, "v": ref.v, "C": ref.C, "F_trial": ref.F_trial}
    for k in got:
        e = rel_err(got[k].cpu().numpy().reshape(exp[k].shape), exp[k])
        assert e < TOL_DERIVED.get(k, TOL), (k, e)


@pytest.mark.parametrize("pipe", PIPES)
def test_heterogeneous_masses(dev, pipe):
    """The round-4 verdict's reference-semantics gap: one chunk whose masses
    span more than 2^52.  A particle 1e-17 as heavy as the 200 others of its
    tile (one chunk) has a contribution below the chunk's fixed-point
    resolution, so the nodes only its stencil reaches sum to mass 0 -- where
    the reference's grid_m (2e-21) is <= 1e-15 and v_out stays at the reset
    value 0 (utils.py:177-183).  The heavy blob moves away (+x, 3 m/s) from
    the light particle, whose stencil shares nodes with the blob's trailing
    edge at first: those nodes had v_out ~ 3 while the blob covered them.  A
    grid update that skipped every massless node left that stale 3 for the
    light particle to keep gathering (it would follow the blob); one that
    stores every node inside a stencil box gives it the reference's 0."""
    import torch
    import oracle as O
    from gsmpm.sim import Simulator
    rng = np.random.default_rng(7)
    ng, ext, dt, steps = 32, 2.0, 1e-3, 60
    nb = 200
    blob = np.stack([rng.uniform(0.80, 0.95, nb), rng.uniform(0.85, 1.0, nb), rng.uniform(0.60, 0.75, nb)], 1)
    light = np.array([[0.66, 0.92, 0.67]])
    x = np.concatenate([blob, light]).astype(np.float32)
    v = np.zeros_like(x)
    v[:nb, 0] = 3.0
    cov = np.tile(np.array([1e-4, 0, 0, 1e-4, 0, 1e-4], np.float32), (len(x), 1))
    vol = O.particle_volume(x, ng, ext).astype(np.float32)
    vol[nb] = vol[:nb].mean() * 1e-17
    kw = dict(n_grid=ng, grid_extent=ext, material="jelly", E=2e4, nu=0.3, density=200.0, gravity=(0.0, 0.0, 0.0))
    ref = O.OracleMPM(x, cov, vol, v=v, **kw)  # jelly as written, as Simulator runs it
    sim = Simulator(len(x), phased=pipe == "phased", **kw)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    sim.set_particles(t(x), t(cov), t(vol), t(v))
    for _ in range(steps):
        ref.substep(dt, [], [])
    sim.step(dt, [0] * steps)
    gx = sim.get("x").cpu().numpy().reshape(-1, 3)
    gv = sim.get("v").cpu().numpy().reshape(-1, 3)
    # the blob really left the light particle's stencil, so some of its nodes
    # went from heavy to (reference) massless during the run
    assert ref.x[:nb, 0].min() - ref.x[nb, 0] > 3 * ext / ng
    vmax = np.abs(ref.v).max()
    assert np.abs(gv[nb] - ref.v[nb]).max() < 1e-4 * vmax, (gv[nb], ref.v[nb])
    assert np.abs(gx[nb] - ref.x[nb]).max() < 1e-4 * np.abs(ref.x).max(), (gx[nb], ref.x[nb])
    assert rel_err(gx, ref.x) < TOL and rel_err(gv, ref.v) < TOL


@pytest.mark.parametrize("pipe", PIPES)
def test_nonfinite_position_reported(dev, pipe):
    """SURVEY 5's per-frame NaN / Inf check on x: a non-finite particle
    position -- given at set_particles, or produced during a step -- is
    reported by check_finite() and by the next step() call (GSMPM_ESTATE, a
    RuntimeError), and a fresh state clears it."""
    import torch
    import oracle as O
    from gsmpm.sim import Simulator
    rng = np.random.default_rng(0)
    n, ng, dt = 2000, 32, 1e-4
    x = rng.uniform(0.7, 1.3, size=(n, 3)).astype(np.float32)
    cov = np.tile(np.array([1e-4, 0, 0, 1e-4, 0, 1e-4], np.float32), (n, 1))
    vol = O.particle_volume(x, ng, 2.0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    sim = Simulator(n, n_grid=ng, grid_extent=2.0, material="metal", E=2e5, nu=0.3, density=200.0,
                    phased=pipe == "phased")
    sim.set_particles(t(x), t(cov), t(vol))
    sim.step(dt, [0] * 10)
    sim.check_finite()  # a finite state raises nothing
    # NaN given at set_particles
    xb = x.copy()
    xb[17, 1] = np.nan
    sim.set_particles(t(xb), t(cov), t(vol))
    sim.step(dt, [0] * 10)
    with pytest.raises(RuntimeError, match="non-finite"):
        sim.check_finite()
    with pytest.raises(RuntimeError, match="non-finite"):
        sim.step(dt, [0] * 10)
    # a fresh finite state clears it
    sim.set_particles(t(x), t(cov), t(vol))
    sim.step(dt, [0] * 10)
    sim.check_finite()
    # Inf produced during a step: one particle's velocity is infinite
    vb = sim.get("v").clone()
    vb.view(-1, 3)[5, 0] = float("inf")
    sim.set("v", vb)
    sim.step(dt, [0] * 10)
    with pytest.raises(RuntimeError, match="non-finite"):
        sim.check_finite(clear=True)
    sim.check_finite()  # cleared


def test_particles_binned_outside_the_grid(dev):
    """Particles outside the grid (base cell beyond n_grid: every stencil node
    out of bounds) are binned into the fused pipeline's "outside" chunk and
    take the bounds-checked global path: they gather nothing, so after a step
    their v and C are exactly 0 and x is unchanged (the oracle's bounds-checked
    reading of the reference's out-of-range region).  60 of them start with
    random velocities beside 1,500 particles inside; after 45 substeps (two
    re-binnings, and launches that reuse the lane order of the last P2G on the
    same bins) every field matches the oracle.  Round 4 left the outside
    chunk's lane order unwritten, so the next launch's lanes took stale rows
    (the same particle several times -- the others kept their initial v -- or
    rows past the live ones: an illegal address in a GPU suite run)."""
    import torch
    import oracle as O
    from gsmpm.sim import Simulator
    rng = np.random.default_rng(5)
    ng, ext, dt, steps = 32, 2.0, 2e-4, 45
    n_in, n_out = 1500, 60
    xin = rng.uniform(0.3, 0.9, size=(n_in, 3))
    xout = np.stack([rng.uniform(2.05, 2.3, n_out), rng.uniform(0.4, 0.8, n_out), rng.uniform(0.4, 0.8, n_out)], 1)
    x = np.concatenate([xin, xout]).astype(np.float32)
    v = rng.normal(0, 0.5, size=x.shape).astype(np.float32)
    cov = np.tile(np.array([1e-4, 0, 0, 1e-4, 0, 1e-4], np.float32), (len(x), 1))
    vol = O.particle_volume(x, ng, ext)
    kw = dict(n_grid=ng, grid_extent=ext, material="jelly", E=2e4, nu=0.3, density=200.0, gravity=(0.0, -9.8, 0.0))
    ref = O.OracleMPM(x, cov, vol, v=v, **kw)  # jelly as written, as Simulator runs it
    sim = Simulator(len(x), **kw)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    sim.set_particles(t(x), t(cov), t(vol), t(v))
    for _ in range(steps):
        ref.substep(dt, [], [])
    sim.step(dt, [0] * steps)
    got = {k: sim.get(k).cpu().numpy().reshape(getattr(ref, k).shape) for k in ("x", "v", "C", "F_trial")}
    assert np.isfinite(ref.x).all() and np.abs(ref.v[n_in:]).max() == 0.0  # the oracle's reading
    assert np.array_equal(got["x"][n_in:], x[n_in:])
    assert np.abs(got["v"][n_in:]).max() == 0.0 and np.abs(got["C"][n_in:]).max() == 0.0
    for k, g in got.items():
        e = rel_err(g, getattr(ref, k))
        assert e < TOL, (k, e)
