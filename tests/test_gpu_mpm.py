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
    """Per-substep launches and the cached hipGraph replay give identical state."""
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
