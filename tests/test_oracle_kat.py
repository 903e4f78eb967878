"""Known-answer tests that pin the CPU oracle.

The reference has no tests, fixtures or golden vectors and its Taichi kernels
cannot run here, so the oracle is pinned by first-principles
properties of the algorithm it restates.
"""
import math

import numpy as np
import pytest

import oracle as O
from conftest import rel_err


def _sim(x, v=None, n_grid=32, material="jelly", gravity=(0.0, 0.0, 0.0), vol=None, **kw):
    x = np.asarray(x, np.float32)
    n = len(x)
    cov = np.tile(np.array([1e-4, 0, 0, 1e-4, 0, 1e-4], np.float32), (n, 1))
    vol = np.full(n, 1e-4, np.float32) if vol is None else vol
    return O.OracleMPM(x, cov, vol, n_grid=n_grid, grid_extent=2.0, material=material, E=2e5, nu=0.3,
                       density=200.0, gravity=gravity, v=v, **kw)


# ---------------------------------------------------------------- 2f: SVD --
def test_svd_properties():
    rng = np.random.default_rng(0)
    for t in range(3000):
        A = (np.eye(3) + 0.4 * rng.standard_normal((3, 3))).astype(np.float32)
        if t % 3 == 0:
            A = rng.standard_normal((3, 3)).astype(np.float32)
        if t % 7 == 0:
            A[:, 2] = -A[:, 2]  # inverted
        U, s, V = O.svd3(A)
        assert np.abs(U @ np.diag(s) @ V.T - A).max() < 2e-5 * max(1.0, np.abs(A).max())
        assert abs(np.linalg.det(U) - 1) < 1e-4 and abs(np.linalg.det(V) - 1) < 1e-4
        assert np.abs(U.T @ U - np.eye(3)).max() < 1e-5
        assert s[0] >= s[1] - 1e-5 and s[1] >= abs(s[2]) - 1e-5 and s[1] >= 0
        assert np.sign(s[2]) == np.sign(np.linalg.det(A)) or abs(s[2]) < 1e-6
        ref = np.linalg.svd(A.astype(np.float64), compute_uv=False)
        assert np.allclose(np.abs(s), ref, rtol=1e-4, atol=1e-5)


def test_svd_identity_and_diagonal():
    U, s, V = O.svd3(np.eye(3))
    assert np.allclose(s, 1) and np.allclose(U @ V.T, np.eye(3), atol=1e-6)
    D = np.diag([0.5, 3.0, 2.0]).astype(np.float32)
    U, s, V = O.svd3(D)
    assert np.allclose(s, [3.0, 2.0, 0.5], atol=1e-5)


# --------------------------------------------------- 2a/2b: P2G conservation --
def test_p2g_mass_and_momentum_conservation():
    rng = np.random.default_rng(1)
    n = 500
    x = rng.uniform(0.6, 1.4, size=(n, 3)).astype(np.float32)
    v = rng.normal(0, 1, size=(n, 3)).astype(np.float32)
    s = _sim(x, v)
    s.C[:] = rng.normal(0, 0.5, size=(n, 9)).astype(np.float32)
    O.lib().om_p2g(O.ctypes.byref(s._st), O.ctypes.c_float(1e-4))
    assert rel_err(s.gm.sum(), s.mass.sum()) < 1e-5
    # APIC: sum_i w (v + C (x_i - x_p)) = v because sum_i w (x_i - x_p) = 0 (quadratic B-spline)
    mom = (s.mass[:, None] * v).sum(0)
    assert np.abs(s.gv_in.sum(0) - mom).max() < 1e-4 * np.abs(mom).max() + 1e-6


# ------------------------------------------------ 2c: affine reproduction --
def test_g2p_reproduces_affine_field():
    n_grid = 32
    s = _sim(np.random.default_rng(2).uniform(0.7, 1.3, size=(50, 3)), n_grid=n_grid)
    A = np.array([[0.1, -0.2, 0.05], [0.3, 0.0, -0.1], [0.02, 0.04, -0.3]], np.float32)
    v0 = np.array([0.5, -0.25, 1.0], np.float32)
    dx = 2.0 / n_grid
    idx = np.stack(np.meshgrid(*[np.arange(n_grid)] * 3, indexing="ij"), -1).reshape(-1, 3) * dx
    s.gv_out[:] = (v0 + idx @ A.T).astype(np.float32)
    x0 = s.x.copy()
    O.lib().om_g2p(O.ctypes.byref(s._st), O.ctypes.c_float(1e-3))
    assert np.abs(s.v - (v0 + x0 @ A.T)).max() < 1e-5
    assert np.abs(s.C.reshape(-1, 3, 3) - A).max() < 1e-4     # C = A (APIC, D^-1 = 4/dx^2)
    dv = s.F_trial.reshape(-1, 3, 3)                          # F_trial = (I + dt grad v) I
    assert np.abs(dv - (np.eye(3) + 1e-3 * A)).max() < 1e-6


# ------------------------------------------------------ 2d: free fall --
def test_free_fall():
    g = (0.0, 0.0, -9.0)
    x = np.random.default_rng(3).uniform(0.8, 1.2, size=(200, 3))
    s = _sim(x, gravity=g)
    dt, steps = 1e-3, 20
    for _ in range(steps):
        s.substep(dt)
    assert np.abs(s.v - np.array(g) * dt * steps).max() < 1e-4
    # x_n = x_0 + dt * sum_k g k dt
    expect = np.asarray(x, np.float32) + np.array(g) * dt * dt * steps * (steps + 1) / 2
    assert np.abs(s.x - expect).max() < 1e-5


# --------------------------------------------------- 2e: postprocess at F = I --
def test_postprocess_identity():
    s = _sim(np.random.default_rng(4).uniform(0.8, 1.2, size=(20, 3)))
    s.init_cov[:] = np.random.default_rng(5).uniform(0, 1e-3, size=s.init_cov.shape).astype(np.float32)
    s.postprocess()
    assert np.array_equal(s.cov, s.init_cov)
    assert np.allclose(s.R.reshape(-1, 3, 3), np.eye(3), atol=1e-6)


def test_postprocess_rotation():
    s = _sim(np.full((1, 3), 1.0))
    th = 0.7
    Rz = np.array([[math.cos(th), -math.sin(th), 0], [math.sin(th), math.cos(th), 0], [0, 0, 1]], np.float32)
    F = Rz @ np.diag([1.2, 0.9, 1.0]).astype(np.float32)
    s.F_trial[0] = F.reshape(9)
    A = np.array([[2e-3, 1e-4, 0], [1e-4, 1e-3, 0], [0, 0, 5e-4]], np.float32)
    s.init_cov[0] = [A[0, 0], A[0, 1], A[0, 2], A[1, 1], A[1, 2], A[2, 2]]
    s.postprocess()
    C = F @ A @ F.T
    assert np.allclose(s.cov[0], [C[0, 0], C[0, 1], C[0, 2], C[1, 1], C[1, 2], C[2, 2]], rtol=1e-5, atol=1e-9)
    assert np.allclose(s.R[0].reshape(3, 3), Rz.T, atol=1e-5)  # particle_R = (U V^T)^T


# ---------------------------------------------------------- 2g: collider --
def test_collider_removes_inward_velocity():
    n_grid = 20
    s = _sim(np.full((1, 3), 1.0), n_grid=n_grid)
    s.add_collider([0.0, 0.0, 0.4], [0.0, 0.0, 2.0])  # normal normalised in f64
    rng = np.random.default_rng(6)
    s.gv_out[:] = rng.normal(0, 1, size=s.gv_out.shape).astype(np.float32)
    before = s.gv_out.copy().reshape(n_grid, n_grid, n_grid, 3)
    O.lib().om_grid_ops(O.ctypes.byref(s._st), 1, _ops(s), (O.ctypes.c_int32 * 1)(1))
    after = s.gv_out.reshape(n_grid, n_grid, n_grid, 3)
    dx = np.float32(2.0 / n_grid)
    for k in range(n_grid):
        z = np.float32(k) * dx - np.float32(0.4)
        b, a = before[:, :, k], after[:, :, k]
        if z < 0:
            exp = b.copy()
            exp[..., 2] = np.maximum(b[..., 2], 0.0)
            assert np.allclose(a, exp * np.float32(0.99), atol=1e-6)
        else:
            assert np.array_equal(a, b)


def _ops(s):
    ops = (O._GridOp * len(s.ops))()
    for i, (k, a, b, fr) in enumerate(s.ops):
        ops[i].kind, ops[i].friction = k, fr
        ops[i].a[:] = list(a)
        ops[i].b[:] = list(b)
    return ops


def test_fixed_cube_zeroes_nodes():
    n_grid = 16
    s = _sim(np.full((1, 3), 1.0), n_grid=n_grid)
    s.add_fixed_box([1.0, 1.2, 0.5], [1.0, 0.8, 0.3])
    s.gv_out[:] = 1.0
    O.lib().om_grid_ops(O.ctypes.byref(s._st), 1, _ops(s), (O.ctypes.c_int32 * 1)(1))
    g = s.gv_out.reshape(n_grid, n_grid, n_grid, 3)
    dx = np.float32(2.0 / n_grid)
    for i, j, k in [(8, 10, 4), (0, 10, 4), (8, 3, 4), (8, 10, 8)]:
        p = np.array([i, j, k], np.float32) * dx
        inside = np.all(np.abs(p - np.array([1.0, 1.2, 0.5], np.float32)) < np.array([1.0, 0.8, 0.3], np.float32))
        assert (g[i, j, k] == 0).all() == bool(inside)


# ------------------------------------------------------------ volumes --
def test_particle_volume():
    x = np.array([[0.01, 0.01, 0.01], [0.02, 0.03, 0.01], [1.0, 1.0, 1.0]], np.float32)
    vol = O.particle_volume(x, 10, 2.0)
    dx3 = np.float32(0.2) ** 3
    assert np.allclose(vol, [dx3 / 2, dx3 / 2, dx3])


# ----------------------------------------------------- 2h: rasterizer --
def _cam(W, H, t=0.5, dist=3.0):
    view = np.eye(4, dtype=np.float32)
    view[3, 2] = dist
    zn, zf = 0.01, 100.0
    P = np.zeros((4, 4), np.float32)
    P[0, 0] = P[1, 1] = 1 / t
    P[3, 2], P[2, 2], P[2, 3] = 1.0, zf / (zf - zn), -(zf * zn) / (zf - zn)
    return view, (view @ P.T).astype(np.float32)


def test_raster_single_gaussian_footprint():
    W = H = 64
    t = 0.5
    view, full = _cam(W, H, t)
    var = 2e-3
    means = np.zeros((1, 3), np.float32)
    c6 = np.array([[var, 0, 0, var, 0, var]], np.float32)
    col = np.array([[1.0, 0.5, 0.25]], np.float32)
    op = np.array([0.8], np.float32)
    img, radii, K, depth, _ = O.raster_forward(means, op, view, full, np.zeros(3), np.zeros(3), W, H, t, t,
                                               colors_precomp=col, cov3D_precomp=c6)
    f = W / (2 * t)
    s2 = var * (f / 3.0) ** 2 + 0.3                    # EWA at depth 3 + low-pass
    assert radii[0] == math.ceil(3 * math.sqrt(s2))
    assert depth[0] == pytest.approx(3.0)
    cx = cy = (W - 1) / 2                               # ndc 0 -> pixel (S-1)/2
    yy, xx = np.mgrid[0:H, 0:W]
    a = np.minimum(0.99, 0.8 * np.exp(-0.5 * ((xx - cx) ** 2 + (yy - cy) ** 2) / s2))
    a[a < 1 / 255] = 0
    for ch in range(3):
        assert np.abs(img[ch] - a * col[0, ch]).max() < 1e-5


def test_raster_zero_opacity_is_background():
    W, H = 40, 30
    view, full = _cam(W, H)
    bg = np.array([0.1, 0.2, 0.3], np.float32)
    img, radii, K, _, _ = O.raster_forward(np.zeros((3, 3), np.float32), np.zeros(3, np.float32), view, full,
                                           np.zeros(3), bg, W, H, 0.5, 0.5, colors_precomp=np.ones((3, 3)),
                                           cov3D_precomp=np.tile([[1e-2, 0, 0, 1e-2, 0, 1e-2]], (3, 1)))
    assert np.allclose(img, bg[:, None, None])


def test_raster_depth_order_composite():
    """Two coincident splats: front-to-back blend C = c1 a1 + c2 a2 (1 - a1)."""
    W = H = 32
    view, full = _cam(W, H)
    means = np.array([[0, 0, 0.5], [0, 0, -0.5]], np.float32)  # second is nearer (depth 2.5)
    c6 = np.tile(np.array([[1.0, 0, 0, 1.0, 0, 1.0]], np.float32), (2, 1))  # huge -> alpha ~ opacity at centre
    col = np.array([[1, 0, 0], [0, 1, 0]], np.float32)
    op = np.array([0.5, 0.6], np.float32)
    img, _, _, _, _ = O.raster_forward(means, op, view, full, np.zeros(3), np.zeros(3), W, H, 0.5, 0.5,
                                       colors_precomp=col, cov3D_precomp=c6)
    px = img[:, 15, 15]
    # pixel 15 is 0.5 px from centre: alpha = o * exp(-0.5*conic*d^2) ~ o (within 1e-4)
    assert px[1] == pytest.approx(0.6, abs=2e-3)
    assert px[0] == pytest.approx(0.5 * 0.4, abs=2e-3)


def test_fluid_return_mapping_known_answers():
    """fluid_return_mapping (constitutive_models.py:142-213), from its own
    algebra in float64: below the yield surface F_trial comes back unchanged;
    above it the returned F keeps F_trial's singular vectors and the volumetric
    log-strain, and its deviatoric Kirchhoff norm is s_trial - yield_value /
    plastic_factor.  The StVK stress it is paired with is symmetric."""
    rng = np.random.default_rng(11)
    n, mu, lam, dt, pv = 400, 8.3e4, 5.6e4, 1e-4, 0.008
    Q1 = np.linalg.qr(rng.standard_normal((n, 3, 3)))[0]
    Q2 = np.linalg.qr(rng.standard_normal((n, 3, 3)))[0]
    s = np.stack([rng.uniform(1.15, 1.3, n), rng.uniform(0.95, 1.05, n), rng.uniform(0.7, 0.85, n)], 1)
    F = (Q1 * s[:, None, :]) @ Q2.transpose(0, 2, 1)
    F *= np.sign(np.linalg.det(F))[:, None, None]
    F = F.astype(np.float32)
    # elastic: a yield stress far above any trial deviatoric stress
    Fo, tau = O.fluid_return_mapping(F, mu, lam, 1e9, dt, pv)
    assert np.array_equal(Fo, F)
    assert np.abs(tau - tau.transpose(0, 2, 1)).max() == 0.0
    # plastic
    yld = 0.005
    Fo, _ = O.fluid_return_mapping(F, mu, lam, yld, dt, pv)
    for i in range(n):
        U, sig, Vt = np.linalg.svd(F[i].astype(np.float64))
        eps = np.log(np.maximum(np.abs(sig), 0.01))
        tr = eps.sum()
        st = 2 * mu * (eps - tr / 3)
        stn = np.linalg.norm(st)
        y = stn - math.sqrt(2 / 3) * yld
        assert y > 0
        pf = 1 + pv / (2 * mu * (sig ** 2).sum() / 3 * dt)
        want_dev = stn - y / pf
        so = np.linalg.svd(Fo[i].astype(np.float64), compute_uv=False)
        eo = np.log(so)
        assert abs(eo.sum() - tr) < 2e-5
        assert abs(2 * mu * np.linalg.norm(eo - eo.sum() / 3) - want_dev) < 1e-4 * stn
        # same singular vectors: U^T Fo V is diagonal
        D = U.T @ Fo[i].astype(np.float64) @ Vt.T
        assert np.abs(D - np.diag(np.diag(D))).max() < 2e-5
