"""Rasterizer backward oracle (oracle/raster_oracle.c or_backward) against
float64 autograd of the forward (tests/raster_torch_ref.py).

Upstream's backward (graphdeco-inria diff-gaussian-rasterization, not in the
reference) is restated, so this pins the restatement's adjoint to
its own forward: "parity unpinned" against upstream itself.  Scenes are small
(autograd runs a per-pixel Python loop).  Tolerance: 2e-3 of each output's
max magnitude (f32 oracle vs f64 reference).
"""
from __future__ import annotations

import math

import numpy as np
import pytest
import torch

from conftest import rel_err


def _camera(W, H, fovx, dist=3.0, yaw=0.3):
    fovy = 2 * math.atan(math.tan(fovx / 2) * H / W)
    c, s = math.cos(yaw), math.sin(yaw)
    w2c = np.eye(4)
    w2c[:3, :3] = [[c, 0, -s], [0, 1, 0], [s, 0, c]]
    w2c[:3, 3] = [0.1, -0.05, dist]
    zn, zf = 0.01, 100.0
    tx, ty = math.tan(fovx / 2), math.tan(fovy / 2)
    P = np.zeros((4, 4))
    P[0, 0], P[1, 1] = 1 / tx, 1 / ty
    P[3, 2], P[2, 2], P[2, 3] = 1.0, zf / (zf - zn), -(zf * zn) / (zf - zn)
    return (w2c.T.astype(np.float32), (P @ w2c).T.astype(np.float32),
            np.linalg.inv(w2c)[:3, 3].astype(np.float32), tx, ty)


def _scene(P, seed, wide=False):
    rng = np.random.default_rng(seed)
    means = np.stack([rng.uniform(-0.6, 0.6, P), rng.uniform(-0.6, 0.6, P), rng.uniform(-0.5, 0.5, P)],
                     1).astype(np.float32)
    A = rng.normal(0, 1, size=(P, 3, 3)) * 0.06
    A[::3] *= 2.5  # wide opaque ones: many pixels near their centre
    if wide:  # half of them beyond 1.3 x the fov, large enough to reach into the image
        k = P // 2
        means[:k, 0] = np.sign(rng.normal(size=k)) * rng.uniform(2.6, 3.0, k)
        A[:k] *= 5.0
    cov = A @ A.transpose(0, 2, 1) + np.eye(3) * 2e-3
    c6 = np.stack([cov[:, 0, 0], cov[:, 0, 1], cov[:, 0, 2], cov[:, 1, 1], cov[:, 1, 2], cov[:, 2, 2]],
                  1).astype(np.float32)
    opa = rng.uniform(0.2, 0.95, size=(P, 1)).astype(np.float32)
    opa[::3] = 0.999  # alpha = min(0.99, o G) clamps near their centres
    shs = rng.normal(0, 0.3, size=(P, 16, 3)).astype(np.float32)
    shs[:, 0] += 0.6
    scales = np.exp(rng.normal(-2.5, 0.3, (P, 3))).astype(np.float32)
    rots = rng.normal(0, 1, (P, 4)).astype(np.float32)
    rots /= np.linalg.norm(rots, axis=1, keepdims=True)
    return means, c6, opa, shs, scales, rots


def _compare(P, W, H, seed, D=3, use_sr=False, colors=False, bg=0.3, wide=False):
    import oracle as O
    from raster_torch_ref import forward
    means, c6, opa, shs, scales, rots = _scene(P, seed, wide)
    view, full, campos, tx, ty = _camera(W, H, 1.0)
    bgv = np.full(3, bg, np.float32)
    rng = np.random.default_rng(seed + 1)
    cols = rng.uniform(0, 1, (P, 3)).astype(np.float32)
    wgt = rng.normal(0, 1, (3, H, W)).astype(np.float32)
    kw = dict(colors_precomp=cols) if colors else dict(shs=shs, sh_degree=D)
    kw.update(dict(scales=scales, rotations=rots) if use_sr else dict(cov3D_precomp=c6))
    g = O.raster_backward(wgt, means, opa, view, full, campos, bgv, W, H, tx, ty, **kw)
    img32, radii32, _, _, _ = O.raster_forward(means, opa, view, full, campos, bgv, W, H, tx, ty, **kw)
    d = lambda a: torch.tensor(np.asarray(a, np.float64), requires_grad=True)
    inp = {"means3D": d(means), "opacities": d(opa), "viewmatrix": d(view).detach(), "projmatrix": d(full).detach(),
           "campos": d(campos).detach(), "bg": d(bgv).detach()}
    if colors:
        inp["colors_precomp"] = d(cols)
    else:
        inp["shs"] = d(shs)
    if use_sr:
        inp["scales"], inp["rotations"] = d(scales), d(rots)
    else:
        inp["cov3D_precomp"] = d(c6)
    img, ndc, radii, stats = forward(inp, W, H, tx, ty, D=D)
    assert np.array_equal(radii, radii32), "f64 reference made different culling decisions"
    hom = np.c_[means, np.ones(P)] @ view[:, :3]
    n_clamped = int(((np.abs(hom[:, 0] / hom[:, 2]) > 1.3 * tx) & (radii32 > 0)).sum())
    assert np.abs(img.detach().numpy() - img32).max() < 1e-4
    (img * torch.from_numpy(wgt.astype(np.float64))).sum().backward()
    checks = [("means3D", inp["means3D"].grad), ("opacity", inp["opacities"].grad.view(-1)),
              ("means2D", ndc.grad)]
    checks.append(("colors", inp["colors_precomp"].grad) if colors else ("sh", inp["shs"].grad))
    if use_sr:
        checks += [("scales", inp["scales"].grad), ("rotations", inp["rotations"].grad)]
    else:
        checks.append(("cov3D", inp["cov3D_precomp"].grad))
    errs = {}
    for k, ref in checks:
        got = g[k]
        if k == "means2D":
            got = got[:, :2]
        if k == "sh" and D < 3:
            ref = ref[:, :(D + 1) ** 2]
            got = got[:, :(D + 1) ** 2]
        errs[k] = rel_err(got, ref.numpy())
    return errs, g, n_clamped, stats


@pytest.mark.parametrize("D,bg", [(3, 0.3), (1, 0.0)])
def test_raster_backward_cov3d_sh(D, bg):
    errs, g, _, stats = _compare(14, 40, 36, seed=11 + D, D=D, bg=bg)
    assert stats["alpha_clamped"] > 0, stats
    assert all(e < 2e-3 for e in errs.values()), errs
    assert g["scales"] is None and np.abs(g["means3D"]).max() > 0


def test_raster_backward_scales_rotations_colors():
    errs, _, _, _ = _compare(12, 36, 36, seed=5, use_sr=True, colors=True)
    assert all(e < 2e-3 for e in errs.values()), errs


def test_raster_backward_fov_clamp_quirk():
    """Gaussians outside 1.3 x the fov: the t.x clamp rule of upstream."""
    errs, _, n_clamped, _ = _compare(16, 40, 40, seed=21, wide=True)
    assert n_clamped >= 2, n_clamped
    assert all(e < 2e-3 for e in errs.values()), errs
