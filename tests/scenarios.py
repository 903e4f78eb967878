"""Seeded synthetic inputs shared by the oracle, the golden generator and the
GPU parity tests.  numpy only: no device code here."""
from __future__ import annotations

import json
import math
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONFIGS = os.path.join(ROOT, "gaussian-splatting-mpm_amd", "configs")


def load_config(name):
    with open(os.path.join(CONFIGS, name)) as f:
        return json.load(f)


def synthetic_gaussians(n, seed=0, box=((-0.65, -0.65, -0.55), (0.65, 0.65, 0.55)), sh_rest=15):
    """Same draws, same order as GaussianModel.init_synthetic."""
    rng = np.random.default_rng(seed)
    lo, hi = np.asarray(box[0]), np.asarray(box[1])
    xyz = rng.uniform(lo, hi, size=(n, 3))
    scl = rng.normal(-4.5, 0.5, size=(n, 3))
    rot = rng.normal(0.0, 1.0, size=(n, 4))
    rot /= np.linalg.norm(rot, axis=1, keepdims=True)
    opa = rng.normal(2.0, 1.5, size=(n, 1))
    dc = rng.normal(0.5, 0.5, size=(n, 1, 3))
    rest = rng.normal(0.0, 0.05, size=(n, sh_rest, 3))
    f = lambda a: a.astype(np.float32)
    return dict(xyz=f(xyz), scale_log=f(scl), rot=f(rot), opacity_logit=f(opa), f_dc=f(dc), f_rest=f(rest))


def covariance6(scale_log, rot):
    """Upper-6 of (R S)(R S)^T (GaussianModel.get_covariance), f32."""
    s = np.exp(scale_log.astype(np.float32))
    q = rot / np.sqrt((rot.astype(np.float32) ** 2).sum(1, keepdims=True))
    w, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
                  2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
                  2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], 1).reshape(-1, 3, 3)
    L = R * s[:, None, :]
    S = L @ L.transpose(0, 2, 1)
    return np.stack([S[:, 0, 0], S[:, 0, 1], S[:, 0, 2], S[:, 1, 1], S[:, 1, 2], S[:, 2, 2]], 1).astype(np.float32)


def world2grid_np(x, grid_extent):
    """transform_utils.py:8-15 in f32."""
    x = x.astype(np.float32)
    lo, hi = x.min(0), x.max(0)
    c = ((lo + hi) / np.float32(2.0)).astype(np.float32)
    s = np.float32(grid_extent / 2.0) / np.float32((hi - lo).max())
    xg = ((x - c) * s + np.float32(grid_extent / 2.0)).astype(np.float32)
    return xg, c, np.float32(s)


LEGO_BOX = ((-0.65, -0.65, -0.55), (0.65, 0.65, 0.55))
BICYCLE_BOX = ((0.05, 0.05, 0.05), (0.95, 0.95, 0.95))


def lego_problem(n, n_grid, seed=0, config="lego.json", box=None):
    """Synthetic lego (config D with config="bicycle.json"):
    grid-space particles + BC list.  The box defaults to the config's SURVEY 8(d) box."""
    import oracle as O  # test infrastructure only
    cfg = load_config(config)["mpm"]
    if box is None:
        box = BICYCLE_BOX if config.startswith("bicycle") else LEGO_BOX
    g = synthetic_gaussians(n, seed, box=box)
    cov = covariance6(g["scale_log"], g["rot"])
    lo, hi = np.asarray(cfg["sim_area"][0]), np.asarray(cfg["sim_area"][1])
    mask = np.all((g["xyz"] >= lo) & (g["xyz"] <= hi), axis=1)
    x = g["xyz"][mask]
    cov = cov[mask]
    xg, c, s = world2grid_np(x, cfg["grid_extent"])
    covg = (cov * (s * s)).astype(np.float32)
    vol = O.particle_volume(xg, n_grid, cfg["grid_extent"])
    return dict(x=xg, cov=covg, vol=vol, center=c, scale=s, cfg=cfg, n_grid=n_grid, gaussians=g, mask=mask)


class BC:
    """Minimal host BC record for the oracle side (mirrors boundary_conditions.py:15-16,30-31)."""

    def __init__(self, kind, d, substep_dt):
        self.kind = kind
        self.start = d.get("start_time", 0)
        self.end = d.get("start_time", 0) + substep_dt * d.get("num_dt", 0)
        self.d = d

    def active(self, t):
        return self.start <= t < self.end


def build_oracle_sim(prob, material=None, jelly_quirk=True, with_collider=True, threaded=False):
    """threaded=True: the OpenMP build of the same restatement (P2G summation
    order differs from the serial one by f32 rounding only), for the
    BASELINE-size parity runs."""
    import oracle as O
    cfg = prob["cfg"]
    sim = O.OracleMPM(prob["x"], prob["cov"], prob["vol"], n_grid=prob["n_grid"], grid_extent=cfg["grid_extent"],
                      material=material or cfg["material"], E=cfg["E"], nu=cfg["nu"], density=cfg["density"],
                      gravity=cfg["gravity"], jelly_quirk=jelly_quirk, threaded=threaded)
    imps, ops = [], []
    for d in cfg["boundary_conditions"]:
        if d["type"] == "fixed_cube":
            sim.add_fixed_box(d["center"], d["size"])
            ops.append(BC("fixed_cube", d, cfg["substep_dt"]))
        elif d["type"] == "impulse":
            sim.add_impulse(d["center"], d["size"], d["force"], cfg["substep_dt"])
            imps.append(BC("impulse", d, cfg["substep_dt"]))
    if with_collider:
        sim.add_collider([0.0, 0.0, 0.4], [0.0, 0.0, 1.0], 0.0)
        ops.append(None)
    return sim, imps, ops


def oracle_run(sim, imps, ops, dt, n, t0=0.0):
    t = t0
    for _ in range(n):
        ia = [int(b.active(t)) for b in imps]
        oa = [1 if b is None else int(b.active(t)) for b in ops]
        sim.substep(dt, ia, oa)
        t += dt
    return t
