"""Golden vectors from the CPU oracle on seeded synthetic inputs.

  oracle_lego_A.npz  configs[0]: lego.json jelly as written, 5k synthetic
                     Gaussians, 64^3, 50 substeps, lego BCs + ground collider;
                     inputs (x, cov, vol) and outputs (x, v, C, F_trial after 50
                     substeps; cov, R after postprocess).
  oracle_raster.npz  one 3DGS forward (600 Gaussians, SH deg 3, 96x64).

The oracle is a restatement, not the reference (parity
unpinned); these goldens freeze it (tests/test_oracle_goldens.py re-derives
them bit for bit) and give the GPU tests fixed expected outputs.

    python tests/golden/make_oracle_goldens.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import oracle as O  # noqa: E402
from scenarios import build_oracle_sim, lego_problem, oracle_run  # noqa: E402


def lego_A():
    prob = lego_problem(5000, 64)
    sim, imps, ops = build_oracle_sim(prob)
    dt = prob["cfg"]["substep_dt"]
    oracle_run(sim, imps, ops, dt, 50)
    out = dict(x_in=prob["x"], cov_in=prob["cov"], vol_in=prob["vol"], x=sim.x, v=sim.v, C=sim.C, F_trial=sim.F_trial)
    sim.postprocess()
    out.update(cov=sim.cov, R=sim.R)
    return out


def raster_scene(P=600, W=96, H=64, seed=11):
    import math
    rng = np.random.default_rng(seed)
    means = rng.uniform(-0.7, 0.7, size=(P, 3)).astype(np.float32)
    A = rng.normal(0, 1, size=(P, 3, 3)) * 0.04
    cov = A @ A.transpose(0, 2, 1) + np.eye(3) * 1e-4
    c6 = np.stack([cov[:, 0, 0], cov[:, 0, 1], cov[:, 0, 2], cov[:, 1, 1], cov[:, 1, 2], cov[:, 2, 2]], 1)
    opa = rng.uniform(0.05, 0.99, size=(P, 1)).astype(np.float32)
    shs = rng.normal(0, 0.3, size=(P, 16, 3)).astype(np.float32)
    shs[:, 0] += 0.8
    fovx = 0.9
    fovy = 2 * math.atan(math.tan(fovx / 2) * H / W)
    w2c = np.eye(4)
    w2c[:3, 3] = [0.05, -0.02, 3.0]
    zn, zf = 0.01, 100.0
    tx, ty = math.tan(fovx / 2), math.tan(fovy / 2)
    Pm = np.zeros((4, 4))
    Pm[0, 0], Pm[1, 1] = 1 / tx, 1 / ty
    Pm[3, 2], Pm[2, 2], Pm[2, 3] = 1.0, zf / (zf - zn), -(zf * zn) / (zf - zn)
    return dict(means=means, cov6=c6.astype(np.float32), opacity=opa, shs=shs,
                view=w2c.T.astype(np.float32), proj=(Pm @ w2c).T.astype(np.float32),
                campos=np.linalg.inv(w2c)[:3, 3].astype(np.float32), bg=np.array([0.1, 0.2, 0.3], np.float32),
                W=np.int32(W), H=np.int32(H), tanx=np.float32(tx), tany=np.float32(ty))


def raster():
    s = raster_scene()
    img, radii, K, _, _ = O.raster_forward(s["means"], s["opacity"], s["view"], s["proj"], s["campos"], s["bg"],
                                     int(s["W"]), int(s["H"]), float(s["tanx"]), float(s["tany"]), shs=s["shs"],
                                     sh_degree=3, cov3D_precomp=s["cov6"])
    s.update(image=img, radii=radii, num_rendered=np.int32(K))
    return s


if __name__ == "__main__":
    np.savez_compressed(os.path.join(HERE, "oracle_lego_A.npz"), **lego_A())
    np.savez_compressed(os.path.join(HERE, "oracle_raster.npz"), **raster())
    print("wrote oracle_lego_A.npz, oracle_raster.npz")
