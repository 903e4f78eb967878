"""End-to-end drop-in run of main.py (the reference's frame loop,
main.py:297-333): `main.py --config_path configs/lego.json --synthetic 5000
--n_grid 64 --num_frames 2` writes images/0000..0002.png through the HIP
simulator and rasterizer; every PNG must equal the oracle's frame (oracle
MPM 100 substeps per frame with lego.json's BCs and the ground collider,
grid2world + render-space shift, oracle rasterizer, to8b truncation) up to
one 8-bit level on a handful of pixels: float pixels agree to 1e-3
(test_gpu_raster.py), and to8b truncates, so a value within 1e-3 of a level
boundary can land one level apart.
"""
from __future__ import annotations

import os

import numpy as np
import pytest

from scenarios import CONFIGS, build_oracle_sim, covariance6, lego_problem, oracle_run
from test_gpu_configs import _grid2world_np, _lego_camera

pytestmark = pytest.mark.gpu


def test_main_py_frames_match_oracle(dev, tmp_path):
    import math

    import oracle as O
    from PIL import Image

    import main as drv
    from utils.render_utils import to8b
    out = str(tmp_path / "lego")
    drv.main(["--config_path", os.path.join(CONFIGS, "lego.json"), "--synthetic", "5000", "--n_grid", "64",
              "--num_frames", "2", "--output_path", out])
    frames = [np.asarray(Image.open(os.path.join(out, "images", f"{f:04d}.png"))) for f in range(3)]
    assert frames[0].shape == (800, 800, 3) and frames[0].dtype == np.uint8

    prob = lego_problem(5000, 64)
    ref, imps, ops = build_oracle_sim(prob)
    dt, spf = prob["cfg"]["substep_dt"], 100
    cam = _lego_camera(prob, dev)
    g, mask = prob["gaussians"], prob["mask"]
    shs = np.concatenate([g["f_dc"], g["f_rest"]], 1)[mask].astype(np.float32)
    opa = (1.0 / (1.0 + np.exp(-g["opacity_logit"][mask].astype(np.float64)))).astype(np.float32).reshape(-1)
    view, full = cam.view_mat.cpu().numpy(), cam.full_proj_mat.cpu().numpy()
    campos = np.asarray(cam.cam_center.cpu().numpy() if hasattr(cam.cam_center, "cpu") else cam.cam_center,
                        np.float32)
    tx, ty = math.tan(cam.FovX * 0.5), math.tan(cam.FovY * 0.5)
    half = prob["cfg"]["grid_extent"] / 2.0
    t, worst = 0.0, []
    for f in range(3):
        if f > 0:
            t = oracle_run(ref, imps, ops, dt, spf, t0=t)
            ref.postprocess()
            m, c6 = _grid2world_np(ref.x, ref.cov, prob["scale"], prob["center"], half, True)
        else:
            # frame 0 renders the world-space Gaussians themselves (main.py), through the
            # same render-space shift
            c = prob["center"].astype(np.float32)
            m = (c + (g["xyz"][mask] - np.float32(1.0)) / np.float32(1.0)).astype(np.float32)
            c6 = covariance6(g["scale_log"], g["rot"])[mask]
        img, _, _, _, _ = O.raster_forward(m, opa, view, full, campos, np.zeros(3, np.float32), 800, 800, tx, ty,
                                           shs=shs, sh_degree=3, cov3D_precomp=c6)
        exp = to8b(img.transpose(1, 2, 0))
        d = np.abs(frames[f].astype(np.int32) - exp.astype(np.int32))
        worst.append((int(d.max()), int((d > 0).sum())))
        assert d.max() <= 1, (f, worst)
        assert (d > 0).sum() <= 2e-4 * d.size, (f, worst)
    print("main.py frames vs oracle (max level diff, pixels differing):", worst)
