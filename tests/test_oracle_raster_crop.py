"""The oracle rasterizer's tile crop (oracle/raster_oracle.c or_forward_crop,
used by the large-frame GPU parity tests): the cropped tiles' pixels, radii,
tiles_touched and num_rendered equal the full frame's bit for bit."""
import numpy as np

import oracle as O


def test_crop_equals_full_frame_tiles():
    rng = np.random.default_rng(5)
    P, W, H = 3000, 150, 110  # partial tiles on both axes
    means = rng.uniform(-0.8, 0.8, size=(P, 3)).astype(np.float32)
    c6 = np.tile(np.array([3e-3, 0, 0, 2e-3, 0, 2e-3], np.float32), (P, 1))
    c6 *= rng.uniform(0.05, 3.0, size=(P, 1)).astype(np.float32)
    opa = rng.uniform(0.05, 0.95, size=P).astype(np.float32)
    col = rng.uniform(0, 1, size=(P, 3)).astype(np.float32)
    view = np.eye(4, dtype=np.float32)
    view[3, 2] = 3.0
    t = 0.6
    proj = np.array([[1 / t, 0, 0, 0], [0, 1 / t, 0, 0], [0, 0, 100 / 99.99, 1], [0, 0, -1 / 99.99, 0]], np.float32)
    full = view @ proj
    args = (means, opa, view, full, np.zeros(3, np.float32), np.zeros(3, np.float32), W, H, t, t)
    kw = dict(colors_precomp=col, cov3D_precomp=c6)
    c_all, r_all, k_all, d_all, tt_all = O.raster_forward(*args, **kw)
    for crop in ((2, 1, 7, 5), (0, 0, 10, 7), (8, 5, 10, 7)):
        c, r, k, d, tt = O.raster_forward(*args, crop_tiles=crop, **kw)
        assert k == k_all
        assert np.array_equal(r, r_all) and np.array_equal(tt, tt_all) and np.array_equal(d, d_all)
        y0, y1, x0, x1 = crop[1] * 16, min(H, crop[3] * 16), crop[0] * 16, min(W, crop[2] * 16)
        assert np.array_equal(c[:, y0:y1, x0:x1], c_all[:, y0:y1, x0:x1])
        outside = np.ones((H, W), bool)
        outside[y0:y1, x0:x1] = False
        assert not c[:, outside].any()
