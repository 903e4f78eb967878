"""Rasterizer forward parity: HIP (drop-in GaussianRasterizer) vs the CPU oracle.

Tolerance (BASELINE north_star): 1e-3 absolute on pixel values (images in
[0, ~1]); radii and num_rendered must match exactly.
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _camera(W, H, fovx, dist=3.0, yaw=0.3):
    fovy = 2 * math.atan(math.tan(fovx / 2) * H / W)
    c, s = math.cos(yaw), math.sin(yaw)
    Rw = np.array([[c, 0, -s], [0, 1, 0], [s, 0, c]])  # world -> view rotation
    w2c = np.eye(4)
    w2c[:3, :3] = Rw
    w2c[:3, 3] = [0.1, -0.05, dist]
    zn, zf = 0.01, 100.0
    tx, ty = math.tan(fovx / 2), math.tan(fovy / 2)
    P = np.zeros((4, 4))
    P[0, 0], P[1, 1] = 1 / tx, 1 / ty
    P[3, 2], P[2, 2], P[2, 3] = 1.0, zf / (zf - zn), -(zf * zn) / (zf - zn)
    view = w2c.T.astype(np.float32)
    full = (P @ w2c).T.astype(np.float32)
    campos = np.linalg.inv(w2c)[:3, 3].astype(np.float32)
    return view, full, campos, tx, ty


def _scene(P, seed, sh_deg=3):
    rng = np.random.default_rng(seed)
    means = rng.uniform(-0.8, 0.8, size=(P, 3)).astype(np.float32)
    A = rng.normal(0, 1, size=(P, 3, 3)) * 0.03
    cov = A @ A.transpose(0, 2, 1) + np.eye(3) * 1e-4
    c6 = np.stack([cov[:, 0, 0], cov[:, 0, 1], cov[:, 0, 2], cov[:, 1, 1], cov[:, 1, 2], cov[:, 2, 2]], 1)
    opa = rng.uniform(0.05, 0.99, size=(P, 1)).astype(np.float32)
    shs = (rng.normal(0, 0.3, size=(P, 16, 3))).astype(np.float32)
    shs[:, 0] += 0.8
    return means, c6.astype(np.float32), opa, shs


@pytest.mark.parametrize("P,W,H,sh_deg,bg", [(2000, 200, 200, 3, 0.0), (5000, 320, 176, 2, 1.0),
                                              (800, 97, 61, 0, 0.0), (3000, 256, 256, 1, 0.5)])
def test_render_vs_oracle(dev, P, W, H, sh_deg, bg):
    import oracle as O
    import torch
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    means, c6, opa, shs = _scene(P, seed=P + W)
    view, full, campos, tx, ty = _camera(W, H, 0.9)
    bgv = np.full(3, bg, np.float32)
    oc, orad, oK, _, _ = O.raster_forward(means, opa, view, full, campos, bgv, W, H, tx, ty, shs=shs,
                                          sh_degree=sh_deg, cov3D_precomp=c6)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    st = GaussianRasterizationSettings(image_height=H, image_width=W, tanfovx=tx, tanfovy=ty, bg=t(bgv),
                                       scale_modifier=1.0, viewmatrix=t(view), projmatrix=t(full), sh_degree=sh_deg,
                                       campos=t(campos), prefiltered=False, debug=False)
    color, radii = GaussianRasterizer(st)(means3D=t(means), means2D=None, opacities=t(opa), shs=t(shs),
                                          cov3D_precomp=t(c6))
    assert np.array_equal(radii.cpu().numpy(), orad)
    err = np.abs(color.cpu().numpy() - oc)
    assert err.max() < 1e-3, (err.max(), (err > 1e-3).sum())


def test_scale_rotation_path(dev):
    import oracle as O
    import torch
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    rng = np.random.default_rng(3)
    P, W, H = 1500, 160, 120
    means = rng.uniform(-0.7, 0.7, size=(P, 3)).astype(np.float32)
    scales = np.exp(rng.normal(-3.5, 0.4, size=(P, 3))).astype(np.float32)
    rots = rng.normal(0, 1, size=(P, 4)).astype(np.float32)
    rots /= np.linalg.norm(rots, axis=1, keepdims=True)
    opa = rng.uniform(0.1, 0.9, size=(P, 1)).astype(np.float32)
    cols = rng.uniform(0, 1, size=(P, 3)).astype(np.float32)
    view, full, campos, tx, ty = _camera(W, H, 1.0)
    bgv = np.zeros(3, np.float32)
    oc, orad, _, _, _ = O.raster_forward(means, opa, view, full, campos, bgv, W, H, tx, ty, colors_precomp=cols,
                                         scales=scales, rotations=rots, scale_modifier=1.3)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    st = GaussianRasterizationSettings(H, W, tx, ty, t(bgv), 1.3, t(view), t(full), 0, t(campos), False, False)
    color, radii = GaussianRasterizer(st)(means3D=t(means), means2D=None, opacities=t(opa), colors_precomp=t(cols),
                                          scales=t(scales), rotations=t(rots))
    assert np.array_equal(radii.cpu().numpy(), orad)
    assert np.abs(color.cpu().numpy() - oc).max() < 1e-3


def test_empty_and_culled(dev):
    import torch
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    W, H = 64, 32
    view, full, campos, tx, ty = _camera(W, H, 0.8)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    bgv = np.array([0.2, 0.4, 0.6], np.float32)
    st = GaussianRasterizationSettings(H, W, tx, ty, t(bgv), 1.0, t(view), t(full), 0, t(campos), False, False)
    # all behind the camera -> background, radii 0
    means = np.tile(np.array([[0.0, 0.0, -10.0]], np.float32), (10, 1))
    c6 = np.tile(np.array([[1e-2, 0, 0, 1e-2, 0, 1e-2]], np.float32), (10, 1))
    color, radii = GaussianRasterizer(st)(means3D=t(means), means2D=None, opacities=t(np.ones((10, 1), np.float32)),
                                          colors_precomp=t(np.ones((10, 3), np.float32)), cov3D_precomp=t(c6))
    assert int(radii.abs().sum()) == 0
    assert np.allclose(color.cpu().numpy(), bgv[:, None, None])
    with pytest.raises(Exception):
        GaussianRasterizer(st)(means3D=t(means), means2D=None, opacities=t(np.ones((10, 1), np.float32)),
                               cov3D_precomp=t(c6))


@pytest.mark.parametrize("W,H", [(240, 160), (1104, 1000)])
def test_narrow_keys_match_upstream_keys(dev, monkeypatch, W, H):
    """The depth-ordered binning (depth sort, then a stable sort on the tile
    index alone: the chunked counting sort for <= 4096 tiles, rocPRIM onesweep
    above or with GSMPM_RASTER_ONESWEEP=1) gives the same sorted pair lists as
    upstream's 64-bit (tile << 32 | depth bits) keys: images, radii and every
    input gradient bitwise equal; equal depths (ties broken by Gaussian index)
    included.  1104 x 1000 has 4347 tiles (onesweep fallback)."""
    import torch
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    P = 4000
    means, c6, opa, shs = _scene(P, seed=11)
    means[1::7, 2] = means[::7, 2][: len(means[1::7])]  # depth ties
    view, full, campos, tx, ty = _camera(W, H, 0.9)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    st = GaussianRasterizationSettings(image_height=H, image_width=W, tanfovx=tx, tanfovy=ty,
                                       bg=t(np.zeros(3, np.float32)), scale_modifier=1.0, viewmatrix=t(view),
                                       projmatrix=t(full), sh_degree=3, campos=t(campos), prefiltered=False,
                                       debug=False)
    outs = []
    # (wide keys, onesweep, per-tile depth sort: GSMPM_RASTER_TILE_DSORT, chunked path only)
    for wide, onesweep, tds in (("1", "0", "0"), ("0", "0", "0"), ("0", "1", "0"), ("0", "0", "1")):
        monkeypatch.setenv("GSMPM_RASTER_WIDE_KEYS", wide)
        monkeypatch.setenv("GSMPM_RASTER_ONESWEEP", onesweep)
        monkeypatch.setenv("GSMPM_RASTER_TILE_DSORT", tds)
        m, s, o, c = (t(a).requires_grad_(True) for a in (means, shs, opa, c6))
        color, radii = GaussianRasterizer(st)(means3D=m, means2D=None, opacities=o, shs=s, cov3D_precomp=c)
        (color * torch.linspace(0.5, 1.5, color.numel(), device=dev).reshape(color.shape)).sum().backward()
        outs.append([x.detach().cpu().numpy() for x in (color, radii, m.grad, s.grad, o.grad, c.grad)])
    for other in outs[1:]:
        for a, b in zip(outs[0], other):
            assert np.array_equal(a, b)


@pytest.mark.parametrize("P", [3000, 12000])
def test_tile_depth_sort_size_classes(dev, monkeypatch, P):
    """GSMPM_RASTER_TILE_DSORT=1 on lists of every size class: a 48 x 48 image
    (9 tiles) under P Gaussians puts 1,024 < n <= 8,192 (P = 3000) and n > 8,192
    (P = 12000: the rank fallback) entries in a tile; images, radii and every
    input gradient equal the global depth sort's bitwise, depth ties included."""
    import torch
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    W = H = 48
    means, c6, opa, shs = _scene(P, seed=5)
    means[:, :2] *= 0.15  # all in front of the small image
    means[1::5, 2] = means[::5, 2][: len(means[1::5])]  # depth ties
    view, full, campos, tx, ty = _camera(W, H, 0.9)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    st = GaussianRasterizationSettings(image_height=H, image_width=W, tanfovx=tx, tanfovy=ty,
                                       bg=t(np.zeros(3, np.float32)), scale_modifier=1.0, viewmatrix=t(view),
                                       projmatrix=t(full), sh_degree=3, campos=t(campos), prefiltered=False,
                                       debug=False)
    outs = []
    for tds in ("0", "1"):
        monkeypatch.setenv("GSMPM_RASTER_TILE_DSORT", tds)
        m, s, o, c = (t(a).requires_grad_(True) for a in (means, shs, opa, c6))
        color, radii = GaussianRasterizer(st)(means3D=m, means2D=None, opacities=o, shs=s, cov3D_precomp=c)
        (color * torch.linspace(0.5, 1.5, color.numel(), device=dev).reshape(color.shape)).sum().backward()
        outs.append([x.detach().cpu().numpy() for x in (color, radii, m.grad, s.grad, o.grad, c.grad)])
    assert (outs[0][1] > 0).sum() > 0.9 * P
    for a, b in zip(outs[0], outs[1]):
        assert np.array_equal(a, b)


def _dense_scene(P, seed, lo, hi):
    """Heavy tiles (~1000 pairs each) of faint Gaussians (opacity log-uniform in
    [lo, hi]): most list entries fall to k_render's sub-tile culling, and T
    falls below the 1e-4 stop at different depths per pixel (11-72 % of the
    pixels stop for the cases below)."""
    rng = np.random.default_rng(seed)
    means = (rng.uniform(-1, 1, size=(P, 3)) * np.array([1.3, 0.975, 0.5])).astype(np.float32)
    A = rng.normal(0, 1, size=(P, 3, 3)) * 0.05
    cov = A @ A.transpose(0, 2, 1) + np.eye(3) * 1e-3
    c6 = np.stack([cov[:, 0, 0], cov[:, 0, 1], cov[:, 0, 2], cov[:, 1, 1], cov[:, 1, 2], cov[:, 2, 2]], 1)
    opa = np.exp(rng.uniform(np.log(lo), np.log(hi), size=(P, 1))).astype(np.float32)
    shs = (rng.normal(0, 0.3, size=(P, 16, 3))).astype(np.float32)
    shs[:, 0] += 0.8
    return means, c6.astype(np.float32), opa, shs


@pytest.mark.parametrize("P,W,H,lo,hi", [(8000, 100, 72, 0.02, 0.3), (8000, 100, 72, 0.03, 0.5),
                                         (4000, 64, 48, 0.05, 0.7)])
def test_segmented_blend_vs_oracle(dev, P, W, H, lo, hi):
    import oracle as O
    import torch
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    means, c6, opa, shs = _dense_scene(P, P, lo, hi)
    view, full, campos, tx, ty = _camera(W, H, 0.9)
    bgv = np.full(3, 0.5, np.float32)
    oc, orad, oK, _, _ = O.raster_forward(means, opa, view, full, campos, bgv, W, H, tx, ty, shs=shs,
                                          sh_degree=3, cov3D_precomp=c6)
    assert oK > 40 * ((W + 15) // 16) * ((H + 15) // 16)  # lists far longer than one 64-entry segment
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    st = GaussianRasterizationSettings(image_height=H, image_width=W, tanfovx=tx, tanfovy=ty, bg=t(bgv),
                                       scale_modifier=1.0, viewmatrix=t(view), projmatrix=t(full), sh_degree=3,
                                       campos=t(campos), prefiltered=False, debug=False)
    color, radii = GaussianRasterizer(st)(means3D=t(means), means2D=None, opacities=t(opa), shs=t(shs),
                                          cov3D_precomp=t(c6))
    assert np.array_equal(radii.cpu().numpy(), orad)
    err = np.abs(color.cpu().numpy() - oc)
    assert err.max() < 1e-3, (err.max(), (err > 1e-3).sum())


@pytest.mark.parametrize("scene,path", [("dense", "chunked"), ("sparse", "chunked"), ("sparse", "onesweep"),
                                        ("dense", "wide")])
def test_subtile_culling_changes_nothing(dev, monkeypatch, scene, path):
    """k_render's sub-tile culling and the tight binning (each Gaussian binned
    into the tiles its alpha-reach box meets) only drop Gaussians upstream's
    loop skips (alpha < 1/255 at every pixel of the sub-tile): pixels, final T
    and last contributor -- hence the backward's gradients -- are bit-identical
    with both off (GSMPM_RASTER_RENDER_MODE=1, 3-sigma rects), on the chunked
    tile sort, the onesweep sort and upstream's 64-bit keys."""
    import torch
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    monkeypatch.setenv("GSMPM_RASTER_ONESWEEP", "1" if path == "onesweep" else "0")
    monkeypatch.setenv("GSMPM_RASTER_WIDE_KEYS", "1" if path == "wide" else "0")
    if scene == "dense":
        P, W, H = 8000, 100, 72
        means, c6, opa, shs = _dense_scene(P, P, 0.03, 0.5)
    else:
        P, W, H = 3000, 256, 192
        means, c6, opa, shs = _scene(P, seed=7)
    view, full, campos, tx, ty = _camera(W, H, 0.9)
    rng = np.random.default_rng(1)
    wgt = torch.from_numpy(rng.normal(0, 1, (3, H, W)).astype(np.float32)).to(dev)
    t = lambda a, g=False: torch.from_numpy(np.ascontiguousarray(a)).to(dev).requires_grad_(g)
    st = GaussianRasterizationSettings(image_height=H, image_width=W, tanfovx=tx, tanfovy=ty,
                                       bg=t(np.full(3, 0.25, np.float32)), scale_modifier=1.0, viewmatrix=t(view),
                                       projmatrix=t(full), sh_degree=3, campos=t(campos), prefiltered=False,
                                       debug=False)
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("GSMPM_RASTER_RENDER_MODE", mode)
        m3, o1, s1, cv = t(means, True), t(opa, True), t(shs, True), t(c6, True)
        img, _ = GaussianRasterizer(st)(means3D=m3, means2D=None, opacities=o1, shs=s1, cov3D_precomp=cv)
        (img * wgt).sum().backward()
        out[mode] = [x.detach().cpu().numpy() for x in (img, m3.grad, o1.grad, s1.grad, cv.grad)]
    for a, b in zip(out["0"], out["1"]):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("P,W,H,tiles", [(2000, 200, 200, 169), (20000, 1024, 1024, 4096), (6000, 272, 3856, 4097),
                                         (8000, 100, 72, 35)])
def test_num_rendered_and_radii_exact(dev, P, W, H, tiles):
    """num_rendered (K = sum of tiles touched, upstream's binning count that the
    backward and the API rely on) and every radius equal the oracle's exactly.
    Cases: K over many 2048-pair sort chunks; exactly 4096 tiles (the largest
    grid on the chunked counting sort); 4097 tiles (first on the onesweep
    fallback); dense tiles with >1000 pairs each."""
    import oracle as O
    import torch
    from gsmpm import raster
    assert ((W + 15) // 16) * ((H + 15) // 16) == tiles
    means, c6, opa, shs = _dense_scene(P, P + 1, 0.03, 0.5) if tiles == 35 else _scene(P, seed=P + W)
    view, full, campos, tx, ty = _camera(W, H, 0.9)
    bgv = np.zeros(3, np.float32)
    oc, orad, oK, _, _ = O.raster_forward(means, opa, view, full, campos, bgv, W, H, tx, ty, shs=shs, sh_degree=3,
                                          cov3D_precomp=c6)
    assert oK > 4 * 2048
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    K, color, radii = raster.forward(t(means), t(opa), t(view), t(full), t(campos), t(bgv), H, W, tx, ty,
                                     sh_degree=3, shs=t(shs), cov3D_precomp=t(c6))
    assert K == oK, (K, oK)
    assert np.array_equal(radii.cpu().numpy(), orad)
    assert np.abs(color.cpu().numpy() - oc).max() < 1e-3


@pytest.mark.parametrize("P,W,H,tiles", [(6000, 272, 3856, 4097), (20000, 1600, 1200, 7500),
                                         (20000, 4200, 4200, 69169)])
def test_digit_tile_sort_matches_onesweep(dev, monkeypatch, P, W, H, tiles):
    """Above 4,096 tiles, the hand-written LSD digit sort (k_lsd_*, the default
    there: two 8-bit passes, three above 65,535 tiles) against the library's
    onesweep (GSMPM_RASTER_LSD=0): pixels, final T, last contributor and every
    gradient equal bit for bit -- both are stable sorts of the same
    depth-ordered emission."""
    import torch
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    assert ((W + 15) // 16) * ((H + 15) // 16) == tiles
    means, c6, opa, shs = _scene(P, seed=P + W)
    view, full, campos, tx, ty = _camera(W, H, 0.9)
    rng = np.random.default_rng(3)
    wgt = torch.from_numpy(rng.normal(0, 1, (3, H, W)).astype(np.float32)).to(dev)
    t = lambda a, g=False: torch.from_numpy(np.ascontiguousarray(a)).to(dev).requires_grad_(g)
    st = GaussianRasterizationSettings(image_height=H, image_width=W, tanfovx=tx, tanfovy=ty,
                                       bg=t(np.full(3, 0.25, np.float32)), scale_modifier=1.0, viewmatrix=t(view),
                                       projmatrix=t(full), sh_degree=3, campos=t(campos), prefiltered=False,
                                       debug=False)
    out = {}
    # "wide": the digit rows' prefixes by a workgroup per row (k_rows_wide), as bicycle-sized frames take them
    # "lsd16": 4,096-pair chunks (GSMPM_RASTER_LSD_I=16; the default takes 8,192)
    for form, lsd, wide, li in (("onesweep", "0", None, None), ("lsd", "1", None, None), ("wide", "1", "1", None),
                                ("lsd16", "1", "1", "16")):
        monkeypatch.setenv("GSMPM_RASTER_LSD", lsd)
        if wide:
            monkeypatch.setenv("GSMPM_RASTER_ROWS_WIDE_MIN", wide)
        if li:
            monkeypatch.setenv("GSMPM_RASTER_LSD_I", li)
        m3, o1, s1, cv = t(means, True), t(opa, True), t(shs, True), t(c6, True)
        img, radii = GaussianRasterizer(st)(means3D=m3, means2D=None, opacities=o1, shs=s1, cov3D_precomp=cv)
        (img * wgt).sum().backward()
        out[form] = [x.detach().cpu().numpy() for x in (img, radii, m3.grad, o1.grad, s1.grad, cv.grad)]
    assert (out["lsd"][1] > 0).sum() > P // 4
    for form in ("lsd", "wide", "lsd16"):
        for a, b in zip(out[form], out["onesweep"]):
            assert np.array_equal(a, b), form


@pytest.mark.parametrize("P,W,H", [(20000, 800, 800), (20000, 1024, 1024)])
def test_digit_sort_below_4096_tiles_matches_chunked(dev, monkeypatch, P, W, H):
    """GSMPM_RASTER_CHUNKED=0 takes the LSD digit sort (k_lsd_*, k_ranges32) at
    tile counts where the chunked counting sort is the default (2,500 and
    4,096 tiles): pixels, radii and every gradient equal bit for bit."""
    import torch
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    means, c6, opa, shs = _scene(P, seed=P + W + 1)
    view, full, campos, tx, ty = _camera(W, H, 0.9)
    rng = np.random.default_rng(5)
    wgt = torch.from_numpy(rng.normal(0, 1, (3, H, W)).astype(np.float32)).to(dev)
    t = lambda a, g=False: torch.from_numpy(np.ascontiguousarray(a)).to(dev).requires_grad_(g)
    st = GaussianRasterizationSettings(image_height=H, image_width=W, tanfovx=tx, tanfovy=ty,
                                       bg=t(np.full(3, 0.1, np.float32)), scale_modifier=1.0, viewmatrix=t(view),
                                       projmatrix=t(full), sh_degree=3, campos=t(campos), prefiltered=False,
                                       debug=False)
    out = {}
    for form in ("1", "0"):
        monkeypatch.setenv("GSMPM_RASTER_CHUNKED", form)
        m3, o1, s1, cv = t(means, True), t(opa, True), t(shs, True), t(c6, True)
        img, radii = GaussianRasterizer(st)(means3D=m3, means2D=None, opacities=o1, shs=s1, cov3D_precomp=cv)
        (img * wgt).sum().backward()
        out[form] = [x.detach().cpu().numpy() for x in (img, radii, m3.grad, o1.grad, s1.grad, cv.grad)]
    assert (out["1"][1] > 0).sum() > P // 4
    for a, b in zip(out["0"], out["1"]):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("P,W,H", [(20000, 1024, 1024), (6000, 272, 3856)])
def test_tight_binning_pair_counts(dev, monkeypatch, P, W, H):
    """The tight binning sorts fewer pairs than upstream's 3-sigma count (which
    num_rendered keeps), and exactly that count with it off (render mode 1)."""
    import torch
    from gsmpm import raster
    means, c6, opa, shs = _scene(P, seed=P + W)
    view, full, campos, tx, ty = _camera(W, H, 0.9)
    bgv = np.zeros(3, np.float32)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    counts = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("GSMPM_RASTER_RENDER_MODE", mode)
        ctx = raster.shared_context(dev.index or 0)
        K, _, _ = raster.forward(t(means), t(opa), t(view), t(full), t(campos), t(bgv), H, W, tx, ty,
                                 sh_degree=3, shs=t(shs), cov3D_precomp=t(c6), context=ctx)
        binned, rendered = raster.pair_counts(ctx)
        assert rendered == K
        counts[mode] = (binned, K)
    (b0, k0), (b1, k1) = counts["0"], counts["1"]
    assert k0 == k1 and b1 == k1, counts
    assert 0 < b0 < k0, counts
    print("binned / 3-sigma pairs", b0, k0, round(b0 / k0, 3))


@pytest.mark.parametrize("case", ["spread", "wide", "layers", "flat", "culled", "none", "many"])
def test_depth_order_matches_library_sort(dev, monkeypatch, case):
    """Both forms of the hand-written depth order (csrc/dsort.h) against the
    library's stable radix sort + scan (GSMPM_RASTER_DSORT=lib): num_rendered,
    radii and every pixel bit-identical.  "bucket": bucketed on the depth bits,
    each bucket ranked by (bits, index) in a wave or, above 256 entries, a
    bitonic workgroup; "lsd": 8-bit LSD passes over (bits - lo), the passes
    beyond the span's bit length skipped on the device.  Cases: depths spread
    over a box ("spread"), a far outlier stretching the range ("wide": all four
    LSD passes), depths on 3 exact values (buckets of ~1,000: the workgroup
    sort, "layers"), all depths equal (one bucket of 20,000 > 8,192: the
    overflow flag and the LSD-form fallback; one LSD pass, "flat"), a third of
    the Gaussians behind the camera (culled: the tail of the order, "culled"),
    all of them behind it (no pair: K = 0, "none"), and 300,000 Gaussians
    ("many")."""
    import torch
    from gsmpm import raster
    P, W, H, yaw = {"spread": (3000, 256, 192, 0.3), "wide": (20000, 640, 480, 0.3), "layers": (3000, 256, 192, 0.0),
                    "flat": (20000, 512, 512, 0.0), "culled": (20000, 640, 480, 0.3), "none": (5000, 256, 192, 0.3),
                    "many": (300000, 800, 800, 0.3)}[case]
    means, c6, opa, shs = _scene(P, seed=P + 7)
    if case == "wide":
        means[0] = (0.0, 0.0, 60.0)  # far behind the scene
    if case == "layers":
        means[:, 2] = np.float32([-0.2, 0.1, 0.4])[np.arange(P) % 3]
    if case == "flat":
        means[:, 2] = np.float32(0.1)
    if case == "culled":
        means[::3, 2] = np.float32(-4.0)  # view depth < 0.2: culled
    if case == "none":
        means[:, 2] = np.float32(-4.0)  # every Gaussian culled: no pair, the image is the background
    view, full, campos, tx, ty = _camera(W, H, 0.9, yaw=yaw)
    bgv = np.zeros(3, np.float32)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    args = (t(means), t(opa), t(view), t(full), t(campos), t(bgv), H, W, tx, ty)
    kw = dict(sh_degree=3, shs=t(shs), cov3D_precomp=t(c6))
    out = {}
    # early: the hand-written forms publish the pair count from their own kernels (dsort.h ds_publish);
    # "0": from the one-lane kernel after the order, as the library path does
    for mode, early in (("bucket", "1"), ("lsd", "1"), ("bucket", "0"), ("lsd", "0"), ("lib", "1")):
        monkeypatch.setenv("GSMPM_RASTER_DSORT", mode)
        monkeypatch.setenv("GSMPM_RASTER_EARLY_COUNT", early)
        for ctx in (None, raster.RasterContext()):  # the workspace form and the context form
            K, color, radii = raster.forward(*args, **kw, context=ctx)
            torch.cuda.synchronize()
            out[(mode, early, ctx is None)] = (K, color.cpu().numpy(), radii.cpu().numpy())
    K0, c0, r0 = out[("lib", "1", False)]
    if case == "none":
        assert K0 == 0 and (r0 == 0).all() and c0.max() == 0.0  # bgv is black
    else:
        assert K0 > 0 and c0.max() > 0
    if case == "culled":
        assert (r0 == 0).sum() >= P // 3, int((r0 == 0).sum())
    for key, (K, c, r) in out.items():
        assert K == K0, (key, K, K0)
        assert np.array_equal(r, r0), key
        assert np.array_equal(c, c0), (key, float(np.abs(c - c0).max()))


def test_depth_bucket_overflow_takes_lsd_fallback(dev, monkeypatch):
    """The round-4 verdict's item 5: a depth bucket of more than 8,192
    Gaussians (a camera-facing plane: 12,000 Gaussians at one depth) makes the
    bucket form fall back to the hand-written LSD form (from the bucket form's
    state: lo from it, all four digit passes), not to the library sort.  The
    context's diagnostics report the overflow and the fallback; num_rendered,
    radii and every pixel equal the library path's (GSMPM_RASTER_DSORT=lib) and
    the forced LSD form's, in the context and the workspace forms."""
    import torch
    from gsmpm import raster
    P, W, H = 12000, 384, 320
    means, c6, opa, shs = _scene(P, seed=11)
    means[:, 2] = np.float32(0.25)
    view, full, campos, tx, ty = _camera(W, H, 0.9, yaw=0.0)
    bgv = np.zeros(3, np.float32)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    args = (t(means), t(opa), t(view), t(full), t(campos), t(bgv), H, W, tx, ty)
    kw = dict(sh_degree=3, shs=t(shs), cov3D_precomp=t(c6))
    out = {}
    ctx = raster.RasterContext()
    for mode in ("bucket", "lsd", "lib"):
        monkeypatch.setenv("GSMPM_RASTER_DSORT", mode)
        for c in (None, ctx):
            before = raster.dsort_stats(ctx)["fallbacks"]
            K, color, radii = raster.forward(*args, **kw, context=c)
            torch.cuda.synchronize()
            out[(mode, c is None)] = (K, color.cpu().numpy(), radii.cpu().numpy())
            if mode == "bucket" and c is ctx:
                st = raster.dsort_stats(ctx)
                assert st["overflow"] == 1 and st["max_bucket"] > 8192, st
                assert st["fallbacks"] == before + 1, st
    K0, c0, r0 = out[("lib", False)]
    assert K0 > 0 and c0.max() > 0 and (r0 > 0).sum() > P // 2
    for key, (K, c, r) in out.items():
        assert K == K0, (key, K, K0)
        assert np.array_equal(r, r0), key
        assert np.array_equal(c, c0), (key, float(np.abs(c - c0).max()))
    # and the state is left idle: a spread scene through the bucket form right after is exact
    monkeypatch.setenv("GSMPM_RASTER_DSORT", "bucket")
    m2, c62, o2, s2 = _scene(3000, seed=12)
    a2 = (t(m2), t(o2), t(view), t(full), t(campos), t(bgv), H, W, tx, ty)
    Kb, cb, rb = raster.forward(*a2, sh_degree=3, shs=t(s2), cov3D_precomp=t(c62), context=ctx)
    monkeypatch.setenv("GSMPM_RASTER_DSORT", "lib")
    Kl, cl, rl = raster.forward(*a2, sh_degree=3, shs=t(s2), cov3D_precomp=t(c62), context=ctx)
    assert Kb == Kl and torch.equal(rb, rl) and torch.equal(cb, cl)


def test_async_forward_matches_workspace_forward(dev):
    """gsmpm_raster_forward_async (the round-4 verdict's item 4: no host
    round trip on the pair count): the image and radii bit-identical to the
    workspace form's, counts = {K, num_rendered, flags = 0, .} once the stream is past
    it; a capacity below K raises flag bit 1 (no fault, the caller re-renders);
    a depth bucket above 8,192 raises bit 0; P = 0 gives the background and
    zero counts; and the whole forward captured in a graph and replayed on new
    means renders what the synchronous form renders."""
    import torch
    from gsmpm import raster
    P, W, H = 20000, 800, 800
    means, c6, opa, shs = _scene(P, seed=21)
    view, full, campos, tx, ty = _camera(W, H, 0.9, yaw=0.3)
    bgv = np.array([0.1, 0.2, 0.3], np.float32)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    args = [t(means), t(opa), t(view), t(full), t(campos), t(bgv), H, W, tx, ty]
    kw = dict(sh_degree=3, shs=t(shs), cov3D_precomp=t(c6))
    K, col, rad = raster.forward(*args, **kw)  # the workspace form (host count)
    ctx = raster.RasterContext()
    raster.forward(*args, **kw, context=ctx)
    binned, _ = raster.pair_counts(ctx)
    ws = raster.Workspace(dev)
    ar = raster.forward_async(*args, **kw, pairs_cap=binned + binned // 4 + 64, ws=ws)
    nr, flags = ar.result()
    assert flags == 0 and nr == K and int(ar.counts[0]) == binned
    assert torch.equal(ar.radii, rad) and torch.equal(ar.color, col)
    # too small a capacity: flagged, and the next full-capacity call is exact again (the state stays idle)
    small = raster.forward_async(*args, **kw, pairs_cap=binned // 2, ws=ws)
    assert small.result()[1] & 2
    again = raster.forward_async(*args, **kw, pairs_cap=binned + 1, ws=ws)
    assert again.result()[1] == 0 and torch.equal(again.color, col)
    # a camera-facing plane: one depth bucket above 8,192 Gaussians -> flag bit 0
    # (the camera looks along z: yaw 0, as test_depth_order_matches_library_sort's "flat")
    mflat = means.copy()
    mflat[:, 2] = np.float32(0.1)
    view0, full0, campos0, tx0, ty0 = _camera(W, H, 0.9, yaw=0.0)
    flat = raster.forward_async(t(mflat), args[1], t(view0), t(full0), t(campos0), args[5], H, W, tx0, ty0, **kw,
                                pairs_cap=64 * P, ws=ws)
    assert flat.result()[1] & 1
    # no Gaussians: the background
    empty = raster.forward_async(t(np.zeros((0, 3), np.float32)), t(np.zeros((0, 1), np.float32)), *args[2:],
                                 sh_degree=3, shs=t(np.zeros((0, 16, 3), np.float32)),
                                 cov3D_precomp=t(np.zeros((0, 6), np.float32)), ws=ws)
    assert empty.result() == (0, 0) and torch.equal(empty.color, t(bgv).view(3, 1, 1).expand(3, H, W))
    # captured once, replayed on new means (copied into the captured input buffer)
    m_in = t(means).clone()
    col_out = torch.empty((3, H, W), dtype=torch.float32, device=dev)
    rad_out = torch.empty(P, dtype=torch.int32, device=dev)
    cnt = torch.zeros(4, dtype=torch.int32, pin_memory=True)
    cap = 2 * binned
    raster.forward_async(m_in, *args[1:], **kw, pairs_cap=cap, ws=ws, counts=cnt, color=col_out, radii=rad_out)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        raster.forward_async(m_in, *args[1:], **kw, pairs_cap=cap, ws=ws, counts=cnt, color=col_out, radii=rad_out)
    m2 = means + np.float32(0.05)
    K2, col2, rad2 = raster.forward(t(m2), *args[1:], **kw)
    m_in.copy_(t(m2))
    g.replay()
    torch.cuda.synchronize()
    assert int(cnt[2]) == 0 and int(cnt[1]) == K2
    assert torch.equal(rad_out, rad2) and torch.equal(col_out, col2)


@pytest.mark.parametrize("P,W,H", [(3000, 256, 192), (20000, 1100, 1000)])
def test_workspace_forward_matches_context(dev, P, W, H):
    """SURVEY 8(b) b2's caller-owned workspace: gsmpm_raster_forward_ws into a
    torch byte tensor (gsmpm_raster_workspace_size) gives bit-identical pixels,
    radii and num_rendered to the library-owned context form, at <= 4,096
    tiles (chunked tile sort) and above (4,345 tiles: onesweep).  A workspace
    sized for too few pairs reports GSMPM_ESPACE with the count it needs
    (outputs unwritten), and one sized for that count then succeeds."""
    import ctypes
    import torch
    from gsmpm import _lib, raster
    means, c6, opa, shs = _scene(P, seed=P + 1)
    view, full, campos, tx, ty = _camera(W, H, 0.9)
    bgv = np.zeros(3, np.float32)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    args = (t(means), t(opa), t(view), t(full), t(campos), t(bgv), H, W, tx, ty)
    kw = dict(sh_degree=3, shs=t(shs), cov3D_precomp=t(c6))
    K0, c0, r0 = raster.forward(*args, **kw, context=raster.RasterContext())
    ws = raster.Workspace(dev)
    ws.ensure(P, H, W, 16)  # far too few pairs
    a, keep = raster._args(*args, kw["sh_degree"], kw["shs"], None, None, None, kw["cov3D_precomp"], 1.0, False)
    color = torch.full((3, H, W), -7.0, device=dev)
    radii = torch.empty(P, dtype=torch.int32, device=dev)
    nr, need = ctypes.c_int32(0), ctypes.c_int64(0)
    rc = _lib.LIB.gsmpm_raster_forward_ws(ctypes.byref(a), _lib.ptr(color), _lib.ptr(radii), ctypes.byref(nr),
                                         ws.ptr(), ws.nbytes(), ctypes.byref(need), _lib.stream_of(dev))
    torch.cuda.synchronize()
    assert rc == _lib.ESPACE and need.value > 16, (rc, need.value)
    assert bool((color == -7.0).all())  # nothing rendered into the outputs
    ws.ensure(P, H, W, int(need.value))
    K1, c1, r1 = raster.forward(*args, **kw, ws=ws)
    assert K1 == K0
    assert torch.equal(r1, r0)
    assert torch.equal(c1, c0)
    K2, c2, _ = raster.forward(*args, **kw)  # the default: the device's cached workspace, grown on demand
    assert K2 == K0 and torch.equal(c2, c0)


@pytest.mark.parametrize("scene,onesweep", [("dense", "0"), ("sparse", "0"), ("sparse", "1")])
def test_tile_shared_render_matches_quarter_render(dev, monkeypatch, scene, onesweep):
    """k_render4 (one workgroup per tile, each list entry read and gathered once
    for the four quarter waves) against the one-workgroup-per-quarter k_render
    (the default; k_render4 with GSMPM_RASTER_TILE_SHARED=1): pixels and, through the backward, final T and
    last contributor are bit-identical -- with sub-tile masks (chunked sort)
    and without (onesweep: the quarter test on the gathered conic)."""
    import torch
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    if scene == "dense":
        P, W, H = 8000, 100, 72
        means, c6, opa, shs = _dense_scene(P, P, 0.03, 0.5)
    else:
        P, W, H = 3000, 256, 192
        means, c6, opa, shs = _scene(P, seed=9)
    view, full, campos, tx, ty = _camera(W, H, 0.9)
    rng = np.random.default_rng(2)
    wgt = torch.from_numpy(rng.normal(0, 1, (3, H, W)).astype(np.float32)).to(dev)
    t = lambda a, g=False: torch.from_numpy(np.ascontiguousarray(a)).to(dev).requires_grad_(g)
    st = GaussianRasterizationSettings(image_height=H, image_width=W, tanfovx=tx, tanfovy=ty,
                                       bg=t(np.full(3, 0.25, np.float32)), scale_modifier=1.0, viewmatrix=t(view),
                                       projmatrix=t(full), sh_degree=3, campos=t(campos), prefiltered=False,
                                       debug=False)
    monkeypatch.setenv("GSMPM_RASTER_ONESWEEP", onesweep)
    out = {}
    for quarters in ("1", "0"):
        monkeypatch.setenv("GSMPM_RASTER_TILE_SHARED", "0" if quarters == "1" else "1")
        m3, o1, s1, cv = t(means, True), t(opa, True), t(shs, True), t(c6, True)
        img, _ = GaussianRasterizer(st)(means3D=m3, means2D=None, opacities=o1, shs=s1, cov3D_precomp=cv)
        (img * wgt).sum().backward()
        out[quarters] = [x.detach().cpu().numpy() for x in (img, m3.grad, o1.grad, s1.grad, cv.grad)]
    for a, b in zip(out["0"], out["1"]):
        assert np.array_equal(a, b)


def test_in_frame_timing(dev):
    """gsmpm_raster_set_timing / gsmpm_raster_timing: with timing on, each
    forward records its k_render and whole-forward times on its own stream;
    the read returns their sums and count and clears them; off, nothing is
    recorded."""
    import torch
    from gsmpm import raster
    P, W, H = 5000, 320, 240
    means, c6, opa, shs = _scene(P, seed=5)
    view, full, campos, tx, ty = _camera(W, H, 0.9)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    args = [t(means), t(opa), t(view), t(full), t(campos), t(np.zeros(3, np.float32)), H, W, tx, ty]
    kw = dict(sh_degree=3, shs=t(shs), cov3D_precomp=t(c6))
    raster.timing()
    raster.set_timing(True)
    try:
        s = torch.cuda.Stream(dev)
        with torch.cuda.stream(s):
            for _ in range(3):
                raster.forward(*args, **kw)
        kr, fw, n = raster.timing()
        assert n == 3 and 0 < kr <= fw, (kr, fw, n)
        assert raster.timing()[2] == 0  # read once
    finally:
        raster.set_timing(False)
    raster.forward(*args, **kw)
    assert raster.timing()[2] == 0


def test_default_workspaces_bounded_and_released(dev):
    """The default workspace cache (gsmpm.raster.workspace) keeps at most
    _WS_KEEP per process -- short-lived streams evict the least recently used
    one after a device sync instead of leaking a workspace each -- and
    release_workspace drops one explicitly."""
    import torch
    from gsmpm import raster
    streams = [torch.cuda.Stream(dev) for _ in range(raster._WS_KEEP + 4)]
    for st in streams:
        raster.workspace(dev.index or 0, st)
    assert len(raster._WS) <= raster._WS_KEEP
    last = streams[-1]
    assert raster.release_workspace(last, dev.index or 0) is True
    assert raster.release_workspace(last, dev.index or 0) is False
