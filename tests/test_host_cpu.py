"""CPU tests of the host side and the boundary (no GPU, no compute calls).

* libgsmpm.so loads and binds every entry point include/gsmpm.h declares.
* arguments: ParamGroup semantics of the --config_path interface
  (reference arguments/__init__.py:7-34,83).
* BC activity from the float64 host clock (boundary_conditions.py:15-16,30-31,
  solver.py:19,52).
* GaussianModel PLY I/O and getters against a fixture cut from the
  reference's own udon PLY (tests/golden/make_ply_fixture.py).
* Camera orbit helpers (transform_utils.py:136-216) by their defining properties.
"""
from __future__ import annotations

import json
import os
import re
from argparse import ArgumentParser

import numpy as np
import pytest

from conftest import GOLDEN, PKG, ROOT

HEADER = os.path.join(ROOT, "include", "gsmpm.h")


def _declared():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(gsmpm_\w+)\s*\(", txt)))


# ----------------------------------------------------------------- C-ABI --
def test_header_declares_the_boundary():
    names = _declared()
    for must in ("gsmpm_mpm_create", "gsmpm_mpm_set_particles", "gsmpm_mpm_step", "gsmpm_mpm_postprocess",
                 "gsmpm_mpm_get", "gsmpm_mpm_add_fixed_cube", "gsmpm_mpm_add_impulse",
                 "gsmpm_mpm_add_plane_collider", "gsmpm_raster_forward", "gsmpm_particle_volume",
                 "gsmpm_mpm_slab_init", "gsmpm_mpm_slab_step", "gsmpm_rccl_comm_init", "gsmpm_last_error"):
        assert must in names


def test_library_loads_and_exports_every_declared_symbol():
    import ctypes
    from gsmpm import _lib  # loads libgsmpm.so (no HIP call is made)
    names = _declared()
    missing_sig = [n for n in names if n not in _lib._SIGS]
    assert not missing_sig, f"declared in gsmpm.h but not bound in _lib.py: {missing_sig}"
    for n in names:
        assert isinstance(getattr(_lib.LIB, n), ctypes._CFuncPtr), n
    assert _lib.LIB.gsmpm_version() >= 1


def test_raster_workspace_entry_points_validate_without_a_gpu():
    """gsmpm_raster_workspace_size / gsmpm_raster_forward_ws (the caller-owned
    workspace form): bad sizes and an unaligned workspace are
    refused before any HIP call; sizing itself needs the device (rocPRIM's
    temporary-size queries read its properties) and fails with the HIP error
    here rather than crashing."""
    import ctypes
    from gsmpm import _lib
    nb = ctypes.c_uint64(0)
    assert _lib.LIB.gsmpm_raster_workspace_size(-1, 800, 800, 0, ctypes.byref(nb)) == _lib.GSMPM_EINVAL
    assert "bad argument" in _lib.last_error()
    assert _lib.LIB.gsmpm_raster_workspace_size(10, 0, 800, 0, ctypes.byref(nb)) == _lib.GSMPM_EINVAL
    a = _lib.RasterArgs()
    a.P, a.W, a.H = 10, 64, 64
    need = ctypes.c_int64(0)
    nr = ctypes.c_int32(0)
    assert _lib.LIB.gsmpm_raster_forward_ws(ctypes.byref(a), None, None, ctypes.byref(nr), 0x1001, 1 << 20,
                                            ctypes.byref(need), None) == _lib.GSMPM_EINVAL
    assert "256-byte aligned" in _lib.last_error()
    rc = _lib.LIB.gsmpm_raster_workspace_size(100_000, 800, 800, 500_000, ctypes.byref(nb))
    assert rc == 0 or (rc == _lib.GSMPM_EHIP and _lib.last_error()), (rc, _lib.last_error())


def test_null_arguments_fail_loudly_without_a_gpu():
    """Argument validation happens before any HIP call."""
    import ctypes
    from gsmpm import _lib
    p = _lib.MpmParams()
    p.n_particles, p.n_grid, p.grid_extent, p.material = 10, 16, 2.0, 7
    h = ctypes.c_void_p()
    assert _lib.LIB.gsmpm_mpm_create(ctypes.byref(p), ctypes.byref(h)) < 0
    assert "Material not supported yet" in _lib.last_error()  # model.py:30
    assert _lib.LIB.gsmpm_mpm_step(None, ctypes.c_float(1e-4), 1, None, None) < 0
    assert _lib.LIB.gsmpm_mpm_field_width(_lib.FIELD["C"]) == 9
    assert _lib.LIB.gsmpm_mpm_field_width(99) < 0


# ------------------------------------------------------------- arguments --
def _parse(cfg, cli):
    from arguments import ModelParams, MPMParams, RenderParams
    parser = ArgumentParser()
    m, s, r = ModelParams(parser, cfg["model"]), MPMParams(parser, cfg["mpm"]), RenderParams(parser, cfg["render"])
    a = parser.parse_args(cli)
    return m.extract(a), s.extract(a), r.extract(a)


def test_param_group_semantics():
    with open(os.path.join(PKG, "configs", "lego.json")) as f:
        cfg = json.load(f)
    m, s, r = _parse(cfg, [])
    assert s.n_grid == 50 and s.substep_dt == 1e-4 and s.frame_dt == 0.01
    assert s.steps_per_frame == int(0.01 / 1e-4) == 100        # arguments/__init__.py:83 (int truncation)
    assert s.gravity == [0.0, 0.0, -100.0] and s.material == "jelly"
    assert len(s.boundary_conditions) == 3
    assert not hasattr(r, "steps_per_frame") and not hasattr(m, "n_grid")
    # JSON keys a group does not declare are ignored (lego's model.white_background)
    assert r.white_background is False
    # CLI overrides JSON, typed by the default's type
    m2, s2, r2 = _parse(cfg, ["--n_grid", "128", "--material", "metal", "--white_background", "--num_frames", "3"])
    assert s2.n_grid == 128 and isinstance(s2.n_grid, int) and s2.material == "metal"
    assert r2.white_background is True and r2.num_frames == 3
    # additions are off by default
    assert s.jelly_fcr is False and m.synthetic == 0


def test_steps_per_frame_truncates():
    cfg = {"model": {}, "mpm": {"frame_dt": 0.03, "substep_dt": 0.0007}, "render": {}}
    _, s, _ = _parse(cfg, [])
    assert s.steps_per_frame == 42  # int(42.857...)


# ------------------------------------------------------------------- BCs --
def _lego_specs():
    from gsmpm.bc import BCSpec
    with open(os.path.join(PKG, "configs", "lego.json")) as f:
        bcs = json.load(f)["mpm"]["boundary_conditions"]
    specs = []
    for bit, d in enumerate(bcs):
        specs.append(BCSpec(d["type"], bit, d["start_time"], d["start_time"] + 1e-4 * d["num_dt"]))
    specs.append(BCSpec("collider", len(bcs)))
    return specs


def test_lego_impulse_window_on_f64_clock():
    """lego's impulse [0.8, 0.8 + 10 dt) is live on substeps 8001..8010 of the
    f64 clock (time += 1e-4 accumulates below 0.8 at substep 8000)."""
    from gsmpm.bc import substep_masks
    specs = _lego_specs()
    masks, t = substep_masks(specs, 0.0, 1e-4, 8100)
    imp = [i for i, m in enumerate(masks) if m & (1 << 2)]
    assert imp == list(range(8001, 8011))
    # the long fixed cube is always on; the 1-substep cube only on substep 0; colliders carry no bit
    assert all(m & 1 for m in masks)
    assert [i for i, m in enumerate(masks) if m & 2] == [0]
    assert all(not (m >> 3) for m in masks)
    # chunked calls give the same masks as one long call (the clock is threaded through)
    a, t1 = substep_masks(specs, 0.0, 1e-4, 5000)
    b, t2 = substep_masks(specs, t1, 1e-4, 3100)
    assert a + b == masks and t2 == t


# ------------------------------------------------------------ PLY / model --
def test_ply_fixture_getters_and_roundtrip(tmp_path):
    import torch
    from gaussian_splatting.scene import GaussianModel
    exp = np.load(os.path.join(GOLDEN, "udon64_expected.npz"))
    g = GaussianModel(3, device="cpu")
    g.load_ply(os.path.join(GOLDEN, "udon64.ply"))
    f = lambda t: t.detach().double().numpy()
    assert g.get_xyz.shape == (64, 3) and g.get_features.shape == (64, 16, 3)
    np.testing.assert_allclose(f(g.get_xyz), exp["xyz"], rtol=0, atol=0)
    np.testing.assert_allclose(f(g.get_opacity)[:, 0], exp["opacity"], rtol=1e-6)
    np.testing.assert_allclose(f(g.get_features), exp["features"], rtol=0, atol=0)
    np.testing.assert_allclose(f(g.get_scaling), exp["scaling"], rtol=1e-6)
    cov = f(g.get_covariance())
    np.testing.assert_allclose(cov, exp["cov6"], rtol=1e-4, atol=1e-6 * np.abs(exp["cov6"]).max())
    # save -> load is the identity on the raw parameters
    p = tmp_path / "rt.ply"
    g.save_ply(str(p))
    h = GaussianModel(3, device="cpu")
    h.load_ply(str(p))
    for a, b in ((g._xyz, h._xyz), (g._features_rest, h._features_rest), (g._rotation, h._rotation),
                 (g._opacity, h._opacity), (g._scaling, h._scaling)):
        assert torch.equal(a, b)
    # load_multiple_plys concatenates and skips missing files (main.py:47)
    m = GaussianModel(3, device="cpu")
    m.load_multiple_plys([str(p), str(tmp_path / "missing.ply"), os.path.join(GOLDEN, "udon64.ply")])
    assert m.get_xyz.shape == (128, 3)
    with pytest.raises(FileNotFoundError):
        m.load_multiple_plys([str(tmp_path / "nope.ply")])


def test_ply_rejects_non_float_and_ascii(tmp_path):
    from gaussian_splatting.scene import GaussianModel
    p = tmp_path / "bad.ply"
    p.write_bytes(b"ply\nformat ascii 1.0\nelement vertex 1\nproperty float x\nend_header\n0\n")
    with pytest.raises(ValueError):
        GaussianModel(3, device="cpu").load_ply(str(p))


# --------------------------------------------------------------- camera --
def test_camera_orbit_helpers():
    from utils.transform_utils import (generate_local_coord, get_camera_position_and_rotation,
                                       get_point_on_sphere)
    rng = np.random.default_rng(1)
    for vert in [np.array([0.0, 0.0, 1.0]), np.array([1.0, -1.0, 0.0]), rng.normal(size=3)]:
        v, h1, h2 = generate_local_coord(vert.copy())
        basis = np.stack([h1, h2, v])
        np.testing.assert_allclose(basis @ basis.T, np.eye(3), atol=1e-12)      # orthonormal
        np.testing.assert_allclose(v, vert / np.linalg.norm(vert), atol=1e-12)
        np.testing.assert_allclose(np.cross(h1, v), h2, atol=1e-12)             # h2 = h1 x v
        obs = np.column_stack((h1, h2, v))
        center = rng.normal(size=3)
        for az, el, rad in ((130.0, 10.0, 5.75), (-45.0, 60.0, 2.0)):
            p = get_point_on_sphere(az, el, rad, center, obs)
            assert abs(np.linalg.norm(p - center) - rad) < 1e-12
            # elevation = angle above the plane orthogonal to the vertical axis
            assert abs(np.dot(p - center, v) - rad * np.sin(np.radians(el))) < 1e-12
            pos, R = get_camera_position_and_rotation(az, el, rad, center, obs)
            np.testing.assert_allclose(pos, p, atol=1e-12)
            np.testing.assert_allclose(R.T @ R, np.eye(3), atol=1e-12)
            fwd = (center - pos) / np.linalg.norm(center - pos)
            np.testing.assert_allclose(R[:, 2], fwd, atol=1e-12)                 # 3rd column looks at the center
            assert np.dot(R[:, 1], -v) >= -1e-9                                  # 2nd column points "down"
            assert abs(np.linalg.det(R) - 1.0) < 1e-12


def test_to8b_truncates():
    from utils.render_utils import to8b
    x = np.array([-1.0, 0.0, 0.5, 1 / 255, 0.999, 1.0, 7.0])
    assert to8b(x).tolist() == [0, 0, 127, 1, 254, 255, 255]  # uint8(255 * clip(x)) truncates


def test_camera_known_answers():
    """Hand-derived answers for the orbit camera (transform_utils.py:136-216,
    main.py:84-106) and the projection (graphics_utils getProjectionMatrix).
    Vertical axis z: generate_local_coord gives h1 = (1,1,0)/sqrt2 and
    h2 = h1 x z = (1,-1,0)/sqrt2; azimuth 0 / elevation 0 puts the camera at
    center + r h1 looking back along -h1 with its y axis along -z, so
    R = [(-1,1,0)/sqrt2 | (0,0,-1) | (-1,-1,0)/sqrt2].  modify_cam's W2C maps
    the view center to (0, 0, r), and its campos is the W2C translation
    (SURVEY F8), (0, 0, r) - R^T center."""
    import math as _m
    import torch
    from gaussian_splatting.utils.graphics_utils import getProjectionMatrix
    from utils.render_utils import TinyCam
    from utils.transform_utils import generate_local_coord, get_camera_position_and_rotation
    import main as M
    s2 = 1.0 / _m.sqrt(2.0)
    v, h1, h2 = generate_local_coord(np.array([0.0, 0.0, 2.0]))
    np.testing.assert_allclose(v, [0, 0, 1], atol=1e-15)
    np.testing.assert_allclose(h1, [s2, s2, 0], atol=1e-15)
    np.testing.assert_allclose(h2, [s2, -s2, 0], atol=1e-15)
    obs = np.column_stack((h1, h2, v))
    r = 5.75
    pos, R = get_camera_position_and_rotation(0.0, 0.0, r, np.zeros(3), obs)
    np.testing.assert_allclose(pos, [r * s2, r * s2, 0], atol=1e-14)
    np.testing.assert_allclose(R, np.column_stack(([-s2, s2, 0], [0, 0, -1], [-s2, -s2, 0])), atol=1e-15)
    pos, R = get_camera_position_and_rotation(90.0, 0.0, r, np.zeros(3), obs)
    np.testing.assert_allclose(pos, [r * s2, -r * s2, 0], atol=1e-14)
    # projection at 90 degrees both ways: diag(1, 1, f/(f-n)), P[2,3] = -f n/(f-n), P[3,2] = 1
    P = getProjectionMatrix(znear=0.01, zfar=100, fovX=_m.pi / 2, fovY=_m.pi / 2).numpy()
    n_, f_ = 0.01, 100.0
    want = np.array([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, f_ / (f_ - n_), -f_ * n_ / (f_ - n_)], [0, 0, 1, 0]])
    np.testing.assert_allclose(P, want, rtol=1e-6, atol=1e-7)
    # modify_cam (azimuth 130, elevation 10, radius 5.75) around two centers
    for center in (np.zeros(3), np.array([0.3, -0.2, 0.9])):
        cam = TinyCam(width=64, height=48, FovX=_m.pi / 2, FovY=_m.pi / 2, cam_center=np.zeros(3, np.float32),
                      view_mat=None, full_proj_mat=None)
        cam = M.modify_cam(cam, center, obs, device="cpu")
        W2C = cam.view_mat.numpy().T  # the rasterizer's transposed convention
        pc = W2C @ np.append(center, 1.0)
        np.testing.assert_allclose(pc[:3], [0, 0, r], atol=1e-5)
        _, Rc = get_camera_position_and_rotation(130, 10, r, center, obs)
        np.testing.assert_allclose(cam.cam_center, np.array([0, 0, r]) - Rc.T @ center, atol=1e-5)
        np.testing.assert_allclose(cam.full_proj_mat.numpy(), cam.view_mat.numpy() @ want.T, rtol=1e-5, atol=1e-5)
