"""CPU oracle for the PhysGaussian hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg
may import this module.  The product package never does.

It wraps ``liboracle.so`` (``mpm_oracle.c`` / ``raster_oracle.c``), a scalar f32
restatement of the reference kernels:

* MPM substep: ``mpm_solver/solver.py:27-52`` driving ``mpm_solver/utils.py``
  (stress 13-54, p2g 89-134, grid 177-183, g2p 218-282, postprocess 376-433),
  ``constitutive_models.py``, ``boundary_conditions.py:23-45``,
  ``collider.py:13-44``; init from ``model.py:35-59`` and
  ``internel_filling/filling.py:11-42``.
* Rasterizer forward: upstream diff-gaussian-rasterization (pre-2024), not in
  the reference tree -- "parity unpinned" against upstream, pinned by KATs.

PARITY UNPINNED against the reference itself: no reference test, fixture or
golden vector exists for this path, taichi and the graphdeco
submodules are not installed, and running the reference's Python to generate
fixtures was refused in this pipeline.  The oracle is pinned by
first-principles known-answer tests in ``tests/test_oracle_kat.py``.
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIBS = {}

F32P = ctypes.POINTER(ctypes.c_float)
I32P = ctypes.POINTER(ctypes.c_int32)


class _State(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_int), ("ng", ctypes.c_int),
        ("dx", ctypes.c_float), ("inv_dx", ctypes.c_float),
        ("gravity", ctypes.c_float * 3),
        ("material", ctypes.c_int), ("jelly_quirk", ctypes.c_int),
        ("alpha", ctypes.c_float), ("hardening", ctypes.c_float), ("xi", ctypes.c_float),
        ("plastic_viscosity", ctypes.c_float),
        ("x", F32P), ("v", F32P), ("C", F32P), ("F", F32P), ("F_trial", F32P), ("stress", F32P),
        ("cov", F32P), ("init_cov", F32P), ("R", F32P),
        ("vol", F32P), ("mass", F32P), ("mu", F32P), ("lam", F32P), ("yield_stress", F32P),
        ("gm", F32P), ("gv_in", F32P), ("gv_out", F32P),
    ]


class _GridOp(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int), ("a", ctypes.c_float * 3), ("b", ctypes.c_float * 3),
                ("friction", ctypes.c_float)]


class _Impulse(ctypes.Structure):
    _fields_ = [("center", ctypes.c_float * 3), ("size", ctypes.c_float * 3), ("force", ctypes.c_float * 3),
                ("substep_dt", ctypes.c_float)]


class _RArgs(ctypes.Structure):
    _fields_ = [("P", ctypes.c_int), ("D", ctypes.c_int), ("M", ctypes.c_int), ("W", ctypes.c_int), ("H", ctypes.c_int),
                ("means3D", F32P), ("shs", F32P), ("colors_precomp", F32P), ("opacities", F32P),
                ("scales", F32P), ("rotations", F32P), ("cov3D_precomp", F32P),
                ("scale_modifier", ctypes.c_float),
                ("viewmatrix", F32P), ("projmatrix", F32P), ("campos", F32P), ("bg", F32P),
                ("tanfovx", ctypes.c_float), ("tanfovy", ctypes.c_float)]


def lib(threaded=False):
    """Load (building if needed) liboracle.so, with threaded=True the OpenMP
    build liboracle_omp.so (checker of the BASELINE-size parity runs), or with
    threaded="fast" liboracle_fast.so (OpenMP, -O3 -ffast-math, AVX2/FMA:
    bench.py's timed CPU baseline, and in the long-horizon parity tests one
    member of the spread of valid reference outputs -- never the checker)."""
    name = "liboracle_fast.so" if threaded == "fast" else ("liboracle_omp.so" if threaded else "liboracle.so")
    variant = os.environ.get("GSMPM_ORACLE_VARIANT", "")
    if variant in ("asan", "debug"):  # the host sanitizer / bounds-checked builds (oracle/Makefile)
        name = name.replace(".so", f"_{variant}.so")
    elif variant:
        raise ValueError(f"GSMPM_ORACLE_VARIANT={variant!r}: expected asan or debug")
    if name not in _LIBS:
        path = os.path.join(_HERE, name)
        if not os.path.exists(path):
            subprocess.check_call(["make", "-s", "-C", _HERE, name])
        L = ctypes.CDLL(path)
        L.or_forward.restype = ctypes.c_int
        L.or_forward_crop.restype = ctypes.c_long
        _LIBS[name] = L
    return _LIBS[name]


def _p(a):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"]
    if a.dtype == np.float32:
        return a.ctypes.data_as(F32P)
    if a.dtype == np.int32:
        return a.ctypes.data_as(I32P)
    raise TypeError(a.dtype)


def svd3(A):
    A = np.ascontiguousarray(A, dtype=np.float32).reshape(9)
    U = np.zeros(9, np.float32); V = np.zeros(9, np.float32); s = np.zeros(3, np.float32)
    lib().om_svd3(_p(A), _p(U), _p(s), _p(V))
    return U.reshape(3, 3), s, V.reshape(3, 3)


MATERIALS = {"jelly": 0, "metal": 1, "sand": 2, "foam": 3}


def fluid_return_mapping(F_trial, mu, lam, yield_stress, dt, plastic_viscosity=0.008):
    """fluid_return_mapping (constitutive_models.py:142-213) on n particles,
    plus the StVK Kirchhoff stress of the returned F the GPU build pairs it
    with (symmetrised).  The reference never dispatches it (utils.py:13-54)."""
    F = np.ascontiguousarray(F_trial, np.float32).reshape(-1, 9)
    n = F.shape[0]
    a = lambda v: np.ascontiguousarray(np.broadcast_to(np.asarray(v, np.float32), (n,)))
    mu, lam, y = a(mu), a(lam), a(yield_stress)
    Fo = np.zeros_like(F); tau = np.zeros_like(F)
    lib().om_fluid(ctypes.c_int(n), _p(F), _p(mu), _p(lam), _p(y), ctypes.c_float(plastic_viscosity),
                   ctypes.c_float(dt), _p(Fo), _p(tau))
    return Fo.reshape(n, 3, 3), tau.reshape(n, 3, 3)


def mu_lam(E: float, nu: float, n: int):
    """model.py:42-44 (host f64 -> f32 storage) + utils.py:349-362 (device f32)."""
    logE = np.full(n, math.log10(E), np.float32)
    y = np.full(n, -math.log(0.49 / nu - 1), np.float32)
    mu = np.zeros(n, np.float32); lam = np.zeros(n, np.float32)
    lib().om_mu_lam(ctypes.c_int(n), _p(logE), _p(y), _p(mu), _p(lam))
    return mu, lam


def particle_volume(x, n_grid: int, grid_extent: float):
    """internel_filling/filling.py:27-42 (uniform=False)."""
    x = np.ascontiguousarray(x, np.float32)
    n = x.shape[0]
    cnt = np.zeros(n_grid ** 3, np.int32)
    vol = np.zeros(n, np.float32)
    lib().om_particle_volume(ctypes.c_int(n), _p(x), ctypes.c_int(n_grid),
                             ctypes.c_float(grid_extent / n_grid), _p(cnt), _p(vol))
    return vol


class OracleMPM:
    """Mirror of ``MPM_Simulator`` (solver.py:9-177) on the CPU oracle."""

    def __init__(self, x, cov6, vol, *, n_grid, grid_extent=2.0, material="jelly", E=2e6, nu=0.4,
                 density=1000.0, gravity=(0.0, -9.81, 0.0), jelly_quirk=True, v=None, threaded=False):
        x = np.ascontiguousarray(x, np.float32).reshape(-1, 3)
        n = x.shape[0]
        self.n, self.ng = n, n_grid
        code = MATERIALS.get(material, -1)
        if code not in (0, 1, 2, 3):
            raise TypeError("Material not supported yet")
        f = lambda *shape: np.zeros(shape, np.float32)
        eye = np.tile(np.eye(3, dtype=np.float32).reshape(1, 9), (n, 1))
        self.x = x.copy()
        self.v = f(n, 3) if v is None else np.ascontiguousarray(v, np.float32).reshape(n, 3).copy()
        self.C = f(n, 9); self.F = eye.copy(); self.F_trial = eye.copy(); self.stress = f(n, 9)
        self.init_cov = np.ascontiguousarray(cov6, np.float32).reshape(n, 6).copy()
        self.cov = self.init_cov.copy(); self.R = f(n, 9)
        self.vol = np.ascontiguousarray(vol, np.float32).reshape(n).copy()
        self.mass = (np.float32(density) * self.vol).astype(np.float32)
        self.mu, self.lam = mu_lam(E, nu, n)
        self.yield_stress = np.full(n, 0.005, np.float32)
        nn = n_grid ** 3
        self.gm = f(nn); self.gv_in = f(nn, 3); self.gv_out = f(nn, 3)
        st = _State()
        st.n, st.ng = n, n_grid
        st.dx = grid_extent / n_grid
        st.inv_dx = n_grid / grid_extent
        st.gravity[:] = [float(g) for g in gravity]
        st.material, st.jelly_quirk = code, int(bool(jelly_quirk))
        sin_phi = math.sin(25.0 / 180.0 * 3.141592653589793)
        st.alpha = math.sqrt(2.0 / 3.0) * 2.0 * sin_phi / (3.0 - sin_phi)
        st.hardening, st.xi, st.plastic_viscosity = 1.0, 1.0, 0.008
        for name in ("x", "v", "C", "F", "F_trial", "stress", "cov", "init_cov", "R", "vol", "mass", "mu", "lam",
                     "yield_stress", "gm", "gv_in", "gv_out"):
            setattr(st, name, _p(getattr(self, name)))
        self._st = st
        self._L = lib(threaded)
        self.ops = []       # grid postprocess list (fixed_cube / collider) in order
        self.impulses = []

    def add_fixed_box(self, center, size):
        self.ops.append((0, center, size, 0.0))
        return len(self.ops) - 1

    def add_collider(self, point, normal, friction=0.0):
        s = 1.0 / math.sqrt(float(sum(c * c for c in normal)))
        self.ops.append((1, point, [s * c for c in normal], friction))
        return len(self.ops) - 1

    def add_impulse(self, center, size, force, substep_dt):
        self.impulses.append((center, size, force, substep_dt))
        return len(self.impulses) - 1

    def substep(self, dt, imp_active=None, op_active=None):
        ops = (_GridOp * max(1, len(self.ops)))()
        for i, (k, a, b, fr) in enumerate(self.ops):
            ops[i].kind = k; ops[i].a[:] = list(a); ops[i].b[:] = list(b); ops[i].friction = fr
        imps = (_Impulse * max(1, len(self.impulses)))()
        for i, (c, s, fo, sdt) in enumerate(self.impulses):
            imps[i].center[:] = list(c); imps[i].size[:] = list(s); imps[i].force[:] = list(fo); imps[i].substep_dt = sdt
        ia = np.zeros(max(1, len(self.impulses)), np.int32)
        oa = np.zeros(max(1, len(self.ops)), np.int32)
        if imp_active is not None:
            ia[:len(imp_active)] = imp_active
        if op_active is not None:
            oa[:len(op_active)] = op_active
        self._L.om_substep(ctypes.byref(self._st), ctypes.c_float(dt), ctypes.c_int(len(self.impulses)), imps, _p(ia),
                         ctypes.c_int(len(self.ops)), ops, _p(oa))

    # ---- split substep (multi-GPU slab tests: the halo exchange sits between the halves) ----
    def _tables(self, imp_active, op_active):
        ops = (_GridOp * max(1, len(self.ops)))()
        for i, (k, a, b, fr) in enumerate(self.ops):
            ops[i].kind = k; ops[i].a[:] = list(a); ops[i].b[:] = list(b); ops[i].friction = fr
        imps = (_Impulse * max(1, len(self.impulses)))()
        for i, (c, s, fo, sdt) in enumerate(self.impulses):
            imps[i].center[:] = list(c); imps[i].size[:] = list(s); imps[i].force[:] = list(fo); imps[i].substep_dt = sdt
        ia = np.zeros(max(1, len(self.impulses)), np.int32)
        oa = np.zeros(max(1, len(self.ops)), np.int32)
        if imp_active is not None:
            ia[:len(imp_active)] = imp_active
        if op_active is not None:
            oa[:len(op_active)] = op_active
        return imps, ia, ops, oa

    def substep_begin(self, dt, imp_active=None):
        """solver.py:27-40: grid reset, impulses, stress, P2G (om_substep's first half)."""
        imps, ia, _, _ = self._tables(imp_active, None)
        self.gm[:] = 0; self.gv_in[:] = 0; self.gv_out[:] = 0
        L, st = self._L, ctypes.byref(self._st)
        L.om_impulses(st, ctypes.c_int(len(self.impulses)), imps, _p(ia))
        L.om_stress(st, ctypes.c_float(dt))
        L.om_p2g(st, ctypes.c_float(dt))

    def window_sums(self, x0, nx):
        """(m v, m) of planes [x0, x0 + nx) as [nx, n, n, 4] (planes outside the grid: 0)."""
        ng = self.ng
        out = np.zeros((nx, ng, ng, 4), np.float32)
        lo, hi = max(0, x0), min(ng, x0 + nx)
        if lo < hi:
            gv = self.gv_in.reshape(ng, ng, ng, 3)
            gm = self.gm.reshape(ng, ng, ng)
            out[lo - x0:hi - x0, :, :, :3] = gv[lo:hi]
            out[lo - x0:hi - x0, :, :, 3] = gm[lo:hi]
        return out

    def set_window_sums(self, x0, arr):
        ng, nx = self.ng, arr.shape[0]
        lo, hi = max(0, x0), min(ng, x0 + nx)
        if lo < hi:
            self.gv_in.reshape(ng, ng, ng, 3)[lo:hi] = arr[lo - x0:hi - x0, :, :, :3]
            self.gm.reshape(ng, ng, ng)[lo:hi] = arr[lo - x0:hi - x0, :, :, 3]

    def substep_end(self, dt, op_active=None):
        """solver.py:41-52: grid normalisation, grid postprocess list, G2P."""
        _, _, ops, oa = self._tables(None, op_active)
        L, st = self._L, ctypes.byref(self._st)
        L.om_grid_normalize(st, ctypes.c_float(dt))
        L.om_grid_ops(st, ctypes.c_int(len(self.ops)), ops, _p(oa))
        L.om_g2p(st, ctypes.c_float(dt))

    def postprocess(self):
        self._L.om_postprocess(ctypes.byref(self._st))


def raster_forward(means3D, opacities, viewmatrix, projmatrix, campos, bg, W, H, tanfovx, tanfovy,
                   shs=None, sh_degree=3, colors_precomp=None, cov3D_precomp=None, scales=None, rotations=None,
                   scale_modifier=1.0, crop_tiles=None, threaded=False):
    """Returns (color (3,H,W), radii (P,), num_rendered, depth, tiles_touched).
    crop_tiles=(tx0, ty0, tx1, ty1): blend only those 16x16 tiles (the rest of
    color stays 0); radii / num_rendered / depth / tiles_touched are global.
    threaded=True: the OpenMP build (per-tile sorts and blends in parallel,
    the same arithmetic and lists: a full bicycle frame in seconds);
    threaded="fast": the -O3 -ffast-math build (bench.py's CPU baseline)."""
    c = lambda a: None if a is None else np.ascontiguousarray(np.asarray(a, np.float32))
    means3D = c(means3D).reshape(-1, 3)
    P = means3D.shape[0]
    a = _RArgs()
    a.P, a.W, a.H = P, W, H
    a.D = sh_degree
    keep = []
    shs_c = c(shs)
    a.M = 0 if shs_c is None else int(shs_c.reshape(P, -1, 3).shape[1])
    for name, arr in (("means3D", means3D), ("shs", shs_c), ("colors_precomp", c(colors_precomp)),
                      ("opacities", c(opacities)), ("scales", c(scales)), ("rotations", c(rotations)),
                      ("cov3D_precomp", c(cov3D_precomp)), ("viewmatrix", c(viewmatrix)),
                      ("projmatrix", c(projmatrix)), ("campos", c(campos)), ("bg", c(bg))):
        keep.append(arr)
        setattr(a, name, _p(arr))
    a.scale_modifier = scale_modifier
    a.tanfovx, a.tanfovy = tanfovx, tanfovy
    color = np.zeros((3, H, W), np.float32)
    radii = np.zeros(P, np.int32)
    depth = np.zeros(P, np.float32)
    tt = np.zeros(P, np.int32)
    L = lib(threaded)
    if crop_tiles is None:
        K = int(L.or_forward_crop(ctypes.byref(a), _p(color), _p(radii), _p(depth), _p(tt), None))
    else:
        crop = np.ascontiguousarray(np.asarray(crop_tiles, np.int32).reshape(4))
        K = int(L.or_forward_crop(ctypes.byref(a), _p(color), _p(radii), _p(depth), _p(tt), _p(crop)))
    return color, radii, K, depth, tt


def raster_backward(dL_dcolor, means3D, opacities, viewmatrix, projmatrix, campos, bg, W, H, tanfovx, tanfovy,
                    shs=None, sh_degree=3, colors_precomp=None, cov3D_precomp=None, scales=None, rotations=None,
                    scale_modifier=1.0):
    """Backward of raster_forward for dL/dcolor (3,H,W).  Returns a dict:
    means2D (P,3), colors (P,3), opacity (P,), means3D (P,3), cov3D (P,6),
    sh (P,M,3) or None, scales (P,3) or None, rotations (P,4) or None."""
    c = lambda a: None if a is None else np.ascontiguousarray(np.asarray(a, np.float32))
    means3D = c(means3D).reshape(-1, 3)
    P = means3D.shape[0]
    a = _RArgs()
    a.P, a.W, a.H = P, W, H
    a.D = sh_degree
    keep = []
    shs_c = c(shs)
    a.M = 0 if shs_c is None else int(shs_c.reshape(P, -1, 3).shape[1])
    for name, arr in (("means3D", means3D), ("shs", shs_c), ("colors_precomp", c(colors_precomp)),
                      ("opacities", c(opacities)), ("scales", c(scales)), ("rotations", c(rotations)),
                      ("cov3D_precomp", c(cov3D_precomp)), ("viewmatrix", c(viewmatrix)),
                      ("projmatrix", c(projmatrix)), ("campos", c(campos)), ("bg", c(bg))):
        keep.append(arr)
        setattr(a, name, _p(arr))
    a.scale_modifier = scale_modifier
    a.tanfovx, a.tanfovy = tanfovx, tanfovy
    g = c(dL_dcolor).reshape(3, H, W)
    z = lambda *shape: np.zeros(shape, np.float32)
    out = {"means2D": z(P, 3), "colors": z(P, 3), "opacity": z(P), "means3D": z(P, 3), "cov3D": z(P, 6),
           "sh": z(P, max(a.M, 1), 3) if shs_c is not None else None,
           "scales": z(P, 3) if scales is not None else None, "rotations": z(P, 4) if rotations is not None else None}
    lib().or_backward(ctypes.byref(a), _p(g), _p(out["means2D"]), _p(out["colors"]), _p(out["opacity"]),
                      _p(out["means3D"]), _p(out["cov3D"]), _p(out["sh"]), _p(out["scales"]), _p(out["rotations"]))
    return out


# ------------------------------------------------------------------ differentiable path --
class _DState(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("ng", ctypes.c_int), ("L", ctypes.c_int),
                ("dx", ctypes.c_float), ("inv_dx", ctypes.c_float), ("gravity", ctypes.c_float * 3)] + \
               [(nm, F32P) for nm in ("x", "v", "F", "C", "stress", "gx", "gv", "gF", "gC", "gstress", "vol", "mass",
                                      "logE", "y", "mu", "lam", "glogE", "gy", "gmu", "glam", "init_cov", "cov", "gcov",
                                      "gm", "gv_in", "gv_out", "g_gv_in", "g_gv_out")] + \
               [("n_box", ctypes.c_int), ("box_c", ctypes.c_float * 3), ("box_s", ctypes.c_float * 3), ("g_gm", F32P)]


class OracleDiff:
    """Mirror of MPM_Simulator with args.fitting=True (MPM_state_opt,
    p2g2p_forward/backward, postprocess_forward/backward, learn, clear_grads,
    cycle_init) on the CPU restatement in diff_oracle.c."""

    def __init__(self, x, cov6, vol, *, n_grid, grid_extent=2.0, E=2e6, nu=0.4, density=1000.0,
                 gravity=(0.0, -9.81, 0.0), init_v=None, levels=31, ground_only=False, exact_mass_grad=False):
        x = np.ascontiguousarray(x, np.float32).reshape(-1, 3)
        n, L = x.shape[0], levels
        self.n, self.ng, self.L = n, n_grid, L
        f = lambda *shape: np.zeros(shape, np.float32)
        self.x = f(L, n, 3); self.v = f(L, n, 3); self.F = f(L, n, 9); self.C = f(L, n, 9); self.stress = f(L, n, 9)
        self.gx = f(L, n, 3); self.gv = f(L, n, 3); self.gF = f(L, n, 9); self.gC = f(L, n, 9)
        self.gstress = f(L, n, 9)
        self.x[0] = x
        if init_v is not None:
            self.v[0] = np.asarray(init_v, np.float32).reshape(n, 3)
        self.F[0] = np.tile(np.eye(3, dtype=np.float32).reshape(1, 9), (n, 1))
        self.vol = np.ascontiguousarray(vol, np.float32).reshape(n).copy()
        self.mass = (np.float32(density) * self.vol).astype(np.float32)
        self.logE = np.full(n, math.log10(E), np.float32)
        self.y = np.full(n, -math.log(0.49 / nu - 1), np.float32)
        self.mu = f(n); self.lam = f(n); self.glogE = f(n); self.gy = f(n); self.gmu = f(n); self.glam = f(n)
        self.init_cov = np.ascontiguousarray(cov6, np.float32).reshape(n * 6).copy()
        self.cov = self.init_cov.copy(); self.gcov = f(n * 6)
        nn = n_grid ** 3
        self.gm = f(nn); self.gv_in = f(nn, 3); self.gv_out = f(nn, 3); self.g_gv_in = f(nn, 3); self.g_gv_out = f(nn, 3)
        st = _DState()
        st.n, st.ng, st.L = n, n_grid, L
        st.dx, st.inv_dx = grid_extent / n_grid, n_grid / grid_extent
        st.gravity[:] = [float(g) for g in gravity]
        for nm, _ in _DState._fields_:
            if hasattr(self, nm) and isinstance(getattr(self, nm), np.ndarray):
                setattr(st, nm, _p(getattr(self, nm)))
        st.n_box = 0
        if exact_mass_grad:  # test-only, see oracle.h
            self.g_gm = f(nn)
            st.g_gm = _p(self.g_gm)
        self._st = st
        self._L = lib()
        if ground_only:
            self.set_bc_ground_only()
        self._L.od_mu_lam(ctypes.byref(st))

    def set_bc_ground_only(self):
        """StickyGroundBC (boundary_conditions.py:88-95) as grid_postprocess[0]."""
        self.set_fixed_box([1.0, 0.6, 1.0], [1.0, 0.1, 1.0])

    def set_fixed_box(self, center, size):
        self._st.n_box = 1
        self._st.box_c[:] = list(center)
        self._st.box_s[:] = list(size)

    def mu_lam(self):
        self._L.od_mu_lam(ctypes.byref(self._st))

    def p2g2p_forward(self, dt, s):
        self._L.od_substep_forward(ctypes.byref(self._st), ctypes.c_float(dt), ctypes.c_int(s))

    def p2g2p_backward(self, dt, s):
        self._L.od_substep_backward(ctypes.byref(self._st), ctypes.c_float(dt), ctypes.c_int(s))

    def postprocess_forward(self):
        self._L.od_cov_forward(ctypes.byref(self._st))

    def postprocess_backward(self):
        self._L.od_cov_backward(ctypes.byref(self._st))

    def set_grads(self, xyz_grad, cov_grad):
        self.gx[self.L - 1] = np.asarray(xyz_grad, np.float32).reshape(self.n, 3)
        self.gcov[:] = np.asarray(cov_grad, np.float32).reshape(-1)

    def learn(self):
        self._L.od_learn(ctypes.byref(self._st))

    def cycle_init(self):
        self._L.od_cycle_init(ctypes.byref(self._st))

    def clear_grads(self):
        self._L.od_clear_grads(ctypes.byref(self._st))
