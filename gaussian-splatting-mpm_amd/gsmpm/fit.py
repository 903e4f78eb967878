"""Torch-facing wrapper of the differentiable-MPM C-ABI (gsmpm_fit_*).

Mirrors what MPM_Simulator does with args.fitting=True (solver.py:54-108,
131-133, 167-177; model.py:135-223): ``forward(dt, s)`` = p2g2p_forward,
``backward(dt, s)`` = p2g2p_backward, and so on.  All tensors live on the
current HIP device; calls are asynchronous on torch's current stream.
"""
from __future__ import annotations

import ctypes
import math

import torch

from . import _lib
from ._lib import LIB, check, ptr, stream_of

STICKY_GROUND = ((1.0, 0.6, 1.0), (1.0, 0.1, 1.0))  # StickyGroundBC, boundary_conditions.py:88-95
_LEVELED = {"x", "v", "F", "C", "stress", "gx", "gv", "gF", "gC", "gstress"}


class FitSimulator:
    def __init__(self, n_particles: int, *, n_grid: int, grid_extent: float = 2.0, levels: int = 31,
                 E: float = 2e6, nu: float = 0.4, density: float = 1000.0, gravity=(0.0, -9.81, 0.0), device=None):
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        self.n, self.n_grid, self.levels = int(n_particles), int(n_grid), int(levels)
        p = _lib.FitParams()
        p.n_particles, p.n_grid, p.grid_extent, p.levels = self.n, self.n_grid, float(grid_extent), self.levels
        p.E, p.nu, p.density = float(E), float(nu), float(density)
        p.gravity[:] = [float(g) for g in gravity]
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(LIB.gsmpm_fit_create(ctypes.byref(p), ctypes.byref(h)), "gsmpm_fit_create")
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            LIB.gsmpm_fit_destroy(h)
            self._h = None

    def _s(self):
        return stream_of(self.device)

    def _f32(self, t, shape):
        t = t.to(device=self.device, dtype=torch.float32).contiguous()
        if t.numel() != math.prod(shape):
            raise ValueError(f"expected {math.prod(shape)} values, got {t.numel()}")
        return t

    def set_particles(self, xyz, cov6, vol, init_v=None):
        n = self.n
        self._keep = [self._f32(xyz, (n, 3)), self._f32(cov6, (n, 6)), self._f32(vol, (n,)),
                      None if init_v is None else self._f32(init_v, (n, 3))]
        x, c, v, iv = self._keep
        check(LIB.gsmpm_fit_set_particles(self._h, ptr(x), ptr(c), ptr(v), ptr(iv), self._s()),
              "gsmpm_fit_set_particles")

    def set_fixed_cube(self, center, size):
        d3 = lambda a: (ctypes.c_double * 3)(*[float(x) for x in a])
        check(LIB.gsmpm_fit_set_fixed_cube(self._h, d3(center), d3(size)), "gsmpm_fit_set_fixed_cube")

    def set_bc_ground_only(self):
        self.set_fixed_cube(*STICKY_GROUND)

    def forward(self, dt: float, s: int):
        check(LIB.gsmpm_fit_forward(self._h, ctypes.c_float(dt), int(s), self._s()), "gsmpm_fit_forward")

    def backward(self, dt: float, s: int):
        check(LIB.gsmpm_fit_backward(self._h, ctypes.c_float(dt), int(s), self._s()), "gsmpm_fit_backward")

    def postprocess_forward(self):
        check(LIB.gsmpm_fit_postprocess_forward(self._h, self._s()), "gsmpm_fit_postprocess_forward")

    def postprocess_backward(self):
        check(LIB.gsmpm_fit_postprocess_backward(self._h, self._s()), "gsmpm_fit_postprocess_backward")

    def set_grads(self, xyz_grad, cov_grad):
        g1, g2 = self._f32(xyz_grad, (self.n, 3)), self._f32(cov_grad, (self.n * 6,))
        check(LIB.gsmpm_fit_set_grads(self._h, ptr(g1), ptr(g2), self._s()), "gsmpm_fit_set_grads")
        self._keep_grads = (g1, g2)

    def learn(self):
        check(LIB.gsmpm_fit_learn(self._h, self._s()), "gsmpm_fit_learn")

    def cycle_init(self):
        check(LIB.gsmpm_fit_cycle_init(self._h, self._s()), "gsmpm_fit_cycle_init")

    def clear_grads(self):
        check(LIB.gsmpm_fit_clear_grads(self._h, self._s()), "gsmpm_fit_clear_grads")

    def mu_lam(self):
        check(LIB.gsmpm_fit_mu_lam(self._h, self._s()), "gsmpm_fit_mu_lam")

    def get(self, field: str, level: int = 0) -> torch.Tensor:
        fid = _lib.FIT_FIELD[field]
        w = LIB.gsmpm_fit_field_width(fid)
        out = torch.empty((self.n, w) if w > 1 else (self.n,), dtype=torch.float32, device=self.device)
        check(LIB.gsmpm_fit_get(self._h, fid, int(level), ptr(out), self._s()), f"gsmpm_fit_get({field})")
        return out

    def set(self, field: str, t, level: int = 0):
        fid = _lib.FIT_FIELD[field]
        w = LIB.gsmpm_fit_field_width(fid)
        t = self._f32(t, (self.n, w))
        check(LIB.gsmpm_fit_set(self._h, fid, int(level), ptr(t), self._s()), f"gsmpm_fit_set({field})")
        self._keep_set = t

    def get_grid(self, which: str) -> torch.Tensor:
        code = {"mass": 0, "v_in": 1, "v_out": 2, "v_in_grad": 3, "v_out_grad": 4}[which]
        ng = self.n_grid
        shape = (ng, ng, ng) if code == 0 else (ng, ng, ng, 3)
        out = torch.empty(shape, dtype=torch.float32, device=self.device)
        check(LIB.gsmpm_fit_get_grid(self._h, code, ptr(out), self._s()), "gsmpm_fit_get_grid")
        return out
