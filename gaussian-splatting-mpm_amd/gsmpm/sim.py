"""Torch-facing wrapper of the MPM C-ABI (gsmpm_mpm_*).

All tensors live on the current HIP device; every call is asynchronous on
torch's current stream.  This is plumbing: the math runs in libgsmpm.so.
"""
from __future__ import annotations

import ctypes
import math

import torch

from . import _lib
from ._lib import LIB, check, ptr, stream_of

MATERIALS = {"jelly": 0, "metal": 1, "sand": 2, "foam": 3}  # mpm_solver/utils.py:5-10

_WIDTH = {"x": 3, "v": 3, "C": 9, "F_trial": 9, "cov": 6, "init_cov": 6, "R": 9, "mass": 1, "vol": 1, "mu": 1,
          "lam": 1, "yield_stress": 1}


def _d3(v):
    return (ctypes.c_double * 3)(*[float(a) for a in v])


class Simulator:
    """One MPM domain: particle state + dense n^3 grid on one GPU."""

    def __init__(self, n_particles: int, *, n_grid: int, grid_extent: float = 2.0, material: str | int = "jelly",
                 E: float = 2e6, nu: float = 0.4, density: float = 1000.0, gravity=(0.0, -9.81, 0.0),
                 yield_stress: float = 0.005, hardening: float = 1.0, xi: float = 1.0,
                 plastic_viscosity: float = 0.008, friction_angle: float = 25.0, jelly_fcr: bool = False,
                 keep_grid: bool = False, use_graph: bool = True, sort: bool = True, phased: bool = False,
                 device=None):
        code = MATERIALS.get(material, -1) if isinstance(material, str) else int(material)
        if code not in (0, 1, 2, 3):
            raise TypeError("Material not supported yet")  # model.py:27-30
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        self.n = int(n_particles)
        self.n_grid = int(n_grid)
        self.grid_extent = float(grid_extent)
        p = _lib.MpmParams()
        p.n_particles = self.n
        p.n_grid = self.n_grid
        p.grid_extent = self.grid_extent
        p.material = code
        p.E, p.nu, p.density = float(E), float(nu), float(density)
        p.gravity[:] = [float(g) for g in gravity]
        p.yield_stress, p.hardening, p.xi = float(yield_stress), float(hardening), float(xi)
        p.plastic_viscosity, p.friction_angle_deg = float(plastic_viscosity), float(friction_angle)
        flags = 0
        if jelly_fcr:
            flags |= _lib.FLAG_JELLY_FCR
        if keep_grid:
            flags |= _lib.FLAG_KEEP_GRID
        if not use_graph:
            flags |= _lib.FLAG_NO_GRAPH
        if not sort:
            flags |= _lib.FLAG_NO_SORT
        if phased:
            flags |= _lib.FLAG_PHASED
        p.flags = flags
        self.params = p
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(LIB.gsmpm_mpm_create(ctypes.byref(p), ctypes.byref(h)), "gsmpm_mpm_create")
        self._h = h

    # -------------------------------------------------------------- setup --
    def set_particles(self, x, cov6, vol, v=None):
        f = lambda t: None if t is None else t.detach().to(self.device, torch.float32).contiguous()
        x, cov6, vol, v = f(x), f(cov6), f(vol), f(v)
        assert x.numel() == 3 * self.n and cov6.numel() == 6 * self.n and vol.numel() == self.n
        assert v is None or v.numel() == 3 * self.n
        check(LIB.gsmpm_mpm_set_particles(self._h, ptr(x), ptr(cov6), ptr(vol), ptr(v), stream_of(self.device)),
              "gsmpm_mpm_set_particles")

    def add_fixed_cube(self, center, size) -> int:
        return check(LIB.gsmpm_mpm_add_fixed_cube(self._h, _d3(center), _d3(size)), "add_fixed_cube")

    def add_impulse(self, center, size, force, substep_dt) -> int:
        return check(LIB.gsmpm_mpm_add_impulse(self._h, _d3(center), _d3(size), _d3(force), float(substep_dt)),
                     "add_impulse")

    def add_plane_collider(self, point, normal, friction=0.0) -> int:
        return check(LIB.gsmpm_mpm_add_plane_collider(self._h, _d3(point), _d3(normal), float(friction)),
                     "add_plane_collider")

    # ------------------------------------------------------------ stepping --
    def step(self, dt: float, masks):
        n = len(masks)
        if n == 0:
            return
        arr = (ctypes.c_uint32 * n)(*[int(m) & 0xFFFFFFFF for m in masks])
        check(LIB.gsmpm_mpm_step(self._h, ctypes.c_float(dt), n, arr, stream_of(self.device)), "gsmpm_mpm_step")

    def check_finite(self, clear: bool = False):
        """SURVEY 5's per-frame NaN / Inf check: waits for the stream and
        raises RuntimeError if any substep so far produced non-finite particle
        state -- a position, or a P2G scatter input (mass, velocity, C,
        stress) -- (``step`` also raises, at the call after)."""
        check(LIB.gsmpm_mpm_check_finite(self._h, int(bool(clear)), stream_of(self.device)), "check_finite")

    # ---------------------------------------------------------- slab mode --
    def slab_init(self, rank: int, world: int, lo: int, hi: int, margin: int = 2, interval: int = 10):
        """Make this simulator (created with n_particles = capacity) rank `rank`
        of a `world`-slab domain owning grid planes [lo, hi) (csrc/slab.h)."""
        with torch.cuda.device(self.device):  # the slab's comm stream / buffers live on this device
            check(LIB.gsmpm_mpm_slab_init(self._h, int(rank), int(world), int(lo), int(hi), int(margin),
                                          int(interval)), "gsmpm_mpm_slab_init")

    def slab_set_particles(self, x, cov6, vol, gid, v=None):
        f = lambda t: None if t is None else t.detach().to(self.device, torch.float32).contiguous()
        x, cov6, vol, v = f(x), f(cov6), f(vol), f(v)
        gid = gid.detach().to(self.device, torch.int32).contiguous()
        n = int(gid.numel())
        assert x.numel() == 3 * n and cov6.numel() == 6 * n and vol.numel() == n
        check(LIB.gsmpm_mpm_slab_set_particles(self._h, n, ptr(x) if n else None, ptr(cov6) if n else None,
                                               ptr(vol) if n else None, ptr(v) if n and v is not None else None,
                                               ptr(gid) if n else None, stream_of(self.device)),
              "gsmpm_mpm_slab_set_particles")

    def slab_step(self, dt: float, masks, transport):
        """`len(masks)` substeps with the window exchange every substep and the
        particle migration every `interval` substeps through `transport`
        (gsmpm.dist.RcclTransport / CallbackTransport)."""
        n = len(masks)
        if n == 0:
            return
        arr = (ctypes.c_uint32 * n)(*[int(m) & 0xFFFFFFFF for m in masks])
        xp = None if transport is None else ctypes.byref(transport.struct)
        with torch.cuda.device(self.device):
            check(LIB.gsmpm_mpm_slab_step(self._h, ctypes.c_float(dt), n, arr, xp, stream_of(self.device)),
                  "gsmpm_mpm_slab_step")

    @property
    def count(self) -> int:
        """Particles this simulator holds now (a slab's count changes with migration)."""
        return check(LIB.gsmpm_mpm_count(self._h), "gsmpm_mpm_count")

    def get_gid(self) -> torch.Tensor:
        out = torch.empty(self.count, dtype=torch.int32, device=self.device)
        if out.numel():
            check(LIB.gsmpm_mpm_get_gid(self._h, ptr(out), stream_of(self.device)), "gsmpm_mpm_get_gid")
        return out

    def slab_stats(self):
        b = (ctypes.c_int64 * 12)()
        check(LIB.gsmpm_mpm_slab_stats(self._h, b), "gsmpm_mpm_slab_stats")
        keys = ("migrations", "migrated", "lo", "hi", "margin", "interval", "window_planes", "capacity", "deferred",
                "payload_capacity", "host_syncs", "step_calls")
        return dict(zip(keys, [int(v) for v in b]))

    def slab_rects(self):
        """The exchanged yz rect of the lower and upper window: [(y0, ny, z0, nz)] * 2."""
        b = (ctypes.c_int32 * 8)()
        check(LIB.gsmpm_mpm_slab_rects(self._h, b), "gsmpm_mpm_slab_rects")
        return [tuple(int(v) for v in b[4 * w:4 * w + 4]) for w in (0, 1)]

    def slab_set_rebalance(self, on: bool = True, tolerance: float = 0.05):
        """Re-cut the slabs at step-call boundaries when the most loaded one holds
        more than (1 + tolerance) x the mean (gsmpm_mpm_slab_set_rebalance)."""
        check(LIB.gsmpm_mpm_slab_set_rebalance(self._h, 1 if on else 0, ctypes.c_float(tolerance)),
              "gsmpm_mpm_slab_set_rebalance")

    def slab_set_weight(self, weight: float):
        """This rank's share weight in the re-cut (gsmpm_mpm_slab_set_weight)."""
        check(LIB.gsmpm_mpm_slab_set_weight(self._h, ctypes.c_float(weight)), "gsmpm_mpm_slab_set_weight")

    def slab_bounds(self, world: int):
        """(every slab's bounds [world + 1], re-cuts so far)."""
        b = (ctypes.c_int32 * (world + 1))()
        n = ctypes.c_int64(0)
        check(LIB.gsmpm_mpm_slab_bounds(self._h, b, world + 1, ctypes.byref(n)), "gsmpm_mpm_slab_bounds")
        return [int(v) for v in b], int(n.value)

    def profile(self, dt: float, masks):
        """Eager substeps with a hipEvent pair per kernel -> summed ms of
        (k_p2g, k_grid, k_g2p, binning); fused pipeline: (k_fused, k_grid_f, binning, 0)."""
        n = len(masks)
        arr = (ctypes.c_uint32 * max(1, n))(*[int(m) & 0xFFFFFFFF for m in masks])
        out = (ctypes.c_float * 4)()
        check(LIB.gsmpm_mpm_profile_substeps(self._h, ctypes.c_float(dt), n, arr, out, stream_of(self.device)),
              "gsmpm_mpm_profile_substeps")
        return tuple(float(v) for v in out)

    def time_kernels(self, dt: float, mask: int, reps: int = 20):
        """Per-launch ms of (k_p2g, k_grid, k_g2p, binning) -- fused pipeline:
        (k_fused, k_grid_f, binning, 0) -- from hipEvents around `reps`
        back-to-back launches of each on this stream; state restored."""
        out = (ctypes.c_float * 4)()
        check(LIB.gsmpm_mpm_time_kernels(self._h, ctypes.c_float(dt), int(mask) & 0xFFFFFFFF, int(reps), out,
                                         stream_of(self.device)), "gsmpm_mpm_time_kernels")
        return tuple(float(v) for v in out)

    def debug_stats(self):
        b = (ctypes.c_int32 * 8)()
        check(LIB.gsmpm_mpm_debug_stats(self._h, b, stream_of(self.device)), "gsmpm_mpm_debug_stats")
        keys = ("active_tiles", "max_per_tile", "outside", "chunks", "touched_tiles", "binned", "parity", "since_sort")
        return dict(zip(keys, list(b)))

    def live_box(self):
        b = (ctypes.c_int32 * 6)()
        check(LIB.gsmpm_mpm_live_box(self._h, b, stream_of(self.device)), "gsmpm_mpm_live_box")
        return list(b[:3]), list(b[3:])

    @property
    def pipeline(self) -> str:
        """'fused' (k_fused + k_grid_f per substep) or 'phased' (k_p2g, k_grid, k_g2p, binning)."""
        code = check(LIB.gsmpm_mpm_pipeline(self._h), "gsmpm_mpm_pipeline")
        return "fused" if code == _lib.PIPE_FUSED else "phased"

    @property
    def folded(self) -> bool:
        """True when each substep's grid update is folded into the next k_fused
        launch (gsmpm_mpm_folded; one launch per substep)."""
        return bool(check(LIB.gsmpm_mpm_folded(self._h), "gsmpm_mpm_folded"))

    def escapes(self, clear: bool = False) -> int:
        """Particle scatters that left their chunk window since set_particles or
        the last clear (gsmpm_mpm_escapes; syncs the stream)."""
        out = ctypes.c_int64(0)
        check(LIB.gsmpm_mpm_escapes(self._h, int(bool(clear)), ctypes.byref(out), stream_of(self.device)),
              "gsmpm_mpm_escapes")
        return int(out.value)

    def rebin_state(self):
        """{interval, auto, rebins_last_call, vmax} (gsmpm_mpm_rebin_state): the
        longest spacing, whether the re-binnings adapt to the particles' speed,
        how many the last step call ran (0: from the interval) and the fastest
        velocity component seen."""
        b = (ctypes.c_int32 * 3)()
        v = ctypes.c_float(0.0)
        check(LIB.gsmpm_mpm_rebin_state(self._h, b, ctypes.byref(v)), "gsmpm_mpm_rebin_state")
        return {"interval": int(b[0]), "auto": bool(b[1]), "rebins_last_call": int(b[2]), "vmax": float(v.value)}

    def set_rebin_interval(self, substeps: int):
        """Fused pipeline: substeps between particle re-binnings (any value >= 1 is correct)."""
        check(LIB.gsmpm_mpm_set_rebin_interval(self._h, int(substeps)), "gsmpm_mpm_set_rebin_interval")

    def resort(self, interval: int = -1):
        """Re-sort storage into Morton order now; interval >= 0 sets the automatic period."""
        check(LIB.gsmpm_mpm_resort(self._h, int(interval), stream_of(self.device)), "gsmpm_mpm_resort")

    def postprocess(self):
        if self.count == 0:
            return
        check(LIB.gsmpm_mpm_postprocess(self._h, stream_of(self.device)), "gsmpm_mpm_postprocess")

    # ------------------------------------------------------------------ io --
    def get(self, name: str) -> torch.Tensor:
        w, n = _WIDTH[name], self.count
        out = torch.empty((n, w) if w > 1 else (n,), dtype=torch.float32, device=self.device)
        if n:
            check(LIB.gsmpm_mpm_get(self._h, _lib.FIELD[name], ptr(out), stream_of(self.device)), f"get {name}")
        return out

    def set(self, name: str, t: torch.Tensor):
        t = t.detach().to(self.device, torch.float32).contiguous()
        assert t.numel() == self.n * _WIDTH[name]
        check(LIB.gsmpm_mpm_set(self._h, _lib.FIELD[name], ptr(t), stream_of(self.device)), f"set {name}")

    def get_grid(self, which: str) -> torch.Tensor:
        code = {"mass": 0, "v_in": 1, "v_out": 2}[which]
        ng = self.n_grid
        shape = (ng, ng, ng) if code == 0 else (ng, ng, ng, 3)
        out = torch.empty(shape, dtype=torch.float32, device=self.device)
        check(LIB.gsmpm_mpm_get_grid(self._h, code, ptr(out), stream_of(self.device)), f"get_grid {which}")
        return out

    def world_outputs(self, scale, center, render_space: bool, means_out=None, cov_out=None):
        """Fused grid2world (+ render shift) of x and cov, in caller order."""
        n = self.count
        means_out = torch.empty((n, 3), dtype=torch.float32, device=self.device) if means_out is None else means_out
        cov_out = torch.empty((n, 6), dtype=torch.float32, device=self.device) if cov_out is None else cov_out
        if n == 0:
            return means_out, cov_out
        c = (ctypes.c_float * 3)(*[float(a) for a in center])
        check(LIB.gsmpm_mpm_world_outputs(self._h, ctypes.c_float(float(scale)), c, int(bool(render_space)),
                                          ptr(means_out), ptr(cov_out), stream_of(self.device)), "world_outputs")
        return means_out, cov_out

    def close(self):
        if getattr(self, "_h", None):
            LIB.gsmpm_mpm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def particle_volume(x: torch.Tensor, n_grid: int, grid_extent: float) -> torch.Tensor:
    """internel_filling/filling.py:27-42 on the GPU (i32 atomics, floor cells)."""
    x = x.detach().to(torch.float32).contiguous()
    n = x.shape[0]
    scratch = torch.empty(n_grid ** 3, dtype=torch.int32, device=x.device)
    vol = torch.empty(n, dtype=torch.float32, device=x.device)
    check(LIB.gsmpm_particle_volume(ptr(x), n, n_grid, float(grid_extent), ptr(scratch), ptr(vol),
                                    stream_of(x.device)), "gsmpm_particle_volume")
    return vol


def alpha_from_friction(friction_angle_deg: float) -> float:
    """model.py:48-51 (f64)."""
    s = math.sin(friction_angle_deg / 180.0 * 3.141592653589793)
    return math.sqrt(2.0 / 3.0) * 2.0 * s / (3.0 - s)
