"""ctypes binding of libgsmpm.so (the C-ABI declared in include/gsmpm.h).

The HIP library is the only compute path: if it is missing or fails to load,
importing this module raises -- there is no CPU fallback.  torch is imported
first so that libgsmpm.so binds to the HIP runtime torch already loaded
(both carry SONAME libamdhip64.so.7), which makes torch device pointers and
streams valid inside the library.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("GSMPM_LIB", os.path.join(PKG_ROOT, "libgsmpm.so"))

c_float_p = ctypes.POINTER(ctypes.c_float)
c_void_p = ctypes.c_void_p


class MpmParams(ctypes.Structure):
    _fields_ = [
        ("n_particles", ctypes.c_int32),
        ("n_grid", ctypes.c_int32),
        ("grid_extent", ctypes.c_double),
        ("material", ctypes.c_int32),
        ("E", ctypes.c_double),
        ("nu", ctypes.c_double),
        ("density", ctypes.c_double),
        ("gravity", ctypes.c_double * 3),
        ("yield_stress", ctypes.c_double),
        ("hardening", ctypes.c_double),
        ("xi", ctypes.c_double),
        ("plastic_viscosity", ctypes.c_double),
        ("friction_angle_deg", ctypes.c_double),
        ("flags", ctypes.c_uint32),
    ]


class RasterArgs(ctypes.Structure):
    _fields_ = [
        ("P", ctypes.c_int32), ("D", ctypes.c_int32), ("M", ctypes.c_int32),
        ("W", ctypes.c_int32), ("H", ctypes.c_int32),
        ("means3D", c_void_p), ("shs", c_void_p), ("colors_precomp", c_void_p), ("opacities", c_void_p),
        ("scales", c_void_p), ("rotations", c_void_p), ("cov3D_precomp", c_void_p),
        ("scale_modifier", ctypes.c_float),
        ("viewmatrix", c_void_p), ("projmatrix", c_void_p), ("campos", c_void_p), ("bg", c_void_p),
        ("tanfovx", ctypes.c_float), ("tanfovy", ctypes.c_float),
        ("prefiltered", ctypes.c_int32),
    ]


class FitParams(ctypes.Structure):
    _fields_ = [
        ("n_particles", ctypes.c_int32),
        ("n_grid", ctypes.c_int32),
        ("grid_extent", ctypes.c_double),
        ("levels", ctypes.c_int32),
        ("E", ctypes.c_double),
        ("nu", ctypes.c_double),
        ("density", ctypes.c_double),
        ("gravity", ctypes.c_double * 3),
    ]


# entry point -> (restype, argtypes); mirrors include/gsmpm.h
_SIGS = {
    "gsmpm_last_error": (ctypes.c_char_p, []),
    "gsmpm_version": (ctypes.c_int, []),
    "gsmpm_mpm_create": (ctypes.c_int, [ctypes.POINTER(MpmParams), ctypes.POINTER(c_void_p)]),
    "gsmpm_mpm_destroy": (ctypes.c_int, [c_void_p]),
    "gsmpm_mpm_set_particles": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "gsmpm_mpm_add_fixed_cube": (ctypes.c_int, [c_void_p, ctypes.c_double * 3, ctypes.c_double * 3]),
    "gsmpm_mpm_add_impulse": (ctypes.c_int, [c_void_p, ctypes.c_double * 3, ctypes.c_double * 3,
                                             ctypes.c_double * 3, ctypes.c_double]),
    "gsmpm_mpm_add_plane_collider": (ctypes.c_int, [c_void_p, ctypes.c_double * 3, ctypes.c_double * 3,
                                                    ctypes.c_double]),
    "gsmpm_mpm_step": (ctypes.c_int, [c_void_p, ctypes.c_float, ctypes.c_int32, ctypes.POINTER(ctypes.c_uint32),
                                      c_void_p]),
    "gsmpm_rccl_unique_id": (ctypes.c_int, [c_void_p]),
    "gsmpm_rccl_comm_init": (ctypes.c_int, [c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(c_void_p)]),
    "gsmpm_rccl_comm_destroy": (ctypes.c_int, [c_void_p]),
    "gsmpm_mpm_slab_init": (ctypes.c_int, [c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                           ctypes.c_int32, ctypes.c_int32]),
    "gsmpm_mpm_slab_set_particles": (ctypes.c_int, [c_void_p, ctypes.c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
                                                    c_void_p, c_void_p]),
    "gsmpm_mpm_slab_step": (ctypes.c_int, [c_void_p, ctypes.c_float, ctypes.c_int32, ctypes.POINTER(ctypes.c_uint32),
                                           c_void_p, c_void_p]),
    "gsmpm_mpm_count": (ctypes.c_int, [c_void_p]),
    "gsmpm_mpm_get_gid": (ctypes.c_int, [c_void_p, c_void_p, c_void_p]),
    "gsmpm_mpm_slab_stats": (ctypes.c_int, [c_void_p, ctypes.POINTER(ctypes.c_int64)]),
    "gsmpm_mpm_slab_rects": (ctypes.c_int, [c_void_p, ctypes.POINTER(ctypes.c_int32)]),
    "gsmpm_mpm_slab_set_rebalance": (ctypes.c_int, [c_void_p, ctypes.c_int32, ctypes.c_float]),
    "gsmpm_mpm_slab_set_weight": (ctypes.c_int, [c_void_p, ctypes.c_float]),
    "gsmpm_mpm_slab_bounds": (ctypes.c_int, [c_void_p, ctypes.POINTER(ctypes.c_int32), ctypes.c_int32,
                                             ctypes.POINTER(ctypes.c_int64)]),
    "gsmpm_mpm_resort": (ctypes.c_int, [c_void_p, ctypes.c_int32, c_void_p]),
    "gsmpm_mpm_set_rebin_interval": (ctypes.c_int, [c_void_p, ctypes.c_int32]),
    "gsmpm_mpm_check_finite": (ctypes.c_int, [c_void_p, ctypes.c_int32, c_void_p]),
    "gsmpm_mpm_pipeline": (ctypes.c_int, [c_void_p]),
    "gsmpm_mpm_folded": (ctypes.c_int, [c_void_p]),
    "gsmpm_mpm_rebin_state": (ctypes.c_int, [c_void_p, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_float)]),
    "gsmpm_mpm_escapes": (ctypes.c_int, [c_void_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_int64), c_void_p]),
    "gsmpm_mpm_postprocess": (ctypes.c_int, [c_void_p, c_void_p]),
    "gsmpm_mpm_field_width": (ctypes.c_int, [ctypes.c_int32]),
    "gsmpm_mpm_get": (ctypes.c_int, [c_void_p, ctypes.c_int32, c_void_p, c_void_p]),
    "gsmpm_mpm_set": (ctypes.c_int, [c_void_p, ctypes.c_int32, c_void_p, c_void_p]),
    "gsmpm_mpm_get_grid": (ctypes.c_int, [c_void_p, ctypes.c_int32, c_void_p, c_void_p]),
    "gsmpm_mpm_world_outputs": (ctypes.c_int, [c_void_p, ctypes.c_float, ctypes.c_float * 3, ctypes.c_int32,
                                               c_void_p, c_void_p, c_void_p]),
    "gsmpm_mpm_profile_substeps": (ctypes.c_int, [c_void_p, ctypes.c_float, ctypes.c_int32,
                                                   ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_float),
                                                   c_void_p]),
    "gsmpm_mpm_time_kernels": (ctypes.c_int, [c_void_p, ctypes.c_float, ctypes.c_uint32, ctypes.c_int32,
                                              ctypes.POINTER(ctypes.c_float), c_void_p]),
    "gsmpm_mpm_debug_stats": (ctypes.c_int, [c_void_p, ctypes.POINTER(ctypes.c_int32), c_void_p]),
    "gsmpm_debug_stamps": (ctypes.c_int, [c_void_p, c_void_p]),
    "gsmpm_mpm_live_box": (ctypes.c_int, [c_void_p, ctypes.POINTER(ctypes.c_int32), c_void_p]),
    "gsmpm_svd3": (ctypes.c_int, [c_void_p, ctypes.c_int32, c_void_p, c_void_p, c_void_p, c_void_p]),
    "gsmpm_constitutive": (ctypes.c_int, [ctypes.c_int32, c_void_p, ctypes.c_int32, c_void_p, c_void_p, c_void_p,
                                          ctypes.c_float, c_void_p, c_void_p, c_void_p]),
    "gsmpm_particle_volume": (ctypes.c_int, [c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_double, c_void_p,
                                             c_void_p, c_void_p]),
    "gsmpm_fit_create": (ctypes.c_int, [ctypes.POINTER(FitParams), ctypes.POINTER(c_void_p)]),
    "gsmpm_fit_destroy": (ctypes.c_int, [c_void_p]),
    "gsmpm_fit_set_particles": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "gsmpm_fit_set_fixed_cube": (ctypes.c_int, [c_void_p, ctypes.c_double * 3, ctypes.c_double * 3]),
    "gsmpm_fit_forward": (ctypes.c_int, [c_void_p, ctypes.c_float, ctypes.c_int32, c_void_p]),
    "gsmpm_fit_backward": (ctypes.c_int, [c_void_p, ctypes.c_float, ctypes.c_int32, c_void_p]),
    "gsmpm_fit_postprocess_forward": (ctypes.c_int, [c_void_p, c_void_p]),
    "gsmpm_fit_postprocess_backward": (ctypes.c_int, [c_void_p, c_void_p]),
    "gsmpm_fit_set_grads": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "gsmpm_fit_learn": (ctypes.c_int, [c_void_p, c_void_p]),
    "gsmpm_fit_cycle_init": (ctypes.c_int, [c_void_p, c_void_p]),
    "gsmpm_fit_clear_grads": (ctypes.c_int, [c_void_p, c_void_p]),
    "gsmpm_fit_mu_lam": (ctypes.c_int, [c_void_p, c_void_p]),
    "gsmpm_fit_field_width": (ctypes.c_int, [ctypes.c_int32]),
    "gsmpm_fit_get": (ctypes.c_int, [c_void_p, ctypes.c_int32, ctypes.c_int32, c_void_p, c_void_p]),
    "gsmpm_fit_set": (ctypes.c_int, [c_void_p, ctypes.c_int32, ctypes.c_int32, c_void_p, c_void_p]),
    "gsmpm_fit_get_grid": (ctypes.c_int, [c_void_p, ctypes.c_int32, c_void_p, c_void_p]),
    "gsmpm_raster_create": (ctypes.c_int, [ctypes.POINTER(c_void_p)]),
    "gsmpm_raster_destroy": (ctypes.c_int, [c_void_p]),
    "gsmpm_raster_forward": (ctypes.c_int, [c_void_p, ctypes.POINTER(RasterArgs), c_void_p, c_void_p,
                                            ctypes.POINTER(ctypes.c_int32), c_void_p]),
    "gsmpm_raster_backward": (ctypes.c_int, [c_void_p, ctypes.POINTER(RasterArgs), c_void_p, c_void_p] +
                              [c_void_p] * 8 + [c_void_p]),
    "gsmpm_raster_mark_visible": (ctypes.c_int, [c_void_p, ctypes.c_int32, c_void_p, c_void_p, c_void_p, c_void_p]),
    "gsmpm_raster_set_forward_only": (ctypes.c_int, [c_void_p, ctypes.c_int32]),
    "gsmpm_raster_pair_counts": (ctypes.c_int, [c_void_p, c_void_p, c_void_p]),
    "gsmpm_raster_dsort_stats": (ctypes.c_int, [c_void_p, c_void_p]),
    "gsmpm_raster_workspace_size": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64,
                                                   ctypes.POINTER(ctypes.c_uint64)]),
    "gsmpm_raster_forward_ws": (ctypes.c_int, [ctypes.POINTER(RasterArgs), c_void_p, c_void_p,
                                               ctypes.POINTER(ctypes.c_int32), c_void_p, ctypes.c_uint64,
                                               ctypes.POINTER(ctypes.c_int64), c_void_p]),
    "gsmpm_raster_forward_async": (ctypes.c_int, [ctypes.POINTER(RasterArgs), c_void_p, c_void_p, c_void_p,
                                                  ctypes.c_uint64, ctypes.c_int64, c_void_p, c_void_p]),
    "gsmpm_raster_set_timing": (ctypes.c_int, [ctypes.c_int32]),
    "gsmpm_raster_timing": (ctypes.c_int, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(ctypes.c_int64)]),
}
GSMPM_OK, GSMPM_EINVAL, GSMPM_EHIP, GSMPM_ESTATE = 0, -1, -2, -3
ESPACE = GSMPM_ESPACE = -4  # a caller-owned workspace is too small

# slab transports (include/gsmpm.h)
XPORT_NONE, XPORT_RCCL, XPORT_CALLBACK = 0, 1, 2
EXCHANGE_FN = ctypes.CFUNCTYPE(ctypes.c_int, c_void_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32),
                               ctypes.POINTER(c_void_p), ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(c_void_p),
                               ctypes.POINTER(ctypes.c_size_t))


class Transport(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("rank", ctypes.c_int32), ("world", ctypes.c_int32), ("comm", c_void_p),
                ("fn", EXCHANGE_FN), ("user", c_void_p)]


# field ids (include/gsmpm.h)
FIELD = {"x": 0, "v": 1, "C": 2, "F_trial": 3, "cov": 4, "init_cov": 5, "R": 6, "mass": 7, "vol": 8, "mu": 9,
         "lam": 10, "yield_stress": 11}
FIT_FIELD = {k: i for i, k in enumerate(
    ("x", "v", "F", "C", "stress", "gx", "gv", "gF", "gC", "gstress", "logE", "y", "mu", "lam", "glogE", "gy", "gmu",
     "glam", "cov", "gcov", "init_cov", "vol", "mass"))}
FLAG_JELLY_FCR, FLAG_KEEP_GRID, FLAG_NO_GRAPH, FLAG_NO_SORT, FLAG_PHASED = 1, 2, 4, 8, 16
PIPE_PHASED, PIPE_FUSED = 0, 1


class GsmpmError(RuntimeError):
    pass


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libgsmpm.so not found at {LIB_PATH}: the HIP extension is the only compute path; "
            "build it with `python -c 'import __graft_entry__ as g; g.build()'` (or make -C "
            "gaussian-splatting-mpm_amd/csrc)")
    L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in _SIGS.items():
        fn = getattr(L, name)  # AttributeError here = ABI drift between header and library
        fn.restype = res
        fn.argtypes = args
    return L


LIB = _load()


def last_error() -> str:
    msg = LIB.gsmpm_last_error()
    return msg.decode() if msg else ""


def check(rc: int, what: str = "") -> int:
    if rc < 0:
        raise GsmpmError(f"{what}: {last_error()} (status {rc})")
    return rc


def ptr(t) -> int | None:
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError("expected a device (cuda/hip) tensor")
    if not t.is_contiguous():
        raise ValueError("expected a contiguous tensor")
    return t.data_ptr()


def stream_of(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream
