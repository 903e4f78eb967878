"""Torch-facing wrapper of the rasterizer C-ABI (gsmpm_raster_*)."""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import LIB, check, ptr, stream_of

_CTX = {}


def _context(device_index: int):
    h = _CTX.get(device_index)
    if h is None:
        h = ctypes.c_void_p()
        check(LIB.gsmpm_raster_create(ctypes.byref(h)), "gsmpm_raster_create")
        _CTX[device_index] = h
    return h


def _f32(t):
    if t is None:
        return None
    if t.numel() == 0:
        return None
    return t.detach().to(torch.float32).contiguous()


def forward(means3D, opacities, viewmatrix, projmatrix, campos, bg, image_height, image_width, tanfovx, tanfovy,
            sh_degree=0, shs=None, colors_precomp=None, scales=None, rotations=None, cov3D_precomp=None,
            scale_modifier=1.0, prefiltered=False):
    """Returns (num_rendered, color [3,H,W], radii [P] int32)."""
    dev = means3D.device
    means3D = _f32(means3D)
    P = means3D.shape[0] if means3D is not None else 0
    shs, colors_precomp = _f32(shs), _f32(colors_precomp)
    scales, rotations, cov3D_precomp = _f32(scales), _f32(rotations), _f32(cov3D_precomp)
    opacities = _f32(opacities)
    vm, pm, cp, bgc = _f32(viewmatrix), _f32(projmatrix), _f32(campos), _f32(bg)
    color = torch.empty((3, image_height, image_width), dtype=torch.float32, device=dev)
    radii = torch.zeros(P, dtype=torch.int32, device=dev)
    a = _lib.RasterArgs()
    a.P, a.D = P, int(sh_degree)
    a.M = 0 if shs is None else int(shs.reshape(P, -1, 3).shape[1]) if P > 0 else 0
    a.W, a.H = int(image_width), int(image_height)
    a.means3D = ptr(means3D) if P > 0 else None
    a.shs = ptr(shs)
    a.colors_precomp = ptr(colors_precomp)
    a.opacities = ptr(opacities) if P > 0 else None
    a.scales, a.rotations, a.cov3D_precomp = ptr(scales), ptr(rotations), ptr(cov3D_precomp)
    a.scale_modifier = float(scale_modifier)
    a.viewmatrix, a.projmatrix, a.campos, a.bg = ptr(vm), ptr(pm), ptr(cp), ptr(bgc)
    a.tanfovx, a.tanfovy = float(tanfovx), float(tanfovy)
    a.prefiltered = int(bool(prefiltered))
    if P == 0:
        # nothing to splat: the image is the background (upstream behaviour)
        color[:] = bgc.view(3, 1, 1)
        return 0, color, radii
    nr = ctypes.c_int32(0)
    with torch.cuda.device(dev):
        check(LIB.gsmpm_raster_forward(_context(dev.index or 0), ctypes.byref(a), ptr(color), ptr(radii),
                                       ctypes.byref(nr), stream_of(dev)), "rasterize_gaussians")
    return int(nr.value), color, radii


def mark_visible(positions, viewmatrix, projmatrix):
    positions = _f32(positions)
    P = positions.shape[0]
    vis = torch.zeros(P, dtype=torch.uint8, device=positions.device)
    if P:
        check(LIB.gsmpm_raster_mark_visible(ptr(positions), P, ptr(_f32(viewmatrix)), ptr(_f32(projmatrix)),
                                            ptr(vis), stream_of(positions.device)), "mark_visible")
    return vis.bool()
