"""Drop-in for the ``diff_gaussian_rasterization`` package (forward path).

Same Python surface as the graphdeco-inria extension the reference imports at
main.py:16 / extra.py:16 (pre-2024 API: the forward returns ``(color, radii)``,
consumed as ``rendered_image, _ = rasterizer(...)`` at main.py:148), backed by
the HIP kernels in libgsmpm.so.  The backward (upstream's
_RasterizeGaussians.backward, used by extra.py's loss.backward()) returns the
gradients of means3D, means2D (w.r.t. NDC, as upstream), shs / colors_precomp,
opacities, scales / rotations or cov3D_precomp; a forward that needs them runs
on a context of its own (leased from a per-device pool) that keeps its
binning and per-pixel state until the backward.
"""
from __future__ import annotations

from typing import NamedTuple

import torch
import torch.nn as nn

from gsmpm import raster as _raster


class GaussianRasterizationSettings(NamedTuple):
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool
    debug: bool


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                        raster_settings):
    return _RasterizeGaussians.apply(means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                                     cov3Ds_precomp, raster_settings)


def _opt(t):
    return None if t is None or t.numel() == 0 else t


class _RasterizeGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                raster_settings):
        s = raster_settings
        kw = dict(sh_degree=s.sh_degree, shs=_opt(sh), colors_precomp=_opt(colors_precomp), scales=_opt(scales),
                  rotations=_opt(rotations), cov3D_precomp=_opt(cov3Ds_precomp), scale_modifier=s.scale_modifier,
                  prefiltered=s.prefiltered)
        args = (means3D, opacities.reshape(-1), s.viewmatrix, s.projmatrix, s.campos, s.bg, s.image_height,
                s.image_width, s.tanfovx, s.tanfovy)
        if any(ctx.needs_input_grad[:8]):
            lease = _raster.ContextLease(means3D.device.index or 0)
            num_rendered, color, radii, a, keep = _raster.forward(*args, **kw, context=lease.context,
                                                                  return_args=True)
            ctx.state = (lease, a, keep, radii)
            ctx.shapes = [None if t is None else (t.shape, t.dtype) for t in
                          (means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp)]
        else:
            num_rendered, color, radii = _raster.forward(*args, **kw)
        ctx.num_rendered = num_rendered
        ctx.mark_non_differentiable(radii)
        return color, radii

    @staticmethod
    def backward(ctx, grad_out_color, _):
        lease, a, keep, radii = ctx.state
        shp = ctx.shapes
        P = a.P

        def cast(t, i):
            if t is None or shp[i] is None or shp[i][0].numel() == 0 or not ctx.needs_input_grad[i]:
                return None
            return t.reshape(shp[i][0]).to(shp[i][1])
        if P == 0:
            return (None,) * 9
        g = _raster.backward(lease.context, keep, a, radii, grad_out_color)
        lease.release()  # back to the pool: the next iteration's forward reuses its buffers
        ctx.state = None
        return (cast(g["means3D"], 0), cast(g["means2D"], 1), cast(g["sh"], 2), cast(g["colors"], 3),
                cast(g["opacity"], 4), cast(g["scales"], 5), cast(g["rotations"], 6), cast(g["cov3D"], 7), None)


class GaussianRasterizer(nn.Module):
    def __init__(self, raster_settings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions):
        with torch.no_grad():
            s = self.raster_settings
            return _raster.mark_visible(positions, s.viewmatrix, s.projmatrix)

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
                cov3D_precomp=None):
        s = self.raster_settings
        if (shs is None and colors_precomp is None) or (shs is not None and colors_precomp is not None):
            raise Exception("Please provide excatly one of either SHs or precomputed colors!")
        if ((scales is None or rotations is None) and cov3D_precomp is None) or \
                ((scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception("Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!")
        empty = torch.Tensor([])
        return rasterize_gaussians(means3D, means2D, empty if shs is None else shs,
                                   empty if colors_precomp is None else colors_precomp, opacities,
                                   empty if scales is None else scales, empty if rotations is None else rotations,
                                   empty if cov3D_precomp is None else cov3D_precomp, s)
