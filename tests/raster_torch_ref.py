"""Float64 torch restatement of the rasterizer forward, differentiated by
autograd -- the check for the hand-derived backward (oracle/raster_oracle.c
or_backward, and through it the HIP kernels).  Test infrastructure.

Same math as the forward (oracle/raster_oracle.c, Appendix B of SURVEY),
with upstream's two gradient conventions expressed as autograd rules:
  * alpha = min(0.99, o G) passes the gradient of o G (straight-through);
  * the 1.3 x fov clamp of t: a clamped t.x (t.y) is a constant.
The discrete decisions (frustum/radius culling, tile membership, depth order,
alpha < 1/255 skips, the T < 1e-4 stop) are made once on detached values.
dL/dmeans2D is read at the NDC position, as upstream returns it.
"""
from __future__ import annotations

import math

import numpy as np
import torch

SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396]
SH_C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
         1.445305721320277, -0.5900435899266435]


def _sh(D, sh, d):
    x, y, z = d[:, 0:1], d[:, 1:2], d[:, 2:3]
    r = SH_C0 * sh[:, 0]
    if D > 0:
        r = r - SH_C1 * y * sh[:, 1] + SH_C1 * z * sh[:, 2] - SH_C1 * x * sh[:, 3]
    if D > 1:
        xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
        r = (r + SH_C2[0] * xy * sh[:, 4] + SH_C2[1] * yz * sh[:, 5] + SH_C2[2] * (2 * zz - xx - yy) * sh[:, 6]
             + SH_C2[3] * xz * sh[:, 7] + SH_C2[4] * (xx - yy) * sh[:, 8])
    if D > 2:
        r = (r + SH_C3[0] * y * (3 * xx - yy) * sh[:, 9] + SH_C3[1] * xy * z * sh[:, 10]
             + SH_C3[2] * y * (4 * zz - xx - yy) * sh[:, 11] + SH_C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[:, 12]
             + SH_C3[4] * x * (4 * zz - xx - yy) * sh[:, 13] + SH_C3[5] * z * (xx - yy) * sh[:, 14]
             + SH_C3[6] * x * (xx - 3 * yy) * sh[:, 15])
    return r + 0.5


def _cov_from_sr(s, mod, q):
    S = mod * s
    r, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y),
                     2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x),
                     2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], 1).view(-1, 3, 3)
    M = R * S[:, None, :]
    Sg = M @ M.transpose(1, 2)
    return torch.stack([Sg[:, 0, 0], Sg[:, 0, 1], Sg[:, 0, 2], Sg[:, 1, 1], Sg[:, 1, 2], Sg[:, 2, 2]], 1)


def forward(inp, W, H, tanx, tany, D=3, scale_modifier=1.0):
    """inp: dict of float64 leaf tensors (means3D, opacities, viewmatrix, projmatrix,
    campos, bg, and shs or colors_precomp, cov3D_precomp or scales+rotations).
    Returns (image (3,H,W), ndc (P,2) with retain_grad, radii np.int, stats dict)."""
    m = inp["means3D"]
    P = m.shape[0]
    vm, pm = inp["viewmatrix"], inp["projmatrix"]
    fx, fy = W / (2 * tanx), H / (2 * tany)
    hom = torch.cat([m, torch.ones(P, 1, dtype=m.dtype)], 1)
    t = hom @ vm[:, :3]          # view space (matrices are transposed, row vectors)
    ph = hom @ pm
    pw = 1.0 / (ph[:, 3] + 1e-7)
    ndc = torch.stack([ph[:, 0] * pw, ph[:, 1] * pw], 1)
    ndc.retain_grad()
    px = ((ndc[:, 0] + 1.0) * W - 1.0) * 0.5
    py = ((ndc[:, 1] + 1.0) * H - 1.0) * 0.5
    c6 = inp["cov3D_precomp"] if "cov3D_precomp" in inp else _cov_from_sr(inp["scales"], scale_modifier,
                                                                            inp["rotations"])
    limx, limy = 1.3 * tanx, 1.3 * tany
    tz = t[:, 2]
    txtz, tytz = t[:, 0] / tz, t[:, 1] / tz
    cx = (txtz < -limx) | (txtz > limx)
    cy = (tytz < -limy) | (tytz > limy)
    tx = torch.where(cx, (txtz.clamp(-limx, limx) * tz).detach(), t[:, 0])
    ty = torch.where(cy, (tytz.clamp(-limy, limy) * tz).detach(), t[:, 1])
    J00, J02 = fx / tz, -(fx * tx) / (tz * tz)
    J11, J12 = fy / tz, -(fy * ty) / (tz * tz)
    Wm = vm[:3, :3].T             # math rotation, W[r][c] = vm[c*4 + r]
    T0 = J00[:, None] * Wm[0] + J02[:, None] * Wm[2]
    T1 = J11[:, None] * Wm[1] + J12[:, None] * Wm[2]
    V = torch.stack([c6[:, 0], c6[:, 1], c6[:, 2], c6[:, 1], c6[:, 3], c6[:, 4], c6[:, 2], c6[:, 4], c6[:, 5]],
                    1).view(-1, 3, 3)
    VT0, VT1 = (V @ T0[:, :, None])[..., 0], (V @ T1[:, :, None])[..., 0]
    a = (T0 * VT0).sum(1) + 0.3
    b = (T0 * VT1).sum(1)
    c = (T1 * VT1).sum(1) + 0.3
    det = a * c - b * b
    con = torch.stack([c / det, -b / det, a / det], 1)
    if "shs" in inp:
        d = m - inp["campos"]
        d = d / d.norm(dim=1, keepdim=True)
        raw = _sh(D, inp["shs"], d)
        rgb = torch.clamp(raw, min=0.0)   # torch's clamp: zero gradient where clamped (upstream's rule)
    else:
        rgb = inp["colors_precomp"]
    opa = inp["opacities"].view(-1)
    # ---- discrete decisions, as the forward makes them
    with torch.no_grad():
        mid = 0.5 * (a + c)
        l1 = mid + torch.sqrt(torch.clamp(mid * mid - det, min=0.1))
        rad = torch.ceil(3 * torch.sqrt(l1)).long().numpy()
        gx, gy = (W + 15) // 16, (H + 15) // 16
        keep = (tz.detach().numpy() > 0.2) & (det.numpy() != 0)
        rect = []
        for i in range(P):
            r = int(rad[i])
            x0 = min(gx, max(0, int((px[i].item() - r) / 16)))
            y0 = min(gy, max(0, int((py[i].item() - r) / 16)))
            x1 = min(gx, max(0, int((px[i].item() + r + 15) / 16)))
            y1 = min(gy, max(0, int((py[i].item() + r + 15) / 16)))
            rect.append((x0, y0, x1, y1))
            keep[i] &= (x1 - x0) * (y1 - y0) > 0
        order = sorted([i for i in range(P) if keep[i]], key=lambda i: (tz[i].item(), i))
    radii = np.where(keep, rad, 0)
    bg = inp["bg"]
    out = [[None] * W for _ in range(H)]
    stats = {"alpha_clamped": 0, "t_clamped": int((cx | cy).sum()), "pairs": 0}
    for yy in range(H):
        for xx in range(W):
            tile = (xx // 16, yy // 16)
            ids = [i for i in order if rect[i][0] <= tile[0] < rect[i][2] and rect[i][1] <= tile[1] < rect[i][3]]
            Tv = torch.ones((), dtype=m.dtype)
            col = torch.zeros(3, dtype=m.dtype)
            for i in ids:
                dx, dy = px[i] - xx, py[i] - yy
                power = -0.5 * (con[i, 0] * dx * dx + con[i, 2] * dy * dy) - con[i, 1] * dx * dy
                if power.item() > 0:
                    continue
                G = torch.exp(power)
                oG = opa[i] * G
                alpha = oG - torch.clamp(oG - 0.99, min=0.0).detach()
                stats["alpha_clamped"] += int(oG.item() > 0.99)
                stats["pairs"] += 1
                if alpha.item() < 1.0 / 255.0:
                    continue
                test_T = Tv * (1 - alpha)
                if test_T.item() < 1e-4:
                    break
                col = col + rgb[i] * alpha * Tv
                Tv = test_T
            out[yy][xx] = col + Tv * bg
    img = torch.stack([torch.stack(row, 1) for row in out], 1)
    return img, ndc, radii, stats
