"""Torch-facing wrapper of the rasterizer C-ABI (gsmpm_raster_*)."""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import LIB, check, ptr, stream_of

_CTX = {}


class SharedContext:
    """A forward-only library-owned context (gsmpm_raster_create): its buffers
    grow inside the library.  The default forward uses a caller-owned
    workspace instead (Workspace); this form remains for the diagnostics
    (pair_counts) and as the C-ABI's context entry point."""

    def __init__(self):
        self.h = ctypes.c_void_p()
        check(LIB.gsmpm_raster_create(ctypes.byref(self.h)), "gsmpm_raster_create")
        check(LIB.gsmpm_raster_set_forward_only(self.h, 1), "gsmpm_raster_set_forward_only")


def shared_context(device_index: int = 0) -> SharedContext:
    c = _CTX.get(device_index)
    if c is None:
        c = _CTX[device_index] = SharedContext()
    return c


def pair_counts(context) -> tuple:
    """(binned pairs, num_rendered) of `context`'s last forward (diagnostics:
    the tight binning's pair count vs the 3-sigma one)."""
    b, n = ctypes.c_uint32(), ctypes.c_uint32()
    check(LIB.gsmpm_raster_pair_counts(context.h, ctypes.byref(b), ctypes.byref(n)), "gsmpm_raster_pair_counts")
    return int(b.value), int(n.value)


def dsort_stats(context) -> dict:
    """The hand-written depth order's diagnostics for `context`'s last forward (csrc/dsort.h)."""
    o = (ctypes.c_int64 * 8)()
    check(LIB.gsmpm_raster_dsort_stats(context.h, o), "gsmpm_raster_dsort_stats")
    return dict(zip(("buckets", "wave_buckets", "wg_buckets", "max_bucket", "overflow", "visible", "fallbacks",
                     "shift"), list(o)))


class Workspace:
    """A caller-owned rasterizer workspace: one torch byte tensor
    (gsmpm_raster_workspace_size / gsmpm_raster_forward_ws), as upstream's
    RasterizeGaussiansCUDA keeps its geometry / binning / image buffers in
    torch byte tensors.  Sized for the last frame's Gaussians, image and
    binned pairs; when a frame bins more pairs than it holds, the library
    reports how many (GSMPM_ESPACE) and the forward is repeated once on a
    workspace grown for 1.25x that many."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.buf = None
        self.key = None  # (P, H, W, pairs) the buffer is sized for

    def ensure(self, P, H, W, pairs):
        if self.key is not None and self.key[0] >= P and self.key[1:3] == (H, W) and self.key[3] >= pairs:
            return
        if self.key is not None and self.key[1:3] == (H, W):
            P, pairs = max(P, self.key[0]), max(pairs, self.key[3])
        nb = ctypes.c_uint64()
        check(LIB.gsmpm_raster_workspace_size(int(P), int(H), int(W), int(pairs), ctypes.byref(nb)),
              "gsmpm_raster_workspace_size")
        if self.buf is not None:
            # the old buffer may still be in use by kernels queued on this stream
            # (GSMPM_ESPACE returns with the depth-order kernels queued): the
            # caching allocator must not hand it out before they finish
            self.buf.record_stream(torch.cuda.current_stream(self.device))
        self.buf = None  # release before allocating the larger one
        # zero-filled once: the library keeps its depth-order state zero between forwards (csrc/dsort.h)
        self.buf = torch.zeros(int(nb.value) + 256, dtype=torch.uint8, device=self.device)
        self.key = (P, H, W, pairs)

    def ptr(self):
        a = self.buf.data_ptr()
        return (a + 255) & ~255  # 256-byte aligned start

    def nbytes(self):
        return self.buf.numel() - (self.ptr() - self.buf.data_ptr())


_WS = __import__("collections").OrderedDict()  # (device, stream handle) -> Workspace, least recently used first
_WS_LOCK = __import__("threading").Lock()
_WS_KEEP = 8  # default workspaces kept; a process cycling through more streams evicts the oldest


def _drop_workspace(device_index: int):
    # the evicted workspace may still be in use by a forward queued on its stream:
    # let the device drain before its buffer goes back to the allocator
    torch.cuda.synchronize(torch.device("cuda", device_index))


def workspace(device_index: int = 0, stream=None) -> Workspace:
    """The default workspace of (device, stream).  One per stream: the library
    keeps the workspace's depth-order state zero between forwards
    (csrc/dsort.h), which holds only while its forwards are ordered, so two
    streams (e.g. bench's render worker and the default stream) never share
    one.  At most _WS_KEEP are kept (least recently used evicted, after a
    device sync), so short-lived streams do not leak workspaces;
    release_workspace(stream) drops one explicitly."""
    if stream is None:
        stream = torch.cuda.current_stream(torch.device("cuda", device_index))
    key = (device_index, int(stream.cuda_stream))
    evict = []
    with _WS_LOCK:
        w = _WS.get(key)
        if w is None:
            w = _WS[key] = Workspace(torch.device("cuda", device_index))
            while len(_WS) > _WS_KEEP:
                evict.append(_WS.popitem(last=False))
        else:
            _WS.move_to_end(key)
    for (dev, _), _w in evict:
        _drop_workspace(dev)
    return w


def release_workspace(stream=None, device_index: int = 0) -> bool:
    """Drop the default workspace of (device, stream), e.g. before the stream
    is destroyed (a later stream could otherwise get the same handle and with
    it this workspace).  Returns whether one was held."""
    if stream is None:
        stream = torch.cuda.current_stream(torch.device("cuda", device_index))
    key = (device_index, int(stream.cuda_stream))
    with _WS_LOCK:
        w = _WS.pop(key, None)
    if w is not None:
        _drop_workspace(device_index)
    return w is not None


class RasterContext:
    """A dedicated gsmpm_raster context: holds one forward's binning and
    per-pixel state until its backward (upstream keeps geom/binning/image
    buffers in the autograd context for the same reason)."""

    def __init__(self):
        self.h = ctypes.c_void_p()
        check(LIB.gsmpm_raster_create(ctypes.byref(self.h)), "gsmpm_raster_create")

    def __del__(self):
        # LIB is None when the interpreter tears the module down before this object
        if getattr(self, "h", None) is not None and self.h.value and LIB is not None:
            LIB.gsmpm_raster_destroy(self.h)
            self.h = None


_POOL = {}   # device index -> idle RasterContexts (buffers kept grown)
_POOL_KEEP = 4


class ContextLease:
    """A pooled RasterContext for one forward + backward.  Contexts are reused
    across training iterations instead of created and destroyed per call
    (creation is a pinned allocation plus ~20 device allocations, and the
    destroy's hipFree synchronises the device).  The context goes back to the
    pool on release() or when the lease is dropped (autograd graph freed
    without a backward)."""

    def __init__(self, device_index: int):
        self.dev = device_index
        idle = _POOL.setdefault(device_index, [])
        self.context = idle.pop() if idle else RasterContext()

    def release(self):
        c, self.context = getattr(self, "context", None), None
        if c is not None:
            idle = _POOL.setdefault(self.dev, [])
            if len(idle) < _POOL_KEEP:
                idle.append(c)

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass


def _f32(t):
    if t is None:
        return None
    if t.numel() == 0:
        return None
    return t.detach().to(torch.float32).contiguous()


def _args(means3D, opacities, viewmatrix, projmatrix, campos, bg, image_height, image_width, tanfovx, tanfovy,
          sh_degree, shs, colors_precomp, scales, rotations, cov3D_precomp, scale_modifier, prefiltered):
    """(RasterArgs, the f32 tensors it points into)."""
    means3D = _f32(means3D)
    P = means3D.shape[0] if means3D is not None else 0
    shs, colors_precomp = _f32(shs), _f32(colors_precomp)
    scales, rotations, cov3D_precomp = _f32(scales), _f32(rotations), _f32(cov3D_precomp)
    opacities = _f32(opacities)
    vm, pm, cp, bgc = _f32(viewmatrix), _f32(projmatrix), _f32(campos), _f32(bg)
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
    keep = dict(means3D=means3D, shs=shs, colors_precomp=colors_precomp, scales=scales, rotations=rotations,
                cov3D_precomp=cov3D_precomp, opacities=opacities, vm=vm, pm=pm, cp=cp, bg=bgc)
    return a, keep


def backward(context, keep, a, radii, grad_color):
    """gsmpm_raster_backward on the state of `context`'s forward.  Returns a dict of
    means2D [P,3], colors [P,3], opacity [P], means3D [P,3], cov3D [P,6],
    sh [P,M,3] | None, scales [P,3] | None, rotations [P,4] | None."""
    dev = keep["means3D"].device
    P = a.P
    z = lambda *shape: torch.empty(shape, dtype=torch.float32, device=dev)
    g = {"means2D": z(P, 3), "colors": z(P, 3), "opacity": z(P), "means3D": z(P, 3), "cov3D": z(P, 6),
         "sh": z(P, a.M, 3) if keep["shs"] is not None else None,
         "scales": z(P, 3) if keep["scales"] is not None else None,
         "rotations": z(P, 4) if keep["rotations"] is not None else None}
    grad_color = grad_color.detach().to(torch.float32).contiguous()
    with torch.cuda.device(dev):
        check(LIB.gsmpm_raster_backward(context.h, ctypes.byref(a), ptr(radii), ptr(grad_color), ptr(g["means2D"]),
                                        ptr(g["colors"]), ptr(g["opacity"]), ptr(g["means3D"]), ptr(g["cov3D"]),
                                        ptr(g["sh"]), ptr(g["scales"]), ptr(g["rotations"]), stream_of(dev)),
              "rasterize_gaussians_backward")
    return g


def forward(means3D, opacities, viewmatrix, projmatrix, campos, bg, image_height, image_width, tanfovx, tanfovy,
            sh_degree=0, shs=None, colors_precomp=None, scales=None, rotations=None, cov3D_precomp=None,
            scale_modifier=1.0, prefiltered=False, context=None, return_args=False, ws=None):
    """Returns (num_rendered, color [3,H,W], radii [P] int32) [+ (args, kept tensors)
    when return_args].  `context` (a RasterContext, or a SharedContext) keeps
    this forward's state (for `backward`, or the diagnostics); by default the
    forward runs in the device's caller-owned Workspace (or `ws`)."""
    dev = means3D.device
    a, keep = _args(means3D, opacities, viewmatrix, projmatrix, campos, bg, image_height, image_width, tanfovx,
                    tanfovy, sh_degree, shs, colors_precomp, scales, rotations, cov3D_precomp, scale_modifier,
                    prefiltered)
    P = a.P
    color = torch.empty((3, image_height, image_width), dtype=torch.float32, device=dev)
    radii = torch.empty(P, dtype=torch.int32, device=dev)  # k_preprocess writes every entry (0 when culled)
    nr = ctypes.c_int32(0)
    if P == 0:
        # nothing to splat: the image is the background (upstream behaviour)
        color[:] = keep["bg"].view(3, 1, 1)
    elif context is not None:
        with torch.cuda.device(dev):
            check(LIB.gsmpm_raster_forward(context.h, ctypes.byref(a), ptr(color), ptr(radii), ctypes.byref(nr),
                                           stream_of(dev)), "rasterize_gaussians")
    else:
        w = ws if ws is not None else workspace(dev.index or 0, torch.cuda.current_stream(dev))
        H, W = int(image_height), int(image_width)
        w.ensure(P, H, W, w.key[3] if w.key else 8 * P + 4096)
        need = ctypes.c_int64(0)
        with torch.cuda.device(dev):
            for attempt in range(2):
                rc = LIB.gsmpm_raster_forward_ws(ctypes.byref(a), ptr(color), ptr(radii), ctypes.byref(nr), w.ptr(),
                                                 w.nbytes(), ctypes.byref(need), stream_of(dev))
                if rc != _lib.ESPACE or attempt == 1:
                    break
                w.ensure(P, H, W, int(need.value) + int(need.value) // 4 + 1024)
            check(rc, "rasterize_gaussians")
    if return_args:
        return int(nr.value), color, radii, a, keep
    return int(nr.value), color, radii


class AsyncRender:
    """One in-flight render of forward_async: the image and radii it writes and
    its counts {K, num_rendered, flags, internal} in pinned host memory, valid
    once the stream has passed the render (done())."""

    def __init__(self, color, radii, counts, event, args):
        self.color, self.radii, self.counts, self.event, self._args = color, radii, counts, event, args

    def done(self) -> bool:
        return self.event is None or self.event.query()

    def result(self):
        """(num_rendered, flags) after the stream reached it (waits for it)."""
        if self.event is not None:
            self.event.synchronize()
        c = self.counts.tolist()
        return int(c[1]), int(c[2])

    @property
    def valid(self) -> bool:
        return self.result()[1] == 0


def forward_async(means3D, opacities, viewmatrix, projmatrix, campos, bg, image_height, image_width, tanfovx, tanfovy,
                  sh_degree=0, shs=None, colors_precomp=None, cov3D_precomp=None, scales=None, rotations=None,
                  scale_modifier=1.0, pairs_cap=None, ws=None, counts=None, color=None, radii=None):
    """gsmpm_raster_forward_async: the forward with no host synchronisation
    (the pair count stays on the device; buffers carved for pairs_cap pairs,
    default the workspace's).  Returns an AsyncRender; a frame whose flags
    are set (a depth bucket overflow, or more pairs than pairs_cap) must be
    rendered again by forward()."""
    dev = means3D.device
    a, keep = _args(means3D, opacities, viewmatrix, projmatrix, campos, bg, image_height, image_width, tanfovx,
                    tanfovy, sh_degree, shs, colors_precomp, scales, rotations, cov3D_precomp, scale_modifier, False)
    H, W = int(image_height), int(image_width)
    color = torch.empty((3, H, W), dtype=torch.float32, device=dev) if color is None else color
    radii = torch.empty(a.P, dtype=torch.int32, device=dev) if radii is None else radii
    counts = torch.zeros(4, dtype=torch.int32, pin_memory=True) if counts is None else counts
    w = ws if ws is not None else workspace(dev.index or 0, torch.cuda.current_stream(dev))
    cap = int(pairs_cap) if pairs_cap else (w.key[3] if w.key else 8 * a.P + 4096)
    w.ensure(a.P, H, W, cap)
    with torch.cuda.device(dev):
        check(LIB.gsmpm_raster_forward_async(ctypes.byref(a), ptr(color), ptr(radii), w.ptr(), w.nbytes(), cap,
                                             ctypes.c_void_p(counts.data_ptr()), stream_of(dev)),
              "rasterize_gaussians (async)")
        ev = None
        if not torch.cuda.is_current_stream_capturing():  # a graph replay is waited on by its caller
            ev = torch.cuda.Event()
            ev.record()
    return AsyncRender(color, radii, counts, ev, (a, keep))


def set_timing(on):
    """gsmpm_raster_set_timing: record k_render's and each forward's in-stream
    time from now on (process-wide; forwards under a stream capture excluded)."""
    check(LIB.gsmpm_raster_set_timing(1 if on else 0), "set_timing")


def timing():
    """gsmpm_raster_timing: (k_render ms, whole forward ms, forwards) summed
    over the forwards recorded since the last call (waits for them)."""
    kr, fw, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
    check(LIB.gsmpm_raster_timing(ctypes.byref(kr), ctypes.byref(fw), ctypes.byref(n)), "timing")
    return kr.value, fw.value, n.value


def mark_visible(positions, viewmatrix, projmatrix):
    positions = _f32(positions)
    P = positions.shape[0]
    vis = torch.zeros(P, dtype=torch.uint8, device=positions.device)
    if P:
        check(LIB.gsmpm_raster_mark_visible(ptr(positions), P, ptr(_f32(viewmatrix)), ptr(_f32(projmatrix)),
                                            ptr(vis), stream_of(positions.device)), "mark_visible")
    return vis.bool()
