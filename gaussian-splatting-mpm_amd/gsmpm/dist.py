"""Multi-GPU MPM: one scene cut into spatial slabs, one rank per GPU.

SURVEY.md 8(e).  The reference runs its substep (mpm_solver/solver.py:27-52)
on one device (main.py:28); here it is sharded by slab along grid axis 0
(csrc/slab.h has the kernels, csrc/slab_host.inc the per-substep sequence):

* ``slab_bounds`` cuts the planes [0, n_grid) into ``world`` slabs of about
  equal particle count (quantiles of the particles' base planes,
  trunc(x * inv_dx - 0.5), utils.py:95), each at least 2 * margin + 2 planes
  thick.  Rank r owns planes [bounds[r], bounds[r+1]) and the particles whose
  base plane lies there.
* Every substep the partial (m v, m) sums of the 2 * margin + 2 planes around
  each shared bound are swapped with the neighbour and both sides update the
  node from the same f32 sum (lower rank's partial + upper rank's): the
  pairwise all-reduce of boundary grid nodes, over RCCL (``RcclTransport``,
  grouped ncclSend/ncclRecv on the simulator's comm stream, overlapping the
  interior grid update) or, for tests, a host callback over
  torch.distributed (``CallbackTransport``, gloo).
* Every ``interval`` substeps the particles whose base plane left the slab
  migrate to the neighbour (wave-ballot compaction on the GPU, counts then
  payloads through the transport).  A particle drifting more than ``margin``
  planes between migrations would have scattered outside the exchanged
  windows; the library detects it (and a slab over capacity) and ``step``
  raises on every rank at the same migration, since every rank's migration
  record goes to every rank.

``SlabDomain`` is one rank's view: the engine (``gsmpm.sim.Simulator`` in
slab mode), the transport, and ``gather`` of per-particle outputs to one rank
in global particle order (the renderer does not shard by slab: compositing
order is view-dependent).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from ._lib import LIB, check


def base_planes(x_grid, inv_dx: float):
    """trunc(x * inv_dx - 0.5) of the axis-0 coordinate, f32 as the kernels compute it."""
    xs = np.asarray(x_grid, dtype=np.float32).reshape(-1, 3)[:, 0]
    with np.errstate(invalid="ignore"):
        return np.trunc(xs * np.float32(inv_dx) - np.float32(0.5)).astype(np.int64)


def slab_bounds(x_grid, n_grid: int, grid_extent: float, world: int, margin: int = 2):
    """Plane bounds [0 = b_0 < b_1 < ... < b_world = n_grid] of `world` slabs of
    about equal particle count, each >= 2 * margin + 2 planes thick.  Raises
    ValueError if the grid cannot hold that many slabs."""
    thick = 2 * margin + 2
    if world == 1:
        return [0, n_grid]
    if world * thick > n_grid:
        raise ValueError(f"cannot cut {n_grid} planes into {world} slabs of >= {thick} planes")
    bx = np.clip(base_planes(x_grid, n_grid / grid_extent), 0, n_grid - 1)
    q = np.quantile(bx, [r / world for r in range(1, world)]) if len(bx) else \
        np.linspace(0, n_grid, world + 1)[1:-1]
    b = [0] + [int(round(v)) for v in q] + [n_grid]
    for r in range(1, world):  # forward: every slab at least `thick`
        b[r] = max(b[r], b[r - 1] + thick)
    for r in range(world - 1, 0, -1):  # backward: room for the slabs above
        b[r] = min(b[r], b[r + 1] - thick)
    return b


def owner_of(x_grid, bounds, n_grid: int, grid_extent: float):
    """Rank owning each particle: the slab holding its base plane (clipped to the grid)."""
    bx = np.clip(base_planes(x_grid, n_grid / grid_extent), 0, n_grid - 1)
    return np.searchsorted(np.asarray(bounds[1:-1]), bx, side="right").astype(np.int32)


# ------------------------------------------------------------- transports --
class RcclTransport:
    """GSMPM_XPORT_RCCL: an RCCL communicator of the library's own (unique id
    from rank 0, broadcast over the torch.distributed group), used by
    gsmpm_mpm_slab_step for grouped ncclSend/ncclRecv between neighbours."""

    def __init__(self, rank: int, world: int, group=None, device=None):
        uid = (ctypes.c_uint8 * 128)()
        if rank == 0:
            check(LIB.gsmpm_rccl_unique_id(uid), "gsmpm_rccl_unique_id")
        obj = [bytes(uid)]
        dist.broadcast_object_list(obj, src=0, group=group)
        uid = (ctypes.c_uint8 * 128).from_buffer_copy(obj[0])
        comm = ctypes.c_void_p()
        with torch.cuda.device(device if device is not None else torch.cuda.current_device()):
            check(LIB.gsmpm_rccl_comm_init(uid, int(rank), int(world), ctypes.byref(comm)), "gsmpm_rccl_comm_init")
        self.comm = comm
        self.struct = _lib.Transport(_lib.XPORT_RCCL, int(rank), int(world), comm, _lib.EXCHANGE_FN(), None)

    def close(self):
        """Destroy the communicator.  Every simulator that stepped with it must be
        closed first: its captured chunk graphs hold RCCL work on the
        communicator (ncclCommDestroy behind a live graph blocked in
        tools/probe/rccl_graph_probe.cpp)."""
        if self.comm is not None and self.comm.value:
            check(LIB.gsmpm_rccl_comm_destroy(self.comm), "gsmpm_rccl_comm_destroy")
            self.comm = None


class CallbackTransport:
    """GSMPM_XPORT_CALLBACK over torch.distributed point-to-point: the library
    hands pinned host copies of the buffers to `exchange` (gloo moves host
    memory).  Used to run several slab ranks on one GPU in tests; the
    protocol (sizes, order, peers) is the one the RCCL transport runs."""

    def __init__(self, rank: int, world: int, group=None):
        self.rank, self.world, self.group = int(rank), int(world), group
        self.error = None
        self._fn = _lib.EXCHANGE_FN(self._callback)  # kept alive with the object
        self.struct = _lib.Transport(_lib.XPORT_CALLBACK, self.rank, self.world, None, self._fn, None)

    def exchange(self, peers, sends, recvs):
        """send sends[i] to peers[i] and receive recvs[i] from it (CPU tensors)."""
        ops = []
        for p, s, r in zip(peers, sends, recvs):
            if s.numel():
                ops.append(dist.P2POp(dist.isend, s, int(p), self.group))
            if r.numel():
                ops.append(dist.P2POp(dist.irecv, r, int(p), self.group))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()

    def _callback(self, user, n, peers, send, sb, recv, rb):
        try:
            view = lambda addr, nb: torch.frombuffer((ctypes.c_uint8 * nb).from_address(addr), dtype=torch.uint8) \
                if nb else torch.empty(0, dtype=torch.uint8)
            self.exchange([peers[i] for i in range(n)], [view(send[i], sb[i]) for i in range(n)],
                          [view(recv[i], rb[i]) for i in range(n)])
            return 0
        except Exception as e:  # surfaced by the library as a failed exchange; kept for the caller
            self.error = e
            return 1

    def close(self):
        pass


def make_transport(rank: int, world: int, group=None, device=None):
    """RCCL when the process group is nccl (one rank per GPU), else the host callback."""
    if world > 1 and dist.get_backend(group) == "nccl":
        return RcclTransport(rank, world, group, device)
    return CallbackTransport(rank, world, group)


# ------------------------------------------------------------------ domain --
def _default_gravity(engine_factory):
    """The gravity an engine uses when none is passed: the ``gravity`` default
    of its constructor (Simulator: (0, -9.81, 0), utils/solver defaults), else
    that same vector."""
    import inspect
    try:
        p = inspect.signature(engine_factory).parameters.get("gravity")
    except (TypeError, ValueError):
        p = None
    if p is not None and p.default is not inspect.Parameter.empty:
        return tuple(float(g) for g in p.default)
    return (0.0, -9.81, 0.0)


class SlabDomain:
    """Rank `rank`'s slab of one MPM scene.

    Every rank passes the WHOLE scene (grid-space x, cov6, vol, optional v;
    the same arrays on every rank, e.g. built from the same seed / PLY); the
    slab keeps its particles, with their index in those arrays as global id.
    ``sim_kwargs`` go to gsmpm.sim.Simulator (material, E, nu, density,
    gravity, ...); ``engine_factory`` replaces Simulator (tests: a CPU engine
    built on the oracle that runs the same slab protocol)."""

    def __init__(self, x_grid, cov6, vol, *, rank: int, world: int, transport, n_grid: int, grid_extent: float = 2.0,
                 margin: int = 2, interval: int = 10, capacity: int | None = None, v=None, device=None,
                 engine_factory=None, group=None, rebalance: bool = True, rebalance_tol: float = 0.05,
                 cut_axis="longest", **sim_kwargs):
        from .sim import Simulator
        engine_factory = engine_factory or Simulator
        self.rank, self.world, self.transport = int(rank), int(world), transport
        self.group = group  # the process group of the slab ranks (None: the default group)
        self.n_grid, self.grid_extent = int(n_grid), float(grid_extent)
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        self.margin, self.interval = int(margin), int(interval)
        xh = (x_grid.detach().cpu().numpy() if torch.is_tensor(x_grid) else np.asarray(x_grid)).reshape(-1, 3)
        self.n_total = len(xh)
        # SURVEY 8(e) cuts along the bbox's longest axis.  The library's slabs are
        # planes of its grid axis 0, so the domain runs the engine in a frame whose
        # axis 0 is the cut axis: coordinates, velocities, matrices, covariances,
        # gravity and every BC are permuted on the way in and back on the way out
        # (the grid is cubic and the update is axis-symmetric, so this is the same
        # computation up to f32 operand order).  Axis 0 is kept unless another is
        # more than 1 / 0.9 times longer (lego: x and y tie at 1.3; bicycle: a
        # cube, whose sampled extents differ in the 5th digit), where nothing is
        # permuted.
        ext = (xh.max(0) - xh.min(0)) if len(xh) else np.zeros(3)
        if cut_axis == "longest":
            a = int(np.argmax(ext))
            a = 0 if ext[0] >= 0.9 * ext[a] else a
        else:
            a = int(cut_axis)
        if not 0 <= a < 3:
            raise ValueError(f"cut_axis must be 'longest' or 0, 1, 2 (got {cut_axis!r})")
        self.cut_axis = a
        self.cut_axis_ratio = float(ext[a] / max(float(ext.max()), 1e-30)) if len(xh) else 1.0
        self._perm = [a] + [i for i in range(3) if i != a]  # engine axis i = scene axis _perm[i]
        self._inv = [self._perm.index(i) for i in range(3)]  # scene axis i = engine axis _inv[i]
        self._permuted = a != 0
        if self._permuted:
            xh = xh[:, self._perm]
            x_grid = self._vec_in(x_grid)
            cov6 = self._cov_in(cov6)
            v = None if v is None else self._vec_in(v)
            # gravity is a scene vector too: the engine's default is read in the
            # engine's (permuted) axes, so it is filled in before the swap
            sim_kwargs["gravity"] = self._p3(sim_kwargs.get("gravity", _default_gravity(engine_factory)))
        self._bounds0 = slab_bounds(xh, self.n_grid, self.grid_extent, self.world, margin)
        owner = owner_of(xh, self._bounds0, self.n_grid, self.grid_extent)
        mine = torch.from_numpy(np.nonzero(owner == self.rank)[0]).to(self.device)
        cap = capacity or max(4096, 2 * (self.n_total // self.world) + 4096)
        self.engine = engine_factory(cap, n_grid=self.n_grid, grid_extent=self.grid_extent, device=self.device,
                                     **sim_kwargs)
        self.engine.slab_init(self.rank, self.world, self._bounds0[self.rank], self._bounds0[self.rank + 1], margin,
                              interval)
        if hasattr(self.engine, "slab_set_rebalance"):  # the library re-cuts by itself (slab_host.inc)
            self.engine.slab_set_rebalance(rebalance, rebalance_tol)
        t = lambda a: (a if torch.is_tensor(a) else torch.from_numpy(np.ascontiguousarray(a))).to(self.device)
        sel = lambda a: None if a is None else t(a).reshape(self.n_total, -1)[mine]
        self.engine.slab_set_particles(sel(x_grid), sel(cov6), sel(vol), mine.to(torch.int32), v=sel(v))

    # ---- the cut-axis frame (engine axis 0 = the cut axis) ----
    _UP = ((0, 0), (0, 1), (0, 2), (1, 1), (1, 2), (2, 2))  # upper-6 layout [xx, xy, xz, yy, yz, zz]

    def _p3(self, a):
        return [float(a[i]) for i in self._perm]

    @staticmethod
    def _take(t, idx):
        if torch.is_tensor(t):
            return t[..., torch.as_tensor(idx, device=t.device)]
        return np.asarray(t)[..., list(idx)]

    def _vec_in(self, t):
        return self._take(self._rows(t, 3), self._perm)

    def _vec_out(self, t):
        return self._take(t, self._inv)

    def _mat_idx(self, p):
        return [3 * p[i] + p[j] for i in range(3) for j in range(3)]

    def _cov_idx(self, p):
        up = self._UP
        return [up.index(tuple(sorted((p[i], p[j])))) for i, j in up]

    def _cov_in(self, t):
        return self._take(self._rows(t, 6), self._cov_idx(self._perm))

    def _rows(self, t, w):
        return t.reshape(-1, w) if torch.is_tensor(t) else np.asarray(t).reshape(-1, w)

    def _out(self, name, t):
        """An engine field in the scene's axes."""
        if not self._permuted:
            return t
        if name in ("x", "v"):
            return self._vec_out(t)
        if name in ("C", "F_trial", "R"):
            return self._take(t, self._mat_idx(self._inv))
        if name in ("cov", "init_cov"):
            return self._take(t, self._cov_idx(self._inv))
        return t

    @property
    def bounds(self):
        """Every slab's current planes [world + 1]: the init quantiles until the
        library re-cuts them (every rank computes the same re-cut)."""
        if hasattr(self.engine, "slab_bounds"):
            b, _ = self.engine.slab_bounds(self.world)
            if min(b) >= 0:
                return b
        return list(self._bounds0)

    @property
    def rebalances(self) -> int:
        return self.engine.slab_bounds(self.world)[1] if hasattr(self.engine, "slab_bounds") else 0

    # configuration and stepping: the engine's, with the transport
    # (BC geometry in the scene's axes, permuted into the engine's)
    def add_fixed_cube(self, center, size):
        if self._permuted:
            center, size = self._p3(center), self._p3(size)
        return self.engine.add_fixed_cube(center, size)

    def add_impulse(self, center, size, force, substep_dt):
        if self._permuted:
            center, size, force = self._p3(center), self._p3(size), self._p3(force)
        return self.engine.add_impulse(center, size, force, substep_dt)

    def add_plane_collider(self, point, normal, friction=0.0):
        if self._permuted:
            point, normal = self._p3(point), self._p3(normal)
        return self.engine.add_plane_collider(point, normal, friction)

    def step(self, dt: float, masks):
        try:
            self.engine.slab_step(dt, masks, self.transport)
        except _lib.GsmpmError:
            err = getattr(self.transport, "error", None)
            if err is not None:
                raise RuntimeError(f"rank {self.rank}: slab exchange failed") from err
            raise

    def postprocess(self):
        self.engine.postprocess()

    def set_weight(self, weight: float):
        """This rank's share weight in the library's re-cut (1: even;
        gsmpm_mpm_slab_set_weight); takes effect at the next step calls."""
        if hasattr(self.engine, "slab_set_weight"):
            self.engine.slab_set_weight(float(weight))

    def set_render_share(self, sim_ms: float, render_ms: float, world: int | None = None,
                         floor: float = 0.1) -> float:
        """The render-aware re-cut: the rank that renders the gathered frame
        takes a smaller particle share so that its simulation plus the render
        matches the other ranks' simulation.  `sim_ms` must be this rank's
        simulation time at an EVEN share (weight 1, i.e. before any call to
        this), `render_ms` its render time.  The library's re-cut gives this
        rank the share w / (w + W - 1) of the particles (W = world), so with a
        simulation time linear in the particle count the balancing weight is
            w = (W s - (W - 1) r) / (W s + r)
        (rank 0: W s w / (w + W - 1) + r = the others' W s / (w + W - 1)),
        clamped to [floor, 1].  Returns the weight set."""
        W = self.world if world is None else int(world)
        s, r = float(sim_ms), float(render_ms)
        w = (W * s - (W - 1) * r) / max(W * s + r, 1e-9)
        w = max(float(floor), min(1.0, w))
        self.set_weight(w)
        return w

    @property
    def n(self) -> int:
        return self.engine.count

    def stats(self):
        return self.engine.slab_stats()

    # outputs in global order on one rank
    def gather(self, rows: torch.Tensor, dst: int = 0):
        """Per-particle rows of this rank ([n, w] in the engine's row order)
        -> on rank `dst` (a rank of the slab group) the [n_total, w] tensor in
        global particle order (None elsewhere).  One max-reduce of the counts,
        then a gather to `dst` of count-padded blocks whose last column is the
        global id as int32 bits (a block's unused rows carry id -1)."""
        gid = self.engine.get_gid()
        n = gid.numel()
        rows = rows.reshape(n, -1).to(torch.float32)
        w = rows.shape[1]
        on_dev = dist.get_backend(self.group) == "nccl"
        dev = self.device if on_dev else torch.device("cpu")
        nmax = torch.tensor([n], dtype=torch.int64, device=dev)
        dist.all_reduce(nmax, op=dist.ReduceOp.MAX, group=self.group)
        nmax = int(nmax.item())
        blk = torch.empty((nmax, w + 1), dtype=torch.float32, device=dev)
        blk[:n, :w] = rows.to(dev)
        ids = blk[:, w:].view(torch.int32)  # the id column, reinterpreted: exact for any count
        ids.fill_(-1)
        ids[:n, 0] = gid.to(dev)
        me = dist.get_rank(self.group) if self.group is not None else self.rank
        g_dst = dist.get_global_rank(self.group, dst) if self.group is not None else dst
        parts = [torch.empty_like(blk) for _ in range(self.world)] if me == dst else None
        dist.gather(blk, parts, dst=g_dst, group=self.group)
        if me != dst:
            return None
        allb = torch.cat(parts).to(self.device)
        idx = allb[:, w:].contiguous().view(torch.int32).reshape(-1).to(torch.int64)
        keep = idx >= 0
        out = torch.empty((self.n_total, w), dtype=torch.float32, device=self.device)
        out[idx[keep]] = allb[keep, :w]
        return out

    def gather_field(self, name: str, dst: int = 0):
        out = self.gather(self.engine.get(name), dst)
        return None if out is None else self._out(name, out)

    def gather_world(self, scale, center, render_space: bool, dst: int = 0):
        """Fused grid2world (+ render shift) of every particle, on rank `dst`:
        (means [N, 3], cov6 [N, 6]) in global order."""
        if self._permuted:
            center = self._p3(center)
        m, c = self.engine.world_outputs(scale, center, render_space)
        full = self.gather(torch.cat([m, c], 1), dst)
        if full is None:
            return None, None
        m, c = full[:, :3], full[:, 3:]
        return self._out("x", m).contiguous(), self._out("cov", c).contiguous()
