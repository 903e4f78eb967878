"""Multi-GPU MPM: one shared grid split into x-slabs, one rank per GPU.

SURVEY.md 8(e).  The reference is single-GPU; this is the MI355X-side
decomposition of its substep (mpm_solver/solver.py:27-52):

* Particles are owned by rank: ``slab_partition`` splits them into ``world``
  x-slabs of about equal count by their base plane
  (trunc(x * inv_dx - 0.5), utils.py:95), slab bounds rounded to 8-plane tiles.
  Every rank runs a full-size grid but only its particles touch it, so the work
  (tiles, chunks) is its slab's.
* A node receives contributions from two ranks only near a shared slab bound
  b: the halo window [b - H, b + H) (H = 8 planes by default).  After P2G each
  rank writes its partial (m, m v) of every window node; the two ranks sharing
  the window exchange partials with one send/recv pair (RCCL over xGMI, or
  gloo), and both add them in the same order (a + b == b + a in f32), so the
  grid update, BCs and G2P see the same node values on both sides -- the
  "all-reduce of boundary grid nodes" of the north star, done pairwise.
* No particle migration: a rank may touch only planes [b_r - H, b_{r+1} + H).
  The library flags any touched tile outside that range and ``step`` raises
  (never a silently wrong answer); re-partition (``repartition``) when that
  happens.

The engine is anything with ``set_halo / substep_begin / substep_end /
halo_escaped`` -- ``gsmpm.sim.Simulator`` on the GPU, or a CPU engine in the
tests.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

TILE = 8


def base_planes(x_grid, inv_dx: float):
    """trunc(x * inv_dx - 0.5) of the x coordinate, f32 as the kernels compute it."""
    xs = np.asarray(x_grid, dtype=np.float32)[:, 0]
    return np.trunc(xs * np.float32(inv_dx) - np.float32(0.5)).astype(np.int64)


def slab_partition(x_grid, n_grid: int, grid_extent: float, world: int, halo: int = TILE):
    """Split particles into `world` x-slabs of about equal count.

    Returns (owner[N] int32, bounds[world + 1]) with bounds[0] = 0,
    bounds[world] = n_grid rounded up to a tile, every bound a multiple of 8,
    and slabs at least 2 * halo planes thick (so the two windows of a rank never
    overlap).  Raises ValueError if the grid cannot hold that many slabs.
    """
    inv_dx = n_grid / grid_extent
    bx = base_planes(x_grid, inv_dx)
    top = (n_grid + TILE - 1) // TILE * TILE
    if world == 1:
        return np.zeros(len(bx), np.int32), [0, top]
    qs = np.quantile(np.clip(bx, 0, n_grid - 1), [r / world for r in range(1, world)])
    bounds = [0]
    for q in qs:
        b = int(round(q / TILE)) * TILE
        b = max(b, bounds[-1] + 2 * halo)
        bounds.append(b)
    bounds.append(top)
    for r in range(world):
        if bounds[r + 1] - bounds[r] < 2 * halo or (r + 1 < world and bounds[r + 1] + halo > top):
            raise ValueError(f"cannot cut {n_grid} planes into {world} slabs of >= {2 * halo} planes "
                             f"around the particles (bounds {bounds})")
    owner = (np.searchsorted(np.asarray(bounds[1:-1]), bx, side="right")).astype(np.int32)
    return owner, bounds


def windows_of(rank: int, world: int, bounds, halo: int = TILE):
    """Halo windows of `rank` in increasing x: lower (shared with rank - 1) and upper (rank + 1)."""
    w = []
    if rank > 0:
        w.append(bounds[rank] - halo)
    if rank < world - 1:
        w.append(bounds[rank + 1] - halo)
    return w


class SlabSimulator:
    """One rank's slab of a shared-grid MPM domain (see module docstring)."""

    def __init__(self, engine, rank: int, world: int, bounds, halo: int = TILE, group=None):
        self.engine, self.rank, self.world, self.bounds, self.halo = engine, rank, world, list(bounds), halo
        self.group = group
        self.x0s = windows_of(rank, world, bounds, halo)
        lo = max(0, bounds[rank] - halo) if rank > 0 else 0
        hi = bounds[rank + 1] + halo if rank < world - 1 else 1 << 30
        self.part, self.total = engine.set_halo(self.x0s, 2 * halo, allow=(lo, hi))
        self.n = engine.n
        self._host = None
        if world > 1 and dist.get_backend(group) == "gloo" and self.part.is_cuda:
            # gloo moves host memory: stage the windows through pinned buffers
            self._host = (torch.empty(self.part.shape, pin_memory=True), torch.empty(self.part.shape, pin_memory=True))
        self.recv = torch.empty_like(self.part) if self.part is not None else None

    # ------------------------------------------------------------ exchange --
    def _exchange(self):
        if self.part is None:  # world == 1
            return
        part, recv = self.part, self.recv
        if self._host is not None:
            hp, hr = self._host
            hp.copy_(part)
            part, recv = hp, hr
        ops = []
        k = 0
        if self.rank > 0:
            ops.append(dist.P2POp(dist.isend, part[k], self.rank - 1, self.group))
            ops.append(dist.P2POp(dist.irecv, recv[k], self.rank - 1, self.group))
            k += 1
        if self.rank < self.world - 1:
            ops.append(dist.P2POp(dist.isend, part[k], self.rank + 1, self.group))
            ops.append(dist.P2POp(dist.irecv, recv[k], self.rank + 1, self.group))
        for req in dist.batch_isend_irecv(ops):
            req.wait()
        if self._host is not None:
            self.recv.copy_(recv, non_blocking=True)
        # both sharing ranks add the same two partials: identical window sums
        torch.add(self.part, self.recv, out=self.total)

    # ---------------------------------------------------------------- step --
    def step(self, dt: float, masks):
        for m in masks:
            self.engine.substep_begin(dt, m)
            self._exchange()
            self.engine.substep_end(dt, m)
        if self.engine.halo_escaped():
            raise RuntimeError(f"rank {self.rank}: particles left planes [{self.bounds[self.rank]} - {self.halo}, "
                               f"{self.bounds[self.rank + 1]} + {self.halo}); re-partition the slabs")

    def __getattr__(self, name):
        # postprocess / get / world_outputs / ... act on this rank's particles
        return getattr(self.engine, name)
