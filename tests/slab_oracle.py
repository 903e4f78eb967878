"""CPU slab engine for the multi-rank tests -- TEST INFRASTRUCTURE (oracle).

Runs the slab protocol of csrc/slab.h / slab_host.inc on the CPU oracle's
split substep, with the same sequence the library runs: per substep P2G
(oracle substep_begin), this rank's partial (m v, m) of the window planes
[b - M, b + M + 2) around each shared bound, the swap through the transport
(gsmpm.dist.CallbackTransport.exchange, gloo), total = lower rank's partial +
upper rank's (f32), grid update + G2P (substep_end); every `interval`
substeps the migration (every rank's record {send to lower, send to upper,
stayers, error bits, capacity} to every other rank, then the payloads;
stayers first, then arrivals from below, then from above).  Errors (a drift
past the margin, a slab over capacity) are checked on the records, so every
rank raises the same error at the same migration, as the library does.  gsmpm.dist.SlabDomain drives it exactly as it
drives gsmpm.sim.Simulator, so the CPU tests exercise the domain code
(partition, chunking, transport, gather) against the single-domain oracle.
"""
from __future__ import annotations

import numpy as np
import torch

import oracle as O  # test infrastructure

FIELDS = (("x", 3), ("v", 3), ("C", 9), ("F_trial", 9), ("mass", 1), ("vol", 1), ("mu", 1), ("lam", 1),
          ("yield_stress", 1), ("init_cov", 6), ("cov", 6), ("R", 9))
WIDTH = sum(w for _, w in FIELDS) + 1  # + global id (int32 bits)


class OracleSlabEngine:
    def __init__(self, capacity, *, n_grid, grid_extent=2.0, device=None, **kw):
        self.cap, self.ng, self.ext, self.kw = capacity, n_grid, grid_extent, kw
        self.inv_dx = n_grid / grid_extent
        self.o = None
        self.bcs = []  # ("op"|"imp", args) in add order = mask bit order
        self.since = 0
        self.migrated = 0
        self.err = 0  # bit 0: a particle drifted past the margin (reported at the next migration)

    # -- slab setup
    def slab_init(self, rank, world, lo, hi, margin, interval):
        self.rank, self.world, self.lo, self.hi, self.M, self.R = rank, world, lo, hi, margin, interval
        self.W = 2 * margin + 2
        self.on = [rank > 0, rank < world - 1]
        self.a = [lo - margin, hi - margin]

    def slab_set_particles(self, x, cov6, vol, gid, v=None):
        f = lambda t: None if t is None else t.detach().cpu().numpy().astype(np.float32)
        self._build(f(x), f(cov6), f(vol), f(v))
        self.gid = gid.detach().cpu().numpy().astype(np.int32)

    def _build(self, x, cov6, vol, v=None):
        self.o = O.OracleMPM(x.reshape(-1, 3), cov6.reshape(-1, 6), vol.reshape(-1), v=v, n_grid=self.ng,
                             grid_extent=self.ext, **self.kw)
        for kind, args in self.bcs:
            (self.o.add_collider if kind == "col" else self.o.add_fixed_box if kind == "box" else self.o.add_impulse)(*args)

    def add_fixed_cube(self, c, s):
        self.bcs.append(("box", (c, s)))
        self.o.add_fixed_box(c, s)
        return len(self.bcs) - 1

    def add_plane_collider(self, p, n, friction=0.0):
        self.bcs.append(("col", (p, n, friction)))
        self.o.add_collider(p, n, friction)
        return len(self.bcs) - 1

    def add_impulse(self, c, s, f, sdt):
        self.bcs.append(("imp", (c, s, f, sdt)))
        self.o.add_impulse(c, s, f, sdt)
        return len(self.bcs) - 1

    # -- stepping
    def _masks(self, mask):
        ia = [(mask >> b) & 1 for b, (k, _) in enumerate(self.bcs) if k == "imp"]
        oa = [(mask >> b) & 1 for b, (k, _) in enumerate(self.bcs) if k != "imp"]
        return ia, oa

    def _peers(self):
        return [self.rank + (-1 if w == 0 else 1) for w in range(2) if self.on[w]], [w for w in range(2) if self.on[w]]

    def _substep(self, dt, mask, xp):
        ia, oa = self._masks(mask)
        b = np.trunc(self.o.x[:, 0] * np.float32(self.inv_dx) - np.float32(0.5)).astype(np.int64)
        if len(b) and ((b < self.lo - self.M) | (b >= self.hi + self.M)).any():
            self.err |= 1
        self.o.substep_begin(dt, ia)
        peers, ws = self._peers()
        mine = [self.o.window_sums(self.a[w], self.W) for w in ws]
        recv = [np.empty_like(m) for m in mine]
        xp.exchange(peers, [torch.from_numpy(m.view(np.uint8).reshape(-1)) for m in mine],
                    [torch.from_numpy(r.view(np.uint8).reshape(-1)) for r in recv])
        for w, m, r in zip(ws, mine, recv):
            tot = (r + m) if w == 0 else (m + r)  # lower rank's partial first
            self.o.set_window_sums(self.a[w], tot.astype(np.float32))
        self.o.substep_end(dt, oa)

    def _migrate(self, xp):
        o = self.o
        b = np.trunc(o.x[:, 0] * np.float32(self.inv_dx) - np.float32(0.5)).astype(np.int64)
        dest = np.ones(len(b), np.int64)
        if self.on[0]:
            dest[b < self.lo] = 0
        if self.on[1]:
            dest[b >= self.hi] = 2
        rows = np.concatenate([getattr(o, k).reshape(len(b), w).astype(np.float32) for k, w in FIELDS] +
                              [self.gid.view(np.float32).reshape(-1, 1)], 1)
        peers, ws = self._peers()
        send = [np.ascontiguousarray(rows[dest == (0 if w == 0 else 2)]) for w in ws]
        u8 = lambda a: torch.from_numpy(a.view(np.uint8).reshape(-1))
        recs = np.zeros((self.world, 8), np.int32)
        recs[self.rank, :5] = [(dest == 0).sum(), (dest == 2).sum(), (dest == 1).sum(), self.err, self.cap]
        others = [r for r in range(self.world) if r != self.rank]
        xp.exchange(others, [u8(recs[self.rank].copy()) for _ in others], [u8(recs[r]) for r in others])
        for r in range(self.world):
            if recs[r, 3] & 1:
                raise RuntimeError(f"rank {r}: a particle drifted past the slab margin")
            n_new = recs[r, 2] + (recs[r - 1, 1] if r > 0 else 0) + (recs[r + 1, 0] if r < self.world - 1 else 0)
            if n_new > recs[r, 4]:
                raise RuntimeError(f"rank {r}: {n_new} particles after the migration, in a slab of capacity "
                                   f"{recs[r, 4]}")
        cnt_r = [recs[self.rank + (-1 if w == 0 else 1), 1 if w == 0 else 0] for w in ws]
        recv = [np.empty((int(c), WIDTH), np.float32) for c in cnt_r]
        xp.exchange(peers, [u8(s) for s in send], [u8(r) for r in recv])
        got = {0: np.zeros((0, WIDTH), np.float32), 2: np.zeros((0, WIDTH), np.float32)}
        for w, r in zip(ws, recv):
            got[0 if w == 0 else 2] = r
        new = np.concatenate([rows[dest == 1], got[0], got[2]], 0)
        self.migrated += sum(len(s) for s in send)
        cols, c0 = {}, 0
        for k, w in FIELDS:
            cols[k] = np.ascontiguousarray(new[:, c0:c0 + w])
            c0 += w
        self.gid = np.ascontiguousarray(new[:, c0]).view(np.int32).copy()
        self._build(cols["x"], cols["init_cov"], cols["vol"], cols["v"])
        for k, w in FIELDS:
            getattr(self.o, k)[...] = cols[k].reshape(getattr(self.o, k).shape)
        self.o.F[...] = self.o.F_trial

    def slab_step(self, dt, masks, xp):
        done = 0
        while done < len(masks):
            k = min(len(masks) - done, self.R - self.since % self.R)
            for s in range(k):
                self._substep(dt, int(masks[done + s]), xp)
            done += k
            self.since += k
            if self.since % self.R == 0 and self.world > 1:
                self._migrate(xp)

    # -- outputs
    @property
    def count(self):
        return len(self.gid)

    def get_gid(self):
        return torch.from_numpy(self.gid.copy())

    def get(self, name):
        return torch.from_numpy(np.ascontiguousarray(getattr(self.o, name)).copy())

    def postprocess(self):
        self.o.postprocess()

    def slab_stats(self):
        return {"migrated": self.migrated, "lo": self.lo, "hi": self.hi}
