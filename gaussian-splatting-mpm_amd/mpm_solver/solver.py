"""``MPM_Simulator`` drop-in (mpm_solver/solver.py:9-177) over libgsmpm.so.

``p2g2p(dt)`` keeps the reference's per-substep call and float64 host clock
(solver.py:27-52) but does not launch per call: the substep's BC activity
mask is decided on the host (exactly as ``isActive`` at the current
``self.time``) and queued; the queue is flushed as one ``gsmpm_mpm_step`` --
a cached hipGraph of fused kernels -- when state is read, ``postprocess()``
runs, or ``flush()`` is called.  Results are identical to launching per call.
"""
from __future__ import annotations

import math

from gsmpm.sim import Simulator
from mpm_solver.boundary_conditions import (StickyGroundBC, boundaryConditionTypeCallBacks, init_bc,
                                            postprocess_bc, preprocess_bc)
from mpm_solver.collider import MPM_Collider, collideTypeCallBacks
from mpm_solver.model import MPM_model, MPM_state

_MAX_QUEUE = 1 << 14


class MPM_Simulator:
    def __init__(self, xyzs, covs, volumes, args, init_v=None):
        self.n_particles = int(xyzs.shape[0])
        self.mpm_model = MPM_model(self.n_particles, args)
        if getattr(args, "fitting", False):
            raise NotImplementedError("fitting=True (extra.py differentiable path) is not implemented yet "
                                      "(SURVEY §8(f) item 1)")
        self._sim = Simulator(
            self.n_particles, n_grid=args.n_grid, grid_extent=args.grid_extent, material=args.material, E=args.E,
            nu=args.nu, density=args.density, gravity=args.gravity, jelly_fcr=bool(getattr(args, "jelly_fcr", False)),
            keep_grid=bool(getattr(args, "keep_grid", False)), device=xyzs.device if xyzs.is_cuda else None)
        self._sim.set_particles(xyzs.reshape(-1, 3), covs.reshape(-1, 6), volumes.reshape(-1), init_v)
        self.mpm_model._bind(self)
        self.mpm_state = MPM_state(self, args)
        self.time = 0.0
        self.collider_params = []
        self.particle_preprocess = []
        self.grid_postprocess = []
        self.init_particles = []
        self._queue = []
        self._queue_dt = None

    # ------------------------------------------------------------ stepping --
    def _mask_now(self):
        m = 0
        for pp in self.particle_preprocess:
            if pp.isActive(self.time):
                m |= 1 << pp.bit
        for gp in self.grid_postprocess:
            if not gp.isCollide and gp.isActive(self.time):
                m |= 1 << gp.bit
        return m

    def p2g2p(self, dt):
        """One substep (solver.py:27-52); queued, see module docstring."""
        if self._queue and dt != self._queue_dt:
            self.flush()
        self._queue_dt = dt
        self._queue.append(self._mask_now())
        self.time += dt  # float64 host clock, solver.py:52
        if len(self._queue) >= _MAX_QUEUE:
            self.flush()

    def flush(self):
        if self._queue:
            q, self._queue = self._queue, []
            self._sim.step(float(self._queue_dt), q)

    def postprocess(self):
        """compute_cov_from_F + compute_R_from_F (solver.py:135-137)."""
        self.flush()
        self._sim.postprocess()

    # ----------------------------------------------------------------- BCs --
    def set_boundary_conditions(self, bc_args_arr, sim_args):
        for bc_args in bc_args_arr:
            bc = boundaryConditionTypeCallBacks[bc_args["type"]](self.n_particles, bc_args, sim_args)
            if bc.type in preprocess_bc:
                bc.bit = self._sim.add_impulse(bc.center, bc.size, bc.force, bc.substep_dt)
                self.particle_preprocess.append(bc)
            if bc.type in postprocess_bc:
                bc.bit = self._sim.add_fixed_cube(bc.center, bc.size)
                self.grid_postprocess.append(bc)
            if bc.type in init_bc:
                self.init_particles.append(bc)
        for pp in self.init_particles:
            pp.apply(self.mpm_state, self.mpm_model)

    def set_bc_ground_only(self):
        bc = StickyGroundBC()
        bc.bit = self._sim.add_fixed_cube(bc.center, bc.size)
        self.grid_postprocess.append(bc)

    def add_surface_collider(self, point, normal, surface="sticky", friction=0.0, start_time=0.0, end_time=999.0):
        point = list(point)
        scale = 1.0 / math.sqrt(float(sum(x ** 2 for x in normal)))
        normal = [scale * x for x in normal]
        cp = MPM_Collider(point, normal, friction)
        self.collider_params.append(cp)
        cl = collideTypeCallBacks["ground"](cp.point, cp.normal, cp.friction)
        cl.bit = self._sim.add_plane_collider(point, normal, friction)
        self.grid_postprocess.append(cl)

    # ---------------------------------------------- differentiable (phase 2) --
    def _phase2(self, *a, **k):
        raise NotImplementedError("differentiable MPM (p2g2p_forward/backward, learn) is not implemented yet "
                                  "(SURVEY §8(f) item 1)")

    p2g2p_forward = p2g2p_backward = postprocess_forward = postprocess_backward = learn = clear_grads = _phase2
