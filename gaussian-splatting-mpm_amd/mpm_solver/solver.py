"""``MPM_Simulator`` drop-in (mpm_solver/solver.py:9-177) over libgsmpm.so.

``p2g2p(dt)`` keeps the reference's per-substep call and float64 host clock
(solver.py:27-52) but does not launch per call: the substep's BC activity
mask is decided on the host (exactly as ``isActive`` at the current
``self.time``) and queued; the queue is flushed as one ``gsmpm_mpm_step`` --
a cached hipGraph of fused kernels -- when state is read, ``postprocess()``
runs, or ``flush()`` is called.  Results are identical to launching per call.

With ``args.fitting=True`` the simulator is the differentiable one
(MPM_state_opt, 31 state levels; gsmpm/fit.py over gsmpm_fit_*):
``p2g2p_forward / p2g2p_backward / postprocess_forward / _backward / learn /
clear_grads`` and ``mpm_state.set_grads / cycle_init`` as in the reference.
"""
from __future__ import annotations

import math

from gsmpm.fit import FitSimulator
from gsmpm.sim import Simulator
from mpm_solver.boundary_conditions import (StickyGroundBC, boundaryConditionTypeCallBacks, init_bc,
                                            postprocess_bc, preprocess_bc)
from mpm_solver.collider import MPM_Collider, collideTypeCallBacks
from mpm_solver.model import MPM_model, MPM_state, MPM_state_opt

_MAX_QUEUE = 1 << 14


class MPM_Simulator:
    def __init__(self, xyzs, covs, volumes, args, init_v=None):
        self.n_particles = int(xyzs.shape[0])
        self.mpm_model = MPM_model(self.n_particles, args)
        self.fitting = bool(getattr(args, "fitting", False))
        self.time = 0.0
        self.collider_params = []
        self.particle_preprocess = []
        self.grid_postprocess = []
        self.init_particles = []
        self._queue = []
        self._queue_dt = None
        if self.fitting:  # MPM_state_opt (model.py:135-223) on gsmpm_fit_*
            self._sim = None
            self._fit = FitSimulator(self.n_particles, n_grid=args.n_grid, grid_extent=args.grid_extent, levels=31,
                                     E=args.E, nu=args.nu, density=args.density, gravity=args.gravity,
                                     device=xyzs.device if xyzs.is_cuda else None)
            self._fit.set_particles(xyzs.reshape(-1, 3), covs.reshape(-1, 6), volumes.reshape(-1), init_v)
            self._fit_bc = None
            self.mpm_model._bind_fit(self)
            self.mpm_state = MPM_state_opt(self, args)
            return
        self._sim = Simulator(
            self.n_particles, n_grid=args.n_grid, grid_extent=args.grid_extent, material=args.material, E=args.E,
            nu=args.nu, density=args.density, gravity=args.gravity, jelly_fcr=bool(getattr(args, "jelly_fcr", False)),
            keep_grid=bool(getattr(args, "keep_grid", False)), phased=bool(getattr(args, "phased", False)),
            device=xyzs.device if xyzs.is_cuda else None)
        self._sim.set_particles(xyzs.reshape(-1, 3), covs.reshape(-1, 6), volumes.reshape(-1), init_v)
        self.mpm_model._bind(self)
        self.mpm_state = MPM_state(self, args)

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

    def p2g2p(self, dt, s=None):
        """One substep (solver.py:27-52); queued, see module docstring.

        With fitting=True, ``p2g2p(dt, s)`` runs ``p2g2p_forward(dt, s)``:
        extra.py:207 calls it that way although the reference's ``p2g2p``
        takes only ``dt``; the intended call is used."""
        if self.fitting:
            if s is None:
                raise TypeError("p2g2p(dt) steps the forward-only state; with fitting=True use p2g2p_forward(dt, s)")
            return self.p2g2p_forward(dt, s)
        if s is not None:
            raise TypeError("p2g2p() takes 2 positional arguments but 3 were given")  # solver.py:27
        if self._queue and dt != self._queue_dt:
            self.flush()
        self._queue_dt = dt
        self._queue.append(self._mask_now())
        self.time += dt  # float64 host clock, solver.py:52
        if len(self._queue) >= _MAX_QUEUE:
            self.flush()

    def flush(self):
        if self.fitting:
            return
        if self._queue:
            q, self._queue = self._queue, []
            self._sim.step(float(self._queue_dt), q)

    def postprocess(self):
        """compute_cov_from_F + compute_R_from_F (solver.py:135-137)."""
        if self.fitting:
            raise TypeError("postprocess() reads the forward-only state; with fitting=True use postprocess_forward()")
        self.flush()
        self._sim.postprocess()

    # ----------------------------------------------------------------- BCs --
    def set_boundary_conditions(self, bc_args_arr, sim_args):
        if self.fitting:
            for bc_args in bc_args_arr:
                bc = boundaryConditionTypeCallBacks[bc_args["type"]](self.n_particles, bc_args, sim_args)
                if bc.type in postprocess_bc:
                    self.grid_postprocess.append(bc)
                elif bc.type in preprocess_bc or bc.type in init_bc:
                    # the _opt path never applies particle_preprocess / init_particles (solver.py:54-69)
                    (self.particle_preprocess if bc.type in preprocess_bc else self.init_particles).append(bc)
            return
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
        if self.fitting:
            self.grid_postprocess.append(bc)
            return
        bc.bit = self._sim.add_fixed_cube(bc.center, bc.size)
        self.grid_postprocess.append(bc)

    def add_surface_collider(self, point, normal, surface="sticky", friction=0.0, start_time=0.0, end_time=999.0):
        point = list(point)
        scale = 1.0 / math.sqrt(float(sum(x ** 2 for x in normal)))
        normal = [scale * x for x in normal]
        cp = MPM_Collider(point, normal, friction)
        self.collider_params.append(cp)
        cl = collideTypeCallBacks["ground"](cp.point, cp.normal, cp.friction)
        if self.fitting:  # only grid_postprocess[0] runs on the fitting path (solver.py:64)
            self.grid_postprocess.append(cl)
            return
        cl.bit = self._sim.add_plane_collider(point, normal, friction)
        self.grid_postprocess.append(cl)

    # ------------------------------------------- differentiable (fitting) --
    def _need_fit(self, name):
        if not self.fitting:
            raise AttributeError(f"{name} needs args.fitting=True (MPM_state_opt)")
        if not self.grid_postprocess:
            raise IndexError("list index out of range")  # grid_postprocess[0], solver.py:64
        bc = self.grid_postprocess[0]
        if bc is not self._fit_bc:
            if getattr(bc, "isCollide", False) or not hasattr(bc, "center"):
                raise NotImplementedError("grid_postprocess[0] must be a fixed-cube BC on the fitting path")
            self._fit.set_fixed_cube(bc.center, bc.size)
            self._fit_bc = bc

    def p2g2p_forward(self, dt, s):
        """solver.py:54-69: stress, P2G, grid update, grid_postprocess[0], G2P; level s -> s+1."""
        self._need_fit("p2g2p_forward")
        self._fit.forward(float(dt), int(s))
        self.time += dt

    def p2g2p_backward(self, dt, s):
        """solver.py:71-90: redo P2G + grid of level s, then the adjoint chain."""
        self._need_fit("p2g2p_backward")
        self._fit.backward(float(dt), int(s))

    def learn(self):
        """solver.py:92-108: clipped SGD on logE (lr 0.8) and y (lr 1.6)."""
        self._need_fit("learn")
        self._fit.learn()

    def postprocess_forward(self):
        """solver.py:167-168: compute_cov_from_F_opt (covariances from F[30])."""
        self._need_fit("postprocess_forward")
        self._fit.postprocess_forward()

    def postprocess_backward(self):
        self._need_fit("postprocess_backward")
        self._fit.postprocess_backward()

    def clear_grads(self):
        """solver.py:173-175: MPM_model.clear_grad + MPM_state_opt.clear_grad."""
        if not self.fitting:
            raise AttributeError("clear_grads needs args.fitting=True")
        self._fit.clear_grads()
