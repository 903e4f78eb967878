"""Model / state containers (mpm_solver/model.py:6-132) as views over device state.

The reference keeps Taichi fields (AOS, one per quantity).  Here the state
lives in libgsmpm.so as SoA planes in Morton order; each attribute below is a
``FieldView`` whose ``to_torch()`` / ``from_torch()`` convert to and from the
reference's Taichi ``to_torch`` shapes and particle order.  Reads first flush
any substeps queued by ``MPM_Simulator.p2g2p``.
"""
from __future__ import annotations

import math

import torch

from mpm_solver.utils import material_types


class FieldView:
    """Stand-in for a Taichi field: to_torch / from_torch / to_numpy / fill / shape (+ .grad)."""

    def __init__(self, owner, getter, setter=None, shape=None, grad=None):
        self._owner = owner
        self._get = getter
        self._set = setter
        self.shape = shape
        self.grad = grad

    def to_torch(self, device=None):
        self._owner.flush()
        t = self._get()
        return t if device is None else t.to(device)

    def to_numpy(self):
        return self.to_torch().cpu().numpy()

    def from_torch(self, t):
        if self._set is None:
            raise AttributeError("field is read-only in the HIP backend")
        self._owner.flush()
        self._set(t)

    def from_numpy(self, a):
        self.from_torch(torch.as_tensor(a))

    def fill(self, value):
        t = self.to_torch()
        self.from_torch(torch.full_like(t, float(value)))


class MPM_model:
    """Material + grid constants (model.py:6-73)."""

    def __init__(self, n_particles: int, args):
        self.args = args
        self.n_particles = n_particles
        self.grid_extent = args.grid_extent
        self.n_grid = args.n_grid
        self.dx = args.grid_extent / args.n_grid
        self.inv_dx = args.n_grid / args.grid_extent
        code = material_types.get(args.material, -1)
        if code not in (0, 1, 2, 3):
            raise TypeError("Material not supported yet")  # model.py:27-30
        self.material_code = code
        self.gravity = list(args.gravity)
        self.friction_angle = 25.0
        sin_phi = math.sin(self.friction_angle / 180.0 * 3.141592653589793)
        self.alpha = math.sqrt(2.0 / 3.0) * 2.0 * sin_phi / (3.0 - sin_phi)
        self.hardening = 1
        self.xi = 1
        self.plastic_viscosity = 0.008
        self.softening = 1.0
        self._logE = math.log10(args.E)
        self._y = -math.log(0.49 / args.nu - 1)
        self._owner = None

    def _bind(self, owner):
        self._owner = owner
        sim = owner._sim
        n = self.n_particles
        dev = sim.device
        self.material = FieldView(owner, lambda: torch.full((n,), float(self.material_code), device=dev), shape=(n,))
        self.logE = FieldView(owner, lambda: torch.full((n,), self._logE, dtype=torch.float32, device=dev), shape=(n,))
        self.y = FieldView(owner, lambda: torch.full((n,), self._y, dtype=torch.float32, device=dev), shape=(n,))
        self.mu = FieldView(owner, lambda: sim.get("mu"), lambda t: sim.set("mu", t), shape=(n,))
        self.lam = FieldView(owner, lambda: sim.get("lam"), lambda t: sim.set("lam", t), shape=(n,))
        self.yield_stress = FieldView(owner, lambda: sim.get("yield_stress"), lambda t: sim.set("yield_stress", t),
                                      shape=(n,))


    def _bind_fit(self, owner):
        """logE / y / mu / lam and their .grad on the fitting path (model.py:35-44)."""
        self._owner = owner
        fit = owner._fit
        n = self.n_particles

        def fv(name):
            g = FieldView(owner, lambda: fit.get("g" + name), lambda t: fit.set("g" + name, t), (n,))
            return FieldView(owner, lambda: fit.get(name), lambda t: fit.set(name, t), (n,), grad=g)
        self.logE, self.y, self.mu, self.lam = fv("logE"), fv("y"), fv("mu"), fv("lam")
        self.material = FieldView(owner, lambda: torch.full((n,), float(self.material_code), device=fit.device),
                                  shape=(n,))

    def clear_grad(self):
        if self._owner is not None and getattr(self._owner, "fitting", False):
            for k in ("glogE", "gy", "gmu", "glam"):
                self._owner._fit.set(k, torch.zeros(self.n_particles))


class MPM_state_opt:
    """Differentiable particle + grid state (model.py:135-223): fields with 31
    levels; ``to_torch()`` returns the reference's (31, N, ...) shapes."""

    def __init__(self, owner, args):
        fit = owner._fit
        n, L, ng = owner.n_particles, fit.levels, args.n_grid
        self.n_particles = n
        self._fit = fit

        def leveled(name, tail):
            def get(nm=name):
                return torch.stack([fit.get(nm, s).view(n, *tail) for s in range(L)])

            def put(t, nm=name):
                t = t.reshape(L, n, -1)
                for s in range(L):
                    fit.set(nm, t[s], s)
            return get, put

        def view(name, tail):
            g, p = leveled(name, tail)
            gg, gp = leveled("g" + name, tail)
            return FieldView(owner, g, p, (L, n, *tail), grad=FieldView(owner, gg, gp, (L, n, *tail)))
        self.particle_xyz = view("x", (3,))
        self.particle_vel = view("v", (3,))
        self.particle_F = view("F", (3, 3))
        self.particle_stress = view("stress", (3, 3))
        self.particle_C = view("C", (3, 3))
        self.particle_cov = FieldView(owner, lambda: fit.get("cov").view(-1), lambda t: fit.set("cov", t), (6 * n,),
                                      grad=FieldView(owner, lambda: fit.get("gcov").view(-1),
                                                     lambda t: fit.set("gcov", t), (6 * n,)))
        self.particle_init_cov = FieldView(owner, lambda: fit.get("init_cov").view(-1), None, (6 * n,))
        self.particle_vol = FieldView(owner, lambda: fit.get("vol"), None, (n,))
        self.particle_mass = FieldView(owner, lambda: fit.get("mass"), None, (n,))
        density = float(args.density)
        self.particle_density = FieldView(owner, lambda: torch.full((n,), density, device=fit.device), None, (n,))
        self.grid_mass = FieldView(owner, lambda: fit.get_grid("mass"), None, (ng, ng, ng))
        self.grid_v_in = FieldView(owner, lambda: fit.get_grid("v_in"), None, (ng, ng, ng, 3),
                                   grad=FieldView(owner, lambda: fit.get_grid("v_in_grad"), None, (ng, ng, ng, 3)))
        self.grid_v_out = FieldView(owner, lambda: fit.get_grid("v_out"), None, (ng, ng, ng, 3),
                                    grad=FieldView(owner, lambda: fit.get_grid("v_out_grad"), None, (ng, ng, ng, 3)))

    def set_grads(self, xyz_grad, cov_grad):
        """model.py:192-202: x.grad[30] = xyz_grad, cov.grad = cov_grad (numpy, as
        extra.py:226-228 passes them, or tensors)."""
        self._fit.set_grads(torch.as_tensor(xyz_grad), torch.as_tensor(cov_grad))

    def cycle_init(self):
        """model.py:216-223: level 30 -> level 0 for x, v, F, stress, C."""
        self._fit.cycle_init()

    def clear_grad(self):
        """model.py:204-214 (the state half of clear_grads; the reference's own
        MPM_model.clear_grad is the other half): the library clears both, so the
        model's adjoints are put back."""
        keep = {k: self._fit.get(k) for k in ("glogE", "gy", "gmu", "glam")}
        self._fit.clear_grads()
        for k, t in keep.items():
            self._fit.set(k, t)

    def reset_grid_state(self):
        pass  # done inside every gsmpm_fit_forward / _backward


class MPM_state:
    """Particle + grid state (model.py:76-132)."""

    def __init__(self, owner, args):
        sim = owner._sim
        n = owner.n_particles
        ng = args.n_grid
        self.n_particles = n
        dev = sim.device
        density = float(args.density)
        self.particle_xyz = FieldView(owner, lambda: sim.get("x"), lambda t: sim.set("x", t.reshape(-1, 3)), (n, 3))
        self.particle_vel = FieldView(owner, lambda: sim.get("v"), lambda t: sim.set("v", t.reshape(-1, 3)), (n, 3))
        self.particle_C = FieldView(owner, lambda: sim.get("C").view(n, 3, 3), lambda t: sim.set("C", t), (n, 3, 3))
        self.particle_F_trial = FieldView(owner, lambda: sim.get("F_trial").view(n, 3, 3),
                                          lambda t: sim.set("F_trial", t), (n, 3, 3))
        self.particle_cov = FieldView(owner, lambda: sim.get("cov").view(-1), None, (6 * n,))
        self.particle_init_cov = FieldView(owner, lambda: sim.get("init_cov").view(-1), None, (6 * n,))
        self.particle_R = FieldView(owner, lambda: sim.get("R").view(n, 3, 3), None, (n, 3, 3))
        self.particle_mass = FieldView(owner, lambda: sim.get("mass"), None, (n,))
        self.particle_vol = FieldView(owner, lambda: sim.get("vol"), None, (n,))
        self.particle_density = FieldView(owner, lambda: torch.full((n,), density, device=dev), None, (n,))
        self.grid_mass = FieldView(owner, lambda: sim.get_grid("mass"), None, (ng, ng, ng))
        self.grid_v_in = FieldView(owner, lambda: sim.get_grid("v_in"), None, (ng, ng, ng, 3))
        self.grid_v_out = FieldView(owner, lambda: sim.get_grid("v_out"), None, (ng, ng, ng, 3))

    @property
    def particle_F(self):
        # The hot loop keeps one F plane (F_trial between substeps, the
        # return-mapped F only inside k_p2g), so particle_F is not materialised.
        raise AttributeError("particle_F is not materialised by the HIP backend; read particle_F_trial")

    @property
    def particle_stress(self):
        raise AttributeError("particle_stress lives in registers inside k_p2g and is not stored")
