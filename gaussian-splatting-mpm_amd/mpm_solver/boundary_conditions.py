"""Boundary-condition descriptors (mpm_solver/boundary_conditions.py:6-117).

Same constructor arguments, attributes, ``isActive`` windows and type
registries as the reference; the per-node / per-particle work runs inside the
fused HIP kernels (fixed cubes in k_grid, impulses in k_p2g).
"""
from __future__ import annotations


class BasicBC:
    """fixed_cube: zero v_out on nodes with |i*dx - center| < size (boundary_conditions.py:6-31)."""

    def __init__(self, n_particles, bc_args, sim_args):
        self.n_particles = n_particles
        self.substep_dt = sim_args.substep_dt
        self.id = bc_args["id"]
        self.type = bc_args["type"]
        self.start_time = bc_args["start_time"]
        # float64 on the host, as boundary_conditions.py:16
        self.end_time = bc_args["start_time"] + sim_args.substep_dt * bc_args["num_dt"]
        self.center = bc_args["center"]
        self.size = bc_args["size"]
        self.isCollide = False
        self.bit = None  # library bc id (bit of the activity mask)

    def isActive(self, time):
        return time >= self.start_time and time < self.end_time


class ImpulseBC(BasicBC):
    """impulse: v += force / m * substep_dt inside the box (boundary_conditions.py:34-45)."""

    def __init__(self, n_particles, bc_args, sim_args):
        self.force = list(bc_args["force"][:3])
        super().__init__(n_particles, bc_args, sim_args)


class MaterialParamsModifier(BasicBC):
    """additional_params (boundary_conditions.py:47-72).

    In the reference its apply() writes ``model.nu[p]`` / ``model.E[p]``,
    fields MPM_model never defines, so any config using it raises
    AttributeError.  Kept as an error here too.
    """

    def __init__(self, n_particles, bc_args, sim_args):
        self.mu = bc_args["mu"]
        self.density = bc_args["density"]
        self.E = bc_args["E"]
        self.nu = bc_args["nu"]
        self.isMaterial = False
        super().__init__(n_particles, bc_args, sim_args)

    def apply(self, state, model):
        raise AttributeError("'MPM_model' object has no attribute 'nu' "
                             "(additional_params is broken in the reference, SURVEY F9)")


class MaterialTypeModifier(BasicBC):
    """modify_material (boundary_conditions.py:74-85): writes a string into the f32
    material field in the reference, which Taichi rejects."""

    def __init__(self, n_particles, bc_args, sim_args):
        self.material = bc_args["material"]
        self.isMaterial = True
        super().__init__(n_particles, bc_args, sim_args)

    def apply(self, state, model):
        raise TypeError("modify_material assigns a string to the f32 material field "
                        "(broken in the reference, SURVEY F9)")


class StickyGroundBC(BasicBC):
    """sticky_ground (boundary_conditions.py:87-94): always-active fixed cube."""

    def __init__(self):
        self.center = [1.0, 0.6, 1.0]
        self.size = [1.0, 0.1, 1.0]
        self.type = "sticky_ground"
        self.isCollide = False
        self.start_time, self.end_time = 0.0, float("inf")
        self.bit = None

    def isActive(self, time):
        return True


# boundary_conditions.py:97-109 -- note preprocess_bc is a *string*, so
# ``type in preprocess_bc`` is a substring test exactly as in the reference.
preprocess_bc = ("impulse")
postprocess_bc = ("fixed_cube", "sticky_ground")
init_bc = ("additional_params", "modify_material")

boundaryConditionTypeCallBacks = {
    "fixed_cube": BasicBC,
    "impulse": ImpulseBC,
    "sticky_ground": StickyGroundBC,
    "additional_params": MaterialParamsModifier,
    "modify_material": MaterialTypeModifier,
}
