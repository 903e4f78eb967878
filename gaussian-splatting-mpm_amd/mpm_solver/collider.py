"""Plane collider descriptor (mpm_solver/collider.py:4-49).

The collide pass itself (remove the inward normal velocity below the plane,
friction, x0.99) runs inside the fused grid kernel k_grid (csrc/mpm.hip).
"""


class MPM_Collider:
    def __init__(self, point, normal, friction):
        self.point = point
        self.normal = normal
        self.friction = friction
        self.isCollide = True
        self.bit = None  # library bc id


collideTypeCallBacks = {"ground": MPM_Collider}
