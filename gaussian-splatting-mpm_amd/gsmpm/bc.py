"""Host-side boundary-condition scheduling (pure Python, no device code).

The reference decides BC activity on the host from a float64 clock:
``MPM_Simulator.time += dt`` after every substep (mpm_solver/solver.py:19,52)
and ``BasicBC.isActive`` = ``start_time <= time < start_time + substep_dt*num_dt``
(mpm_solver/boundary_conditions.py:15-16,30-31), evaluated before the substep's
kernels run.  Colliders bypass the test (``isCollide``, solver.py:42-43).

This module reproduces that clock exactly (same float64 additions in the same
order) and turns it into one activity bit-mask per substep for
``gsmpm_mpm_step`` (e.g. lego's impulse at [0.8, 0.801) is live on
substeps 8001-8010, not 8000-8009).
"""
from __future__ import annotations

from dataclasses import dataclass, field


@dataclass
class BCSpec:
    kind: str              # "fixed_cube" | "impulse" | "collider"
    bit: int               # id returned by the library (bit of the activity mask)
    start_time: float = 0.0
    end_time: float = float("inf")
    params: dict = field(default_factory=dict)

    def is_active(self, time: float) -> bool:
        if self.kind == "collider":
            return True
        return self.start_time <= time < self.end_time


def bc_window(start_time, substep_dt, num_dt):
    """boundary_conditions.py:15-16 -- end_time computed in float64."""
    return start_time, start_time + substep_dt * num_dt


def substep_masks(specs, time: float, dt: float, n: int):
    """Activity masks for n substeps starting at host time ``time``.

    Returns (masks, time_after).  The clock advances with ``time += dt``
    exactly as solver.py:52 does, so BC windows flip on the same substep.
    """
    masks = []
    t = time
    for _ in range(n):
        m = 0
        for s in specs:
            if s.kind != "collider" and s.is_active(t):
                m |= 1 << s.bit
        masks.append(m)
        t += dt
    return masks, t
