"""Helpers that drive the HIP path the way main.py does (device code only via libgsmpm.so)."""
from __future__ import annotations

import types

import numpy as np
import torch


def sim_args_from_cfg(cfg, n_grid, **over):
    a = types.SimpleNamespace(**cfg)
    a.n_grid = n_grid
    a.fitting = False
    a.jelly_fcr = False
    a.steps_per_frame = int(a.frame_dt / a.substep_dt)
    for k, v in over.items():
        setattr(a, k, v)
    return a


def dropin_sim(prob, dev, n_grid=None, with_collider=True, **over):
    from mpm_solver.solver import MPM_Simulator
    args = sim_args_from_cfg(prob["cfg"], n_grid or prob["n_grid"], **over)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    s = MPM_Simulator(t(prob["x"]), t(prob["cov"]), t(prob["vol"]), args)
    s.set_boundary_conditions(args.boundary_conditions, args)
    if with_collider:
        s.add_surface_collider((0.0, 0.0, 0.4), (0.0, 0.0, 1.0))
    return s, args
