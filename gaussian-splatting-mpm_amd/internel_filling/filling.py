"""Particle volume initialisation (internel_filling/filling.py:27-42) on the GPU.

vol_p = dx^3 / (number of particles in p's cell), cell = floor(x / dx),
counted with i32 atomics in libgsmpm.so (k_fill_count / k_fill_vol).
"""
import torch

from gsmpm.sim import particle_volume


def get_particle_volume(pos: torch.Tensor, args, uniform: bool = False):
    vol = particle_volume(pos, args.n_grid, args.grid_extent)
    if uniform:  # same volume for all particles (filling.py:39-40)
        return torch.mean(vol).repeat(pos.shape[0])
    return vol
