"""How much could wave-level pre-aggregation save in k_fused's P2G scatter?

Pre-aggregation (sum the contributions of lanes that hit the same node
before the LDS atomic) pays when many particles share a base cell: lanes
with equal base cells have identical 27-node stencils, so one lane can
issue the 108 u64 atomics for all of them.  This probe builds the bench's
synthetic scenes on the CPU (bench.build_scene's generator and world2grid,
no GPU) and counts, per scene:

  * particles per occupied base cell, and the fraction of the scatter's
    atomics a perfect per-cell aggregation would remove (1 - cells/particles);
  * contributions per touched node (what a node-centric, gather-style P2G
    would reduce over).

    python tools/p2g_multiplicity.py            # lego 100k / 128^3 (config B)
    python tools/p2g_multiplicity.py --bicycle  # config D 1M / 256^3
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gaussian-splatting-mpm_amd")
sys.path.insert(0, PKG)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bicycle", action="store_true")
    a = ap.parse_args()
    from argparse import ArgumentParser
    from arguments import MPMParams
    from gaussian_splatting.scene import GaussianModel
    from utils.transform_utils import world2grid

    name, n, n_grid = ("bicycle.json", 1_000_000, 256) if a.bicycle else ("lego.json", 100_000, 128)
    box = ((0.05,) * 3, (0.95,) * 3) if a.bicycle else ((-0.65, -0.65, -0.55), (0.65, 0.65, 0.55))
    with open(os.path.join(PKG, "configs", name)) as f:
        cfg = json.load(f)
    p = ArgumentParser()
    s = MPMParams(p, cfg["mpm"]).extract(p.parse_args(["--n_grid", str(n_grid)]))
    xyz = GaussianModel(3, device="cpu").init_synthetic(n, seed=0, box=box).get_xyz
    b = torch.tensor(s.sim_area)
    xg = world2grid(xyz[((xyz <= b[1]).all(1) & (xyz >= b[0]).all(1))], s)[0]
    inv_dx = n_grid / s.grid_extent
    base = np.floor(xg.numpy().astype(np.float64) * inv_dx - 0.5).astype(np.int64)  # utils.py:95
    ng = n_grid + 2
    cells, cnt = np.unique((base[:, 0] * ng + base[:, 1]) * ng + base[:, 2], return_counts=True)
    off = np.stack(np.meshgrid([0, 1, 2], [0, 1, 2], [0, 1, 2], indexing="ij"), -1).reshape(27, 3)
    nodes = (base[:, None, :] + off[None]).reshape(-1, 3)
    touched = np.unique((nodes[:, 0] * ng + nodes[:, 1]) * ng + nodes[:, 2]).size
    out = {
        "scene": name, "particles": int(base.shape[0]), "n_grid": n_grid,
        "occupied_cells": int(cells.size),
        "particles_per_occupied_cell": round(float(cnt.mean()), 3),
        "particles_sharing_a_cell": round(float(cnt[cnt > 1].sum() / base.shape[0]), 4),
        "atomics_removable_by_cell_aggregation": round(1.0 - cells.size / base.shape[0], 4),
        "touched_nodes": int(touched),
        "contributions_per_touched_node": round(27.0 * base.shape[0] / touched, 2),
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
