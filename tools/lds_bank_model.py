"""What is left of k_fused's P2G bank conflicts after the lane balance, and
what any lane assignment could still remove (CPU model of the bench scenes).

The P2G scatter issues, per particle, 108 ds_add_u64 (27 stencil nodes x 4
channels) with the same node offset on every lane: the LDS serves a wave in
4 groups of 16 lanes, and a group costs as many cycles as the most lanes
whose u64 address falls on one bank pair, i.e. whose base node is the same
mod 16 (same address included: tools/ubench/lds_banks.hip, "pairs" and
"res16").  The lane balance (fused.h balanced_lane) puts a particle whose
base node has residue r on a lane L = r mod 16 while the residue has lanes
left, and the rest on the leftover lanes in order.

For each chunk (the bench scene's particles binned into 8x8x7 tiles,
<= 256 a chunk, in a random order as the binning leaves them) this counts
  * in order:  the cycles with lanes in particle order (no balance);
  * balanced:  with fused.h's assignment;
  * bound:     a lower bound for ANY assignment of the chunk's particles to
               its ceil(cnt / 16) lane groups: every group costs >= 1 cycle, a
               residue r can be spread over at most G groups, so at least
               E = sum_r max(0, c_r - G) particles share their group with a
               particle of the same residue, and a 2-cycle group holds at
               most 8 of them: >= G + ceil(E / 8) cycles; and a full group
               of multiplicity 1 holds one particle of every residue, so at
               most min_r c_r of the G - 1 full groups cost 1 cycle and the
               others >= 2: >= 2 G - 1 - min(min_r c_r, G - 1) cycles.
  * largest_first / spread: a greedy assignment (below), over the chunk's
               groups / over every group of its active waves.
and reports conflict cycles / all cycles, the figure SQ_LDS_BANK_CONFLICT /
SQ_LDS_IDX_ACTIVE gives for the scatter.

    python tools/lds_bank_model.py            # lego 100k / 128^3 (config B)
    python tools/lds_bank_model.py --bicycle  # config D 1M / 256^3
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

FT = (8, 8, 7)          # tile (fused.h kFT0..2)
FW = (12, 12, 11)       # window (kFW0..2): base cells in [o - 1, o + T]


def balanced(res, cnt):
    """fused.h balanced_lane: lane of each particle (in its residue's rank order)."""
    rc = np.bincount(res, minlength=16)
    lanes = np.empty(cnt, np.int64)
    rank = np.zeros(16, np.int64)
    for i, r in enumerate(res):
        k = rank[r]
        rank[r] += 1
        Lr = (cnt - r + 15) >> 4
        if k < Lr:
            lanes[i] = k * 16 + r
            continue
        o = k - Lr
        for q in range(r):
            o += max(0, rc[q] - ((cnt - q + 15) >> 4))
        acc = 0
        for q in range(16):
            Lq = (cnt - q + 15) >> 4
            d = max(0, Lq - rc[q])
            if o < acc + d:
                lanes[i] = (rc[q] + (o - acc)) * 16 + q
                break
            acc += d
    return lanes


def largest_first(res, cnt, spread=False):
    """groups filled one at a time with the residues of most remaining
    particles, one each, then (when fewer distinct residues remain than the
    group has lanes) second copies of the largest: cycles of that assignment.
    spread: over every 16-lane group of the chunk's active waves (the idle
    lanes of its last wave dealt out, as evenly as possible)."""
    c = np.bincount(res, minlength=16).astype(np.int64)
    G = 4 * ((cnt + 63) // 64) if spread else (cnt + 15) // 16
    caps = [len(a) for a in np.array_split(np.arange(cnt), G)] if spread else \
        [min(16, cnt - 16 * g) for g in range(G)]
    cyc = 0
    for g in range(G):
        cap = caps[g]
        take = np.zeros(16, np.int64)
        while cap > 0:
            avail = np.flatnonzero(c - take > 0)
            if avail.size == 0:
                break
            pick = avail[np.argsort(-(c - take)[avail], kind="stable")][:cap]
            take[pick] += 1
            cap -= pick.size
        c -= take
        cyc += int(take.max())
    return cyc


def group_cycles(res_by_lane):
    """sum over 16-lane groups of the largest residue multiplicity (-1: idle lane)."""
    cyc = 0
    for g in range(0, len(res_by_lane), 16):
        r = res_by_lane[g:g + 16]
        r = r[r >= 0]
        if r.size:
            cyc += int(np.bincount(r, minlength=16).max())
    return cyc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bicycle", action="store_true")
    ap.add_argument("--chunks", type=int, default=400, help="chunks sampled (0: all)")
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
    tile = base // np.array(FT)
    wloc = base - tile * np.array(FT) + 1                      # window coordinates 1..T
    res = ((wloc[:, 0] * FW[1] + wloc[:, 1]) * FW[2] + wloc[:, 2]) & 15
    tid = (tile[:, 0] * 64 + tile[:, 1]) * 64 + tile[:, 2]
    rng = np.random.default_rng(0)
    order = rng.permutation(len(tid))
    tid, res = tid[order], res[order]
    srt = np.argsort(tid, kind="stable")
    tid, res = tid[srt], res[srt]
    starts = np.flatnonzero(np.r_[True, tid[1:] != tid[:-1]])
    ends = np.r_[starts[1:], len(tid)]
    chunks = []
    for s0, e0 in zip(starts, ends):
        for c0 in range(s0, e0, 256):
            chunks.append(res[c0:min(c0 + 256, e0)])
    if a.chunks and len(chunks) > a.chunks:
        chunks = [chunks[i] for i in rng.choice(len(chunks), a.chunks, replace=False)]
    tot = {"in_order": 0, "balanced": 0, "largest_first": 0, "spread": 0, "bound": 0, "ideal": 0}
    for r in chunks:
        cnt = len(r)
        G = (cnt + 15) // 16
        tot["ideal"] += G
        tot["in_order"] += group_cycles(r)
        lanes = balanced(r, cnt)
        byl = -np.ones(G * 16, np.int64)
        byl[lanes] = r
        tot["balanced"] += group_cycles(byl)
        tot["largest_first"] += largest_first(r, cnt)
        tot["spread"] += largest_first(r, cnt, spread=True)
        c = np.bincount(r, minlength=16)
        E = int(np.maximum(0, c - G).sum())
        # and a full group of multiplicity 1 holds one particle of EVERY
        # residue, so at most min_r c_r of the G - 1 full groups are clean
        tot["bound"] += max(G + (E + 7) // 8, 2 * G - 1 - min(int(c.min()), G - 1))
    sizes = np.array([len(r) for r in chunks])
    out = {"scene": name, "chunks_sampled": len(chunks), "particles_per_chunk_mean": round(float(sizes.mean()), 1)}
    for k in ("in_order", "balanced", "largest_first", "spread", "bound"):
        out[f"conflict_frac_{k}"] = round(1 - tot["ideal"] / tot[k], 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
