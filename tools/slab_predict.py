"""Predicted N-GPU frame time of a scene through the slab path -- config D
(bicycle 1M, 256^3) by default, or the lego headline (--config lego.json
--particles 100000 --n_grid 128) -- from pieces measured on ONE GPU (SURVEY
8(e); the round-5 verdict's item 2).  Run on the GPU box:

    python3 tools/slab_predict.py [--gpus 2,4,8] [--out profiles/r06/slab_prediction_D.json]

For each N the scene is cut exactly as gsmpm.dist.SlabDomain cuts it (count
quantiles of the base planes along the longest bbox axis, bicycle: axis 0),
and the most loaded rank's particles are simulated ALONE on this GPU (the
unsharded single-domain pipeline on the full 256^3 grid: the kernels a slab
rank runs, without its exchange) for whole frames -- its sim ms per frame and
the per-launch k_fused / k_grid_f times.  The window exchange of that rank
is priced from the geometry the library agrees on (slab_host.inc: float4
partials of W = 2 margin + 2 planes over the yz rect the particles near the
bound can reach, both neighbours) at the xGMI link rate, plus a fixed RCCL
latency per exchange round; the exchange overlaps the interior grid pass, so
only its excess over that pass is added.  Per frame: 100 substeps, a
migration round every 10 substeps (counts + payloads: two latencies), and on
rank 0 the gather of the frame (36 B a particle) and the 4946x3286 render,
which the render-aware re-cut balances against the other ranks' simulation
(rank 0 takes the share that equalises sim + render).  The model's constants
are printed with the result; the driver's first 8-GPU SCALE run checks it.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-mpm_amd"))

LINK_GBPS = 150.0       # one xGMI link, one direction (MI355X_MICROARCH.md: 7 links x ~153 GB/s)
RCCL_LAT_US = 10.0      # one grouped send/recv round between neighbours inside a graph (assumed)
MARGIN, INTERVAL = 2, 10  # bench.py make_sim's slab parameters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", default="1,2,4,8")
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--out", default=None)
    ap.add_argument("--config", default="bicycle.json")
    ap.add_argument("--particles", type=int, default=1_000_000)
    ap.add_argument("--n_grid", type=int, default=256)
    a = ap.parse_args()
    # a slab rank runs the unfolded pipeline (k_grid_f every substep, split around the exchange):
    # measure the rank's kernels in that form
    os.environ["GSMPM_FOLD"] = "0"
    import numpy as np
    import torch
    import bench as B
    from gsmpm.bc import substep_masks
    from gsmpm.dist import base_planes, slab_bounds
    from gsmpm import raster

    dev = torch.device("cuda", 0)
    ns = argparse.Namespace(config=a.config, material=None, particles=a.particles, n_grid=a.n_grid)
    sc = B.build_scene(ns, dev)
    sa = sc["sargs"]
    ng, ext = sa.n_grid, sa.grid_extent
    xg = sc["xg"]
    xh = xg.cpu().numpy()
    ntot = len(xh)
    spf, dt = sa.steps_per_frame, sa.substep_dt
    W = 2 * MARGIN + 2
    inv_dx = ng / ext
    ext3 = xh.max(0) - xh.min(0)
    axis = int(np.argmax(ext3))
    axis = 0 if ext3[0] >= 0.9 * ext3[axis] else axis

    # rank 0's render and the gather volume (measured once, whole scene)
    cam, g, mask = sc["cam"], sc["g"], sc["mask"]
    full, fspecs = B.make_sim(sc, dev)
    masks, _ = substep_masks(fspecs, 0.0, dt, spf)
    full.step(dt, masks)
    full.postprocess()
    m_r, c_r = full.world_outputs(float(sc["s"]), [float(v) for v in sc["c"].reshape(-1).tolist()], render_space=True)
    feats, opac = g.get_features[mask].contiguous(), g.get_opacity[mask].reshape(-1).contiguous()
    tx, ty = math.tan(cam.FovX * 0.5), math.tan(cam.FovY * 0.5)
    bg = torch.zeros(3, device=dev)
    rf = lambda: raster.forward(m_r, opac, cam.view_mat, cam.full_proj_mat, cam.cam_center, bg, cam.height,
                                cam.width, tx, ty, sh_degree=3, shs=feats, cov3D_precomp=c_r)
    rf()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        rf()
    torch.cuda.synchronize()
    render_ms = (time.perf_counter() - t0) / 3 * 1e3
    del full, m_r, c_r
    torch.cuda.empty_cache()

    res = {"config": f"{a.config} {ntot} particles, {ng}^3", "cut_axis": axis, "window_planes": W,
           "constants": {"xgmi_link_GBps": LINK_GBPS, "rccl_round_latency_us": RCCL_LAT_US,
                         "gather_bytes_per_particle": 36, "migration_rounds_per_frame": 2 * spf // INTERVAL},
           "render_ms_rank0": round(render_ms, 3), "per_n": {}}
    bp_all = base_planes(xh[:, [axis, (axis + 1) % 3, (axis + 2) % 3]], inv_dx)  # along the cut axis
    for N in [int(v) for v in a.gpus.split(",")]:
        if N == 1:
            bounds = [0, ng]
        else:
            xs = xh[:, [axis] + [i for i in range(3) if i != axis]]
            bounds = slab_bounds(xs, ng, ext, N, MARGIN)
        owner = np.searchsorted(np.asarray(bounds[1:-1]), np.clip(bp_all, 0, ng - 1), side="right")
        counts = np.bincount(owner, minlength=N)
        r = int(np.argmax(counts))
        sel = np.nonzero(owner == r)[0]
        # the rank's exchange rects: particles within MARGIN + 3 planes of each bound, their yz node bbox
        xb = []
        for wdx, bnd in ((0, bounds[r]), (1, bounds[r + 1])):
            if (wdx == 0 and r == 0) or (wdx == 1 and r == N - 1):
                continue
            near = np.abs(bp_all - bnd) <= MARGIN + 3
            if not near.any():
                continue
            o = [i for i in range(3) if i != axis]
            lo = np.floor(xh[near][:, o] * inv_dx - 0.5).min(0) - MARGIN
            hi = np.floor(xh[near][:, o] * inv_dx - 0.5).max(0) + 3 + MARGIN
            ny, nz = [int(min(ng, h) - max(0, l)) for l, h in zip(lo, hi)]
            xb.append(16 * W * ny * nz)
        t = torch.from_numpy(sel).to(dev)
        sub = dict(sc)
        sub["xg"], sub["covs"], sub["vols"] = sc["xg"][t], sc["covs"][t], sc["vols"][t]
        sim, specs = B.make_sim(sub, dev)
        tt = 0.0
        masks, tt = substep_masks(specs, tt, dt, spf)
        sim.step(dt, masks)  # capture
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.frames):
            masks, tt = substep_masks(specs, tt, dt, spf)
            sim.step(dt, masks)
        e1.record()
        e1.synchronize()
        sim_ms = e0.elapsed_time(e1) / a.frames
        masks, tt = substep_masks(specs, tt, dt, spf)
        prof = sim.profile(dt, masks)
        ngrid = int(prof[3]) if prof[3] > 0 else spf
        kf_us, kg_us = prof[0] / (spf + 1) * 1e3, prof[1] / ngrid * 1e3
        del sim
        torch.cuda.empty_cache()
        # slab ranks run the unfolded pipeline (k_grid_f every substep, in two passes around the exchange):
        # per substep k_fused + k_grid_f, plus the exchange's excess over the interior pass (~half of k_grid_f)
        x_us = (max(xb) / (LINK_GBPS * 1e3) + RCCL_LAT_US) if xb else 0.0
        sub_us = kf_us + kg_us + max(0.0, x_us - 0.5 * kg_us) + (3.0 if xb else 0.0)  # + k_win_update
        mig_ms = (2 * spf // INTERVAL) * RCCL_LAT_US * 1e-3 if N > 1 else 0.0
        sim_pred_ms = spf * sub_us * 1e-3 + mig_ms
        gather_ms = (36 * ntot * (N - 1) / N) / (LINK_GBPS * 1e6 * min(N - 1, 7)) + 0.05 if N > 1 else 0.0
        # render-aware share: rank 0 simulates w / (w + N - 1) of the scene and renders; the others balance it
        frame_pred_ms = max(sim_pred_ms, (sim_pred_ms * N + render_ms) / N) + gather_ms if N > 1 \
            else sim_ms + render_ms
        res["per_n"][str(N)] = {
            "bounds": [int(b) for b in bounds], "max_rank": r, "max_rank_particles": int(counts[r]),
            "per_rank_particles": [int(c) for c in counts],
            "measured_one_gpu": {"rank_sim_ms_per_frame_unfolded": round(sim_ms, 4),
                                 "k_fused_us": round(kf_us, 2), "k_grid_f_us": round(kg_us, 2),
                                 "k_grid_f_launches_per_frame": ngrid},
            "exchange_bytes_per_substep_per_window": xb, "exchange_us_per_substep": round(x_us, 2),
            "predicted_substep_us": round(sub_us, 2), "predicted_sim_ms_per_frame": round(sim_pred_ms, 3),
            "predicted_gather_ms": round(gather_ms, 3), "predicted_frame_ms": round(frame_pred_ms, 3),
            "predicted_particle_substeps_per_s": ntot * spf / (frame_pred_ms * 1e-3)}
        print(N, json.dumps(res["per_n"][str(N)]), flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
