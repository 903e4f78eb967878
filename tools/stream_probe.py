"""GPU diagnostic: does work on a second stream run beside a simulator frame?

bench.py's frame loop renders frame f - 1 on a second stream while frame f's
captured graph runs; a kernel trace showed the render starting only when the
graph ended.  This launches one lego frame (100 substeps, the captured graph)
on stream A and then small work on stream B, and reports when B's work
completed relative to A's (host clock after event syncs), for A = the default
stream and A = a second pool stream, and B's work = a torch elementwise op
or one raster.forward of the previous frame.

    python3 tools/stream_probe.py
"""
import math
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'gaussian-splatting-mpm_amd'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import torch  # noqa: E402

import bench  # noqa: E402
from gsmpm import raster  # noqa: E402
from gsmpm.bc import substep_masks  # noqa: E402


class A:
    particles, n_grid, config, material = 100000, 128, 'lego.json', None


dev = torch.device('cuda:0')
torch.cuda.set_device(dev)
scene = bench.build_scene(A, dev)
sa = scene['sargs']
cam, g, mask = scene['cam'], scene['g'], scene['mask']
feats, opac = g.get_features[mask].contiguous(), g.get_opacity[mask].reshape(-1).contiguous()
bg = torch.zeros(3, device=dev)


def trial(sim_on_default, work, reps=3):
    sstream = torch.cuda.current_stream() if sim_on_default else torch.cuda.Stream()
    bstream = torch.cuda.Stream()
    with torch.cuda.stream(sstream):
        sim, specs = bench.make_sim(scene, dev)
        t = 0.0
        for _ in range(2):  # capture + warm the graphs
            masks, t = substep_masks(specs, t, sa.substep_dt, sa.steps_per_frame)
            sim.step(sa.substep_dt, masks)
        sim.postprocess()
        means_r, covs_r = sim.world_outputs(float(scene['s']), [float(v) for v in scene['c'].reshape(-1).tolist()],
                                            render_space=True)
        ev_ready = torch.cuda.Event()
        ev_ready.record(sstream)
    torch.cuda.synchronize()
    x = torch.ones(1 << 20, device=dev)
    out = []
    for _ in range(reps):
        with torch.cuda.stream(sstream):
            masks, t = substep_masks(specs, t, sa.substep_dt, sa.steps_per_frame)
            t0 = time.perf_counter()
            sim.step(sa.substep_dt, masks)
            t_launch = time.perf_counter()
            ea = torch.cuda.Event()
            ea.record(sstream)
        with torch.cuda.stream(bstream):
            bstream.wait_event(ev_ready)  # complete long ago
            if work == 'elementwise':
                y = x * 2.0
            else:
                raster.forward(means_r, opac, cam.view_mat, cam.full_proj_mat, cam.cam_center, bg, cam.height,
                               cam.width, math.tan(cam.FovX * 0.5), math.tan(cam.FovY * 0.5), sh_degree=3,
                               shs=feats, cov3D_precomp=covs_r)
            t_b_issued = time.perf_counter()
            eb = torch.cuda.Event()
            eb.record(bstream)
        eb.synchronize()
        t_b = time.perf_counter()
        ea.synchronize()
        t_a = time.perf_counter()
        out.append((1e3 * (t_launch - t0), 1e3 * (t_b_issued - t0), 1e3 * (t_b - t0), 1e3 * (t_a - t0)))
    torch.cuda.synchronize()
    del sim
    return out


def trial_bench(timing, reps=3):
    """bench.py's pattern: B waits on an event recorded behind the previous
    frame's world_outputs, i.e. one that completes as this frame's graph starts."""
    sim, specs = bench.make_sim(scene, dev)
    bstream = torch.cuda.Stream()
    t = 0.0
    for _ in range(2):
        masks, t = substep_masks(specs, t, sa.substep_dt, sa.steps_per_frame)
        sim.step(sa.substep_dt, masks)
    torch.cuda.synchronize()
    out = []
    for _ in range(reps + 1):
        masks, t = substep_masks(specs, t, sa.substep_dt, sa.steps_per_frame)
        t0 = time.perf_counter()
        sim.step(sa.substep_dt, masks)  # frame f - 1
        sim.postprocess()
        means_r, covs_r = sim.world_outputs(float(scene['s']), [float(v) for v in scene['c'].reshape(-1).tolist()],
                                            render_space=True)
        ev = torch.cuda.Event(enable_timing=timing)
        ev.record()
        masks, t = substep_masks(specs, t, sa.substep_dt, sa.steps_per_frame)
        sim.step(sa.substep_dt, masks)  # frame f
        ea = torch.cuda.Event()
        ea.record()
        with torch.cuda.stream(bstream):
            bstream.wait_event(ev)
            raster.forward(means_r, opac, cam.view_mat, cam.full_proj_mat, cam.cam_center, bg, cam.height,
                           cam.width, math.tan(cam.FovX * 0.5), math.tan(cam.FovY * 0.5), sh_degree=3,
                           shs=feats, cov3D_precomp=covs_r)
            eb = torch.cuda.Event()
            eb.record(bstream)
        eb.synchronize()
        t_b = time.perf_counter()
        ea.synchronize()
        t_a = time.perf_counter()
        out.append((1e3 * (t_b - t0), 1e3 * (t_a - t0)))
    torch.cuda.synchronize()
    del sim
    return out[1:]


for timing in (False, True):
    for b_done, a_done in trial_bench(timing):
        print(f"bench pattern, event timing={timing}: render done at {b_done:6.3f} ms, the two frames done at "
              f"{a_done:6.3f} ms", flush=True)

for sim_on_default in (True, False):
    for work in ('elementwise', 'render'):
        r = trial(sim_on_default, work)
        for launch, issued, b_done, a_done in r[1:]:
            print(f"sim on {'default' if sim_on_default else 'pool'} stream, B = {work:11s}: graph launch "
                  f"{launch:6.3f} ms, B issued at {issued:6.3f}, B done at {b_done:6.3f}, frame done at "
                  f"{a_done:6.3f} ms", flush=True)
