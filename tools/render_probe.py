"""GPU diagnostic: the lego frame's render alone (no concurrent simulation),
REPS forwards after one simulated frame, for rocprofv3 --kernel-trace --stats."""
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
    particles = int(os.environ.get('N', 100000))
    n_grid = int(os.environ.get('NG', 128))
    config = os.environ.get('CONFIG', 'lego.json')
    material = None


dev = torch.device('cuda:0')
scene = bench.build_scene(A, dev)
sim, specs = bench.make_sim(scene, dev)
sa = scene['sargs']
masks, _ = substep_masks(specs, 0.0, sa.substep_dt, sa.steps_per_frame)
sim.step(sa.substep_dt, masks)
sim.postprocess()
cam, g, mask = scene['cam'], scene['g'], scene['mask']
means_r, covs_r = sim.world_outputs(float(scene['s']), [float(v) for v in scene['c'].reshape(-1).tolist()],
                                    render_space=True)
feats, opac = g.get_features[mask].contiguous(), g.get_opacity[mask].reshape(-1).contiguous()
bg = torch.zeros(3, device=dev)


def fwd():
    return raster.forward(means_r, opac, cam.view_mat, cam.full_proj_mat, cam.cam_center, bg, cam.height, cam.width,
                          math.tan(cam.FovX * 0.5), math.tan(cam.FovY * 0.5), sh_degree=3, shs=feats,
                          cov3D_precomp=covs_r)


# RSTREAM=1: render on a second stream, as bench.py's frame loop does (EVENTS=1: hipEvents on it, 5 renders)
rstream = torch.cuda.Stream() if os.environ.get('RSTREAM') == '1' else torch.cuda.current_stream()
with torch.cuda.stream(rstream):
    for _ in range(3):
        fwd()
    torch.cuda.synchronize()
    reps = int(os.environ.get('REPS', 20))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(rstream)
    for _ in range(reps):
        K = fwd()[0]
    e1.record(rstream)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if os.environ.get('EVENTS') == '1':
        el = e0.elapsed_time(e1) / 1e3
ctx = raster.shared_context(dev.index or 0)
raster.forward(means_r, opac, cam.view_mat, cam.full_proj_mat, cam.cam_center, bg, cam.height, cam.width,
               math.tan(cam.FovX * 0.5), math.tan(cam.FovY * 0.5), sh_degree=3, shs=feats, cov3D_precomp=covs_r,
               context=ctx)
binned, _ = raster.pair_counts(ctx)
print(f"render {1e3 * el / reps:.4f} ms/frame, K {K}, binned {binned}")
