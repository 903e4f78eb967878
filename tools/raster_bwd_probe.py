"""GPU diagnostic: rasterizer forward + backward (the extra.py loss.backward()
path) on the lego frame (100k Gaussians, 800x800, SH degree 3, precomputed
covariances as main.py/extra.py pass them), REPS iterations, for timing and
rocprofv3 --kernel-trace --stats.  Prints ms per forward and per
forward + backward."""
import math
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'gaussian-splatting-mpm_amd'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import torch  # noqa: E402

import bench  # noqa: E402
from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer  # noqa: E402
from gsmpm.bc import substep_masks  # noqa: E402


class A:
    particles = int(os.environ.get('N', 100000))
    n_grid = int(os.environ.get('NG', 128))
    config = os.environ.get('CONFIG', 'lego.json')
    material = None


REPS = int(os.environ.get('REPS', 20))
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
feats = g.get_features[mask].contiguous()
opac = g.get_opacity[mask].reshape(-1, 1).contiguous()
st = GaussianRasterizationSettings(image_height=cam.height, image_width=cam.width,
                                   tanfovx=math.tan(cam.FovX * 0.5), tanfovy=math.tan(cam.FovY * 0.5),
                                   bg=torch.zeros(3, device=dev), scale_modifier=1.0, viewmatrix=cam.view_mat,
                                   projmatrix=cam.full_proj_mat, sh_degree=3, campos=cam.cam_center,
                                   prefiltered=False, debug=False)
ras = GaussianRasterizer(st)
m3 = means_r.detach().clone().requires_grad_(True)
c6 = covs_r.detach().clone().requires_grad_(True)
sh = feats.detach().clone().requires_grad_(True)
op = opac.detach().clone().requires_grad_(True)
target = torch.rand(3, cam.height, cam.width, device=dev)


def fwd():
    img, _ = ras(means3D=m3, means2D=None, shs=sh, colors_precomp=None, opacities=op, scales=None, rotations=None,
                 cov3D_precomp=c6)
    return img


def step():
    img = fwd()
    (img - target).abs().mean().backward()


for _ in range(3):
    step()
torch.cuda.synchronize()
t0 = time.perf_counter()
with torch.no_grad():
    for _ in range(REPS):
        fwd()
torch.cuda.synchronize()
t1 = time.perf_counter()
for _ in range(REPS):
    step()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"forward (no grad) {(t1 - t0) / REPS * 1e3:.3f} ms; forward+backward with the L1 loss "
      f"{(t2 - t1) / REPS * 1e3:.3f} ms per iteration ({REPS} reps)")
