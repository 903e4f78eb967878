"""GPU diagnostic for rocprofv3 --pmc passes: one eager lego frame (NSUB
substeps, re-binning launches included) and, with RENDER=1, postprocess +
world outputs + two rasterizer forwards of that frame."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'gaussian-splatting-mpm_amd'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import math  # noqa: E402

import torch  # noqa: E402

import bench  # noqa: E402
from gsmpm import raster  # noqa: E402
from gsmpm.bc import substep_masks  # noqa: E402


class A:
    particles = int(os.environ.get('N', 100000))
    n_grid = int(os.environ.get('NG', 128))
    config = os.environ.get('CONFIG', 'lego.json')
    material = os.environ.get('MAT')


dev = torch.device('cuda:0')
scene = bench.build_scene(A, dev)
sim, specs = bench.make_sim(scene, dev)
sa = scene['sargs']
masks, t = substep_masks(specs, 0.0, sa.substep_dt, int(os.environ.get('NSUB', 100)))
sim.profile(sa.substep_dt, masks)
if os.environ.get('RENDER') == '1':
    sim.postprocess()
    cam, g, mask = scene['cam'], scene['g'], scene['mask']
    means_r, covs_r = sim.world_outputs(float(scene['s']), [float(v) for v in scene['c'].reshape(-1).tolist()],
                                        render_space=True)
    for _ in range(2):
        raster.forward(means_r, g.get_opacity[mask].reshape(-1).contiguous(), cam.view_mat, cam.full_proj_mat,
                       cam.cam_center, torch.zeros(3, device=dev), cam.height, cam.width, math.tan(cam.FovX * 0.5),
                       math.tan(cam.FovY * 0.5), sh_degree=3, shs=g.get_features[mask].contiguous(),
                       cov3D_precomp=covs_r)
torch.cuda.synchronize()
print("done")
