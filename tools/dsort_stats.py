"""GPU diagnostic: the hand-written depth order's bucket statistics
(gsmpm_raster_dsort_stats) on the lego and bicycle frames of bench.py."""
import math
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'gaussian-splatting-mpm_amd'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import torch  # noqa: E402

os.environ.setdefault("GSMPM_RASTER_DSORT", "bucket")  # the bucket form's statistics at both sizes

import bench  # noqa: E402
from gsmpm import raster  # noqa: E402


class A:
    particles, n_grid, config, material = 100000, 128, 'lego.json', None


dev = torch.device('cuda:0')
for cfg, n, ng in (('lego.json', 100000, 128), ('bicycle.json', 1000000, 256)):
    A.config, A.particles, A.n_grid = cfg, n, ng
    scene = bench.build_scene(A, dev)
    sim, specs = bench.make_sim(scene, dev)
    sim.postprocess()
    cam, g, mask = scene['cam'], scene['g'], scene['mask']
    means_r, covs_r = sim.world_outputs(float(scene['s']), [float(v) for v in scene['c'].reshape(-1).tolist()],
                                        render_space=True)
    feats, opac = g.get_features[mask].contiguous(), g.get_opacity[mask].reshape(-1).contiguous()
    ctx = raster.RasterContext()
    raster.forward(means_r, opac, cam.view_mat, cam.full_proj_mat, cam.cam_center, torch.zeros(3, device=dev),
                   cam.height, cam.width, math.tan(cam.FovX * 0.5), math.tan(cam.FovY * 0.5), sh_degree=3, shs=feats,
                   cov3D_precomp=covs_r, context=ctx)
    torch.cuda.synchronize()
    print(cfg, n, raster.dsort_stats(ctx))
