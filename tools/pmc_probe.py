"""Runs a few eager lego substeps (for rocprofv3 --pmc passes; GPU diagnostic)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'gaussian-splatting-mpm_amd'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import torch
import bench
from gsmpm.bc import substep_masks
class A: particles = int(os.environ.get('N', 100000)); n_grid = int(os.environ.get('NG', 128)); config = os.environ.get('CONFIG', 'lego.json'); material = os.environ.get('MAT')
dev = torch.device('cuda:0')
scene = bench.build_scene(A, dev)
sim, specs = bench.make_sim(scene, dev)
sa = scene['sargs']
masks, t = substep_masks(specs, 0.0, sa.substep_dt, int(os.environ.get('NSUB', 20)))
sim.profile(sa.substep_dt, masks)
torch.cuda.synchronize()
print("done")
