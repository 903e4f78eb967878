"""Stamps of k_scan_tiles phases during one eager substep (GPU diagnostic)."""
import os, sys, ctypes
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'gaussian-splatting-mpm_amd'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import numpy as np, torch
import bench
from gsmpm.bc import substep_masks
from gsmpm._lib import LIB, stream_of
class A: particles = 100000; n_grid = 128; config = 'lego.json'; material = None
dev = torch.device('cuda:0')
scene = bench.build_scene(A, dev)
sim, specs = bench.make_sim(scene, dev)
sa = scene['sargs']
masks, t = substep_masks(specs, 0.0, sa.substep_dt, 20)
sim.profile(sa.substep_dt, masks)
sim.profile(sa.substep_dt, masks[:1])
buf = np.zeros((4, 4096, 8), np.uint64)
LIB.gsmpm_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p), stream_of(dev))
r = buf[0, 0].astype(np.int64)
print("scan stamps (us from start): staged %.2f counted %.2f scanned %.2f written %.2f end %.2f" % tuple((r[[2, 3, 4, 5, 1]] - r[0]) / 100))
