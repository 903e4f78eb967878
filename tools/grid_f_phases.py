"""Per-workgroup phases of k_grid_f in a replayed lego substep graph (GPU
diagnostic; the stamps build: GSMPM_LIB=.../libgsmpm_stamps.so).  Stamps of
slot 3 (fused.h): 0 workgroup start, 2 the tile id and the touched count
read, 3 the covering chunks' ranges and boxes in LDS (the cover record, or
the tile tables with GSMPM_COVER_RECORDS=0), 4 the node's <= 8 slot loads,
update and store done, 1 end.  Prints the median / p90 of each phase over
the workgroups of the last of 10 replays, and the span, in us
(s_memrealtime, 100 MHz)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'gaussian-splatting-mpm_amd'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import numpy as np
import torch

import bench
from gsmpm._lib import LIB, stream_of
from gsmpm.bc import substep_masks


class A:
    particles = int(os.environ.get('N', 100000))
    n_grid = int(os.environ.get('NG', 128))
    config = 'lego.json'
    material = os.environ.get('MAT')


dev = torch.device('cuda:0')
scene = bench.build_scene(A, dev)
sim, specs = bench.make_sim(scene, dev)
sa = scene['sargs']
masks, t = substep_masks(specs, 0.0, sa.substep_dt, 400)
sim.step(sa.substep_dt, masks[:100])
sim.step(sa.substep_dt, masks[100:200])
rows = []
for rep in range(10):
    sim.step(sa.substep_dt, masks[200 + 3 * rep:203 + 3 * rep])
    torch.cuda.synchronize()
    buf = np.zeros((4, 8192, 8), np.uint64)
    LIB.gsmpm_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p), stream_of(dev))
    torch.cuda.synchronize()
    g = buf[3].astype(np.int64)
    g = g[(g[:, 0] > 0) & (g[:, 4] > 0)]  # workgroups that owned a tile part
    ph = np.stack([g[:, 2] - g[:, 0], g[:, 3] - g[:, 2], g[:, 4] - g[:, 3], g[:, 1] - g[:, 4]], 1) / 100.0
    rows.append([np.median(ph, 0), np.percentile(ph, 90, 0), (g[:, 1].max() - g[:, 0].min()) / 100.0,
                 (g[:, 0].max() - g[:, 0].min()) / 100.0, len(g)])
med, p90, span, ramp, n = rows[-1]
tag = os.environ.get("TAG", "")
print(f"[{tag}] k_grid_f {n} WGs: phases (start->tile, tile->cover, cover->slots+store, ->end) "
      f"median {med.round(2).tolist()} p90 {p90.round(2).tolist()}; start ramp {ramp:.2f}, span {span:.2f} us; "
      f"spans of 10 replays {[round(r[2], 2) for r in rows]}")
