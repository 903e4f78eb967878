"""Kernel-boundary gaps of the replayed substep graph (GPU diagnostic; needs the
stamps build: GSMPM_LIB=.../libgsmpm_stamps.so).  One graph replay of three
substeps launches k_fused(P2G) k_grid_f k_fused k_grid_f k_fused k_grid_f
k_fused(G2P); the stamps kept are the last of each slot: k_fused<.,3> (slot 0),
k_fused<.,1> (slot 1), k_grid_f (slot 3).  Prints, in us on the
s_memrealtime clock: the last full k_fused (first WG start -> last WG end),
the gap to the first k_grid_f WG, k_grid_f's span, and the gap to the G2P-only
k_fused that follows it."""
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

    def span(k):
        b = buf[k].astype(np.int64)
        b = b[b[:, 0] > 0]
        return b[:, 0].min(), b[:, 1].max()

    k3, k1, gr = span(0), span(1), span(3)
    if rep == 9:
        g = buf[3].astype(np.int64)
        g = g[g[:, 0] > 0]
        st, du = (g[:, 0] - g[:, 0].min()) / 100, (g[:, 1] - g[:, 0]) / 100
        print(f"k_grid_f: {len(g)} WGs; start p50/p90/p99/max {np.percentile(st, [50, 90, 99, 100]).round(2).tolist()}"
              f"; duration p50/p90/max {np.percentile(du, [50, 90, 100]).round(2).tolist()}")
        f = buf[0].astype(np.int64)
        f = f[f[:, 0] > 0]
        st, du = (f[:, 0] - f[:, 0].min()) / 100, (f[:, 1] - f[:, 0]) / 100
        print(f"k_fused: {len(f)} WGs; start p50/p90/p99/max {np.percentile(st, [50, 90, 99, 100]).round(2).tolist()}"
              f"; duration p50/p90/max {np.percentile(du, [50, 90, 100]).round(2).tolist()}")
    rows.append([(k3[1] - k3[0]) / 100, (gr[0] - k3[1]) / 100, (gr[1] - gr[0]) / 100, (k1[0] - gr[1]) / 100])
r = np.array(rows)
print("k_fused span, gap -> k_grid_f, k_grid_f span, gap -> next k_fused (us), median of 10 replays:",
      np.median(r, 0).round(2).tolist())
print("all:", r.round(2).tolist())
