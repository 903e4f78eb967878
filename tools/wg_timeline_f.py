"""Workgroup timeline of one fused-pipeline k_fused launch (G2P + P2G) on the
bench scene (GPU diagnostic).  Stamps: 0 start, 2 window staged, 3 G2P done,
4 scatter done, 1 end (s_memrealtime, 100 MHz)."""
import os, sys, ctypes
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'gaussian-splatting-mpm_amd'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import numpy as np, torch
import bench
from gsmpm.bc import substep_masks
from gsmpm._lib import LIB, stream_of
class A: particles = int(os.environ.get('N', 100000)); n_grid = int(os.environ.get('NG', 128)); config = 'lego.json'; material = os.environ.get('MAT')
dev = torch.device('cuda:0')
scene = bench.build_scene(A, dev)
sim, specs = bench.make_sim(scene, dev)
sa = scene['sargs']
masks, t = substep_masks(specs, 0.0, sa.substep_dt, 300)
sim.step(sa.substep_dt, masks[:100]); sim.step(sa.substep_dt, masks[100:200])
print('stats', sim.debug_stats(), 'pipeline', sim.pipeline)
ms = sim.profile(sa.substep_dt, masks[200:203])  # K(P2G), grid, K, grid, K, grid, K(G2P)
print('event ms K/grid/bins per 3 substeps', ms)
buf = np.zeros((4, 8192, 8), np.uint64)
LIB.gsmpm_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p), stream_of(dev))
b = buf[0].astype(np.int64)
b = b[b[:, 0] > 0]
t0 = b[:, 0].min()
ok = b[:, 2] > 0
dur = (b[:, 1] - b[:, 0]) / 100
print(f"k_fused: {len(b)} WGs ({ok.sum()} with a chunk); start spread {(b[:,0].max()-t0)/100:.1f} us; end {(b[:,1].max()-t0)/100:.1f} us")
print("  WG dur percentiles 50/90/99/max:", np.percentile(dur[ok], [50, 90, 99, 100]).round(2))
seg = lambda a, c: (b[ok, c] - b[ok, a]) / 100
for name, a, c in (("start->staged", 0, 2), ("staged->g2p", 2, 3), ("g2p->scattered", 3, 4), ("scattered->end", 4, 1)):
    x = seg(a, c)
    print(f"  {name}: median {np.median(x):.2f} p90 {np.percentile(x, 90):.2f} max {x.max():.2f}")
st = (b[ok, 0] - t0) / 100
print("  start histogram", np.histogram(st, bins=10)[0].tolist(), "edges", np.histogram(st, bins=10)[1].round(1).tolist())
print("  WGs per XCC", np.bincount(b[ok, 7] & 0xf).tolist())
cnt = b[ok, 5]
print("  chunk sizes: mean", cnt.mean().round(1), "<=64:", (cnt <= 64).sum(), ">=200:", (cnt >= 200).sum())
big = cnt >= 200
print("  dur by size >=200 median", np.median(dur[ok][big]).round(2), "<64 median", np.median(dur[ok][cnt < 64]).round(2))
order = np.argsort(-dur[ok])[:12]
print("  slowest WGs: (dur, cnt, staged, g2p, scatter, store)")
for i in order:
    r = b[ok][i]
    print("   ", round(dur[ok][i], 2), int(r[5]), [round((r[c] - r[a]) / 100, 2) for a, c in ((0, 2), (2, 3), (3, 4), (4, 1))],
          "start", round((r[0] - t0) / 100, 2))
# per-CU load: HW_ID (slot 6) cu_id [11:8], sh_id [12], se_id [15:13]; XCC (slot 7)
hw = b[:, 6]; xcc = b[:, 7] & 0xf
cu = (xcc << 8) | (((hw >> 13) & 7) << 5) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15)
cuk = cu[ok]; sizes = cnt.astype(np.int64); durs = dur[ok]
u, inv = np.unique(cuk, return_inverse=True)
load = np.bincount(inv, weights=sizes); nwg = np.bincount(inv)
print(f"  CUs used {len(u)}; WGs per CU hist {np.bincount(nwg).tolist()}; particles per CU p50/p90/max {np.percentile(load,[50,90,100]).round(0).tolist()}")
maxdur = np.zeros(len(u)); np.maximum.at(maxdur, inv, durs)
for lo_, hi_ in ((0, 300), (300, 450), (450, 600), (600, 2000)):
    m = (load >= lo_) & (load < hi_)
    if m.any(): print(f"    CU load [{lo_},{hi_}): {m.sum()} CUs, max WG dur median {np.median(maxdur[m]):.2f} max {maxdur[m].max():.2f}")
same = {}
for i in np.nonzero(ok)[0]:
    same.setdefault(int(cu[i]), []).append(int(i))
print("  WG sets sharing a CU (sample):", list(same.values())[:8])
# the SIMD of each workgroup's wave 0 (HW_ID simd_id [5:4]): are the three
# workgroups of a CU starting on the same SIMD (small chunks' only wave
# stacked on it) or spread?
simd0 = (hw >> 4) & 3
print("  wave-0 SIMD histogram (WGs with a chunk):", np.bincount(simd0[ok], minlength=4).tolist())
tuples = {}
for c_, idx in same.items():
    if len(idx) == 3:
        key = tuple(sorted(int(simd0[i]) for i in idx))
        tuples[key] = tuples.get(key, 0) + 1
print("  wave-0 SIMDs of the 3 WGs of a CU (count):", sorted(tuples.items(), key=lambda kv: -kv[1])[:8])
# second-chunk WGs (grid-stride): count WGs whose end - start >> single chunk
ms2 = sim.time_kernels(sa.substep_dt, masks[203], reps=20)
print('time_kernels K/grid/bins', ms2)
g = buf[3].astype(np.int64)
g = g[g[:, 0] > 0]
t0 = g[:, 0].min()
okg = g[:, 2] > 0
print(f"k_grid_f: {len(g)} WGs ({okg.sum()} with a tile); start spread {(g[:,0].max()-t0)/100:.1f} us; end {(g[:,1].max()-t0)/100:.1f} us")
segg = lambda a, c: (g[okg, c] - g[okg, a]) / 100
for name, a, c in (("start->tile", 0, 2), ("tile->covers", 2, 3), ("covers->nodes", 3, 4), ("nodes->end", 4, 1)):
    x = segg(a, c)
    print(f"  {name}: median {np.median(x):.2f} p90 {np.percentile(x, 90):.2f} max {x.max():.2f}")
d = (g[okg, 1] - g[okg, 0]) / 100
print("  WG dur percentiles 50/90/99/max:", np.percentile(d, [50, 90, 99, 100]).round(2))
st = (g[okg, 0] - t0) / 100
print("  start histogram", np.histogram(st, bins=10)[0].tolist(), "edges", np.histogram(st, bins=10)[1].round(1).tolist())
