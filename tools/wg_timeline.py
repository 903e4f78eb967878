"""Workgroup timeline of one eager substep (GPU diagnostic)."""
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
ms = sim.profile(sa.substep_dt, masks[:1])
buf = np.zeros((4, 4096, 8), np.uint64)
LIB.gsmpm_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p), stream_of(dev))
print('event ms p2g/grid/g2p', ms)
for k, name in enumerate(('p2g', 'g2p')):
    st = buf[k, :, 0].astype(np.int64); en = buf[k, :, 1].astype(np.int64)
    valid = st > 0
    n = int(valid.sum())
    if n == 0:
        print(name, ': no stamps'); continue
    st, en = st[:n], en[:n]
    t0 = st.min()
    dur = (en - st) / 100.0  # us
    print(f"{name}: {n} WGs; start spread {(st.max()-t0)/100:.1f} us; end {(en.max()-t0)/100:.1f} us; WG dur us: min {dur.min():.1f} med {np.median(dur):.1f} max {dur.max():.1f}")
    order = np.argsort(st)
    print('  first starts (us):', ((st[order[:8]] - t0) / 100).round(1), ' last starts:', ((st[order[-8:]] - t0) / 100).round(1))
    hist = np.histogram((st - t0) / 100, bins=10)
    print('  start histogram', hist[0].tolist(), 'edges', hist[1].round(1).tolist())

st = buf[1, :, :].astype(np.int64)
v = st[:, 0] > 0
st = st[v]
seg = lambda a, b: (st[:, b] - st[:, a]) / 100.0
ok = st[:, 2] > 0
print('g2p first-chunk segments (us): start->staged', np.median(seg(0, 2)[ok]), ' staged->particles', np.median(seg(2, 3)[ok]),
      ' particles->reserved', np.median(seg(3, 4)[ok]), ' reserved->end', np.median(seg(4, 1)[ok]))
print('  max:', seg(0, 2)[ok].max(), seg(2, 3)[ok].max(), seg(3, 4)[ok].max(), seg(4, 1)[ok].max())

p = buf[0].astype(np.int64); p = p[p[:, 0] > 0]
ok = p[:, 2] > 0
sg = lambda a, b: np.median((p[ok, b] - p[ok, a]) / 100.0)
print('p2g first-chunk median segments (us): start->front', sg(0, 2), ' front->scattered', sg(2, 3), ' scattered->written', sg(3, 4), ' ->end', sg(4, 1))
order = np.argsort(-(st[:, 1] - st[:, 0]))
print("slowest WGs: dur, seg staged/part/resv/end, cnt, tile, hwreg")
for i in order[:12]:
    r = st[i]
    print(((r[1]-r[0])/100), ((r[2]-r[0])/100, (r[3]-r[2])/100, (r[4]-r[3])/100, (r[1]-r[4])/100), r[5], r[6], hex(r[7]))
print("fastest:")
for i in order[-4:]:
    r = st[i]
    print(((r[1]-r[0])/100), r[5], r[6], hex(r[7]))
d = (st[:, 1] - st[:, 0]) / 100
print("dur percentiles 50/75/90/95/99:", np.percentile(d, [50, 75, 90, 95, 99]).round(1))
f = buf[2].astype(np.int64); f = f[f[:, 0] > 0]
if len(f):
    t0 = f[:, 0].min()
    sg = lambda a, b: np.median((f[:, b] - f[:, a]) / 100.0)
    print(f'finish_bins: {len(f)} WGs; start spread {(f[:,0].max()-t0)/100:.1f} us, end {(f[:,1].max()-t0)/100:.1f} us; median staged {sg(0,2)} counted+scanned {sg(2,3)} written {sg(3,4)} scattered {sg(4,1)}')
# P2G: duration vs co-residency on the same CU (HW_ID: CU_ID bits 8-11, SH bit 12, SE bits 13-15 on gfx9)
p = buf[0].astype(np.int64); p = p[p[:, 0] > 0]
if len(p):
    hw = p[:, 6]
    cu = (hw >> 8) & 0xF; sh = (hw >> 12) & 1; se = (hw >> 13) & 0x7
    key = se * 32 + sh * 16 + cu
    xcc = None
    dur = (p[:, 1] - p[:, 0]) / 100.0
    from collections import Counter
    occ = Counter(key.tolist())
    per = np.array([occ[k] for k in key.tolist()])
    for n in sorted(set(per.tolist())):
        sel = per == n
        print(f"p2g WGs on CUs hosting {n} WGs: {sel.sum()} WGs, median dur {np.median(dur[sel]):.1f} us, max {dur[sel].max():.1f}, mean cnt {p[sel,5].mean():.0f}")
    big = p[:, 5] >= 200
    print(f"p2g dur by chunk size: >=200: median {np.median(dur[big]):.1f}; <200: median {np.median(dur[~big]):.1f}; distinct CU keys {len(occ)}")
