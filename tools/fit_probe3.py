"""Probe: run-to-run spread of the GPU fit adjoints (atomic summation order) vs the oracle."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting-mpm_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np, torch
import oracle as O
import test_gpu_fit as T
from conftest import rel_err
from gsmpm.fit import FitSimulator
dev = torch.device("cuda:0")
n = 2000
x, cov, v = T._scene(n, 3)
vol = O.particle_volume(x, T.NG, T.EXT)
t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)

def run(engine):
    out = []
    for it in range(2):
        for s in range(30):
            engine.forward(T.DT, s)
        engine.postprocess_forward()
        xs = engine.get("x", 30)
        gx = (xs - xs.mean(0)).cpu().numpy() if it == 0 else None
        out.append(None)
    return out

res = []
o = O.OracleDiff(x, cov, vol, n_grid=T.NG, grid_extent=T.EXT, gravity=T.GRAV, init_v=v, ground_only=True, **T.MAT)
gxs = []
ref = []
for it in range(2):
    for s in range(30):
        o.p2g2p_forward(T.DT, s)
    o.postprocess_forward()
    gx = (o.x[30] - o.x[30].mean(0)).astype(np.float32); gxs.append(gx)
    o.clear_grads(); o.set_grads(gx, np.full(n * 6, 10, np.float32)); o.postprocess_backward()
    for s in reversed(range(30)):
        o.p2g2p_backward(T.DT, s)
    ref.append((o.glogE.copy(), o.gy.copy()))
    o.learn(); o.cycle_init()
runs = []
for r in range(12):
    g = FitSimulator(n, n_grid=T.NG, grid_extent=T.EXT, gravity=T.GRAV, **T.MAT)
    g.set_particles(t(x), t(cov), t(vol), t(v)); g.set_bc_ground_only()
    per = []
    for it in range(2):
        for s in range(30):
            g.forward(T.DT, s)
        g.postprocess_forward()
        g.clear_grads(); g.set_grads(t(gxs[it]), t(np.full(n * 6, 10, np.float32))); g.postprocess_backward()
        for s in reversed(range(30)):
            g.backward(T.DT, s)
        per.append((g.get("glogE").cpu().numpy(), g.get("gy").cpu().numpy()))
        g.learn(); g.cycle_init()
    runs.append(per)
    del g
def pct(a, b):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    r = np.abs(a - b) / (np.abs(b) + 1e-3 * np.abs(b).max() + 1e-30)
    return [float((r > t).mean()) for t in (5e-3, 2e-2, 5e-2)], float(np.percentile(r, 99))
for it in range(2):
    fo = [pct(runs[r][it][0], ref[it][0]) for r in range(12)]
    fg = [pct(runs[r][it][0], runs[0][it][0]) for r in range(1, 12)]
    print(it, "frac>(5e-3,2e-2,5e-2) gpu-vs-oracle worst", [max(f[0][k] for f in fo) for k in range(3)], "p99", max(f[1] for f in fo),
          "| gpu-vs-gpu worst", [max(f[0][k] for f in fg) for k in range(3)], "p99", max(f[1] for f in fg))
for it in range(2):
    vo = [rel_err(runs[r][it][0], ref[it][0]) for r in range(12)]
    vg = [rel_err(runs[r][it][0], runs[0][it][0]) for r in range(1, 12)]
    print(it, "glogE gpu-vs-oracle max %.2e med %.2e | gpu-vs-gpu max %.2e med %.2e" % (max(vo), np.median(vo), max(vg), np.median(vg)))
    b = ref[it][0]
    worst = int(np.argmax([rel_err(runs[r][it][0], b) for r in range(12)]))
    d = np.abs(runs[worst][it][0] - b); i = d.argmax()
    print("   worst run", worst, "particle", i, runs[worst][it][0][i], b[i], "x", x[i])
