"""Probe: GPU fit path vs oracle over two extra.py-style iterations (prints errors)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting-mpm_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np, torch
import oracle as O
import test_gpu_fit as T
from conftest import rel_err
from gsmpm.fit import FitSimulator
dev = torch.device("cuda:0")
n = int(os.environ.get("N", "2000"))
x, cov, v = T._scene(n, 3)
vol = O.particle_volume(x, T.NG, T.EXT)
o = O.OracleDiff(x, cov, vol, n_grid=T.NG, grid_extent=T.EXT, gravity=T.GRAV, init_v=v, ground_only=True, **T.MAT)
g = FitSimulator(n, n_grid=T.NG, grid_extent=T.EXT, gravity=T.GRAV, **T.MAT)
t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
g.set_particles(t(x), t(cov), t(vol), t(v)); g.set_bc_ground_only()
for it in range(3):
    for s in range(30):
        o.p2g2p_forward(T.DT, s); g.forward(T.DT, s)
    o.postprocess_forward(); g.postprocess_forward()
    xs = o.x[30]
    print(it, "x30", rel_err(g.get("x", 30).cpu().numpy(), xs), "F30", rel_err(g.get("F", 30).cpu().numpy(), o.F[30]),
          "v30", rel_err(g.get("v", 30).cpu().numpy(), o.v[30]), "minJ", np.linalg.det(o.F[30].reshape(-1, 3, 3)).min())
    gx = (xs - xs.mean(0)).astype(np.float32); gc = np.full(n * 6, 10, np.float32)
    o.clear_grads(); g.clear_grads(); o.set_grads(gx, gc); g.set_grads(t(gx), t(gc))
    o.postprocess_backward(); g.postprocess_backward()
    for s in reversed(range(30)):
        o.p2g2p_backward(T.DT, s); g.backward(T.DT, s)
        if s in (29, 20, 10, 0):
            print("   s", s, "gF", rel_err(g.get("gF", s).cpu().numpy(), o.gF[s]), "gx", rel_err(g.get("gx", s).cpu().numpy(), o.gx[s]),
                  "gmu", rel_err(g.get("gmu").cpu().numpy(), o.gmu))
    a, b = g.get("glogE").cpu().numpy(), o.glogE
    r = np.abs(a - b) / (np.abs(b) + 1e-3 * np.abs(b).max())
    print(it, "glogE", rel_err(a, b), "elem p50/p99/max", np.percentile(r, 50), np.percentile(r, 99), r.max(), "argmax", r.argmax(), a[r.argmax()], b[r.argmax()])
    o.learn(); g.learn(); o.cycle_init(); g.cycle_init()
