"""Probe: the drop-in MPM_Simulator(fitting=True) loop vs the oracle (prints errors)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting-mpm_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np, torch
import oracle as O
import test_gpu_fit as T
from conftest import rel_err
from argparse import ArgumentParser
from arguments import MPMParams
from mpm_solver.solver import MPM_Simulator
dev = torch.device("cuda:0")
x, cov, v = T._scene(2000, 3)
vol = O.particle_volume(x, T.NG, T.EXT)
parser = ArgumentParser()
group = MPMParams(parser, {"n_grid": T.NG, "grid_extent": T.EXT, "E": T.MAT["E"], "nu": T.MAT["nu"],
                           "density": T.MAT["density"], "gravity": list(T.GRAV)})
args = group.extract(parser.parse_args([]))
args.fitting = True
print({k: getattr(args, k) for k in ("n_grid", "grid_extent", "E", "nu", "density", "gravity")})
t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
sim = MPM_Simulator(t(x), t(cov), t(vol), args, init_v=t(v))
sim.set_bc_ground_only()
o = O.OracleDiff(x, cov, vol, n_grid=T.NG, grid_extent=T.EXT, gravity=T.GRAV, init_v=v, ground_only=True, **T.MAT)
for it in range(2):
    for s in range(T.NSUB):
        sim.p2g2p(T.DT, s); o.p2g2p_forward(T.DT, s)
    sim.postprocess_forward(); o.postprocess_forward()
    means = sim.mpm_state.particle_xyz.to_torch()[30]
    covs = sim.mpm_state.particle_cov.to_torch()
    print(it, "x30", rel_err(means.cpu().numpy(), o.x[30]), "cov", rel_err(covs.cpu().numpy(), o.cov))
    gx = (means - means.mean(0)).detach(); gc = torch.ones_like(covs) * 10
    sim.clear_grads(); o.clear_grads()
    sim.mpm_state.set_grads(gx, gc); o.set_grads(gx.cpu().numpy(), gc.cpu().numpy())
    sim.postprocess_backward(); o.postprocess_backward()
    print("  gF30", rel_err(sim._fit.get("gF", 30).cpu().numpy(), o.gF[30]), "gx30", rel_err(sim._fit.get("gx", 30).cpu().numpy(), o.gx[30]))
    for s in reversed(range(T.NSUB)):
        sim.p2g2p_backward(T.DT, s); o.p2g2p_backward(T.DT, s)
        if s in (29, 15, 0):
            print("   s", s, "gF", rel_err(sim._fit.get("gF", s).cpu().numpy(), o.gF[s]), "gx", rel_err(sim._fit.get("gx", s).cpu().numpy(), o.gx[s]))
    a, b = sim.mpm_model.logE.grad.to_torch().cpu().numpy(), o.glogE
    print(it, "glogE", rel_err(a, b), np.abs(b).max(), np.abs(a - b).argmax(), a[np.abs(a - b).argmax()], b[np.abs(a - b).argmax()])
    sim.learn(); o.learn(); sim.mpm_state.cycle_init(); o.cycle_init()
