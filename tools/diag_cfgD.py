"""Diagnostic: config D (bicycle 1M, 256^3) one substep, where do C errors sit."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "gaussian-splatting-mpm_amd")]
import torch
from scenarios import build_oracle_sim, lego_problem, oracle_run
from gpu_helpers import dropin_sim
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
ng = int(sys.argv[2]) if len(sys.argv) > 2 else 256
dev = torch.device("cuda:0")
prob = lego_problem(n, ng, config="bicycle.json")
ref, imps, ops = build_oracle_sim(prob, threaded=True)
dt = prob["cfg"]["substep_dt"]
s, _ = dropin_sim(prob, dev)
oracle_run(ref, imps, ops, dt, 1)
s.p2g2p(dt)
C = s.mpm_state.particle_C.to_torch().cpu().numpy().reshape(-1, 9)
v = s.mpm_state.particle_vel.to_torch().cpu().numpy()
e = np.abs(C - ref.C).max(1)
print("max|C_ref|", np.abs(ref.C).max(), "max|C_gpu|", np.abs(C).max(), "max err", e.max())
idx = np.argsort(-e)[:12]
np.set_printoptions(precision=5, linewidth=200)
for i in idx:
    print(i, "x_g", prob["x"][i], "vol", prob["vol"][i], "err", e[i])
    print("   C_gpu", C[i]); print("   C_ref", ref.C[i]); print("   v", v[i], ref.v[i])
print("n particles with err > 1e-3*max:", int((e > 1e-3 * np.abs(ref.C).max()).sum()))
