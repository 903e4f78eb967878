"""GPU diagnostic: one substep with a prescribed deformed F_trial, KEEP_GRID,
grid momentum vs oracle (isolates the P2G stress-force path)."""
import sys
sys.path[:0] = ['tests', 'oracle', 'gaussian-splatting-mpm_amd']
import numpy as np, torch
from scenarios import *
from conftest import rel_err
from gpu_helpers import dropin_sim
dev = torch.device('cuda:0')
for mat, quirk in (('jelly', False), ('metal', True)):
    prob = lego_problem(4000, 48)
    rng = np.random.default_rng(1)
    F = (np.eye(3)[None] + 0.01 * rng.standard_normal((len(prob['x']), 3, 3))).astype(np.float32).reshape(-1, 9)
    ref, imps, ops = build_oracle_sim(prob, material=mat, jelly_quirk=quirk, with_collider=False)
    ref.F_trial[:] = F
    s, _ = dropin_sim(prob, dev, material=mat, jelly_fcr=not quirk, keep_grid=True, with_collider=False)
    s.mpm_state.particle_F_trial.from_torch(torch.from_numpy(F).to(dev))
    ref.substep(1e-4, [0] * len(imps), [0] * len(ops))
    s.p2g2p(1e-4)
    gm = s.mpm_state.grid_mass.to_torch().cpu().numpy().reshape(-1)
    gvin = s.mpm_state.grid_v_in.to_torch().cpu().numpy().reshape(-1, 3)
    print(mat, 'grid mass', rel_err(gm, ref.gm), 'v_in', rel_err(gvin, ref.gv_in), 'max|v_in|', np.abs(ref.gv_in).max(),
          'stress max', np.abs(ref.stress).max())
    d = np.abs(gvin - ref.gv_in).max(1); i = int(d.argmax())
    print('  worst node', i, gvin[i], ref.gv_in[i], 'mass', gm[i], ref.gm[i])
