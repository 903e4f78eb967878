"""GPU diagnostic: FCR jelly divergence by substep + device SVD vs oracle SVD."""
import sys, os
sys.path[:0] = ['tests', 'oracle', 'gaussian-splatting-mpm_amd']
import numpy as np, torch
from scenarios import *
from conftest import rel_err
from gpu_helpers import dropin_sim
import oracle as O
from gsmpm._lib import LIB, ptr, stream_of
dev = torch.device('cuda:0')
rng = np.random.default_rng(0)
A = (np.eye(3)[None] + 1e-3 * rng.standard_normal((20000, 3, 3))).astype(np.float32)
A[:5000] = rng.standard_normal((5000, 3, 3))
At = torch.from_numpy(A.reshape(-1, 9)).to(dev)
U = torch.empty_like(At); V = torch.empty_like(At); S = torch.empty(len(A), 3, device=dev)
LIB.gsmpm_svd3(ptr(At), len(A), ptr(U), ptr(S), ptr(V), stream_of())
torch.cuda.synchronize()
U, S, V = U.cpu().numpy().reshape(-1, 3, 3), S.cpu().numpy(), V.cpu().numpy().reshape(-1, 3, 3)
worst = 0; wr = 0; bitexact = 0
for i in range(len(A)):
    u, s, v = O.svd3(A[i])
    worst = max(worst, np.abs(s - S[i]).max())
    wr = max(wr, np.abs(u @ v.T - U[i] @ V[i].T).max())
    bitexact += np.array_equal(u, U[i]) and np.array_equal(s, S[i]) and np.array_equal(v, V[i])
print('svd: max |sig diff|', worst, 'max |UV^T diff|', wr, 'bit-exact', bitexact, '/', len(A))
for mat, quirk in (('jelly', False), ('metal', True)):
    prob = lego_problem(4000, 48)
    ref, imps, ops = build_oracle_sim(prob, material=mat, jelly_quirk=quirk)
    s, _ = dropin_sim(prob, dev, material=mat, jelly_fcr=not quirk)
    t = 0.0
    for k in range(12):
        t = oracle_run(ref, imps, ops, 1e-4, 1, t)
        s.p2g2p(1e-4)
        st = s.mpm_state
        gv = st.particle_vel.to_torch().cpu().numpy(); gx = st.particle_xyz.to_torch().cpu().numpy()
        gF = st.particle_F_trial.to_torch().cpu().numpy().reshape(-1, 9)
        dv = np.abs(gv - ref.v).max(1)
        i = int(dv.argmax())
        print(mat, k + 1, 'x', f'{rel_err(gx, ref.x):.2e}', 'v', f'{rel_err(gv, ref.v):.2e}', 'F', f'{rel_err(gF, ref.F_trial):.2e}',
              'worst p', i, 'v gpu', gv[i], 'v ref', ref.v[i], 'x', ref.x[i])
