"""Fused vs per-phase pipeline on config A, per substep (GPU diagnostic)."""
import os, sys
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path[:0] = [os.path.join(ROOT, 'gaussian-splatting-mpm_amd'), os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'oracle')]
import numpy as np, torch
from scenarios import lego_problem
from gpu_helpers import dropin_sim

dev = torch.device('cuda:0')
prob = lego_problem(5000, 64)
dt = prob['cfg']['substep_dt']
R = int(os.environ.get('R', '10'))
a, _ = dropin_sim(prob, dev, phased=False)
b, _ = dropin_sim(prob, dev, phased=True)
a._sim.set_rebin_interval(R)


def rel(p, q):
    return float(np.abs(p - q).max() / max(np.abs(q).max(), 1e-30))


def fields(s):
    st = s.mpm_state
    return {k: getattr(st, f).to_torch().cpu().numpy().reshape(len(prob['x']), -1)
            for k, f in (('x', 'particle_xyz'), ('v', 'particle_vel'), ('C', 'particle_C'), ('F', 'particle_F_trial'))}


fa, fb = fields(a), fields(b)
print('init', {k: rel(fa[k], fb[k]) for k in fa})
a.p2g2p(dt)
b.p2g2p(dt)
fields(a), fields(b)  # flush the wrappers' pending substeps
ga =a._sim.get_grid('v_out').cpu().numpy()
gb = b._sim.get_grid('v_out').cpu().numpy()
d = np.abs(ga - gb).max(-1)
bad = np.argwhere(d > 1e-4 * np.abs(gb).max())
print('grid v_out rel', rel(ga, gb), 'bad nodes', len(bad), 'nonzero phased', int((np.abs(gb).max(-1) > 0).sum()),
      'nonzero fused', int((np.abs(ga).max(-1) > 0).sum()))
fa, fb = fields(a), fields(b)
badp = np.nonzero(np.abs(fa['v'] - fb['v']).max(1) > 1e-3 * np.abs(fb['v']).max())[0]
goodp = np.nonzero(np.abs(fa['v'] - fb['v']).max(1) <= 1e-3 * np.abs(fb['v']).max())[0]
np.set_printoptions(precision=5, suppress=False, linewidth=200)
print('bad particles', len(badp), 'x', fb['x'][badp[:4]], '\n v fused', fa['v'][badp[:4]], '\n v phased', fb['v'][badp[:4]])
print('good particles', len(goodp), 'v fused', fa['v'][goodp[:3]], '\n v phased', fb['v'][goodp[:3]])
print('max|v| fused', np.abs(fa['v']).max(0), 'phased', np.abs(fb['v']).max(0))
if len(bad):
    print(' first bad', bad[:10].tolist(), 'fused', ga[tuple(bad[0])], 'phased', gb[tuple(bad[0])])
    print(' bad (i%8, j%8, k%7) hist', np.unique(np.stack([bad[:, 0] % 8, bad[:, 1] % 8, bad[:, 2] % 7], 1), axis=0,
                                                 return_counts=True)[1][:20])
for s in range(12):
    a.p2g2p(dt)
    b.p2g2p(dt)
    fa, fb = fields(a), fields(b)
    e = {k: rel(fa[k], fb[k]) for k in fa}
    bad = np.abs(fa['v'] - fb['v']).max(1) > 1e-3 * np.abs(fb['v']).max()
    print(s + 1, {k: f'{v:.2e}' for k, v in e.items()}, 'bad rows', int(bad.sum()), np.nonzero(bad)[0][:8],
          'stats', a._sim.debug_stats())
