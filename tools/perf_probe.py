"""Per-frame kernel timings + bucket stats for the bench scene (GPU diagnostic)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'gaussian-splatting-mpm_amd'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import torch
import bench
from gsmpm.bc import substep_masks
class A: particles = int(os.environ.get('N', 100000)); n_grid = int(os.environ.get('NG', 128)); config = 'lego.json'; material = os.environ.get('MAT')
dev = torch.device('cuda:0')
scene = bench.build_scene(A, dev)
sim, specs = bench.make_sim(scene, dev)
sa = scene['sargs']; t = 0.0
for f in range(int(os.environ.get('FRAMES', 10))):
    st = sim.debug_stats()
    masks, t = substep_masks(specs, t, sa.substep_dt, 10)
    ms = sim.profile(sa.substep_dt, masks)
    masks, t = substep_masks(specs, t, sa.substep_dt, 90)
    torch.cuda.synchronize(); t0 = time.perf_counter()
    sim.step(sa.substep_dt, masks); torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(f"frame {f}: {st}  eager us/launch p2g {ms[0]*100:.1f} grid {ms[1]*100:.1f} g2p {ms[2]*100:.1f} | graph 90 substeps {el*1e3:.2f} ms = {el/90*1e6:.1f} us/substep", flush=True)
