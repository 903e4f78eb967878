"""Probe: the slab RCCL path with every rank on cuda:0, stage by stage.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29533 tools/probe/rccl_shared_probe.py [stage]

Each rank gets an NCCL_HOSTID of its own (RCCL then accepts both ranks on one
device, over its socket transport).  Stages, each printed when done:
  1 torch.distributed nccl group + all_reduce
  2 the library's own RCCL communicator (gsmpm.dist.RcclTransport)
  3 a 2-slab scene stepped eagerly (GSMPM_SLAB_GRAPH=0)
  4 the same stepped through the captured step-call graph
faulthandler prints the Python stack of a crash."""
import faulthandler
import os
import sys

SEGV = None
if os.environ.get("SEGV_TRACE"):  # native backtrace of a crash (tools/probe/segv_trace.c)
    import ctypes
    SEGV = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "segv_trace.so"))
else:
    faulthandler.enable()
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting-mpm_amd"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "oracle")]
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
os.environ.update(NCCL_HOSTID=f"gsmpm-probe-rank{rank}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")
last = int(sys.argv[1]) if len(sys.argv) > 1 else 4

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def say(*a):
    print(f"[rank {rank}]", *a, flush=True)


torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", device_id=dev)
t = torch.full((4,), float(rank + 1), device=dev)
dist.all_reduce(t)
torch.cuda.synchronize()
say("stage 1: all_reduce", t.tolist())
if os.environ.get("TORCH_GRAPH"):  # RCCL inside a captured graph, without the library
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    u = torch.ones(8, device=dev)
    with torch.cuda.stream(s):
        dist.all_reduce(u)  # warm-up outside capture
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            dist.all_reduce(u)
    u.fill_(1.0)
    g.replay()
    torch.cuda.synchronize()
    say("stage 1g: captured all_reduce replayed", u.tolist()[:2])
if last < 2:
    sys.exit(0)
from gsmpm.dist import RcclTransport, SlabDomain  # noqa: E402
xp = RcclTransport(rank, world, device=dev)
say("stage 2: comm", hex(xp.comm.value or 0))
if last >= 3:
    from test_dist_slab import EXT, FIXED, KW, NG, scene  # noqa: E402
    x, v, cov, vol = scene()
    for stage, graph in ((3, "0"), (4, "1")):
        if stage > last:
            break
        os.environ["GSMPM_SLAB_GRAPH"] = graph
        if SEGV is not None:
            SEGV.segv_trace_reinstall()
        dom = SlabDomain(x, cov, vol, v=v, rank=rank, world=world, transport=xp, n_grid=NG, grid_extent=EXT,
                         margin=2, interval=10, device=dev, jelly_fcr=True, **KW)
        dom.add_fixed_cube(*FIXED)
        dom.add_plane_collider([0, 0, 0.4], [0, 0, 1])
        for s in range(3):
            dom.step(1e-4, [0b11] * 20)
            torch.cuda.synchronize()
            say(f"stage {stage}: call {s} ok, n = {dom.n}, stats {dom.stats()}")
        xs = dom.gather_field("x")
        if rank == 0:
            say(f"stage {stage}: gathered", tuple(xs.shape))
        dom.engine.close()
xp.close()
dist.destroy_process_group()
say("done")
