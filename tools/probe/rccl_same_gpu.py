"""Probe: can two RCCL ranks share one GPU on this box? (multi-rank rehearsal)"""
import os
import torch
import torch.distributed as dist
rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
t = torch.full((1024,), float(rank), device="cuda")
r = torch.empty_like(t)
ops = [dist.P2POp(dist.isend, t, 1 - rank), dist.P2POp(dist.irecv, r, 1 - rank)]
for q in dist.batch_isend_irecv(ops):
    q.wait()
torch.cuda.synchronize()
print("rank", rank, "got", float(r[0]), flush=True)
dist.destroy_process_group()
