"""Rehearse the RCCL code paths with 2 ranks on one GPU (if RCCL allows it)."""
import os, sys, time
sys.path.insert(0, os.getcwd())
import torch
import torch.distributed as dist
rank = int(os.environ["RANK"]); world = int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
from sda_amd.parallel.comm import Comm
c = Comm()
t = torch.full((4,), rank + 1, dtype=torch.int64, device="cuda")
b = c.broadcast(t.clone(), src=0)
r = c.reduce_sum(t.clone(), dst=0)
peer = 1 - rank
send = torch.full((1 << 20,), rank + 7, dtype=torch.uint8, device="cuda")
recv = torch.empty_like(send)
h = c.exchange_async([(peer, send)], [(peer, recv)])
h.wait()
c.barrier()
ok = bool(b.eq(1).all()) and (rank != 0 or bool(r.eq(3).all())) and bool(recv.eq(peer + 7).all())
print(f"rank {rank} rccl same-device ok={ok}", flush=True)
dist.destroy_process_group()
