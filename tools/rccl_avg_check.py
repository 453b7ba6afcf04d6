"""One-rank RCCL process group: the AVG all-reduce GradBucket uses at N > 1 is supported by this
torch / RCCL build (a 1-GPU box cannot run two ranks; the multi-rank math is covered by the gloo
tests). Usage (GPU box): python tools/rccl_avg_check.py"""
import os

import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
t = torch.arange(8, dtype=torch.float32, device="cuda:0")
dist.all_reduce(t, op=dist.ReduceOp.AVG)
torch.cuda.synchronize()
assert torch.equal(t.cpu(), torch.arange(8, dtype=torch.float32)), t
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lesion_gnn_amd import dist as ldist
p = torch.nn.Parameter(torch.zeros(4, device="cuda:0"))
p.grad = torch.full((4,), 2.0, device="cuda:0")
b = ldist.GradBucket([p], 4, 4)
b.pack(); b.reduce(); b.unpack()
torch.cuda.synchronize()
assert b.avg and p.grad.data_ptr() == b.flat.data_ptr() and torch.all(p.grad == 2.0)
print("rccl AVG all-reduce ok; GradBucket avg =", b.avg)
dist.destroy_process_group()
