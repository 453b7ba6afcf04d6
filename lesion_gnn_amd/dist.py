"""Data parallelism over the GPUs of one node (new capability — the reference trains on one
device, src/lesion_gnn/training.py:64-66).

Graphs are independent (k-NN edges never cross graphs), so a global batch is split into
contiguous per-rank shards with no halo exchange; the only exchange is ONE all-reduce of the
flat fp32 gradient per step (RCCL over xGMI on MI355X via backend "nccl"; gloo on CPU for tests).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_bounds(costs: list[int] | torch.Tensor, world: int) -> list[int]:
    """Contiguous split of items with per-item `costs` (e.g. edges per graph) into `world`
    shards of near-equal total cost (greedy prefix split). Returns world+1 item offsets."""
    c = torch.as_tensor(costs, dtype=torch.float64)
    n = c.numel()
    pref = torch.cat([torch.zeros(1, dtype=torch.float64), torch.cumsum(c, 0)])
    total = pref[-1].item()
    bounds = [0]
    for r in range(1, world):
        target = total * r / world
        i = int(torch.searchsorted(pref, torch.tensor(target, dtype=torch.float64)).item())
        i = max(bounds[-1], min(i, n))
        bounds.append(i)
    bounds.append(n)
    return bounds


def allreduce_grads(params: list[torch.nn.Parameter], local_count: int, global_count: int,
                    group=None) -> None:
    """grad <- sum_r (n_r / N) grad_r: the gradient of the global-batch mean loss when each rank
    holds the gradient of its local-batch mean loss. One flat bucket, one all-reduce."""
    grads = [p.grad for p in params if p.grad is not None]
    if not grads:
        return
    flat = torch._utils._flatten_dense_tensors(grads)
    flat.mul_(local_count / global_count)
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    for g, f in zip(grads, torch._utils._unflatten_dense_tensors(flat, grads)):
        g.copy_(f)


def broadcast_params(module: torch.nn.Module, src: int = 0, group=None) -> None:
    """Start every replica from rank `src`'s weights."""
    for t in list(module.parameters()) + list(module.buffers()):
        dist.broadcast(t.data, src=src, group=group)
