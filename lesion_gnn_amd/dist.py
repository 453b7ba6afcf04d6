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


_SEGMENTS = None  # the SegmentedCapture in progress on this process, if any


def sync_all_reduce(t: torch.Tensor, group) -> None:
    """SUM all-reduce of the SyncBN sums over `group`. Eager: the collective runs here. Inside a
    SegmentedCapture: the HIP graph being captured ends here, the collective is recorded to run
    eagerly between that graph and the next one on replay, and capture resumes — so a step whose
    forward and backward exchange statistics still replays as graphs (no collective is ever
    captured)."""
    seg = _SEGMENTS
    if seg is not None and seg.capturing:
        seg.split(lambda: dist.all_reduce(t, group=group))
    else:
        dist.all_reduce(t, group=group)


class SegmentedCapture:
    """A training step captured as a chain of HIP graphs split at its collectives:
        replay() = graph_0, collective_0, graph_1, collective_1, ..., graph_n
    Every graph shares one memory pool and is replayed in capture order (torch's rule for
    graphs sharing a pool), so a tensor a collective reduces keeps its address from the graph
    that writes it to the one that reads it. The split points come from sync_all_reduce (the
    SyncBN exchanges of GIN, inside forward AND backward: the backward's split happens on the
    autograd thread, which runs on the capture stream); `extra` collectives (the gradient
    all-reduce) are added with add_collective between two capture() calls."""

    def __init__(self, dev):
        self.dev = torch.device(dev)
        self.pool = torch.cuda.graph_pool_handle()
        self.stream = torch.cuda.Stream(self.dev)
        self.items: list = []  # ("graph", CUDAGraph) | ("collective", callable)
        self.capturing = False
        self._cur = None

    def _begin(self) -> None:
        self._cur = torch.cuda.CUDAGraph()
        with torch.cuda.stream(self.stream):
            # relaxed: the backward's split points end and begin captures on the autograd thread
            self._cur.capture_begin(pool=self.pool, capture_error_mode="relaxed")

    def _end(self) -> None:
        with torch.cuda.stream(self.stream):
            self._cur.capture_end()
        self.items.append(("graph", self._cur))
        self._cur = None

    def split(self, collective) -> None:
        self._end()
        self.items.append(("collective", collective))
        self._begin()

    def add_collective(self, collective) -> None:
        self.items.append(("collective", collective))

    def capture(self, fn) -> None:
        """Capture fn() (on the capture stream) as one or more graphs."""
        global _SEGMENTS
        if _SEGMENTS is not None:
            raise RuntimeError("nested SegmentedCapture")
        cur = torch.cuda.current_stream(self.dev)
        self.stream.wait_stream(cur)
        torch.cuda.synchronize(self.dev)
        _SEGMENTS = self
        self.capturing = True
        self._begin()
        try:
            with torch.cuda.stream(self.stream):
                fn()
        finally:
            self._end()
            self.capturing = False
            _SEGMENTS = None
        cur.wait_stream(self.stream)

    @property
    def num_graphs(self) -> int:
        return sum(1 for k, _ in self.items if k == "graph")

    def plan(self) -> tuple:
        return tuple("graph" if k == "graph" else "rccl" for k, _ in self.items)

    def replay(self) -> None:
        for kind, obj in self.items:
            if kind == "graph":
                obj.replay()
            else:
                obj()


def broadcast_params(module: torch.nn.Module, src: int = 0, group=None) -> None:
    """Start every replica from rank `src`'s weights."""
    for t in list(module.parameters()) + list(module.buffers()):
        dist.broadcast(t.data, src=src, group=group)


class GradBucket:
    """The flat-gradient exchange split into its device part and its collective, so a training
    step captured in HIP graphs keeps every copy kernel inside the graphs and only the RCCL call
    outside them (a collective is never captured):
      pack()    flat <- concat(grad_i) [* local / global]  (capturable: ONE cat kernel at the end
                                                            of the backward graph)
      reduce()  all_reduce(flat, AVG | SUM)                (eager, RCCL over xGMI)
      unpack()  grad_i <- flat[slice_i]                    (no kernel: grad_i becomes a view of
                                                            the reduced buffer, which the optimizer
                                                            then reads in place)
    With equal shards (local / global = 1 / world) on RCCL the mean is the collective's own AVG,
    so pack is the concatenation alone; otherwise (gloo, unequal shards) pack pre-scales and the
    collective sums. The flat buffer is allocated once, so replays of the captured parts reuse it.
    Equivalent to allreduce_grads (tests/test_distributed.py)."""

    def __init__(self, params: list[torch.nn.Parameter], local_count: int, global_count: int,
                 group=None):
        self.params = list(params)
        self.scale = local_count / global_count
        self.group = group
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.avg = (dist.is_initialized() and dist.get_backend(group) == "nccl"
                    and local_count * world == global_count)
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device if self.params else torch.device("cpu")
        self.flat = torch.empty(n, dtype=torch.float32, device=dev)
        self.views = []
        off = 0
        for p in self.params:
            self.views.append(self.flat[off:off + p.numel()].view_as(p))
            off += p.numel()

    def pack(self) -> None:
        torch.cat([p.grad.reshape(-1) for p in self.params], out=self.flat)
        if not self.avg and self.scale != 1.0:
            self.flat.mul_(self.scale)

    def reduce(self) -> None:
        op = dist.ReduceOp.AVG if self.avg else dist.ReduceOp.SUM
        dist.all_reduce(self.flat, op=op, group=self.group)

    def unpack(self) -> None:
        for p, v in zip(self.params, self.views):
            p.grad = v
