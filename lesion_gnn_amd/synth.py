"""Seeded synthetic k-NN lesion-graph batches.

The real inputs (DDR / APTOS lesion graphs, reference datasets/nodes/lesions.py:111-177) need
offline segmentation models and data that are not in this environment, so benchmarks and tests
use graphs of the same shape: lesion centroids `pos ~ U[0,1)^2` (float64, like the reference's
centroids, lesions.py:175), KNNGraph(k, loop=True) topology (configs/config.py:47: each node's k
nearest nodes including itself, flow source_to_target, neighbours ordered by (distance, index)),
node features x ~ N(0,1) fp32 and graph labels y ~ U{0..C-1}, collated like PyG Batch.

This is data plumbing on the host (CPU torch), not the timed hot path.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch


@dataclass
class Batch:
    x: torch.Tensor            # fp32 [sumN, d_in]
    edge_index: torch.Tensor   # int64 [2, sumE], rows (source, target), grouped by target
    batch: torch.Tensor        # int64 [sumN], sorted graph id
    ptr: torch.Tensor          # int64 [B+1]
    y: torch.Tensor            # int64 [B]
    pos: torch.Tensor          # fp64 [sumN, 2]
    num_graphs: int

    def to(self, device) -> "Batch":
        return Batch(self.x.to(device), self.edge_index.to(device), self.batch.to(device),
                     self.ptr.to(device), self.y.to(device), self.pos.to(device),
                     self.num_graphs)

    @property
    def num_nodes(self) -> int:
        return self.x.size(0)

    @property
    def num_edges(self) -> int:
        return self.edge_index.size(1)


def knn_edges(pos: torch.Tensor, k: int, loop: bool = True) -> torch.Tensor:
    """k-NN graph of G same-size graphs at once. pos [G, n, 2] fp64 -> local edge_index
    [G, 2, n*kk] with kk = min(k, n) (loop) / min(k+1, n) - 1 (no loop)."""
    G, n, _ = pos.shape
    d2 = ((pos[:, :, None, :] - pos[:, None, :, :]) ** 2).sum(-1)  # [G, query, cand]
    order = torch.sort(d2, dim=-1, stable=True).indices
    kk = min(k if loop else k + 1, n)
    nb = order[:, :, :kk]  # [G, query, kk]
    q = torch.arange(n).view(1, n, 1).expand(G, n, kk)
    if not loop:
        keep = nb != q
        nb = nb[keep].view(G, n, kk - 1)
        q = q[keep].view(G, n, kk - 1)
    return torch.stack([nb.reshape(G, -1), q.reshape(G, -1)], dim=1)


def graph_sizes(num_graphs: int, dist: str, gen: torch.Generator, n: int = 64,
                lo: int = 16, hi: int = 512) -> list[int]:
    """'fixed': all n; 'lognormal': clip(round(LogNormal(ln 24, 1)), 1, 512) (C3);
    'powerlaw': discrete power law alpha=2 on [lo, hi] (C5)."""
    if dist == "fixed":
        return [n] * num_graphs
    if dist == "lognormal":
        z = torch.randn(num_graphs, generator=gen, dtype=torch.float64)
        s = torch.exp(math.log(24.0) + z).round().clamp(1, 512)
        return [int(v) for v in s]
    if dist == "powerlaw":
        vals = torch.arange(lo, hi + 1, dtype=torch.float64)
        p = vals.pow(-2.0)
        idx = torch.multinomial(p / p.sum(), num_graphs, replacement=True, generator=gen)
        return [int(vals[i]) for i in idx]
    raise ValueError(dist)


def make_batch(num_graphs: int, n: int = 64, k: int = 8, d_in: int = 128, num_classes: int = 5,
               seed: int = 0, sizes: list[int] | str | None = None, loop: bool = True,
               last_channel_class: bool = False) -> Batch:
    """Collated batch of `num_graphs` synthetic lesion graphs (deterministic in `seed`)."""
    gen = torch.Generator().manual_seed(seed)
    if sizes is None or isinstance(sizes, str):
        sizes = graph_sizes(num_graphs, sizes or "fixed", gen, n)
    assert len(sizes) == num_graphs
    total = sum(sizes)
    pos = torch.rand(total, 2, generator=gen, dtype=torch.float64)
    x = torch.randn(total, d_in, generator=gen, dtype=torch.float32)
    if last_channel_class:  # reference node features: 1024 encoder channels + lesion class id
        x[:, -1] = torch.randint(0, 5, (total,), generator=gen).float()
    y = torch.randint(0, num_classes, (num_graphs,), generator=gen)
    offsets = [0]
    for s in sizes:
        offsets.append(offsets[-1] + s)
    ptr = torch.tensor(offsets, dtype=torch.int64)
    batch = torch.repeat_interleave(torch.arange(num_graphs), torch.tensor(sizes))
    # k-NN per graph, vectorised over graphs of equal size, collated in graph order
    pieces: list[torch.Tensor | None] = [None] * num_graphs
    by_size: dict[int, list[int]] = {}
    for g, s in enumerate(sizes):
        by_size.setdefault(s, []).append(g)
    for s, gs in by_size.items():
        idx = torch.tensor(gs)
        starts = ptr[idx]
        local_pos = torch.stack([pos[offsets[g]:offsets[g] + s] for g in gs])
        ei = knn_edges(local_pos, k, loop) + starts.view(-1, 1, 1)
        for j, g in enumerate(gs):
            pieces[g] = ei[j]
    edge_index = (torch.cat(pieces, dim=1) if num_graphs else
                  torch.empty(2, 0, dtype=torch.int64))
    return Batch(x, edge_index.contiguous(), batch, ptr, y, pos, num_graphs)
