"""Message-passing layers with PyG 2.5.1 constructor signatures and state_dict keys, computed by
the HIP kernels of liblgnn.so.

GCNConv  — PyG GCNConv(in, out): keys `lin.weight`, `bias` (added conv)
GINConv  — PyG GINConv(nn, eps=0): keys `nn.*`, `eps` (reference gin.py:23)
global_mean_pool / global_add_pool — reference gin.py:33 / gat.py:56 (+ add)
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from . import _lib, ops
from .graph import Graph, as_graph


def glorot_(t: torch.Tensor) -> None:
    a = math.sqrt(6.0 / (t.size(-2) + t.size(-1)))
    with torch.no_grad():
        t.uniform_(-a, a)


class GCNConv(nn.Module):
    """out = D^-1/2 (A + I) D^-1/2 X W^T + b (gcn_norm with add_remaining_self_loops)."""

    def __init__(self, in_channels: int, out_channels: int):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.lin = nn.Linear(in_channels, out_channels, bias=False)
        self.bias = nn.Parameter(torch.zeros(out_channels))
        glorot_(self.lin.weight)

    def forward(self, x: torch.Tensor, edge_index, act: int = _lib.LGNN_ACT_NONE) -> torch.Tensor:
        g = as_graph(edge_index, x.size(0))
        return ops.node_linear(x, self.lin.weight, self.bias, g, "gcn", 0.0, act)


def global_mean_pool(x: torch.Tensor, batch: torch.Tensor, size: int | None = None,
                     graph: Graph | None = None) -> torch.Tensor:
    g = graph if graph is not None else _pool_graph(x, batch, size)
    return ops.segment_pool(x, g, mean=True)


def global_add_pool(x: torch.Tensor, batch: torch.Tensor, size: int | None = None,
                    graph: Graph | None = None) -> torch.Tensor:
    g = graph if graph is not None else _pool_graph(x, batch, size)
    return ops.segment_pool(x, g, mean=False)


def _pool_graph(x: torch.Tensor, batch: torch.Tensor, size: int | None) -> Graph:
    _lib.require_gpu(x, batch)
    empty = torch.empty(2, 0, dtype=torch.int64, device=x.device)
    return Graph(empty, x.size(0), batch, size)
