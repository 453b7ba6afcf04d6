"""Message-passing layers with PyG 2.5.1 constructor signatures and state_dict keys, computed by
the HIP kernels of liblgnn.so.

GCNConv  — PyG GCNConv(in, out): keys `lin.weight`, `bias` (added conv)
GINConv  — PyG GINConv(nn, eps=0): keys `nn.*`, `eps` (reference gin.py:23)
GraphConv — PyG GraphConv(in, out): keys `lin_rel.*`, `lin_root.weight` (DRGNet,
           reference models/drgnet.py:30-33,55)
global_mean_pool / global_add_pool — reference gin.py:33 / gat.py:56 (+ add)
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from . import _lib, dropout, ops
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


class GraphConv(nn.Module):
    """out_i = lin_rel(sum_{j->i} w_ji x_j) + lin_root(x_i) (aggr 'add', no self loops), with the
    optional per-edge weight of the reference's GaussianDistance transform (drgnet.py:55, :103).

    The weighted aggregation runs in the HIP segmented-sum kernel (lgnn_spmm, transpose CSR in
    the backward) on whichever side of lin_rel has a width divisible by 4 — A(X) W^T == A(X W^T)
    — so DRGNet's wide input layer (d_in 1025) aggregates its `hidden` outputs and the final
    GraphConv(hidden, 1) its inputs; the two Linears run on the tile kernels or the library GEMM
    (ops.linear_auto)."""

    def __init__(self, in_channels: int, out_channels: int):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.lin_rel = nn.Linear(in_channels, out_channels, bias=True)
        self.lin_root = nn.Linear(in_channels, out_channels, bias=False)

    def forward(self, x: torch.Tensor, edge_index, edge_weight: torch.Tensor | None = None
                ) -> torch.Tensor:
        _lib.require_gpu(x)
        g = as_graph(edge_index, x.size(0))
        if edge_weight is None and g.adj_values is not None:  # weighted adj_t (ToSparseTensor)
            edge_weight = g.adj_values
        kind = g.weighted(edge_weight) if edge_weight is not None else "gin"
        K, N = self.in_channels, self.out_channels
        root = ops.linear_auto(x, self.lin_root.weight)
        if K % 4 == 0 and (N % 4 != 0 or K <= N):
            rel = ops.linear_auto(ops.spmm(x, g, kind), self.lin_rel.weight, self.lin_rel.bias)
        elif N % 4 == 0:
            rel = ops.spmm(ops.linear_auto(x, self.lin_rel.weight), g, kind) + self.lin_rel.bias
        else:  # neither width divisible by 4: zero-pad the input columns for the aggregation
            pad = (-K) % 4
            agg = ops.spmm(torch.nn.functional.pad(x, (0, pad)), g, kind)[:, :K]
            rel = ops.linear_auto(agg, self.lin_rel.weight, self.lin_rel.bias)
        return rel + root


class BatchNorm(nn.Module):
    """torch_geometric.nn.norm.BatchNorm: torch.nn.BatchNorm1d wrapped as `.module` (state_dict
    keys `module.{weight,bias,running_mean,running_var,num_batches_tracked}`)."""

    def __init__(self, in_channels: int, eps: float = 1e-5, momentum: float = 0.1):
        super().__init__()
        self.module = nn.BatchNorm1d(in_channels, eps=eps, momentum=momentum)


class MLP(nn.Module):
    """Parameter container with PyG MLP(channel_list, act="ELU", dropout=p) structure
    (norm="batch_norm", plain_last=True): `lins.{i}`, `norms.{i}.module`. The 3-entry form of the
    reference GIN (gin.py:23) is computed by the fused GINConv kernel chain."""

    def __init__(self, channel_list: list[int], dropout: float = 0.0):
        super().__init__()
        if len(channel_list) != 3:
            raise ValueError("the fused GIN MLP supports channel_list [d1, d2, d3] (reference "
                             "gin.py:23 uses [d1, d2, d2])")
        self.channel_list = list(channel_list)
        self.dropout = float(dropout)
        self._dropout_key = repr(self.dropout)
        self.lins = nn.ModuleList([nn.Linear(a, b) for a, b in
                                   zip(channel_list[:-1], channel_list[1:])])
        self.norms = nn.ModuleList([BatchNorm(channel_list[1])])


class GINConv(nn.Module):
    """PyG GINConv(nn, eps=0, train_eps=False): nn((1 + eps) x_i + sum_{j->i} x_j), with `nn` a
    2-layer MLP with BatchNorm + ELU (reference gin.py:23); keys `nn.*` and the `eps` buffer."""

    def __init__(self, mlp: MLP, eps: float = 0.0):
        super().__init__()
        self.nn = mlp
        self.initial_eps = float(eps)  # train_eps=False: eps stays at its initial value
        self.register_buffer("eps", torch.full((1,), float(eps)))
        self.sync_group = None  # torch.distributed group for SyncBN (None: per-replica stats)
        self.sync_count = None  # fixed global node count under SyncBN (None: all-reduced)

    def _mask(self, x: torch.Tensor, mask):
        """The MLP's dropout mask: the model's (drawn with its other masks in one launch), else
        one drawn here from the device's global generator; None when dropout is inactive."""
        mlp = self.nn
        if mask is not None or mlp.dropout == 0.0 or not self.training:
            return mask if (mlp.dropout > 0.0 and self.training) else None
        return dropout.masks(dropout.global_state(x.device),
                             [(x.size(0), mlp.channel_list[1])], dropout.key(mlp, mlp.dropout))[0]

    def forward(self, x: torch.Tensor, edge_index, act: int = _lib.LGNN_ACT_NONE,
                mask: torch.Tensor | None = None) -> torch.Tensor:
        g = as_graph(edge_index, x.size(0))
        mlp = self.nn
        bn = mlp.norms[0].module
        mask = self._mask(x, mask)
        return ops.gin_conv(x, mlp.lins[0].weight, mlp.lins[0].bias, bn, mlp.lins[1].weight,
                            mlp.lins[1].bias, g, self.initial_eps, mask, act, self.sync_group,
                            self.sync_count)

    def stack_spec(self, x: torch.Tensor, act: int, mask: torch.Tensor | None = None) -> dict:
        """This conv's weights, BatchNorm, eps and dropout mask for ops.gin_stack."""
        mlp = self.nn
        mask = self._mask(x, mask)
        return dict(W1=mlp.lins[0].weight, b1=mlp.lins[0].bias, bn=mlp.norms[0].module,
                    W2=mlp.lins[1].weight, b2=mlp.lins[1].bias, eps=self.initial_eps, mask=mask,
                    act=act, group=self.sync_group, sync_count=self.sync_count)

    def head_fusable(self, x: torch.Tensor) -> bool:
        mlp = self.nn
        return ops.gin_conv_head_eligible(x, mlp.lins[0].weight, mlp.lins[1].weight)

    def forward_head(self, x: torch.Tensor, g, act: int, W_out: torch.Tensor,
                     b_out: torch.Tensor, mean: bool, mask: torch.Tensor | None = None
                     ) -> torch.Tensor:
        """forward(x) followed by global pool + out_proj (W_out, b_out) in one autograd node
        (ops.gin_conv_head): the model's last conv and readout. Returns the logits."""
        mlp = self.nn
        bn = mlp.norms[0].module
        mask = self._mask(x, mask)
        return ops.gin_conv_head(x, mlp.lins[0].weight, mlp.lins[0].bias, bn, mlp.lins[1].weight,
                                 mlp.lins[1].bias, W_out, b_out, g, self.initial_eps, mask, act,
                                 self.sync_group, self.sync_count, mean)


class GATConv(nn.Module):
    """PyG 2.5.1 GATConv(in, out, heads, dropout) with concat=True, negative_slope=0.2,
    add_self_loops=True, bias=True (reference gat.py:31). state_dict: `lin.weight`, `att_src`,
    `att_dst` [1, H, C], `bias` [H*C]."""

    def __init__(self, in_channels: int, out_channels: int, heads: int = 1, dropout: float = 0.0,
                 negative_slope: float = 0.2):
        super().__init__()
        self.in_channels, self.out_channels, self.heads = in_channels, out_channels, heads
        self.negative_slope, self.dropout = negative_slope, dropout
        self._dropout_key = repr(float(dropout))
        self.lin = nn.Linear(in_channels, heads * out_channels, bias=False)
        self.att_src = nn.Parameter(torch.empty(1, heads, out_channels))
        self.att_dst = nn.Parameter(torch.empty(1, heads, out_channels))
        self.bias = nn.Parameter(torch.zeros(heads * out_channels))
        glorot_(self.lin.weight)
        glorot_(self.att_src)
        glorot_(self.att_dst)

    def mask_shape(self, g) -> tuple:
        """The attention-dropout mask: one multiplier per (target-CSR slot, head)."""
        return (g.csr("gat").col.numel(), self.heads)

    def _mask(self, x: torch.Tensor, g, mask):
        if self.dropout == 0.0 or not self.training:
            return None
        if mask is not None:
            return mask
        return dropout.masks(dropout.global_state(x.device), [self.mask_shape(g)],
                             dropout.key(self, self.dropout))[0]

    def forward(self, x: torch.Tensor, edge_index, act: int = _lib.LGNN_ACT_NONE,
                bf16: bool = False, mask: torch.Tensor | None = None,
                planes: tuple | None = None) -> torch.Tensor:
        """planes: (lin.weight's, its transpose's) split-3 planes from ops.s3_weight_bundle."""
        g = as_graph(edge_index, x.size(0))
        mask = self._mask(x, g, mask)
        return ops.gat_conv(x, self.lin.weight, self.att_src, self.att_dst, self.bias, g,
                            self.heads, self.negative_slope, mask, act, bf16, planes)

    def forward_head(self, x: torch.Tensor, g, act: int, W_out: torch.Tensor,
                     b_out: torch.Tensor, mean: bool, bf16: bool = False,
                     mask: torch.Tensor | None = None, planes: tuple | None = None
                     ) -> torch.Tensor:
        """forward(x) followed by global pool + out_proj (W_out, b_out) in one autograd node
        (ops.gat_conv_head): the model's last conv and readout. Returns the logits."""
        mask = self._mask(x, g, mask)
        return ops.gat_conv_head(x, self.lin.weight, self.att_src, self.att_dst, self.bias,
                                 W_out, b_out, g, self.heads, self.negative_slope, mask, act,
                                 bf16, mean, planes)


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


class SortAggregation(nn.Module):
    """PyG 2.5.1 SortAggregation(k) (reference models/drgnet.py:37, :59): per graph, rows sorted
    by the last channel (descending, stable), top k kept (zero rows when fewer), elements equal
    to min(x) - 1 zeroed; [ΣN, D] -> [B, k * D]. HIP: lgnn_sort_pool_fwd / _bwd."""

    def __init__(self, k: int):
        super().__init__()
        self.k = int(k)

    def forward(self, x: torch.Tensor, index: torch.Tensor | None = None,
                ptr: torch.Tensor | None = None, dim_size: int | None = None, dim: int = -2,
                graph: Graph | None = None) -> torch.Tensor:
        if dim not in (-2, 0) or x.dim() != 2:
            raise ValueError("SortAggregation: x must be [num_nodes, channels], dim=-2")
        if graph is None:
            if index is None:
                raise ValueError("SortAggregation needs the batch index (or a Graph)")
            graph = _pool_graph(x, index, dim_size)
        return ops.sort_pool(x, graph, self.k)

    def __repr__(self) -> str:
        return f"{self.__class__.__name__}(k={self.k})"
