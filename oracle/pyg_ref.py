"""CPU oracle: plain-torch restatement of the PyG 2.5.1 op sequence on the lesion-gnn hot path.

TEST INFRASTRUCTURE ONLY. Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module, and only as the checker / the timed CPU baseline.
The product path (``lesion_gnn_amd``) never imports it and has no CPU fallback.

Parity status: **unpinned against PyG itself.** torch_geometric / torch_scatter / torch_sparse /
torch_cluster are not installed in this image and the reference (zacharielegault/lesion-gnn @ v2)
holds no test or fixture on the GNN path. This file restates the documented
PyG 2.5.1 operator sequence (pinned in requirements.lock:407 of the reference) with the same ATen
primitives PyG runs on CPU (index_select -> message -> scatter_add_ / scatter_reduce_), and is
pinned by analytic known-answer tests (tests/test_oracle.py) plus the only reference fixture that
exists (the GaussianDistance KATs, reference test/test_transforms.py:20,29,38).

Reference call sites restated here (paths relative to the reference root):
  * GIN:  src/lesion_gnn/models/gin.py:17-35  (GINConv(MLP([d1,d2,d2], act="ELU", dropout)) :23,
          F.elu :31, dropout :32, global_mean_pool :33)
  * GAT:  src/lesion_gnn/models/gat.py:17-59  (GATConv(d1, d2 // heads, heads, dropout) :31,
          F.elu :51, global_mean_pool :56)
  * GCN:  NEW: skeleton of gin.py:17-35 with PyG GCNConv semantics.
  * Loss: src/lesion_gnn/models/base.py:88-96 (criterion), :196-201 (training_step).
  * Graph: configs/config.py:47 (KNNGraph(k, loop=True)); PyG Batch collation
          (src/lesion_gnn/datasets/datamodule.py:63-69).
"""
from __future__ import annotations

import math
from itertools import pairwise

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch import Tensor

# ----------------------------------------------------------------------------------------------
# dropout masks: the device generator of lgnn_dropout_masks (include/lgnn.h), restated in numpy
# ----------------------------------------------------------------------------------------------

_GOLD = np.uint64(0x9E3779B97F4A7C15)
_STREAM = np.uint64(0xD1B54A32D192ED03)


def _mix64(z: np.ndarray) -> np.ndarray:
    """splitmix64 finalizer (uint64 arithmetic wraps mod 2^64 in numpy arrays)."""
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


class DropoutMasks:
    """The masks one lgnn_dropout_masks launch draws from generator state (seed, counter): mask
    j (the j-th shape of the launch) element i is scale when its 24 bits u(j, i) >= thr, else 0.
    The oracle applies them where torch's F.dropout draws its Bernoulli mask (same semantics:
    keep with probability 1 - p, scale 1 / (1 - p)); the models below take them as `masks`.
    Test infrastructure: it restates the product's generator so parity can be checked with
    dropout on; it is not torch's generator (no PyG run could be pinned to it anyway)."""

    def __init__(self, seed: int, counter: int, p: float):
        with np.errstate(over="ignore"):
            z = np.array([seed & (2 ** 64 - 1)], dtype=np.uint64) ^ \
                (np.array([counter & (2 ** 64 - 1)], dtype=np.uint64) * _GOLD)
            self.key = _mix64(z)[0]
        self.thr = int(p * 16777216.0)
        self.scale = np.float32(1.0 / (1.0 - p))
        self.p = p

    def mask(self, j: int, n: int) -> Tensor:
        """Elements 0..n-1 of mask j, fp32."""
        with np.errstate(over="ignore"):
            i = np.arange(n, dtype=np.uint64)
            base = (np.array([self.key], dtype=np.uint64)
                    + np.array([j], dtype=np.uint64) * _STREAM)
            h = _mix64(base + i * _GOLD)
        u = (h >> np.uint64(40)).astype(np.int64)
        return torch.from_numpy(np.where(u >= self.thr, self.scale, np.float32(0.0))
                                .astype(np.float32))


def _dropout(x: Tensor, p: float, training: bool, m: Tensor | None) -> Tensor:
    """F.dropout, or x * m when the step's device mask m is given (parity runs)."""
    if m is None or not training or p == 0.0:
        return F.dropout(x, p=p, training=training)
    return x * m.view_as(x)


# ----------------------------------------------------------------------------------------------
# scatter helpers (PyG 2.5.1 torch_geometric.utils.scatter on CPU == ATen scatter_add_/reduce_)
# ----------------------------------------------------------------------------------------------


def scatter_sum(src: Tensor, index: Tensor, dim_size: int) -> Tensor:
    out = src.new_zeros((dim_size,) + tuple(src.shape[1:]))
    idx = index.view((-1,) + (1,) * (src.dim() - 1)).expand_as(src)
    return out.scatter_add_(0, idx, src)


def scatter_max(src: Tensor, index: Tensor, dim_size: int) -> Tensor:
    out = src.new_zeros((dim_size,) + tuple(src.shape[1:]))
    idx = index.view((-1,) + (1,) * (src.dim() - 1)).expand_as(src)
    return out.scatter_reduce_(0, idx, src, reduce="amax", include_self=False)


def scatter_mean(src: Tensor, index: Tensor, dim_size: int) -> Tensor:
    """PyG scatter(reduce='mean'): sum / count.clamp(min=1)."""
    count = src.new_zeros(dim_size).scatter_add_(0, index, src.new_ones(src.size(0)))
    count = count.clamp(min=1)
    out = scatter_sum(src, index, dim_size)
    return out / count.view((-1,) + (1,) * (src.dim() - 1))


# ----------------------------------------------------------------------------------------------
# graph construction: KNNGraph (configs/config.py:47) + Batch collation (datamodule.py:63-69)
# ----------------------------------------------------------------------------------------------


def knn_graph(pos: Tensor, k: int, loop: bool = True) -> Tensor:
    """torch_cluster.knn_graph for ONE graph, flow='source_to_target'.

    Returns edge_index [2, E] = [neighbor (source), query (target)], grouped by query in node
    order, each query's neighbors ordered by (squared distance, index) ascending. With loop=True a
    node is its own nearest neighbor (distance 0). k is clipped to the node count, as knn does.
    loop=False asks for k+1 neighbours and drops the self pair (PyG knn_graph).
    """
    n = pos.size(0)
    if n == 0:
        return torch.empty(2, 0, dtype=torch.long)
    kk = min(k if loop else k + 1, n)
    d = ((pos[:, None, :] - pos[None, :, :]) ** 2).sum(-1)  # [query, cand]
    rows, cols = [], []
    for q in range(n):
        order = sorted(range(n), key=lambda c: (d[q, c].item(), c))[:kk]
        for c in order:
            if not loop and c == q:
                continue
            rows.append(c)
            cols.append(q)
    return torch.tensor([rows, cols], dtype=torch.long).view(2, -1)


def radius_graph(pos: Tensor, r: float, loop: bool = False, max_num_neighbors: int = 32) -> Tensor:
    """torch_cluster.radius_graph for ONE graph, flow='source_to_target' (torch_cluster 1.6.3 —
    not under /root/reference; the reference sweep builds it through PyG's RadiusGraph(r),
    scripts/sweep.py:113-118, defaults loop=False, max_num_neighbors=32).

    radius_graph calls radius(x, x, r, limit = max_num_neighbors (+ 1 without loop)); radius
    walks each query's candidates in INDEX order and takes c when the squared distance < r * r
    (strict), stopping at `limit` (the CUDA kernel radius_cuda.cu; the CPU path's nanoflann search
    with sorted=False keeps a traversal-order subset when more than `limit` are in range — that
    case is parity-unpinned and this restatement follows the CUDA rule); without loop the self
    pair is dropped afterwards, so up to max_num_neighbors + 1 neighbours can remain. Returns
    [2, E] = [neighbour (source), query (target)], grouped by query, neighbours ascending.
    Squared distances: ((p_q - p_c) ** 2).sum(-1) in fp64."""
    n = pos.size(0)
    if n == 0:
        return torch.empty(2, 0, dtype=torch.long)
    pos = pos.to(torch.float64)
    d = ((pos[:, None, :] - pos[None, :, :]) ** 2).sum(-1)  # [query, cand]
    r2 = float(r) * float(r)
    limit = max_num_neighbors if loop else max_num_neighbors + 1
    inr = d < r2
    taken = inr & (torch.cumsum(inr.to(torch.int64), 1) <= limit)  # first `limit` in index order
    if not loop:
        taken &= ~torch.eye(n, dtype=torch.bool)
    q, c = torch.nonzero(taken, as_tuple=True)  # row-major: grouped by query, c ascending
    return torch.stack([c, q]).to(torch.long)


def radius_graph_batch(pos: Tensor, r: float, ptr: list[int], loop: bool = False,
                       max_num_neighbors: int = 32) -> Tensor:
    """radius_graph per graph of a collated batch (node offsets `ptr`), concatenated."""
    parts = [radius_graph(pos[a:b], r, loop, max_num_neighbors) + a for a, b in pairwise(ptr)]
    return torch.cat(parts, 1) if parts else torch.empty(2, 0, dtype=torch.long)


def collate(graphs: list[dict]) -> dict:
    """PyG Batch.from_data_list for graphs {'x', 'edge_index', 'y'}: concat x, offset edges,
    build batch (graph id per node) and ptr."""
    xs, eis, ys, batch, ptr = [], [], [], [], [0]
    off = 0
    for g, d in enumerate(graphs):
        n = d["x"].size(0)
        xs.append(d["x"])
        eis.append(d["edge_index"] + off)
        ys.append(d["y"].view(-1))
        batch.append(torch.full((n,), g, dtype=torch.long))
        off += n
        ptr.append(off)
    return {
        "x": torch.cat(xs, 0),
        "edge_index": torch.cat(eis, 1),
        "y": torch.cat(ys, 0),
        "batch": torch.cat(batch, 0),
        "ptr": torch.tensor(ptr, dtype=torch.long),
        "num_graphs": len(graphs),
    }


# ----------------------------------------------------------------------------------------------
# self-loop utilities (torch_geometric.utils.loop, 2.5.1)
# ----------------------------------------------------------------------------------------------


def remove_self_loops(edge_index: Tensor) -> Tensor:
    mask = edge_index[0] != edge_index[1]
    return edge_index[:, mask]


def add_self_loops(edge_index: Tensor, num_nodes: int) -> Tensor:
    loop = torch.arange(num_nodes, dtype=edge_index.dtype).view(1, -1).repeat(2, 1)
    return torch.cat([edge_index, loop], dim=1)


def add_remaining_self_loops(edge_index: Tensor, edge_weight: Tensor, fill_value: float,
                             num_nodes: int) -> tuple[Tensor, Tensor]:
    """Drop existing loops from the list, append one loop per node at the end; a node that had a
    loop keeps that loop's weight (the last one in edge order), others get fill_value."""
    mask = edge_index[0] != edge_index[1]
    loop_index = torch.arange(num_nodes, dtype=edge_index.dtype).view(1, -1).repeat(2, 1)
    loop_attr = edge_weight.new_full((num_nodes,), fill_value)
    inv = ~mask
    loop_attr[edge_index[0][inv]] = edge_weight[inv]
    edge_weight = torch.cat([edge_weight[mask], loop_attr], dim=0)
    edge_index = torch.cat([edge_index[:, mask], loop_index], dim=1)
    return edge_index, edge_weight


def gcn_norm(edge_index: Tensor, num_nodes: int, improved: bool = False,
             add_loops: bool = True) -> tuple[Tensor, Tensor]:
    """torch_geometric.nn.conv.gcn_conv.gcn_norm, edge_index (COO) path, flow source_to_target."""
    fill = 2.0 if improved else 1.0
    edge_weight = torch.ones(edge_index.size(1), dtype=torch.float32)
    if add_loops:
        edge_index, edge_weight = add_remaining_self_loops(edge_index, edge_weight, fill, num_nodes)
    row, col = edge_index[0], edge_index[1]
    deg = scatter_sum(edge_weight, col, num_nodes)
    dis = deg.pow(-0.5)
    dis = dis.masked_fill(dis == float("inf"), 0.0)
    edge_weight = dis[row] * edge_weight * dis[col]
    return edge_index, edge_weight


# ----------------------------------------------------------------------------------------------
# message-passing layers
# ----------------------------------------------------------------------------------------------


def glorot_(t: Tensor) -> None:
    a = math.sqrt(6.0 / (t.size(-2) + t.size(-1)))
    with torch.no_grad():
        t.uniform_(-a, a)


class GCNConv(nn.Module):
    """PyG GCNConv(in, out): lin (no bias, glorot) -> gcn_norm -> propagate(add) -> + bias."""

    def __init__(self, in_channels: int, out_channels: int):
        super().__init__()
        self.lin = nn.Linear(in_channels, out_channels, bias=False)
        self.bias = nn.Parameter(torch.zeros(out_channels))
        glorot_(self.lin.weight)

    def forward(self, x: Tensor, edge_index: Tensor) -> Tensor:
        n = x.size(0)
        ei, w = gcn_norm(edge_index, n)
        x = self.lin(x)
        x_j = x.index_select(0, ei[0])  # propagate: collect x_j
        msg = w.view(-1, 1) * x_j  # message: edge_weight * x_j
        out = scatter_sum(msg, ei[1], n)  # aggregate 'add' at target
        return out + self.bias


class BatchNorm(nn.Module):
    """torch_geometric.nn.norm.BatchNorm: wraps torch.nn.BatchNorm1d as `.module`."""

    def __init__(self, channels: int):
        super().__init__()
        self.module = nn.BatchNorm1d(channels)

    def forward(self, x: Tensor) -> Tensor:
        return self.module(x)


class MLP(nn.Module):
    """PyG MLP(channel_list, act='ELU', dropout=p): norm='batch_norm', plain_last=True,
    act_first=False: Lin -> BN -> ELU -> Dropout for every layer but the last; last Lin plain."""

    def __init__(self, channel_list: list[int], dropout: float = 0.0):
        super().__init__()
        self.lins = nn.ModuleList([nn.Linear(a, b) for a, b in pairwise(channel_list)])
        self.norms = nn.ModuleList([BatchNorm(c) for c in channel_list[1:-1]])
        self.dropout = dropout

    def forward(self, x: Tensor, m: Tensor | None = None) -> Tensor:
        for lin, norm in zip(self.lins[:-1], self.norms):
            x = lin(x)
            x = norm(x)
            x = F.elu(x)
            x = _dropout(x, self.dropout, self.training, m)
        return self.lins[-1](x)


class GINConv(nn.Module):
    """PyG GINConv(nn, eps=0, train_eps=False): nn((1 + eps) * x_i + sum_{j->i} x_j)."""

    def __init__(self, mlp: nn.Module):
        super().__init__()
        self.nn = mlp
        self.register_buffer("eps", torch.zeros(1))

    def forward(self, x: Tensor, edge_index: Tensor, m: Tensor | None = None) -> Tensor:
        x_j = x.index_select(0, edge_index[0])
        out = scatter_sum(x_j, edge_index[1], x.size(0))
        out = out + (1 + self.eps) * x
        return self.nn(out, m)


def edge_softmax(src: Tensor, index: Tensor, num_nodes: int) -> Tensor:
    """torch_geometric.utils.softmax (index path): exp(e - max.detach()) / (sum + 1e-16)."""
    src_max = scatter_max(src.detach(), index, num_nodes)
    out = (src - src_max.index_select(0, index)).exp()
    out_sum = scatter_sum(out, index, num_nodes) + 1e-16
    return out / out_sum.index_select(0, index)


def _r16(t: Tensor) -> Tensor:
    return t.to(torch.bfloat16).float()


class _Bf16Linear(torch.autograd.Function):
    """bf16 GEMM semantics of BASELINE config C3 (the GPU path's lesion_gnn_amd.ops.mm_dense):
    every GEMM — forward y = x W^T, and backward dW = dy^T x, dx = dy W — takes bf16-rounded
    operands and accumulates / returns fp32; bias and its gradient stay fp32."""

    @staticmethod
    def forward(ctx, x, W, b):
        ctx.save_for_backward(x, W)
        ctx.has_b = b is not None
        return F.linear(_r16(x), _r16(W), b)

    @staticmethod
    def backward(ctx, dy):
        x, W = ctx.saved_tensors
        dW = _r16(dy).t() @ _r16(x)
        dx = _r16(dy) @ _r16(W)
        return dx, dW, dy.sum(0) if ctx.has_b else None


def linear(x: Tensor, W: Tensor, b: Tensor | None, bf16: bool) -> Tensor:
    """nn.Linear, or with bf16 the bf16-operand GEMMs of _Bf16Linear."""
    return _Bf16Linear.apply(x, W, b) if bf16 else F.linear(x, W, b)


class GATConv(nn.Module):
    """PyG 2.5.1 GATConv(in, out, heads, dropout), concat=True, negative_slope=0.2,
    add_self_loops=True, bias=True (state_dict: lin.weight, att_src, att_dst, bias)."""

    def __init__(self, in_channels: int, out_channels: int, heads: int = 1, dropout: float = 0.0,
                 negative_slope: float = 0.2):
        super().__init__()
        self.heads, self.out_channels = heads, out_channels
        self.negative_slope, self.dropout = negative_slope, dropout
        self.lin = nn.Linear(in_channels, heads * out_channels, bias=False)
        self.att_src = nn.Parameter(torch.empty(1, heads, out_channels))
        self.att_dst = nn.Parameter(torch.empty(1, heads, out_channels))
        self.bias = nn.Parameter(torch.zeros(heads * out_channels))
        glorot_(self.lin.weight)
        glorot_(self.att_src)
        glorot_(self.att_dst)

    def forward(self, x: Tensor, edge_index: Tensor, masks: DropoutMasks | None = None,
                stream: int = 0) -> Tensor:
        """masks: the step's device masks (parity with dropout on). The device mask of this conv
        is indexed by target-CSR position (rows by target, edge order within a row, the
        appended self loop last) x head: the stable sort of this edge list by target."""
        H, C = self.heads, self.out_channels
        n = x.size(0)
        xs = linear(x, self.lin.weight, None, getattr(self, "bf16", False)).view(-1, H, C)
        a_src = (xs * self.att_src).sum(-1)
        a_dst = (xs * self.att_dst).sum(-1)
        ei = add_self_loops(remove_self_loops(edge_index), n)
        src, dst = ei[0], ei[1]
        alpha = a_src.index_select(0, src) + a_dst.index_select(0, dst)  # alpha_j + alpha_i
        alpha = F.leaky_relu(alpha, self.negative_slope)
        alpha = edge_softmax(alpha, dst, n)
        m = None
        if masks is not None and self.training and self.dropout > 0.0:
            perm = torch.sort(dst, stable=True).indices
            m = torch.empty(alpha.shape)
            m[perm] = masks.mask(stream, alpha.numel()).view(alpha.shape)
        alpha = _dropout(alpha, self.dropout, self.training, m)
        msg = alpha.unsqueeze(-1) * xs.index_select(0, src)
        out = scatter_sum(msg, dst, n)
        return out.view(-1, H * C) + self.bias


def global_mean_pool(x: Tensor, batch: Tensor, size: int | None = None) -> Tensor:
    size = int(batch.max()) + 1 if size is None else size
    return scatter_mean(x, batch, size)


def global_add_pool(x: Tensor, batch: Tensor, size: int | None = None) -> Tensor:
    size = int(batch.max()) + 1 if size is None else size
    return scatter_sum(x, batch, size)


# ----------------------------------------------------------------------------------------------
# models (same constructor signatures and state_dict keys as the build's modules)
# ----------------------------------------------------------------------------------------------


def _pool(kind: str):
    return {"mean": global_mean_pool, "add": global_add_pool}[kind]


class GCN(nn.Module):
    """NEW model: skeleton of reference gin.py:17-35 with GCNConv."""

    def __init__(self, input_features: int, hidden_channels: list[int], num_classes: int,
                 dropout: float, pool: str = "mean"):
        super().__init__()
        self.in_proj = nn.Linear(input_features, hidden_channels[0])
        self.convs = nn.ModuleList([GCNConv(a, b) for a, b in pairwise(hidden_channels)])
        self.out_proj = nn.Linear(hidden_channels[-1], num_classes)
        self.dropout = nn.Dropout(dropout)
        self.pool = pool

    def forward(self, x, edge_index, batch, num_graphs=None, masks: DropoutMasks | None = None):
        """masks: the step's device masks; mask l follows conv l."""
        x = self.in_proj(x)
        for i, conv in enumerate(self.convs):
            x = F.elu(conv(x, edge_index))
            m = masks.mask(i, x.numel()) if masks is not None else None
            x = _dropout(x, self.dropout.p, self.training, m)
        x = _pool(self.pool)(x, batch, num_graphs)
        return self.out_proj(x)


class GIN(nn.Module):
    """Reference gin.py:17-35 (+ pool option, default 'mean')."""

    def __init__(self, input_features: int, hidden_channels: list[int], num_classes: int,
                 dropout: float, pool: str = "mean"):
        super().__init__()
        self.in_proj = nn.Linear(input_features, hidden_channels[0])
        self.convs = nn.ModuleList(
            [GINConv(MLP([a, b, b], dropout=dropout)) for a, b in pairwise(hidden_channels)])
        self.out_proj = nn.Linear(hidden_channels[-1], num_classes)
        self.dropout = nn.Dropout(dropout)
        self.pool = pool

    def forward(self, x, edge_index, batch, num_graphs=None, masks: DropoutMasks | None = None):
        """masks: the step's device masks; conv l's MLP dropout takes mask 2l, the dropout after
        conv l (gin.py:32) mask 2l + 1."""
        x = self.in_proj(x)
        for i, conv in enumerate(self.convs):
            n = x.size(0) * conv.nn.lins[0].out_features
            m1 = masks.mask(2 * i, n) if masks is not None else None
            x = F.elu(conv(x, edge_index, m1))
            m2 = masks.mask(2 * i + 1, x.numel()) if masks is not None else None
            x = _dropout(x, self.dropout.p, self.training, m2)
        x = _pool(self.pool)(x, batch, num_graphs)
        return self.out_proj(x)


class GAT(nn.Module):
    """Reference gat.py:17-59 (SetTransformer readout branch :33-43 out of scope)."""

    def __init__(self, input_features: int, hiddden_channels: list[int], num_classes: int,
                 heads: int, dropout: float, num_st_seed_points=None, pool: str = "mean",
                 precision: str = "fp32"):
        super().__init__()
        assert num_st_seed_points is None
        self.bf16 = precision == "bf16"
        self.in_proj = nn.Linear(input_features, hiddden_channels[0])
        self.convs = nn.ModuleList([GATConv(a, b // heads, heads=heads, dropout=dropout)
                                    for a, b in pairwise(hiddden_channels)])
        self.out_proj = nn.Linear(hiddden_channels[-1], num_classes)
        self.pool = pool

    def forward(self, x, edge_index, batch, num_graphs=None, masks: DropoutMasks | None = None):
        """masks: the step's device masks; conv l's attention dropout takes mask l."""
        x = linear(x, self.in_proj.weight, self.in_proj.bias, self.bf16)
        for i, conv in enumerate(self.convs):
            conv.bf16 = self.bf16
            x = F.elu(conv(x, edge_index, masks, i))
        x = _pool(self.pool)(x, batch, num_graphs)
        return self.out_proj(x)


def criterion(kind: str, logits: Tensor, y: Tensor, num_classes: int,
              class_weights: Tensor | None = None) -> Tensor:
    """Reference base.py:88-96 + training_step :196-201 (+ regression clamp gin.py:66-67)."""
    if kind == "CE":
        return F.cross_entropy(logits, y, weight=class_weights)
    pred = torch.clamp(logits.squeeze(1), min=0, max=num_classes - 1)
    if kind == "MSE":
        return F.mse_loss(pred, y.float())
    if kind == "SmoothL1":
        return F.smooth_l1_loss(pred, y.float())
    raise ValueError(kind)


def gaussian_distance(edge_index: Tensor, pos: Tensor, sigma: float) -> Tensor:
    """Reference transforms.py:32-79 (EDGE_WEIGHT_REPLACE): exp(-d^2 / 2s^2) / sqrt(2 pi s^2)."""
    row, col = edge_index
    sq = (pos[row] - pos[col]).pow(2).sum(-1)
    return torch.exp(-sq / (2 * sigma ** 2)) / math.sqrt(2 * math.pi * sigma ** 2)


class GraphConv(nn.Module):
    """PyG 2.5.1 GraphConv(in, out) as DRGNet stacks it (reference models/drgnet.py:30-33,
    called with edge_weight at :55): out_i = lin_rel(sum_{j->i} w_ji x_j) + lin_root(x_i);
    aggr='add' via scatter_add_ by target, no self loops; lin_rel has the bias, lin_root none."""

    def __init__(self, in_channels: int, out_channels: int):
        super().__init__()
        self.lin_rel = nn.Linear(in_channels, out_channels, bias=True)
        self.lin_root = nn.Linear(in_channels, out_channels, bias=False)

    def forward(self, x: Tensor, edge_index: Tensor, edge_weight: Tensor | None = None) -> Tensor:
        src, dst = edge_index
        msg = x.index_select(0, src)
        if edge_weight is not None:
            msg = msg * edge_weight.view(-1, 1)
        agg = scatter_sum(msg, dst, x.size(0))
        return self.lin_rel(agg) + self.lin_root(x)


def to_dense_batch(x: Tensor, batch: Tensor, fill_value: float | Tensor,
                   batch_size: int | None = None) -> tuple[Tensor, Tensor]:
    """PyG 2.5.1 torch_geometric.utils.to_dense_batch (called by SortAggregation): [ΣN, D] ->
    [B, Nmax, D] with fill_value padding, rows in node order within each graph."""
    if batch_size is None:
        batch_size = int(batch.max()) + 1 if batch.numel() else 0
    counts = torch.bincount(batch, minlength=batch_size)
    cum = torch.cat([counts.new_zeros(1), counts.cumsum(0)])
    nmax = int(counts.max()) if counts.numel() else 0
    idx = torch.arange(batch.numel()) - cum[batch] + batch * nmax
    out = x.new_full((batch_size * nmax, x.size(1)), 0.0) + fill_value
    out = out.index_put((idx,), x)  # out-of-place so autograd reaches x
    mask = torch.zeros(batch_size * nmax, dtype=torch.bool)
    mask[idx] = True
    return out.view(batch_size, nmax, x.size(1)), mask.view(batch_size, nmax)


def sort_aggregation(x: Tensor, batch: Tensor, k: int, batch_size: int | None = None) -> Tensor:
    """PyG 2.5.1 SortAggregation(k) (reference models/drgnet.py:37, called at :59): pad each
    graph with fill = min(x) - 1, sort its rows by the last channel (descending; ties by node
    order — torch's CPU sort is stable), keep the first k rows (pad with fill rows when the
    graph has fewer), zero every element equal to fill, flatten to [B, k * D]."""
    fill_value = x.detach().min() - 1
    bx, _ = to_dense_batch(x, batch, fill_value, batch_size)
    B, N, D = bx.size()
    _, perm = bx[:, :, -1].sort(dim=-1, descending=True, stable=True)
    perm = perm + (torch.arange(B) * N).view(-1, 1)
    bx = bx.reshape(B * N, D)[perm].view(B, N, D)
    if N >= k:
        bx = bx[:, :k].contiguous()
    else:
        bx = torch.cat([bx, bx.new_full((B, k - N, D), 0.0) + fill_value], dim=1)
    bx = bx.masked_fill(bx == fill_value, 0.0)
    return bx.view(B, k * D)


class MLPPlain(nn.Module):
    """PyG 2.5.1 MLP(channel_list, dropout, norm=None, act=F.elu), plain_last=True (reference
    drgnet.py:48): Lin -> act -> dropout ... -> Lin; state_dict keys lins.{i}.*."""

    def __init__(self, channel_list: list[int], dropout: float = 0.0):
        super().__init__()
        self.lins = nn.ModuleList([nn.Linear(a, b) for a, b in pairwise(channel_list)])
        self.dropout = dropout

    def forward(self, x: Tensor) -> Tensor:
        for lin in self.lins[:-1]:
            x = F.dropout(F.elu(lin(x)), self.dropout, self.training)
        return self.lins[-1](x)


class DRGNet(nn.Module):
    """Reference models/drgnet.py:16-69: GraphConv stack (ELU after each, outputs concatenated),
    SortAggregation(k), Conv1d(1, c0, D, stride D) -> ELU -> MaxPool1d(2, 2) -> Conv1d(c0, c1, 5)
    -> ELU -> flatten -> MLP([dense, 128, C], dropout 0.5)."""

    def __init__(self, input_features: int, gnn_hidden_dim: int, num_layers: int,
                 sortpool_k: int, num_classes: int, conv_hidden_dims: tuple[int, int] = (16, 32),
                 dropout: float = 0.5):
        super().__init__()
        dims = [input_features] + [gnn_hidden_dim] * num_layers
        self.graph_convs = nn.ModuleList([GraphConv(a, b) for a, b in pairwise(dims)])
        self.graph_convs.append(GraphConv(gnn_hidden_dim, 1))
        total = gnn_hidden_dim * num_layers + 1
        self.k = sortpool_k
        self.conv1 = nn.Conv1d(1, conv_hidden_dims[0], kernel_size=total, stride=total)
        self.max_pool = nn.MaxPool1d(2, 2)
        self.conv2 = nn.Conv1d(conv_hidden_dims[0], conv_hidden_dims[1], kernel_size=5, stride=1)
        dense = int((sortpool_k - 2) / 2 + 1)
        dense = (dense - 5 + 1) * conv_hidden_dims[1]
        self.mlp = MLPPlain([dense, 128, num_classes], dropout=dropout)

    def forward(self, x: Tensor, edge_index: Tensor, batch: Tensor,
                edge_weight: Tensor | None = None, num_graphs: int | None = None) -> Tensor:
        xs = []
        for conv in self.graph_convs:
            x = F.elu(conv(x, edge_index, edge_weight))
            xs.append(x)
        x = sort_aggregation(torch.cat(xs, dim=1), batch, self.k, num_graphs).unsqueeze(1)
        x = self.max_pool(F.elu(self.conv1(x)))
        x = F.elu(self.conv2(x))
        return self.mlp(x.view(x.size(0), -1))


def extract_features_by_cc(cc: Tensor, features: Tensor, nlabel: int,
                           reduce: str = "mean") -> Tensor:
    """Reference datasets/nodes/lesions.py:88-93: features (1, C, H, W), cc (H, W) int64
    component labels -> per-label mean (or sum) of the pixel features, [max(cc) + 1, C]
    (torch_scatter.scatter along dim 0: sum, then / clamp(count, 1) for mean). nlabel == 1
    returns the global average (1, C)."""
    if nlabel == 1:
        return features.mean((2, 3))
    f = features.squeeze(0).flatten(1, 2).transpose(0, 1)  # (H*W, C)
    idx = cc.flatten()
    size = int(idx.max()) + 1
    if reduce == "max":  # PyG scatter(reduce="max"): scatter_reduce_ amax, include_self=False
        ix = idx.view(-1, 1).expand_as(f)
        return f.new_zeros(size, f.size(1)).scatter_reduce_(0, ix, f, "amax", include_self=False)
    if reduce not in ("sum", "add", "mean"):
        raise ValueError(reduce)
    out = f.new_zeros(size, f.size(1)).index_add_(0, idx, f)
    if reduce == "mean":
        cnt = torch.bincount(idx, minlength=size).clamp_min(1).to(f.dtype)
        out = out / cnt.view(-1, 1)
    return out
