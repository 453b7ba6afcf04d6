"""Second, independent restatement of the hot-path models for cross-checking the oracle:
float64, DENSE adjacency (no index_select / scatter), written from the PyG 2.5.1 operator
definitions rather than from oracle/pyg_ref.py's op sequence. Test-only.

Edge multiplicities matter (PyG sums one message per edge), so adjacency entries COUNT edges:
A[i, j] = number of edges j -> i.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

D = torch.float64


def count_adj(edge_index: torch.Tensor, n: int) -> torch.Tensor:
    A = torch.zeros(n, n, dtype=D)
    A.index_put_((edge_index[1], edge_index[0]), torch.ones(edge_index.size(1), dtype=D),
                 accumulate=True)
    return A


def gcn_adj(edge_index: torch.Tensor, n: int) -> torch.Tensor:
    """gcn_norm with add_remaining_self_loops (fill 1): every node gets exactly one loop of
    weight 1 (an existing loop keeps weight 1), non-loop edges keep their multiplicity."""
    A = count_adj(edge_index, n)
    A.fill_diagonal_(1.0)
    deg = A.sum(1)
    dis = torch.where(deg > 0, deg.rsqrt(), torch.zeros_like(deg))
    return dis[:, None] * A * dis[None, :]


def pool(x, batch, B, kind):
    P = torch.zeros(B, x.size(0), dtype=D)
    P[batch, torch.arange(x.size(0))] = 1.0
    s = P @ x
    if kind == "mean":
        s = s / P.sum(1, keepdim=True).clamp(min=1)
    return s


def p(sd, k):
    return sd[k]


def gcn_forward(sd, x, edge_index, batch, B, L, pool_kind="mean"):
    n = x.size(0)
    Ah = gcn_adj(edge_index, n)
    h = x.to(D) @ p(sd, "in_proj.weight").T + p(sd, "in_proj.bias")
    for i in range(L):
        h = F.elu(Ah @ (h @ p(sd, f"convs.{i}.lin.weight").T) + p(sd, f"convs.{i}.bias"))
    return pool(h, batch, B, pool_kind) @ p(sd, "out_proj.weight").T + p(sd, "out_proj.bias")


def gin_forward(sd, x, edge_index, batch, B, L, pool_kind="mean", eps_bn=1e-5):
    n = x.size(0)
    A = count_adj(edge_index, n) + torch.eye(n, dtype=D)  # (1 + eps) x_i with eps = 0
    h = x.to(D) @ p(sd, "in_proj.weight").T + p(sd, "in_proj.bias")
    for i in range(L):
        pre = f"convs.{i}.nn."
        z = (A @ h) @ p(sd, pre + "lins.0.weight").T + p(sd, pre + "lins.0.bias")
        mu = z.mean(0)
        var = z.var(0, unbiased=False)
        z = (z - mu) / torch.sqrt(var + eps_bn) * p(sd, pre + "norms.0.module.weight") + \
            p(sd, pre + "norms.0.module.bias")
        z = F.elu(z)
        h = F.elu(z @ p(sd, pre + "lins.1.weight").T + p(sd, pre + "lins.1.bias"))
    return pool(h, batch, B, pool_kind) @ p(sd, "out_proj.weight").T + p(sd, "out_proj.bias")


def gat_forward(sd, x, edge_index, batch, B, L, heads, slope=0.2, pool_kind="mean"):
    n = x.size(0)
    A = count_adj(edge_index, n)
    A.fill_diagonal_(1.0)  # remove_self_loops + add_self_loops: exactly one loop per node
    h = x.to(D) @ p(sd, "in_proj.weight").T + p(sd, "in_proj.bias")
    for i in range(L):
        W = p(sd, f"convs.{i}.lin.weight")
        C = W.size(0) // heads
        xs = (h @ W.T).view(n, heads, C)
        a_s = (xs * p(sd, f"convs.{i}.att_src")).sum(-1)  # [n, H]
        a_d = (xs * p(sd, f"convs.{i}.att_dst")).sum(-1)
        out = torch.zeros(n, heads, C, dtype=D)
        for hh in range(heads):
            e = F.leaky_relu(a_d[:, hh, None] + a_s[None, :, hh], slope)  # [i, j]
            e = torch.where(A > 0, e, torch.full_like(e, -float("inf")))
            w = A * torch.exp(e - e.max(1, keepdim=True).values.detach())
            w = w / w.sum(1, keepdim=True)
            out[:, hh] = w @ xs[:, hh]
        h = F.elu(out.reshape(n, heads * C) + p(sd, f"convs.{i}.bias"))
    return pool(h, batch, B, pool_kind) @ p(sd, "out_proj.weight").T + p(sd, "out_proj.bias")
