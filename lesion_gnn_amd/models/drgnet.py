"""DRGNet graph classifier — reference src/lesion_gnn/models/drgnet.py:16-108 (DRGNet,
DRGNetModelConfig, DRGNetLightning): a GraphConv stack with the GaussianDistance edge weights
(ELU after each conv, outputs concatenated), SortAggregation(k), then a Conv1d / MaxPool1d /
Conv1d / MLP head over the k sorted node rows.

On the GPU: every GraphConv is the HIP weighted segmented sum (lgnn_spmm, transpose CSR in the
backward) + the node-linear kernels or the library GEMM for the 1025-wide input layer; the graph
is built once (one `Graph` shared by every conv, the weighted CSR cached per weight tensor);
SortAggregation is lgnn_sort_pool_fwd/_bwd. The head (B x k rows, a few KFLOP per graph) runs on
torch's GPU Conv1d / MaxPool1d / Linear, as the reference's own modules do — same state_dict keys:
graph_convs.{i}.lin_rel.{weight,bias}, graph_convs.{i}.lin_root.weight, conv1.*, conv2.*,
mlp.lins.{0,1}.*.
"""
from __future__ import annotations

import dataclasses
from itertools import pairwise

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..conv import GraphConv, SortAggregation
from ..graph import as_graph
from ..utils.placeholder import Placeholder
from .base import BaseModelConfig, BaseModule


class MLP(nn.Module):
    """PyG 2.5.1 MLP(channel_list, dropout, norm=None, act=F.elu) with plain_last=True
    (reference drgnet.py:48): Lin -> ELU -> Dropout -> ... -> Lin; keys lins.{i}.*."""

    def __init__(self, channel_list: list[int], dropout: float = 0.0):
        super().__init__()
        self.channel_list = list(channel_list)
        self.dropout = float(dropout)
        self.lins = nn.ModuleList([nn.Linear(a, b) for a, b in pairwise(channel_list)])

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        for lin in self.lins[:-1]:
            x = F.dropout(F.elu(lin(x)), self.dropout, self.training)
        return self.lins[-1](x)


class DRGNet(nn.Module):
    def __init__(self, input_features: int, gnn_hidden_dim: int, num_layers: int,
                 sortpool_k: int, num_classes: int, conv_hidden_dims: tuple[int, int] = (16, 32),
                 dropout: float = 0.5):
        super().__init__()
        gnn_dims = [input_features] + [gnn_hidden_dim] * num_layers
        self.graph_convs = nn.ModuleList([GraphConv(a, b) for a, b in pairwise(gnn_dims)])
        self.graph_convs.append(GraphConv(gnn_hidden_dim, 1))
        total_latent_dim = gnn_hidden_dim * num_layers + 1
        self.sort_pool = SortAggregation(sortpool_k)
        kernel_size = 5  # reference drgnet.py:40
        self.conv1 = nn.Conv1d(1, conv_hidden_dims[0], kernel_size=total_latent_dim,
                               stride=total_latent_dim)
        self.max_pool = nn.MaxPool1d(2, 2)
        self.conv2 = nn.Conv1d(conv_hidden_dims[0], conv_hidden_dims[1], kernel_size=kernel_size,
                               stride=1)
        dense_dim = int((sortpool_k - 2) / 2 + 1)  # reference drgnet.py:46-47
        dense_dim = (dense_dim - kernel_size + 1) * conv_hidden_dims[1]
        if dense_dim <= 0:
            raise ValueError(f"sortpool_k={sortpool_k} leaves no positions for conv2 (need >= 10)")
        self.mlp = MLP([dense_dim, 128, num_classes], dropout=dropout)

    def forward(self, x: torch.Tensor, edge_index, batch: torch.Tensor,
                edge_weight: torch.Tensor | None = None,
                num_graphs: int | None = None) -> torch.Tensor:
        g = as_graph(edge_index, x.size(0), batch, num_graphs)
        xs = []
        for conv in self.graph_convs:
            x = F.elu(conv(x, g, edge_weight))
            xs.append(x)
        x = self.sort_pool(torch.cat(xs, dim=1), graph=g)  # [B, k * (h * L + 1)]
        x = x.unsqueeze(1)
        x = self.max_pool(F.elu(self.conv1(x)))
        x = F.elu(self.conv2(x))
        return self.mlp(x.view(x.size(0), -1))


@dataclasses.dataclass(kw_only=True)
class DRGNetModelConfig(BaseModelConfig):
    input_features: Placeholder[int] = dataclasses.field(default_factory=Placeholder, init=False)
    gnn_hidden_dim: int
    num_layers: int
    sortpool_k: int
    conv_hidden_dims: tuple[int, int] = (16, 32)
    compile: bool = False
    name: str = dataclasses.field(default="DRGNet", init=False)


class DRGNetModule(BaseModule):
    """Reference DRGNetLightning (drgnet.py:88-108): forwards data.edge_weight."""

    def __init__(self, config: DRGNetModelConfig):
        super().__init__(config)
        model = DRGNet(
            input_features=config.input_features.value,
            gnn_hidden_dim=config.gnn_hidden_dim,
            num_layers=config.num_layers,
            sortpool_k=config.sortpool_k,
            num_classes=1 if self.is_regression else config.num_classes.value,
            conv_hidden_dims=config.conv_hidden_dims,
        )
        # reference drgnet.py:103: the model is compiled when the config asks (library.py holds the
        # lgnn:: custom ops + fake kernels Dynamo traces)
        self.model = torch.compile(model, dynamic=True) if config.compile else model

    def _model_logits(self, data) -> torch.Tensor:
        """The one hook BaseModule.forward and training_step call: DRGNet takes the per-edge
        GaussianDistance weights in the 4th position (reference drgnet.py:103)."""
        edge_index = getattr(data, "adj_t", None)
        if edge_index is None:
            edge_index = data.edge_index
        return self.model(data.x, edge_index, data.batch, getattr(data, "edge_weight", None),
                          getattr(data, "num_graphs", None))
