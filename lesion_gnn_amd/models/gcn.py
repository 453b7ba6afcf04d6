"""GCN graph classifier (NEW model): the skeleton of the reference GIN
(src/lesion_gnn/models/gin.py:17-35 — in_proj -> convs with F.elu -> dropout -> global pool ->
out_proj) with PyG GCNConv convs, plus the `pool` option ("mean" keeps reference behaviour,
"add" = global_add_pool).

forward(x, edge_index | Graph, batch) is the drop-in boundary `self.model(data.x, edge_index,
data.batch)` (reference gin.py:64). With dropout inactive the whole body runs as one fused HIP
autograd node (ops.gcn_stack); otherwise layer by layer on the same kernels.
"""
from __future__ import annotations

import dataclasses
from itertools import pairwise

import torch
import torch.nn as nn

from .. import _lib, ops
from .. import dropout as lgnn_dropout
from ..conv import GCNConv
from ..graph import as_graph
from ..utils.placeholder import Placeholder
from .base import BaseModelConfig, BaseModule


class GCN(nn.Module):
    def __init__(self, input_features: int, hidden_channels: list[int], num_classes: int,
                 dropout: float, pool: str = "mean"):
        super().__init__()
        assert all(d > 0 for d in hidden_channels)
        if pool not in ("mean", "add"):
            raise ValueError(f"pool must be 'mean' or 'add', got {pool!r}")
        self.in_proj = nn.Linear(input_features, hidden_channels[0])
        self.convs = nn.ModuleList([GCNConv(a, b) for a, b in pairwise(hidden_channels)])
        self.out_proj = nn.Linear(hidden_channels[-1], num_classes)
        self.dropout = nn.Dropout(dropout)
        self.pool = pool
        self._dropout_key = repr(float(dropout))
        # the dropout generator (lesion_gnn_amd.dropout; not in state_dict)
        # (seeded by the generator state and this model's initial weights)
        self.register_buffer("_dropout_rng",
                             lgnn_dropout.new_state(salt=lgnn_dropout.param_salt(self)),
                             persistent=False)

    def flat_params(self) -> list[torch.Tensor]:
        ps = [self.in_proj.weight, self.in_proj.bias]
        for c in self.convs:
            ps += [c.lin.weight, c.bias]
        return ps + [self.out_proj.weight, self.out_proj.bias]

    def forward(self, x: torch.Tensor, edge_index, batch: torch.Tensor,
                num_graphs: int | None = None) -> torch.Tensor:
        g = as_graph(edge_index, x.size(0), batch, num_graphs)
        mean = self.pool == "mean"
        if self.dropout.p == 0.0 or not self.training:
            return ops.gcn_stack(x, g, self.flat_params(), len(self.convs), mean)
        # the dropout after each conv (mask l follows conv l), all masks in one launch
        ms = lgnn_dropout.masks(self._dropout_rng,
                                [(x.size(0), c.out_channels) for c in self.convs],
                                lgnn_dropout.key(self, self.dropout.p))
        h = ops.node_linear(x, self.in_proj.weight, self.in_proj.bias)
        for conv, m in zip(self.convs, ms):
            h = lgnn_dropout.mask_mul(conv(h, g, act=_lib.LGNN_ACT_ELU), m)
        return ops.pool_head(h, self.out_proj.weight, self.out_proj.bias, g, mean)


    def forward_loss(self, x: torch.Tensor, edge_index, batch: torch.Tensor, y: torch.Tensor,
                     weight: torch.Tensor | None = None, num_graphs: int | None = None):
        """(logits, loss) of forward() followed by nn.CrossEntropyLoss(weight) (the reference's
        criterion, base.py:93-94, as its training_step applies it, :196-201). Without dropout the
        model and the criterion are one autograd node (ops.gcn_stack_ce): the backward forms the
        logits gradient inside its own launches. Otherwise forward() then ops.cross_entropy."""
        if self.dropout.p == 0.0 or not self.training:
            if not torch.compiler.is_compiling():
                g = as_graph(edge_index, x.size(0), batch, num_graphs)
                return ops.gcn_stack_ce(x, g, self.flat_params(), len(self.convs), y, weight,
                                        self.pool == "mean")
        logits = self(x, edge_index, batch, num_graphs)
        return logits, ops.cross_entropy(logits, y, weight)


@dataclasses.dataclass(kw_only=True)
class GCNConfig(BaseModelConfig):
    input_features: Placeholder[int] = dataclasses.field(default_factory=Placeholder, init=False)
    hidden_channels: list[int]
    dropout: float
    compile: bool
    pool: str = "mean"
    name: str = dataclasses.field(default="GCN", init=False)


class GCNModule(BaseModule):
    """LightningModule-shaped wrapper (reference GINLightning gin.py:47-69 pattern)."""

    def __init__(self, config: GCNConfig):
        super().__init__(config)
        model = GCN(
            input_features=config.input_features.value,
            hidden_channels=config.hidden_channels,
            num_classes=1 if self.is_regression else config.num_classes.value,
            dropout=config.dropout,
            pool=config.pool,
        )
        # reference gin.py:56: the model is compiled when the config asks (library.py holds the
        # lgnn:: custom ops + fake kernels Dynamo traces)
        self.model = torch.compile(model, dynamic=True) if config.compile else model
