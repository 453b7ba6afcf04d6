"""GIN graph classifier — reference src/lesion_gnn/models/gin.py:17-69 (GIN, GINConfig,
GINLightning) with the `pool` option of SURVEY.md §0.3 ("mean" = reference behaviour, "add" =
global_add_pool for BASELINE config C4).

forward(x, edge_index | Graph, batch) is the drop-in boundary `self.model(data.x, edge_index,
data.batch)` (reference gin.py:64). Each GINConv (aggregate -> Lin -> BatchNorm -> ELU -> Lin)
plus the model's F.elu (gin.py:31) runs as one HIP autograd node (ops.gin_conv).
"""
from __future__ import annotations

import dataclasses
from itertools import pairwise

import torch
import torch.nn as nn

from .. import _lib, ops
from .. import dropout as lgnn_dropout
from ..conv import MLP, GINConv
from ..graph import as_graph
from ..utils.placeholder import Placeholder
from .base import BaseModelConfig, BaseModule


# the GIN model as one autograd node (ops.gin_stack) when eligible; STACK = False: per-conv
STACK = True


class GIN(nn.Module):
    def __init__(self, input_features: int, hidden_channels: list[int], num_classes: int,
                 dropout: float, pool: str = "mean"):
        super().__init__()
        assert all(d > 0 for d in hidden_channels)
        if pool not in ("mean", "add"):
            raise ValueError(f"pool must be 'mean' or 'add', got {pool!r}")
        self.in_proj = nn.Linear(input_features, hidden_channels[0])
        self.convs = nn.ModuleList([GINConv(MLP([d1, d2, d2], dropout=dropout))
                                    for d1, d2 in pairwise(hidden_channels)])
        self.out_proj = nn.Linear(hidden_channels[-1], num_classes)
        self.dropout = nn.Dropout(dropout)
        self.pool = pool
        self._dropout_key = repr(float(dropout))
        # the dropout generator (lesion_gnn_amd.dropout; not in state_dict)
        # (seeded by the generator state and this model's initial weights)
        self.register_buffer("_dropout_rng",
                             lgnn_dropout.new_state(salt=lgnn_dropout.param_salt(self)),
                             persistent=False)

    def dropout_masks(self, x: torch.Tensor) -> list | None:
        """This forward's masks in one launch: conv l's MLP dropout (mask 2l, reference gin.py:23)
        and the dropout after conv l (mask 2l + 1, gin.py:32); None when dropout is inactive."""
        if self.dropout.p == 0.0 or not self.training or not len(self.convs):
            return None
        M = x.size(0)
        shapes = []
        for c in self.convs:
            shapes += [(M, c.nn.channel_list[1]), (M, c.nn.channel_list[2])]
        return lgnn_dropout.masks(self._dropout_rng, shapes,
                                  lgnn_dropout.key(self, self.dropout.p))

    def set_sync_bn(self, group, global_count: int | None = None) -> None:
        """SyncBatchNorm over a torch.distributed group (RCCL): BN statistics and their backward
        sums are all-reduced, so N replicas compute exactly the single-device batch statistics.
        global_count: the total node count over the group when every step has the same one
        (skips the per-step count all-reduce and its host read, so the step can be captured
        in a HIP graph); None = all-reduce the count every step."""
        for c in self.convs:
            c.sync_group = group
            c.sync_count = global_count

    def forward(self, x: torch.Tensor, edge_index, batch: torch.Tensor,
                num_graphs: int | None = None) -> torch.Tensor:
        g = as_graph(edge_index, x.size(0), batch, num_graphs)
        drop = self.dropout.p > 0.0 and self.training
        if STACK and not drop and ops.gin_stack_eligible(
                x, self.in_proj.weight,
                [(c.nn.lins[0].weight, c.nn.lins[1].weight) for c in self.convs]):
            # the whole model as one autograd node: each conv's aggregation backward is gathered
            # by the layer below it instead of a separate transpose pass
            convs = [c.stack_spec(x, _lib.LGNN_ACT_ELU) for c in self.convs]
            return ops.gin_stack(x, self.in_proj.weight, self.in_proj.bias, convs,
                                 self.out_proj.weight, self.out_proj.bias, g, self.pool == "mean")
        ms = self.dropout_masks(x) if drop else None
        h = ops.node_linear(x, self.in_proj.weight, self.in_proj.bias)
        last = len(self.convs) - 1
        for i, conv in enumerate(self.convs):
            if i == last and not drop and conv.head_fusable(h):
                # last conv + readout as one node: no dH tensor in the backward
                return conv.forward_head(h, g, _lib.LGNN_ACT_ELU, self.out_proj.weight,
                                         self.out_proj.bias, self.pool == "mean")
            h = conv(h, g, act=_lib.LGNN_ACT_ELU, mask=ms[2 * i] if drop else None)
            if drop:
                h = lgnn_dropout.mask_mul(h, ms[2 * i + 1])
        return ops.pool_head(h, self.out_proj.weight, self.out_proj.bias, g, self.pool == "mean")


@dataclasses.dataclass(kw_only=True)
class GINConfig(BaseModelConfig):
    input_features: Placeholder[int] = dataclasses.field(default_factory=Placeholder, init=False)
    hidden_channels: list[int]
    dropout: float
    compile: bool
    pool: str = "mean"
    name: str = dataclasses.field(default="GIN", init=False)


class GINModule(BaseModule):
    """Reference GINLightning (gin.py:47-69)."""

    def __init__(self, config: GINConfig):
        super().__init__(config)
        model = GIN(
            input_features=config.input_features.value,
            hidden_channels=config.hidden_channels,
            num_classes=1 if self.is_regression else config.num_classes.value,
            dropout=config.dropout,
            pool=config.pool,
        )
        # reference gin.py:56: the model is compiled when the config asks (library.py holds the
        # lgnn:: custom ops + fake kernels Dynamo traces)
        self.model = torch.compile(model, dynamic=True) if config.compile else model
