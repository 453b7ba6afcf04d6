"""GAT graph classifier — reference src/lesion_gnn/models/gat.py:17-97 (GAT, GATConfig,
GATLightning), including the config field typo `hiddden_channels` (gat.py:65, used by
configs/config.py:61). The SetTransformer readout branch (gat.py:33-43, `num_st_seed_points`)
is out of scope (no config enables it); passing it raises.

forward(x, edge_index | Graph, batch) is the drop-in boundary `self.model(data.x, edge_index,
data.batch)` (reference gat.py:92): in_proj -> L x ELU(GATConv) -> global_mean_pool -> out_proj,
every conv one HIP autograd node (ops.gat_conv) with the ELU fused.
"""
from __future__ import annotations

import dataclasses
from itertools import pairwise

import torch
import torch.nn as nn

from .. import _lib, ops
from .. import dropout as lgnn_dropout
from ..conv import GATConv
from ..graph import as_graph
from ..utils.placeholder import Placeholder
from .base import BaseModelConfig, BaseModule


# the last GATConv + readout as one autograd node (ops.gat_conv_head); HEAD_FOLD = False: separate
HEAD_FOLD = True
# fp32: every split-3 weight operand of a step in one launch (GAT.weight_planes); 0: per GEMM
WEIGHT_BUNDLE = True


class GAT(nn.Module):
    def __init__(self, input_features: int, hiddden_channels: list[int], num_classes: int,
                 heads: int, dropout: float, num_st_seed_points: int | None = None,
                 pool: str = "mean", precision: str = "fp32"):
        super().__init__()
        if precision not in ("fp32", "bf16"):
            raise ValueError(f"precision must be 'fp32' or 'bf16', got {precision!r}")
        # bf16 (BASELINE config C3): in_proj and every GATConv.lin on bf16-rounded operands with
        # fp32 accumulation and fp32 activations; attention, softmax, pool and out_proj in fp32
        self.bf16 = precision == "bf16"
        assert all(d % heads == 0 for d in hiddden_channels)
        if num_st_seed_points is not None:
            raise NotImplementedError("SetTransformerAggregation readout (reference gat.py:33-43)"
                                      " is out of scope for this build")
        if pool not in ("mean", "add"):
            raise ValueError(f"pool must be 'mean' or 'add', got {pool!r}")
        self.in_proj = nn.Linear(input_features, hiddden_channels[0])
        self.convs = nn.ModuleList([GATConv(d1, d2 // heads, heads=heads, dropout=dropout)
                                    for d1, d2 in pairwise(hiddden_channels)])
        self.st = None
        self.out_proj = nn.Linear(hiddden_channels[-1], num_classes)
        self.pool = pool
        self.dropout_p = float(dropout)
        self._dropout_key = repr(self.dropout_p)
        # the attention-dropout generator (lesion_gnn_amd.dropout; not in state_dict)
        # (seeded by the generator state and this model's initial weights)
        self.register_buffer("_dropout_rng",
                             lgnn_dropout.new_state(salt=lgnn_dropout.param_salt(self)),
                             persistent=False)

    def dropout_masks(self, g) -> list | None:
        """Every conv's attention-dropout mask of this forward, in one launch (mask l -> conv l);
        None when dropout is inactive."""
        if self.dropout_p == 0.0 or not self.training or not len(self.convs):
            return None
        return lgnn_dropout.masks(self._dropout_rng, [c.mask_shape(g) for c in self.convs],
                                  lgnn_dropout.key(self, self.dropout_p))

    def weight_planes(self):
        """fp32: every split-3 weight operand of this step — in_proj's (when it runs on the dense
        GEMMs), each conv's lin W and (for its dx) W^T — in ONE launch (ops.s3_weight_bundle)
        instead of one per GEMM. Returns (in_proj's planes | None, [(W's, W^T's) per conv])."""
        none = (None, [None] * len(self.convs))
        if self.bf16 or not ops.GAT_S3 or not len(self.convs) or not WEIGHT_BUNDLE:
            return none
        grad = torch.is_grad_enabled()
        specs = [(self.in_proj.weight, False)] if ops.dense_path(self.in_proj.weight, False) \
            else []
        for c in self.convs:
            specs += [(c.lin.weight, False)] + ([(c.lin.weight, True)] if grad else [])
        views = ops.s3_weight_bundle(specs, False)
        wp = views.pop(0) if len(specs) > len(self.convs) * (2 if grad else 1) else None
        per = 2 if grad else 1
        return wp, [(views[per * i], views[per * i + 1] if grad else None)
                    for i in range(len(self.convs))]

    def forward(self, x: torch.Tensor, edge_index, batch: torch.Tensor,
                num_graphs: int | None = None) -> torch.Tensor:
        g = as_graph(edge_index, x.size(0), batch, num_graphs)
        if self.bf16 and not torch.compiler.is_compiling():
            # every bf16 GEMM's weight operands for this step in one launch
            ops.bf16_prepare_weights([self.in_proj.weight] + [c.lin.weight for c in self.convs])
        ms = self.dropout_masks(g)
        wp, planes = self.weight_planes()
        h = ops.linear_auto(x, self.in_proj.weight, self.in_proj.bias, self.bf16, wp)
        last = len(self.convs) - 1
        for i, conv in enumerate(self.convs):
            m = ms[i] if ms is not None else None
            if i == last and HEAD_FOLD:
                # last conv + readout as one node: the readout's backward is formed inside the
                # attention backward's load, no dH tensor
                return conv.forward_head(h, g, _lib.LGNN_ACT_ELU, self.out_proj.weight,
                                         self.out_proj.bias, self.pool == "mean", self.bf16,
                                         mask=m, planes=planes[i])
            h = conv(h, g, act=_lib.LGNN_ACT_ELU, bf16=self.bf16, mask=m, planes=planes[i])
        return ops.pool_head(h, self.out_proj.weight, self.out_proj.bias, g, self.pool == "mean")


@dataclasses.dataclass(kw_only=True)
class GATConfig(BaseModelConfig):
    input_features: Placeholder[int] = dataclasses.field(default_factory=Placeholder, init=False)
    hiddden_channels: list[int]
    heads: int
    dropout: float
    compile: bool
    num_st_seed_points: int | None = None
    pool: str = "mean"
    precision: str = "fp32"
    name: str = dataclasses.field(default="GAT", init=False)


class GATModule(BaseModule):
    """Reference GATLightning (gat.py:73-97)."""

    def __init__(self, config: GATConfig):
        super().__init__(config)
        model = GAT(
            input_features=config.input_features.value,
            hiddden_channels=config.hiddden_channels,
            num_classes=1 if self.is_regression else config.num_classes.value,
            heads=config.heads,
            dropout=config.dropout,
            num_st_seed_points=config.num_st_seed_points,
            pool=config.pool,
            precision=config.precision,
        )
        # reference gat.py:84: the model is compiled when the config asks (library.py holds the
        # lgnn:: custom ops + fake kernels Dynamo traces)
        self.model = torch.compile(model, dynamic=True) if config.compile else model
