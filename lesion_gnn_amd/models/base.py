"""The boundary caller: loss + step around `self.model(x, edge_index, batch)`.

Mirrors the reference's BaseLightningModule contract (src/lesion_gnn/models/base.py:82-233) for
the parts on the hot path — criterion selection (:88-96), the regression clamp of the
XLightning.forward methods (gin.py:58-69, gat.py:86-97), training_step (:196-201) and
configure_optimizers (:162-188) — as a plain nn.Module (Lightning, torchmetrics and W&B are not
part of this build; metrics/logging are out of scope).
"""
from __future__ import annotations

import dataclasses
from enum import Enum
from typing import Any, Literal

import torch
import torch.nn as nn

from .. import ops
from ..utils import ClassWeights
from ..utils.placeholder import Placeholder


class OptimizerAlgo(str, Enum):
    ADAM = "adam"
    ADAMW = "adamw"
    SGD = "sgd"


class LossType(str, Enum):
    MSE = "MSE"
    CE = "CE"
    SMOOTH_L1 = "SmoothL1"


@dataclasses.dataclass(kw_only=True)
class LRSchedulerConfig:
    name: str
    kwargs: dict[str, Any]
    monitor: str = "val_loss"
    interval: Literal["epoch", "step"] = "epoch"
    frequency: int = 1


@dataclasses.dataclass(kw_only=True)
class OptimizerConfig:
    lr: float = 0.001
    lr_scheduler: LRSchedulerConfig | None = None
    weight_decay: float = 0.01
    algo: OptimizerAlgo = OptimizerAlgo.ADAMW
    loss_type: LossType = LossType.CE
    class_weights_mode: ClassWeights = ClassWeights.UNIFORM
    class_weights: Placeholder[torch.Tensor] = dataclasses.field(default_factory=Placeholder,
                                                                 init=False)


@dataclasses.dataclass(kw_only=True)
class BaseModelConfig:
    num_classes: Placeholder[int] = dataclasses.field(default_factory=Placeholder, init=False)
    optimizer: OptimizerConfig
    name: str


class CrossEntropyLoss(nn.Module):
    """nn.CrossEntropyLoss(weight) (mean reduction) on the HIP criterion kernels
    (ops.cross_entropy); `weight` is kept as a buffer so .to(device) moves it."""

    def __init__(self, weight: torch.Tensor | None = None):
        super().__init__()
        self.register_buffer("weight", None if weight is None else weight.float().clone())

    def forward(self, logits: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        return ops.cross_entropy(logits, target, self.weight)


class RegressionLoss(nn.Module):
    """nn.MSELoss() / nn.SmoothL1Loss() (mean reduction, reference base.py:95-96) on the HIP
    regression criterion (ops.regression_loss); BaseModule.training_step runs the regression
    clamp in the same launch."""

    def __init__(self, kind: str):
        super().__init__()
        self.kind = kind

    def forward(self, pred: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        inf = float("inf")
        return ops.regression_loss(pred, target, -inf, inf, self.kind)[1]


def make_criterion(cfg: OptimizerConfig) -> nn.Module:
    kind = LossType(cfg.loss_type)
    if kind is LossType.CE:
        # reference base.py:93-94 reads the placeholder (unset -> ValueError, as there)
        return CrossEntropyLoss(weight=cfg.class_weights.value)
    return RegressionLoss(kind.value)


class BaseModule(nn.Module):
    """Holds `self.model` (set by subclasses), the criterion and the step logic."""

    model: nn.Module

    def __init__(self, config: BaseModelConfig):
        super().__init__()
        opt = config.optimizer
        self.loss_type = LossType(opt.loss_type)
        self.num_classes = config.num_classes.value
        self.criterion = make_criterion(opt)
        self.lr, self.weight_decay = opt.lr, opt.weight_decay
        self.optimizer_algo = OptimizerAlgo(opt.algo)
        self.lr_scheduler_config = opt.lr_scheduler

    @property
    def is_regression(self) -> bool:
        return self.loss_type in (LossType.MSE, LossType.SMOOTH_L1)

    def _model_logits(self, data) -> torch.Tensor:
        edge_index = getattr(data, "adj_t", None)
        if edge_index is None:
            edge_index = data.edge_index
        return self.model(data.x, edge_index, data.batch, getattr(data, "num_graphs", None))

    def forward(self, data) -> torch.Tensor:
        """data: object with x, edge_index (or adj_t / a Graph), batch [, num_graphs]."""
        logits = self._model_logits(data)
        if self.is_regression:
            logits = torch.clamp(logits.squeeze(1), min=0, max=self.num_classes - 1)
        return logits

    def training_step(self, batch, batch_idx: int = 0) -> torch.Tensor:
        if self.is_regression and isinstance(self.criterion, RegressionLoss):
            # the clamp (forward) and the criterion in one HIP launch each way; y read as given
            # (the reference's y.float() happens in the kernel)
            return ops.regression_loss(self._model_logits(batch), batch.y, 0.0,
                                       float(self.num_classes - 1), self.criterion.kind)[1]
        # model + criterion as one node where the model offers it (GCN; the eager model only:
        # a compiled model keeps the reference's logits -> criterion sequence)
        fused = None if hasattr(self.model, "_orig_mod") else getattr(self.model, "forward_loss",
                                                                         None)
        if fused is not None and isinstance(self.criterion, CrossEntropyLoss):
            edge_index = getattr(batch, "adj_t", None)
            if edge_index is None:
                edge_index = batch.edge_index
            return fused(batch.x, edge_index, batch.batch, batch.y, self.criterion.weight,
                         getattr(batch, "num_graphs", None))[1]
        logits = self(batch)
        y = batch.y.float() if self.is_regression else batch.y
        return self.criterion(logits, y)

    def configure_optimizers(self):
        """Reference base.py:162-188: the optimizer, plus a torch.optim.lr_scheduler by name or
        pl_bolts' LinearWarmupCosineAnnealingLR (restated in lesion_gnn_amd.optim). Adam and
        AdamW step in one HIP launch (lesion_gnn_amd.optim, same update as torch's)."""
        from .. import optim as lgnn_optim

        ctor = {
            OptimizerAlgo.ADAM: lgnn_optim.Adam,
            OptimizerAlgo.ADAMW: lgnn_optim.AdamW,
            OptimizerAlgo.SGD: torch.optim.SGD,
        }[self.optimizer_algo]
        optimizer = ctor(self.parameters(), lr=self.lr, weight_decay=self.weight_decay)
        sc = self.lr_scheduler_config
        if sc is None:
            return optimizer
        if sc.name == "LinearWarmupCosineAnnealingLR":  # reference base.py:174-175 (pl_bolts)
            scheduler = lgnn_optim.LinearWarmupCosineAnnealingLR(optimizer, **sc.kwargs)
        else:
            scheduler = getattr(torch.optim.lr_scheduler, sc.name)(optimizer, **sc.kwargs)
        return {"optimizer": optimizer,
                "lr_scheduler": {"scheduler": scheduler, "monitor": sc.monitor,
                                 "interval": sc.interval, "frequency": sc.frequency}}
