"""Model registry (reference src/lesion_gnn/models/__init__.py:10,22-35: isinstance dispatch on
the config type), restricted to the message-passing families of the hot path."""
from .base import (BaseModelConfig, BaseModule, LossType, LRSchedulerConfig, OptimizerAlgo,
                   OptimizerConfig)
from .gcn import GCN, GCNConfig, GCNModule
from .gat import GAT, GATConfig, GATModule
from .gin import GIN, GINConfig, GINModule
from .drgnet import DRGNet, DRGNetModelConfig, DRGNetModule

ModelConfig = DRGNetModelConfig | GCNConfig | GINConfig | GATConfig

__all__ = ["GCN", "GCNConfig", "GCNModule", "GIN", "GINConfig", "GINModule", "GAT", "GATConfig",
           "GATModule", "DRGNet", "DRGNetModelConfig", "DRGNetModule", "BaseModule",
           "BaseModelConfig", "OptimizerConfig", "OptimizerAlgo", "LossType", "LRSchedulerConfig",
           "ModelConfig", "get_model"]


def get_model(config) -> BaseModule:
    if isinstance(config, DRGNetModelConfig):
        return DRGNetModule(config)
    if isinstance(config, GCNConfig):
        return GCNModule(config)
    if isinstance(config, GINConfig):
        return GINModule(config)
    if isinstance(config, GATConfig):
        return GATModule(config)
    raise ValueError(f"Unknown model config type {type(config)}")
