"""Reference src/lesion_gnn/datasets/datamodule.py:27-34 (`DataConfig`) and the transform
composition of `DataModule.__init__` (:42-48): the configured transforms in order, plus
`ToSparseTensor` when the model is not compiled (:44-45). The Lightning DataModule, the image
datasets and the PyG DataLoader are out of scope; `compose_transforms` returns the
per-batch transform chain this package runs on the GPU (KNNGraph, GaussianDistance) so a
synthetic or pre-collated batch goes through the same graph construction the reference applies
per sample."""
from __future__ import annotations

import dataclasses

from ..transforms import TransformConfig, get_transform
from .aptos import AptosConfig
from .ddr import DDRConfig


@dataclasses.dataclass(kw_only=True)
class DataConfig:
    train_datasets: list[AptosConfig | DDRConfig]
    val_datasets: list[AptosConfig | DDRConfig]
    test_datasets: list[AptosConfig | DDRConfig]
    transforms: list[TransformConfig]
    batch_size: int
    num_workers: int


class Compose:
    """torch_geometric.transforms.Compose: apply the transforms in order."""

    def __init__(self, transforms: list):
        self.transforms = list(transforms)

    def __call__(self, data):
        for t in self.transforms:
            data = t(data)
        return data

    def __repr__(self) -> str:
        return f"Compose({self.transforms!r})"


class ToSparseTensor:
    """The reference appends torch_geometric's ToSparseTensor when `compile=False`
    (datamodule.py:44-45) so the model receives `adj_t` (target-major CSR). This package's
    models build that CSR on the GPU from either input (graph.py), so the transform records
    the choice and leaves `edge_index` in place; `as_graph` accepts both forms."""

    def __call__(self, data):
        return data

    def __repr__(self) -> str:
        return "ToSparseTensor()"


def compose_transforms(config: DataConfig, compile: bool = False) -> Compose:
    """The transform chain of DataModule.__init__ (datamodule.py:43-45)."""
    t = Compose([get_transform(c) for c in config.transforms])
    if not compile:
        t.transforms.append(ToSparseTensor())
    return t
