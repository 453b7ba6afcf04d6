"""Edge-weight transform of lesion graphs on the GPU (liblgnn `lgnn_gaussian_distance`).

Mirrors `lesion_gnn.transforms.GaussianDistance` and `SaveAs` (reference
src/lesion_gnn/transforms.py:26-79; its known-answer tests, test/test_transforms.py:8-77, are
restated in tests/test_gpu_edge.py): same constructor, same three `save_as` modes, same
warning-and-return on a graph without edges, same dtype handling (weights evaluated in the
precision of `pos`, then cast to `dtype`). The weights feed DRGNet's GraphConv stack
(models/drgnet.py:55, edge_weight at :103) through `lesion_gnn_amd.conv.GraphConv`.
"""
from __future__ import annotations

import dataclasses
import math
import warnings
from enum import Enum
from typing import Any

import torch

from . import _lib


class SaveAs(Enum):
    EDGE_WEIGHT_REPLACE = "edge_weight_replace"
    EDGE_ATTR_CAT = "edge_attr_cat"
    EDGE_ATTR_REPLACE = "edge_attr_replace"


def gaussian_distance(edge_index: torch.Tensor, pos: torch.Tensor, sigma: float,
                      dtype: torch.dtype = torch.float32) -> torch.Tensor:
    """w[e] = exp(-|pos[row_e] - pos[col_e]|^2 / (2 sigma^2)) / sqrt(2 pi sigma^2), one HIP
    launch for a whole collated batch. Raises on out-of-range indices (one host sync)."""
    _lib.require_gpu(edge_index, pos)
    if edge_index.dim() != 2 or edge_index.size(0) != 2:
        raise ValueError("edge_index must be [2, E]")
    if pos.dim() != 2:
        raise ValueError("pos must be [N, D]")
    if dtype not in (torch.float32, torch.float64):
        raise ValueError("dtype must be torch.float32 or torch.float64")
    if not sigma > 0:
        raise ValueError("sigma must be positive")
    dev = pos.device
    pos_f64 = pos.dtype == torch.float64
    pos = pos.contiguous() if pos.dtype in (torch.float32, torch.float64) else \
        pos.to(torch.float32).contiguous()
    ei = edge_index.to(torch.int64).contiguous()
    E = ei.size(1)
    out = torch.empty(E, dtype=dtype, device=dev)
    err = torch.empty(1, dtype=torch.int32, device=dev)
    _lib.call("lgnn_gaussian_distance", _lib.ptr(pos), int(pos_f64), pos.size(0), pos.size(1),
              _lib.ptr(ei), E, float(sigma), _lib.ptr(out), int(dtype == torch.float64),
              _lib.ptr(err), _lib.stream(dev))
    if E and int(err.item()):
        raise IndexError(f"edge_index has {int(err.item())} edges outside [0, {pos.size(0)})")
    return out


class GaussianDistance:
    """Reference GaussianDistance(sigma, save_as, dtype) (transforms.py:32-79), on the GPU."""

    def __init__(self, sigma: float, save_as: SaveAs = SaveAs.EDGE_WEIGHT_REPLACE,
                 dtype: torch.dtype = torch.float32):
        self.sigma = sigma
        self._norm_const = math.sqrt(2 * math.pi * sigma ** 2)
        self.save_as = save_as
        self.dtype = dtype

    def __call__(self, data):
        if data.edge_index.numel() == 0:
            warnings.warn("The graph has no edges, returning the original data object.")
            return data
        pseudo = getattr(data, "edge_attr", None)
        dist = gaussian_distance(data.edge_index, data.pos, self.sigma, self.dtype)
        if self.save_as == SaveAs.EDGE_WEIGHT_REPLACE:
            data.edge_weight = dist
        elif self.save_as == SaveAs.EDGE_ATTR_CAT:
            dist = dist.view(-1, 1)
            if pseudo is not None:
                pseudo = pseudo.view(-1, 1) if pseudo.dim() == 1 else pseudo
                data.edge_attr = torch.cat([pseudo, dist.type_as(pseudo)], dim=-1)
            else:
                data.edge_attr = dist
        elif self.save_as == SaveAs.EDGE_ATTR_REPLACE:
            data.edge_attr = dist.view(-1, 1)
        return data

    def __repr__(self) -> str:
        return f"{self.__class__.__name__}(sigma={self.sigma})"


@dataclasses.dataclass(kw_only=True)
class TransformConfig:
    """Reference transforms.py:13-16: a transform by name plus its keyword arguments."""

    name: str
    kwargs: dict[str, Any] = dataclasses.field(default_factory=dict)


def get_transform(config: TransformConfig):
    """Reference transforms.py:19-23: GaussianDistance by name, otherwise the
    torch_geometric.transforms class of that name. The graph-building transforms the reference
    configs and sweep use run on the GPU here (KNNGraph, RadiusGraph — sweep.py:105-118 —,
    GaussianDistance); ToSparseTensor is accepted (the models take either input form); any other
    PyG transform is outside the hot path and raises."""
    kw = dict(config.kwargs)
    if config.name == "GaussianDistance":
        return GaussianDistance(**kw)
    if config.name == "KNNGraph":
        from .knn import KNNGraph

        return KNNGraph(**kw)
    if config.name == "RadiusGraph":
        from .knn import RadiusGraph

        return RadiusGraph(**kw)
    if config.name == "ToSparseTensor":
        from .datasets.datamodule import ToSparseTensor

        return ToSparseTensor()
    raise NotImplementedError(f"transform {config.name!r} is not part of this package (the "
                              "reference configs use KNNGraph, RadiusGraph and GaussianDistance)")
