"""Lesion-node extractor configuration (reference src/lesion_gnn/datasets/nodes/lesions.py:
22-71: the feature sources, `FeaturesReduction`, `LesionsNodesConfig`).

The extractor itself (`LesionsExtractor.__call__`, :111-177: fundus segmentation, a timm encoder
from the HF hub, OpenCV connected components) needs network weights and image data and is out
of scope; its per-component feature pooling `extract_features_by_cc` (:88-93,
called at :172) is the scatter that produces the d_in = encoder channels + 1 node features, and
runs here on the HIP kernel lgnn_cc_pool.
"""
from __future__ import annotations

import dataclasses
from enum import Enum

import torch


@dataclasses.dataclass(kw_only=True)
class SegmentationEncoderFeatures:
    layer: int


@dataclasses.dataclass(kw_only=True)
class SegmentationDecoderFeatures:
    pass


@dataclasses.dataclass(kw_only=True)
class TimmEncoderFeatures:
    timm_model: str
    layer: int


FeatureSource = SegmentationEncoderFeatures | SegmentationDecoderFeatures | TimmEncoderFeatures


class FeaturesReduction(str, Enum):
    MEAN = "mean"
    MAX = "max"


@dataclasses.dataclass(kw_only=True)
class LesionsNodesConfig:
    feature_source: FeatureSource
    features_reduction: FeaturesReduction = FeaturesReduction.MEAN
    reinterpolation: tuple[int, int] | None = None
    compile: bool = True


def extract_features_by_cc(cc: torch.Tensor, features: torch.Tensor, nlabel: int,
                           reduce: str | FeaturesReduction = "mean") -> torch.Tensor:
    """Reference lesions.py:88-93. cc (H, W) int64 component labels (OpenCV
    connectedComponents), features (1, C, H, W) fp32 on the GPU -> [max(cc) + 1, C]: the mean
    (or max) feature of each component's pixels (torch_scatter.scatter(features.view(C, H*W).T,
    cc.flatten(), 0, reduce)); nlabel == 1 -> features.mean((2, 3)), the (1, C) global mean.
    One HIP launch pair (lgnn_cc_pool) reading the channel-major map once; the output size is
    read from the device (one host sync, as max(cc) + 1 is in torch_scatter)."""
    from ... import ops

    reduce = FeaturesReduction(reduce).value
    if features.dim() != 4 or features.size(0) != 1:
        raise ValueError("features must be (1, C, H, W)")
    C, H, W = features.shape[1:]
    if cc.numel() != H * W:
        raise ValueError("cc must be (H, W) like the feature map")
    f = features.reshape(C, H * W)
    if nlabel == 1:
        return ops.cc_pool(f, torch.zeros_like(cc), 1, reduce_max=False).view(1, C)
    size = int(cc.max().item()) + 1
    return ops.cc_pool(f, cc, size, reduce_max=(reduce == "max"))
