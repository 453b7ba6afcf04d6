"""Lesion-node extractor configuration (reference src/lesion_gnn/datasets/nodes/lesions.py:
22-71: the feature sources, `FeaturesReduction`, `LesionsNodesConfig`).

The extractor itself (`LesionsExtractor.__call__`, :111-177: fundus segmentation, a timm encoder
from the HF hub, OpenCV connected components) needs network weights and image data and is out
of scope; only its output contract matters to the hot path (d_in = encoder
channels + 1 lesion-class channel).
"""
from __future__ import annotations

import dataclasses
from enum import Enum


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
