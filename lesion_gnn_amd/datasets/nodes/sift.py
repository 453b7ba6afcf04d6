"""Reference src/lesion_gnn/datasets/nodes/sift.py:11-14 (`SiftNodesConfig`). The OpenCV SIFT
extractor itself is out of scope (image preprocessing)."""
from __future__ import annotations

import dataclasses


@dataclasses.dataclass(kw_only=True)
class SiftNodesConfig:
    num_keypoints: int
    sigma: float
