"""Reference src/lesion_gnn/datasets/base.py:17-24 (`BaseDatasetConfig`). The InMemoryDataset
behind it (base.py:27-115: the processed `data.pt` cache of image-derived graphs) is out of
scope — no dataset is available offline."""
from __future__ import annotations

import dataclasses
from typing import Any, Callable

from .nodes.lesions import LesionsNodesConfig
from .nodes.sift import SiftNodesConfig


@dataclasses.dataclass(kw_only=True)
class BaseDatasetConfig:
    name: str
    root: str
    nodes: LesionsNodesConfig | SiftNodesConfig
    transform: Callable[..., Any] | None = None
    log: bool = True
    num_workers: int = 0
