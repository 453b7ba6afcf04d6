"""Reference src/lesion_gnn/datasets/ddr.py:11-20 (`DDRVariant`, `DDRConfig`, name fixed to
"DDR")."""
from __future__ import annotations

import dataclasses
from enum import Enum

from .base import BaseDatasetConfig


class DDRVariant(str, Enum):
    TRAIN = "train"
    VALID = "valid"
    TEST = "test"


@dataclasses.dataclass(kw_only=True)
class DDRConfig(BaseDatasetConfig):
    variant: DDRVariant
    name: str = dataclasses.field(default="DDR", init=False)
