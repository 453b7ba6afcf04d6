"""Reference src/lesion_gnn/datasets/aptos.py:12-14 (`AptosConfig`, name fixed to "Aptos")."""
from __future__ import annotations

import dataclasses

from .base import BaseDatasetConfig


@dataclasses.dataclass(kw_only=True)
class AptosConfig(BaseDatasetConfig):
    name: str = dataclasses.field(default="Aptos", init=False)
