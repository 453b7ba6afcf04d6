"""Config helpers mirroring reference src/lesion_gnn/utils (Placeholder, ClassWeights)."""
from enum import Enum

from .placeholder import Placeholder


class ClassWeights(str, Enum):
    """Reference src/lesion_gnn/utils/__init__.py:4-8."""

    UNIFORM = "uniform"
    INVERSE = "inverse"
    QUADRATIC_INVERSE = "quadratic_inverse"
    INVERSE_FREQUENCY = "inverse_frequency"


__all__ = ["Placeholder", "ClassWeights"]
