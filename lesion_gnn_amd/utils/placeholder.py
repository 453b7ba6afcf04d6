"""Runtime-filled config value (reference src/lesion_gnn/utils/placeholder.py:6-21 semantics)."""
from typing import Generic, TypeVar

T = TypeVar("T")


class Placeholder(Generic[T]):
    """A config field filled from the dataset at run time; reading it unset is an error."""

    def __init__(self) -> None:
        self._value: T | None = None

    @property
    def value(self) -> T:
        if self._value is None:
            raise ValueError("Placeholder value not set")
        return self._value

    @value.setter
    def value(self, value: T) -> None:
        self._value = value

    def __repr__(self) -> str:
        return "Placeholder" if self._value is None else repr(self._value)
