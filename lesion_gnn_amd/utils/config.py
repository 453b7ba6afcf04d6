"""Experiment configuration (reference src/lesion_gnn/utils/config.py:17-80): the `Config`
dataclass tree and the Python-file loader, so an experiment file such as the reference's
configs/config.py loads unchanged against this package.

Such a file imports the reference's module paths (`from lesion_gnn.models.gat import
GATConfig`, ...). `get_config` (and `install_reference_alias`) resolve `lesion_gnn` and every
`lesion_gnn.<sub>` module to `lesion_gnn_amd.<sub>` — the same module objects, so the config
classes the file builds are this package's and `get_model`'s isinstance dispatch
(models/__init__.py) takes them. The alias is only installed when the real `lesion_gnn` is not
already imported.
"""
from __future__ import annotations

import dataclasses
import importlib
import importlib.abc
import importlib.util
import os
import sys
import warnings
from argparse import ArgumentParser

from ..datasets.datamodule import DataConfig
from ..models import ModelConfig

REFERENCE_PACKAGE = "lesion_gnn"
PACKAGE = __name__.split(".")[0]  # lesion_gnn_amd


@dataclasses.dataclass(kw_only=True)
class Config:
    dataset: DataConfig
    model: ModelConfig
    monitored_metric: str
    monitor_mode: str
    early_stopping_patience: int | None = None
    max_epochs: int
    seed: int
    project_name: str
    tags: list[str] | None = None


class _AliasLoader(importlib.abc.Loader):
    def __init__(self, target: str):
        self.target = target

    def create_module(self, spec):
        return importlib.import_module(self.target)

    def exec_module(self, module):  # the target module is already executed
        pass


class _ReferenceAlias(importlib.abc.MetaPathFinder):
    """`lesion_gnn[.sub]` -> `lesion_gnn_amd[.sub]` (module swap at import time)."""

    def find_spec(self, fullname, path=None, target=None):
        if fullname != REFERENCE_PACKAGE and not fullname.startswith(REFERENCE_PACKAGE + "."):
            return None
        real = PACKAGE + fullname[len(REFERENCE_PACKAGE):]
        if importlib.util.find_spec(real) is None:
            return None
        is_pkg = importlib.util.find_spec(real).submodule_search_locations is not None
        return importlib.util.spec_from_loader(fullname, _AliasLoader(real), is_package=is_pkg)


def install_reference_alias() -> bool:
    """Make `import lesion_gnn...` resolve to this package. Returns False (and does nothing)
    when a real `lesion_gnn` is already imported."""
    mod = sys.modules.get(REFERENCE_PACKAGE)
    if mod is not None and not getattr(mod, "__name__", "").startswith(PACKAGE):
        return False
    if not any(isinstance(f, _ReferenceAlias) for f in sys.meta_path):
        sys.meta_path.insert(0, _ReferenceAlias())
    return True


def get_config(file_path: str | os.PathLike, module_name: str | None = None,
               alias_reference: bool = True) -> Config:
    """Reference utils/config.py:30-56: exec the Python file and return its `cfg`; with
    `module_name`, register the module in sys.modules under that name."""
    if alias_reference:
        install_reference_alias()
    name = module_name or "experiment_config"
    spec = importlib.util.spec_from_file_location(name, file_path)
    assert spec is not None, f"Could not load config file {file_path}"
    assert spec.loader is not None, f"Could not load config file {file_path}"
    module = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(module)
    if module_name is not None:
        sys.modules[name] = module
    return module.cfg


def parse_args(argv: list[str] | None = None) -> Config:
    """Reference utils/config.py:59-80: `--config FILE` is required; further arguments are
    ignored with a warning (the reference disabled CLI overrides, :74-75)."""
    parser = ArgumentParser()
    parser.add_argument("--config", type=str, help="Path to Python config file.", metavar="FILE",
                        required=True)
    args, remaining = parser.parse_known_args(argv)
    config = get_config(args.config)
    if remaining:
        warnings.warn("Overriding config values with command line arguments is disabled")
    return config
