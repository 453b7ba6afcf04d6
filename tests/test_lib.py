"""CPU checks of the C-ABI library: it loads without a GPU, exports every symbol include/lgnn.h
declares, and the ctypes signature table matches the header. No compute calls."""
import ctypes
import os
import re

import pytest

from lesion_gnn_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "lgnn.h")


def declared_functions() -> dict[str, int]:
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    out = {}
    for m in re.finditer(r"^\s*[a-zA-Z_][\w\s\*]*?\b(lgnn_\w+)\s*\(([^;]*?)\)\s*;", text,
                         flags=re.M | re.S):
        args = m.group(2).strip()
        out[m.group(1)] = 0 if args in ("", "void") else args.count(",") + 1
    return out


def test_header_parses():
    fns = declared_functions()
    assert "lgnn_node_linear_fwd" in fns and "lgnn_graph_build" in fns
    assert len(fns) >= 12


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for name in declared_functions():
        assert hasattr(lib, name), f"liblgnn.so does not export {name}"


def test_ctypes_table_matches_header():
    fns = declared_functions()
    assert set(fns) == set(_lib.SIGNATURES), set(fns) ^ set(_lib.SIGNATURES)
    for name, nargs in fns.items():
        assert len(_lib.SIGNATURES[name][1]) == nargs, name


def test_abi_version_and_status_strings():
    lib = _lib.load()
    assert lib.lgnn_abi_version() == _lib.ABI_VERSION
    assert lib.lgnn_status_string(0) == b"ok"
    assert lib.lgnn_status_string(-22) == b"invalid argument"


def test_argument_validation_without_gpu():
    lib = _lib.load()
    # invalid shapes are rejected before any launch
    assert lib.lgnn_node_linear_fwd(None, 10, 0, None, None, None, 0.0, None, None, 4, 0, None,
                                    None, None) == -22
    assert lib.lgnn_bwd_num_partials(100, 0, 128, 0) == -22
    assert lib.lgnn_bwd_num_partials(65536, 128, 128, 0) > 0
    assert lib.lgnn_graph_build(None, 0, -1, 1, 1, None, None, None, None, None, None, None,
                                None, None, 0, None, None, None, 0, None) == -22
    # too large for the 30-bit chained scan
    assert lib.lgnn_graph_build(None, 1 << 30, 1, 1, 1, 1, 1, None, None, None, None, None,
                                None, None, 0, None, None, None, 0, None) == -22


def test_product_path_refuses_cpu_tensors():
    import torch

    from lesion_gnn_amd.graph import Graph

    with pytest.raises(_lib.LgnnError):
        Graph(torch.zeros(2, 3, dtype=torch.long), 4)


def test_stack_fwd_validation_without_gpu():
    import ctypes

    lib = _lib.load()
    arr = (ctypes.c_void_p * 2)(None, None)
    widths = (ctypes.c_int * 2)(128, 128)
    assert lib.lgnn_gcn_stack_fwd(None, -1, 128, 1, None, None, None, 1, arr, arr, widths, arr,
                                  None, None) == -22
    big = (ctypes.c_int * 2)(256, 128)  # widths beyond the tile fast path are refused
    assert lib.lgnn_gcn_stack_fwd(None, 10, 128, 1, None, None, None, 1, arr, arr, big, arr,
                                  None, None) == -22
    # a conv stack needs the tile flags (closed tiles are aggregated on chip)
    assert lib.lgnn_gcn_stack_fwd(None, 10, 128, 1, 1, 1, None, 1, arr, arr, widths, arr,
                                  None, None) == -22
    assert lib.lgnn_tile_count(65) == 2 and lib.lgnn_tile_count(64) == 1


def test_dropout_seeds_distinct_without_cpu_draws():
    """Two unsalted constructions with no CPU generator draw in between (a lone conv, meta
    parameters) get different dropout seeds: derived_seed mixes a per-process counter into the
    hash of the generator state, and leaves the generator untouched."""
    import torch

    from lesion_gnn_amd import dropout

    torch.manual_seed(0)
    before = torch.default_generator.get_state().clone()
    a, b = dropout.derived_seed(), dropout.derived_seed()
    assert a != b
    assert torch.equal(torch.default_generator.get_state(), before)
    assert 0 <= a < 2 ** 62 and 0 <= b < 2 ** 62


def test_dropout_seed_reproducible_under_manual_seed():
    """Re-seeding and rebuilding reproduces a model's dropout seed, whatever was built in
    between (the seed is salted with the model's initial weights, not a process counter); two
    models with different weights get different seeds, and building leaves the generator where
    weight init left it."""
    import torch

    from lesion_gnn_amd.models.gat import GAT
    from lesion_gnn_amd.models.gcn import GCN
    from lesion_gnn_amd.models.gin import GIN

    builders = {"GCN": lambda: GCN(16, [32, 32], 3, 0.35), "GIN": lambda: GIN(16, [32, 32], 3, 0.35),
                "GAT": lambda: GAT(16, [32, 32], 3, 2, 0.35)}
    for name, build in builders.items():
        torch.manual_seed(7)
        m1 = build()
        after = torch.default_generator.get_state().clone()
        build()  # a construction in between
        torch.manual_seed(7)
        m2 = build()
        assert torch.equal(torch.default_generator.get_state(), after)
        m3 = build()
        s1, s2, s3 = (int(m._dropout_rng[0]) for m in (m1, m2, m3))
        assert s1 == s2 and s3 != s1, name


def test_dropout_scale_is_fp32_rounding_without_torch_scalars():
    """dropout.threshold_scale rounds 1 / (1 - p) to fp32 in plain Python (a torch scalar there
    was a Tensor.item() graph break under torch.compile): equal to numpy's float32 rounding."""
    import random

    import numpy as np

    from lesion_gnn_amd import dropout

    rnd = random.Random(7)
    ps = [0.0, 0.1, 0.25, 0.35, 0.5, 0.9, 1 / 3] + [rnd.random() * 0.999 for _ in range(20000)]
    for p in ps:
        thr, scale = dropout.threshold_scale(p)
        assert scale == float(np.float32(1.0 / (1.0 - p))), p
        assert thr == int(p * 16777216.0)
