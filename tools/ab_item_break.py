"""A/B helper: bench.py with the round-5 dropout scale rounding (a torch scalar + .item(), which
graph-breaks the compiled GAT on the GPU box) patched back in. Usage: python tools/ab_item_break.py
<bench args...>"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lesion_gnn_amd import dropout  # noqa: E402


def threshold_scale(p):
    if not 0.0 <= p < 1.0:
        raise ValueError(p)
    return int(p * 16777216.0), float(torch.tensor(1.0 / (1.0 - p), dtype=torch.float32))


dropout.threshold_scale = threshold_scale
import bench  # noqa: E402

sys.argv = ["bench.py"] + sys.argv[1:]
bench.main()
