"""Micro-timing of the split-3 GEMMs at the reference in_proj / lin shapes (tuning aid):
python tools/s3_micro.py -> one line per (kernel, shape): average us over 50 launches.
--inproj: only the in_proj shape (42,279 x 1025 -> 128), e.g. under rocprofv3 --pmc, so that
k_s3_wgrad2's per-launch HBM bytes belong to that shape alone (the step also runs it on the lins)."""
import sys

import torch

from lesion_gnn_amd import ops


def timeit(fn, n=50):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


dev = torch.device("cuda:0")
SHAPES = [(42279, 1025, 128)] if "--inproj" in sys.argv else [(42279, 1025, 128), (42279, 128, 128)]
if "--kalign" in sys.argv:  # the in_proj at 16-B aligned row strides (1024, 1028) vs 1025
    SHAPES = [(42279, 1024, 128), (42279, 1025, 128), (42279, 1028, 128)]
if "--lin" in sys.argv:  # the reference GATConv.lin shape alone (42,279 x 128 -> 128)
    SHAPES = [(42279, 128, 128)]
if "--wide" in sys.argv:  # the sweep's GIN [512]*4 linears (scripts/sweep.py:126)
    SHAPES += [(65536, 512, 512), (65536, 128, 512)]
for M, K, N in SHAPES:
    A = torch.randn(M, K, device=dev)
    W = torch.randn(N, K, device=dev)
    dY = torch.randn(M, N, device=dev)
    wp = ops.dense_planes(W, False, False)
    t_f = timeit(lambda: ops.dense_mm(A, wp, N, None, False))
    t_w = timeit(lambda: ops.dense_wgrad(dY, A, False))
    print(f"M={M} K={K} N={N}: gemm {t_f:.1f} us  wgrad(+reduce) {t_w:.1f} us", flush=True)
