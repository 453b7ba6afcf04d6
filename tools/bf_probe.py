"""Timing probe for the bf16 GEMM kernels (csrc/bflin.hip) at C3 shapes: python tools/bf_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lesion_gnn_amd import _lib, ops  # noqa: E402


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


dev = torch.device("cuda:0")
M, N = 42279, 128
for K in (1024, 1025, 1028, 128):
    x = torch.randn(M, K, device=dev)
    W = torch.randn(N, K, device=dev)
    Wb, _ = ops.bf16_weight_operands(W, False)
    dyb = torch.randn(M, N, device=dev).to(torch.bfloat16)
    xb = x.to(torch.bfloat16) if K % 4 == 0 else None
    t1 = timeit(lambda: ops.bf16_gemm(x, Wb, None, N))
    t2 = timeit(lambda: ops.bf16_gemm(x, Wb, None, N, want_yb=True))
    t3 = timeit(lambda: ops.bf16_wgrad(dyb, x, N))
    line = f"K={K}: gemm f32 {t1:.1f} us (+yb {t2:.1f}), wgrad f32 (+reduce) {t3:.1f} us"
    if xb is not None:
        t4 = timeit(lambda: ops.bf16_gemm(xb, Wb, None, N))
        t5 = timeit(lambda: ops.bf16_wgrad(dyb, xb, N))
        line += f"; bf16 A gemm {t4:.1f}, wgrad {t5:.1f}"
    print(line, flush=True)
