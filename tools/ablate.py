"""Timing-only ablation of the tile kernels (cdna_hip_programming.md §7 'Ablate').

Builds liblgnn variants with -DLGNN_ABLATE=<mask> (1 no MFMA, 2 no aggregation, 4 no global
stores, 16 no global row loads) under tools/_abl/, then times the C2 conv-forward and
conv-backward launches of each variant with HIP events (launches queued behind a spin kernel).
Outputs of ablated builds are garbage by design; only the times matter.

  python tools/ablate.py build          # here (hipcc cross-compiles gfx950)
  python tools/ablate.py run            # on the GPU box
"""
from __future__ import annotations

import ctypes
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tools", "_abl")
MASKS = [0, 1, 2, 4, 16, 1 | 2, 2 | 4 | 16, 1 | 2 | 4 | 16, 32]


def build():
    os.makedirs(OUT, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(ROOT, "lesion_gnn_amd", "csrc", "*.hip")))
    procs = []
    for m in MASKS:
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
               "-shared", f"-DLGNN_ABLATE={m}", *srcs, "-o", os.path.join(OUT, f"liblgnn_{m}.so")]
        procs.append(subprocess.Popen(cmd))
    for p in procs:
        assert p.wait() == 0


def run():
    sys.path.insert(0, ROOT)
    import torch

    from lesion_gnn_amd import _lib, ops, synth
    from lesion_gnn_amd.graph import Graph

    dev = torch.device("cuda:0")
    b = synth.make_batch(1024, n=64, k=8, d_in=128, seed=0).to(dev)
    g = Graph(b.edge_index, b.num_nodes, b.batch, b.num_graphs)
    csr = g.csr("gcn")
    M, K, N = b.num_nodes, 128, 128
    W = torch.randn(N, K, device=dev) / 11.3
    bias = torch.randn(N, device=dev)
    Y = torch.empty(M, N, device=dev)
    S = torch.empty(M, K, device=dev)
    dS = torch.randn(M, N, device=dev)
    P = ops.num_partials(M, N, K, False)
    dWp = torch.empty(P * N * K, device=dev)
    dbp = torch.empty(P * N, device=dev)
    dX = torch.empty(M, K, device=dev)
    s = torch.cuda.current_stream()
    with torch.no_grad():
        H, S0 = ops.linear_fwd(b.x, W, bias, _lib.LGNN_ACT_ELU, csr, save_s=True)

    def timed(fn, reps=20):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(10_000_000)
        e0.record(s)
        for _ in range(reps):
            fn()
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3

    print(f"{'mask':>5} {'fwd_gather_us':>14} {'fwd_plain_us':>13} {'bwd_transpose_us':>17}")
    for m in MASKS:
        lib = ctypes.CDLL(os.path.join(OUT, f"liblgnn_{m}.so"))
        for name, (res, args) in _lib.SIGNATURES.items():
            f = getattr(lib, name)
            f.restype, f.argtypes = res, args

        def fwd_gather():
            lib.lgnn_node_linear_fwd(b.x.data_ptr(), M, K, csr.rowptr.data_ptr(),
                                     csr.col.data_ptr(), csr.w.data_ptr(), 0.0, W.data_ptr(),
                                     bias.data_ptr(), N, 1, Y.data_ptr(), S.data_ptr(),
                                     s.cuda_stream)

        def fwd_plain():
            lib.lgnn_node_linear_fwd(b.x.data_ptr(), M, K, None, None, None, 0.0, W.data_ptr(),
                                     bias.data_ptr(), N, 0, Y.data_ptr(), None, s.cuda_stream)

        def bwd():
            lib.lgnn_node_linear_bwd(2, dS.data_ptr(), None, None, 1, csr.tptr.data_ptr(),
                                     csr.tidx.data_ptr(), csr.tw.data_ptr(), 0.0, H.data_ptr(),
                                     1, S0.data_ptr(), M, K, None, None, None, 0.0, W.data_ptr(),
                                     N, dX.data_ptr(), dWp.data_ptr(), dbp.data_ptr(), P,
                                     s.cuda_stream)

        print(f"{m:5d} {timed(fwd_gather):14.2f} {timed(fwd_plain):13.2f} {timed(bwd):17.2f}",
              flush=True)


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
