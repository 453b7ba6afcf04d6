"""Run the C2 fused split-3 backward (k_s3_fbwd<3, true>, the step's CE-free entry with the
logits gradient) N times on the in-tree library, for profilers that attribute samples to
instructions (rocprofv3 PC sampling). Diagnostics only.

  rocprofv3 --pc-sampling-beta-enabled ... -- python3 tools/fbwd_loop.py [N]
"""
from __future__ import annotations

import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(n: int = 200) -> None:
    import torch

    from lesion_gnn_amd import _lib, ops, synth
    from lesion_gnn_amd.graph import Graph

    dev = torch.device("cuda:0")
    b = synth.make_batch(1024, n=64, k=8, d_in=128, seed=0).to(dev)
    g = Graph(b.edge_index, b.num_nodes, b.batch, b.num_graphs)
    csr = g.csr("gcn")
    open_ = g.tile_open("gcn")
    M, L, D = b.num_nodes, 2, 128
    gen = torch.Generator(device=dev).manual_seed(0)
    Ws = [torch.randn(D, D, device=dev, generator=gen) / 11.3 for _ in range(L + 1)]
    Hs = [torch.randn(M, D, device=dev, generator=gen) for _ in range(L + 1)]
    W_out = torch.randn(5, D, device=dev, generator=gen) / 11.3
    dlog = torch.randn(b.num_graphs, 5, device=dev, generator=gen)
    dS_ws = torch.empty(2 * M * 128, device=dev)
    keep: dict = {}
    ops.stack_fwd(b.x, g, Ws, [torch.zeros(D, device=dev)] * (L + 1), keep)
    planes_t = keep["planes_t"]
    adjt = keep.get("adjt")
    adjt_ptr = adjt.data_ptr() if adjt is not None else ops._adjt_ptr(planes_t, L)
    lib = _lib.load()
    P = lib.lgnn_gcn_stack_bwd_partials(M)
    slabs = [torch.empty(P * (D * D + D), device=dev) for _ in range(L + 1)]
    arr = ctypes.c_void_p * (L + 1)
    args = (None, g.batch.data_ptr(), g.gptr.data_ptr(), 1, b.num_graphs,
            csr.rowptr.data_ptr(), csr.col.data_ptr(), csr.w.data_ptr(), csr.tptr.data_ptr(),
            csr.tidx.data_ptr(), csr.tw.data_ptr(), b.x.data_ptr(), M, L, planes_t.data_ptr(),
            arr(*[W.data_ptr() for W in Ws]), arr(*[h.data_ptr() for h in Hs]),
            (ctypes.c_void_p * L)(*[h.data_ptr() for h in Hs[1:]]),
            (ctypes.c_int * (L + 2))(D, D, D, D),
            arr(*[t.data_ptr() for t in slabs]), arr(*[t.data_ptr() + P * D * D * 4 for t in slabs]),
            P, dS_ws.data_ptr(), open_.data_ptr(), dlog.data_ptr(), W_out.data_ptr(),
            W_out.size(0), adjt_ptr, torch.cuda.current_stream().cuda_stream)
    for _ in range(n):
        assert lib.lgnn_gcn_stack_bwd_s3f_all(*args) == 0
    torch.cuda.synchronize()
    print("done", n)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 200)
