"""Timing variants + phase stamps of the fused GCN stack backward (k_stack_bwd), diagnostics only.

  python tools/stamps_bwd.py build        # here: builds tools/_abl/liblgnn_bwd_<variant>.so
  python tools/stamps_bwd.py run          # GPU box: per-launch time of every variant, phase
                                          # cycles (s_memtime) of the stamped build
Variant libraries live outside the package and are never loaded by it.
"""
from __future__ import annotations

import ctypes
import glob
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tools", "_abl", "liblgnn_bwd_%s.so")
VARIANTS = {
    "default": [],
    "stamps": ["-DLGNN_STAMPS"],
}


def build():
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(ROOT, "lesion_gnn_amd", "csrc", "*.hip")))
    procs = [subprocess.Popen(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC",
                               "--offload-arch=gfx950", "-shared", *flags, *srcs, "-o", LIB % v])
             for v, flags in VARIANTS.items()]
    assert all(p.wait() == 0 for p in procs)


def run():
    sys.path.insert(0, ROOT)
    import torch

    from lesion_gnn_amd import _lib, synth
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
    dP = torch.randn(b.num_graphs, D, device=dev, generator=gen)
    s = torch.cuda.current_stream().cuda_stream
    arr = ctypes.c_void_p * (L + 1)
    for v in VARIANTS:
        lib = ctypes.CDLL(LIB % v)
        for name, (res, args) in _lib.SIGNATURES.items():
            f = getattr(lib, name)
            f.restype, f.argtypes = res, args
        P = lib.lgnn_gcn_stack_bwd_partials(M)
        slabs = [torch.empty(P * (D * D + D), device=dev) for _ in range(L + 1)]
        dWp = arr(*[t.data_ptr() for t in slabs])
        dbp = arr(*[t.data_ptr() + P * D * D * 4 for t in slabs])
        args = (dP.data_ptr(), g.batch.data_ptr(), g.gptr.data_ptr(), 1, csr.rowptr.data_ptr(),
                csr.col.data_ptr(), csr.w.data_ptr(), b.x.data_ptr(), M, L,
                arr(*[w.data_ptr() for w in Ws]), arr(*[h.data_ptr() for h in Hs]),
                (ctypes.c_int * (L + 2))(D, D, D, D), dWp, dbp, P, open_.data_ptr(), s)
        for _ in range(3):
            assert lib.lgnn_gcn_stack_bwd(*args) == 0
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            lib.lgnn_gcn_stack_bwd(*args)
        e1.record()
        torch.cuda.synchronize()
        print(f"{v:10s} {e0.elapsed_time(e1) / 20 * 1e3:8.1f} us per launch", flush=True)
        if v == "stamps":
            lib.lgnn_debug_stamps.argtypes = [ctypes.c_void_p]
            buf = (ctypes.c_ulonglong * (1024 * 64))()
            assert lib.lgnn_debug_stamps(buf) == 0
            a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 64)[:P].astype(np.int64)
            n = int((a[0] > 0).sum())
            d = np.diff(a[:, :n], axis=1)
            names = ["tile start (scatter, dZ_L)", "l2 G + write", "l2 dW + DX",
                     "l2 dZ write", "l1 G + write", "l1 dW + DX", "l1 dZ write", "l0 dW + sync"]
            print(f"stamps per block: {n}; mean span {(a[:, n - 1] - a[:, 0]).mean():.0f} cycles")
            for i in range(min(n - 1, 24)):
                print(f"{i:2d} {names[i % 8]:26s} mean {d[:, i].mean():8.0f}  "
                      f"p90 {np.percentile(d[:, i], 90):8.0f}")


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
