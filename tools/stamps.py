"""Phase timing of k_stack_fwd from in-kernel s_memtime stamps (diagnostic build, -DLGNN_STAMPS).

  python tools/stamps.py build     # here
  python tools/stamps.py run       # GPU box: average cycles between consecutive stamps
The stamped build's run time is not quoted anywhere; only the phase shares are read.
"""
from __future__ import annotations

import ctypes
import glob
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tools", "_abl", "liblgnn_stamps%s.so")


VARIANTS = {"": [], "_u1": ["-DLGNN_AGG_UNROLL=1"], "_u4": ["-DLGNN_AGG_UNROLL=4"]}


def build():
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(ROOT, "lesion_gnn_amd", "csrc", "*.hip")))
    procs = [subprocess.Popen(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC",
                               "--offload-arch=gfx950", "-shared", "-DLGNN_STAMPS", *flags, *srcs,
                               "-o", LIB % v]) for v, flags in VARIANTS.items()]
    assert all(p.wait() == 0 for p in procs)


def run():
    for v in VARIANTS:
        print("== variant", v or "default")
        run_one(LIB % v)


def run_one(libpath):
    sys.path.insert(0, ROOT)
    import torch

    from lesion_gnn_amd import _lib, synth
    from lesion_gnn_amd.graph import Graph

    lib = ctypes.CDLL(libpath)
    for name, (res, args) in _lib.SIGNATURES.items():
        f = getattr(lib, name)
        f.restype, f.argtypes = res, args
    lib.lgnn_debug_stamps.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda:0")
    b = synth.make_batch(1024, n=64, k=8, d_in=128, seed=0).to(dev)
    g = Graph(b.edge_index, b.num_nodes, b.batch, b.num_graphs)
    csr = g.csr("gcn")
    M, L = b.num_nodes, 2
    Ws = [torch.randn(128, 128, device=dev) / 11.3 for _ in range(L + 1)]
    bs = [torch.randn(128, device=dev) for _ in range(L + 1)]
    hs = [torch.empty(M, 128, device=dev) for _ in range(L + 1)]
    ss = [torch.empty(M, 128, device=dev) for _ in range(L + 1)]
    arr = ctypes.c_void_p * (L + 1)
    Wp, bp = arr(*[w.data_ptr() for w in Ws]), arr(*[x.data_ptr() for x in bs])
    Hp, Sp = arr(*[x.data_ptr() for x in hs]), arr(*[x.data_ptr() for x in ss])
    widths = (ctypes.c_int * (L + 1))(128, 128, 128)
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        assert lib.lgnn_gcn_stack_fwd(b.x.data_ptr(), M, 128, 1, csr.rowptr.data_ptr(),
                                      csr.col.data_ptr(), csr.w.data_ptr(), L, Wp, bp, widths,
                                      Hp, Sp, None, s) == 0
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        lib.lgnn_gcn_stack_fwd(b.x.data_ptr(), M, 128, 1, csr.rowptr.data_ptr(),
                               csr.col.data_ptr(), csr.w.data_ptr(), L, Wp, bp, widths, Hp, Sp,
                               None, s)
    e1.record()
    torch.cuda.synchronize()
    print(f"stamped build: {e0.elapsed_time(e1) / 10 * 1e3:.1f} us per launch (shares only)")
    buf = (ctypes.c_ulonglong * (1024 * 64))()
    assert lib.lgnn_debug_stamps(buf) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 64)[:512].astype(np.int64)
    n = int((a[0] > 0).sum())
    d = np.diff(a[:, :n], axis=1)
    names = ["start->tile0 ready", "MFMA0", "epi0 sync", "H0 store",
             "agg1", "MFMA1", "epi1 sync", "H1 store", "agg2", "MFMA2", "epi2 sync",
             "H2 store+sync", "->tile1 ready", "MFMA0", "epi0 sync", "H0 store", "agg1", "MFMA1",
             "epi1 sync", "H1 store", "agg2", "MFMA2", "epi2 sync", "H2 store+sync"]
    tot = (a[:, n - 1] - a[:, 0]).mean()
    print(f"stamps per block: {n}; mean kernel span {tot:.0f} cycles")
    for i in range(n - 1):
        nm = names[i] if i < len(names) else str(i)
        print(f"{i:2d} {nm:22s} mean {d[:, i].mean():9.0f}  p90 {np.percentile(d[:, i], 90):9.0f}")


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
