"""Phase stamps + ablations of the fused split-3 GCN backward (k_s3_fbwd), diagnostics only.

  python tools/stamps_s3f.py build        # here: builds tools/_abl/liblgnn_s3f_<variant>.so
  python tools/stamps_s3f.py run          # GPU box: per-launch time of every variant and the
                                          # phase cycles (s_memtime) of the stamped build
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
LIB = os.path.join(ROOT, "tools", "_abl", "liblgnn_s3f_%s.so")
VARIANTS = {"default": [], "stamps": ["-DLGNN_STAMPS"]}
if os.environ.get("STAMPS_ABLATIONS"):
    for k, v in [("nomfma", 1), ("noglobal", 16)]:
        VARIANTS[k] = [f"-DLGNN_ABLATE={v}"]
    VARIANTS["sb"] = ["-DLGNN_S3F_SB"]
    VARIANTS["sb_stamps"] = ["-DLGNN_S3F_SB", "-DLGNN_STAMPS"]
NAMES = ["prologue: stage + load wait", "prologue: dZ_L", "prologue: Â planes", "l2 G, G image",
         "l2 H image", "l2 dW", "l2 dH+dZ", "l1 G, G image", "l1 H image", "l1 dW", "l1 dH+dZ",
         "l0 X + dW", "tile tail"]


# variant libraries built from another source tree (tools/build_base_lib.sh: git HEAD's sources
# as tools/_abl/liblgnn_s3f_base.so, an A/B baseline on the same box); not rebuilt here
PREBUILT = ["base", "base_stamps"]


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
    dP = torch.randn(b.num_graphs, D, device=dev, generator=gen)
    W_out = torch.randn(5, D, device=dev, generator=gen) / 11.3
    dlog = torch.randn(b.num_graphs, 5, device=dev, generator=gen)
    dS_ws = torch.empty(2 * M * 128, device=dev)
    # the forward's Â^T planes handed to the backward (STAMPS_ADJT=0: rebuilt from the CSR)
    keep = {}
    ops.stack_fwd(b.x, g, Ws, [torch.zeros(D, device=dev)] * (L + 1), keep)
    planes_t = keep["planes_t"]
    adjt_ptr = ops._adjt_ptr(planes_t, L) if os.environ.get("STAMPS_ADJT", "1") != "0" else None
    s = torch.cuda.current_stream().cuda_stream
    arr = ctypes.c_void_p * (L + 1)
    for v in [*VARIANTS, *[p for p in PREBUILT if os.path.exists(LIB % p)]]:
        lib = ctypes.CDLL(LIB % v)
        for name, (res, args) in _lib.SIGNATURES.items():
            f = getattr(lib, name, None)  # a variant built from an older source may lack some
            if f is not None:
                f.restype, f.argtypes = res, args
        P = lib.lgnn_gcn_stack_bwd_partials(M)
        slabs = [torch.empty(P * (D * D + D), device=dev) for _ in range(L + 1)]
        dWp = arr(*[t.data_ptr() for t in slabs])
        dbp = arr(*[t.data_ptr() + P * D * D * 4 for t in slabs])
        # the step's entry: the _all launch with the logits gradient (dZ_L = dlogits W_out
        # formed in the prologue), as ops.stack_bwd runs it at C2
        args = (None, g.batch.data_ptr(), g.gptr.data_ptr(), 1, b.num_graphs,
                csr.rowptr.data_ptr(), csr.col.data_ptr(), csr.w.data_ptr(), csr.tptr.data_ptr(),
                csr.tidx.data_ptr(), csr.tw.data_ptr(), b.x.data_ptr(), M, L,
                planes_t.data_ptr(), arr(*[W.data_ptr() for W in Ws]),
                arr(*[h.data_ptr() for h in Hs]), (ctypes.c_void_p * L)(*[h.data_ptr() for h in Hs[1:]]),
                (ctypes.c_int * (L + 2))(D, D, D, D), dWp, dbp, P, dS_ws.data_ptr(),
                open_.data_ptr(), dlog.data_ptr(), W_out.data_ptr(), W_out.size(0), adjt_ptr, s)
        for _ in range(3):
            assert lib.lgnn_gcn_stack_bwd_s3f_all(*args) == 0
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            lib.lgnn_gcn_stack_bwd_s3f_all(*args)
        e1.record()
        torch.cuda.synchronize()
        print(f"{v:14s} {e0.elapsed_time(e1) / 20 * 1e3:8.1f} us per launch", flush=True)
        if v.endswith("stamps"):
            lib.lgnn_debug_stamps_s3b.argtypes = [ctypes.c_void_p]
            buf = (ctypes.c_ulonglong * (1024 * 64))()
            assert lib.lgnn_debug_stamps_s3b(buf) == 0
            a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 64)[:P].astype(np.int64)
            n = int((a[0, :62] > 0).sum())
            d = np.diff(a[:, :n], axis=1)
            print(f"stamps per block: {n}; mean span {(a[:, n - 1] - a[:, 0]).mean():.0f} ticks")
            names = NAMES
            per = len(names)
            for i in range(per):  # phases of the 2nd and later tiles, averaged
                cols = [j for j in range(i, n - 1, per) if j >= per]
                if cols:
                    print(f"{i:2d} {names[i]:22s} mean {d[:, cols].mean():8.0f}")


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
