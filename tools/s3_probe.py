"""Timing-only ablation of the split-3 forward k_s3_fwd (stack3.hip, -DLGNN_S3_ABLATE=<mask>).

  python tools/s3_probe.py build     # here: one library per mask under tools/_abl/
  python tools/s3_probe.py run       # GPU box: HIP-event time per launch of each variant (C2)
Outputs of ablated builds are garbage by design; only the times are read.
"""
from __future__ import annotations

import ctypes
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tools", "_abl")
MASKS = {0: "product", 1: "no GEMM1", 2: "no GEMM2", 3: "no MFMA", 4: "no H stores",
         8: "no ELU", 16: "no plane split", 32: "no W reloads", 64: "no X prefetch",
         4 | 8 | 16: "no epilogue work", 1 | 2 | 4 | 8 | 16 | 32 | 64: "skeleton",
         "fastelu": "LGNN_FAST_ELU"}


STAMP_NAMES = ["prologue+B1", "scatter+in_proj GEMM", "B2", "in_proj epilogue",
               "Â planes+B4", "L1 W load+GEMM1", "L1 P split", "L1 GEMM2", "L1 B5",
               "L1 epilogue", "L1 B6", "L2 W load+GEMM1", "L2 P split", "L2 GEMM2", "L2 B5",
               "L2 epilogue"]


def lib_path(m):
    return os.path.join(OUT, f"liblgnn_s3_{m}.so")


def build():
    os.makedirs(OUT, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(ROOT, "lesion_gnn_amd", "csrc", "*.hip")))
    procs = []
    for m in MASKS:
        flag = "-DLGNN_FAST_ELU" if m == "fastelu" else f"-DLGNN_S3_ABLATE={m}"
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
               "-shared", flag, *srcs, "-o", lib_path(m)]
        procs.append(subprocess.Popen(cmd))
    procs.append(subprocess.Popen(
        ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-shared",
         "-DLGNN_S3_STAMPS", *srcs, "-o", lib_path("stamps")]))
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
    csr, open_ = g.csr("gcn"), g.tile_open("gcn")
    M, L = b.num_nodes, 2
    Ws = [torch.randn(128, 128, device=dev) / 11.3 for _ in range(L + 1)]
    bs = [torch.randn(128, device=dev) for _ in range(L + 1)]
    hs = [torch.empty(M, 128, device=dev) for _ in range(L + 1)]
    planes, _ = ops.weight_planes(Ws, 128)
    arr = ctypes.c_void_p * (L + 1)
    bp, Hp = arr(*[x.data_ptr() for x in bs]), arr(*[x.data_ptr() for x in hs])
    widths = (ctypes.c_int * (L + 1))(128, 128, 128)
    s = torch.cuda.current_stream().cuda_stream
    for m, name in MASKS.items():
        lib = ctypes.CDLL(lib_path(m))
        f = lib.lgnn_gcn_stack_fwd_s3
        f.restype, f.argtypes = _lib.SIGNATURES["lgnn_gcn_stack_fwd_s3"]

        def launch():
            assert f(b.x.data_ptr(), M, 128, 1, csr.rowptr.data_ptr(), csr.col.data_ptr(),
                     csr.w.data_ptr(), L, planes.data_ptr(), bp, widths, Hp, open_.data_ptr(),
                     None, s) == 0
        for _ in range(3):
            launch()
        torch.cuda.synchronize()
        torch.cuda._sleep(10_000_000)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            launch()
        e1.record()
        torch.cuda.synchronize()
        print(f"{str(m):8s} {name:18s} {e0.elapsed_time(e1) / 20 * 1e3:8.1f} us", flush=True)
    # phase stamps (cycles of s_memtime) of the stamped build, one launch
    import numpy as np
    lib = ctypes.CDLL(lib_path("stamps"))
    f = lib.lgnn_gcn_stack_fwd_s3
    f.restype, f.argtypes = _lib.SIGNATURES["lgnn_gcn_stack_fwd_s3"]
    lib.lgnn_s3_debug_stamps.argtypes = [ctypes.c_void_p]
    for _ in range(3):
        assert f(b.x.data_ptr(), M, 128, 1, csr.rowptr.data_ptr(), csr.col.data_ptr(),
                 csr.w.data_ptr(), L, planes.data_ptr(), bp, widths, Hp, open_.data_ptr(), None,
                 s) == 0
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (1024 * 64))()
    assert lib.lgnn_s3_debug_stamps(buf) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 64)[:512].astype(np.int64)
    n = int((a[0] > 0).sum())
    d = np.diff(a[:, :n], axis=1)
    per = len(STAMP_NAMES)
    print(f"stamps per block {n}; mean span {(a[:, n - 1] - a[:, 0]).mean():.0f} cycles")
    for i in range(n - 1):
        print(f"{i:2d} {STAMP_NAMES[i % per]:22s} mean {d[:, i].mean():8.0f}  "
              f"p90 {np.percentile(d[:, i], 90):8.0f}")


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
