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


VARIANTS = {"": [], "_noslp": ["-fno-slp-vectorize"], "_fastelu": ["-DLGNN_FAST_ELU"],
            "_both": ["-fno-slp-vectorize", "-DLGNN_FAST_ELU"], "_abl8": ["-DLGNN_ABLATE=8"]}


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
    open_ = g.tile_open("gcn")
    M, L = b.num_nodes, 2
    Ws = [torch.randn(128, 128, device=dev) / 11.3 for _ in range(L + 1)]
    bs = [torch.randn(128, device=dev) for _ in range(L + 1)]
    hs = [torch.empty(M, 128, device=dev) for _ in range(L + 1)]
    arr = ctypes.c_void_p * (L + 1)
    Wp, bp = arr(*[w.data_ptr() for w in Ws]), arr(*[x.data_ptr() for x in bs])
    Hp = arr(*[x.data_ptr() for x in hs])
    widths = (ctypes.c_int * (L + 1))(128, 128, 128)
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        assert lib.lgnn_gcn_stack_fwd(b.x.data_ptr(), M, 128, 1, csr.rowptr.data_ptr(),
                                      csr.col.data_ptr(), csr.w.data_ptr(), L, Wp, bp, widths,
                                      Hp, open_.data_ptr(), s) == 0
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        lib.lgnn_gcn_stack_fwd(b.x.data_ptr(), M, 128, 1, csr.rowptr.data_ptr(),
                               csr.col.data_ptr(), csr.w.data_ptr(), L, Wp, bp, widths, Hp,
                               open_.data_ptr(), s)
    e1.record()
    torch.cuda.synchronize()
    print(f"stamped build: {e0.elapsed_time(e1) / 10 * 1e3:.1f} us per launch (shares only)")
    buf = (ctypes.c_ulonglong * (1024 * 64))()
    assert lib.lgnn_debug_stamps(buf) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 64)[:512].astype(np.int64)
    n = int((a[0] > 0).sum())
    d = np.diff(a[:, :n], axis=1)
    names = ["start->tile ready", "l0 lin MFMA+sync", "l0 epi", "l0 sync", "l0 store",
             "l1 lin MFMA+sync", "l1 P write+agg MFMA", "l1 epi", "l1 sync", "l1 store",
             "l2 lin MFMA+sync", "l2 P write+agg MFMA", "l2 epi", "l2 sync", "l2 store",
             "tile end sync->next ready"]
    # co-residence: workgroups on one CU (HW_ID cu/sh/se fields + XCC_ID), their phase overlap
    full = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 64)[:512]
    hwid, xcc = full[:, 62].astype(np.int64), full[:, 63].astype(np.int64)
    cu_key = (xcc & 0xF) * 4096 + ((hwid >> 8) & 0xF) + 16 * ((hwid >> 12) & 1) + 32 * ((hwid >> 13) & 7)
    groups = {}
    for i, k in enumerate(cu_key):
        groups.setdefault(int(k), []).append(i)
    sizes = np.bincount([len(v) for v in groups.values()])
    print("workgroups per CU histogram:", dict(enumerate(sizes.tolist())))
    lin = [1, 3, 6]  # lin MFMA phase indices within a tile cycle (diff index into d)
    ov, tot_lin = 0.0, 0.0
    for v in groups.values():
        if len(v) != 2:
            continue
        ivs = []
        for wg in v:
            st = a[wg, :n]
            ph = []
            for i in range(n - 1):
                c = 0 if i == 0 else 1 + (i - 1) % 15
                if c in (1, 5, 10):
                    ph.append((st[i], st[i + 1]))
            ivs.append(ph)
        for (s0, e0) in ivs[0]:
            tot_lin += e0 - s0
            for (s1, e1) in ivs[1]:
                ov += max(0, min(e0, e1) - max(s0, s1))
    if tot_lin:
        print(f"pairs: lin-MFMA time of WG A overlapped by WG B's lin-MFMA: {ov / tot_lin:.2f}")
        print("first pairs (blockIdx):", [v for v in list(groups.values())[:6]])
    tot = (a[:, n - 1] - a[:, 0]).mean()
    print(f"stamps per block: {n}; mean kernel span {tot:.0f} cycles")
    for i in range(min(n - 1, 40)):
        nm = names[0] if i == 0 else names[1 + (i - 1) % 15]
        print(f"{i:2d} {nm:22s} mean {d[:, i].mean():9.0f}  p90 {np.percentile(d[:, i], 90):9.0f}")


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
