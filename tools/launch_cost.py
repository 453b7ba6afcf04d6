"""Per-launch cost of verdict-reading no-op kernels inside a replayed HIP graph (the graph build's
general-path launches on target-sorted input). Graph = [writer, K x variant]; the per-kernel
cost is the slope of replay time over K. Usage (GPU box): python tools/launch_cost.py
(builds tools/probe/liblaunch_cost.so first: hipcc --offload-arch=gfx950 -O3 -shared -fPIC)."""
import ctypes
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "probe", "liblaunch_cost.so"))
lib.probe_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_int, ctypes.c_void_p]


def replay_ms(variant, K, grid, flag, out, nwords, reps=400):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())

    def body():
        st = torch.cuda.current_stream().cuda_stream
        lib.probe_launch(9, 1, flag.data_ptr(), 0, 1, st)
        for _ in range(K):
            assert lib.probe_launch(variant, grid, flag.data_ptr(), out.data_ptr(), nwords,
                                    st) == 0
    with torch.cuda.stream(s):
        body()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    for _ in range(30):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda", 0)
    flag = torch.zeros(1024 + 64, dtype=torch.int32, device=dev)
    out = torch.zeros(1024 * 256 * 2, dtype=torch.int32, device=dev)
    names = {0: "empty", 1: "flag via kernarg", 2: "OR of 1024 words", 3: "flag + 60 KB LDS",
             4: "flag via device global"}
    for grid in (256, 512):
        for v, name in names.items():
            rows = [(K, replay_ms(v, K, grid, flag, out, 1024)) for K in (2, 4, 8, 16)]
            slope = (rows[-1][1] - rows[0][1]) / (rows[-1][0] - rows[0][0])
            print(f"grid {grid:4d} {name:24s}: " +
                  ", ".join(f"K={k}: {ms * 1e3:.1f}" for k, ms in rows) +
                  f" us -> {slope * 1e3:.2f} us per launch", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
