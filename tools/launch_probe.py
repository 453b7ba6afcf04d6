"""What one extra kernel costs inside a replayed HIP graph: graphs of K tiny kernels (an in-place
add on a 1-element tensor, and on a 256-workgroup tensor) replayed back to back; the per-kernel
cost is the slope of replay time over K.
Usage (GPU box): python tools/launch_probe.py
"""
import time

import torch


def per_replay_ms(t, K, reps=300):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(K):
            t.add_(1.0)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(K):
            t.add_(1.0)
    for _ in range(20):
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
    for name, n in (("1 workgroup", 1), ("256 workgroups", 256 * 256), ("1024 workgroups",
                                                                         1024 * 256)):
        t = torch.zeros(n, device=dev)
        rows = []
        for K in (1, 2, 4, 8, 16, 32):
            rows.append((K, per_replay_ms(t, K)))
        slope = (rows[-1][1] - rows[2][1]) / (rows[-1][0] - rows[2][0])
        print(f"{name}: " + ", ".join(f"K={k}: {ms * 1e3:.1f} us" for k, ms in rows) +
              f" -> {slope * 1e3:.2f} us per extra kernel", flush=True)
    # host side: time to enqueue one replay of a 13-kernel graph
    t = torch.zeros(256 * 256, device=dev)
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        t.add_(1.0)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        for _ in range(13):
            t.add_(1.0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        g.replay()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"host enqueue of a 13-kernel graph replay: {(t1 - t0) / 200 * 1e6:.1f} us", flush=True)


if __name__ == "__main__":
    main()
