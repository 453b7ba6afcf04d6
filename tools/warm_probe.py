"""Per-step timing of the bench step from a cold start (where does a short run lose time?).

Builds the same step as bench.py (workload, plan, graph capture), then replays it STEPS times
with a HIP event before every replay and one after the last: prints the GPU time of each of the
first 40 steps, window means after that, and the host enqueue time per replay. A second pass
after a 2 s idle shows whether the GPU clocks down between runs.
Usage (GPU box): python tools/warm_probe.py [--workload c2] [--steps 400]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def run_pass(step, n, dev, label):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(n):
        ev[i].record()
        step()
    ev[n].record()
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize(dev)
    t_all = time.perf_counter() - t0
    ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(n)]
    print(f"[{label}] host enqueue {t_host / n * 1e3:.4f} ms/step, wall {t_all / n * 1e3:.4f} "
          f"ms/step over {n} steps")
    print(f"[{label}] first 40:", " ".join(f"{x:.4f}" for x in ms[:40]))
    for a in (0, 5, 25, 50, 100, 200, 300):
        for w in (20, 100):
            if a + w <= n:
                seg = ms[a:a + w]
                print(f"[{label}] steps {a}..{a + w}: mean {sum(seg) / w:.4f} ms")
    return ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--steps", type=int, default=400)
    args = ap.parse_args()
    wl = bench.WORKLOADS[args.workload]
    dev = torch.device("cuda", 0)
    B = 1024
    b = bench.make_batch(wl, B, seed=100).to(dev)
    model = bench.build_model(wl).to(dev)
    run = torch.compile(model, dynamic=True) if wl.get("compile") else model
    from lesion_gnn_amd import optim as lgnn_optim
    opt = lgnn_optim.Adam(list(model.parameters()), lr=1e-3, weight_decay=2e-6)
    one = torch.ones((), device=dev)

    def fwd_bwd():
        bench.loss_fn(wl, run(b.x, b.edge_index, b.batch, B), b.y).backward(one)

    step = bench.make_step(bench.step_plan(1, True, False), fwd_bwd, None, opt, dev)
    run_pass(step, args.steps, dev, "cold")
    time.sleep(2.0)
    run_pass(step, args.steps, dev, "after 2 s idle")
    run_pass(step, args.steps, dev, "back to back")


if __name__ == "__main__":
    main()
