"""Where do the device-to-device copies of a bench step come from? Runs a few eager (or, with
the workload's compile flag, compiled) steps of one workload under torch.profiler and prints
every aten::copy_ / clone / contiguous-style op that reached the GPU, with its Python stack.
Usage (GPU box): python tools/copy_probe.py <workload> [steps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    name = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    wl = bench.WORKLOADS[name]
    dev = torch.device("cuda", 0)
    b = bench.make_batch(wl, 1024, seed=100).to(dev)
    model = bench.build_model(wl).to(dev)
    run = torch.compile(model, dynamic=True) if wl.get("compile") else model
    from lesion_gnn_amd import optim as lgnn_optim
    opt = lgnn_optim.Adam(list(model.parameters()), lr=1e-3, weight_decay=2e-6)

    def step():
        opt.zero_grad(set_to_none=True)
        bench.loss_fn(wl, run(b.x, b.edge_index, b.batch, 1024), b.y).backward()
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize(dev)
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, with_stack=True) as prof:
        for _ in range(steps):
            step()
        torch.cuda.synchronize(dev)
    seen = {}
    for ev in prof.events():
        if ev.name in ("aten::copy_", "aten::clone", "aten::_to_copy", "aten::contiguous",
                       "aten::index_put_", "aten::cat"):
            stack = " <- ".join(s for s in (ev.stack or [])[:6])
            key = (ev.name, stack)
            seen[key] = seen.get(key, 0) + 1
    for (n, st), c in sorted(seen.items(), key=lambda kv: -kv[1]):
        print(f"{c / steps:5.1f}/step {n}: {st}")
    names = {}
    for ev in prof.events():
        if ev.device_type == torch.autograd.DeviceType.CUDA and "opy" in ev.name:
            names[ev.name] = names.get(ev.name, 0) + 1
    print({k: v / steps for k, v in names.items()})
    return 0


if __name__ == "__main__":
    sys.exit(main())
