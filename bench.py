"""Benchmark: graphs/s of one training step of the lesion-graph GNN (BASELINE.json `metric`).

Workload (BASELINE.json configs[1], "C2"): 2-layer GCN (in_proj -> 2 x GCNConv+ELU -> mean pool
-> out_proj), hidden 128, d_in 128, 5 classes, synthetic k-NN lesion graphs N=64, k=8, 1024
graphs per GPU, fp32. One step = forward (incl. the per-forward graph build from edge_index) +
cross-entropy + backward + (N>1: RCCL all-reduce of the flat gradient) + Adam step, inputs
resident in HBM. Weak scaling: every rank processes its own 1024-graph shard.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]; N>1 under torch.distributed.run.
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: 8.0 TB/s spec
MFMA_F32_PEAK_TF = 157.3  # MI355X_MICROARCH.md: fp32 MFMA (= vector) peak

# algorithmic bytes per graph for the whole fwd+bwd step:
# B_graph = s*N*(2*d_in + h*(6L + 4 + 4*M*L)) + 2*L*(4E + 4(N+1)); GCN: M = 0
def bytes_per_graph(n=64, k=8, d_in=128, h=128, L=2, s=4, m=0):
    e = n * k
    return s * n * (2 * d_in + h * (6 * L + 4 + 4 * m * L)) + 2 * L * (4 * e + 4 * (n + 1))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--graphs-per-gpu", type=int, default=1024)
    ap.add_argument("--nodes", type=int, default=64)
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--hidden", type=int, default=128)
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="bounded CPU-baseline sample (rank 0, N=1 only); 0 disables")
    ap.add_argument("--no-kernel-timing", action="store_true")
    return ap.parse_args()


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, torch.device("cuda", local)


def time_dominant_kernel(model, b, dev, reps=20):
    """Average duration of the dominant kernel — the fused GCN conv backward exactly as the step
    launches it (transposed aggregation of dS + ELU' prologue, dW = dZ^T S and dX = dZ W fp32
    MFMA GEMMs, S streamed from the forward) — with HIP events on the stream it runs on."""
    from lesion_gnn_amd import _lib, ops
    from lesion_gnn_amd.graph import Graph

    g = Graph(b.edge_index, b.num_nodes, b.batch, b.num_graphs)
    csr = g.csr("gcn")
    with torch.no_grad():
        h0 = ops.linear_fwd(b.x, model.in_proj.weight, model.in_proj.bias, _lib.LGNN_ACT_NONE)
        c0 = model.convs[0]
        h1, s1 = ops.linear_fwd(h0, c0.lin.weight, c0.bias, _lib.LGNN_ACT_ELU, csr, save_s=True)
    M, K = s1.shape
    W = c0.lin.weight.detach().contiguous()
    N = W.size(0)
    dS = torch.randn(M, N, device=dev)
    P = ops.num_partials(M, N, K, False)
    dWp = torch.empty(P * N * K, device=dev)
    dbp = torch.empty(P * N, device=dev)
    dX = torch.empty(M, K, device=dev)
    s = torch.cuda.current_stream(dev)

    def launch():
        _lib.call("lgnn_node_linear_bwd", _lib.LGNN_GRAD_TRANSPOSE, dS.data_ptr(), None, None, 1,
                  csr.tptr.data_ptr(), csr.tidx.data_ptr(), csr.tw.data_ptr(), 0.0,
                  h1.data_ptr(), _lib.LGNN_ACT_ELU, s1.data_ptr(), M, K, None, None, None, 0.0,
                  W.data_ptr(), N, dX.data_ptr(), dWp.data_ptr(), dbp.data_ptr(), P,
                  s.cuda_stream)

    for _ in range(3):
        launch()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    # park the stream on a spin kernel so every timed launch is queued before the GPU reaches
    # the first event: the events then bracket back-to-back kernels, not host launch latency
    torch.cuda._sleep(10_000_000)
    e0.record(s)
    for _ in range(reps):
        launch()
    e1.record(s)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    flops = 4.0 * M * N * K  # dW = dZ^T S (2MNK) + dX = dZ W (2MNK)
    return {"kernel": "lgnn_tile::k_bwd<GRAD_TRANSPOSE,ELU,DX> (GCN conv backward)",
            "ms": ms, "flops": flops, "trace_name": "void lgnn_tile::k_bwd<2, 1, true>"}


def pmc_traffic(trace_name: str):
    """HBM bytes per launch of `trace_name` from the committed rocprofv3 PMC passes
    (profiles/traffic.json, written by tools/summarize_prof.py from separate FETCH_SIZE and
    WRITE_SIZE passes of this same bench command: (2*FETCH_SIZE + WRITE_SIZE) * 1024)."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(path):
        return None, None
    for k, v in json.load(open(path)).items():
        if k.startswith(trace_name):
            return v["bytes_per_launch"], v["source"]
    return None, None


def cpu_baseline(args, seconds):
    """Oracle (plain-torch CPU restatement of the PyG path) on the host cores: same model, same
    step (fwd + CE + bwd + Adam), bounded sample of the same workload."""
    import oracle.pyg_ref as ref
    from lesion_gnn_amd import synth

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    B = args.graphs_per_gpu
    b = synth.make_batch(B, n=args.nodes, k=args.k, d_in=128, seed=11)
    torch.manual_seed(0)
    m = ref.GCN(128, [args.hidden] * (args.layers + 1), 5, 0.0)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=2e-6)

    def step():
        opt.zero_grad(set_to_none=True)
        loss = torch.nn.functional.cross_entropy(m(b.x, b.edge_index, b.batch, B), b.y)
        loss.backward()
        opt.step()

    step()
    times = []
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end or len(times) < 3:
        t0 = time.perf_counter()
        step()
        times.append(time.perf_counter() - t0)
    med = statistics.median(times)
    return {"value": round(B / med, 2), "unit": "graphs/s", "cores": threads, "kind": "port",
            "sample": f"{len(times)} steps x {B} graphs (N={args.nodes}, k={args.k}), median "
                      f"{med * 1e3:.1f} ms/step, torch CPU fp32 with {threads} threads"}


def main():
    args = parse()
    world, rank, dev = setup_dist(args)
    from lesion_gnn_amd import dist as ldist
    from lesion_gnn_amd import synth
    from lesion_gnn_amd.models.gcn import GCN

    B = args.graphs_per_gpu
    b = synth.make_batch(B, n=args.nodes, k=args.k, d_in=128, seed=100 + rank).to(dev)
    torch.manual_seed(1234)
    model = GCN(128, [args.hidden] * (args.layers + 1), 5, dropout=0.0).to(dev)
    if world > 1:
        ldist.broadcast_params(model)
    params = list(model.parameters())
    opt = torch.optim.Adam(params, lr=1e-3, weight_decay=2e-6)

    def step():
        opt.zero_grad(set_to_none=True)
        logits = model(b.x, b.edge_index, b.batch, B)
        loss = torch.nn.functional.cross_entropy(logits, b.y)
        loss.backward()
        if world > 1:  # one flat RCCL all-reduce; equal shards -> weights 1/world
            ldist.allreduce_grads(params, B, B * world)
        opt.step()

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    ms_per_step = elapsed / args.steps * 1e3
    value = B * world * args.steps / elapsed

    out = {
        "metric": "graphs/sec (fwd+bwd) on batched k-NN lesion graphs at 1/2/4/8 MI355X",
        "value": round(value, 1), "unit": "graphs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic k-NN lesion graphs (pos~U[0,1)^2, x~N(0,1)), random-init weights",
        "config": {"workload": "C2: 2-layer GCN fwd+CE+bwd+Adam, graph build per forward",
                   "model": "GCN(128,[128,128,128],5,dropout=0,pool=mean)",
                   "graphs_per_gpu": B, "global_batch": B * world, "nodes_per_graph": args.nodes,
                   "k": args.k, "d": 128, "parallelism": f"dp{world}"},
    }
    bpg = bytes_per_graph(args.nodes, args.k, 128, args.hidden, args.layers)
    out["step_hbm_roofline"] = {
        "bytes_per_graph": bpg, "achieved_GBps_per_gpu": round(value / world * bpg / 1e9, 1),
        "frac_of_8TBps": round(value / world * bpg / (HBM_PEAK_GBS * 1e9), 4)}
    if rank == 0 and not args.no_kernel_timing:
        kt = time_dominant_kernel(model, b, dev)
        achieved = kt["flops"] / (kt["ms"] * 1e-3) / 1e12
        traffic, tsrc = pmc_traffic(kt["trace_name"])
        out["roofline"] = {"bound": "mfma", "achieved": round(achieved, 2),
                           "peak": MFMA_F32_PEAK_TF, "unit": "TFLOP/s",
                           "frac": round(achieved / MFMA_F32_PEAK_TF, 4),
                           "traffic": round(traffic) if traffic else None,
                           "traffic_source": tsrc,
                           "kernel": kt["kernel"], "avg_launch_ms": round(kt["ms"], 5),
                           "flops_per_launch": kt["flops"]}
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        out["cpu_baseline"] = cpu_baseline(args, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
