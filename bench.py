"""Benchmark: graphs/s of one training step of the lesion-graph GNN (BASELINE.json `metric`).

Default workload (BASELINE.json configs[1], "C2"): 2-layer GCN (in_proj -> 2 x GCNConv+ELU ->
mean pool -> out_proj), hidden 128, d_in 128, 5 classes, synthetic k-NN lesion graphs N=64,
k=8, 1024 graphs per GPU, fp32. One step = forward (incl. the per-forward graph build from
edge_index) + cross-entropy + backward + (N>1: RCCL all-reduce of the flat gradient) + Adam
step, inputs resident in HBM. Weak scaling: every rank processes its own 1024-graph shard.

Other workloads (--workload): c3 (3-layer GAT, 4 heads, d_in 1025, log-normal N, k=6, MSE;
computed in fp32), c4 (GIN + global_add_pool, SyncBN over the ranks), c5k4 / c5k16 (GCN on
power-law N in [16, 512], k = 4 / 16).

Step launch (--graph 1, default): the forward+backward and the optimizer step are each captured
once in a HIP graph and replayed — every kernel runs every step, only host launch overhead is
removed; with N>1 the RCCL gradient all-reduce runs eagerly between the two graphs.
--graph 0 runs everything eagerly.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2]; N>1 under
torch.distributed.run. Prints ONE JSON line on rank 0.
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

METRIC = "graphs/sec (fwd+bwd) on batched k-NN lesion graphs at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: 8.0 TB/s spec
MFMA_F32_PEAK_TF = 157.3  # MI355X_MICROARCH.md: fp32 MFMA (= vector) peak
# split-3 kernels compute fp32-accurate products as 6 bf16 MFMA products: dense bf16 peak
# (16 x the fp32 rate, MI355X_MICROARCH.md) / 6, priced in useful fp32 FLOP
MFMA_S3_PEAK_TF = round(16 * MFMA_F32_PEAK_TF / 6, 1)

WORKLOADS = {
    "c2": dict(model="gcn", sizes="fixed", n=64, k=8, d_in=128, hidden=[128, 128, 128],
               classes=5, loss="CE", pool="mean",
               desc="C2: 2-layer GCN fwd+CE+bwd+Adam, graph build per forward"),
    "c3": dict(model="gat", sizes="lognormal", n=64, k=6, d_in=1025, hidden=[128] * 4, heads=4,
               classes=5, loss="MSE", pool="mean", last_channel_class=True, precision="bf16",
               desc="C3: 3-layer GAT (4 heads), d_in 1025, log-normal N, k=6, MSE, bf16 GEMMs"),
    "c3f32": dict(model="gat", sizes="lognormal", n=64, k=6, d_in=1025, hidden=[128] * 4,
                  heads=4, classes=5, loss="MSE", pool="mean", last_channel_class=True,
                  desc="C3 in fp32: 3-layer GAT (4 heads), d_in 1025, log-normal N, k=6, MSE"),
    "refcfg": dict(model="gat", sizes="lognormal", n=64, k=6, d_in=1025, hidden=[128] * 4,
                   heads=2, classes=5, loss="MSE", pool="mean", last_channel_class=True,
                   dropout=0.35, compile=True,
                   desc="reference experiment (configs/config.py:47-65): GAT [128]*4, heads 2, "
                        "dropout 0.35, torch.compile(dynamic=True), d_in 1025, KNN k=6, MSE, "
                        "fp32, log-normal N"),
    "c4": dict(model="gin", sizes="fixed", n=64, k=8, d_in=128, hidden=[128, 128, 128],
               classes=5, loss="CE", pool="add",
               desc="C4: GIN + global_add_pool, SyncBN across ranks, fwd+CE+bwd+Adam"),
    "c5k4": dict(model="gcn", sizes="powerlaw", n=64, k=4, d_in=128, hidden=[128, 128, 128],
                 classes=5, loss="CE", pool="mean",
                 desc="C5: GCN, power-law N in [16,512], k=4"),
    "c5k16": dict(model="gcn", sizes="powerlaw", n=64, k=16, d_in=128, hidden=[128, 128, 128],
                  classes=5, loss="CE", pool="mean",
                  desc="C5: GCN, power-law N in [16,512], k=16"),
    # the reference sweep's space off the fused fast paths (scripts/sweep.py:126-141: widths
    # {32..512}, 1-8 layers, heads {1, 2, 4, 8}): timed as lines of their own, not the metric
    "sweep_gcn3": dict(model="gcn", sizes="fixed", n=64, k=8, d_in=128, hidden=[128] * 4,
                       classes=5, loss="CE", pool="mean",
                       desc="sweep: GCN with 3 convs (layer-major split-3 backward)"),
    "sweep_gat256h8": dict(model="gat", sizes="lognormal", n=64, k=6, d_in=1025,
                           hidden=[256] * 4, heads=8, classes=5, loss="MSE", pool="mean",
                           last_channel_class=True, dropout=0.35,
                           desc="sweep: GAT [256]*4, heads 8, dropout 0.35, d_in 1025, fp32"),
    "sweep_gat512h4": dict(model="gat", sizes="lognormal", n=64, k=6, d_in=1025,
                           hidden=[512] * 3, heads=4, classes=5, loss="MSE", pool="mean",
                           last_channel_class=True, dropout=0.35,
                           desc="sweep: GAT [512]*3, heads 4, dropout 0.35, d_in 1025, fp32"),
    "sweep_gat128h8": dict(model="gat", sizes="lognormal", n=64, k=6, d_in=1025,
                           hidden=[128] * 4, heads=8, classes=5, loss="MSE", pool="mean",
                           last_channel_class=True, dropout=0.35,
                           desc="sweep: GAT [128]*4, heads 8 (16 channels per head), dropout 0.35, "
                                "d_in 1025, fp32"),
    "sweep_gcn_k16": dict(model="gcn", sizes="fixed", n=64, k=16, d_in=128, hidden=[128] * 3,
                          classes=5, loss="CE", pool="mean",
                          desc="sweep: 2-layer GCN, N = 64, k = 16 (closed 64-row tiles of 1024 "
                               "CSR entries)"),
    "sweep_gcn_k32": dict(model="gcn", sizes="fixed", n=64, k=32, d_in=128, hidden=[128] * 3,
                          classes=5, loss="CE", pool="mean",
                          desc="sweep: 2-layer GCN, N = 64, k = 32 (the sweep's largest k, "
                               "scripts/sweep.py:110)"),
    "sweep_gin512": dict(model="gin", sizes="fixed", n=64, k=8, d_in=128, hidden=[512] * 4,
                         classes=5, loss="CE", pool="add",
                         desc="sweep: GIN [512]*4 + global_add_pool (generic-shape kernels)"),
}


def step_bytes(b, wl) -> float:
    """Algorithmic HBM bytes of one fwd+bwd step over batch b, summed per graph:
    B_graph = s*N*(2*d_in + h*(6L + 4 + 4*M*L)) + 2*L*(4E + 4(N+1)) [+ GAT: 2*L*E*H*4 for alpha]
    with s = 4 (fp32), M = 1 for GIN (MLP hidden), 0 otherwise; E = the edges of the batch's
    k-NN graph (self loops included, as KNNGraph(loop=True) builds them)."""
    h = wl["hidden"][1]
    L = len(wl["hidden"]) - 1
    m = 1 if wl["model"] == "gin" else 0
    n = (b.ptr[1:] - b.ptr[:-1]).double().cpu()
    e = torch.bincount(b.batch.cpu()[b.edge_index[1].cpu()], minlength=b.num_graphs).double()
    tot = 4 * n * (2 * wl["d_in"] + h * (6 * L + 4 + 4 * m * L)) + 2 * L * (4 * e + 4 * (n + 1))
    if wl["model"] == "gat":
        tot = tot + 2 * L * e * wl["heads"] * 4
    return float(tot.sum())


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c2")
    ap.add_argument("--graphs-per-gpu", type=int, default=1024)
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="bounded CPU-baseline sample (rank 0, N=1 only); 0 disables")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--opt", choices=["lgnn", "fused", "foreach"], default="lgnn",
                    help="Adam implementation, inside the timed step either way: lgnn = one "
                         "HIP launch (lesion_gnn_amd.optim.Adam); fused / foreach = torch's")
    ap.add_argument("--graph", type=int, default=1,
                    help="1: replay the captured fwd+bwd and optimizer HIP graphs; 0: eager")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="process-group backend for N > 1 (nccl = RCCL over xGMI on ROCm)")
    ap.add_argument("--force-dist", action="store_true",
                    help="run the N > 1 step plan (process group, gradient bucket + all-reduce, "
                         "SyncBN for GIN) even at --gpus 1, over a one-rank group: times the plan "
                         "a multi-GPU run executes on one GPU")
    ap.add_argument("--rccl-eager", action="store_true",
                    help="N > 1: run the collectives eagerly between captured graph segments "
                         "instead of capturing them into the step's graph")
    ap.add_argument("--sync-bn", choices=["auto", "on", "off"], default="auto",
                    help="GIN with a process group: auto/on = SyncBN (full-batch statistics, "
                         "all-reduces inside forward and backward), off = per-replica statistics "
                         "(torch DDP's default)")
    ap.add_argument("--entries", type=int, default=1,
                    help="1: per-entry HIP-event profile of an eager step (rank 0, after the "
                         "timed region)")
    ap.add_argument("--path-option", action="append", default=[], metavar="NAME=VALUE",
                    help="A/B only: set an lgnn_set_option path option before the run "
                         "(gat_pipe, gat_bpc, graph_sorted; include/lgnn.h LGNN_OPT_*)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher/rank plumbing only: set up the process group, all-reduce a "
                         "gradient-sized buffer once, print the JSON line with value null; "
                         "touches no GPU (CPU tests drive this over gloo)")
    return ap.parse_args()


def launch_ranks(args) -> int:
    """`--gpus N` with N > 1 and no torch.distributed environment: start N ranks on this node
    as ONE child `torch.distributed.run` process (rendezvous on 127.0.0.1, a free port) and
    return its exit code. Runs before anything touches the GPU, and never replaces this
    process (no exec)."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get(
        "HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.run(cmd, env=env).returncode


def _free_port() -> int:
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def setup_dist(args):
    """One process per GPU (LOCAL_RANK = device). Refuses a rank count that differs from
    --gpus, so a run cannot report fewer GPUs than it was asked for."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.dry_run:
        dev = torch.device("cpu")
        if world > 1:
            dist.init_process_group(args.backend)
    else:
        dev = torch.device("cuda", local)
        if world > 1 or args.force_dist:
            torch.cuda.set_device(local)
            kw = {"device_id": dev} if args.backend == "nccl" else {}
            if world == 1:  # --force-dist: a one-rank group on this process
                os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
                os.environ.setdefault("MASTER_PORT", str(_free_port()))
                kw.update(rank=0, world_size=1)
            dist.init_process_group(args.backend, **kw)
    if world > 1 and dist.get_world_size() != args.gpus:
        raise SystemExit(f"bench.py: process group has {dist.get_world_size()} ranks, "
                         f"--gpus {args.gpus}")
    return world, rank, dev


def make_batch(wl, B, seed):
    from lesion_gnn_amd import synth

    return synth.make_batch(B, n=wl["n"], k=wl["k"], d_in=wl["d_in"], num_classes=wl["classes"],
                            seed=seed, sizes=wl["sizes"],
                            last_channel_class=wl.get("last_channel_class", False))


def build_model(wl, oracle=False):
    torch.manual_seed(1234)
    if oracle:
        import oracle.pyg_ref as ref

        mods = {"gcn": ref.GCN, "gin": ref.GIN, "gat": ref.GAT}
    else:
        from lesion_gnn_amd import models

        mods = {"gcn": models.GCN, "gin": models.GIN, "gat": models.GAT}
    out = 1 if wl["loss"] == "MSE" else wl["classes"]
    p = wl.get("dropout", 0.0)
    if wl["model"] == "gat":
        return mods["gat"](wl["d_in"], wl["hidden"], out, heads=wl["heads"], dropout=p,
                           precision=wl.get("precision", "fp32"))
    return mods[wl["model"]](wl["d_in"], wl["hidden"], out, p, pool=wl["pool"])


def loss_fn(wl, logits, y, oracle=False):
    if wl["loss"] == "CE":
        if oracle:
            return torch.nn.functional.cross_entropy(logits, y)
        from lesion_gnn_amd import ops  # HIP criterion (reference nn.CrossEntropyLoss)

        return ops.cross_entropy(logits, y)
    # reference regression head: clamp(logits.squeeze(1), 0, C-1) then MSE (gat.py:94-95)
    if oracle:
        return torch.nn.functional.mse_loss(logits.squeeze(1).clamp(0, wl["classes"] - 1),
                                            y.float())
    from lesion_gnn_amd import ops  # HIP clamp + criterion (one launch each way)

    return ops.regression_loss(logits, y, 0.0, float(wl["classes"] - 1), "MSE")[1]


def _time_launches(launch, dev, reps=20):
    """Average duration of `launch` with HIP events on the launch stream; the launches are
    queued behind a spin kernel so the events bracket back-to-back kernels, not host latency."""
    s = torch.cuda.current_stream(dev)
    for _ in range(3):
        launch()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    torch.cuda._sleep(10_000_000)
    e0.record(s)
    for _ in range(reps):
        launch()
    e1.record(s)
    torch.cuda.synchronize(dev)
    return e0.elapsed_time(e1) / reps


def time_dominant_kernels(model, b, dev):
    """The two largest kernels of the C2 step, each launched alone with the step's arguments:
    * lgnn_s3::k_s3_fbwd<L + 1, true, false> (`lgnn_gcn_stack_bwd_s3f_ce`, stack3_bwd.hip) — the fused
      split-3 backward of in_proj + L GCN convs with the CE logits gradient and out_proj's dP
      formed in its prologue; useful FLOP per launch 2*M*(d_in*h + L*h*h) (dW) + 2*M*L*h*h
      (dH = G W) + 2*nnz*h*L (the transposed aggregation);
    * lgnn_s3::k_s3_fwd<true> (`lgnn_gcn_stack_fwd_s3`, stack3.hip) — the fused split-3 forward,
      2*M*(d_in*h + L*h*h) + 2*nnz*h*L.
    The tile aggregation runs as a dense 64 x 64 MFMA product; its zeros are not counted. (The fp32
    kernels lgnn_tile::k_stack_fwd / k_stack_bwd are timed instead when MFMA_MODE / BWD_MODE
    select them.)"""
    import ctypes

    from lesion_gnn_amd import _lib, ops
    from lesion_gnn_amd.graph import Graph

    g = Graph(b.edge_index, b.num_nodes, b.batch, b.num_graphs)
    csr = g.csr("gcn")
    open_ = g.tile_open("gcn")
    Ws = [model.in_proj.weight.detach()] + [c.lin.weight.detach() for c in model.convs]
    bs = [model.in_proj.bias.detach()] + [c.bias.detach() for c in model.convs]
    with torch.no_grad():
        hs, _ = ops.stack_fwd(b.x, g, Ws, bs)
    M, h = hs[1].shape
    d_in = b.x.size(1)
    L = len(Ws) - 1
    nnz = int(csr.rowptr[-1].item())
    s = torch.cuda.current_stream(dev).cuda_stream
    arr = ctypes.c_void_p * (L + 1)
    Wp = arr(*[W.data_ptr() for W in Ws])
    bp = arr(*[x.data_ptr() for x in bs])
    Hp = arr(*[x.data_ptr() for x in hs])
    widths = [d_in] + [W.size(0) for W in Ws]
    lib = _lib.load()
    P = lib.lgnn_gcn_stack_bwd_partials(M)
    slabs = [torch.empty(P * (widths[l + 1] * widths[l] + widths[l + 1]), device=dev)
             for l in range(L + 1)]
    dWp = arr(*[t.data_ptr() for t in slabs])
    dbp = arr(*[t.data_ptr() + P * widths[l + 1] * widths[l] * 4 for l, t in enumerate(slabs)])
    dP = torch.randn(b.num_graphs, h, device=dev)
    agg = 2.0 * nnz * h * L
    lin = 2.0 * M * (d_in * h + L * h * h)
    out = []

    def bwd():
        _lib.call("lgnn_gcn_stack_bwd", dP.data_ptr(), g.batch.data_ptr(), g.gptr.data_ptr(), 1,
                  csr.rowptr.data_ptr(), csr.col.data_ptr(), csr.w.data_ptr(), b.x.data_ptr(), M,
                  L, Wp, Hp, (ctypes.c_int * (L + 2))(*widths), dWp, dbp, P, open_.data_ptr(), s)

    bwd_flops = lin + 2.0 * M * L * h * h + agg
    if ops.MFMA_MODE == "s3" and ops.BWD_MODE == "s3f" and L <= 2:
        # the step's backward: the fused split-3 kernel (stack3_bwd.hip), priced against the
        # split-3 peak like the forward
        _, planes_t = ops.weight_planes(Ws, d_in, transposed=True)
        # the Â^T planes the step's forward hands over (as the step: the backward loads them)
        adjt = torch.empty(ops.adjt_numel(M), dtype=torch.int16, device=dev) if ops.ADJT else None
        planes_f, _ = ops.weight_planes(Ws, d_in)
        _lib.call("lgnn_gcn_stack_fwd_s3", b.x.data_ptr(), M, d_in, 1, csr.rowptr.data_ptr(),
                  csr.col.data_ptr(), csr.w.data_ptr(), L, planes_f.data_ptr(), bp,
                  (ctypes.c_int * (L + 1))(*widths[1:]), Hp, open_.data_ptr(), _lib.ptr(adjt), s)

        # the step's launch: the CE entry (the model + criterion node, ops.gcn_stack_ce): the
        # logits gradient formed per graph in the prologue from the CE forward's values, then
        # dP = dlogits W_out as the dZ_L product — as ops.stack_bwd runs it in the step
        W_out = model.out_proj.weight.detach()
        C = W_out.size(0)
        z = torch.randn(b.num_graphs, C, device=dev)
        y = b.y.to(dev)
        # the readout's CE factors (lgnn_pool_head_ce_fwd): pm = softmax(z) - onehot(y), wt = 1
        pm = (torch.softmax(z, 1) - torch.nn.functional.one_hot(y.long(), C).float()).contiguous()
        wt = torch.ones(b.num_graphs, device=dev)
        ce_out = torch.full((2,), float(b.num_graphs), device=dev)
        gloss = torch.ones(1, device=dev)
        ce = _lib.CeSrc(pm.data_ptr(), wt.data_ptr(), ce_out.data_ptr() + 4, gloss.data_ptr())
        dS_ws = torch.empty(2 * M * 128, dtype=torch.float32, device=dev)
        Sp = (ctypes.c_void_p * L)(*[x.data_ptr() for x in hs[1:]])  # open tiles only (none)

        def bwd_s3f():
            _lib.call("lgnn_gcn_stack_bwd_s3f_ce", g.batch.data_ptr(),
                      g.gptr.data_ptr(), 1, b.num_graphs, csr.rowptr.data_ptr(),
                      csr.col.data_ptr(), csr.w.data_ptr(), csr.tptr.data_ptr(),
                      csr.tidx.data_ptr(), csr.tw.data_ptr(), b.x.data_ptr(), M, L,
                      planes_t.data_ptr(), Wp, Hp, Sp, (ctypes.c_int * (L + 2))(*widths), dWp,
                      dbp, P, dS_ws.data_ptr(), open_.data_ptr(), ctypes.byref(ce),
                      W_out.data_ptr(), C, _lib.ptr(adjt), s)

        out.append({"kernel": f"lgnn_s3::k_s3_fbwd<{L + 1}, {str(ops.ADJT).lower()}, false> "
                              "(fused GCN "
                              "backward, all layers, "
                              "split-3 bf16 MFMA)",
                    "ms": _time_launches(bwd_s3f, dev), "flops": bwd_flops,
                    "peak": MFMA_S3_PEAK_TF,
                    "trace_name": f"void lgnn_s3::k_s3_fbwd<{L + 1}, "
                                  f"{str(ops.ADJT).lower()}, false>"})
    else:
        out.append({"kernel": f"lgnn_tile::k_stack_bwd<{L + 1}> (fused GCN backward, all "
                              "layers)",
                    "ms": _time_launches(bwd, dev), "flops": bwd_flops,
                    "trace_name": f"void lgnn_tile::k_stack_bwd<{L + 1}>"})

    if ops.MFMA_MODE == "s3":
        planes, _ = ops.weight_planes(Ws, d_in)
        adjt_f = torch.empty(ops.adjt_numel(M), dtype=torch.int16, device=dev) \
            if ops.BWD_MODE == "s3f" and L <= 2 and ops.ADJT else None

        def fwd():  # as in the step: with the Â^T planes for the fused backward when it runs
            _lib.call("lgnn_gcn_stack_fwd_s3", b.x.data_ptr(), M, d_in, 1,
                      csr.rowptr.data_ptr(), csr.col.data_ptr(), csr.w.data_ptr(), L,
                      planes.data_ptr(), bp, (ctypes.c_int * (L + 1))(*widths[1:]), Hp,
                      open_.data_ptr(), _lib.ptr(adjt_f), s)

        out.append({"kernel": "lgnn_s3::k_s3_fwd<true> (fused GCN forward, all layers, "
                              "split-3 bf16 MFMA)",
                    "ms": _time_launches(fwd, dev), "flops": lin + agg, "peak": MFMA_S3_PEAK_TF,
                    "trace_name": "void lgnn_s3::k_s3_fwd<true>("})
        return out

    def fwd():
        _lib.call("lgnn_gcn_stack_fwd", b.x.data_ptr(), M, d_in, 1, csr.rowptr.data_ptr(),
                  csr.col.data_ptr(), csr.w.data_ptr(), L, Wp, bp,
                  (ctypes.c_int * (L + 1))(*widths[1:]), Hp, open_.data_ptr(), s)

    out.append({"kernel": "lgnn_tile::k_stack_fwd<true> (fused GCN forward, all layers)",
                "ms": _time_launches(fwd, dev), "flops": lin + agg,
                "trace_name": "void lgnn_tile::k_stack_fwd<true>"})
    return out


def time_gat_in_proj(model, b, dev, wl):
    """The GAT workloads' two largest launches, both on the in_proj nn.Linear(d_in, 128) (the
    reference's 1024 encoder channels + lesion class, gat.py:29), timed alone on the step's own
    node features: the forward GEMM Y = X W^T + b and the weight gradient dW = dY^T X (+ db),
    split-3 bf16 MFMA at fp32 accuracy (s3gemm.hip) in fp32 mode, the one-plane bf16 kernels
    (bflin.hip) in bf16 mode. Useful FLOP per launch 2 M d_in h; algorithmic HBM bytes per launch
    X once (M d_in 4) + Y (or dY) once (M h 4)."""
    from lesion_gnn_amd import _lib, ops

    x = b.x
    M, K = x.shape
    W = model.in_proj.weight.detach()
    bias = model.in_proj.bias.detach()
    N = W.size(0)
    dy = torch.randn(M, N, device=dev)
    flops = 2.0 * M * K * N
    nbytes = 4.0 * M * K + 4.0 * M * N
    lib = _lib.load()
    s = torch.cuda.current_stream(dev).cuda_stream
    out = []
    if wl.get("precision") == "bf16":
        Wb, _ = ops.bf16_weight_operands(W, False)
        Y = torch.empty(M, N, device=dev)
        S = lib.lgnn_bf16_wgrad_partials(M, K)
        part = torch.empty(S * N * K, device=dev)
        dyb = dy.to(torch.bfloat16)

        def fwd():
            _lib.call("lgnn_bf16_gemm", x.data_ptr(), 1, M, K, Wb.data_ptr(), bias.data_ptr(), N,
                      Y.data_ptr(), None, None, s)

        def wgrad():
            _lib.call("lgnn_bf16_wgrad", dyb.data_ptr(), N, x.data_ptr(), 1, M, K,
                      part.data_ptr(), S, s)
        names = ("void lgnn_bf::k_bf_gemm<true, false, 17", "void lgnn_bf::k_bf_wgrad<true")
        peak = 16 * MFMA_F32_PEAK_TF  # dense bf16: one plane product per product
        label = "bf16 MFMA (bflin.hip)"
    else:
        Wp = ops.dense_planes(W, False, False)
        Y = torch.empty(M, N, device=dev)
        S = lib.lgnn_s3_wgrad_partials(M, K, N)
        part = torch.empty(S * N * K, device=dev)
        dbp = torch.empty(S * N, device=dev)

        def fwd():
            _lib.call("lgnn_s3_gemm", x.data_ptr(), M, K, Wp.data_ptr(), N, 3, bias.data_ptr(),
                      Y.data_ptr(), None, s)

        def wgrad():
            _lib.call("lgnn_s3_wgrad", dy.data_ptr(), N, x.data_ptr(), M, K, 3, part.data_ptr(),
                      S, dbp.data_ptr(), s)
        # the forward kernel runs only at this shape; k_s3_wgrad2 also runs on the lins, so its
        # traffic entry is the in_proj-only PMC pass of tools/s3_micro.py --inproj
        names = ("void lgnn_s3g::k_s3_gemm<3, false, 17, false>",
                 "void lgnn_s3g::k_s3_wgrad2<3> [in_proj 42279 x 1025 -> 128]")
        peak = MFMA_S3_PEAK_TF
        label = "split-3 bf16 MFMA at fp32 accuracy (s3gemm.hip)"
    for what, fn, name in (("forward GEMM Y = X W^T + b", fwd, names[0]),
                           ("weight gradient dW = dY^T X (+ db)", wgrad, names[1])):
        out.append({"kernel": f"in_proj {what} [{M} x {K}] -> {N}, {label}",
                    "ms": _time_launches(fn, dev), "flops": flops, "bytes": nbytes,
                    "peak": peak, "trace_name": name})
    return out


class GraphStats:
    """Host-side sizes of the batch's CSR the algorithmic byte / FLOP models need: entries (nnz)
    of the graph kind the model builds, and the rows / entries that sit in open 64-row tiles
    (an edge leaves the tile or it holds > 1024 entries: the layer-wise kernels take those)."""

    def __init__(self, b, kind):
        from lesion_gnn_amd.graph import Graph

        g = Graph(b.edge_index, b.num_nodes, b.batch, b.num_graphs)
        csr = g.csr(kind)
        rp = csr.rowptr.cpu().long()
        self.M, self.B = b.num_nodes, b.num_graphs
        self.nnz = int(rp[-1])
        self.open_rows = self.open_nnz = 0
        if csr.tile_open is not None:
            T = (self.M + 63) // 64
            flags = csr.tile_open[:T].cpu()
            for t in torch.nonzero(flags).flatten().tolist():
                r0, r1 = 64 * t, min(64 * t + 64, self.M)
                self.open_rows += r1 - r0
                self.open_nnz += int(rp[r1] - rp[r0])

    def rows(self, tile_open, want_open):
        """(rows, entries) a *_tiles launch processes."""
        if tile_open is None:
            return self.M, self.nnz
        if want_open:
            return self.open_rows, self.open_nnz
        return self.M - self.open_rows, self.nnz - self.open_nnz


def _entry_model(name, a, gs):
    """Algorithmic (bytes, useful FLOP) of one C-ABI launch from its arguments (the positions of
    include/lgnn.h), fp32: every activation row the launch reads or writes counted once, the CSR
    entries it walks once (8 B: index + weight), a weight gradient once (N K 4, not the partial
    slabs); FLOP = the GEMMs + 2 nnz width per aggregation. None for entries without a model."""
    f4 = 4.0
    if name in ("lgnn_node_linear_fwd", "lgnn_node_linear_fwd_tiles", "lgnn_node_linear_fwd_bn"):
        M, K, rowptr, N, S = a[1], a[2], a[3], a[9], a[12]
        R, nz = gs.rows(a[13], a[14]) if name.endswith("_tiles") else (M, gs.nnz)
        by = f4 * R * (K + N) + (f4 * R * K if S else 0) + ((8.0 * nz + 4 * R) if rowptr else 0)
        if name.endswith("_bn"):  # BN_IN: the dropout mask and A1 = ELU(BN(Z1)) (+ mask)
            by += (f4 * R * K if a[16] else 0) + (f4 * R * K if a[17] else 0)
        return by, 2.0 * R * K * N + (2.0 * nz * K if rowptr else 0)
    if name in ("lgnn_node_linear_bwd", "lgnn_node_linear_bwd_tiles"):
        mode, H, M, K, rowptr, N, dX = a[0], a[9], a[12], a[13], a[14], a[19], a[20]
        R, nz = gs.rows(a[24], a[25]) if name.endswith("_tiles") else (M, gs.nnz)
        by = f4 * R * K + f4 * N * K  # X (or S) read once, dW written once
        fl = 2.0 * R * K * N
        if mode != 1:  # DIRECT / TRANSPOSE: the output gradient rows (POOL: [B, N], negligible)
            by += f4 * R * N
        if mode == 2:  # the transposed aggregation of dY
            by += 8.0 * nz + 4 * R
            fl += 2.0 * nz * N
        if H:
            by += f4 * R * N
        if rowptr:  # S recomputed from the forward CSR
            by += 8.0 * nz + 4 * R
            fl += 2.0 * nz * K
        if dX:
            by += f4 * R * K
            fl += 2.0 * R * K * N
        return by, fl
    if name in ("lgnn_node_linear_bwd_bn", "lgnn_node_linear_bwd_bn_pool",
                "lgnn_node_linear_bwd_bn_gather"):
        g = name.endswith("_gather")
        if g:  # dS, tptr, tidx, tw, tself, H, act, X, M, K, W, N, dX, ..., bn_Z, bn_mask, ...
            H, M, K, N, dX, Z, mask = a[5], a[8], a[9], a[11], a[12], a[16], a[17]
        else:  # bn_mode, dY, H, act, X, M, K, W, N, dX, ..., bn_Z, bn_mask, ...
            H, M, K, N, dX, Z, mask = a[2], a[5], a[6], a[8], a[9], a[13], a[14]
        by = f4 * M * K + f4 * N * K + (f4 * M * N if H else 0) + (f4 * M * K if dX else 0)
        by += (f4 * M * K if Z else 0) + (f4 * M * K if mask else 0)
        fl = 2.0 * M * K * N + (2.0 * M * K * N if dX else 0)
        if not name.endswith("_pool"):  # the output gradient rows (pool: [B, N])
            by += f4 * M * N
        if g:
            by += 8.0 * gs.nnz + 4 * M
            fl += 2.0 * gs.nnz * N
        return by, fl
    # split-3 dense GEMMs (s3gemm.hip: the wide GIN / GCN linears, the GAT lins / in_proj)
    if name in ("lgnn_s3_gemm", "lgnn_s3_gemm_act"):  # A, M, K, Wp, N, ...: Y = A W^T (+ b)
        M, K, N = a[1], a[2], a[4]
        return f4 * M * (K + N) + 6.0 * N * K, 2.0 * M * K * N
    if name == "lgnn_s3_wgrad":  # dY, N, X, M, K, ...: dW = dY^T X (the slab written once)
        N, M, K = a[1], a[3], a[4]
        return f4 * M * (K + N) + f4 * N * K, 2.0 * M * K * N
    if name == "lgnn_spmm":  # rowptr, col, w, self_scale, X, M, D, Y: Y = (s I + A) X
        M, D = a[5], a[6]
        return 2 * f4 * M * D + 8.0 * gs.nnz + 4 * M, 2.0 * (gs.nnz + M) * D
    if name in ("lgnn_gcn_stack_fwd_s3_all", "lgnn_gcn_stack_bwd_s3"):
        if name.endswith("_all"):  # X, M, d_in, has_in_proj, rowptr, col, w, L, planes, W, b, widths
            M, L, wd = a[1], a[7], list(a[11])
            wd = [a[2]] + wd  # widths of lgnn_gcn_stack_fwd_s3_all: the layers' outputs
        else:  # dP, batch, gptr, mean, B, rowptr, col, w, X, M, L, planes_t, H, widths
            M, L, wd = a[9], a[10], list(a[13])
        R, nz = gs.rows(1, 0) if gs.open_rows else (M, gs.nnz)
        conv = sum(2.0 * R * wd[l] * wd[l + 1] + 2.0 * nz * wd[l] for l in range(1, L + 1))
        if name.endswith("_all"):  # reads X, writes H_0..H_L, walks the CSR once per conv
            by = f4 * M * (wd[0] + sum(wd[1:L + 2])) + 8.0 * nz * L
            return by, 2.0 * R * wd[0] * wd[1] + conv
        # layer-major backward: H_{l-1} and dZ_l read, dZ_{l-1} written per conv, X and dZ_0 for
        # in_proj, H_L for the top ELU', the CSR once per conv
        by = f4 * M * (wd[L + 1] + sum(wd[l] + wd[l + 1] + wd[l] for l in range(1, L + 1))
                       + wd[0] + wd[1]) + 8.0 * nz * L
        return by, 2.0 * R * wd[0] * wd[1] + 2 * conv
    if name in ("lgnn_gcn_stack_bwd_s3f_ce", "lgnn_gcn_stack_bwd_s3f_all"):
        # fused split-3 backward (closed tiles; the open ones add their layer-wise bodies): per
        # conv dW_l and dH (2 M K N each) and G = Â^T dZ (2 nnz N); in_proj's dW in the kernel for
        # L <= 2, outside it (dZ_0 written, the lgnn_s3_wgrad entry) for L = 3. Reads H_0..H_L,
        # X (L <= 2), the forward's Â tiles (64 x 64 fp32 per 64 rows); dW written once
        i = 11 if name.endswith("_ce") else 12
        M, L, wd = a[i], a[i + 1], list(a[i + 6])
        conv = sum(4.0 * M * wd[l] * wd[l + 1] + 2.0 * gs.nnz * wd[l + 1] for l in range(1, L + 1))
        inproj = L <= 2
        by = f4 * M * (sum(wd[1:L + 2]) + (wd[0] if inproj else wd[1]) + 64) \
            + f4 * sum(wd[l] * wd[l + 1] for l in range(0 if inproj else 1, L + 1))
        return by, conv + (2.0 * M * wd[0] * wd[1] if inproj else 0.0)
    return None


# the MFMA roof of a modelled entry (useful fp32 FLOP): split-3 bf16 entries against dense bf16 / 6,
# the fp32-MFMA tile kernels against the fp32 peak
_S3_ENTRIES = ("lgnn_s3_gemm", "lgnn_s3_gemm_act", "lgnn_s3_wgrad", "lgnn_gcn_stack_fwd_s3_all",
               "lgnn_gcn_stack_bwd_s3", "lgnn_gcn_stack_bwd_s3f_ce", "lgnn_gcn_stack_bwd_s3f_all")


# kernel-name fragments of the modelled entries without a _entry_kernel mapping (PMC lookups)
_ENTRY_TRACE = {"lgnn_s3_gemm": "lgnn_s3::k_s3_gemm", "lgnn_s3_gemm_act": "lgnn_s3::k_s3_gemm",
                "lgnn_s3_wgrad": "lgnn_s3::k_s3_wgrad2", "lgnn_spmm": "::k_spmm",
                "lgnn_gcn_stack_fwd_s3_all": "lgnn_s3::k_s3_fwd",
                "lgnn_gcn_stack_bwd_s3": "lgnn_s3::k_s3_bwd",
                "lgnn_gcn_stack_bwd_s3f_ce": "lgnn_s3::k_s3_fbwd",
                "lgnn_gcn_stack_bwd_s3f_all": "lgnn_s3::k_s3_fbwd"}


def _entry_kernel(name, a):
    """The HIP kernel (rocprofv3 name prefix) a layer-wise launch runs, from its arguments: the
    tile.hip templates k_fwd<GATHER, ACT, BN> / k_bwd<GRAD_MODE, ACT, DX, BN>. Launches of one
    entry with different template arguments are aggregated separately. None: not mapped."""
    t = lambda v: "true" if v else "false"  # noqa: E731
    if name in ("lgnn_node_linear_fwd", "lgnn_node_linear_fwd_tiles"):
        return f"void lgnn_tile::k_fwd<{t(a[3])}, {a[10]}, 0>"
    if name == "lgnn_node_linear_fwd_bn":
        bn = 1 if a[13] else (2 if a[14] else 0)
        return f"void lgnn_tile::k_fwd<{t(a[3])}, {a[10]}, {bn}>"
    if name in ("lgnn_node_linear_bwd", "lgnn_node_linear_bwd_tiles"):
        return f"void lgnn_tile::k_bwd<{a[0]}, {a[10]}, {t(a[20])}, 0>"
    if name == "lgnn_node_linear_bwd_bn":
        return f"void lgnn_tile::k_bwd<0, {a[3]}, {t(a[9])}, {a[0]}>"
    if name == "lgnn_node_linear_bwd_bn_pool":
        return f"void lgnn_tile::k_bwd<1, {a[3]}, true, 3>"
    if name == "lgnn_node_linear_bwd_bn_gather":
        return f"void lgnn_tile::k_bwd<2, {a[6]}, true, 3>"
    return None


class EntryTracer:
    """HIP-event timing of every C-ABI launch of one eager step (lesion_gnn_amd._lib.set_tracer):
    each launch is bracketed by two events on the current stream, and the step is queued behind
    a spin kernel long enough that the whole step is enqueued before the GPU reaches it, so the
    event pairs bracket back-to-back device work, not host latency."""

    def __init__(self, dev):
        self.dev = dev
        self.rows = []

    def __call__(self, name, args, launch):
        s = torch.cuda.current_stream(self.dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        st = launch()
        e1.record(s)
        self.rows.append((name, tuple(args), e0, e1))
        return st


def profile_entries(step, dev, gs, reps=5):
    """Per-entry average launch time over `reps` eager steps (after one untimed), with the
    algorithmic bytes / FLOP of each launch (_entry_model). Returns rows sorted by time per step,
    plus the traced share of the step."""
    from lesion_gnn_amd import _lib

    # spin length: ~40 ms (calibrated), doubled until the step is enqueued before it drains
    torch.cuda.synchronize(dev)
    c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    c0.record()
    torch.cuda._sleep(1_000_000)
    c1.record()
    torch.cuda.synchronize(dev)
    cycles = int(1_000_000 * 40.0 / max(c0.elapsed_time(c1), 1e-3))
    tracer = EntryTracer(dev)
    agg: dict = {}
    step()
    done, tries = 0, 0
    while done < reps and tries < 4 * reps:
        tries += 1
        torch.cuda.synchronize(dev)
        tracer.rows = []
        t0, t1, spun = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        torch.cuda._sleep(cycles)
        spun.record()
        t0.record()
        _lib.set_tracer(tracer)
        try:
            step()
        finally:
            _lib.set_tracer(None)
        t1.record()
        late = spun.query()  # the spin drained before the host finished enqueueing the step
        torch.cuda.synchronize(dev)
        if late:
            cycles *= 2
            continue
        done += 1
        for name, args, e0, e1 in tracer.rows:
            kern = _entry_kernel(name, args)
            r = agg.setdefault((name, kern), {"calls": 0, "ms": 0.0, "bytes": 0.0, "flops": 0.0,
                                              "modelled": True, "max_ms": 0.0})
            ms = e0.elapsed_time(e1)
            r["calls"] += 1
            r["ms"] += ms
            r["max_ms"] = max(r["max_ms"], ms)
            m = _entry_model(name, args, gs)
            if m is None:
                r["modelled"] = False
            else:
                r["bytes"] += m[0]
                r["flops"] += m[1]
        agg.setdefault("_step", {"ms": 0.0})["ms"] += t0.elapsed_time(t1)
    step_ms = agg.pop("_step")["ms"] / max(done, 1)
    rows = []
    for (name, kern), r in agg.items():
        n = r["calls"]
        row = {"entry": name, "kernel": kern, "calls_per_step": round(n / done, 2),
               "avg_launch_ms": round(r["ms"] / n, 5), "ms_per_step": round(r["ms"] / done, 5)}
        if r["modelled"]:
            sec = r["ms"] * 1e-3
            row.update({"bytes_per_launch": round(r["bytes"] / n),
                        "flops_per_launch": round(r["flops"] / n),
                        "GBps": round(r["bytes"] / sec / 1e9, 1),
                        "TFLOPs": round(r["flops"] / sec / 1e12, 2)})
        rows.append(row)
    rows.sort(key=lambda r: -r["ms_per_step"])
    traced = sum(r["ms_per_step"] for r in rows)
    return rows, {"eager_step_ms": round(step_ms, 4), "traced_ms": round(traced, 4),
                  "steps": done, "spin_cycles": cycles}


def layer_roofline(rows, workload):
    """roofline / roofline_next for the layer-wise workloads (C4 GIN, C5 GCN): the longest modelled
    launches of the per-entry profile (tile.hip k_fwd / k_bwd: fp32 MFMA GEMMs + CSR gathers).
    Both roofs are reported; `bound` is the one the kernel is closer to. For C5 (BASELINE
    configs[4]: "rocprof HBM GB/s vs roofline") the HBM side also carries the rocprofv3 PMC bytes
    per launch over the same HIP-event launch time (`pmc_GBps`)."""
    cand = [r for r in rows if "bytes_per_launch" in r]
    cand.sort(key=lambda r: -r["avg_launch_ms"])
    out = []
    for r in cand[:3]:
        sec = r["avg_launch_ms"] * 1e-3
        gbs, tf = r["bytes_per_launch"] / sec / 1e9, r["flops_per_launch"] / sec / 1e12
        mpeak = MFMA_S3_PEAK_TF if r["entry"] in _S3_ENTRIES else MFMA_F32_PEAK_TF
        f_hbm, f_mfma = gbs / HBM_PEAK_GBS, tf / mpeak
        traffic, tsrc = pmc_traffic(r["kernel"] or _ENTRY_TRACE.get(r["entry"], r["entry"]),
                                    workload)
        hbm = f_hbm >= f_mfma
        what = ("split-3 bf16 MFMA at fp32 accuracy" if r["entry"] in _S3_ENTRIES else
                "fp32 MFMA + CSR gather, tile.hip" if r["kernel"] else "CSR gather")
        row = {"bound": "hbm" if hbm else "mfma", "achieved": round(gbs if hbm else tf, 2),
               "peak": HBM_PEAK_GBS if hbm else mpeak,
               "unit": "GB/s" if hbm else "TFLOP/s", "frac": round(max(f_hbm, f_mfma), 4),
               "frac_hbm": round(f_hbm, 4), "frac_mfma": round(f_mfma, 4),
               "achieved_GBps": round(gbs, 1), "achieved_TFLOPs": round(tf, 2),
               "traffic": round(traffic) if traffic else None, "traffic_source": tsrc,
               "pmc_GBps": round(traffic / sec / 1e9, 1) if traffic else None,
               "frac_pmc_hbm": round(traffic / sec / 1e9 / HBM_PEAK_GBS, 4) if traffic else None,
               "kernel": f"{r['entry']} -> {r['kernel'] or 'its kernels'} ({what})",
               "trace_name": r["kernel"], "calls_per_step": r["calls_per_step"],
               "avg_launch_ms": r["avg_launch_ms"],
               "bytes_per_launch": r["bytes_per_launch"],
               "flops_per_launch": r["flops_per_launch"],
               "timing": "HIP events around the launch on its stream, eager step queued behind a "
                         "spin kernel (bench.profile_entries)"}
        out.append(row)
    if not out:
        return None, []
    return out[0], out[1:]


def time_knn(b, wl, dev):
    """The data-side k-NN graph build of this batch (KNNGraph(k, loop=True), reference
    configs/config.py:47): GPU (lgnn_knn_graph, one launch for the whole batch, HIP events) vs
    the vectorised CPU restatement (synth.knn_edges per size group, one thread). Not part of the
    timed step; reported beside it."""
    from lesion_gnn_amd import synth
    from lesion_gnn_amd.knn import knn_graph

    k = wl["k"]
    knn_graph(b.pos, k, b.batch, loop=True, num_graphs=b.num_graphs)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    reps = 10
    for _ in range(reps):
        ei = knn_graph(b.pos, k, b.batch, loop=True, num_graphs=b.num_graphs)
    e1.record()
    torch.cuda.synchronize(dev)
    gpu_ms = e0.elapsed_time(e1) / reps
    same = bool(torch.equal(ei, b.edge_index))
    pos, ptr = b.pos.cpu(), b.ptr.cpu().tolist()
    sizes = [ptr[i + 1] - ptr[i] for i in range(len(ptr) - 1)]
    nthreads = torch.get_num_threads()
    torch.set_num_threads(1)
    t0 = time.perf_counter()
    by_size: dict[int, list[int]] = {}
    for g, n in enumerate(sizes):
        by_size.setdefault(n, []).append(g)
    for n, gs in by_size.items():
        synth.knn_edges(torch.stack([pos[ptr[g]:ptr[g] + n] for g in gs]), k, True)
    cpu_ms = (time.perf_counter() - t0) * 1e3
    torch.set_num_threads(nthreads)
    return {"graphs": b.num_graphs, "nodes": b.num_nodes, "k": k,
            "gpu_ms_incl_host_sizing": round(gpu_ms, 4), "cpu_ms_1thread": round(cpu_ms, 2),
            "bitexact_vs_batch_edge_index": same}


def pmc_traffic(trace_name: str, workload: str | None = None):
    """HBM bytes per launch of `trace_name` from the committed rocprofv3 PMC passes
    (profiles/traffic.json, written by tools/summarize_prof.py from separate FETCH_SIZE and
    WRITE_SIZE passes of this same bench command: (2*FETCH_SIZE + WRITE_SIZE) * 1024). Keys
    "<workload>:<kernel>" (passes recorded per workload) are preferred over bare kernel names."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(path):
        return None, None
    data = json.load(open(path))
    prefixes = ([f"{workload}:{trace_name}"] if workload else []) + [trace_name]
    for pre in prefixes:
        for k, v in data.items():
            if k.startswith(pre):
                return v["bytes_per_launch"], v["source"]
    if workload and "::" in trace_name and "(" not in trace_name:  # a bare kernel name
        for k, v in data.items():
            if k.startswith(f"{workload}:") and trace_name in k:
                return v["bytes_per_launch"], v["source"]
    return None, None


def cpu_share() -> int:
    """CPUs this process may actually use: its affinity mask, capped by the cgroup CPU quota
    (cgroup v2 cpu.max) and by OMP_NUM_THREADS when the environment sets it. On the GPU box the affinity mask lists every host CPU (256) while the
    job's quota is 16 CPUs; torch with 256 threads under a 16-CPU quota runs ~500x slower
    (measured r02c: 23 s per 1024-graph step)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(float(quota) / float(period))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:  # the box exports its CPU share here (16 per GPU)
        n = min(n, int(omp))
    return n


def cpu_baseline(wl, B, seconds, c1: bool = False):
    """Oracle (plain-torch CPU restatement of the PyG path) on the host cores:
    same model, same step (fwd + loss + bwd + Adam), same per-graph shapes. Two legs, each 3
    warmup steps then the median of up to 10 timed steps (fewer if a leg passes `seconds`):
      * all cores this process may run on (cpu_share: affinity capped by the cgroup quota),
        B graphs per step;
      * 1 thread, on a B/8-graph sample of the same workload (a 1024-graph step takes seconds
        on one core; the per-graph cost does not depend on the batch size at these sizes).
    `value` / `cores` are the all-cores leg; the host's os.cpu_count() and OMP_NUM_THREADS are
    reported beside them. c1 (the C2 workload): two more legs at SURVEY §8d's C1 shape — the same
    GCN step on 32 graphs (the reference's CPU plumbing config), all cores and 1 thread."""
    host = os.cpu_count() or 1
    avail = cpu_share()
    legs = []
    plan = [(avail, B), (1, max(1, B // 8))]
    if c1:
        plan += [(avail, 32), (1, 32)]
    for threads, nb in plan:
        torch.set_num_threads(threads)
        b = make_batch(wl, nb, seed=11)
        m = build_model(wl, oracle=True)
        opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=2e-6)

        def step():
            opt.zero_grad(set_to_none=True)
            loss_fn(wl, m(b.x, b.edge_index, b.batch, nb), b.y, oracle=True).backward()
            opt.step()

        for _ in range(3):
            step()
        times = []
        t_end = time.perf_counter() + seconds / 2
        while len(times) < 10 and (time.perf_counter() < t_end or len(times) < 3):
            t0 = time.perf_counter()
            step()
            times.append(time.perf_counter() - t0)
        med = statistics.median(times)
        legs.append({"threads": threads, "graphs_per_step": nb, "steps": len(times),
                     "median_ms": round(med * 1e3, 2), "value": round(nb / med, 2)})
    main_leg = legs[0]
    extra = {}
    if c1:
        extra["c1"] = {"graphs_per_step": 32, "value": legs[2]["value"], "cores": legs[2]["threads"],
                       "one_thread_value": legs[3]["value"]}
    return {**{"value": main_leg["value"], "unit": "graphs/s", "cores": main_leg["threads"]},
            **extra,
            "kind": "port", "host_cpu_count": host, "cpu_share": avail,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "one_thread_value": legs[1]["value"], "legs": legs,
            "sample": f"{wl['desc']}; all-cores leg {main_leg['steps']} steps x "
                      f"{main_leg['graphs_per_step']} graphs, 1-thread leg {legs[1]['steps']} "
                      f"steps x {legs[1]['graphs_per_step']} graphs"
                      + ("; C1 legs (32 graphs, all cores / 1 thread)" if c1 else "")
                      + "; median step time after 3 warmups; torch CPU fp32"}


def dry_run(args, wl, world, rank):
    """Plumbing check for the launcher (no GPU, no measurement): every rank all-reduces a
    buffer the size of the model's flat gradient once; rank 0 prints the JSON line."""
    n = sum(p.numel() for p in build_model(wl).parameters())  # module init only, on CPU
    flat = torch.full((n,), float(rank + 1))
    if world > 1:
        dist.all_reduce(flat)
        dist.barrier()
    ok = bool(torch.all(flat == world * (world + 1) / 2))
    if rank == 0:
        emit({"metric": METRIC, "value": None, "unit": "graphs/s", "n_gpus": world,
              "dry_run": True, "allreduce_ok": ok,
              "dist": {"backend": args.backend if world > 1 else None, "world_size": world},
              "config": {"workload": wl["desc"], "name": args.workload,
                         "parallelism": f"dp{world}"}})
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        raise SystemExit("bench.py --dry-run: all-reduce result wrong")


def step_plan(world: int, capture: bool, collectives_in_fwd: bool,
              rccl_capture: bool = False) -> tuple:
    """How one training step runs:
      ("eager",)                                   --graph 0
      ("graph:step",)                              N = 1: forward + backward + Adam, one graph
      ("graph:step+rccl",)                         N > 1 over RCCL (the default): the same one
                                                   graph with the collectives captured in it —
                                                   the SyncBN exchanges where forward and backward
                                                   issue them, then the gradient bucket (pack,
                                                   all-reduce, unpack) before Adam
    With rccl_capture False (gloo, or --rccl-eager) no collective is captured:
      ("graph:fwd_bwd+pack", "rccl", "graph:unpack+opt")   N > 1: the gradient bucket is packed
                                                   (and scaled) at the end of the first graph and
                                                   unpacked at the head of the second; only the
                                                   flat RCCL all-reduce runs between them
      ("graph:segments+pack", "rccl", "graph:unpack+opt")  N > 1 with SyncBN (GIN, C4): its
                                                   all-reduces sit inside forward and backward, so
                                                   the first part is captured as a chain of graphs
                                                   split at each SyncBN exchange (dist.
                                                   SegmentedCapture), the exchanges eager between
                                                   them."""
    if not capture:
        return ("eager",)
    if world == 1:
        return ("graph:step",)
    if rccl_capture:
        return ("graph:step+rccl",)
    if collectives_in_fwd:
        return ("graph:segments+pack", "rccl", "graph:unpack+opt")
    return ("graph:fwd_bwd+pack", "rccl", "graph:unpack+opt")


def eager_step_fn(fwd_bwd, bucket, opt):
    """The step run eagerly: zero the gradients, forward + backward, exchange the flat gradient
    (N > 1) and step the optimizer."""
    def eager_step():
        opt.zero_grad(set_to_none=True)
        fwd_bwd()
        if bucket is not None:
            bucket.pack()
            bucket.reduce()
            bucket.unpack()
        opt.step()
    return eager_step


def make_step(plan: tuple, fwd_bwd, bucket, opt, dev, info: dict | None = None):
    """The step callable for `plan` (step_plan). Graph plans warm up eagerly on a side stream,
    then capture. `info` (optional) receives the executed launch sequence of a segmented plan."""
    eager_step = eager_step_fn(fwd_bwd, bucket, opt)
    if plan == ("eager",):
        return eager_step
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for _ in range(3):
            eager_step()
    torch.cuda.current_stream(dev).wait_stream(side)
    opt.zero_grad(set_to_none=True)
    if plan == ("graph:step",):
        g_step = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g_step):
            fwd_bwd()
            opt.step()
        return g_step.replay
    if plan == ("graph:step+rccl",):
        # N > 1 over RCCL: the collectives (the SyncBN exchanges inside forward and backward,
        # the gradient bucket) are captured into the step's one graph with everything else
        g_all = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g_all):
            fwd_bwd()
            bucket.pack()
            bucket.reduce()
            bucket.unpack()
            opt.step()
        return g_all.replay
    if plan[0] == "graph:segments+pack":
        from lesion_gnn_amd.dist import SegmentedCapture

        seg = SegmentedCapture(dev)

        def first():
            fwd_bwd()
            bucket.pack()

        def second():
            bucket.unpack()
            opt.step()
        seg.capture(first)
        seg.add_collective(bucket.reduce)
        seg.capture(second)
        if info is not None:
            info["segments"] = " | ".join(seg.plan())
        return seg.replay
    g_fb, g_opt = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(g_fb):
        fwd_bwd()
        bucket.pack()
    with torch.cuda.graph(g_opt):
        bucket.unpack()
        opt.step()

    def step():
        g_fb.replay()
        bucket.reduce()  # RCCL stays outside the captured graphs
        g_opt.replay()
    return step


_JSON_OUT = None  # the process's original stdout: the one JSON line goes there


def emit(obj) -> None:
    """Print the bench's JSON line on the real stdout (library banners went to stderr)."""
    line = json.dumps(obj) + "\n"
    if _JSON_OUT is None:
        sys.stdout.write(line)
        sys.stdout.flush()
    else:
        os.write(_JSON_OUT, line.encode())


def main():
    global _JSON_OUT
    args = parse()
    wl = WORKLOADS[args.workload]
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    # everything the libraries print on stdout (RCCL's version banner at communicator creation,
    # ...) goes to stderr, so stdout holds exactly the one JSON line
    sys.stdout.flush()
    _JSON_OUT = os.dup(1)
    os.dup2(2, 1)
    world, rank, dev = setup_dist(args)
    if args.dry_run:
        return dry_run(args, wl, world, rank)
    from lesion_gnn_amd import dist as ldist

    for opt in args.path_option:
        from lesion_gnn_amd import _lib as llib
        name, val = opt.split("=")
        llib.load().lgnn_set_option(getattr(llib, "LGNN_OPT_" + name.upper()), int(val))
    B = args.graphs_per_gpu
    b = make_batch(wl, B, seed=100 + rank).to(dev)
    model = build_model(wl).to(dev)
    run = model
    if wl.get("compile"):  # reference gat.py:84: torch.compile(model, dynamic=True)
        run = torch.compile(model, dynamic=True)
    multi = world > 1 or args.force_dist  # the N > 1 plan (process group + gradient bucket)
    sync_bn = wl["model"] == "gin" and multi and args.sync_bn != "off"
    if multi:
        ldist.broadcast_params(model)
        if sync_bn:  # SyncBN: full-batch statistics across the ranks
            model.set_sync_bn(dist.group.WORLD, global_count=b.num_nodes * world)
    params = list(model.parameters())
    if args.opt == "lgnn":
        from lesion_gnn_amd import optim as lgnn_optim
        opt = lgnn_optim.Adam(params, lr=1e-3, weight_decay=2e-6)
    else:
        okw = {"fused": True} if args.opt == "fused" else {"foreach": True}
        if args.graph:
            okw["capturable"] = True
        opt = torch.optim.Adam(params, lr=1e-3, weight_decay=2e-6, **okw)

    one = torch.ones((), device=dev)  # the loss gradient, allocated once (no fill per step)

    fused_ce = wl["loss"] == "CE" and hasattr(run, "forward_loss") and not wl.get("compile")

    def fwd_bwd():
        if fused_ce:  # model + criterion as one node (GCN.forward_loss = training_step's pair)
            run.forward_loss(b.x, b.edge_index, b.batch, b.y, None, B)[1].backward(one)
        else:
            loss_fn(wl, run(b.x, b.edge_index, b.batch, B), b.y).backward(one)

    # GIN under SyncBN all-reduces inside its forward and backward (RCCL collectives)
    plan = step_plan(2 if multi else 1, bool(args.graph), sync_bn,
                     rccl_capture=multi and args.backend == "nccl" and not args.rccl_eager)
    bucket = ldist.GradBucket(params, B, B * world) if multi else None
    plan_info: dict = {}
    step = make_step(plan, fwd_bwd, bucket, opt, dev, plan_info)
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
        "metric": METRIC, "value": round(value, 1), "unit": "graphs/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "bf16 GEMM operands, f32 accumulate" if wl.get("precision") == "bf16" else "f32",
        "data": "synthetic k-NN lesion graphs (pos~U[0,1)^2, x~N(0,1)), random-init weights",
        "config": {"workload": wl["desc"], "name": args.workload,
                   "step_launch": " | ".join(plan),
                   "criterion": "CE fused with the model node (forward_loss)" if fused_ce else
                   ("CE (ops.cross_entropy)" if wl["loss"] == "CE" else "clamp + MSE"),
                   "sync_bn": sync_bn, "process_group": multi,
                   "adam": args.opt, "graphs_per_gpu": B, "global_batch": B * world,
                   "nodes": b.num_nodes, "edges": b.num_edges, "k": wl["k"], "d_in": wl["d_in"],
                   "hidden": wl["hidden"], "parallelism": f"dp{world}"},
        "dist": {"backend": args.backend if multi else None, "world_size": world},
    }
    if plan_info.get("segments"):
        out["config"]["step_segments"] = plan_info["segments"]
    bpb = step_bytes(b, wl)
    out["step_hbm_roofline"] = {
        "bytes_per_graph": round(bpb / B, 1),
        "achieved_GBps_per_gpu": round(value / world * bpb / B / 1e9, 1),
        "frac_of_8TBps": round(value / world * bpb / B / (HBM_PEAK_GBS * 1e9), 4)}
    if rank == 0 and not args.no_kernel_timing and args.workload == "c2":
        rows = []
        for kt in time_dominant_kernels(model, b, dev):
            achieved = kt["flops"] / (kt["ms"] * 1e-3) / 1e12
            traffic, tsrc = pmc_traffic(kt["trace_name"], args.workload)
            peak = kt.get("peak", MFMA_F32_PEAK_TF)
            rows.append({"bound": "mfma", "achieved": round(achieved, 2),
                         "peak": peak, "unit": "TFLOP/s",
                         "frac": round(achieved / peak, 4),
                         "traffic": round(traffic) if traffic else None,
                         "traffic_source": tsrc, "kernel": kt["kernel"],
                         # the same useful fp32 FLOP against the fp32 MFMA peak (what an fp32
                         # GEMM kernel of these shapes is bounded by); `frac` prices the split-3
                         # algorithm's own ceiling (6 bf16 products per fp32 product)
                         "frac_of_fp32_mfma_peak": round(achieved / MFMA_F32_PEAK_TF, 4),
                         "avg_launch_ms": round(kt["ms"], 5), "flops_per_launch": kt["flops"]})
        rows.sort(key=lambda r: -r["avg_launch_ms"])
        out["roofline"] = rows[0]  # the dominant kernel (longest launch)
        out["roofline_next"] = rows[1:]
    if rank == 0 and not args.no_kernel_timing and wl["model"] == "gat":
        rows = []
        for kt in time_gat_in_proj(model, b, dev, wl):
            sec = kt["ms"] * 1e-3
            tf = kt["flops"] / sec / 1e12
            gbs = kt["bytes"] / sec / 1e9
            f_mfma, f_hbm = tf / kt["peak"], gbs / HBM_PEAK_GBS
            traffic, tsrc = pmc_traffic(kt["trace_name"], args.workload)
            mfma_bound = f_mfma >= f_hbm  # the roof the kernel is closer to
            rows.append({"bound": "mfma" if mfma_bound else "hbm",
                         "achieved": round(tf if mfma_bound else gbs, 2),
                         "peak": kt["peak"] if mfma_bound else HBM_PEAK_GBS,
                         "unit": "TFLOP/s" if mfma_bound else "GB/s",
                         "frac": round(max(f_mfma, f_hbm), 4),
                         "frac_mfma": round(f_mfma, 4), "frac_hbm": round(f_hbm, 4),
                         "achieved_TFLOPs": round(tf, 2), "achieved_GBps": round(gbs, 1),
                         "traffic": round(traffic) if traffic else None, "traffic_source": tsrc,
                         "kernel": kt["kernel"], "avg_launch_ms": round(kt["ms"], 5),
                         "flops_per_launch": kt["flops"], "algorithmic_bytes_per_launch":
                         kt["bytes"]})
        rows.sort(key=lambda r: -r["avg_launch_ms"])
        out["roofline"] = rows[0]
        out["roofline_next"] = rows[1:]
    # one rank only: the eager step's gradient all-reduce (and GIN's SyncBN) would wait on ranks
    # that have left for destroy_process_group
    if rank == 0 and world == 1 and args.entries and not args.no_kernel_timing:
        kind = {"gcn": "gcn", "gin": "gin", "gat": "gat"}[wl["model"]]
        rows, tot = profile_entries(eager_step_fn(fwd_bwd, bucket, opt), dev,
                                    GraphStats(b, kind))
        out["entries"] = rows[:16]
        out["entries_total"] = tot
        if args.workload in ("c4", "c5k4", "c5k16") or "roofline" not in out:
            out["roofline"], out["roofline_next"] = layer_roofline(rows, args.workload)
    if rank == 0 and not args.no_kernel_timing:
        out["knn_graph"] = time_knn(b, wl, dev)
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        out["cpu_baseline"] = cpu_baseline(wl, B, args.cpu_seconds, c1=args.workload == "c2")
    if rank == 0:
        emit(out)
    if multi:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
