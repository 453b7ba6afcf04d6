"""Data-parallel HIP path on one GPU box: 2 ranks (processes) on cuda:0 over gloo (RCCL needs one
GPU per rank; the collectives are the same torch.distributed calls bench.py makes on RCCL).

* GCN: sharded batch + flat gradient all-reduce == single-process full-batch gradients.
* GIN with SyncBN: all-reduced BatchNorm sums make 2 replicas reproduce the single-process
  full-batch forward AND gradients.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

B, N, K = 16, 40, 6


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def build(kind):
    from lesion_gnn_amd.models import GCN, GIN

    torch.manual_seed(5)
    if kind == "gcn":
        return GCN(32, [64, 64, 64], 5, 0.0)
    return GIN(32, [64, 64, 64], 5, 0.0, pool="add")  # gin, gin_fixed


def shard(b, g0, g1):
    n0, n1 = int(b.ptr[g0]), int(b.ptr[g1])
    m = (b.edge_index[1] >= n0) & (b.edge_index[1] < n1)
    return b.x[n0:n1], b.edge_index[:, m] - n0, b.batch[n0:n1] - g0, b.y[g0:g1]


def worker(rank, world, port, kind, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from lesion_gnn_amd import dist as ldist
    from lesion_gnn_amd import synth

    dev = torch.device("cuda:0")
    b = synth.make_batch(B, n=N, k=K, d_in=32, seed=17)
    m = build(kind).to(dev).train()
    if kind == "gin":
        m.set_sync_bn(dist.group.WORLD)
    elif kind == "gin_fixed":  # known global node count: no per-step count all-reduce
        m.set_sync_bn(dist.group.WORLD, global_count=B * N)
    g0, g1 = rank * B // world, (rank + 1) * B // world
    x, ei, bt, y = (t.to(dev) for t in shard(b, g0, g1))
    logits = m(x, ei, bt, g1 - g0)
    torch.nn.functional.cross_entropy(logits, y).backward()
    ldist.allreduce_grads(list(m.parameters()), g1 - g0, B)
    # numpy arrays pickle by value (torch CPU tensors would travel through shared memory owned
    # by this process, which may have exited before the parent reads the queue)
    out = {"logits": logits.detach().cpu().numpy(),
           "grads": {k: p.grad.detach().cpu().numpy() for k, p in m.named_parameters()}}
    if kind != "gcn":
        out["state"] = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()
                        if "running" in k}
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["gcn", "gin", "gin_fixed"])
def test_two_ranks_match_full_batch(cuda, kind):
    from lesion_gnn_amd import synth

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, 2, port, kind, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    b = synth.make_batch(B, n=N, k=K, d_in=32, seed=17)
    m = build(kind).to(cuda).train()
    logits = m(b.x.to(cuda), b.edge_index.to(cuda), b.batch.to(cuda), B)
    torch.nn.functional.cross_entropy(logits, b.y.to(cuda)).backward()
    full = logits.detach().cpu()
    got = torch.cat([torch.from_numpy(res[0]["logits"]), torch.from_numpy(res[1]["logits"])])
    torch.testing.assert_close(got, full, rtol=0, atol=1e-4 * max(1.0, full.abs().max().item()))
    for k, p in m.named_parameters():
        want = p.grad.cpu()
        for r in range(2):
            torch.testing.assert_close(torch.from_numpy(res[r]["grads"][k]), want, rtol=0,
                                       atol=max(1e-4 * want.abs().max().item(), 5e-6),
                                       msg=lambda s: f"rank {r} {k}: {s}")
    if kind != "gcn":
        for k, v in m.state_dict().items():
            if "running" in k:
                torch.testing.assert_close(torch.from_numpy(res[0]["state"][k]), v.cpu(),
                                           rtol=1e-5, atol=1e-6)


def plan_worker(rank, world, port, q, backend="gloo"):
    """bench.py's N > 1 GIN + SyncBN plan, captured: graph segments split at the SyncBN
    exchanges (forward and backward), the gradient bucket exchange, the optimizer graph."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    kw = {"device_id": dev} if backend == "nccl" else {}
    dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    import bench
    from lesion_gnn_amd import dist as ldist
    from lesion_gnn_amd import ops, synth

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    b = synth.make_batch(B, n=N, k=K, d_in=32, seed=17)
    m = build("gin").to(dev).train()
    m.set_sync_bn(dist.group.WORLD, global_count=B * N)
    g0, g1 = rank * B // world, (rank + 1) * B // world
    x, ei, bt, y = (t.to(dev) for t in shard(b, g0, g1))
    params = list(m.parameters())
    # SGD: Adam would normalise the analytically-zero gradient of the bias that feeds BatchNorm
    # (round-off noise) into +-lr steps that differ between the replicas and the full batch
    opt = torch.optim.SGD(params, lr=0.05)
    bucket = ldist.GradBucket(params, g1 - g0, B)

    def fwd_bwd():
        ops.cross_entropy(m(x, ei, bt, g1 - g0), y).backward()

    plan = bench.step_plan(max(world, 2), True, True, rccl_capture=backend == "nccl")
    info = {}
    step = bench.make_step(plan, fwd_bwd, bucket, opt, dev, info)
    for _ in range(3):
        step()
    torch.cuda.synchronize(dev)
    q.put((rank, {"plan": plan, "segments": info.get("segments"),
                  "state": {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}}))
    dist.barrier()
    dist.destroy_process_group()


def test_segmented_syncbn_plan_matches_full_batch(cuda):
    """The captured N > 1 GIN + SyncBN step (bench.step_plan -> SegmentedCapture) on 2 ranks:
    after the 3 warm-up eager steps make_step runs and 3 replays, every replica holds the weights
    and BN running statistics of 6 full-batch single-process steps."""
    from lesion_gnn_amd import ops, synth

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=plan_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert res[0]["plan"] == ("graph:segments+pack", "rccl", "graph:unpack+opt")
    seg = res[0]["segments"].split(" | ")
    # per GINConv: one exchange in the forward, one in the backward; then the gradient bucket
    assert seg.count("rccl") == 2 * 2 + 1 and seg[-1] == "graph", seg
    b = synth.make_batch(B, n=N, k=K, d_in=32, seed=17)
    m = build("gin").to(cuda).train()
    opt = torch.optim.SGD(list(m.parameters()), lr=0.05)
    x, ei, bt, y = b.x.to(cuda), b.edge_index.to(cuda), b.batch.to(cuda), b.y.to(cuda)
    for _ in range(6):
        opt.zero_grad(set_to_none=True)
        ops.cross_entropy(m(x, ei, bt, B), y).backward()
        opt.step()
    for k, v in m.state_dict().items():
        for r in range(2):
            got = torch.from_numpy(res[r]["state"][k])
            if got.dtype.is_floating_point:
                torch.testing.assert_close(got, v.cpu(), rtol=1e-4, atol=1e-5,
                                           msg=lambda s: f"rank {r} {k}: {s}")
            else:
                assert torch.equal(got, v.cpu()), k


def test_rccl_captured_plan_one_rank(cuda):
    """bench.py's default N > 1 plan over RCCL (step_plan -> "graph:step+rccl": the SyncBN
    exchanges and the gradient all-reduce captured into the step's one HIP graph), run on a
    one-rank RCCL group (RCCL needs one GPU per rank): 3 replays after make_step's 3 eager steps
    hold the weights and BN statistics of 6 single-process steps."""
    from lesion_gnn_amd import ops, synth

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=plan_worker, args=(0, 1, free_port(), q, "nccl"))
    p.start()
    rank, res = q.get(timeout=300)
    p.join(timeout=120)
    assert p.exitcode == 0
    assert res["plan"] == ("graph:step+rccl",)
    b = synth.make_batch(B, n=N, k=K, d_in=32, seed=17)
    m = build("gin").to(cuda).train()
    opt = torch.optim.SGD(list(m.parameters()), lr=0.05)
    x, ei, bt, y = b.x.to(cuda), b.edge_index.to(cuda), b.batch.to(cuda), b.y.to(cuda)
    for _ in range(6):
        opt.zero_grad(set_to_none=True)
        ops.cross_entropy(m(x, ei, bt, B), y).backward()
        opt.step()
    for k, v in m.state_dict().items():
        got = torch.from_numpy(res["state"][k])
        if got.dtype.is_floating_point:
            torch.testing.assert_close(got, v.cpu(), rtol=1e-4, atol=1e-5, msg=lambda s: f"{k}: {s}")
        else:
            assert torch.equal(got, v.cpu()), k
