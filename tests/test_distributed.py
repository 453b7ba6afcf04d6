"""N > 1 data-parallel path on CPU (gloo, world_size 2): sharding + the flat-gradient
all-reduce reproduce the single-process full-batch gradients. The model here is the CPU oracle
(the HIP model is GPU-only); the same lesion_gnn_amd.dist helpers drive bench.py on RCCL."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle.pyg_ref as ref
from lesion_gnn_amd import dist as ldist
from lesion_gnn_amd import synth


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def sub_batch(b, g0, g1):
    n0, n1 = int(b.ptr[g0]), int(b.ptr[g1])
    m = (b.edge_index[1] >= n0) & (b.edge_index[1] < n1)
    return (b.x[n0:n1], b.edge_index[:, m] - n0, b.batch[n0:n1] - g0, b.y[g0:g1])


def make_model(kind):
    torch.manual_seed(7)
    if kind == "gcn":
        return ref.GCN(16, [16, 16, 16], 5, 0.0)
    return ref.GAT(16, [16, 16], 5, heads=2, dropout=0.0)


def worker(rank, world, port, kind, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    b = synth.make_batch(10, d_in=16, k=4, seed=3, sizes="lognormal")
    costs = (b.ptr[1:] - b.ptr[:-1]).tolist()
    bounds = ldist.shard_bounds(costs, world)
    g0, g1 = bounds[rank], bounds[rank + 1]
    m = make_model(kind)
    ldist.broadcast_params(m)
    x, ei, bt, y = sub_batch(b, g0, g1)
    loss = torch.nn.functional.cross_entropy(m(x, ei, bt, g1 - g0), y)
    loss.backward()
    ldist.allreduce_grads(list(m.parameters()), g1 - g0, b.num_graphs)
    if rank == 0:
        out.put({k: p.grad.numpy().copy() for k, p in m.named_parameters()})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["gcn", "gat"])
def test_two_rank_gradients_match_full_batch(kind):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, 2, port, kind, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    b = synth.make_batch(10, d_in=16, k=4, seed=3, sizes="lognormal")
    m = make_model(kind)
    torch.nn.functional.cross_entropy(m(b.x, b.edge_index, b.batch, b.num_graphs), b.y).backward()
    for k, p in m.named_parameters():
        torch.testing.assert_close(torch.from_numpy(got[k]), p.grad, atol=1e-6, rtol=1e-5,
                                   msg=lambda s: f"{k}: {s}")


def test_shard_bounds_balance_edges():
    costs = [1, 1, 1, 1, 100, 1, 1, 1]
    b = ldist.shard_bounds(costs, 2)
    assert b[0] == 0 and b[-1] == 8 and b == sorted(b)
    assert ldist.shard_bounds([5] * 8, 4) == [0, 2, 4, 6, 8]
    assert ldist.shard_bounds([], 3) == [0, 0, 0, 0]


def test_bench_step_plan():
    """bench.py's step structure: over RCCL the N > 1 step is one graph with its collectives
    captured in it; with collectives that cannot be captured (gloo, --rccl-eager) SyncBN (GIN,
    C4) is captured as graph segments split at its all-reduces (which sit inside forward and
    backward), and otherwise the flat-gradient all-reduce is the only eager part between two
    graphs."""
    import bench

    assert bench.step_plan(1, True, False) == ("graph:step",)
    assert bench.step_plan(1, True, True) == ("graph:step",)  # one rank: SyncBN is local
    assert bench.step_plan(2, True, False) == ("graph:fwd_bwd+pack", "rccl", "graph:unpack+opt")
    assert bench.step_plan(8, True, True) == ("graph:segments+pack", "rccl", "graph:unpack+opt")
    assert bench.step_plan(4, False, False) == ("eager",)
    assert bench.step_plan(4, False, True) == ("eager",)
    # over RCCL (the default backend) the collectives are captured into the step's graph
    assert bench.step_plan(8, True, True, rccl_capture=True) == ("graph:step+rccl",)
    assert bench.step_plan(2, True, False, rccl_capture=True) == ("graph:step+rccl",)
    assert bench.step_plan(1, True, True, rccl_capture=True) == ("graph:step",)
    assert bench.step_plan(4, False, True, rccl_capture=True) == ("eager",)


class _SyncNormNet(torch.nn.Module):
    """A SyncBN-shaped CPU model: the forward normalises with batch statistics all-reduced over
    the group (autograd through the all-reduce, as SyncBN's backward all-reduces too)."""

    def __init__(self):
        super().__init__()
        torch.manual_seed(5)
        self.lin = torch.nn.Linear(6, 4)
        self.out = torch.nn.Linear(4, 3)

    def forward(self, x, world):
        z = self.lin(x)
        s = torch.stack([z.sum(0), (z * z).sum(0)])
        n = torch.tensor(float(x.size(0)))
        if world > 1:
            import torch.distributed.nn.functional as dnf

            s = dnf.all_reduce(s)
            n = n * world
        mean = s[0] / n
        var = s[1] / n - mean * mean
        return self.out(torch.nn.functional.elu((z - mean) / torch.sqrt(var + 1e-5)))


def _plan_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    import bench

    g = torch.Generator().manual_seed(0)
    X, Y = torch.randn(16, 6, generator=g), torch.randint(0, 3, (16,), generator=g)
    x, y = X[8 * rank:8 * rank + 8], Y[8 * rank:8 * rank + 8]
    m = _SyncNormNet()
    ldist.broadcast_params(m)
    params = list(m.parameters())
    opt = torch.optim.SGD(params, lr=0.1)
    bucket = ldist.GradBucket(params, 8, 16)

    def fwd_bwd():
        torch.nn.functional.cross_entropy(m(x, world), y).backward()

    # CPU: the eager form of the plan (--graph 0); the captured segments run on the GPU
    # (tests/test_gpu_dist.py)
    plan = bench.step_plan(world, False, True)
    step = bench.make_step(plan, fwd_bwd, bucket, opt, torch.device("cpu"))
    for _ in range(3):
        step()
    # the bucket exchange equals allreduce_grads on the same gradients
    opt.zero_grad(set_to_none=True)
    fwd_bwd()
    ref_grads = [p.grad.clone() for p in params]
    bucket.pack()
    bucket.reduce()
    bucket.unpack()
    # unpack launches nothing: every grad is now a view of the reduced flat buffer
    same_ptr = all(p.grad.data_ptr() == v.data_ptr() for p, v in zip(params, bucket.views))
    via_bucket = [p.grad.clone() for p in params]
    for p, g0 in zip(params, ref_grads):
        p.grad = g0
    ldist.allreduce_grads(params, 8, 16)
    same = same_ptr and not bucket.avg and all(
        torch.allclose(a, p.grad, atol=1e-7) for a, p in zip(via_bucket, params))
    if rank == 0:
        out.put(({k: v.detach().numpy().copy() for k, v in m.state_dict().items()}, same, plan))
    dist.barrier()
    dist.destroy_process_group()


def test_syncbn_step_plan_two_ranks_matches_full_batch():
    """bench.py's N > 1 step for a model with collectives inside forward / backward (the C4 GIN
    + SyncBN structure), world size 2 on gloo: three steps of the plan bench would run leave the
    same weights as three full-batch single-process steps; the GradBucket exchange equals the
    flat all-reduce."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_plan_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    state, same, plan = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert plan == ("eager",) and same
    g = torch.Generator().manual_seed(0)
    X, Y = torch.randn(16, 6, generator=g), torch.randint(0, 3, (16,), generator=g)
    m = _SyncNormNet()
    opt = torch.optim.SGD(m.parameters(), lr=0.1)
    for _ in range(3):
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(X, 1), Y).backward()
        opt.step()
    for k, v in m.state_dict().items():
        torch.testing.assert_close(torch.from_numpy(state[k]), v, atol=1e-6, rtol=1e-5)
