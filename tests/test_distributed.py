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
