"""GPU radius graph construction (liblgnn lgnn_radius_count / lgnn_radius_graph via
lesion_gnn_amd.knn.radius_graph / RadiusGraph) vs the CPU restatement of torch_cluster 1.6.3's
radius_graph (oracle.pyg_ref.radius_graph, itself checked against the literal per-query walk in
tests/test_oracle.py). The reference sweep's alternative connectivity: RadiusGraph(r) with PyG's
defaults loop=False, max_num_neighbors=32, r in [1, 1536] pixels (scripts/sweep.py:113-118).

Bar: edge_index bit-exact (same neighbours, same order). Cases: log-normal (C3-shaped) and
power-law (C5-shaped) ragged batches in pixel coordinates; radii from sparse to "everything in
range", so rows hit the 32-neighbour cap (the walk keeps the first 33 in index order and drops
the self pair: 32 or 33 neighbours); loop=True; 3-D positions; coincident points; r = 0;
single-node graphs; one graph larger than the LDS candidate chunk (1024); max_num_neighbors 1;
flow='target_to_source'; the transform resolved by name (transforms.get_transform).
"""
import pytest
import torch

import oracle.pyg_ref as ref
from lesion_gnn_amd import synth, transforms
from lesion_gnn_amd.knn import radius_graph

pytestmark = pytest.mark.gpu


def batch_of(sizes):
    return torch.repeat_interleave(torch.arange(len(sizes)), torch.tensor(sizes))


def ptr_of(sizes):
    return [0] + torch.cumsum(torch.tensor(sizes), 0).tolist()


def check(pos, sizes, r, loop, max_nb, cuda, dims=2):
    want = ref.radius_graph_batch(pos, r, ptr_of(sizes), loop, max_nb)
    got = radius_graph(pos.to(cuda), r, batch_of(sizes).to(cuda), loop=loop,
                       max_num_neighbors=max_nb).cpu()
    assert got.dtype == torch.int64 and got.shape == want.shape, (got.shape, want.shape)
    assert torch.equal(got, want)
    return want


@pytest.mark.parametrize("sizes_kind,r", [("lognormal", 60.0), ("lognormal", 400.0),
                                          ("lognormal", 1536.0), ("powerlaw", 200.0),
                                          ("powerlaw", 1536.0)])
@pytest.mark.parametrize("loop", [False, True])
def test_radius_graph_ragged_batches(cuda, sizes_kind, r, loop):
    g = torch.Generator().manual_seed(7)
    sizes = synth.graph_sizes(96 if sizes_kind == "lognormal" else 48, sizes_kind, g)
    pos = torch.rand(sum(sizes), 2, generator=g, dtype=torch.float64) * 1536.0
    want = check(pos, sizes, r, loop, 32, cuda)
    if r == 1536.0:  # every pair in range: the cap binds on every row of graphs > 33 nodes
        deg = torch.bincount(want[1], minlength=sum(sizes))
        assert int(deg.max()) == (32 if loop else 33)


def test_radius_graph_edge_cases(cuda):
    g = torch.Generator().manual_seed(3)
    # single-node graphs, a graph of coincident points (cap + ties), r = 0 (no edges)
    sizes = [1, 40, 5, 1, 70]
    pos = torch.rand(sum(sizes), 2, generator=g, dtype=torch.float64) * 100
    pos[1:41] = 7.0
    check(pos, sizes, 3.0, False, 32, cuda)
    check(pos, sizes, 3.0, True, 32, cuda)
    assert check(pos, sizes, 0.0, False, 32, cuda).numel() == 0
    check(pos, sizes, 50.0, False, 1, cuda)
    # 3-D positions
    pos3 = torch.rand(sum(sizes), 3, generator=g, dtype=torch.float64)
    want = ref.radius_graph_batch(pos3, 0.4, ptr_of(sizes), False, 32)
    got = radius_graph(pos3.to(cuda), 0.4, batch_of(sizes).to(cuda)).cpu()
    assert torch.equal(got, want)
    # one graph past the 1024-candidate LDS chunk, no batch vector
    big = torch.rand(1500, 2, generator=g, dtype=torch.float64)
    want = ref.radius_graph(big, 0.03, False, 32)
    assert torch.equal(radius_graph(big.to(cuda), 0.03).cpu(), want)
    # flow='target_to_source' swaps the rows
    got = radius_graph(big.to(cuda), 0.03, flow="target_to_source").cpu()
    assert torch.equal(got, want.flip(0))
    # nodes but num_graphs = 0: rejected (the batch vector cannot index an empty ptr)
    from lesion_gnn_amd._lib import LgnnError
    with pytest.raises(LgnnError):
        radius_graph(big.to(cuda), 0.03, torch.zeros(1500, dtype=torch.int64, device=cuda),
                     num_graphs=0)
    # no nodes: no edges
    assert radius_graph(big[:0].to(cuda), 0.03).numel() == 0


def test_radius_transform_by_name(cuda):
    """transforms.get_transform(TransformConfig(name="RadiusGraph", kwargs={"r": ...})) — how the
    sweep builds it (sweep.py:113-118) — on a collated batch."""
    g = torch.Generator().manual_seed(11)
    sizes = [30, 64, 12]
    pos = torch.rand(sum(sizes), 2, generator=g, dtype=torch.float64) * 1536.0

    class Data:
        pass

    d = Data()
    d.pos = pos.to(cuda)
    d.batch = batch_of(sizes).to(cuda)
    d.num_graphs = len(sizes)
    d.edge_attr = torch.ones(3)
    t = transforms.get_transform(transforms.TransformConfig(name="RadiusGraph",
                                                            kwargs={"r": 500.0}))
    t(d)
    assert d.edge_attr is None
    assert torch.equal(d.edge_index.cpu(), ref.radius_graph_batch(pos, 500.0, ptr_of(sizes)))
