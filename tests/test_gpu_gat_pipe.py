"""GPU: the row-pipelined GATConv kernels (gat.hip k_gat_fwd_p / k_gat_bwd_edge_p /
k_gat_bwd_node_p: a half wave walks many rows with the next rows' indices in flight, per-edge
scalars loaded edge-parallel and handed over by ds_bpermute; taken when H*C <= 128 (5..8 heads:
each edge lane holds a second head),
i.e. the reference config's GAT (heads 2, C 64; gat.py:31, configs/config.py:59-64) and C3's,
and also when 128 < H*C <= 512 with C >= 32: two 128-feature strips per row and launch)
are bit-identical to the per-row kernels they replace (path option LGNN_OPT_GAT_PIPE = 0): forward
outputs and
every parameter gradient, with dropout masks, with the readout folded into the last layer's edge
kernel and without, on rows longer than one 8-entry batch (k = 10, hub nodes: the batched walk),
1-node graphs and launches with fewer rows than workgroups. Plus the oracle at the reference
config shape, so the pair is pinned, not only consistent."""
import pytest
import torch

import oracle.pyg_ref as ref
from lesion_gnn_amd import _lib, synth
from lesion_gnn_amd.models import gat as gat_mod
from lesion_gnn_amd.models.gat import GAT

pytestmark = pytest.mark.gpu


def _batch(kind):
    if kind == "refcfg":
        return synth.make_batch(64, k=6, d_in=64, seed=31, sizes="lognormal")
    if kind == "k10":  # every target row has 11 entries: all rows take the long walk
        return synth.make_batch(24, k=10, d_in=64, seed=32, sizes="lognormal")
    if kind == "tiny":  # 3 nodes: fewer rows than the 8 XCD row ranges
        return synth.make_batch(2, k=2, d_in=64, seed=33, sizes=[1, 2])
    # hubs: node 5 gathers 40 extra sources (long target row), node 7 feeds 30 targets (long
    # transpose row), duplicated edges, 1-node graphs
    b = synth.make_batch(7, k=6, d_in=64, seed=34, sizes=[1, 3, 7, 64, 2, 130, 9])
    n = b.num_nodes
    src = torch.cat([torch.arange(40) % n, torch.full((30,), 7), torch.tensor([9, 9])])
    dst = torch.cat([torch.full((40,), 5), (torch.arange(30) * 3) % n, torch.tensor([10, 10])])
    b.edge_index = torch.cat([b.edge_index, torch.stack([src, dst])], 1)
    return b


def _run(m, b, cuda, rng):
    m._dropout_rng.copy_(rng)
    out = m(b.x.to(cuda), b.edge_index.to(cuda), b.batch.to(cuda), b.num_graphs)
    m.zero_grad(set_to_none=True)
    out.square().sum().backward()
    return out.detach().cpu(), {n: p.grad.detach().cpu() for n, p in m.named_parameters()}


@pytest.mark.parametrize("kind,heads,hidden,dropout,fold", [
    ("refcfg", 2, [128] * 4, 0.35, True),
    ("refcfg", 4, [128] * 4, 0.0, False),
    ("refcfg", 1, [128, 128], 0.2, True),
    ("k10", 2, [128, 64, 128], 0.35, True),
    ("k10", 4, [32, 32], 0.0, False),
    ("hubs", 2, [128, 128], 0.3, True),
    ("hubs", 4, [64, 128], 0.0, False),
    ("tiny", 2, [128, 128], 0.0, True),
    # 8 heads at H*C <= 128 (C = 16, 8): two head slots per edge lane
    ("refcfg", 8, [128] * 4, 0.35, True),
    ("k10", 8, [128, 64, 128], 0.35, False),
    ("hubs", 8, [64, 128], 0.3, True),
    ("tiny", 8, [128, 128], 0.0, False),
    ("refcfg", 6, [96, 96], 0.2, True),
    # H*C = 256 (the sweep's width 256): the two-strip form, 2..8 heads
    ("refcfg", 8, [256, 256], 0.35, True),
    ("k10", 2, [256, 256], 0.0, False),
    ("hubs", 4, [256, 128], 0.3, True),
    ("tiny", 8, [256, 256], 0.0, True),
    # H*C = 512: two launches of the two-strip form per kernel
    ("refcfg", 4, [512, 512], 0.35, True),
    ("hubs", 8, [512, 256], 0.3, False),
    ("k10", 8, [512, 512], 0.0, True),
])
def test_pipelined_kernels_bitwise(cuda, monkeypatch, kind, heads, hidden, dropout, fold):
    b = _batch(kind)
    torch.manual_seed(len(hidden) * 7 + heads)
    m = GAT(64, hidden, 1, heads=heads, dropout=dropout, pool="mean").to(cuda).train()
    monkeypatch.setattr(gat_mod, "HEAD_FOLD", fold)
    rng = m._dropout_rng.clone()
    res = []
    for pipe in (1, 0):
        with _lib.path_option(_lib.LGNN_OPT_GAT_PIPE, pipe):
            res.append(_run(m, b, cuda, rng))
    assert torch.equal(res[0][0], res[1][0])
    for n in res[1][1]:
        assert torch.equal(res[0][1][n], res[1][1][n]), n


def test_pipelined_reference_config_vs_oracle(cuda):
    """The reference model (GAT [128]*4, heads 2) through the pipelined kernels (the default
    path option) vs the oracle, tests/test_gpu_gat.py's fp32 bar."""
    assert _lib.load().lgnn_get_option(_lib.LGNN_OPT_GAT_PIPE) == 1
    b = _batch("hubs")
    torch.manual_seed(5)
    ours = GAT(64, [128] * 4, 1, heads=2, dropout=0.0)
    oref = ref.GAT(64, [128] * 4, 1, heads=2, dropout=0.0)
    oref.load_state_dict(ours.state_dict())
    out = ours.to(cuda).train()(b.x.to(cuda), b.edge_index.to(cuda), b.batch.to(cuda),
                                b.num_graphs)
    want = oref(b.x, b.edge_index, b.batch, b.num_graphs)
    torch.testing.assert_close(out.detach().cpu(), want.detach(), rtol=0,
                               atol=1e-4 * max(1.0, want.abs().max().item()))
    out.square().sum().backward()
    want.square().sum().backward()
    gr = dict(oref.named_parameters())
    for n, p in ours.named_parameters():
        scale = gr[n].grad.abs().max().item()
        torch.testing.assert_close(p.grad.cpu(), gr[n].grad, rtol=0, atol=max(1e-4 * scale, 1e-6),
                                   msg=lambda s: f"{n}: {s}")


@pytest.mark.parametrize("bpc", [1, 3])
def test_pipelined_grid_override(cuda, bpc):
    """LGNN_OPT_GAT_BPC (workgroups per CU of the persistent grid, a tuning option) changes only
    which half wave walks which rows, never the results."""
    b = _batch("refcfg")
    torch.manual_seed(3)
    m = GAT(64, [128] * 3, 1, heads=2, dropout=0.35).to(cuda).train()
    rng = m._dropout_rng.clone()
    base = _run(m, b, cuda, rng)
    with _lib.path_option(_lib.LGNN_OPT_GAT_BPC, bpc):
        got = _run(m, b, cuda, rng)
    assert torch.equal(base[0], got[0])
    for n in base[1]:
        assert torch.equal(base[1][n], got[1][n]), n
