"""Windowed dense aggregation (lgnn_window_aggregate, csrc/window.hip): the layer-wise GCN
path's open-tile aggregation A_hat H (forward, target CSR) and A_hat^T dY (backward, transpose
CSR) as dense 64 x 64 blocks per source chunk on split-3 MFMA, against a float64 restatement of
the CSR sum (PyG propagate with gcn_norm weights). Bar: 2e-6 of the row scale (fp32-accurate;
the per-row order is the MFMA's, not CSR order). Cases: C5-shaped power-law batches (k = 4, 16),
every tile (mask NULL) and the open tiles only (rows of other tiles untouched, and NaN rows of
unselected tiles never read), the per-row fallback (max_chunks = 1), the transpose CSR.
"""
import pytest
import torch

from lesion_gnn_amd import ops, synth
from lesion_gnn_amd.graph import as_graph

pytestmark = pytest.mark.gpu


def ref_agg(rowptr, col, w, inp):
    rp = rowptr.cpu().long()
    nnz = int(rp[-1])  # col / w have capacity E + N
    rows = torch.repeat_interleave(torch.arange(rp.numel() - 1), rp[1:] - rp[:-1])
    out = torch.zeros(rp.numel() - 1, inp.size(1), dtype=torch.float64)
    src = inp.cpu().double()[col.cpu().long()[:nnz]]
    out.index_add_(0, rows, w.cpu().double()[:nnz].view(-1, 1) * src)
    return out


def graph_of(k, num_graphs, cuda, seed=0):
    b = synth.make_batch(num_graphs, k=k, sizes="powerlaw", seed=seed)
    M = b.x.size(0)
    g = as_graph(b.edge_index.to(cuda), M, b.batch.to(cuda), b.num_graphs)
    return g, M


def tile_rows(mask, M):
    sel = torch.repeat_interleave(mask.cpu()[: (M + 63) // 64] != 0, 64)[:M]
    return sel


@pytest.mark.parametrize("k", [4, 16])
@pytest.mark.parametrize("transpose", [False, True])
def test_window_aggregate_open_tiles(cuda, k, transpose):
    g, M = graph_of(k, 160, cuda)
    csr = g.csr("gcn")
    open_ = g.tile_open("gcn")
    ptr, idx, w = (csr.tptr, csr.tidx, csr.tw) if transpose else (csr.rowptr, csr.col, csr.w)
    gen = torch.Generator().manual_seed(1)
    inp = torch.randn(M, 128, generator=gen).to(cuda)
    sel = tile_rows(open_, M)
    assert sel.any()  # power-law batches: most (at k = 4 often all) tiles are open
    inp_nan = inp.clone()
    inp_nan[sel.logical_not().to(cuda)] = float("nan")  # rows of closed tiles: never read
    out = torch.full((M, 128), 7.0, device=cuda)
    ops.window_aggregate(ptr, idx, w, M, inp_nan, out, open_)
    want = ref_agg(ptr, idx, w, inp)
    got = out.cpu()
    assert torch.all(got[~sel] == 7.0)  # other tiles' rows untouched
    err = (got[sel].double() - want[sel]).abs().max().item()
    scale = want[sel].abs().max().item()
    assert err <= 2e-6 * max(scale, 1.0), (err, scale)


@pytest.mark.parametrize("max_chunks", [1, 20])
def test_window_aggregate_every_tile(cuda, max_chunks):
    g, M = graph_of(16, 96, cuda, seed=3)
    csr = g.csr("gcn")
    gen = torch.Generator().manual_seed(2)
    inp = torch.randn(M, 128, generator=gen).to(cuda)
    out = torch.empty(M, 128, device=cuda)
    old = ops.WINDOW_CHUNKS
    ops.WINDOW_CHUNKS = max_chunks  # 1: every straddling tile takes the per-row gather
    try:
        ops.window_aggregate(csr.rowptr, csr.col, csr.w, M, inp, out, None)
    finally:
        ops.WINDOW_CHUNKS = old
    want = ref_agg(csr.rowptr, csr.col, csr.w, inp)
    err = (out.cpu().double() - want).abs().max().item()
    assert err <= 2e-6 * max(want.abs().max().item(), 1.0), err


def test_window_layerwise_stack_matches_gather(cuda, monkeypatch):
    """The C5 GCN step's open-tile layers with the windowed aggregation equal the per-entry
    gather path (LGNN_WINDOW=0) to fp32 accuracy: forward H_l and every parameter gradient."""
    from lesion_gnn_amd.models.gcn import GCN
    torch.manual_seed(0)
    b = synth.make_batch(192, k=16, sizes="powerlaw", seed=5)
    model = GCN(128, [128, 128, 128], 5, dropout=0.0).to(cuda)
    x, ei, batch = b.x.to(cuda), b.edge_index.to(cuda), b.batch.to(cuda)
    res = {}
    for win in (True, False):
        monkeypatch.setattr(ops, "WINDOW", win)
        model.zero_grad()
        logits = model(x, ei, batch, b.num_graphs)
        logits.square().sum().backward()
        res[win] = (logits.detach().cpu(), [p.grad.detach().cpu().clone()
                                            for p in model.parameters()])
    (lw, gw), (lg, gg) = res[True], res[False]
    assert (lw - lg).abs().max().item() <= 1e-4 * max(lg.abs().max().item(), 1.0)
    for a, c in zip(gw, gg):
        assert (a - c).abs().max().item() <= 1e-4 * max(c.abs().max().item(), 1e-6)
