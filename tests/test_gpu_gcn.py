"""GPU parity: the HIP path (through liblgnn.so's C ABI) vs the CPU oracle (oracle/pyg_ref.py).

Tolerances: fp32 logits / activations atol 1e-4 (north_star), gradients rtol 1e-4 + atol 1e-5
(fp32 sums over up to 65,536 nodes in a different association order); graph structure (CSR
indices) bit-exact; GCN edge weights exact.
"""
import pytest
import torch

import oracle.pyg_ref as ref
from lesion_gnn_amd import _lib, ops, synth
from lesion_gnn_amd.conv import GCNConv, global_add_pool, global_mean_pool
from lesion_gnn_amd.graph import Graph
from lesion_gnn_amd.models.gcn import GCN

pytestmark = pytest.mark.gpu


def ref_csr(edge_index: torch.Tensor, n: int):
    """CPU restatement of the CSR the kernels must build: gcn_norm edge list, stably grouped by
    target (rows) and by source (transpose)."""
    ei, w = ref.gcn_norm(edge_index, n)
    o = torch.sort(ei[1], stable=True).indices
    rowptr = torch.zeros(n + 1, dtype=torch.int64)
    rowptr[1:] = torch.cumsum(torch.bincount(ei[1], minlength=n), 0)
    ot = torch.sort(ei[0], stable=True).indices
    tptr = torch.zeros(n + 1, dtype=torch.int64)
    tptr[1:] = torch.cumsum(torch.bincount(ei[0], minlength=n), 0)
    return rowptr, ei[0][o], w[o], tptr, ei[1][ot], w[ot]


def check_csr(edge_index, n, cuda):
    g = Graph(edge_index.to(cuda), n)
    c = g.csr("gcn")
    rowptr, col, w, tptr, tidx, tw = ref_csr(edge_index, n)
    e = int(rowptr[-1])
    assert torch.equal(c.rowptr.cpu().long(), rowptr)
    assert torch.equal(c.col.cpu()[:e].long(), col)
    assert torch.equal(c.w.cpu()[:e], w)
    assert torch.equal(c.tptr.cpu().long(), tptr)
    assert torch.equal(c.tidx.cpu()[:e].long(), tidx)
    assert torch.equal(c.tw.cpu()[:e], tw)
    assert g.dropped_edges("gcn") == 0


def test_graph_build_knn(cuda):
    b = synth.make_batch(16, n=64, k=8, seed=1)
    check_csr(b.edge_index, b.num_nodes, cuda)


def test_graph_build_irregular(cuda):
    # loop=False k-NN, variable sizes incl. 1-node graphs and N < k, shuffled edge order,
    # duplicated edges and duplicated self loops.
    b = synth.make_batch(12, k=8, seed=2, sizes=[1, 3, 7, 64, 65, 2, 130, 1, 9, 16, 8, 33],
                         loop=False)
    ei = b.edge_index
    gen = torch.Generator().manual_seed(0)
    perm = torch.randperm(ei.size(1), generator=gen)
    ei = ei[:, perm]
    extra = torch.tensor([[5, 5, 5, 70, 70], [5, 5, 6, 71, 71]])
    ei = torch.cat([ei, extra], 1)
    check_csr(ei, b.num_nodes, cuda)


def test_graph_build_invalid_edges_dropped(cuda):
    ei = torch.tensor([[0, 1, 7, -1], [1, 0, 0, 2]])
    g = Graph(ei.to(cuda), 3)
    assert g.dropped_edges("gcn") == 2
    check_csr(torch.tensor([[0, 1], [1, 0]]), 3, cuda)


def test_batch_ptr_with_empty_graphs(cuda):
    batch = torch.tensor([0, 0, 2, 2, 2, 5])
    g = Graph(torch.empty(2, 0, dtype=torch.long, device=cuda), 6, batch.to(cuda), 7)
    assert g.gptr.cpu().tolist() == [0, 2, 2, 5, 5, 5, 6, 6]


@pytest.mark.parametrize("M,K,N,gather", [(1000, 128, 128, True), (64, 128, 128, False),
                                          (333, 64, 32, True), (130, 1025, 128, False),
                                          (257, 36, 256, False), (77, 128, 5, False)])
def test_node_linear_fwd(cuda, M, K, N, gather):
    torch.manual_seed(0)
    x = torch.randn(M, K)
    W = torch.randn(N, K) / K ** 0.5
    b = torch.randn(N)
    if gather:
        bt = synth.make_batch((M + 49) // 50, k=6, seed=3, sizes="lognormal")
        ei = bt.edge_index[:, bt.edge_index.max(0).values < M]
        g = Graph(ei.to(cuda), M)
        e, w = ref.gcn_norm(ei, M)
        agg = ref.scatter_sum(w.view(-1, 1) * x.index_select(0, e[0]), e[1], M)
        want = torch.nn.functional.elu(agg @ W.T + b)
        got = ops.linear_fwd(x.to(cuda), W.to(cuda), b.to(cuda), _lib.LGNN_ACT_ELU, g.csr("gcn"))
    else:
        want = x @ W.T + b
        got = ops.linear_fwd(x.to(cuda), W.to(cuda), b.to(cuda), _lib.LGNN_ACT_NONE)
    torch.testing.assert_close(got.cpu(), want, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("M,K,N,gather", [(1000, 128, 128, True), (200, 128, 128, False),
                                          (130, 1025, 128, False), (300, 64, 32, True),
                                          (150, 128, 256, False)])
def test_node_linear_bwd(cuda, M, K, N, gather):
    torch.manual_seed(1)
    x = torch.randn(M, K, requires_grad=True)
    W = (torch.randn(N, K) / K ** 0.5).requires_grad_()
    b = torch.randn(N, requires_grad=True)
    dy = torch.randn(M, N)
    if gather:
        bt = synth.make_batch((M + 49) // 50, k=6, seed=4, sizes="lognormal")
        ei = bt.edge_index[:, bt.edge_index.max(0).values < M]
        e, w = ref.gcn_norm(ei, M)
        g = Graph(ei.to(cuda), M)
        h = ref.scatter_sum(w.view(-1, 1) * x.index_select(0, e[0]), e[1], M)
    else:
        g = None
        h = x
    y = torch.nn.functional.elu(h @ W.T + b)
    y.backward(dy)
    xg = x.detach().to(cuda).requires_grad_()
    Wg = W.detach().to(cuda).requires_grad_()
    bg = b.detach().to(cuda).requires_grad_()
    yg = ops.node_linear(xg, Wg, bg, g, "gcn", 0.0, _lib.LGNN_ACT_ELU)
    torch.testing.assert_close(yg.detach().cpu(), y.detach(), atol=1e-4, rtol=1e-4)
    yg.backward(dy.to(cuda))
    torch.testing.assert_close(Wg.grad.cpu(), W.grad, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(bg.grad.cpu(), b.grad, atol=1e-4, rtol=1e-4)
    if N <= 128:
        torch.testing.assert_close(xg.grad.cpu(), x.grad, atol=1e-4, rtol=1e-4)


def make_pair(hidden, d_in=128, classes=5, pool="mean", seed=1234):
    torch.manual_seed(seed)
    ours = GCN(d_in, hidden, classes, dropout=0.0, pool=pool)
    oref = ref.GCN(d_in, hidden, classes, dropout=0.0, pool=pool)
    oref.load_state_dict(ours.state_dict())
    return ours, oref


def run_step(model, b, device, num_graphs=None):
    x = b.x.to(device)
    logits = model(x, b.edge_index.to(device), b.batch.to(device), num_graphs)
    loss = torch.nn.functional.cross_entropy(logits, b.y.to(device))
    model.zero_grad(set_to_none=True)
    loss.backward()
    grads = {k: p.grad.detach().cpu() for k, p in model.named_parameters()}
    return logits.detach().cpu(), loss.detach().cpu(), grads


@pytest.mark.parametrize("B,pool", [(32, "mean"), (32, "add"), (1024, "mean")])
def test_gcn_model_parity(cuda, B, pool):
    """C1 (B=32) and C2 (B=1024) shapes: 2-layer GCN, N=64, d=128, k=8."""
    b = synth.make_batch(B, n=64, k=8, d_in=128, seed=0)
    ours, oref = make_pair([128, 128, 128], pool=pool)
    lo, losso, go = run_step(ours.to(cuda), b, cuda, B)
    lr_, lossr, gr = run_step(oref, b, "cpu", B)
    torch.testing.assert_close(lo, lr_, atol=1e-4, rtol=0)
    torch.testing.assert_close(losso, lossr, atol=1e-5, rtol=1e-5)
    for k in gr:
        torch.testing.assert_close(go[k], gr[k], atol=1e-5, rtol=1e-4, msg=lambda m: f"{k}: {m}")


def test_gcn_model_irregular_graphs(cuda):
    """Mixed sizes (1-node graphs, N < k, N > 64), lesion-class last channel, 3 layers, widths
    not multiples of 64 nodes."""
    sizes = [1, 5, 64, 200, 2, 33, 512, 17]
    b = synth.make_batch(len(sizes), k=6, d_in=96, seed=5, sizes=sizes, last_channel_class=True)
    ours, oref = make_pair([64, 64, 64, 64], d_in=96)
    lo, _, go = run_step(ours.to(cuda), b, cuda)
    lr_, _, gr = run_step(oref, b, "cpu")
    torch.testing.assert_close(lo, lr_, atol=1e-4, rtol=0)
    for k in gr:
        torch.testing.assert_close(go[k], gr[k], atol=1e-5, rtol=1e-4, msg=lambda m: f"{k}: {m}")


def test_gcn_dropout_path_matches_fused_in_eval(cuda):
    b = synth.make_batch(8, seed=6)
    torch.manual_seed(0)
    m = GCN(128, [128, 128, 128], 5, dropout=0.5).to(cuda)
    m.eval()
    a = m(b.x.to(cuda), b.edge_index.to(cuda), b.batch.to(cuda))
    m.dropout.p = 0.0
    m.train()
    c = m(b.x.to(cuda), b.edge_index.to(cuda), b.batch.to(cuda))
    assert torch.equal(a, c)
    # layer-wise (dropout active) path with p -> tiny keeps results close to the fused path
    m.dropout.p = 1e-9
    d = m(b.x.to(cuda), b.edge_index.to(cuda), b.batch.to(cuda))
    torch.testing.assert_close(d, c, atol=1e-5, rtol=1e-5)


def test_gcn_deterministic(cuda):
    b = synth.make_batch(256, seed=7)
    ours, _ = make_pair([128, 128, 128])
    ours = ours.to(cuda)
    l1, _, g1 = run_step(ours, b, cuda)
    l2, _, g2 = run_step(ours, b, cuda)
    assert torch.equal(l1, l2)
    for k in g1:
        assert torch.equal(g1[k], g2[k]), k


def test_gcnconv_and_pools_standalone(cuda):
    b = synth.make_batch(10, seed=8, sizes="lognormal")
    torch.manual_seed(0)
    conv = GCNConv(128, 64)
    rconv = ref.GCNConv(128, 64)
    rconv.load_state_dict(conv.state_dict())
    x = b.x.clone().requires_grad_()
    xg = b.x.to(cuda).requires_grad_()
    yr = rconv(x, b.edge_index)
    yg = conv.to(cuda)(xg, b.edge_index.to(cuda))
    torch.testing.assert_close(yg.detach().cpu(), yr.detach(), atol=1e-4, rtol=1e-4)
    pr = ref.global_mean_pool(yr, b.batch) + ref.global_add_pool(yr, b.batch)
    pg = (global_mean_pool(yg, b.batch.to(cuda)) + global_add_pool(yg, b.batch.to(cuda)))
    torch.testing.assert_close(pg.detach().cpu(), pr.detach(), atol=1e-4, rtol=1e-4)
    pr.sum().backward()
    pg.sum().backward()
    torch.testing.assert_close(xg.grad.cpu(), x.grad, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(conv.lin.weight.grad.cpu(), rconv.lin.weight.grad, atol=1e-4,
                               rtol=1e-4)


def test_cpu_tensors_rejected(cuda):
    b = synth.make_batch(2, seed=9)
    m = GCN(128, [128, 128], 5, 0.0)
    with pytest.raises(_lib.LgnnError):
        m(b.x, b.edge_index, b.batch)


class _FakeStorage:
    def __init__(self, row, col):
        self._row, self._col = row, col

    def row(self):
        return self._row

    def col(self):
        return self._col


class FakeSparseTensor:
    """Duck-typed torch_sparse.SparseTensor as ToSparseTensor builds it (row = target)."""

    def __init__(self, edge_index):
        o = torch.argsort(edge_index[1] * (edge_index.max() + 1) + edge_index[0])
        self.storage = _FakeStorage(edge_index[1][o], edge_index[0][o])


@pytest.mark.parametrize("form", ["torch_sparse", "sparse_csr"])
def test_adj_t_input_matches_edge_index(cuda, form):
    """Reference gin.py:59-62 / gat.py:87-90: the model accepts adj_t (compile=False path)."""
    b = synth.make_batch(16, seed=21, sizes="lognormal")
    ours, _ = make_pair([128, 128, 128])
    ours = ours.to(cuda).eval()
    ei = b.edge_index.to(cuda)
    if form == "torch_sparse":
        adj = FakeSparseTensor(ei)
    else:
        n = b.num_nodes
        adj = torch.sparse_coo_tensor(torch.stack([ei[1], ei[0]]),
                                      torch.ones(ei.size(1), device=cuda), (n, n)).coalesce()
        adj = adj.to_sparse_csr()
    want = ours(b.x.to(cuda), ei, b.batch.to(cuda))
    got = ours(b.x.to(cuda), adj, b.batch.to(cuda))
    torch.testing.assert_close(got, want, atol=1e-5, rtol=1e-5)


def test_tile_open_flags(cuda):
    """Graph-build tile flags == the standalone lgnn_tile_open, and == a CPU recomputation."""
    from lesion_gnn_amd import _lib
    sizes = [64, 64, 30, 34, 64, 100, 28, 64, 1]
    b = synth.make_batch(len(sizes), k=6, d_in=8, seed=22, sizes=sizes)
    g = Graph(b.edge_index.to(cuda), b.num_nodes)
    nt = (b.num_nodes + 63) // 64
    got_all = g.tile_open("gcn").cpu()
    # barrier words, then the partial-slot skip words (zero after a build)
    assert got_all.numel() == nt + _lib.LGNN_TILE_OPEN_EXTRA
    assert got_all[nt + 1:].tolist() == [0] * (_lib.LGNN_TILE_OPEN_EXTRA - 1)
    got = got_all[:nt + 1]
    c = g.csr("gcn")
    ref_t = torch.empty_like(got_all, device=cuda)
    _lib.call("lgnn_tile_open", c.rowptr.data_ptr(), c.col.data_ptr(), b.num_nodes,
              ref_t.data_ptr(), _lib.stream())
    assert torch.equal(got_all, ref_t.cpu())
    src, dst = b.edge_index
    want = torch.zeros_like(got)
    cross = (src // 64) != (dst // 64)
    want[(src[cross] // 64)] = 1
    want[(dst[cross] // 64)] = 1
    want[-1] = int(want[:-1].sum())  # trailing entry: the number of open tiles
    assert torch.equal(got, want)
    # all tiles closed: count 0 (the masked launches return at once)
    b2 = synth.make_batch(4, n=64, k=6, d_in=8, seed=23)
    assert Graph(b2.edge_index.to(cuda), b2.num_nodes).tile_open("gcn").cpu().tolist()[:5] == [0] * 5


@pytest.mark.parametrize("bwd", ["f32", "s3", "s3f"])
@pytest.mark.parametrize("case", ["c2_L2", "irregular_L2", "irregular_L1_add", "dense_tiles",
                                  "wide_tiles", "c2_L3", "irregular_L3"])
def test_gcn_fused_backward(cuda, case, bwd, monkeypatch):
    """lgnn_gcn_stack_bwd (closed tiles, fused) + masked accumulating layer-wise backward (open
    tiles) vs the layer-wise backward and the oracle. dense_tiles: 64-node graphs with k = 40
    (2560 CSR entries per tile > the 2048 a closed tile takes) are flagged open by the graph
    build. wide_tiles: k = 20 and k = 32 (1280 and 2048 entries: closed tiles whose entries past
    the 1024 staged in registers are read from the CSR as the tile's Â is built).
    c2_L3: three convs (fp32: layer-wise backward on recomputed aggregates; split-3: fused).
    irregular_L3: three convs on graphs that straddle tiles (split-3: the layer-major kernels,
    the open tiles then run in separate launches).
    bwd: the fp32 fused kernel (lgnn_gcn_stack_bwd), the split-3 layer-major kernels
    (lgnn_gcn_stack_bwd_s3) or the fused split-3 kernel (lgnn_gcn_stack_bwd_s3f; c2_L3: the
    single-launch entry with three conv layers' dW in the kernel and the in_proj weight gradient
    as a split-3 GEMM on the dZ_0 it writes)."""
    pool = "add" if case.endswith("add") else "mean"
    hidden = [128, 128] if "L1" in case else [128] * 4 if "L3" in case else [128, 128, 128]
    if case.startswith("c2"):
        b = synth.make_batch(300, n=64, k=8, d_in=128, seed=31)
    elif case == "dense_tiles":
        b = synth.make_batch(6, n=64, k=40, d_in=128, seed=32, sizes=[64, 64, 30, 34, 64, 64])
    elif case == "wide_tiles":
        b1 = synth.make_batch(3, n=64, k=20, d_in=128, seed=34)
        b2 = synth.make_batch(3, n=64, k=32, d_in=128, seed=35)
        b = synth.Batch(torch.cat([b1.x, b2.x]),
                        torch.cat([b1.edge_index, b2.edge_index + b1.num_nodes], 1),
                        torch.cat([b1.batch, b2.batch + 3]), None, torch.cat([b1.y, b2.y]),
                        None, 6)
    else:
        b = synth.make_batch(9, k=6, d_in=128, seed=33, sizes=[1, 5, 64, 200, 2, 33, 512, 17, 64])
    ours, oref = make_pair(hidden, pool=pool)
    ours = ours.to(cuda)
    monkeypatch.setattr(ops, "BWD_MODE", bwd)
    monkeypatch.setattr(ops, "BWD_S3", bwd != "f32")
    if case in ("dense_tiles", "wide_tiles"):
        g = Graph(b.edge_index.to(cuda), b.num_nodes)
        want = [1, 1, 1, 1, 1, 5] if case == "dense_tiles" else [0, 0, 0, 0, 0, 0]
        assert g.tile_open("gcn").cpu().tolist()[:6] == want
    monkeypatch.setattr(ops, "FUSED_BWD", True)
    lf, _, gf = run_step(ours, b, cuda)
    monkeypatch.setattr(ops, "FUSED_BWD", False)
    ll, _, gl = run_step(ours, b, cuda)
    lr_, _, gr = run_step(oref, b, "cpu")
    assert torch.equal(lf, ll)
    torch.testing.assert_close(lf, lr_, atol=1e-4, rtol=0)
    for k in gr:
        torch.testing.assert_close(gf[k], gl[k], atol=1e-6, rtol=1e-5, msg=lambda m: f"{k}: {m}")
        torch.testing.assert_close(gf[k], gr[k], atol=1e-5, rtol=1e-4, msg=lambda m: f"{k}: {m}")
    monkeypatch.setattr(ops, "FUSED_BWD", True)
    _, _, gf2 = run_step(ours, b, cuda)
    for k in gf:
        assert torch.equal(gf[k], gf2[k]), k


@pytest.mark.parametrize("convs", [2, 3])
@pytest.mark.parametrize("open_in_fused", [True, False])
def test_open_tiles_in_fused_launch(cuda, open_in_fused, convs, monkeypatch):
    """Open tiles (graphs straddling 64-node tiles, an over-capacity tile) processed inside the
    fused split-3 launches (layer by layer behind grid barriers) == the separate layer-wise
    launches == the oracle; the same Graph reused for a second step (the barrier words re-arm
    themselves: every word back to 0, no barrier gave up). convs = 3: the open phase gathers the
    open tiles' dZ_0 rows for the in_proj GEMM (layer-major s3 backward without open_in_fused)."""
    from lesion_gnn_amd.graph import Graph

    monkeypatch.setattr(ops, "OPEN_IN_FUSED", open_in_fused)
    monkeypatch.setattr(ops, "OPEN_IN_FUSED_BWD", open_in_fused)
    sizes = [1, 5, 64, 200, 2, 33, 512, 17, 64, 64, 30, 34]
    b = synth.make_batch(len(sizes), k=6, d_in=128, seed=41, sizes=sizes)
    ours, oref = make_pair([128] * (convs + 1))
    ours = ours.to(cuda)
    g = Graph(b.edge_index.to(cuda), b.num_nodes, b.batch.to(cuda), b.num_graphs)
    nt = (b.num_nodes + 63) // 64
    results = []
    for _ in range(2):
        logits = ours(b.x.to(cuda), g, b.batch.to(cuda), b.num_graphs)
        loss = torch.nn.functional.cross_entropy(logits, b.y.to(cuda))
        ours.zero_grad(set_to_none=True)
        loss.backward()
        results.append((logits.detach().cpu(),
                        {k: p.grad.detach().cpu() for k, p in ours.named_parameters()}))
        words = g.tile_open("gcn_lazy" if ops.LAZY_TRANSPOSE else "gcn").cpu().tolist()
        assert words[nt] > 0  # this batch has open tiles
        assert words[nt + 1:nt + 7] == [0] * 6, words[nt:nt + 7]  # barrier words re-armed
        assert g.barrier_timeouts("gcn_lazy" if ops.LAZY_TRANSPOSE else "gcn") == 0
    lr_, _, gr = run_step(oref, b, "cpu")
    for lo, go in results:
        torch.testing.assert_close(lo, lr_, atol=1e-4, rtol=0)
        for k in gr:
            torch.testing.assert_close(go[k], gr[k], atol=1e-5, rtol=1e-4,
                                       msg=lambda m: f"{k}: {m}")
    assert torch.equal(results[0][0], results[1][0])


@pytest.mark.parametrize("classes,pool,convs", [(5, "mean", 2), (8, "add", 2), (12, "mean", 2),
                                                (8, "add", 3), (12, "mean", 3)])
def test_head_backward_folded_into_stack(cuda, classes, pool, convs, monkeypatch):
    """out_proj backward folded into the single split-3 backward launch (dP = dlogits W_out
    formed in the pool prologue of closed tiles and in the open-tile phase, dW_out / db_out as
    jobs of the slab reduction; <= 8 classes, 12 falls back to lgnn_pool_head_bwd) and the same
    step with the fold off: both == the oracle."""
    from lesion_gnn_amd.graph import Graph

    monkeypatch.setattr(ops, "OPEN_IN_FUSED", "1")
    monkeypatch.setattr(ops, "OPEN_IN_FUSED_BWD", "1")
    sizes = [1, 5, 64, 200, 2, 33, 512, 17, 64, 64, 30, 34] * 3
    b = synth.make_batch(len(sizes), k=6, d_in=128, seed=43, sizes=sizes)
    b.y = b.y % classes
    ours, oref = make_pair([128] * (convs + 1), classes=classes, pool=pool)
    ours = ours.to(cuda)
    if ops.BWD_S3:
        g = Graph(b.edge_index.to(cuda), b.num_nodes, b.batch.to(cuda), b.num_graphs)
        assert ops.head_in_stack_bwd(g, convs, classes, True) == (classes <= 8)
    results = []
    for fold in (True, False):
        monkeypatch.setattr(ops, "HEAD_FOLD", fold)
        results.append(run_step(ours, b, cuda, b.num_graphs))
    lr_, _, gr = run_step(oref, b, "cpu", b.num_graphs)
    for lo, _, go in results:
        torch.testing.assert_close(lo, lr_, atol=1e-4, rtol=0)
        for k in gr:
            torch.testing.assert_close(go[k], gr[k], atol=1e-5, rtol=1e-4,
                                       msg=lambda m: f"{k}: {m}")



@pytest.mark.parametrize("case", ["aligned", "ragged", "capacity"])
def test_lazy_transpose_build(cuda, case):
    """lgnn_graph_build_lazy (the fused GCN stack's build): the target CSR and the tile flags
    (cross edges marked in the count pass, the > 2048-entry capacity rule in the scan) equal the
    full build's bit for bit; the source CSR (tptr / tidx / tw) is built exactly when some tile
    is open (ragged graphs, dense tiles) and then equals the full build's (aligned k-NN input
    takes the target-sorted path, which leaves it unwritten)."""
    if case == "aligned":
        b = synth.make_batch(64, n=64, k=8, d_in=8, seed=51)
    elif case == "ragged":
        b = synth.make_batch(9, k=6, d_in=8, seed=52, sizes=[1, 5, 64, 200, 2, 33, 512, 17, 64])
    else:
        b = synth.make_batch(6, n=64, k=40, d_in=8, seed=53, sizes=[64, 64, 64, 64, 64, 64])
    g = Graph(b.edge_index.to(cuda), b.num_nodes)
    g.keep_build_workspace = True  # build_path() below
    full, lazy = g.csr("gcn"), g.csr("gcn_lazy")
    nnz = int(full.rowptr[-1])  # arrays have capacity E + N; entries past nnz are unused
    for name in ("rowptr", "err"):
        assert torch.equal(getattr(full, name), getattr(lazy, name)), name
    for name in ("col", "w"):
        assert torch.equal(getattr(full, name)[:nnz], getattr(lazy, name)[:nnz]), name
    to_full, to_lazy = g.tile_open("gcn").cpu(), g.tile_open("gcn_lazy").cpu()
    assert torch.equal(to_full, to_lazy)
    nt = (b.num_nodes + 63) // 64
    n_open = int(to_lazy[nt])
    assert (n_open == 0) == (case == "aligned")
    assert g.build_path("gcn_lazy") == {"aligned": "sorted", "ragged": "sorted_open",
                                        "capacity": "general"}[case]
    if n_open:
        assert int(full.tptr[-1]) == nnz
        assert torch.equal(full.tptr, lazy.tptr)
        assert torch.equal(full.tidx[:nnz], lazy.tidx[:nnz])
        assert torch.equal(full.tw[:nnz], lazy.tw[:nnz])


def test_fused_grid_capacity(cuda):
    """The open-tile phase of the fused split-3 launches runs behind grid barriers, so every
    workgroup must be resident: the device's capacity (occupancy x CUs) covers both launches'
    largest grids on MI355X (forward 512, backward lgnn_gcn_stack_bwd_partials), so
    _open_in_fused keeps the one-launch path there; a smaller capacity turns it off."""
    from lesion_gnn_amd import _lib
    from lesion_gnn_amd.graph import Graph

    fwd = ops.fused_grid_capacity("fwd", cuda)
    bwd = ops.fused_grid_capacity("bwd", cuda)
    assert fwd >= 512 and bwd >= _lib.load().lgnn_gcn_stack_bwd_partials(1 << 20), (fwd, bwd)
    b = synth.make_batch(64, k=8, d_in=128, seed=3)
    g = Graph(b.edge_index.to(cuda), b.num_nodes, b.batch.to(cuda), b.num_graphs)
    assert ops._open_in_fused("auto", g, "fwd") and ops._open_in_fused("auto", g, "bwd")
    ops._CAPACITY[("fwd", torch.device(cuda).index)] = 1
    try:
        assert not ops._open_in_fused("auto", g, "fwd")
    finally:
        ops._CAPACITY.clear()
