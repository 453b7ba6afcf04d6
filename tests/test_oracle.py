"""Pins the CPU oracle (oracle/pyg_ref.py) with known answers: analytic identities of the PyG
operators and the only fixture the reference holds (GaussianDistance KATs, reference
test/test_transforms.py:20,29,38, rtol = atol = 1e-3 as there). Also checks the synthetic
generator's k-NN topology bit-exactly against the oracle's restatement."""
import math

import pytest
import torch

import oracle.pyg_ref as ref
from lesion_gnn_amd import synth


def small_graph(seed=0, n=12, k=4):
    g = torch.Generator().manual_seed(seed)
    pos = torch.rand(n, 2, generator=g, dtype=torch.float64)
    return pos, ref.knn_graph(pos, k, loop=True)


def test_knn_graph_structure():
    pos, ei = small_graph()
    n, k = 12, 4
    assert ei.shape == (2, n * k)
    assert torch.equal(ei[1], torch.arange(n).repeat_interleave(k))  # grouped by query
    assert torch.equal(ei[0][::k], torch.arange(n))  # self is the nearest
    d = ((pos[ei[0]] - pos[ei[1]]) ** 2).sum(-1).view(n, k)
    assert (d[:, 1:] >= d[:, :-1]).all()


def test_synth_knn_matches_oracle_bitexact():
    b = synth.make_batch(6, n=20, k=8, d_in=4, seed=3, sizes=[20, 5, 1, 20, 9, 33])
    for g in range(b.num_graphs):
        lo, hi = int(b.ptr[g]), int(b.ptr[g + 1])
        want = ref.knn_graph(b.pos[lo:hi], 8, loop=True) + lo
        mask = (b.edge_index[1] >= lo) & (b.edge_index[1] < hi)
        assert torch.equal(b.edge_index[:, mask], want)
    b2 = synth.make_batch(3, n=15, k=5, d_in=4, seed=4, loop=False)
    want = torch.cat([ref.knn_graph(b2.pos[15 * g:15 * (g + 1)], 5, loop=False) + 15 * g
                      for g in range(3)], 1)
    assert torch.equal(b2.edge_index, want)


def test_gcn_norm_regular_knn_is_one_over_k():
    _, ei = small_graph(k=6)
    ei2, w = ref.gcn_norm(ei, 12)
    assert ei2.size(1) == ei.size(1)  # loops already present: none added
    torch.testing.assert_close(w, torch.full_like(w, 1 / 6), rtol=1e-6, atol=0)
    # loops moved to the end
    assert torch.equal(ei2[0, -12:], torch.arange(12)) and torch.equal(ei2[1, -12:],
                                                                      torch.arange(12))


def test_gcn_norm_isolated_node_and_missing_loops():
    ei = torch.tensor([[0, 1], [1, 0]])
    ei2, w = ref.gcn_norm(ei, 3)  # node 2 isolated: only its loop, deg 1
    assert ei2.size(1) == 5
    torch.testing.assert_close(w, torch.tensor([0.5, 0.5, 0.5, 0.5, 1.0]))


def test_gat_softmax_rows_sum_to_one():
    torch.manual_seed(0)
    _, ei = small_graph(k=5)
    conv = ref.GATConv(8, 4, heads=3)
    x = torch.randn(12, 8)
    xs = conv.lin(x).view(-1, 3, 4)
    a_s, a_d = (xs * conv.att_src).sum(-1), (xs * conv.att_dst).sum(-1)
    e = ref.add_self_loops(ref.remove_self_loops(ei), 12)
    alpha = ref.edge_softmax(torch.nn.functional.leaky_relu(a_s[e[0]] + a_d[e[1]], 0.2), e[1], 12)
    s = ref.scatter_sum(alpha, e[1], 12)
    torch.testing.assert_close(s, torch.ones_like(s))


def test_gin_self_loops_only_is_mlp_of_2x():
    torch.manual_seed(0)
    n = 7
    ei = torch.stack([torch.arange(n), torch.arange(n)])
    mlp = ref.MLP([5, 6, 6]).eval()
    conv = ref.GINConv(mlp)
    x = torch.randn(n, 5)
    torch.testing.assert_close(conv(x, ei), mlp(2 * x))


def test_pools():
    x = torch.full((9, 3), 2.5)
    batch = torch.tensor([0, 0, 0, 1, 1, 3, 3, 3, 3])
    m = ref.global_mean_pool(x, batch)
    assert m.shape == (4, 3)
    torch.testing.assert_close(m[[0, 1, 3]], torch.full((3, 3), 2.5))
    assert (m[2] == 0).all()  # empty graph -> 0 (count clamped to 1)
    a = ref.global_add_pool(x, batch)
    torch.testing.assert_close(a[:, 0], torch.tensor([7.5, 5.0, 0.0, 10.0]))


@pytest.mark.parametrize("model", ["gcn", "gin", "gat"])
def test_models_permutation_equivariant_within_graph(model):
    torch.manual_seed(0)
    b = synth.make_batch(3, n=10, k=4, d_in=16, seed=1)
    if model == "gcn":
        m = ref.GCN(16, [16, 16, 16], 5, 0.0)
    elif model == "gin":
        m = ref.GIN(16, [16, 16, 16], 5, 0.0)
    else:
        m = ref.GAT(16, [16, 16], 5, heads=2, dropout=0.0)
    m.eval()
    out = m(b.x, b.edge_index, b.batch)
    perm = torch.cat([torch.randperm(10) + 10 * g for g in range(3)])
    inv = torch.empty_like(perm)
    inv[perm] = torch.arange(30)
    out2 = m(b.x[perm], inv[b.edge_index], b.batch[perm])
    torch.testing.assert_close(out, out2, atol=1e-5, rtol=1e-5)


def test_gaussian_distance_reference_kats():
    """Reference test/test_transforms.py:20,29,38 (sigma 1, 0.5, 2 at d = 1)."""
    ei = torch.tensor([[0, 1], [1, 0]])
    pos = torch.tensor([[0.0, 0.0], [1.0, 0.0]])
    for sigma, want in [(1.0, 0.2420), (0.5, 0.1080), (2.0, 0.1760)]:
        w = ref.gaussian_distance(ei, pos, sigma)
        torch.testing.assert_close(w, torch.tensor([want, want]), rtol=1e-3, atol=1e-3)
    assert math.isclose(ref.gaussian_distance(ei, pos, 1.0)[0].item(),
                        math.exp(-0.5) / math.sqrt(2 * math.pi), rel_tol=1e-6)


def test_criterion_regression_clamp():
    logits = torch.tensor([[-1.0], [2.0], [9.0]])
    y = torch.tensor([0, 2, 4])
    assert ref.criterion("MSE", logits, y, 5).item() == 0.0


def test_graphconv_oracle_dense_form():
    """oracle GraphConv == dense A_w X W_rel^T + b_rel + X W_root^T (A_w[i, j] = sum of the
    weights of edges j -> i, duplicates and self loops included as given)."""
    torch.manual_seed(0)
    n, K, N = 7, 5, 3
    ei = torch.tensor([[0, 1, 2, 3, 3, 6, 5, 4, 4], [1, 0, 0, 2, 2, 6, 4, 5, 0]])
    w = torch.rand(ei.size(1), dtype=torch.float64)
    x = torch.randn(n, K, dtype=torch.float64)
    conv = ref.GraphConv(K, N).double()
    A = torch.zeros(n, n, dtype=torch.float64)
    for e in range(ei.size(1)):
        A[ei[1, e], ei[0, e]] += w[e]
    want = A @ x @ conv.lin_rel.weight.T + conv.lin_rel.bias + x @ conv.lin_root.weight.T
    torch.testing.assert_close(conv(x, ei, w), want)
    A1 = (A > 0).double() * 0
    for e in range(ei.size(1)):
        A1[ei[1, e], ei[0, e]] += 1
    want1 = A1 @ x @ conv.lin_rel.weight.T + conv.lin_rel.bias + x @ conv.lin_root.weight.T
    torch.testing.assert_close(conv(x, ei), want1)


def test_sort_aggregation_known_answer():
    """PyG SortAggregation semantics (reference drgnet.py:37,59): rows by last channel
    descending, ties in node order, top k, short graphs zero-padded, x.min()-1 fill zeroed."""
    x = torch.tensor([[1., 5.], [2., 7.], [3., 5.], [4., -1.], [9., 0.]])
    batch = torch.tensor([0, 0, 0, 1, 1])
    out = ref.sort_aggregation(x, batch, 3).view(2, 3, 2)
    assert torch.equal(out[0], torch.tensor([[2., 7.], [1., 5.], [3., 5.]]))
    assert torch.equal(out[1], torch.tensor([[9., 0.], [4., -1.], [0., 0.]]))
    out2 = ref.sort_aggregation(x, batch, 2).view(2, 2, 2)
    assert torch.equal(out2[0], torch.tensor([[2., 7.], [1., 5.]]))


def test_extract_features_by_cc_known_answer():
    """lesions.py:88-93: per-label mean / max over the (H*W, C) view of (1, C, H, W)."""
    feats = torch.arange(8, dtype=torch.float32).view(1, 2, 2, 2)  # c0: 0..3, c1: 4..7
    cc = torch.tensor([[0, 1], [1, 0]])
    mean = ref.extract_features_by_cc(cc, feats, 2, "mean")
    assert torch.equal(mean, torch.tensor([[1.5, 5.5], [1.5, 5.5]]))
    mx = ref.extract_features_by_cc(cc, feats, 2, "max")
    assert torch.equal(mx, torch.tensor([[3., 7.], [2., 6.]]))
    assert torch.equal(ref.extract_features_by_cc(cc, feats, 1), feats.mean((2, 3)))


def _radius_loop(pos, r, loop, max_nb):
    """torch_cluster 1.6.3 radius_cuda.cu's per-query walk, literally (one graph): candidates in
    index order, taken while the squared distance < r * r, at most `limit`; radius_graph then
    swaps to (source, target) and drops the self pair without loop."""
    n = pos.size(0)
    limit = max_nb if loop else max_nb + 1
    rows, cols = [], []
    for q in range(n):
        count = 0
        for c in range(n):
            d = float(((pos[q] - pos[c]) ** 2).sum())
            if d < r * r:
                if loop or c != q:
                    rows.append(c)
                    cols.append(q)
                count += 1
            if count >= limit:
                break
    return torch.tensor([rows, cols], dtype=torch.long).view(2, -1)


@pytest.mark.parametrize("seed,n,r,loop,max_nb", [(0, 40, 0.3, False, 32), (1, 90, 0.5, False, 8),
                                                 (2, 50, 0.2, True, 32), (3, 7, 10.0, True, 3),
                                                 (4, 1, 1.0, False, 32), (5, 64, 0.0, False, 32)])
def test_radius_graph_oracle_matches_literal_walk(seed, n, r, loop, max_nb):
    g = torch.Generator().manual_seed(seed)
    pos = torch.rand(n, 2, generator=g, dtype=torch.float64)
    assert torch.equal(ref.radius_graph(pos, r, loop, max_nb), _radius_loop(pos, r, loop, max_nb))


def test_radius_graph_known_answers():
    """Points on a line at 0..9: r = 1.5 links neighbours at distance 1 only; r = 1 links nothing
    (the comparison is strict); 40 coincident points with the default cap (32, no loop): the walk
    takes the first 33 in index order, so nodes 0..32 keep 32 neighbours (their self pair was
    among the 33 and is dropped) and nodes 33..39 keep 33 (torch_cluster's behaviour)."""
    line = torch.stack([torch.arange(10, dtype=torch.float64), torch.zeros(10, dtype=torch.float64)], 1)
    ei = ref.radius_graph(line, 1.5)
    want = sorted([(q - 1, q) for q in range(1, 10)] + [(q + 1, q) for q in range(9)],
                  key=lambda e: (e[1], e[0]))
    assert ei.t().tolist() == [list(e) for e in want]
    assert ref.radius_graph(line, 1.0).numel() == 0
    same = torch.zeros(40, 2, dtype=torch.float64)
    ei = ref.radius_graph(same, 1.0)
    cnt = torch.bincount(ei[1], minlength=40)
    assert cnt.tolist() == [32] * 33 + [33] * 7
    assert ei[0][ei[1] == 35].tolist() == list(range(33))  # the first 33 in index order
