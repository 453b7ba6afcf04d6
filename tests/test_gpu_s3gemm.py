"""GPU: the split-3 dense GEMMs (s3gemm.hip: lgnn_s3_gemm / lgnn_s3_wgrad / lgnn_s3_weight_planes)
that replaced the library GEMMs on the fp32 in_proj (nn.Linear(1025, 128), reference gat.py:29 —
the reference's own experiment trains it in fp32, configs/config.py:52-65) and on every lin wider
than 128 (the sweep's widths, scripts/sweep.py:126).

Accuracy bar (fp32 mode): against a float64 restatement, the kernel's error is at most 4x that of
torch's own fp32 CPU GEMM on the same operands (whose blocked summation is unusually accurate),
or the statistical error of fp32 accumulation, 2^-24 sqrt(K) max_ij sum_k |a_ik||b_kj| — i.e.
fp32-class (the split-3 products themselves are exact to 2^-24).
bf16 mode (planes = 1): equal to a float64 GEMM of the RNE-rounded operands within fp32
accumulation error (2e-6 of the scale). Shapes: the C3 / reference-config in_proj at full size
(42,279 x 1025 -> 128), ragged M, K % 4 != 0, K < 64, N > 128 in 128-column blocks, N odd.
"""
import pytest
import torch

from lesion_gnn_amd import ops

pytestmark = pytest.mark.gpu


def _bound(ref64, torch32, absprod=None):
    err_t = (torch32.double() - ref64).abs().max().item()
    acc = 0.0
    if absprod is not None:
        K, mag = absprod
        acc = 2.0 ** -24 * K ** 0.5 * mag
    return max(4 * err_t, acc) + 1e-7 * ref64.abs().max().item()


def _mag(A, B):
    """max_ij sum_k |A_ik| |B_kj| (the accumulation error's scale)."""
    return (A.abs().double() @ B.abs().double()).max().item()


SHAPES = [(42279, 1025, 128), (1000, 1025, 128), (333, 256, 512), (130, 37, 300), (64, 128, 256),
          (7, 5, 3), (257, 64, 130)]


@pytest.mark.parametrize("M,K,N", SHAPES)
def test_s3_gemm_forward(cuda, M, K, N):
    g = torch.Generator().manual_seed(M + K + N)
    A = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g)
    want64 = A.double() @ W.double().T + b.double()
    got = ops.dense_mm(A.to(cuda), ops.dense_planes(W.to(cuda), False, False), N, b.to(cuda),
                       False).cpu()
    err = (got.double() - want64).abs().max().item()
    assert err <= _bound(want64, A @ W.T + b, (K, _mag(A, W.T))), err
    # Y = A W (the transposed operand: dX = dY W of a backward)
    Wt = torch.randn(K, N, generator=g) / K ** 0.5  # W^T-shaped weight [K][N] -> Y [M][N]
    want64 = A.double() @ Wt.double()
    got = ops.dense_mm(A.to(cuda), ops.dense_planes(Wt.to(cuda), True, False), N, None,
                       False).cpu()
    assert (got.double() - want64).abs().max().item() <= _bound(want64, A @ Wt, (K, _mag(A, Wt)))


@pytest.mark.parametrize("M,K,N", SHAPES)
def test_s3_wgrad_and_bias_grad(cuda, M, K, N):
    g = torch.Generator().manual_seed(7 * M + K + N)
    dY = torch.randn(M, N, generator=g)
    X = torch.randn(M, K, generator=g)
    dW, db = ops.dense_wgrad(dY.to(cuda), X.to(cuda), False, want_db=True)
    want64 = dY.double().T @ X.double()
    err = (dW.cpu().double() - want64).abs().max().item()
    assert err <= _bound(want64, dY.T @ X, (M, _mag(dY.T, X))), err
    db64 = dY.double().sum(0)
    assert (db.cpu().double() - db64).abs().max().item() <= \
        3 * (dY.sum(0).double() - db64).abs().max().item() + 1e-6 * db64.abs().max().item()
    again, _ = ops.dense_wgrad(dY.to(cuda), X.to(cuda), False)
    assert torch.equal(again, dW)  # fixed-order reduction: deterministic


@pytest.mark.parametrize("M,K,N", [(1000, 1025, 128), (333, 256, 512), (130, 37, 300)])
def test_bf16_plane_mode(cuda, M, K, N):
    """planes = 1: bf16 RNE operands (torch's .to(bfloat16)), fp32 accumulation — the bf16 GEMM
    semantics of the oracle's _Bf16Linear, for widths the bf16 tile kernel does not take."""
    g = torch.Generator().manual_seed(M * 3 + N)
    A = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) / K ** 0.5
    r16 = lambda t: t.to(torch.bfloat16).double()
    want = r16(A) @ r16(W).T
    got = ops.dense_mm(A.to(cuda), ops.dense_planes(W.to(cuda), False, True), N, None, True).cpu()
    assert (got.double() - want).abs().max().item() <= 2e-6 * want.abs().max().item()
    dY = torch.randn(M, N, generator=g)
    dW, _ = ops.dense_wgrad(dY.to(cuda), A.to(cuda), True)
    want = r16(dY).T @ r16(A)
    assert (dW.cpu().double() - want).abs().max().item() <= 2e-6 * want.abs().max().item()


@pytest.mark.parametrize("K,N,bf16", [(1025, 128, False), (128, 256, False), (96, 512, True)])
def test_dense_linear_autograd(cuda, K, N, bf16):
    """_DenseLinear (linear_auto's path for these shapes) forward + backward vs float64 autograd
    (bf16: vs the oracle's bf16-operand semantics, 1e-3 relative)."""
    import oracle.pyg_ref as ref

    g = torch.Generator().manual_seed(K + N)
    M = 777
    x = torch.randn(M, K, generator=g, dtype=torch.float64)
    W = torch.randn(N, K, generator=g, dtype=torch.float64) / K ** 0.5
    b = torch.randn(N, generator=g, dtype=torch.float64)
    dy = torch.randn(M, N, generator=g, dtype=torch.float64)
    xr, Wr, br = (t.clone().requires_grad_() for t in (x, W, b))
    if bf16:
        y = ref.linear(xr.float(), Wr.float(), br.float(), True).double()
    else:
        y = xr @ Wr.T + br
    y.backward(dy)
    xg, Wg, bg = (t.float().to(cuda).requires_grad_() for t in (x, W, b))
    yg = ops.linear_auto(xg, Wg, bg, bf16)
    yg.backward(dy.float().to(cuda))
    tol = 1e-3 if bf16 else 2e-6
    for got, want in ((yg, y), (xg.grad, xr.grad), (Wg.grad, Wr.grad), (bg.grad, br.grad)):
        err = (got.detach().cpu().double() - want.detach()).abs().max().item()
        assert err <= tol * want.abs().max().item(), (err, want.abs().max().item())


def test_no_library_gemm_in_gat_fp32_step(cuda):
    """The fp32 GAT step (d_in 1025, the reference model) launches no vendor-library GEMM: every
    kernel of forward + backward is one of liblgnn.so's (profiled by name)."""
    from torch.profiler import ProfilerActivity, profile

    from lesion_gnn_amd import synth
    from lesion_gnn_amd.models import GAT

    torch.manual_seed(0)
    m = GAT(1025, [128] * 4, 1, heads=2, dropout=0.35).to(cuda).train()
    b = synth.make_batch(64, k=6, d_in=1025, seed=2, sizes="lognormal",
                         last_channel_class=True).to(cuda)
    m(b.x, b.edge_index, b.batch, b.num_graphs).sum().backward()  # warm-up
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        m(b.x, b.edge_index, b.batch, b.num_graphs).sum().backward()
        torch.cuda.synchronize()
    names = {e.name for e in prof.events() if e.device_type.name == "CUDA"}
    lib = [n for n in names if n.startswith(("Cijk", "Custom_Cijk")) or "gemm" in n.lower()
           and "lgnn" not in n and "k_" not in n]
    assert not lib, sorted(lib)
    assert any("k_s3_gemm" in n for n in names), sorted(names)  # the in_proj ran on ours
    assert any("k_s3_wgrad" in n for n in names), sorted(names)


def test_weight_bundle_equals_per_gemm_planes(cuda):
    """ops.s3_weight_bundle (one lgnn_s3_weight_planes_multi launch, more than 16 operands split
    over launches) writes, per (W, transposed), exactly dense_planes' bytes."""
    g = torch.Generator().manual_seed(5)
    shapes = [(128, 1025), (128, 128), (256, 128), (300, 37), (5, 3)] * 4  # 20 operands
    Ws = [torch.randn(r, c, generator=g).to(cuda) for r, c in shapes]
    specs = [(W, i % 2 == 1) for i, W in enumerate(Ws)]
    for bf16 in (False, True):
        views = ops.s3_weight_bundle(specs, bf16)
        for (W, t), v in zip(specs, views):
            assert torch.equal(v, ops.dense_planes(W, t, bf16))


@pytest.mark.parametrize("compiled", [False, True])
def test_gat_weight_bundle_bitwise(cuda, monkeypatch, compiled):
    """The fp32 GAT step with its weight operands from one bundle launch (GAT.weight_planes) is
    bit-identical to one plane launch per GEMM — eager and compiled (the bundle rides through the
    lgnn:: custom ops)."""
    from lesion_gnn_amd import synth
    from lesion_gnn_amd.models import GAT
    from lesion_gnn_amd.models import gat as gat_mod

    torch.manual_seed(0)
    b = synth.make_batch(48, k=6, d_in=1025, seed=2, sizes="lognormal",
                         last_channel_class=True).to(cuda)
    m = GAT(1025, [128] * 4, 1, heads=2, dropout=0.35).to(cuda).train()
    run = torch.compile(m, dynamic=True) if compiled else m
    rng = m._dropout_rng.clone()
    res = []
    for bundle in (True, False):
        monkeypatch.setattr(gat_mod, "WEIGHT_BUNDLE", bundle)
        torch._dynamo.reset()
        m._dropout_rng.copy_(rng)
        out = run(b.x, b.edge_index, b.batch, b.num_graphs)
        m.zero_grad(set_to_none=True)
        out.square().sum().backward()
        res.append((out.detach().cpu(), {n: p.grad.detach().cpu() for n, p in m.named_parameters()}))
    assert torch.equal(res[0][0], res[1][0])
    for n in res[0][1]:
        assert torch.equal(res[0][1][n], res[1][1][n]), n


@pytest.mark.parametrize("heads,C,K", [(2, 64, 1025), (4, 32, 128), (1, 128, 128), (8, 8, 37)])
def test_s3_gemm_att_scores(cuda, heads, C, K):
    """lgnn_s3_gemm_att (the fp32 GATConv.lin with the attention scores in its epilogue): Y equals
    lgnn_s3_gemm's bit for bit, and a_s / a_d (one fmaf chain per row and head) match
    lgnn_gat_att's (dot4 + butterfly sums) within fp32 summation error."""
    from lesion_gnn_amd import _lib

    g = torch.Generator().manual_seed(heads * 100 + C)
    M, N = 777, heads * C
    A = torch.randn(M, K, generator=g).to(cuda)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(cuda)
    att_s = torch.randn(N, generator=g).to(cuda)
    att_d = torch.randn(N, generator=g).to(cuda)
    wp = ops.dense_planes(W, False, False)
    Y = torch.empty(M, N, device=cuda)
    a_s = torch.empty(M, heads, device=cuda)
    a_d = torch.empty(M, heads, device=cuda)
    _lib.call("lgnn_s3_gemm_att", A.data_ptr(), M, K, wp.data_ptr(), N, 3, Y.data_ptr(),
              att_s.data_ptr(), att_d.data_ptr(), heads, C, a_s.data_ptr(), a_d.data_ptr(),
              _lib.stream())
    assert torch.equal(Y, ops.dense_mm(A, wp, N, None, False))
    r_s = torch.empty_like(a_s)
    r_d = torch.empty_like(a_d)
    _lib.call("lgnn_gat_att", Y.data_ptr(), M, heads, C, att_s.data_ptr(), att_d.data_ptr(),
              r_s.data_ptr(), r_d.data_ptr(), _lib.stream())
    for got, want in ((a_s, r_s), (a_d, r_d)):
        scale = (Y.view(M, heads, C).abs() * att_s.view(heads, C).abs()).sum(-1).max().item()
        assert (got - want).abs().max().item() <= 2e-6 * scale


@pytest.mark.parametrize("bf16", [False, True])
def test_in_proj_past_32bit_offsets(cuda, bf16):
    """the in_proj GEMMs take 32-bit buffer offsets, so a launch over more than
    ~523 k rows of 1025 channels would be refused (LGNN_EINVAL). ops splits such operands into
    row blocks (ops._row_blocks): here M is just above one block (two launches), the rows on
    both sides of the block boundary and the last rows are checked against float64, and the
    weight / bias gradients (partial slabs of both blocks in one fixed-order reduction) against
    float64 over all rows."""
    K, N = 1025, 128
    blocks = ops._row_blocks(10 ** 7, K, N)
    M = blocks[0][1] + 1000  # one block + 1000 rows
    assert len(ops._row_blocks(M, K, N)) == 2
    g = torch.Generator(device=cuda).manual_seed(7)
    A = torch.randn(M, K, device=cuda, generator=g)
    W = torch.randn(N, K, device=cuda, generator=g) / K ** 0.5
    b = torch.randn(N, device=cuda, generator=g)
    if bf16:
        Wb, _ = ops.bf16_weight_operands(W, False)
        Y = ops.bf16_gemm(A, Wb, b, N)[0]
        Ar, Wr = A.bfloat16().double(), W.bfloat16().double()
    else:
        Y = ops.dense_mm(A, ops.dense_planes(W, False, False), N, b, False)
        Ar, Wr = A.double(), W.double()
    r0 = blocks[0][1]
    for rows in (slice(0, 64), slice(r0 - 64, r0 + 64), slice(M - 64, M)):
        want = Ar[rows] @ Wr.T + b.double()
        err = (Y[rows].double() - want).abs().max().item()
        assert err <= (2e-6 if bf16 else 2e-5) * max(1.0, want.abs().max().item()), (rows, err)
    dy = torch.randn(M, N, device=cuda, generator=g) / M ** 0.5
    if bf16:
        dW = ops.bf16_wgrad(dy.bfloat16(), A, N)
        want = dy.bfloat16().double().T @ Ar
        tol = 2e-6
    else:
        dW, db = ops.dense_wgrad(dy, A, False, want_db=True)
        want = dy.double().T @ A.double()
        torch.testing.assert_close(db.double(), dy.double().sum(0), rtol=0, atol=1e-5)
        tol = 2e-5
    err = (dW.double() - want).abs().max().item()
    assert err <= tol * max(1.0, want.abs().max().item()), err
