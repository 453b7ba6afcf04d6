"""GPU parity of the GAT path (reference gat.py:17-59: in_proj -> ELU(GATConv) x L -> mean pool
-> out_proj; BASELINE config C3 shapes: d_in = 1025 (1024 encoder channels + lesion class),
4 heads, h = 128, k = 6, log-normal graph sizes, MSE regression with clamp) vs the CPU oracle.
fp32 tolerances as tests/test_gpu_gcn.py; attention rows checked to sum to 1."""
import pytest
import torch

import oracle.pyg_ref as ref
from lesion_gnn_amd import ops, synth
from lesion_gnn_amd.graph import Graph
from lesion_gnn_amd.models.gat import GAT

pytestmark = pytest.mark.gpu


def make_pair(d_in, hidden, classes, heads, seed=1234, precision="fp32"):
    torch.manual_seed(seed)
    ours = GAT(d_in, hidden, classes, heads=heads, dropout=0.0, precision=precision)
    oref = ref.GAT(d_in, hidden, classes, heads=heads, dropout=0.0, precision=precision)
    oref.load_state_dict(ours.state_dict())
    return ours, oref


def step(model, b, device, loss_kind, classes):
    logits = model(b.x.to(device), b.edge_index.to(device), b.batch.to(device), b.num_graphs)
    loss = ref.criterion(loss_kind, logits, b.y.to(device), classes)
    model.zero_grad(set_to_none=True)
    loss.backward()
    return (logits.detach().cpu(), loss.detach().cpu(),
            {k: p.grad.detach().cpu() for k, p in model.named_parameters()})


def check(ours, oref, b, cuda, loss_kind="MSE", classes=5, tol=1e-4):
    lo, losso, go = step(ours.to(cuda).train(), b, cuda, loss_kind, classes)
    lr_, lossr, gr = step(oref.train(), b, "cpu", loss_kind, classes)
    torch.testing.assert_close(lo, lr_, rtol=0, atol=tol)
    torch.testing.assert_close(losso, lossr, rtol=10 * tol, atol=1e-6)
    for k in gr:
        scale = gr[k].abs().max().item()
        torch.testing.assert_close(go[k], gr[k], rtol=0, atol=max(tol * scale, 1e-6),
                                   msg=lambda m: f"{k}: {m}")


def test_gat_c3_shape(cuda):
    """C3: 3-layer GAT, 4 heads, d_in 1025, lognormal N, k = 6, MSE (256 graphs, fp32)."""
    b = synth.make_batch(256, k=6, d_in=1025, seed=3, sizes="lognormal", last_channel_class=True)
    ours, oref = make_pair(1025, [128] * 4, 1, heads=4)
    check(ours, oref, b, cuda)


def test_gat_c3_bf16(cuda):
    """C3 as BASELINE.json states it (bf16): in_proj and GATConv.lin GEMMs on bf16-rounded
    operands with fp32 accumulation (hipBLASLt), attention/softmax/aggregation fp32; vs the oracle
    with the same bf16 GEMM semantics (oracle.pyg_ref._Bf16Linear). The two differ in fp32
    summation order, and a last-bit fp32 difference can flip the bf16 rounding of a GEMM operand
    (one bf16 ulp = 2^-8 relative), so the bar is 1e-3 (logits absolute, gradients relative to
    each tensor's max) — 50x below the bf16-vs-fp32 gap asserted below."""
    b = synth.make_batch(256, k=6, d_in=1025, seed=3, sizes="lognormal", last_channel_class=True)
    ours, oref = make_pair(1025, [128] * 4, 1, heads=4, precision="bf16")
    check(ours, oref, b, cuda, tol=1e-3)
    # and bf16 differs from fp32 by bf16 rounding, not by a bug: same weights, fp32 oracle
    o32 = ref.GAT(1025, [128] * 4, 1, heads=4, dropout=0.0)
    o32.load_state_dict(oref.state_dict())
    l16, _, _ = step(oref, b, "cpu", "MSE", 5)
    l32, _, _ = step(o32, b, "cpu", "MSE", 5)
    d = (l16 - l32).abs().max().item()
    assert 1e-6 < d < 5e-2, d


def test_gat_reference_config(cuda):
    """configs/config.py:47,59-64: hiddden_channels=[128]*4, heads=2 (C = 64), KNN k=6 loop."""
    b = synth.make_batch(64, k=6, d_in=64, seed=10, sizes="lognormal")
    ours, oref = make_pair(64, [128] * 4, 1, heads=2)
    check(ours, oref, b, cuda)


@pytest.mark.parametrize("heads,hidden", [(1, [128, 128]), (8, [128, 128]), (2, [64, 256, 32]),
                                          (1, [64, 256, 64]), (1, [32, 512]), (2, [512, 512]),
                                          (8, [32, 32])])
def test_gat_heads_and_widths(cuda, heads, hidden):
    b = synth.make_batch(24, k=5, d_in=32, num_classes=3, seed=11, sizes="lognormal")
    ours, oref = make_pair(32, hidden, 3, heads=heads)
    check(ours, oref, b, cuda, "CE", 3)


def test_gat_unsupported_head_width_raises(cuda):
    """Head widths must be powers of two in [4, 512] (the reference sweep's space)."""
    from lesion_gnn_amd import _lib

    b = synth.make_batch(2, k=4, d_in=8, seed=1)
    m = GAT(8, [48, 96], 1, heads=4, dropout=0.0).to(cuda)  # C = 24
    with pytest.raises(_lib.LgnnError):
        m(b.x.to(cuda), b.edge_index.to(cuda), b.batch.to(cuda))


def test_gat_irregular_edges(cuda):
    """loop=False input (self loops added by the conv), duplicated edges, explicit self loops,
    shuffled edge order, 1-node graphs."""
    sizes = [1, 3, 7, 64, 2, 130, 9]
    b = synth.make_batch(len(sizes), k=6, d_in=16, seed=12, sizes=sizes, loop=False)
    ei = b.edge_index
    perm = torch.randperm(ei.size(1), generator=torch.Generator().manual_seed(0))
    extra = torch.tensor([[5, 5, 5, 20, 20], [5, 5, 6, 21, 21]])
    b.edge_index = torch.cat([ei[:, perm], extra], 1)
    ours, oref = make_pair(16, [32, 32, 32], 1, heads=2)
    check(ours, oref, b, cuda)


def test_gat_alpha_rows_sum_to_one(cuda):
    b = synth.make_batch(16, k=6, d_in=32, seed=13, sizes="lognormal")
    torch.manual_seed(0)
    m = GAT(32, [64, 64], 1, heads=4, dropout=0.0).to(cuda)
    g = Graph(b.edge_index.to(cuda), b.num_nodes)
    conv = m.convs[0]
    x = torch.randn(b.num_nodes, 64, device=cuda)
    ctxout = ops._GATConv.forward  # noqa: F841 (documented entry)
    csr = g.csr("gat")
    y = ops.gat_conv(x, conv.lin.weight, conv.att_src, conv.att_dst, conv.bias, g, 4)
    assert torch.isfinite(y).all()
    # recompute alpha through the C ABI and check row sums
    from lesion_gnn_amd import _lib
    XP = ops.linear_fwd(x, conv.lin.weight.detach(), None, _lib.LGNN_ACT_NONE)
    a_s = torch.empty(b.num_nodes, 4, device=cuda)
    a_d = torch.empty(b.num_nodes, 4, device=cuda)
    _lib.call("lgnn_gat_att", XP.data_ptr(), b.num_nodes, 4, 16,
              conv.att_src.detach().contiguous().data_ptr(),
              conv.att_dst.detach().contiguous().data_ptr(), a_s.data_ptr(), a_d.data_ptr(),
              _lib.stream())
    alpha = torch.empty(csr.col.numel(), 4, device=cuda)
    out = torch.empty(b.num_nodes, 64, device=cuda)
    _lib.call("lgnn_gat_fwd", csr.rowptr.data_ptr(), csr.col.data_ptr(), XP.data_ptr(),
              a_s.data_ptr(), a_d.data_ptr(), b.num_nodes, 4, 16, 0.2, None, None, 0,
              alpha.data_ptr(), out.data_ptr(), None, _lib.stream())
    nnz = int(csr.rowptr[-1])
    rows = torch.repeat_interleave(torch.arange(b.num_nodes, device=cuda),
                                   (csr.rowptr[1:] - csr.rowptr[:-1]).long())
    s = torch.zeros(b.num_nodes, 4, device=cuda).index_add_(0, rows, alpha[:nnz])
    torch.testing.assert_close(s, torch.ones_like(s), rtol=0, atol=1e-6)


def test_gat_dropout_and_determinism(cuda):
    b = synth.make_batch(32, k=6, d_in=64, seed=14, sizes="lognormal")
    torch.manual_seed(0)
    m = GAT(64, [128] * 4, 1, heads=2, dropout=0.35).to(cuda).train()
    out = m(b.x.to(cuda), b.edge_index.to(cuda), b.batch.to(cuda))
    out.sum().backward()
    assert torch.isfinite(out).all()
    assert all(torch.isfinite(p.grad).all() for p in m.parameters())
    m.eval()
    o1 = m(b.x.to(cuda), b.edge_index.to(cuda), b.batch.to(cuda))
    o2 = m(b.x.to(cuda), b.edge_index.to(cuda), b.batch.to(cuda))
    assert torch.equal(o1, o2)


def test_reference_config_training_step(cuda):
    """configs/config.py model section through get_model + training_step (MSE + clamp), dropout
    set to 0 for parity, vs the oracle criterion on the same weights."""
    from lesion_gnn_amd.models import get_model
    from tests.test_config import reference_model_section

    cfg = reference_model_section()
    cfg.dropout = 0.0
    cfg.num_classes.value = 5
    cfg.input_features.value = 64
    cfg.optimizer.class_weights.value = torch.ones(5)
    torch.manual_seed(0)
    module = get_model(cfg).to(cuda).train()
    oref = ref.GAT(64, [128] * 4, 1, heads=2, dropout=0.0)
    # compile=True in the reference section: the model is torch.compile'd (gat.py:84), so the
    # training step below runs the compiled lgnn:: graph
    oref.load_state_dict(getattr(module.model, "_orig_mod", module.model).state_dict())
    b = synth.make_batch(32, k=6, d_in=64, seed=15, sizes="lognormal")
    loss = module.training_step(b.to(cuda))
    want = ref.criterion("MSE", oref(b.x, b.edge_index, b.batch, b.num_graphs), b.y, 5)
    torch.testing.assert_close(loss.detach().cpu(), want.detach(), rtol=1e-5, atol=1e-6)



def test_gat_bf16_copies_match_torch_cast(cuda, monkeypatch):
    """bf16 GAT: the bf16 operand copies the attention kernels write beside their fp32 outputs
    (lgnn_gat_fwd's Y_bf16, lgnn_gat_bwd_node's dXP_bf16) equal torch's RNE cast, so a C3 step
    with them is bit-identical to the same step casting in torch (LGNN_BF16_OUT=0)."""
    from lesion_gnn_amd import ops

    b = synth.make_batch(96, k=6, d_in=1025, seed=17, sizes="lognormal", last_channel_class=True)
    torch.manual_seed(5)
    m = GAT(1025, [128] * 4, 1, heads=4, dropout=0.0, precision="bf16").to(cuda).train()
    res = []
    for on in (True, False):
        monkeypatch.setattr(ops, "BF16_OUT", on)
        out = m(b.x.to(cuda), b.edge_index.to(cuda), b.batch.to(cuda), b.num_graphs)
        loss = torch.nn.functional.mse_loss(out.squeeze(1), b.y.to(cuda).float())
        m.zero_grad(set_to_none=True)
        loss.backward()
        res.append((out.detach().cpu(), {k: p.grad.detach().cpu() for k, p in m.named_parameters()}))
    assert torch.equal(res[0][0], res[1][0])
    for k in res[1][1]:
        assert torch.equal(res[0][1][k], res[1][1][k]), k


def test_gat_bf16_batched_weight_prep_bitwise(cuda, monkeypatch):
    """bf16 GAT: the weight operands prepared for the whole step in one launch
    (lgnn_bf16_weight_prep_multi) and the attention / lin slab sums batched per layer give a
    step bit-identical to per-layer preparation; and no prepared operand survives the step."""
    from lesion_gnn_amd import ops

    b = synth.make_batch(64, k=6, d_in=1025, seed=23, sizes="lognormal", last_channel_class=True)
    torch.manual_seed(7)
    m = GAT(1025, [128] * 4, 1, heads=4, dropout=0.0, precision="bf16").to(cuda).train()
    real = ops.bf16_prepare_weights
    res = []
    for batched in (True, False):
        monkeypatch.setattr(ops, "bf16_prepare_weights", real if batched else (lambda ws: None))
        out = m(b.x.to(cuda), b.edge_index.to(cuda), b.batch.to(cuda), b.num_graphs)
        assert not ops._PREPARED
        m.zero_grad(set_to_none=True)
        out.square().sum().backward()
        res.append((out.detach().cpu(), {n: p.grad.detach().cpu() for n, p in m.named_parameters()}))
    assert torch.equal(res[0][0], res[1][0])
    for n in res[1][1]:
        assert torch.equal(res[0][1][n], res[1][1][n]), n


@pytest.mark.parametrize("precision,pool,dropout", [("bf16", "mean", 0.0), ("fp32", "add", 0.0),
                                                    ("fp32", "mean", 0.3)])
def test_gat_last_conv_readout_fused_bitwise(cuda, monkeypatch, precision, pool, dropout):
    """The last GATConv + global pool + out_proj as one node (ops.gat_conv_head: the readout's
    backward formed inside lgnn_gat_bwd_edge_pool's load) is bit-identical to the separate conv
    and pool_head nodes (k_head_bwd's fmaf chain, then k_pool_bwd's division), same dropout
    masks — except out_proj's own dW / db, summed as outer-product jobs of the layer's slab
    reduction in another fixed order (within 1e-6 of their scale); and matches the oracle."""
    from lesion_gnn_amd.models import gat as gat_mod

    b = synth.make_batch(48, k=6, d_in=64, seed=27, sizes="lognormal")
    torch.manual_seed(9)
    m = GAT(64, [128] * 4, 1, heads=4, dropout=dropout, precision=precision,
            pool=pool).to(cuda).train()
    res = []
    rng = m._dropout_rng.clone()  # both runs draw the same device dropout masks
    for fold in (True, False):
        monkeypatch.setattr(gat_mod, "HEAD_FOLD", fold)
        m._dropout_rng.copy_(rng)
        out = m(b.x.to(cuda), b.edge_index.to(cuda), b.batch.to(cuda), b.num_graphs)
        m.zero_grad(set_to_none=True)
        out.square().sum().backward()
        res.append((out.detach().cpu(), {n: p.grad.detach().cpu() for n, p in m.named_parameters()}))
    assert torch.equal(res[0][0], res[1][0])
    for n in res[1][1]:
        if n.startswith("out_proj."):
            torch.testing.assert_close(res[0][1][n], res[1][1][n], rtol=0,
                                       atol=1e-6 * res[1][1][n].abs().max().item())
        else:
            assert torch.equal(res[0][1][n], res[1][1][n]), n
    if dropout == 0.0 and precision == "fp32":
        oref = ref.GAT(64, [128] * 4, 1, heads=4, dropout=0.0, pool=pool)
        oref.load_state_dict(m.state_dict())
        want = oref(b.x, b.edge_index, b.batch, b.num_graphs)
        torch.testing.assert_close(res[0][0], want.detach(), rtol=0,
                                   atol=1e-4 * max(1.0, want.abs().max().item()))


def test_gat_scores_in_gemm_epilogue(cuda, monkeypatch):
    """bf16 GAT: the attention scores computed in the lin GEMM's epilogue (lgnn_bf16_gemm_att,
    an fmaf chain per (row, head) over the staged fp32 Y tile) against lgnn_gat_att (the same
    products summed as dot4 + butterfly): outputs and gradients within 1e-3 of their scale,
    the bf16 bar (a last-bit difference in a score can flip a later operand's bf16 rounding,
    2^-8 relative; test_gat_c3_bf16)."""
    from lesion_gnn_amd import ops

    b = synth.make_batch(96, k=6, d_in=1025, seed=29, sizes="lognormal", last_channel_class=True)
    torch.manual_seed(4)
    m = GAT(1025, [128] * 4, 1, heads=4, dropout=0.0, precision="bf16").to(cuda).train()
    res = []
    for on in (True, False):
        monkeypatch.setattr(ops, "GAT_GEMM_ATT", on)
        out = m(b.x.to(cuda), b.edge_index.to(cuda), b.batch.to(cuda), b.num_graphs)
        m.zero_grad(set_to_none=True)
        out.square().sum().backward()
        res.append((out.detach().cpu(), {n: p.grad.detach().cpu() for n, p in m.named_parameters()}))
    torch.testing.assert_close(res[0][0], res[1][0], rtol=0,
                               atol=1e-3 * max(1.0, res[1][0].abs().max().item()))
    for n in res[1][1]:
        torch.testing.assert_close(res[0][1][n], res[1][1][n], rtol=0,
                                   atol=max(1e-3 * res[1][1][n].abs().max().item(), 1e-8),
                                   msg=lambda msg: f"{n}: {msg}")
