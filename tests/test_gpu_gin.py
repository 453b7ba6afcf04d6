"""GPU parity of the GIN path (reference gin.py:17-35 + global_add_pool, BASELINE config C4) vs
the CPU oracle: BatchNorm in training and eval mode, running statistics, irregular graphs,
widths off the fast path, determinism. Tolerances as tests/test_gpu_gcn.py."""
import pytest
import torch

import oracle.pyg_ref as ref
from lesion_gnn_amd import ops, synth
from lesion_gnn_amd.models.gin import GIN

pytestmark = pytest.mark.gpu


def make_pair(d_in, hidden, classes=5, pool="add", seed=1234):
    torch.manual_seed(seed)
    ours = GIN(d_in, hidden, classes, dropout=0.0, pool=pool)
    oref = ref.GIN(d_in, hidden, classes, dropout=0.0, pool=pool)
    oref.load_state_dict(ours.state_dict())
    return ours, oref


def step(model, b, device):
    # labels must index the logits (an out-of-range target faults nll_loss on the GPU)
    assert int(b.y.max()) < model.out_proj.out_features
    logits = model(b.x.to(device), b.edge_index.to(device), b.batch.to(device), b.num_graphs)
    loss = torch.nn.functional.cross_entropy(logits, b.y.to(device))
    model.zero_grad(set_to_none=True)
    loss.backward()
    return (logits.detach().cpu(), loss.detach().cpu(),
            {k: p.grad.detach().cpu() for k, p in model.named_parameters()},
            {k: v.detach().cpu() for k, v in model.state_dict().items()})


def assert_grads(go, gr):
    for k in gr:
        scale = gr[k].abs().max().item()
        torch.testing.assert_close(go[k], gr[k], rtol=0, atol=max(1e-4 * scale, 1e-6),
                                   msg=lambda m: f"{k}: {m}")


@pytest.mark.parametrize("bn_fused", [True, False])
@pytest.mark.parametrize("B,pool", [(1024, "add"), (32, "mean")])
def test_gin_c4_shape(cuda, B, pool, bn_fused, monkeypatch):
    """bn_fused: BatchNorm inside the MLP's linear kernels (lgnn_node_linear_fwd_bn / _bwd_bn,
    the default) or the separate lgnn_bn_* passes."""
    monkeypatch.setattr(ops, "BN_FUSED", bn_fused)
    b = synth.make_batch(B, n=64, k=8, d_in=128, seed=4)
    ours, oref = make_pair(128, [128, 128, 128], pool=pool)
    lo, losso, go, so = step(ours.to(cuda).train(), b, cuda)
    lr_, lossr, gr, sr = step(oref.train(), b, "cpu")
    scale = lr_.abs().max().item()
    torch.testing.assert_close(lo, lr_, rtol=0, atol=1e-4 * max(1.0, scale))
    torch.testing.assert_close(losso, lossr, rtol=1e-5, atol=1e-5)
    assert_grads(go, gr)
    for k in sr:
        if "running" in k or "num_batches" in k:
            torch.testing.assert_close(so[k], sr[k], rtol=1e-5, atol=1e-6)


def test_gin_eval_mode_uses_running_stats(cuda):
    b = synth.make_batch(16, n=40, k=6, d_in=64, seed=7)
    ours, oref = make_pair(64, [64, 64, 64])
    step(ours.to(cuda).train(), b, cuda)  # one training step moves the running stats
    step(oref.train(), b, "cpu")
    lo, _, go, _ = step(ours.eval(), b, cuda)
    lr_, _, gr, _ = step(oref.eval(), b, "cpu")
    torch.testing.assert_close(lo, lr_, rtol=0, atol=1e-4)
    assert_grads(go, gr)


def test_gin_irregular_and_wide(cuda):
    """Mixed graph sizes (1-node graphs, N < k, N = 512), loop=False k-NN, widths off the tile
    fast path (160 > 128) and odd class count."""
    sizes = [1, 5, 64, 200, 2, 33, 512, 17]
    b = synth.make_batch(len(sizes), k=6, d_in=96, num_classes=3, seed=5, sizes=sizes,
                         loop=False)
    ours, oref = make_pair(96, [64, 160, 64], classes=3, pool="mean")
    lo, _, go, _ = step(ours.to(cuda).train(), b, cuda)
    lr_, _, gr, _ = step(oref.train(), b, "cpu")
    torch.testing.assert_close(lo, lr_, rtol=0, atol=1e-4)
    assert_grads(go, gr)


def test_gin_deterministic(cuda):
    b = synth.make_batch(128, seed=8)
    ours, _ = make_pair(128, [128, 128, 128])
    ours = ours.to(cuda).train()
    sd = {k: v.clone() for k, v in ours.state_dict().items()}
    l1, _, g1, _ = step(ours, b, cuda)
    ours.load_state_dict(sd)
    l2, _, g2, _ = step(ours, b, cuda)
    assert torch.equal(l1, l2)
    for k in g1:
        assert torch.equal(g1[k], g2[k]), k


def test_gin_dropout_runs(cuda):
    b = synth.make_batch(8, seed=9)
    torch.manual_seed(0)
    m = GIN(128, [128, 128, 128], 5, dropout=0.35).to(cuda).train()
    out = m(b.x.to(cuda), b.edge_index.to(cuda), b.batch.to(cuda))
    out.sum().backward()
    assert torch.isfinite(out).all()
    assert all(torch.isfinite(p.grad).all() for p in m.parameters())


def test_gin_bn_fused_matches_unfused_with_dropout(cuda, monkeypatch):
    """The BN-fused kernels against the separate BN passes on the same
    dropout masks (MLP and
    between convs), training mode, ragged graphs: the same arithmetic up to the order of the fp64
    statistic sums, so within 1e-5 of each tensor's scale; running statistics too."""
    sizes = [1, 5, 64, 200, 2, 33, 90, 17] * 4
    b = synth.make_batch(len(sizes), k=6, d_in=64, seed=15, sizes=sizes)
    torch.manual_seed(3)
    m = GIN(64, [64, 128, 96], 5, dropout=0.35).to(cuda).train()
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    rng = m._dropout_rng.clone()  # every run draws the same device dropout masks
    res = []
    for fused in (True, False):
        monkeypatch.setattr(ops, "BN_FUSED", fused)
        m.load_state_dict(sd)
        m._dropout_rng.copy_(rng)
        res.append(step(m, b, cuda))
    _, (l2, _, g2, s2) = res
    for l1, _, g1, s1 in (res[0],):
        torch.testing.assert_close(l1, l2, rtol=0, atol=1e-5 * max(1.0, l2.abs().max().item()))
        for k in g2:
            torch.testing.assert_close(g1[k], g2[k], rtol=0,
                                       atol=max(1e-5 * g2[k].abs().max().item(), 1e-7),
                                       msg=lambda msg: f"{k}: {msg}")
        for k in s2:
            torch.testing.assert_close(s1[k].float(), s2[k].float(), rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("pool", ["add", "mean"])
def test_gin_last_conv_readout_fused_bitexact(cuda, pool, monkeypatch):
    """The last conv + global pool + out_proj as one node (ops.gin_conv_head: the readout's
    backward folded into Lin2's backward load) is bit-identical to the separate conv and
    pool_head nodes (same arithmetic: k_head_bwd's fmaf chain, then / |graph|), and matches the
    oracle; ragged graphs, SyncBN-free training mode."""
    from lesion_gnn_amd.models import gin as gin_mod

    monkeypatch.setattr(gin_mod, "STACK", False)  # per-conv nodes (the model-wide one: below)
    sizes = [1, 5, 64, 200, 2, 33, 90, 17] * 4
    b = synth.make_batch(len(sizes), k=6, d_in=64, seed=21, sizes=sizes)
    ours, oref = make_pair(64, [64, 128, 96], pool=pool)
    ours = ours.to(cuda).train()
    sd = {k: v.clone() for k, v in ours.state_dict().items()}
    res = []
    for fused in (True, False):
        if not fused:
            monkeypatch.setattr(ops, "gin_conv_head_eligible", lambda *a: False)
        ours.load_state_dict(sd)
        res.append(step(ours, b, cuda))
    (l1, _, g1, s1), (l2, _, g2, s2) = res
    assert torch.equal(l1, l2)
    for k in g2:
        assert torch.equal(g1[k], g2[k]), k
    for k in s2:
        assert torch.equal(s1[k], s2[k]), k
    lr_, _, gr, _ = step(oref.train(), b, "cpu")
    torch.testing.assert_close(l1, lr_, rtol=0, atol=1e-4 * max(1.0, lr_.abs().max().item()))
    assert_grads(g1, gr)


@pytest.mark.parametrize("sizes,pool,eval_mode", [
    ([64] * 1024, "add", False),                      # C4 shape: every tile closed
    ([1, 5, 64, 200, 2, 33, 90, 17] * 4, "mean", False),  # ragged: open tiles, global gathers
    ([1, 5, 64, 200, 2, 33, 90, 17] * 4, "add", True),    # eval: running statistics
])
def test_gin_stack_node(cuda, sizes, pool, eval_mode, monkeypatch):
    """The whole GIN model as one autograd node (ops.gin_stack: each conv's aggregation backward
    gathered by the layer below — lgnn_node_linear_bwd_bn_gather / in_proj in transpose mode —
    instead of a transpose spmm) against the per-conv nodes (within 1e-5 of each tensor's scale:
    the same sums, the self term added after the neighbours instead of before) and the oracle;
    running statistics identical in value."""
    from lesion_gnn_amd.models import gin as gin_mod

    b = synth.make_batch(len(sizes), k=8 if len(sizes) > 100 else 6, d_in=128, seed=31,
                         sizes=sizes)
    ours, oref = make_pair(128, [128, 128, 96], pool=pool)
    ours = ours.to(cuda).train()
    if eval_mode:  # one training step first so the running statistics are not the initial ones
        step(ours, b, cuda)
        step(oref.train(), b, "cpu")
        ours.eval()
        oref.eval()
    sd = {k: v.clone() for k, v in ours.state_dict().items()}
    res = []
    for stack in (True, False):
        monkeypatch.setattr(gin_mod, "STACK", stack)
        ours.load_state_dict(sd)
        res.append(step(ours, b, cuda))
    (l1, _, g1, s1), (l2, _, g2, s2) = res
    torch.testing.assert_close(l1, l2, rtol=0, atol=1e-5 * max(1.0, l2.abs().max().item()))
    for k in g2:
        torch.testing.assert_close(g1[k], g2[k], rtol=0,
                                   atol=max(1e-5 * g2[k].abs().max().item(), 1e-7),
                                   msg=lambda msg: f"{k}: {msg}")
    for k in s2:
        torch.testing.assert_close(s1[k].float(), s2[k].float(), rtol=1e-6, atol=1e-7)
    lr_, _, gr, _ = step(oref, b, "cpu")
    torch.testing.assert_close(l1, lr_, rtol=0, atol=1e-4 * max(1.0, lr_.abs().max().item()))
    for k in gr:  # 5e-6 floor: in_proj.bias feeds BatchNorm through equal-degree aggregation,
        # so its gradient vanishes analytically (parity bar)
        torch.testing.assert_close(g1[k], gr[k], rtol=0,
                                   atol=max(1e-4 * gr[k].abs().max().item(), 5e-6),
                                   msg=lambda m: f"{k}: {m}")
