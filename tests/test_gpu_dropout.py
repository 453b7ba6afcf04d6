"""GPU parity with dropout ON — the configuration the reference actually trains
(configs/config.py:52-65: GAT [128]*4, heads 2, dropout 0.35, compile=True, MSE; and GIN's MLP +
between-conv dropout, gin.py:23,32).

The device masks come from lgnn_dropout_masks (a counter-based generator, include/lgnn.h); the
oracle regenerates the same masks from the model's generator state (oracle.pyg_ref.DropoutMasks)
and applies them where torch's F.dropout would draw its own, so logits, loss and every gradient
are compared at the suite's fp32 bars (logits 1e-4 absolute; gradients 1e-4 x max|grad| per
tensor, floor 1e-6; 1e-5 for the GIN biases BatchNorm cancels; bf16 GEMMs 1e-3).
"""
import pytest
import torch

import oracle.pyg_ref as ref
from lesion_gnn_amd import dropout, synth
from lesion_gnn_amd.models import GAT, GCN, GIN

pytestmark = pytest.mark.gpu

BN_FED = ("in_proj.bias", "convs.0.nn.lins.0.bias", "convs.1.nn.lins.0.bias")


@pytest.mark.parametrize("p", [0.35, 0.5, 0.05])
def test_masks_bitexact_vs_oracle_generator(cuda, p):
    """Every mask of one launch (ragged sizes, a size below 4, an empty one) equals the oracle's
    restatement bit for bit; the counter advances by one per launch; keep rate ~ 1 - p."""
    st = dropout.new_state(987654321).to(cuda)
    shapes = [(1000, 3), (7,), (0,), (65536, 128), (3,)]
    for it in range(2):
        seed, ctr = dropout.get_state(st)
        assert (seed, ctr) == (987654321, it)
        got = dropout.masks(st, shapes, p)
        gen = ref.DropoutMasks(seed, ctr, p)
        for j, (g, s) in enumerate(zip(got, shapes)):
            want = gen.mask(j, g.numel()).view(s)
            assert torch.equal(g.cpu(), want), (j, s)
        big = got[3]
        keep = (big != 0).float().mean().item()
        assert abs(keep - (1 - p)) < 0.01, keep
        assert torch.equal(big[big != 0].unique().cpu(),
                           torch.tensor([1.0 / (1.0 - p)], dtype=torch.float32))
    assert dropout.get_state(st) == (987654321, 2)


def test_masks_fresh_per_graph_replay(cuda):
    """A captured HIP graph draws new masks on every replay (the counter lives on the device)."""
    st = dropout.new_state(5).to(cuda)
    shapes = [(4096,)]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        dropout.masks(st, shapes, 0.35)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        m = dropout.masks(st, shapes, 0.35)[0]
    seen = []
    for i in range(3):
        g.replay()
        torch.cuda.synchronize()
        seen.append(m.clone().cpu())
        # replay i uses counter 1 + i (the warm-up call used 0; capture runs nothing)
        assert torch.equal(seen[-1], ref.DropoutMasks(5, 1 + i, 0.35).mask(0, 4096))
    assert not torch.equal(seen[0], seen[1])
    assert dropout.get_state(st) == (5, 4)


def test_mask_mul_forward_backward(cuda):
    x = torch.randn(1001, 37, device=cuda, requires_grad=True)
    m = dropout.masks(dropout.new_state(1).to(cuda), [(1001, 37)], 0.3)[0]
    y = dropout.mask_mul(x, m)
    assert torch.equal(y, x.detach() * m)
    y.backward(torch.ones_like(y) * 2)
    assert torch.equal(x.grad, 2 * m)


def _check(lo, go, lr_, gr, tol, floors=()):
    torch.testing.assert_close(lo, lr_, rtol=0, atol=tol * max(1.0, lr_.abs().max().item()))
    for k in gr:
        s = gr[k].abs().max().item()
        floor = 1e-5 if k in floors else 1e-6
        torch.testing.assert_close(go[k], gr[k], rtol=0, atol=max(tol * s, floor),
                                   msg=lambda m: f"{k}: {m}")


def _strip(d):
    return {k.replace("_orig_mod.", ""): v for k, v in d.items()}


@pytest.mark.parametrize("compiled", [True, False])
def test_reference_config_gat_dropout_training_step(cuda, compiled):
    """The reference experiment's model (configs/config.py:52-65): GATModule with GAT [128]*4,
    heads 2, dropout 0.35, compile=True, MSE regression (clamp to [0, C-1]), d_in 1025 (1024
    encoder channels + the lesion class, lesions.py:142,169), kNN k = 6, log-normal graph sizes;
    training_step + backward vs the oracle with the same masks."""
    from lesion_gnn_amd.models import get_model
    from tests.test_config import reference_model_section

    cfg = reference_model_section()
    cfg.compile = compiled
    cfg.num_classes.value = 5
    cfg.input_features.value = 1025
    cfg.optimizer.class_weights.value = torch.ones(5)
    torch.manual_seed(1234)
    torch._dynamo.reset()
    module = get_model(cfg).to(cuda).train()
    b = synth.make_batch(192, k=6, d_in=1025, seed=31, sizes="lognormal",
                         last_channel_class=True)
    oref = ref.GAT(1025, [128] * 4, 1, heads=2, dropout=0.35).train()
    oref.load_state_dict(_strip(module.model.state_dict()))
    rng = module.model._dropout_rng
    seen = []  # the inner model's logits of the step (forward hook; compiled or not)
    module.model.register_forward_hook(lambda m, a, out: seen.append(out.detach().cpu()))
    for step in range(2):  # the second step draws new masks (counter + 1)
        seed, ctr = dropout.get_state(rng)
        assert ctr == step
        module.zero_grad(set_to_none=True)
        seen.clear()
        loss = module.training_step(b.to(cuda))
        loss.backward()
        assert len(seen) == 1
        go = {k: p.grad.detach().cpu() for k, p in _strip(dict(module.model.named_parameters()))
              .items()}
        oref.zero_grad(set_to_none=True)
        logits = oref(b.x, b.edge_index, b.batch, b.num_graphs,
                      masks=ref.DropoutMasks(seed, ctr, 0.35))
        want = ref.criterion("MSE", logits, b.y, 5)
        want.backward()
        gr = {k: p.grad for k, p in oref.named_parameters()}
        torch.testing.assert_close(loss.detach().cpu(), want.detach(), rtol=1e-5, atol=1e-6)
        # the raw logits and the clamped predictions the criterion saw (gat.py:94-95)
        _check(seen[0], go, logits.detach(), gr, 1e-4)
        torch.testing.assert_close(seen[0].squeeze(1).clamp(0, 4),
                                   logits.detach().squeeze(1).clamp(0, 4), rtol=0, atol=1e-4)
    # dropout changed the result: the same forward without masks gives other logits (the
    # clamped MSE itself can barely move when most predictions sit at a clamp bound)
    with torch.no_grad():
        plain = oref.eval()(b.x, b.edge_index, b.batch, b.num_graphs)
    assert (plain - logits.detach()).abs().max().item() > 1e-3


@pytest.mark.parametrize("precision,heads,tol", [("fp32", 2, 1e-4), ("bf16", 4, 1e-3)])
def test_gat_dropout_logits_and_grads(cuda, precision, heads, tol):
    """GAT logits and gradients with attention dropout on (fp32 and the bf16 C3 GEMM mode, whose
    bar is 1e-3 as in test_gpu_gat.py), irregular graphs incl. single-node graphs."""
    torch.manual_seed(3)
    sizes = [1, 5, 64, 200, 2, 33, 17, 90]
    b = synth.make_batch(len(sizes), k=6, d_in=128, seed=8, sizes=sizes)
    ours = GAT(128, [128] * 4, 3, heads=heads, dropout=0.35, precision=precision)
    oref = ref.GAT(128, [128] * 4, 3, heads=heads, dropout=0.35, precision=precision)
    oref.load_state_dict(ours.state_dict())
    ours = ours.to(cuda).train()
    seed, ctr = dropout.get_state(ours._dropout_rng)
    lo = ours(b.x.to(cuda), b.edge_index.to(cuda), b.batch.to(cuda), b.num_graphs)
    torch.nn.functional.cross_entropy(lo, b.y.to(cuda) % 3).backward()
    lr_ = oref.train()(b.x, b.edge_index, b.batch, b.num_graphs,
                       masks=ref.DropoutMasks(seed, ctr, 0.35))
    torch.nn.functional.cross_entropy(lr_, b.y % 3).backward()
    _check(lo.detach().cpu(), {k: p.grad.cpu() for k, p in ours.named_parameters()},
           lr_.detach(), {k: p.grad for k, p in oref.named_parameters()}, tol)


@pytest.mark.parametrize("pool,compiled", [("mean", False), ("add", False), ("mean", True)])
def test_gin_dropout_logits_and_grads(cuda, pool, compiled):
    """GIN [128]*3 with dropout 0.35: the MLP's dropout after BatchNorm + ELU (gin.py:23) inside
    the fused GINConv kernels and the dropout after each conv (gin.py:32) by lgnn_mask_mul;
    BatchNorm in training mode; eager and compiled."""
    torch.manual_seed(4)
    b = synth.make_batch(96, n=64, k=8, d_in=128, seed=12)
    ours = GIN(128, [128, 128, 128], 5, 0.35, pool=pool)
    oref = ref.GIN(128, [128, 128, 128], 5, 0.35, pool=pool)
    oref.load_state_dict(ours.state_dict())
    ours = ours.to(cuda).train()
    torch._dynamo.reset()
    run = torch.compile(ours, dynamic=True, fullgraph=True) if compiled else ours
    seed, ctr = dropout.get_state(ours._dropout_rng)
    lo = run(b.x.to(cuda), b.edge_index.to(cuda), b.batch.to(cuda), b.num_graphs)
    torch.nn.functional.cross_entropy(lo, b.y.to(cuda)).backward()
    lr_ = oref.train()(b.x, b.edge_index, b.batch, b.num_graphs,
                       masks=ref.DropoutMasks(seed, ctr, 0.35))
    torch.nn.functional.cross_entropy(lr_, b.y).backward()
    _check(lo.detach().cpu(), {k: p.grad.cpu() for k, p in ours.named_parameters()},
           lr_.detach(), {k: p.grad for k, p in oref.named_parameters()}, 1e-4, BN_FED)
    # BatchNorm running statistics saw the same (dropped) activations
    for k, v in oref.state_dict().items():
        if "running" in k:
            torch.testing.assert_close(ours.state_dict()[k].cpu(), v, rtol=1e-5, atol=1e-6)


def test_gcn_dropout_logits_and_grads(cuda):
    torch.manual_seed(5)
    b = synth.make_batch(64, n=64, k=8, d_in=128, seed=13)
    ours = GCN(128, [128, 128, 128], 5, 0.35)
    oref = ref.GCN(128, [128, 128, 128], 5, 0.35)
    oref.load_state_dict(ours.state_dict())
    ours = ours.to(cuda).train()
    seed, ctr = dropout.get_state(ours._dropout_rng)
    lo = ours(b.x.to(cuda), b.edge_index.to(cuda), b.batch.to(cuda), b.num_graphs)
    torch.nn.functional.cross_entropy(lo, b.y.to(cuda)).backward()
    lr_ = oref.train()(b.x, b.edge_index, b.batch, b.num_graphs,
                       masks=ref.DropoutMasks(seed, ctr, 0.35))
    torch.nn.functional.cross_entropy(lr_, b.y).backward()
    _check(lo.detach().cpu(), {k: p.grad.cpu() for k, p in ours.named_parameters()},
           lr_.detach(), {k: p.grad for k, p in oref.named_parameters()}, 1e-4)


def test_eval_mode_draws_no_masks(cuda):
    m = GAT(32, [32, 32], 2, heads=2, dropout=0.35).to(cuda).eval()
    b = synth.make_batch(8, k=6, d_in=32, seed=1).to(cuda)
    before = dropout.get_state(m._dropout_rng)
    a = m(b.x, b.edge_index, b.batch, b.num_graphs)
    c = m(b.x, b.edge_index, b.batch, b.num_graphs)
    assert torch.equal(a, c) and dropout.get_state(m._dropout_rng) == before
