"""GPU: the GCN model and its cross-entropy criterion as one autograd node (ops.gcn_stack_ce,
GCN.forward_loss; reference models/base.py:93-94 criterion + training_step :196-201).

The fused backward forms the CE logits gradient where it is consumed (the split-3 backward's
prologue, the open-tile phase, the out_proj reduction jobs) with lgnn_ce_bwd's expression, so
its gradients must equal the unfused sequence (gcn_stack -> ops.cross_entropy -> backward)
BITWISE; both are also checked against the CPU oracle at the suite's fp32 bars. Cases: C2 tiles
(all closed), ragged power-law graphs (open tiles: the open phase forms the gradient too), class
weights, out-of-range-free targets, the logits also differentiated (falls back to lgnn_ce_bwd),
BaseModule.training_step, and a captured HIP graph replay.
"""
import pytest
import torch

import oracle.pyg_ref as ref
from lesion_gnn_amd import ops, synth
from lesion_gnn_amd.models import GCN

pytestmark = pytest.mark.gpu


def _model(cuda, d_in=128, C=5):
    torch.manual_seed(21)
    return GCN(d_in, [128, 128, 128], C, 0.0).to(cuda).train()


def _grads(m):
    return {k: p.grad.detach().clone() for k, p in m.named_parameters()}


@pytest.mark.parametrize("case", ["c2", "ragged", "weighted"])
def test_fused_ce_bitwise_equals_unfused(cuda, case):
    if case == "ragged":
        b = synth.make_batch(96, k=8, d_in=128, seed=5, sizes="powerlaw")
    else:
        # the bench's C2 batch size (BASELINE configs[1]: 1024 graphs)
        b = synth.make_batch(1024, n=64, k=8, d_in=128, seed=4)
    w = torch.tensor([0.5, 2.0, 1.0, 3.0, 0.25], device=cuda) if case == "weighted" else None
    m = _model(cuda)
    x, ei, bt, y = (t.to(cuda) for t in (b.x, b.edge_index, b.batch, b.y))
    logits, loss = m.forward_loss(x, ei, bt, y, w, b.num_graphs)
    loss.backward()
    g_fused = _grads(m)
    m.zero_grad(set_to_none=True)
    lo2 = m(x, ei, bt, b.num_graphs)
    loss2 = ops.cross_entropy(lo2, y, w)
    loss2.backward()
    g_plain = _grads(m)
    assert torch.equal(logits, lo2) and torch.equal(loss, loss2)
    for k in g_plain:
        assert torch.equal(g_fused[k], g_plain[k]), k
    # and the oracle at the fp32 bars
    oref = ref.GCN(128, [128, 128, 128], 5, 0.0)
    oref.load_state_dict({k: v.cpu() for k, v in m.state_dict().items()})
    lr_ = oref(b.x, b.edge_index, b.batch, b.num_graphs)
    want = torch.nn.functional.cross_entropy(lr_, b.y, weight=None if w is None else w.cpu())
    want.backward()
    torch.testing.assert_close(logits.detach().cpu(), lr_.detach(), rtol=0, atol=1e-4)
    torch.testing.assert_close(loss.detach().cpu(), want.detach(), rtol=1e-5, atol=1e-6)
    for k, p in oref.named_parameters():
        s = p.grad.abs().max().item()
        torch.testing.assert_close(g_fused[k].cpu(), p.grad, rtol=0, atol=max(1e-4 * s, 1e-6),
                                   msg=lambda e: f"{k}: {e}")


def test_fused_ce_logits_also_differentiated(cuda):
    """loss + a term on the logits: the node forms dlogits with lgnn_ce_bwd and adds the logits'
    own gradient (the unfused result)."""
    b = synth.make_batch(64, n=64, k=8, d_in=128, seed=6)
    m = _model(cuda)
    x, ei, bt, y = (t.to(cuda) for t in (b.x, b.edge_index, b.batch, b.y))
    logits, loss = m.forward_loss(x, ei, bt, y, None, b.num_graphs)
    (loss + 0.1 * logits.square().mean()).backward()
    g1 = _grads(m)
    m.zero_grad(set_to_none=True)
    lo2 = m(x, ei, bt, b.num_graphs)
    (ops.cross_entropy(lo2, y) + 0.1 * lo2.square().mean()).backward()
    g2 = _grads(m)
    for k in g2:
        torch.testing.assert_close(g1[k], g2[k], rtol=1e-6, atol=1e-7, msg=lambda e: f"{k}: {e}")


def test_training_step_uses_fused_node(cuda):
    from lesion_gnn_amd.models import GCNConfig, OptimizerConfig, get_model

    cfg = GCNConfig(optimizer=OptimizerConfig(loss_type="CE"), hidden_channels=[128, 128, 128],
                    dropout=0.0, compile=False)
    cfg.num_classes.value, cfg.input_features.value = 5, 128
    cfg.optimizer.class_weights.value = torch.tensor([1.0, 2.0, 0.5, 1.0, 4.0])
    torch.manual_seed(3)
    module = get_model(cfg).to(cuda).train()
    b = synth.make_batch(128, n=64, k=8, d_in=128, seed=8).to(cuda)
    loss = module.training_step(b)
    assert loss.grad_fn is not None and "GCNStackCE" in type(loss.grad_fn).__name__
    loss.backward()
    g1 = _grads(module.model)
    module.zero_grad(set_to_none=True)
    ops.cross_entropy(module(b), b.y, module.criterion.weight).backward()
    g2 = _grads(module.model)
    for k in g2:
        assert torch.equal(g1[k], g2[k]), k


def test_fused_ce_in_captured_graph(cuda):
    """The bench's step shape: forward_loss + backward captured once, replayed; every replay's
    gradients equal an eager step's on the same weights."""
    b = synth.make_batch(128, n=64, k=8, d_in=128, seed=9)
    m = _model(cuda)
    x, ei, bt, y = (t.to(cuda) for t in (b.x, b.edge_index, b.batch, b.y))
    one = torch.ones((), device=cuda)

    def step():
        m.forward_loss(x, ei, bt, y, None, b.num_graphs)[1].backward(one)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            m.zero_grad(set_to_none=True)
            step()
    torch.cuda.current_stream().wait_stream(s)
    m.zero_grad(set_to_none=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    g.replay()
    torch.cuda.synchronize()
    got = _grads(m)
    m.zero_grad(set_to_none=True)
    ops.cross_entropy(m(x, ei, bt, b.num_graphs), y).backward()
    for k, v in _grads(m).items():
        assert torch.equal(got[k], v), k
