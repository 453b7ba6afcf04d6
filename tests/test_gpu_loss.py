"""GPU parity of the HIP criterion (reference models/base.py:93-94, nn.CrossEntropyLoss(weight),
mean reduction) and of the batched slab reduction, vs torch on CPU (fp32; 1e-6 relative)."""
import pytest
import torch

import oracle.pyg_ref as ref
from lesion_gnn_amd import ops, synth
from lesion_gnn_amd.models.base import CrossEntropyLoss

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,C,weighted", [(1024, 5, False), (1024, 5, True), (3, 2, True),
                                          (5000, 7, False)])
def test_cross_entropy_matches_torch(cuda, B, C, weighted):
    g = torch.Generator().manual_seed(B + C)
    z = torch.randn(B, C, generator=g) * 3
    y = torch.randint(0, C, (B,), generator=g)
    w = torch.rand(C, generator=g) + 0.1 if weighted else None
    zr = z.clone().requires_grad_()
    want = torch.nn.functional.cross_entropy(zr, y, weight=w)
    want.backward()
    zg = z.to(cuda).requires_grad_()
    got = ops.cross_entropy(zg, y.to(cuda), w.to(cuda) if w is not None else None)
    got.backward()
    torch.testing.assert_close(got.detach().cpu(), want.detach(), rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(zg.grad.cpu(), zr.grad, rtol=1e-5, atol=1e-8)
    # criterion module (BaseModule) and bitwise determinism
    crit = CrossEntropyLoss(w).to(cuda)
    a = crit(z.to(cuda), y.to(cuda))
    b = crit(z.to(cuda), y.to(cuda))
    assert torch.equal(a, b)


def test_cross_entropy_validates_targets(cuda):
    z = torch.randn(4, 3, device=cuda)
    y = torch.tensor([0, 1, 3, 2], device=cuda)
    with pytest.raises(ValueError):
        ops.cross_entropy(z, y, validate=True)


def test_reduce_multi(cuda):
    jobs = []
    want = []
    for P, n in [(512, 16384), (7, 5), (1, 100), (300, 129)]:
        part = torch.randn(P * n, device=cuda)
        out = torch.empty(n, device=cuda)
        jobs.append((part, P, n, out))
        want.append(part.view(P, n).double().sum(0).float())
    ops.reduce_multi(jobs, cuda)
    for (_, _, _, out), w in zip(jobs, want):
        torch.testing.assert_close(out, w, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("kind", ["MSE", "SmoothL1"])
@pytest.mark.parametrize("ydtype", [torch.int64, torch.float32])
def test_regression_head_and_criterion(cuda, kind, ydtype):
    """ops.regression_loss (lgnn_regression_fwd / _bwd: clamp(logits.squeeze(1), 0, C-1) + mean
    MSE / SmoothL1 in one launch each way) against torch's clamp + mse_loss / smooth_l1_loss, as
    the reference computes them (gat.py:94-95, models/base.py:95-96): values below, inside and
    above the clamp range and exactly on its bounds; the gradient of the clamped prediction too."""
    from lesion_gnn_amd import ops

    g = torch.Generator().manual_seed(3)
    B, C = 1000, 5
    z = (torch.rand(B, 1, generator=g) * 8 - 2)
    z[:4, 0] = torch.tensor([0.0, 4.0, -1.0, 6.0])
    y = torch.randint(0, C, (B,), generator=g)
    zc = z.clone().to(cuda).requires_grad_(True)
    pred, loss = ops.regression_loss(zc, y.to(cuda).to(ydtype), 0.0, C - 1.0, kind)
    (loss * 3.0 + (pred * torch.linspace(0, 1, B, device=cuda)).sum()).backward()
    zr = z.clone().requires_grad_(True)
    pr = torch.clamp(zr.squeeze(1), 0, C - 1)
    fn = torch.nn.functional.mse_loss if kind == "MSE" else torch.nn.functional.smooth_l1_loss
    lr_ = fn(pr, y.float())
    (lr_ * 3.0 + (pr * torch.linspace(0, 1, B)).sum()).backward()
    assert torch.equal(pred.detach().cpu(), pr.detach())
    torch.testing.assert_close(loss.detach().cpu(), lr_.detach(), rtol=1e-6, atol=0)
    torch.testing.assert_close(zc.grad.cpu(), zr.grad, rtol=1e-5, atol=1e-7)


def test_regression_module_training_step_matches_oracle(cuda):
    """BaseModule.training_step for a regression config runs the fused clamp + criterion; its
    loss equals the oracle criterion on the same logits."""
    from lesion_gnn_amd.models import get_model
    from tests.test_config import reference_model_section

    cfg = reference_model_section()
    cfg.dropout = 0.0
    cfg.compile = False
    cfg.num_classes.value = 5
    cfg.input_features.value = 32
    cfg.optimizer.class_weights.value = torch.ones(5)
    torch.manual_seed(0)
    module = get_model(cfg).to(cuda).train()
    b = synth.make_batch(24, k=6, d_in=32, seed=5, sizes="lognormal").to(cuda)
    loss = module.training_step(b)
    logits = module.model(b.x, b.edge_index, b.batch, b.num_graphs)
    want = ref.criterion("MSE", logits.detach().cpu(), b.y.cpu(), 5)
    torch.testing.assert_close(loss.detach().cpu(), want, rtol=1e-6, atol=1e-7)
