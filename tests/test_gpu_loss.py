"""GPU parity of the HIP criterion (reference models/base.py:93-94, nn.CrossEntropyLoss(weight),
mean reduction) and of the batched slab reduction, vs torch on CPU (fp32; 1e-6 relative)."""
import pytest
import torch

from lesion_gnn_amd import ops
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
