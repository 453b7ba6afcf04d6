"""GPU: the readout (lgnn_pool_head_fwd: global_mean_pool / global_add_pool + out_proj, reference
gin.py:33, gat.py:56-58) against a float64 restatement on few large graphs (the GAT configs),
ragged and empty graphs; deterministic run to run."""
import pytest
import torch

from lesion_gnn_amd import _lib

pytestmark = pytest.mark.gpu


def _ref(H, sizes, mean, W, b):
    out, off = [], 0
    for n in sizes:
        seg = H[off:off + n].double()
        s = seg.sum(0) if n else torch.zeros(H.size(1), dtype=torch.float64)
        out.append(s / max(n, 1) if mean else s)
        off += n
    p = torch.stack(out)
    return p, p @ W.double().T + b.double()


@pytest.mark.parametrize("sizes,D,mean", [([660] * 64, 128, True), ([1, 0, 3000, 7, 64, 5], 128, False),
                                          ([300] * 17 + [0, 2], 256, True), ([40] * 200, 64, True)])
def test_readout(cuda, sizes, D, mean):
    g = torch.Generator().manual_seed(len(sizes) + D)
    M, B = sum(sizes), len(sizes)
    H = torch.randn(M, D, generator=g)
    W = torch.randn(5, D, generator=g)
    b = torch.randn(5, generator=g)
    gptr = torch.tensor([0] + list(torch.tensor(sizes).cumsum(0)), dtype=torch.int32)
    Hc, Wc, bc, gc = H.to(cuda), W.to(cuda), b.to(cuda), gptr.to(cuda)
    outs = []
    for _ in range(2):
        pooled = torch.empty(B, D, device=cuda)
        logits = torch.empty(B, 5, device=cuda)
        _lib.call("lgnn_pool_head_fwd", Hc.data_ptr(), gc.data_ptr(), B, D, int(mean),
                  Wc.data_ptr(), bc.data_ptr(), 5, pooled.data_ptr(), logits.data_ptr(),
                  _lib.stream())
        outs.append((pooled.cpu(), logits.cpu()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    p64, l64 = _ref(H, sizes, mean, W, b)
    scale = max(1.0, p64.abs().max().item())
    assert (outs[0][0].double() - p64).abs().max().item() <= 4e-6 * scale * (1 if mean else 50)
    lscale = scale * W.abs().sum(1).max().item()
    assert (outs[0][1].double() - l64).abs().max().item() <= 4e-6 * lscale * (1 if mean else 50)
