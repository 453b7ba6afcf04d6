"""GPU: the split readout (lgnn_pool_head_fwd_split: each graph's rows over several workgroups,
the last to arrive sums the partials in split order) — global_mean_pool / global_add_pool +
out_proj (reference gin.py:33, gat.py:56-58) — against a float64 restatement and against the
one-workgroup-per-graph kernel, on few large graphs, ragged and empty graphs; deterministic run
to run, tickets left zero. (Opt-in, LGNN_POOL_SPLITS: slower in every step measured, see
ops.pool_splits.)"""
import pytest
import torch

from lesion_gnn_amd import _lib, ops

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
def test_split_readout(cuda, sizes, D, mean):
    g = torch.Generator().manual_seed(len(sizes) + D)
    M, B = sum(sizes), len(sizes)
    H = torch.randn(M, D, generator=g)
    W = torch.randn(5, D, generator=g)
    b = torch.randn(5, generator=g)
    gptr = torch.tensor([0] + list(torch.tensor(sizes).cumsum(0)), dtype=torch.int32)
    Hc, Wc, bc, gc = H.to(cuda), W.to(cuda), b.to(cuda), gptr.to(cuda)
    S = 4
    outs = []
    for _ in range(2):
        pooled = torch.empty(B, D, device=cuda)
        logits = torch.empty(B, 5, device=cuda)
        part = torch.empty(B * S * D, device=cuda)
        tickets = ops.pool_tickets(cuda, B)
        _lib.call("lgnn_pool_head_fwd_split", Hc.data_ptr(), gc.data_ptr(), B, D, int(mean),
                  Wc.data_ptr(), bc.data_ptr(), 5, S, part.data_ptr(), tickets.data_ptr(),
                  pooled.data_ptr(), logits.data_ptr(), _lib.stream())
        outs.append((pooled.cpu(), logits.cpu()))
        assert int(tickets[:B].abs().sum()) == 0
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    p64, l64 = _ref(H, sizes, mean, W, b)
    tol = 1e-6 * max(1.0, p64.abs().max().item())
    assert (outs[0][0].double() - p64).abs().max().item() <= tol * (1 if mean else 50)
    one = torch.empty(B, D, device=cuda)
    one_l = torch.empty(B, 5, device=cuda)
    _lib.call("lgnn_pool_head_fwd", Hc.data_ptr(), gc.data_ptr(), B, D, int(mean), Wc.data_ptr(),
              bc.data_ptr(), 5, one.data_ptr(), one_l.data_ptr(), _lib.stream())
    # the same terms summed in another fixed order: fp32 summation error of the scale
    scale = max(1.0, p64.abs().max().item())
    torch.testing.assert_close(outs[0][0], one.cpu(), rtol=0, atol=4e-6 * scale)
    torch.testing.assert_close(outs[0][1], one_l.cpu(), rtol=0,
                               atol=4e-6 * scale * W.abs().sum(1).max().item())
