"""GPU: the wide linears (K or N > 128 — the reference sweep's widths 256 / 512,
scripts/sweep.py:126) on the split-3 dense GEMMs: ops.linear_fwd / linear_bwd run the aggregation
(lgnn_spmm), lgnn_s3_gemm_act (ELU in the epilogue), lgnn_act_bwd and lgnn_s3_wgrad instead of the
fp32 generic node kernels. Parity against the CPU oracle at the suite's fp32 bars (logits 1e-4 of
their scale, gradients 1e-4 of each tensor's max), and against the generic kernels
(LGNN_WIDE=f32) for GIN with BatchNorm in training and eval mode, GCN, ragged graphs whose tiles
are open, add and mean pools."""
import pytest
import torch

import oracle.pyg_ref as ref
from lesion_gnn_amd import _lib, ops, synth
from lesion_gnn_amd.models import GCN, GIN

pytestmark = pytest.mark.gpu


def _step(model, b, device):
    logits = model(b.x.to(device), b.edge_index.to(device), b.batch.to(device), b.num_graphs)
    loss = torch.nn.functional.cross_entropy(logits, b.y.to(device))
    model.zero_grad(set_to_none=True)
    loss.backward()
    return (logits.detach().cpu(), {k: p.grad.detach().cpu() for k, p in model.named_parameters()},
            {k: v.detach().cpu() for k, v in model.state_dict().items()})


def _close(got, want, what):
    logits, grads, state = got
    wl, wg, ws = want
    torch.testing.assert_close(logits, wl, rtol=0, atol=1e-4 * max(1.0, wl.abs().max().item()))
    for k in wg:
        s = wg[k].abs().max().item()
        torch.testing.assert_close(grads[k], wg[k], rtol=0, atol=max(1e-4 * s, 5e-6),
                                   msg=lambda m: f"{what} {k}: {m}")
    for k in ws:
        if "running" in k:
            torch.testing.assert_close(state[k], ws[k], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("model,hidden,pool,sizes,eval_mode", [
    ("gin", [256, 256, 256], "add", [64] * 128, False),
    ("gin", [192, 256, 128], "mean", [1, 5, 64, 200, 2, 33, 90, 17] * 4, False),
    ("gin", [256, 256, 256], "add", [1, 5, 64, 200, 2, 33, 90, 17] * 4, True),
    ("gcn", [128, 256, 256, 256], "mean", [64] * 128, False),
    ("gcn", [256, 256, 256], "add", [1, 5, 64, 200, 2, 33, 90, 17] * 4, False),
])
def test_wide_models_match_oracle_and_generic(cuda, monkeypatch, model, hidden, pool, sizes,
                                              eval_mode):
    b = synth.make_batch(len(sizes), k=6, d_in=128, seed=61, sizes=sizes)
    torch.manual_seed(7)
    Ours, Ref = (GIN, ref.GIN) if model == "gin" else (GCN, ref.GCN)
    ours = Ours(128, hidden, 5, dropout=0.0, pool=pool).to(cuda).train()
    oref = Ref(128, hidden, 5, dropout=0.0, pool=pool)
    oref.load_state_dict({k: v.cpu() for k, v in ours.state_dict().items()})
    if eval_mode:  # one training step first, so the running statistics are not the initial ones
        _step(ours, b, cuda)
        _step(oref.train(), b, "cpu")
        ours.eval()
        oref.eval()
    sd = {k: v.clone() for k, v in ours.state_dict().items()}
    res = {}
    for wide in ("s3", "f32"):
        monkeypatch.setattr(ops, "WIDE", wide)
        ours.load_state_dict(sd)
        res[wide] = _step(ours, b, cuda)
    want = _step(oref, b, "cpu")
    _close(res["s3"], want, "s3 vs oracle")
    _close(res["s3"], res["f32"], "s3 vs generic")


@pytest.mark.parametrize("M,K,N", [(1000, 256, 512), (333, 512, 128), (77, 128, 260)])
def test_wide_linear_elu_and_act_bwd(cuda, M, K, N):
    """lgnn_s3_gemm_act (ELU epilogue) and lgnn_act_bwd against torch's F.elu and its autograd
    on the same operands (float64 reference, the split-3 bound)."""
    g = torch.Generator().manual_seed(M + K + N)
    x = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g)
    y = ops.linear_fwd(x.to(cuda), W.to(cuda), b.to(cuda), _lib.LGNN_ACT_ELU).cpu()
    want = torch.nn.functional.elu(x.double() @ W.double().T + b.double())
    torch.testing.assert_close(y.double(), want, rtol=0, atol=2e-5)
    dy = torch.randn(M, N, generator=g)
    dz = torch.empty(M, N, device=cuda)
    yc, dyc = y.to(cuda), dy.to(cuda)
    _lib.call("lgnn_act_bwd", _lib.ptr(dyc), _lib.ptr(yc), _lib.ptr(dz), M * N, _lib.LGNN_ACT_ELU,
              _lib.stream(cuda))
    want_dz = dy * torch.where(y > 0, torch.ones_like(y), y + 1)
    assert torch.equal(dz.cpu(), want_dz)


@pytest.mark.parametrize("D", [4, 64, 128, 200, 512])
def test_spmm_tiles_closed_open_and_partial(cuda, D):
    """lgnn_spmm stages a 64-row tile in LDS when none of its CSR entries leaves it and gathers
    from global memory otherwise: a CSR whose tiles are closed (graphs of 64 and 32 nodes), open
    (a 100-node graph straddles two tiles, one edge reaches the previous tile) and a partial last
    tile, with weights and a self term, in several feature widths (chunks of 128, a 72-wide tail),
    against a float64 dense restatement."""
    from lesion_gnn_amd.graph import Graph

    b = synth.make_batch(7, k=6, d_in=D, seed=17, sizes=[64, 32, 32, 100, 64, 64, 37])
    ei = b.edge_index.clone()
    # an edge from node 10 (tile 0) into graph 1 (tile 1): both tiles open; the 100-node graph
    # straddles tiles 2 and 3
    assert 64 <= int(ei[1, 400]) < 96
    ei[0, 400] = 10
    g = Graph(ei.to(cuda), b.num_nodes)
    csr = g.csr("gcn")
    x = torch.randn(b.num_nodes, D, generator=torch.Generator().manual_seed(3))
    y = ops.spmm_raw(csr.rowptr, csr.col, csr.w, 0.75, x.to(cuda)).cpu().double()
    rp, cl, w = csr.rowptr.cpu(), csr.col.cpu(), csr.w.cpu().double()
    A = torch.zeros(b.num_nodes, b.num_nodes, dtype=torch.float64)
    for i in range(b.num_nodes):
        for e in range(int(rp[i]), int(rp[i + 1])):
            A[i, int(cl[e])] += w[e]
    want = A @ x.double() + 0.75 * x.double()
    torch.testing.assert_close(y, want, rtol=0, atol=1e-5 * max(1.0, want.abs().max().item()))
