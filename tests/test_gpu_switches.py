"""GPU: the off-state of every environment switch that no other test flips. Each
switch selects between a default fast path and the earlier path it replaced; both must give the
oracle's answer. fp32 models: logits and gradients against the CPU oracle at the suite's fp32 bars
(1e-4 of the logits' scale, 1e-4 of each gradient's max), with the switch on and off. bf16 GAT
(BF16_MFMA): the hand-written bf16 MFMA kernels against the one-plane split GEMMs they replaced,
at the bf16 bar of test_gpu_gat.py::test_gat_c3_bf16 (1e-3)."""
import pytest
import torch

import oracle.pyg_ref as ref
from lesion_gnn_amd import ops, synth
from lesion_gnn_amd.models import GAT, GCN, GIN

pytestmark = pytest.mark.gpu

RAGGED = [1, 5, 64, 200, 2, 33, 90, 17] * 4


def _step(model, b, device, loss_kind):
    logits = model(b.x.to(device), b.edge_index.to(device), b.batch.to(device), b.num_graphs)
    loss = ref.criterion(loss_kind, logits, b.y.to(device), 5)
    model.zero_grad(set_to_none=True)
    loss.backward()
    return logits.detach().cpu(), {k: p.grad.detach().cpu() for k, p in model.named_parameters()}


def _close(got, want, tol, what):
    (lo, go), (lw, gw) = got, want
    torch.testing.assert_close(lo, lw, rtol=0, atol=tol * max(1.0, lw.abs().max().item()),
                               msg=lambda m: f"{what} logits: {m}")
    for k in gw:
        s = gw[k].abs().max().item()
        torch.testing.assert_close(go[k], gw[k], rtol=0, atol=max(tol * s, 5e-6),
                                   msg=lambda m: f"{what} {k}: {m}")


def _pair(kind, precision="fp32"):
    torch.manual_seed(11)
    if kind == "gcn":
        return GCN(128, [128, 128, 128], 5, dropout=0.0), ref.GCN(128, [128, 128, 128], 5,
                                                                  dropout=0.0)
    if kind == "gin":
        return GIN(128, [128, 128], 5, dropout=0.0), ref.GIN(128, [128, 128], 5, dropout=0.0)
    ours = GAT(64, [128, 128], 5, heads=4, dropout=0.0, precision=precision)
    return ours, ref.GAT(64, [128, 128], 5, heads=4, dropout=0.0, precision=precision)


@pytest.mark.parametrize("switch,kind,sizes", [
    ("ADJT", "gcn", [64] * 64),              # closed tiles: Â^T planes from the forward vs rebuilt
    ("LAZY_TRANSPOSE", "gcn", [64] * 64),    # transpose CSR skipped vs always built
    ("LAZY_TRANSPOSE", "gcn", RAGGED),       # open tiles: the transpose is needed either way
    ("HEAD_JOBS", "gin", RAGGED),            # out_proj dW/db as slab jobs vs lgnn_pool_head_bwd
    ("HEAD_JOBS", "gat", RAGGED),
    ("GAT_S3", "gat", RAGGED),               # split-3 dense GEMMs vs the fp32-MFMA tile kernels
])
def test_switch_off_matches_oracle(cuda, monkeypatch, switch, kind, sizes):
    b = synth.make_batch(len(sizes), k=6, d_in=64 if kind == "gat" else 128, seed=23, sizes=sizes)
    loss_kind = "CE"
    ours, oref = _pair(kind)
    oref.load_state_dict(ours.state_dict())
    ours = ours.to(cuda).train()
    want = _step(oref.train(), b, "cpu", loss_kind)
    sd = {k: v.clone() for k, v in ours.state_dict().items()}
    for on in (True, False):
        monkeypatch.setattr(ops, switch, on)
        ours.load_state_dict(sd)
        _close(_step(ours, b, cuda, loss_kind), want, 1e-4, f"{switch}={on}")


def test_bf16_mfma_off_matches_on(cuda, monkeypatch):
    b = synth.make_batch(len(RAGGED), k=6, d_in=64, seed=29, sizes=RAGGED)
    ours, _ = _pair("gat", "bf16")
    ours = ours.to(cuda).train()
    sd = {k: v.clone() for k, v in ours.state_dict().items()}
    res = {}
    for on in (True, False):
        monkeypatch.setattr(ops, "BF16_MFMA", on)
        ours.load_state_dict(sd)
        res[on] = _step(ours, b, cuda, "CE")
    _close(res[False], res[True], 1e-3, "BF16_MFMA=0 vs 1")
