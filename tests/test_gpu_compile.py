"""torch.compile(model, dynamic=True) on the GPU — the reference's compile=True path (gat.py:84,
gin.py:56, drgnet.py:103; configs/config.py:64) — through the lgnn:: custom ops
(lesion_gnn_amd/library.py).

Each compiled model (default Inductor backend, fullgraph=True so a graph break fails the test)
runs one training step and is compared with
  * the eager model on the same weights — BIT-EXACT for GCN / GIN / GAT: the compiled graph holds
    only lgnn ops, i.e. the same HIP kernels in the same order;
  * the CPU oracle at the suite's bars (fp32 1e-4; bf16 GEMMs 1e-3, see test_gpu_gat.py);
and is called again on a batch of a different size, which must reuse the dynamic-shape graph
(no recompilation) and still match eager bit for bit.
"""
import pytest
import torch

import oracle.pyg_ref as ref
from lesion_gnn_amd import synth
from lesion_gnn_amd.models import DRGNet, GAT, GCN, GIN

pytestmark = pytest.mark.gpu


def step(model, b, dev, loss="CE", extra=()):
    out = model(b.x.to(dev), b.edge_index.to(dev), b.batch.to(dev),
                *[e.to(dev) for e in extra], b.num_graphs)
    y = b.y.to(dev)
    if loss == "MSE":
        l = torch.nn.functional.mse_loss(out.squeeze(1).clamp(0, 4), y.float())
    else:
        l = torch.nn.functional.cross_entropy(out, y)
    model.zero_grad(set_to_none=True)
    l.backward()
    return out.detach().cpu(), {k: p.grad.detach().cpu() for k, p in model.named_parameters()}


def clone_to(model, dev):
    import copy

    return copy.deepcopy(model).to(dev)


# biases whose gradient is analytically zero in GIN: a per-channel constant that BatchNorm removes
# (in_proj.bias reaches BN through an aggregation over k-regular rows, nn.lins.0.bias directly);
# both sides hold fp32 cancellation noise, hence a 1e-5 floor (as tests/test_gpu_configs.py)
BN_FED = ("in_proj.bias", "convs.0.nn.lins.0.bias", "convs.1.nn.lins.0.bias")


def check_vs_oracle(lo, go, lr_, gr, tol, gin=False):
    torch.testing.assert_close(lo, lr_, rtol=0, atol=tol * max(1.0, lr_.abs().max().item()))
    for k in gr:
        s = gr[k].abs().max().item()
        floor = 1e-5 if gin and k in BN_FED else 1e-6
        torch.testing.assert_close(go[k], gr[k], rtol=0, atol=max(tol * s, floor),
                                   msg=lambda m: f"{k}: {m}")


def strip(d):
    return {k.replace("_orig_mod.", ""): v for k, v in d.items()}


CASES = {
    "gat_c3_bf16": dict(d_in=1025, sizes="lognormal", k=6, B=(256, 97), loss="MSE", tol=1e-3),
    "gat_fp32": dict(d_in=128, sizes="lognormal", k=6, B=(64, 33), loss="MSE", tol=1e-4),
    "gin_add_train": dict(d_in=128, sizes="fixed", k=8, B=(256, 100), loss="CE", tol=1e-4),
    "gcn": dict(d_in=128, sizes="powerlaw", k=8, B=(128, 57), loss="CE", tol=1e-4),
    # graphs aligned to tiles (C2's shape): the single-launch backward with its open-tile phase
    "gcn_c2": dict(d_in=128, sizes="fixed", k=8, B=(128, 64), loss="CE", tol=1e-4),
    # three convs on graphs aligned to tiles: the fused backward with in_proj's GEMM outside it
    "gcn3": dict(d_in=128, sizes="fixed", k=8, B=(128, 64), loss="CE", tol=1e-4),
}


def build(name):
    torch.manual_seed(1234)
    c = CASES[name]
    if name.startswith("gat"):
        prec = "bf16" if "bf16" in name else "fp32"
        ours = GAT(c["d_in"], [128] * 4, 1, heads=4, dropout=0.0, precision=prec)
        oref = ref.GAT(c["d_in"], [128] * 4, 1, heads=4, dropout=0.0, precision=prec)
    elif name.startswith("gin"):
        ours = GIN(128, [128, 128, 128], 5, 0.0, pool="add")
        oref = ref.GIN(128, [128, 128, 128], 5, 0.0, pool="add")
    else:
        hidden = [128] * (4 if name == "gcn3" else 3)
        ours = GCN(128, hidden, 5, 0.0)
        oref = ref.GCN(128, hidden, 5, 0.0)
    oref.load_state_dict(ours.state_dict())
    return ours.train(), oref.train()


@pytest.mark.parametrize("name", list(CASES))
def test_compiled_model_matches_eager_and_oracle(cuda, name):
    c = CASES[name]
    ours, oref = build(name)
    eager = clone_to(ours, cuda)
    torch._dynamo.reset()
    torch._dynamo.utils.counters.clear()
    compiled = torch.compile(clone_to(ours, cuda), dynamic=True, fullgraph=True)
    for i, B in enumerate(c["B"]):
        b = synth.make_batch(B, n=64, k=c["k"], d_in=c["d_in"], seed=40 + i, sizes=c["sizes"],
                             last_channel_class=c["d_in"] > 128)
        lc, gc = step(compiled, b, cuda, c["loss"])
        le, ge = step(eager, b, cuda, c["loss"])
        gc = strip(gc)
        assert torch.equal(lc, le), (lc - le).abs().max()
        for k in ge:
            assert torch.equal(gc[k], ge[k]), k
        if i == 0:
            lr_, gr = step(oref, b, "cpu", c["loss"])
            check_vs_oracle(lc, gc, lr_, gr, c["tol"], gin=name.startswith("gin"))
    # BatchNorm running statistics (GIN, training) updated identically through the mutating op
    for (k, v), (k2, v2) in zip(strip(compiled.state_dict()).items(), eager.state_dict().items()):
        assert k == k2 and torch.equal(v.cpu(), v2.cpu()), k
    assert torch._dynamo.utils.counters["stats"]["unique_graphs"] <= 2  # no per-size recompile


def test_compiled_dropout_model_is_one_graph(cuda):
    """The reference experiment trains the compiled GAT with dropout 0.35 (configs/config.py:
    52-65): with fullgraph=True a graph break (round 5: the mask scale's fp32 rounding went
    through a torch scalar and `.item()` on the GPU box) fails the compile; the compiled step then
    draws the same masks as the eager one (same generator state) and matches it bit for bit."""
    torch.manual_seed(1234)
    m = GAT(1025, [128] * 4, 1, heads=2, dropout=0.35).train()
    eager, comp = clone_to(m, cuda), clone_to(m, cuda)
    torch._dynamo.reset()
    compiled = torch.compile(comp, dynamic=True, fullgraph=True)
    b = synth.make_batch(64, n=64, k=6, d_in=1025, seed=44, sizes="lognormal",
                         last_channel_class=True)
    lc, gc = step(compiled, b, cuda, "MSE")
    le, ge = step(eager, b, cuda, "MSE")
    gc = strip(gc)
    assert torch.equal(lc, le), (lc - le).abs().max()
    for k in ge:
        assert torch.equal(gc[k], ge[k]), k


def test_compiled_drgnet(cuda):
    """DRGNet (drgnet.py:103 compiles it): lgnn ops for the GraphConv stack, the weighted CSR and
    SortAggregation; the head's torch ops go through Inductor, so the compiled model matches
    eager to fp32 rounding rather than bitwise."""
    b = synth.make_batch(48, n=24, k=6, d_in=16, seed=32, sizes="lognormal")
    ew = ref.gaussian_distance(b.edge_index, b.pos, 0.1).float()
    torch.manual_seed(1234)
    m = DRGNet(16, 8, 2, 10, 5).eval()
    eager = clone_to(m, cuda)
    torch._dynamo.reset()
    compiled = torch.compile(clone_to(m, cuda), dynamic=True, fullgraph=True)
    lc, gc = step(compiled, b, cuda, extra=(ew,))
    le, ge = step(eager, b, cuda, extra=(ew,))
    torch.testing.assert_close(lc, le, rtol=0, atol=1e-5)
    gc = strip(gc)
    for k in ge:
        s = ge[k].abs().max().item()
        torch.testing.assert_close(gc[k], ge[k], rtol=0, atol=max(1e-5 * s, 1e-7),
                                   msg=lambda msg: f"{k}: {msg}")


def test_config_compile_true_module(cuda):
    """GATModule built from a config with compile=True (configs/config.py:59-64) trains through
    the compiled model and matches the same module with compile=False."""
    from lesion_gnn_amd.models import GATConfig, OptimizerConfig, get_model

    def module(compile_):
        cfg = GATConfig(hiddden_channels=[128] * 4, heads=2, dropout=0.0, compile=compile_,
                        optimizer=OptimizerConfig(loss_type="MSE"))
        cfg.input_features.value = 64
        cfg.num_classes.value = 5
        torch.manual_seed(7)
        return get_model(cfg).to(cuda)

    b = synth.make_batch(64, k=6, d_in=64, seed=10, sizes="lognormal").to(cuda)
    torch._dynamo.reset()
    mc, me = module(True), module(False)
    lc = mc.training_step(b)
    le = me.training_step(b)
    lc.backward()
    le.backward()
    assert torch.equal(lc, le)
    for (k, p), (k2, q) in zip(mc.named_parameters(), me.named_parameters()):
        assert k.replace("_orig_mod.", "") == k2 and torch.equal(p.grad, q.grad), k


def test_compiled_reference_config_step_runs_only_lgnn_kernels(cuda):
    """The reference experiment's step (configs/config.py:52-65: GAT heads 2, dropout 0.35,
    compile=True, MSE, d_in 1025) under torch.compile launches no Triton kernel (Inductor has
    nothing to generate: every op is an lgnn custom op) and no vendor-library GEMM, and no
    device copy (the attention / bias gradients come out of one reduction buffer as views)."""
    from torch.profiler import ProfilerActivity, profile

    from lesion_gnn_amd.models import get_model
    from tests.test_config import reference_model_section

    cfg = reference_model_section()
    cfg.num_classes.value = 5
    cfg.input_features.value = 1025
    cfg.optimizer.class_weights.value = torch.ones(5)
    torch.manual_seed(1234)
    torch._dynamo.reset()
    module = get_model(cfg).to(cuda).train()
    b = synth.make_batch(64, k=6, d_in=1025, seed=3, sizes="lognormal",
                         last_channel_class=True).to(cuda)
    for _ in range(2):  # compile + warm up
        module.zero_grad(set_to_none=True)
        module.training_step(b).backward()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        module.zero_grad(set_to_none=True)
        module.training_step(b).backward()
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if e.device_type.name == "CUDA"]
    assert names and any("k_gat_fwd" in n for n in names), sorted(set(names))
    assert not [n for n in names if "triton" in n.lower()], sorted(set(names))
    assert not [n for n in names if n.startswith(("Cijk", "Custom_Cijk"))], sorted(set(names))
    assert not [n for n in names if "copyBuffer" in n or "Memcpy" in n], sorted(set(names))
