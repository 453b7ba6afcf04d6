"""Parity at the BASELINE configs' full sizes: every workload bench.py times (bench.WORKLOADS, the
same synthetic batch builder, model init and criterion) runs one training step — forward from
edge_index (graph build included), loss, backward — on the HIP path and on the CPU oracle, and
the logits, loss and every parameter gradient are compared.

  C2   GCN, 1024 graphs, N = 64, k = 8, fp32               (BASELINE configs[1])
  C3   GAT, 3 convs, 4 heads, d_in 1025, log-normal N, k = 6, MSE, bf16 GEMMs, 1024 graphs
  C3f32 the same in fp32
  C4   GIN + global_add_pool, 8192 graphs on one GPU (the 8-GPU global batch)
  C5   GCN, power-law N in [16, 512], k = 4 and k = 16, 1024 graphs
  refcfg the reference experiment (configs/config.py:52-65): GAT [128]*4, heads 2, dropout 0.35,
       torch.compile(dynamic=True), d_in 1025, MSE, 1024 graphs — the oracle replays the step's
       dropout masks (oracle.pyg_ref.DropoutMasks)
  sweep_* the reference sweep's space (scripts/sweep.py:105-141): GCN with 3 convs, GCN at
       k = 16 and k = 32 (closed tiles up to 2048 CSR entries), GAT [256]*4 heads 8 (dropout
       0.35), GAT [128]*3 heads 8 (C = 16), GAT [512]*3 heads 4, GIN [512]*4, 1024 graphs each

Bars (written per case): fp32 logits within 1e-4 absolute (× max(1, |logits|) for the add pool,
whose logits sum 64 rows), gradients within 1e-4 × max|grad| per tensor (floor 1e-6); bf16 (C3)
1e-3 — a last-bit fp32 difference can flip the bf16 rounding of a GEMM operand (2^-8 relative),
see tests/test_gpu_gat.py::test_gat_c3_bf16. The CPU oracle takes ≤ 5 s per case here."""
import pytest
import torch

import bench
import oracle.pyg_ref as ref

pytestmark = pytest.mark.gpu

CASES = [("c2", 1024), ("c3", 1024), ("c3f32", 1024), ("c4", 8192), ("c5k4", 1024),
         ("c5k16", 1024), ("refcfg", 1024), ("sweep_gcn3", 1024), ("sweep_gat256h8", 1024),
         ("sweep_gin512", 1024), ("sweep_gcn_k16", 1024), ("sweep_gcn_k32", 1024),
         ("sweep_gat128h8", 1024), ("sweep_gat512h4", 1024)]


def run_step(wl, model, b, dev, oracle, masks=None):
    kw = {"masks": masks} if masks is not None else {}
    logits = model(b.x.to(dev), b.edge_index.to(dev), b.batch.to(dev), b.num_graphs, **kw)
    loss = bench.loss_fn(wl, logits, b.y.to(dev), oracle=oracle)
    model.zero_grad(set_to_none=True)
    loss.backward()
    return (logits.detach().cpu(), loss.detach().cpu(),
            {k: p.grad.detach().cpu() for k, p in model.named_parameters()})


@pytest.mark.parametrize("name,B", CASES)
def test_bench_config_step_vs_oracle(cuda, name, B):
    wl = bench.WORKLOADS[name]
    b = bench.make_batch(wl, B, seed=100)
    ours = bench.build_model(wl).to(cuda).train()
    oref = bench.build_model(wl, oracle=True).train()
    oref.load_state_dict({k: v.cpu() for k, v in ours.state_dict().items()})
    tol = 1e-3 if wl.get("precision") == "bf16" else 1e-4
    masks = None
    run = ours
    if wl.get("dropout"):  # the oracle applies the masks the device step draws
        from lesion_gnn_amd import dropout

        seed, ctr = dropout.get_state(ours._dropout_rng)
        masks = ref.DropoutMasks(seed, ctr, wl["dropout"])
    if wl.get("compile"):  # as bench.py runs it (reference gat.py:84)
        torch._dynamo.reset()
        run = torch.compile(ours, dynamic=True)
    lo, losso, go = run_step(wl, run, b, cuda, oracle=False)
    go = {k.replace("_orig_mod.", ""): v for k, v in go.items()}
    lr_, lossr, gr = run_step(wl, oref, b, "cpu", oracle=True, masks=masks)
    scale = max(1.0, lr_.abs().max().item()) if wl["pool"] == "add" else 1.0
    torch.testing.assert_close(lo, lr_, rtol=0, atol=tol * scale)
    torch.testing.assert_close(losso, lossr, rtol=10 * tol, atol=1e-6)
    assert go.keys() == gr.keys()
    for k in gr:
        s = gr[k].abs().max().item()
        # a Linear bias that feeds BatchNorm (GIN nn.lins.0.bias) has an analytically zero
        # gradient: both sides hold fp32 cancellation noise of a 524k-row sum, hence the floor
        floor = 1e-5 if k.endswith("nn.lins.0.bias") else 1e-6
        torch.testing.assert_close(go[k], gr[k], rtol=0, atol=max(tol * s, floor),
                                   msg=lambda m: f"{name} {k}: {m}")
