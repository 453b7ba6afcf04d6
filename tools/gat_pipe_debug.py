"""Gradient differences between the row-pipelined GAT kernels and the per-row ones
(path option LGNN_OPT_GAT_PIPE 1 / 0) for one shape. Usage (GPU box): python tools/gat_pipe_debug.py heads hidden fold"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lesion_gnn_amd import _lib, synth  # noqa: E402
from lesion_gnn_amd.models import gat as gat_mod  # noqa: E402
from lesion_gnn_amd.models.gat import GAT  # noqa: E402


def main():
    heads = int(sys.argv[1])
    hidden = [int(v) for v in sys.argv[2].split(",")]
    gat_mod.HEAD_FOLD = sys.argv[3] == "1"
    dev = torch.device("cuda", 0)
    b = synth.make_batch(64, k=6, d_in=64, seed=31, sizes="lognormal")
    torch.manual_seed(5)
    m = GAT(64, hidden, 1, heads=heads, dropout=0.0, pool="mean").to(dev).train()
    res = {}
    for pipe in ("1", "0"):
        _lib.load().lgnn_set_option(_lib.LGNN_OPT_GAT_PIPE, int(pipe))
        out = m(b.x.to(dev), b.edge_index.to(dev), b.batch.to(dev), b.num_graphs)
        m.zero_grad(set_to_none=True)
        out.square().sum().backward()
        res[pipe] = ({n: p.grad.detach().cpu() for n, p in m.named_parameters()}, out.detach().cpu())
    print(heads, hidden, "fold", gat_mod.HEAD_FOLD, "logits equal", torch.equal(res["1"][1], res["0"][1]))
    for n in res["0"][0]:
        a, c = res["1"][0][n], res["0"][0][n]
        print("  ", n, "equal" if torch.equal(a, c) else
              f"max diff {(a - c).abs().max().item():.3e} scale {c.abs().max().item():.3e}")


if __name__ == "__main__":
    main()
