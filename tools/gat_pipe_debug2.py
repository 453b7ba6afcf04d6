"""lgnn_gat_fwd / lgnn_gat_bwd_edge / lgnn_gat_bwd_node called directly with the row-pipelined
kernels and the per-row ones (path option LGNN_OPT_GAT_PIPE 1 / 0) on the same inputs; prints which outputs differ.
Usage (GPU box): python tools/gat_pipe_debug2.py heads C"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lesion_gnn_amd import _lib, synth  # noqa: E402
from lesion_gnn_amd.graph import Graph  # noqa: E402

P = _lib.ptr


def main():
    H, C = int(sys.argv[1]), int(sys.argv[2])
    HC = H * C
    dev = torch.device("cuda", 0)
    b = synth.make_batch(64, k=6, d_in=8, seed=31, sizes="lognormal")
    g = Graph(b.edge_index.to(dev), b.num_nodes)
    csr = g.csr("gat")
    M = b.num_nodes
    gen = torch.Generator().manual_seed(0)
    XP = torch.randn(M, HC, generator=gen).to(dev)
    att_s = torch.randn(HC, generator=gen).to(dev)
    att_d = torch.randn(HC, generator=gen).to(dev)
    a_s = torch.empty(M, H, device=dev)
    a_d = torch.empty(M, H, device=dev)
    s = _lib.stream(dev)
    _lib.call("lgnn_gat_att", P(XP), M, H, C, P(att_s), P(att_d), P(a_s), P(a_d), s)
    cap = csr.col.numel()
    dY = torch.randn(M, HC, generator=gen).to(dev)
    res = {}
    for pipe in ("1", "0"):
        _lib.load().lgnn_set_option(_lib.LGNN_OPT_GAT_PIPE, int(pipe))
        alpha = torch.zeros(cap, H, device=dev)
        Y = torch.empty(M, HC, device=dev)
        _lib.call("lgnn_gat_fwd", P(csr.rowptr), P(csr.col), P(XP), P(a_s), P(a_d), M, H, C,
                  0.2, None, None, 1, P(alpha), P(Y), None, s)
        dZ = torch.empty(M, HC, device=dev)
        da_e = torch.zeros(cap, H, device=dev)
        da_d = torch.empty(M, H, device=dev)
        _lib.call("lgnn_gat_bwd_edge", P(csr.rowptr), P(csr.col), P(XP), P(a_s), P(a_d), P(alpha),
                  None, P(dY), P(Y), 1, M, H, C, 0.2, P(dZ), P(da_e), P(da_d), s)
        NP = _lib.load().lgnn_gat_bwd_num_partials(M)
        part = torch.empty(NP * 3 * HC, device=dev)
        dXP = torch.empty(M, HC, device=dev)
        _lib.call("lgnn_gat_bwd_node", P(csr.tptr), P(csr.tidx), P(csr.tmap), P(alpha), None,
                  P(da_e), P(da_d), P(dZ), P(XP), P(att_s), P(att_d), M, H, C, P(dXP), P(part),
                  NP, None, s)
        torch.cuda.synchronize()
        res[pipe] = dict(alpha=alpha.cpu(), Y=Y.cpu(), dZ=dZ.cpu(), da_e=da_e.cpu(),
                         da_d=da_d.cpu(), dXP=dXP.cpu(), part=part.view(NP, 3, HC).sum(0).cpu())
    for k in res["0"]:
        a, c = res["1"][k], res["0"][k]
        if torch.equal(a, c):
            print(f"H={H} C={C} {k}: equal")
        else:
            bad = (a != c).nonzero()
            print(f"H={H} C={C} {k}: {bad.size(0)} differ, max {(a - c).abs().max().item():.3e}; "
                  f"first {bad[:6].tolist()}")


if __name__ == "__main__":
    main()
