"""Split-3 fused GCN stack forward (stack3.hip): bf16 MFMA on three-plane operands.

Checks: the weight planes bit-exactly against a numpy restatement of the split (RNE bf16, feature
order perm16); the stack outputs H_0..H_L against a float64 restatement of the same layers, with
the split-3 error bounded by the fp32-MFMA path's own error (tolerance: max|err_s3| <=
3 * max|err_f32| + 2e-7 * max|H|, and <= 1e-5 absolute) on exact (k = 8) and inexact (k = 6)
tile adjacencies, ragged graphs (open tiles) and widths below 128.
"""
import ctypes

import numpy as np
import pytest
import torch

import oracle.pyg_ref as ref
from lesion_gnn_amd import _lib, ops, synth
from lesion_gnn_amd.graph import Graph

pytestmark = pytest.mark.gpu


def bf16_rne(x: np.ndarray) -> np.ndarray:
    """fp32 -> bf16 bits, round to nearest even (finite inputs)."""
    b = x.astype(np.float32).view(np.uint32).astype(np.uint64)
    return ((b + 0x7FFF + ((b >> 16) & 1)) >> 16).astype(np.uint16)


def bf16_to_f32(h: np.ndarray) -> np.ndarray:
    return (h.astype(np.uint32) << 16).view(np.float32)


def split3(x: np.ndarray):
    out, r = [], x.astype(np.float32)
    for _ in range(3):
        h = bf16_rne(r)
        out.append(h)
        r = (r - bf16_to_f32(h)).astype(np.float32)
    return out


def perm16(k: np.ndarray) -> np.ndarray:
    return (k & ~12) | ((k & 4) << 1) | ((k & 8) >> 1)


def planes_ref(Ws, d_in):
    nl = len(Ws)
    P = np.zeros((nl, 3, 128, 128), np.uint16)
    PT = np.zeros((nl, 3, 128, 128), np.uint16)
    for l, W in enumerate(Ws):
        W = W.cpu().numpy()
        N, K = W.shape
        sp = split3(W)
        n = np.arange(N)[:, None]
        k = np.arange(K)[None, :]
        for p in range(3):
            P[l, p][n, perm16(k)] = sp[p]
            PT[l, p][k, perm16(n)] = sp[p]
    return P, PT


def unfrag(planes: torch.Tensor) -> np.ndarray:
    """Fragment order [l][plane][row / 32][s][h][row % 32][8] -> [l][plane][row][16 s + 8 h + j]."""
    a = planes.cpu().numpy().view(np.uint16).reshape(-1, 3, 4, 8, 2, 32, 8)
    return a.transpose(0, 1, 2, 5, 3, 4, 6).reshape(-1, 3, 128, 128)


@pytest.mark.parametrize("widths", [[128, 128, 128, 128], [64, 96, 128, 32]])
def test_weight_planes_bitexact(cuda, widths):
    torch.manual_seed(3)
    d_in = widths[0]
    Ws = [torch.randn(widths[i + 1], widths[i], device=cuda) * 0.3 for i in range(len(widths) - 1)]
    Ws[0][0, :4] = torch.tensor([1e-30, -3.0e-39, 65504.0, 0.0])  # tiny / subnormal / exact
    planes, planes_t = ops.weight_planes(Ws, d_in, transposed=True)
    P, PT = planes_ref(Ws, d_in)
    gp, gp_t = unfrag(planes), unfrag(planes_t)
    assert np.array_equal(gp, P)
    assert np.array_equal(gp_t, PT)
    # the three planes carry W to 2^-24 relative
    for l, W in enumerate(Ws):
        p = gp[l].astype(np.uint32)
        rec = sum(bf16_to_f32(p[i].astype(np.uint16)).astype(np.float64) for i in range(3))
        N, K = W.shape
        want = W.cpu().numpy().astype(np.float64)
        got = rec[np.arange(N)[:, None], perm16(np.arange(K))[None, :]]
        # (fp32 subnormals keep fewer bits: absolute floor 2^-133)
        assert np.all(np.abs(got - want) <= 2.0 ** -24 * np.abs(want) + 2.0 ** -133)


def ref_stack64(x, edge_index, n, Ws, bs):
    """float64 restatement of in_proj + L x ELU(GCNConv) (PyG order: lin, propagate, bias)."""
    ei, w = ref.gcn_norm(edge_index, n)
    h = x.double() @ Ws[0].double().T + bs[0].double()
    out = [h]
    for W, b in zip(Ws[1:], bs[1:]):
        p = h @ W.double().T
        agg = torch.zeros_like(p).index_add_(0, ei[1], w.double()[:, None] * p[ei[0]])
        h = torch.nn.functional.elu(agg + b.double())
        out.append(h)
    return out


CASES = {
    "c2_exact": dict(B=96, n=64, k=8, widths=[128, 128, 128, 128]),
    "k6_inexact": dict(B=96, n=64, k=6, widths=[128, 128, 128, 128]),
    "ragged": dict(B=9, n=None, k=6, widths=[128, 128, 128, 128],
                   sizes=[1, 5, 64, 200, 2, 33, 512, 17, 64]),
    "narrow": dict(B=40, n=64, k=8, widths=[64, 96, 128, 32]),
    "L1": dict(B=40, n=64, k=8, widths=[128, 128, 128]),
    "L3": dict(B=40, n=64, k=8, widths=[128, 128, 128, 128, 128]),
}


def run_stack(x, g, Ws, bs, mode, monkeypatch):
    monkeypatch.setattr(ops, "MFMA_MODE", mode)
    hs, _ = ops.stack_fwd(x, g, Ws, bs)
    torch.cuda.synchronize()
    return [h.cpu() for h in hs]


@pytest.mark.parametrize("case", list(CASES))
def test_stack_fwd_s3_accuracy(cuda, case, monkeypatch):
    c = CASES[case]
    wd = c["widths"]
    b = synth.make_batch(c["B"], n=c["n"] or 64, k=c["k"], d_in=wd[0], seed=11,
                         sizes=c.get("sizes"))
    torch.manual_seed(5)
    Ws = [torch.randn(wd[i + 1], wd[i]) / wd[i] ** 0.5 for i in range(len(wd) - 1)]
    bs = [torch.randn(wd[i + 1]) * 0.1 for i in range(len(wd) - 1)]
    want = ref_stack64(b.x, b.edge_index, b.num_nodes, Ws, bs)
    g = Graph(b.edge_index.to(cuda), b.num_nodes)
    xd = b.x.to(cuda)
    Wd = [W.to(cuda) for W in Ws]
    bd = [v.to(cuda) for v in bs]
    got_s3 = run_stack(xd, g, Wd, bd, "s3", monkeypatch)
    got_f32 = run_stack(xd, g, Wd, bd, "f32", monkeypatch)
    for l, (s3, f32, w64) in enumerate(zip(got_s3, got_f32, want)):
        e_s3 = (s3.double() - w64).abs().max().item()
        e_f32 = (f32.double() - w64).abs().max().item()
        scale = w64.abs().max().item()
        assert e_s3 <= 3 * e_f32 + 2e-7 * scale, (l, e_s3, e_f32, scale)
        assert e_s3 <= 1e-5, (l, e_s3)


def test_stack_fwd_s3_without_in_proj(cuda):
    """has_in_proj = 0: layer 1 reads X as H_0; must equal the full stack's H_1..H_L."""
    b = synth.make_batch(50, n=64, k=8, d_in=128, seed=12)
    torch.manual_seed(6)
    Ws = [(torch.randn(128, 128) / 128 ** 0.5).to(cuda) for _ in range(3)]
    bs = [(torch.randn(128) * 0.1).to(cuda) for _ in range(3)]
    g = Graph(b.edge_index.to(cuda), b.num_nodes)
    x = b.x.to(cuda)
    hs, _ = ops.stack_fwd(x, g, Ws, bs)
    csr, open_ = g.csr("gcn"), g.tile_open("gcn")
    assert open_.cpu().tolist()[-1] == 0
    M, L = x.size(0), 2
    planes, _ = ops.weight_planes(Ws, 128)
    out = [torch.zeros(M, 128, device=cuda) for _ in range(L + 1)]
    arr = ctypes.c_void_p * (L + 1)
    _lib.call("lgnn_gcn_stack_fwd_s3", _lib.ptr(hs[0]), M, 128, 0, _lib.ptr(csr.rowptr),
              _lib.ptr(csr.col), _lib.ptr(csr.w), L, _lib.ptr(planes),
              arr(*[v.data_ptr() for v in bs]), (ctypes.c_int * (L + 1))(128, 128, 128),
              arr(*[t.data_ptr() for t in out]), _lib.ptr(open_), None, _lib.stream(cuda))
    torch.cuda.synchronize()
    for l in (1, 2):
        assert torch.equal(out[l], hs[l]), l


def test_stack_fwd_s3_deterministic(cuda):
    b = synth.make_batch(300, n=64, k=6, d_in=128, seed=13)
    torch.manual_seed(7)
    Ws = [(torch.randn(128, 128) / 128 ** 0.5).to(cuda) for _ in range(3)]
    bs = [(torch.randn(128) * 0.1).to(cuda) for _ in range(3)]
    g = Graph(b.edge_index.to(cuda), b.num_nodes)
    x = b.x.to(cuda)
    h1, _ = ops.stack_fwd(x, g, Ws, bs)
    h2, _ = ops.stack_fwd(x, g, Ws, bs)
    for a, c in zip(h1, h2):
        assert torch.equal(a, c)
