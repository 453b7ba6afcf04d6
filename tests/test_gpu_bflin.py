"""bf16 dense GEMMs (csrc/bflin.hip): the C3 in_proj / GATConv.lin kernels, forward and backward.

Reference semantics: the GEMM of bf16-rounded operands (RNE, as torch's .to(torch.bfloat16)) with
fp32 accumulation (oracle.pyg_ref._Bf16Linear). Checks: the weight operands bit-exactly against
a numpy RNE restatement; Y, dX and dW against a float64 product of the same rounded operands,
within fp32 summation error (|err| <= 2^-20 * sum_k |a_k b_k| + 1e-30: the kernels sum in a
different order than any reference, so bit equality is not defined); the bf16 output copy equal
to torch's cast of the fp32 output; ragged M (tails of the 64-row tiles), K = 1025 (the
reference's in_proj width: unaligned rows, a 1-wide last k-chunk), K = 1, N < 128, bf16 A.
"""
import numpy as np
import pytest
import torch

from lesion_gnn_amd import _lib, ops

pytestmark = pytest.mark.gpu


def bf16_rne(x: np.ndarray) -> np.ndarray:
    b = x.astype(np.float32).view(np.uint32).astype(np.uint64)
    return ((b + 0x7FFF + ((b >> 16) & 1)) >> 16).astype(np.uint16)


def bf16_to_f32(h: np.ndarray) -> np.ndarray:
    return (h.astype(np.uint32) << 16).view(np.float32)


def rounded(t: torch.Tensor) -> np.ndarray:
    return bf16_to_f32(bf16_rne(t.detach().float().cpu().numpy())).astype(np.float64)


def check_product(got: torch.Tensor, a: np.ndarray, b: np.ndarray, add=0.0):
    """got ~ a @ b + add (float64 of the rounded operands) within fp32 summation error."""
    ref = a @ b + add
    bound = 2.0 ** -20 * (np.abs(a) @ np.abs(b) + np.abs(add)) + 1e-30
    err = np.abs(got.double().cpu().numpy() - ref)
    assert (err <= bound).all(), f"max err {err.max():.3e}, worst ratio {(err / bound).max():.2f}"


def frag_order(mat: np.ndarray) -> np.ndarray:
    """[128][width] -> the kernels' fragment order (include/lgnn.h, lgnn_bf16_weight_prep)."""
    j = np.arange(mat.size)
    e, lane, w, cs = j & 7, (j >> 3) & 63, (j >> 9) & 3, j >> 11
    return mat[32 * w + (lane & 31), cs * 16 + 8 * (lane >> 5) + e]


def _weights(N, K, dev, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(N, K, generator=g) / K ** 0.5).to(dev)


@pytest.mark.parametrize("N,K", [(128, 1025), (128, 128), (62, 33), (128, 1)])
def test_weight_prep_bitexact(cuda, N, K):
    W = _weights(N, K, cuda)
    Wb, WTb = ops.bf16_weight_operands(W, True)
    kp, npad = _lib.load().lgnn_bf16_kpad(K), _lib.load().lgnn_bf16_kpad(N)
    want = np.zeros((128, kp), np.uint16)
    want[:N, :K] = bf16_rne(W.cpu().numpy())
    assert np.array_equal(Wb.view(torch.int16).cpu().numpy().view(np.uint16), frag_order(want))
    if K <= 128:
        wt = np.zeros((128, npad), np.uint16)
        wt[:K, :N] = bf16_rne(W.cpu().numpy()).T
        got = WTb.view(torch.int16).cpu().numpy().view(np.uint16)
        assert np.array_equal(got, frag_order(wt))
    else:
        assert WTb is None


@pytest.mark.parametrize("M,K,N,a_bf16,bias", [
    (42279, 1025, 128, False, True),   # C3 in_proj
    (4133, 128, 128, True, False),     # GATConv.lin on the previous layer's bf16 copy
    (4133, 128, 128, False, False),
    (100, 36, 62, False, True),        # K % 4 == 0 fp32, N < 128
    (65, 1, 128, False, True),         # K = 1
    (1, 1025, 128, False, False),
    (63, 200, 96, True, True),
])
def test_gemm_vs_rounded_product(cuda, M, K, N, a_bf16, bias):
    g = torch.Generator().manual_seed(M + K + N)
    A = torch.randn(M, K, generator=g).to(cuda)
    W = _weights(N, K, cuda, seed=1)
    b = torch.randn(N, generator=g).to(cuda) if bias else None
    Wb, _ = ops.bf16_weight_operands(W, False)
    Ain = A.to(torch.bfloat16) if a_bf16 else A
    Y, Yb = ops.bf16_gemm(Ain, Wb, b, N, want_yb=True)
    torch.cuda.synchronize()
    a, w = rounded(A), rounded(W)
    ref_b = b.double().cpu().numpy() if bias else 0.0
    check_product(Y, a, w.T, ref_b)
    assert torch.equal(Yb, Y.to(torch.bfloat16))


@pytest.mark.parametrize("M,K,N,x_bf16", [
    (42279, 1025, 128, False),   # C3 in_proj dW (x fp32, rounded in the kernel)
    (42279, 128, 128, True),     # GATConv.lin dW (bf16 copy of x)
    (4133, 128, 128, False),
    (130, 33, 62, False),
    (1, 1025, 128, False),
    (0, 128, 128, True),
])
def test_wgrad_vs_rounded_product(cuda, M, K, N, x_bf16):
    g = torch.Generator().manual_seed(M * 7 + K + N)
    X = torch.randn(M, K, generator=g).to(cuda)
    dY = torch.randn(M, N, generator=g).to(cuda)
    dYb = dY.to(torch.bfloat16)
    Xin = X.to(torch.bfloat16) if x_bf16 else X
    dW = ops.bf16_wgrad(dYb, Xin, N)
    torch.cuda.synchronize()
    check_product(dW, rounded(dY).T, rounded(X))


def test_dx_through_transposed_weights(cuda):
    """dX = dY W with W^T as the weight operand (the lin backward), K < 128."""
    M, N, K = 5000, 128, 96
    g = torch.Generator().manual_seed(3)
    dY = torch.randn(M, N, generator=g).to(cuda)
    W = _weights(N, K, cuda, seed=4)
    _, WTb = ops.bf16_weight_operands(W, True)
    dX, _ = ops.bf16_gemm(dY.to(torch.bfloat16), WTb, None, K)
    torch.cuda.synchronize()
    check_product(dX, rounded(dY), rounded(W))


def test_wgrad_deterministic(cuda):
    M, K, N = 42279, 1025, 128
    g = torch.Generator().manual_seed(9)
    X = torch.randn(M, K, generator=g).to(cuda)
    dYb = torch.randn(M, N, generator=g).to(cuda).to(torch.bfloat16)
    assert torch.equal(ops.bf16_wgrad(dYb, X, N), ops.bf16_wgrad(dYb, X, N))


def test_bad_arguments_refused(cuda):
    lib = _lib.load()
    A = torch.zeros(64, 30, dtype=torch.bfloat16, device=cuda)   # bf16 A needs K % 4 == 0
    Wb = torch.zeros(128 * 64, dtype=torch.bfloat16, device=cuda)
    Y = torch.empty(64, 128, device=cuda)
    rc = lib.lgnn_bf16_gemm(_lib.ptr(A), 0, 64, 30, _lib.ptr(Wb), None, 128, _lib.ptr(Y), None,
                            None, None)
    assert rc == -22  # LGNN_EINVAL
    rc = lib.lgnn_bf16_gemm(_lib.ptr(A), 0, 64, 32, _lib.ptr(Wb), None, 129, _lib.ptr(Y), None,
                            None, None)
    assert rc == -22  # LGNN_EINVAL


@pytest.mark.parametrize("M,bias", [(42279, False), (4133, True), (1, True)])
def test_colsum_rides_along(cuda, M, bias):
    """want_colsum: the per-tile column sums the GEMM writes reduce (fixed order) to Y.sum(0);
    colsum_of refuses a Y modified in place."""
    K, N = 128, 128
    g = torch.Generator().manual_seed(M)
    A = torch.randn(M, K, generator=g).to(cuda).to(torch.bfloat16)
    W = _weights(N, K, cuda, seed=5)
    b = torch.randn(N, generator=g).to(cuda) if bias else None
    Wb, _ = ops.bf16_weight_operands(W, False)
    Y, _ = ops.bf16_gemm(A, Wb, b, N, want_colsum=True)
    cs = ops.colsum_of(Y)
    ref = Y.double().sum(0)
    bound = 2.0 ** -18 * Y.double().abs().sum(0) + 1e-30
    assert ((cs.double() - ref).abs() <= bound).all()
    Y.add_(1.0)
    assert ops.colsum_of(Y) is None
