"""Autograd ops over the HIP kernels of liblgnn.so. No CPU path: every op requires GPU tensors.

- `node_linear`     Y = act(P(X) W^T + b), P = identity or the CSR aggregation (GCN/GIN conv)
- `spmm`            Y = A X (+ self term) — torch_sparse spmm / PyG propagate(aggr='add')
- `pool_head`       logits = pool(H) Wout^T + bout (global_mean/add_pool + out_proj)
- `segment_pool`    pool(H) alone
- `gcn_stack`       the whole GCN model body as ONE autograd node: in_proj -> L x (GCNConv, ELU)
                    -> pool -> out_proj, with a fused backward chain (pool-broadcast and the
                    transposed aggregation feed the next kernel's prologue, never materialised).
"""
from __future__ import annotations

import torch

from . import _lib
from .graph import Csr, Graph


def _f32c(t: torch.Tensor) -> torch.Tensor:
    if t.dtype != torch.float32:
        raise TypeError(f"expected float32, got {t.dtype}")
    return t.contiguous()


def _s(dev) -> int:
    return _lib.stream(dev)


# ----------------------------------------------------------------------------------------------
# raw launches
# ----------------------------------------------------------------------------------------------


def fast_shape(K: int, N: int) -> bool:
    """Shapes served by the tile fast path (tile.hip): S can be saved in the forward."""
    return K <= 128 and N <= 128 and K % 4 == 0 and N % 4 == 0


def linear_fwd(x: torch.Tensor, W: torch.Tensor, b: torch.Tensor | None, act: int,
               csr: Csr | None = None, self_scale: float = 0.0, save_s: bool = False):
    """Y = act(P(x) W^T + b). With save_s (aggregating fast-path shapes) also returns S = P(x)."""
    M, K = x.shape
    N = W.size(0)
    y = torch.empty(M, N, dtype=torch.float32, device=x.device)
    s_out = torch.empty(M, K, dtype=torch.float32, device=x.device) if save_s else None
    _lib.call("lgnn_node_linear_fwd", _lib.ptr(x), M, K,
              _lib.ptr(csr.rowptr) if csr else None, _lib.ptr(csr.col) if csr else None,
              _lib.ptr(csr.w) if csr else None, float(self_scale), _lib.ptr(W), _lib.ptr(b), N,
              act, _lib.ptr(y), _lib.ptr(s_out), _s(x.device))
    return (y, s_out) if save_s else y


def num_partials(M: int, N: int, K: int, gather: bool = False) -> int:
    p = _lib.load().lgnn_bwd_num_partials(M, N, K, int(gather))
    _lib.check(0 if p > 0 else p, "lgnn_bwd_num_partials")
    return p


def linear_bwd(grad_mode: int, dY: torch.Tensor, *, H: torch.Tensor | None, act: int,
               X: torch.Tensor, W: torch.Tensor, csr: Csr | None = None, self_scale: float = 0.0,
               graph: Graph | None = None, pool_mean: bool = True, tcsr: Csr | None = None,
               tself: float = 0.0, want_dx: bool = True, want_db: bool = True):
    """Returns (dXpre or None, dW, db or None). dXpre = dZ W (pre-aggregation input grad)."""
    M, K = X.shape
    N = W.size(0)
    dev = X.device
    P = num_partials(M, N, K, csr is not None)
    slab = torch.empty(P * N * K + (P * N if want_db else 0), dtype=torch.float32, device=dev)
    dWp = slab[: P * N * K]
    dbp = slab[P * N * K:] if want_db else None
    dX = torch.empty(M, K, dtype=torch.float32, device=dev) if want_dx else None
    batch = graph.batch if graph is not None else None
    gptr = graph.gptr if graph is not None else None
    _lib.call(
        "lgnn_node_linear_bwd", grad_mode, _lib.ptr(dY), _lib.ptr(batch), _lib.ptr(gptr),
        int(pool_mean), _lib.ptr(tcsr.tptr) if tcsr else None,
        _lib.ptr(tcsr.tidx) if tcsr else None, _lib.ptr(tcsr.tw) if tcsr else None, float(tself),
        _lib.ptr(H), act, _lib.ptr(X), M, K, _lib.ptr(csr.rowptr) if csr else None,
        _lib.ptr(csr.col) if csr else None, _lib.ptr(csr.w) if csr else None, float(self_scale),
        _lib.ptr(W), N, _lib.ptr(dX), _lib.ptr(dWp), _lib.ptr(dbp), P, _s(dev))
    dW = torch.empty(N, K, dtype=torch.float32, device=dev)
    _lib.call("lgnn_reduce_partials", _lib.ptr(dWp), P, N * K, _lib.ptr(dW), _s(dev))
    db = None
    if want_db:
        db = torch.empty(N, dtype=torch.float32, device=dev)
        _lib.call("lgnn_reduce_partials", _lib.ptr(dbp), P, N, _lib.ptr(db), _s(dev))
    return dX, dW, db


def spmm_raw(rowptr, col, w, self_scale: float, x: torch.Tensor) -> torch.Tensor:
    M, D = x.shape
    y = torch.empty_like(x)
    _lib.call("lgnn_spmm", _lib.ptr(rowptr), _lib.ptr(col), _lib.ptr(w), float(self_scale),
              _lib.ptr(x), M, D, _lib.ptr(y), _s(x.device))
    return y


def pool_head_fwd(H: torch.Tensor, graph: Graph, mean: bool, Wout=None, bout=None):
    B, D = graph.num_graphs, H.size(1)
    pooled = torch.empty(B, D, dtype=torch.float32, device=H.device)
    C = Wout.size(0) if Wout is not None else 0
    logits = torch.empty(B, C, dtype=torch.float32, device=H.device) if Wout is not None else None
    _lib.call("lgnn_pool_head_fwd", _lib.ptr(H), _lib.ptr(graph.gptr), B, D, int(mean),
              _lib.ptr(Wout), _lib.ptr(bout), C, _lib.ptr(pooled), _lib.ptr(logits),
              _s(H.device))
    return pooled, logits


def pool_head_bwd(dlogits: torch.Tensor, pooled: torch.Tensor, Wout: torch.Tensor):
    B, D = pooled.shape
    C = Wout.size(0)
    dev = pooled.device
    dp = torch.empty(B, D, dtype=torch.float32, device=dev)
    dWo = torch.empty(C, D, dtype=torch.float32, device=dev)
    dbo = torch.empty(C, dtype=torch.float32, device=dev)
    _lib.call("lgnn_pool_head_bwd", _lib.ptr(dlogits), _lib.ptr(pooled), B, D, _lib.ptr(Wout), C,
              _lib.ptr(dp), _lib.ptr(dWo), _lib.ptr(dbo), _s(dev))
    return dp, dWo, dbo


def pool_bwd(dpooled: torch.Tensor, graph: Graph, mean: bool, M: int) -> torch.Tensor:
    D = dpooled.size(1)
    dH = torch.empty(M, D, dtype=torch.float32, device=dpooled.device)
    _lib.call("lgnn_pool_bwd", _lib.ptr(dpooled), _lib.ptr(graph.batch), _lib.ptr(graph.gptr), M,
              D, int(mean), _lib.ptr(dH), _s(dpooled.device))
    return dH


# ----------------------------------------------------------------------------------------------
# autograd functions
# ----------------------------------------------------------------------------------------------


class _NodeLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, b, graph, kind, self_scale, act):
        _lib.require_gpu(x, W)
        x, W = _f32c(x), _f32c(W)
        b = _f32c(b) if b is not None else None
        csr = graph.csr(kind) if graph is not None else None
        y = linear_fwd(x, W, b, act, csr, self_scale)
        ctx.save_for_backward(x, W, y)
        ctx.graph, ctx.kind, ctx.self_scale, ctx.act = graph, kind, self_scale, act
        ctx.has_b = b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, W, y = ctx.saved_tensors
        csr = ctx.graph.csr(ctx.kind) if ctx.graph is not None else None
        want_dx = ctx.needs_input_grad[0]
        dxpre, dW, db = linear_bwd(_lib.LGNN_GRAD_DIRECT, _f32c(dy), H=y, act=ctx.act, X=x, W=W,
                                   csr=csr, self_scale=ctx.self_scale, want_dx=want_dx,
                                   want_db=ctx.has_b)
        dx = None
        if want_dx:
            dx = dxpre if csr is None else spmm_raw(csr.tptr, csr.tidx, csr.tw, ctx.self_scale,
                                                     dxpre)
        return dx, dW, db, None, None, None, None


def node_linear(x, W, b=None, graph: Graph | None = None, kind: str = "gcn",
                self_scale: float = 0.0, act: int = _lib.LGNN_ACT_NONE):
    return _NodeLinear.apply(x, W, b, graph, kind, self_scale, act)


class _Spmm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, graph, kind, self_scale):
        _lib.require_gpu(x)
        c = graph.csr(kind)
        ctx.graph, ctx.kind, ctx.self_scale = graph, kind, self_scale
        return spmm_raw(c.rowptr, c.col, c.w, self_scale, _f32c(x))

    @staticmethod
    def backward(ctx, dy):
        c = ctx.graph.csr(ctx.kind)
        return spmm_raw(c.tptr, c.tidx, c.tw, ctx.self_scale, _f32c(dy)), None, None, None


def spmm(x, graph: Graph, kind: str = "gin", self_scale: float = 0.0):
    return _Spmm.apply(x, graph, kind, self_scale)


class _Pool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, graph, mean):
        _lib.require_gpu(x)
        pooled, _ = pool_head_fwd(_f32c(x), graph, mean)
        ctx.graph, ctx.mean, ctx.M = graph, mean, x.size(0)
        return pooled

    @staticmethod
    def backward(ctx, dp):
        return pool_bwd(_f32c(dp), ctx.graph, ctx.mean, ctx.M), None, None


def segment_pool(x, graph: Graph, mean: bool = True):
    return _Pool.apply(x, graph, mean)


class _PoolHead(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, Wout, bout, graph, mean):
        _lib.require_gpu(x, Wout)
        pooled, logits = pool_head_fwd(_f32c(x), graph, mean, _f32c(Wout), _f32c(bout))
        ctx.save_for_backward(pooled, Wout)
        ctx.graph, ctx.mean, ctx.M = graph, mean, x.size(0)
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        pooled, Wout = ctx.saved_tensors
        dp, dWo, dbo = pool_head_bwd(_f32c(dlogits), pooled, Wout)
        dx = pool_bwd(dp, ctx.graph, ctx.mean, ctx.M) if ctx.needs_input_grad[0] else None
        return dx, dWo, dbo, None, None


def pool_head(x, Wout, bout, graph: Graph, mean: bool = True):
    return _PoolHead.apply(x, Wout, bout, graph, mean)


class _GCNStack(torch.autograd.Function):
    """in_proj -> L x ELU(GCNConv) -> pool -> out_proj as one autograd node (dropout p = 0 or
    eval). params = [W_in, b_in, (W_l, b_l) * L, W_out, b_out]."""

    @staticmethod
    def forward(ctx, x, graph, mean, L, *params):
        _lib.require_gpu(x, *params)
        x = _f32c(x)
        params = [_f32c(p) for p in params]
        csr = graph.csr("gcn")
        W_in, b_in = params[0], params[1]
        hs = [linear_fwd(x, W_in, b_in, _lib.LGNN_ACT_NONE)]
        ss = []  # aggregated conv inputs S_l = A_hat H_{l-1} (saved when the fast path applies)
        ctx.saved_s = []
        for l in range(L):
            W, b = params[2 + 2 * l], params[3 + 2 * l]
            fast = fast_shape(W.size(1), W.size(0))
            if fast:
                h, s_ = linear_fwd(hs[-1], W, b, _lib.LGNN_ACT_ELU, csr, save_s=True)
            else:
                h, s_ = linear_fwd(hs[-1], W, b, _lib.LGNN_ACT_ELU, csr), hs[-1]
            hs.append(h)
            ss.append(s_)
            ctx.saved_s.append(fast)
        W_out, b_out = params[2 + 2 * L], params[3 + 2 * L]
        pooled, logits = pool_head_fwd(hs[-1], graph, mean, W_out, b_out)
        ctx.save_for_backward(x, pooled, *hs, *ss, *params)
        ctx.graph, ctx.mean, ctx.L = graph, mean, L
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        L = ctx.L
        saved = ctx.saved_tensors
        x, pooled = saved[0], saved[1]
        hs = saved[2:3 + L]
        ss = saved[3 + L:3 + 2 * L]
        params = saved[3 + 2 * L:]
        graph = ctx.graph
        csr = graph.csr("gcn")
        W_out = params[2 + 2 * L]
        dp, dWo, dbo = pool_head_bwd(_f32c(dlogits), pooled, W_out)
        grads = [None] * len(params)
        grads[2 + 2 * L], grads[3 + 2 * L] = dWo, dbo
        dS = None
        for l in reversed(range(L)):
            W = params[2 + 2 * l]
            if l == L - 1:
                mode, dY, tc = _lib.LGNN_GRAD_POOL, dp, None
            else:
                mode, dY, tc = _lib.LGNN_GRAD_TRANSPOSE, dS, csr
            saved_s = ctx.saved_s[l]
            dS, dW, db = linear_bwd(mode, dY, H=hs[l + 1], act=_lib.LGNN_ACT_ELU,
                                    X=ss[l] if saved_s else hs[l], W=W,
                                    csr=None if saved_s else csr, graph=graph,
                                    pool_mean=ctx.mean, tcsr=tc)
            grads[2 + 2 * l], grads[3 + 2 * l] = dW, db
        # in_proj: dH0 = A^T dS_1 (transposed aggregation in the prologue); dx = dH0 W_in
        want_dx = ctx.needs_input_grad[0]
        if L > 0:
            mode, dY, tc = _lib.LGNN_GRAD_TRANSPOSE, dS, csr
        else:
            mode, dY, tc = _lib.LGNN_GRAD_POOL, dp, None
        dx, dW, db = linear_bwd(mode, dY, H=None, act=_lib.LGNN_ACT_NONE, X=x, W=params[0],
                                graph=graph, pool_mean=ctx.mean, tcsr=tc,
                                want_dx=want_dx)
        grads[0], grads[1] = dW, db
        return (dx, None, None, None, *grads)


def gcn_stack(x, graph: Graph, params: list[torch.Tensor], L: int, mean: bool = True):
    return _GCNStack.apply(x, graph, mean, L, *params)
