"""torch.library registration of the HIP ops: the `torch.compile(model, dynamic=True)` path.

The reference wraps its models in `torch.compile(model, dynamic=True)` when the config asks for
it (src/lesion_gnn/models/gin.py:56, gat.py:84, drgnet.py:103; configs/config.py:64 sets
compile=True for the GAT run). Under Dynamo every op of this package dispatches here instead of
to its eager `torch.autograd.Function` (ops.py): each HIP op is a `torch.library.custom_op` in
namespace `lgnn` with
  * a real (CUDA-key, i.e. HIP) implementation that runs the same eager code — the same kernels
    through the same C ABI — on a stub autograd context,
  * a fake (meta) implementation giving output shapes from symbolic input shapes (dynamic=True),
  * `register_autograd` wiring its backward to a second custom op (`lgnn::<op>_bwd`).
The graph structure is built by `lgnn::graph_build` / `lgnn::batch_ptr` / `lgnn::weighted_csr`,
so a compiled model's FX graph holds only `lgnn` ops: no graph break, and nothing for Inductor to
generate (every kernel is already a hand-written fused HIP kernel).

A graph's CSR travels between ops as one `list[Tensor]` bundle (`GPARTS` order below); an absent
member is a 0-element uint8 tensor (`_none`). SyncBatchNorm (a torch.distributed all-reduce in the
middle of GINConv) is not supported under compile and raises.
"""
from __future__ import annotations

import types
from typing import Optional

import torch
from torch import Tensor
from torch.library import custom_op

from . import _lib
from .graph import Csr

GPARTS = ("rowptr", "col", "w", "tptr", "tidx", "tw", "tmap", "tile_open", "err", "batch", "gptr")


def _none(dev) -> Tensor:
    return torch.empty(0, dtype=torch.uint8, device=dev)


def _is_none(t: Tensor | None) -> bool:
    return t is None or (t.dtype == torch.uint8 and t.numel() == 0)


def _opt(t: Tensor) -> Tensor | None:
    return None if _is_none(t) else t


def _enc(t: Tensor | None, dev) -> Tensor:
    return _none(dev) if t is None else t


class _Ctx:
    """Stand-in for an autograd ctx: lets a custom op's real implementation run the eager
    autograd.Function's forward / backward body unchanged."""

    def __init__(self, needs_input_grad=()):
        self.saved_tensors = ()
        self.needs_input_grad = tuple(needs_input_grad)

    def save_for_backward(self, *ts):
        self.saved_tensors = ts

    def mark_non_differentiable(self, *ts):
        pass


class TGraph:
    """The graph view the eager op bodies read (csr(kind), tile_open(kind), batch, gptr,
    num_graphs), rebuilt from a GPARTS bundle inside a custom op's real implementation."""

    def __init__(self, parts: list[Tensor], kind: str = ""):
        p = dict(zip(GPARTS, parts))
        self.batch = _opt(p["batch"])
        self.gptr = _opt(p["gptr"])
        self.num_graphs = self.gptr.numel() - 1 if self.gptr is not None else None
        self.num_nodes = p["rowptr"].numel() - 1 if not _is_none(p["rowptr"]) else (
            self.batch.numel() if self.batch is not None else 0)
        self._kind = kind
        self._csr = None
        if not _is_none(p["rowptr"]):
            self._csr = Csr(rowptr=p["rowptr"], col=p["col"], w=p["w"], tptr=p["tptr"],
                            tidx=p["tidx"], tw=p["tw"], tmap=_opt(p["tmap"]),
                            tile_open=_opt(p["tile_open"]), err=p["err"])

    def csr(self, kind: str) -> Csr:
        if self._csr is None:
            raise RuntimeError(f"graph bundle carries no CSR (asked for {kind!r})")
        return self._csr

    def csr_planes(self, kind: str, planes=None) -> tuple[Csr, bool]:
        return self.csr(kind), False  # built by its own op: the caller splits the planes

    def tile_open(self, kind: str) -> Tensor:
        return self.csr(kind).tile_open


def gparts(graph, kind: str | None) -> list[Tensor]:
    """GPARTS bundle of a (traced) Graph for one CSR kind (None: pool-only, batch + gptr)."""
    dev = graph.device
    c = graph.csr(kind) if kind is not None else None
    vals = [None] * 9 if c is None else [c.rowptr, c.col, c.w, c.tptr, c.tidx, c.tw, c.tmap,
                                         c.tile_open, c.err]
    return [_enc(t, dev) for t in vals] + [_enc(graph.batch, dev), _enc(graph.gptr, dev)]


# ----------------------------------------------------------------------------------------------
# graph structure
# ----------------------------------------------------------------------------------------------


@custom_op("lgnn::graph_build", mutates_args=(), device_types="cuda")
def graph_build(edge_index: Tensor, num_nodes: int, kind: str) -> list[Tensor]:
    """lgnn_graph_build for one kind: [rowptr, col, w, tptr, tidx, tw, tmap, tile_open, err]."""
    from .graph import Graph

    g = Graph(edge_index, num_nodes)
    c = g.csr(kind)
    dev = edge_index.device
    return [c.rowptr, c.col, c.w, c.tptr, c.tidx, c.tw, _enc(c.tmap, dev),
            _enc(c.tile_open, dev), c.err]


@graph_build.register_fake
def _(edge_index, num_nodes, kind):
    return _graph_build_fake(edge_index, num_nodes, kind)


@custom_op("lgnn::graph_build_b", mutates_args=(), device_types="cuda")
def graph_build_b(edge_index: Tensor, num_nodes: int, kind: str, batch: Tensor,
                  num_graphs: int) -> list[Tensor]:
    """graph_build with the batch vector: the graph offsets (Batch.ptr) ride along with the
    build's first launch (no separate lgnn_batch_ptr launch): [graph_build's nine, gptr]."""
    from .graph import Graph

    g = Graph(edge_index, num_nodes, batch, num_graphs)
    c = g.csr(kind)
    dev = edge_index.device
    return [c.rowptr, c.col, c.w, c.tptr, c.tidx, c.tw, _enc(c.tmap, dev),
            _enc(c.tile_open, dev), c.err, g.gptr]


@graph_build_b.register_fake
def _(edge_index, num_nodes, kind, batch, num_graphs):
    return _graph_build_fake(edge_index, num_nodes, kind) + [
        batch.new_empty(num_graphs + 1, dtype=torch.int32)]


def _graph_build_fake(edge_index, num_nodes, kind):
    n = num_nodes
    cap = edge_index.shape[1] + n
    i32 = dict(dtype=torch.int32)
    f32 = dict(dtype=torch.float32)
    e = edge_index
    return [e.new_empty(n + 1, **i32), e.new_empty(cap, **i32), e.new_empty(cap, **f32),
            e.new_empty(n + 1, **i32), e.new_empty(cap, **i32), e.new_empty(cap, **f32),
            e.new_empty(cap if kind == "gat" else 0, **(i32 if kind == "gat" else
                                                       dict(dtype=torch.uint8))),
            e.new_empty((n + 63) // 64 + _lib.LGNN_TILE_OPEN_EXTRA if kind == "gcn" else 0,
                        **(i32 if kind == "gcn" else dict(dtype=torch.uint8))),
            e.new_empty(1, **i32)]


@custom_op("lgnn::batch_ptr", mutates_args=(), device_types="cuda")
def batch_ptr(batch: Tensor, num_graphs: int) -> Tensor:
    """lgnn_batch_ptr: Batch.ptr (int32 [B + 1]) from the sorted batch vector."""
    from . import _lib

    gptr = torch.empty(num_graphs + 1, dtype=torch.int32, device=batch.device)
    _lib.call("lgnn_batch_ptr", _lib.ptr(batch), batch.numel(), num_graphs, _lib.ptr(gptr),
              _lib.stream(batch.device))
    return gptr


@batch_ptr.register_fake
def _(batch, num_graphs):
    return batch.new_empty(num_graphs + 1, dtype=torch.int32)


@custom_op("lgnn::weighted_csr", mutates_args=(), device_types="cuda")
def weighted_csr(edge_index: Tensor, edge_weight: Tensor, num_nodes: int,
                 w_like: Tensor) -> list[Tensor]:
    """Per-edge weights gathered into the CSR pair's slots (Graph.weighted): [w, tw]."""
    n = num_nodes
    bad = ((edge_index < 0) | (edge_index >= n)).any(0)
    perm = torch.argsort(edge_index[1].masked_fill(bad, n), stable=True)
    tperm = torch.argsort(edge_index[0].masked_fill(bad, n), stable=True)
    w = edge_weight.detach().to(torch.float32)
    cw, ctw = torch.zeros_like(w_like), torch.zeros_like(w_like)
    cw[: w.numel()] = w[perm]
    ctw[: w.numel()] = w[tperm]
    return [cw, ctw]


@weighted_csr.register_fake
def _(edge_index, edge_weight, num_nodes, w_like):
    return [torch.empty_like(w_like), torch.empty_like(w_like)]


# ----------------------------------------------------------------------------------------------
# node linear (aggregate + Linear + bias + act), dense (library) linear, spmm
# ----------------------------------------------------------------------------------------------


def _grad_list(ts, dev) -> list[Tensor]:
    return [_enc(t, dev) for t in ts]


@custom_op("lgnn::node_linear", mutates_args=(), device_types="cuda")
def node_linear(x: Tensor, W: Tensor, b: Optional[Tensor], g: list[Tensor], kind: str,
                self_scale: float, act: int) -> Tensor:
    from .ops import _NodeLinear

    graph = TGraph(g, kind) if kind else None
    return _NodeLinear.forward(_Ctx(), x, W, b, graph, kind, self_scale, act)


@node_linear.register_fake
def _(x, W, b, g, kind, self_scale, act):
    return x.new_empty(x.shape[0], W.shape[0], dtype=torch.float32)


@custom_op("lgnn::node_linear_bwd", mutates_args=(), device_types="cuda")
def node_linear_bwd(dy: Tensor, x: Tensor, W: Tensor, y: Tensor, has_b: bool, g: list[Tensor],
                    kind: str, self_scale: float, act: int, want_dx: bool) -> list[Tensor]:
    from .ops import _NodeLinear

    ctx = _Ctx((want_dx,))
    ctx.save_for_backward(x.contiguous(), W.contiguous(), y)
    ctx.graph = TGraph(g, kind) if kind else None
    ctx.kind, ctx.self_scale, ctx.act, ctx.has_b = kind, self_scale, act, has_b
    dx, dW, db = _NodeLinear.backward(ctx, dy)[:3]
    return _grad_list([dx, dW, db], x.device)


@node_linear_bwd.register_fake
def _(dy, x, W, y, has_b, g, kind, self_scale, act, want_dx):
    return [torch.empty_like(x) if want_dx else _none(x.device), torch.empty_like(W),
            W.new_empty(W.shape[0]) if has_b else _none(x.device)]


def _node_linear_setup(ctx, inputs, output):
    x, W, b, g, kind, self_scale, act = inputs
    ctx.save_for_backward(x, W, output, *g)
    ctx.meta = (b is not None, kind, self_scale, act)


def _node_linear_backward(ctx, dy):
    x, W, y, *g = ctx.saved_tensors
    has_b, kind, self_scale, act = ctx.meta
    dx, dW, db = torch.ops.lgnn.node_linear_bwd(dy, x, W, y, has_b, g, kind, self_scale, act,
                                                ctx.needs_input_grad[0])
    return _opt(dx), dW, _opt(db), [None] * len(g), None, None, None


node_linear.register_autograd(_node_linear_backward, setup_context=_node_linear_setup)


@custom_op("lgnn::s3_weight_planes_multi", mutates_args=(), device_types="cuda")
def s3_weight_planes_multi(Ws: list[Tensor], transposed: list[bool], bf16: bool) -> Tensor:
    """ops.s3_weight_bundle: every split-3 weight operand of a step in one flat buffer."""
    from .ops import s3_bundle_raw

    return s3_bundle_raw(Ws, transposed, bf16)


@s3_weight_planes_multi.register_fake
def _(Ws, transposed, bf16):
    from .ops import _s3_bundle_sizes

    n = sum(_s3_bundle_sizes([tuple(W.shape) for W in Ws], transposed, bf16))
    return Ws[0].new_empty(n, dtype=torch.int16)


@custom_op("lgnn::dense_linear", mutates_args=(), device_types="cuda")
def dense_linear(x: Tensor, W: Tensor, b: Optional[Tensor], bf16: bool,
                 wp: Optional[Tensor]) -> Tensor:
    from .ops import _DenseLinear

    return _DenseLinear.forward(_Ctx(), x, W, b, bf16, wp)


@dense_linear.register_fake
def _(x, W, b, bf16, wp=None):
    return x.new_empty(x.shape[0], W.shape[0], dtype=torch.float32)


@custom_op("lgnn::dense_linear_bwd", mutates_args=(), device_types="cuda")
def dense_linear_bwd(dy: Tensor, x: Tensor, W: Tensor, has_b: bool, bf16: bool,
                     want_dx: bool) -> list[Tensor]:
    from .ops import _DenseLinear, bf16_mfma_fits

    ctx = _Ctx((want_dx,))
    # the MFMA kernels round an fp32 x themselves (as the eager path hands it over)
    xs = x.to(torch.bfloat16) if bf16 and not bf16_mfma_fits(W.shape[0]) else x.contiguous()
    ctx.save_for_backward(xs, W.contiguous())
    ctx.bf16, ctx.has_b = bf16, has_b
    dx, dW, db = _DenseLinear.backward(ctx, dy)[:3]
    return _grad_list([dx, dW, db], x.device)


@dense_linear_bwd.register_fake
def _(dy, x, W, has_b, bf16, want_dx):
    return [torch.empty_like(x) if want_dx else _none(x.device), torch.empty_like(W),
            W.new_empty(W.shape[0]) if has_b else _none(x.device)]


def _dense_setup(ctx, inputs, output):
    x, W, b, bf16, _wp = inputs
    ctx.save_for_backward(x, W)
    ctx.meta = (b is not None, bf16)


def _dense_backward(ctx, dy):
    x, W = ctx.saved_tensors
    has_b, bf16 = ctx.meta
    dx, dW, db = torch.ops.lgnn.dense_linear_bwd(dy, x, W, has_b, bf16, ctx.needs_input_grad[0])
    return _opt(dx), dW, _opt(db), None, None


dense_linear.register_autograd(_dense_backward, setup_context=_dense_setup)


@custom_op("lgnn::spmm", mutates_args=(), device_types="cuda")
def spmm(x: Tensor, g: list[Tensor], self_scale: float, transpose: bool) -> Tensor:
    """Y = A X (+ self_scale X) over the bundle's target CSR, or over its transpose."""
    from .ops import _f32c, spmm_raw

    c = TGraph(g).csr("")
    if transpose:
        return spmm_raw(c.tptr, c.tidx, c.tw, self_scale, _f32c(x))
    return spmm_raw(c.rowptr, c.col, c.w, self_scale, _f32c(x))


@spmm.register_fake
def _(x, g, self_scale, transpose):
    return torch.empty_like(x)


def _spmm_setup(ctx, inputs, output):
    x, g, self_scale, transpose = inputs
    ctx.save_for_backward(*g)
    ctx.meta = (self_scale, transpose)


def _spmm_backward(ctx, dy):
    self_scale, transpose = ctx.meta
    g = list(ctx.saved_tensors)
    return torch.ops.lgnn.spmm(dy, g, self_scale, not transpose), [None] * len(g), None, None


spmm.register_autograd(_spmm_backward, setup_context=_spmm_setup)


# ----------------------------------------------------------------------------------------------
# pooling (+ out_proj)
# ----------------------------------------------------------------------------------------------


@custom_op("lgnn::pool_head", mutates_args=(), device_types="cuda")
def pool_head(x: Tensor, Wout: Tensor, bout: Tensor, g: list[Tensor],
              mean: bool) -> list[Tensor]:
    from .ops import _f32c, pool_head_fwd

    pooled, logits = pool_head_fwd(_f32c(x), TGraph(g), mean, _f32c(Wout), _f32c(bout))
    return [logits, pooled]


@pool_head.register_fake
def _(x, Wout, bout, g, mean):
    B = g[GPARTS.index("gptr")].shape[0] - 1
    return [x.new_empty(B, Wout.shape[0]), x.new_empty(B, x.shape[1])]


@custom_op("lgnn::pool_head_bwd", mutates_args=(), device_types="cuda")
def pool_head_bwd(dlogits: Tensor, pooled: Tensor, Wout: Tensor, g: list[Tensor], mean: bool,
                  num_nodes: int, want_dx: bool) -> list[Tensor]:
    from .ops import _f32c, pool_bwd, pool_head_bwd as phb

    dp, dWo, dbo = phb(_f32c(dlogits), pooled, Wout)
    dx = pool_bwd(dp, TGraph(g), mean, num_nodes) if want_dx else None
    return _grad_list([dx, dWo, dbo], pooled.device)


@pool_head_bwd.register_fake
def _(dlogits, pooled, Wout, g, mean, num_nodes, want_dx):
    dx = pooled.new_empty(num_nodes, pooled.shape[1]) if want_dx else _none(pooled.device)
    return [dx, torch.empty_like(Wout), Wout.new_empty(Wout.shape[0])]


def _pool_head_setup(ctx, inputs, output):
    x, Wout, bout, g, mean = inputs
    ctx.save_for_backward(output[1], Wout, *g)
    ctx.meta = (mean, x.shape[0])


def _pool_head_backward(ctx, grads):
    pooled, Wout, *g = ctx.saved_tensors
    mean, M = ctx.meta
    dx, dWo, dbo = torch.ops.lgnn.pool_head_bwd(grads[0], pooled, Wout, g, mean, M,
                                                ctx.needs_input_grad[0])
    return _opt(dx), dWo, dbo, [None] * len(g), None


pool_head.register_autograd(_pool_head_backward, setup_context=_pool_head_setup)


@custom_op("lgnn::segment_pool", mutates_args=(), device_types="cuda")
def segment_pool(x: Tensor, g: list[Tensor], mean: bool) -> Tensor:
    from .ops import _f32c, pool_head_fwd

    return pool_head_fwd(_f32c(x), TGraph(g), mean)[0]


@segment_pool.register_fake
def _(x, g, mean):
    return x.new_empty(g[GPARTS.index("gptr")].shape[0] - 1, x.shape[1])


@custom_op("lgnn::segment_pool_bwd", mutates_args=(), device_types="cuda")
def segment_pool_bwd(dp: Tensor, g: list[Tensor], mean: bool, num_nodes: int) -> Tensor:
    from .ops import _f32c, pool_bwd

    return pool_bwd(_f32c(dp), TGraph(g), mean, num_nodes)


@segment_pool_bwd.register_fake
def _(dp, g, mean, num_nodes):
    return dp.new_empty(num_nodes, dp.shape[1])


def _segpool_setup(ctx, inputs, output):
    x, g, mean = inputs
    ctx.save_for_backward(*g)
    ctx.meta = (mean, x.shape[0])


def _segpool_backward(ctx, dp):
    mean, M = ctx.meta
    g = list(ctx.saved_tensors)
    return torch.ops.lgnn.segment_pool_bwd(dp, g, mean, M), [None] * len(g), None


segment_pool.register_autograd(_segpool_backward, setup_context=_segpool_setup)


# ----------------------------------------------------------------------------------------------
# dropout (lesion_gnn_amd.dropout): masks from the device generator, the mask product
# ----------------------------------------------------------------------------------------------


@custom_op("lgnn::dropout_masks", mutates_args=("state",), device_types="cuda",
           tags=(torch.Tag.nondeterministic_seeded,))
def dropout_masks(state: Tensor, numels: list[int], thr: int, scale: float) -> Tensor:
    """lgnn_dropout_masks: every mask in one flat fp32 tensor (lesion_gnn_amd.dropout layout),
    the state's counter advanced. Tagged nondeterministic_seeded so the compiler neither merges
    two calls nor recomputes one in the backward (the backward needs the forward's masks)."""
    from .dropout import dropout_masks_raw

    return dropout_masks_raw(state, list(numels), thr, scale)


@dropout_masks.register_fake
def _(state, numels, thr, scale):
    tot = 0
    for n in numels:
        tot += (n + 3) // 4 * 4
    return state.new_empty(tot, dtype=torch.float32)


@custom_op("lgnn::mask_mul", mutates_args=(), device_types="cuda")
def mask_mul(x: Tensor, m: Tensor) -> Tensor:
    """lgnn_mask_mul: x * m (dropout between convs)."""
    from .dropout import _mul

    return _mul(x, m)


@mask_mul.register_fake
def _(x, m):
    return torch.empty_like(x)


def _mask_mul_setup(ctx, inputs, output):
    ctx.save_for_backward(inputs[1])


def _mask_mul_backward(ctx, grad):
    (m,) = ctx.saved_tensors
    return torch.ops.lgnn.mask_mul(grad, m), None


mask_mul.register_autograd(_mask_mul_backward, setup_context=_mask_mul_setup)


# ----------------------------------------------------------------------------------------------
# GATConv
# ----------------------------------------------------------------------------------------------


@custom_op("lgnn::gat_conv", mutates_args=(), device_types="cuda")
def gat_conv(x: Tensor, W: Tensor, att_src: Tensor, att_dst: Tensor, bias: Optional[Tensor],
             g: list[Tensor], heads: int, slope: float, mask: Optional[Tensor], act: int,
             bf16: bool, wp: Optional[Tensor], wpt: Optional[Tensor]) -> list[Tensor]:
    """[Y, XP, a_s, a_d, alpha] (the eager _GATConv forward and what it saves)."""
    from .ops import _GATConv

    ctx = _Ctx()
    Y = _GATConv.forward(ctx, x, W, att_src, att_dst, bias, TGraph(g, "gat"), heads, slope, mask,
                         act, bf16, wp)
    _x, _W, _as, _ad, XP, a_s, a_d, alpha, _Y, _m = ctx.saved_tensors
    return [Y, XP, a_s, a_d, alpha]


@gat_conv.register_fake
def _(x, W, att_src, att_dst, bias, g, heads, slope, mask, act, bf16, wp=None, wpt=None):
    M, HC = x.shape[0], W.shape[0]
    cap = g[GPARTS.index("col")].shape[0]
    return [x.new_empty(M, HC), x.new_empty(M, HC), x.new_empty(M, heads),
            x.new_empty(M, heads), x.new_empty(cap, heads)]


@custom_op("lgnn::gat_conv_bwd", mutates_args=(), device_types="cuda")
def gat_conv_bwd(dY: Tensor, x: Tensor, W: Tensor, att_src: Tensor, att_dst: Tensor,
                 XP: Tensor, a_s: Tensor, a_d: Tensor, alpha: Tensor, Y: Tensor,
                 mask: Optional[Tensor], g: list[Tensor], heads: int, slope: float, act: int,
                 bf16: bool, has_bias: bool, want_dx: bool,
                 wpt: Optional[Tensor]) -> list[Tensor]:
    from .ops import GAT_S3, _GATConv, fast_shape

    HC = W.shape[0]
    ctx = _Ctx((want_dx,))
    ctx.wpt = wpt
    ctx.save_for_backward(x.contiguous(), W.contiguous(), att_src.reshape(-1),
                          att_dst.reshape(-1), XP, a_s, a_d, alpha, Y, mask)
    ctx.graph, ctx.heads, ctx.slope, ctx.act = TGraph(g, "gat"), heads, slope, act
    ctx.bf16, ctx.dense = bf16, bf16 or not fast_shape(W.shape[1], HC) or GAT_S3
    ctx.has_bias = has_bias
    ctx.att_shape = tuple(att_src.shape)
    dx, dW = _GATConv.backward(ctx, dY)[:2]
    # the attention / bias gradients are ONE reduction buffer [att_src | att_dst | bias]
    # (outputs of a custom op may not alias each other): returned whole and split into views by
    # the autograd formula below, instead of three copies
    return _grad_list([dx, dW, ctx.red], x.device)


@gat_conv_bwd.register_fake
def _(dY, x, W, att_src, att_dst, XP, a_s, a_d, alpha, Y, mask, g, heads, slope, act, bf16,
      has_bias, want_dx, wpt=None):
    dev = x.device
    return [torch.empty_like(x) if want_dx else _none(dev), torch.empty_like(W),
            W.new_empty(3 * W.shape[0])]


def _gat_setup(ctx, inputs, output):
    x, W, att_src, att_dst, bias, g, heads, slope, mask, act, bf16, _wp, wpt = inputs
    Y, XP, a_s, a_d, alpha = output
    ctx.save_for_backward(x, W, att_src, att_dst, XP, a_s, a_d, alpha, Y,
                          _enc(mask, x.device), _enc(wpt, x.device), *g)
    ctx.meta = (heads, slope, act, bf16, bias is not None)


def _gat_backward(ctx, grads):
    x, W, att_src, att_dst, XP, a_s, a_d, alpha, Y, mask, wpt, *g = ctx.saved_tensors
    heads, slope, act, bf16, has_bias = ctx.meta
    dx, dW, red = torch.ops.lgnn.gat_conv_bwd(
        grads[0], x, W, att_src, att_dst, XP, a_s, a_d, alpha, Y, _opt(mask), g, heads, slope,
        act, bf16, has_bias, ctx.needs_input_grad[0], _opt(wpt))
    HC = W.shape[0]
    da_s = red[:HC].view(att_src.shape)
    da_d = red[HC:2 * HC].view(att_dst.shape)
    db = red[2 * HC:] if has_bias else None
    return (_opt(dx), dW, da_s, da_d, db, [None] * len(g), None, None, None, None, None, None,
            None)


gat_conv.register_autograd(_gat_backward, setup_context=_gat_setup)


@custom_op("lgnn::gat_conv_head", mutates_args=(), device_types="cuda")
def gat_conv_head(x: Tensor, W: Tensor, att_src: Tensor, att_dst: Tensor, bias: Optional[Tensor],
                  W_out: Tensor, b_out: Tensor, g: list[Tensor], heads: int, slope: float,
                  mask: Optional[Tensor], act: int, bf16: bool, mean: bool,
                  wp: Optional[Tensor], wpt: Optional[Tensor]) -> list[Tensor]:
    """The GAT model's last conv + global pool + out_proj as one node (ops._GATConvHead):
    [logits, Y, XP, a_s, a_d, alpha, pooled]."""
    from .ops import _GATConvHead

    ctx = _Ctx()
    logits = _GATConvHead.forward(ctx, x, W, att_src, att_dst, bias, W_out, b_out,
                                  TGraph(g, "gat"), heads, slope, mask, act, bf16, mean, wp)
    s = ctx.saved_tensors  # x, W, att_src, att_dst, XP, a_s, a_d, alpha, Y, mask, pooled, W_out
    return [logits, s[8], s[4], s[5], s[6], s[7], s[10]]


@gat_conv_head.register_fake
def _(x, W, att_src, att_dst, bias, W_out, b_out, g, heads, slope, mask, act, bf16, mean,
      wp=None, wpt=None):
    M, HC = x.shape[0], W.shape[0]
    cap = g[GPARTS.index("col")].shape[0]
    B = g[GPARTS.index("gptr")].shape[0] - 1
    return [x.new_empty(B, W_out.shape[0]), x.new_empty(M, HC), x.new_empty(M, HC),
            x.new_empty(M, heads), x.new_empty(M, heads), x.new_empty(cap, heads),
            x.new_empty(B, HC)]


@custom_op("lgnn::gat_conv_head_bwd", mutates_args=(), device_types="cuda")
def gat_conv_head_bwd(dlogits: Tensor, x: Tensor, W: Tensor, att_src: Tensor, att_dst: Tensor,
                      XP: Tensor, a_s: Tensor, a_d: Tensor, alpha: Tensor, Y: Tensor,
                      mask: Optional[Tensor], pooled: Tensor, W_out: Tensor, g: list[Tensor],
                      heads: int, slope: float, act: int, bf16: bool, has_bias: bool, mean: bool,
                      want_dx: bool, wpt: Optional[Tensor]) -> list[Tensor]:
    """[dx, dW, red (= [datt_src | datt_dst | dbias]), dW_out, db_out]: the readout's backward
    formed inside the edge kernel's load (lgnn_gat_bwd_edge_pool), no dH tensor."""
    from .ops import GAT_S3, _GATConvHead, _SubCtx, fast_shape

    HC = W.shape[0]
    sub = _SubCtx(want_dx)
    sub.graph, sub.heads, sub.slope, sub.act = TGraph(g, "gat"), heads, slope, act
    sub.bf16, sub.dense = bf16, bf16 or not fast_shape(W.shape[1], HC) or GAT_S3
    sub.has_bias = has_bias
    sub.att_shape = tuple(att_src.shape)
    sub.wt = None
    sub.wpt = wpt
    ctx = _Ctx((want_dx,))
    ctx.save_for_backward(x.contiguous(), W.contiguous(), att_src.reshape(-1),
                          att_dst.reshape(-1), XP, a_s, a_d, alpha, Y, mask, pooled, W_out)
    ctx.sub, ctx.head_graph, ctx.head_mean = sub, TGraph(g, "gat"), mean
    grads = _GATConvHead.backward(ctx, dlogits)
    return _grad_list([grads[0], grads[1], sub.red, grads[5], grads[6]], x.device)


@gat_conv_head_bwd.register_fake
def _(dlogits, x, W, att_src, att_dst, XP, a_s, a_d, alpha, Y, mask, pooled, W_out, g, heads,
      slope, act, bf16, has_bias, mean, want_dx, wpt=None):
    dev = x.device
    return [torch.empty_like(x) if want_dx else _none(dev), torch.empty_like(W),
            W.new_empty(3 * W.shape[0]), torch.empty_like(W_out), W_out.new_empty(W_out.shape[0])]


def _gat_head_setup(ctx, inputs, output):
    (x, W, att_src, att_dst, bias, W_out, b_out, g, heads, slope, mask, act, bf16, mean, _wp,
     wpt) = inputs
    _logits, Y, XP, a_s, a_d, alpha, pooled = output
    ctx.save_for_backward(x, W, att_src, att_dst, XP, a_s, a_d, alpha, Y, _enc(mask, x.device),
                          pooled, W_out, _enc(wpt, x.device), *g)
    ctx.meta = (heads, slope, act, bf16, bias is not None, mean)


def _gat_head_backward(ctx, grads):
    (x, W, att_src, att_dst, XP, a_s, a_d, alpha, Y, mask, pooled, W_out, wpt,
     *g) = ctx.saved_tensors
    heads, slope, act, bf16, has_bias, mean = ctx.meta
    dx, dW, red, dWo, dbo = torch.ops.lgnn.gat_conv_head_bwd(
        grads[0], x, W, att_src, att_dst, XP, a_s, a_d, alpha, Y, _opt(mask), pooled, W_out, g,
        heads, slope, act, bf16, has_bias, mean, ctx.needs_input_grad[0], _opt(wpt))
    HC = W.shape[0]
    da_s = red[:HC].view(att_src.shape)
    da_d = red[HC:2 * HC].view(att_dst.shape)
    db = red[2 * HC:] if has_bias else None
    return (_opt(dx), dW, da_s, da_d, db, dWo, dbo, [None] * len(g), None, None, None, None,
            None, None, None, None)


gat_conv_head.register_autograd(_gat_head_backward, setup_context=_gat_head_setup)


# ----------------------------------------------------------------------------------------------
# GINConv (MLP with BatchNorm; running statistics mutated in place)
# ----------------------------------------------------------------------------------------------


def _bn_stub(gamma, beta, running_mean, running_var, nbt, bn_eps, momentum):
    track = running_mean is not None
    return types.SimpleNamespace(
        weight=gamma, bias=beta, affine=gamma is not None, track_running_stats=track,
        running_mean=running_mean, running_var=running_var, num_batches_tracked=nbt,
        eps=bn_eps, momentum=None if momentum < 0 else momentum)


@custom_op("lgnn::gin_conv", mutates_args=(), device_types="cuda")
def gin_conv(x: Tensor, W1: Tensor, b1: Tensor, gamma: Optional[Tensor], beta: Optional[Tensor],
             W2: Tensor, b2: Tensor, running_mean: Optional[Tensor],
             running_var: Optional[Tensor], g: list[Tensor], training: bool, eps: float,
             bn_eps: float, mask: Optional[Tensor], act: int) -> list[Tensor]:
    """[H, S or none, Z1, A1, mean, invstd, scale, shift, sums or none] (the eager _GINConv
    forward). Functional: in training the BatchNorm running statistics are NOT updated here —
    lgnn::bn_running_update does it from the returned batch sums (a mutating op cannot carry an
    autograd formula); in eval the running statistics are read."""
    from .ops import _GINConv

    ctx = _Ctx()
    rm, rv = (None, None) if training else (running_mean, running_var)
    bn = _bn_stub(gamma, beta, rm, rv, None, bn_eps, 0.1)
    H = _GINConv.forward(ctx, x, W1, b1, gamma, beta, W2, b2, TGraph(g, "gin"), bn, training,
                         eps, mask, act, None, None)
    S, Z1, A1, _H, _W1, _W2, mean, invstd, scale, shift, _m = ctx.saved_tensors
    return [H, _none(x.device) if ctx.gathered else S, Z1, A1, mean, invstd, scale, shift,
            _enc(ctx.bn_sums, x.device)]


@custom_op("lgnn::bn_running_update", mutates_args=("running_mean", "running_var", "nbt"),
           device_types="cuda")
def bn_running_update(running_mean: Tensor, running_var: Tensor, nbt: Optional[Tensor],
                      sums: Tensor, count: int, bn_eps: float, momentum: float) -> None:
    """BatchNorm1d running statistics from a batch's (sum z, sum z^2) (lgnn_bn_finalize in
    training mode), torch semantics (unbiased variance; momentum < 0: cumulative average)."""
    from .ops import bn_finalize

    bn = _bn_stub(None, None, running_mean, running_var, nbt, bn_eps, momentum)
    bn_finalize(sums, float(count), bn, True, running_mean.numel(), running_mean.device)


@bn_running_update.register_fake
def _(running_mean, running_var, nbt, sums, count, bn_eps, momentum):
    return None


@gin_conv.register_fake
def _(x, W1, b1, gamma, beta, W2, b2, running_mean, running_var, g, training, eps, bn_eps,
      mask, act):
    from .ops import fast_shape, wide_shape

    M, N1 = x.shape[0], W1.shape[0]
    # the eager rule (_GINConv.forward): S is saved for the tile fast path and the wide path
    gathered = not (fast_shape(W1.shape[1], N1) or wide_shape(W1.shape[1], N1))
    S = _none(x.device) if gathered else torch.empty_like(x)
    sums = x.new_empty(2 * N1, dtype=torch.float64) if training else _none(x.device)
    return [x.new_empty(M, W2.shape[0]), S, x.new_empty(M, N1), x.new_empty(M, N1)] + \
        [x.new_empty(N1) for _ in range(4)] + [sums]


@custom_op("lgnn::gin_conv_bwd", mutates_args=(), device_types="cuda")
def gin_conv_bwd(dH: Tensor, S: Tensor, Z1: Tensor, A1: Tensor, H: Tensor, W1: Tensor,
                 W2: Tensor, mean: Tensor, invstd: Tensor, scale: Tensor, shift: Tensor,
                 mask: Optional[Tensor], g: list[Tensor], training: bool, count: int,
                 act: int, affine: bool, gathered: bool, eps: float,
                 want_dx: bool) -> list[Tensor]:
    from .ops import _GINConv, gin_bn_fused

    ctx = _Ctx((want_dx,))
    ctx.save_for_backward(S.contiguous(), Z1, A1, H, W1.contiguous(), W2.contiguous(), mean,
                          invstd, scale, shift, mask)
    ctx.graph, ctx.self_scale, ctx.gathered = TGraph(g, "gin"), 1.0 + eps, gathered
    ctx.training, ctx.count, ctx.group, ctx.act = training, float(count), None, act
    ctx.affine = affine
    ctx.bn_fused = gin_bn_fused(W1.shape[1], W1.shape[0], W2.shape[0])
    grads = _GINConv.backward(ctx, dH)[:7]
    return _grad_list(grads, H.device)


@gin_conv_bwd.register_fake
def _(dH, S, Z1, A1, H, W1, W2, mean, invstd, scale, shift, mask, g, training, count, act,
      affine, gathered, eps, want_dx):
    dev = H.device
    N1 = W1.shape[0]
    dx = S.new_empty(S.shape[0], W1.shape[1]) if want_dx else _none(dev)
    dgb = [W1.new_empty(N1), W1.new_empty(N1)] if affine else [_none(dev), _none(dev)]
    return [dx, torch.empty_like(W1), W1.new_empty(N1)] + dgb + \
        [torch.empty_like(W2), W2.new_empty(W2.shape[0])]


def _gin_setup(ctx, inputs, output):
    (x, W1, b1, gamma, beta, W2, b2, running_mean, running_var, g, training, eps, bn_eps,
     mask, act) = inputs
    H, S, Z1, A1, mean, invstd, scale, shift, _sums = output
    gathered = _is_none(S)
    ctx.save_for_backward(x if gathered else S, Z1, A1, H, W1, W2, mean, invstd, scale, shift,
                          _enc(mask, x.device), *g)
    ctx.meta = (training, x.shape[0], act, gamma is not None, gathered, eps)


def _gin_backward(ctx, grads):
    S, Z1, A1, H, W1, W2, mean, invstd, scale, shift, mask, *g = ctx.saved_tensors
    training, count, act, affine, gathered, eps = ctx.meta
    dx, dW1, db1, dg, dbt, dW2, db2 = torch.ops.lgnn.gin_conv_bwd(
        grads[0], S, Z1, A1, H, W1, W2, mean, invstd, scale, shift, _opt(mask), g, training,
        count, act, affine, gathered, eps, ctx.needs_input_grad[0])
    return (_opt(dx), dW1, db1, _opt(dg), _opt(dbt), dW2, db2, None, None,
            [None] * len(g), None, None, None, None, None)


gin_conv.register_autograd(_gin_backward, setup_context=_gin_setup)


# ----------------------------------------------------------------------------------------------
# the fused GCN model body
# ----------------------------------------------------------------------------------------------


def _gcn_layout(params, L):
    from .ops import STACK_MAX, fast_shape, wide_shape

    Ws = [params[2 * l] for l in range(L + 1)]
    fused = L + 1 <= STACK_MAX and all(fast_shape(W.shape[1], W.shape[0]) for W in Ws)
    # the eager rule (_GCNStack._fwd): S_l is saved for fast-path and wide layers
    saved_s = [True] * L if fused else [
        fast_shape(params[2 + 2 * l].shape[1], params[2 + 2 * l].shape[0]) or
        wide_shape(params[2 + 2 * l].shape[1], params[2 + 2 * l].shape[0]) for l in range(L)]
    return fused, saved_s


@custom_op("lgnn::gcn_stack", mutates_args=(), device_types="cuda")
def gcn_stack(x: Tensor, g: list[Tensor], mean: bool, L: int,
              params: list[Tensor]) -> list[Tensor]:
    """[logits, pooled, H_0..H_L, S_1..S_L, planes_t or none] (the eager _GCNStack forward)."""
    from .ops import _GCNStack, adjt_in_planes

    ctx = _Ctx()
    with adjt_in_planes():  # the op's planes output is a fresh buffer (planes + Â^T room)
        logits = _GCNStack.forward(ctx, x, TGraph(g, "gcn"), mean, L, *params)
    sv = ctx.saved_tensors
    hs = list(sv[2:3 + L])
    ss = [s if s.data_ptr() != x.data_ptr() and all(s.data_ptr() != h.data_ptr() for h in hs)
          else s.clone() for s in sv[3 + L:3 + 2 * L]]
    return [logits, sv[1]] + hs + ss + [_enc(ctx.planes_t, x.device)]


@gcn_stack.register_fake
def _(x, g, mean, L, params):
    from .ops import BWD_S3, MFMA_MODE

    B = g[GPARTS.index("gptr")].shape[0] - 1
    M = x.shape[0]
    Ws = [params[2 * l] for l in range(L + 1)]
    fused, saved_s = _gcn_layout(params, L)
    hs = [x.new_empty(M, W.shape[0]) for W in Ws]
    ss = [x.new_empty(M, Ws[l + 1].shape[1]) for l in range(L)]
    from .ops import bwd_planes_numel

    planes = (x.new_empty(bwd_planes_numel(L, M), dtype=torch.int16)
              if fused and MFMA_MODE == "s3" and BWD_S3 and L >= 1 else _none(x.device))
    return [x.new_empty(B, params[2 + 2 * L].shape[0]), x.new_empty(B, Ws[-1].shape[0])] + hs + \
        ss + [planes]


@custom_op("lgnn::gcn_stack_bwd", mutates_args=(), device_types="cuda")
def gcn_stack_bwd(dlogits: Tensor, x: Tensor, pooled: Tensor, hs: list[Tensor],
                  ss: list[Tensor], params: list[Tensor], planes_t: Tensor, g: list[Tensor],
                  mean: bool, L: int, want_dx: bool) -> list[Tensor]:
    """[dx or none, dparams...]

    The graph's tile_open (in g) is written here although the op declares no mutation: the fused
    backward's barrier words and partial-slot skip words (include/lgnn.h LGNN_SLOT_FLAG0) are
    scratch set and consumed inside this one call, and the next graph build zeroes them; the tile
    flags proper, the only part of tile_open other ops read, are left unchanged."""
    from .ops import _GCNStack

    fused, saved_s = _gcn_layout(params, L)
    ctx = _Ctx((want_dx,))
    ctx.save_for_backward(x.contiguous(), pooled, *hs, *ss, *[p.contiguous() for p in params])
    ctx.fused, ctx.planes_t, ctx.saved_s = fused, _opt(planes_t), saved_s
    ctx.graph, ctx.mean, ctx.L = TGraph(g, "gcn"), mean, L
    out = _GCNStack.backward(ctx, dlogits)
    return _grad_list([out[0]] + list(out[4:]), x.device)


@gcn_stack_bwd.register_fake
def _(dlogits, x, pooled, hs, ss, params, planes_t, g, mean, L, want_dx):
    return [torch.empty_like(x) if want_dx else _none(x.device)] + \
        [torch.empty_like(p) for p in params]


def _gcn_setup(ctx, inputs, output):
    x, g, mean, L, params = inputs
    logits, pooled, *rest = output
    hs, ss, planes = rest[:L + 1], rest[L + 1:2 * L + 1], rest[2 * L + 1]
    ctx.save_for_backward(x, pooled, planes, *hs, *ss, *params, *g)
    ctx.meta = (mean, L, len(params), len(g))


def _gcn_backward(ctx, grads):
    mean, L, npar, ng = ctx.meta
    x, pooled, planes, *rest = ctx.saved_tensors
    hs, ss = rest[:L + 1], rest[L + 1:2 * L + 1]
    params = rest[2 * L + 1:2 * L + 1 + npar]
    g = rest[2 * L + 1 + npar:]
    out = torch.ops.lgnn.gcn_stack_bwd(grads[0], x, pooled, list(hs), list(ss), list(params),
                                       planes, list(g), mean, L, ctx.needs_input_grad[0])
    return _opt(out[0]), [None] * ng, None, None, list(out[1:])


gcn_stack.register_autograd(_gcn_backward, setup_context=_gcn_setup)


# ----------------------------------------------------------------------------------------------
# SortAggregation
# ----------------------------------------------------------------------------------------------


@custom_op("lgnn::sort_pool", mutates_args=(), device_types="cuda")
def sort_pool(x: Tensor, g: list[Tensor], k: int) -> list[Tensor]:
    """[out, rank, fill]"""
    from .ops import _SortPool

    ctx = _Ctx()
    out = _SortPool.forward(ctx, x, TGraph(g), k)
    _x, rank, fill = ctx.saved_tensors
    return [out, rank, fill]


@sort_pool.register_fake
def _(x, g, k):
    B = g[GPARTS.index("gptr")].shape[0] - 1
    return [x.new_empty(B, k * x.shape[1]), x.new_empty(x.shape[0], dtype=torch.int32),
            x.new_empty(1)]


@custom_op("lgnn::sort_pool_bwd", mutates_args=(), device_types="cuda")
def sort_pool_bwd(dout: Tensor, x: Tensor, rank: Tensor, fill: Tensor, g: list[Tensor],
                  k: int) -> Tensor:
    from .ops import _SortPool

    ctx = _Ctx()
    ctx.save_for_backward(x.contiguous(), rank, fill)
    ctx.graph, ctx.k = TGraph(g), k
    return _SortPool.backward(ctx, dout)[0]


@sort_pool_bwd.register_fake
def _(dout, x, rank, fill, g, k):
    return torch.empty_like(x)


def _sort_setup(ctx, inputs, output):
    x, g, k = inputs
    ctx.save_for_backward(x, output[1], output[2], *g)
    ctx.k = k


def _sort_backward(ctx, grads):
    x, rank, fill, *g = ctx.saved_tensors
    return (torch.ops.lgnn.sort_pool_bwd(grads[0], x, rank, fill, list(g), ctx.k),
            [None] * len(g), None)


sort_pool.register_autograd(_sort_backward, setup_context=_sort_setup)


def gparts_empty(dev) -> list[Tensor]:
    return [_none(dev) for _ in GPARTS]
