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

import ctypes
import weakref

import torch

from . import _lib
from .graph import Csr, Graph


def _compiling() -> bool:
    """True while torch.compile / torch.export traces: the ops then dispatch to their
    torch.library custom ops (library.py) instead of the eager autograd.Functions."""
    return torch.compiler.is_compiling()


def _lgnn():
    from . import library

    return library


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


# Wide linears (K or N > 128: the reference sweep's widths 256 / 512, scripts/sweep.py:126) run as
# the aggregation (lgnn_spmm) + the split-3 dense GEMMs (s3gemm.hip) instead of the fp32 generic
# node kernels, which stream the weight per 128-wide block and re-derive dZ per output block
# (GIN [512]*4: dX 1.4 ms per launch). WIDE = "f32" keeps the generic kernels (A/B).
WIDE = "s3"


def wide_shape(K: int, N: int) -> bool:
    return WIDE == "s3" and (K > 128 or N > 128) and K % 4 == 0 and N % 4 == 0


def linear_fwd(x: torch.Tensor, W: torch.Tensor, b: torch.Tensor | None, act: int,
               csr: Csr | None = None, self_scale: float = 0.0, save_s: bool = False):
    """Y = act(P(x) W^T + b). With save_s (aggregating fast-path and wide shapes) also returns
    S = P(x)."""
    M, K = x.shape
    N = W.size(0)
    if wide_shape(K, N):
        S = spmm_raw(csr.rowptr, csr.col, csr.w, self_scale, x) if csr is not None else x
        Wp = dense_planes(W, False, False)
        y = torch.empty(M, N, dtype=torch.float32, device=x.device)
        for r0, r1 in _row_blocks(M, K, N):
            _lib.call("lgnn_s3_gemm_act", _lib.ptr(S) + r0 * K * 4, r1 - r0, K, _lib.ptr(Wp), N,
                      _lib.ptr(b), act, _lib.ptr(y) + r0 * N * 4, _s(x.device))
        return (y, S) if save_s else y
    y = torch.empty(M, N, dtype=torch.float32, device=x.device)
    s_out = torch.empty(M, K, dtype=torch.float32, device=x.device) if save_s else None
    _lib.call("lgnn_node_linear_fwd", _lib.ptr(x), M, K,
              _lib.ptr(csr.rowptr) if csr else None, _lib.ptr(csr.col) if csr else None,
              _lib.ptr(csr.w) if csr else None, float(self_scale), _lib.ptr(W), _lib.ptr(b), N,
              act, _lib.ptr(y), _lib.ptr(s_out), _s(x.device))
    return (y, s_out) if save_s else y


STACK_MAX = 8  # LGNN_MAX_STACK


# fused stack backward on/off (FUSED_BWD = False selects the layer-wise backward; diagnostics)
FUSED_BWD = True
# the fused stack's graph build skips the transpose CSR when no tile is open
# (LAZY_TRANSPOSE = False: always built)
LAZY_TRANSPOSE = True


# GEMM arithmetic of the fused GCN stack: "s3" = bf16 MFMA on three-plane split operands (fp32
# accuracy, stack3.hip), "f32" = fp32 MFMA (tile.hip). MFMA_MODE = "f32" selects the latter.
MFMA_MODE = "s3"
# Backward of the fused stack (BWD_MODE): "f32" = the fp32 fused kernel (tile.hip k_stack_bwd, one
# launch); "s3" = the split-3 layer-major kernels (stack3_bwd.hip k_s3_bwd: one launch per layer,
# dZ through HBM, 512 partial slots); "s3f" = the fused split-3 kernel (stack3_bwd.hip
# k_s3_fbwd: every layer of a tile in one pass, one launch, 256 slots; the default: 121 us vs
# 154 us for f32 at C2 on MI355X). s3 / s3f need the split-3 forward (their transposed weight
# planes come out of its weight-plane launch); otherwise the f32 kernel runs.
BWD_MODE = "s3f"
BWD_S3 = BWD_MODE in ("s3", "s3f")
# open tiles (an edge leaves them) inside the fused split-3 launches, layer by layer behind grid
# barriers, instead of three layer-wise launches per direction (OPEN_IN_FUSED = "0": separate)
# The fused kernels' open phase saves the six layer-wise launches (~4.5 us each), but runs the
# open tiles ~1.5x slower than the standalone layer-wise kernels (measured C5, r02j). So it is
# taken when open tiles are expected to be rare: "auto" (default) = when every graph could sit
# whole in 64-node tiles (all graphs of one size that divides or is a multiple of 64: the
# batch's node count is B * n with 64 % n == 0 or n % 64 == 0). Either choice is exact; "1" /
# "0" force it (also "fwd" / "bwd" for one direction).
OPEN_IN_FUSED = "auto"
OPEN_IN_FUSED_BWD = OPEN_IN_FUSED
# dP = dlogits W_out formed inside the single-launch split-3 backward (HEAD_FOLD = False: by
# lgnn_pool_head_bwd before it)
HEAD_FOLD = True
_CAPACITY: dict = {}


def fused_grid_capacity(direction: str, dev) -> int:
    """Workgroups of the fused split-3 forward / backward kernel the device holds at once
    (lgnn_fused_grid_capacity: occupancy per CU x CU count), cached per device."""
    key = (direction, torch.device(dev).index)
    cap = _CAPACITY.get(key)
    if cap is None:
        with torch.cuda.device(dev):
            cap = int(_lib.load().lgnn_fused_grid_capacity(0 if direction == "fwd" else 1))
        if cap < 0:
            _lib.check(cap, "lgnn_fused_grid_capacity")
        _CAPACITY[key] = cap
    return cap


def _open_in_fused(mode, graph: Graph, direction: str) -> bool:
    """Run the open tiles inside the fused launch (behind grid barriers)? Only when every
    workgroup of that launch can be resident at once (a partitioned or smaller device, or CUs
    held by other kernels' reservations, refuse it; the C entry refuses it too)."""
    if not _mode_open_in_fused(mode, graph, direction):
        return False
    M = graph.num_nodes
    ntiles = (M + 63) // 64
    grid = min(ntiles, 512) if direction == "fwd" else \
        _lib.load().lgnn_gcn_stack_bwd_partials(M)
    return grid <= fused_grid_capacity(direction, _graph_device(graph))


def _graph_device(graph):
    """The device of a Graph, or of the graph bundle a compiled op body rebuilds (TGraph: no
    edge_index, its CSR / batch tensors instead)."""
    ei = getattr(graph, "edge_index", None)
    if ei is not None:
        return ei.device
    return (graph.gptr if graph.gptr is not None else graph.batch).device


def _mode_open_in_fused(mode, graph: Graph, direction: str) -> bool:
    if mode in ("1", True):
        return True
    if mode in ("0", False):
        return False
    if mode in ("fwd", "bwd"):
        return mode == direction
    M, B = graph.num_nodes, graph.num_graphs
    if not B or M % B:
        return False
    n = M // B
    return n > 0 and (64 % n == 0 or n % 64 == 0)


def plane_buffers(Ws: list, transposed: bool = False, extra: int = 0):
    """Uninitialised buffers for the bf16 three-plane images of the stack weights (split-3
    kernels): (planes [L+1, 3, 128, 128] int16, planes_t or None). planes_t is flat: the
    transposed planes, then `extra` int16 of room (the forward's Â^T planes, bwd_planes_numel)."""
    nl = len(Ws)
    dev = Ws[0].device
    planes = torch.empty(nl, 3, 128, 128, dtype=torch.int16, device=dev)
    planes_t = torch.empty(nl * 3 * 128 * 128 + extra, dtype=torch.int16, device=dev) \
        if transposed else None
    return planes, planes_t


def plane_job(Ws: list, d_in: int, planes, planes_t) -> _lib.PlaneJob:
    """lgnn_plane_job: the split of Ws into `planes` / `planes_t` (lgnn_weight_planes' arguments),
    run by the graph build's first launch (Graph.csr_planes) or by lgnn_weight_planes."""
    nl = len(Ws)
    if nl > _lib.LGNN_PLANE_JOB_MAX:
        raise _lib.LgnnError("plane job: too many layers")
    job = _lib.PlaneJob()
    job.nl = nl
    widths = [d_in] + [W.size(0) for W in Ws]
    for i, v in enumerate(widths):
        job.widths[i] = v
    for i, W in enumerate(Ws):
        job.W[i] = W.data_ptr()
    job.planes = planes.data_ptr()
    job.planes_t = planes_t.data_ptr() if planes_t is not None else None
    job._keep = (Ws, planes, planes_t)  # the pointers' owners live as long as the job
    return job


def run_plane_job(job: _lib.PlaneJob, dev) -> None:
    """The split of `job` as its own launch (lgnn_weight_planes)."""
    arr = ctypes.c_void_p * job.nl
    _lib.call("lgnn_weight_planes", job.nl, arr(*[job.W[i] for i in range(job.nl)]),
              (ctypes.c_int * (job.nl + 1))(*[job.widths[i] for i in range(job.nl + 1)]),
              job.planes, job.planes_t, _s(dev))


def weight_planes(Ws: list, d_in: int, transposed: bool = False, extra: int = 0):
    """bf16 three-plane images of the stack weights for the split-3 kernels (one launch):
    returns (planes [L+1, 3, 128, 128] int16, planes_t or None); see plane_buffers."""
    planes, planes_t = plane_buffers(Ws, transposed, extra)
    run_plane_job(plane_job(Ws, d_in, planes, planes_t), Ws[0].device)
    return planes, planes_t


# The split-3 weight planes are made afresh by every forward, from the live weights: when the
# forward builds its graph the split runs as extra workgroups of the build's first launch
# (lgnn_graph_build_planes), otherwise as its own launch. Nothing is cached across steps, so a
# captured step replays the split and sees any write to the weights between replays
# (load_state_dict, EMA, clipping), eager or captured alike.
_ADJT_IN_PLANES = [0]  # > 0 inside adjt_in_planes()


class adjt_in_planes:
    """Context: stack forwards put the Â^T room after the transposed planes (one buffer) — the
    compiled lgnn::gcn_stack op returns that buffer as an output of its own."""

    def __enter__(self):
        _ADJT_IN_PLANES[0] += 1

    def __exit__(self, *exc):
        _ADJT_IN_PLANES[0] -= 1


def adjt_numel(M) -> int:
    """int16 elements of the Â^T planes the split-3 forward hands to the fused backward."""
    return (M + 63) // 64 * (_lib.LGNN_S3_ADJT_TILE_BYTES // 2)


def bwd_planes_numel(L: int, M) -> int:
    """Size of the buffer the fused GCN forward keeps for its backward (ctx.planes_t): the
    transposed weight planes, plus the Â^T planes when the single-launch split-3 backward runs."""
    return (L + 1) * 3 * 128 * 128 + (adjt_numel(M) if _s3f(L) and ADJT else 0)


def _s3f(L: int) -> bool:
    """The fused split-3 backward takes L <= 2 convs in one launch, and L = 3 with the in_proj
    weight gradient outside it (the kernel writes dZ_0; stack_bwd runs the GEMM) when its
    open-tile phase runs in the same launch (stack_bwd checks that; otherwise layer-major s3)."""
    return BWD_MODE == "s3f" and L <= 3


# the split-3 forward hands each closed tile's Â^T planes to the fused backward (ADJT = False: the
# backward rebuilds them from the CSR)
ADJT = True


def _adjt_ptr(planes_t: torch.Tensor, L: int):
    """Device address of the Â^T planes inside planes_t, or None."""
    base = (L + 1) * 3 * 128 * 128
    return planes_t.data_ptr() + 2 * base if planes_t.numel() > base else None


def stack_fwd(x: torch.Tensor, graph: Graph, Ws: list, bs: list, keep: dict | None = None,
              kind: str = "gcn"):
    """in_proj + L x ELU(GCNConv) forward, every width <= 128: returns ([H_0..H_L],
    [S_1..S_L]). Tiles no edge leaves run fused through every layer (lgnn_gcn_stack_fwd); the
    rest (graphs straddling 64-node tiles) layer by layer (lgnn_node_linear_fwd_tiles), into the
    same buffers. With graphs aligned to tiles (C2: N = 64) the second group is empty.
    kind: the graph build ("gcn", or "gcn_lazy" when only the fused backward follows)."""
    M = x.size(0)
    L = len(Ws) - 1
    dev = x.device
    s3 = MFMA_MODE == "s3" and L >= 1
    if s3:
        # the transposed planes (the split-3 backward's dH = G W_l operand) come from the same
        # split when the caller keeps them; the split rides the graph build when this forward
        # builds the graph
        want_adjt = keep is not None and _s3f(L) and ADJT
        extra = adjt_numel(M) if want_adjt and _ADJT_IN_PLANES[0] else 0
        planes, planes_t = plane_buffers(Ws, transposed=keep is not None, extra=extra)
        job = plane_job(Ws, x.size(1), planes, planes_t)
        csr, split_done = graph.csr_planes(kind, job)
        if not split_done:
            run_plane_job(job, dev)
        if extra:  # the Â^T tiles in the room after the planes (the compiled op's one output)
            adjt_t, adjt = None, _adjt_ptr(planes_t, L)
        else:
            adjt_t = torch.empty(adjt_numel(M), dtype=torch.int16, device=dev) \
                if want_adjt else None
            adjt = _lib.ptr(adjt_t)
        if keep is not None:
            keep["planes_t"] = planes_t
            keep["adjt"] = adjt_t
    else:
        csr = graph.csr(kind)
    open_ = graph.tile_open(kind)
    hs = [torch.empty(M, W.size(0), dtype=torch.float32, device=dev) for W in Ws]
    ss = [torch.empty(M, Ws[l].size(1), dtype=torch.float32, device=dev) for l in range(1, L + 1)]
    arr = ctypes.c_void_p * (L + 1)
    Wp = arr(*[W.data_ptr() for W in Ws])
    bp = arr(*[b.data_ptr() for b in bs])
    Hp = arr(*[h.data_ptr() for h in hs])
    widths = (ctypes.c_int * (L + 1))(*[W.size(0) for W in Ws])
    if s3:
        if _open_in_fused(OPEN_IN_FUSED, graph, "fwd"):  # open tiles in the same launch
            _lib.call("lgnn_gcn_stack_fwd_s3_all", _lib.ptr(x), M, x.size(1), 1,
                      _lib.ptr(csr.rowptr), _lib.ptr(csr.col), _lib.ptr(csr.w), L,
                      _lib.ptr(planes), Wp, bp, widths, Hp,
                      (ctypes.c_void_p * L)(*[t.data_ptr() for t in ss]), _lib.ptr(open_),
                      adjt, _s(dev))
            return hs, ss
        _lib.call("lgnn_gcn_stack_fwd_s3", _lib.ptr(x), M, x.size(1), 1, _lib.ptr(csr.rowptr),
                  _lib.ptr(csr.col), _lib.ptr(csr.w), L, _lib.ptr(planes), bp, widths, Hp,
                  _lib.ptr(open_), adjt, _s(dev))
    else:
        _lib.call("lgnn_gcn_stack_fwd", _lib.ptr(x), M, x.size(1), 1, _lib.ptr(csr.rowptr),
                  _lib.ptr(csr.col), _lib.ptr(csr.w), L, Wp, bp, widths, Hp, _lib.ptr(open_),
                  _s(dev))
    for l in range(L + 1):
        inp = x if l == 0 else hs[l - 1]
        c = csr if l > 0 else None
        s_out = ss[l - 1] if l > 0 else None
        _lib.call("lgnn_node_linear_fwd_tiles", _lib.ptr(inp), M, inp.size(1),
                  _lib.ptr(c.rowptr) if c else None, _lib.ptr(c.col) if c else None,
                  _lib.ptr(c.w) if c else None, 0.0, _lib.ptr(Ws[l]), _lib.ptr(bs[l]),
                  Ws[l].size(0), _lib.LGNN_ACT_ELU if l > 0 else _lib.LGNN_ACT_NONE,
                  _lib.ptr(hs[l]), _lib.ptr(s_out), _lib.ptr(open_), 1, _s(dev))
    return hs, ss


def head_in_stack_bwd(graph: Graph, L: int, C: int, s3: bool) -> bool:
    """True when stack_bwd's single split-3 launch forms dP = dlogits W_out itself (out_proj
    backward folded into the kernel's pool prologue, <= 8 classes)."""
    return (HEAD_FOLD and s3 and BWD_MODE == "s3f" and L <= 3 and C <= 8 and
            _open_in_fused(OPEN_IN_FUSED_BWD, graph, "bwd"))


def stack_bwd(dp: torch.Tensor | None, x: torch.Tensor, graph: Graph, mean: bool, Ws: list,
              hs: list, ss: list, reducer: list, planes_t: torch.Tensor | None = None,
              head: tuple | None = None, kind: str = "gcn", adjt_t: torch.Tensor | None = None):
    """Backward of stack_fwd from the pooled-output gradient dp down to in_proj, L >= 1 convs,
    no input gradient. Closed tiles run fused (one launch; L = 3 with in_proj's weight gradient
    as a split-3 GEMM after it, the layer-major split-3 kernels past that); open tiles inside the
    same launch behind grid barriers, or layer by layer (lgnn_node_linear_bwd_tiles,
    want_open = 1) into the same partial slots. Returns [(dW_l, db_l)] for l = 0..L; the slab reductions are appended
    to `reducer`. head = (dlogits, W_out) replaces dp where head_in_stack_bwd() allows."""
    csr = graph.csr(kind)
    open_ = graph.tile_open(kind)
    M = x.size(0)
    L = len(Ws) - 1
    dev = x.device
    lib = _lib.load()
    s3 = planes_t is not None
    s3f = s3 and _s3f(L) and (L <= 2 or _open_in_fused(OPEN_IN_FUSED_BWD, graph, "bwd"))
    # the forward's Â^T tiles: their own buffer (adjt_t), or room after the planes (weight_planes'
    # `extra`); none -> the backward rebuilds them from the CSR
    adjt = (_lib.ptr(adjt_t) if adjt_t is not None else _adjt_ptr(planes_t, L)) if s3f else None
    P = lib.lgnn_gcn_stack_bwd_s3_partials(M) if s3 and not s3f else \
        lib.lgnn_gcn_stack_bwd_partials(M)
    _lib.check(0 if P > 0 else P, "lgnn_gcn_stack_bwd_partials")
    widths = [x.size(1)] + [W.size(0) for W in Ws]
    per = [widths[l + 1] * widths[l] + widths[l + 1] for l in range(L + 1)]
    slab = torch.empty(P * sum(per), dtype=torch.float32, device=dev)
    dWp, dbp, off = [], [], 0
    for l in range(L + 1):
        nk, n = widths[l + 1] * widths[l], widths[l + 1]
        dWp.append(slab[off:off + P * nk])
        dbp.append(slab[off + P * nk:off + P * (nk + n)])
        off += P * (nk + n)
    arr = ctypes.c_void_p * (L + 1)
    Sx = [x] + list(ss)
    dlog, W_out = head if head is not None else (None, None)
    ce = dlog if isinstance(dlog, _lib.CeSrc) else None  # CE-formed logits gradient
    B = dp.size(0) if dp is not None else (graph.num_graphs if ce is not None else dlog.size(0))
    if s3f and _open_in_fused(OPEN_IN_FUSED_BWD, graph, "bwd"):  # one launch, open tiles last
        # L = 3: the third [M][128] block receives dZ_0, the in_proj output gradient
        dS_ws = torch.empty((3 if L == 3 else 2) * M * 128, dtype=torch.float32, device=dev)
        common = (_lib.ptr(graph.batch), _lib.ptr(graph.gptr), int(mean), B,
                  _lib.ptr(csr.rowptr), _lib.ptr(csr.col), _lib.ptr(csr.w), _lib.ptr(csr.tptr),
                  _lib.ptr(csr.tidx), _lib.ptr(csr.tw), _lib.ptr(x), M, L, _lib.ptr(planes_t),
                  arr(*[W.data_ptr() for W in Ws]), arr(*[h.data_ptr() for h in hs]),
                  (ctypes.c_void_p * L)(*[t.data_ptr() for t in ss]),
                  (ctypes.c_int * (L + 2))(*widths), arr(*[t.data_ptr() for t in dWp]),
                  arr(*[t.data_ptr() for t in dbp]), P, _lib.ptr(dS_ws), _lib.ptr(open_))
        if ce is not None:
            _lib.call("lgnn_gcn_stack_bwd_s3f_ce", *common, ctypes.byref(ce), _lib.ptr(W_out),
                      W_out.size(0), adjt, _s(dev))
        else:
            _lib.call("lgnn_gcn_stack_bwd_s3f_all", _lib.ptr(dp), *common, _lib.ptr(dlog),
                      _lib.ptr(W_out), W_out.size(0) if head else 0, adjt, _s(dev))
        if L == 3:  # in_proj: (dW_0, db_0) = (dZ_0^T X, colsum dZ_0), one split-3 GEMM
            dz0 = dS_ws[2 * M * 128:2 * M * 128 + M * widths[1]].view(M, widths[1])
            first = dense_wgrad(dz0, x, False, want_db=True, reducer=reducer)
            return [first] + _stack_bwd_outputs(L, widths, dWp, dbp, P, dev, reducer, l0=1)
        return _stack_bwd_outputs(L, widths, dWp, dbp, P, dev, reducer)
    assert head is None, "dP from the logits gradient only in the single-launch split-3 path"
    if s3f:  # one fused split-3 launch, every layer of a tile in one pass (stack3_bwd.hip)
        _lib.call("lgnn_gcn_stack_bwd_s3f", _lib.ptr(dp), _lib.ptr(graph.batch),
                  _lib.ptr(graph.gptr), int(mean), dp.size(0), _lib.ptr(csr.rowptr),
                  _lib.ptr(csr.col), _lib.ptr(csr.w), _lib.ptr(x), M, L, _lib.ptr(planes_t),
                  arr(*[h.data_ptr() for h in hs]), (ctypes.c_int * (L + 2))(*widths),
                  arr(*[t.data_ptr() for t in dWp]), arr(*[t.data_ptr() for t in dbp]), P,
                  _lib.ptr(open_), adjt, _s(dev))
    elif s3:  # one split-3 launch per layer (stack3_bwd.hip); dZ between them in dz_ws
        dz_ws = torch.empty(2 * M * 128, dtype=torch.float32, device=dev)
        _lib.call("lgnn_gcn_stack_bwd_s3", _lib.ptr(dp), _lib.ptr(graph.batch),
                  _lib.ptr(graph.gptr), int(mean), dp.size(0), _lib.ptr(csr.rowptr),
                  _lib.ptr(csr.col), _lib.ptr(csr.w), _lib.ptr(x), M, L, _lib.ptr(planes_t),
                  arr(*[h.data_ptr() for h in hs]), (ctypes.c_int * (L + 2))(*widths),
                  arr(*[t.data_ptr() for t in dWp]), arr(*[t.data_ptr() for t in dbp]), P,
                  _lib.ptr(dz_ws), _lib.ptr(open_), _s(dev))
    else:
        _lib.call("lgnn_gcn_stack_bwd", _lib.ptr(dp), _lib.ptr(graph.batch),
                  _lib.ptr(graph.gptr), int(mean), _lib.ptr(csr.rowptr), _lib.ptr(csr.col),
                  _lib.ptr(csr.w), _lib.ptr(x), M, L, arr(*[W.data_ptr() for W in Ws]),
                  arr(*[h.data_ptr() for h in hs]), (ctypes.c_int * (L + 2))(*widths),
                  arr(*[t.data_ptr() for t in dWp]), arr(*[t.data_ptr() for t in dbp]), P,
                  _lib.ptr(open_), _s(dev))
    dS = None
    for l in reversed(range(L + 1)):
        K, N = widths[l], widths[l + 1]
        if l == L:
            mode, dY, tc = _lib.LGNN_GRAD_POOL, dp, None
        else:
            mode, dY, tc = _lib.LGNN_GRAD_TRANSPOSE, dS, csr
        dX = torch.empty(M, K, dtype=torch.float32, device=dev) if l > 0 else None
        _lib.call("lgnn_node_linear_bwd_tiles", mode, _lib.ptr(dY), _lib.ptr(graph.batch),
                  _lib.ptr(graph.gptr), int(mean), _lib.ptr(tc.tptr) if tc else None,
                  _lib.ptr(tc.tidx) if tc else None, _lib.ptr(tc.tw) if tc else None, 0.0,
                  _lib.ptr(hs[l]) if l > 0 else None,
                  _lib.LGNN_ACT_ELU if l > 0 else _lib.LGNN_ACT_NONE, _lib.ptr(Sx[l]), M, K,
                  None, None, None, 0.0, _lib.ptr(Ws[l]), N, _lib.ptr(dX), _lib.ptr(dWp[l]),
                  _lib.ptr(dbp[l]), P, _lib.ptr(open_), 1, 2 if s3f else 1, _s(dev))
        dS = dX
    return _stack_bwd_outputs(L, widths, dWp, dbp, P, dev, reducer)


def _stack_bwd_outputs(L, widths, dWp, dbp, P, dev, reducer, l0=0):
    out = []
    for l in range(l0, L + 1):
        dW = torch.empty(widths[l + 1], widths[l], dtype=torch.float32, device=dev)
        db = torch.empty(widths[l + 1], dtype=torch.float32, device=dev)
        reducer.extend([(dWp[l], P, dW.numel(), dW), (dbp[l], P, db.numel(), db)])
        out.append((dW, db))
    return out


def num_partials(M: int, N: int, K: int, gather: bool = False) -> int:
    p = _lib.load().lgnn_bwd_num_partials(M, N, K, int(gather))
    _lib.check(0 if p > 0 else p, "lgnn_bwd_num_partials")
    return p


def linear_bwd(grad_mode: int, dY: torch.Tensor, *, H: torch.Tensor | None, act: int,
               X: torch.Tensor, W: torch.Tensor, csr: Csr | None = None, self_scale: float = 0.0,
               graph: Graph | None = None, pool_mean: bool = True, tcsr: Csr | None = None,
               tself: float = 0.0, want_dx: bool = True, want_db: bool = True,
               reducer: list | None = None):
    """Returns (dXpre or None, dW, db or None). dXpre = dZ W (pre-aggregation input grad).
    With `reducer` (a list), the dW/db slab reductions are appended to it for one batched
    launch (reduce_multi) instead of running here."""
    M, K = X.shape
    N = W.size(0)
    dev = X.device
    if wide_shape(K, N):
        # the output gradient as given, from the pooled gradient, or gathered through the
        # transpose CSR; dZ = g * act'(H); then dXpre = dZ W and (dW, db) = (dZ^T S, sum dZ)
        if grad_mode == _lib.LGNN_GRAD_POOL:
            g = pool_bwd(_f32c(dY), graph, pool_mean, M)
        elif grad_mode == _lib.LGNN_GRAD_TRANSPOSE:
            g = spmm_raw(tcsr.tptr, tcsr.tidx, tcsr.tw, tself, dY)
        else:
            g = _f32c(dY)
        if act == _lib.LGNN_ACT_ELU:
            dZ = torch.empty_like(g)
            _lib.call("lgnn_act_bwd", _lib.ptr(g), _lib.ptr(H), _lib.ptr(dZ), g.numel(), act,
                      _s(dev))
        else:
            dZ = g
        S = spmm_raw(csr.rowptr, csr.col, csr.w, self_scale, X) if csr is not None else X
        dX = dense_mm(dZ, dense_planes(W, True, False), K, None, False) if want_dx else None
        dW, db = dense_wgrad(dZ, S, False, want_db=want_db, reducer=reducer)
        return dX, dW, db
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
    db = torch.empty(N, dtype=torch.float32, device=dev) if want_db else None
    jobs = [(dWp, P, N * K, dW)] + ([(dbp, P, N, db)] if want_db else [])
    if reducer is not None:  # caller batches the slab reductions of several layers
        reducer.extend(jobs)
    else:
        reduce_multi(jobs, dev)
    return dX, dW, db


CE_PART = object()  # reduce_multi job part: the CE logits gradient, formed in the reduction


def reduce_multi(jobs: list, dev, ce=None, num_classes: int = 0) -> None:
    """Deterministic slab reductions [(partials, P, len, out), ...] in one launch per 16; a job
    (a, P, len, out, f, width) is the outer-product sum out[c, d] = sum_p a[p, c] f[p, d]. A job
    whose partials are CE_PART takes the [P][C] CE logits gradient formed from `ce`
    (_lib.CeSrc, lgnn_reduce_jobs_ce) instead of a materialised dlogits tensor."""
    for i in range(0, len(jobs), 16):
        chunk = jobs[i:i + 16]
        n = len(chunk)
        is_ce = [j[0] is CE_PART for j in chunk]
        parts = (ctypes.c_void_p * n)(*[None if c else j[0].data_ptr()
                                        for j, c in zip(chunk, is_ce)])
        nps = (ctypes.c_int * n)(*[j[1] for j in chunk])
        lens = (ctypes.c_int64 * n)(*[j[2] for j in chunk])
        outs = (ctypes.c_void_p * n)(*[j[3].data_ptr() for j in chunk])
        fac = (ctypes.c_void_p * n)(*[j[4].data_ptr() if len(j) > 4 else None for j in chunk])
        wid = (ctypes.c_int * n)(*[j[5] if len(j) > 4 else 0 for j in chunk])
        if any(is_ce):
            if ce is None:
                raise _lib.LgnnError("reduce_multi: a CE_PART job needs the CE source")
            _lib.call("lgnn_reduce_jobs_ce", n, parts, fac, wid, nps, lens, outs,
                      (ctypes.c_int * n)(*[int(c) for c in is_ce]), ctypes.byref(ce),
                      int(num_classes), _s(dev))
        elif any(len(j) > 4 for j in chunk):
            _lib.call("lgnn_reduce_jobs", n, parts, fac, wid, nps, lens, outs, _s(dev))
        else:
            _lib.call("lgnn_reduce_partials_multi", n, parts, nps, lens, outs, _s(dev))


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
    if _compiling():
        lib = _lgnn()
        g = lib.gparts(graph, kind) if graph is not None else lib.gparts_empty(x.device)
        return torch.ops.lgnn.node_linear(x, W, b, g, kind if graph is not None else "",
                                          float(self_scale), int(act))
    return _NodeLinear.apply(x, W, b, graph, kind, self_scale, act)


def dense_planes(W: torch.Tensor, transposed: bool, bf16: bool) -> torch.Tensor:
    """The weight operand of dense_mm for W [rows][cols] (lgnn_s3_weight_planes): B = W
    (Y = A W^T) or B = W^T (transposed: Y = A W); three bf16 planes (fp32 accuracy) or, in bf16
    mode, one RNE-rounded plane. One launch; the optimizer updates W in place each step, so the
    planes are written afresh by every forward / backward that uses them."""
    W = _f32c(W)
    rows, cols = W.shape
    out, inn = (cols, rows) if transposed else (rows, cols)
    planes = 1 if bf16 else 3
    n = _lib.load().lgnn_s3_weight_planes_numel(out, inn, planes)
    Wp = torch.empty(n, dtype=torch.int16, device=W.device)
    _lib.call("lgnn_s3_weight_planes", _lib.ptr(W), rows, cols, int(transposed), planes,
              _lib.ptr(Wp), _s(W.device))
    return Wp


def _s3_bundle_sizes(shapes, transposed, bf16: bool) -> list:
    """lgnn_s3_weight_planes_numel per operand, restated in Python (Dynamo traces this; a
    ctypes call would break the graph): ceil(out/128) blocks x planes x 128 x kpad(in, 64)."""
    planes = 1 if bf16 else 3
    out = []
    for (rows, cols), t in zip(shapes, transposed):
        o, i = (cols, rows) if t else (rows, cols)
        out.append((o + 127) // 128 * planes * 128 * ((i + 63) // 64 * 64))
    return out


def s3_bundle_raw(Ws: list, transposed: list, bf16: bool) -> torch.Tensor:
    """The planes of every (W, transposed) operand in one flat int16 buffer (each operand's
    numel a multiple of 8192: every view 16 KiB aligned), LGNN_MAX_WPREP jobs per launch."""
    Ws = [_f32c(W) for W in Ws]
    sizes = _s3_bundle_sizes([tuple(W.shape) for W in Ws], transposed, bf16)
    flat = torch.empty(sum(sizes), dtype=torch.int16, device=Ws[0].device)
    views = flat.split(sizes)
    for j0 in range(0, len(Ws), 16):
        js = range(j0, min(j0 + 16, len(Ws)))
        n = len(js)
        P_ = ctypes.c_void_p * n
        I_ = ctypes.c_int * n
        _lib.call("lgnn_s3_weight_planes_multi", n, P_(*[Ws[j].data_ptr() for j in js]),
                  I_(*[Ws[j].size(0) for j in js]), I_(*[Ws[j].size(1) for j in js]),
                  I_(*[int(bool(transposed[j])) for j in js]), 1 if bf16 else 3,
                  P_(*[views[j].data_ptr() for j in js]), _s(flat.device))
    return flat


def s3_weight_bundle(specs: list, bf16: bool) -> list:
    """Every split-3 weight operand of a step — specs = [(W, transposed)] — in one launch
    (lgnn_s3_weight_planes_multi) instead of one dense_planes launch per GEMM: returns, per spec,
    the planes dense_planes(W, transposed, bf16) would (views of one buffer). The optimizer
    updates the weights in place, so a model asks for its bundle afresh every forward."""
    Ws = [W.detach() for W, _ in specs]
    tr = [bool(t) for _, t in specs]
    if _compiling():
        flat = torch.ops.lgnn.s3_weight_planes_multi(Ws, tr, bool(bf16))
    else:
        flat = s3_bundle_raw(Ws, tr, bf16)
    return list(flat.split(_s3_bundle_sizes([tuple(W.shape) for W in Ws], tr, bf16)))


def _row_blocks(M: int, K: int, N: int, pad_rows: int = 64) -> list:
    """Row ranges [r0, r1) of an M-row GEMM operand that the kernels' 32-bit buffer offsets
    address: (rows + pad_rows) * K * 4 < 2^31 and rows * N * 4 < 2^30 (s3gemm.hip / bflin.hip
    refuse bigger launches with LGNN_EINVAL). Blocks start on 64-row boundaries, so per-tile
    outputs (column-sum rows) of consecutive blocks are contiguous. One block below the limits:
    at the reference's d_in = 1025 a block holds ~520 k nodes."""
    if M <= 0:
        return [(0, max(M, 0))]
    rows = min(((1 << 31) - 1) // (4 * max(K, 1)) - pad_rows, ((1 << 30) - 1) // (4 * max(N, 1)))
    rows = max(64, rows // 64 * 64)
    return [(r, min(r + rows, M)) for r in range(0, M, rows)]


def dense_mm(a: torch.Tensor, Wp: torch.Tensor, N: int, bias, bf16: bool,
             want_colsum: bool = False) -> torch.Tensor:
    """Y = a B^T (+ bias) on the split-3 (fp32 accuracy) or bf16-operand MFMA kernel
    (lgnn_s3_gemm); B's planes from dense_planes. a is fp32 (a bf16 copy is widened: exact).
    Operands past the kernel's 32-bit offsets run as several row-block launches."""
    a = a.float().contiguous() if a.dtype != torch.float32 else a.contiguous()
    M, K = a.shape
    Y = torch.empty(M, N, dtype=torch.float32, device=a.device)
    cs = torch.empty((M + 63) // 64 * N, dtype=torch.float32, device=a.device) \
        if want_colsum and M > 0 else None
    bp = _lib.ptr(_f32c(bias) if bias is not None else None)
    for r0, r1 in _row_blocks(M, K, N):
        _lib.call("lgnn_s3_gemm", _lib.ptr(a) + r0 * K * 4, r1 - r0, K, _lib.ptr(Wp), N,
                  1 if bf16 else 3, bp, _lib.ptr(Y) + r0 * N * 4,
                  _lib.ptr(cs) + (r0 // 64) * N * 4 if cs is not None else None, _s(a.device))
    if cs is not None:
        _COLSUMS[id(Y)] = (weakref.ref(Y), Y._version, cs)
        weakref.finalize(Y, _COLSUMS.pop, id(Y), None)
    return Y


def dense_wgrad(dy: torch.Tensor, x: torch.Tensor, bf16: bool, want_db: bool = False,
                reducer: list | None = None):
    """(dW, db) = (dy^T x, dy.sum(0)) on lgnn_s3_wgrad: partial slabs over row splits (and the
    bias gradient's partial rows from the same pass over dy), summed in fixed order by one
    reduction launch (or appended to `reducer`, the caller's batched reduction)."""
    dy = dy.float().contiguous() if dy.dtype != torch.float32 else dy.contiguous()
    x = x.float().contiguous() if x.dtype != torch.float32 else x.contiguous()
    M, K = x.shape
    N = dy.size(1)
    dev = x.device
    if N % 2:  # the kernel reads dY in column pairs: pad one zero column (exact)
        dy = torch.nn.functional.pad(dy, (0, 1))
    Ne = dy.size(1)
    lib = _lib.load()
    # row blocks past the kernel's 32-bit offsets: each block's partial slabs follow the
    # previous block's, so one fixed-order reduction sums them all
    blocks = _row_blocks(M, max(K, Ne), 0, pad_rows=64)
    Ss = [lib.lgnn_s3_wgrad_partials(r1 - r0, K, Ne) for r0, r1 in blocks]
    S = sum(Ss)
    part = torch.empty(S * Ne * K, dtype=torch.float32, device=dev)
    dbp = torch.empty(S * Ne, dtype=torch.float32, device=dev) if want_db else None
    so = 0
    for (r0, r1), Sb in zip(blocks, Ss):
        _lib.call("lgnn_s3_wgrad", _lib.ptr(dy) + r0 * Ne * 4, Ne, _lib.ptr(x) + r0 * K * 4,
                  r1 - r0, K, 1 if bf16 else 3, _lib.ptr(part) + so * Ne * K * 4, Sb,
                  _lib.ptr(dbp) + so * Ne * 4 if dbp is not None else None, _s(dev))
        so += Sb
    dW = torch.empty(Ne, K, dtype=torch.float32, device=dev)
    db = torch.empty(Ne, dtype=torch.float32, device=dev) if want_db else None
    jobs = [(part, S, Ne * K, dW)] + ([(dbp, S, Ne, db)] if want_db else [])
    if reducer is not None:
        reducer.extend(jobs)
    else:
        reduce_multi(jobs, dev)
    if Ne != N:
        dW, db = dW[:N], (db[:N] if db is not None else None)
    return dW, db


# bf16 GEMMs on the hand-written MFMA kernels (csrc/bflin.hip); BF16_MFMA = False (A/B) and widths
# N > 128 route them to the one-plane split GEMMs above (dense_mm / dense_wgrad with bf16=True)
BF16_MFMA = True


def bf16_mfma_fits(N: int) -> bool:
    return BF16_MFMA and 1 <= N <= 128 and N % 2 == 0


# operands prepared ahead for this forward (bf16_prepare_weights), each taken once
_PREPARED: dict = {}


def bf16_prepare_weights(weights: list) -> None:
    """The bf16 operands (Wb and, when K <= 128, WTb) of several weights in one launch
    (lgnn_bf16_weight_prep_multi). Each is handed out ONCE by bf16_weight_operands for the same
    tensor at the same version, so a later step (the optimizer updates weights in place, without
    a version bump) always prepares afresh."""
    ws = [_f32c(W) for W in weights if bf16_mfma_fits(W.size(0))][:8]
    if not ws:
        return
    lib = _lib.load()
    ops_ = []
    for W in ws:
        N, K = W.shape
        Wb = torch.empty(128 * lib.lgnn_bf16_kpad(K), dtype=torch.bfloat16, device=W.device)
        WTb = torch.empty(128 * lib.lgnn_bf16_kpad(N), dtype=torch.bfloat16, device=W.device) \
            if K <= 128 else None
        ops_.append((W, Wb, WTb))
    n = len(ops_)
    P_ = ctypes.c_void_p * n
    I_ = ctypes.c_int * n
    _lib.call("lgnn_bf16_weight_prep_multi", n, P_(*[o[0].data_ptr() for o in ops_]),
              I_(*[o[0].size(0) for o in ops_]), I_(*[o[0].size(1) for o in ops_]),
              P_(*[o[1].data_ptr() for o in ops_]),
              P_(*[o[2].data_ptr() if o[2] is not None else None for o in ops_]),
              _s(ws[0].device))
    for W, Wb, WTb in ops_:
        _PREPARED[id(W)] = (weakref.ref(W), W._version, Wb, WTb)


def bf16_weight_operands(W: torch.Tensor, want_t: bool):
    """(Wb, WTb): bf16 W [128][kpad(K)] and, when want_t and K <= 128, bf16 W^T [128][kpad(N)]
    (zero-padded operands of lgnn_bf16_gemm), in one launch — or the pair bf16_prepare_weights
    made for W in this forward."""
    W = _f32c(W)
    rec = _PREPARED.pop(id(W), None)
    if rec is not None and rec[0]() is W and rec[1] == W._version \
            and (rec[3] is not None or not want_t or W.size(1) > 128):
        return rec[2], rec[3]
    N, K = W.shape
    lib = _lib.load()
    Wb = torch.empty(128 * lib.lgnn_bf16_kpad(K), dtype=torch.bfloat16, device=W.device)
    WTb = torch.empty(128 * lib.lgnn_bf16_kpad(N), dtype=torch.bfloat16, device=W.device) \
        if want_t and K <= 128 else None
    _lib.call("lgnn_bf16_weight_prep", _lib.ptr(W), N, K, _lib.ptr(Wb), _lib.ptr(WTb),
              _s(W.device))
    return Wb, WTb


def bf16_gemm(A: torch.Tensor, Wb: torch.Tensor, bias, N: int, want_yb: bool = False,
              want_colsum: bool = False):
    """Y = bf16(A) bf16(W)^T (+ bias) in fp32 (and its bf16 copy when want_yb): A fp32 (rounded
    in the kernel) or bf16. want_colsum: Y's per-tile column sums are remembered beside Y
    (colsum_of: a following Linear's bias gradient without a pass over Y)."""
    A = A.contiguous()
    M, K = A.shape
    Y = torch.empty(M, N, dtype=torch.float32, device=A.device)
    Yb = torch.empty(M, N, dtype=torch.bfloat16, device=A.device) if want_yb else None
    cs = torch.empty((M + 63) // 64 * N, dtype=torch.float32, device=A.device) \
        if want_colsum and M > 0 else None
    es = A.element_size()
    bp = _lib.ptr(_f32c(bias) if bias is not None else None)
    for r0, r1 in _row_blocks(M, K, N):  # row blocks past the kernel's 32-bit offsets
        _lib.call("lgnn_bf16_gemm", _lib.ptr(A) + r0 * K * es, int(A.dtype == torch.float32),
                  r1 - r0, K, _lib.ptr(Wb), bp, N, _lib.ptr(Y) + r0 * N * 4,
                  _lib.ptr(Yb) + r0 * N * 2 if Yb is not None else None,
                  _lib.ptr(cs) + (r0 // 64) * N * 4 if cs is not None else None, _s(A.device))
    if cs is not None:
        _COLSUMS[id(Y)] = (weakref.ref(Y), Y._version, cs)
        weakref.finalize(Y, _COLSUMS.pop, id(Y), None)
    return Y, Yb


_COLSUMS: dict = {}


def colsum_of(y: torch.Tensor, reducer: list = None):
    """y.sum(0) from the per-tile column sums its producing GEMM wrote (fixed order), if y is
    that output unchanged; else None. With `reducer` the slab reduction is appended to that job
    list (the caller launches the batch, reduce_multi) instead of launched here."""
    rec = _COLSUMS.get(id(y))
    if rec is None:
        return None
    ref, version, cs = rec
    if ref() is not y or y._version != version:
        return None
    N = y.size(1)
    out = torch.empty(N, dtype=torch.float32, device=y.device)
    if reducer is not None:
        reducer.append((cs, cs.numel() // N, N, out))
    else:
        _lib.call("lgnn_reduce_partials", _lib.ptr(cs), cs.numel() // N, N, _lib.ptr(out),
                  _s(y.device))
    return out


def bf16_wgrad(dYb: torch.Tensor, X: torch.Tensor, N: int, reducer: list = None) -> torch.Tensor:
    """dW = bf16(dY)^T bf16(X): partial slabs over row splits, summed in fixed order (with
    `reducer`: the sum is appended to the caller's job list, launched with its other slabs)."""
    X = X.contiguous()
    M, K = X.shape
    if X.dtype != torch.float32 and K % 2:  # bf16 X needs even rows; bf16 -> fp32 is exact
        X = X.float()
    dev = X.device
    lib = _lib.load()
    es = X.element_size()
    blocks = _row_blocks(M, K, 0, pad_rows=32 * 64)  # past the kernel's 32-bit offsets
    Ss = [lib.lgnn_bf16_wgrad_partials(r1 - r0, K) for r0, r1 in blocks]
    S = sum(Ss)
    part = torch.empty(S * N * K, dtype=torch.float32, device=dev)
    so = 0
    for (r0, r1), Sb in zip(blocks, Ss):
        _lib.call("lgnn_bf16_wgrad", _lib.ptr(dYb) + r0 * N * 2, N, _lib.ptr(X) + r0 * K * es,
                  int(X.dtype == torch.float32), r1 - r0, K, _lib.ptr(part) + so * N * K * 4, Sb,
                  _s(dev))
        so += Sb
    dW = torch.empty(N, K, dtype=torch.float32, device=dev)
    if reducer is not None:
        reducer.append((part, S, N * K, dW))
    else:
        _lib.call("lgnn_reduce_partials", _lib.ptr(part), S, N * K, _lib.ptr(dW), _s(dev))
    return dW


def _bf16_operand(t: torch.Tensor) -> torch.Tensor:
    """The bf16 copy a kernel wrote beside t, else t's own cast."""
    tb = _bf16_copy_of(t)
    return tb if tb is not None else t.to(torch.bfloat16)


class _DenseLinear(torch.autograd.Function):
    """y = x W^T + b for shapes outside the tile kernels (K > 128, K % 4 != 0: the reference's
    in_proj with 1025 input channels, gat.py:29 / lesions.py:142,169) or in bf16 mode, on the
    hand-written MFMA GEMMs: bf16 mode with N <= 128 on bflin.hip, everything else on the
    split-3 kernels of s3gemm.hip (fp32 accuracy; bf16 mode N > 128: one rounded plane). The
    backward is dW = dy^T x, db = colsum dy (from the same pass), dx = dy W in the same
    precision."""

    @staticmethod
    def forward(ctx, x, W, b, bf16, wp=None):
        _lib.require_gpu(x, W)
        x, W = _f32c(x), _f32c(W)
        if bf16 and bf16_mfma_fits(W.size(0)):
            # hand-written bf16 MFMA GEMM: an fp32 x is rounded as the kernel loads it (no copy);
            # the output's bf16 copy feeds the next bf16 GEMM
            xb = _bf16_copy_of(x)
            A = xb if xb is not None else x
            Wb, WTb = bf16_weight_operands(W, True)
            y, yb = bf16_gemm(A, Wb, b, W.size(0), want_yb=BF16_OUT)
            if yb is not None:
                _remember_bf16(y, yb)
            ctx.save_for_backward(A, W)
            ctx.wt = WTb
            ctx.bf16, ctx.has_b = bf16, b is not None
            return y
        # split-3 MFMA GEMM at fp32 accuracy (bf16 mode: RNE-rounded operands, N > 128)
        y = dense_mm(x, wp if wp is not None else dense_planes(W, False, bf16), W.size(0), b,
                     bf16)
        ctx.save_for_backward(x, W)
        ctx.bf16, ctx.has_b = bf16, b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, W = ctx.saved_tensors
        dy = _f32c(dy)
        N, K = W.shape
        mfma = ctx.bf16 and bf16_mfma_fits(N)
        jobs = [] if mfma else None  # db's and dW's slab sums in one launch
        db = None
        if ctx.has_b:  # from the column sums dy's producing GEMM wrote, when it was ours
            db = colsum_of(dy, jobs)
            if db is None and mfma:
                db = dy.sum(0)
        if mfma:
            dyb = _bf16_operand(dy)
            dW = bf16_wgrad(dyb, x, N, jobs)
            reduce_multi(jobs, dW.device)
            dx = None
            if ctx.needs_input_grad[0]:
                if K <= 128:
                    WTb = getattr(ctx, "wt", None)
                    if WTb is None:
                        WTb = bf16_weight_operands(W, True)[1]
                    dx, dxb = bf16_gemm(dyb, WTb, None, K, want_yb=BF16_OUT)
                    if dxb is not None:
                        _remember_bf16(dx, dxb)
                else:
                    dx = dense_mm(dyb, dense_planes(W, True, True), K, None, True)
            return dx, dW, db, None, None
        dW, db2 = dense_wgrad(dy, x, ctx.bf16, want_db=ctx.has_b and db is None)
        if db is None and ctx.has_b:
            db = db2
        dx = dense_mm(dy, dense_planes(W, True, ctx.bf16), K, None, ctx.bf16) \
            if ctx.needs_input_grad[0] else None
        return dx, dW, db, None, None


def dense_linear(x, W, b=None, bf16: bool = False, wp=None):
    """wp: W's split-3 planes from s3_weight_bundle (else made here, one launch)."""
    if _compiling():
        return torch.ops.lgnn.dense_linear(x, W, b, bool(bf16), wp)
    return _DenseLinear.apply(x, W, b, bf16, wp)


def dense_path(W, bf16: bool) -> bool:
    """Whether linear_auto runs W on the split-3 GEMMs (so s3_weight_bundle can prepare it)."""
    return not bf16 and not fast_shape(W.size(1), W.size(0))


def linear_auto(x, W, b=None, bf16: bool = False, wp=None):
    """node_linear (tile kernels) where the shape allows and fp32 is asked for; else the
    hand-written dense GEMMs (dense_linear: split-3 s3gemm.hip, or one bf16 plane in bf16 mode)."""
    if not bf16 and fast_shape(W.size(1), W.size(0)):
        return node_linear(x, W, b)
    return dense_linear(x, W, b, bf16, wp)


class _Spmm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, graph, kind, self_scale):
        _lib.require_gpu(x)
        c = graph.csr(kind)
        # the Csr itself, not its key: a later weighted() call may replace the "weighted" entry
        ctx.c, ctx.self_scale = c, self_scale
        return spmm_raw(c.rowptr, c.col, c.w, self_scale, _f32c(x))

    @staticmethod
    def backward(ctx, dy):
        c = ctx.c
        return spmm_raw(c.tptr, c.tidx, c.tw, ctx.self_scale, _f32c(dy)), None, None, None


def spmm(x, graph: Graph, kind: str = "gin", self_scale: float = 0.0):
    if _compiling():
        return torch.ops.lgnn.spmm(x, _lgnn().gparts(graph, kind), float(self_scale), False)
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
    if _compiling():
        return torch.ops.lgnn.segment_pool(x, _lgnn().gparts(graph, None), bool(mean))
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
    if _compiling():
        return torch.ops.lgnn.pool_head(x, Wout, bout, _lgnn().gparts(graph, None),
                                        bool(mean))[0]
    return _PoolHead.apply(x, Wout, bout, graph, mean)


class _GCNStack(torch.autograd.Function):
    """in_proj -> L x ELU(GCNConv) -> pool -> out_proj as one autograd node (dropout p = 0 or
    eval). params = [W_in, b_in, (W_l, b_l) * L, W_out, b_out]."""

    @staticmethod
    def forward(ctx, x, graph, mean, L, *params):
        logits, to_save = _GCNStack._fwd(ctx, x, graph, mean, L, params)
        ctx.save_for_backward(*to_save)
        return logits

    @staticmethod
    def _fwd(ctx, x, graph, mean, L, params):
        _lib.require_gpu(x, *params)
        x = _f32c(x)
        params = [_f32c(p) for p in params]
        W_in, b_in = params[0], params[1]
        Ws = [params[2 * l] for l in range(L + 1)]
        fused = L + 1 <= STACK_MAX and all(fast_shape(W.size(1), W.size(0)) for W in Ws)
        keep = {} if fused and MFMA_MODE == "s3" and BWD_S3 and L >= 1 else None
        # only the fused kernels read this build (the backward's fused path, the condition
        # backward() tests): its transpose CSR is then built only if some tile is open
        lazy = LAZY_TRANSPOSE and isinstance(graph, Graph) and fused and FUSED_BWD and \
            (1 <= L <= 2 or keep is not None) and not ctx.needs_input_grad[0]
        kind = "gcn_lazy" if lazy else "gcn"
        ctx.kind = kind
        # the fused forward builds the graph itself (with the weight-plane split riding along)
        csr = None if fused else graph.csr(kind)
        ctx.fused = fused
        ctx.planes_t = None
        ctx.adjt = None
        if fused:
            hs, ss = stack_fwd(x, graph, Ws, [params[2 * l + 1] for l in range(L + 1)], keep,
                               kind)
            ctx.planes_t = keep.get("planes_t") if keep else None
            ctx.adjt = keep.get("adjt") if keep else None
            ctx.saved_s = [True] * L
        else:
            hs = [linear_fwd(x, W_in, b_in, _lib.LGNN_ACT_NONE)]
            ss = []  # aggregated conv inputs S_l = A_hat H_{l-1} (saved on the fast path)
            ctx.saved_s = []
            for l in range(L):
                W, b = params[2 + 2 * l], params[3 + 2 * l]
                fast = fast_shape(W.size(1), W.size(0)) or wide_shape(W.size(1), W.size(0))
                if fast:
                    h, s_ = linear_fwd(hs[-1], W, b, _lib.LGNN_ACT_ELU, csr, save_s=True)
                else:
                    h, s_ = linear_fwd(hs[-1], W, b, _lib.LGNN_ACT_ELU, csr), hs[-1]
                hs.append(h)
                ss.append(s_)
                ctx.saved_s.append(fast)
        W_out, b_out = params[2 + 2 * L], params[3 + 2 * L]
        pooled, logits = pool_head_fwd(hs[-1], graph, mean, W_out, b_out)
        ctx.graph, ctx.mean, ctx.L = graph, mean, L
        ctx.n_saved = 2 + len(hs) + len(ss) + len(params)
        return logits, (x, pooled, *hs, *ss, *params)

    @staticmethod
    def backward(ctx, dlogits):
        return _GCNStack._bwd(ctx, dlogits, ctx.saved_tensors)

    @staticmethod
    def fused_head(ctx, W_out) -> bool:
        """True when the backward forms dP = dlogits W_out inside the single split-3 launch."""
        return (ctx.fused and (1 <= ctx.L <= 2 or ctx.planes_t is not None) and
                not ctx.needs_input_grad[0] and FUSED_BWD and
                head_in_stack_bwd(ctx.graph, ctx.L, W_out.size(0), ctx.planes_t is not None))

    @staticmethod
    def _bwd(ctx, dlogits, saved, ce=None):
        """ce = (CeSrc, logits): the logits gradient is CE's, formed where it is consumed (the
        fused backward's prologue, the out_proj reduction jobs) — dlogits is None then."""
        L = ctx.L
        x, pooled = saved[0], saved[1]
        hs = saved[2:3 + L]
        ss = saved[3 + L:3 + 2 * L]
        params = saved[3 + 2 * L:]
        graph = ctx.graph
        kind = getattr(ctx, "kind", "gcn")
        csr = graph.csr(kind)
        W_out = params[2 + 2 * L]
        dlogits = _f32c(dlogits) if dlogits is not None else None
        grads = [None] * len(params)
        red: list = []
        s3 = ctx.planes_t is not None
        if ctx.fused and (1 <= L <= 2 or s3) and not ctx.needs_input_grad[0] and FUSED_BWD:
            Ws = [params[2 * l] for l in range(L + 1)]
            if head_in_stack_bwd(graph, L, W_out.size(0), s3):
                # dP is formed inside the stack kernel; out_proj's gradients (dlogits^T pooled,
                # column sums of dlogits) join the stack's slab reductions: no head launch
                C, D = W_out.shape
                B = pooled.size(0)
                dWo = torch.empty_like(W_out)
                dbo = torch.empty(C, dtype=torch.float32, device=x.device)
                part = CE_PART if ce is not None else dlogits
                red += [(part, B, C * D, dWo, pooled, D), (part, B, C, dbo)]
                outs = stack_bwd(None, x, graph, ctx.mean, Ws, hs, ss, red, ctx.planes_t,
                                 head=(ce[0] if ce is not None else dlogits, W_out), kind=kind,
                                 adjt_t=getattr(ctx, "adjt", None))
            else:
                dp, dWo, dbo = pool_head_bwd(dlogits, pooled, W_out)
                outs = stack_bwd(dp, x, graph, ctx.mean, Ws, hs, ss, red, ctx.planes_t,
                                 kind=kind, adjt_t=getattr(ctx, "adjt", None))
            grads[2 + 2 * L], grads[3 + 2 * L] = dWo, dbo
            for l, (dW, db) in enumerate(outs):
                grads[2 * l], grads[2 * l + 1] = dW, db
            reduce_multi(red, x.device, ce=ce[0] if ce is not None else None,
                         num_classes=W_out.size(0))
            return (None, None, None, None, *grads)
        assert ce is None, "the CE-formed logits gradient only on the fused head path"
        dp, dWo, dbo = pool_head_bwd(dlogits, pooled, W_out)
        grads[2 + 2 * L], grads[3 + 2 * L] = dWo, dbo
        if ctx.fused:  # the fused forward saves no aggregated inputs: S_l = Â H_{l-1}
            ss = [spmm_raw(csr.rowptr, csr.col, csr.w, 0.0, hs[l]) for l in range(L)]
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
                                    pool_mean=ctx.mean, tcsr=tc, reducer=red)
            grads[2 + 2 * l], grads[3 + 2 * l] = dW, db
        # in_proj: dH0 = A^T dS_1 (transposed aggregation in the prologue); dx = dH0 W_in
        want_dx = ctx.needs_input_grad[0]
        if L > 0:
            mode, dY, tc = _lib.LGNN_GRAD_TRANSPOSE, dS, csr
        else:
            mode, dY, tc = _lib.LGNN_GRAD_POOL, dp, None
        dx, dW, db = linear_bwd(mode, dY, H=None, act=_lib.LGNN_ACT_NONE, X=x, W=params[0],
                                graph=graph, pool_mean=ctx.mean, tcsr=tc,
                                want_dx=want_dx, reducer=red)
        reduce_multi(red, x.device)
        grads[0], grads[1] = dW, db
        return (dx, None, None, None, *grads)


class _GCNStackCE(torch.autograd.Function):
    """The GCN model and its criterion nn.CrossEntropyLoss(weight) (mean reduction, reference
    models/base.py:93-94, training_step :196-201) as ONE autograd node: outputs (logits, loss).
    Forward: _GCNStack's launches + lgnn_ce_fwd. Backward with only the loss differentiated (the
    training step): the logits gradient is never materialised — the fused split-3 backward forms
    it per graph in its prologue and the out_proj reduction jobs form it per (graph, class), both
    with lgnn_ce_bwd's expression (no lgnn_ce_bwd launch, bitwise the same gradients). Anything
    else (logits also differentiated, shapes off the fused head path) forms dlogits with
    lgnn_ce_bwd and takes _GCNStack's backward."""

    @staticmethod
    def forward(ctx, x, graph, mean, L, y, weight, *params):
        ctx.set_materialize_grads(False)
        yy = y.to(torch.int64).contiguous()
        w = _f32c(weight) if weight is not None else None
        logits, to_save = _GCNStack._fwd(ctx, x, graph, mean, L, params)
        z = logits
        # one single-workgroup launch: loss, lse and the gradient's factors pm / wt
        B, C = z.shape
        dev = z.device
        lse = torch.empty(B, dtype=torch.float32, device=dev)
        out = torch.empty(2, dtype=torch.float32, device=dev)  # loss, sum of weights
        bad = torch.empty(1, dtype=torch.int32, device=dev)
        pm = torch.empty(B, C, dtype=torch.float32, device=dev)
        wt = torch.empty(B, dtype=torch.float32, device=dev)
        _lib.call("lgnn_ce_fwd_factors", _lib.ptr(z), _lib.ptr(yy), _lib.ptr(w), B, C,
                  _lib.ptr(lse), _lib.ptr(out), _lib.ptr(out) + 4, _lib.ptr(bad),
                  _lib.ptr(pm), _lib.ptr(wt), _s(dev))
        ctx.ce_fwd = None
        ctx.has_w = w is not None
        ctx.has_pm = pm is not None
        ctx.save_for_backward(*to_save, z, yy, lse, out, *((w,) if w is not None else ()),
                              *((pm, wt) if pm is not None else ()))
        return logits, out[0]

    @staticmethod
    def backward(ctx, dlogits, dloss):
        saved = ctx.saved_tensors
        n = ctx.n_saved
        stack_saved = saved[:n]
        z, yy, lse, out = saved[n:n + 4]
        w = saved[n + 4] if ctx.has_w else None
        pm, wt = saved[-2:] if ctx.has_pm else (None, None)
        params = stack_saved[3 + 2 * ctx.L:]
        W_out = params[2 + 2 * ctx.L]

        def grads(r):  # _GCNStack's (dx, -, -, -, *param grads) -> this node's inputs
            return (r[0], None, None, None, None, None, *r[4:])

        if dloss is None:
            if dlogits is None:
                return (None,) * (6 + len(params))
            return grads(_GCNStack._bwd(ctx, dlogits, stack_saved))
        g = _f32c(dloss.reshape(1))
        if dlogits is None and pm is not None and _GCNStack.fused_head(ctx, W_out):
            src = _lib.CeSrc(pm.data_ptr(), wt.data_ptr(), out.data_ptr() + 4, g.data_ptr())
            return grads(_GCNStack._bwd(ctx, None, stack_saved, ce=(src, z)))
        B, C = z.shape
        dz = torch.empty_like(z)
        _lib.call("lgnn_ce_bwd", _lib.ptr(z), _lib.ptr(yy), _lib.ptr(w), B, C, _lib.ptr(lse),
                  _lib.ptr(out) + 4, _lib.ptr(g), _lib.ptr(dz), _s(z.device))
        if dlogits is not None:
            dz = dz + dlogits
        return grads(_GCNStack._bwd(ctx, dz, stack_saved))


def gcn_stack_ce(x, graph: Graph, params: list[torch.Tensor], L: int, y: torch.Tensor,
                 weight: torch.Tensor | None = None, mean: bool = True):
    """(logits, loss): the GCN stack and its cross-entropy criterion in one node (_GCNStackCE)."""
    return _GCNStackCE.apply(x, graph, mean, L, y, weight, *params)


def gcn_stack(x, graph: Graph, params: list[torch.Tensor], L: int, mean: bool = True):
    if _compiling():
        return torch.ops.lgnn.gcn_stack(x, _lgnn().gparts(graph, "gcn"), bool(mean), int(L),
                                        list(params))[0]
    return _GCNStack.apply(x, graph, mean, L, *params)


# ----------------------------------------------------------------------------------------------
# BatchNorm1d + ELU (GIN MLP) and the fused GINConv
# ----------------------------------------------------------------------------------------------


def _bn_ws(M: int, N: int, dev) -> torch.Tensor:
    return torch.empty(_lib.load().lgnn_bn_workspace_bytes(M, N), dtype=torch.uint8, device=dev)


def bn_stats(Z: torch.Tensor) -> torch.Tensor:
    """fp64 [2N]: (sum z, sum z^2) over rows."""
    M, N = Z.shape
    sums = torch.empty(2 * N, dtype=torch.float64, device=Z.device)
    ws = _bn_ws(M, N, Z.device)
    _lib.call("lgnn_bn_stats", _lib.ptr(Z), M, N, _lib.ptr(sums), _lib.ptr(ws), ws.numel(),
              _s(Z.device))
    return sums


def bn_finalize(sums, count: float, bn: torch.nn.BatchNorm1d, training: bool, N: int, dev,
                part: tuple | None = None):
    """The BN constants (+ running-stat update). part = (partial rows, P): sums are first reduced
    from the BN-fused kernels' partial rows into `sums`, in the same launch (training only)."""
    f = dict(dtype=torch.float32, device=dev)
    mean, invstd, scale, shift = (torch.empty(N, **f) for _ in range(4))
    track = bn.track_running_stats and bn.running_mean is not None
    rm = bn.running_mean if track else None
    rv = bn.running_var if track else None
    nbt = bn.num_batches_tracked if (track and training) else None
    momentum = bn.momentum if bn.momentum is not None else 0.1
    if nbt is not None and bn.momentum is None:  # cumulative moving average (torch semantics)
        momentum = 1.0 / float(bn.num_batches_tracked.item() + 1)
    if part is not None:
        _lib.call("lgnn_bn_partials_finalize", _lib.ptr(part[0]), part[1], N, _lib.ptr(sums),
                  float(count), _lib.ptr(bn.weight) if bn.affine else None,
                  _lib.ptr(bn.bias) if bn.affine else None, float(bn.eps), float(momentum),
                  _lib.ptr(rm), _lib.ptr(rv), _lib.ptr(nbt), _lib.ptr(mean), _lib.ptr(invstd),
                  _lib.ptr(scale), _lib.ptr(shift), _s(dev))
        return mean, invstd, scale, shift
    _lib.call("lgnn_bn_finalize", _lib.ptr(sums), float(count),
              _lib.ptr(bn.weight) if bn.affine else None, _lib.ptr(bn.bias) if bn.affine else None,
              float(bn.eps), float(momentum), int(training), N, _lib.ptr(rm), _lib.ptr(rv),
              _lib.ptr(nbt), _lib.ptr(mean), _lib.ptr(invstd), _lib.ptr(scale), _lib.ptr(shift),
              _s(dev))
    return mean, invstd, scale, shift


def bn_act(Z, scale, shift, mask=None) -> torch.Tensor:
    M, N = Z.shape
    A = torch.empty_like(Z)
    _lib.call("lgnn_bn_act", _lib.ptr(Z), M, N, _lib.ptr(scale), _lib.ptr(shift), _lib.ptr(mask),
              _lib.ptr(A), _s(Z.device))
    return A


def bn_bwd_stats(dA, Z, mask, scale, shift, mean, invstd) -> torch.Tensor:
    M, N = Z.shape
    sums = torch.empty(2 * N, dtype=torch.float64, device=Z.device)
    ws = _bn_ws(M, N, Z.device)
    _lib.call("lgnn_bn_bwd_stats", _lib.ptr(dA), _lib.ptr(Z), _lib.ptr(mask), M, N,
              _lib.ptr(scale), _lib.ptr(shift), _lib.ptr(mean), _lib.ptr(invstd), _lib.ptr(sums),
              _lib.ptr(ws), ws.numel(), _s(Z.device))
    return sums


def bn_bwd_apply(dA, Z, mask, scale, shift, mean, invstd, sums, count, training, local_sums,
                 want_param_grads: bool):
    M, N = Z.shape
    dev = Z.device
    dZ = torch.empty_like(Z)
    _lib.call("lgnn_bn_bwd_apply", _lib.ptr(dA), _lib.ptr(Z), _lib.ptr(mask), M, N,
              _lib.ptr(scale), _lib.ptr(shift), _lib.ptr(mean), _lib.ptr(invstd), _lib.ptr(sums),
              float(count), int(training), _lib.ptr(dZ), None, None, _s(dev))
    dg = db = None
    if want_param_grads:
        dg = torch.empty(N, dtype=torch.float32, device=dev)
        db = torch.empty(N, dtype=torch.float32, device=dev)
        _lib.call("lgnn_bn_bwd_apply", None, None, None, 0, N, _lib.ptr(scale), _lib.ptr(shift),
                  _lib.ptr(mean), _lib.ptr(invstd), _lib.ptr(local_sums), 1.0, 0, None,
                  _lib.ptr(dg), _lib.ptr(db), _s(dev))
    return dZ, dg, db


# GIN: BatchNorm folded into the MLP's two linear launches (BN_FUSED = False: the separate
# lgnn_bn_* passes)
BN_FUSED = True



def gin_bn_fused(K: int, N1: int, N2: int) -> bool:
    """True when _GINConv runs its BatchNorm inside the linear kernels (fast-path shapes)."""
    return BN_FUSED and fast_shape(K, N1) and fast_shape(N1, N2)


def _global_count(M: int, group, dev, fixed=None) -> float:
    if group is None:
        return float(M)
    if fixed is not None:
        return float(fixed)
    import torch.distributed as dist

    t = torch.tensor([float(M)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, group=group)
    return float(t.item())


class _GINConv(torch.autograd.Function):
    """One GINConv(MLP([d1,d2,d2], act=ELU, norm=batch_norm)) with the model's F.elu fused:
        S  = (1 + eps) x_i + sum_{j->i} x_j      (eps = 0 buffer; edges as given, KNN loops kept)
        Z1 = S W1^T + b1;  A1 = ELU(BN(Z1)) [* dropout mask];  H = act(A1 W2^T + b2)
    Reference: gin.py:23 (GINConv(MLP(...))), gin.py:31 (F.elu). BN per `bn` (training uses batch
    statistics; SyncBN over `group` when given)."""

    @staticmethod
    def forward(ctx, x, W1, b1, gamma, beta, W2, b2, graph, bn, training, eps, mask, act, group,
                sync_count):
        _lib.require_gpu(x, W1, W2)
        x, W1, b1, W2, b2 = (_f32c(t) for t in (x, W1, b1, W2, b2))
        csr = graph.csr("gin")
        self_scale = 1.0 + float(eps)
        M = x.size(0)
        N1 = W1.size(0)
        fast = fast_shape(W1.size(1), N1)
        if gin_bn_fused(W1.size(1), N1, W2.size(0)):
            H, saved = _GINConv._forward_fused(ctx, x, W1, b1, W2, b2, csr, self_scale, graph, bn,
                                               training, mask, act, group, sync_count, gamma)
            ctx.save_for_backward(*saved)
            return H
        if fast or wide_shape(W1.size(1), N1):
            Z1, S = linear_fwd(x, W1, b1, _lib.LGNN_ACT_NONE, csr, self_scale, save_s=True)
        else:
            Z1, S = linear_fwd(x, W1, b1, _lib.LGNN_ACT_NONE, csr, self_scale), None
        count = float(M)
        sums = None
        if training:
            sums = bn_stats(Z1)
            count = _global_count(M, group, x.device, sync_count)
            if count <= 1:
                raise ValueError("Expected more than 1 value per channel when training")
            if group is not None:
                from .dist import sync_all_reduce

                sync_all_reduce(sums, group)
        mean, invstd, scale, shift = bn_finalize(sums, count, bn, training, N1, x.device)
        A1 = bn_act(Z1, scale, shift, mask)
        H = linear_fwd(A1, W2, b2, act)
        ctx.save_for_backward(x if S is None else S, Z1, A1, H, W1, W2, mean, invstd, scale,
                              shift, mask)
        ctx.graph, ctx.self_scale, ctx.gathered = graph, self_scale, S is None
        ctx.training, ctx.count, ctx.group, ctx.act = training, count, group, act
        ctx.bn_sums = sums  # the batch statistics' sums (library.py: running-stat update op)
        ctx.affine = gamma is not None
        return H

    @staticmethod
    def _forward_fused(ctx, x, W1, b1, W2, b2, csr, self_scale, graph, bn, training, mask, act,
                       group, sync_count, gamma):
        """BatchNorm folded into the two linear launches (lgnn_node_linear_fwd_bn): the BN
        statistics in the first one's epilogue, BN + ELU (+ mask) in the second one's prologue.
        Same arithmetic as the unfused sequence except the fixed order of the fp64 sums."""
        M, N1 = x.size(0), W1.size(0)
        dev = x.device
        P = _lib.load().lgnn_bn_fused_partials(M)
        Z1 = torch.empty(M, N1, dtype=torch.float32, device=dev)
        S = torch.empty_like(x)
        count = float(M)
        sums = None
        fname = "lgnn_node_linear_fwd_bn"
        w1, w2 = W1.data_ptr(), W2.data_ptr()
        if training:
            part = torch.empty(P * 2 * N1, dtype=torch.float64, device=dev)
            _lib.call(fname, _lib.ptr(x), M, x.size(1), _lib.ptr(csr.rowptr),
                      _lib.ptr(csr.col), _lib.ptr(csr.w), float(self_scale), w1,
                      _lib.ptr(b1), N1, _lib.LGNN_ACT_NONE, _lib.ptr(Z1), _lib.ptr(S),
                      _lib.ptr(part), None, None, None, None, _s(dev))
            sums = torch.empty(2 * N1, dtype=torch.float64, device=dev)
            count = _global_count(M, group, dev, sync_count)
            if count <= 1:
                raise ValueError("Expected more than 1 value per channel when training")
            if group is None:  # sums + the BN constants in one launch
                mean, invstd, scale, shift = bn_finalize(sums, count, bn, training, N1, dev,
                                                         part=(part, P))
            else:
                from .dist import sync_all_reduce

                _lib.call("lgnn_bn_partials_reduce", _lib.ptr(part), P, N1, _lib.ptr(sums), None,
                          None, _s(dev))
                sync_all_reduce(sums, group)
                mean, invstd, scale, shift = bn_finalize(sums, count, bn, training, N1, dev)
        else:
            Z1, S = linear_fwd(x, W1, b1, _lib.LGNN_ACT_NONE, csr, self_scale, save_s=True)
            mean, invstd, scale, shift = bn_finalize(sums, count, bn, training, N1, dev)
        A1 = torch.empty_like(Z1)
        N2 = W2.size(0)
        H = torch.empty(M, N2, dtype=torch.float32, device=dev)
        _lib.call(fname, _lib.ptr(Z1), M, N1, None, None, None, 0.0, w2, _lib.ptr(b2), N2, act,
                  _lib.ptr(H), None, None, _lib.ptr(scale), _lib.ptr(shift), _lib.ptr(mask),
                  _lib.ptr(A1), _s(dev))
        ctx.graph, ctx.self_scale, ctx.gathered = graph, self_scale, False
        ctx.training, ctx.count, ctx.group, ctx.act = training, count, group, act
        ctx.bn_sums = sums
        ctx.affine = gamma is not None
        ctx.bn_fused = True
        return H, (S, Z1, A1, H, W1, W2, mean, invstd, scale, shift, mask)

    @staticmethod
    def _backward_fused(ctx, dH, pool: tuple | None = None, gather: tuple | None = None,
                        defer_dx: bool = False, extra_red: list | None = None):
        """pool = (dlogits, W_out, graph, mean): the output gradient comes from the pooled readout
        (global pool + out_proj backward folded into Lin2's backward load; dH is None).
        gather = (dS, tself): the output gradient is the next conv's aggregation backward,
        tself dS + A^T dS, gathered as Lin2's backward loads it (dH is None). defer_dx: return
        this conv's pre-aggregation input gradient (for the previous layer to gather) instead
        of aggregating it here. extra_red: more slab / outer-product jobs for this conv's
        reduction launch."""
        S, Z1, A1, H, W1, W2, mean, invstd, scale, shift, mask = ctx.saved_tensors[:11]
        csr = ctx.graph.csr("gin")
        M, N1 = Z1.shape
        N2 = W2.size(0)
        K = S.size(1)
        dev = Z1.device
        P = _lib.load().lgnn_bn_fused_partials(M)
        red: list = []
        fname = "lgnn_node_linear_bwd_bn"
        w1, w2 = W1.data_ptr(), W2.data_ptr()
        # Lin2 backward; its dX (= dA1) epilogue also sums the BN backward's (g, g xhat)
        dA1 = torch.empty_like(Z1)
        slab2 = torch.empty(P * (N2 * N1 + N2), dtype=torch.float32, device=dev)
        gpart = torch.empty(P * 2 * N1, dtype=torch.float64, device=dev)
        if gather is not None:
            dS, tself = gather
            _lib.call("lgnn_node_linear_bwd_bn_gather", _lib.ptr(dS), _lib.ptr(csr.tptr),
                      _lib.ptr(csr.tidx), _lib.ptr(csr.tw), float(tself), _lib.ptr(H), ctx.act,
                      _lib.ptr(A1), M, N1, w2, N2, _lib.ptr(dA1), _lib.ptr(slab2),
                      _lib.ptr(slab2[P * N2 * N1:]), P, _lib.ptr(Z1), _lib.ptr(mask),
                      _lib.ptr(scale), _lib.ptr(shift), _lib.ptr(mean), _lib.ptr(invstd),
                      _lib.ptr(gpart), _s(dev))
        elif pool is not None:
            dlog, W_out, pg, pmean = pool
            _lib.call("lgnn_node_linear_bwd_bn_pool", _lib.LGNN_BN_GSTATS, None, _lib.ptr(H),
                      ctx.act, _lib.ptr(A1), M, N1, w2, N2, _lib.ptr(dA1), _lib.ptr(slab2),
                      _lib.ptr(slab2[P * N2 * N1:]), P, _lib.ptr(Z1), _lib.ptr(mask),
                      _lib.ptr(scale), _lib.ptr(shift), _lib.ptr(mean), _lib.ptr(invstd),
                      _lib.ptr(gpart), None, 0.0, int(ctx.training), _lib.ptr(pg.batch),
                      _lib.ptr(pg.gptr), int(pmean), _lib.ptr(dlog), _lib.ptr(W_out),
                      W_out.size(0), _s(dev))
        else:
            _lib.call(fname, _lib.LGNN_BN_GSTATS, _lib.ptr(_f32c(dH)), _lib.ptr(H),
                      ctx.act, _lib.ptr(A1), M, N1, w2, N2, _lib.ptr(dA1), _lib.ptr(slab2),
                      _lib.ptr(slab2[P * N2 * N1:]), P, _lib.ptr(Z1), _lib.ptr(mask),
                      _lib.ptr(scale), _lib.ptr(shift), _lib.ptr(mean), _lib.ptr(invstd),
                      _lib.ptr(gpart), None, 0.0, int(ctx.training), _s(dev))
        dW2 = torch.empty(N2, N1, dtype=torch.float32, device=dev)
        db2 = torch.empty(N2, dtype=torch.float32, device=dev)
        red += [(slab2[:P * N2 * N1], P, N2 * N1, dW2), (slab2[P * N2 * N1:], P, N2, db2)]
        local = torch.empty(2 * N1, dtype=torch.float64, device=dev)
        dg = dbt = None
        if ctx.affine:  # the affine gradients come out of the same launch (local sums)
            dg = torch.empty(N1, dtype=torch.float32, device=dev)
            dbt = torch.empty(N1, dtype=torch.float32, device=dev)
        _lib.call("lgnn_bn_partials_reduce", _lib.ptr(gpart), P, N1, _lib.ptr(local),
                  _lib.ptr(dg), _lib.ptr(dbt), _s(dev))
        sums = local
        if ctx.training and ctx.group is not None:
            from .dist import sync_all_reduce

            sums = local.clone()
            sync_all_reduce(sums, ctx.group)
        # Lin1 backward with the BN backward applied to dA1 as it is loaded
        want_dx = ctx.needs_input_grad[0]
        dxpre = torch.empty(M, K, dtype=torch.float32, device=dev) if want_dx else None
        slab1 = torch.empty(P * (N1 * K + N1), dtype=torch.float32, device=dev)
        _lib.call(fname, _lib.LGNN_BN_GIN, _lib.ptr(dA1), None,
                  _lib.LGNN_ACT_NONE, _lib.ptr(S), M, K, w1, N1, _lib.ptr(dxpre),
                  _lib.ptr(slab1), _lib.ptr(slab1[P * N1 * K:]), P, _lib.ptr(Z1), _lib.ptr(mask),
                  _lib.ptr(scale), _lib.ptr(shift), _lib.ptr(mean), _lib.ptr(invstd), None,
                  _lib.ptr(sums), float(ctx.count), int(ctx.training), _s(dev))
        dW1 = torch.empty(N1, K, dtype=torch.float32, device=dev)
        db1 = torch.empty(N1, dtype=torch.float32, device=dev)
        red += [(slab1[:P * N1 * K], P, N1 * K, dW1), (slab1[P * N1 * K:], P, N1, db1)]
        if extra_red:  # e.g. out_proj's dW / db as outer-product jobs (no k_head_bwd launch)
            red += extra_red
        reduce_multi(red, dev)
        dx = None
        if want_dx:
            dx = dxpre if defer_dx else spmm_raw(csr.tptr, csr.tidx, csr.tw, ctx.self_scale,
                                                 dxpre)
        return (dx, dW1, db1, dg, dbt, dW2, db2, None, None, None, None, None, None, None,
                None)

    @staticmethod
    def backward(ctx, dH):
        if getattr(ctx, "bn_fused", False):
            return _GINConv._backward_fused(ctx, dH)
        S, Z1, A1, H, W1, W2, mean, invstd, scale, shift, mask = ctx.saved_tensors
        csr = ctx.graph.csr("gin")
        dA1, dW2, db2 = linear_bwd(_lib.LGNN_GRAD_DIRECT, _f32c(dH), H=H, act=ctx.act, X=A1, W=W2)
        local = bn_bwd_stats(dA1, Z1, mask, scale, shift, mean, invstd)
        sums = local
        if ctx.training and ctx.group is not None:
            from .dist import sync_all_reduce

            sums = local.clone()
            sync_all_reduce(sums, ctx.group)
        dZ1, dg, dbt = bn_bwd_apply(dA1, Z1, mask, scale, shift, mean, invstd, sums, ctx.count,
                                    ctx.training, local, ctx.affine)
        want_dx = ctx.needs_input_grad[0]
        if ctx.gathered:
            dxpre, dW1, db1 = linear_bwd(_lib.LGNN_GRAD_DIRECT, dZ1, H=None,
                                         act=_lib.LGNN_ACT_NONE, X=S, W=W1, csr=csr,
                                         self_scale=ctx.self_scale, want_dx=want_dx)
        else:
            dxpre, dW1, db1 = linear_bwd(_lib.LGNN_GRAD_DIRECT, dZ1, H=None,
                                         act=_lib.LGNN_ACT_NONE, X=S, W=W1, want_dx=want_dx)
        dx = None
        if want_dx:
            dx = spmm_raw(csr.tptr, csr.tidx, csr.tw, ctx.self_scale, dxpre)
        return (dx, dW1, db1, dg, dbt, dW2, db2, None, None, None, None, None, None, None,
                None)


class _GINConvHead(torch.autograd.Function):
    """The GIN model's last conv + global pool + out_proj as one autograd node (BN-fused fp32
    path): its backward forms each row's output gradient from dlogits (out_proj backward + pool
    backward folded into Lin2's backward load, lgnn_node_linear_bwd_bn_pool) instead of
    materialising dH; out_proj's dW / db come from lgnn_pool_head_bwd (same arithmetic as the
    unfused chain)."""

    @staticmethod
    def forward(ctx, x, W1, b1, gamma, beta, W2, b2, W_out, b_out, graph, bn, training, eps,
                mask, act, group, sync_count, mean):
        _lib.require_gpu(x, W1, W2, W_out)
        x, W1, b1, W2, b2 = (_f32c(t) for t in (x, W1, b1, W2, b2))
        W_out, b_out = _f32c(W_out), _f32c(b_out)
        csr = graph.csr("gin")
        H, saved = _GINConv._forward_fused(ctx, x, W1, b1, W2, b2, csr, 1.0 + float(eps), graph,
                                           bn, training, mask, act, group, sync_count, gamma)
        pooled, logits = pool_head_fwd(H, graph, mean, W_out, b_out)
        ctx.save_for_backward(*saved, pooled, W_out)
        ctx.head_graph, ctx.head_mean = graph, mean
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        pooled, W_out = ctx.saved_tensors[11:13]
        dlogits = _f32c(dlogits)
        B, D = pooled.shape
        C = W_out.size(0)
        dev = pooled.device
        dWo = torch.empty(C, D, dtype=torch.float32, device=dev)
        dbo = torch.empty(C, dtype=torch.float32, device=dev)
        _lib.call("lgnn_pool_head_bwd", _lib.ptr(dlogits), _lib.ptr(pooled), B, D,
                  _lib.ptr(W_out), C, None, _lib.ptr(dWo), _lib.ptr(dbo), _s(dev))
        g = _GINConv._backward_fused(ctx, None, pool=(dlogits, W_out, ctx.head_graph,
                                                      ctx.head_mean))
        return (*g[:7], dWo, dbo) + (None,) * 9


# out_proj's dW / db as outer-product jobs of a layer's slab reduction (GIN / GAT model nodes);
# HEAD_JOBS = False: the separate lgnn_pool_head_bwd launch
HEAD_JOBS = True


class _SubCtx:
    """The per-conv state _GINConv._forward_fused / _backward_fused keep on an autograd ctx,
    for one conv inside the _GINStack node."""

    def __init__(self, needs_dx: bool):
        self.needs_input_grad = (needs_dx,)
        self.saved_tensors = ()

    def save_for_backward(self, *t):
        self.saved_tensors = t


class _GINStack(torch.autograd.Function):
    """The whole GIN model (in_proj + every GINConv + global pool + out_proj, reference
    gin.py:17-35) as one autograd node on the BN-fused fp32 kernels. Same kernels as the
    per-conv nodes, except the backward of each conv's aggregation: instead of a transpose-CSR
    pass over its input gradient (spmm), the previous layer's backward gathers that gradient as
    it loads it (lgnn_node_linear_bwd_bn_gather for a conv's Lin2, lgnn_node_linear_bwd in
    LGNN_GRAD_TRANSPOSE mode for in_proj), so no aggregated gradient goes through HBM."""

    @staticmethod
    def forward(ctx, x, graph, mean, specs, W_in, b_in, W_out, b_out, *flat):
        _lib.require_gpu(x, W_in, W_out)
        x, W_in, b_in, W_out, b_out = (_f32c(t) for t in (x, W_in, b_in, W_out, b_out))
        csr = graph.csr("gin")
        h = linear_fwd(x, W_in, b_in, _lib.LGNN_ACT_NONE)
        subs, saved = [], [x, W_in]
        for i, sp in enumerate(specs):
            W1, b1, gamma, beta, W2, b2 = flat[6 * i:6 * i + 6]
            sub = _SubCtx(True)
            h, sv = _GINConv._forward_fused(sub, h, _f32c(W1), _f32c(b1), _f32c(W2), _f32c(b2),
                                            csr, 1.0 + float(sp["eps"]), graph, sp["bn"],
                                            sp["training"], sp["mask"], sp["act"], sp["group"],
                                            sp["sync_count"], gamma)
            sub.n_saved = len(sv)
            saved += list(sv)
            subs.append(sub)
        pooled, logits = pool_head_fwd(h, graph, mean, W_out, b_out)
        ctx.save_for_backward(*saved, pooled, W_out)
        ctx.subs, ctx.graph, ctx.mean = subs, graph, mean
        ctx.in_self = [1.0 + float(sp["eps"]) for sp in specs]
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        saved = ctx.saved_tensors
        x, W_in = saved[0], saved[1]
        pooled, W_out = saved[-2], saved[-1]
        dlogits = _f32c(dlogits)
        B, D = pooled.shape
        C = W_out.size(0)
        dev = pooled.device
        dWo = torch.empty(C, D, dtype=torch.float32, device=dev)
        dbo = torch.empty(C, dtype=torch.float32, device=dev)
        # out_proj's dW = dlogits^T pooled and db = colsum dlogits join the last conv's slab
        # reductions (outer-product jobs): no k_head_bwd launch
        head_jobs = [(dlogits, B, C * D, dWo, pooled, D), (dlogits, B, C, dbo)]
        if not HEAD_JOBS:
            _lib.call("lgnn_pool_head_bwd", _lib.ptr(dlogits), _lib.ptr(pooled), B, D,
                      _lib.ptr(W_out), C, None, _lib.ptr(dWo), _lib.ptr(dbo), _s(dev))
            head_jobs = None
        off = 2
        for sub in ctx.subs:
            sub.saved_tensors = saved[off:off + sub.n_saved]
            off += sub.n_saved
        L = len(ctx.subs)
        grads = [None] * L
        dS = None
        # each layer's dW / db slabs are summed right after that layer, while they are still in
        # the caches (one launch at the end measured 10 us slower per C4 step)
        for i in range(L - 1, -1, -1):
            sub = ctx.subs[i]
            if i == L - 1:
                g = _GINConv._backward_fused(sub, None, pool=(dlogits, W_out, ctx.graph,
                                                               ctx.mean), defer_dx=True,
                                             extra_red=head_jobs)
            else:
                g = _GINConv._backward_fused(sub, None, gather=(dS, ctx.in_self[i + 1]),
                                             defer_dx=True)
            dS = g[0]
            grads[i] = g[1:7]
        # in_proj: its output gradient is the first conv's aggregation backward, gathered
        dx, dW_in, db_in = linear_bwd(_lib.LGNN_GRAD_TRANSPOSE, dS, H=None, act=_lib.LGNN_ACT_NONE,
                                      X=x, W=W_in, tcsr=ctx.graph.csr("gin"),
                                      tself=ctx.in_self[0], want_dx=ctx.needs_input_grad[0])
        flat = [t for g in grads for t in g]
        return (dx, None, None, None, dW_in, db_in, dWo, dbo, *flat)


def gin_stack_eligible(x, W_in, convs_W) -> bool:
    """Whether the GIN model runs as one _GINStack node (eager, BN-fused fp32 kernels, every
    layer on the fast-path shapes)."""
    return (not _compiling() and fast_shape(x.size(1), W_in.size(0)) and
            all(gin_bn_fused(W1.size(1), W1.size(0), W2.size(0)) for W1, W2 in convs_W))


def gin_stack(x, W_in, b_in, convs: list, W_out, b_out, graph: Graph, mean: bool):
    """convs: per GINConv a dict (W1, b1, bn, W2, b2, eps, mask, act, group, sync_count)."""
    specs, flat = [], []
    for c in convs:
        bn = c["bn"]
        training = bn.training or not bn.track_running_stats
        specs.append(dict(bn=bn, training=training, eps=c["eps"], mask=c["mask"], act=c["act"],
                          group=c["group"], sync_count=c["sync_count"]))
        flat += [c["W1"], c["b1"], bn.weight if bn.affine else None,
                 bn.bias if bn.affine else None, c["W2"], c["b2"]]
    return _GINStack.apply(x, graph, mean, specs, W_in, b_in, W_out, b_out, *flat)


def gin_conv_head_eligible(x, W1, W2) -> bool:
    """Whether gin_conv_head runs fused (eager, BN-fused fp32 kernels, fast-path shapes)."""
    return (not _compiling() and
            gin_bn_fused(x.size(1), W1.size(0), W2.size(0)))


def gin_conv_head(x, W1, b1, bn, W2, b2, W_out, b_out, graph: Graph, eps: float = 0.0,
                  mask=None, act: int = _lib.LGNN_ACT_ELU, group=None, sync_count=None,
                  mean: bool = True):
    """gin_conv followed by pool_head (the GIN model's last conv and readout) as one node."""
    training = bn.training or not bn.track_running_stats
    gamma = bn.weight if bn.affine else None
    beta = bn.bias if bn.affine else None
    return _GINConvHead.apply(x, W1, b1, gamma, beta, W2, b2, W_out, b_out, graph, bn, training,
                              eps, mask, act, group, sync_count, mean)


def gin_conv(x, W1, b1, bn, W2, b2, graph: Graph, eps: float = 0.0, mask=None,
             act: int = _lib.LGNN_ACT_ELU, group=None, sync_count=None):
    """bn: the torch.nn.BatchNorm1d holding gamma/beta and the running statistics."""
    training = bn.training or not bn.track_running_stats
    gamma = bn.weight if bn.affine else None
    beta = bn.bias if bn.affine else None
    if _compiling():
        if group is not None:
            raise NotImplementedError("SyncBatchNorm (GIN.set_sync_bn) is not supported under "
                                      "torch.compile")
        track = bn.track_running_stats and bn.running_mean is not None
        out = torch.ops.lgnn.gin_conv(x, W1, b1, gamma, beta, W2, b2,
                                      bn.running_mean if track else None,
                                      bn.running_var if track else None,
                                      _lgnn().gparts(graph, "gin"), bool(training), float(eps),
                                      float(bn.eps), mask, int(act))
        if training and track:
            torch.ops.lgnn.bn_running_update(
                bn.running_mean, bn.running_var, bn.num_batches_tracked, out[8], x.size(0),
                float(bn.eps), -1.0 if bn.momentum is None else float(bn.momentum))
        return out[0]
    return _GINConv.apply(x, W1, b1, gamma, beta, W2, b2, graph, bn, training, eps, mask, act,
                          group, sync_count)


# ----------------------------------------------------------------------------------------------
# GATConv
# ----------------------------------------------------------------------------------------------


class _GATConv(torch.autograd.Function):
    """PyG 2.5.1 GATConv (reference gat.py:31) + the model's F.elu (gat.py:51):
        XP = x W^T (lin, no bias) viewed [M, H, C];  a_s = <XP, att_src>, a_d = <XP, att_dst>
        alpha = softmax_dst(leaky_relu(a_s[j] + a_d[i]));  out_i = sum_j alpha_ij mask_ij XP_j
        Y = act(out.view(M, H*C) + bias)
    over remove_self_loops + add_self_loops of edge_index (graph kind "gat")."""

    @staticmethod
    def forward(ctx, x, W, att_src, att_dst, bias, graph, heads, slope, mask, act, bf16=False,
                wp=None, wpt=None):
        _lib.require_gpu(x, W, att_src, att_dst)
        x, W = _f32c(x), _f32c(W)
        att_src, att_dst = _f32c(att_src).view(-1), _f32c(att_dst).view(-1)
        bias = _f32c(bias) if bias is not None else None
        csr = graph.csr("gat")
        M = x.size(0)
        HC = W.size(0)
        C = HC // heads
        dev = x.device
        # fp32: the lin on the split-3 MFMA GEMMs (s3gemm.hip) at every width — they beat the
        # fp32-MFMA tile kernels (2.7x the MFMA rate at fp32 accuracy); GAT_S3 = False: tiles
        dense = bf16 or not fast_shape(W.size(1), HC) or GAT_S3
        mfma = bf16 and bf16_mfma_fits(HC)
        ctx.wt = None
        if mfma:  # hand-written bf16 MFMA lin; x rounded in the kernel unless a copy exists
            xb = _bf16_copy_of(x)
            xg, Wg = (xb if xb is not None else x), W
            Wb, ctx.wt = bf16_weight_operands(W, True)
        else:  # fp32, or bf16 wider than 128: the operands are split / rounded in the GEMMs
            xg, Wg = x, W
        a_s = torch.empty(M, heads, dtype=torch.float32, device=dev)
        a_d = torch.empty(M, heads, dtype=torch.float32, device=dev)
        scored = False
        if mfma and GAT_GEMM_ATT and 64 < xg.size(1) <= 128:
            # the attention scores come out of the lin GEMM's epilogue (no lgnn_gat_att pass)
            XP = torch.empty(M, HC, dtype=torch.float32, device=dev)
            xg = xg.contiguous()
            _lib.call("lgnn_bf16_gemm_att", _lib.ptr(xg), int(xg.dtype == torch.float32), M,
                      xg.size(1),
                      _lib.ptr(Wb), HC, _lib.ptr(XP), None, _lib.ptr(att_src), _lib.ptr(att_dst),
                      heads, C, _lib.ptr(a_s), _lib.ptr(a_d), _s(dev))
            scored = True
        elif mfma:
            XP = bf16_gemm(xg, Wb, None, HC)[0]
        elif dense and not bf16 and GAT_GEMM_ATT and HC <= 128:
            # split-3 (or one rounded plane) with the attention scores in the GEMM's epilogue
            XP = torch.empty(M, HC, dtype=torch.float32, device=dev)
            xg = xg.contiguous()
            _lib.call("lgnn_s3_gemm_att", _lib.ptr(xg), M, xg.size(1),
                      _lib.ptr(wp if wp is not None else dense_planes(Wg, False, False)), HC, 3,
                      _lib.ptr(XP), _lib.ptr(att_src), _lib.ptr(att_dst), heads,
                      C, _lib.ptr(a_s), _lib.ptr(a_d), _s(dev))
            scored = True
        elif dense:  # split-3 MFMA GEMM (fp32 accuracy), or one rounded plane in bf16 mode
            XP = dense_mm(xg, wp if wp is not None else dense_planes(Wg, False, bf16), HC, None,
                          bf16)
        else:
            XP = linear_fwd(x, W, None, _lib.LGNN_ACT_NONE)
        if not scored:
            _lib.call("lgnn_gat_att", _lib.ptr(XP), M, heads, C, _lib.ptr(att_src),
                      _lib.ptr(att_dst), _lib.ptr(a_s), _lib.ptr(a_d), _s(dev))
        cap = csr.col.numel()
        alpha = torch.empty(cap, heads, dtype=torch.float32, device=dev)
        Y = torch.empty(M, HC, dtype=torch.float32, device=dev)
        # bf16 mode: the kernel also writes Y in bf16 for the next layer's GEMM (no cast pass)
        Yb = torch.empty(M, HC, dtype=torch.bfloat16, device=dev) if bf16 and BF16_OUT else None
        _lib.call("lgnn_gat_fwd", _lib.ptr(csr.rowptr), _lib.ptr(csr.col), _lib.ptr(XP),
                  _lib.ptr(a_s), _lib.ptr(a_d), M, heads, C, float(slope), _lib.ptr(mask),
                  _lib.ptr(bias), act, _lib.ptr(alpha), _lib.ptr(Y), _lib.ptr(Yb), _s(dev))
        ctx.save_for_backward(xg, Wg, att_src, att_dst, XP, a_s, a_d, alpha, Y, mask)
        ctx.graph, ctx.heads, ctx.slope, ctx.act = graph, heads, slope, act
        ctx.bf16, ctx.dense = bf16, dense
        ctx.wpt = wpt if dense and not mfma else None  # W^T's planes for dx (s3_weight_bundle)
        ctx.has_bias = bias is not None
        ctx.att_shape = (1, heads, C)
        if Yb is not None:
            _remember_bf16(Y, Yb)
        return Y

    @staticmethod
    def backward(ctx, dY, pool: tuple | None = None, extra_red: list | None = None):
        """pool = (dlogits, W_out, graph, mean): the output gradient is formed from the readout's
        gradient inside the edge kernel (lgnn_gat_bwd_edge_pool; dY is None). extra_red: more
        slab / outer-product jobs for this layer's reduction launch."""
        x, W, att_src, att_dst, XP, a_s, a_d, alpha, Y, mask = ctx.saved_tensors[:10]
        csr = ctx.graph.csr("gat")
        M, HC = Y.shape
        H = ctx.heads
        C = HC // H
        dev = Y.device
        dZ = torch.empty_like(Y)
        da_e = torch.empty_like(alpha)
        da_d = torch.empty(M, H, dtype=torch.float32, device=dev)
        if pool is not None:
            dlog, W_out, pg, pmean = pool
            _lib.call("lgnn_gat_bwd_edge_pool", _lib.ptr(csr.rowptr), _lib.ptr(csr.col),
                      _lib.ptr(XP), _lib.ptr(a_s), _lib.ptr(a_d), _lib.ptr(alpha), _lib.ptr(mask),
                      _lib.ptr(Y), ctx.act, M, H, C, float(ctx.slope), _lib.ptr(pg.batch),
                      _lib.ptr(pg.gptr), int(pmean), _lib.ptr(dlog), _lib.ptr(W_out),
                      W_out.size(0), _lib.ptr(dZ), _lib.ptr(da_e), _lib.ptr(da_d), _s(dev))
        else:
            _lib.call("lgnn_gat_bwd_edge", _lib.ptr(csr.rowptr), _lib.ptr(csr.col),
                      _lib.ptr(XP), _lib.ptr(a_s), _lib.ptr(a_d), _lib.ptr(alpha),
                      _lib.ptr(mask), _lib.ptr(_f32c(dY)), _lib.ptr(Y), ctx.act, M, H, C,
                      float(ctx.slope), _lib.ptr(dZ), _lib.ptr(da_e), _lib.ptr(da_d), _s(dev))
        P = _lib.load().lgnn_gat_bwd_num_partials(M)
        part = torch.empty(P * 3 * HC, dtype=torch.float32, device=dev)
        dXP = torch.empty_like(XP)
        # bf16 MFMA lin: the kernel also writes dXP in bf16 (the GEMMs' operand, no cast pass)
        dXPb = torch.empty(M, HC, dtype=torch.bfloat16, device=dev) \
            if ctx.bf16 and bf16_mfma_fits(HC) and BF16_OUT else None
        _lib.call("lgnn_gat_bwd_node", _lib.ptr(csr.tptr), _lib.ptr(csr.tidx),
                  _lib.ptr(csr.tmap), _lib.ptr(alpha), _lib.ptr(mask), _lib.ptr(da_e),
                  _lib.ptr(da_d), _lib.ptr(dZ), _lib.ptr(XP), _lib.ptr(att_src),
                  _lib.ptr(att_dst), M, H, C, _lib.ptr(dXP), _lib.ptr(part), P, _lib.ptr(dXPb),
                  _s(dev))
        red = torch.empty(3 * HC, dtype=torch.float32, device=dev)
        want_dx = ctx.needs_input_grad[0]
        if ctx.bf16 and bf16_mfma_fits(HC):
            dg = dXPb if dXPb is not None else dXP.to(torch.bfloat16)
            # the attention partials and lin's dW slabs summed in one launch
            jobs = [(part, P, 3 * HC, red)] + (extra_red or [])
            dW = bf16_wgrad(dg, x, HC, jobs)
            reduce_multi(jobs, dev)
            dx = None
            if want_dx:
                K = W.size(1)
                if K <= 128:
                    WTb = getattr(ctx, "wt", None)
                    if WTb is None:
                        WTb = bf16_weight_operands(W, True)[1]
                    # dx's column sums ride along: the in_proj backward's bias gradient
                    dx, dxb = bf16_gemm(dg, WTb, None, K, want_yb=BF16_OUT, want_colsum=True)
                    if dxb is not None:
                        _remember_bf16(dx, dxb)
                else:
                    dx = dense_mm(dg, dense_planes(W, True, True), K, None, True)
        else:
            jobs = [(part, P, 3 * HC, red)] + (extra_red or [])
            if ctx.dense:  # split-3 (or bf16-rounded) MFMA GEMMs on the fp32 dXP
                # lin's dW slabs join the attention partials' reduction: one launch per conv
                dW = dense_wgrad(dXP, x, ctx.bf16, reducer=jobs)[0]
                reduce_multi(jobs, dev)
                wpt = getattr(ctx, "wpt", None)
                dx = dense_mm(dXP, wpt if wpt is not None else dense_planes(W, True, ctx.bf16),
                              W.size(1), None, ctx.bf16) if want_dx else None
            else:
                if extra_red:
                    reduce_multi(jobs, dev)
                else:
                    _lib.call("lgnn_reduce_partials", _lib.ptr(part), P, 3 * HC, _lib.ptr(red),
                              _s(dev))
                dx, dW, _ = linear_bwd(_lib.LGNN_GRAD_DIRECT, dXP, H=None,
                                       act=_lib.LGNN_ACT_NONE, X=x, W=W, want_dx=want_dx,
                                       want_db=False)
        ctx.red = red  # the compiled path returns the one buffer (lgnn::gat_conv_bwd)
        datt_s = red[:HC].view(ctx.att_shape)
        datt_d = red[HC:2 * HC].view(ctx.att_shape)
        dbias = red[2 * HC:] if ctx.has_bias else None
        return dx, dW, datt_s, datt_d, dbias, None, None, None, None, None, None, None, None


GAT_S3 = True
# bf16 GAT: the attention kernels write their fp32 outputs' bf16 copies for the following bf16
# GEMMs (BF16_OUT = False: torch casts instead; the values are identical, RNE both ways)
BF16_OUT = True
# bf16 GATConv.lin forward with the attention scores in its epilogue (lgnn_bf16_gemm_att)
GAT_GEMM_ATT = True
_BF16_COPIES: dict = {}


def _remember_bf16(y: torch.Tensor, yb: torch.Tensor) -> None:
    key = id(y)
    _BF16_COPIES[key] = (weakref.ref(y), y._version, yb)
    weakref.finalize(y, _BF16_COPIES.pop, key, None)


def _bf16_copy_of(x: torch.Tensor):
    """The bf16 copy a GAT layer wrote beside its output x, if x is that output unchanged."""
    rec = _BF16_COPIES.get(id(x))
    if rec is None:
        return None
    ref, version, xb = rec
    if ref() is not x or x._version != version:
        return None
    return xb


class _GATConvHead(torch.autograd.Function):
    """The GAT model's last GATConv + global pool + out_proj as one autograd node: its backward
    forms the conv's output gradient from dlogits inside the edge kernel (out_proj backward +
    pool backward folded into the load, lgnn_gat_bwd_edge_pool) instead of writing dH
    (k_pool_bwd); out_proj's dW / db are outer-product jobs of the layer's slab reduction.
    Bitwise the separate nodes except out_proj's dW / db (another fixed summation order)."""

    @staticmethod
    def forward(ctx, x, W, att_src, att_dst, bias, W_out, b_out, graph, heads, slope, mask, act,
                bf16, mean, wp=None, wpt=None):
        sub = _SubCtx(True)
        Y = _GATConv.forward(sub, x, W, att_src, att_dst, bias, graph, heads, slope, mask, act,
                             bf16, wp, wpt)
        W_out, b_out = _f32c(W_out), _f32c(b_out)
        pooled, logits = pool_head_fwd(Y, graph, mean, W_out, b_out)
        ctx.save_for_backward(*sub.saved_tensors, pooled, W_out)
        sub.saved_tensors = ()
        ctx.sub, ctx.head_graph, ctx.head_mean = sub, graph, mean
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        saved = ctx.saved_tensors
        pooled, W_out = saved[10], saved[11]
        dlogits = _f32c(dlogits)
        B, D = pooled.shape
        C = W_out.size(0)
        dev = pooled.device
        dWo = torch.empty(C, D, dtype=torch.float32, device=dev)
        dbo = torch.empty(C, dtype=torch.float32, device=dev)
        sub = ctx.sub
        sub.saved_tensors = saved[:10]
        sub.needs_input_grad = (ctx.needs_input_grad[0],)
        # out_proj's dW / db as outer-product jobs of the layer's reduction (no k_head_bwd)
        head_jobs = [(dlogits, B, C * D, dWo, pooled, D), (dlogits, B, C, dbo)]
        if not HEAD_JOBS:
            _lib.call("lgnn_pool_head_bwd", _lib.ptr(dlogits), _lib.ptr(pooled), B, D,
                      _lib.ptr(W_out), C, None, _lib.ptr(dWo), _lib.ptr(dbo), _s(dev))
            head_jobs = None
        g = _GATConv.backward(sub, None, pool=(dlogits, W_out, ctx.head_graph, ctx.head_mean),
                              extra_red=head_jobs)
        sub.saved_tensors = ()
        return (*g[:5], dWo, dbo) + (None,) * 9


def gat_conv_head(x, W, att_src, att_dst, bias, W_out, b_out, graph: Graph, heads: int,
                  slope: float = 0.2, mask=None, act: int = _lib.LGNN_ACT_NONE,
                  bf16: bool = False, mean: bool = True, planes=None):
    """gat_conv followed by pool_head (the GAT model's last conv and readout) as one node."""
    wp, wpt = planes if planes is not None else (None, None)
    if _compiling():
        return torch.ops.lgnn.gat_conv_head(
            x, W, att_src, att_dst, bias, W_out, b_out, _lgnn().gparts(graph, "gat"), int(heads),
            float(slope), mask, int(act), bool(bf16), bool(mean), wp, wpt)[0]
    return _GATConvHead.apply(x, W, att_src, att_dst, bias, W_out, b_out, graph, heads, slope,
                              mask, act, bf16, mean, wp, wpt)


def gat_conv(x, W, att_src, att_dst, bias, graph: Graph, heads: int, slope: float = 0.2,
             mask=None, act: int = _lib.LGNN_ACT_NONE, bf16: bool = False, planes=None):
    """bf16: the lin GEMM (and its backward) on bf16-rounded operands, fp32 accumulate/out;
    attention, softmax and aggregation stay fp32. planes = (W's, W^T's) split-3 planes from
    s3_weight_bundle (fp32 / dense path), else each GEMM prepares its own."""
    wp, wpt = planes if planes is not None else (None, None)
    if _compiling():
        return torch.ops.lgnn.gat_conv(x, W, att_src, att_dst, bias, _lgnn().gparts(graph, "gat"),
                                       int(heads), float(slope), mask, int(act), bool(bf16), wp,
                                       wpt)[0]
    return _GATConv.apply(x, W, att_src, att_dst, bias, graph, heads, slope, mask, act, bf16, wp,
                          wpt)


# ----------------------------------------------------------------------------------------------
# criterion
# ----------------------------------------------------------------------------------------------


class _Regression(torch.autograd.Function):
    """The regression head and criterion: pred = clamp(z.squeeze(1), lo, hi) (reference
    gat.py:94-95 / gin.py:66-67) and loss = nn.MSELoss / nn.SmoothL1Loss (models/base.py:95-96)
    of (pred, y.float()), in one HIP launch forward (lgnn_regression_fwd) and one backward,
    instead of torch's clamp / compare / mse / mean / where kernels. Returns (pred, loss)."""

    @staticmethod
    def forward(ctx, z, y, lo, hi, smooth):
        _lib.require_gpu(z, y)
        ctx.needs_reshape = z.dim() == 2
        z = _f32c(z).reshape(-1)
        B = z.numel()
        if y.numel() != B:
            raise ValueError("regression target must have one value per graph")
        yi64 = y.dtype == torch.int64
        yc = y.contiguous() if yi64 else y.to(torch.float32).contiguous()
        pred = torch.empty(B, dtype=torch.float32, device=z.device)
        loss = torch.empty((), dtype=torch.float32, device=z.device)
        _lib.call("lgnn_regression_fwd", _lib.ptr(z), _lib.ptr(yc), int(yi64), B, float(lo),
                  float(hi), int(smooth), _lib.ptr(pred), _lib.ptr(loss), _s(z.device))
        ctx.save_for_backward(z, yc)
        ctx.cfg = (int(yi64), B, float(lo), float(hi), int(smooth))
        ctx.set_materialize_grads(False)
        return pred, loss

    @staticmethod
    def backward(ctx, gpred, gloss):
        z, yc = ctx.saved_tensors
        yi64, B, lo, hi, smooth = ctx.cfg
        dz = torch.empty_like(z)
        if gpred is None and gloss is None:
            return None, None, None, None, None
        _lib.call("lgnn_regression_bwd", _lib.ptr(z), _lib.ptr(yc), yi64, B, lo, hi, smooth,
                  _lib.ptr(_f32c(gloss) if gloss is not None else None),
                  _lib.ptr(_f32c(gpred).reshape(-1) if gpred is not None else None),
                  _lib.ptr(dz), _s(z.device))
        return dz.view(-1, 1) if ctx.needs_reshape else dz, None, None, None, None


def regression_loss(logits: torch.Tensor, y: torch.Tensor, lo: float, hi: float,
                    kind: str = "MSE"):
    """(pred, loss): pred = clamp(logits.squeeze(1), lo, hi); loss = MSE or SmoothL1 (beta 1,
    mean) of (pred, y.float()). lo = -inf, hi = inf: the bare criterion."""
    if kind not in ("MSE", "SmoothL1"):
        raise ValueError(kind)
    if logits.dim() == 2 and logits.size(1) != 1:
        raise ValueError("regression logits must be [B] or [B, 1]")
    return _Regression.apply(logits, y, lo, hi, kind == "SmoothL1")


class _CrossEntropy(torch.autograd.Function):
    """nn.CrossEntropyLoss(weight) with mean reduction (reference models/base.py:93-94) in two
    HIP kernels (lgnn_ce_fwd / lgnn_ce_bwd) instead of log_softmax + nll_loss + their backward."""

    @staticmethod
    def forward(ctx, logits, target, weight, validate):
        _lib.require_gpu(logits, target)
        z = _f32c(logits)
        y = target.to(torch.int64).contiguous()
        B, C = z.shape
        dev = z.device
        lse = torch.empty(B, dtype=torch.float32, device=dev)
        out = torch.empty(2, dtype=torch.float32, device=dev)  # loss, sum of weights
        bad = torch.empty(1, dtype=torch.int32, device=dev)
        w = _f32c(weight) if weight is not None else None
        _lib.call("lgnn_ce_fwd", _lib.ptr(z), _lib.ptr(y), _lib.ptr(w), B, C, _lib.ptr(lse),
                  _lib.ptr(out), _lib.ptr(out) + 4, _lib.ptr(bad), _s(dev))
        if validate and int(bad.item()):
            raise ValueError("cross_entropy: a target is outside [0, num_classes)")
        ctx.save_for_backward(z, y, w, lse, out)
        return out[0]

    @staticmethod
    def backward(ctx, g):
        z, y, w, lse, out = ctx.saved_tensors
        B, C = z.shape
        dz = torch.empty_like(z)
        g = _f32c(g.reshape(1))
        _lib.call("lgnn_ce_bwd", _lib.ptr(z), _lib.ptr(y), _lib.ptr(w), B, C, _lib.ptr(lse),
                  _lib.ptr(out) + 4, _lib.ptr(g), _lib.ptr(dz), _s(z.device))
        return dz, None, None, None


def cross_entropy(logits, target, weight=None, validate: bool = False):
    """Weighted-mean cross-entropy of [B, C] logits vs int64 targets. validate=True checks the
    targets (one host read); otherwise out-of-range targets are skipped silently."""
    return _CrossEntropy.apply(logits, target, weight, validate)


# ----------------------------------------------------------------------------------------------
# SortAggregation (DRGNet) and per-component feature pooling
# ----------------------------------------------------------------------------------------------


class _SortPool(torch.autograd.Function):
    """PyG 2.5.1 SortAggregation(k) (reference drgnet.py:37,59) on lgnn_sort_pool_fwd/_bwd."""

    @staticmethod
    def forward(ctx, x, graph, k):
        _lib.require_gpu(x)
        x = _f32c(x)
        M, D = x.shape
        B = graph.num_graphs
        dev = x.device
        out = torch.empty(B, k * D, dtype=torch.float32, device=dev)
        rank = torch.empty(M, dtype=torch.int32, device=dev)
        fill = torch.empty(1, dtype=torch.float32, device=dev)
        nws = _lib.load().lgnn_sort_pool_workspace_bytes()
        ws = torch.empty(nws, dtype=torch.uint8, device=dev)
        _lib.call("lgnn_sort_pool_fwd", _lib.ptr(x), M, D, _lib.ptr(graph.gptr), B, int(k),
                  _lib.ptr(out), _lib.ptr(rank), _lib.ptr(fill), _lib.ptr(ws), nws, _s(dev))
        ctx.save_for_backward(x, rank, fill)
        ctx.graph, ctx.k = graph, int(k)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, rank, fill = ctx.saved_tensors
        M, D = x.shape
        dx = torch.empty_like(x)
        _lib.call("lgnn_sort_pool_bwd", _lib.ptr(_f32c(dout)), _lib.ptr(x), _lib.ptr(rank),
                  _lib.ptr(ctx.graph.batch), _lib.ptr(fill), M, D, ctx.k, _lib.ptr(dx),
                  _s(x.device))
        return dx, None, None


def sort_pool(x, graph: Graph, k: int):
    """x [ΣN, D] -> [B, k * D]; graph carries batch / Batch.ptr."""
    if graph.batch is None:
        raise ValueError("sort_pool needs the graph's batch vector")
    if _compiling():
        return torch.ops.lgnn.sort_pool(x, _lgnn().gparts(graph, None), int(k))[0]
    return _SortPool.apply(x, graph, k)


def cc_pool(features: torch.Tensor, cc: torch.Tensor, num_segments: int, reduce_max: bool,
            validate: bool = True) -> torch.Tensor:
    """features (C, P) fp32 channel-major, cc (P,) int64 -> (num_segments, C): per-label mean or
    max (lgnn_cc_pool). validate: raise if a label falls outside [0, num_segments) (one host
    read)."""
    _lib.require_gpu(features, cc)
    f = _f32c(features)
    C, P = f.shape
    lab = cc.reshape(-1).to(torch.int64).contiguous()
    if lab.numel() != P:
        raise ValueError("cc must hold one label per pixel")
    dev = f.device
    out = torch.empty(num_segments, C, dtype=torch.float32, device=dev)
    err = torch.empty(1, dtype=torch.int32, device=dev)
    nws = _lib.load().lgnn_cc_pool_workspace_bytes(P, C, num_segments)
    ws = torch.empty(nws, dtype=torch.uint8, device=dev)
    _lib.call("lgnn_cc_pool", _lib.ptr(f), C, P, _lib.ptr(lab), int(num_segments),
              int(reduce_max), _lib.ptr(out), None, _lib.ptr(err), _lib.ptr(ws), nws, _s(dev))
    if validate and int(err.item()):
        raise IndexError(f"cc_pool: {int(err.item())} labels outside [0, {num_segments})")
    return out
