"""Batched-graph structure on the GPU: CSR by target + CSR by source, Batch.ptr.

Replaces the per-forward edge_index preprocessing PyG does inside each conv (gcn_norm for
GCNConv, remove/add_self_loops for GATConv) and torch_sparse's adj_t CSR
(reference src/lesion_gnn/datasets/datamodule.py:44-45). A `Graph` is built once per forward and
shared by every conv of the model; it is also accepted in place of `edge_index` (the analogue of
the reference's SparseTensor `adj_t` input, gin.py:59-62).
"""
from __future__ import annotations

from dataclasses import dataclass

import ctypes

import torch

from . import _lib

KEEP_BUILD_WS = False

KIND = {
    # kind: (loops mode, norm mode, self_scale of the aggregation)
    "gcn": (_lib.LGNN_LOOPS_REMAINING, _lib.LGNN_NORM_GCN),
    # the "gcn" build for the fused GCN stack alone: its source (transpose) CSR is built only
    # when some tile is open (lgnn_graph_build_lazy) — the closed tiles' backward never reads it
    "gcn_lazy": (_lib.LGNN_LOOPS_REMAINING, _lib.LGNN_NORM_GCN),
    "gin": (_lib.LGNN_LOOPS_KEEP, _lib.LGNN_NORM_NONE),
    "gat": (_lib.LGNN_LOOPS_READD, _lib.LGNN_NORM_NONE),
}


@dataclass
class Csr:
    rowptr: torch.Tensor  # int32 [N+1]
    col: torch.Tensor     # int32 [cap] source of each entry, grouped by target
    w: torch.Tensor       # fp32 [cap]
    tptr: torch.Tensor    # int32 [N+1]
    tidx: torch.Tensor    # int32 [cap] target of each entry, grouped by source
    tw: torch.Tensor      # fp32 [cap]
    tmap: torch.Tensor | None  # int32 [cap] target-CSR position of each transpose entry (GAT)
    tile_open: torch.Tensor | None  # int32 [ceil(N/64) + LGNN_TILE_OPEN_EXTRA] tiles an edge leaves, their count,
    # and the fused stack kernels' grid-barrier words (LGNN_TILE_OPEN_EXTRA)
    err: torch.Tensor     # int32 [1] count of dropped out-of-range edges


class Graph:
    """edge_index [2, E] int64 (source, target) + sorted `batch` [N] -> device CSR views."""

    def __init__(self, edge_index: torch.Tensor, num_nodes: int, batch: torch.Tensor | None = None,
                 num_graphs: int | None = None):
        _lib.require_gpu(edge_index)
        if edge_index.dim() != 2 or edge_index.size(0) != 2:
            raise ValueError("edge_index must be [2, E]")
        self.edge_index = edge_index.to(torch.int64).contiguous()
        self.num_nodes = int(num_nodes)
        self.device = edge_index.device
        self._csr: dict[str, Csr] = {}
        self._aux: dict[str, torch.Tensor] = {}
        self.adj_values: torch.Tensor | None = None  # values of an adj_t input (as_graph)
        # keep the last eager build's workspace for build_path() (tests / diagnostics only: it
        # holds several (E + N)-sized arrays for the Graph's lifetime); KEEP_BUILD_WS = True sets it
        self.keep_build_workspace = KEEP_BUILD_WS
        self.batch = None
        self._gptr = None
        self.num_graphs = None
        if batch is not None:
            self.set_batch(batch, num_graphs)

    @property
    def num_edges(self) -> int:
        return self.edge_index.size(1)

    def set_batch(self, batch: torch.Tensor, num_graphs: int | None = None) -> None:
        _lib.require_gpu(batch)
        if batch.numel() != self.num_nodes:
            raise ValueError("batch must have one entry per node")
        self.batch = batch.to(torch.int64).contiguous()
        if num_graphs is None:
            # PyG: int(batch.max()) + 1 (a device->host read; pass num_graphs to avoid it)
            num_graphs = int(self.batch[-1].item()) + 1 if self.num_nodes > 0 else 0
        self.num_graphs = int(num_graphs)
        self._gptr = None  # computed by the first CSR build, or on first use

    @property
    def gptr(self) -> torch.Tensor | None:
        """int32 [num_graphs + 1] graph offsets (Batch.ptr)."""
        if self._gptr is None and self.batch is not None and torch.compiler.is_compiling():
            self._gptr = torch.ops.lgnn.batch_ptr(self.batch, self.num_graphs)
        if self._gptr is None and self.batch is not None:
            self._gptr = torch.empty(self.num_graphs + 1, dtype=torch.int32, device=self.device)
            _lib.call("lgnn_batch_ptr", _lib.ptr(self.batch), self.num_nodes, self.num_graphs,
                      _lib.ptr(self._gptr), _lib.stream(self.device))
        return self._gptr

    def csr(self, kind: str) -> Csr:
        return self.csr_planes(kind)[0]

    def csr_planes(self, kind: str, planes: "_lib.PlaneJob | None" = None) -> tuple[Csr, bool]:
        """csr(kind), with the split-3 weight planes of `planes` written by the build's first
        launch when this call builds the CSR (lgnn_graph_build_planes). Returns (csr, True) when
        the planes were written, (csr, False) when the CSR was already built (or is traced):
        the caller then makes them itself (lgnn_weight_planes)."""
        if kind in self._csr:
            return self._csr[kind], False
        if torch.compiler.is_compiling():  # traced: the graph build is one opaque lgnn op
            if self._gptr is None and self.batch is not None:  # Batch.ptr rides along
                rp, col, w, tp, ti, tw, tmap, topen, err, self._gptr = \
                    torch.ops.lgnn.graph_build_b(self.edge_index, self.num_nodes, kind,
                                                 self.batch, self.num_graphs)
            else:
                rp, col, w, tp, ti, tw, tmap, topen, err = torch.ops.lgnn.graph_build(
                    self.edge_index, self.num_nodes, kind)
            c = Csr(rowptr=rp, col=col, w=w, tptr=tp, tidx=ti, tw=tw,
                    tmap=tmap if kind == "gat" else None,
                    tile_open=topen if kind == "gcn" else None, err=err)
            self._csr[kind] = c
            return c, False
        loops, norm = KIND[kind]
        n, e = self.num_nodes, self.num_edges
        cap = e + n
        dev = self.device
        i32 = dict(dtype=torch.int32, device=dev)
        c = Csr(
            rowptr=torch.empty(n + 1, **i32), col=torch.empty(cap, **i32),
            w=torch.empty(cap, dtype=torch.float32, device=dev),
            tptr=torch.empty(n + 1, **i32), tidx=torch.empty(cap, **i32),
            tw=torch.empty(cap, dtype=torch.float32, device=dev),
            tmap=torch.empty(cap, **i32) if kind == "gat" else None,
            tile_open=torch.empty((n + 63) // 64 + _lib.LGNN_TILE_OPEN_EXTRA, **i32)
            if kind in ("gcn", "gcn_lazy") else None,
            err=torch.empty(1, **i32),
        )
        lib = _lib.load()
        ws_bytes = lib.lgnn_graph_workspace_bytes(n, e)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        gptr = None  # the graph offsets ride along with the first build
        if self._gptr is None and self.batch is not None:
            gptr = self._gptr = torch.empty(self.num_graphs + 1, dtype=torch.int32, device=dev)
        args = (_lib.ptr(self.edge_index), e, n, loops, norm,
                _lib.ptr(c.rowptr), _lib.ptr(c.col), _lib.ptr(c.w), _lib.ptr(c.tptr),
                _lib.ptr(c.tidx), _lib.ptr(c.tw), _lib.ptr(c.tmap), _lib.ptr(c.tile_open),
                _lib.ptr(self.batch) if gptr is not None else None,
                self.num_graphs if gptr is not None else 0, _lib.ptr(gptr), _lib.ptr(c.err),
                _lib.ptr(ws), ws_bytes)
        if planes is not None:
            _lib.call("lgnn_graph_build_planes", *args, int(kind == "gcn_lazy"),
                      ctypes.byref(planes), _lib.stream(dev))
        else:
            _lib.call("lgnn_graph_build_lazy" if kind == "gcn_lazy" else "lgnn_graph_build",
                      *args, _lib.stream(dev))
        self._csr[kind] = c
        if self.keep_build_workspace:
            self._last_ws = (kind, ws)
        return c, planes is not None

    def build_path(self, kind: str) -> str:
        """Which launches the last eager build of `kind` took: "sorted" (the target-sorted fast
        path: k-NN input grouped by target), "sorted_open" (target-sorted, but an edge leaves its
        64-row tile: the sorted path writes the target CSR, the counting sort only the source
        CSR) or "general" (the counting sort for both). Synchronises.
        Needs keep_build_workspace set before the build."""
        k, ws = getattr(self, "_last_ws", (None, None))
        if k != kind:
            raise ValueError(f"no eager build of {kind!r} on this graph kept its workspace "
                             "(set Graph.keep_build_workspace = True, or KEEP_BUILD_WS = True)")
        r = _lib.load().lgnn_graph_build_path(_lib.ptr(ws), self.num_nodes, self.num_edges,
                                              _lib.stream(self.device))
        _lib.check(r if r < 0 else 0, "lgnn_graph_build_path")
        return {1: "sorted", 2: "sorted_open"}.get(r, "general")

    def weighted(self, edge_weight: torch.Tensor) -> str:
        """Register the CSR pair carrying per-edge weights `edge_weight` [E] (edge order, e.g.
        GaussianDistance output) for GraphConv (reference models/drgnet.py:55); returns its kind
        key for csr(). The structure is the "gin" build (edges as given, no loops, rows in
        edge-id order), so the weights are gathered by the stable (target | source, edge id)
        order on the device. Edges the build drops (an index outside [0, N)) sort after every
        valid one, so they never shift a valid edge's weight. One weighted entry per Graph,
        reused only for the same tensor object at the same version."""
        _lib.require_gpu(edge_weight)
        if edge_weight.dim() != 1 or edge_weight.numel() != self.num_edges:
            raise ValueError("edge_weight must be [E]")
        key = "weighted"
        if torch.compiler.is_compiling():
            base = self.csr("gin")
            cw, ctw = torch.ops.lgnn.weighted_csr(self.edge_index, edge_weight, self.num_nodes,
                                                  base.w)
            self._csr[key] = Csr(rowptr=base.rowptr, col=base.col, w=cw, tptr=base.tptr,
                                 tidx=base.tidx, tw=ctw, tmap=None, tile_open=None, err=base.err)
            return key
        src = self._aux.get("w_src")
        if key in self._csr and src is not None and src[0] is edge_weight \
                and src[1] == edge_weight._version:
            return key
        base = self.csr("gin")
        w = edge_weight.detach().to(torch.float32)
        if "perm" not in self._aux:
            n = self.num_nodes
            ei = self.edge_index
            bad = ((ei < 0) | (ei >= n)).any(0)
            self._aux["perm"] = torch.argsort(ei[1].masked_fill(bad, n), stable=True)
            self._aux["tperm"] = torch.argsort(ei[0].masked_fill(bad, n), stable=True)
        cw, ctw = torch.zeros_like(base.w), torch.zeros_like(base.tw)
        cw[: self.num_edges] = w[self._aux["perm"]]
        ctw[: self.num_edges] = w[self._aux["tperm"]]
        self._csr[key] = Csr(rowptr=base.rowptr, col=base.col, w=cw, tptr=base.tptr,
                             tidx=base.tidx, tw=ctw, tmap=None, tile_open=None, err=base.err)
        self._aux["w_src"] = (edge_weight, edge_weight._version)  # holds the tensor: id stays
        return key

    def tile_open(self, kind: str) -> torch.Tensor:
        """int32 [ceil(N/64) + LGNN_TILE_OPEN_EXTRA]: 1 for the 64-node tiles an edge leaves or that exceed the
        on-chip CSR capacity, then the number of such tiles (from the graph build for kind
        "gcn"; lgnn_tile_open otherwise)."""
        c = self.csr(kind)
        if c.tile_open is not None:
            return c.tile_open
        key = "open:" + kind
        if key not in self._aux:
            n_t = _lib.load().lgnn_tile_count(self.num_nodes)
            t = torch.empty(n_t + _lib.LGNN_TILE_OPEN_EXTRA, dtype=torch.int32,
                            device=self.device)
            _lib.call("lgnn_tile_open", _lib.ptr(c.rowptr), _lib.ptr(c.col), self.num_nodes,
                      _lib.ptr(t), _lib.stream(self.device))
            self._aux[key] = t
        return self._aux[key]

    def barrier_timeouts(self, kind: str = "gcn") -> int:
        """Grid barriers of the fused stack kernels' open-tile phase that gave up waiting since
        this graph's build (forward + backward words of tile_open; synchronises). Non-zero means
        a launch whose workgroups were not all resident: its results are wrong."""
        c = self._csr.get(kind)
        if c is None or c.tile_open is None:
            return 0
        n = (self.num_nodes + 63) // 64
        t = c.tile_open
        return int(t[n + 3].item()) + int(t[n + 6].item())

    def dropped_edges(self, kind: str) -> int:
        """Number of edges with an out-of-range index (synchronises)."""
        return int(self.csr(kind).err.item())


def adj_t_to_edge_index(adj_t, with_values: bool = False):
    """The reference's `adj_t` input (ToSparseTensor, datasets/datamodule.py:44-45; selected at
    gin.py:59-62 / gat.py:87-90): a transposed adjacency whose row is the TARGET and column the
    SOURCE. Accepts a torch_sparse.SparseTensor (duck-typed: `.storage.row()/.col()/.value()`) or
    a torch sparse COO/CSR tensor. Returns edge_index [2, E] = (source, target) in row-major
    order; with `with_values`, also the stored values [E] (ToSparseTensor moves `edge_weight`
    there; PyG GraphConv's spmm(adj_t, x) aggregates with them) or None."""
    vals = None
    if hasattr(adj_t, "storage") and hasattr(adj_t.storage, "row"):
        row, col = adj_t.storage.row(), adj_t.storage.col()
        if hasattr(adj_t.storage, "value"):
            vals = adj_t.storage.value()
    elif isinstance(adj_t, torch.Tensor) and adj_t.layout == torch.sparse_csr:
        crow = adj_t.crow_indices()
        col = adj_t.col_indices()
        row = torch.repeat_interleave(torch.arange(crow.numel() - 1, device=crow.device),
                                      crow[1:] - crow[:-1])
        vals = adj_t.values()
    elif isinstance(adj_t, torch.Tensor) and adj_t.layout == torch.sparse_coo:
        adj_t = adj_t.coalesce()
        idx = adj_t.indices()
        row, col = idx[0], idx[1]
        vals = adj_t.values()
    else:
        raise TypeError(f"unsupported adjacency input {type(adj_t)}")
    ei = torch.stack([col.to(torch.int64), row.to(torch.int64)])
    return (ei, vals) if with_values else ei


def as_graph(edge_index, num_nodes: int, batch=None, num_graphs=None) -> Graph:
    """edge_index [2, E] | Graph | adj_t -> Graph. An adj_t's stored values ride along as
    `Graph.adj_values` (the edge weights of a weighted conv given no explicit edge_weight)."""
    vals = None
    if not isinstance(edge_index, (Graph, torch.Tensor)) or (
            isinstance(edge_index, torch.Tensor) and edge_index.layout != torch.strided):
        edge_index, vals = adj_t_to_edge_index(edge_index, with_values=True)
    if isinstance(edge_index, Graph):
        g = edge_index
        if batch is not None and g.batch is None:
            g.set_batch(batch, num_graphs)
        return g
    g = Graph(edge_index, num_nodes, batch, num_graphs)
    g.adj_values = vals
    return g
