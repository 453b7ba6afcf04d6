"""GPU k-NN and radius graph construction for batches of lesion graphs (liblgnn
`lgnn_knn_graph`, `lgnn_radius_count` / `lgnn_radius_graph`).

Mirrors `torch_cluster.knn_graph(x, k, batch, loop, flow='source_to_target')` and PyG 2.5.1's
`KNNGraph(k, loop, force_undirected=False, flow='source_to_target')` transform, which the
reference applies to every lesion graph while loading (configs/config.py:47
`KNNGraph(k=6, loop=True)`, datasets/datamodule.py:43-48; sweep.py:105-120 draws k in [2, 32]).
Here a whole collated batch is built in one launch on the GPU instead of graph by graph on the
host: for every node, its k nearest nodes of the same graph (itself included when `loop`),
ordered by (fp64 squared distance, node index), as edges (neighbour, node) grouped by node —
bit-exact against the CPU restatement `synth.knn_edges`.

Not reproduced: `force_undirected=True` and `cosine=True` (neither is used by the reference's
configs); they raise.

`radius_graph` / `RadiusGraph` mirror `torch_cluster.radius_graph` and PyG's `RadiusGraph(r,
loop=False, max_num_neighbors=32)`, the reference sweep's other connectivity
(scripts/sweep.py:113-118): every node's in-range nodes of its graph (fp64 squared distance
< r^2) in index order, at most max_num_neighbors (+ 1 before the self pair is dropped when not
`loop`) — torch_cluster's CUDA selection rule (include/lgnn.h).
"""
from __future__ import annotations

import torch

from . import _lib


def knn_graph(pos: torch.Tensor, k: int, batch: torch.Tensor | None = None, loop: bool = False,
              flow: str = "source_to_target", cosine: bool = False,
              num_graphs: int | None = None) -> torch.Tensor:
    """edge_index [2, E] int64 of the k-NN graph of `pos` [N, 2 or 3] (per graph of the sorted
    `batch` vector). Defaults as torch_cluster.knn_graph (loop=False)."""
    if flow not in ("source_to_target", "target_to_source"):
        raise ValueError(f"flow must be 'source_to_target' or 'target_to_source', got {flow!r}")
    if cosine:
        raise NotImplementedError("cosine distance is not supported (unused by the reference)")
    _lib.require_gpu(pos)
    if pos.dim() != 2 or pos.size(1) not in (2, 3):
        raise ValueError("pos must be [N, 2] or [N, 3]")
    if not 1 <= k <= 32:
        raise ValueError("k must be in [1, 32]")
    dev = pos.device
    pos = pos.to(torch.float64).contiguous()
    N = pos.size(0)
    if batch is None:
        batch = torch.zeros(N, dtype=torch.int64, device=dev)
        num_graphs = 1 if N > 0 else 0
    batch = batch.to(device=dev, dtype=torch.int64).contiguous()
    if num_graphs is None:
        num_graphs = int(batch.max().item()) + 1 if N > 0 else 0
    B = int(num_graphs)
    ptr = torch.empty(B + 1, dtype=torch.int32, device=dev)
    _lib.call("lgnn_batch_ptr", _lib.ptr(batch), N, B, _lib.ptr(ptr), _lib.stream(dev))
    n = (ptr[1:] - ptr[:-1]).to(torch.int64)
    kk = torch.clamp(n, max=k) if loop else torch.clamp(torch.clamp(n, max=k + 1) - 1, min=0)
    E = int((n * kk).sum().item()) if B > 0 else 0  # one host sync: sizes the output
    out = torch.empty(2, E, dtype=torch.int64, device=dev)
    ws = torch.empty(max(1, _lib.load().lgnn_knn_workspace_bytes(B)), dtype=torch.uint8,
                     device=dev)
    _lib.call("lgnn_knn_graph", _lib.ptr(pos), N, pos.size(1), _lib.ptr(batch), _lib.ptr(ptr), B,
              int(k), int(bool(loop)), _lib.ptr(out), E, _lib.ptr(ws), ws.numel(),
              _lib.stream(dev))
    if flow == "target_to_source":
        out = out.flip(0)
    return out


def _batch_ptr(pos, batch, num_graphs):
    dev = pos.device
    N = pos.size(0)
    if batch is None:
        batch = torch.zeros(N, dtype=torch.int64, device=dev)
        num_graphs = 1 if N > 0 else 0
    batch = batch.to(device=dev, dtype=torch.int64).contiguous()
    if num_graphs is None:
        num_graphs = int(batch.max().item()) + 1 if N > 0 else 0
    B = int(num_graphs)
    ptr = torch.empty(B + 1, dtype=torch.int32, device=dev)
    _lib.call("lgnn_batch_ptr", _lib.ptr(batch), N, B, _lib.ptr(ptr), _lib.stream(dev))
    return batch, ptr, B


def radius_graph(pos: torch.Tensor, r: float, batch: torch.Tensor | None = None,
                 loop: bool = False, max_num_neighbors: int = 32,
                 flow: str = "source_to_target", num_workers: int = 1,
                 num_graphs: int | None = None) -> torch.Tensor:
    """edge_index [2, E] int64 of the radius graph of `pos` [N, 2 or 3] (per graph of the sorted
    `batch` vector), torch_cluster.radius_graph's arguments and defaults (num_workers is a CPU
    knob there; ignored). Two launches, one host read of the edge count, one launch."""
    if flow not in ("source_to_target", "target_to_source"):
        raise ValueError(f"flow must be 'source_to_target' or 'target_to_source', got {flow!r}")
    _lib.require_gpu(pos)
    if pos.dim() != 2 or pos.size(1) not in (2, 3):
        raise ValueError("pos must be [N, 2] or [N, 3]")
    if int(max_num_neighbors) < 1:
        raise ValueError("max_num_neighbors must be >= 1")
    if not float(r) >= 0.0:
        raise ValueError("r must be >= 0")
    dev = pos.device
    pos = pos.to(torch.float64).contiguous()
    N = pos.size(0)
    batch, ptr, B = _batch_ptr(pos, batch, num_graphs)
    lib = _lib.load()
    ws = torch.empty(max(1, lib.lgnn_radius_workspace_bytes(N)), dtype=torch.uint8, device=dev)
    args = (_lib.ptr(pos), N, pos.size(1), _lib.ptr(batch), _lib.ptr(ptr), B, float(r),
            int(max_num_neighbors), int(bool(loop)))
    _lib.call("lgnn_radius_count", *args, _lib.ptr(ws), ws.numel(), _lib.stream(dev))
    E = int(ws[8 * N:8 * N + 8].view(torch.int64).item())  # one host sync: sizes the output
    out = torch.empty(2, E, dtype=torch.int64, device=dev)
    _lib.call("lgnn_radius_graph", *args, _lib.ptr(out), E, _lib.ptr(ws), ws.numel(),
              _lib.stream(dev))
    if flow == "target_to_source":
        out = out.flip(0)
    return out


class RadiusGraph:
    """PyG `torch_geometric.transforms.RadiusGraph` on the GPU, for a single graph or a collated
    batch (`data.batch` present): sets `data.edge_index` and drops `edge_attr`, as PyG does."""

    def __init__(self, r: float, loop: bool = False, max_num_neighbors: int = 32,
                 flow: str = "source_to_target", num_workers: int = 1):
        self.r, self.loop, self.max_num_neighbors = r, loop, max_num_neighbors
        self.flow, self.num_workers = flow, num_workers

    def __call__(self, data):
        data.edge_attr = None
        batch = getattr(data, "batch", None)
        num_graphs = getattr(data, "num_graphs", None)
        data.edge_index = radius_graph(data.pos, self.r, batch, self.loop,
                                       max_num_neighbors=self.max_num_neighbors, flow=self.flow,
                                       num_graphs=num_graphs)
        return data

    def __repr__(self) -> str:
        return f"{self.__class__.__name__}(r={self.r})"


class KNNGraph:
    """PyG `torch_geometric.transforms.KNNGraph` on the GPU, for a single graph or a collated
    batch (`data.batch` present): sets `data.edge_index` (and drops `edge_attr`, as PyG does)."""

    def __init__(self, k: int = 6, loop: bool = False, force_undirected: bool = False,
                 flow: str = "source_to_target", cosine: bool = False):
        if force_undirected:
            raise NotImplementedError("force_undirected=True is not supported (unused by the "
                                      "reference configs)")
        self.k, self.loop, self.flow, self.cosine = k, loop, flow, cosine

    def __call__(self, data):
        batch = getattr(data, "batch", None)
        num_graphs = getattr(data, "num_graphs", None)
        data.edge_index = knn_graph(data.pos, self.k, batch, loop=self.loop, flow=self.flow,
                                    cosine=self.cosine, num_graphs=num_graphs)
        if hasattr(data, "edge_attr"):
            data.edge_attr = None
        return data

    def __repr__(self) -> str:
        return f"{self.__class__.__name__}(k={self.k})"
