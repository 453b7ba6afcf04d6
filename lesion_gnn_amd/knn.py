"""GPU k-NN graph construction for batches of lesion graphs (liblgnn `lgnn_knn_graph`).

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
