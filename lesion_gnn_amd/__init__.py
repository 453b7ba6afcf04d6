"""lesion_gnn_amd — MI355X-native (gfx950 HIP) lesion-graph message-passing path.

Drop-in for the reference's `self.model(data.x, edge_index, data.batch)` (zacharielegault/
lesion-gnn src/lesion_gnn/models/gin.py:64, gat.py:92): same constructor signatures, configs and
state_dict keys; forward/backward run on the hand-written kernels of liblgnn.so (C ABI:
include/lgnn.h). GPU only — there is no CPU fallback.
"""
from . import _lib
from . import library  # noqa: F401  (registers the lgnn:: custom ops for torch.compile)
from .conv import GCNConv, GraphConv, global_add_pool, global_mean_pool
from .graph import Graph
from .knn import KNNGraph, knn_graph
from .transforms import GaussianDistance, SaveAs, gaussian_distance
from .models import GCN, GCNConfig, get_model

__all__ = ["GCN", "GCNConfig", "GCNConv", "GaussianDistance", "Graph", "GraphConv", "KNNGraph",
           "SaveAs", "gaussian_distance", "get_model", "global_mean_pool", "global_add_pool",
           "knn_graph", "load_library"]


def load_library():
    return _lib.load()
