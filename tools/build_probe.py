"""Graph-build timing probe: builds the CSR of one bench workload's batch `reps` times (eager,
no model), so rocprofv3 can time the build kernels alone. Usage (GPU box):
  rocprofv3 --kernel-trace --stats -d <dir> -- python3 tools/build_probe.py <workload> <kind> [reps]
kind: gcn_lazy | gcn | gin | gat; [sorted] 0 turns the target-sorted path off (LGNN_OPT_GRAPH_SORTED)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from lesion_gnn_amd.graph import Graph  # noqa: E402


def main():
    wl, kind = sys.argv[1], sys.argv[2]
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    if len(sys.argv) > 4:
        from lesion_gnn_amd import _lib
        _lib.load().lgnn_set_option(_lib.LGNN_OPT_GRAPH_SORTED, int(sys.argv[4]))
    dev = torch.device("cuda", 0)
    b = bench.make_batch(bench.WORKLOADS[wl], 1024, seed=100).to(dev)
    for _ in range(reps):
        g = Graph(b.edge_index, b.num_nodes, b.batch, b.num_graphs)
        g.csr(kind)
    torch.cuda.synchronize(dev)
    print(wl, kind, "nodes", b.num_nodes, "edges", b.num_edges)


if __name__ == "__main__":
    main()
