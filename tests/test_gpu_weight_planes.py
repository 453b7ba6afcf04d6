"""GPU: the split-3 weight planes of the fused GCN stack are made from the live weights by every
forward (the split rides the graph build's first launch, lgnn_graph_build_planes, or runs as its
own launch when the graph is already built), so a captured training step sees weights written
between replays (the round-4 plane cache did not: its validity check ran once, at capture).

* capture the bench's C2-shaped step (forward_loss + backward + lesion_gnn_amd.optim.Adam) in a
  HIP graph, replay it, load new weights in place (load_state_dict: outside the graph), replay
  again: the replay's logits and loss are the oracle's on the loaded weights (fp32 bars);
* the eager step's launch trace has no lgnn_weight_planes launch when the forward builds its
  graph, and one when it is handed a prebuilt Graph; both give bitwise the same logits.
"""
import pytest
import torch

import oracle.pyg_ref as ref
from lesion_gnn_amd import _lib, optim, synth
from lesion_gnn_amd.graph import Graph
from lesion_gnn_amd.models import GCN

pytestmark = pytest.mark.gpu


class _Names:
    def __init__(self):
        self.names = []

    def __call__(self, name, args, launch):
        self.names.append(name)
        return launch()


def test_captured_step_sees_weights_loaded_between_replays(cuda):
    torch.manual_seed(0)
    m = GCN(128, [128, 128, 128], 5, 0.0).to(cuda).train()
    b = synth.make_batch(128, n=64, k=8, d_in=128, seed=3)
    x, ei, bt, y = (t.to(cuda) for t in (b.x, b.edge_index, b.batch, b.y))
    B = b.num_graphs
    opt = optim.Adam(m.parameters(), lr=1e-2, weight_decay=2e-6)
    out = {}

    def step():
        logits, loss = m.forward_loss(x, ei, bt, y, None, B)
        loss.backward()
        opt.step()
        out["logits"], out["loss"] = logits, loss

    side = torch.cuda.Stream(cuda)
    side.wait_stream(torch.cuda.current_stream(cuda))
    with torch.cuda.stream(side):
        for _ in range(2):
            step()
    torch.cuda.current_stream(cuda).wait_stream(side)
    opt.zero_grad(set_to_none=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    g.replay()
    torch.manual_seed(1)
    fresh = GCN(128, [128, 128, 128], 5, 0.0)
    m.load_state_dict(fresh.state_dict())  # in-place copies, outside the graph
    g.replay()
    torch.cuda.synchronize()
    oref = ref.GCN(128, [128, 128, 128], 5, 0.0)
    oref.load_state_dict(fresh.state_dict())
    want = oref(b.x, b.edge_index, b.batch, B)
    want_loss = torch.nn.functional.cross_entropy(want, b.y)
    torch.testing.assert_close(out["logits"].cpu(), want, rtol=0, atol=1e-4)
    torch.testing.assert_close(out["loss"].cpu(), want_loss, rtol=0, atol=1e-5)


def test_split_rides_the_build_or_runs_alone(cuda):
    torch.manual_seed(2)
    m = GCN(128, [128, 128, 128], 5, 0.0).to(cuda).train()
    b = synth.make_batch(64, n=64, k=8, d_in=128, seed=4)
    x, ei, bt = (t.to(cuda) for t in (b.x, b.edge_index, b.batch))
    res = []
    for prebuilt in (False, True):
        graph = Graph(ei, b.num_nodes, bt, b.num_graphs) if prebuilt else ei
        if prebuilt:
            graph.csr("gcn_lazy")
            graph.csr("gcn")
        tr = _Names()
        _lib.set_tracer(tr)
        try:
            lo = m(x, graph, bt, b.num_graphs)
        finally:
            _lib.set_tracer(None)
        assert ("lgnn_weight_planes" in tr.names) == prebuilt, tr.names
        if not prebuilt:
            assert "lgnn_graph_build_planes" in tr.names, tr.names
        res.append(lo)
    assert torch.equal(res[0], res[1])
