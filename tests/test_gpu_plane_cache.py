"""GPU: split-3 weight planes kept across training steps (ops.cached_weight_planes) and rewritten
by the optimizer launch (lgnn_adam_step_planes), so the C2 step runs no weight-plane launch.

* after an Adam step the cached planes equal a fresh lgnn_weight_planes of the new weights,
  bitwise (normal and transposed);
* the next forward launches no lgnn_weight_planes (C-ABI tracer);
* an in-place update outside the optimizer (a version bump) makes the next forward rebuild them;
* three training steps (forward_loss + Adam, the bench's step) give bitwise the same weights with
  the cache on and off.
"""
import pytest
import torch

from lesion_gnn_amd import _lib, ops, optim, synth
from lesion_gnn_amd.models import GCN

pytestmark = pytest.mark.gpu


class _Count:
    def __init__(self):
        self.names = []

    def __call__(self, name, args, launch):
        self.names.append(name)
        return launch()


def _setup(cuda, seed=0):
    torch.manual_seed(seed)
    m = GCN(128, [128, 128, 128], 5, 0.0).to(cuda).train()
    b = synth.make_batch(128, n=64, k=8, d_in=128, seed=3)
    data = tuple(t.to(cuda) for t in (b.x, b.edge_index, b.batch, b.y))
    return m, data, b.num_graphs


def _step(m, opt, data, B):
    x, ei, bt, y = data
    opt.zero_grad(set_to_none=True)
    m.forward_loss(x, ei, bt, y, None, B)[1].backward()
    opt.step()


def test_adam_rewrites_cached_planes_bitwise(cuda):
    ops.invalidate_weight_planes()
    m, data, B = _setup(cuda)
    opt = optim.Adam(m.parameters(), lr=1e-2, weight_decay=2e-6)
    for _ in range(2):
        _step(m, opt, data, B)
    Ws = [m.in_proj.weight] + [c.lin.weight for c in m.convs]
    planes, planes_t = ops.cached_weight_planes(Ws, 128, True)
    fresh, fresh_t = ops.weight_planes(Ws, 128, True)
    assert torch.equal(planes, fresh) and torch.equal(planes_t, fresh_t)
    tr = _Count()
    _lib.set_tracer(tr)
    try:
        x, ei, bt, y = data
        m.forward_loss(x, ei, bt, y, None, B)
    finally:
        _lib.set_tracer(None)
    assert "lgnn_weight_planes" not in tr.names, tr.names


def test_outside_update_rebuilds_planes(cuda):
    ops.invalidate_weight_planes()
    m, data, B = _setup(cuda, 1)
    opt = optim.Adam(m.parameters(), lr=1e-2)
    _step(m, opt, data, B)
    with torch.no_grad():
        m.convs[0].lin.weight.mul_(0.5)  # a version bump
    tr = _Count()
    _lib.set_tracer(tr)
    try:
        x, ei, bt, y = data
        lo = m(x, ei, bt, B)
    finally:
        _lib.set_tracer(None)
    assert "lgnn_weight_planes" in tr.names
    ops.invalidate_weight_planes()
    with ops.no_plane_cache():
        want = m(x, ei, bt, B)
    assert torch.equal(lo, want)


def test_training_with_and_without_cache_bitwise(cuda):
    states = []
    for cache in (True, False):
        ops.invalidate_weight_planes()
        old = ops.PLANE_CACHE
        ops.PLANE_CACHE = cache
        try:
            m, data, B = _setup(cuda, 2)
            opt = optim.Adam(m.parameters(), lr=1e-2, weight_decay=2e-6)
            for _ in range(3):
                _step(m, opt, data, B)
            torch.cuda.synchronize()
            states.append({k: v.clone() for k, v in m.state_dict().items()})
        finally:
            ops.PLANE_CACHE = old
    for k in states[0]:
        assert torch.equal(states[0][k], states[1][k]), k
