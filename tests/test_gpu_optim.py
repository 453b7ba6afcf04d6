"""GPU: lesion_gnn_amd.optim.Adam / AdamW (one HIP launch per step) vs torch.optim.Adam / AdamW
on the same parameters and gradients. fp32; the update order of operations differs from
torch's kernels in the last bits only (rtol 1e-5, atol 1e-7)."""
import pytest
import torch

from lesion_gnn_amd import optim

pytestmark = pytest.mark.gpu


def _params(cuda, shapes, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return [torch.randn(*s, generator=g).to(cuda).requires_grad_() for s in shapes]


@pytest.mark.parametrize("kind,wd,maximize,n", [("adam", 2e-6, False, 5), ("adam", 0.1, True, 5),
                                                ("adamw", 1e-2, False, 5),
                                                ("adam", 1e-3, False, 40)])
def test_adam_matches_torch(cuda, kind, wd, maximize, n):
    shapes = [(128, 128), (128,), (5, 128), (5,), (3, 7, 2)] * (n // 5)
    ours, ref = _params(cuda, shapes, 0), _params(cuda, shapes, 0)
    cls = optim.Adam if kind == "adam" else optim.AdamW
    tcls = torch.optim.Adam if kind == "adam" else torch.optim.AdamW
    o = cls(ours, lr=1e-2, betas=(0.8, 0.95), eps=1e-7, weight_decay=wd, maximize=maximize)
    r = tcls(ref, lr=1e-2, betas=(0.8, 0.95), eps=1e-7, weight_decay=wd, maximize=maximize,
             foreach=False)
    gen = torch.Generator(device="cpu").manual_seed(1)
    for _ in range(6):
        for a, b in zip(ours, ref):
            gr = torch.randn(a.shape, generator=gen).to(cuda)
            a.grad, b.grad = gr.clone(), gr.clone()
        o.step()
        r.step()
    for a, b in zip(ours, ref):
        torch.testing.assert_close(a.detach(), b.detach(), rtol=1e-5, atol=1e-7)
    st = o.state[ours[0]]
    torch.testing.assert_close(st["exp_avg"], r.state[ref[0]]["exp_avg"], rtol=1e-5, atol=1e-7)
    assert float(st["step"]) == 6.0


def test_adam_graph_capture(cuda):
    """The step replays from a captured HIP graph and keeps counting steps on the device."""
    p = _params(cuda, [(64, 32), (32,)], 3)
    q = _params(cuda, [(64, 32), (32,)], 3)
    for a in p + q:
        a.grad = torch.full_like(a, 0.5)
    o = optim.Adam(p, lr=1e-2, weight_decay=1e-4)
    r = torch.optim.Adam(q, lr=1e-2, weight_decay=1e-4, foreach=False)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        o.step()
    torch.cuda.current_stream().wait_stream(s)
    r.step()
    gph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gph):
        o.step()
    for _ in range(4):
        gph.replay()
        r.step()
    torch.cuda.synchronize()
    for a, b in zip(p, q):
        torch.testing.assert_close(a.detach(), b.detach(), rtol=1e-5, atol=1e-7)
    assert float(o.state[p[0]]["step"]) == 5.0


def test_adam_rejects_cpu_and_amsgrad(cuda):
    from lesion_gnn_amd import _lib
    with pytest.raises(NotImplementedError):
        optim.Adam([torch.zeros(2, device=cuda, requires_grad=True)], amsgrad=True)
    w = torch.zeros(2, requires_grad=True)
    w.grad = torch.zeros(2)
    with pytest.raises(_lib.LgnnError):
        optim.Adam([w]).step()


def test_adam_many_tensors_captured_no_host_sync(cuda):
    """Many small tensors (three launches of LGNN_MAX_ADAM, so several step readers per step) plus
    numel-0 tensors — whose workgroups run no loop iteration but still read the step count and
    take a ticket — replayed from a captured graph 12 times back to back with no host sync in
    between: the device step counter and every parameter match torch.optim.Adam."""
    shapes = [(3,), (0,), (17, 5), (1,), (64,), (0, 4), (130,), (2, 2)] * 5
    p, q = _params(cuda, shapes, 11), _params(cuda, shapes, 11)
    gen = torch.Generator(device="cpu").manual_seed(2)
    grads = [torch.randn(s, generator=gen).to(cuda) for s in shapes]
    for a, b, g in zip(p, q, grads):
        a.grad, b.grad = g.clone(), g.clone()
    o = optim.Adam(p, lr=3e-3, betas=(0.85, 0.99), weight_decay=1e-3)
    r = torch.optim.Adam(q, lr=3e-3, betas=(0.85, 0.99), weight_decay=1e-3, foreach=False)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        o.step()  # warm-up: allocates the state outside capture
    torch.cuda.current_stream().wait_stream(s)
    r.step()
    gph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gph):
        o.step()
    for _ in range(12):
        gph.replay()
    for _ in range(12):
        r.step()
    torch.cuda.synchronize()
    assert float(o.state[p[0]]["step"]) == 13.0
    for a, b in zip(p, q):
        torch.testing.assert_close(a.detach(), b.detach(), rtol=1e-5, atol=1e-7)
