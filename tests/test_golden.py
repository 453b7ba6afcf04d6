"""Golden vectors (tests/golden/*.npz, made by tests/golden/make_golden.py) on CPU:

1. the synthetic generator still produces the exact inputs (sha256 of x / edge_index / batch);
2. the oracle (oracle/pyg_ref.py) reproduces the committed logits, loss and gradients;
3. an independent float64 DENSE-adjacency restatement (tests/dense_ref.py) agrees with the
   golden logits, loss and gradients — two different formulations of the PyG 2.5.1 operators
   pin each other (parity against PyG itself stays unpinned: SURVEY.md §8c).
GPU parity against the same files lives in tests/test_gpu_*.py.
"""
import hashlib
import os

import numpy as np
import pytest
import torch

import oracle.pyg_ref as ref
from tests import dense_ref
from tests.golden import make_golden as mg

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with np.load(os.path.join(HERE, f"{name}.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def golden_state(g):
    return {k[len("params/"):]: torch.from_numpy(v) for k, v in g.items()
            if k.startswith("params/")}


@pytest.mark.parametrize("name", list(mg.CASES))
def test_inputs_regenerate(name):
    g = load(name)
    b = mg.make_batch(mg.CASES[name][2])
    for key, t in (("x", b.x), ("edge_index", b.edge_index), ("batch", b.batch)):
        assert hashlib.sha256(t.contiguous().numpy().tobytes()).hexdigest() == str(g["sha_" + key])
    assert np.array_equal(g["y"], b.y.numpy())


@pytest.mark.parametrize("name", list(mg.CASES))
def test_oracle_reproduces_golden(name):
    torch.set_num_threads(1)
    g = load(name)
    kind, mkw, bkw, loss_kind, seed = mg.CASES[name]
    m = mg.MODELS[kind](**mkw)
    m.load_state_dict(golden_state(g))
    m.train()
    b = mg.make_batch(bkw)
    logits = m(b.x, b.edge_index, b.batch, b.num_graphs)
    loss = ref.criterion(loss_kind, logits, b.y, mkw["num_classes"] if loss_kind == "CE" else 5)
    loss.backward()
    np.testing.assert_allclose(logits.detach().numpy(), g["logits"], rtol=1e-6, atol=1e-7)
    for k, p in m.named_parameters():
        np.testing.assert_allclose(p.grad.numpy(), g[f"grads/{k}"], rtol=1e-5, atol=1e-8,
                                   err_msg=k)


def dense_step(name, g):
    kind, mkw, bkw, loss_kind, _ = mg.CASES[name]
    b = mg.make_batch(bkw)
    sd = {k: v.to(torch.float64).requires_grad_(v.is_floating_point() and "running" not in k)
          for k, v in golden_state(g).items()}
    L = len(mkw.get("hidden_channels", mkw.get("hiddden_channels"))) - 1
    args = (sd, b.x, b.edge_index, b.batch, b.num_graphs, L)
    if kind == "gcn":
        logits = dense_ref.gcn_forward(*args, pool_kind=mkw["pool"])
    elif kind == "gin":
        logits = dense_ref.gin_forward(*args, pool_kind=mkw["pool"])
    else:
        logits = dense_ref.gat_forward(*args, heads=mkw["heads"])
    y = b.y
    if loss_kind == "CE":
        loss = torch.nn.functional.cross_entropy(logits, y)
    else:
        loss = torch.nn.functional.mse_loss(logits.squeeze(1).clamp(0, 4), y.to(torch.float64))
    loss.backward()
    return logits, loss, sd


@pytest.mark.parametrize("name", list(mg.CASES))
def test_dense_float64_restatement_agrees(name):
    g = load(name)
    logits, loss, sd = dense_step(name, g)
    np.testing.assert_allclose(logits.detach().numpy(), g["logits"], rtol=0, atol=2e-5)
    np.testing.assert_allclose(loss.item(), float(g["loss"]), rtol=1e-5)
    for k, t in sd.items():
        if t.requires_grad and f"grads/{k}" in g:
            want = g[f"grads/{k}"]
            scale = max(np.abs(want).max(), 1e-6)
            # atol floor: grads that vanish in exact arithmetic (a bias feeding BatchNorm) hold
            # only fp32 rounding noise in the golden file
            np.testing.assert_allclose(t.grad.numpy(), want, rtol=0, atol=max(1e-4 * scale, 5e-6),
                                       err_msg=k)
