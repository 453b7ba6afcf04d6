"""CPU: LinearWarmupCosineAnnealingLR (pl_bolts 0.7.0, the scheduler the reference's
configure_optimizers builds by name, models/base.py:174-175) against pl_bolts' recursive get_lr()
restated step by step here, and wired through BaseModule.configure_optimizers."""
import math

import pytest
import torch

from lesion_gnn_amd.optim import LinearWarmupCosineAnnealingLR


def pl_bolts_recursive(base, warmup, max_epochs, start, eta, epochs):
    """pl_bolts LinearWarmupCosineAnnealingLR.get_lr(), one value per epoch 0..epochs-1: every
    step updates the group's current lr from the previous one."""
    lr, out = None, []
    for e in range(epochs):
        if e == 0:
            lr = start
        elif e < warmup:
            lr = lr + (base - start) / (warmup - 1)
        elif e == warmup:
            lr = base
        elif (e - 1 - max_epochs) % (2 * (max_epochs - warmup)) == 0:
            lr = lr + (base - eta) * (1 - math.cos(math.pi / (max_epochs - warmup))) / 2
        else:
            lr = ((1 + math.cos(math.pi * (e - warmup) / (max_epochs - warmup)))
                  / (1 + math.cos(math.pi * (e - warmup - 1) / (max_epochs - warmup)))
                  * (lr - eta) + eta)
        out.append(lr)
    return out


@pytest.mark.parametrize("warmup,max_epochs,start,eta", [(10, 100, 0.0, 0.0), (5, 40, 1e-4, 1e-5),
                                                        (3, 7, 0.0, 1e-6), (0, 20, 1e-4, 0.0),
                                                        (1, 20, 1e-4, 0.0), (0, 9, 0.0, 1e-6)])
def test_schedule_matches_pl_bolts(warmup, max_epochs, start, eta):
    base = 1e-3
    p = torch.nn.Parameter(torch.zeros(2))
    opt = torch.optim.SGD([p], lr=base)
    sch = LinearWarmupCosineAnnealingLR(opt, warmup_epochs=warmup, max_epochs=max_epochs,
                                        warmup_start_lr=start, eta_min=eta)
    got = []
    for _ in range(max_epochs + 1):
        got.append(opt.param_groups[0]["lr"])
        opt.step()
        sch.step()
    want = pl_bolts_recursive(base, warmup, max_epochs, start, eta, max_epochs + 1)
    for e, (g, w) in enumerate(zip(got, want)):
        assert g == pytest.approx(w, rel=1e-9, abs=1e-15), e
    if warmup > 0:
        assert got[warmup] == pytest.approx(base)
        assert got[max_epochs] == pytest.approx(eta, abs=1e-15)
    else:  # pl_bolts starts at warmup_start_lr and decays from it (never reaches base)
        assert got[0] == start


def test_configure_optimizers_builds_warmup_cosine():
    from lesion_gnn_amd.models import GCNConfig, OptimizerConfig, get_model
    from lesion_gnn_amd.models.base import LRSchedulerConfig

    sc = LRSchedulerConfig(name="LinearWarmupCosineAnnealingLR",
                           kwargs={"warmup_epochs": 5, "max_epochs": 50})
    cfg = GCNConfig(optimizer=OptimizerConfig(lr_scheduler=sc, loss_type="MSE"),
                    hidden_channels=[16, 16], dropout=0.0, compile=False)
    cfg.num_classes.value, cfg.input_features.value = 5, 8
    out = get_model(cfg).configure_optimizers()
    assert isinstance(out["lr_scheduler"]["scheduler"], LinearWarmupCosineAnnealingLR)
    assert out["lr_scheduler"]["monitor"] == "val_loss"
    assert out["optimizer"].param_groups[0]["lr"] == 0.0  # warmup_start_lr at epoch 0
