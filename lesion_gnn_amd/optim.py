"""Optimizers whose step is one HIP launch (lgnn_adam_step) — drop-ins for torch.optim.Adam /
AdamW (amsgrad=False) as the reference's configure_optimizers builds them (models/base.py:
162-188). torch runs the same update as multi_tensor_apply launches plus a step-count kernel.

State per parameter mirrors torch's ('step', 'exp_avg', 'exp_avg_sq'); every parameter of a
group shares one device step tensor. Graph-capturable: the launch reads only device pointers
(lr / betas / eps / weight_decay are launch arguments, so fixed inside a captured graph).
No CPU path: parameters and gradients must be contiguous fp32 GPU tensors.
"""
from __future__ import annotations

import ctypes
import math
import warnings

import torch

from . import _lib

MAX_TENSORS = 16  # LGNN_MAX_ADAM


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, maximize: bool = False, amsgrad: bool = False,
                 decoupled: bool = False):
        if amsgrad:
            raise NotImplementedError("lgnn Adam: amsgrad")
        if not 0.0 <= lr or not 0.0 <= eps or not 0.0 <= weight_decay:
            raise ValueError("lgnn Adam: lr, eps and weight_decay must be >= 0")
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay,
                        maximize=maximize)
        super().__init__(params, defaults)
        self._decoupled = decoupled
        self._tickets: dict[int, torch.Tensor] = {}

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            ps = [p for p in group["params"] if p.grad is not None]
            if not ps:
                continue
            _lib.require_gpu(*ps)
            dev = ps[0].device
            step_t = None
            for p in ps:
                if p.dtype != torch.float32 or not p.is_contiguous() or \
                        p.grad.dtype != torch.float32 or not p.grad.is_contiguous():
                    raise _lib.LgnnError("lgnn Adam: contiguous fp32 parameters and gradients")
                st = self.state[p]
                if not st:
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                step_t = st.get("step", step_t)
            if step_t is None:
                step_t = torch.zeros((), dtype=torch.float32, device=dev)
            for p in ps:
                self.state[p]["step"] = step_t
            ticket = self._tickets.get(gi)
            if ticket is None:
                # lgnn_adam_step's two-level ticket: 9 words, zeroed once, left zero
                ticket = self._tickets[gi] = torch.zeros(9, dtype=torch.int32, device=dev)
            b1, b2 = group["betas"]

            for c in range(0, len(ps), MAX_TENSORS):
                chunk = ps[c:c + MAX_TENSORS]
                n = len(chunk)
                arr = ctypes.c_void_p * n
                args = (n, arr(*[p.data_ptr() for p in chunk]),
                        arr(*[p.grad.data_ptr() for p in chunk]),
                        arr(*[self.state[p]["exp_avg"].data_ptr() for p in chunk]),
                        arr(*[self.state[p]["exp_avg_sq"].data_ptr() for p in chunk]),
                        (ctypes.c_int64 * n)(*[p.numel() for p in chunk]),
                        step_t.data_ptr(), ticket.data_ptr(), float(group["lr"]), float(b1),
                        float(b2), float(group["eps"]), float(group["weight_decay"]),
                        int(self._decoupled), int(group["maximize"]),
                        int(c + MAX_TENSORS >= len(ps)))
                _lib.call("lgnn_adam_step", *args, _lib.stream(dev))
        return loss


class AdamW(Adam):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 1e-2, maximize: bool = False, amsgrad: bool = False):
        super().__init__(params, lr, betas, eps, weight_decay, maximize, amsgrad, decoupled=True)


class LinearWarmupCosineAnnealingLR(torch.optim.lr_scheduler.LRScheduler):
    """pl_bolts.optimizers.lr_scheduler.LinearWarmupCosineAnnealingLR (pl_bolts 0.7.0), the
    scheduler the reference's configure_optimizers builds by name (models/base.py:174-175; pl_bolts
    is not installed here). A closed-form schedule per base lr b, epoch e (= last_epoch), warmup
    w, max m, start s, minimum eta, as pl_bolts' _get_closed_form_lr():
      e < w:  s + e (b - s) / max(1, w - 1)          (linear warmup from s to b)
      e >= w: eta + (b - eta) (1 + cos(pi (e - w) / (m - w))) / 2   (cosine to eta at e = m)
    get_lr() is pl_bolts' recursive form (each step from the group's current lr), restated case
    for case, so the schedule equals pl_bolts' for every warmup including w = 0 (where pl_bolts
    starts at warmup_start_lr and decays from there, unlike the closed form)."""

    def __init__(self, optimizer, warmup_epochs: int, max_epochs: int,
                 warmup_start_lr: float = 0.0, eta_min: float = 0.0, last_epoch: int = -1):
        self.warmup_epochs = int(warmup_epochs)
        self.max_epochs = int(max_epochs)
        self.warmup_start_lr = float(warmup_start_lr)
        self.eta_min = float(eta_min)
        super().__init__(optimizer, last_epoch)

    def _closed_form(self, base_lr: float) -> float:
        e, w, m = self.last_epoch, self.warmup_epochs, self.max_epochs
        if e < w:
            return self.warmup_start_lr + e * (base_lr - self.warmup_start_lr) / max(1, w - 1)
        span = max(1, m - w)
        return self.eta_min + 0.5 * (base_lr - self.eta_min) * (1 + math.cos(math.pi * (e - w)
                                                                               / span))

    def _get_closed_form_lr(self):
        return [self._closed_form(b) for b in self.base_lrs]

    def get_lr(self):
        if not getattr(self, "_get_lr_called_within_step", True):
            warnings.warn("To get the last learning rate computed by the scheduler, please use "
                          "`get_last_lr()`.", UserWarning)
        e, w, m, s, eta = (self.last_epoch, self.warmup_epochs, self.max_epochs,
                           self.warmup_start_lr, self.eta_min)
        span = max(1, m - w)
        groups = self.optimizer.param_groups
        if e == 0:
            return [s] * len(self.base_lrs)
        if e < w:
            return [g["lr"] + (b - s) / max(1, w - 1) for b, g in zip(self.base_lrs, groups)]
        if e == w:
            return list(self.base_lrs)
        if (e - 1 - m) % (2 * span) == 0:
            return [g["lr"] + (b - eta) * (1 - math.cos(math.pi / span)) / 2
                    for b, g in zip(self.base_lrs, groups)]
        return [(1 + math.cos(math.pi * (e - w) / span)) / (1 + math.cos(math.pi * (e - w - 1) / span))
                * (g["lr"] - eta) + eta for g in groups]

