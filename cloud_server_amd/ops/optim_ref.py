"""Flat-buffer optimizers: PyTorch reference implementations (numerics oracle + CPU path).

Semantics follow TF1's ``GradientDescent``/``Adagrad``/``Adam``/``Adadelta`` (the four
choices of the reference option catalog, apps/construction/util/options.py:26-37), so a
reference config trains the same way.  The MI355X path runs the same math in ONE fused
HIP launch over the whole flat buffer (``ops.fused.optimizer_step``).
"""
from __future__ import annotations

import math
from typing import Dict

import torch

OPT_SGD, OPT_ADAGRAD, OPT_ADAM, OPT_ADADELTA = 0, 1, 2, 3
OPT_IDS = {
    "GradientDescentOptimizer": OPT_SGD,
    "AdagradOptimizer": OPT_ADAGRAD,
    "AdamOptimizer": OPT_ADAM,
    "AdadeltaOptimizer": OPT_ADADELTA,
}
ADAGRAD_INIT = 0.1            # tf.train.AdagradOptimizer initial_accumulator_value
ADAM_B1, ADAM_B2, ADAM_EPS = 0.9, 0.999, 1e-8
ADADELTA_RHO, ADADELTA_EPS = 0.95, 1e-8


def n_slots(opt_id: int) -> int:
    return {OPT_SGD: 0, OPT_ADAGRAD: 1, OPT_ADAM: 2, OPT_ADADELTA: 2}[opt_id]


def init_slots(opt_id: int, numel: int, device) -> torch.Tensor:
    """Slots stacked [n_slots, numel] (a [0, numel] tensor for SGD)."""
    s = torch.zeros(n_slots(opt_id), numel, device=device, dtype=torch.float32)
    if opt_id == OPT_ADAGRAD:
        s.fill_(ADAGRAD_INIT)
    return s


def adam_lr_t(lr: float, step: int) -> float:
    """TF Adam bias correction with the 1-based step count."""
    return lr * math.sqrt(1.0 - ADAM_B2 ** step) / (1.0 - ADAM_B1 ** step)


@torch.no_grad()
def step_ref(opt_id: int, w: torch.Tensor, g: torch.Tensor, slots: torch.Tensor, lr: float,
             step: int) -> None:
    """In-place update of flat ``w`` with flat ``g``; ``step`` is 1-based."""
    if opt_id == OPT_SGD:
        w.add_(g, alpha=-lr)
    elif opt_id == OPT_ADAGRAD:
        acc = slots[0]
        acc.addcmul_(g, g)
        w.addcdiv_(g, acc.sqrt(), value=-lr)
    elif opt_id == OPT_ADAM:
        m, v = slots[0], slots[1]
        m.mul_(ADAM_B1).add_(g, alpha=1 - ADAM_B1)
        v.mul_(ADAM_B2).addcmul_(g, g, value=1 - ADAM_B2)
        w.addcdiv_(m, v.sqrt().add_(ADAM_EPS), value=-adam_lr_t(lr, step))
    elif opt_id == OPT_ADADELTA:
        acc, acc_up = slots[0], slots[1]
        acc.mul_(ADADELTA_RHO).addcmul_(g, g, value=1 - ADADELTA_RHO)
        upd = (acc_up + ADADELTA_EPS).sqrt().div_((acc + ADADELTA_EPS).sqrt()).mul_(g)
        acc_up.mul_(ADADELTA_RHO).addcmul_(upd, upd, value=1 - ADADELTA_RHO)
        w.add_(upd, alpha=-lr)
    else:
        raise ValueError(opt_id)
