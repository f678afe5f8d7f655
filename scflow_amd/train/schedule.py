"""The training step's learning-rate schedule (configs/refine_models/scflow_ycbv_real.py:299-306:
``param_scheduler = [dict(type='OneCycleLR', eta_max=4e-4, total_steps=100100, pct_start=0.05,
anneal_strategy='linear')]`` under an ``IterBasedTrainLoop(max_iters=100000)``, :323).

mmengine (absent here) resolves 'OneCycleLR' to its ``OneCycleParamScheduler`` on ``lr``, whose
published algorithm is torch's ``OneCycleLR`` without momentum cycling: the lr starts at
``eta_max / div_factor``, moves to ``eta_max`` over the first ``pct_start·total_steps − 1`` steps,
then to ``initial / final_div_factor`` at step ``total_steps − 1`` (``three_phase``: up, back down
to the initial lr, then to the minimum), each phase annealed linearly or by a half cosine.
Step k of training (0-based) runs at ``lr_at(k)``; the optimizer is constructed at ``lr_at(0)``.
"""
from __future__ import annotations

import math


class OneCycleLR:
    """Per-iteration one-cycle schedule; ``lr_at(k)`` is the lr of training iteration k."""

    def __init__(self, eta_max: float, total_steps: int, pct_start: float = 0.3,
                 anneal_strategy: str = "cos", div_factor: float = 25.0,
                 final_div_factor: float = 1e4, three_phase: bool = False) -> None:
        if total_steps <= 0:
            raise ValueError(f"OneCycleLR: total_steps must be positive, got {total_steps}")
        if not 0.0 <= pct_start <= 1.0:
            raise ValueError(f"OneCycleLR: pct_start must be in [0, 1], got {pct_start}")
        if anneal_strategy not in ("cos", "linear"):
            raise ValueError(f"OneCycleLR: anneal_strategy must be 'cos' or 'linear', got "
                             f"{anneal_strategy!r}")
        self.eta_max = float(eta_max)
        self.total_steps = int(total_steps)
        self.anneal_strategy = anneal_strategy
        self.initial_lr = self.eta_max / div_factor
        self.min_lr = self.initial_lr / final_div_factor
        up = float(pct_start * self.total_steps) - 1
        if three_phase:
            self.phases = [(up, self.initial_lr, self.eta_max),
                           (float(2 * pct_start * self.total_steps) - 2, self.eta_max, self.initial_lr),
                           (self.total_steps - 1, self.initial_lr, self.min_lr)]
        else:
            self.phases = [(up, self.initial_lr, self.eta_max),
                           (self.total_steps - 1, self.eta_max, self.min_lr)]

    def _anneal(self, start: float, end: float, pct: float) -> float:
        if self.anneal_strategy == "linear":
            return (end - start) * pct + start
        return end + (start - end) / 2.0 * (math.cos(math.pi * pct) + 1)

    def lr_at(self, step: int) -> float:
        """Steps past the schedule's last (``total_steps − 1``) stay at its minimum lr — torch
        raises there, and a linear anneal evaluated at ``total_steps`` would dip below zero."""
        if step < 0:
            raise ValueError(f"OneCycleLR: step {step} is negative")
        step = min(step, self.total_steps - 1)
        start_step = 0.0
        for i, (end_step, lo, hi) in enumerate(self.phases):
            if step <= end_step or i == len(self.phases) - 1:
                return self._anneal(lo, hi, (step - start_step) / (end_step - start_step))
            start_step = end_step
        raise AssertionError("unreachable")


def reference_schedule(eta_max: float = 4e-4) -> OneCycleLR:
    """The configured schedule (scflow_ycbv_real.py:299-306)."""
    return OneCycleLR(eta_max, total_steps=100100, pct_start=0.05, anneal_strategy="linear")
