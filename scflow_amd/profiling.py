"""HIP-event timing of individual kernel launches inside a live run (bench.py roofline).

``KernelTimer`` is installed as ``decoder.kernel_hooks[name]``; the decoder calls it right
before and right after the launch it names.  Events are recorded on the current stream — the
stream the kernels are enqueued on — so each pair brackets exactly that launch.
"""
from __future__ import annotations

import torch


class KernelTimer:
    def __init__(self) -> None:
        self.pairs = []
        self._start = None
        self.enabled = True

    def __call__(self, start: bool) -> None:
        if not self.enabled:
            return
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        if start:
            self._start = ev
        else:
            self.pairs.append((self._start, ev))
            self._start = None

    def reset(self) -> None:
        self.pairs = []

    def mean_ms(self) -> float:
        if not self.pairs:
            return float("nan")
        return sum(s.elapsed_time(e) for s, e in self.pairs) / len(self.pairs)

    def count(self) -> int:
        return len(self.pairs)
