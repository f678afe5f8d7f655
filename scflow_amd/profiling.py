"""Timing of individual kernel launches inside a live run (bench.py roofline).

``KernelTimer`` is installed as ``decoder.kernel_hooks[name]``; the decoder calls it right
before and right after the launch it names.  Each call enqueues ``scflow_timestamp`` — a
one-thread kernel storing the GPU's constant-rate wall clock (s_memrealtime, 100 MHz on
MI355X) — on the current stream, the stream the timed kernel is enqueued on, so each pair
brackets exactly that launch (plus the dispatch gap).  Being ordinary kernels, the stamps are
also nodes of a captured hipGraph and every replay re-stamps: after replays, ``mean_ms`` is the
mean over the launches of the last replay.  (torch refuses external events on ROCm, and a
hipEventRecordWithFlags(external) inside a capture is rejected by this runtime.)
"""
from __future__ import annotations

import torch

from . import _lib


class KernelTimer:
    def __init__(self, capacity: int = 4096) -> None:
        self.capacity = capacity
        self.stamps = None
        self.n = 0
        self.enabled = True
        self._khz = None

    def __call__(self, start: bool) -> None:
        if not self.enabled:
            return
        if self.stamps is None:
            self.stamps = torch.zeros(self.capacity, dtype=torch.int64, device=torch.cuda.current_device())
        if self.n >= self.capacity:
            raise RuntimeError("KernelTimer capacity exceeded")
        if (self.n % 2 == 0) != start:
            raise RuntimeError("KernelTimer: unbalanced start/stop")
        lib = _lib.load()
        _lib.check(lib.scflow_timestamp(self.stamps.data_ptr(), self.n,
                                        torch.cuda.current_stream().cuda_stream), "scflow_timestamp")
        self.n += 1

    def reset(self) -> None:
        self.n = 0

    def durations_ms(self):
        if self._khz is None:
            self._khz = int(_lib.load().scflow_wallclock_khz())
        torch.cuda.synchronize()
        s = self.stamps[: self.n].cpu().tolist()
        return [(s[i + 1] - s[i]) / self._khz for i in range(0, self.n - 1, 2)]

    def mean_ms(self) -> float:
        d = self.durations_ms() if self.n >= 2 else []
        return sum(d) / len(d) if d else float("nan")

    def count(self) -> int:
        return self.n // 2


class EventTimer:
    """Eager-mode alternative: torch (HIP) timing events on the current stream — queue packets
    rather than kernel dispatches, so cheaper, but not usable inside a hipGraph capture."""

    def __init__(self, stride: int = 1) -> None:
        """``stride`` > 1 brackets only every stride-th launch (an event pair costs a few µs of
        queue time between dependent kernels); with stride = launches per step + 1 the bracketed
        launch moves one position every step, so K steps sample K different launch positions."""
        self.pairs = []
        self._start = None
        self.enabled = True
        self.stride = max(1, stride)
        self._calls = 0
        # device-scope timing events (scflow_timing_event_create): no system-scope cache
        # writeback inside the bracket
        self.device_scope = True

    def __call__(self, start: bool) -> None:
        if not self.enabled:
            return
        if start:
            self._calls += 1
        if (self._calls - 1) % self.stride:
            return
        if self.device_scope:
            from . import ops
            ev = ops.SyncEvent(timing=True)
            ev.record(ops.raw_stream(torch.cuda.current_device()))
        else:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
        if start:
            self._start = ev
        else:
            self.pairs.append((self._start, ev))

    def reset(self) -> None:
        self.pairs = []
        self._calls = 0

    def mean_ms(self) -> float:
        if not self.pairs:
            return float("nan")
        torch.cuda.synchronize()
        if self.device_scope:
            return sum(a.elapsed_ms(b) for a, b in self.pairs) / len(self.pairs)
        return sum(a.elapsed_time(b) for a, b in self.pairs) / len(self.pairs)

    def count(self) -> int:
        return len(self.pairs)
