"""Per-segment GPU timers (the reference has no timers at all).

``SegmentTimer`` records HIP events around named segments of a step
(backbone / correlation / NC / loss / backward / all-reduce / optimizer) on
the current stream.  Recording an event does not synchronise; the elapsed
times are resolved only when ``collect()`` is called (once per log interval),
so enabling the timer does not serialise the step.  On CPU it falls back to
``time.perf_counter``.  With no timer installed (the default) ``segment()``
returns a null context, so the hot path pays one global lookup per segment.
Segments are skipped while a HIP graph is being captured (timed events cannot
be recorded into a graph).

Usage::

    timer = SegmentTimer()
    set_active(timer)
    with segment("backbone"):
        f = trunk(x)
    ...
    ms = timer.collect()          # {"backbone": 2.7, ...}, mean ms since the last collect
"""
from __future__ import annotations

import contextlib
import time
from collections import defaultdict

import torch

_ACTIVE: "SegmentTimer | None" = None


class SegmentTimer:
    def __init__(self, enabled: bool = True, device: torch.device | str | None = None):
        self.enabled = enabled
        self.gpu = enabled and torch.cuda.is_available() and (device is None or torch.device(device).type == "cuda")
        self._pending: list[tuple[str, object, object]] = []
        self._acc: dict[str, float] = defaultdict(float)
        self._count: dict[str, int] = defaultdict(int)

    @contextlib.contextmanager
    def __call__(self, name: str):
        if not self.enabled or (self.gpu and torch.cuda.is_current_stream_capturing()):
            yield
            return
        if self.gpu:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            try:
                yield
            finally:
                e.record()
                self._pending.append((name, s, e))
        else:
            t0 = time.perf_counter()
            try:
                yield
            finally:
                self._pending.append((name, t0, time.perf_counter()))

    def collect(self, reset: bool = True) -> dict[str, float]:
        """Resolve pending events (waits for the last one) -> mean ms per occurrence of each segment."""
        if not self.enabled:
            return {}
        if self.gpu and self._pending:
            self._pending[-1][2].synchronize()
        for name, s, e in self._pending:
            ms = s.elapsed_time(e) if self.gpu else (e - s) * 1e3
            self._acc[name] += ms
            self._count[name] += 1
        self._pending.clear()
        out = {k: round(self._acc[k] / max(self._count[k], 1), 4) for k in self._acc}
        if reset:
            self._acc.clear()
            self._count.clear()
        return out


def active() -> SegmentTimer | None:
    return _ACTIVE


def set_active(timer: SegmentTimer | None):
    """Install ``timer`` as the process-wide timer that model and trainer code report into."""
    global _ACTIVE
    _ACTIVE = timer


def segment(name: str):
    """Context manager timing ``name`` on the active timer (null context when none is installed)."""
    t = _ACTIVE
    if t is None or not t.enabled:
        return contextlib.nullcontext()
    return t(name)
