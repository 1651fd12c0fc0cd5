"""Tracing and phase timing (SURVEY §5 'Tracing / profiling').

The reference has no profiler: it times the 10-batch probe and each global
epoch with ``time.time()`` and no device synchronisation
(BAR/dataloader.py:120,134-136; BAR/trainer.py:39,179-180), so GPU time is
mis-measured.  Here:

* ``trace_range(name)`` pushes a roctx range through the native extension
  (``_C.trace_push``/``trace_pop``, linked against rocprofiler-sdk-roctx), so
  ``rocprofv3 --marker-trace`` shows forward / backward / comm-bucket /
  optimizer phases on the timeline next to the kernels.  Without the native
  extension (CPU hosts) it is a no-op.
* ``PhaseTimer`` brackets phases with HIP events recorded on the current
  stream.  Recording costs no host sync; the elapsed times are resolved once,
  when ``summary()`` is called (or, on CPU, with ``perf_counter``).

Both are off unless enabled (``--trace`` on the CLI, or ``LDNN_TRACE=1``).
"""
from __future__ import annotations

import contextlib
import os
import time
from collections import defaultdict

import torch

_enabled = os.environ.get("LDNN_TRACE", "0") not in ("", "0")
_native = None


def enable(flag: bool = True):
    global _enabled
    _enabled = bool(flag)


def enabled() -> bool:
    return _enabled


def _C():
    global _native
    if _native is None:
        try:
            from ..ops import _ext
            _native = _ext.C() if _ext.native_available() else False
        except Exception:  # pragma: no cover - extension import failure on a CPU host
            _native = False
    return _native


@contextlib.contextmanager
def trace_range(name: str):
    """roctx range around a phase (no-op when tracing is off or no native extension)."""
    if not _enabled:
        yield
        return
    C = _C()
    if C:
        C.trace_push(name)
    try:
        yield
    finally:
        if C:
            C.trace_pop()


def mark(name: str):
    if _enabled and _C():
        _C().trace_mark(name)


class PhaseTimer:
    """Per-phase device time without per-step host syncs.

    >>> t = PhaseTimer(torch.device("cpu"))
    >>> with t.phase("fwd"):
    ...     pass
    >>> sorted(t.summary())
    ['fwd']
    """

    def __init__(self, device=None, enabled: bool | None = None, max_pending: int = 4096):
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.gpu = self.device.type == "cuda" and torch.cuda.is_available()
        self.on = _enabled if enabled is None else enabled
        self.max_pending = max_pending
        self._pending: list[tuple[str, object, object]] = []
        self.total_ms: dict[str, float] = defaultdict(float)
        self.count: dict[str, int] = defaultdict(int)

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.on:
            yield
            return
        with trace_range(name):
            if self.gpu:
                a = torch.cuda.Event(enable_timing=True)
                b = torch.cuda.Event(enable_timing=True)
                a.record()
                try:
                    yield
                finally:
                    b.record()
                    self._pending.append((name, a, b))
                    if len(self._pending) >= self.max_pending:
                        self._resolve()
            else:
                t0 = time.perf_counter()
                try:
                    yield
                finally:
                    self.total_ms[name] += (time.perf_counter() - t0) * 1e3
                    self.count[name] += 1

    def _resolve(self):
        if not self._pending:
            return
        self._pending[-1][2].synchronize()
        for name, a, b in self._pending:
            self.total_ms[name] += a.elapsed_time(b)
            self.count[name] += 1
        self._pending.clear()

    def summary(self) -> dict[str, dict[str, float]]:
        """{phase: {"total_ms", "count", "mean_ms"}} (syncs once on the last pending event)."""
        self._resolve()
        return {k: {"total_ms": v, "count": self.count[k], "mean_ms": v / max(self.count[k], 1)}
                for k, v in self.total_ms.items()}

    def reset(self):
        self._resolve()
        self.total_ms.clear()
        self.count.clear()


_null_timer = PhaseTimer(enabled=False)


def null_timer() -> PhaseTimer:
    return _null_timer
