"""Clock abstraction for deterministic tests (internal/clock/clock.go:48-109)."""
from __future__ import annotations

import threading
import time
from typing import Protocol


class Clock(Protocol):
    def now(self) -> float:  # seconds since the epoch
        ...

    def monotonic(self) -> float:
        ...


class SystemClock:
    """Wall clock (clock.System)."""

    def now(self) -> float:
        return time.time()

    def monotonic(self) -> float:
        return time.monotonic()


class FakeClock:
    """Manually advanced clock (clock.Fake with Set/Advance)."""

    def __init__(self, initial: float = 0.0):
        self._lock = threading.Lock()
        self._now = float(initial)

    def now(self) -> float:
        with self._lock:
            return self._now

    def monotonic(self) -> float:
        return self.now()

    def set(self, t: float) -> None:
        with self._lock:
            self._now = float(t)

    def advance(self, d: float) -> None:
        with self._lock:
            self._now += float(d)


SYSTEM = SystemClock()
