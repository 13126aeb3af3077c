"""Bounded insertion-ordered set for long-lived dedupe state.

Parity: the reference caps its unacked-submit map at 1024 entries and, when
full, drops the oldest half (internal/engine/run.go:720-726,944-957). The same
policy bounds the engine's submitted-share keys here, so a long block (or a
pool that never sends clean_jobs) cannot grow memory without limit.
"""
from __future__ import annotations

from typing import Hashable, Iterable, Iterator


class BoundedSet:
    __slots__ = ("cap", "_d", "evicted")

    def __init__(self, cap: int = 1024, items: Iterable[Hashable] = ()):
        if cap < 2:
            raise ValueError("cap must be >= 2")
        self.cap = cap
        self._d: dict = {}
        self.evicted = 0  # entries dropped by the halving policy (observability)
        for x in items:
            self.add(x)

    def add(self, key: Hashable) -> None:
        if key in self._d:
            return
        if len(self._d) >= self.cap:
            drop = len(self._d) // 2
            for k in list(self._d)[:drop]:  # dicts iterate in insertion order: the oldest half
                del self._d[k]
            self.evicted += drop
        self._d[key] = None

    def discard(self, key: Hashable) -> None:
        self._d.pop(key, None)

    def clear(self) -> None:
        self._d.clear()

    def __contains__(self, key: object) -> bool:
        return key in self._d

    def __len__(self) -> int:
        return len(self._d)

    def __iter__(self) -> Iterator:
        return iter(self._d)

    def __eq__(self, other: object) -> bool:
        if isinstance(other, BoundedSet):
            return self._d.keys() == other._d.keys()
        if isinstance(other, (set, frozenset)):
            return set(self._d) == other
        return NotImplemented

    def __repr__(self) -> str:
        return f"BoundedSet(cap={self.cap}, n={len(self._d)})"
