"""Zero-dependency Prometheus text-format (0.0.4) registry.

Parity: internal/metrics/metrics.go (Registry, Counter, Gauge, WriteText,
RegisterCollector, name/label validation, cross-type guard) and
internal/metrics/runtime.go (RuntimeCollector; the reference never registers it
in production — SURVEY §7.6 — here the engine registers it).

Semantics kept byte-compatible: entries sorted by (name, label key), HELP/TYPE
emitted once per name, label values escaped (\\, ", \\n), help escaped (\\, \\n),
floats rendered like Go's %g with NaN/+Inf/-Inf.
"""
from __future__ import annotations

import gc
import math
import os
import re
import resource
import sys
import threading
import time
from typing import Callable, TextIO

_NAME_RE = re.compile(r"^[a-zA-Z_:][a-zA-Z0-9_:]*$")
_LABEL_RE = re.compile(r"^[a-zA-Z_][a-zA-Z0-9_]*$")

CollectFunc = Callable[[TextIO], None]


class MetricsError(ValueError):
    """Invalid metric/label name or counter/gauge type clash (the reference panics)."""


def _metric_key(name: str, labels: dict[str, str] | None) -> str:
    if not labels:
        return name
    return name + "".join(f",{k}={labels[k]}" for k in sorted(labels))


def escape_label(v: str) -> str:
    return v.replace("\\", "\\\\").replace('"', '\\"').replace("\n", "\\n")


def escape_help(v: str) -> str:
    return v.replace("\\", "\\\\").replace("\n", "\\n")


def render_labels(labels: dict[str, str] | None) -> str:
    if not labels:
        return ""
    return "{" + ",".join(f'{k}="{escape_label(str(labels[k]))}"' for k in sorted(labels)) + "}"


def format_float(v: float) -> str:
    """Go's fmt ``%g`` for float64: shortest round-trip digits; exponent form
    (``d.ddde±XX``) when the decimal exponent is < -4 or >= 6."""
    v = float(v)
    if math.isnan(v):
        return "NaN"
    if math.isinf(v):
        return "+Inf" if v > 0 else "-Inf"
    if v == 0:
        return "-0" if math.copysign(1.0, v) < 0 else "0"
    if 1e-4 <= abs(v) < 1e6:
        # Fixed-point range of %g: Python's repr is the same shortest round-trip digits, without an exponent.
        r = repr(v)
        return r[:-2] if r.endswith(".0") else r
    return _format_float_exp(v)


def _format_float_exp(v: float) -> str:
    from decimal import Decimal

    sign, digits, exp = Decimal(repr(abs(v))).as_tuple()
    ds = "".join(map(str, digits)).rstrip("0") or "0"
    lead = len("".join(map(str, digits)).lstrip("0"))
    nd_all = len(digits)
    e10 = exp + nd_all - 1 - (nd_all - lead)  # exponent of the first significant digit
    neg = "-" if v < 0 else ""
    ds = ds.lstrip("0") or "0"
    if e10 < -4 or e10 >= 6:
        m = ds[0] + ("." + ds[1:] if len(ds) > 1 else "")
        return f"{neg}{m}e{'+' if e10 >= 0 else '-'}{abs(e10):02d}"
    if e10 >= 0:
        ip = ds[: e10 + 1].ljust(e10 + 1, "0")
        fp = ds[e10 + 1 :]
        return f"{neg}{ip}" + (f".{fp}" if fp else "")
    return f"{neg}0." + "0" * (-e10 - 1) + ds


class Counter:
    __slots__ = ("name", "help", "labels", "key", "prefix", "_v", "_lock")

    def __init__(self, name: str, help: str, labels: dict[str, str] | None):
        self.name, self.help, self.labels = name, help, dict(labels or {})
        # Labels are fixed for a series' lifetime: its sort key and exposition prefix are rendered once.
        self.key, self.prefix = _metric_key(name, self.labels), f"{name}{render_labels(self.labels)} "
        self._v = 0
        self._lock = threading.Lock()

    def inc(self) -> None:
        with self._lock:
            self._v += 1

    def add(self, delta: int) -> None:
        if delta < 0:
            raise MetricsError("counter delta must be non-negative")
        with self._lock:
            self._v = (self._v + int(delta)) & 0xFFFFFFFFFFFFFFFF

    def value(self) -> int:
        return self._v

    def text(self) -> str:
        return str(self._v)


class FloatCounter(Counter):
    """Counter of a real-valued quantity (e.g. accepted share difficulty, which is fractional below 1)."""

    __slots__ = ()

    def __init__(self, name: str, help: str, labels: dict[str, str] | None):
        super().__init__(name, help, labels)
        self._v = 0.0

    def add(self, delta: float) -> None:
        if not delta >= 0:
            raise MetricsError("counter delta must be non-negative")
        with self._lock:
            self._v += float(delta)

    def text(self) -> str:
        return format_float(self._v)


class Gauge:
    __slots__ = ("name", "help", "labels", "key", "prefix", "_v", "_lock", "_fv", "_ft")

    def __init__(self, name: str, help: str, labels: dict[str, str] | None):
        self.name, self.help, self.labels = name, help, dict(labels or {})
        self.key, self.prefix = _metric_key(name, self.labels), f"{name}{render_labels(self.labels)} "
        self._v = 0.0
        self._fv, self._ft = 0.0, "0"  # last formatted value (Go %g formatting is the costly part of a scrape)
        self._lock = threading.Lock()

    def set(self, v: float) -> None:
        with self._lock:
            self._v = float(v)

    def add(self, d: float) -> None:
        with self._lock:
            self._v += float(d)

    def value(self) -> float:
        return self._v

    def text(self) -> str:
        v = self._v
        if v != self._fv or math.copysign(1.0, v) != math.copysign(1.0, self._fv):  # NaN always re-formats
            self._ft, self._fv = format_float(v), v
        return self._ft


class Registry:
    def __init__(self) -> None:
        self._lock = threading.RLock()
        self._counters: dict[str, Counter] = {}
        self._gauges: dict[str, Gauge] = {}
        self._collectors: list[CollectFunc] = []

    @staticmethod
    def _validate(name: str, labels: dict[str, str] | None) -> None:
        if not _NAME_RE.match(name or ""):
            raise MetricsError(f"invalid metric name {name!r} (must match [a-zA-Z_:][a-zA-Z0-9_:]*)")
        for k in labels or {}:
            if not _LABEL_RE.match(k):
                raise MetricsError(f"invalid label name {k!r} on metric {name!r} (must match [a-zA-Z_][a-zA-Z0-9_]*)")

    def new_counter(self, name: str, help: str, labels: dict[str, str] | None = None,
                    float_value: bool = False) -> Counter:
        """``float_value``: a FloatCounter (real-valued increments) instead of the reference's uint64 counter."""
        self._validate(name, labels)
        key = _metric_key(name, labels)
        with self._lock:
            if key in self._counters:
                return self._counters[key]
            if any(g.name == name for g in self._gauges.values()):
                raise MetricsError(f"name {name!r} already registered as a gauge; cannot also be a counter")
            c = (FloatCounter if float_value else Counter)(name, help, labels)
            self._counters[key] = c
            return c

    def new_gauge(self, name: str, help: str, labels: dict[str, str] | None = None) -> Gauge:
        self._validate(name, labels)
        key = _metric_key(name, labels)
        with self._lock:
            if key in self._gauges:
                return self._gauges[key]
            if any(c.name == name for c in self._counters.values()):
                raise MetricsError(f"name {name!r} already registered as a counter; cannot also be a gauge")
            g = Gauge(name, help, labels)
            self._gauges[key] = g
            return g

    def register_collector(self, fn: CollectFunc) -> None:
        with self._lock:
            self._collectors.append(fn)

    def names(self) -> set[str]:
        with self._lock:
            return {c.name for c in self._counters.values()} | {g.name for g in self._gauges.values()}

    def write_text(self, w: TextIO) -> None:
        with self._lock:
            entries = [(c.name, c.key, c.help, "counter", c.prefix, c.text()) for c in self._counters.values()]
            entries += [(g.name, g.key, g.help, "gauge", g.prefix, g.text()) for g in self._gauges.values()]
            fns = list(self._collectors)
        entries.sort(key=lambda e: (e[0], e[1]))
        out: list[str] = []
        seen: set[str] = set()
        for name, _key, help_, kind, prefix, text in entries:
            if name not in seen:
                seen.add(name)
                out.append(f"# HELP {name} {escape_help(help_)}\n# TYPE {name} {kind}\n")
            out.append(f"{prefix}{text}\n")
        w.write("".join(out))
        for fn in fns:
            fn(w)

    def render(self) -> str:
        import io

        buf = io.StringIO()
        self.write_text(buf)
        return buf.getvalue()


_START = time.time()


def runtime_collector() -> CollectFunc:
    """Process/runtime gauges (the Go build's go_* series become python_*/process_*)."""
    pyver = sys.version.split()[0]

    def collect(w: TextIO) -> None:
        ru = resource.getrusage(resource.RUSAGE_SELF)
        try:
            with open("/proc/self/statm") as f:
                rss = int(f.read().split()[1]) * os.sysconf("SC_PAGE_SIZE")
        except OSError:
            rss = ru.ru_maxrss * 1024
        gcs = gc.get_stats()
        entries = [
            ("python_threads", "Number of Python threads that currently exist.", "gauge", "",
             str(threading.active_count())),
            ("python_info", "Information about the Python environment.", "gauge",
             f'{{version="{escape_label(pyver)}"}}', "1"),
            ("process_resident_memory_bytes", "Resident memory size in bytes.", "gauge", "", str(rss)),
            ("process_cpu_seconds_total", "Total user and system CPU time spent in seconds.", "counter", "",
             format_float(ru.ru_utime + ru.ru_stime)),
            ("process_start_time_seconds", "Start time of the process since unix epoch in seconds.", "gauge", "",
             format_float(_START)),
            ("python_gc_collections_total", "Total number of completed GC collections (all generations).",
             "counter", "", str(sum(g.get("collections", 0) for g in gcs))),
            ("python_gc_objects_collected_total", "Objects collected by the GC.", "counter", "",
             str(sum(g.get("collected", 0) for g in gcs))),
        ]
        w.write("".join(f"# HELP {n} {h}\n# TYPE {n} {k}\n{n}{lab} {v}\n" for n, h, k, lab, v in entries))

    return collect
