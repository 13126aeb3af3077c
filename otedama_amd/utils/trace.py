"""roctx spans for the Python control plane.

``rocprofv3 --marker-trace --kernel-trace -- python3 bench.py`` (or ``-- python3 -m otedama_amd run``)
then shows the node tick collectives (R1/R2/R3), share submit/ack marks and bench steps on the same
timeline as the gfx950 kernels and the native miner's ``otd.*.batch`` / ``otd.verify_candidates``
ranges (csrc/include/otedama/trace.h). The reference has no tracer; its closest aid is pprof
(`/debug/pprof/*`), which the API server also serves.

Tracing is an observer, never a dependency: without the native extension the calls are no-ops.
"""
from __future__ import annotations

import contextlib

_N = None
_tried = False


def _native():
    global _N, _tried
    if not _tried:
        _tried = True
        try:
            from otedama_amd.ops.native import load

            _N = load(build_if_missing=False)
        except Exception:  # noqa: BLE001
            _N = None
    return _N


@contextlib.contextmanager
def span(name: str):
    """Nested host range; use only where push/pop stay on one thread (not across ``await``)."""
    n = _native()
    if n is None:
        yield
        return
    n.trace_push(name)
    try:
        yield
    finally:
        n.trace_pop()


def mark(name: str) -> None:
    """Instant event (safe anywhere, including asyncio tasks)."""
    n = _native()
    if n is not None:
        n.trace_mark(name)
