"""The in-tree native extension builds for gfx950 and is newer than every source.

Guards against running GPU jobs on a stale .so after a source edit whose compile
failed (the build is incremental: this is a no-op when everything is current).
"""
from pathlib import Path

from otedama_amd import _build


def test_native_build_is_current():
    out = _build.build()
    assert out.exists()
    newest_src = max(p.stat().st_mtime for p in (Path(_build.CSRC)).rglob("*") if p.suffix in (".hip", ".cpp", ".h"))
    assert out.stat().st_mtime >= newest_src
