"""The in-tree native extensions build for gfx950 and each is newer than every one of its sources.

Guards against running GPU jobs on a stale .so after a source edit whose compile
failed (the build is incremental: this is a no-op when everything is current).
"""
from pathlib import Path

from otedama_amd import _build


def test_native_build_is_current():
    out = _build.build()
    assert out.exists()
    rccl_out = _build.ext_path("_rccl")
    assert rccl_out.exists()
    csrc = Path(_build.CSRC)
    rccl_srcs = {csrc / s for s in _build.RCCL_SOURCES}
    sources = [p for p in csrc.rglob("*") if p.suffix in (".hip", ".cpp", ".h")]
    headers = [p for p in sources if p.suffix == ".h"]
    newest_native = max(p.stat().st_mtime for p in sources if p not in rccl_srcs)
    newest_rccl = max(p.stat().st_mtime for p in [*rccl_srcs, *headers])
    assert out.stat().st_mtime >= newest_native
    assert rccl_out.stat().st_mtime >= newest_rccl
