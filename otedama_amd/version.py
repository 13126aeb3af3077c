"""Build metadata (internal/version/version.go:19-75).

Version/commit/build date can be stamped at packaging time through the
``OTEDAMA_VERSION`` / ``OTEDAMA_COMMIT`` / ``OTEDAMA_BUILD_DATE`` environment
variables (the Go build uses -ldflags for the same three variables).
"""
from __future__ import annotations

import os
import platform
import subprocess
import sys
from dataclasses import asdict, dataclass
from pathlib import Path

VERSION = "v3.0.0-alpha.1-mi355x"


def _git_commit() -> str:
    root = Path(__file__).resolve().parent.parent
    try:
        out = subprocess.run(["git", "-C", str(root), "rev-parse", "--short", "HEAD"], capture_output=True,
                             text=True, timeout=2)
        return out.stdout.strip() or "unknown"
    except Exception:  # noqa: BLE001
        return "unknown"


@dataclass(frozen=True)
class Info:
    version: str
    commit: str
    build_date: str
    python_version: str
    platform: str
    gpu_arch: str = "gfx950"

    def to_dict(self) -> dict:
        return asdict(self)

    def __str__(self) -> str:
        return (f"otedama {self.version} ({self.commit}) built {self.build_date} with "
                f"python{self.python_version} for {self.platform} [{self.gpu_arch}]")


_cached: Info | None = None


def get() -> Info:
    global _cached
    if _cached is None:
        _cached = Info(
            version=os.environ.get("OTEDAMA_VERSION", VERSION),
            commit=os.environ.get("OTEDAMA_COMMIT") or _git_commit(),
            build_date=os.environ.get("OTEDAMA_BUILD_DATE", "unknown"),
            python_version=platform.python_version(),
            platform=f"{sys.platform}/{platform.machine()}",
        )
    return _cached
