"""Loader for the in-tree native extension ``otedama_amd._native``.

The extension is built by ``otedama_amd._build`` (``__graft_entry__.build()``).
On a machine with a GPU a missing extension is an error, never a silent
fallback: every GPU op calls :func:`require_native`.
"""
from __future__ import annotations

import importlib
import os
import sys
import threading

_lock = threading.Lock()
_mod = None
_err: Exception | None = None


def load(build_if_missing: bool = True):
    """Import (building first if needed) and return the native module."""
    global _mod, _err
    with _lock:
        if _mod is not None:
            return _mod
        # torch must load its bundled HIP runtime BEFORE the extension: the
        # extension's libamdhip64.so.7 / libhsa-runtime64.so.1 needs are then
        # satisfied by torch's copies (same sonames). Loading the extension
        # first pulls /opt/rocm's runtime and torch then adds a second one, and
        # two HSA runtimes in one process cannot both enumerate the GPU.
        # A host without /dev/kfd has no GPU for either runtime to enumerate, so a CPU-only process skips the
        # ~2 s torch import (startup to first hash stays well under the reference's 1 s budget).
        # A device process (engine/devproc.py) never imports torch (OTEDAMA_NO_TORCH=1): the extension then binds
        # to /opt/rocm's runtime alone, and start-up skips torch's ~1-2 s import.
        no_torch = os.environ.get("OTEDAMA_NO_TORCH") == "1" and "torch" not in sys.modules
        if not no_torch and (os.path.exists("/dev/kfd") or os.environ.get("OTEDAMA_IMPORT_TORCH_FIRST") == "1"):
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
        try:
            _mod = importlib.import_module("otedama_amd._native")
            return _mod
        except ImportError as exc:  # not built yet
            _err = exc
        if build_if_missing and os.environ.get("OTEDAMA_NO_AUTOBUILD") != "1":
            try:
                from otedama_amd import _build

                _build.build()
                _mod = importlib.import_module("otedama_amd._native")
                return _mod
            except Exception as exc:  # noqa: BLE001 - surfaced by require_native
                _err = exc
        return None


def loaded():
    """The native module if this process already imported it, else None. Never imports: the extension links the HIP
    runtime (libamdhip64, libhsa-runtime64, comgr), ~1.4 s to page in on a cold GPU host, which a GPU-free engine
    (device processes own the GPUs) must not pay for an optional fast path."""
    return _mod if _mod is not None else sys.modules.get("otedama_amd._native")


def available() -> bool:
    return load() is not None


def require_native():
    mod = load()
    if mod is None:
        raise RuntimeError(f"otedama_amd._native is not available (build with `python -m otedama_amd._build`): {_err}")
    return mod


def gpu_count() -> int:
    """Number of visible HIP devices (0 when the extension or driver is missing)."""
    mod = load()
    if mod is None:
        return 0
    try:
        return int(mod.gpu_device_count())
    except Exception:  # noqa: BLE001
        return 0
