"""gfx950 HIP kernel ops and the native-extension loader."""
from otedama_amd.ops.native import available, gpu_count, load, require_native

__all__ = ["available", "gpu_count", "load", "require_native"]
