"""Resident set of a device process through its start-up (the ~1 GB of anonymous memory seen in
profiles/r3/m_devproc): RSS after the extension import, the miner thread's HIP start-up, the first SHA-256d job,
and with a few runtime knobs. Usage: python tools/rss_probe.py  (prints one JSON line)"""
from __future__ import annotations

import json
import os
import sys
import time

os.environ["OTEDAMA_NO_TORCH"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def rss() -> float:
    with open("/proc/self/statm") as f:
        return round(int(f.read().split()[1]) * os.sysconf("SC_PAGE_SIZE") / 2**20, 1)


def top(n: int = 6) -> list:
    sizes: dict[str, float] = {}
    name = "?"
    with open("/proc/self/smaps") as f:
        for line in f:
            parts = line.split()
            if parts and "-" in parts[0] and len(parts) >= 5:
                name = parts[5] if len(parts) >= 6 else "[anon]"
            elif parts and parts[0] == "Rss:":
                sizes[name] = sizes.get(name, 0.0) + int(parts[1]) / 1024
    return [(k, round(v, 1)) for k, v in sorted(sizes.items(), key=lambda kv: -kv[1])[:n]]


def main() -> int:
    out = {"start": rss()}
    from otedama_amd.models.header import int_to_hash
    from otedama_amd.ops.native import require_native

    N = require_native()
    out["native_imported"] = rss()
    N.gpu_cu_count(0)
    out["hip_runtime_up"] = rss()
    out["top_after_runtime"] = top()
    m = N.GpuMiner(0, "gpu-0", batch_nonces=1 << 32)
    m.start()
    time.sleep(1.0)
    out["miner_thread_up"] = rss()
    hdr = bytes(range(76)) + bytes(4)
    m.set_job({"header": hdr, "target": int_to_hash((1 << 200) - 1), "job_id": "r", "epoch": 1,
               "algo": "sha256d", "version_mask": 0x1FFFE000})
    time.sleep(1.5)
    out["sha_running"] = rss()
    out["top_sha_running"] = top()
    out["miner_phases_rss_mb"] = m.stats().get("startup_rss_mb")
    out["miner_phases_ms"] = m.stats().get("startup_ms")
    m.stop()
    out["stopped"] = rss()
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
