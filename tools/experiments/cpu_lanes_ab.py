"""CPU SHA-256d scan: single-thread rate for 1-4 nonces in flight (interleaved SHA-NI chains), rounds interleaved.
Prints one JSON line: MH/s per lane count per round and the medians."""
from __future__ import annotations

import json
import statistics
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/experiments/", 1)[0])
from otedama_amd.models.header import GENESIS_HEADER_HEX, int_to_hash  # noqa: E402
from otedama_amd.ops.native import require_native  # noqa: E402


def main() -> int:
    N = require_native()
    hdr = bytes.fromhex(GENESIS_HEADER_HEX)
    tgt = int_to_hash((1 << 200) - 1)
    n = 1 << 23
    res: dict[int, list[float]] = {l: [] for l in (1, 2, 3, 4)}
    for _ in range(3):
        for lanes in res:
            t0 = time.perf_counter()
            N._cpu_scan_lanes(lanes, hdr, tgt, 0, n)
            res[lanes].append(round(n / (time.perf_counter() - t0) / 1e6, 2))
    print(json.dumps({"mhs": res, "median": {l: statistics.median(v) for l, v in res.items()},
                      "sha_ni": bool(N.cpu_has_sha_ni()) if hasattr(N, "cpu_has_sha_ni") else None}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
