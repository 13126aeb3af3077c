"""Idle gaps between consecutive kernels in a rocprofv3 kernel trace.

python tools/kernel_gaps.py <kernel_trace.csv> [--min-kernels N]

For each kernel name: count, total busy ns, and the idle gap that precedes it (previous kernel's end to its
start, same queue). Prints one JSON line with the whole-trace busy fraction between the first and last kernel,
which is what a hipGraph (or any launch-overhead fix) could at most recover for a back-to-back kernel chain.
"""
from __future__ import annotations

import csv
import json
import statistics
import sys


def main(argv: list[str]) -> int:
    if not argv:
        print(__doc__)
        return 2
    rows = []
    with open(argv[0], newline="") as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", "")))
    rows.sort()
    per: dict[str, dict] = {}
    prev_end = None
    gaps = []
    for start, end, name, _q in rows:
        short = name.split("(")[0][:60]
        d = per.setdefault(short, {"count": 0, "busy_ns": 0, "gap_ns": []})
        d["count"] += 1
        d["busy_ns"] += end - start
        if prev_end is not None and start >= prev_end:
            d["gap_ns"].append(start - prev_end)
            gaps.append(start - prev_end)
        prev_end = max(prev_end or 0, end)
    span = rows[-1][1] - rows[0][0] if rows else 0
    busy = sum(e - s for s, e, _, _ in rows)
    out = {
        "kernels": len(rows), "span_ms": span / 1e6, "busy_ms": busy / 1e6,
        "busy_fraction": busy / span if span else None,
        "gap_median_us": statistics.median(gaps) / 1e3 if gaps else None,
        "gap_p95_us": sorted(gaps)[int(0.95 * (len(gaps) - 1))] / 1e3 if gaps else None,
        "per_kernel": {k: {"count": v["count"], "busy_ms": v["busy_ns"] / 1e6,
                           "gap_median_us": statistics.median(v["gap_ns"]) / 1e3 if v["gap_ns"] else None}
                       for k, v in per.items()},
    }
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
