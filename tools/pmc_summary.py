"""Per-kernel summary of rocprofv3 --pmc / --kernel-trace CSVs.

python tools/pmc_summary.py <pmc_dir> [<pmc_dir> ...] [--nonces N] [--lanes-per-nonce k=v,...]
Sums every counter per kernel over dispatches and derives per-nonce instruction counts
(SQ_INSTS_* are wave-level: x64 lanes / nonces) and the LDS bank-conflict share.
"""
from __future__ import annotations

import argparse
import collections
import csv
import re
import sys


def short(name: str) -> str:
    m = re.search(r"(k_[a-z0-9_]+(?:<[a-z]+>)?)", name)
    if m:
        return m.group(1)
    return name.split("(")[0][-48:]


def load(dirs):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for d in dirs:
        with open(f"{d}/run_counter_collection.csv") as f:
            for row in csv.DictReader(f):
                k = short(row["Kernel_Name"])
                tot[k][row["Counter_Name"]] += float(row["Counter_Value"])
                disp[(d, k)].add(row["Dispatch_Id"])
                tot[k]["_vgpr"] = float(row["VGPR_Count"])
                tot[k]["_lds"] = float(row["LDS_Block_Size"])
    return tot


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--nonces", type=float, default=0, help="nonces processed per kernel over the profiled run")
    a = ap.parse_args()
    tot = load(a.dirs)
    cols = ["SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE",
            "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS", "SQ_BUSY_CYCLES"]
    w = csv.writer(sys.stdout)
    hdr = ["kernel", "vgpr", "lds_bytes"] + cols
    if a.nonces:
        hdr += ["valu_per_nonce", "lds_per_nonce"]
    hdr += ["lds_conflict_pct"]
    w.writerow(hdr)
    for k, c in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_BUSY_CYCLES", 0)):
        if not k.startswith("k_") and not k.startswith("otd"):
            continue
        row = [k, int(c["_vgpr"]), int(c["_lds"])] + [f"{c.get(x, 0):.4g}" for x in cols]
        if a.nonces:
            row += [f"{c.get('SQ_INSTS_VALU', 0) * 64 / a.nonces:.0f}", f"{c.get('SQ_INSTS_LDS', 0) * 64 / a.nonces:.0f}"]
        idx = c.get("SQ_LDS_IDX_ACTIVE", 0)
        row += [f"{100 * c.get('SQ_LDS_BANK_CONFLICT', 0) / idx:.1f}" if idx else ""]
        w.writerow(row)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
