"""Why does the production miner run scrypt slower inside bench.py than in a torch-free process? Each variant is a
fresh child running engine/miner_probe.measure_miner: torch-free or with torch's HIP context (and a few torch
streams, as bench.py holds by then), at the scrypt diff-1 share target (~270 candidates/s) or at a target that finds
nothing. One JSON line per variant.

Usage: python tools/miner_ctx_ab.py [--algo scrypt] [--seconds 6]"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CHILD = r'''
import json, os, sys
sys.path.insert(0, sys.argv[1])
algo, secs, with_torch, target_bits = sys.argv[2], float(sys.argv[3]), sys.argv[4] == "1", int(sys.argv[5])
hold = None
if with_torch:
    import torch
    torch.cuda.init()
    torch.zeros(1, device="cuda:0")
    streams = [torch.cuda.Stream("cuda:0") for _ in range(3)]
    pad = os.environ.get("CTX_PAD", "")
    if pad:  # a 128 GiB torch allocation like bench.py's ops-API scrypt pad, written once, then freed or held
        big = torch.empty(128 << 30, dtype=torch.uint8, device="cuda:0")
        big.fill_(1)
        torch.cuda.synchronize()
        if pad == "freed":
            del big
            torch.cuda.empty_cache()
        else:
            hold = big
    heat = float(os.environ.get("CTX_HEAT", "0"))
    if heat > 0:  # keep the GPU busy first (bench.py's kernel sections run ~1 min before the miner sections)
        import time as _t
        from otedama_amd.ops.search import ScryptSearch
        from otedama_amd.models.header import int_to_hash as _ih
        from otedama_amd.ops.native import require_native as _rn
        _N = _rn()
        sc = ScryptSearch("cuda:0")
        prm = _N.scrypt_prepare(bytes(80), _ih((1 << 200) - 1))
        t_end = _t.monotonic() + heat
        b = 0
        while _t.monotonic() < t_end:
            sc.launch(prm, b)
            torch.cuda.synchronize()
            b += sc.batch
        del sc
        torch.cuda.empty_cache()
else:
    os.environ["OTEDAMA_NO_TORCH"] = "1"
from otedama_amd.ops.native import require_native
from otedama_amd.engine.miner_probe import measure_miner
N = require_native()
tgt = (0xFFFF << 224) if target_bits == 0 else (1 << target_bits) - 1
r = measure_miner(N, 0, algo, tgt, seconds=secs, warmup=2.0, recheck=8)
print(json.dumps({k: r[k] for k in ("hashes_per_sec", "launches", "shares", "window_device_seconds",
                                     "rejected_candidates", "dropped", "verify_dropped")}))
'''


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--algo", default="scrypt")
    ap.add_argument("--seconds", type=float, default=6.0)
    ap.add_argument("--pad", action="store_true", help="variants: a bench-like 128 GiB torch pad freed / held, 60 s of "
                                                     "scrypt load first")
    a = ap.parse_args()
    hits = 0 if a.algo == "scrypt" else 236  # scrypt: diff 1 (0xFFFF << 224); X11: 2^-20, as in bench.py
    variants = [("torch_free_hits", "0", hits, {}), ("torch_free_no_hits", "0", 200, {}),
                ("torch_hits", "1", hits, {}), ("torch_no_hits", "1", 200, {})]
    if a.pad:
        variants = [("torch_hits", "1", hits, {}), ("torch_pad_freed", "1", hits, {"CTX_PAD": "freed"}),
                    ("torch_pad_held", "1", hits, {"CTX_PAD": "held"}),
                    ("torch_heat_60s", "1", hits, {"CTX_HEAT": "60"}), ("torch_hits_again", "1", hits, {})]
    for name, torch_on, bits, extra in variants:
        out = subprocess.run([sys.executable, "-c", CHILD, ROOT, a.algo, str(a.seconds), torch_on, str(bits)],
                             capture_output=True, text=True, timeout=200, env=dict(os.environ, **extra))
        line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
        rec = json.loads(line[0]) if line else {"error": out.returncode, "stderr": out.stderr[-800:]}
        print(json.dumps({"variant": name, "algo": a.algo, **rec}), flush=True)
        if not line:
            return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
