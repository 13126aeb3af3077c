"""Interleaved A/B of the production GPU miner (native GpuMiner: launches, hit ring, abort word, verification)
between two source trees on one GPU, each measurement a fresh process.

python tools/ab_miner.py --a . --b ab_old [--rounds 3] [--seconds 10]
Prints one JSON line: SHA-256d hashes/s per round for A and B and the median ratio A/B.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys

CHILD = r'''
import os, sys, time, json
sys.path.insert(0, sys.argv[1])
os.environ["OTEDAMA_NO_TORCH"] = "1"
from otedama_amd.ops.native import require_native
from otedama_amd.models.header import int_to_hash
N = require_native()
secs = float(sys.argv[2])
algo = sys.argv[3] if len(sys.argv) > 3 else "sha256d"
m = N.GpuMiner(0, "gpu-0", batch_nonces=1 << 32, grid=N.gpu_cu_count(0) * 6, queue_cap=4096, sha_variants=128)
hdr = bytes(range(76)) + bytes(4)
m.set_job({"header": hdr, "target": int_to_hash((1 << (224 if algo == "sha256d" else 200)) - 1), "job_id": "ab",
           "epoch": 1, "algo": algo, "version_mask": 0x1FFFE000})
m.start()
time.sleep(3.0)

def edge():
    # the moment the completed-hash counter moves: a window between two such moments holds whole launches, so the
    # rate is exact (sampling at arbitrary times quantizes it by one 2^32-hash launch, +-2% over 10 s)
    h = m.stats()["hashes"]
    while True:
        h2 = m.stats()["hashes"]
        if h2 != h:
            return h2, time.monotonic()
        time.sleep(0.0002)

h0, t0 = edge()
time.sleep(secs)
h1, t1 = edge()
m.stop()
print(json.dumps({"hps": (h1 - h0) / (t1 - t0)}))
'''


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--a", default=".")
    ap.add_argument("--b", default="ab_old")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--env-a", default="", help="KEY=VALUE[,KEY=VALUE] for the A processes")
    ap.add_argument("--env-b", default="", help="KEY=VALUE[,KEY=VALUE] for the B processes")
    ap.add_argument("--algo", default="sha256d", choices=("sha256d", "scrypt", "x11"))
    a = ap.parse_args()

    def env_of(spec: str) -> dict:
        e = dict(os.environ)
        for kv in filter(None, spec.split(",")):
            k, _, v = kv.partition("=")
            e[k] = v
        return e

    res = {"a": [], "b": []}
    for _ in range(a.rounds):
        for key, tree, spec in (("a", a.a, a.env_a), ("b", a.b, a.env_b)):
            out = subprocess.run([sys.executable, "-c", CHILD, os.path.abspath(tree), str(a.seconds), a.algo],
                                 capture_output=True, text=True, timeout=120, env=env_of(spec))
            line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
            if out.returncode != 0 or not line:
                print(json.dumps({"error": key, "stderr": out.stderr[-2000:]}))
                return 1
            res[key].append(json.loads(line[0])["hps"])
    res["median_a"], res["median_b"] = statistics.median(res["a"]), statistics.median(res["b"])
    res["a_over_b"] = res["median_a"] / res["median_b"]
    res["algo"], res["env_a"], res["env_b"] = a.algo, a.env_a, a.env_b
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
