#!/bin/bash
# Round 4, GPU pass h: which bench.py section makes the production miner's scrypt / X11 rate lower inside bench.py
# (16.4 / 388 vs 17.3 / 397 in fresh processes)? Short benches with sections switched off, miner sections kept.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/r4h
mkdir -p $D
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
BASE="--steps 2 --warmup 1 --no-latency --node-seconds 0 --pool-seconds 0 --cpu-seconds 0 --miner-seconds 6"
timeout -k 10 240 python bench.py $BASE > $D/all.json 2> $D/all.err && echo "all ok" &&
timeout -k 10 240 python bench.py $BASE --single-midstate-headers 0 > $D/no_single.json 2> $D/no_single.err && echo "no_single ok" &&
timeout -k 10 240 python bench.py $BASE --x11-steps 0 > $D/no_x11.json 2> $D/no_x11.err && echo "no_x11 ok" &&
timeout -k 10 240 python bench.py $BASE --grid 256 --single-midstate-headers 0 > $D/small_sha.json 2> $D/small_sha.err && echo "small_sha ok" &&
python - <<'PY'
import json
for n in ("all", "no_single", "no_x11", "small_sha"):
    d = json.load(open(f"gpurun_out/r4h/{n}.json"))
    m = d["scrypt"].get("miner", {})
    x = d.get("x11", {}).get("miner", {})
    print(n, "scrypt kernel", round(d["scrypt"].get("kernel_path_hashes_per_sec", 0) / 1e6, 3), "miner",
          round(m.get("hashes_per_sec", 0) / 1e6, 3), "x11 miner", round(x.get("hashes_per_sec", 0) / 1e6, 1))
PY
