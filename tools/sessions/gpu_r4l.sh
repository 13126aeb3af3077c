#!/bin/bash
# Round 4, GPU pass l: the bench's SHA-256d steps with and without the per-step stream join (old = joined), rounds
# interleaved, kernel section only. (tools/bench_join_old.py was the previous bench.py, removed after the run.)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/r4l
mkdir -p $D
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
ARGS="--steps 8 --warmup 1 --single-midstate-headers 0 --scrypt-steps 0 --x11-steps 0 --no-latency --node-seconds 0 --pool-seconds 0 --cpu-seconds 0 --miner-seconds 0"
for r in 1 2 3; do
  timeout -k 10 120 python bench.py $ARGS > $D/new_$r.json 2> $D/new_$r.err || exit 1
  timeout -k 10 120 python tools/bench_join_old.py $ARGS > $D/old_$r.json 2> $D/old_$r.err || exit 1
done
python - <<'PY'
import json, statistics
r = {k: [json.load(open(f"gpurun_out/r4l/{k}_{i}.json")) for i in (1, 2, 3)] for k in ("new", "old")}
for k, v in r.items():
    print(k, [round(d["value"] / 1e9, 3) for d in v], "hits", [(d["hits_found"], d["hits_verified"], d["hits_duplicate"], d["hits_outside_window"]) for d in v])
print("ratio", statistics.median(d["value"] for d in r["new"]) / statistics.median(d["value"] for d in r["old"]))
PY
