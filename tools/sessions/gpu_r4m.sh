#!/bin/bash
# Torch-free supervisor store on the GPU: the node GPU tests, then the 1-GPU bench (its node section runs
# `otedama node --gpus 1` under the new store and reports the supervisor's RSS).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/r4m
mkdir -p $D
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 400 python -u -m pytest tests/test_gpu_node.py tests/test_gpu_runtime.py -m gpu -x -v --timeout 180 --timeout-method thread > $D/pytest_gpu.log 2>&1; rc=$?
tail -3 $D/pytest_gpu.log; [ $rc -eq 0 ] &&
timeout -k 10 600 python -u bench.py > $D/bench.json 2> $D/bench.err && echo "bench ok" && python - <<'PY'
import json
d = json.load(open("gpurun_out/r4m/bench.json"))
n = d.get("node", {})
print(json.dumps({"value": d["value"], "node_total": n.get("total_hashes_per_sec"), "rss_mib": n.get("rss_mib"),
                  "scrypt": d.get("scrypt_hashes_per_sec"), "x11": d.get("x11_hashes_per_sec")}))
PY
