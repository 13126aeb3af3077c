#!/bin/bash
# Round 4, GPU pass j: miner-probe GPU tests (in-process and device process) and a bench whose scrypt / X11 miner
# sections run in device processes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/r4j
mkdir -p $D
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 200 python -u -m pytest tests/test_miner_probe.py -m gpu -x -v --timeout 120 --timeout-method thread > $D/pytest_miner_probe.log 2>&1; rc=$?
tail -3 $D/pytest_miner_probe.log; [ $rc -eq 0 ] &&
timeout -k 10 600 python bench.py > $D/bench.json 2> $D/bench.err && echo "bench ok" &&
python - <<'PY'
import json
d = json.load(open("gpurun_out/r4j/bench.json"))
for a in ("scrypt", "x11"):
    m = d[a].get("miner", {})
    print(a, d[f"{a}_hashes_per_sec"], d[a].get("rate_source"), d[a].get("kernel_path_hashes_per_sec"), m.get("path"),
          m.get("shares"), m.get("shares_recheck_ok"), m.get("window_device_seconds"), m.get("window_wall_seconds"))
print("value", d["value"], "node", d["node_hashes_per_sec"], "switch", d["job_switch_ms"])
PY
