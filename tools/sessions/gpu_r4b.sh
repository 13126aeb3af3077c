#!/bin/bash
# Round 4, second GPU pass: the GPU tests touched this round (runtime drop accounting, the node with device
# processes, X11 / scrypt miners), then the job-switch / rate A/Bs and the device-process RSS breakdown.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r4b
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 600 python -u -m pytest tests/test_gpu_runtime.py tests/test_gpu_node.py tests/test_x11_gpu.py tests/test_gpu_devproc.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r4b/pytest.log 2>&1; rc=$?
tail -4 gpurun_out/r4b/pytest.log; [ $rc -eq 0 ] &&
bash tools/gpu_switch_ab.sh &&
timeout -k 10 300 python tools/rss_breakdown.py > gpurun_out/r4b/rss.jsonl 2> gpurun_out/r4b/rss.err && echo "rss ok" &&
OTEDAMA_DIST_BACKEND=gloo timeout -k 10 300 python -c "
import json
from otedama_amd.parallel.node_probe import measure_node
print(json.dumps(measure_node(2, seconds=10, expected_per_gpu=9.7e9, shares_per_gpu=25.0)))
" > gpurun_out/r4b/node2_gloo.json 2> gpurun_out/r4b/node2_gloo.err && echo "node2 ok"
