#!/bin/bash
# Round 4, second GPU pass (r4b plus the host-written abort word probe): can the CPU move the abort word without a
# control stream (tools/abort_host_write.hip), then the GPU tests touched this round, the job-switch / rate A/Bs, the
# device-process RSS breakdown and a 2-rank gloo node on the one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r4c
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 60 tools/bin/abort_host_write > gpurun_out/r4c/abort_host_write.jsonl 2> gpurun_out/r4c/abort_host_write.err; echo "abort probe rc=$?"
cat gpurun_out/r4c/abort_host_write.jsonl | head -60
timeout -k 10 600 python -u -m pytest tests/test_gpu_runtime.py tests/test_gpu_node.py tests/test_x11_gpu.py tests/test_gpu_devproc.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r4c/pytest.log 2>&1; rc=$?
tail -4 gpurun_out/r4c/pytest.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python tools/rss_breakdown.py > gpurun_out/r4c/rss.jsonl 2> gpurun_out/r4c/rss.err && echo "rss ok" &&
bash tools/gpu_switch_ab.sh &&
OTEDAMA_DIST_BACKEND=gloo timeout -k 10 300 python -c "
import json
from otedama_amd.parallel.node_probe import measure_node
print(json.dumps(measure_node(2, seconds=10, expected_per_gpu=9.7e9, shares_per_gpu=25.0)))
" > gpurun_out/r4c/node2_gloo.json 2> gpurun_out/r4c/node2_gloo.err && echo "node2 ok"
