#!/bin/bash
# Round 3: one shared high-priority control stream; one vs two search streams in `otedama run` (hashrate, RSS).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R3_TAG:-r3p}
mkdir -p $O
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
true &&
timeout -k 10 240 python -u -m pytest tests/test_gpu_runtime.py -m gpu -x -v -s --timeout 90 --timeout-method thread > $O/pytest_runtime.txt 2>&1 && echo "runtime tests ok" &&
for i in 1 2; do
  timeout -k 10 150 python tools/gpu_node_rehearsal.py --run-only --seconds 20 --out-dir $O/run2_$i > $O/run_2streams_$i.json 2> $O/run2_$i.err || exit 1
  OTEDAMA_SEARCH_STREAMS=1 timeout -k 10 150 python tools/gpu_node_rehearsal.py --run-only --seconds 20 --out-dir $O/run1_$i > $O/run_1stream_$i.json 2> $O/run1_$i.err || exit 1
done && echo "stream A/B ok"
