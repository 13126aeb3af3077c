#!/bin/bash
# roctx marker + kernel trace (no PMC counters in these runs) of the native miner and bench.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats -d gpurun_out/trace_miner -o run --output-format csv -- python3 tools/trace_miner.py 3 > gpurun_out/trace_miner.log 2>&1 && echo "trace miner ok" &&
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats -d gpurun_out/trace_bench -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 > gpurun_out/trace_bench.log 2>&1 && echo "trace bench ok"
