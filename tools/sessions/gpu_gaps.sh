#!/bin/bash
# Kernel-trace (no counters) of the X11 chain bench and the native miner, for inter-kernel idle gaps
# (tools/kernel_gaps.py). Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/gaps_x11 -o run --output-format csv -- python3 tools/bench_x11.py --iters 3 > gpurun_out/gaps_x11.log 2>&1 && echo "x11 trace ok" &&
timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/gaps_miner -o run --output-format csv -- python3 tools/trace_miner.py 3 > gpurun_out/gaps_miner.log 2>&1 && echo "miner trace ok"
