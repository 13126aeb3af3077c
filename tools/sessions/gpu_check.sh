#!/bin/bash
# One gpurun call: GPU tests, smoke, kernel sweeps, bench. Every GPU step has its
# own time limit and the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
true &&

timeout -k 10 300 python tools/sweep_kernels.py --algo sha256d > gpurun_out/sweep_sha.jsonl 2>&1 && echo "sweep sha ok" &&
timeout -k 10 300 python tools/sweep_kernels.py --algo scrypt > gpurun_out/sweep_scrypt.jsonl 2>&1 && echo "sweep scrypt ok" &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-latency > gpurun_out/bench.json 2> gpurun_out/bench.err && echo "bench ok"
