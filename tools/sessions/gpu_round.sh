#!/bin/bash
# Round-end rehearsal in one gpurun call: the GPU test suite (as the driver runs it), smoke(),
# then the 1-GPU bench. Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] &&
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log &&
timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err && echo "bench ok" && cat gpurun_out/bench.json
