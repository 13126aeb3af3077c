#!/bin/bash
# Round 4 round-end rehearsal: every GPU test (as the driver runs them), smoke(), the 1-GPU bench, then a rocprofv3
# kernel trace of the production miner (one process: SHA-256d, scrypt, X11). Each GPU step has its own limit and the
# chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/r4f
mkdir -p $D
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $D/pytest_gpu.log 2>&1; rc=$?
tail -3 $D/pytest_gpu.log; [ $rc -eq 0 ] &&
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 && tail -1 $D/smoke.log &&
timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > $D/bench.json 2> $D/bench.err && echo "bench ok" && cut -c1-400 $D/bench.json &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $D/trace -o run --output-format csv -- python3 tools/trace_native_miner.py 4 > $D/trace.log 2>&1 && echo "trace ok" && grep -h '^{' $D/trace.log
