#!/bin/bash
# Round 5 rehearsal of the driver's round end on the current tree: smoke, every GPU test, a kernel-trace profile of
# the production miner (SHA-256d, scrypt, X11 in one process), then bench.py with the driver's defaults (N=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r5k}
mkdir -p "$out"
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$out/pytest.log" 2>&1 \
  || exit $?
timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run --output-format csv \
  -- python3 tools/trace_native_miner.py 3 > "$out/prof.log" 2>&1 || exit $?
timeout -k 10 700 python bench.py > "$out/bench.json" 2> "$out/bench.err"
