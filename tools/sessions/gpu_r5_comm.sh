#!/bin/bash
# Round 5: the GPU tests and the comm-under-load A/B (legacy vs the node's high-priority layout).
set -o pipefail
out=gpurun_out/${1:-r5d}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$out/pytest.log" 2>&1 || exit $?
timeout -k 10 400 python -m otedama_amd.parallel.comm_probe --seconds 4 --windows 2 > "$out/comm.json" 2> "$out/comm.err"
