#!/bin/bash
# Round 3: device-process GPU tests (kill/restart, start-up, share latency with the pool in its own process).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R3_TAG:-r3aa}
mkdir -p $O
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
true &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_devproc.py -m gpu -x -v -s --timeout 200 --timeout-method thread > $O/pytest_devproc.txt 2>&1 && echo "devproc tests ok"
