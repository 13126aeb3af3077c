#!/bin/bash
# Round 3: device-process kill/restart on the GPU, KFD enumeration, rehearsal with RSS breakdown.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R3_TAG:-r3m}
mkdir -p $O
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
true &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_devproc.py -m gpu -x -v -s --timeout 200 --timeout-method thread > $O/pytest_devproc.txt 2>&1 && echo "devproc tests ok" &&
timeout -k 10 300 python tools/gpu_node_rehearsal.py --seconds 15 --out-dir $O/node_rehearsal > $O/node_rehearsal.json 2> $O/node_rehearsal.err && echo "rehearsal ok"
