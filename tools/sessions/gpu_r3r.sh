#!/bin/bash
# Round 3: production miner A/B: split abort poll (this tree) vs the previous commit (ab_prev) vs pre-abort (ab_old).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R3_TAG:-r3r}
mkdir -p $O
export TMPDIR=/tmp
true &&
timeout -k 10 240 env PYTHONPATH=$PWD python -u -m pytest tests/test_gpu_runtime.py -m gpu -x -q --timeout 90 --timeout-method thread > $O/pytest_runtime.txt 2>&1 && echo "runtime tests ok" &&
timeout -k 10 300 python tools/ab_miner.py --a . --b ab_prev --rounds 3 --seconds 10 > $O/ab_miner_prev.json 2> $O/ab_miner_prev.err && echo "ab prev ok" &&
timeout -k 10 300 python tools/ab_miner.py --a . --b ab_old --rounds 3 --seconds 10 > $O/ab_miner_old.json 2> $O/ab_miner_old.err && echo "ab old ok"
