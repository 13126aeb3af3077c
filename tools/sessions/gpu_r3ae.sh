#!/bin/bash
# Round 3: single-midstate SHA-256d with the peek poll in production; grid sweep (7 waves/SIMD = 7 blocks per CU
# resident) and the single-kernel GPU tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R3_TAG:-r3ae}
mkdir -p $O
true &&
timeout -k 10 150 tools/bin/sha_single_ab 3 1536 1792 2048 3584 7168 16384 > $O/single_grids.json 2> $O/single.err && echo "grids ok" &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "sha256d_genesis or easy_target or tie_filtered or wraps_nonce or runtime_shares" -p no:cacheprovider > $O/pytest_single.txt 2>&1 && echo "tests ok"
