#!/bin/bash
# Round 3: SHA-256d launch paths in one process (bench's ops launches vs the production miner).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R3_TAG:-r3s}
mkdir -p $O
export TMPDIR=/tmp
true &&
timeout -k 10 300 python tools/sha_paths.py > $O/sha_paths.json 2> $O/sha_paths.err && echo "sha paths ok"
