#!/bin/bash
# Round 3: scrypt pad-size sweep (blocks per CU) now that new work aborts a batch at the next ROMix phase.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R3_TAG:-r3z}
mkdir -p $O
export TMPDIR=/tmp
true &&
timeout -k 10 600 python tools/scrypt_grid.py --rounds 2 > $O/scrypt_grid.json 2> $O/scrypt_grid.err && echo "scrypt grid ok"
