#!/bin/bash
# Round 3: single-midstate SHA-256d grid sweep past 64 blocks per CU, then bench.py N=1 with the new default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R3_TAG:-r3af}
mkdir -p $O
true &&
timeout -k 10 150 tools/bin/sha_single_ab 3 8192 16384 32768 65536 > $O/single_grids.json 2> $O/single.err && echo "grids ok" &&
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err && echo "bench ok"
