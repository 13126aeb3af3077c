#!/bin/bash
# Round 3: bench with 2^32-hash launches on two streams per step, next to the launch-path comparison on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R3_TAG:-r3t}
mkdir -p $O
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
true &&
timeout -k 10 300 python tools/sha_paths.py > $O/sha_paths.json 2> $O/sha_paths.err && echo "sha paths ok" &&
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-latency > $O/bench_n1.json 2> $O/bench_n1.err && echo "bench ok"
