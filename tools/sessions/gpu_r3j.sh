#!/bin/bash
# Round 3: high-priority control stream (job switch at 2^32 with other streams in the process), X11 variants,
# engine start-up phases incl. the SV2 dial steps, bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R3_TAG:-r3j}
mkdir -p $O
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
true &&
timeout -k 10 240 python -u -m pytest tests/test_gpu_runtime.py -m gpu -x -v -s --timeout 90 --timeout-method thread > $O/pytest_runtime.txt 2>&1 && echo "runtime tests ok" &&
timeout -k 10 120 tools/bin/x11_variants 3 > $O/x11_variants.json 2> $O/x11_variants.err && echo "x11 variants ok" &&
timeout -k 10 300 python tools/gpu_node_rehearsal.py --seconds 20 --out-dir $O/node_rehearsal > $O/node_rehearsal.json 2> $O/node_rehearsal.err && echo "rehearsal ok" &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $O/bench_n1.json 2> $O/bench_n1.err && echo "bench ok"
