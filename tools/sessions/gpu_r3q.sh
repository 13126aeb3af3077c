#!/bin/bash
# Round 3: the round-end sequence after the stream / start-up / device-process changes: GPU suite, smoke, bench,
# and the production rehearsal (run vs 2-rank gloo node).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R3_TAG:-r3y}
mkdir -p $O
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
true &&
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.txt 2>&1 && echo "pytest gpu ok" &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && echo "smoke ok" &&
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > $O/bench_n1.json 2> $O/bench_n1.err && echo "bench ok" &&
timeout -k 10 300 python tools/gpu_node_rehearsal.py --seconds 25 --out-dir $O/node_rehearsal > $O/node_rehearsal.json 2> $O/node_rehearsal.err && echo "rehearsal ok"
