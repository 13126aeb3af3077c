#!/bin/bash
# Round 3: JH / SHAvite kernel variants, X11 numerics, engine start-up phases, GPU tests, smoke, bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R3_TAG:-r3i}
mkdir -p $O
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
true &&
timeout -k 10 120 tools/bin/x11_variants 3 > $O/x11_variants.json 2> $O/x11_variants.err && echo "x11 variants ok" &&
timeout -k 10 240 python -u -m pytest tests/test_x11_gpu.py tests/test_gpu_runtime.py -m gpu -x -v -s --timeout 90 --timeout-method thread > $O/pytest_runtime.txt 2>&1 && echo "x11 + runtime tests ok" &&
timeout -k 10 300 python tools/gpu_node_rehearsal.py --seconds 15 --out-dir $O/node_rehearsal > $O/node_rehearsal.json 2> $O/node_rehearsal.err && echo "rehearsal ok" &&
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 && echo "pytest gpu ok" &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && echo "smoke ok" &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $O/bench_n1.json 2> $O/bench_n1.err && echo "bench ok"
